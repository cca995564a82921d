// Device-resident state of a loopback channel (csrc/kernels/loopback.hip) and
// the pinned status block its kernels report to (csrc/loop_fabric.cpp).
#pragma once
#include <stdint.h>

#define LOOP_HEADERS 64  // message headers in flight per channel

enum : uint32_t {
  LOOP_OK = 0,
  LOOP_ERR_ABORT = 1,     // the host aborted the data plane (watchdog)
  LOOP_ERR_TIMEOUT = 2,   // a device wait exceeded the channel's spin limit
  LOOP_ERR_MISMATCH = 3,  // posted receive size != size of the message at the channel head
};

struct LoopChan {
  // written by the sender's kernels only (stream-ordered)
  uint64_t s_seq, s_off;
  uint32_t s_ticket, r_ticket;    // last-block tickets of the op in flight (reset by that block)
  // written by the receiver's release only; polled by the sender
  uint64_t r_seq, r_off;
  // constant after creation
  uint64_t cap;         // ring bytes
  uint64_t spin_limit;  // s_memrealtime ticks (100 MHz) a wait may last
  uint8_t* ring;        // the owner's address (diagnostics only: kernels take theirs as an argument)
  uint32_t id, pad;
  uint64_t stall_from;  // fault injection (tests): messages >= this are never published
  // message headers: tag = seq + 1 once {size, off} and the payload are visible
  uint64_t h_tag[LOOP_HEADERS];
  uint64_t h_size[LOOP_HEADERS];
  uint64_t h_off[LOOP_HEADERS];
};

// Pinned (fine-grained) host memory, mapped into the device: the host sets
// `abort`; kernels record the first error they hit.
struct LoopStatus {
  uint32_t abort;
  uint32_t err;
  uint32_t err_chan;
  uint32_t pad;
};
