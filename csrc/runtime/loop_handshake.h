// Host-side enqueue handshake of a device loopback channel, free of HIP so it
// can be built and stress-tested on its own under ThreadSanitizer
// (csrc/runtime/tests/loop_handshake_stress.cpp).  csrc/loop_fabric.cpp uses
// it for every channel of the single-GPU rehearsal of the RCCL pipeline edges
// (parallel/comm.py DeviceLoopTransport / IpcLoopTransport).
//
// Rule (loop_fabric.cpp module comment): per channel,
//   receive #n may be enqueued only after send #n was enqueued;
//   send #n only after the receives that free its header slot and its ring
//   bytes were enqueued.
// Each side's mirror words are written by the one thread (or process) that
// owns that side and read by the other: the owner publishes a count with a
// release store after the byte position it covers, the peer acquire-loads the
// count before the position.  A mirror is one 64-B line (it may live in a
// POSIX shared-memory block shared by two processes).
#pragma once

#include <atomic>
#include <chrono>
#include <cstdint>
#include <functional>
#include <stdexcept>
#include <string>
#include <thread>

namespace lsd_rt {

constexpr uint64_t kLoopHeaders = 64;  // == LOOP_HEADERS (csrc/kernels/loopback.h)

// Ring placement of a message: 256-B aligned, never straddling the ring's end
// (it skips to the next lap).  Must equal the device kernels' place().
inline uint64_t loop_place(uint64_t head, uint64_t bytes, uint64_t cap) {
  head = (head + 255) & ~(uint64_t)255;
  const uint64_t o = head % cap;
  return (o + bytes > cap) ? head + (cap - o) : head;
}

struct alignas(64) LoopMirror {
  std::atomic<uint64_t> send_n, send_end;  // sender side: messages enqueued, ring end
  std::atomic<uint64_t> recv_n, recv_end;  // receiver side
  std::atomic<uint64_t> stall_from;        // fault injection (tests)
};
static_assert(sizeof(LoopMirror) == 64, "one cache line per channel mirror");

inline void loop_mirror_init(LoopMirror* m) {
  m->send_n.store(0, std::memory_order_relaxed);
  m->send_end.store(0, std::memory_order_relaxed);
  m->recv_n.store(0, std::memory_order_relaxed);
  m->recv_end.store(0, std::memory_order_relaxed);
  m->stall_from.store(~0ull, std::memory_order_release);
}

// May receive #(recv_n + k) be enqueued?  (k: earlier receives of the same
// I/O list on this channel, not yet mirrored.)  Receiver thread only.
inline bool loop_can_recv(const LoopMirror* m, uint64_t k) {
  return m->send_n.load(std::memory_order_acquire) > m->recv_n.load(std::memory_order_relaxed) + k;
}

// May send #(send_n + k) of `bytes` at ring head `head` be enqueued?  Sender
// thread only.  The receive count is loaded before the ring end it covers.
inline bool loop_can_send(const LoopMirror* m, uint64_t k, uint64_t head, uint64_t bytes, uint64_t cap) {
  const uint64_t rn = m->recv_n.load(std::memory_order_acquire);
  const uint64_t rend = m->recv_end.load(std::memory_order_acquire);
  const uint64_t n = m->send_n.load(std::memory_order_relaxed) + k;
  const uint64_t off = loop_place(head, bytes, cap);
  return n - rn < kLoopHeaders && off + bytes - rend <= cap;
}

// The owner side's mirror after it enqueued one op (send: dir 0, receive: 1):
// the ring end first, then the count with release, so a peer that sees the
// count also sees the end.
inline void loop_advance(LoopMirror* m, int dir, uint64_t bytes, uint64_t cap) {
  auto& n = dir ? m->recv_n : m->send_n;
  auto& end = dir ? m->recv_end : m->send_end;
  end.store(loop_place(end.load(std::memory_order_relaxed), bytes, cap) + bytes, std::memory_order_release);
  n.store(n.load(std::memory_order_relaxed) + 1, std::memory_order_release);
}

// Wait until `ok()` holds: yield-spin briefly, then sleep (several stage
// threads wait at once and must not take the CPUs their peers need).  Throws
// `aborted_msg` once `aborted()` turns true and `timeout_msg` after
// `timeout_s` (non-positive: 600 s).
inline void loop_wait_until(const std::function<bool()>& ok, const std::function<bool()>& aborted,
                            double timeout_s, const std::string& aborted_msg, const std::string& timeout_msg) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  const double limit = timeout_s > 0 ? timeout_s : 600.0;
  for (uint64_t spins = 0;; ++spins) {
    if (ok()) return;
    if (aborted()) throw std::runtime_error(aborted_msg);
    if (spins < 64) {
      std::this_thread::yield();
      continue;
    }
    if (std::chrono::duration<double>(clk::now() - t0).count() > limit) throw std::runtime_error(timeout_msg);
    std::this_thread::sleep_for(std::chrono::microseconds(spins < 256 ? 5 : 25));
  }
}

}  // namespace lsd_rt
