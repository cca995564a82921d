// Device-side loopback channels: the RCCL-shaped data plane of the
// single-GPU pipeline rehearsal (parallel/comm.py DeviceLoopTransport).
//
// The reference relays every hidden state through its coordinator over HTTP
// (`server.py:171-181`).  On an 8-GPU node a pipeline edge is an RCCL
// ncclSend / ncclRecv pair on a 2-rank communicator whose kernels spin on a
// FIFO of slots in the peer's memory.  On ONE MI355X the rehearsal needs the
// same semantics -- ops enqueued on the lane stream (eagerly or captured in a
// hipGraph), matched strictly in per-channel FIFO order, device-side waits,
// no host synchronisation -- so a channel here is that FIFO: a byte ring in
// HBM plus a ring of message headers, written by the sending stage's kernels
// and drained by the receiving stage's.
//
// Protocol (one channel = one (edge, lane) of one pipeline):
//   send  = wait for ring space, copy the payload into the ring, publish the
//           header {size, offset} and tag = seq + 1
//   recv  = wait for the tag, check the size, copy out, release the space
// One launch per op; its last block (agent-scope ticket, every block drained
// and released first) publishes the tag / releases the space.  Every
// cross-stream word is an agent-scope atomic (tags / consumed counters),
// every wait is polled by ONE lane per block, bounded in time (s_memrealtime)
// and abortable through a word in pinned host memory (the watchdog's abort):
// no spin in this file can outlive its deadline.
//
// Header size check: a receive whose posted size differs from the message at
// the head of its channel records LOOP_ERR_MISMATCH instead of copying -- the
// RCCL op-ordering contract (same op sequence on both ends of a communicator)
// checked on every transfer.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "loopback.h"

namespace {

typedef uint64_t u64;
typedef uint32_t u32;

constexpr int THREADS = 256;
constexpr int CHUNK = THREADS * 16 * 4;  // bytes per block per pass (4 x 16 B per thread)

__device__ __forceinline__ u64 ld_agent(const u64* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent_release(u64* p, u64 v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u32 ld_sys(const u32* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void set_err(LoopStatus* st, u32 code, u32 chan) {
  // vector stores to the pinned status block (first error is enough; a
  // later one may overwrite it -- any non-zero code fails the engine)
  __hip_atomic_store(&st->err_chan, chan, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(&st->err, code, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Ring placement: a message occupies [off, off + bytes) of the monotonic byte
// stream, starts 256-B aligned (16-B vector copies on both ends; the ring
// itself is 256-B aligned) and never straddles the ring's end (it skips to
// the next lap).  The host handshake mirrors this function exactly.
__device__ __host__ __forceinline__ u64 place(u64 head, u64 bytes, u64 cap) {
  head = (head + 255) & ~(u64)255;
  const u64 o = head % cap;
  return (o + bytes > cap) ? head + (cap - o) : head;
}

// Bounded wait helper: ONE lane polls; every 64 polls it also reads the
// host abort word.  Returns 0 (condition met), LOOP_ERR_ABORT or
// LOOP_ERR_TIMEOUT.
template <typename Cond>
__device__ u32 bounded_wait(Cond cond, const LoopStatus* st, u64 limit_ticks) {
  const u64 t0 = __builtin_amdgcn_s_memrealtime();
  for (u32 n = 0;; ++n) {
    if (cond()) return 0;
    if ((n & 63) == 63) {
      if (ld_sys(&st->abort)) return LOOP_ERR_ABORT;
      if (__builtin_amdgcn_s_memrealtime() - t0 > limit_ticks) return LOOP_ERR_TIMEOUT;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

// 16-byte vector copy of [0, bytes) when both ends are 16-B aligned, 4-byte
// words otherwise (every wire tensor is fp32 / bf16 / int32: sizes % 2 == 0;
// a trailing odd half-word is copied bytewise).
__device__ __forceinline__ void copy_part(uint8_t* dst, const uint8_t* src, u64 bytes) {
  const u64 tid = (u64)blockIdx.x * THREADS + threadIdx.x;
  const u64 nth = (u64)gridDim.x * THREADS;
  if ((((uintptr_t)dst | (uintptr_t)src) & 15) == 0) {
    const u64 n16 = bytes >> 4;
    const uint4* s = reinterpret_cast<const uint4*>(src);
    uint4* d = reinterpret_cast<uint4*>(dst);
    for (u64 i = tid; i < n16; i += nth) d[i] = s[i];
    for (u64 i = (n16 << 4) + tid; i < bytes; i += nth) dst[i] = src[i];
  } else if ((((uintptr_t)dst | (uintptr_t)src) & 3) == 0) {
    const u64 n4 = bytes >> 2;
    const u32* s = reinterpret_cast<const u32*>(src);
    u32* d = reinterpret_cast<u32*>(dst);
    for (u64 i = tid; i < n4; i += nth) d[i] = s[i];
    for (u64 i = (n4 << 2) + tid; i < bytes; i += nth) dst[i] = src[i];
  } else {
    for (u64 i = tid; i < bytes; i += nth) dst[i] = src[i];
  }
}

// One kernel per op, on at most MAX_BLOCKS blocks: in every block ONE lane
// polls (bounded) before the block copies its share; the last block to finish
// (agent-scope ticket) publishes the message / releases its ring space.  The
// block cap bounds the waves that waiting ops can hold -- MAX_BLOCKS x 4 per
// op, a few percent of the chip even with every lane of eight stages waiting
// -- so a waiting op never takes the CUs the kernel it waits for needs.  (The
// first version spun on up to 256 blocks per op; eight stage threads' prefill
// sends filled the chip with spinning waves and the receives that would free
// their ring space could not start: a device-wait timeout in the 8-stage
// rehearsal.  The second ran wait / copy / finish as three launches, ~6 extra
// kernels per decode item: profiles/r4_rehearsal_graph_io.log.)
//
// `ring` is this process's address of the channel's ring (an IPC mapping when
// the peer process owns it): pointers never travel through the shared state.
constexpr int MAX_BLOCKS = 16;

__device__ __forceinline__ bool send_space(const LoopChan* ch, u64 seq, u64 off, u64 bytes) {
  // header slot free and [r_off, off + bytes) within one ring
  return seq - ld_agent(&ch->r_seq) < LOOP_HEADERS && off + bytes - ld_agent(&ch->r_off) <= ch->cap;
}

// The calling block is the last of the launch to get here (ticket), after
// every block drained its memory operations.  Single lane.
__device__ __forceinline__ bool last_block(u32* ticket) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // this block's stores / completed reads first
  const u32 t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (t != gridDim.x - 1) return false;
  __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next op
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // every other block's release before ours
  return true;
}

__global__ __launch_bounds__(THREADS) void loop_send_kernel(LoopChan* ch, uint8_t* ring, const uint8_t* src,
                                                            u64 bytes, LoopStatus* st) {
  __shared__ u32 verdict;
  const u64 cap = ch->cap, seq = ch->s_seq;  // sender-private: stream-ordered
  const u64 off = place(ch->s_off, bytes, cap);
  if (threadIdx.x == 0) {
    const u32 v = bounded_wait([&] { return send_space(ch, seq, off, bytes); }, st, ch->spin_limit);
    if (v) set_err(st, v, ch->id);
    verdict = v;
  }
  __syncthreads();
  if (verdict) return;  // the data plane is failed: nothing is published
  copy_part(ring + off % cap, src, bytes);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
  __syncthreads();
  if (threadIdx.x == 0 && last_block(&ch->s_ticket) && seq < ch->stall_from) {  // stall_from: tests
    const u32 k = (u32)(seq % LOOP_HEADERS);
    __hip_atomic_store(&ch->h_size[k], bytes, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&ch->h_off[k], off, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    st_agent_release(&ch->h_tag[k], seq + 1);
    ch->s_seq = seq + 1;  // read by the channel's next send (stream order)
    ch->s_off = off + bytes;
  }
}

__global__ __launch_bounds__(THREADS) void loop_recv_kernel(LoopChan* ch, const uint8_t* ring, uint8_t* dst,
                                                            u64 bytes, LoopStatus* st) {
  __shared__ u32 verdict;
  __shared__ u64 s_off;
  const u64 seq = ch->r_seq;  // receiver-private: stream-ordered
  if (threadIdx.x == 0) {
    const u32 k = (u32)(seq % LOOP_HEADERS);
    u32 v = bounded_wait([&] { return ld_agent(&ch->h_tag[k]) == seq + 1; }, st, ch->spin_limit);
    if (!v) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      s_off = ld_agent(&ch->h_off[k]);
      if (ld_agent(&ch->h_size[k]) != bytes) v = LOOP_ERR_MISMATCH;
    }
    if (v) set_err(st, v, ch->id);
    verdict = v;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (verdict) return;
  const u64 off = s_off;
  copy_part(dst, ring + off % ch->cap, bytes);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this block's ring reads are done
  __syncthreads();
  if (threadIdx.x == 0 && last_block(&ch->r_ticket)) {
    st_agent_release(&ch->r_off, off + bytes);  // the ring space is free again
    st_agent_release(&ch->r_seq, seq + 1);
  }
}

int copy_blocks(u64 bytes) {
  const u64 b = (bytes + CHUNK - 1) / CHUNK;
  return (int)(b < 1 ? 1 : (b > MAX_BLOCKS ? MAX_BLOCKS : b));
}

}  // namespace

extern "C" hipError_t lsd_loop_send(LoopChan* ch, void* ring, const void* src, uint64_t bytes,
                                    LoopStatus* st, hipStream_t s) {
  hipLaunchKernelGGL(loop_send_kernel, dim3(copy_blocks(bytes)), dim3(THREADS), 0, s, ch,
                     static_cast<uint8_t*>(ring), static_cast<const uint8_t*>(src), bytes, st);
  return hipGetLastError();
}

extern "C" hipError_t lsd_loop_recv(LoopChan* ch, const void* ring, void* dst, uint64_t bytes,
                                    LoopStatus* st, hipStream_t s) {
  hipLaunchKernelGGL(loop_recv_kernel, dim3(copy_blocks(bytes)), dim3(THREADS), 0, s, ch,
                     static_cast<const uint8_t*>(ring), static_cast<uint8_t*>(dst), bytes, st);
  return hipGetLastError();
}

extern "C" uint64_t lsd_loop_place(uint64_t head, uint64_t bytes, uint64_t cap) {
  return place(head, bytes, cap);
}
