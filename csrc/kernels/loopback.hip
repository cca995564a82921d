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
// Up to 128 KiB one block does the whole op (drain + agent-scope release
// before the tag); above that a 1-block wait, a many-block copy and a 1-block
// publish / release kernel run in stream order, so kernel boundaries order
// the payload before its publish and the reads before the release.  Every
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

// No copy kernel ever spins: a wait runs in ONE block (of its own launch for
// large messages), so however many ops are waiting, they hold a handful of
// waves -- never the CUs the kernels they wait for need.  (The first version
// let every block of a 256-block copy spin for ring space; eight stage
// threads' prefill sends filled the chip with spinning waves and the
// receives that would free the space could not start: a device-wait timeout
// in the 8-stage rehearsal, profiles/r4_rehearsal_graph_io.log.)
//
// `ring` is this process's address of the channel's ring (an IPC mapping when
// the peer process owns it): pointers never travel through the shared state.

__device__ __forceinline__ bool send_space(const LoopChan* ch, u64 seq, u64 off, u64 bytes) {
  // header slot free and [r_off, off + bytes) within one ring
  return seq - ld_agent(&ch->r_seq) < LOOP_HEADERS && off + bytes - ld_agent(&ch->r_off) <= ch->cap;
}

// publish message `seq` at `off` (after the payload is visible device-wide)
__device__ __forceinline__ void publish(LoopChan* ch, u64 seq, u64 off, u64 bytes) {
  const u32 k = (u32)(seq % LOOP_HEADERS);
  __hip_atomic_store(&ch->h_size[k], bytes, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(&ch->h_off[k], off, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  st_agent_release(&ch->h_tag[k], seq + 1);
  ch->s_seq = seq + 1;
  ch->s_off = off + bytes;
}

// wait for message `seq`; 0 and its ring offset in *off, or an error code
__device__ __forceinline__ u32 recv_head(const LoopChan* ch, u64 seq, u64 bytes, const LoopStatus* st, u64* off) {
  const u32 k = (u32)(seq % LOOP_HEADERS);
  u32 v = bounded_wait([&] { return ld_agent(&ch->h_tag[k]) == seq + 1; }, st, ch->spin_limit);
  if (v) return v;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  *off = ld_agent(&ch->h_off[k]);
  return ld_agent(&ch->h_size[k]) == bytes ? 0u : (u32)LOOP_ERR_MISMATCH;
}

__device__ __forceinline__ void release_recv(LoopChan* ch, u64 seq, u64 off, u64 bytes) {
  st_agent_release(&ch->r_off, off + bytes);
  st_agent_release(&ch->r_seq, seq + 1);
}

// --- small messages: one block does wait + copy + publish / release --------
__global__ __launch_bounds__(THREADS) void loop_send_small(LoopChan* ch, uint8_t* ring, const uint8_t* src,
                                                           u64 bytes, LoopStatus* st) {
  __shared__ u32 verdict;
  const u64 cap = ch->cap, seq = ch->s_seq;  // sender-private: stream-ordered
  const u64 off = place(ch->s_off, bytes, cap);
  if (threadIdx.x == 0) {
    u32 v = bounded_wait([&] { return send_space(ch, seq, off, bytes); }, st, ch->spin_limit);
    if (v) set_err(st, v, ch->id);
    verdict = v;
  }
  __syncthreads();
  if (verdict) return;
  copy_part(ring + off % cap, src, bytes);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
  __syncthreads();
  if (threadIdx.x == 0 && seq < ch->stall_from) {    // stall_from: fault injection
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    publish(ch, seq, off, bytes);
  }
}

__global__ __launch_bounds__(THREADS) void loop_recv_small(LoopChan* ch, const uint8_t* ring, uint8_t* dst,
                                                           u64 bytes, LoopStatus* st) {
  __shared__ u32 verdict;
  __shared__ u64 s_off;
  const u64 seq = ch->r_seq;  // receiver-private: stream-ordered
  if (threadIdx.x == 0) {
    u64 off = 0;
    const u32 v = recv_head(ch, seq, bytes, st, &off);
    if (v) set_err(st, v, ch->id);
    verdict = v;
    s_off = off;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (verdict) return;
  copy_part(dst, ring + s_off % ch->cap, bytes);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the ring reads are done
  __syncthreads();
  if (threadIdx.x == 0) release_recv(ch, seq, s_off, bytes);
}

// --- large messages: wait (1 block) / copy (many blocks) / finish (1 block) --
__global__ void loop_send_wait(LoopChan* ch, u64 bytes, LoopStatus* st) {
  if (threadIdx.x != 0) return;
  const u64 seq = ch->s_seq, off = place(ch->s_off, bytes, ch->cap);
  const u32 v = bounded_wait([&] { return send_space(ch, seq, off, bytes); }, st, ch->spin_limit);
  if (v) set_err(st, v, ch->id);
  ch->s_verdict = v;
}

__global__ __launch_bounds__(THREADS) void loop_send_copy(const LoopChan* ch, uint8_t* ring, const uint8_t* src,
                                                          u64 bytes) {
  if (ch->s_verdict) return;
  copy_part(ring + place(ch->s_off, bytes, ch->cap) % ch->cap, src, bytes);
}

__global__ void loop_send_publish(LoopChan* ch, u64 bytes) {
  if (threadIdx.x != 0 || ch->s_verdict) return;
  const u64 seq = ch->s_seq;
  if (seq >= ch->stall_from) return;  // fault injection: the peer waits on the device
  // the payload (previous kernel) is visible: kernel boundary
  publish(ch, seq, place(ch->s_off, bytes, ch->cap), bytes);
}

__global__ void loop_recv_wait(LoopChan* ch, u64 bytes, LoopStatus* st) {
  if (threadIdx.x != 0) return;
  u64 off = 0;
  const u32 v = recv_head(ch, ch->r_seq, bytes, st, &off);
  if (v) set_err(st, v, ch->id);
  ch->r_verdict = v;
  ch->r_cur = off;
}

__global__ __launch_bounds__(THREADS) void loop_recv_copy(const LoopChan* ch, const uint8_t* ring, uint8_t* dst,
                                                          u64 bytes) {
  if (ch->r_verdict) return;
  copy_part(dst, ring + ch->r_cur % ch->cap, bytes);
}

__global__ void loop_recv_release(LoopChan* ch, u64 bytes) {
  if (threadIdx.x != 0 || ch->r_verdict) return;
  // the copy kernel's reads of the ring completed before this kernel began
  release_recv(ch, ch->r_seq, ch->r_cur, bytes);
}

constexpr u64 SMALL = 128 << 10;  // one-block ops up to this many bytes

int copy_blocks(u64 bytes) {
  const u64 b = (bytes + CHUNK - 1) / CHUNK;
  return (int)(b < 1 ? 1 : (b > 256 ? 256 : b));
}

}  // namespace

extern "C" hipError_t lsd_loop_send(LoopChan* ch, void* ring, const void* src, uint64_t bytes,
                                    LoopStatus* st, hipStream_t s) {
  auto* r = static_cast<uint8_t*>(ring);
  auto* p = static_cast<const uint8_t*>(src);
  if (bytes <= SMALL) {
    hipLaunchKernelGGL(loop_send_small, dim3(1), dim3(THREADS), 0, s, ch, r, p, bytes, st);
  } else {
    hipLaunchKernelGGL(loop_send_wait, dim3(1), dim3(64), 0, s, ch, bytes, st);
    hipLaunchKernelGGL(loop_send_copy, dim3(copy_blocks(bytes)), dim3(THREADS), 0, s, ch, r, p, bytes);
    hipLaunchKernelGGL(loop_send_publish, dim3(1), dim3(64), 0, s, ch, bytes);
  }
  return hipGetLastError();
}

extern "C" hipError_t lsd_loop_recv(LoopChan* ch, const void* ring, void* dst, uint64_t bytes,
                                    LoopStatus* st, hipStream_t s) {
  auto* r = static_cast<const uint8_t*>(ring);
  auto* p = static_cast<uint8_t*>(dst);
  if (bytes <= SMALL) {
    hipLaunchKernelGGL(loop_recv_small, dim3(1), dim3(THREADS), 0, s, ch, r, p, bytes, st);
  } else {
    hipLaunchKernelGGL(loop_recv_wait, dim3(1), dim3(64), 0, s, ch, bytes, st);
    hipLaunchKernelGGL(loop_recv_copy, dim3(copy_blocks(bytes)), dim3(THREADS), 0, s, ch, r, p, bytes);
    hipLaunchKernelGGL(loop_recv_release, dim3(1), dim3(64), 0, s, ch, bytes);
  }
  return hipGetLastError();
}

extern "C" uint64_t lsd_loop_place(uint64_t head, uint64_t bytes, uint64_t cap) {
  return place(head, bytes, cap);
}
