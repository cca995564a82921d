// On-device sampler: greedy argmax or temperature + top-k + multinomial.
//
// K14/K15 of SURVEY.md §2.5.  The reference ships [1, S, 50257] fp32 logits
// to the coordinator as JSON and samples on the host (`server.py:151,183-206`:
// logits[0,-1] / 0.6 -> topk(40) -> softmax -> multinomial).  Here only the
// sampled id (int32) leaves the last stage.
//
// Per row (one 1024-thread block):
//   greedy: block argmax (lowest index on ties).
//   top-k : 4-pass 8-bit radix select over order-preserving uint32 keys finds
//           the k-th largest logit; the k winners are collected, sorted by
//           (value desc, index asc) with a bitonic sort in LDS (deterministic
//           order regardless of atomic arrival), softmax over value/T, and an
//           inverse-CDF draw with u = splitmix64(seed * FNV + step) -- the same
//           counter-based generator as runtime/batch.py:counter_uniform, so a
//           seeded request reproduces across batch layouts and stage counts.
#include "common.h"

namespace lsd {

constexpr int SMAX = 1024;  // max top_k supported on device (host validates)

__device__ __forceinline__ unsigned fkey(float x) {
  unsigned u = __float_as_uint(x);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ float counter_uniform(long long seed, long long step) {
  const unsigned long long z =
      mix64((unsigned long long)seed * 0x100000001B3ull + (unsigned long long)step);
  return (float)((double)(z >> 40) / 16777216.0);
}

__global__ __launch_bounds__(1024) void sample_kernel(const float* __restrict__ logits, long ld,
                                                      int V, const float* __restrict__ temp,
                                                      const int* __restrict__ topk,
                                                      const int* __restrict__ greedy,
                                                      const long long* __restrict__ seeds,
                                                      const long long* __restrict__ step,
                                                      int* __restrict__ out) {
  __shared__ unsigned hist[256];
  __shared__ float cval[2 * SMAX];
  __shared__ int cidx[2 * SMAX];
  __shared__ float redv[16];
  __shared__ int redi[16];
  __shared__ unsigned s_prefix, s_need, s_ngt, s_neq;
  const int row = blockIdx.x, tid = threadIdx.x;
  const float* x = logits + (long)row * ld;

  if (greedy[row]) {
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for (int i = tid; i < V; i += blockDim.x) {
      const float v = x[i];
      if (v > best || (v == best && i < bi)) { best = v; bi = i; }
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      const float ov = shfl_xor(best, m);
      const int oi = shfl_xor(bi, m);
      if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
    }
    if (lane_id() == 0) { redv[tid >> 6] = best; redi[tid >> 6] = bi; }
    __syncthreads();
    if (tid == 0) {
      for (int w = 1; w < (int)(blockDim.x >> 6); ++w)
        if (redv[w] > best || (redv[w] == best && redi[w] < bi)) { best = redv[w]; bi = redi[w]; }
      out[row] = bi;
    }
    return;
  }

  const int k = min(max(topk[row], 1), min(SMAX, V));
  // ---- radix select: the k-th largest key
  unsigned prefix = 0, mask = 0, need = k;
  for (int pass = 0; pass < 4; ++pass) {
    const int shift = 24 - 8 * pass;
    for (int i = tid; i < 256; i += blockDim.x) hist[i] = 0;
    __syncthreads();
    for (int i = tid; i < V; i += blockDim.x) {
      const unsigned kk = fkey(x[i]);
      if ((kk & mask) == prefix) atomicAdd(&hist[(kk >> shift) & 255u], 1u);
    }
    __syncthreads();
    if (tid == 0) {
      unsigned cum = 0;
      int d = 255;
      for (; d >= 0; --d) {
        if (cum + hist[d] >= need) break;
        cum += hist[d];
      }
      s_prefix = prefix | ((unsigned)d << shift);
      s_need = need - cum;
    }
    __syncthreads();
    prefix = s_prefix;
    need = s_need;
    mask |= 255u << shift;
    __syncthreads();
  }
  // keys > prefix: k - need of them; keys == prefix: take the `need` lowest indices
  if (tid == 0) { s_ngt = 0; s_neq = 0; }
  __syncthreads();
  const unsigned n_gt = k - need;
  for (int i = tid; i < V; i += blockDim.x) {
    const unsigned kk = fkey(x[i]);
    if (kk > prefix) {
      const unsigned slot = atomicAdd(&s_ngt, 1u);
      cval[slot] = x[i];
      cidx[slot] = i;
    } else if (kk == prefix) {
      const unsigned slot = atomicAdd(&s_neq, 1u);
      if (slot < (unsigned)SMAX) { cval[SMAX + slot] = x[i]; cidx[SMAX + slot] = i; }
    }
  }
  __syncthreads();
  // equal keys: keep the `need` smallest indices (selection by thread 0; ties are rare)
  if (tid == 0) {
    const unsigned neq = min(s_neq, (unsigned)SMAX);
    for (unsigned a = 0; a < need; ++a) {
      unsigned best = a;
      for (unsigned b2 = a + 1; b2 < neq; ++b2)
        if (cidx[SMAX + b2] < cidx[SMAX + best]) best = b2;
      const int ti = cidx[SMAX + a]; cidx[SMAX + a] = cidx[SMAX + best]; cidx[SMAX + best] = ti;
      const float tv = cval[SMAX + a]; cval[SMAX + a] = cval[SMAX + best]; cval[SMAX + best] = tv;
      cval[n_gt + a] = cval[SMAX + a];
      cidx[n_gt + a] = cidx[SMAX + a];
    }
  }
  __syncthreads();
  // ---- bitonic sort of the k winners: (value desc, index asc); pad to pow2
  int n2 = 1;
  while (n2 < k) n2 <<= 1;
  for (int i = k + tid; i < n2; i += blockDim.x) { cval[i] = -INFINITY; cidx[i] = 0x7fffffff; }
  __syncthreads();
  for (int size = 2; size <= n2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < n2; i += blockDim.x) {
        const int j = i ^ stride;
        if (j > i) {
          const bool up = (i & size) == 0;  // "up" = descending by our order
          const float vi = cval[i], vj = cval[j];
          const int ii = cidx[i], ij = cidx[j];
          const bool i_first = (vi > vj) || (vi == vj && ii < ij);
          if (up != i_first) {
            cval[i] = vj; cval[j] = vi; cidx[i] = ij; cidx[j] = ii;
          }
        }
      }
      __syncthreads();
    }
  }
  // ---- softmax over value/T and inverse-CDF draw
  if (tid == 0) {
    const float T = temp[row];
    const float x0 = cval[0] / T;
    float tot = 0.f;
    for (int i = 0; i < k; ++i) {
      tot += __expf(cval[i] / T - x0);
      cval[SMAX + i] = tot;  // running (unnormalised) CDF
    }
    const float u = counter_uniform(seeds[row], step[row]) * tot;
    int j = 0;
    while (j < k - 1 && cval[SMAX + j] < u) ++j;
    out[row] = cidx[j];
  }
}

}  // namespace lsd

using namespace lsd;

extern "C" hipError_t lsd_sample(const float* logits, long ld, int B, int V, const float* temp,
                                 const int* topk, const int* greedy, const long long* seeds,
                                 const long long* step, int* out, hipStream_t st) {
  if (B == 0) return hipSuccess;
  hipLaunchKernelGGL(sample_kernel, dim3(B), dim3(1024), 0, st, logits, ld, V, temp, topk, greedy,
                     seeds, step, out);
  return hipGetLastError();
}
