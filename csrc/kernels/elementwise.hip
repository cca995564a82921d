// SiLU(gate) * up over a gate/up-interleaved GEMM output (Llama MLP).
//
// The gate_up weight is stored in 32-row blocks [gate 16 | up 16]
// (ops/hip.py interleave_gate_up), so the fused GEMM epilogue (gemm.hip
// EPI_SILU_MUL) pairs each gate column with the up column 16 to its right.
// When the GEMM itself runs elsewhere (the hipBLASLt A/B oracle, LSD_ROUTING
// blaslt=1: 64-128 decode rows, csrc/blaslt.cpp) its bf16 output [M, 2F]
// goes through this pass: one thread
// per 8 outputs, 16-byte loads of the gate and up chunks, fp32 math, one
// 16-byte store -- out[m, 16 j + i] = silu(y[m, 32 j + i]) * y[m, 32 j + 16 + i].
#include "common.h"

namespace lsd {

__global__ __launch_bounds__(256) void silu_mul_kernel(const bf16* __restrict__ y, long ldy,
                                                       bf16* __restrict__ out, long ldo, int M, int F) {
  const long per_row = F / 8;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)M * per_row) return;
  const int m = (int)(idx / per_row);
  const int o = (int)(idx % per_row) * 8;  // first of 8 outputs
  const int j = o >> 4, i = o & 15;
  const bf16* row = y + (long)m * ldy + (long)j * 32 + i;
  const bf16x8 g = ld8(row), u = ld8(row + 16);
  bf16x8 r;
#pragma unroll
  for (int e = 0; e < 8; ++e) r[e] = f2bf(silu(bf2f(g[e])) * bf2f(u[e]));
  st8(out + (long)m * ldo + o, r);
}

// QKV epilogue over an fp32 GEMM output (hipBLASLt, csrc/blaslt.cpp) -- the
// same math as gemm.hip EPI_QKV: y = acc + bias; RoPE on adjacent (even, odd)
// column pairs of q and k (weights pre-permuted, ops/hip.py
// rope_pair_permutation) with the (cos, sin) of the token's position; q ->
// out bf16 [M, q_size]; k / v -> the caches at [slot][kv head][pos][d].  One
// thread per 8 columns: two 16-byte fp32 loads, one 16-byte bf16 store (8
// columns never straddle a head: hd % 8 == 0).
__global__ __launch_bounds__(256) void qkv_post_kernel(const float* __restrict__ y, long ldy,
                                                       const bf16* __restrict__ bias, const int* __restrict__ tslot,
                                                       const int* __restrict__ tpos, const float* __restrict__ rope,
                                                       bf16* __restrict__ q, bf16* __restrict__ kc,
                                                       bf16* __restrict__ vc, int M, int q_size, int kv_size, int hd,
                                                       int n_kv, int max_seq) {
  const int N = q_size + 2 * kv_size, per_row = N / 8;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)M * per_row) return;
  const int m = (int)(idx / per_row);
  const int n = (int)(idx % per_row) * 8;
  const f32x4* src = reinterpret_cast<const f32x4*>(y + (long)m * ldy + n);
  const f32x4 a = src[0], b = src[1];
  float v[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  if (bias) {
    const bf16x8 bb = ld8(bias + n);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += bf2f(bb[j]);
  }
  const int qk = q_size + kv_size;
  const int pos = tpos[m];
  if (rope != nullptr && n < qk) {
    const int d0 = (n < q_size ? n : n - q_size) % hd;
    const f32x4* cs = reinterpret_cast<const f32x4*>(rope + ((long)pos * (hd >> 1) + (d0 >> 1)) * 2);
    const f32x4 c0 = cs[0], c1 = cs[1];  // (cos, sin) of pairs d0/2 .. d0/2 + 3
    const float cc[4] = {c0[0], c0[2], c1[0], c1[2]}, ss[4] = {c0[1], c0[3], c1[1], c1[3]};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float e = v[2 * k], o = v[2 * k + 1];
      v[2 * k] = e * cc[k] - o * ss[k];
      v[2 * k + 1] = o * cc[k] + e * ss[k];
    }
  }
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = f2bf(v[j]);
  if (n < q_size) {
    st8(q + (long)m * q_size + n, r);
  } else {
    const int c = n < qk ? n - q_size : n - qk;
    bf16* cache = n < qk ? kc : vc;
    st8(cache + (((long)tslot[m] * n_kv + c / hd) * max_seq + pos) * hd + c % hd, r);
  }
}

}  // namespace lsd

using namespace lsd;

extern "C" hipError_t lsd_silu_mul(const bf16* y, long ldy, bf16* out, long ldo, int M, int F,
                                   hipStream_t st) {
  if (M == 0) return hipSuccess;
  if (F % 16 != 0) return hipErrorInvalidValue;
  const long n = (long)M * (F / 8);
  hipLaunchKernelGGL(silu_mul_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, y, ldy, out, ldo, M, F);
  return hipGetLastError();
}

extern "C" hipError_t lsd_qkv_post(const float* y, long ldy, const bf16* bias, const int* tslot, const int* tpos,
                                   const float* rope, bf16* q, bf16* kc, bf16* vc, int M, int q_size, int kv_size,
                                   int hd, int n_kv, int max_seq, hipStream_t st) {
  if (M == 0) return hipSuccess;
  if (hd % 8 != 0 || q_size % hd != 0 || kv_size % hd != 0) return hipErrorInvalidValue;
  const long n = (long)M * ((q_size + 2 * kv_size) / 8);
  hipLaunchKernelGGL(qkv_post_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, y, ldy, bias, tslot, tpos,
                     rope, q, kc, vc, M, q_size, kv_size, hd, n_kv, max_seq);
  return hipGetLastError();
}

namespace lsd {

// Composition change of a decode group (runtime/plan.py Row; the host side is
// parallel/pipeline.py _apply_rows): the new rows' state arrives as ONE packed
// int32 buffer (one host-to-device copy) laid out by the group capacity `cap`
//   [0, 2 cap)      int64 sampler seeds        [2 cap, 4 cap)  int64 sampler steps
//   [4 cap]         n (live rows)              then, from f = 4 cap + 1:
//   f[0, cap) KV slots  f[cap, 2 cap) positions  f[2 cap, 3 cap) temperatures (fp32 bits)
//   f[3 cap, 4 cap) top-k  f[4 cap, 5 cap) greedy  f[5 cap, 6 cap) stage 0's gather index
// and this kernel scatters it into the group's row-state vectors: rows [0, n)
// live, pad rows [n, b) idle on the scratch slot (position 0, inactive,
// temperature 1, top-k 1, greedy, seed 0, step 0, gather index 0).  Stage 0
// also gathers the rows' input tokens out of the previous token-return vector
// in place (tin[i] = tin[src[i]], staged through LDS: a source may be a row
// this same launch overwrites).  One workgroup: b <= 16384 (64 KB of LDS).
// Replaces ~10 copy / index_select launches per changed item and lets the
// native executor (csrc/stage_exec.cpp) issue composition-change items.
__global__ __launch_bounds__(1024) void apply_rows_kernel(const int* __restrict__ buf, int b, int cap, int scratch,
                                                          int* __restrict__ slots, int* __restrict__ pos,
                                                          int* __restrict__ act, float* __restrict__ temp,
                                                          int* __restrict__ topk, int* __restrict__ greedy,
                                                          long long* __restrict__ seeds, long long* __restrict__ sstep,
                                                          int* tin) {
  extern __shared__ int gath[];
  const int n = buf[4 * cap];
  const int* f = buf + 4 * cap + 1;
  const long long* s64 = reinterpret_cast<const long long*>(buf);
  for (int i = threadIdx.x; i < b; i += blockDim.x) {
    const bool live = i < n;
    slots[i] = live ? f[i] : scratch;
    pos[i] = live ? f[cap + i] : 0;
    act[i] = live ? 1 : 0;
    if (temp != nullptr) {
      temp[i] = live ? __int_as_float(f[2 * cap + i]) : 1.0f;
      topk[i] = live ? f[3 * cap + i] : 1;
      greedy[i] = live ? f[4 * cap + i] : 1;
      seeds[i] = live ? s64[i] : 0;
      sstep[i] = live ? s64[cap + i] : 0;
    }
    if (tin != nullptr) gath[i] = tin[live ? f[5 * cap + i] : 0];
  }
  if (tin == nullptr) return;  // uniform across the workgroup
  __syncthreads();
  for (int i = threadIdx.x; i < b; i += blockDim.x) tin[i] = gath[i];
}

}  // namespace lsd

// args: the host int64 record [cap, scratch, buf, slots, pos, act, temp, topk,
// greedy, seeds, sstep, tin] (device pointers; 0 = the field is absent on this
// stage) -- the native executor passes the same record it got from Python.
extern "C" hipError_t lsd_apply_rows(const int64_t* args, int b, hipStream_t st) {
  if (b <= 0) return hipSuccess;
  const int cap = (int)args[0];
  if (b > cap || b > 16384 || args[2] == 0 || args[3] == 0 || args[4] == 0 || args[5] == 0) return hipErrorInvalidValue;
  if (args[6] != 0 && (args[7] == 0 || args[8] == 0 || args[9] == 0 || args[10] == 0)) return hipErrorInvalidValue;
  const unsigned threads = b >= 1024 ? 1024u : (unsigned)((b + 63) / 64 * 64);
  const size_t lds = args[11] != 0 ? (size_t)b * sizeof(int) : 0;
  auto P = [&](int k) { return reinterpret_cast<void*>(args[k]); };
  hipLaunchKernelGGL(lsd::apply_rows_kernel, dim3(1), dim3(threads), lds, st, static_cast<const int*>(P(2)), b, cap,
                     (int)args[1], static_cast<int*>(P(3)), static_cast<int*>(P(4)), static_cast<int*>(P(5)),
                     static_cast<float*>(P(6)), static_cast<int*>(P(7)), static_cast<int*>(P(8)),
                     static_cast<long long*>(P(9)), static_cast<long long*>(P(10)), static_cast<int*>(P(11)));
  return hipGetLastError();
}
