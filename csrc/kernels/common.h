// Common CDNA4 (gfx950 / MI355X) helpers for the engine kernels.
//
// Conventions used by every kernel in this directory:
//   * wave64: lane = threadIdx.x & 63, all cross-lane reductions span 64 lanes
//   * bf16 storage, fp32 math; 16-byte vector loads for every streamed tensor
//   * MFMA: v_mfma_f32_16x16x32_bf16.  Operand maps (lane l, r = l & 15, g = l >> 4):
//       A[row r][k = 8g + j]   B[k = 8g + j][col r]   (j = 0..7, one 16-byte fragment)
//       C/D: col = r, row = 4g + i (i = 0..3)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lsd {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int WAVE = 64;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }  // v_cvt_pk_bf16_f32, RNE, NaN-safe

// 16-byte loads/stores through an integer vector type (hipcc does not
// auto-vectorise bf16 scalar loads: guide Guideline 13).
__device__ __forceinline__ bf16x8 ld8(const bf16* p) {
  u32x4 v = *reinterpret_cast<const u32x4*>(p);
  return __builtin_bit_cast(bf16x8, v);
}
// Streaming (non-temporal) 16-byte load: data read once per step (KV cache)
// need not displace reusable lines (weights re-read by the next microbatch).
__device__ __forceinline__ bf16x8 ld8_nt(const bf16* p) {
  u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return __builtin_bit_cast(bf16x8, v);
}
__device__ __forceinline__ void st8(bf16* p, bf16x8 v) {
  *reinterpret_cast<u32x4*>(p) = __builtin_bit_cast(u32x4, v);
}
__device__ __forceinline__ bf16x4 ld4(const bf16* p) {
  u32x2 v = *reinterpret_cast<const u32x2*>(p);
  return __builtin_bit_cast(bf16x4, v);
}
__device__ __forceinline__ void st4(bf16* p, bf16x4 v) {
  *reinterpret_cast<u32x2*>(p) = __builtin_bit_cast(u32x2, v);
}

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <typename T>
__device__ __forceinline__ T shfl_xor(T v, int m) { return __shfl_xor(v, m, 64); }

// Partner exchange across lane bit log2(OFF) without the LDS crossbar
// (ds_bpermute costs an LDS round trip per step): DPP quad permutes for
// OFF = 1, 2; row half-mirror / mirror (lane i <-> 7-i / 15-i) for 4, 8;
// v_permlane16/32_swap for 16, 32.  Each is an involution that pairs lanes
// differing in that bit, which is all a butterfly reduction needs; the
// partner is lane ^ OFF except for OFF = 4, 8 (mirror order).
template <int OFF>
__device__ __forceinline__ float wave_xchg(float v) {
  const int x = __builtin_bit_cast(int, v);
  if constexpr (OFF == 1) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false));
  } else if constexpr (OFF == 2) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false));
  } else if constexpr (OFF == 4) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, x, 0x141, 0xF, 0xF, false));
  } else if constexpr (OFF == 8) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, x, 0x140, 0xF, 0xF, false));
  } else if constexpr (OFF == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
    return __builtin_bit_cast(float, (threadIdx.x & 16) ? (int)r[0] : (int)r[1]);
  } else {
    static_assert(OFF == 32, "offset must be a power of two <= 32");
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
    return __builtin_bit_cast(float, (threadIdx.x & 32) ? (int)r[0] : (int)r[1]);
  }
}

// wave_xchg with an offset that is a compile-time constant after unrolling
__device__ __forceinline__ float wave_xchg_n(float v, int off) {
  switch (off) {
    case 1: return wave_xchg<1>(v);
    case 2: return wave_xchg<2>(v);
    case 4: return wave_xchg<4>(v);
    case 8: return wave_xchg<8>(v);
    case 16: return wave_xchg<16>(v);
    default: return wave_xchg<32>(v);
  }
}

// Exact lane ^ off partner (values of non-equivalent lanes, e.g. merging
// per-dimension partials): mirrors replaced by ds_bpermute for 4 and 8.
__device__ __forceinline__ float wave_xor_n(float v, int off) {
  switch (off) {
    case 1: return wave_xchg<1>(v);
    case 2: return wave_xchg<2>(v);
    case 16: return wave_xchg<16>(v);
    case 32: return wave_xchg<32>(v);
    default: return shfl_xor(v, off);
  }
}

__device__ __forceinline__ float wave_sum(float v) {
  v += wave_xchg<1>(v);
  v += wave_xchg<2>(v);
  v += wave_xchg<4>(v);
  v += wave_xchg<8>(v);
  v += wave_xchg<16>(v);
  v += wave_xchg<32>(v);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, shfl_xor(v, m));
  return v;
}

// Mean / variance statistics (count, mean, M2 = sum of squared deviations),
// merged with Chan's pairwise formula in a form symmetric in its two operands
// (m = (na ma + nb mb) / n), so both lanes of a butterfly pair -- and every
// thread of a block -- end with bit-identical results.
struct Wf {
  float n, m, M;
};
__device__ __forceinline__ Wf wf_merge(Wf a, Wf b) {
  const float n = a.n + b.n;
  if (n == 0.f) return a;
  const float d = b.m - a.m, rn = 1.f / n;
  return {n, (a.n * a.m + b.n * b.m) * rn, a.M + b.M + d * d * (a.n * b.n) * rn};
}
template <int OFF>
__device__ __forceinline__ Wf wf_xchg(Wf v) {
  return {wave_xchg<OFF>(v.n), wave_xchg<OFF>(v.m), wave_xchg<OFF>(v.M)};
}
// Block-wide merge in ONE LDS round (red: >= 3 x waves floats)
__device__ __forceinline__ Wf block_welford(Wf v, float* red) {
  v = wf_merge(v, wf_xchg<1>(v));
  v = wf_merge(v, wf_xchg<2>(v));
  v = wf_merge(v, wf_xchg<4>(v));
  v = wf_merge(v, wf_xchg<8>(v));
  v = wf_merge(v, wf_xchg<16>(v));
  v = wf_merge(v, wf_xchg<32>(v));
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane_id() == 0) {
    red[3 * w] = v.n;
    red[3 * w + 1] = v.m;
    red[3 * w + 2] = v.M;
  }
  __syncthreads();
  Wf t = {red[0], red[1], red[2]};
  for (int i = 1; i < nw; ++i) t = wf_merge(t, Wf{red[3 * i], red[3 * i + 1], red[3 * i + 2]});
  return t;
}

// Block-wide sum for blockDim.x = nwaves*64 (<= 1024); `red` holds >= 16 floats.
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane_id() == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

// gelu_new (tanh approximation) -- [tf5.15] activations.py:59-66
//   0.5 x (1 + tanh(u)) = x * sigmoid(2u) = x / (1 + exp(-2u)),
//   u = sqrt(2/pi) (x + 0.044715 x^3)
// Six VALU ops, two of them transcendental (v_exp_f32, v_rcp_f32, ~1 ulp
// each), no IEEE division and no cancellation; saturates to x / -0 at +-inf
// without NaNs.  The prefill FC epilogue evaluates it 420M times per GEMM on
// GPT-2 XL, where the libm/division form cost ~a quarter of the kernel.
__device__ __forceinline__ float gelu_new(float x) {
  constexpr float k = -2.f * 0.7978845608028654f * 1.4426950408889634f;  // -2 sqrt(2/pi) log2(e)
  const float y = x * fmaf(k * 0.044715f, x * x, k);                      // -2u log2(e)
  return x * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(y));
}
__device__ __forceinline__ float silu(float x) {
  return x * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-1.4426950408889634f * x));
}

// Bijective XCD-aware remap of a 1-D workgroup id (guide §5.5 T1, "XCD
// swizzle must be bijective"): consecutive logical tiles land on one XCD so
// tiles sharing an operand panel share that XCD's L2.  Speed only.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int nx = 8;
  if (nwg < nx) return bid;
  const int q = nwg / nx, r = nwg % nx, x = bid % nx;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / nx;
}

}  // namespace lsd
