// Single-stream decode: one persistent launch per layer chain vs one launch per
// GEMV (verdict r3 "Next round" item 6: "one kernel per layer at batch <= 8,
// with grid-wide barriers between the phases ... or a profiles/ log shows the
// persistent kernel losing, with per-phase stamps").
//
// The batch-1 decode layer of GPT-2 (the reference's
// block loop `/root/reference/server.py:84-85,99-100`) is five dependent
// launches in production: QKV (+LN1, +KV append), attention, out-projection
// (+residual), FC (+LN2, +GELU), projection (+residual).  Every GEMV pays a
// fixed ~3 us (ramp, first weight load, reduction, drain:
// profiles/r2_single_stream_analysis.log).  Here the four GEMVs of a layer run
// as the SAME phase bodies three ways, captured in one hipGraph over 48 layers:
//   A  launches    -- out-proj, FC, proj, QKV, attention: 5 launches per layer
//   B  persistent  -- out-proj | FC | proj | QKV in ONE launch (256 workgroups,
//                     one per CU) with a grid barrier between phases, the next
//                     phase's weights issued into registers BEFORE each barrier
//                     (they do not depend on it), + the attention launch:
//                     2 launches per layer
//   C  persistent, weights issued after each barrier (no prefetch)
// The attention is a stand-in copy kernel (its real cost, ~5.7 us, is the
// same in all three and is added back in the report).
//
// Phase body (one wave per output row, R rows per wave, the full K per wave,
// as lsd::gemv_kernel): weights straight to VGPRs (16-B nt loads), the input
// vector (LayerNorm'd where the phase has a norm) as a zero-padded bf16 image
// in LDS, v_dot2c_f32_bf16, a wave butterfly, lane 0 stores the epilogue.
//
// Grid barrier (MI355X_MICROARCH "Valid forms", hand-off table row 1): every
// storing wave drains its stores (`s_waitcnt vmcnt(n)` leaves only the
// prefetched weight loads outstanding: the counter is in order), a workgroup
// barrier, ONE lane adds to its shard of an 8-way sharded agent-scope counter;
// 8 lanes of wave 0 poll all 8 shards with `sc1` loads until each reached its
// generation target; every activation the phases hand over is stored `sc1`
// (4 or 16 B) and read `sc1` -- no fences.  Every spin is bounded (100 ms on
// the 100 MHz constant clock) and sets an error flag instead of hanging.
//
// Correctness: A, B and C compute the same rows on the same waves in the same
// order, so their final residual stream and QKV outputs must be bit-identical
// (a stale hand-off shows up as a mismatch); the host checks every word.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../kernels/common.h"

using namespace lsd;

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__);     \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

constexpr int NT = 256;   // threads per workgroup (4 waves)
constexpr int G = 256;    // workgroups: one per CU
constexpr int NWV = G * 4;
constexpr int NSTAMP = 9;  // per workgroup per layer (mode B/C)

enum Kind : int { OPROJ = 0, FC = 1, PROJ2 = 2, QKV = 3 };

struct LayerW {
  const bf16 *wo, *bo, *wfc, *bfc, *wp2, *bp2, *wq, *bq, *g1, *b1, *g2, *b2;
};

struct Bufs {
  float* x;        // residual stream [H] fp32
  float* h;        // MLP hidden [FF] fp32
  bf16* qkv;       // [3H] bf16 (consumed by the next launch)
  bf16* o;         // attention output [H] bf16 (written by the previous launch)
  unsigned* bar;   // 8 shards x 32 words
  int* err;
  unsigned long long* stamps;  // [layers][G][NSTAMP]
};

template <int H, int FF>
struct Dims {
  static constexpr int NBH = (H / 8 + 63) / 64;   // 16-B chunks per lane per row, K = H
  static constexpr int NBF = (FF / 8 + 63) / 64;  // K = FF
  static constexpr int RO = (H + NWV - 1) / NWV;  // rows per wave
  static constexpr int RF = (FF + NWV - 1) / NWV;
  static constexpr int RQ = (3 * H + NWV - 1) / NWV;
  static constexpr int KSH = NBH * 512;  // LDS image lengths (bf16), zero past K
  static constexpr int KSF = NBF * 512;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, bytes, 0x00020000);
}
// 16-B / 4-B loads and stores with the sc1 bit (aux 16): L1 bypassed, stores written through
__device__ __forceinline__ f32x4 ld_sc1_x4(__amdgpu_buffer_rsrc_t r, int off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16));
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ float dot8(bf16x8 a, bf16x8 b, float acc) {
#define LSD_PR(v, j) __builtin_shufflevector(v, v, 2 * (j), 2 * (j) + 1)
  acc = __builtin_amdgcn_fdot2_f32_bf16(LSD_PR(a, 0), LSD_PR(b, 0), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(LSD_PR(a, 1), LSD_PR(b, 1), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(LSD_PR(a, 2), LSD_PR(b, 2), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(LSD_PR(a, 3), LSD_PR(b, 3), acc, false);
#undef LSD_PR
  return acc;
}

__device__ __forceinline__ void stamp(const Bufs& b, int layer, int k) {
  if (b.stamps && threadIdx.x == 0)
    b.stamps[((long)layer * G + blockIdx.x) * NSTAMP + k] = __builtin_amdgcn_s_memrealtime();
}

// ---- weights of R rows x NB chunks per lane, straight to VGPRs
template <int R, int NB>
struct WRegs {
  bf16x8 v[R][NB];
  float bias[R];
};

template <int R, int NB>
__device__ __forceinline__ void issue_w(WRegs<R, NB>& w, const bf16* W, const bf16* bias, int N, int K) {
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6), lane = lane_id();
  const int KC = K >> 3;
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const bf16* wr = W + (long)min(gw + j * NWV, N - 1) * K;
#pragma unroll
    for (int i = 0; i < NB; ++i) w.v[j][i] = ld8_nt(wr + min(lane + 64 * i, KC - 1) * 8);
  }
#pragma unroll
  for (int j = 0; j < R; ++j) w.bias[j] = bf2f(bias[min(gw + j * NWV, N - 1)]);
}

// ---- dot products against the LDS image, wave-reduced (every lane holds the sums)
template <int R, int NB>
__device__ __forceinline__ void dots(const WRegs<R, NB>& w, const bf16* xs, float (&acc)[R]) {
  const int lane = lane_id();
#pragma unroll
  for (int j = 0; j < R; ++j) acc[j] = 0.f;
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const bf16x8 xv = *reinterpret_cast<const bf16x8*>(xs + (lane + 64 * i) * 8);
#pragma unroll
    for (int j = 0; j < R; ++j) acc[j] = dot8(w.v[j][i], xv, acc[j]);
  }
#pragma unroll
  for (int j = 0; j < R; ++j) acc[j] = wave_sum(acc[j]);
}

// ---- inputs -> bf16 LDS image
// LayerNorm of the fp32 residual (sc1 loads: written by other workgroups this launch)
template <int H>
__device__ __forceinline__ void input_ln(const float* x, const bf16* g, const bf16* bta, bf16* xs, float* red) {
  constexpr int NV = (H / 4 + NT - 1) / NT;
  const __amdgpu_buffer_rsrc_t r = rsrc(x, H * 4);
  f32x4 v[NV];
  float s = 0.f, cnt = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (threadIdx.x + NT * i) * 4;
    v[i] = c < H ? ld_sc1_x4(r, c * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int i = 0; i < NV; ++i)
    if ((threadIdx.x + NT * i) * 4 < H) {
      s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
      cnt += 4.f;
    }
  const float mt = cnt > 0.f ? s / cnt : 0.f;
  float m2 = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
    if ((threadIdx.x + NT * i) * 4 < H) {
      const f32x4 d = v[i] - mt;
      m2 += d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3];
    }
  const Wf st = block_welford(Wf{cnt, mt, m2}, red);
  const float rstd = rsqrtf(st.M / H + 1e-5f);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (threadIdx.x + NT * i) * 4;
    if (c < H) {
      const bf16x4 gg = ld4(g + c), bb = ld4(bta + c);
      bf16x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = f2bf((v[i][e] - st.m) * rstd * bf2f(gg[e]) + bf2f(bb[e]));
      st4(xs + c, o);
    }
  }
}

// fp32 vector (sc1) -> bf16 image
template <int K>
__device__ __forceinline__ void input_f32(const float* h, bf16* xs) {
  constexpr int NV = (K / 4 + NT - 1) / NT;
  const __amdgpu_buffer_rsrc_t r = rsrc(h, K * 4);
  f32x4 v[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (threadIdx.x + NT * i) * 4;
    v[i] = c < K ? ld_sc1_x4(r, c * 4) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (threadIdx.x + NT * i) * 4;
    if (c < K) st4(xs + c, bf16x4{f2bf(v[i][0]), f2bf(v[i][1]), f2bf(v[i][2]), f2bf(v[i][3])});
  }
}

// bf16 vector from the previous launch (plain loads) -> image
template <int K>
__device__ __forceinline__ void input_bf16(const bf16* o, bf16* xs) {
  for (int c = threadIdx.x * 8; c < K; c += NT * 8) st8(xs + c, ld8(o + c));
}

template <int KS, int K>
__device__ __forceinline__ void zero_pad(bf16* xs) {
  for (int c = K + threadIdx.x; c < KS; c += NT) xs[c] = f2bf(0.f);
}

// ---- grid barrier: sharded counter, every shard polled (see header)
template <int OUTSTANDING>
__device__ __forceinline__ void grid_sync(const Bufs& b, unsigned gen) {
  // this wave's epilogue stores drained; only the OUTSTANDING prefetched
  // weight loads issued after them may still be in flight (in-order counter)
  if constexpr (OUTSTANDING == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    __builtin_amdgcn_s_waitcnt((OUTSTANDING & 0xF) | ((OUTSTANDING >> 4) << 14) | (0x7 << 4) | (0xF << 8));
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    if (lane == 0)
      __hip_atomic_fetch_add(b.bar + 32 * (blockIdx.x & 7), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (lane < 8) {
      const unsigned per = (unsigned)((G - lane + 7) / 8);  // workgroups in shard `lane`
      const unsigned target = gen * per;
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(b.bar + 32 * lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > 10000000ull) {  // 100 ms
          __hip_atomic_store(b.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
    }
  }
  __syncthreads();
}

// ---- epilogues (lane 0 of the wave, rows < N)
template <int R>
__device__ __forceinline__ void epi_resid(const float (&acc)[R], const float (&bias)[R], float (&xr)[R], float* x,
                                          int N) {
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (lane_id() != 0) return;
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const int r = gw + j * NWV;
    if (r < N) {
      xr[j] += acc[j] + bias[j];
      st_sc1(x + r, xr[j]);
    }
  }
}

template <int R>
__device__ __forceinline__ void epi_gelu(const float (&acc)[R], const float (&bias)[R], float* h, int N) {
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (lane_id() != 0) return;
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const int r = gw + j * NWV;
    if (r < N) st_sc1(h + r, gelu_new(acc[j] + bias[j]));
  }
}

template <int R>
__device__ __forceinline__ void epi_qkv(const float (&acc)[R], const float (&bias)[R], bf16* q, int N) {
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (lane_id() != 0) return;
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const int r = gw + j * NWV;
    if (r < N) q[r] = f2bf(acc[j] + bias[j]);
  }
}

template <int R>
__device__ __forceinline__ void load_rows(float (&xr)[R], const float* x, int N) {
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
#pragma unroll
  for (int j = 0; j < R; ++j) xr[j] = ld_sc1(x + min(gw + j * NWV, N - 1));
}

// ---------------------------------------------------------------------------
// Mode A: one launch per phase
// ---------------------------------------------------------------------------
template <int H, int FF, int KIND>
__global__ __launch_bounds__(NT) void phase_kernel(LayerW L, Bufs b) {
  using D = Dims<H, FF>;
  __shared__ __attribute__((aligned(16))) bf16 xs[KIND == PROJ2 ? D::KSF : D::KSH];
  __shared__ float red[16];
  if constexpr (KIND == OPROJ) {
    WRegs<D::RO, D::NBH> w;
    float xr[D::RO], acc[D::RO];
    load_rows(xr, b.x, H);
    issue_w(w, L.wo, L.bo, H, H);
    zero_pad<D::KSH, H>(xs);
    input_bf16<H>(b.o, xs);
    __syncthreads();
    dots(w, xs, acc);
    epi_resid(acc, w.bias, xr, b.x, H);
  } else if constexpr (KIND == FC) {
    WRegs<D::RF, D::NBH> w;
    float acc[D::RF];
    issue_w(w, L.wfc, L.bfc, FF, H);
    zero_pad<D::KSH, H>(xs);
    input_ln<H>(b.x, L.g2, L.b2, xs, red);
    __syncthreads();
    dots(w, xs, acc);
    epi_gelu(acc, w.bias, b.h, FF);
  } else if constexpr (KIND == PROJ2) {
    WRegs<D::RO, D::NBF> w;
    float xr[D::RO], acc[D::RO];
    load_rows(xr, b.x, H);
    issue_w(w, L.wp2, L.bp2, H, FF);
    zero_pad<D::KSF, FF>(xs);
    input_f32<FF>(b.h, xs);
    __syncthreads();
    dots(w, xs, acc);
    epi_resid(acc, w.bias, xr, b.x, H);
  } else {
    WRegs<D::RQ, D::NBH> w;
    float acc[D::RQ];
    issue_w(w, L.wq, L.bq, 3 * H, H);
    zero_pad<D::KSH, H>(xs);
    input_ln<H>(b.x, L.g1, L.b1, xs, red);
    __syncthreads();
    dots(w, xs, acc);
    epi_qkv(acc, w.bias, b.qkv, 3 * H);
  }
}

// Attention stand-in: o = q (the real decode attention is ~5.7 us at batch 1
// on GPT-2 XL, profiles/r2_single_stream_analysis.log; identical in all modes)
template <int H>
__global__ __launch_bounds__(NT) void attn_standin(Bufs b) {
  const int i = blockIdx.x * NT + threadIdx.x;
  if (i < H) b.o[i] = b.qkv[i];
}

// ---------------------------------------------------------------------------
// Modes B / C: the four GEMV phases of a layer in one launch
// ---------------------------------------------------------------------------
template <int H, int FF, bool PREFETCH>
__global__ __launch_bounds__(NT) void chain_kernel(LayerW L, Bufs b, int layer) {
  using D = Dims<H, FF>;
  __shared__ __attribute__((aligned(16))) bf16 xh[D::KSH];
  __shared__ __attribute__((aligned(16))) bf16 xf[D::KSF];
  __shared__ float red[16];
  const unsigned gen0 = (unsigned)layer * 3;
  stamp(b, layer, 0);
  WRegs<D::RO, D::NBH> wo;
  WRegs<D::RF, D::NBH> wf;
  WRegs<D::RO, D::NBF> wp;
  WRegs<D::RQ, D::NBH> wq;
  float xr[D::RO];
  load_rows(xr, b.x, H);
  issue_w(wo, L.wo, L.bo, H, H);
  zero_pad<D::KSH, H>(xh);
  zero_pad<D::KSF, FF>(xf);
  // ---- out-projection + residual
  input_bf16<H>(b.o, xh);
  __syncthreads();
  {
    float acc[D::RO];
    dots(wo, xh, acc);
    stamp(b, layer, 1);
    epi_resid(acc, wo.bias, xr, b.x, H);
  }
  asm volatile("" ::: "memory");  // the epilogue stores issue before the prefetch
  if constexpr (PREFETCH) {
    issue_w(wf, L.wfc, L.bfc, FF, H);
    grid_sync<D::RF * D::NBH + D::RF>(b, gen0 + 1);
  } else {
    grid_sync<0>(b, gen0 + 1);
    issue_w(wf, L.wfc, L.bfc, FF, H);
  }
  stamp(b, layer, 2);
  // ---- LN2 + FC + GELU
  input_ln<H>(b.x, L.g2, L.b2, xh, red);
  __syncthreads();
  {
    float acc[D::RF];
    dots(wf, xh, acc);
    stamp(b, layer, 3);
    epi_gelu(acc, wf.bias, b.h, FF);
  }
  asm volatile("" ::: "memory");  // the epilogue stores issue before the prefetch
  if constexpr (PREFETCH) {
    issue_w(wp, L.wp2, L.bp2, H, FF);
    grid_sync<D::RO * D::NBF + D::RO>(b, gen0 + 2);
  } else {
    grid_sync<0>(b, gen0 + 2);
    issue_w(wp, L.wp2, L.bp2, H, FF);
  }
  stamp(b, layer, 4);
  // ---- projection + residual (same rows on the same wave as the out-projection)
  input_f32<FF>(b.h, xf);
  __syncthreads();
  {
    float acc[D::RO];
    dots(wp, xf, acc);
    stamp(b, layer, 5);
    epi_resid(acc, wp.bias, xr, b.x, H);
  }
  asm volatile("" ::: "memory");  // the epilogue stores issue before the prefetch
  if constexpr (PREFETCH) {
    issue_w(wq, L.wq, L.bq, 3 * H, H);
    grid_sync<D::RQ * D::NBH + D::RQ>(b, gen0 + 3);
  } else {
    grid_sync<0>(b, gen0 + 3);
    issue_w(wq, L.wq, L.bq, 3 * H, H);
  }
  stamp(b, layer, 6);
  // ---- LN1 (next layer's; same weights here) + QKV
  input_ln<H>(b.x, L.g1, L.b1, xh, red);
  __syncthreads();
  {
    float acc[D::RQ];
    dots(wq, xh, acc);
    stamp(b, layer, 7);
    epi_qkv(acc, wq.bias, b.qkv, 3 * H);
  }
  stamp(b, layer, 8);
}

// ---------------------------------------------------------------------------
__global__ void fill_kernel(bf16* p, long n, unsigned seed, float scale) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    unsigned z = (unsigned)i * 2654435761u ^ seed;
    z ^= z >> 15;
    z *= 2246822519u;
    z ^= z >> 13;
    p[i] = f2bf(((float)(z & 0xFFFF) / 65536.f - 0.5f) * scale);
  }
}

template <int H, int FF>
struct Model {
  int layers;
  std::vector<LayerW> L;
  bf16* slab = nullptr;
  Model(int n) : layers(n) {
    const long wsz = (long)H * H + 3L * H * H + 2L * H * FF;  // weights
    const long vsz = H + 3L * H + FF + H + 4L * H;            // biases + 2 LN (gamma, beta)
    const long tot = (wsz + vsz + 64) * n;
    CK(hipMalloc(&slab, tot * sizeof(bf16)));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, slab, tot, 12345u, 0.05f);
    CK(hipGetLastError());
    bf16* p = slab;
    auto take = [&](long k) { bf16* q = p; p += (k + 63) / 64 * 64; return q; };
    for (int l = 0; l < n; ++l) {
      LayerW w;
      w.wo = take((long)H * H); w.bo = take(H);
      w.wfc = take((long)FF * H); w.bfc = take(FF);
      w.wp2 = take((long)H * FF); w.bp2 = take(H);
      w.wq = take(3L * H * H); w.bq = take(3 * H);
      bf16* g1 = take(H); w.g1 = g1; w.b1 = take(H);
      bf16* g2 = take(H); w.g2 = g2; w.b2 = take(H);
      L.push_back(w);
    }
    // LN gammas near 1
    std::vector<bf16> ones(H);
    for (int i = 0; i < H; ++i) ones[i] = (bf16)(1.0f + 0.01f * (i % 7));
    for (auto& w : L) {
      CK(hipMemcpy(const_cast<bf16*>(w.g1), ones.data(), H * sizeof(bf16), hipMemcpyHostToDevice));
      CK(hipMemcpy(const_cast<bf16*>(w.g2), ones.data(), H * sizeof(bf16), hipMemcpyHostToDevice));
    }
  }
};

struct Result {
  double us_per_layer;
  std::vector<float> x;
  std::vector<unsigned short> q;
  int err;
};

// mode 0 = launches, 1 = persistent + prefetch, 2 = persistent, no prefetch
template <int H, int FF>
Result run(Model<H, FF>& m, int mode, Bufs b, const std::vector<float>& x0, int reps, bool stamps,
           std::vector<unsigned long long>* st_out) {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  Bufs bb = b;
  if (!stamps) bb.stamps = nullptr;
  // graph: reset x and the barrier counters, then every layer
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  CK(hipMemcpyAsync(b.x, x0.data(), H * sizeof(float), hipMemcpyHostToDevice, s));
  CK(hipMemsetAsync(b.bar, 0, 8 * 32 * sizeof(unsigned), s));
  CK(hipMemsetAsync(b.o, 0, H * sizeof(bf16), s));
  for (int l = 0; l < m.layers; ++l) {
    const LayerW& w = m.L[l];
    if (mode == 0) {
      hipLaunchKernelGGL((phase_kernel<H, FF, OPROJ>), dim3(G), dim3(NT), 0, s, w, bb);
      hipLaunchKernelGGL((phase_kernel<H, FF, FC>), dim3(G), dim3(NT), 0, s, w, bb);
      hipLaunchKernelGGL((phase_kernel<H, FF, PROJ2>), dim3(G), dim3(NT), 0, s, w, bb);
      hipLaunchKernelGGL((phase_kernel<H, FF, QKV>), dim3(G), dim3(NT), 0, s, w, bb);
    } else if (mode == 1) {
      hipLaunchKernelGGL((chain_kernel<H, FF, true>), dim3(G), dim3(NT), 0, s, w, bb, l);
    } else {
      hipLaunchKernelGGL((chain_kernel<H, FF, false>), dim3(G), dim3(NT), 0, s, w, bb, l);
    }
    hipLaunchKernelGGL((attn_standin<H>), dim3((H + NT - 1) / NT), dim3(NT), 0, s, bb);
  }
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipMemset(b.err, 0, sizeof(int)));
  for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, s));
  for (int i = 0; i < reps; ++i) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  Result r;
  r.us_per_layer = ms * 1000.0 / reps / m.layers;
  r.x.resize(H);
  r.q.resize(3 * H);
  CK(hipMemcpy(r.x.data(), b.x, H * sizeof(float), hipMemcpyDeviceToHost));
  CK(hipMemcpy(r.q.data(), b.qkv, 3 * H * sizeof(bf16), hipMemcpyDeviceToHost));
  CK(hipMemcpy(&r.err, b.err, sizeof(int), hipMemcpyDeviceToHost));
  if (st_out) {
    st_out->resize((size_t)m.layers * G * NSTAMP);
    CK(hipMemcpy(st_out->data(), b.stamps, st_out->size() * 8, hipMemcpyDeviceToHost));
  }
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipStreamDestroy(s));
  return r;
}

template <int H, int FF>
int bench(const char* name, int layers, int reps) {
  Model<H, FF> m(layers);
  Bufs b;
  CK(hipMalloc(&b.x, H * 4));
  CK(hipMalloc(&b.h, FF * 4));
  CK(hipMalloc(&b.qkv, 3 * H * 2));
  CK(hipMalloc(&b.o, H * 2));
  CK(hipMalloc(&b.bar, 8 * 32 * 4));
  CK(hipMalloc(&b.err, 4));
  CK(hipMalloc(&b.stamps, (size_t)layers * G * NSTAMP * 8));
  CK(hipMemset(b.stamps, 0, (size_t)layers * G * NSTAMP * 8));
  std::vector<float> x0(H);
  for (int i = 0; i < H; ++i) x0[i] = 0.5f * std::sin(0.37f * i) + 0.1f * (i % 13);
  CK(hipDeviceSynchronize());
  using D = Dims<H, FF>;
  std::printf("== %s: H %d FF %d, %d layers, grid %d x %d threads; rows per wave o/fc/proj/qkv %d/%d/%d/%d, "
              "chunks per lane K=H %d K=FF %d\n",
              name, H, FF, layers, G, NT, D::RO, D::RF, D::RO, D::RQ, D::NBH, D::NBF);
  const char* lab[3] = {"A launches (4 GEMV + attn per layer)", "B persistent + weight prefetch (1 + attn)",
                        "C persistent, no prefetch (1 + attn)"};
  Result res[3];
  for (int mode = 0; mode < 3; ++mode) {
    res[mode] = run(m, mode, b, x0, reps, false, nullptr);
    std::printf("  %-44s %8.2f us per layer%s\n", lab[mode], res[mode].us_per_layer,
                res[mode].err ? "  (BARRIER TIMEOUT)" : "");
  }
  // second pass, reversed order (box drift)
  for (int mode = 2; mode >= 0; --mode) {
    Result r = run(m, mode, b, x0, reps, false, nullptr);
    std::printf("  %-44s %8.2f us per layer (repeat)%s\n", lab[mode], r.us_per_layer, r.err ? "  (BARRIER TIMEOUT)" : "");
  }
  int bad = 0;
  for (int mode = 1; mode < 3; ++mode) {
    long dx = 0, dq = 0;
    for (int i = 0; i < H; ++i) dx += std::memcmp(&res[mode].x[i], &res[0].x[i], 4) != 0;
    for (int i = 0; i < 3 * H; ++i) dq += res[mode].q[i] != res[0].q[i];
    std::printf("  check %c vs A: residual words differing %ld / %d, qkv %ld / %d -> %s\n", 'A' + mode, dx, H, dq,
                3 * H, dx || dq ? "MISMATCH" : "bit-identical");
    bad += dx || dq;
  }
  bool finite = true;
  for (float v : res[0].x) finite &= std::isfinite(v);
  std::printf("  residual finite: %s (x[0] %.5f x[H-1] %.5f)\n", finite ? "yes" : "NO", res[0].x[0], res[0].x[H - 1]);
  // per-phase stamps of mode B (one replay)
  std::vector<unsigned long long> st;
  Result r = run(m, 1, b, x0, 1, true, &st);
  const char* ph[8] = {"start -> out-proj dots", "out-proj dots -> barrier 1 out", "barrier 1 -> FC dots (LN2)",
                       "FC dots -> barrier 2 out", "barrier 2 -> proj dots", "proj dots -> barrier 3 out",
                       "barrier 3 -> QKV dots (LN1)", "QKV dots -> epilogue done"};
  std::printf("  B per-phase spans (10 ns ticks -> us), median / max over workgroups, mean over layers 4..%d:\n",
              layers - 1);
  for (int k = 0; k < 8; ++k) {
    double med = 0, mx = 0;
    int nl = 0;
    for (int l = 4; l < layers; ++l) {
      std::vector<double> d(G);
      for (int w = 0; w < G; ++w) {
        const unsigned long long* p = &st[((size_t)l * G + w) * NSTAMP];
        d[w] = (double)(p[k + 1] - p[k]) * 0.01;
      }
      std::sort(d.begin(), d.end());
      med += d[G / 2];
      mx += d[G - 1];
      ++nl;
    }
    std::printf("    %-34s %6.2f / %6.2f us\n", ph[k], med / nl, mx / nl);
  }
  {
    double span = 0;
    int nl = 0;
    for (int l = 4; l < layers; ++l) {
      unsigned long long lo = ~0ull, hi = 0;
      for (int w = 0; w < G; ++w) {
        const unsigned long long* p = &st[((size_t)l * G + w) * NSTAMP];
        lo = std::min(lo, p[0]);
        hi = std::max(hi, p[8]);
      }
      span += (hi - lo) * 0.01;
      ++nl;
    }
    std::printf("    %-34s %6.2f us (first workgroup start -> last end)\n", "launch span", span / nl);
  }
  std::printf("  stamped replay barrier timeouts: %d\n", r.err);
  CK(hipFree(m.slab));
  return bad;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 50;
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  std::printf("device %s, %d CUs\n", p.name, p.multiProcessorCount);
  int bad = 0;
  bad += bench<1600, 6400>("GPT-2 XL", 48, reps);
  bad += bench<768, 3072>("GPT-2 small", 12, reps * 4);
  std::printf("%s\n", bad ? "RESULT: MISMATCH" : "RESULT: all modes bit-identical");
  return bad ? 1 : 0;
}
