// Embedding gather and (residual-combine +) LayerNorm / RMSNorm.
//
// K1-K3 of SURVEY.md §2.5: wte[ids] + wpe[pos] (`server.py:79-83`; dropout is a
// no-op in eval).  K4: LayerNorm eps 1e-5 ([tf5.15] modeling_gpt2.py:252-254,
// `server.py:101`), RMSNorm for Llama.
//
// The norm kernel is also the split-K reduction point: a residual GEMM that
// split K across workgroups leaves fp32 slabs [S][T][H]; this kernel computes
//   x[t] += bias + sum_s slab[s][t]       (written back, fp32 residual stream)
//   y[t]  = norm(x[t]) * w (+ b)          (bf16, the next GEMM's A operand)
// in one pass over the row -- the "combine in the next kernel's prologue"
// launch-boundary reduce (guide §5 Projection GEMM item 2), deterministic.
#include "common.h"

namespace lsd {

// One block per token row; each thread moves 8 contiguous elements per step.
__global__ __launch_bounds__(256) void embed_kernel(const int* __restrict__ ids,
                                                    const int* __restrict__ pos,
                                                    const bf16* __restrict__ wte,
                                                    const bf16* __restrict__ wpe, float* out,
                                                    int H, int vocab) {
  const int t = blockIdx.x;
  int id = ids[t];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);  // never read out of bounds
  const bf16* e = wte + (long)id * H;
  const bf16* pe = wpe ? wpe + (long)pos[t] * H : nullptr;
  float* o = out + (long)t * H;
  for (int c = threadIdx.x * 8; c < H; c += blockDim.x * 8) {
    bf16x8 a = ld8(e + c);
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = bf2f(a[j]);
    if (pe) {
      bf16x8 b = ld8(pe + c);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] += bf2f(b[j]);
    }
    *reinterpret_cast<f32x4*>(o + c) = f32x4{v[0], v[1], v[2], v[3]};
    *reinterpret_cast<f32x4*>(o + c + 4) = f32x4{v[4], v[5], v[6], v[7]};
  }
}

// Row kernel: H <= 4 * 256 * MAXV floats kept in registers between passes.
// SPL >= 0: exactly SPL split-K slabs, every slab load of the row issued
// before the first add (one memory round trip instead of one per slab: the
// runtime-count loop serialised them, ~1 us each); SPL < 0: runtime count.
// SB: the slabs are bf16 (LSD_SLAB_BF16: half the bytes), else fp32.
template <int MAXV, bool RMS, int SPL, bool SB = false>
__global__ __launch_bounds__(256) void norm_kernel(float* x, const void* __restrict__ slab_,
                                                   int splits, const bf16* __restrict__ pbias,
                                                   const bf16* __restrict__ w,
                                                   const bf16* __restrict__ b, bf16* out, int T,
                                                   int H, float eps, const int* __restrict__ rows) {
  __shared__ float red[24];
  const float* slab = static_cast<const float*>(slab_);
  const bf16* slab_h = static_cast<const bf16*>(slab_);
  // one slab element group of 4 at (split s, row, column c)
  auto slab4 = [&](int s, int row, int c) -> f32x4 {
    if constexpr (SB) {
      // read-once slabs: non-temporal loads (+0.6-1.3 % on the headline
      // over default-policy loads, profiles/r4_slab_bf16.log)
      const bf16x4 h = __builtin_bit_cast(
          bf16x4, __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(slab_h + ((long)s * T + row) * H + c)));
      return f32x4{bf2f(h[0]), bf2f(h[1]), bf2f(h[2]), bf2f(h[3])};
    } else {
      return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(slab + ((long)s * T + row) * H + c));
    }
  };
  const int t = blockIdx.x;
  // gamma / beta are issued first: their latency overlaps the row loads
  // instead of adding a second memory round trip after the reductions
  bf16x4 wv[MAXV], bv[MAXV];
  if (out != nullptr) {
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int c = min((threadIdx.x + i * 256) * 4, H - 4);
      wv[i] = ld4(w + c);
      if (!RMS) bv[i] = ld4(b + c);
    }
  }
  const int src = rows ? rows[t] : t;  // optional row gather (last-token rows)
  float* xr = x + (long)src * H;
  f32x4 v[MAXV];
  float s1 = 0.f, s2 = 0.f;
  // GRP column groups of the row are loaded per round trip (all of them
  // unless the slab count would blow the register budget)
  constexpr int NL = SPL > 0 ? SPL : 0;
  constexpr int GRP = MAXV * (NL + 1) <= 24 ? MAXV : 1;
#pragma unroll
  for (int i0 = 0; i0 < MAXV; i0 += GRP) {
    f32x4 xa[GRP], part[GRP][NL > 0 ? NL : 1];
    bf16x4 pbv[GRP];
#pragma unroll
    for (int g = 0; g < GRP; ++g) {
      const int cc = min((threadIdx.x + (i0 + g) * 256) * 4, H - 4);  // clamped: always valid
      xa[g] = *reinterpret_cast<const f32x4*>(xr + cc);
      if (slab && pbias) pbv[g] = ld4(pbias + cc);
#pragma unroll
      for (int s = 0; s < NL; ++s) part[g][s] = slab4(s, src, cc);
    }
#pragma unroll
    for (int g = 0; g < GRP; ++g) {
      const int i = i0 + g;
      const int c = (threadIdx.x + i * 256) * 4;
      if (c < H) {
        f32x4 a = xa[g];
#pragma unroll
        for (int s = 0; s < NL; ++s) a += part[g][s];
        if (SPL < 0 && slab)
          for (int s = 0; s < splits; ++s) a += slab4(s, src, c);
        if (slab) {
          if (pbias) {
            const bf16x4 pb = pbv[g];
            a += f32x4{bf2f(pb[0]), bf2f(pb[1]), bf2f(pb[2]), bf2f(pb[3])};
          }
          *reinterpret_cast<f32x4*>(xr + c) = a;
        }
        v[i] = a;
        if (!RMS) s1 += a[0] + a[1] + a[2] + a[3];
        else s2 += a[0] * a[0] + a[1] * a[1] + a[2] * a[2] + a[3] * a[3];
      } else {
        v[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
  if (out == nullptr) return;  // combine-only (flush)
  // LayerNorm: each thread's (count, mean, M2) over its own <= 4 MAXV values
  // (exact two-pass in registers), merged across the block in ONE LDS round
  // (Chan) instead of a mean reduction followed by a variance reduction
  float mean = 0.f, var;
  if (RMS) {
    var = block_sum(s2, red) / H;
  } else {
    float cnt = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) cnt += (threadIdx.x + i * 256) * 4 < H ? 4.f : 0.f;
    const float mt = cnt > 0.f ? s1 / cnt : 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      if ((threadIdx.x + i * 256) * 4 < H) {
        const f32x4 d = v[i] - mt;
        s2 += d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3];
      }
    }
    const Wf st = block_welford(Wf{cnt, mt, s2}, red);
    mean = st.m;
    var = st.M / H;
  }
  const float rstd = rsqrtf(var + eps);
  bf16* o = out + (long)t * H;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int c = (threadIdx.x + i * 256) * 4;
    if (c < H) {
      f32x4 y = (v[i] - mean) * rstd;
      bf16x4 r;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float z = y[j] * bf2f(wv[i][j]);
        if (!RMS) z += bf2f(bv[i][j]);
        r[j] = f2bf(z);
      }
      st4(o + c, r);
    }
  }
}

// Wave-per-row norm: 4 rows per 256-thread block, a row's 16-byte chunks
// spread over its wave's 64 lanes and all issued before the first use, the
// statistics merged inside the wave (DPP / permlane butterflies: no LDS, no
// barrier).  Up to 32 rows in flight per CU where the block kernel above
// holds 8 (2048 threads / 256 per row): GPT-2 XL prefill, 32 K rows x 1600,
// the block kernel streams ~4.5 TB/s (profiles/r4_rejected_norm_loop.log).
// SPL > 0: first fold SPL split-K slabs (bf16 when SB) and the projection
// bias into the fp32 residual row, written back -- the block kernel's decode
// job, every slab load of the row issued with the row's (H <= 1024).  Which
// row counts take this kernel: lsd_norm below.
template <int MAXC, bool RMS, int SPL = 0, bool SB = false>
__global__ __launch_bounds__(256) void norm_wave_kernel(float* __restrict__ x, const void* __restrict__ slab_,
                                                        const bf16* __restrict__ pbias, const bf16* __restrict__ w,
                                                        const bf16* __restrict__ b, bf16* __restrict__ out,
                                                        int T, int H, float eps) {
  const int lane = lane_id();
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= T) return;  // wave-uniform
  float* xr = x + (long)row * H;
  const int nch = H >> 2;  // 16-byte chunks of the row
  // the norm weights first: L2-resident, independent of the row, so their
  // round trip hides behind the row / slab loads instead of following the fold
  bf16x4 wv[MAXC], bv[MAXC];
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = 4 * min(lane + i * 64, nch - 1);
    wv[i] = ld4(w + c);
    if (!RMS) bv[i] = ld4(b + c);
  }
  f32x4 v[MAXC];
#pragma unroll
  for (int i = 0; i < MAXC; ++i) v[i] = *reinterpret_cast<const f32x4*>(xr + 4 * min(lane + i * 64, nch - 1));
  if constexpr (SPL > 0) {
    f32x4 part[MAXC][SPL];
    bf16x4 pb[MAXC];
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
      const int c = 4 * min(lane + i * 64, nch - 1);
#pragma unroll
      for (int s = 0; s < SPL; ++s) {
        if constexpr (SB) {
          const bf16x4 h = __builtin_bit_cast(bf16x4, __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(
                                                          static_cast<const bf16*>(slab_) + ((long)s * T + row) * H + c)));
          part[i][s] = f32x4{bf2f(h[0]), bf2f(h[1]), bf2f(h[2]), bf2f(h[3])};
        } else {
          part[i][s] = __builtin_nontemporal_load(
              reinterpret_cast<const f32x4*>(static_cast<const float*>(slab_) + ((long)s * T + row) * H + c));
        }
      }
      if (pbias) pb[i] = ld4(pbias + c);
    }
#pragma unroll
    for (int i = 0; i < MAXC; ++i) {
      f32x4 a = v[i];
#pragma unroll
      for (int s = 0; s < SPL; ++s) a += part[i][s];
      if (pbias) a += f32x4{bf2f(pb[i][0]), bf2f(pb[i][1]), bf2f(pb[i][2]), bf2f(pb[i][3])};
      v[i] = a;
      if (lane + i * 64 < nch) *reinterpret_cast<f32x4*>(xr + 4 * (lane + i * 64)) = a;
    }
  }
  float mean = 0.f, var;
  if (RMS) {
    float s2 = 0.f;
#pragma unroll
    for (int i = 0; i < MAXC; ++i)
      if (lane + i * 64 < nch) s2 += v[i][0] * v[i][0] + v[i][1] * v[i][1] + v[i][2] * v[i][2] + v[i][3] * v[i][3];
    s2 += wave_xchg<1>(s2);
    s2 += wave_xchg<2>(s2);
    s2 += wave_xchg<4>(s2);
    s2 += wave_xchg<8>(s2);
    s2 += wave_xchg<16>(s2);
    s2 += wave_xchg<32>(s2);
    var = s2 / H;
  } else {
    float cnt = 0.f, s1 = 0.f;
#pragma unroll
    for (int i = 0; i < MAXC; ++i)
      if (lane + i * 64 < nch) {
        cnt += 4.f;
        s1 += v[i][0] + v[i][1] + v[i][2] + v[i][3];
      }
    const float mt = cnt > 0.f ? s1 / cnt : 0.f;
    float m2 = 0.f;
#pragma unroll
    for (int i = 0; i < MAXC; ++i)
      if (lane + i * 64 < nch) {
        const f32x4 d = v[i] - mt;
        m2 += d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3];
      }
    Wf st{cnt, mt, m2};
    st = wf_merge(st, wf_xchg<1>(st));
    st = wf_merge(st, wf_xchg<2>(st));
    st = wf_merge(st, wf_xchg<4>(st));
    st = wf_merge(st, wf_xchg<8>(st));
    st = wf_merge(st, wf_xchg<16>(st));
    st = wf_merge(st, wf_xchg<32>(st));
    mean = st.m;
    var = st.M / H;
  }
  const float rstd = rsqrtf(var + eps);
  bf16* o = out + (long)row * H;
#pragma unroll
  for (int i = 0; i < MAXC; ++i) {
    const int c = lane + i * 64;
    if (c < nch) {
      const f32x4 y = (v[i] - mean) * rstd;
      bf16x4 r;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float z = y[j] * bf2f(wv[i][j]);
        if (!RMS) z += bf2f(bv[i][j]);
        r[j] = f2bf(z);
      }
      st4(o + 4 * c, r);
    }
  }
}

}  // namespace lsd

using namespace lsd;

extern "C" hipError_t lsd_embed(const int* ids, const int* pos, const bf16* wte, const bf16* wpe,
                                float* out, int T, int H, int vocab, hipStream_t st) {
  if (T == 0) return hipSuccess;
  hipLaunchKernelGGL(embed_kernel, dim3(T), dim3(256), 0, st, ids, pos, wte, wpe, out, H, vocab);
  return hipGetLastError();
}

// Wave-per-row kernel from g_norm_wave_min rows (any H <= 4096) and from
// g_norm_wave_narrow_min rows when H <= 1024 (0 = off).  The choice depends on
// (T, H) only, never on whether slabs are pending: a norm that folds slabs
// and the same norm after a separate fold (a pipeline stage boundary flushes
// pending slabs, parallel/pipeline.py) then compute their statistics with the
// same kernel, so a P-stage pipeline stays bit-identical to one stage.
static int g_norm_wave_min = 0;
extern "C" void lsd_norm_set_wave_min(int v) { g_norm_wave_min = v; }
static int g_norm_wave_narrow_min = 0;
extern "C" void lsd_norm_set_wave_narrow_min(int v) { g_norm_wave_narrow_min = v; }

static int norm_wave_rows(int H) {
  int m = g_norm_wave_min;
  if (H <= 1024 && g_norm_wave_narrow_min > 0 && (m == 0 || g_norm_wave_narrow_min < m)) m = g_norm_wave_narrow_min;
  return m;
}

extern "C" hipError_t lsd_norm(float* x, const void* slab, int slab_bf16, int splits, const bf16* pbias,
                               const bf16* w, const bf16* b, bf16* out, int T, int H, float eps,
                               int rms, const int* rows, int nrows, hipStream_t st) {
  const int n = rows ? nrows : T;
  if (n == 0) return hipSuccess;
  const int wmin = norm_wave_rows(H);
  const bool wave = !rows && out && H % 4 == 0 && H <= 4096 && wmin > 0 && T >= wmin;
  // 4 rows (one wave each) per block: 1- and 2-row blocks measured within
  // noise on GPT-2 small decode and the XL prefill (profiles/r6_normwave_rpb.log)
  const dim3 wg((T + 3) / 4), wb(256);
  if (wave && slab && H <= 1024 && splits >= 1 && splits <= 8) {
    // slabs folded in the wave kernel: its row and every slab load in registers
#define LSD_NORM_WS(S, SB)                                                                                           \
  if (rms) hipLaunchKernelGGL((norm_wave_kernel<4, true, S, SB>), wg, wb, 0, st, x, slab, pbias, w, b, out, T, H, eps); \
  else hipLaunchKernelGGL((norm_wave_kernel<4, false, S, SB>), wg, wb, 0, st, x, slab, pbias, w, b, out, T, H, eps);
#define LSD_NORM_WB(S)     \
  if (slab_bf16) {         \
    LSD_NORM_WS(S, true)   \
  } else {                 \
    LSD_NORM_WS(S, false)  \
  }
    switch (splits) {
      case 1: LSD_NORM_WB(1) break;
      case 2: LSD_NORM_WB(2) break;
      case 3: LSD_NORM_WB(3) break;
      case 4: LSD_NORM_WB(4) break;
      case 5: LSD_NORM_WB(5) break;
      case 6: LSD_NORM_WB(6) break;
      case 7: LSD_NORM_WB(7) break;
      default: LSD_NORM_WB(8) break;
    }
#undef LSD_NORM_WB
#undef LSD_NORM_WS
    return hipGetLastError();
  }
  if (wave && slab) {
    // other slab counts / widths: fold first (the block kernel's combine-only
    // pass, the same add order), then the slab-free wave kernel below
    const hipError_t e = lsd_norm(x, slab, slab_bf16, splits, pbias, nullptr, nullptr, nullptr, T, H, eps, rms,
                                  nullptr, 0, st);
    if (e != hipSuccess) return e;
    slab = nullptr;
  }
  if (wave) {
    const int nch = H / 4;
#define LSD_NORM_W(MC)                                                                                           \
  if (rms) hipLaunchKernelGGL((norm_wave_kernel<MC, true>), wg, wb, 0, st, x, nullptr, nullptr, w, b, out, T, H, eps); \
  else hipLaunchKernelGGL((norm_wave_kernel<MC, false>), wg, wb, 0, st, x, nullptr, nullptr, w, b, out, T, H, eps);
    if (nch <= 256) {
      LSD_NORM_W(4)
    } else if (nch <= 512) {
      LSD_NORM_W(8)
    } else {
      LSD_NORM_W(16)
    }
#undef LSD_NORM_W
    return hipGetLastError();
  }
  const int maxv = (H + 1023) / 1024;
#define LSD_NORM_T(MV, S, SB)                                                                     \
  if (rms)                                                                                        \
    hipLaunchKernelGGL((norm_kernel<MV, true, S, SB>), dim3(n), dim3(256), 0, st, x, slab, splits, \
                       pbias, w, b, out, T, H, eps, rows);                                        \
  else                                                                                            \
    hipLaunchKernelGGL((norm_kernel<MV, false, S, SB>), dim3(n), dim3(256), 0, st, x, slab,      \
                       splits, pbias, w, b, out, T, H, eps, rows);
#define LSD_NORM_S(MV, S)      \
  if (slab_bf16 && slab) {     \
    LSD_NORM_T(MV, S, true)    \
  } else {                     \
    LSD_NORM_T(MV, S, false)   \
  }
#define LSD_NORM(MV)                   \
  switch (slab ? splits : 0) {         \
    case 0: LSD_NORM_S(MV, 0) break;   \
    case 1: LSD_NORM_S(MV, 1) break;   \
    case 2: LSD_NORM_S(MV, 2) break;   \
    case 3: LSD_NORM_S(MV, 3) break;   \
    case 4: LSD_NORM_S(MV, 4) break;   \
    case 5: LSD_NORM_S(MV, 5) break;   \
    case 6: LSD_NORM_S(MV, 6) break;   \
    case 7: LSD_NORM_S(MV, 7) break;   \
    case 8: LSD_NORM_S(MV, 8) break;   \
    default: LSD_NORM_S(MV, -1) break; \
  }
  if (maxv <= 2) {
    LSD_NORM(2)
  } else if (maxv <= 4) {
    LSD_NORM(4)
  } else if (maxv <= 8) {
    LSD_NORM(8)
  } else {
    return hipErrorInvalidValue;
  }
#undef LSD_NORM_T
#undef LSD_NORM_S
#undef LSD_NORM
  return hipGetLastError();
}
