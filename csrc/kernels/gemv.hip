// Small-M decode GEMV (M <= 8 rows): C[M,N] = norm?(A)[M,K] . W[N,K]^T (+ epilogue)
//
// Single-stream and small-batch decode (SURVEY.md §7.4 hard part 1: "decode
// GEMMs are skinny") is pure weight streaming: every W byte is used M <= 8
// times, so the only goal is to keep HBM busy and pay as few kernel
// boundaries as possible.  The split-K MFMA kernel (gemm.hip, gemm_sk) pays a
// cross-workgroup combine (release/acquire ticket) per launch and needs a
// separate norm kernel in front of every QKV / MLP-up / lm_head GEMM; at
// M = 1 that was ~7 us of fixed cost per launch (profiles/r1_microbench_gemm_m1_256.log).
//
// Design (guide §5 "GEMV / M <= 16 decode weights": load straight to VGPRs,
// deep unroll, late vmcnt):
//   * one wave owns CPW whole W rows (output columns) over the FULL K: no
//     split-K, no partial slabs, no cross-workgroup hand-off at all;
//   * every 16-byte W chunk of the wave's rows is issued up front (NB x 4
//     chunks per lane per row, fully unrolled), the activation rows are
//     requested BEFORE them (L2-resident, they land first), so the input
//     prologue below runs while the weight stream is in flight;
//   * fused input norm (NORM = LayerNorm / RMSNorm): the workgroup normalises
//     the fp32 residual rows itself (block-wide two-pass statistics) and
//     writes the bf16 result to LDS -- the separate norm launch disappears;
//   * dot products with v_dot2c_f32_bf16 against the LDS image (zero-padded
//     past K, so the clamped tail chunks contribute nothing);
//   * butterfly reduce-scatter across the 64 lanes (CPW*MR values, one value
//     per lane group at the end), then the fused epilogue: bias, gelu_new,
//     silu(gate)*up, fp32 logits, residual add, or QKV + RoPE + KV-cache append.
// Replaces, for decode at M <= 8, the reference's per-token HF Conv1D /
// nn.Linear calls (`[tf5.15] modeling_gpt2.py:185,223,239,241`, `server.py:102`).
#include "common.h"
#include "gemm_params.h"

namespace lsd {
namespace gv {
enum : int { BF16 = 0, GELU = 1, SILU = 2, F32 = 3, RESID = 4, QKV = 6 };
enum : int { NONE = 0, LN = 1, RMS = 2 };
}  // namespace gv

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

// Pairs (2j, 2j+1) of a bf16x8 as the bf16x2 operand of v_dot2c_f32_bf16.
// (A __builtin_bit_cast of a u32x4 element to bf16x2 miscompiles on ROCm 7.2:
// hipcc loads one dword and feeds it to all four dot2 instructions.)
#define LSD_PAIR(v, j) __builtin_shufflevector(v, v, 2 * (j), 2 * (j) + 1)
__device__ __forceinline__ float dot8(bf16x8 a, bf16x8 b, float acc) {
  acc = __builtin_amdgcn_fdot2_f32_bf16(LSD_PAIR(a, 0), LSD_PAIR(b, 0), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(LSD_PAIR(a, 1), LSD_PAIR(b, 1), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(LSD_PAIR(a, 2), LSD_PAIR(b, 2), acc, false);
  acc = __builtin_amdgcn_fdot2_f32_bf16(LSD_PAIR(a, 3), LSD_PAIR(b, 3), acc, false);
  return acc;
}

// W row j (0..CPW-1) of global wave gw.  SiLU: the gate/up rows are
// interleaved in 16-row blocks (ops/hip.py interleave_gate_up), so output
// column c needs rows 32*(c/16) + c%16 (gate) and that + 16 (up).
template <int EPI, int CPW>
__device__ __forceinline__ int gv_row(int gw, int j) {
  if constexpr (EPI == gv::SILU) {
    const int col = gw * (CPW / 2) + (j >> 1);
    return (col >> 4) * 32 + (col & 15) + (j & 1) * 16;
  } else {
    return gw * CPW + j;
  }
}

// One butterfly step at lane bit OFF over the first N live values: lanes with
// the bit set keep the upper half, the others the lower half, each adding
// the partner's copy of the half it keeps (N == 1: plain pairwise sum).
template <int OFF, int N, int V>
__device__ __forceinline__ void gv_step(float (&acc)[V], int& idx, int lane) {
  if constexpr (N == 1) {
    acc[0] += wave_xchg<OFF>(acc[0]);
  } else {
    constexpr int h = N / 2;
    const bool up = (lane & OFF) != 0;
#pragma unroll
    for (int i = 0; i < h; ++i) {
      const float send = up ? acc[i] : acc[i + h];
      const float keep = up ? acc[i + h] : acc[i];
      acc[i] = keep + wave_xchg<OFF>(send);
    }
    if (up) idx += h;
  }
}

// Block-wide sums of MR values at once (one LDS round for all rows).
template <int MR>
__device__ __forceinline__ void block_sums(float (&v)[MR], float* red) {
#pragma unroll
  for (int m = 0; m < MR; ++m) v[m] = wave_sum(v[m]);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if (lane_id() == 0) {
#pragma unroll
    for (int m = 0; m < MR; ++m) red[w * MR + m] = v[m];
  }
  __syncthreads();
#pragma unroll
  for (int m = 0; m < MR; ++m) v[m] = red[m] + red[MR + m] + red[2 * MR + m] + red[3 * MR + m];
}

template <int MR, int NB, int NORM>
constexpr bool gv_ok() {
  return MR * NB <= 16 && (NORM == gv::NONE || MR * NB <= 4);
}

template <int MR, int CPW, int EPI, int NORM, int NB>
__global__ __launch_bounds__(256) void gemv_kernel(GemvParams p) {
  if constexpr (!gv_ok<MR, NB, NORM>()) {
    return;
  } else {
    constexpr int SLOTS = 4 * NB;    // 16-byte chunks per lane per W row
    constexpr int KS = SLOTS * 512;  // LDS image row length (elements), zero past K
    constexpr int V = CPW * MR;      // partial sums per lane
    static_assert((V & (V - 1)) == 0 && V <= 16, "V must be a power of two <= 16");
    __shared__ __attribute__((aligned(16))) bf16 xs[MR * KS];
    __shared__ float red[4 * 16];
    const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
    const int gw = blockIdx.x * 4 + w;
    const int KC = p.K >> 3;  // valid 16-byte chunks per row
    const int M = p.M;

    // ---- 0. the epilogue's own operands, fetched NOW (they do not depend on
    // the dot products): bias, the residual value the RESID epilogue adds to,
    // the QKV rows' position / cache slot and the RoPE partner's bias.  Loaded
    // after the reduction they cost one dependent memory round trip at the
    // tail of every launch (the single-stream layer is five such tails).
    constexpr int NOUT = EPI == gv::SILU ? V / 2 : V;
    const bool epi_thread = tid < 4 * NOUT;
    const int e_w2 = tid / NOUT, e_o = tid % NOUT;
    const int e_j = e_o / MR, e_m = e_o % MR;
    const int e_n = (blockIdx.x * 4 + e_w2) * CPW + e_j;  // output column (non-SiLU)
    const bool e_live = epi_thread && e_m < M && e_n < p.N;
    float e_bias = 0.f, e_biasp = 0.f, e_x = 0.f;
    int e_pos = 0, e_slot = 0;
    if constexpr (EPI != gv::SILU) {
      if (e_live) {
        if (p.bias) e_bias = bf2f(p.bias[e_n]);
        if constexpr (EPI == gv::RESID) e_x = reinterpret_cast<const float*>(p.out)[(long)e_m * p.ldo + e_n];
        if constexpr (EPI == gv::QKV) {
          e_pos = p.tpos[e_m];
          if (e_n >= p.q_size) e_slot = p.tslot[e_m];
          if (CPW % 2 == 0 && p.rope != nullptr && p.bias && e_n < p.q_size + p.kv_size) e_biasp = bf2f(p.bias[e_n ^ 1]);
        }
      }
    }

    // ---- 1. activation rows first (L2-resident: they land before the weights)
    constexpr int NV = NORM != gv::NONE ? 2 * NB : 1;  // f32x4 per thread per row
    constexpr int NA = NORM != gv::NONE ? 1 : MR * NB;  // bf16x8 copy chunks per thread
    f32x4 xr[NORM != gv::NONE ? MR : 1][NV];
    bf16x4 gmv[NV], btv[NV];
    bf16x8 av[NA];
    if constexpr (NORM != gv::NONE) {
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int c = min((tid + 256 * i) * 4, p.K - 4);  // clamped: always a valid address
        gmv[i] = ld4(p.gamma + c);
        if constexpr (NORM == gv::LN) btv[i] = ld4(p.beta + c);
#pragma unroll
        for (int m = 0; m < MR; ++m)
          xr[m][i] = *reinterpret_cast<const f32x4*>(p.X + (long)min(m, M - 1) * p.ldx + c);
      }
    } else {
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int q = tid + 256 * i;
        const int m = q / (SLOTS * 64), c = q % (SLOTS * 64);
        av[i] = ld8(p.A + (long)min(m, M - 1) * p.lda + min(c, KC - 1) * 8);
      }
    }

    // ---- 2. the weight stream: every chunk of this wave's rows, issued now
    bf16x8 wv[CPW][SLOTS];
    // waves past N re-read row N-1 (never stored)
    if (p.nt) {  // wave-uniform: weights read once per token need not stay cached
#pragma unroll
      for (int j = 0; j < CPW; ++j) {
        const bf16* wr = p.W + (long)min(gv_row<EPI, CPW>(gw, j), p.N - 1) * p.ldw;
#pragma unroll
        for (int i = 0; i < SLOTS; ++i) wv[j][i] = ld8_nt(wr + min(lane + 64 * i, KC - 1) * 8);
      }
    } else {
#pragma unroll
      for (int j = 0; j < CPW; ++j) {
        const bf16* wr = p.W + (long)min(gv_row<EPI, CPW>(gw, j), p.N - 1) * p.ldw;
#pragma unroll
        for (int i = 0; i < SLOTS; ++i) wv[j][i] = ld8(wr + min(lane + 64 * i, KC - 1) * 8);
      }
    }

    // ---- 3. input prologue -> LDS (runs while the weights are in flight)
    if constexpr (NORM != gv::NONE) {
      float mean[MR], rstd[MR];
#pragma unroll
      for (int m = 0; m < MR; ++m) mean[m] = 0.f;
      if constexpr (NORM == gv::LN) {
#pragma unroll
        for (int m = 0; m < MR; ++m) {
          float s = 0.f;
#pragma unroll
          for (int i = 0; i < NV; ++i)
            if ((tid + 256 * i) * 4 < p.K) s += xr[m][i][0] + xr[m][i][1] + xr[m][i][2] + xr[m][i][3];
          mean[m] = s;
        }
        block_sums<MR>(mean, red);
#pragma unroll
        for (int m = 0; m < MR; ++m) mean[m] /= p.K;
      }
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < NV; ++i)
          if ((tid + 256 * i) * 4 < p.K) {
            const f32x4 d = xr[m][i] - mean[m];
            s += d[0] * d[0] + d[1] * d[1] + d[2] * d[2] + d[3] * d[3];
          }
        rstd[m] = s;
      }
      block_sums<MR>(rstd, red);
#pragma unroll
      for (int m = 0; m < MR; ++m) rstd[m] = rsqrtf(rstd[m] / p.K + p.eps);
#pragma unroll
      for (int m = 0; m < MR; ++m)
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          const int c = (tid + 256 * i) * 4;  // covers [0, KS): zero past K and for rows >= M
          bf16x4 r;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float z = (xr[m][i][e] - mean[m]) * rstd[m] * bf2f(gmv[i][e]);
            if constexpr (NORM == gv::LN) z += bf2f(btv[i][e]);
            r[e] = f2bf((c < p.K && m < M) ? z : 0.f);
          }
          st4(xs + m * KS + c, r);
        }
    } else {
      const bf16x8 zero = {};
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        const int q = tid + 256 * i;
        const int m = q / (SLOTS * 64), c = q % (SLOTS * 64);
        st8(xs + m * KS + c * 8, (m < M && c < KC) ? av[i] : zero);
      }
    }
    __syncthreads();

    // the RoPE (cos, sin) of this epilogue thread's position: issued before the
    // dot products (its position arrived with the first loads)
    float e_cs0 = 0.f, e_cs1 = 0.f;
    if constexpr (EPI == gv::QKV) {
      if (CPW % 2 == 0 && p.rope != nullptr && e_live && e_n < p.q_size + p.kv_size) {
        const int d = (e_n < p.q_size ? e_n : e_n - p.q_size) % p.hd;
        const float* cs = p.rope + ((long)e_pos * (p.hd >> 1) + (d >> 1)) * 2;
        e_cs0 = cs[0];
        e_cs1 = cs[1];
      }
    }

    // ---- 4. dot products (W from registers, x from LDS)
    float acc[V];
#pragma unroll
    for (int v = 0; v < V; ++v) acc[v] = 0.f;
#pragma unroll
    for (int i = 0; i < SLOTS; ++i) {
      const int c = lane + 64 * i;
#pragma unroll
      for (int m = 0; m < MR; ++m) {
        const bf16x8 xv = *reinterpret_cast<const bf16x8*>(xs + m * KS + c * 8);
#pragma unroll
        for (int j = 0; j < CPW; ++j) acc[j * MR + m] = dot8(wv[j][i], xv, acc[j * MR + m]);
      }
    }

    // ---- 5. butterfly reduce-scatter over the wave (DPP / permlane swaps):
    // halving steps leave each lane group with the full sum of one value
    // idx; the remaining steps are plain pairwise sums
    int idx = 0;
    gv_step<32, V>(acc, idx, lane);
    gv_step<16, (V > 1 ? V / 2 : 1)>(acc, idx, lane);
    gv_step<8, (V > 2 ? V / 4 : 1)>(acc, idx, lane);
    gv_step<4, (V > 4 ? V / 8 : 1)>(acc, idx, lane);
    gv_step<2, (V > 8 ? V / 16 : 1)>(acc, idx, lane);
    gv_step<1, 1>(acc, idx, lane);
    if ((lane & (64 / V - 1)) == 0) red[w * 16 + idx] = acc[0];
    __syncthreads();

    // ---- 6. fused epilogue, one thread per (wave, output); operands prefetched in step 0
    if (epi_thread) {
      const int w2 = e_w2, o = e_o;
      const int gw2 = blockIdx.x * 4 + w2;
      const float* rv = red + w2 * 16;
      if constexpr (EPI == gv::SILU) {
        const int jj = o / MR, m = o % MR;
        const int col = gw2 * (CPW / 2) + jj;
        if (m < M && col < (p.N >> 1)) {
          const float g = rv[(2 * jj) * MR + m], u = rv[(2 * jj + 1) * MR + m];
          reinterpret_cast<bf16*>(p.out)[(long)m * p.ldo + col] = f2bf(silu(g) * u);
        }
      } else if (e_live) {
        const int j = e_j, m = e_m, n = e_n;
        float y = rv[j * MR + m] + e_bias;
        if constexpr (EPI == gv::F32) {
          reinterpret_cast<float*>(p.out)[(long)m * p.ldo + n] = y;
          if (p.segmax && tid == 0) {
            // this workgroup's 8 columns are one sampler segment: its maximum
            // per row, from the same fp32 values stored above (bit-equal to a
            // max over the stored logits)
#pragma unroll
            for (int mm = 0; mm < MR; ++mm) {
              if (mm >= M) break;
              float mx = -INFINITY;
#pragma unroll
              for (int w3 = 0; w3 < 4; ++w3)
#pragma unroll
                for (int j3 = 0; j3 < CPW; ++j3) {
                  const int n3 = (blockIdx.x * 4 + w3) * CPW + j3;
                  if (n3 < p.N) mx = fmaxf(mx, red[w3 * 16 + j3 * MR + mm] + (p.bias ? bf2f(p.bias[n3]) : 0.f));
                }
              p.segmax[(long)mm * p.ldseg + blockIdx.x] = mx;
            }
          }
        } else if constexpr (EPI == gv::RESID) {
          reinterpret_cast<float*>(p.out)[(long)m * p.ldo + n] = e_x + y;
        } else if constexpr (EPI == gv::BF16 || EPI == gv::GELU) {
          reinterpret_cast<bf16*>(p.out)[(long)m * p.ldo + n] = f2bf(EPI == gv::GELU ? gelu_new(y) : y);
        } else if constexpr (EPI == gv::QKV) {
          const int qk = p.q_size + p.kv_size;
          const int pos = e_pos;
          if (CPW % 2 == 0 && p.rope != nullptr && n < qk) {
            // RoPE pairs (2i, 2i+1) are this wave's rows j, j^1 (ops/hip.py
            // rope_pair_permutation makes the rotated pairs adjacent)
            const float yp = rv[(j ^ 1) * MR + m] + e_biasp;
            const int d = (n < p.q_size ? n : n - p.q_size) % p.hd;
            y = (d & 1) ? (y * e_cs0 + yp * e_cs1) : (y * e_cs0 - yp * e_cs1);
          }
          if (n < p.q_size) {
            reinterpret_cast<bf16*>(p.out)[(long)m * p.ldo + n] = f2bf(y);
          } else {
            const int c = n < qk ? n - p.q_size : n - qk;
            bf16* cache = n < qk ? p.kc : p.vc;
            cache[(((long)e_slot * p.n_kv + c / p.hd) * p.max_seq + pos) * p.hd + c % p.hd] = f2bf(y);
          }
        }
      }
    }
  }
}

template <int EPI, int NORM>
hipError_t gemv_launch(const GemvParams& p, int mr, int nb, hipStream_t st) {
  constexpr int CPW = EPI == gv::RESID ? 1 : 2;
  const int grid = (p.N + 4 * CPW - 1) / (4 * CPW);
#define LSD_GV(MR_, NB_)                                                                    \
  if (mr == MR_ && nb == NB_) {                                                             \
    if constexpr (gv_ok<MR_, NB_, NORM>()) {                                                \
      hipLaunchKernelGGL((gemv_kernel<MR_, CPW, EPI, NORM, NB_>), dim3(grid), dim3(256), 0, \
                         st, p);                                                            \
      return hipGetLastError();                                                             \
    } else {                                                                                \
      return hipErrorInvalidValue;                                                          \
    }                                                                                       \
  }
  LSD_GV(1, 1) LSD_GV(1, 2) LSD_GV(1, 4) LSD_GV(1, 7)
  LSD_GV(2, 1) LSD_GV(2, 2) LSD_GV(2, 4) LSD_GV(2, 7)
  LSD_GV(4, 1) LSD_GV(4, 2) LSD_GV(4, 4)
  LSD_GV(8, 1) LSD_GV(8, 2)
#undef LSD_GV
  return hipErrorInvalidValue;
}

}  // namespace lsd

using namespace lsd;

// Row bucket and K bucket of a GEMV launch; 0 when the shape is not eligible.
static int gv_mr(int M) { return M <= 1 ? 1 : M <= 2 ? 2 : M <= 4 ? 4 : M <= 8 ? 8 : 0; }
static int gv_nb(int K) { return K <= 2048 ? 1 : K <= 4096 ? 2 : K <= 8192 ? 4 : K <= 14336 ? 7 : 0; }

extern "C" int lsd_gemv_ok(int M, int K, int epi, int norm) {
  const int mr = gv_mr(M), nb = gv_nb(K);
  if (M < 1 || mr == 0 || nb == 0 || K % 8 != 0) return 0;
  if (mr * nb > 16) return 0;
  if (norm != gv::NONE && mr * nb > 4) return 0;
  if (epi == 5) return 0;  // no slab epilogue: the GEMV never splits K
  // exactly the (epilogue, norm) pairs lsd_gemv dispatches: a pair it does not
  // instantiate must read "not ok" so the caller materialises the norm first
  switch (epi * 4 + norm) {
    case gv::BF16 * 4 + gv::NONE: case gv::GELU * 4 + gv::NONE: case gv::GELU * 4 + gv::LN:
    case gv::SILU * 4 + gv::NONE: case gv::SILU * 4 + gv::RMS: case gv::F32 * 4 + gv::NONE:
    case gv::F32 * 4 + gv::LN: case gv::F32 * 4 + gv::RMS: case gv::RESID * 4 + gv::NONE:
    case gv::QKV * 4 + gv::NONE: case gv::QKV * 4 + gv::LN: case gv::QKV * 4 + gv::RMS:
      return 1;
    default:
      return 0;
  }
}

static int g_gemv_nt = 0;
extern "C" void lsd_gemv_set_nt(int v) { g_gemv_nt = v; }

extern "C" hipError_t lsd_gemv(const GemvParams* pin, int epi, int norm, hipStream_t st) {
  if (!lsd_gemv_ok(pin->M, pin->K, epi, norm)) return hipErrorInvalidValue;
  GemvParams q = *pin;
  q.nt = g_gemv_nt;
  const GemvParams* p = &q;
  const int mr = gv_mr(p->M), nb = gv_nb(p->K);
  switch (epi * 4 + norm) {
    case gv::BF16 * 4 + gv::NONE: return gemv_launch<gv::BF16, gv::NONE>(*p, mr, nb, st);
    case gv::GELU * 4 + gv::NONE: return gemv_launch<gv::GELU, gv::NONE>(*p, mr, nb, st);
    case gv::GELU * 4 + gv::LN: return gemv_launch<gv::GELU, gv::LN>(*p, mr, nb, st);
    case gv::SILU * 4 + gv::NONE: return gemv_launch<gv::SILU, gv::NONE>(*p, mr, nb, st);
    case gv::SILU * 4 + gv::RMS: return gemv_launch<gv::SILU, gv::RMS>(*p, mr, nb, st);
    case gv::F32 * 4 + gv::NONE: return gemv_launch<gv::F32, gv::NONE>(*p, mr, nb, st);
    case gv::F32 * 4 + gv::LN: return gemv_launch<gv::F32, gv::LN>(*p, mr, nb, st);
    case gv::F32 * 4 + gv::RMS: return gemv_launch<gv::F32, gv::RMS>(*p, mr, nb, st);
    case gv::RESID * 4 + gv::NONE: return gemv_launch<gv::RESID, gv::NONE>(*p, mr, nb, st);
    case gv::QKV * 4 + gv::NONE: return gemv_launch<gv::QKV, gv::NONE>(*p, mr, nb, st);
    case gv::QKV * 4 + gv::LN: return gemv_launch<gv::QKV, gv::LN>(*p, mr, nb, st);
    case gv::QKV * 4 + gv::RMS: return gemv_launch<gv::QKV, gv::RMS>(*p, mr, nb, st);
    default: return hipErrorInvalidValue;
  }
}
