// MFMA GEMMs with fused epilogues:  C[M,N] = A[M,K] . W[N,K]^T  (+ epilogue)
//
// Replaces the reference's HF Conv1D / nn.Linear calls on CPU (SURVEY.md
// §2.5 K5, K8, K10, K12, K13: `[tf5.15] modeling_gpt2.py:185,223,239,241`,
// `server.py:102`).  Weights are stored [N][K] (K-contiguous) so a
// 16x16x32 B-operand fragment is one 16-byte load.
//
// Two kernels:
//  * gemm_skinny  -- M <= 64 (decode microbatches).  Weight-bandwidth bound:
//    W is streamed HBM -> VGPRs with 16-byte loads, no LDS round trip (guide
//    §5 "GEMV / M <= 16 decode weights"), the block's 4 waves split K and
//    reduce through LDS, optional cross-workgroup split-K writes fp32 slabs
//    that the next norm kernel folds in (no atomics, deterministic).
//  * gemm_tiled   -- M > 64 (prefill / large microbatches).  128x128x64 block
//    tile, 4 waves of 64x64, operands staged HBM -> LDS with 16-byte
//    global_load_lds (LDS-DMA), XOR-swizzled on the source address so the
//    ds_read_b128 fragment reads are bank-conflict free, double buffered,
//    XCD-aware tile order.
//
// Epilogues (fused, no extra pass): bias, gelu_new, silu(gate)*up, fp32
// store, residual add into the fp32 residual stream, split-K slab, and the
// QKV epilogue that applies RoPE (Llama) and scatters K/V straight into the
// shard-local KV cache at (slot, position).
#include "common.h"
#include "gemm_params.h"

namespace lsd {

enum Epi : int {
  EPI_BF16 = 0,      // out bf16 = acc + bias
  EPI_GELU = 1,      // out bf16 = gelu_new(acc + bias)
  EPI_SILU_MUL = 2,  // out bf16 [M, N/2] = silu(gate) * up; W rows interleaved in 16-row blocks
  EPI_F32 = 3,       // out f32 = acc
  EPI_RESID = 4,     // x f32 += acc + bias
  EPI_SLAB = 5,      // slab[split][M][N] = acc
  EPI_QKV = 6,       // q -> out bf16, k/v -> KV cache (+ RoPE)
};


// Stores the 4 accumulator values of one 16x16 MFMA tile owned by this lane:
// column n, rows row0 + i.  All lanes of the wave must call it (RoPE uses a
// cross-lane exchange).  `v2` carries the paired tile for EPI_SILU_MUL.
template <int EPI>
__device__ __forceinline__ void epilogue4(const GemmParams& p, int row0, int n, f32x4 v, f32x4 v2,
                                          int split) {
  if constexpr (EPI == EPI_SLAB) {
    float* s = p.slab + (long)split * p.M * p.N;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (row0 + i < p.M) s[(long)(row0 + i) * p.N + n] = v[i];
    return;
  }
  if constexpr (EPI == EPI_F32) {
    float* o = reinterpret_cast<float*>(p.out);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (row0 + i < p.M) o[(long)(row0 + i) * p.ldo + n] = v[i];
    return;
  }
  const float b = p.bias ? bf2f(p.bias[n]) : 0.f;
  if constexpr (EPI == EPI_RESID) {
    float* x = reinterpret_cast<float*>(p.out);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (row0 + i < p.M) x[(long)(row0 + i) * p.ldo + n] += v[i] + b;
    return;
  }
  if constexpr (EPI == EPI_BF16 || EPI == EPI_GELU) {
    bf16* o = reinterpret_cast<bf16*>(p.out);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float y = v[i] + b;
      if constexpr (EPI == EPI_GELU) y = gelu_new(y);
      if (row0 + i < p.M) o[(long)(row0 + i) * p.ldo + n] = f2bf(y);
    }
    return;
  }
  if constexpr (EPI == EPI_SILU_MUL) {
    // n is the gate column inside an interleaved [gate16 | up16] 32-row block
    bf16* o = reinterpret_cast<bf16*>(p.out);
    const int col = (n >> 5) * 16 + (n & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (row0 + i < p.M) o[(long)(row0 + i) * p.ldo + col] = f2bf(silu(v[i]) * v2[i]);
    return;
  }
  if constexpr (EPI == EPI_QKV) {
    float y[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) y[i] = v[i] + b;
    const int qk = p.q_size + p.kv_size;
    if (p.rope != nullptr && n < qk) {  // uniform per 16-column tile (q/k sizes are multiples of hd)
      const int d = (n < p.q_size ? n : n - p.q_size) % p.hd;
      const int half = p.hd >> 1;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float partner = shfl_xor(y[i], 1);
        const int m = min(row0 + i, p.M - 1);
        const int pos = p.tpos[m];
        const float* cs = p.rope + ((long)pos * half + (d >> 1)) * 2;
        const float c = cs[0], s = cs[1];
        y[i] = (d & 1) ? (y[i] * c + partner * s) : (y[i] * c - partner * s);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = row0 + i;
      if (m >= p.M) continue;
      if (n < p.q_size) {
        reinterpret_cast<bf16*>(p.out)[(long)m * p.ldo + n] = f2bf(y[i]);
      } else {
        const int c = n < qk ? n - p.q_size : n - qk;
        const int head = c / p.hd, d = c % p.hd;
        bf16* cache = n < qk ? p.kc : p.vc;
        const long idx = (((long)p.tslot[m] * p.n_kv + head) * p.max_seq + p.tpos[m]) * p.hd + d;
        cache[idx] = f2bf(y[i]);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Skinny GEMM (M <= 64)
// ---------------------------------------------------------------------------
// grid = (N / (16*NW), splits); block = 256 = 4 waves splitting the block's K range.
template <int MT, int NW, int U, int EPI>
__global__ __launch_bounds__(256) void gemm_skinny_kernel(GemmParams p) {
  const int lane = lane_id(), wk = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int nb = blockIdx.x * 16 * NW;
  const int split = blockIdx.y;
  const int KT = p.K >> 5;
  const int kb = (int)((long)KT * split / p.splits), ke = (int)((long)KT * (split + 1) / p.splits);
  const int len = ke - kb;
  const int wb = kb + len * wk / 4, we = kb + len * (wk + 1) / 4;

  const bf16* wp[NW];
#pragma unroll
  for (int ns = 0; ns < NW; ++ns) wp[ns] = p.W + (long)(nb + 16 * ns + r) * p.ldw + g * 8;
  const bf16* ap[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) ap[mt] = p.A + (long)min(mt * 16 + r, p.M - 1) * p.lda + g * 8;

  f32x4 acc[MT][NW];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int ns = 0; ns < NW; ++ns) acc[mt][ns] = f32x4{0.f, 0.f, 0.f, 0.f};

  int s = wb;
  for (; s + U <= we; s += U) {
    bf16x8 wv[U][NW], av[U][MT];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int ns = 0; ns < NW; ++ns) wv[u][ns] = ld8(wp[ns] + (long)(s + u) * 32);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) av[u][mt] = ld8(ap[mt] + (long)(s + u) * 32);
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int ns = 0; ns < NW; ++ns) acc[mt][ns] = mfma16(av[u][mt], wv[u][ns], acc[mt][ns]);
  }
  for (; s < we; ++s) {
    bf16x8 wv[NW], av[MT];
#pragma unroll
    for (int ns = 0; ns < NW; ++ns) wv[ns] = ld8(wp[ns] + (long)s * 32);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) av[mt] = ld8(ap[mt] + (long)s * 32);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int ns = 0; ns < NW; ++ns) acc[mt][ns] = mfma16(av[mt], wv[ns], acc[mt][ns]);
  }

  // Reduce the 4 waves' K-partials through LDS; wave 0 runs the epilogue.
  __shared__ f32x4 red[3][MT * NW][64];
  if (wk > 0) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int ns = 0; ns < NW; ++ns) red[wk - 1][mt * NW + ns][lane] = acc[mt][ns];
  }
  __syncthreads();
  if (wk != 0) return;
#pragma unroll
  for (int j = 0; j < 3; ++j)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int ns = 0; ns < NW; ++ns) acc[mt][ns] += red[j][mt * NW + ns][lane];

#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int row0 = mt * 16 + 4 * g;
    if constexpr (EPI == EPI_SILU_MUL) {
#pragma unroll
      for (int ns = 0; ns < NW; ns += 2)
        epilogue4<EPI>(p, row0, nb + 16 * ns + r, acc[mt][ns], acc[mt][ns + 1], split);
    } else {
#pragma unroll
      for (int ns = 0; ns < NW; ++ns)
        epilogue4<EPI>(p, row0, nb + 16 * ns + r, acc[mt][ns], acc[mt][ns], split);
    }
  }
}

// ---------------------------------------------------------------------------
// Tiled GEMM (M > 64): 128x128x64, glds-staged, swizzled, double-buffered
// ---------------------------------------------------------------------------
constexpr int TBM = 128, TBN = 128, TBK = 64;
constexpr int TILE_BYTES = TBM * TBK * 2;  // 16 KiB per operand tile

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void gbl_cvoid;

// Stage a [128 rows][64 k] bf16 tile: LDS image is row-major 128-B rows with
// the 16-B chunk index XOR-swizzled by (row>>1)&7.  glds writes lane-linear
// (base + 16*lane), so the swizzle goes on the per-lane SOURCE address and the
// same XOR is applied on the read (guide §5.4 rule 21).
__device__ __forceinline__ void stage_tile(char* lds_tile, const bf16* src, long ld, int row0,
                                           int row_max, int k0) {
  const int lane = lane_id(), w = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int inst = w * 4 + q;           // 16 wave-instructions of 1 KiB per tile
    const int row = inst * 8 + (lane >> 3);
    const int pch = lane & 7;
    const int lch = pch ^ ((row >> 1) & 7);
    const int grow = min(row0 + row, row_max);
    const bf16* gp = src + (long)grow * ld + k0 + lch * 8;
    __builtin_amdgcn_global_load_lds((gbl_cvoid*)gp, (lds_void*)(lds_tile + inst * 1024), 16, 0, 0);
  }
}

__device__ __forceinline__ bf16x8 lds_frag(const char* tile, int row, int chunk) {
  const int pch = chunk ^ ((row >> 1) & 7);
  return *reinterpret_cast<const bf16x8*>(tile + row * 128 + pch * 16);
}

template <int EPI>
__global__ __launch_bounds__(256) void gemm_tiled_kernel(GemmParams p, int tiles_m, int tiles_n) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TILE_BYTES];  // [buf][A|W]
  const int nwg = gridDim.x;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int per_split = tiles_m * tiles_n;
  const int split = bid / per_split;
  const int t = bid % per_split;
  const int tm = t % tiles_m, tn = t / tiles_m;  // M-fastest: blocks sharing a W panel adjacent
  const int m0 = tm * TBM, n0 = tn * TBN;
  const int KT = p.K / TBK;
  const int kb = (int)((long)KT * split / p.splits), ke = (int)((long)KT * (split + 1) / p.splits);

  const int lane = lane_id(), w = threadIdx.x >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int r = lane & 15, g = lane >> 4;

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (kb < ke) {
    stage_tile(smem, p.A, p.lda, m0, p.M - 1, kb * TBK);
    stage_tile(smem + TILE_BYTES, p.W, p.ldw, n0, p.N - 1, kb * TBK);
    __syncthreads();
  }
  int cur = 0;
  for (int kt = kb; kt < ke; ++kt) {
    if (kt + 1 < ke) {
      char* nb = smem + (cur ^ 1) * 2 * TILE_BYTES;
      stage_tile(nb, p.A, p.lda, m0, p.M - 1, (kt + 1) * TBK);
      stage_tile(nb + TILE_BYTES, p.W, p.ldw, n0, p.N - 1, (kt + 1) * TBK);
    }
    const char* ta = smem + cur * 2 * TILE_BYTES;
    const char* tw = ta + TILE_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[4], wf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = lds_frag(ta, wm * 64 + i * 16 + r, kk * 4 + g);
#pragma unroll
      for (int j = 0; j < 4; ++j) wf[j] = lds_frag(tw, wn * 64 + j * 16 + r, kk * 4 + g);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af[i], wf[j], acc[i][j]);
    }
    __syncthreads();  // waits the in-flight glds (vmcnt(0)) and the buffer's readers
    cur ^= 1;
  }

#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row0 = m0 + wm * 64 + i * 16 + 4 * g;
    if constexpr (EPI == EPI_SILU_MUL) {
#pragma unroll
      for (int j = 0; j < 4; j += 2) {
        const int n = n0 + wn * 64 + j * 16 + r;
        if (n < p.N) epilogue4<EPI>(p, row0, n, acc[i][j], acc[i][j + 1], split);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wn * 64 + j * 16 + r;
        // N % 64 == 0 (host-checked): a whole 16-col tile is in or out, so the
        // RoPE lane exchange never straddles the predicate.
        if (n0 + wn * 64 + j * 16 < p.N) epilogue4<EPI>(p, row0, n, acc[i][j], acc[i][j], split);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------
template <int EPI>
static hipError_t launch_skinny(const GemmParams& p, hipStream_t st) {
  const int MT = (p.M + 15) / 16;
  const int NW = (EPI == EPI_SILU_MUL) ? 2 : 1;
  dim3 grid(p.N / (16 * NW), p.splits), block(256);
#define LSD_SK(mt, u)                                                               \
  hipLaunchKernelGGL((gemm_skinny_kernel<mt, (EPI == EPI_SILU_MUL ? 2 : 1), u, EPI>), grid, \
                     block, 0, st, p)
  switch (MT) {
    case 1: LSD_SK(1, 8); break;
    case 2: LSD_SK(2, 4); break;
    case 3: LSD_SK(3, 4); break;
    case 4: LSD_SK(4, 4); break;
    default: return hipErrorInvalidValue;
  }
#undef LSD_SK
  (void)NW;
  return hipGetLastError();
}

template <int EPI>
static hipError_t launch_tiled(const GemmParams& p, hipStream_t st) {
  const int tm = (p.M + TBM - 1) / TBM, tn = (p.N + TBN - 1) / TBN;
  dim3 grid(tm * tn * p.splits), block(256);
  hipLaunchKernelGGL((gemm_tiled_kernel<EPI>), grid, block, 0, st, p, tm, tn);
  return hipGetLastError();
}

}  // namespace lsd

using namespace lsd;

// C ABI used by csrc/bindings.cpp; shapes are validated there.
extern "C" hipError_t lsd_gemm(const GemmParams* p, int epi, int tiled, hipStream_t st) {
#define LSD_DISPATCH(E) \
  case E: return tiled ? launch_tiled<E>(*p, st) : launch_skinny<E>(*p, st);
  switch (epi) {
    LSD_DISPATCH(EPI_BF16)
    LSD_DISPATCH(EPI_GELU)
    LSD_DISPATCH(EPI_SILU_MUL)
    LSD_DISPATCH(EPI_F32)
    LSD_DISPATCH(EPI_RESID)
    LSD_DISPATCH(EPI_SLAB)
    LSD_DISPATCH(EPI_QKV)
    default: return hipErrorInvalidValue;
  }
#undef LSD_DISPATCH
}
