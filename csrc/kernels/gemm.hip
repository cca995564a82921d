// MFMA GEMMs with fused epilogues:  C[M,N] = A[M,K] . W[N,K]^T  (+ epilogue)
//
// Replaces the reference's HF Conv1D / nn.Linear calls on CPU (SURVEY.md
// §2.5 K5, K8, K10, K12, K13: `[tf5.15] modeling_gpt2.py:185,223,239,241`,
// `server.py:102`).  Weights are stored [N][K] (K-contiguous) so a
// 16x16x32 B-operand fragment is one 16-byte load.
//
// Four kernels:
//  * gemm_sk      -- decode microbatches (M <= 64; narrow GEMMs to 128 rows).  Weight-bandwidth bound:
//    W streamed HBM -> VGPRs (read once, no LDS round trip), the small A
//    operand staged through LDS with full-line LDS-DMA, split-K across
//    workgroups for occupancy with an in-kernel last-arriver combine that
//    runs the fused epilogue (deterministic: fixed summation order).
//  * gemm_tiled   -- larger M (prefill, vocab projection).  128x128x64 block
//    tile, 4 waves of 64x64, operands staged HBM -> LDS with 16-byte
//    global_load_lds (LDS-DMA), XOR-swizzled on the source address so the
//    ds_read_b128 fragment reads are bank-conflict free, double buffered,
//    XCD-aware tile order.
//  * gemm_ring    -- the tiled kernel's grids of <= 256 workgroups (decode
//    microbatches of 65-256 rows): 128x64 (or 128x128) tiles, a 3-slot LDS
//    ring with two k-steps in flight, 1 block/CU.
//  * gemm_big     -- large prefill GEMMs: 256x256 tiles, 8 waves, 4-slot ring.
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


// (head, dim) of column c inside the q / k / v block: shifts and a mask for the
// power-of-two head dims of every model here (a wave-uniform branch; integer
// division by a runtime divisor is a ~40-instruction sequence per call, paid
// for every 16-byte chunk of the prefill QKV epilogue)
__device__ __forceinline__ void hd_split(int hd, int c, int& head, int& d) {
  if ((hd & (hd - 1)) == 0) {
    head = c >> __builtin_ctz(hd);
    d = c & (hd - 1);
  } else {
    head = c / hd;
    d = c % hd;
  }
}

// Stores the 4 accumulator values of one 16x16 MFMA tile owned by this lane:
// column n, rows row0 + i.  All lanes of the wave must call it (RoPE uses a
// cross-lane exchange).  `v2` carries the paired tile for EPI_SILU_MUL.
template <int EPI>
__device__ __forceinline__ void epilogue4(const GemmParams& p, int row0, int n, f32x4 v, f32x4 v2,
                                          int split) {
  if constexpr (EPI == EPI_SLAB) {
    if (p.slab_bf16) {
      bf16* s = reinterpret_cast<bf16*>(p.slab) + (long)split * p.M * p.N;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (row0 + i < p.M) s[(long)(row0 + i) * p.N + n] = f2bf(v[i]);
      return;
    }
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
      int hh, d;
      hd_split(p.hd, n < p.q_size ? n : n - p.q_size, hh, d);
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
        int head, d;
        hd_split(p.hd, c, head, d);
        bf16* cache = n < qk ? p.kc : p.vc;
        const long idx = (((long)p.tslot[m] * p.n_kv + head) * p.max_seq + p.tpos[m]) * p.hd + d;
        cache[idx] = f2bf(y[i]);
      }
    }
  }
}

// Row-contiguous epilogue of 8 consecutive columns [n, n+8) of row m (the
// tiled kernel's LDS-transposed output): every store is one 16-byte vector.
// n % 8 == 0; bias / out / x / caches are 16-byte aligned (host-checked).
//
// Split in three so a store pass can issue the global reads of ALL its chunks
// before its first store (store_pass below): CDNA4's vmcnt counts loads and
// stores in one in-order counter, so a load issued after a store is waited for
// together with that store, and a chunk-at-a-time loop (load bias / residual,
// wait, compute, store) serialises one store round trip per chunk (the p8
// epilogue: 16 per thread, most of its 6-12 us).
//   epi8_pre  -- bias, residual x, QKV position / slot      (independent loads)
//   epi8_pre2 -- QKV RoPE (cos, sin) of that position        (dependent loads)
//   epi8_post -- the math and the stores
// s_waitcnt immediate for vmcnt(n) alone (gfx9 layout: vmcnt[3:0] | vmcnt[5:4] << 14)
constexpr int vmcnt_imm(int n) { return (n & 0xF) | ((n >> 4) << 14) | (0x7 << 4) | (0xF << 8); }

struct Epi8Pre {
  bf16x8 b;
  f32x4 x0, x1, cs0, cs1;
  int pos, slot;
};

template <int EPI>
__device__ __forceinline__ void epi8_pre(const GemmParams& p, int m, int n, Epi8Pre& e) {
  if constexpr (EPI == EPI_SLAB || EPI == EPI_F32 || EPI == EPI_SILU_MUL) return;
  if (p.bias) e.b = ld8(p.bias + n);
  if constexpr (EPI == EPI_RESID) {
    const f32x4* x = reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(p.out) + (long)m * p.ldo + n);
    e.x0 = x[0];
    e.x1 = x[1];
  }
  if constexpr (EPI == EPI_QKV) {
    e.pos = p.tpos[m];
    e.slot = n >= p.q_size ? p.tslot[m] : 0;
  }
}

template <int EPI>
__device__ __forceinline__ void epi8_pre2(const GemmParams& p, int n, Epi8Pre& e) {
  if constexpr (EPI == EPI_QKV) {
    if (p.rope != nullptr && n < p.q_size + p.kv_size) {
      int hh, d0;
      hd_split(p.hd, n < p.q_size ? n : n - p.q_size, hh, d0);
      const f32x4* cs = reinterpret_cast<const f32x4*>(p.rope + ((long)e.pos * (p.hd >> 1) + (d0 >> 1)) * 2);
      e.cs0 = cs[0];
      e.cs1 = cs[1];
    }
  }
}

template <int EPI>
__device__ __forceinline__ void epi8_post(const GemmParams& p, int m, int n, const float* v, int split,
                                          const Epi8Pre& e) {
  if constexpr (EPI == EPI_SLAB) {
    if (p.slab_bf16) {  // half the slab bytes for the GEMM to write and the norm to read
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(v[j]);
      st8(reinterpret_cast<bf16*>(p.slab) + (long)split * p.M * p.N + (long)m * p.N + n, o);
      return;
    }
  }
  if constexpr (EPI == EPI_SLAB || EPI == EPI_F32) {
    float* o = EPI == EPI_SLAB ? p.slab + (long)split * p.M * p.N + (long)m * p.N + n
                               : reinterpret_cast<float*>(p.out) + (long)m * p.ldo + n;
    reinterpret_cast<f32x4*>(o)[0] = f32x4{v[0], v[1], v[2], v[3]};
    reinterpret_cast<f32x4*>(o)[1] = f32x4{v[4], v[5], v[6], v[7]};
    if constexpr (EPI == EPI_F32) {
      // lm_head: the chunk's maximum for the sampler (one float per 8 logits)
      if (p.segmax) {
        const float m01 = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
        const float m23 = fmaxf(fmaxf(v[4], v[5]), fmaxf(v[6], v[7]));
        p.segmax[(long)m * p.ldseg + (n >> 3)] = fmaxf(m01, m23);
      }
    }
    return;
  }
  float y[8];
  if (p.bias) {
#pragma unroll
    for (int j = 0; j < 8; ++j) y[j] = v[j] + bf2f(e.b[j]);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) y[j] = v[j];
  }
  if constexpr (EPI == EPI_RESID) {
    f32x4* x = reinterpret_cast<f32x4*>(reinterpret_cast<float*>(p.out) + (long)m * p.ldo + n);
    f32x4 x0 = e.x0, x1 = e.x1;
#pragma unroll
    for (int j = 0; j < 4; ++j) { x0[j] += y[j]; x1[j] += y[4 + j]; }
    x[0] = x0;
    x[1] = x1;
    return;
  }
  if constexpr (EPI == EPI_BF16 || EPI == EPI_GELU) {
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(EPI == EPI_GELU ? gelu_new(y[j]) : y[j]);
    st8(reinterpret_cast<bf16*>(p.out) + (long)m * p.ldo + n, o);
    return;
  }
  if constexpr (EPI == EPI_QKV) {
    const int qk = p.q_size + p.kv_size;
    if (p.rope != nullptr && n < qk) {  // adjacent (even, odd) pairs rotate together
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 t = h ? e.cs1 : e.cs0;  // (cos, sin) of pairs d0/2 + 2h, d0/2 + 2h + 1
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const float c = t[2 * q], sn = t[2 * q + 1];
          const float a = y[4 * h + 2 * q], b = y[4 * h + 2 * q + 1];
          y[4 * h + 2 * q] = a * c - b * sn;
          y[4 * h + 2 * q + 1] = b * c + a * sn;
        }
      }
    }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(y[j]);
    if (n < p.q_size) {
      st8(reinterpret_cast<bf16*>(p.out) + (long)m * p.ldo + n, o);
    } else {
      const int c = n < qk ? n - p.q_size : n - qk;
      bf16* cache = n < qk ? p.kc : p.vc;
      int head, d;
      hd_split(p.hd, c, head, d);
      st8(cache + (((long)e.slot * p.n_kv + head) * p.max_seq + e.pos) * p.hd + d, o);
    }
  }
}

template <int EPI>
__device__ __forceinline__ void epilogue8(const GemmParams& p, int m, int n, const float* v, int split) {
  Epi8Pre e;
  epi8_pre<EPI>(p, m, n, e);
  epi8_pre2<EPI>(p, n, e);
  epi8_post<EPI>(p, m, n, v, split, e);
}

// One store pass over the 8-column row chunks c = threadIdx.x + i * NT (i < NCH,
// c < nchunks) of an fp32 C image in LDS.  at(c, m, n, src) maps a chunk to its
// output row / column and its 8 floats in LDS (false: out of range).  Every
// global read of the thread's chunks is issued before its first store (see
// epi8_pre); SiLU·up pairs each gate chunk with the up chunk 16 columns right
// (interleaved [gate16 | up16] 32-column blocks in one tile: `up` = src + UPOFF).
template <int EPI, int NCH, int NT, class At>
__device__ __forceinline__ void store_pass(const GemmParams& p, int nchunks, int split, At at) {
  Epi8Pre e[NCH];
  int mm[NCH], nn[NCH];
  const float* sp[NCH];
  bool ok[NCH];
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int c = (int)threadIdx.x + i * NT;
    ok[i] = c < nchunks && at(c, mm[i], nn[i], sp[i]);
    if (ok[i]) epi8_pre<EPI>(p, mm[i], nn[i], e[i]);
  }
  // one explicit wait for all of them: the compiler's own waits after the
  // branchy chunk bodies below would be vmcnt(0) per chunk (joins lose count),
  // i.e. one store round trip per chunk again
  __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));
  if constexpr (EPI == EPI_QKV) {
    if (p.rope != nullptr) {  // wave-uniform: GPT-2 has no RoPE loads to wait for
#pragma unroll
      for (int i = 0; i < NCH; ++i)
        if (ok[i]) epi8_pre2<EPI>(p, nn[i], e[i]);
      __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));
    }
  }
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    if (!ok[i]) continue;
    const f32x4 lo = *reinterpret_cast<const f32x4*>(sp[i]);
    const f32x4 hi = *reinterpret_cast<const f32x4*>(sp[i] + 4);
    const float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    epi8_post<EPI>(p, mm[i], nn[i], v, split, e[i]);
  }
}

// ---------------------------------------------------------------------------
// Decode GEMM (M <= 128): split-K across workgroups, last-arriver combine
// ---------------------------------------------------------------------------
// grid = (N / (64*NW) column tiles, S k-splits); block = 4 waves, wave w owns
// columns [16*NW*w, 16*NW*(w+1)) of the block's tile and the whole K range of
// the split.  Per round of up to 512 k (256 k for M > 64):
//   * A[0:M, k-range] -> LDS with 16-B LDS-DMA (global_load_lds), whole 128-B
//     lines per instruction (not 16-row fragment-shaped loads, which double
//     TA traffic: guide §5 "x operand through LDS in full lines"), one image of
//     256-B rows per 128-k chunk, 16-B chunks XOR-swizzled by (row & 15) so the
//     ds_read_b128 fragment reads are conflict-free;
//   * every W fragment of the round is issued straight to VGPRs (W is read
//     once: no LDS round trip), so a block costs ONE memory round trip;
//   * one barrier, then MFMAs out of LDS (A) and registers (W).
// S > 1: each split stores its fp32 partial tile, the last arriver (agent-scope
// release/acquire ticket, guide §5 "In-launch split-K reduction") sums the S
// partials and runs the fused epilogue -- so any epilogue (QKV scatter + RoPE,
// GELU, residual add) works with any split and no extra launch is needed.
// 32-k MFMA steps per round: 16 (512 k) up to M = 64; 8 (256 k) for M <= 128
// so the A image stays at 64 KiB (2 blocks / CU) while the rows double.
// Rounds are double-buffered (2 LDS images): 4 steps (128 k) above 64 rows,
// 8 up to 64 rows, 16 up to 32 rows keep both images at <= 64 KiB (2 blocks/CU).
template <int MT>
constexpr int sk_round_steps() {
#ifdef LSD_SK_ROUND
  return LSD_SK_ROUND;
#else
  return MT > 4 ? 4 : (MT > 2 ? 8 : 16);
#endif
}
// s_waitcnt simm16 (gfx9 layout) for lgkmcnt(0) alone
constexpr int LGKM0_SK = 0xC07F;

__device__ __forceinline__ void glds16(const void* g, void* lds) {
  __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) const void*)g,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

// Diagnostic phase stamps (100 MHz constant clock), written by thread 0 only
// when p.stamps != null; slot 7 = XCC id.  Never on in production.
#define LSD_STAMP(k)                                                                       \
  if (p.stamps && threadIdx.x == 0)                                                        \
    p.stamps[(((long)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * 8 + (k)] = \
        __builtin_amdgcn_s_memrealtime();

template <int MT, int NW, int EPI>
__global__ __launch_bounds__(256) void gemm_sk_kernel(GemmParams p, int* __restrict__ cnt,
                                                      float* __restrict__ ws) {
  constexpr int ROWS = MT * 16;
  constexpr int CHUNK_BYTES = ROWS * 256;  // one [ROWS][128 k] bf16 image
  constexpr int BNB = 64 * NW;             // block tile columns
  constexpr int SK_ROUND_STEPS = sk_round_steps<MT>();
  constexpr int NCHUNK = SK_ROUND_STEPS / 4;
  __shared__ __attribute__((aligned(16))) char smem[2 * NCHUNK * CHUNK_BYTES + 16];
  int* s_flag = reinterpret_cast<int*>(smem + 2 * NCHUNK * CHUNK_BYTES);

  LSD_STAMP(0)
  if (p.stamps && threadIdx.x == 0)
    p.stamps[(((long)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * 8 + 7] =
        __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11));  // HW_REG_XCC_ID[3:0]
  const int lane = lane_id(), w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int split = blockIdx.y, S = p.splits;
  // row block (blockIdx.z): M > rows-per-block runs as independent row
  // blocks that share each W tile through L2, instead of deeper K splits
  const int rb0 = blockIdx.z * ROWS;
  const int tile = blockIdx.x;
  const int tile_id = blockIdx.z * gridDim.x + tile;  // ticket / workspace index
  const int n_w = tile * BNB + w * 16 * NW;
  const int KT = p.K >> 5;
  const int kb = (int)((long)KT * split / S), ke = (int)((long)KT * (split + 1) / S);

  const bf16* wrow[NW];
#pragma unroll
  // a partial last tile (N % (64 NW) != 0) re-reads row N-1; its columns are never stored
  for (int ns = 0; ns < NW; ++ns) wrow[ns] = p.W + (long)min(n_w + 16 * ns + r, p.N - 1) * p.ldw + g * 8;

  f32x4 acc[MT][NW];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int ns = 0; ns < NW; ++ns) acc[mt][ns] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Double-buffered rounds: round r+1's W fragments (second register set) and
  // A image (second LDS buffer) are issued BEFORE round r's MFMAs, so a split
  // with several rounds pays one HBM latency instead of one per round.  Every
  // round issues the same number of loads per thread (partial rounds re-load
  // clamped addresses), so "round r has landed" is the counted wait
  // vmcnt(LOADS) -- raw s_barrier, never __syncthreads (it would drain the
  // next round's LDS-DMA too: guide §5 "Pipelining across barriers").
  constexpr int LOADS = SK_ROUND_STEPS * NW + NCHUNK * MT;  // per thread per round
  static_assert(LOADS <= 63, "vmcnt holds at most 63 outstanding loads");
  constexpr int WAIT_PREV = (LOADS & 0xF) | ((LOADS >> 4) << 14) | (0x7 << 4) | (0xF << 8);
  constexpr int WAIT_ALL = (0x7 << 4) | (0xF << 8);  // vmcnt(0)
  constexpr int BUF_BYTES = NCHUNK * CHUNK_BYTES;
  const int nrounds = (ke - kb + SK_ROUND_STEPS - 1) / SK_ROUND_STEPS;

  auto issue = [&](int rd, bf16x8 (&wv)[SK_ROUND_STEPS][NW], char* buf) {
    const int k0 = kb + rd * SK_ROUND_STEPS;
    const int nst = min(SK_ROUND_STEPS, ke - k0);
    // No per-load guard: a runtime "if (j < nst) load" makes hipcc branch
    // around each load and wait vmcnt(0) per element (guide §5 trap (c));
    // steps past the round end re-load the last valid step, never consumed.
#pragma unroll
    for (int j = 0; j < SK_ROUND_STEPS; ++j)
#pragma unroll
      for (int ns = 0; ns < NW; ++ns) wv[j][ns] = ld8(wrow[ns] + (long)(k0 + min(j, nst - 1)) * 32);
    // A chunks (after W: the HBM-latency loads go first, the L2-resident
    // activations overlap them): MT*4 wave-instructions (1 KiB = 4 rows of
    // 256 B) per chunk; chunks past the round end re-load a valid chunk
#pragma unroll
    for (int i = 0; i < NCHUNK * MT; ++i) {
      const int inst = w + 4 * i;
      const int c = inst / (MT * 4), q = inst % (MT * 4);
      const int row = q * 4 + (lane >> 4);
      const int lch = (lane & 15) ^ (row & 15);
      const int kk = min((k0 + min(c * 4, nst - 1)) * 32 + lch * 8, p.K - 8);
      glds16(p.A + (long)min(rb0 + row, p.M - 1) * p.lda + kk, buf + c * CHUNK_BYTES + q * 1024);
    }
  };
  // A fragments come from LDS one step ahead of the MFMAs that use them, so
  // the ds_read latency of step j+1 hides under step j's MFMAs for any round
  // length (the round count nst is wave-uniform).
  auto compute = [&](int rd, bf16x8 (&wv)[SK_ROUND_STEPS][NW], const char* buf) {
    const int nst = min(SK_ROUND_STEPS, ke - (kb + rd * SK_ROUND_STEPS));
    auto read_a = [&](int j, bf16x8 (&a)[MT]) {
      const char* img = buf + (j >> 2) * CHUNK_BYTES;
      const int lch = (j & 3) * 4 + g;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int row = mt * 16 + r;
        a[mt] = *reinterpret_cast<const bf16x8*>(img + row * 256 + ((lch ^ (row & 15)) << 4));
      }
    };
    // Fully unrolled (static indices keep wv[] in VGPRs -- a rolled loop sends
    // it to scratch, guide rule 20) and branch-free.
    bf16x8 a_cur[MT];
    read_a(0, a_cur);
#pragma unroll
    for (int j = 0; j < SK_ROUND_STEPS; ++j) {
      bf16x8 a_nxt[MT];
      read_a(min(j + 1, nst - 1), a_nxt);
      // Steps past the round end multiply a zeroed W fragment (A there is a
      // valid, finite LDS row) -- no branch, so the accumulators stay in AGPRs.
#pragma unroll
      for (int ns = 0; ns < NW; ++ns) {
        const u32x4 z = {0u, 0u, 0u, 0u};
        const u32x4 wb = __builtin_bit_cast(u32x4, wv[j][ns]);
        wv[j][ns] = __builtin_bit_cast(bf16x8, j < nst ? wb : z);
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int ns = 0; ns < NW; ++ns) acc[mt][ns] = mfma16(a_cur[mt], wv[j][ns], acc[mt][ns]);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) a_cur[mt] = a_nxt[mt];
    }
    // every wave's reads of `buf` retire before anyone re-fills it
    __builtin_amdgcn_s_waitcnt(LGKM0_SK);
    __builtin_amdgcn_s_barrier();
  };
  // round rd with round rd+1 issued first (straight-line, so hipcc's own
  // register waits count exactly like the explicit one)
  auto body_more = [&](int rd, bf16x8 (&cur)[SK_ROUND_STEPS][NW], char* cbuf,
                       bf16x8 (&nxt)[SK_ROUND_STEPS][NW], char* nbuf) {
    issue(rd + 1, nxt, nbuf);
    __builtin_amdgcn_s_waitcnt(WAIT_PREV);  // this thread's round-rd loads landed
    __builtin_amdgcn_s_barrier();           // ... and every other wave's A DMA
    if (rd == 0) { LSD_STAMP(1) }
    compute(rd, cur, cbuf);
  };
  auto body_last = [&](int rd, bf16x8 (&cur)[SK_ROUND_STEPS][NW], char* cbuf) {
    __builtin_amdgcn_s_waitcnt(WAIT_ALL);
    __builtin_amdgcn_s_barrier();
    if (rd == 0) { LSD_STAMP(1) }
    compute(rd, cur, cbuf);
  };

  bf16x8 wv0[SK_ROUND_STEPS][NW], wv1[SK_ROUND_STEPS][NW];
  char* buf0 = smem;
  char* buf1 = smem + BUF_BYTES;
  int rd = 0;
  if (nrounds > 0) issue(0, wv0, buf0);
  for (; rd + 2 < nrounds; rd += 2) {
    body_more(rd, wv0, buf0, wv1, buf1);
    body_more(rd + 1, wv1, buf1, wv0, buf0);
  }
  if (nrounds - rd == 2) {
    body_more(rd, wv0, buf0, wv1, buf1);
    body_last(rd + 1, wv1, buf1);
  } else if (nrounds - rd == 1) {
    body_last(rd, wv0, buf0);
  }
  LSD_STAMP(2)

  // EPI_SLAB (deferred combine): every split writes its raw partial tile to
  // slab[split] and the consumer (the next norm kernel, which reads the rows
  // anyway) sums the S slabs -- no publish, ticket or reducer tail here.
  if (S > 1 && EPI != EPI_SLAB) {
    // ---- publish this split's partial tile; the last arriver combines.
    // Slab layout is lane-major ([wave][mt][ns][lane] x f32x4) so every lane
    // moves 16 contiguous bytes; stores are write-through (sc1) and every
    // reducer load is sc1, so no agent release/acquire fence is needed (guide
    // §5 "In-launch split-K reduction", sc1 form; a buffer_wbl2 release per
    // block cost ~5 us here).
    constexpr int PER_BLOCK = 4 * MT * NW * 64;  // f32x4 per split tile
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        ws + (long)tile_id * S * PER_BLOCK * 4, (short)0, S * PER_BLOCK * 16, 0x00020000);
    const int lane_off = ((w * MT * NW) * 64 + lane) * 16;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int ns = 0; ns < NW; ++ns)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[mt][ns]), rs,
                                               split * PER_BLOCK * 16 + lane_off + (mt * NW + ns) * 1024,
                                               0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const int t = __hip_atomic_fetch_add(cnt + tile_id, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *s_flag = (t == S - 1);
      if (t == S - 1) __hip_atomic_store(cnt + tile_id, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    LSD_STAMP(3)
    if (*s_flag == 0) return;
    // Sum ALL S partials (own included, from the slab) in fixed split order:
    // the result must not depend on which split arrived last.
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int ns = 0; ns < NW; ++ns) acc[mt][ns] = f32x4{0.f, 0.f, 0.f, 0.f};
    // Issue every slab load of a group before summing (no per-load branch:
    // clamped index x 0/1 mask), so the reduce is one round trip per group
    // instead of one per split.
    // group size: <= 128 VGPRs of in-flight partials (the W registers are dead here)
    constexpr int RG = (32 / (MT * NW)) < 4 ? 4 : ((32 / (MT * NW)) > 16 ? 16 : 32 / (MT * NW));
    for (int s0 = 0; s0 < S; s0 += RG) {
      f32x4 v[RG][MT][NW];
#pragma unroll
      for (int u = 0; u < RG; ++u) {
        const int s2 = min(s0 + u, S - 1);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int ns = 0; ns < NW; ++ns)
            v[u][mt][ns] = __builtin_bit_cast(
                f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                           rs, s2 * PER_BLOCK * 16 + lane_off + (mt * NW + ns) * 1024, 0, 16));
      }
#pragma unroll
      for (int u = 0; u < RG; ++u) {
        const float msk = (s0 + u < S) ? 1.f : 0.f;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
          for (int ns = 0; ns < NW; ++ns) acc[mt][ns] += v[u][mt][ns] * msk;
      }
    }
  }
  LSD_STAMP(4)

  // Epilogue through LDS (free: the last round ended with every DMA drained
  // and a barrier): the MFMA layout gives a lane 4 rows x 1 column, i.e.
  // 2-4-byte stores scattered over 4 rows (KV-cache scatter, bf16 outputs,
  // slabs); transposed through an fp32 [ROWS][BNB] tile, every store is a
  // row-contiguous 16-byte vector (epilogue8, as in the tiled kernels).
  constexpr int CLD = BNB + 4;  // row stride: 4 rows x 16 columns hit 64 distinct banks
  constexpr bool LDS_EPI = EPI != EPI_SILU_MUL && ROWS * CLD * 4 <= 2 * NCHUNK * CHUNK_BYTES;
  if constexpr (LDS_EPI) {
    float* ct = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int ns = 0; ns < NW; ++ns)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          ct[(mt * 16 + 4 * g + q) * CLD + w * 16 * NW + ns * 16 + r] = acc[mt][ns][q];
    __syncthreads();
    const int n0 = tile * BNB;
    store_pass<EPI, (ROWS * (BNB / 8) + 255) / 256, 256>(
        p, ROWS * (BNB / 8), split, [&](int c, int& m, int& n, const float*& src) {
          const int row = c / (BNB / 8), ch = c % (BNB / 8);
          m = rb0 + row;
          n = n0 + ch * 8;
          src = ct + row * CLD + ch * 8;
          return m < p.M && n < p.N;
        });
  } else {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int row0 = rb0 + mt * 16 + 4 * g;
      if constexpr (EPI == EPI_SILU_MUL) {
#pragma unroll
        for (int ns = 0; ns < NW; ns += 2)
          epilogue4<EPI>(p, row0, n_w + 16 * ns + r, acc[mt][ns], acc[mt][ns + 1], 0);
      } else {
#pragma unroll
        for (int ns = 0; ns < NW; ++ns)  // 16-column sub-tiles past N: wave-uniform skip
          if (n_w + 16 * ns < p.N) epilogue4<EPI>(p, row0, n_w + 16 * ns + r, acc[mt][ns], acc[mt][ns], split);
      }
    }
  }
  LSD_STAMP(5)
}

// ---------------------------------------------------------------------------
// Tiled GEMM (M > 64): 128x128x64, glds-staged, swizzled, double-buffered
// ---------------------------------------------------------------------------
constexpr int TBM = 128, TBN = 128, TBK = 64;
constexpr int TILE_BYTES = TBM * TBK * 2;  // 16 KiB per operand tile
constexpr int CT_LD = TBN + 4;              // epilogue fp32 C tile row stride (bank skew)
constexpr int SMEM_TILED = TBM * CT_LD * 4 > 4 * TILE_BYTES ? TBM * CT_LD * 4 : 4 * TILE_BYTES;

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void gbl_cvoid;

// Stage a [128 rows][64 k] bf16 tile: LDS image is row-major 128-B rows with
// the 16-B chunk index XOR-swizzled by (row>>1)&7.  glds writes lane-linear
// (base + 16*lane), so the swizzle goes on the per-lane SOURCE address and the
// same XOR is applied on the read (guide §5.4 rule 21).
// kStageBL: the 4- and 8-wave decode / tiled stagers (stage_tile, stage8) issue buffer_load ...
// lds from a wave-uniform resource at (row0, k0) with 32-bit lane offsets instead of
// global_load_lds with 64-bit lane addresses (-DLSD_GLDS_GLOBAL restores the latter for A/B).
#ifdef LSD_GLDS_GLOBAL
constexpr bool kStageBL = false;
#else
constexpr bool kStageBL = false;
#endif

template <int ROWS = TBM, bool BL = kStageBL>
__device__ __forceinline__ void stage_tile(char* lds_tile, const bf16* src, long ld, int row0,
                                           int row_max, int k0) {
  const int lane = lane_id(), w = threadIdx.x >> 6;
  constexpr int PER_WAVE = ROWS / 32;  // wave-instructions of 1 KiB (8 rows of 64 k) per wave
  if constexpr (BL) {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(src + (long)row0 * ld + k0), 0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int q = 0; q < PER_WAVE; ++q) {
      const int inst = w * PER_WAVE + q;
      const int row = inst * 8 + (lane >> 3);
      const int lch = (lane & 7) ^ ((row >> 1) & 7);
      const int off = ((min(row0 + row, row_max) - row0) * (int)ld + lch * 8) * 2;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(lds_tile + inst * 1024), 16, off, 0, 0, 0);
    }
    return;
  }
#pragma unroll
  for (int q = 0; q < PER_WAVE; ++q) {
    const int inst = w * PER_WAVE + q;
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

// Store loop of an fp32 [TM][TN + 4] C tile in LDS: NT threads, one 8-column
// row chunk each per pass, 16-byte global stores (epilogue8).
template <int EPI, int TN, int TM, int NT>
__device__ __forceinline__ void ct_store(const GemmParams& p, const float* ct, int m0, int n0, int split) {
  constexpr int CLD = TN + 4;
  constexpr int CPR = TN / 8;  // 8-column chunks per row
  if constexpr (EPI != EPI_SILU_MUL) {
    store_pass<EPI, (TM * CPR + NT - 1) / NT, NT>(p, TM * CPR, split, [&](int c, int& m, int& n, const float*& src) {
      const int row = c / CPR;
      m = m0 + row;
      n = n0 + (c % CPR) * 8;
      src = ct + row * CLD + (c % CPR) * 8;
      return m < p.M && n < p.N;
    });
    return;
  }
  for (int c = threadIdx.x; c < TM * CPR; c += NT) {
    const int row = c / CPR, n = n0 + (c % CPR) * 8, m = m0 + row;
    if (m >= p.M || n >= p.N) continue;
    const float* src = ct + row * CLD + (c % CPR) * 8;
    const f32x4 lo = *reinterpret_cast<const f32x4*>(src);
    const f32x4 hi = *reinterpret_cast<const f32x4*>(src + 4);
    float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    if constexpr (EPI == EPI_SILU_MUL) {
      // interleaved [gate16 | up16] 32-column blocks: gate chunks pair with
      // the up chunk 16 columns right, in the same tile
      if ((c & 3) >= 2) continue;
      const float* up = src + 16;
      const f32x4 ulo = *reinterpret_cast<const f32x4*>(up);
      const f32x4 uhi = *reinterpret_cast<const f32x4*>(up + 4);
      const float u[8] = {ulo[0], ulo[1], ulo[2], ulo[3], uhi[0], uhi[1], uhi[2], uhi[3]};
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = f2bf(silu(v[e]) * u[e]);
      st8(reinterpret_cast<bf16*>(p.out) + (long)m * p.ldo + (n >> 5) * 16 + (n & 15), o);
    } else {
      epilogue8<EPI>(p, m, n, v, split);
    }
  }
}

// Epilogue through LDS (free after the main loop's last barrier): the MFMA C
// layout gives each lane 4 rows x 1 column, i.e. 2-4-byte scattered stores;
// transposing the 128x128 fp32 tile through LDS turns every global store
// into a 16-byte row-contiguous vector (256 B per 16 lanes).
// TN = tile columns (128, or 64 for the narrow ring tiles); wave (wm, wn)
// holds rows wm*64 + [0, 64) and columns wn*TN/2 + [0, TN/2).
template <int EPI, int TN = TBN, int MI = 4>
__device__ __forceinline__ void tiled_epilogue(const GemmParams& p, f32x4 (&acc)[MI][TN / 32], char* smem,
                                               int m0, int n0, int split, int wm, int wn, int r,
                                               int g) {
  constexpr int CLD = TN + 4;  // bank skew
  constexpr int TM = 32 * MI;  // tile rows (wave rows of 16 * MI)
  float* ct = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < TN / 32; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q)
        ct[(wm * 16 * MI + i * 16 + 4 * g + q) * CLD + wn * (TN / 2) + j * 16 + r] = acc[i][j][q];
  __syncthreads();
  ct_store<EPI, TN, TM, 256>(p, ct, m0, n0, split);
}

template <int EPI>
__global__ __launch_bounds__(256) void gemm_tiled_kernel(GemmParams p, int tiles_m, int tiles_n) {
  __shared__ __attribute__((aligned(16))) char smem[SMEM_TILED];  // [buf][A|W]; then C tile
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

  tiled_epilogue<EPI>(p, acc, smem, m0, n0, split, wm, wn, r, g);
}

// Ring variant of the tiled kernel (decode-sized M, few tiles): the
// two-buffer loop above drains every LDS-DMA at each __syncthreads, so one
// k-step of MFMAs (~512 cycles) is all that covers a load's latency.  Here a
// ring of SLOTS k-steps keeps SLOTS-1 in flight while step kt computes:
// counted `s_waitcnt vmcnt` retires only this thread's step-kt loads (LPS glds
// per step: 4 A + TN/32 W), one raw s_barrier per step publishes them AND
// proves every wave finished step kt-1, whose slot is then refilled (guide §5
// "Pipelining across barriers").  Tiles are 128 x TN (TN = 128, or 64: twice
// the workgroups on the under-filled decode grids; 4 waves of 64 x TN/2).
// 3 slots of 24 KiB (TN = 64) / 32 KiB (TN = 128).  Measured at 256 rows
// (tools/microbench.py tiled3, GPT-2 XL): QKV 25.8 (double buffer) -> 20.5
// (ring, 128 x 128) -> 15.6 us (ring, 128 x 64); MLP-up 29.4 -> 23.5 -> 17.3 us;
// split-K decode kernel 23.3 / 26.2 us, hipBLASLt 19.3 / 20.0 us.
template <int SLOTS, int TN, int TM = TBM>
constexpr int smem_ring() {
  return TM * (TN + 4) * 4 > SLOTS * (TM + TN) * TBK * 2 ? TM * (TN + 4) * 4 : SLOTS * (TM + TN) * TBK * 2;
}


// MI = 16-row MFMA tiles per wave: 4 (128-row tiles) or 3 (96-row tiles: a
// 256-row decode GEMM as 3 row tiles -- 3/4 of the A bytes per workgroup
// where 3 x the column tiles still fit the chip in one round).
template <int EPI, int SLOTS, int TN, int MI = 4>
__global__ __launch_bounds__(256) void gemm_ring_kernel(GemmParams p, int tiles_m, int tiles_n) {
  constexpr int D = SLOTS - 1;                    // prefetch distance (k-steps in flight)
  constexpr int JT = TN / 32;                     // 16-column MFMA tiles per wave
  constexpr int TM = 32 * MI;                     // tile rows
  constexpr int A_BYTES = TM * TBK * 2;
  constexpr int SLOT_BYTES = A_BYTES + TN * TBK * 2;
  constexpr int LPS = MI + TN / 32;               // glds per thread per k-step (A + W)
  __shared__ __attribute__((aligned(16))) char smem[smem_ring<SLOTS, TN, TM>()];  // [slot][A|W]; then C tile
  const int nwg = gridDim.x;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int per_split = tiles_m * tiles_n;
  const int split = bid / per_split;
  const int t = bid % per_split;
  const int tm = t % tiles_m, tn = t / tiles_m;
  const int m0 = tm * TM, n0 = tn * TN;
  const int KT = p.K / TBK;
  const int kb = (int)((long)KT * split / p.splits), ke = (int)((long)KT * (split + 1) / p.splits);

  const int lane = lane_id(), w = threadIdx.x >> 6;
  const int wm = w >> 1, wn = w & 1;
  const int r = lane & 15, g = lane >> 4;

  f32x4 acc[MI][JT];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < JT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int kt, int slot) {
    char* b = smem + slot * SLOT_BYTES;
    stage_tile<TM>(b, p.A, p.lda, m0, p.M - 1, kt * TBK);
    stage_tile<TN>(b + A_BYTES, p.W, p.ldw, n0, p.N - 1, kt * TBK);
  };
  static_assert(SLOTS == 3 || SLOTS == 4, "ring of 3 or 4 slots");
  static_assert(2 * LPS <= 63, "vmcnt holds at most 63 outstanding loads");
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (kb + d < ke) issue(kb + d, d);
  int slot = 0;
  for (int kt = kb; kt < ke; ++kt) {
    const int later = min(D - 1, ke - 1 - kt);  // steps after kt already issued
    if (later >= 2) __builtin_amdgcn_s_waitcnt(vmcnt_imm(2 * LPS));
    else if (later == 1) __builtin_amdgcn_s_waitcnt(vmcnt_imm(LPS));
    else __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));
    __builtin_amdgcn_s_barrier();
    if (kt + D < ke) issue(kt + D, slot == 0 ? SLOTS - 1 : slot - 1);
    const char* ta = smem + slot * SLOT_BYTES;
    const char* tw = ta + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[MI], wf[JT];
#pragma unroll
      for (int i = 0; i < MI; ++i) af[i] = lds_frag(ta, wm * 16 * MI + i * 16 + r, kk * 4 + g);
#pragma unroll
      for (int j = 0; j < JT; ++j) wf[j] = lds_frag(tw, wn * (TN / 2) + j * 16 + r, kk * 4 + g);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < JT; ++j) acc[i][j] = mfma16(af[i], wf[j], acc[i][j]);
    }
    slot = slot == SLOTS - 1 ? 0 : slot + 1;
  }
  __syncthreads();  // every wave's fragment reads retired before the C tile overwrites the slots
  tiled_epilogue<EPI, TN, MI>(p, acc, smem, m0, n0, split, wm, wn, r, g);
}

// Stage a [ROWS][64 k] tile (the lds_frag image) with NWAVES waves sharing
// the ROWS / 8 wave-instructions; `wi` = this wave's index among them.
// BL: buffer_load ... lds from a wave-uniform resource at (row0, k0) with 32-bit lane
// offsets instead of global_load_lds with 64-bit lane addresses (fewer issue cycles
// per DMA instruction: prefill GEMM +6-25 %, profiles/r3_p8_buffer_lds.log).
template <int ROWS, int NWAVES, int AUX = 0, bool BL = false>
__device__ __forceinline__ void stage_rows(char* lds_tile, const bf16* src, long ld, int row0, int row_max,
                                           int k0, int wi) {
  const int lane = lane_id();
  constexpr int PER_WAVE = ROWS / 8 / NWAVES;
  static_assert(PER_WAVE * 8 * NWAVES == ROWS, "rows split evenly over the loading waves");
  if constexpr (BL) {
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(src + (long)row0 * ld + k0), 0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int q = 0; q < PER_WAVE; ++q) {
      const int inst = wi * PER_WAVE + q;
      const int row = inst * 8 + (lane >> 3);
      const int lch = (lane & 7) ^ ((row >> 1) & 7);
      const int off = ((min(row0 + row, row_max) - row0) * (int)ld + lch * 8) * 2;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(lds_tile + inst * 1024), 16, off, 0, 0, AUX);
    }
    return;
  }
#pragma unroll
  for (int q = 0; q < PER_WAVE; ++q) {
    const int inst = wi * PER_WAVE + q;
    const int row = inst * 8 + (lane >> 3);
    const int lch = (lane & 7) ^ ((row >> 1) & 7);
    const bf16* gp = src + (long)min(row0 + row, row_max) * ld + k0 + lch * 8;
    __builtin_amdgcn_global_load_lds((gbl_cvoid*)gp, (lds_void*)(lds_tile + inst * 1024), 16, 0, AUX);
  }
}

// Stage the same [ROWS][64 k] image from a k-block-packed operand
// [K/64][M][64] (activations: every row's 64-k slice of block kb contiguous,
// rows consecutive -> a tile's k-step is ROWS x 128 B contiguous) or
// [N/64][K/64][64][64] (weights: one 8 KiB block per 64 rows x 64 k).  Each
// wave-instruction then reads 1 KiB of consecutive bytes (A/B experiment:
// the row-strided image reads 8 rows x 128 B at a K x 2 B pitch).
template <int ROWS, int NWAVES, int WPACK>
__device__ __forceinline__ void stage_rows_packed(char* lds_tile, const bf16* src, int rows_total, int KB,
                                                  int row0, int row_max, int kb, int wi) {
  const int lane = lane_id();
  constexpr int PER_WAVE = ROWS / 8 / NWAVES;
#pragma unroll
  for (int q = 0; q < PER_WAVE; ++q) {
    const int inst = wi * PER_WAVE + q;
    const int row = inst * 8 + (lane >> 3);
    const int lch = (lane & 7) ^ ((row >> 1) & 7);
    const int r = min(row0 + row, row_max);
    const bf16* gp = WPACK ? src + (((long)(r >> 6) * KB + kb) << 12) + (r & 63) * 64 + lch * 8
                           : src + ((long)kb * rows_total + r) * 64 + lch * 8;
    __builtin_amdgcn_global_load_lds((gbl_cvoid*)gp, (lds_void*)(lds_tile + inst * 1024), 16, 0, 0);
  }
}

// 8-wave variant of the 128x64 decode ring (512 threads, same tiles, same
// 3-slot ring, same grid).  In the 4-wave ring every wave issues its 6 LDS-DMA
// instructions per k-step (each ~60-185 issue cycles beside MFMAs, microarch
// 'LDS-DMA piece issue cost') in the same instruction stream as its 16 MFMAs,
// so a step costs issue + MFMA + reads instead of their max.  Two layouts:
//   VAR 1: waves 0-3 compute (64 x 32 each, as the 4-wave ring) and never touch
//          VMEM; waves 4-7 are loaders (6 glds per step) -- one of each per SIMD;
//   VAR 2: all 8 waves compute 32 x 32 and each issues 3 glds per step.
// One raw s_barrier per k-step publishes step kt's slot (every loader waited
// its own DMAs with a counted vmcnt) and proves step kt-1's slot free.
// A/B knobs: NTW = weights staged non-temporal (aux nt: once-read bytes,
// microarch 'nt-weights'); rot = each tile starts its K loop at a different
// k-step (tile-dependent rotation, fixed per tile, so results stay
// deterministic) so that the workgroups of an XCD do not all read the same
// A k-slice at the same time.
//
// K splits (p.splits > 1): EPI_SLAB writes its partial slab (residual
// projections; the next norm folds the slabs).  Any other epilogue (QKV /
// MLP-up at 129-256 rows, VAR 2 only): every split publishes its fp32
// partial tile write-through (sc1 stores) in a lane-major layout (each
// thread's 16-byte accumulators contiguous across the workgroup: whole-line
// stores and loads), takes an agent-scope ticket, and the last-arriving split
// reloads the other partials (sc1 loads) and sums all S in split order
// (deterministic) before the fused epilogue (guide §5 "In-launch split-K
// reduction", sc1 form: no release / acquire fences).
// Measured and removed (round 5): a W-line L2 prefetch, one extra 4-byte-per-lane
// LDS-DMA touch per k-step of the rows 2-6 k-steps ahead -- 7-16 % slower on every
// GPT-2 XL shape, bench 50.1-50.5k -> 46.5-47.3k (profiles/r5_rejected_ring8_prefetch.log).
template <int EPI, int VAR, int SLOTS, int NTW = 0, int PK = 0, bool BL = kStageBL>
__global__ __launch_bounds__(512) void gemm_ring8_kernel(GemmParams p, int tiles_m, int tiles_n, int rot,
                                                         int* __restrict__ cnt, float* __restrict__ ws) {
  constexpr int D = SLOTS - 1, TN = 64, TM = TBM;
  constexpr int CW = VAR == 1 ? 4 : 8;           // computing waves
  constexpr int LWN = VAR == 1 ? 4 : 8;          // loading waves
  constexpr int MI = TM / 16 / (CW / 2);         // 16-row MFMA tiles per computing wave: 4 / 2
  constexpr int JT = 2;                          // 16-column MFMA tiles per computing wave (32 cols)
  constexpr int A_BYTES = TM * TBK * 2;
  constexpr int SLOT_BYTES = A_BYTES + TN * TBK * 2;
  constexpr int LPS = (TM + TN) / 8 / LWN;      // glds per loading wave per k-step: 6 / 3
  constexpr int CLD = TN + 4;
  constexpr int SMEM = SLOTS * SLOT_BYTES > TM * CLD * 4 ? SLOTS * SLOT_BYTES : TM * CLD * 4;
  static_assert(VAR == 1 || VAR == 2, "ring8 layout");
  static_assert(SLOTS >= 3 && SLOTS <= 5 && (SLOTS - 2) * LPS <= 63, "ring depth / vmcnt range");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];  // [slot][A|W]; then the C tile
  const int nwg = gridDim.x;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int per_split = tiles_m * tiles_n;
  const int split = bid / per_split;
  const int t = bid % per_split;
  const int tm = t % tiles_m, tn = t / tiles_m;
  const int m0 = tm * TM, n0 = tn * TN;
  const int KT = p.K / TBK;
  const int kb = (int)((long)KT * split / p.splits), ke = (int)((long)KT * (split + 1) / p.splits);

  const int lane = lane_id(), w = threadIdx.x >> 6;
  const bool loader = VAR == 2 || w >= 4;
  const bool compute = VAR == 2 || w < 4;
  const int lw = VAR == 1 ? w - 4 : w;
  const int wm = (w & (CW - 1)) >> 1, wn = w & 1;
  const int r = lane & 15, g = lane >> 4;

  f32x4 acc[MI][JT];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < JT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = ke - kb, r0 = rot && nk > 0 ? (t * 7) % nk : 0;
  auto issue = [&](int kt, int slot) {
    char* b = smem + slot * SLOT_BYTES;
    int k = kt - kb + r0;
    k = kb + (k >= nk ? k - nk : k);
    if constexpr (PK & 2) stage_rows_packed<TM, LWN, 0>(b, p.A, p.M, p.K / 64, m0, p.M - 1, k, lw);
    else stage_rows<TM, LWN, 0, BL>(b, p.A, p.lda, m0, p.M - 1, k * TBK, lw);
    if constexpr (PK & 1) stage_rows_packed<TN, LWN, 1>(b + A_BYTES, p.W, p.N, p.K / 64, n0, p.N - 1, k, lw);
    else stage_rows<TN, LWN, NTW ? 2 : 0, BL>(b + A_BYTES, p.W, p.ldw, n0, p.N - 1, k * TBK, lw);
  };
  if (loader) {
#pragma unroll
    for (int d = 0; d < D; ++d)
      if (kb + d < ke) issue(kb + d, d);
  }
  int slot = 0;
  for (int kt = kb; kt < ke; ++kt) {
    if (loader) {  // this wave's DMAs of step kt landed; the later issued steps stay in flight
      const int later = min(D - 1, ke - 1 - kt);
      if (D >= 4 && later >= 3) __builtin_amdgcn_s_waitcnt(vmcnt_imm(3 * LPS));
      else if (D >= 3 && later == 2) __builtin_amdgcn_s_waitcnt(vmcnt_imm(2 * LPS));
      else if (later == 1) __builtin_amdgcn_s_waitcnt(vmcnt_imm(LPS));
      else __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));
    }
    __builtin_amdgcn_s_barrier();
    if (loader && kt + D < ke) issue(kt + D, slot == 0 ? SLOTS - 1 : slot - 1);
    if (compute) {
      const char* ta = smem + slot * SLOT_BYTES;
      const char* tw = ta + A_BYTES;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 af[MI], wf[JT];
#pragma unroll
        for (int i = 0; i < MI; ++i) af[i] = lds_frag(ta, wm * 16 * MI + i * 16 + r, kk * 4 + g);
#pragma unroll
        for (int j = 0; j < JT; ++j) wf[j] = lds_frag(tw, wn * 32 + j * 16 + r, kk * 4 + g);
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < JT; ++j) acc[i][j] = mfma16(af[i], wf[j], acc[i][j]);
      }
    }
    slot = slot == SLOTS - 1 ? 0 : slot + 1;
  }
  __syncthreads();  // fragment reads retired (and no DMA pending) before the C tile overwrites the slots
  if constexpr (VAR == 2 && EPI != EPI_SLAB) {
    const int S = p.splits;
    if (S > 1) {
      constexpr int PER = MI * JT * 512;  // f32x4 per split tile
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          ws + (long)t * S * PER * 4, (short)0, S * PER * 16, 0x00020000);
      const int toff = threadIdx.x * 16;
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < JT; ++j)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs,
                                                 split * PER * 16 + (i * JT + j) * 8192 + toff, 0, 16);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      int* s_flag = reinterpret_cast<int*>(smem);
      if (threadIdx.x == 0) {
        const int tk = __hip_atomic_fetch_add(cnt + t, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *s_flag = (tk == S - 1);
        if (tk == S - 1) __hip_atomic_store(cnt + t, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      if (*s_flag == 0) return;
      __syncthreads();  // every wave has read the flag before the C tile overwrites it
      // every partial of a group in flight before the adds (its own one too:
      // no per-load register-or-load select); clamped split index x 0/1 mask,
      // no per-load branch (guide §5 trap (c))
      constexpr int RG = 4;
      f32x4 sum[MI][JT];
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < JT; ++j) sum[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      for (int s0 = 0; s0 < S; s0 += RG) {
        f32x4 v[RG][MI][JT];
#pragma unroll
        for (int u = 0; u < RG; ++u) {
          const int s2 = min(s0 + u, S - 1);
#pragma unroll
          for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < JT; ++j)
              v[u][i][j] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                  rs, s2 * PER * 16 + (i * JT + j) * 8192 + toff, 0, 16));
        }
#pragma unroll
        for (int u = 0; u < RG; ++u) {
          const float msk = (s0 + u < S) ? 1.f : 0.f;
#pragma unroll
          for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < JT; ++j) sum[i][j] += v[u][i][j] * msk;
        }
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < JT; ++j) acc[i][j] = sum[i][j];
    }
  }
  float* ct = reinterpret_cast<float*>(smem);
  if (compute) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < JT; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          ct[(wm * 16 * MI + i * 16 + 4 * g + q) * CLD + wn * 32 + j * 16 + r] = acc[i][j][q];
  }
  __syncthreads();
  ct_store<EPI, TN, TM, 512>(p, ct, m0, n0, split);
}

// ---------------------------------------------------------------------------
// Large GEMM (prefill, M >= 256): 256x256 tile, 8 waves (2 M x 4 N, 128x64
// per wave), 4-slot LDS ring of BK=32 k-steps, fragments double-buffered in
// registers across the barrier
// ---------------------------------------------------------------------------
// The 128x128 kernel above is the "two-barrier" structure: its __syncthreads
// drains every LDS-DMA (vmcnt(0)) each k-step, and after each barrier every
// wave stalls on its first ds_read before the MFMAs restart.  Here all LDS is
// one array holding a ring of 4 slots of [256 rows][32 k] for A and W
// (32 KiB per slot, 128 KiB, 1 block/CU).  Iteration s:
//   * counted `s_waitcnt vmcnt(4|0)` retires this thread's glds of step s+1
//     (step s+2's stay in flight), raw s_barrier publishes them to all waves;
//   * glds of step s+3 into the slot step s-1 used (WAR-safe: that slot's
//     fragments were read in iteration s-2 and consumed by MFMAs before this
//     barrier);
//   * 12 ds_read_b128 of step s+1's fragments into the idle register set;
//   * 32 MFMAs of step s from the register set read one iteration earlier --
//     they never wait on LDS, the reads above complete under them.
// No other VMEM op sits in the loop, so the vmcnt counts are exact (guide §5
// "Pipelining across barriers", traps 4(a)/(b)).
//
// LDS image per operand per slot: 64-B rows (32 k), the 16-B chunk index
// XOR-swizzled by f((row >> 2) & 3), f = {0, 2, 3, 1}: with the ds_read_b128
// lane groups of CDNA4 ({0-3,12-15,20-27}, {4-11,16-19,28-31}, and +32)
// every group of a fragment read covers 16 distinct 16-B bank slots.  glds
// writes lane-linear, so the swizzle goes on the per-lane source address.
constexpr int GBM = 256, GBN = 256, GBK = 32, GSLOTS = 4;
constexpr int GOP_BYTES = GBM * GBK * 2;           // 16 KiB per operand per slot
constexpr int GSLOT_BYTES = 2 * GOP_BYTES;         // A | W
constexpr int GSMEM = GSLOTS * GSLOT_BYTES;        // 128 KiB (== 256 x 128 fp32 C half-tile)

// s_waitcnt simm16 (gfx9 layout): vmcnt[3:0]+[15:14]=63, expcnt[6:4]=7, lgkmcnt[11:8]=0
constexpr int LGKM0 = 0xC07F;

// A/B knob (guide §5.5 T5): s_setprio(1) around the MFMA clusters
#ifdef LSD_BIG_PRIO
#define LSD_PRIO(v) __builtin_amdgcn_s_setprio(v)
#else
#define LSD_PRIO(v) ((void)0)
#endif

__device__ __forceinline__ int big_swz(int q) { return (0x78 >> (2 * q)) & 3; }

__device__ __forceinline__ void stage_big(char* lds, const bf16* src, long ld, int row0, int row_max,
                                          int k0) {
  const int lane = lane_id(), w = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int inst = w * 2 + q;                  // 16 instructions x 1 KiB = 16 rows x 64 B each
    const int row = inst * 16 + (lane >> 2);
    const int lch = (lane & 3) ^ big_swz((lane >> 4) & 3);  // (row >> 2) & 3 == (lane >> 4) & 3
    const bf16* gp = src + (long)min(row0 + row, row_max) * ld + k0 + lch * 8;
    __builtin_amdgcn_global_load_lds((gbl_cvoid*)gp, (lds_void*)(lds + inst * 1024), 16, 0, 0);
  }
}

__device__ __forceinline__ bf16x8 lds_frag_big(const char* op, int row, int g) {
  return *reinterpret_cast<const bf16x8*>(op + row * 64 + ((g ^ big_swz((row >> 2) & 3)) << 4));
}

// Tile order of the large GEMMs.  G = 0: M-fastest (consecutive workgroups
// share a W panel).  G > 0: groups of G row panels, M-fastest inside a group
// and the group's column panels in turn -- the tiles in flight at once (the
// XCD-contiguous ranges of xcd_remap) then cover a few row panels instead of
// sweeping every row panel per column panel, so each A panel is read from
// HBM about once instead of once per column tile.
__device__ __forceinline__ void tile_order(int t, int tiles_m, int tiles_n, int G, int& tm, int& tn) {
  if (G <= 0) {
    tm = t % tiles_m;
    tn = t / tiles_m;
    return;
  }
  const int gsz = G * tiles_n, grp = t / gsz, idx = t % gsz;
  const int gm = min(G, tiles_m - grp * G);
  tm = grp * G + idx % gm;
  tn = idx / gm;
}

template <int EPI>
__global__ __launch_bounds__(512) void gemm_big_kernel(GemmParams p, int tiles_m, int tiles_n, int G) {
  __shared__ __attribute__((aligned(16))) char smem[GSMEM];
  const int nwg = gridDim.x;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int per_split = tiles_m * tiles_n;
  const int split = bid / per_split;
  const int t = bid % per_split;
  int tm, tn;
  tile_order(t, tiles_m, tiles_n, G, tm, tn);
  const int m0 = tm * GBM, n0 = tn * GBN;
  const int KT = p.K / 64;  // split boundaries in 64-deep units: ns is even
  const int kb = 2 * (int)((long)KT * split / p.splits);
  const int ns = 2 * (int)((long)KT * (split + 1) / p.splits) - kb;

  const int lane = lane_id(), w = threadIdx.x >> 6;
  const int wr = w >> 2, wc = w & 3;
  const int r = lane & 15, g = lane >> 4;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto stage = [&](int step) {
    char* slot = smem + (step & (GSLOTS - 1)) * GSLOT_BYTES;
    const int k0 = (kb + step) * GBK;
    stage_big(slot, p.A, p.lda, m0, p.M - 1, k0);
    stage_big(slot + GOP_BYTES, p.W, p.ldw, n0, p.N - 1, k0);
  };
  auto frag_a = [&](int step, int i) {
    return lds_frag_big(smem + (step & (GSLOTS - 1)) * GSLOT_BYTES, wr * 128 + i * 16 + r, g);
  };
  auto frag_w = [&](int step, int j) {
    return lds_frag_big(smem + (step & (GSLOTS - 1)) * GSLOT_BYTES + GOP_BYTES, wc * 64 + j * 16 + r, g);
  };
  // wait for this thread's glds of `step`; steps after it stay in flight
  auto wait_step = [&](int step) {
    if (step + 1 < ns) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  // One k-step of MFMAs from (ac, wcur) while the next step's fragments are
  // read into (an, wn): W and A rows 0-3 first, A rows 4-7 once the current
  // A rows 0-3 are dead (keeps the live set at acc + 48 + 32 VGPRs).
  auto step_mma = [&](int s, bf16x8 (&ac)[8], bf16x8 (&wcur)[4], bf16x8 (&an)[8], bf16x8 (&wn)[4]) {
    // The next-step reads are unconditional (on the last step they read a
    // stale slot and are discarded): a conditional register load would keep
    // the old fragment set live through the loop and spill the accumulators.
    if (s + 1 < ns) {
      wait_step(s + 1);
      if (s + 3 < ns) stage(s + 3);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) wn[j] = frag_w(s + 1, j);
#pragma unroll
    for (int i = 0; i < 4; ++i) an[i] = frag_a(s + 1, i);
    // sched_barrier(0): keep the phase order as written -- hipcc otherwise
    // hoists every read above the MFMAs and spills the accumulators
    __builtin_amdgcn_sched_barrier(0);
    LSD_PRIO(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(ac[i], wcur[j], acc[i][j]);
    LSD_PRIO(0);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 4; i < 8; ++i) an[i] = frag_a(s + 1, i);
    __builtin_amdgcn_sched_barrier(0);
    LSD_PRIO(1);
#pragma unroll
    for (int i = 4; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(ac[i], wcur[j], acc[i][j]);
    LSD_PRIO(0);
    __builtin_amdgcn_sched_barrier(0);
    // Retire the next set's reads (long done under the 32 MFMAs) with a real
    // S_WAITCNT the waitcnt pass understands: the loop header then carries no
    // pending LDS reads and the next step's MFMAs issue without the
    // conservative lgkmcnt(0) hipcc otherwise puts in front of them.
    __builtin_amdgcn_s_waitcnt(LGKM0);
  };

  bf16x8 a0[8], w0[4], a1[8], w1[4];
  if (ns > 0) {
#pragma unroll
    for (int q = 0; q < GSLOTS - 1; ++q)
      if (q < ns) stage(q);
    // step 0 landed: steps 1, 2 may be in flight
    if (ns >= 3) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (ns == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#pragma unroll
    for (int j = 0; j < 4; ++j) w0[j] = frag_w(0, j);
#pragma unroll
    for (int i = 0; i < 8; ++i) a0[i] = frag_a(0, i);
    __builtin_amdgcn_s_waitcnt(LGKM0);
  }
  // ns is even (splits partition K in 64-deep units): two steps per trip,
  // the register sets swap roles without copies.
  for (int s = 0; s < ns; s += 2) {
    step_mma(s, a0, w0, a1, w1);
    step_mma(s + 1, a1, w1, a0, w0);
  }

  // Epilogue: two passes over 128-column halves of the C tile, staged as fp32
  // [256][128] in LDS (chunks of 16 floats XOR-swizzled by (row >> 2) & 3 so
  // the MFMA-layout writes -- 4 rows x 16 columns per instruction -- hit
  // distinct banks), then 16-byte row-contiguous epilogue8 stores.
  float* ct = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    // pass 0: every DMA landed before C overwrites the ring; pass 1: only the
    // LDS reads of pass 0 (its stores stay in flight)
    if (h == 0) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    if ((wc >> 1) == h) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int row = wr * 128 + i * 16 + 4 * g + q;
            const int col = (wc & 1) * 64 + j * 16 + r;
            ct[row * 128 + (col ^ (((row >> 2) & 3) << 4))] = acc[i][j][q];
          }
    }
    __syncthreads();
    if constexpr (EPI != EPI_SILU_MUL) {
      store_pass<EPI, GBM * 16 / 512, 512>(p, GBM * 16, split, [&](int c, int& m, int& n, const float*& src) {
        const int row = c >> 4, ch = c & 15;
        m = m0 + row;
        n = n0 + h * 128 + ch * 8;
        src = ct + row * 128 + ((ch * 8) ^ (((row >> 2) & 3) << 4));
        return m < p.M && n < p.N;
      });
      continue;
    }
    for (int c = threadIdx.x; c < GBM * 16; c += 512) {
      const int row = c >> 4, ch = c & 15, m = m0 + row, n = n0 + h * 128 + ch * 8;
      if (m >= p.M || n >= p.N) continue;
      const float* src = ct + row * 128 + ((ch * 8) ^ (((row >> 2) & 3) << 4));
      const f32x4 lo = *reinterpret_cast<const f32x4*>(src);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(src + 4);
      float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      if constexpr (EPI == EPI_SILU_MUL) {
        if ((ch & 3) >= 2) continue;  // up chunks are read by their gate chunk
        const float* up = ct + row * 128 + (((ch + 2) * 8) ^ (((row >> 2) & 3) << 4));
        const f32x4 ulo = *reinterpret_cast<const f32x4*>(up);
        const f32x4 uhi = *reinterpret_cast<const f32x4*>(up + 4);
        const float u[8] = {ulo[0], ulo[1], ulo[2], ulo[3], uhi[0], uhi[1], uhi[2], uhi[3]};
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = f2bf(silu(v[e]) * u[e]);
        st8(reinterpret_cast<bf16*>(p.out) + (long)m * p.ldo + (n >> 5) * 16 + (n & 15), o);
      } else {
        epilogue8<EPI>(p, m, n, v, split);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Large GEMM, phase-pipelined (prefill): 256x256 tile, BK = 64, 8 waves,
// two LDS buffers of four 16 KiB half-tiles, one glds half-tile per phase
// ---------------------------------------------------------------------------
// A K-tile t (64 deep) is held as four half-tiles in buffer t & 1:
//   A0 = A rows m0 + [0, 128), A1 = A rows m0 + [128, 256),
//   B0 = W rows n0 + [0, 128), B1 = W rows n0 + [128, 256),
// each [128 rows][64 k] with 128-B rows, 16-B chunks XOR-swizzled by
// (row >> 1) & 7 (the 128x128 kernel's conflict-free fragment image).
// Wave (wr, wc) owns four 64 x 32 output blocks, one per (A half, B half):
// rows mh * 128 + wr * 64 + [0, 64), columns nh * 128 + wc * 32 + [0, 32).
// Each K-tile is four phases, one output quadrant (A half mh, B half nh) of
// 16 MFMAs each, in the order (0,0) (0,1) (1,1) (1,0):
//   phase  reads (ds_read_b128)       stages (glds, 2 per thread)  waits
//   q0     A0 frags (8) + B0 frags (4)  B1 of tile t+1
//   q1     B1 frags (4)                 A1 of tile t+1               A1(t)
//   q2     A1 frags (8)                 A0 of tile t+2
//   q3     --  (B0 frags kept)          B0 of tile t+2               A0/B0/B1(t+1)
// so every half-tile is restaged >= 2 phases after its last read (A0 read
// q0 -> restaged q2, B0 q0 -> q3, B1 q1 -> q0 next, A1 q2 -> q1 next) and is
// issued 5-6 phases before it is read; the counted vmcnt waits (q1: 4
// later halves in flight, q3: 3) always sit one phase before the first read
// of what they retire.  Phase body: reads, stage, wait, s_barrier,
// lgkmcnt(0), 16 MFMAs, s_barrier.  The two wave rows run staggered by one
// barrier (wr = 1 takes an extra barrier up front, wr = 0 one at the end), so
// on every SIMD one wave issues its LDS reads and DMA while the other runs
// MFMAs (guide §5 "The 256^2 8-phase template").  All LDS is one array;
// the epilogue reuses it as the fp32 C tile.
constexpr int P8_HALF = 128 * 64 * 2;  // 16 KiB
constexpr int P8_BUF = 4 * P8_HALF;    // A0 A1 B0 B1
constexpr int P8_SMEM = 2 * P8_BUF;    // 128 KiB (== 256 x 128 fp32 C half-tile)

template <bool BUF = false>
__device__ __forceinline__ void p8_stage(char* lds, const bf16* src, long ld, int row0, int row_max,
                                         int k0) {
  const int lane = lane_id(), w = threadIdx.x >> 6;
  if constexpr (BUF) {
    // buffer_load ... lds: a wave-uniform resource at (row0, k0) and 32-bit lane offsets
    // (one address VGPR per lane instead of a 64-bit global address)
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(src + (long)row0 * ld + k0), 0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int inst = w * 2 + q;
      const int row = inst * 8 + (lane >> 3);
      const int lch = (lane & 7) ^ ((row >> 1) & 7);
      const int off = ((min(row0 + row, row_max) - row0) * (int)ld + lch * 8) * 2;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(lds + inst * 1024), 16, off, 0, 0, 0);
    }
    return;
  }
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int inst = w * 2 + q;  // 16 x 1 KiB = 128 rows of 128 B
    const int row = inst * 8 + (lane >> 3);
    const int lch = (lane & 7) ^ ((row >> 1) & 7);
    const bf16* gp = src + (long)min(row0 + row, row_max) * ld + k0 + lch * 8;
    __builtin_amdgcn_global_load_lds((gbl_cvoid*)gp, (lds_void*)(lds + inst * 1024), 16, 0, 0);
  }
}

// VAR 4 (default, gemm_set_big_kind 4): stage with buffer_load ... lds (wave-uniform
// resource, 32-bit lane offsets) instead of global_load_lds with 64-bit lane addresses;
// VAR 0 = kind 1.  Issuing each phase's DMA before its fragment reads, B fragments first
// and a peeled k-loop were measured and removed (profiles/r3_p8_buffer_lds.log,
// r3_rejected_p8_peeled_loop.log).
template <int EPI, int VAR = 0>
__global__ __launch_bounds__(512) void gemm_p8_kernel(GemmParams p, int tiles_m, int tiles_n, int G) {
  __shared__ __attribute__((aligned(16))) char smem[P8_SMEM];
  const int nwg = gridDim.x;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int per_split = tiles_m * tiles_n;
  const int split = bid / per_split;
  int tm, tn;
  tile_order(bid % per_split, tiles_m, tiles_n, G, tm, tn);
  const int m0 = tm * 256, n0 = tn * 256;
  LSD_STAMP(0)
  const int KT = p.K / 64;
  const int kb = (int)((long)KT * split / p.splits);
  const int T = (int)((long)KT * (split + 1) / p.splits) - kb;  // K-tiles of this split

  const int lane = lane_id(), w = threadIdx.x >> 6;
  const int wr = w >> 2, wc = w & 3;
  const int r = lane & 15, g = lane >> 4;

  f32x4 acc[8][4];  // [mh * 4 + i][nh * 2 + j]
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // half h of K-tile t: 0 = A0, 1 = A1, 2 = B0, 3 = B1
  auto stage = [&](int t, int h) {
    char* dst = smem + (t & 1) * P8_BUF + h * P8_HALF;
    const int k0 = (kb + t) * 64;
    if (h < 2) p8_stage<(VAR & 4) != 0>(dst, p.A, p.lda, m0 + h * 128, p.M - 1, k0);
    else p8_stage<(VAR & 4) != 0>(dst, p.W, p.ldw, n0 + (h - 2) * 128, p.N - 1, k0);
  };
  bf16x8 af[4][2], b0[2][2], b1[2][2];
  auto read_a = [&](int t, int mh) {
    const char* src = smem + (t & 1) * P8_BUF + mh * P8_HALF;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) af[i][kk] = lds_frag(src, wr * 64 + i * 16 + r, kk * 4 + g);
  };
  auto read_b = [&](int t, int nh, bf16x8 (&bf)[2][2]) {
    const char* src = smem + (t & 1) * P8_BUF + (2 + nh) * P8_HALF;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) bf[j][kk] = lds_frag(src, wc * 32 + j * 16 + r, kk * 4 + g);
  };
#ifdef LSD_P8_PROF
  // diagnostic build only (LSD_HIPCC_FLAGS=-DLSD_P8_PROF): wave 0's cycles in
  // the loop, in the counted vmcnt waits and in the two barriers of a phase
  long long pf_t0 = 0, pf_vm = 0, pf_b1 = 0, pf_b2 = 0, pf_c = 0;
#define P8_T() __builtin_amdgcn_s_memtime()
#define P8_ACC(acc, stmt) { pf_c = P8_T(); stmt; acc += P8_T() - pf_c; }
#else
#define P8_ACC(acc, stmt) stmt;
#endif
  auto mma = [&](int mh, int nh, bf16x8 (&bf)[2][2]) {
    P8_ACC(pf_b1, __builtin_amdgcn_s_barrier())
    __builtin_amdgcn_s_waitcnt(LGKM0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[mh * 4 + i][nh * 2 + j] = mfma16(af[i][kk], bf[j][kk], acc[mh * 4 + i][nh * 2 + j]);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    P8_ACC(pf_b2, __builtin_amdgcn_s_barrier())
  };

  if (T > 0) {
    // prologue: all of tile 0, then A0 / B0 of tile 1; tile 0 published
    stage(0, 0);
    stage(0, 2);
    stage(0, 3);
    stage(0, 1);
    if (T > 1) {
      stage(1, 0);
      stage(1, 2);
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    LSD_STAMP(1)
    if (wr == 1) __builtin_amdgcn_s_barrier();  // stagger the wave rows by one barrier

#ifdef LSD_P8_PROF
    pf_t0 = P8_T();
#endif
    for (int t = 0; t < T; ++t) {
      const bool n1 = t + 1 < T, n2 = t + 2 < T;
      // q0: (A0, B0)
      read_a(t, 0);
      read_b(t, 0, b0);
      if (n1) stage(t + 1, 3);
      __builtin_amdgcn_sched_barrier(0);
      mma(0, 0, b0);
      // q1: (A0, B1); retire A1(t): 4 later halves in flight when t + 1 exists
      read_b(t, 1, b1);
      if (n1) stage(t + 1, 1);
      P8_ACC(pf_vm, if (n1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory"))
      __builtin_amdgcn_sched_barrier(0);
      mma(0, 1, b1);
      // q2: (A1, B1)
      read_a(t, 1);
      if (n2) stage(t + 2, 0);
      __builtin_amdgcn_sched_barrier(0);
      mma(1, 1, b1);
      // q3: (A1, B0); retire A0 / B0 / B1 of t + 1 (A1(t+1), A0 / B0(t+2) stay in flight)
      if (n2) stage(t + 2, 2);
      P8_ACC(pf_vm, if (n2) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
                    else if (n1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory"))
      __builtin_amdgcn_sched_barrier(0);
      mma(1, 0, b0);
    }
    if (wr == 0) __builtin_amdgcn_s_barrier();  // balance the stagger
#ifdef LSD_P8_PROF
    if (p.stamps && threadIdx.x == 0) {
      long long* ps = p.stamps + (long)blockIdx.x * 8;
      ps[4] = P8_T() - pf_t0;
      ps[5] = pf_vm;
      ps[6] = pf_b1;
      ps[7] = pf_b2;
    }
#endif
  }
#undef P8_ACC
  LSD_STAMP(2)

  // Epilogue: two passes over 128-column halves (nh), the fp32 C half-tile
  // [256][128] staged in LDS (16-float chunks XOR-swizzled by (row >> 2) & 3),
  // then 16-byte row-contiguous epilogue8 stores.
  float* ct = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    // pass 0: every DMA landed before C overwrites the ring; pass 1: only the
    // LDS reads of pass 0 (its stores stay in flight)
    if (h == 0) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int mh = 0; mh < 2; ++mh)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int row = mh * 128 + wr * 64 + i * 16 + 4 * g + q;
            const int col = wc * 32 + j * 16 + r;
            ct[row * 128 + (col ^ (((row >> 2) & 3) << 4))] = acc[mh * 4 + i][h * 2 + j][q];
          }
    __syncthreads();
    if constexpr (EPI != EPI_SILU_MUL) {
      store_pass<EPI, 256 * 16 / 512, 512>(p, 256 * 16, split, [&](int c, int& m, int& n, const float*& src) {
        const int row = c >> 4, ch = c & 15;
        m = m0 + row;
        n = n0 + h * 128 + ch * 8;
        src = ct + row * 128 + ((ch * 8) ^ (((row >> 2) & 3) << 4));
        return m < p.M && n < p.N;
      });
      continue;
    }
    for (int c = threadIdx.x; c < 256 * 16; c += 512) {
      const int row = c >> 4, ch = c & 15, m = m0 + row, n = n0 + h * 128 + ch * 8;
      if (m >= p.M || n >= p.N) continue;
      const float* src = ct + row * 128 + ((ch * 8) ^ (((row >> 2) & 3) << 4));
      const f32x4 lo = *reinterpret_cast<const f32x4*>(src);
      const f32x4 hi = *reinterpret_cast<const f32x4*>(src + 4);
      float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      if constexpr (EPI == EPI_SILU_MUL) {
        if ((ch & 3) >= 2) continue;  // up chunks are read by their gate chunk
        const float* up = ct + row * 128 + (((ch + 2) * 8) ^ (((row >> 2) & 3) << 4));
        const f32x4 ulo = *reinterpret_cast<const f32x4*>(up);
        const f32x4 uhi = *reinterpret_cast<const f32x4*>(up + 4);
        const float u[8] = {ulo[0], ulo[1], ulo[2], ulo[3], uhi[0], uhi[1], uhi[2], uhi[3]};
        bf16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = f2bf(silu(v[e]) * u[e]);
        st8(reinterpret_cast<bf16*>(p.out) + (long)m * p.ldo + (n >> 5) * 16 + (n & 15), o);
      } else {
        epilogue8<EPI>(p, m, n, v, split);
      }
    }
  }
  LSD_STAMP(3)
}

// Measured and removed this round (code in git history, commits 312c1a1 / 4bb62e9 / 0c5def8):
// a persistent one-k-tile-stream variant of the kernel above, one-wave-per-SIMD 4 x 128x128
// kernels on 16x16x32 and 32x32x16 MFMAs, and a peeled k-loop -- 8-30 % slower or within noise
// (profiles/r3_rejected_persistent_prefill_gemm.log, r3_rejected_one_wave_per_simd_gemm.log,
// r3_rejected_p8_peeled_loop.log).

// ---------------------------------------------------------------------------
// Decode GEMM at 129-256 rows: every row in ONE 256 x BN tile, 8 waves
// ---------------------------------------------------------------------------
// The 128x64 ring tiles above read the whole A operand once per column tile
// AND once per 128-row block; at 256 rows that A traffic (L2 -> CU) is 2/3 of
// the bytes a workgroup moves, and the ring runs at ~38 GB/s per CU
// (profiles/r2_decode_gemm_limits.log).  Here a workgroup owns all <= 256
// rows of BN columns (guide §5 "Projection GEMM at M = 256": BN = 64 x all
// rows, 8 waves as 8 (M) x 1 (N), split-K so that (N / BN) x S ~ the CU
// count): 0.83x (BN 64) / 0.58x (BN 128) the operand bytes per output of the
// 128x64 ring, and twice the waves per CU to keep the loads and the MFMAs of
// consecutive k-steps overlapped.
//   * wave w owns rows [32 w, 32 w + 32) x all BN columns: 2 x BN/16 MFMA
//     tiles (v_mfma_f32_16x16x32_bf16), fp32 accumulators;
//   * k-step = 64: A [256][64] (32 KiB) and W [BN][64] staged by LDS-DMA
//     (global_load_lds, 16 B per lane, full 128-B lines, XOR-swizzled on the
//     source address -- the ring kernel's conflict-free image), SLOTS-deep
//     ring, counted vmcnt + one raw s_barrier per step (as gemm_ring_kernel);
//   * S > 1 K splits: EPI_SLAB writes its partial slab (the residual
//     projections: the next norm folds the S slabs, bindings linear_residual);
//     every other epilogue publishes its fp32 partial tile write-through (sc1
//     stores, sc1 loads: guide §5 "In-launch split-K reduction", sc1 form) and
//     the last-arriving split sums the S partials in split order
//     (deterministic) and runs the fused epilogue.  A tile's splits have
//     consecutive remapped ids, so they share an XCD (speed only).
template <int ROWS, bool BL = kStageBL>
__device__ __forceinline__ void stage8(char* lds_tile, const bf16* src, long ld, int row0, int row_max,
                                       int k0) {
  // 8 waves: ROWS / 64 wave-instructions of 1 KiB (8 rows x 128 B) each, the
  // [ROWS][64 k] image with 16-B chunks swizzled by (row >> 1) & 7 (lds_frag)
  stage_rows<ROWS, 8, 0, BL>(lds_tile, src, ld, row0, row_max, k0, threadIdx.x >> 6);
}

template <int BN, int SLOTS>
constexpr int d256_smem() {
  return SLOTS * (256 + BN) * 128 > 256 * (BN + 4) * 4 ? SLOTS * (256 + BN) * 128 : 256 * (BN + 4) * 4;
}

template <int EPI, int BN, int SLOTS>
__global__ __launch_bounds__(512) void gemm_d256_kernel(GemmParams p, int* __restrict__ cnt,
                                                        float* __restrict__ ws) {
  constexpr int NJ = BN / 16;                 // 16-column MFMA tiles per wave
  constexpr int A_BYTES = 256 * 64 * 2;       // 32 KiB
  constexpr int SLOT_BYTES = A_BYTES + BN * 64 * 2;
  constexpr int LPS = 4 + BN / 64;            // glds per thread per k-step (A + W)
  constexpr int D = SLOTS - 1;                // k-steps in flight
  constexpr int SMEM = d256_smem<BN, SLOTS>();
  static_assert(SLOTS >= 2 && SLOTS <= 4 && SLOTS * SLOT_BYTES <= 160 * 1024, "LDS ring");
  static_assert((D - 1) * LPS <= 63, "vmcnt range");
  // ONE __shared__ array: a second LDS object can make hipcc drain the glds
  // every k-step (guide §5 trap 4(a)).  The reducer flag lives in the ring,
  // dead by then (all glds waited, every wave past the publish barrier).
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  int* s_flag = reinterpret_cast<int*>(smem);

  const int S = p.splits;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = bid / S, split = bid % S;
  // tiles are column-major over 256-row blocks: a column tile's row blocks
  // (and its splits) have consecutive remapped ids, so they share an XCD's L2
  // for the W tile (speed only)
  const int RB = (p.M + 255) / 256;
  const int rb = tile % RB, n0 = (tile / RB) * BN, m0 = rb * 256;
  const int KT = p.K / 64;
  const int kb = (int)((long)KT * split / S), ke = (int)((long)KT * (split + 1) / S);
  const int lane = lane_id(), w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  LSD_STAMP(0)

  f32x4 acc[2][NJ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto issue = [&](int kt, int slot) {
    char* b = smem + slot * SLOT_BYTES;
    stage8<256>(b, p.A, p.lda, m0, p.M - 1, kt * 64);
    stage8<BN>(b + A_BYTES, p.W, p.ldw, n0, p.N - 1, kt * 64);
  };
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (kb + d < ke) issue(kb + d, d);
  int slot = 0;
  for (int kt = kb; kt < ke; ++kt) {
    // this thread's glds of step kt landed; the later steps stay in flight
    const int later = min(D - 1, ke - 1 - kt);
    if (D >= 3 && later >= 2) __builtin_amdgcn_s_waitcnt(vmcnt_imm(2 * LPS));
    else if (later == 1) __builtin_amdgcn_s_waitcnt(vmcnt_imm(LPS));
    else __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));
    // publishes every wave's DMA of step kt AND proves every wave is done
    // reading the slot of step kt - 1, which is refilled right after
    __builtin_amdgcn_s_barrier();
    if (kt + D < ke) issue(kt + D, slot == 0 ? SLOTS - 1 : slot - 1);
    const char* ta = smem + slot * SLOT_BYTES;
    const char* tw = ta + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[2], wf[NJ];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = lds_frag(ta, w * 32 + i * 16 + r, kk * 4 + g);
#pragma unroll
      for (int j = 0; j < NJ; ++j) wf[j] = lds_frag(tw, j * 16 + r, kk * 4 + g);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NJ; ++j) acc[i][j] = mfma16(af[i], wf[j], acc[i][j]);
    }
    slot = slot == SLOTS - 1 ? 0 : slot + 1;
  }
  LSD_STAMP(1)

  if (S > 1 && EPI != EPI_SLAB) {
    // ---- publish this split's partial tile (write-through), last arriver
    // sums all S.  Lane-major slab: thread t's (i, j) accumulator at
    // ((i * NJ + j) * 512 + t) * 16 B, so every access is 16 contiguous bytes.
    constexpr int PER_BLOCK = 2 * NJ * 512;  // f32x4 per split tile
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        ws + (long)tile * S * PER_BLOCK * 4, (short)0, S * PER_BLOCK * 16, 0x00020000);
    const int toff = threadIdx.x * 16;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs,
                                               split * PER_BLOCK * 16 + (i * NJ + j) * 8192 + toff, 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const int t = __hip_atomic_fetch_add(cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *s_flag = (t == S - 1);
      if (t == S - 1) __hip_atomic_store(cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (*s_flag == 0) return;
    LSD_STAMP(2)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < NJ; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // every slab load of a group in flight before the adds (one round trip per
    // group); clamped index x 0/1 mask, no per-load branch (guide §5 trap (c))
    constexpr int RG = 16 / NJ;  // splits per group: 32 f32x4 (128 VGPRs) in flight
    for (int s0 = 0; s0 < S; s0 += RG) {
      f32x4 v[RG][2][NJ];
#pragma unroll
      for (int u = 0; u < RG; ++u) {
        const int s2 = min(s0 + u, S - 1);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            v[u][i][j] = __builtin_bit_cast(
                f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, s2 * PER_BLOCK * 16 + (i * NJ + j) * 8192 + toff,
                                                             0, 16));
      }
#pragma unroll
      for (int u = 0; u < RG; ++u) {
        const float msk = (s0 + u < S) ? 1.f : 0.f;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j) acc[i][j] += v[u][i][j] * msk;
      }
    }
  }

  // ---- epilogue through LDS: fp32 [256][BN + 4] C tile, then 16-byte
  // row-contiguous stores (epilogue8); the ring is idle (every glds waited,
  // every wave past the last barrier below)
  constexpr int CLD = BN + 4;
  constexpr int CPR = BN / 8;
  __syncthreads();
  float* ct = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) ct[(w * 32 + i * 16 + 4 * g + q) * CLD + j * 16 + r] = acc[i][j][q];
  __syncthreads();
  if constexpr (EPI != EPI_SILU_MUL) {
    store_pass<EPI, (256 * CPR + 511) / 512, 512>(p, 256 * CPR, split, [&](int c, int& m, int& n, const float*& src) {
      const int row = c / CPR, ch = c % CPR;
      m = m0 + row;
      n = n0 + ch * 8;
      src = ct + row * CLD + ch * 8;
      return m < p.M && n < p.N;
    });
    LSD_STAMP(3)
    return;
  }
  for (int c = threadIdx.x; c < 256 * CPR; c += 512) {
    const int row = c / CPR, ch = c % CPR, m = m0 + row, n = n0 + ch * 8;
    if (m >= p.M || n >= p.N) continue;
    const float* src = ct + row * CLD + ch * 8;
    const f32x4 lo = *reinterpret_cast<const f32x4*>(src);
    const f32x4 hi = *reinterpret_cast<const f32x4*>(src + 4);
    float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    if constexpr (EPI == EPI_SILU_MUL) {
      // interleaved [gate16 | up16] 32-column blocks: a gate chunk pairs with
      // the up chunk 16 columns right (same tile: BN % 32 == 0)
      if ((ch & 3) >= 2) continue;
      const float* up = src + 16;
      const f32x4 ulo = *reinterpret_cast<const f32x4*>(up);
      const f32x4 uhi = *reinterpret_cast<const f32x4*>(up + 4);
      const float u[8] = {ulo[0], ulo[1], ulo[2], ulo[3], uhi[0], uhi[1], uhi[2], uhi[3]};
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = f2bf(silu(v[e]) * u[e]);
      st8(reinterpret_cast<bf16*>(p.out) + (long)m * p.ldo + (n >> 5) * 16 + (n & 15), o);
    } else {
      epilogue8<EPI>(p, m, n, v, split);
    }
  }
  LSD_STAMP(3)
}

// Measured and removed this round: a decode GEMM that streams the weights
// HBM -> VGPRs several k-steps ahead (A alone through an LDS ring; 4 or 8
// waves, 64-128-row tiles).  Equal on GPT-2 XL QKV at 96-row tiles, 20-150 %
// slower elsewhere: issue-bound with one wave per SIMD, 2x TA work from the
// fragment-shaped weight loads (profiles/r5_vw_ab.log, r5_vw8_ab.log,
// r5_pmc_decode_gemm.txt; code in git history, commit 78fca21 and after).

// ---------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------
static int g_big_min_blocks = 160;  // lsd_gemm_set_big_min(): tuning / tests
// lsd_gemm_set_big_group(): tile_order() group (0 = M-fastest).  4: XL prefill
// GEMMs 10-25 % faster than M-fastest, 8 equal, 16+ slower
// (profiles/r2_prefill_tile_order.log)
static int g_big_group = 4;
// lsd_gemm_set_big_kind(): 0 = BK=32 ring kernel (gemm_big), 1 = phase-pipelined BK=64 (gemm_p8)
// with global_load_lds, 4 (default) = the same with buffer_load ... lds staging (+6 % on the GPT-2 XL
// prefill projections and +25 % at 4096^3 over kind 1; profiles/r3_p8_buffer_lds.log)
static int g_big_kind = 4;
// 128x128 launches of at most this many workgroups use the 3-slot ring kernel
// (1 block/CU); larger grids keep the 2-blocks/CU double-buffered one.
// lsd_gemm_set_tiled3_max(): tuning / tests; 0 = off
static int g_tiled3_max_blocks = 0;
static int g_ring_slots = 3;  // lsd_gemm_set_ring_slots(): 3 or 4
static int g_ring_tn = 128;   // lsd_gemm_set_ring_tn(): ring tile columns, 128, 64, 32 or 0 (auto 32/64)
static int g_ring_fill = 128; // auto: 32-wide tiles below this many 64-wide workgroups
static int g_ring_m96 = 0;    // lsd_gemm_set_ring_m96(): largest 96-row-tile ring grid (0 = off)
// lsd_gemm_set_ring8(): 128x64 decode ring on 8 waves (gemm_ring8_kernel): 0 off, 1 loader waves, 2 all compute
static int g_ring8 = 0;
// lsd_gemm_set_ring8_flags(): A/B bits, 1 = rotate each tile's K start, 2 = weights staged nt
static int g_ring8_flags = 0;
// lsd_gemm_set_ring8_pack(): operands in k-block-packed layouts (bit 0 W, bit 1 A; A/B only)
static int g_ring8_pack = 0;
static int g_d256_slots = 3;  // lsd_gemm_set_d256_slots(): gemm_d256 ring depth 2..4 (BN 128: at most 3)
// Decode GEMM row blocking: when the column tiles x K splits leave the chip
// under-filled (< g_rb_fill workgroups, e.g. the deferred-residual projections
// with N = H), M > g_sk_rows rows run as ceil(M / g_sk_rows) row blocks
// (grid z) that share each W tile through L2 -- more workgroups without more
// split-K slab traffic (tools/microbench.py rows: H x H projection at M = 128
// 14.1 -> 12.1 us; well-filled grids gain nothing, lm_head loses).
static int g_sk_rows = 64;
static int g_rb_fill = 192;
// At most 128 rows (MT = 8) per row block: M up to 256 always runs as >= 2
// row blocks.
static int sk_rblocks(int M, int N, int S) {
  const int need = (M + 127) / 128;
  if (M <= g_sk_rows || (N / 64) * S >= g_rb_fill) return need;
  const int rb = (M + g_sk_rows - 1) / g_sk_rows;
  return rb > need ? rb : need;
}
// Row tiles (16 rows each) of one row block: MT is instantiated for
// {1, 2, 3, 4, 6, 8}.  The split-K workspace is sized from this
// (lsd_gemm_sk_rows = row blocks x rows per block), so the two never disagree.
static int sk_mt(int M, int rb) {
  const int mt = ((M + rb - 1) / rb + 15) / 16;
  return mt == 5 || mt == 7 ? mt + 1 : mt;
}

// Column tile width: 64 * NW.  Wide tiles (NW = 2) read A half as often but
// double the weight fragments per wave; measured slower at M = 128 on every
// GPT-2 XL shape (tools/microbench.py rows), so only silu_mul (gate/up pairs)
// uses them by default; lsd_gemm_set_nw2_rows() lowers the row threshold.
static int g_nw2_rows = 1 << 30;
static int sk_nw(int M, int epi) { return (epi == EPI_SILU_MUL || M > g_nw2_rows) ? 2 : 1; }

template <int EPI, int NW>
static hipError_t launch_sk_nw(const GemmParams& p, int* cnt, float* ws, hipStream_t st) {
  const int RB = sk_rblocks(p.M, p.N, p.splits);
  const int MT = sk_mt(p.M, RB);
  dim3 grid((p.N + 64 * NW - 1) / (64 * NW), p.splits, RB), block(256);
  switch (MT) {
    case 1: hipLaunchKernelGGL((gemm_sk_kernel<1, NW, EPI>), grid, block, 0, st, p, cnt, ws); break;
    case 2: hipLaunchKernelGGL((gemm_sk_kernel<2, NW, EPI>), grid, block, 0, st, p, cnt, ws); break;
    case 3: hipLaunchKernelGGL((gemm_sk_kernel<3, NW, EPI>), grid, block, 0, st, p, cnt, ws); break;
    case 4: hipLaunchKernelGGL((gemm_sk_kernel<4, NW, EPI>), grid, block, 0, st, p, cnt, ws); break;
    case 6: hipLaunchKernelGGL((gemm_sk_kernel<6, NW, EPI>), grid, block, 0, st, p, cnt, ws); break;
    case 8: hipLaunchKernelGGL((gemm_sk_kernel<8, NW, EPI>), grid, block, 0, st, p, cnt, ws); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <int EPI>
static hipError_t launch_sk(const GemmParams& p, int* cnt, float* ws, hipStream_t st) {
  if constexpr (EPI == EPI_SILU_MUL) {
    return launch_sk_nw<EPI, 2>(p, cnt, ws, st);
  } else {
    return sk_nw(p.M, EPI) == 2 ? launch_sk_nw<EPI, 2>(p, cnt, ws, st) : launch_sk_nw<EPI, 1>(p, cnt, ws, st);
  }
}

// Launch kinds (lsd_gemm `kind`): 0 split-K decode kernel, 1 tiled family
// (ring / 128x128 / 256x256 by shape), 2 / 3 gemm_d256 with 64 / 128-column
// tiles (M <= 1024 in 256-row blocks, K % 64 == 0; the caller picks it per GEMM).
static int d256_bn(int kind, int M, int N, int K) {
  if (kind < 2 || M < 1 || M > 1024 || K % 64 != 0) return 0;
  return kind == 3 && N % 128 == 0 ? 128 : 64;
}

template <int EPI, int BN>
static hipError_t launch_d256_bn(const GemmParams& p, int* cnt, float* ws, hipStream_t st) {
  const dim3 grid(((p.N + BN - 1) / BN) * ((p.M + 255) / 256) * p.splits), block(512);
  const int slots = BN == 128 ? min(g_d256_slots, 3) : g_d256_slots;
  switch (slots) {
    case 2: hipLaunchKernelGGL((gemm_d256_kernel<EPI, BN, 2>), grid, block, 0, st, p, cnt, ws); break;
    case 4:
      if constexpr (BN == 64) {
        hipLaunchKernelGGL((gemm_d256_kernel<EPI, BN, 4>), grid, block, 0, st, p, cnt, ws);
        break;
      }
      [[fallthrough]];
    default: hipLaunchKernelGGL((gemm_d256_kernel<EPI, BN, 3>), grid, block, 0, st, p, cnt, ws); break;
  }
  return hipGetLastError();
}

template <int EPI>
static hipError_t launch_d256(const GemmParams& p, int kind, int* cnt, float* ws, hipStream_t st) {
  const int bn = d256_bn(kind, p.M, p.N, p.K);
  if (bn == 0) return hipErrorInvalidValue;
  if (p.splits > 1 && EPI != EPI_SLAB && (cnt == nullptr || ws == nullptr)) return hipErrorInvalidValue;
  return bn == 128 ? launch_d256_bn<EPI, 128>(p, cnt, ws, st) : launch_d256_bn<EPI, 64>(p, cnt, ws, st);
}

template <int EPI>
static hipError_t launch_tiled(const GemmParams& p, int* cnt, float* ws, hipStream_t st) {
  // 256x256 pipelined kernel once the problem fills the chip with 1-block/CU
  // tiles; the 128x128 kernel (2 blocks/CU) for smaller M / N.
  const int bm = (p.M + GBM - 1) / GBM, bn = (p.N + GBN - 1) / GBN;
  if (p.M >= GBM && p.K % 64 == 0 && bm * bn * p.splits >= g_big_min_blocks) {
    if (g_big_kind == 1)
      hipLaunchKernelGGL((gemm_p8_kernel<EPI, 0>), dim3(bm * bn * p.splits), dim3(512), 0, st, p, bm, bn,
                         g_big_group);
    else if (g_big_kind == 4)
      hipLaunchKernelGGL((gemm_p8_kernel<EPI, 4>), dim3(bm * bn * p.splits), dim3(512), 0, st, p, bm, bn,
                         g_big_group);
    else
      hipLaunchKernelGGL((gemm_big_kernel<EPI>), dim3(bm * bn * p.splits), dim3(512), 0, st, p, bm, bn,
                         g_big_group);
    return hipGetLastError();
  }
  const int tm = (p.M + TBM - 1) / TBM;
  if (g_ring_tn == 64 || g_ring_tn == 32 || g_ring_tn == 0) {
    // narrow ring tiles: twice the workgroups of the 128-column grid; 32-wide
    // (2 blocks/CU) when 64-wide tiles leave the chip under-filled (auto, 0)
    const int tn64 = (p.N + 63) / 64;
    const bool narrow = g_ring_tn == 32 || (g_ring_tn == 0 && tm * tn64 * p.splits < g_ring_fill);
    if (narrow && (p.N % 32) == 0) {
      const int tn = (p.N + 31) / 32;
      if (tm * tn * p.splits <= 2 * g_tiled3_max_blocks) {
        hipLaunchKernelGGL((gemm_ring_kernel<EPI, 3, 32>), dim3(tm * tn * p.splits), dim3(256), 0, st, p, tm, tn);
        return hipGetLastError();
      }
    }
    // 96-row tiles above 128 rows while 3 x the column tiles fit one round
    // on the chip (GPT-2 XL QKV at 256 rows: 225 workgroups of 512 KB of
    // operand traffic instead of 150 of 614 KB; the ring GEMMs are bound by
    // L2 -> CU bytes per workgroup, profiles/r2_decode_gemm_limits.log).
    // Alone 10-12 % faster (QKV 16.3 -> 14.7 us at 256 rows, MLP-up 17.1 ->
    // 15.0 at 192), but beside the other microbatch lane the extra
    // workgroups cost more than they save (bench: 384 sequences -1 to -1.4 %,
    // 512 within +-0.5 %; profiles/r2_ring_m96.log) -- off by default.
    if (p.splits == 1 && p.M > TBM && g_ring_m96 > 0) {
      const int tm96 = (p.M + 95) / 96;
      if (tm96 * tn64 <= g_ring_m96) {
        hipLaunchKernelGGL((gemm_ring_kernel<EPI, 3, 64, 3>), dim3(tm96 * tn64), dim3(256), 0, st, p, tm96, tn64);
        return hipGetLastError();
      }
    }
    if (tm * tn64 * p.splits <= g_tiled3_max_blocks) {
      const dim3 g8(tm * tn64 * p.splits), b8(512);
      const int rot = (g_ring8_flags & 1) != 0;
      const bool combine = p.splits > 1 && EPI != EPI_SLAB;
      if (combine && (g_ring8 != 2 || cnt == nullptr || ws == nullptr)) return hipErrorInvalidValue;
      if (g_ring8 == 1)
        hipLaunchKernelGGL((gemm_ring8_kernel<EPI, 1, 3>), g8, b8, 0, st, p, tm, tn64, rot, cnt, ws);
      else if (g_ring8 == 2 && g_ring8_pack == 1)
        hipLaunchKernelGGL((gemm_ring8_kernel<EPI, 2, 3, 0, 1>), g8, b8, 0, st, p, tm, tn64, rot, cnt, ws);
      else if (g_ring8 == 2 && g_ring8_pack == 2)
        hipLaunchKernelGGL((gemm_ring8_kernel<EPI, 2, 3, 0, 2>), g8, b8, 0, st, p, tm, tn64, rot, cnt, ws);
      else if (g_ring8 == 2 && g_ring8_pack == 3)
        hipLaunchKernelGGL((gemm_ring8_kernel<EPI, 2, 3, 0, 3>), g8, b8, 0, st, p, tm, tn64, rot, cnt, ws);
      else if (g_ring8 == 2 && (g_ring8_flags & 4))
        hipLaunchKernelGGL((gemm_ring8_kernel<EPI, 2, 3, 0, 0, true>), g8, b8, 0, st, p, tm, tn64, rot, cnt, ws);
      else if (g_ring8 == 2 && (g_ring8_flags & 2))
        hipLaunchKernelGGL((gemm_ring8_kernel<EPI, 2, 3, 1>), g8, b8, 0, st, p, tm, tn64, rot, cnt, ws);
      else if (g_ring8 == 2)
        hipLaunchKernelGGL((gemm_ring8_kernel<EPI, 2, 3>), g8, b8, 0, st, p, tm, tn64, rot, cnt, ws);
      else
        hipLaunchKernelGGL((gemm_ring_kernel<EPI, 3, 64>), dim3(tm * tn64 * p.splits), dim3(256), 0, st, p, tm, tn64);
      return hipGetLastError();
    }
  }
  const int tn = (p.N + TBN - 1) / TBN;
  dim3 grid(tm * tn * p.splits), block(256);
  // the cap counts 128x64 tiles whatever LSD_RING_TN says: a 128x128 ring
  // grid gets half as many workgroups (vocab-wide lm_head grids stay on the
  // 2-blocks/CU kernel; profiles/r1_ab_ring_n64.log)
  const int cap128 = g_tiled3_max_blocks / 2;
  if (tm * tn * p.splits <= cap128 && g_ring_slots == 4)
    hipLaunchKernelGGL((gemm_ring_kernel<EPI, 4, 128>), grid, block, 0, st, p, tm, tn);
  else if (tm * tn * p.splits <= cap128)
    hipLaunchKernelGGL((gemm_ring_kernel<EPI, 3, 128>), grid, block, 0, st, p, tm, tn);
  else
    hipLaunchKernelGGL((gemm_tiled_kernel<EPI>), grid, block, 0, st, p, tm, tn);
  return hipGetLastError();
}

}  // namespace lsd

using namespace lsd;

extern "C" void lsd_gemm_set_big_min(int v) { g_big_min_blocks = v; }
extern "C" void lsd_gemm_set_big_group(int v) { g_big_group = v < 0 ? 0 : v; }
extern "C" void lsd_gemm_set_big_kind(int v) { g_big_kind = (v == 1 || v == 4) ? v : 0; }
extern "C" void lsd_gemm_set_tiled3_max(int v) { g_tiled3_max_blocks = v; }
extern "C" void lsd_gemm_set_ring_slots(int v) { g_ring_slots = v == 4 ? 4 : 3; }
extern "C" void lsd_gemm_set_ring_tn(int v) { g_ring_tn = (v == 64 || v == 32 || v == 0) ? v : 128; }
extern "C" void lsd_gemm_set_ring_fill(int v) { g_ring_fill = v; }
extern "C" void lsd_gemm_set_ring_m96(int v) { g_ring_m96 = v; }
extern "C" void lsd_gemm_set_ring8(int v) { g_ring8 = (v == 1 || v == 2) ? v : 0; }
extern "C" void lsd_gemm_set_ring8_flags(int v) { g_ring8_flags = v & 7; }
extern "C" void lsd_gemm_set_ring8_pack(int v) { g_ring8_pack = v & 3; }
extern "C" void lsd_gemm_set_d256_slots(int v) { g_d256_slots = v < 2 ? 2 : (v > 4 ? 4 : v); }

// columns per gemm_d256 tile of a launch of this kind (0: not a d256 launch):
// the split workspace and ticket counters are sized from it (bindings.cpp)
extern "C" int lsd_gemm_d256_bn(int kind, int M, int N, int K) { return d256_bn(kind, M, N, K); }
// 128x64 tiles of a tiled (kind 1) launch when it runs on gemm_ring8_kernel
// (mirrors launch_tiled), else 0: the split workspace / counters are sized from it
extern "C" int lsd_gemm_ring8_tiles(int M, int N, int K, int S) {
  if (g_ring8 != 2) return 0;
  const int bm = (M + GBM - 1) / GBM, bn = (N + GBN - 1) / GBN;
  if (M >= GBM && K % 64 == 0 && bm * bn * S >= g_big_min_blocks) return 0;
  if (!(g_ring_tn == 64 || g_ring_tn == 32 || g_ring_tn == 0)) return 0;
  const int tm = (M + TBM - 1) / TBM, tn64 = (N + 63) / 64;
  const bool narrow = g_ring_tn == 32 || (g_ring_tn == 0 && tm * tn64 * S < g_ring_fill);
  if (narrow && (N % 32) == 0 && tm * ((N + 31) / 32) * S <= 2 * g_tiled3_max_blocks) return 0;
  if (S == 1 && M > TBM && g_ring_m96 > 0 && ((M + 95) / 96) * tn64 <= g_ring_m96) return 0;
  return tm * tn64 * S <= g_tiled3_max_blocks ? tm * tn64 : 0;
}
extern "C" int lsd_gemm_sk_rblocks(int M, int N, int S) { return sk_rblocks(M, N, S); }
extern "C" int lsd_gemm_sk_rows(int M, int N, int S) {  // rows per row block
  return sk_mt(M, sk_rblocks(M, N, S)) * 16;
}
extern "C" int lsd_gemm_sk_nw(int M, int epi) { return sk_nw(M, epi); }
extern "C" void lsd_gemm_set_nw2_rows(int v) { g_nw2_rows = v; }
extern "C" void lsd_gemm_set_sk_rows(int v) { g_sk_rows = v < 16 ? 16 : (v > 128 ? 128 : v); }

// C ABI used by csrc/bindings.cpp; shapes are validated there.
extern "C" hipError_t lsd_gemm(const GemmParams* p, int epi, int kind, int* cnt, float* ws,
                               hipStream_t st) {
#define LSD_DISPATCH(E)                                                                   \
  case E:                                                                                 \
    return kind >= 2 ? launch_d256<E>(*p, kind, cnt, ws, st)                              \
                     : (kind ? launch_tiled<E>(*p, cnt, ws, st) : launch_sk<E>(*p, cnt, ws, st));
  switch (epi) {
    LSD_DISPATCH(EPI_BF16)
    LSD_DISPATCH(EPI_GELU)
    LSD_DISPATCH(EPI_SILU_MUL)
    LSD_DISPATCH(EPI_F32)
    LSD_DISPATCH(EPI_RESID)
    LSD_DISPATCH(EPI_QKV)
    LSD_DISPATCH(EPI_SLAB)
    default: return hipErrorInvalidValue;
  }
#undef LSD_DISPATCH
}
