// Causal attention over the shard-local KV cache.
//
// K7 of SURVEY.md §2.5 (`[tf5.15] modeling_gpt2.py:201-220`, SDPA causal):
//   softmax(Q K^T / sqrt(hd) + causal) V.  The reference recomputes attention
// over the whole sequence every step and gets causality only implicitly
// (quirk Q3); here the mask is explicit and K/V come from the cache.
//
// Cache layout [slot][kv_head][position][hd] (bf16): one (slot, head) is a
// contiguous run of positions, so every key/value row read is part of one
// linear stream.
//
// attn_decode : one query per sequence (decode).  Memory-bound flash-decoding:
//   block = (sequence, kv head[, key split]); 4 waves stride over the keys; a
//   key row (hd*2 bytes) is read by hd/8 lanes with 16-byte loads, so each
//   wave-instruction streams 1 KiB of contiguous K (then V).  GQA: the G query
//   heads sharing a kv head are served from the same K/V loads.  Online
//   softmax in exp2 domain; waves/splits merged with (m, l) rescaling.
// attn_prefill: packed ragged queries (prefill / chunked prefill).  MFMA
//   16x16x32 bf16 with SWAPPED operands: S^T = K . Q^T puts one query per lane
//   (column) so the row max/sum are lane-local plus a 2-step exchange, and the
//   S^T accumulator registers ARE the P^T B-operand of the PV MFMA (no LDS
//   round trip for P).  V^T fragments come from the row-major V tile via the
//   gfx950 hardware transpose read ds_read_b64_tr_b16.
#include "common.h"

namespace lsd {

constexpr float NEG = -1e30f;

// K/V rows of the decode step are streamed once per layer per step: load them
// non-temporal so they do not evict the weights the other microbatch lane is
// about to re-read from the Infinity Cache (bench A/B, tools/gpu_ab_flags.sh:
// 31.8k -> 32.6k tok/s GPT-2 XL; -DLSD_KV_TEMPORAL restores default policy)
#ifdef LSD_KV_TEMPORAL
#define LSD_KV_LOAD ld8
#else
#define LSD_KV_LOAD ld8_nt
#endif

// NWV waves per block: 4 for full batches; 16 for small ones (fewer
// (sequence, head) items than CUs), where the whole context of an item is
// requested in one round of loads instead of a chain of dependent rounds.
template <int HD, int G, int U, int NWV>
__global__ __launch_bounds__(NWV * 64) void attn_decode_kernel(
    const bf16* __restrict__ q, long ldq, const bf16* __restrict__ kc,
    const bf16* __restrict__ vc, const int* __restrict__ seq_slots,
    const int* __restrict__ qpos, bf16* out, long ldo, float* part_o, float* part_ml, int n_kv,
    int max_seq, int splits, float scale_log2, int n_items) {
  constexpr int LPK = HD / 8;    // lanes per key row
  constexpr int KPI = 64 / LPK;  // keys per wave-instruction
  __shared__ float sm[NWV][G][LPK][10];
  // work item = (sequence, kv head); a capped grid (lsd_attn_set_max_wg) loops
  // over items so the kernel occupies only part of the chip and a concurrent
  // lane's GEMMs keep the rest
  for (int item = blockIdx.x; item < n_items; item += gridDim.x) {
    const int b = item / n_kv, kvh = item % n_kv, split = blockIdx.y;
    const int lane = lane_id(), w = threadIdx.x >> 6;
    const int ds = lane % LPK, kg = lane / LPK;
    const int ctx = qpos[b] + 1;
    const int per = (ctx + splits - 1) / splits;
    const int k_lo = split * per, k_hi = min(ctx, k_lo + per);
    const long base = ((long)seq_slots[b] * n_kv + kvh) * (long)max_seq * HD + ds * 8;

    float qf[G][8];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      bf16x8 qq = ld8(q + (long)b * ldq + (long)(kvh * G + g) * HD + ds * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[g][j] = bf2f(qq[j]) * scale_log2;
    }
    float m[G], l[G], o[G][8];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      m[g] = NEG;
      l[g] = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[g][j] = 0.f;
    }

    for (int c0 = k_lo + w * KPI; c0 < k_hi; c0 += NWV * KPI * U) {
      bf16x8 kv[U], vv[U];
      int key[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        key[u] = c0 + u * NWV * KPI + kg;
        const int kk = min(key[u], k_hi - 1);
        kv[u] = LSD_KV_LOAD(kc + base + (long)kk * HD);
      }
      // small batches: V (independent of the scores) is requested with K, one
      // round trip per item.  Full batches keep V behind the scores: fewer
      // live registers, and the other blocks on the CU hide the latency
      // (measured: moving it costs the 2 x 256 bench ~1.5 %)
      if constexpr (NWV > 4) {
#pragma unroll
        for (int u = 0; u < U; ++u) vv[u] = LSD_KV_LOAD(vc + base + (long)min(key[u], k_hi - 1) * HD);
      }
      float s[G][U];
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int u = 0; u < U; ++u) {
          float acc = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) acc += qf[g][j] * bf2f(kv[u][j]);
#pragma unroll
          for (int msk = 1; msk < LPK; msk <<= 1) acc += wave_xchg_n(acc, msk);
          s[g][u] = key[u] < k_hi ? acc : NEG;
        }
      if constexpr (NWV <= 4) {
#pragma unroll
        for (int u = 0; u < U; ++u) vv[u] = LSD_KV_LOAD(vc + base + (long)min(key[u], k_hi - 1) * HD);
      }
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float mx = s[g][0];
#pragma unroll
        for (int u = 1; u < U; ++u) mx = fmaxf(mx, s[g][u]);
        const float mn = fmaxf(m[g], mx);
        const float alpha = exp2f(m[g] - mn);
        float p[U], ps = 0.f;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          p[u] = exp2f(s[g][u] - mn);
          ps += p[u];
        }
        l[g] = l[g] * alpha + ps;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float a = o[g][j] * alpha;
#pragma unroll
          for (int u = 0; u < U; ++u) a += p[u] * bf2f(vv[u][j]);
          o[g][j] = a;
        }
        m[g] = mn;
      }
    }

    // merge the key groups of this wave (lanes with equal ds)
#pragma unroll
    for (int msk = LPK; msk < 64; msk <<= 1) {
#pragma unroll
      for (int g = 0; g < G; ++g) {
        // lanes of one head-dim slice (equal ds) merge: exact xor partners
        const float mo = wave_xor_n(m[g], msk), lo = wave_xor_n(l[g], msk);
        const float mn = fmaxf(m[g], mo);
        const float a = exp2f(m[g] - mn), bb = exp2f(mo - mn);
        l[g] = l[g] * a + lo * bb;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[g][j] = o[g][j] * a + wave_xor_n(o[g][j], msk) * bb;
        m[g] = mn;
      }
    }
    // merge the 4 waves through LDS
    if (kg == 0) {
#pragma unroll
      for (int g = 0; g < G; ++g) {
        sm[w][g][ds][0] = m[g];
        sm[w][g][ds][1] = l[g];
#pragma unroll
        for (int j = 0; j < 8; ++j) sm[w][g][ds][2 + j] = o[g][j];
      }
    }
    __syncthreads();
    if (w == 0 && kg == 0) {
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float mm = NEG;
#pragma unroll
        for (int ww = 0; ww < NWV; ++ww) mm = fmaxf(mm, sm[ww][g][ds][0]);
        float ll = 0.f, oo[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ww = 0; ww < NWV; ++ww) {
          const float f = exp2f(sm[ww][g][ds][0] - mm);
          ll += sm[ww][g][ds][1] * f;
#pragma unroll
          for (int j = 0; j < 8; ++j) oo[j] += sm[ww][g][ds][2 + j] * f;
        }
        const int h = kvh * G + g;
        if (splits == 1) {
          const float inv = ll > 0.f ? 1.f / ll : 0.f;
          bf16x8 r;
#pragma unroll
          for (int j = 0; j < 8; ++j) r[j] = f2bf(oo[j] * inv);
          st8(out + (long)b * ldo + (long)h * HD + ds * 8, r);
        } else {
          const int nh = n_kv * G;
          const long pi = ((long)b * nh + h) * splits + split;
          float* po = part_o + pi * HD + ds * 8;
#pragma unroll
          for (int j = 0; j < 8; ++j) po[j] = oo[j];
          if (ds == 0) {
            part_ml[pi * 2] = mm;
            part_ml[pi * 2 + 1] = ll;
          }
        }
      }
    }
    __syncthreads();  // sm is reused by this block's next item
  }
}

// Decode attention FUSED with the attention output projection and its
// residual add, for small batches (single stream: B <= 4 rows).  At batch 1
// a GPT-2 XL layer's attention (5.7 us) and out-projection GEMV (4.8 us, a
// 5 MB weight read at 1.1 TB/s) are both latency-bound launches
// (profiles/r2_single_stream_analysis.log); here one launch does both:
//   block (kv head h, column chunk c): attention of every sequence for the G
//   query heads of kv head h (the decode kernel's loop, K and V requested in
//   one round; recomputed by each of the C chunk blocks of h -- L2-served
//   re-reads of a few tens of KB), kept in fp32 in LDS; then the partial
//   out-projection  part[c][h][b][n] = sum_{k in head h's slice} o[b][k] W[n][k]
//   for the chunk's NC output columns (W's [N][nh*HD] rows: the slice is
//   G*HD contiguous bf16 per column).
// The n_kv partials of a column chunk are summed by the chunk's LAST-arriving
// block in kv-head order (deterministic), plus the bias, into the fp32
// residual x.  Hand-off (guide §6 Guideline 16 / MI355X_MICROARCH hand-off
// table row 1): write-through (sc1, relaxed agent-scope) partial stores ->
// every wave's vmcnt(0) -> barrier -> one lane's agent-scope ticket add; the
// block whose add returns n_kv - 1 reads the partials with sc1 loads.
template <int HD, int G, int NWV, int BMAX>
__global__ __launch_bounds__(NWV * 64) void attn_oproj_kernel(
    const bf16* __restrict__ q, long ldq, const bf16* __restrict__ kc, const bf16* __restrict__ vc,
    const int* __restrict__ seq_slots, const int* __restrict__ qpos, int B, int n_kv, int max_seq,
    float scale_log2, const bf16* __restrict__ W, long ldw, const bf16* __restrict__ bias, float* x,
    int N, int NC, float* part, int* cnt) {
  constexpr int LPK = HD / 8;    // lanes per key row
  constexpr int KPI = 64 / LPK;  // keys per wave-instruction
  constexpr int U = 2;
  constexpr int KS = G * HD;     // this kv head's slice of the out-projection's K
  constexpr int LPC = KS / 8 <= 64 ? KS / 8 : 64;  // lanes per output column
  constexpr int R = KS / (8 * LPC);                 // 16-B pieces of W per lane
  constexpr int CPI = 64 / LPC;                     // columns per wave-instruction
  static_assert(64 % LPC == 0 && R * 8 * LPC == KS, "out-projection slice per lane");
  __shared__ float sm[NWV][G][LPK][10];
  __shared__ float so[BMAX][KS];
  __shared__ int s_flag;
  const int kvh = blockIdx.x, c = blockIdx.y;
  const int lane = lane_id(), w = threadIdx.x >> 6;
  const int ds = lane % LPK, kg = lane / LPK;

  for (int b = 0; b < B; ++b) {
    const int ctx = qpos[b] + 1;
    const long base = ((long)seq_slots[b] * n_kv + kvh) * (long)max_seq * HD + ds * 8;
    float qf[G][8];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const bf16x8 qq = ld8(q + (long)b * ldq + (long)(kvh * G + g) * HD + ds * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[g][j] = bf2f(qq[j]) * scale_log2;
    }
    float m[G], l[G], o[G][8];
#pragma unroll
    for (int g = 0; g < G; ++g) {
      m[g] = NEG;
      l[g] = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[g][j] = 0.f;
    }
    for (int c0 = w * KPI; c0 < ctx; c0 += NWV * KPI * U) {
      bf16x8 kv[U], vv[U];
      int key[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {  // K and V of the round requested together
        key[u] = c0 + u * NWV * KPI + kg;
        const int kk = min(key[u], ctx - 1);
        kv[u] = ld8(kc + base + (long)kk * HD);
        vv[u] = ld8(vc + base + (long)kk * HD);
      }
      float sc[G][U];
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int u = 0; u < U; ++u) {
          float acc = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) acc += qf[g][j] * bf2f(kv[u][j]);
#pragma unroll
          for (int msk = 1; msk < LPK; msk <<= 1) acc += wave_xchg_n(acc, msk);
          sc[g][u] = key[u] < ctx ? acc : NEG;
        }
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float mx = sc[g][0];
#pragma unroll
        for (int u = 1; u < U; ++u) mx = fmaxf(mx, sc[g][u]);
        const float mn = fmaxf(m[g], mx);
        const float alpha = exp2f(m[g] - mn);
        float p[U], ps = 0.f;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          p[u] = exp2f(sc[g][u] - mn);
          ps += p[u];
        }
        l[g] = l[g] * alpha + ps;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float a = o[g][j] * alpha;
#pragma unroll
          for (int u = 0; u < U; ++u) a += p[u] * bf2f(vv[u][j]);
          o[g][j] = a;
        }
        m[g] = mn;
      }
    }
#pragma unroll
    for (int msk = LPK; msk < 64; msk <<= 1) {
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const float mo = wave_xor_n(m[g], msk), lo = wave_xor_n(l[g], msk);
        const float mn = fmaxf(m[g], mo);
        const float a = exp2f(m[g] - mn), bb = exp2f(mo - mn);
        l[g] = l[g] * a + lo * bb;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[g][j] = o[g][j] * a + wave_xor_n(o[g][j], msk) * bb;
        m[g] = mn;
      }
    }
    if (kg == 0) {
#pragma unroll
      for (int g = 0; g < G; ++g) {
        sm[w][g][ds][0] = m[g];
        sm[w][g][ds][1] = l[g];
#pragma unroll
        for (int j = 0; j < 8; ++j) sm[w][g][ds][2 + j] = o[g][j];
      }
    }
    __syncthreads();
    if (w == 0 && kg == 0) {
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float mm = NEG;
#pragma unroll
        for (int ww = 0; ww < NWV; ++ww) mm = fmaxf(mm, sm[ww][g][ds][0]);
        float ll = 0.f, oo[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ww = 0; ww < NWV; ++ww) {
          const float f = exp2f(sm[ww][g][ds][0] - mm);
          ll += sm[ww][g][ds][1] * f;
#pragma unroll
          for (int j = 0; j < 8; ++j) oo[j] += sm[ww][g][ds][2 + j] * f;
        }
        const float inv = ll > 0.f ? 1.f / ll : 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) so[b][g * HD + ds * 8 + j] = oo[j] * inv;
      }
    }
    __syncthreads();  // so[b] complete; sm reused by the next sequence
  }

  // ---- partial out-projection of this kv head's slice, NC columns
  const int n0 = c * NC;
  const int sub = lane % LPC;
  for (int cb = w * CPI; cb < NC; cb += NWV * CPI) {  // wave-uniform trip count (lane reductions)
    const int cc = cb + lane / LPC, n = n0 + cc;
    const bool valid = cc < NC && n < N;
    float wf[R][8];
#pragma unroll
    for (int rr = 0; rr < R; ++rr) {
      const bf16x8 wv = ld8(W + (long)min(n, N - 1) * ldw + (long)kvh * KS + (rr * LPC + sub) * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) wf[rr][j] = bf2f(wv[j]);
    }
    for (int b = 0; b < B; ++b) {
      float acc = 0.f;
#pragma unroll
      for (int rr = 0; rr < R; ++rr)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc += so[b][(rr * LPC + sub) * 8 + j] * wf[rr][j];
#pragma unroll
      for (int msk = 1; msk < LPC; msk <<= 1) acc += wave_xchg_n(acc, msk);
      if (valid && sub == 0)
        __hip_atomic_store(part + (((long)c * n_kv + kvh) * B + b) * NC + cc, acc, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const int t = __hip_atomic_fetch_add(cnt + c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_flag = (t == n_kv - 1);
    if (t == n_kv - 1) __hip_atomic_store(cnt + c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!s_flag) return;
  // ---- last arriver: x[b][n] += bias[n] + sum_h part[c][h][b][n], kv heads in order
  for (int i = threadIdx.x; i < B * NC; i += NWV * 64) {
    const int b = i / NC, cc = i % NC, n = n0 + cc;
    if (n >= N) continue;
    float s = 0.f;
#pragma unroll 8
    for (int h = 0; h < n_kv; ++h)
      s += __hip_atomic_load(part + (((long)c * n_kv + h) * B + b) * NC + cc, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    float* xp = x + (long)b * N + n;
    *xp = *xp + (s + (bias ? bf2f(bias[n]) : 0.f));
  }
}

// Merge split-K decode partials: one block per (sequence, head).
template <int HD>
__global__ __launch_bounds__(64) void attn_decode_combine_kernel(const float* part_o,
                                                                 const float* part_ml, bf16* out,
                                                                 long ldo, int nh, int splits) {
  const int b = blockIdx.x / nh, h = blockIdx.x % nh;
  const long p0 = ((long)b * nh + h) * splits;
  float mm = NEG;
  for (int s = 0; s < splits; ++s) mm = fmaxf(mm, part_ml[(p0 + s) * 2]);
  for (int d = threadIdx.x; d < HD; d += 64) {
    float ll = 0.f, oo = 0.f;
    for (int s = 0; s < splits; ++s) {
      const float f = exp2f(part_ml[(p0 + s) * 2] - mm);
      ll += part_ml[(p0 + s) * 2 + 1] * f;
      oo += part_o[(p0 + s) * HD + d] * f;
    }
    out[(long)b * ldo + (long)h * HD + d] = f2bf(ll > 0.f ? oo / ll : 0.f);
  }
}

// ---------------------------------------------------------------------------
// Prefill: 64-query tile per block (4 waves x 16 queries), 64-key tiles in LDS
// ---------------------------------------------------------------------------
typedef short short4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16x4 ds_read_tr(const bf16* lds_ptr) {
  typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
  return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(lds_ptr));
}

template <int HD>
__global__ __launch_bounds__(256) void attn_prefill_kernel(
    const bf16* __restrict__ q, long ldq, const bf16* __restrict__ kc,
    const bf16* __restrict__ vc, const int* __restrict__ tiles,
    const int* __restrict__ seq_slots, const int* __restrict__ q_start,
    const int* __restrict__ cu_q, bf16* out, long ldo, int nh, int n_kv, int max_seq,
    float scale_log2) {
  constexpr int KT = 64;              // keys per tile
  constexpr int LDR = HD + 8;         // padded LDS row (elements): +16 B
  constexpr int CPR = HD / 8;         // 16-B chunks per row
  constexpr int CH = KT * CPR / 256;  // chunks per thread per tile
  __shared__ __attribute__((aligned(16))) bf16 ks[KT * LDR];
  __shared__ __attribute__((aligned(16))) bf16 vs[KT * LDR];

  const int bseq = tiles[blockIdx.x * 2], qoff = tiles[blockIdx.x * 2 + 1];
  const int h = blockIdx.y;
  const int kvh = h / (nh / n_kv);
  const int qlen = cu_q[bseq + 1] - cu_q[bseq];
  const int st = q_start[bseq];
  const int lane = lane_id(), w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int qi = qoff + w * 16 + r;  // this lane's query (row within the sequence)
  const int qrow = cu_q[bseq] + min(qi, qlen - 1);
  const int my_pos = st + qi;
  const int kmax = st + min(qoff + 64, qlen);  // keys [0, kmax) are needed by the tile
  const int ntile = (kmax + KT - 1) / KT;
  const long base = ((long)seq_slots[bseq] * n_kv + kvh) * (long)max_seq * HD;

  bf16x8 qf[HD / 32];
#pragma unroll
  for (int kk = 0; kk < HD / 32; ++kk) qf[kk] = ld8(q + (long)qrow * ldq + (long)h * HD + kk * 32 + g * 8);

  f32x4 o[HD / 16];
#pragma unroll
  for (int di = 0; di < HD / 16; ++di) o[di] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = NEG, lsum = 0.f;

  bf16x8 kreg[CH], vreg[CH];
  auto load_tile = [&](int kt) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int idx = threadIdx.x + c * 256;
      const int key = min(kt * KT + idx / CPR, kmax - 1);
      const long off = base + (long)key * HD + (idx % CPR) * 8;
      kreg[c] = ld8(kc + off);
      vreg[c] = ld8(vc + off);
    }
  };
  load_tile(0);
  for (int kt = 0; kt < ntile; ++kt) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int idx = threadIdx.x + c * 256;
      st8(ks + (idx / CPR) * LDR + (idx % CPR) * 8, kreg[c]);
      st8(vs + (idx / CPR) * LDR + (idx % CPR) * 8, vreg[c]);
    }
    __syncthreads();
    if (kt + 1 < ntile) load_tile(kt + 1);  // in flight under this tile's math

    // S^T[key][q] for 4 subtiles of 16 keys
    f32x4 sacc[4];
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      sacc[ni] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < HD / 32; ++kk) {
        bf16x8 kf = *reinterpret_cast<const bf16x8*>(ks + (ni * 16 + r) * LDR + kk * 32 + g * 8);
        sacc[ni] = mfma16(kf, qf[kk], sacc[ni]);
      }
    }
    // scale, causal mask, tile max (lane-local over 16 keys, then across g)
    float tmax = NEG;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = kt * KT + ni * 16 + 4 * g + i;
        float sv = sacc[ni][i] * scale_log2;
        sv = key <= my_pos ? sv : NEG;
        sacc[ni][i] = sv;
        tmax = fmaxf(tmax, sv);
      }
    tmax = fmaxf(tmax, wave_xchg<16>(tmax));
    tmax = fmaxf(tmax, wave_xchg<32>(tmax));
    const float mn = fmaxf(m, tmax);
    const float alpha = exp2f(m - mn);
    m = mn;
    float ps = 0.f;
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = exp2f(sacc[ni][i] - mn);
        sacc[ni][i] = p;
        ps += p;
      }
    lsum = lsum * alpha + ps;
#pragma unroll
    for (int di = 0; di < HD / 16; ++di) o[di] *= alpha;
    // O^T[d][q] += V^T[d][key] . P^T[key][q]; k-slot j of group g <-> key
    // 32kk + 4g + j (j < 4), 32kk + 16 + 4g + (j - 4) (j >= 4)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 pf;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pf[j] = f2bf(sacc[2 * kk][j]);
        pf[4 + j] = f2bf(sacc[2 * kk + 1][j]);
      }
      const int r0 = kk * 32 + 4 * g + (r >> 2);
#pragma unroll
      for (int di = 0; di < HD / 16; ++di) {
        const int col = di * 16 + 4 * (r & 3);
        bf16x4 lo = ds_read_tr(vs + r0 * LDR + col);
        bf16x4 hi = ds_read_tr(vs + (r0 + 16) * LDR + col);
        bf16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        o[di] = mfma16(vf, pf, o[di]);
      }
    }
    __syncthreads();
  }
  lsum += wave_xchg<16>(lsum);
  lsum += wave_xchg<32>(lsum);
  if (qi < qlen) {
    const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
    bf16* op = out + (long)qrow * ldo + (long)h * HD;
#pragma unroll
    for (int di = 0; di < HD / 16; ++di) {
      bf16x4 rr;
#pragma unroll
      for (int i = 0; i < 4; ++i) rr[i] = f2bf(o[di][i] * inv);
      st4(op + di * 16 + 4 * g, rr);
    }
  }
}

// ---------------------------------------------------------------------------
// Decode, grouped-query heads on MFMA: one wave per (sequence, kv head)
// ---------------------------------------------------------------------------
// The VALU decode kernel above spends per key G x HD multiply-adds on the
// scores and as many on P.V, plus a 16-lane reduction per score: with
// Llama-3's G = 4 query heads of HD = 128 per kv head it is VALU-bound (about
// 3.6 TB/s of KV at 256 sequences against the 6.3 TB/s HBM floor).  Here the
// G queries of one kv head are the columns of an MFMA tile, the prefill
// kernel's swapped-operand scheme with a key tile instead of a query tile:
//   S^T[key][q] = K[key][d] . Q^T[d][q]      (16 keys x 16 columns, G valid)
//   O^T[d][q]  += V^T[d][key] . P^T[key][q]  (P^T straight from S^T's registers,
//                                             V^T via ds_read_b64_tr_b16)
// 32-key tiles of K and V are streamed with non-temporal 16-byte loads into
// registers (the next tile's loads in flight under the current tile's math),
// then staged through this wave's own LDS region for the fragment reads.
// Waves are independent: no block barrier.  The math is ~2% of the HBM time
// of the KV stream, so the kernel runs at the KV roofline.
template <int HD, int G>
__global__ __launch_bounds__(256) void attn_decode_mfma_kernel(
    const bf16* __restrict__ q, long ldq, const bf16* __restrict__ kc, const bf16* __restrict__ vc,
    const int* __restrict__ seq_slots, const int* __restrict__ qpos, bf16* out, long ldo,
    float* part_o, float* part_ml, int n_kv, int max_seq, int splits, float scale_log2,
    int n_items) {
  static_assert(G >= 1 && G <= 16, "G query heads per kv head fit one MFMA column tile");
  constexpr int KT = 32;             // keys per tile
  constexpr int LDR = HD + 8;        // padded LDS row (elements): +16 B
  constexpr int CPR = HD / 8;        // 16-B chunks per key row
  constexpr int CH = KT * CPR / 64;  // chunks per lane per tile (per K and per V)
  __shared__ __attribute__((aligned(16))) bf16 lds[4][2][KT * LDR];
  const int lane = lane_id(), w = threadIdx.x >> 6;
  const int item = blockIdx.x * 4 + w;
  if (item >= n_items) return;  // waves are independent: no barriers below
  bf16* ks = lds[w][0];
  bf16* vs = lds[w][1];
  const int b = item / n_kv, kvh = item % n_kv;
  const int ctx = qpos[b] + 1;
  // split blockIdx.y of the context (long contexts: more waves than items)
  const int per = (ctx + splits - 1) / splits;
  const int k_lo = blockIdx.y * per, k_hi = min(ctx, k_lo + per);
  const long base = ((long)seq_slots[b] * n_kv + kvh) * (long)max_seq * HD;
  const int r = lane & 15, g = lane >> 4;

  // Q^T fragments: column r = query head kvh * G + r (zero columns past G)
  bf16x8 qf[HD / 32];
#pragma unroll
  for (int kk = 0; kk < HD / 32; ++kk) {
    bf16x8 z = {};
    qf[kk] = r < G ? ld8(q + (long)b * ldq + (long)(kvh * G + r) * HD + kk * 32 + g * 8) : z;
  }
  f32x4 o[HD / 16];
#pragma unroll
  for (int di = 0; di < HD / 16; ++di) o[di] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = NEG, lsum = 0.f;

  const int ntile = k_hi > k_lo ? (k_hi - k_lo + KT - 1) / KT : 0;
  bf16x8 kreg[CH], vreg[CH];
  auto load_tile = [&](int t) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int idx = lane + c * 64;
      const int key = min(k_lo + t * KT + idx / CPR, k_hi - 1);
      const long off = base + (long)key * HD + (idx % CPR) * 8;
      kreg[c] = LSD_KV_LOAD(kc + off);
      vreg[c] = LSD_KV_LOAD(vc + off);
    }
  };
  if (ntile > 0) load_tile(0);
  for (int t = 0; t < ntile; ++t) {
    // the previous tile's fragment reads must be done before the overwrite
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      const int idx = lane + c * 64;
      st8(ks + (idx / CPR) * LDR + (idx % CPR) * 8, kreg[c]);
      st8(vs + (idx / CPR) * LDR + (idx % CPR) * 8, vreg[c]);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // this wave's LDS writes landed
    __builtin_amdgcn_wave_barrier();
    if (t + 1 < ntile) load_tile(t + 1);  // in flight under this tile's math

    f32x4 sacc[2];
#pragma unroll
    for (int ni = 0; ni < 2; ++ni) {
      sacc[ni] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < HD / 32; ++kk) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(ks + (ni * 16 + r) * LDR + kk * 32 + g * 8);
        sacc[ni] = mfma16(kf, qf[kk], sacc[ni]);
      }
    }
    float tmax = NEG;
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = k_lo + t * KT + ni * 16 + 4 * g + i;
        const float sv = key < k_hi ? sacc[ni][i] * scale_log2 : NEG;
        sacc[ni][i] = sv;
        tmax = fmaxf(tmax, sv);
      }
    tmax = fmaxf(tmax, wave_xchg<16>(tmax));
    tmax = fmaxf(tmax, wave_xchg<32>(tmax));
    const float mn = fmaxf(m, tmax);
    const float alpha = exp2f(m - mn);
    m = mn;
    float ps = 0.f;
#pragma unroll
    for (int ni = 0; ni < 2; ++ni)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = exp2f(sacc[ni][i] - mn);
        sacc[ni][i] = p;
        ps += p;
      }
    lsum = lsum * alpha + ps;
#pragma unroll
    for (int di = 0; di < HD / 16; ++di) o[di] *= alpha;
    // O^T += V^T . P^T over the 32 keys: k-slot j of group g <-> key 4g + j
    // (j < 4), 16 + 4g + (j - 4) (j >= 4)
    bf16x8 pf;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      pf[j] = f2bf(sacc[0][j]);
      pf[4 + j] = f2bf(sacc[1][j]);
    }
    const int r0 = 4 * g + (r >> 2);
#pragma unroll
    for (int di = 0; di < HD / 16; ++di) {
      const int col = di * 16 + 4 * (r & 3);
      const bf16x4 lo = ds_read_tr(vs + r0 * LDR + col);
      const bf16x4 hi = ds_read_tr(vs + (r0 + 16) * LDR + col);
      const bf16x8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      o[di] = mfma16(vf, pf, o[di]);
    }
  }
  lsum += wave_xchg<16>(lsum);
  lsum += wave_xchg<32>(lsum);
  if (r < G && splits > 1) {  // unnormalised partial for attn_decode_combine_kernel
    const long pi = ((long)b * n_kv * G + kvh * G + r) * splits + blockIdx.y;
    float* po = part_o + pi * HD;
#pragma unroll
    for (int di = 0; di < HD / 16; ++di) *reinterpret_cast<f32x4*>(po + di * 16 + 4 * g) = o[di];
    if (g == 0) {
      part_ml[pi * 2] = m;
      part_ml[pi * 2 + 1] = lsum;
    }
  } else if (r < G) {
    const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
    bf16* op = out + (long)b * ldo + (long)(kvh * G + r) * HD;
#pragma unroll
    for (int di = 0; di < HD / 16; ++di) {
      bf16x4 rr;
#pragma unroll
      for (int i = 0; i < 4; ++i) rr[i] = f2bf(o[di][i] * inv);
      st4(op + di * 16 + 4 * g, rr);
    }
  }
}

}  // namespace lsd

using namespace lsd;

static int g_attn_max_wg = 0;  // 0: one workgroup per (sequence, kv head)
extern "C" void lsd_attn_set_max_wg(int v) { g_attn_max_wg = v; }
static int g_attn_small_waves = 8;  // waves per block for small decode batches (4, 8, 16; 88)
static int g_attn_small_waves128 = 88;  // ... for 128-dim heads
extern "C" void lsd_attn_set_small_waves(int v) { g_attn_small_waves = v; }
extern "C" void lsd_attn_set_small_waves128(int v) { g_attn_small_waves128 = v; }
// waves per block for full decode batches, by head dim (4 or 8); 8 also
// requests V with K (lsd_attn_set_large_waves: tuning / A/B)
static int g_attn_large_waves64 = 4, g_attn_large_waves128 = 4;
// grouped-query decode on MFMA (attn_decode_mfma_kernel) for HD = 128,
// G in {2, 4, 8}, at least this many waves ((sequence, kv head) items x
// context splits); 0 = off (lsd_attn_set_mfma_min).  ops/hip.py picks the
// splits so that long contexts reach it with few sequences.
static int g_attn_mfma_min = 256;
extern "C" void lsd_attn_set_mfma_min(int v) { g_attn_mfma_min = v; }
extern "C" void lsd_attn_set_large_waves(int hd, int v) {
  v = (v == 8 || v == 42 || v == 2) ? v : 4;
  if (hd == 64) g_attn_large_waves64 = v;
  else g_attn_large_waves128 = v;
}

static hipError_t attn_decode_combine(const float* part_o, const float* part_ml, bf16* out, long ldo,
                                      int B, int nh, int hd, int splits, hipStream_t st) {
  if (splits > 1) {
    if (hd == 64)
      hipLaunchKernelGGL((attn_decode_combine_kernel<64>), dim3(B * nh), dim3(64), 0, st, part_o,
                         part_ml, out, ldo, nh, splits);
    else
      hipLaunchKernelGGL((attn_decode_combine_kernel<128>), dim3(B * nh), dim3(64), 0, st, part_o,
                         part_ml, out, ldo, nh, splits);
  }
  return hipGetLastError();
}

extern "C" hipError_t lsd_attn_decode(const bf16* q, long ldq, const bf16* kc, const bf16* vc,
                                      const int* seq_slots, const int* qpos, bf16* out, long ldo,
                                      float* part_o, float* part_ml, int B, int nh, int n_kv,
                                      int hd, int max_seq, int splits, float scale_log2,
                                      hipStream_t st) {
  if (B == 0) return hipSuccess;
  const int G = nh / n_kv;
  const int n_items = B * n_kv;
  const int gx = g_attn_max_wg > 0 ? (n_items < g_attn_max_wg ? n_items : g_attn_max_wg) : n_items;
  // fewer blocks than half the CUs: wider blocks (g_attn_small_waves waves),
  // K and V of an item requested in one round of loads
  if (g_attn_mfma_min > 0 && hd == 128 && g_attn_max_wg == 0 && (long)n_items * splits >= g_attn_mfma_min) {
    const dim3 mgrid((n_items + 3) / 4, splits);
#define LSD_DEC_MFMA(GV)                                                                        \
  if (G == GV) {                                                                                \
    hipLaunchKernelGGL((attn_decode_mfma_kernel<128, GV>), mgrid, dim3(256), 0, st, q, ldq, kc, \
                       vc, seq_slots, qpos, out, ldo, part_o, part_ml, n_kv, max_seq, splits,   \
                       scale_log2, n_items);                                                    \
    return attn_decode_combine(part_o, part_ml, out, ldo, B, nh, hd, splits, st);              \
  }
    LSD_DEC_MFMA(2)
    LSD_DEC_MFMA(4)
    LSD_DEC_MFMA(8)
#undef LSD_DEC_MFMA
  }
  // full batches: 4 waves (unroll 4) by default; 8 waves, 4 waves with
  // unroll 2 (42) and 2 waves (2) for A/B (lsd_attn_set_large_waves)
  const int lw = hd == 64 ? g_attn_large_waves64 : g_attn_large_waves128;
  // small grids: g_attn_small_waves (8; 88 = 8 waves with 8 keys per wave in
  // flight, so a 256-key context of a 128-dim head is one round of loads:
  // Llama-3 8B single stream 3.196 -> 3.172-3.181 ms, batch 4 3.757 -> 3.735;
  // GPT-2 XL's 64-dim heads 1.394 -> 1.43 ms, so 128-dim heads only;
  // profiles/r6_attn_u8.log)
  const int swd = hd == 128 ? g_attn_small_waves128 : g_attn_small_waves;
  const int sw = (long)gx * splits <= 128 ? swd : (lw == 8 || lw == 42 || lw == 2 ? lw : 0);
  dim3 grid(gx, splits);
#define LSD_DEC(HDV, GV)                                                                        \
  if (hd == HDV && G == GV) {                                                                   \
    if (sw == 16)                                                                               \
      hipLaunchKernelGGL((attn_decode_kernel<HDV, GV, 2, 16>), grid, dim3(1024), 0, st, q, ldq, \
                         kc, vc, seq_slots, qpos, out, ldo, part_o, part_ml, n_kv, max_seq,     \
                         splits, scale_log2, n_items);                                          \
    else if (sw == 8)                                                                           \
      hipLaunchKernelGGL((attn_decode_kernel<HDV, GV, 4, 8>), grid, dim3(512), 0, st, q, ldq,   \
                         kc, vc, seq_slots, qpos, out, ldo, part_o, part_ml, n_kv, max_seq,     \
                         splits, scale_log2, n_items);                                          \
    else if (sw == 88 && GV <= 4)                                                               \
      hipLaunchKernelGGL((attn_decode_kernel<HDV, (GV <= 4 ? GV : 1), 8, 8>), grid, dim3(512),  \
                         0, st, q, ldq, kc, vc, seq_slots, qpos, out, ldo, part_o, part_ml,     \
                         n_kv, max_seq, splits, scale_log2, n_items);                           \
    else if (sw == 42)                                                                          \
      hipLaunchKernelGGL((attn_decode_kernel<HDV, GV, 2, 4>), grid, dim3(256), 0, st, q, ldq,   \
                         kc, vc, seq_slots, qpos, out, ldo, part_o, part_ml, n_kv, max_seq,     \
                         splits, scale_log2, n_items);                                          \
    else if (sw == 2)                                                                           \
      hipLaunchKernelGGL((attn_decode_kernel<HDV, GV, 4, 2>), grid, dim3(128), 0, st, q, ldq,   \
                         kc, vc, seq_slots, qpos, out, ldo, part_o, part_ml, n_kv, max_seq,     \
                         splits, scale_log2, n_items);                                          \
    else                                                                                        \
      hipLaunchKernelGGL((attn_decode_kernel<HDV, GV, 4, 4>), grid, dim3(256), 0, st, q, ldq,   \
                         kc, vc, seq_slots, qpos, out, ldo, part_o, part_ml, n_kv, max_seq,     \
                         splits, scale_log2, n_items);                                          \
    goto combine;                                                                               \
  }
  LSD_DEC(64, 1)
  LSD_DEC(64, 2)
  LSD_DEC(64, 4)
  LSD_DEC(128, 1)
  LSD_DEC(128, 2)
  LSD_DEC(128, 4)
  LSD_DEC(128, 8)
#undef LSD_DEC
  return hipErrorInvalidValue;
combine:
  return attn_decode_combine(part_o, part_ml, out, ldo, B, nh, hd, splits, st);
}

extern "C" hipError_t lsd_attn_prefill(const bf16* q, long ldq, const bf16* kc, const bf16* vc,
                                       const int* tiles, int n_tiles, const int* seq_slots,
                                       const int* q_start, const int* cu_q, bf16* out, long ldo,
                                       int nh, int n_kv, int hd, int max_seq, float scale_log2,
                                       hipStream_t st) {
  if (n_tiles == 0) return hipSuccess;
  dim3 grid(n_tiles, nh), block(256);
  if (hd == 64)
    hipLaunchKernelGGL((attn_prefill_kernel<64>), grid, block, 0, st, q, ldq, kc, vc, tiles,
                       seq_slots, q_start, cu_q, out, ldo, nh, n_kv, max_seq, scale_log2);
  else if (hd == 128)
    hipLaunchKernelGGL((attn_prefill_kernel<128>), grid, block, 0, st, q, ldq, kc, vc, tiles,
                       seq_slots, q_start, cu_q, out, ldo, nh, n_kv, max_seq, scale_log2);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

// Fused decode attention + output projection + residual add (B <= 4).
// part: fp32 [C][n_kv][B][NC] workspace, cnt: >= C zeroed ticket counters
// (re-armed by each chunk's last arriver).
extern "C" hipError_t lsd_attn_oproj(const bf16* q, long ldq, const bf16* kc, const bf16* vc,
                                     const int* seq_slots, const int* qpos, int B, int nh, int n_kv,
                                     int hd, int max_seq, float scale_log2, const bf16* W, long ldw,
                                     const bf16* bias, float* x, int N, int NC, float* part, int* cnt,
                                     hipStream_t st) {
  if (B == 0) return hipSuccess;
  if (B > 4 || NC < 1) return hipErrorInvalidValue;
  const int G = nh / n_kv;
  const dim3 grid(n_kv, (N + NC - 1) / NC), block(512);
#define LSD_AOP(HDV, GV)                                                                           \
  if (hd == HDV && G == GV) {                                                                      \
    hipLaunchKernelGGL((attn_oproj_kernel<HDV, GV, 8, 4>), grid, block, 0, st, q, ldq, kc, vc,     \
                       seq_slots, qpos, B, n_kv, max_seq, scale_log2, W, ldw, bias, x, N, NC, part, \
                       cnt);                                                                       \
    return hipGetLastError();                                                                      \
  }
  LSD_AOP(64, 1)
  LSD_AOP(128, 1)
  LSD_AOP(128, 2)
  LSD_AOP(128, 4)
  LSD_AOP(128, 8)
#undef LSD_AOP
  return hipErrorInvalidValue;
}
