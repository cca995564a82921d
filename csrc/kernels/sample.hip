// On-device sampler: greedy argmax or temperature + top-k + multinomial.
//
// K14/K15 of SURVEY.md §2.5.  The reference ships [1, S, 50257] fp32 logits
// to the coordinator as JSON and samples on the host (`server.py:151,183-206`:
// logits[0,-1] / 0.6 -> topk(40) -> softmax -> multinomial).  Here only the
// sampled id (int32) leaves the last stage.
//
// Per row, one 1024-thread block; every pass re-reads the row with 16-byte
// loads (the row -- 200 KB for GPT-2, 500 KB for Llama-3 -- stays L2-resident
// across passes).
//   greedy: block argmax (lowest index on ties).
//   top-k <= 64: threshold = k-th largest of 64 segment maxima (a lower bound
//           of the k-th largest logit), filter pass, sort the ~100 candidates;
//           a GPT-2 row is read from HBM once (both passes from registers).
//   top-k : radix select of the k-th largest order-preserving key in three
//           passes over bits [31:20], [19:8], [7:0] (4096/4096/256 bins; the
//           exponent-heavy top bits are spread over 4096 bins so LDS atomics
//           do not pile onto a few hot bins), each bin search a block-parallel
//           suffix scan.  The winners / candidates are ordered by (value
//           desc, index asc) -- rank selection for k <= 128, a bitonic
//           network in LDS above (deterministic regardless of atomic arrival
//           order) -- then softmax over value/T, inverse-CDF draw with
//           u = splitmix64(seed * FNV + step) -- the same counter-based
//           generator as runtime/batch.py:counter_uniform, so a seeded
//           request reproduces across batch layouts and stage counts.
//   top-k <= 64 with segment maxima (lm_head's epilogue wrote the max of
//           every 8-logit segment, gemm.hip epi8_post): the threshold comes
//           from the segment maxima (25 KB per GPT-2 row instead of 200 KB)
//           and only the segments whose maximum reaches it are read -- the
//           same candidate superset rule, so the same draws.
#include "common.h"

namespace lsd {

constexpr int SMAX = 1024;   // max top_k on device (host validates)
constexpr int NT = 1024;     // threads per row

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

// Block-wide inclusive suffix scan of one value per thread (thread t holds
// the total of its bins; suffix = sum over threads >= t).  `tmp` >= 16 words.
__device__ __forceinline__ unsigned block_suffix(unsigned v, unsigned* tmp) {
  const int lane = lane_id(), w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  unsigned s = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned o = __shfl_down(s, d, 64);
    if (lane + d < 64) s += o;
  }
  __syncthreads();
  if (lane == 0) tmp[w] = s;  // wave total
  __syncthreads();
  unsigned later = 0;
  for (int j = w + 1; j < nw; ++j) later += tmp[j];
  return s + later;
}

// Visit every (value, index) of the row in chunks of CH float4 per thread:
// all CH loads of a chunk are issued before the first visit (addresses
// clamped, not guarded, so no load sits behind a branch).  CH = 13 covers a
// GPT-2 row (50257 <= 13 x 4096) in ONE L2 round trip per pass instead of 13
// (one per float4 step of the plain loop: ~54 us per 128-row batch, almost all
// latency); Llama-3's 128 K vocabulary takes 3.  90 VGPRs, no spills.
// The row stride is a multiple of 64 floats, so a float4 never leaves the row.
constexpr int CH = 13;
template <typename F>
__device__ __forceinline__ void for_row(const float* x, int V, F&& f) {
  const int last = ((V - 1) >> 2) << 2;  // last float4 that starts inside the row
  for (int b0 = 0; b0 < V; b0 += CH * NT * 4) {
    f32x4 q[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i)
      q[i] = *reinterpret_cast<const f32x4*>(x + min(b0 + ((int)threadIdx.x + i * NT) * 4, last));
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int b = b0 + ((int)threadIdx.x + i * NT) * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (b + j < V) f(q[i][j], b + j);
    }
  }
}

// The decode step's per-row counter advance, after the draw: the sampler
// counter and (pos != null) the row's KV position both move by active[row]
// (1 when active is null; pad rows stay put) -- one kernel instead of two
// extra add kernels per group-step.
__device__ __forceinline__ void advance_row(long long* step, int* pos, const int* active, int row,
                                            long long step_r) {
  const int a = active ? active[row] : 1;
  step[row] = step_r + a;
  if (pos) pos[row] += a;
}

// k-th largest of the 64 16-thread group maxima of mx (ties by group): with
// every group maximum an element of the row (or -inf), a lower bound of the
// row's k-th largest element -- the top-k group maxima are k distinct
// elements >= it.  Two block barriers.
__device__ __forceinline__ float kth_group_max(float mx, int k, float* cval, float* redv) {
  const int tid = threadIdx.x;
  mx = fmaxf(mx, wave_xchg<1>(mx));
  mx = fmaxf(mx, wave_xchg<2>(mx));
  mx = fmaxf(mx, wave_xchg<4>(mx));
  mx = fmaxf(mx, wave_xchg<8>(mx));
  if ((tid & 15) == 0) cval[tid >> 4] = mx;
  __syncthreads();
  if (tid < 64) {  // rank of group `tid` among the 64 maxima
    const float sv = cval[tid];
    int rank = 0;
#pragma unroll
    for (int j4 = 0; j4 < 16; ++j4) {
      const f32x4 o = reinterpret_cast<const f32x4*>(cval)[j4];
#pragma unroll
      for (int e = 0; e < 4; ++e) rank += (o[e] > sv || (o[e] == sv && 4 * j4 + e < tid)) ? 1 : 0;
    }
    if (rank == k - 1) redv[0] = sv;
  }
  __syncthreads();
  return redv[0];
}

// Block-wide slot assignment for `cnt` entries of this thread: wave-inclusive
// scan, one LDS atomic per wave on `s_cnt`; returns the thread's first slot.
__device__ __forceinline__ unsigned claim_slots(int cnt, unsigned* s_cnt) {
  const int lane = lane_id();
  int incl = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int o = __shfl_up(incl, d, 64);
    if (lane >= d) incl += o;
  }
  unsigned base = 0;
  if (lane == 63) base = atomicAdd(s_cnt, (unsigned)incl);
  return __shfl(base, 63, 64) + (unsigned)(incl - cnt);
}

constexpr int SCH = 16;  // segment maxima per thread: rows of <= SCH * NT * 8 logits

__global__ __launch_bounds__(NT) void sample_kernel(const float* __restrict__ logits, long ld,
                                                    int V, const float* __restrict__ temp,
                                                    const int* __restrict__ topk,
                                                    const int* __restrict__ greedy,
                                                    const long long* __restrict__ seeds,
                                                    long long* __restrict__ step,
                                                    int* __restrict__ out, int advance,
                                                    const int* __restrict__ active,
                                                    int* __restrict__ pos,
                                                    const float* __restrict__ segmax, long ldseg) {
  __shared__ unsigned hist[4096];
  __shared__ __attribute__((aligned(16))) float cval[SMAX];
  __shared__ __attribute__((aligned(16))) int cidx[SMAX];
  __shared__ unsigned tmp[32];
  __shared__ float redv[16];
  __shared__ int redi[16];
  __shared__ unsigned s_digit, s_need, s_cnt;
  const int row = blockIdx.x, tid = threadIdx.x;
  const float* x = logits + (long)row * ld;

  // per-row parameters up front: their loads overlap the row read instead of
  // adding a dependent round trip at the end
  const int is_greedy = greedy[row];
  const int k_req = topk[row];
  const float T = temp[row];
  const long long seed_r = seeds[row], step_r = step[row];
  if (is_greedy) {
    float best = -INFINITY;
    int bi = 0x7fffffff;
    for_row(x, V, [&](float val, int idx) {
      if (val > best || (val == best && idx < bi)) { best = val; bi = idx; }
    });
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      const float ov = shfl_xor(best, m);
      const int oi = shfl_xor(bi, m);
      if (ov > best || (ov == best && oi < bi)) { best = ov; bi = oi; }
    }
    if (lane_id() == 0) { redv[tid >> 6] = best; redi[tid >> 6] = bi; }
    __syncthreads();
    if (tid == 0) {
      for (int w = 1; w < NT / 64; ++w)
        if (redv[w] > best || (redv[w] == best && redi[w] < bi)) { best = redv[w]; bi = redi[w]; }
      out[row] = bi;
      if (advance) advance_row(step, pos, active, row, step_r);  // all threads read step[row] before the barrier
    }
    return;
  }

  const int k = min(max(k_req, 1), min(SMAX, V));
  // ---- fast path (k <= 64): threshold from segment maxima, then filter.
  // The 64 segments are the 16-thread groups of the row visit; the k-th
  // largest segment maximum tau is <= the k-th largest logit (the top-k
  // segment maxima are k distinct elements >= tau), so {x >= tau} holds the
  // top k.  One pass for the maxima + one filter pass (the row stays in L2),
  // ~100 candidates on real or random logits; the exact (value desc, index
  // asc) order comes from the rank selection below, so the result equals the
  // radix path's.  More than SMAX candidates (flat logits) -> radix path.
  bool fast = k <= 64;
  const int S = (V + 7) >> 3;  // 8-logit segments holding real logits (the last may be partial)
  if (fast && segmax != nullptr && S <= SCH * NT) {
    // ---- segment-maxima path: tau from the lm_head epilogue's segment
    // maxima; a segment whose maximum is below tau holds no candidate, so only
    // the others are read.  The last segment, when partial, also covers padded
    // vocabulary columns: its maximum is taken over the real logits only.
    const float* sm = segmax + (long)row * ldseg;
    const int Sfull = V >> 3, nch = (S + NT - 1) / NT;
    float q[SCH];
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < SCH; ++i)
      if (i < nch) q[i] = sm[min(tid + i * NT, S - 1)];
#pragma unroll
    for (int i = 0; i < SCH; ++i) {
      if (i >= nch) break;
      const int sg = tid + i * NT;
      if (sg >= S) q[i] = -INFINITY;
      if (sg == Sfull && Sfull < S) {
        float pm = -INFINITY;
        for (int j = 8 * sg; j < V; ++j) pm = fmaxf(pm, x[j]);
        q[i] = pm;
      }
      mx = fmaxf(mx, q[i]);
    }
    if (tid == 0) s_cnt = 0;
    const float tau = kth_group_max(mx, k, cval, redv);
    int cnt = 0;
#pragma unroll
    for (int i = 0; i < SCH; ++i) {
      if (i >= nch) break;
      if (q[i] >= tau) {  // -inf segments (past S) never pass unless tau is -inf
        const int sg = tid + i * NT;
        if (sg < S) {
          const f32x4 a = *reinterpret_cast<const f32x4*>(x + 8 * sg);
          const f32x4 b = *reinterpret_cast<const f32x4*>(x + 8 * sg + 4);
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            cnt += (a[j] >= tau && 8 * sg + j < V) ? 1 : 0;
            cnt += (b[j] >= tau && 8 * sg + 4 + j < V) ? 1 : 0;
          }
        }
      }
    }
    unsigned slot = claim_slots(cnt, &s_cnt);
#pragma unroll
    for (int i = 0; i < SCH; ++i) {
      if (i >= nch) break;
      const int sg = tid + i * NT;
      if (q[i] >= tau && sg < S) {  // the segment's 32 bytes again, from L1 / L2
        const f32x4 a = *reinterpret_cast<const f32x4*>(x + 8 * sg);
        const f32x4 b = *reinterpret_cast<const f32x4*>(x + 8 * sg + 4);
        const float v8[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          if (v8[j] >= tau && 8 * sg + j < V) {
            if (slot < SMAX) {
              cval[slot] = v8[j];
              cidx[slot] = 8 * sg + j;
            }
            ++slot;
          }
        }
      }
    }
    __syncthreads();
    fast = s_cnt <= SMAX;  // uniform; more -> radix path over the full row
  } else if (fast) {
    // a row of <= CH * NT * 4 floats (GPT-2's) is loaded ONCE and every pass
    // runs from registers (the tail past V masked to -inf at load time, so
    // no per-element bounds checks); longer rows (Llama-3's) re-read via L2
    const bool one = V <= CH * NT * 4;
    const int last = ((V - 1) >> 2) << 2;
    f32x4 q[CH];
    float mx = -INFINITY;
    if (one) {
#pragma unroll
      for (int i = 0; i < CH; ++i)
        q[i] = *reinterpret_cast<const f32x4*>(x + min((tid + i * NT) * 4, last));
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const int b = (tid + i * NT) * 4;
        if (b + 3 >= V) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (b + j >= V) q[i][j] = -INFINITY;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) mx = fmaxf(mx, q[i][j]);
      }
    } else {
      for_row(x, V, [&](float val, int) { mx = fmaxf(mx, val); });
    }
    if (tid == 0) s_cnt = 0;
    const float tau = kth_group_max(mx, k, cval, redv);
    // compaction without per-element atomics: per-thread candidate count (and
    // bit mask of register positions), wave scan, one LDS atomic per wave
    int cnt = 0;
    unsigned long long msk = 0;
    if (one) {
      // padding past V (-inf in registers) never becomes a candidate: with
      // fewer than k segments holding real logits (V < ~4096) tau is -inf and
      // would otherwise admit it, and its index lies past the row's end
#pragma unroll
      for (int i = 0; i < CH; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          msk |= (q[i][j] >= tau && (tid + i * NT) * 4 + j < V) ? (1ull << (4 * i + j)) : 0ull;
      cnt = __popcll(msk);
    } else {
      for_row(x, V, [&](float val, int) { cnt += val >= tau ? 1 : 0; });
    }
    unsigned slot = claim_slots(cnt, &s_cnt);
    if (one) {
      while (msk) {  // ~0-2 trips per thread; the value comes back from L2
        const int e = __builtin_ctzll(msk);
        msk &= msk - 1;
        const int idx = (tid + (e >> 2) * NT) * 4 + (e & 3);
        if (slot < SMAX) {
          cval[slot] = x[idx];
          cidx[slot] = idx;
        }
        ++slot;
      }
    } else {
      for_row(x, V, [&](float val, int idx) {
        if (val >= tau) {
          if (slot < SMAX) {
            cval[slot] = val;
            cidx[slot] = idx;
          }
          ++slot;
        }
      });
    }
    __syncthreads();
    fast = s_cnt <= SMAX;  // uniform
  }
  const int nsel = fast ? (int)s_cnt : k;  // entries to sort (k winners on the radix path)
  if (!fast) {
  // ---- radix select over 12 + 12 + 8 bits
  unsigned prefix = 0, mask = 0, need = k;
  const int shifts[3] = {20, 8, 0};
  const int widths[3] = {12, 12, 8};
#pragma unroll
  for (int pass = 0; pass < 3; ++pass) {
    const int sh = shifts[pass], nb = 1 << widths[pass];
    for (int i = tid; i < nb; i += NT) hist[i] = 0;
    __syncthreads();
    for_row(x, V, [&](float val, int) {
      const unsigned kk = fkey(val);
      if ((kk & mask) == prefix) atomicAdd(&hist[(kk >> sh) & (nb - 1)], 1u);
    });
    __syncthreads();
    // thread t owns bins [t*bpt, (t+1)*bpt); find the bin where the count of
    // keys in strictly higher bins is < need <= that plus the bin itself
    const int bpt = (nb + NT - 1) / NT;
    unsigned mine = 0;
    for (int j = 0; j < bpt; ++j) {
      const int b = tid * bpt + j;
      if (b < nb) mine += hist[b];
    }
    const unsigned suf = block_suffix(mine, tmp);  // keys in bins >= tid*bpt
    const unsigned above = suf - mine;              // keys in bins > my range
    if (above < need && suf >= need) {
      unsigned cum = above;
      for (int j = bpt - 1; j >= 0; --j) {
        const int b = tid * bpt + j;
        if (b >= nb) continue;
        if (cum + hist[b] >= need) { s_digit = b; s_need = need - cum; break; }
        cum += hist[b];
      }
    }
    __syncthreads();
    prefix |= s_digit << sh;
    need = s_need;
    mask |= (unsigned)(nb - 1) << sh;
    __syncthreads();
  }
  // ---- collect: keys > prefix (k - need of them) and the `need` lowest-index
  // keys == prefix.  Equal keys are rare; take them in index order.
  if (tid == 0) s_cnt = 0;
  __syncthreads();
  for_row(x, V, [&](float val, int idx) {
    if (fkey(val) > prefix) {
      const unsigned slot = atomicAdd(&s_cnt, 1u);
      cval[slot] = val;
      cidx[slot] = idx;
    }
  });
  __syncthreads();
  const unsigned n_gt = k - need;
  if (need > 0) {
    // index-ordered scan of equal keys: each pass takes the smallest index left
    for (unsigned a = 0; a < need; ++a) {
      int my_best = 0x7fffffff;
      const int prev = a == 0 ? -1 : cidx[n_gt + a - 1];
      for_row(x, V, [&](float val, int idx) {
        if (idx > prev && fkey(val) == prefix) my_best = min(my_best, idx);
      });
#pragma unroll
      for (int m = 32; m >= 1; m >>= 1) my_best = min(my_best, shfl_xor(my_best, m));
      if (lane_id() == 0) redi[tid >> 6] = my_best;
      __syncthreads();
      if (tid == 0) {
        int b = redi[0];
        for (int w = 1; w < NT / 64; ++w) b = min(b, redi[w]);
        cidx[n_gt + a] = b;
        cval[n_gt + a] = x[b];
      }
      __syncthreads();
    }
  }
  }  // radix path
  // ---- k <= 128 (every fast-path row; radix rows with k <= 128): rank
  // selection -- thread t counts the entries ahead of entry t in (value desc,
  // index asc) order (LDS broadcast reads, 4 per instruction) and, ranked < k,
  // writes it there: independent work and one barrier for any nsel <= SMAX,
  // instead of a sorting network (a wave network of 28 dependent shuffle
  // stages for <= 128 entries, a barrier per stage in LDS beyond that, which
  // the rows with more than 128 candidates hit).  The draw: wave 0, 2 sorted
  // entries per lane (element e = 2 * lane + r).  Sampler 256 rows x GPT-2
  // vocab, top-k 40: 21.7 -> 20.8 us (16.5 with the segment maxima),
  // profiles/r5_sampler_ab.log.  Rank counting is O(nsel) per thread: rows
  // with more than 256 candidates (top-k 64 takes the smallest of the 64
  // group maxima as its threshold: ~500) keep the LDS network (top-k 64:
  // 65 us ranked vs 32 us sorted, profiles/r5_sampler_final.log).
  if (k <= 128 && nsel <= 256) {
    float* sv = reinterpret_cast<float*>(hist);
    int* si = reinterpret_cast<int*>(hist + SMAX);
    if (tid < nsel) {
      const float cv = cval[tid];
      const int ci = cidx[tid];
      int rk = 0;
      for (int j4 = 0; j4 < nsel; j4 += 4) {
        const f32x4 vv = *reinterpret_cast<const f32x4*>(cval + j4);
        const int4 ii = *reinterpret_cast<const int4*>(cidx + j4);
        const float vj[4] = {vv[0], vv[1], vv[2], vv[3]};
        const int ij[4] = {ii.x, ii.y, ii.z, ii.w};
#pragma unroll
        for (int e = 0; e < 4; ++e)
          rk += (j4 + e < nsel && (vj[e] > cv || (vj[e] == cv && ij[e] < ci))) ? 1 : 0;
      }
      if (rk < k) { sv[rk] = cv; si[rk] = ci; }
    }
    __syncthreads();
    if (tid >= 64) return;
    float v[2];
    int ix[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const bool ok = 2 * tid + r < k;
      v[r] = ok ? sv[2 * tid + r] : -INFINITY;
      ix[r] = ok ? si[2 * tid + r] : 0x7fffffff;
    }
    const int e0 = 2 * tid;
    const float x0 = __shfl(v[0], 0, 64) / T;
    const float u = counter_uniform(seed_r, step_r);
    const float p0 = e0 < k ? __expf(v[0] / T - x0) : 0.f;
    const float p1 = e0 + 1 < k ? __expf(v[1] / T - x0) : 0.f;
    const float target = u * wave_sum(p0 + p1);
    float pre = p0 + p1;  // inclusive prefix of the lane pairs
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const float o = __shfl_up(pre, d, 64);
      if (tid >= d) pre += o;
    }
    const float c1 = pre, c0 = pre - p1;
    const unsigned long long h0 = __ballot(e0 < k && c0 >= target);
    const unsigned long long h1 = __ballot(e0 + 1 < k && c1 >= target);
    int pick = k - 1;
    const int l0 = h0 ? __builtin_ctzll(h0) : 64, l1 = h1 ? __builtin_ctzll(h1) : 64;
    if (l0 < 64 || l1 < 64) pick = l0 <= l1 ? 2 * l0 : 2 * l1 + 1;
    const int win = __shfl(pick & 1 ? ix[1] : ix[0], pick >> 1, 64);
    if (tid == 0) {
      out[row] = win;
      if (advance) advance_row(step, pos, active, row, step_r);
    }
    return;
  }
  // ---- k > 128 or nsel > 256: bitonic sort of the winners / candidates: (value desc, index asc); pad to pow2
  int n2 = 1;
  while (n2 < nsel) n2 <<= 1;
  for (int i = nsel + tid; i < n2; i += NT) { cval[i] = -INFINITY; cidx[i] = 0x7fffffff; }
  __syncthreads();
  for (int size = 2; size <= n2; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < n2; i += NT) {
        const int j = i ^ stride;
        if (j > i) {
          const bool up = (i & size) == 0;
          const float vi = cval[i], vj = cval[j];
          const int ii = cidx[i], ij = cidx[j];
          const bool i_first = (vi > vj) || (vi == vj && ii < ij);
          if (up != i_first) { cval[i] = vj; cval[j] = vi; cidx[i] = ij; cidx[j] = ii; }
        }
      }
      __syncthreads();
    }
  }
  // ---- softmax over value/T and inverse-CDF draw (one wave, k <= 1024)
  if (tid < 64) {
    const float x0 = cval[0] / T;
    // running CDF in chunks of 64: lane l owns element base + l
    const float u = counter_uniform(seed_r, step_r);
    float tot = 0.f;
    for (int base = 0; base < k; base += 64) {
      const int i = base + tid;
      const float e = i < k ? __expf(cval[i] / T - x0) : 0.f;
      tot += wave_sum(e);
    }
    const float target = u * tot;
    float run = 0.f;
    int pick = k - 1;
    for (int base = 0; base < k; base += 64) {
      const int i = base + tid;
      float e = i < k ? __expf(cval[i] / T - x0) : 0.f;
      // inclusive prefix within the wave
      float pre = e;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const float o = __shfl_up(pre, d, 64);
        if (tid >= d) pre += o;
      }
      const float c = run + pre;
      const unsigned long long hit = __ballot(i < k && c >= target);
      if (hit) { pick = base + __builtin_ctzll(hit); break; }
      run += __shfl(pre, 63, 64);
    }
    if (tid == 0) {
      out[row] = cidx[pick];
      if (advance) advance_row(step, pos, active, row, step_r);
    }
  }
}

}  // namespace lsd

using namespace lsd;


// advance != 0: also step[row] += active[row] (1 when active is null) after
// the draw -- the decode step's sampler-counter advance (pad rows stay put),
// folded in instead of a conversion copy + add kernel
extern "C" hipError_t lsd_sample(const float* logits, long ld, int B, int V, const float* temp,
                                 const int* topk, const int* greedy, const long long* seeds,
                                 long long* step, int* out, int advance, const int* active,
                                 int* pos, const float* segmax, long ldseg, hipStream_t st) {
  if (B == 0) return hipSuccess;
  if (ld % 4 != 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(sample_kernel, dim3(B), dim3(NT), 0, st, logits, ld, V, temp, topk, greedy,
                     seeds, step, out, advance, active, pos, segmax, ldseg);
  return hipGetLastError();
}
