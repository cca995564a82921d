// PyTorch bindings for the CDNA4 kernels (csrc/kernels/*.hip).
//
// Every entry point validates dtypes, shapes, strides and alignment on the
// host before launching, so a bad call raises a Python exception instead of
// faulting the GPU.  Launches go on the current HIP stream (graph-capturable:
// no allocation-free syncs, no host<->device copies inside).
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <hip/hip_runtime.h>
#include <cmath>

#include "kernels/gemm_params.h"

typedef lsd_bf16_t bf16;
using lsd::GemmParams;
using lsd::GemvParams;

extern "C" {
hipError_t lsd_gemm(const GemmParams* p, int epi, int tiled, int* cnt, float* ws, hipStream_t st);
void lsd_gemm_set_big_min(int v);
void lsd_gemm_set_big_group(int v);
void lsd_gemm_set_big_kind(int v);
void lsd_gemm_set_tiled3_max(int v);
void lsd_gemm_set_ring_slots(int v);
void lsd_gemm_set_ring_tn(int v);
void lsd_gemm_set_ring_fill(int v);
void lsd_gemm_set_ring_m96(int v);
void lsd_gemm_set_d256_slots(int v);
void lsd_gemm_set_ring8(int v);
void lsd_gemm_set_ring8_flags(int v);
void lsd_gemm_set_ring8_pack(int v);
void lsd_norm_set_wave_narrow_min(int v);
void lsd_norm_set_wave_min(int v);
int lsd_gemm_d256_bn(int kind, int M, int N, int K);
int lsd_gemm_ring8_tiles(int M, int N, int K, int S);
void lsd_attn_set_max_wg(int v);
void lsd_attn_set_small_waves(int v);
void lsd_attn_set_small_waves128(int v);
void lsd_attn_set_large_waves(int hd, int v);
void lsd_attn_set_mfma_min(int v);
int lsd_gemm_sk_rows(int M, int N, int S);
int lsd_gemm_sk_rblocks(int M, int N, int S);
int lsd_gemm_sk_nw(int M, int epi);
void lsd_gemm_set_nw2_rows(int v);
void lsd_gemm_set_sk_rows(int v);
hipError_t lsd_embed(const int* ids, const int* pos, const bf16* wte, const bf16* wpe, float* out,
                     int T, int H, int vocab, hipStream_t st);
hipError_t lsd_norm(float* x, const void* slab, int slab_bf16, int splits, const bf16* pbias, const bf16* w,
                    const bf16* b, bf16* out, int T, int H, float eps, int rms, const int* rows,
                    int nrows, hipStream_t st);
hipError_t lsd_attn_decode(const bf16* q, long ldq, const bf16* kc, const bf16* vc,
                           const int* seq_slots, const int* qpos, bf16* out, long ldo,
                           float* part_o, float* part_ml, int B, int nh, int n_kv, int hd,
                           int max_seq, int splits, float scale_log2, hipStream_t st);
hipError_t lsd_attn_prefill(const bf16* q, long ldq, const bf16* kc, const bf16* vc,
                            const int* tiles, int n_tiles, const int* seq_slots,
                            const int* q_start, const int* cu_q, bf16* out, long ldo, int nh,
                            int n_kv, int hd, int max_seq, float scale_log2, hipStream_t st);
hipError_t lsd_attn_oproj(const bf16* q, long ldq, const bf16* kc, const bf16* vc,
                          const int* seq_slots, const int* qpos, int B, int nh, int n_kv, int hd,
                          int max_seq, float scale_log2, const bf16* W, long ldw, const bf16* bias,
                          float* x, int N, int NC, float* part, int* cnt, hipStream_t st);
int lsd_gemv_ok(int M, int K, int epi, int norm);
void lsd_gemv_set_nt(int v);
hipError_t lsd_gemv(const lsd::GemvParams* p, int epi, int norm, hipStream_t st);
hipError_t lsd_apply_rows(const int64_t* args, int b, hipStream_t st);
hipError_t lsd_silu_mul(const lsd_bf16_t* y, long ldy, lsd_bf16_t* out, long ldo, int M, int F, hipStream_t st);
hipError_t lsd_qkv_post(const float* y, long ldy, const lsd_bf16_t* bias, const int* tslot, const int* tpos,
                        const float* rope, lsd_bf16_t* q, lsd_bf16_t* kc, lsd_bf16_t* vc, int M, int q_size,
                        int kv_size, int hd, int n_kv, int max_seq, hipStream_t st);
hipError_t lsd_sample(const float* logits, long ld, int B, int V, const float* temp,
                      const int* topk, const int* greedy, const long long* seeds,
                      long long* step, int* out, int advance, const int* active, int* pos,
                      const float* segmax, long ldseg, hipStream_t st);
}

namespace {

enum Epi : int { EPI_BF16 = 0, EPI_GELU = 1, EPI_SILU_MUL = 2, EPI_F32 = 3, EPI_RESID = 4,
                 EPI_SLAB = 5, EPI_QKV = 6 };

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_hip(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, what, ": ", hipGetErrorString(e));
}

void need(const torch::Tensor& t, c10::ScalarType dt, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == dt, name, " has dtype ", t.scalar_type(), ", expected ", dt);
}

long long* g_stamps = nullptr;  // diagnostic phase stamps (tools/microbench.py "stamps")

void set_stamps(c10::optional<torch::Tensor> t) {
  if (!t.has_value()) { g_stamps = nullptr; return; }
  need(*t, torch::kInt64, "stamps");
  g_stamps = reinterpret_cast<long long*>(t->data_ptr<int64_t>());
}

void need_rows(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.dim() == 2 && t.stride(1) == 1, name, " must be 2-D with unit last stride");
  TORCH_CHECK(t.stride(0) % 8 == 0, name, " row stride must be a multiple of 8 elements");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0, name, " must be 16-byte aligned");
}

const bf16* bptr(const torch::Tensor& t) { return reinterpret_cast<const bf16*>(t.data_ptr()); }
bf16* bptr_mut(const torch::Tensor& t) { return reinterpret_cast<bf16*>(t.data_ptr()); }

const bf16* opt_bias(const c10::optional<torch::Tensor>& b, int N) {
  if (!b.has_value()) return nullptr;
  need(*b, torch::kBFloat16, "bias");
  TORCH_CHECK(b->is_contiguous() && b->numel() == N, "bias must be contiguous [N]");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(b->data_ptr()) % 16 == 0, "bias must be 16-byte aligned");
  return bptr(*b);
}

// Slab dtype of split-K residual projections: LSD_SLAB_BF16 (default 1),
// overridable at run time (gemm_set_slab_bf16: kernel tests pin fp32).
int g_slab_bf16 = -1;
bool slab_bf16_enabled() {
  if (g_slab_bf16 < 0) {
    const char* e = std::getenv("LSD_SLAB_BF16");
    g_slab_bf16 = (e == nullptr || e[0] != '0') ? 1 : 0;
  }
  return g_slab_bf16 != 0;
}

GemmParams base_params(const torch::Tensor& a, const torch::Tensor& w, int64_t tiled) {
  need(a, torch::kBFloat16, "a");
  need(w, torch::kBFloat16, "w");
  need_rows(a, "a");
  need_rows(w, "w");
  TORCH_CHECK(a.size(1) == w.size(1), "K mismatch: a ", a.sizes(), " w ", w.sizes());
  GemmParams p{};
  p.A = bptr(a); p.lda = a.stride(0);
  p.W = bptr(w); p.ldw = w.stride(0);
  p.M = a.size(0); p.N = w.size(0); p.K = a.size(1);
  p.splits = 1;
  TORCH_CHECK(p.N % 16 == 0, "N must be a multiple of 16 (pad the weight), got ", p.N);
  TORCH_CHECK(tiled >= 0 && tiled <= 3, "GEMM kind must be 0 (split-K), 1 (tiled), 2 / 3 (256-row), got ", tiled);
  if (tiled >= 2)
    TORCH_CHECK(p.M >= 1 && p.M <= 1024, "256-row-block decode GEMM needs 1 <= M <= 1024, got ", p.M);
  if (tiled) {
    TORCH_CHECK(p.K % 64 == 0, "tiled GEMM needs K % 64 == 0, got ", p.K);
  } else {
    TORCH_CHECK(p.M >= 1 && p.M <= 256, "decode GEMM needs 1 <= M <= 256, got ", p.M);
    TORCH_CHECK(p.K % 32 == 0, "decode GEMM needs K % 32 == 0, got ", p.K);
    TORCH_CHECK(p.N % 64 == 0, "decode GEMM needs N % 64 == 0 (pad the weight), got ", p.N);
  }
  return p;
}

// Launch with split-K bookkeeping: the decode path needs persistent zeroed
// ticket counters (one per column tile) and an fp32 partial-tile workspace.
void run_gemm(GemmParams& p, int epi, int64_t tiled, int64_t splits,
              const c10::optional<torch::Tensor>& counters, const torch::Tensor& like,
              const char* what) {
  const int kt = tiled ? p.K / 64 : p.K / 32;
  TORCH_CHECK(splits >= 1 && splits <= kt, what, ": splits must be in [1, ", kt, "], got ", splits);
  p.splits = (int)splits;
  int* cnt = nullptr;
  float* ws = nullptr;
  torch::Tensor wsbuf;
  if (tiled && splits > 1 && epi != EPI_SLAB) {
    // tiled split-K with an in-kernel combine: the 256-row decode kernel
    // (gemm_d256, kind 2 / 3) or the 8-wave 128x64 ring (kind 1) -- ticket
    // counters + fp32 partial tiles per split
    const int bn = lsd_gemm_d256_bn((int)tiled, p.M, p.N, p.K);
    const int r8 = tiled == 1 ? lsd_gemm_ring8_tiles(p.M, p.N, p.K, (int)splits) : 0;
    TORCH_CHECK(bn > 0 || r8 > 0, what, ": tiled split-K with an in-kernel combine needs the 256-row "
                "kernel (kind 2 / 3) or the 8-wave decode ring");
    const long tiles = r8 > 0 ? r8 : (long)((p.N + bn - 1) / bn) * ((p.M + 255) / 256);
    const long tile_floats = r8 > 0 ? 128L * 64 : 256L * bn;
    TORCH_CHECK(counters.has_value(), what, ": split-K needs the ticket counter buffer");
    need(*counters, torch::kInt32, "counters");
    TORCH_CHECK(counters->is_contiguous() && counters->numel() >= tiles,
                what, ": counter buffer too small (", counters->numel(), " < ", tiles, ")");
    cnt = counters->data_ptr<int>();
    TORCH_CHECK(splits * tile_floats * 4 < (1L << 31), what, ": split workspace too large");
    wsbuf = torch::empty({tiles * splits * tile_floats}, like.options().dtype(torch::kFloat32));
    ws = wsbuf.data_ptr<float>();
  }
  if (!tiled && epi != EPI_SLAB) {
    const int nw = lsd_gemm_sk_nw(p.M, epi);  // column tile = 64 * nw (partial last tile masked)
    if (epi == EPI_SILU_MUL)
      TORCH_CHECK(p.N % (64 * nw) == 0, what, ": N must be a multiple of ", 64 * nw);
    const long tiles = (p.N + 64 * nw - 1) / (64 * nw) * lsd_gemm_sk_rblocks(p.M, p.N, (int)splits);
    if (splits > 1) {
      TORCH_CHECK(counters.has_value(), what, ": split-K needs the ticket counter buffer");
      need(*counters, torch::kInt32, "counters");
      TORCH_CHECK(counters->is_contiguous() && counters->numel() >= tiles,
                  what, ": counter buffer too small (", counters->numel(), " < ", tiles, ")");
      cnt = counters->data_ptr<int>();
      const long rows = lsd_gemm_sk_rows(p.M, p.N, (int)splits);  // rows per row block
      const long bytes = tiles * splits * rows * 64 * nw * 4;
      TORCH_CHECK(splits * rows * 64 * nw * 4 < (1L << 31), what, ": split workspace too large");
      wsbuf = torch::empty({bytes / 4}, like.options().dtype(torch::kFloat32));
      ws = wsbuf.data_ptr<float>();
    }
  }
  p.stamps = g_stamps;
  check_hip(lsd_gemm(&p, epi, (int)tiled, cnt, ws, cur_stream()), what);
}


// out = act(a @ w^T + bias), bf16
torch::Tensor linear(torch::Tensor a, torch::Tensor w, c10::optional<torch::Tensor> bias,
                     int64_t act, int64_t tiled, int64_t splits,
                     c10::optional<torch::Tensor> counters) {
  GemmParams p = base_params(a, w, tiled);
  p.bias = opt_bias(bias, p.N);
  int epi = act == 1 ? EPI_GELU : (act == 2 ? EPI_SILU_MUL : EPI_BF16);
  if (epi == EPI_SILU_MUL) TORCH_CHECK(p.N % 32 == 0, "silu_mul needs N % 32 == 0");
  const int n_out = epi == EPI_SILU_MUL ? p.N / 2 : p.N;
  auto out = torch::empty({p.M, n_out}, a.options());
  if (p.M == 0) return out;
  p.out = out.data_ptr(); p.ldo = n_out;
  run_gemm(p, epi, tiled, splits, counters, a, "linear");
  return out;
}

// fp32 logits = a @ w^T.  segmax (tiled kernels only): also the max of every
// 8-column segment, fp32 [M, N / 8] -- the sampler then reads the logits only
// in the segments that can hold a top-k element (sample.hip)
torch::Tensor linear_f32(torch::Tensor a, torch::Tensor w, int64_t tiled, int64_t splits,
                         c10::optional<torch::Tensor> counters, c10::optional<torch::Tensor> segmax) {
  GemmParams p = base_params(a, w, tiled);
  auto out = torch::empty({p.M, p.N}, a.options().dtype(torch::kFloat32));
  if (segmax.has_value()) {
    TORCH_CHECK(tiled != 0, "linear_f32: segment maxima need a tiled kernel");
    need(*segmax, torch::kFloat32, "segmax");
    TORCH_CHECK(segmax->dim() == 2 && segmax->is_contiguous() && segmax->size(0) == p.M &&
                segmax->size(1) == p.N / 8, "segmax must be contiguous fp32 [M, N / 8]");
    p.segmax = segmax->data_ptr<float>();
    p.ldseg = p.N / 8;
  }
  if (p.M == 0) return out;
  p.out = out.data_ptr(); p.ldo = p.N;
  run_gemm(p, EPI_F32, tiled, splits, counters, a, "linear_f32");
  return out;
}

// x += a @ w^T + bias.  Decode path: any split, combined in-kernel -- or,
// with defer, like the tiled path with splits > 1: returns the partial slabs
// [splits, M, N] (bias not applied) that the next norm folds in.  defer with
// one split (prefill): the GEMM writes its output as one bf16 slab instead of
// a read-modify-write of the fp32 residual stream.
c10::optional<torch::Tensor> linear_residual(torch::Tensor a, torch::Tensor w,
                                              c10::optional<torch::Tensor> bias, torch::Tensor x,
                                              int64_t splits, int64_t tiled,
                                              c10::optional<torch::Tensor> counters, bool defer) {
  GemmParams p = base_params(a, w, tiled);
  need(x, torch::kFloat32, "x");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && x.size(0) == p.M && x.size(1) == p.N,
              "residual x must be contiguous [M, N]");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "residual x must be 16-byte aligned");
  if (p.M == 0) return c10::nullopt;
  if ((tiled || defer) && (splits > 1 || (defer && tiled))) {
    // bf16 partial slabs (LSD_SLAB_BF16=0: fp32): half the bytes the GEMM
    // writes and the next norm reads, each partial rounded once to bf16 --
    // the precision of a bf16 GEMM output, folded into the fp32 residual.
    // GPT-2 XL headline +3.3 % (48.6-49.1k -> 50.4-50.6k tok/s); logits vs the
    // fp32 golden at 256-row decode: mean error 1.73 -> 1.99 % of the logit
    // std, top-1 agreement 99.78 -> 99.72 % (profiles/r4_slab_bf16.log)
    const bool slab_bf16 = slab_bf16_enabled();
    auto slab = torch::empty({splits, p.M, p.N}, x.options().dtype(slab_bf16 ? torch::kBFloat16 : torch::kFloat32));
    p.slab = static_cast<float*>(slab.data_ptr());
    p.slab_bf16 = slab_bf16 ? 1 : 0;
    run_gemm(p, EPI_SLAB, tiled, splits, c10::nullopt, x, "linear_residual(split)");
    return slab;
  }
  p.bias = opt_bias(bias, p.N);
  p.out = x.data_ptr(); p.ldo = p.N;
  run_gemm(p, EPI_RESID, tiled, splits, counters, x, "linear_residual");
  return c10::nullopt;
}

// QKV projection: returns q bf16 [M, q_size]; k, v written into the caches.
torch::Tensor linear_qkv(torch::Tensor a, torch::Tensor w, c10::optional<torch::Tensor> bias,
                         torch::Tensor kc, torch::Tensor vc, torch::Tensor tslot,
                         torch::Tensor tpos, int64_t q_size, int64_t kv_size, int64_t hd,
                         c10::optional<torch::Tensor> rope, int64_t tiled, int64_t splits,
                         c10::optional<torch::Tensor> counters) {
  GemmParams p = base_params(a, w, tiled);
  p.bias = opt_bias(bias, p.N);
  need(kc, torch::kBFloat16, "k_cache");
  need(vc, torch::kBFloat16, "v_cache");
  TORCH_CHECK(kc.dim() == 4 && kc.is_contiguous() && vc.sizes() == kc.sizes() && vc.is_contiguous(),
              "caches must be contiguous [slots, n_kv, max_seq, hd]");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(kc.data_ptr()) % 16 == 0 &&
              reinterpret_cast<uintptr_t>(vc.data_ptr()) % 16 == 0, "caches must be 16-byte aligned");
  TORCH_CHECK(kc.size(3) == hd && kc.size(1) * hd == kv_size, "cache shape mismatch");
  TORCH_CHECK(p.N == q_size + 2 * kv_size, "w rows must be q_size + 2*kv_size");
  TORCH_CHECK(q_size % hd == 0 && hd % 16 == 0, "bad head dims");
  need(tslot, torch::kInt32, "token_slots");
  need(tpos, torch::kInt32, "token_pos");
  TORCH_CHECK(tslot.numel() == p.M && tpos.numel() == p.M && tslot.is_contiguous() &&
              tpos.is_contiguous(), "token_slots/token_pos must be contiguous [M]");
  p.kc = bptr_mut(kc); p.vc = bptr_mut(vc);
  p.tslot = tslot.data_ptr<int>(); p.tpos = tpos.data_ptr<int>();
  p.q_size = q_size; p.kv_size = kv_size; p.hd = hd;
  p.max_seq = kc.size(2); p.n_kv = kc.size(1);
  if (rope.has_value()) {
    need(*rope, torch::kFloat32, "rope");
    TORCH_CHECK(rope->is_contiguous() && rope->dim() == 3 && rope->size(1) == hd / 2 &&
                rope->size(2) == 2 && rope->size(0) >= p.max_seq, "rope table must be [>=max_seq, hd/2, 2]");
    p.rope = rope->data_ptr<float>();
  }
  auto q = torch::empty({p.M, q_size}, a.options());
  if (p.M == 0) return q;
  p.out = q.data_ptr(); p.ldo = q_size;
  run_gemm(p, EPI_QKV, tiled, splits, counters, a, "linear_qkv");
  return q;
}

// Small-M GEMV (csrc/kernels/gemv.hip): out = epi(norm?(x) @ w^T + bias).
//   norm 0: x bf16 [M, K];  norm 1 (LayerNorm) / 2 (RMSNorm): x is the fp32
//   residual [M, K], normalised in the kernel with gamma (+ beta).
//   epi: 0 bf16, 1 gelu, 2 silu(gate)*up, 3 f32, 4 residual add into `resid`,
//   6 QKV (q returned, k/v appended to the caches, optional RoPE).
c10::optional<torch::Tensor> gemv(torch::Tensor x, torch::Tensor w, c10::optional<torch::Tensor> bias,
                                  int64_t epi, int64_t norm, c10::optional<torch::Tensor> gamma,
                                  c10::optional<torch::Tensor> beta, double eps,
                                  c10::optional<torch::Tensor> resid,
                                  c10::optional<torch::Tensor> kc, c10::optional<torch::Tensor> vc,
                                  c10::optional<torch::Tensor> tslot, c10::optional<torch::Tensor> tpos,
                                  int64_t q_size, int64_t kv_size, int64_t hd,
                                  c10::optional<torch::Tensor> rope,
                                  c10::optional<torch::Tensor> segmax = c10::nullopt) {
  need(w, torch::kBFloat16, "w");
  need_rows(w, "w");
  TORCH_CHECK(x.dim() == 2 && x.stride(1) == 1, "x must be 2-D with unit last stride");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0, "x must be 16-byte aligned");
  GemvParams p{};
  p.M = x.size(0); p.K = x.size(1); p.N = w.size(0);
  TORCH_CHECK(w.size(1) == p.K, "K mismatch: x ", x.sizes(), " w ", w.sizes());
  TORCH_CHECK(lsd_gemv_ok(p.M, p.K, (int)epi, (int)norm), "gemv: shape M=", p.M, " K=", p.K,
              " epi=", epi, " norm=", norm, " not supported");
  p.W = bptr(w); p.ldw = w.stride(0);
  if (norm == 0) {
    need(x, torch::kBFloat16, "x");
    TORCH_CHECK(x.stride(0) % 8 == 0, "x row stride must be a multiple of 8");
    p.A = bptr(x); p.lda = x.stride(0);
  } else {
    need(x, torch::kFloat32, "x");
    TORCH_CHECK(x.stride(0) % 4 == 0 && p.K % 4 == 0, "x rows must be 16-byte aligned");
    p.X = x.data_ptr<float>(); p.ldx = x.stride(0);
    TORCH_CHECK(gamma.has_value(), "norm needs gamma");
    need(*gamma, torch::kBFloat16, "gamma");
    TORCH_CHECK(gamma->is_contiguous() && gamma->numel() == p.K, "gamma [K]");
    p.gamma = bptr(*gamma);
    if (norm == 1) {
      TORCH_CHECK(beta.has_value(), "layernorm needs beta");
      need(*beta, torch::kBFloat16, "beta");
      TORCH_CHECK(beta->is_contiguous() && beta->numel() == p.K, "beta [K]");
      p.beta = bptr(*beta);
    }
    p.eps = (float)eps;
  }
  if (bias.has_value()) {
    need(*bias, torch::kBFloat16, "bias");
    TORCH_CHECK(bias->is_contiguous() && bias->numel() == p.N, "bias must be contiguous [N]");
    p.bias = bptr(*bias);
  }
  c10::optional<torch::Tensor> ret;
  auto bopt = w.options();
  if (epi == EPI_RESID) {
    TORCH_CHECK(resid.has_value(), "residual epilogue needs the residual");
    need(*resid, torch::kFloat32, "resid");
    TORCH_CHECK(resid->dim() == 2 && resid->is_contiguous() && resid->size(0) == p.M &&
                resid->size(1) == p.N, "residual must be contiguous [M, N]");
    p.out = resid->data_ptr(); p.ldo = p.N;
  } else if (epi == EPI_F32) {
    ret = torch::empty({p.M, p.N}, bopt.dtype(torch::kFloat32));
    p.out = ret->data_ptr(); p.ldo = p.N;
    if (segmax.has_value()) {  // [M, N / 8] maxima of the 8-column segments
      need(*segmax, torch::kFloat32, "segmax");
      TORCH_CHECK(p.N % 8 == 0 && segmax->dim() == 2 && segmax->size(0) == p.M &&
                  segmax->size(1) == p.N / 8 && segmax->stride(1) == 1, "segmax must be [M, N / 8], N % 8 == 0");
      p.segmax = segmax->data_ptr<float>(); p.ldseg = segmax->stride(0);
    }
  } else if (epi == EPI_BF16 || epi == EPI_GELU) {
    ret = torch::empty({p.M, p.N}, bopt);
    p.out = ret->data_ptr(); p.ldo = p.N;
  } else if (epi == EPI_SILU_MUL) {
    TORCH_CHECK(p.N % 32 == 0 && !bias.has_value(), "silu_mul needs N % 32 == 0 and no bias");
    ret = torch::empty({p.M, p.N / 2}, bopt);
    p.out = ret->data_ptr(); p.ldo = p.N / 2;
  } else if (epi == EPI_QKV) {
    TORCH_CHECK(kc.has_value() && vc.has_value() && tslot.has_value() && tpos.has_value(),
                "qkv needs caches and token slots/positions");
    need(*kc, torch::kBFloat16, "k_cache");
    need(*vc, torch::kBFloat16, "v_cache");
    TORCH_CHECK(kc->dim() == 4 && kc->is_contiguous() && vc->sizes() == kc->sizes() && vc->is_contiguous(),
                "caches must be contiguous [slots, n_kv, max_seq, hd]");
    TORCH_CHECK(kc->size(3) == hd && kc->size(1) * hd == kv_size, "cache shape mismatch");
    TORCH_CHECK(p.N == q_size + 2 * kv_size && q_size % hd == 0 && hd % 2 == 0, "bad qkv dims");
    need(*tslot, torch::kInt32, "token_slots");
    need(*tpos, torch::kInt32, "token_pos");
    TORCH_CHECK(tslot->numel() == p.M && tpos->numel() == p.M && tslot->is_contiguous() &&
                tpos->is_contiguous(), "token_slots/token_pos must be contiguous [M]");
    p.kc = bptr_mut(*kc); p.vc = bptr_mut(*vc);
    p.tslot = tslot->data_ptr<int>(); p.tpos = tpos->data_ptr<int>();
    p.q_size = q_size; p.kv_size = kv_size; p.hd = hd;
    p.max_seq = kc->size(2); p.n_kv = kc->size(1);
    if (rope.has_value()) {
      need(*rope, torch::kFloat32, "rope");
      TORCH_CHECK(rope->is_contiguous() && rope->dim() == 3 && rope->size(1) == hd / 2 &&
                  rope->size(2) == 2 && rope->size(0) >= p.max_seq, "rope table must be [>=max_seq, hd/2, 2]");
      p.rope = rope->data_ptr<float>();
    }
    ret = torch::empty({p.M, q_size}, bopt);
    p.out = ret->data_ptr(); p.ldo = q_size;
  } else {
    TORCH_CHECK(false, "gemv: unknown epilogue ", epi);
  }
  TORCH_CHECK(!segmax.has_value() || epi == EPI_F32, "segmax needs the fp32 logits epilogue");
  check_hip(lsd_gemv(&p, (int)epi, (int)norm, cur_stream()), "gemv");
  return ret;
}

torch::Tensor embed(torch::Tensor ids, torch::Tensor pos, torch::Tensor wte,
                    c10::optional<torch::Tensor> wpe) {
  need(ids, torch::kInt32, "ids");
  need(pos, torch::kInt32, "pos");
  need(wte, torch::kBFloat16, "wte");
  TORCH_CHECK(ids.is_contiguous() && pos.is_contiguous() && ids.numel() == pos.numel(), "ids/pos");
  TORCH_CHECK(wte.dim() == 2 && wte.is_contiguous() && wte.size(1) % 8 == 0, "wte [V, H], H % 8 == 0");
  const int T = ids.numel(), H = wte.size(1);
  const bf16* pe = nullptr;
  if (wpe.has_value()) {
    need(*wpe, torch::kBFloat16, "wpe");
    TORCH_CHECK(wpe->is_contiguous() && wpe->size(1) == H, "wpe [P, H]");
    pe = bptr(*wpe);
  }
  auto out = torch::empty({T, H}, wte.options().dtype(torch::kFloat32));
  check_hip(lsd_embed(ids.data_ptr<int>(), pos.data_ptr<int>(), bptr(wte), pe,
                      out.data_ptr<float>(), T, H, wte.size(0), cur_stream()), "embed");
  return out;
}

c10::optional<torch::Tensor> norm(torch::Tensor x, c10::optional<torch::Tensor> slab,
                                  c10::optional<torch::Tensor> pbias, c10::optional<torch::Tensor> w,
                                  c10::optional<torch::Tensor> b, double eps, bool rms,
                                  c10::optional<torch::Tensor> rows, bool want_out) {
  need(x, torch::kFloat32, "x");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous(), "x must be contiguous [T, H]");
  const int T = x.size(0), H = x.size(1);
  TORCH_CHECK(H % 4 == 0 && H <= 8192, "norm needs H % 4 == 0 and H <= 8192");
  const bf16* wp = nullptr;
  if (want_out) {
    TORCH_CHECK(w.has_value(), "norm output needs a weight");
    need(*w, torch::kBFloat16, "w");
    TORCH_CHECK(w->numel() == H, "w [H]");
    wp = bptr(*w);
    if (!rms) {
      TORCH_CHECK(b.has_value(), "layernorm needs a bias");
      need(*b, torch::kBFloat16, "b");
      TORCH_CHECK(b->numel() == H, "b [H]");
    }
  }
  const void* sp = nullptr;
  int splits = 0, slab_bf16 = 0;
  if (slab.has_value()) {
    TORCH_CHECK(slab->is_cuda() && (slab->scalar_type() == torch::kFloat32 || slab->scalar_type() == torch::kBFloat16),
                "slab must be an fp32 or bf16 device tensor");
    TORCH_CHECK(slab->is_contiguous() && slab->dim() == 3 && slab->size(1) == T && slab->size(2) == H,
                "slab must be [S, T, H]");
    sp = slab->data_ptr();
    splits = slab->size(0);
    slab_bf16 = slab->scalar_type() == torch::kBFloat16 ? 1 : 0;
  }
  const bf16* pb = nullptr;
  if (pbias.has_value()) {
    TORCH_CHECK(sp != nullptr, "pending bias without slab");
    need(*pbias, torch::kBFloat16, "pending_bias");
    TORCH_CHECK(pbias->numel() == H, "pending bias [H]");
    pb = bptr(*pbias);
  }
  const int* rp = nullptr;
  int n = T;
  if (rows.has_value()) {
    need(*rows, torch::kInt32, "rows");
    TORCH_CHECK(sp == nullptr, "row gather cannot combine slabs");
    TORCH_CHECK(rows->is_contiguous(), "rows must be contiguous");
    rp = rows->data_ptr<int>();
    n = rows->numel();
  }
  c10::optional<torch::Tensor> out;
  bf16* op = nullptr;
  if (want_out) {
    out = torch::empty({n, H}, x.options().dtype(torch::kBFloat16));
    op = bptr_mut(*out);
  }
  check_hip(lsd_norm(x.data_ptr<float>(), sp, slab_bf16, splits, pb, wp, (want_out && b.has_value()) ? bptr(*b) : nullptr,
                     op, T, H, (float)eps, rms ? 1 : 0, rp, n, cur_stream()), "norm");
  return out;
}

void check_cache(const torch::Tensor& kc, const torch::Tensor& vc) {
  need(kc, torch::kBFloat16, "k_cache");
  need(vc, torch::kBFloat16, "v_cache");
  TORCH_CHECK(kc.dim() == 4 && kc.is_contiguous() && vc.is_contiguous() && kc.sizes() == vc.sizes(),
              "caches must be contiguous [slots, n_kv, max_seq, hd]");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(kc.data_ptr()) % 16 == 0 &&
              reinterpret_cast<uintptr_t>(vc.data_ptr()) % 16 == 0, "caches must be 16-byte aligned");
}

torch::Tensor attn_decode(torch::Tensor q, torch::Tensor kc, torch::Tensor vc,
                          torch::Tensor seq_slots, torch::Tensor qpos, int64_t nh,
                          int64_t splits) {
  need(q, torch::kBFloat16, "q");
  need_rows(q, "q");
  check_cache(kc, vc);
  const int B = q.size(0), n_kv = kc.size(1), hd = kc.size(3);
  TORCH_CHECK(q.size(1) == nh * hd && nh % n_kv == 0, "q must be [B, nh*hd]");
  TORCH_CHECK(hd == 64 || hd == 128, "head_dim must be 64 or 128");
  need(seq_slots, torch::kInt32, "seq_slots");
  need(qpos, torch::kInt32, "qpos");
  TORCH_CHECK(seq_slots.numel() == B && qpos.numel() == B, "seq_slots/qpos [B]");
  TORCH_CHECK(splits >= 1 && splits <= 256, "splits in [1, 256]");
  auto out = torch::empty({B, nh * hd}, q.options());
  torch::Tensor po, pml;
  float* pop = nullptr;
  float* pmlp = nullptr;
  if (splits > 1) {
    po = torch::empty({B, nh, splits, hd}, q.options().dtype(torch::kFloat32));
    pml = torch::empty({B, nh, splits, 2}, q.options().dtype(torch::kFloat32));
    pop = po.data_ptr<float>();
    pmlp = pml.data_ptr<float>();
  }
  const float sl2 = 1.4426950408889634f / std::sqrt((float)hd);
  check_hip(lsd_attn_decode(bptr(q), q.stride(0), bptr(kc), bptr(vc), seq_slots.data_ptr<int>(),
                            qpos.data_ptr<int>(), bptr_mut(out), out.stride(0), pop, pmlp, B, nh,
                            n_kv, hd, kc.size(2), splits, sl2, cur_stream()), "attn_decode");
  return out;
}

// x[B, N] += bias + attention(q, cache) @ w^T in ONE launch (B <= 4 decode
// rows): the fused attention + output projection + residual kernel.
void attn_oproj(torch::Tensor q, torch::Tensor kc, torch::Tensor vc, torch::Tensor seq_slots,
                torch::Tensor qpos, int64_t nh, torch::Tensor w, c10::optional<torch::Tensor> bias,
                torch::Tensor x, int64_t nc, torch::Tensor counters) {
  need(q, torch::kBFloat16, "q");
  need_rows(q, "q");
  check_cache(kc, vc);
  const int B = q.size(0), n_kv = kc.size(1), hd = kc.size(3);
  TORCH_CHECK(B >= 1 && B <= 4, "attn_oproj: 1 <= B <= 4 rows, got ", B);
  TORCH_CHECK(q.size(1) == nh * hd && nh % n_kv == 0, "q must be [B, nh*hd]");
  TORCH_CHECK(hd == 64 || hd == 128, "head_dim must be 64 or 128");
  const int G = nh / n_kv;
  TORCH_CHECK((hd == 64 && G == 1) || (hd == 128 && (G == 1 || G == 2 || G == 4 || G == 8)),
              "attn_oproj: unsupported head_dim / GQA group (", hd, ", ", G, ")");
  need(seq_slots, torch::kInt32, "seq_slots");
  need(qpos, torch::kInt32, "qpos");
  TORCH_CHECK(seq_slots.numel() == B && qpos.numel() == B, "seq_slots/qpos [B]");
  need(w, torch::kBFloat16, "w");
  need_rows(w, "w");
  TORCH_CHECK(w.size(1) == nh * hd, "w must be [N, nh*hd]");
  const int N = w.size(0);
  need(x, torch::kFloat32, "x");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && x.size(0) == B && x.size(1) == N, "x must be contiguous [B, N]");
  TORCH_CHECK(nc >= 1 && nc <= N, "column chunk in [1, N]");
  const int C = (N + nc - 1) / nc;
  need(counters, torch::kInt32, "counters");
  TORCH_CHECK(counters.is_contiguous() && counters.numel() >= C, "counter buffer too small");
  auto part = torch::empty({(long)C * n_kv * B * nc}, x.options());
  const float sl2 = 1.4426950408889634f / std::sqrt((float)hd);
  check_hip(lsd_attn_oproj(bptr(q), q.stride(0), bptr(kc), bptr(vc), seq_slots.data_ptr<int>(),
                           qpos.data_ptr<int>(), B, nh, n_kv, hd, kc.size(2), sl2, bptr(w), w.stride(0),
                           opt_bias(bias, N), x.data_ptr<float>(), N, (int)nc, part.data_ptr<float>(),
                           counters.data_ptr<int>(), cur_stream()),
            "attn_oproj");
}

torch::Tensor attn_prefill(torch::Tensor q, torch::Tensor kc, torch::Tensor vc,
                           torch::Tensor tiles, torch::Tensor seq_slots, torch::Tensor q_start,
                           torch::Tensor cu_q, int64_t nh) {
  need(q, torch::kBFloat16, "q");
  need_rows(q, "q");
  check_cache(kc, vc);
  const int n_kv = kc.size(1), hd = kc.size(3);
  TORCH_CHECK(q.size(1) == nh * hd && nh % n_kv == 0, "q must be [T, nh*hd]");
  TORCH_CHECK(hd == 64 || hd == 128, "head_dim must be 64 or 128");
  need(tiles, torch::kInt32, "tiles");
  TORCH_CHECK(tiles.dim() == 2 && tiles.size(1) == 2 && tiles.is_contiguous(), "tiles [n, 2]");
  need(seq_slots, torch::kInt32, "seq_slots");
  need(q_start, torch::kInt32, "q_start");
  need(cu_q, torch::kInt32, "cu_q");
  TORCH_CHECK(cu_q.numel() == seq_slots.numel() + 1, "cu_q [B+1]");
  auto out = torch::empty_like(q);
  const float sl2 = 1.4426950408889634f / std::sqrt((float)hd);
  check_hip(lsd_attn_prefill(bptr(q), q.stride(0), bptr(kc), bptr(vc), tiles.data_ptr<int>(),
                             tiles.size(0), seq_slots.data_ptr<int>(), q_start.data_ptr<int>(),
                             cu_q.data_ptr<int>(), bptr_mut(out), out.stride(0), nh, n_kv, hd,
                             kc.size(2), sl2, cur_stream()), "attn_prefill");
  return out;
}

void sample_launch(const torch::Tensor& logits, int64_t V, const torch::Tensor& temp,
                   const torch::Tensor& topk, const torch::Tensor& greedy, const torch::Tensor& seeds,
                   torch::Tensor& step, torch::Tensor& out, bool advance,
                   const c10::optional<torch::Tensor>& active = c10::nullopt,
                   const c10::optional<torch::Tensor>& pos = c10::nullopt,
                   const c10::optional<torch::Tensor>& segmax = c10::nullopt) {
  need(logits, torch::kFloat32, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.stride(1) == 1 && V <= logits.size(1) && V >= 1, "logits [B, >=V]");
  TORCH_CHECK(logits.stride(0) % 4 == 0 && logits.size(1) % 4 == 0, "logits row length must be a multiple of 4");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(logits.data_ptr()) % 16 == 0, "logits must be 16-byte aligned");
  const int B = logits.size(0);
  need(temp, torch::kFloat32, "temperature");
  need(topk, torch::kInt32, "top_k");
  need(greedy, torch::kInt32, "greedy");
  need(seeds, torch::kInt64, "seeds");
  need(step, torch::kInt64, "step");
  TORCH_CHECK(temp.numel() == B && topk.numel() == B && greedy.numel() == B && seeds.numel() == B &&
              step.numel() == B, "sampling params must be [B]");
  TORCH_CHECK(step.is_contiguous(), "step must be contiguous");
  need(out, torch::kInt32, "out");
  TORCH_CHECK(out.numel() == B && out.is_contiguous(), "out must be contiguous int32 [B]");
  const int* act = nullptr;
  if (active.has_value()) {
    need(*active, torch::kInt32, "active");
    TORCH_CHECK(active->numel() == B && active->is_contiguous(), "active must be contiguous int32 [B]");
    act = active->data_ptr<int>();
  }
  int* pp = nullptr;
  if (pos.has_value()) {
    need(*pos, torch::kInt32, "pos");
    TORCH_CHECK(pos->numel() == B && pos->is_contiguous(), "pos must be contiguous int32 [B]");
    pp = pos->data_ptr<int>();
  }
  const float* sm = nullptr;
  long ldseg = 0;
  if (segmax.has_value()) {  // linear_f32's segment maxima of these logits
    need(*segmax, torch::kFloat32, "segmax");
    TORCH_CHECK(segmax->dim() == 2 && segmax->is_contiguous() && segmax->size(0) == B &&
                logits.size(1) % 8 == 0 && segmax->size(1) == logits.size(1) / 8,
                "segmax must be contiguous fp32 [B, logits row length / 8]");
    sm = segmax->data_ptr<float>();
    ldseg = segmax->size(1);
  }
  check_hip(lsd_sample(logits.data_ptr<float>(), logits.stride(0), B, V, temp.data_ptr<float>(),
                       topk.data_ptr<int>(), greedy.data_ptr<int>(),
                       reinterpret_cast<const long long*>(seeds.data_ptr<int64_t>()),
                       reinterpret_cast<long long*>(step.data_ptr<int64_t>()),
                       out.data_ptr<int>(), advance ? 1 : 0, act, pp, sm, ldseg, cur_stream()), "sample");
}

// out[m, 16 j + i] = silu(y[m, 32 j + i]) * y[m, 32 j + 16 + i]: the SiLU * up
// pass over a gate/up-interleaved GEMM output (elementwise.hip)
// QKV epilogue over an fp32 GEMM output y [M, q_size + 2 kv_size] (the
// hipBLASLt decode path): returns q bf16 [M, q_size]; k, v (RoPE'd) into the
// caches -- the same contract as linear_qkv.
torch::Tensor qkv_post(torch::Tensor y, c10::optional<torch::Tensor> bias, torch::Tensor kc, torch::Tensor vc,
                       torch::Tensor tslot, torch::Tensor tpos, int64_t q_size, int64_t kv_size, int64_t hd,
                       c10::optional<torch::Tensor> rope) {
  need(y, torch::kFloat32, "y");
  const long M = y.size(0), N = y.size(1);
  TORCH_CHECK(y.dim() == 2 && y.stride(1) == 1 && y.stride(0) % 4 == 0 &&
              reinterpret_cast<uintptr_t>(y.data_ptr()) % 16 == 0, "qkv_post: y [M, N] with 16-byte rows");
  TORCH_CHECK(N == q_size + 2 * kv_size && hd % 8 == 0 && q_size % hd == 0 && kv_size % hd == 0,
              "qkv_post: N must be q_size + 2 kv_size, head dims multiples of 8");
  const lsd_bf16_t* b = opt_bias(bias, N);
  need(kc, torch::kBFloat16, "k_cache");
  need(vc, torch::kBFloat16, "v_cache");
  TORCH_CHECK(kc.dim() == 4 && kc.is_contiguous() && vc.sizes() == kc.sizes() && vc.is_contiguous(),
              "caches must be contiguous [slots, n_kv, max_seq, hd]");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(kc.data_ptr()) % 16 == 0 &&
              reinterpret_cast<uintptr_t>(vc.data_ptr()) % 16 == 0, "caches must be 16-byte aligned");
  TORCH_CHECK(kc.size(3) == hd && kc.size(1) * hd == kv_size, "cache shape mismatch");
  need(tslot, torch::kInt32, "token_slots");
  need(tpos, torch::kInt32, "token_pos");
  TORCH_CHECK(tslot.numel() == M && tpos.numel() == M && tslot.is_contiguous() && tpos.is_contiguous(),
              "token_slots/token_pos must be contiguous [M]");
  const float* rp = nullptr;
  if (rope.has_value()) {
    need(*rope, torch::kFloat32, "rope");
    TORCH_CHECK(rope->is_contiguous() && rope->dim() == 3 && rope->size(1) == hd / 2 && rope->size(2) == 2 &&
                rope->size(0) >= kc.size(2), "rope table must be [>=max_seq, hd/2, 2]");
    rp = rope->data_ptr<float>();
  }
  auto q = torch::empty({M, q_size}, y.options().dtype(torch::kBFloat16));
  check_hip(lsd_qkv_post(y.data_ptr<float>(), y.stride(0), b, tslot.data_ptr<int>(), tpos.data_ptr<int>(), rp,
                         reinterpret_cast<lsd_bf16_t*>(q.data_ptr()), bptr_mut(kc), bptr_mut(vc), (int)M,
                         (int)q_size, (int)kv_size, (int)hd, (int)kc.size(1), (int)kc.size(2), cur_stream()),
            "qkv_post");
  return q;
}

// Composition change of a decode group: args = the host int64 record of
// elementwise.hip lsd_apply_rows (CPU tensor), on the current stream.
void apply_rows(torch::Tensor args, int64_t b) {
  TORCH_CHECK(args.device().is_cpu() && args.scalar_type() == torch::kInt64 && args.is_contiguous() &&
                  args.numel() == 12, "apply_rows: args must be a contiguous CPU int64[12] record");
  check_hip(lsd_apply_rows(args.data_ptr<int64_t>(), (int)b, cur_stream()), "apply_rows");
}

torch::Tensor silu_mul(torch::Tensor y) {
  need(y, torch::kBFloat16, "y");
  TORCH_CHECK(y.dim() == 2 && y.stride(1) == 1 && y.size(1) % 32 == 0, "silu_mul: y [M, 2F], 2F % 32 == 0");
  TORCH_CHECK(y.stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(y.data_ptr()) % 16 == 0, "silu_mul: 16-byte rows");
  const int M = y.size(0), F = y.size(1) / 2;
  auto out = torch::empty({M, F}, y.options());
  check_hip(lsd_silu_mul(bptr(y), y.stride(0), reinterpret_cast<lsd_bf16_t*>(out.data_ptr()), F, M, F,
                         cur_stream()), "silu_mul");
  return out;
}

torch::Tensor sample(torch::Tensor logits, int64_t V, torch::Tensor temp, torch::Tensor topk,
                     torch::Tensor greedy, torch::Tensor seeds, torch::Tensor step,
                     c10::optional<torch::Tensor> segmax) {
  auto out = torch::empty({logits.size(0)}, logits.options().dtype(torch::kInt32));
  sample_launch(logits, V, temp, topk, greedy, seeds, step, out, false, c10::nullopt, c10::nullopt, segmax);
  return out;
}

// Decode-step form: the sampled ids go straight into `out` (the token-return
// vector) and each row's sampler counter -- and, given `pos`, the row's KV
// position of the last stage -- advances by active[row] (1 without `active`)
// in the same kernel.
void sample_into(torch::Tensor logits, int64_t V, torch::Tensor temp, torch::Tensor topk,
                 torch::Tensor greedy, torch::Tensor seeds, torch::Tensor step, torch::Tensor out,
                 c10::optional<torch::Tensor> active, c10::optional<torch::Tensor> pos,
                 c10::optional<torch::Tensor> segmax) {
  sample_launch(logits, V, temp, topk, greedy, seeds, step, out, true, active, pos, segmax);
}

}  // namespace

void lsd_register_comm(pybind11::module& m);  // csrc/comm.cpp
void lsd_register_exec(pybind11::module& m);  // csrc/stage_exec.cpp
void lsd_register_loopback(pybind11::module& m);  // csrc/loop_fabric.cpp
void lsd_register_blaslt(pybind11::module& m);    // csrc/blaslt.cpp

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "CDNA4 (gfx950) kernels for llm_sharding_demo_amd";
  lsd_register_comm(m);
  lsd_register_exec(m);
  lsd_register_loopback(m);
  lsd_register_blaslt(m);
  m.def("linear", &linear);
  m.def("linear_f32", &linear_f32, py::arg("a"), py::arg("w"), py::arg("tiled"), py::arg("splits"),
        py::arg("counters"), py::arg("segmax") = py::none());
  m.def("linear_residual", &linear_residual);
  m.def("linear_qkv", &linear_qkv);
  m.def("embed", &embed);
  m.def("norm", &norm);
  m.def("attn_decode", &attn_decode);
  m.def("attn_prefill", &attn_prefill);
  m.def("attn_oproj", &attn_oproj);
  m.def("sample", &sample, py::arg("logits"), py::arg("V"), py::arg("temp"), py::arg("topk"),
        py::arg("greedy"), py::arg("seeds"), py::arg("step"), py::arg("segmax") = py::none());
  m.def("sample_into", &sample_into, py::arg("logits"), py::arg("V"), py::arg("temp"), py::arg("topk"),
        py::arg("greedy"), py::arg("seeds"), py::arg("step"), py::arg("out"), py::arg("active"),
        py::arg("pos") = py::none(), py::arg("segmax") = py::none());
  m.def("gemv", [](torch::Tensor x, torch::Tensor w, c10::optional<torch::Tensor> bias, int64_t epi,
                   int64_t norm, c10::optional<torch::Tensor> gamma, c10::optional<torch::Tensor> beta,
                   double eps, c10::optional<torch::Tensor> resid, c10::optional<torch::Tensor> kc,
                   c10::optional<torch::Tensor> vc, c10::optional<torch::Tensor> tslot,
                   c10::optional<torch::Tensor> tpos, int64_t q_size, int64_t kv_size, int64_t hd,
                   c10::optional<torch::Tensor> rope) {
    return gemv(x, w, bias, epi, norm, gamma, beta, eps, resid, kc, vc, tslot, tpos, q_size, kv_size, hd, rope);
  });
  // fp32 logits GEMV that also writes the 8-column segment maxima (the sampler's threshold)
  m.def("gemv_logits", [](torch::Tensor x, torch::Tensor w, int64_t norm, c10::optional<torch::Tensor> gamma,
                          c10::optional<torch::Tensor> beta, double eps, torch::Tensor segmax) {
    return gemv(x, w, c10::nullopt, EPI_F32, norm, gamma, beta, eps, c10::nullopt, c10::nullopt,
                c10::nullopt, c10::nullopt, c10::nullopt, 0, 0, 0, c10::nullopt, segmax);
  });
  m.def("silu_mul", &silu_mul);
  m.def("apply_rows", &apply_rows, py::arg("args"), py::arg("b"));
  m.def("qkv_post", &qkv_post);
  // GEMV weight stream with non-temporal loads (A/B knob, LSD_GEMV_NT)
  m.def("gemv_set_nt", [](int64_t v) { lsd_gemv_set_nt((int)v); });
  m.def("gemv_ok", [](int64_t M, int64_t K, int64_t epi, int64_t norm) {
    return lsd_gemv_ok((int)M, (int)K, (int)epi, (int)norm) != 0; });
  m.def("set_stamps", &set_stamps);
  // tiled GEMMs with >= this many 256x256 tiles use the pipelined 256^2 kernel
  m.def("gemm_set_big_min", [](int64_t v) { lsd_gemm_set_big_min((int)v); });
  // large-GEMM tile order: groups of this many row panels (0 = M-fastest)
  m.def("gemm_set_big_group", [](int64_t v) { lsd_gemm_set_big_group((int)v); });
  // large-GEMM kernel: 0 = BK=32 ring (gemm_big), 1 = phase-pipelined BK=64 (gemm_p8)
  m.def("gemm_set_big_kind", [](int64_t v) { lsd_gemm_set_big_kind((int)v); });
  m.def("gemm_set_tiled3_max", [](int64_t v) { lsd_gemm_set_tiled3_max((int)v); });
  m.def("gemm_set_ring_slots", [](int64_t v) { lsd_gemm_set_ring_slots((int)v); });
  m.def("gemm_set_ring_tn", [](int64_t v) { lsd_gemm_set_ring_tn((int)v); });
  m.def("gemm_set_ring_fill", [](int64_t v) { lsd_gemm_set_ring_fill((int)v); });
  m.def("gemm_set_ring_m96", [](int64_t v) { lsd_gemm_set_ring_m96((int)v); });
  // gemm_d256 (launch kind 2 / 3: all <= 256 rows in one tile, 64 / 128 columns): ring depth
  m.def("gemm_set_d256_slots", [](int64_t v) { lsd_gemm_set_d256_slots((int)v); });
  m.def("gemm_set_ring8", [](int64_t v) { lsd_gemm_set_ring8((int)v); });
  m.def("gemm_ring8_tiles", [](int64_t M, int64_t N, int64_t K, int64_t S) {
    return (int64_t)lsd_gemm_ring8_tiles((int)M, (int)N, (int)K, (int)S);
  });
  m.def("gemm_set_ring8_flags", [](int64_t v) { lsd_gemm_set_ring8_flags((int)v); });
  m.def("gemm_set_ring8_pack", [](int64_t v) { lsd_gemm_set_ring8_pack((int)v); });
  // prefill norms: one wave per row from this many rows (0 = the block-per-row kernel only)
  m.def("norm_set_wave_min", [](int64_t v) { lsd_norm_set_wave_min((int)v); });
  m.def("norm_set_wave_narrow_min", [](int64_t v) { lsd_norm_set_wave_narrow_min((int)v); });
  m.def("gemm_d256_bn", [](int64_t kind, int64_t M, int64_t N, int64_t K) {
    return lsd_gemm_d256_bn((int)kind, (int)M, (int)N, (int)K);
  });
  // decode attention: cap the grid (blocks loop over (sequence, head) items)
  m.def("attn_set_max_wg", [](int64_t v) { lsd_attn_set_max_wg((int)v); });
  // decode attention: waves per block when the batch has few (sequence, head) items
  m.def("attn_set_small_waves", [](int64_t v) { lsd_attn_set_small_waves((int)v); });
  m.def("attn_set_small_waves128", [](int64_t v) { lsd_attn_set_small_waves128((int)v); });
  m.def("attn_set_large_waves", [](int64_t hd, int64_t v) { lsd_attn_set_large_waves((int)hd, (int)v); });
  // grouped-query MFMA decode attention from this many (sequence, kv head) items (0 = off)
  m.def("attn_set_mfma_min", [](int64_t v) { lsd_attn_set_mfma_min((int)v); });
  // decode GEMM: rows per row block (M above it runs as several row blocks)
  m.def("gemm_set_sk_rows", [](int64_t v) { lsd_gemm_set_sk_rows((int)v); });
  m.def("gemm_set_slab_bf16", [](int64_t v) { g_slab_bf16 = v ? 1 : 0; });
  m.def("gemm_slab_bf16", [] { return slab_bf16_enabled(); });
  m.def("gemm_sk_rblocks", [](int64_t M, int64_t N, int64_t S) { return lsd_gemm_sk_rblocks((int)M, (int)N, (int)S); });
  // decode GEMM column tile 128 (NW = 2) above this many rows
  m.def("gemm_set_nw2_rows", [](int64_t v) { lsd_gemm_set_nw2_rows((int)v); });
  m.def("gemm_sk_nw", [](int64_t M, int64_t epi) { return lsd_gemm_sk_nw((int)M, (int)epi); });
  // A HIP stream whose kernels may only run on the CUs set in `mask` (32-bit
  // words; bit i = CU i of the device's mask numbering) -- spatial
  // partitioning of the chip between microbatch lanes (parallel/pipeline.py
  // LSD_LANE_CU_MASK).  Returns the raw hipStream_t for torch.cuda.ExternalStream;
  // the stream lives until the process exits.
  m.def("stream_with_cu_mask", [](std::vector<int64_t> mask) {
    std::vector<uint32_t> m32(mask.begin(), mask.end());
    hipStream_t s = nullptr;
    check_hip(hipExtStreamCreateWithCUMask(&s, (uint32_t)m32.size(), m32.data()), "hipExtStreamCreateWithCUMask");
    return reinterpret_cast<int64_t>(s);
  });
  m.def("stream_cu_mask", [](int64_t stream, int64_t words) {
    std::vector<uint32_t> m32((size_t)words, 0u);
    check_hip(hipExtStreamGetCUMask(reinterpret_cast<hipStream_t>(stream), (uint32_t)words, m32.data()),
              "hipExtStreamGetCUMask");
    return std::vector<int64_t>(m32.begin(), m32.end());
  });
  m.def("device_cu_count", []() {
    int dev = 0, n = 0;
    check_hip(hipGetDevice(&dev), "hipGetDevice");
    check_hip(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev), "hipDeviceGetAttribute");
    return n;
  });
  m.attr("arch") = "gfx950";
}
