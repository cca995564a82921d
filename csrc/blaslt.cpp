// hipBLASLt as an opt-in A/B oracle (ops/routing.py `blaslt=1`; off by
// default: every hot-path GEMM runs on the hand-written kernels of
// csrc/kernels).  It runs the projections whose epilogue the library fuses:
//   * MLP-up: y = gelu_new(a @ w^T + b), bf16 out      (HIPBLASLT_EPILOGUE_GELU_BIAS)
//   * residual projections: x += a @ w^T + b, fp32 x   (beta = 1 with C = D = x,
//     HIPBLASLT_EPILOGUE_BIAS; bf16 A / B, fp32 C / D)
//   * a plain fp32-out GEMM (blaslt_f32) for the QKV comparison, whose RoPE /
//     cache append then runs as kernels/elementwise.hip qkv_post.
// Row-major y[M, N] = a[M, K] w[N, K]^T is the column-major D[N, M] =
// op_T(W[K, N]) B[K, M]: transa = T, m = N, n = M; the bias runs along D's
// rows (our columns) as the epilogue expects.
//
// One handle and heuristic cache per device.  Only workspace-free algorithms
// are accepted, so GEMMs issued concurrently -- two lanes of a stage, or the
// stages of a one-GPU multi-stage rehearsal on their own streams, eager or
// graph-captured -- share no scratch memory.  The plan cache is bounded
// (descriptors destroyed when it overflows: prefill M varies with the chunk
// token count) and the fp32 copy of a residual bias is made once per weight.
// The bindings report "no algorithm" (None / false, nothing issued) and the
// caller then keeps the hand-written kernel.
#include <torch/extension.h>

#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>
#include <hipblaslt/hipblaslt.h>

#include <map>
#include <mutex>
#include <stdexcept>
#include <string>
#include <tuple>

namespace {

void lt_check(hipblasStatus_t s, const char* what) {
  if (s != HIPBLAS_STATUS_SUCCESS) throw std::runtime_error(std::string("hipBLASLt ") + what + " failed: " + std::to_string((int)s));
}

constexpr size_t kMaxPlans = 256;

struct Plan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  bool ok = false;
};

struct DeviceState {
  hipblasLtHandle_t handle = nullptr;
  std::map<std::tuple<long, long, long, int, int>, Plan> plans;  // (M, N, K, epilogue, fp32 out)
  std::map<std::pair<const void*, long>, torch::Tensor> bias32;  // fp32 copies of residual biases
};

std::mutex g_mu;
std::map<int, DeviceState> g_dev;

DeviceState& state(const torch::Tensor& like) {
  const int dev = like.get_device();
  auto& s = g_dev[dev];
  if (!s.handle) lt_check(hipblasLtCreate(&s.handle), "create");
  return s;
}

void destroy(Plan& p) {
  if (p.desc) hipblasLtMatmulDescDestroy(p.desc);
  if (p.la) hipblasLtMatrixLayoutDestroy(p.la);
  if (p.lb) hipblasLtMatrixLayoutDestroy(p.lb);
  if (p.lc) hipblasLtMatrixLayoutDestroy(p.lc);
  p = Plan{};
}

// The plan for y[M, N] (bf16, or fp32 accumulated into C = D) = a[M, K] w[N, K]^T
Plan& plan(DeviceState& s, long M, long N, long K, hipblasLtEpilogue_t epi, bool f32out) {
  auto key = std::make_tuple(M, N, K, (int)epi, (int)f32out);
  auto it = s.plans.find(key);
  if (it != s.plans.end()) return it->second;
  if (s.plans.size() >= kMaxPlans) {  // bounded: drop every plan (the stream order keeps
    for (auto& kv : s.plans) destroy(kv.second);  // earlier enqueued GEMMs valid: the
    s.plans.clear();                              // library copies what it needs at launch)
  }
  Plan p;
  lt_check(hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F), "desc");
  const hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
  lt_check(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)), "transa");
  lt_check(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)), "transb");
  lt_check(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi)), "epilogue");
  // the bias type must be D's or the scale type's: bf16 with a bf16 D, fp32
  // (converted per call, N floats) with the fp32 residual
  const hipDataType bt = f32out ? HIP_R_32F : HIP_R_16BF;
  lt_check(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)), "bias type");
  lt_check(hipblasLtMatrixLayoutCreate(&p.la, HIP_R_16BF, K, N, K), "layout A");
  lt_check(hipblasLtMatrixLayoutCreate(&p.lb, HIP_R_16BF, K, M, K), "layout B");
  lt_check(hipblasLtMatrixLayoutCreate(&p.lc, f32out ? HIP_R_32F : HIP_R_16BF, N, M, N), "layout C");
  hipblasLtMatmulPreference_t pref;
  lt_check(hipblasLtMatmulPreferenceCreate(&pref), "preference");
  const uint64_t ws = 0;  // workspace-free algorithms only (see the header)
  lt_check(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &ws, sizeof(ws)),
           "workspace");
  hipblasLtMatmulHeuristicResult_t res[1];
  int n = 0;
  const hipblasStatus_t hs =
      hipblasLtMatmulAlgoGetHeuristic(s.handle, p.desc, p.la, p.lb, p.lc, p.lc, pref, 1, res, &n);
  hipblasLtMatmulPreferenceDestroy(pref);
  if (hs == HIPBLAS_STATUS_SUCCESS && n > 0 && res[0].state == HIPBLAS_STATUS_SUCCESS &&
      res[0].workspaceSize == 0) {
    p.algo = res[0].algo;
    p.ok = true;
  }
  return s.plans.emplace(key, p).first->second;
}

void check_operands(const torch::Tensor& a, const torch::Tensor& w) {
  TORCH_CHECK(a.is_cuda() && w.is_cuda() && a.scalar_type() == torch::kBFloat16 && w.scalar_type() == torch::kBFloat16,
              "blaslt: bf16 device operands");
  TORCH_CHECK(a.dim() == 2 && w.dim() == 2 && a.size(1) == w.size(1), "blaslt: a [M, K], w [N, K]");
  TORCH_CHECK(a.is_contiguous() && w.is_contiguous(), "blaslt: contiguous operands");
}

const void* bias_ptr(const c10::optional<torch::Tensor>& bias, long N) {
  if (!bias.has_value()) return nullptr;
  TORCH_CHECK(bias->scalar_type() == torch::kBFloat16 && bias->numel() == N && bias->is_contiguous(),
              "blaslt: bias must be contiguous bf16 [N]");
  return bias->data_ptr();
}

void run(DeviceState& s, Plan& p, const void* bias, const torch::Tensor& a, const torch::Tensor& w,
         float beta, void* cd) {
  if (bias)
    lt_check(hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bias, sizeof(bias)),
             "bias pointer");
  const float alpha = 1.f;
  auto st = at::hip::getCurrentHIPStream().stream();
  lt_check(hipblasLtMatmul(s.handle, p.desc, &alpha, w.data_ptr(), p.la, a.data_ptr(), p.lb, &beta, cd, p.lc, cd,
                           p.lc, &p.algo, nullptr, 0, st),
           "matmul");
}

}  // namespace

void lsd_register_blaslt(pybind11::module& m) {
  // y = act(a @ w^T + bias), bf16 [M, N]; act 0 none, 1 GELU.  None when the
  // library has no algorithm for the shape (use the hand-written kernel)
  m.def("blaslt_linear", [](torch::Tensor a, torch::Tensor w, c10::optional<torch::Tensor> bias,
                            int64_t act, int64_t lane) -> c10::optional<torch::Tensor> {
    check_operands(a, w);
    const c10::DeviceGuard guard(a.device());
    TORCH_CHECK(act == 0 || act == 1, "blaslt_linear: act 0 (none) or 1 (GELU)");
    const long M = a.size(0), N = w.size(0), K = a.size(1);
    const void* b = bias_ptr(bias, N);
    const hipblasLtEpilogue_t epi = act == 1 ? (b ? HIPBLASLT_EPILOGUE_GELU_BIAS : HIPBLASLT_EPILOGUE_GELU)
                                             : (b ? HIPBLASLT_EPILOGUE_BIAS : HIPBLASLT_EPILOGUE_DEFAULT);
    std::lock_guard<std::mutex> lk(g_mu);
    auto& s = state(a);
    auto& p = plan(s, M, N, K, epi, false);
    if (!p.ok) return c10::nullopt;
    auto y = torch::empty({M, N}, a.options());
    run(s, p, b, a, w, 0.f, y.data_ptr());
    return y;
  }, py::arg("a"), py::arg("w"), py::arg("bias"), py::arg("act"), py::arg("lane") = 0);
  // y = a @ w^T, fp32 [M, N] (no bias: the caller's pass adds it -- the QKV
  // epilogue, kernels/elementwise.hip qkv_post); None when no algorithm
  m.def("blaslt_f32", [](torch::Tensor a, torch::Tensor w, int64_t lane) -> c10::optional<torch::Tensor> {
    check_operands(a, w);
    const c10::DeviceGuard guard(a.device());
    const long M = a.size(0), N = w.size(0), K = a.size(1);
    std::lock_guard<std::mutex> lk(g_mu);
    auto& s = state(a);
    auto& p = plan(s, M, N, K, HIPBLASLT_EPILOGUE_DEFAULT, true);
    if (!p.ok) return c10::nullopt;
    auto y = torch::empty({M, N}, a.options().dtype(torch::kFloat32));
    run(s, p, nullptr, a, w, 0.f, y.data_ptr());
    return y;
  }, py::arg("a"), py::arg("w"), py::arg("lane") = 0);
  // x += a @ w^T + bias (x fp32 [M, N], in place); false when the library has
  // no algorithm for the shape (nothing was issued)
  m.def("blaslt_residual", [](torch::Tensor a, torch::Tensor w, c10::optional<torch::Tensor> bias,
                              torch::Tensor x, int64_t lane) -> bool {
    check_operands(a, w);
    const c10::DeviceGuard guard(a.device());
    const long M = a.size(0), N = w.size(0), K = a.size(1);
    TORCH_CHECK(x.scalar_type() == torch::kFloat32 && x.is_contiguous() && x.dim() == 2 && x.size(0) == M &&
                x.size(1) == N, "blaslt_residual: x must be contiguous fp32 [M, N]");
    const void* bb = bias_ptr(bias, N);  // checks
    std::lock_guard<std::mutex> lk(g_mu);
    auto& s = state(a);
    const void* b = nullptr;
    if (bb) {  // fp32 copy of the (persistent) bias, made once
      auto key = std::make_pair(bb, N);
      auto it = s.bias32.find(key);
      if (it == s.bias32.end()) {
        if (s.bias32.size() >= 1024) s.bias32.clear();
        it = s.bias32.emplace(key, bias->to(torch::kFloat32)).first;
      }
      b = it->second.data_ptr();
    }
    auto& p = plan(s, M, N, K, b ? HIPBLASLT_EPILOGUE_BIAS : HIPBLASLT_EPILOGUE_DEFAULT, true);
    if (!p.ok) return false;
    run(s, p, b, a, w, 1.f, x.data_ptr());
    return true;
  }, py::arg("a"), py::arg("w"), py::arg("bias"), py::arg("x"), py::arg("lane") = 0);
}
