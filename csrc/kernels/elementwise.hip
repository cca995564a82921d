// SiLU(gate) * up over a gate/up-interleaved GEMM output (Llama MLP).
//
// The gate_up weight is stored in 32-row blocks [gate 16 | up 16]
// (ops/hip.py interleave_gate_up), so the fused GEMM epilogue (gemm.hip
// EPI_SILU_MUL) pairs each gate column with the up column 16 to its right.
// When the GEMM itself runs elsewhere (hipBLASLt at 512 decode rows,
// csrc/blaslt.cpp) its bf16 output [M, 2F] goes through this pass: one thread
// per 8 outputs, 16-byte loads of the gate and up chunks, fp32 math, one
// 16-byte store -- out[m, 16 j + i] = silu(y[m, 32 j + i]) * y[m, 32 j + 16 + i].
#include "common.h"

namespace lsd {

__global__ __launch_bounds__(256) void silu_mul_kernel(const bf16* __restrict__ y, long ldy,
                                                       bf16* __restrict__ out, long ldo, int M, int F) {
  const long per_row = F / 8;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)M * per_row) return;
  const int m = (int)(idx / per_row);
  const int o = (int)(idx % per_row) * 8;  // first of 8 outputs
  const int j = o >> 4, i = o & 15;
  const bf16* row = y + (long)m * ldy + (long)j * 32 + i;
  const bf16x8 g = ld8(row), u = ld8(row + 16);
  bf16x8 r;
#pragma unroll
  for (int e = 0; e < 8; ++e) r[e] = f2bf(silu(bf2f(g[e])) * bf2f(u[e]));
  st8(out + (long)m * ldo + o, r);
}

}  // namespace lsd

using namespace lsd;

extern "C" hipError_t lsd_silu_mul(const bf16* y, long ldy, bf16* out, long ldo, int M, int F,
                                   hipStream_t st) {
  if (M == 0) return hipSuccess;
  if (F % 16 != 0) return hipErrorInvalidValue;
  const long n = (long)M * (F / 8);
  hipLaunchKernelGGL(silu_mul_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, y, ldy, out, ldo, M, F);
  return hipGetLastError();
}
