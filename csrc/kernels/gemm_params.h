// GEMM launch parameters shared by csrc/kernels/gemm.hip and csrc/bindings.cpp.
#pragma once

#if defined(__clang__)
typedef __bf16 lsd_bf16_t;
#else
typedef unsigned short lsd_bf16_t;  // host-only: storage-compatible, pointers only
#endif

namespace lsd {

struct GemmParams {
  const lsd_bf16_t* A; long lda;
  const lsd_bf16_t* W; long ldw;
  int M, N, K;
  const lsd_bf16_t* bias;
  void* out; long ldo;
  float* slab;
  int splits;
  // QKV epilogue
  lsd_bf16_t* kc; lsd_bf16_t* vc;  // [slots][n_kv][max_seq][hd]
  const int* tslot; const int* tpos;
  int q_size, kv_size, hd, max_seq, n_kv;
  const float* rope;  // [max_pos][hd/2][2] (cos, sin), or null
  long long* stamps;  // diagnostic builds only: per-workgroup s_memrealtime phase stamps
  int slab_bf16;      // EPI_SLAB: partial slabs stored bf16 instead of fp32 (LSD_SLAB_BF16)
  // EPI_F32 (tiled kernels): also the max of every 8-column segment,
  // segmax[m * ldseg + n / 8] -- the sampler's first pass, fused (sample.hip)
  float* segmax; long ldseg;
};

// Small-M (M <= 8) weight-streaming GEMV with an optional fused input norm
// (csrc/kernels/gemv.hip).  Epilogue codes are the GemmParams ones.
struct GemvParams {
  const lsd_bf16_t* A; long lda;      // bf16 input rows [M][K] (norm == 0)
  const float* X; long ldx;           // fp32 residual rows [M][K] (norm != 0)
  const lsd_bf16_t* gamma;            // norm weight [K]
  const lsd_bf16_t* beta;             // LayerNorm bias [K] (null: RMSNorm)
  float eps;
  const lsd_bf16_t* W; long ldw;      // [N][K]
  int M, N, K;
  const lsd_bf16_t* bias;             // [N] or null
  void* out; long ldo;                // bf16 / f32 out, or the fp32 residual (EPI_RESID)
  // QKV epilogue (same meaning as GemmParams)
  lsd_bf16_t* kc; lsd_bf16_t* vc;
  const int* tslot; const int* tpos;
  int q_size, kv_size, hd, max_seq, n_kv;
  const float* rope;
  int nt;                             // 1: stream W with non-temporal loads
  // fp32 logits epilogue: also the max of every 8-column segment (one
  // workgroup = 8 columns) per row, [M][ldseg] -- the sampler's top-k threshold
  float* segmax; long ldseg;
};

}  // namespace lsd
