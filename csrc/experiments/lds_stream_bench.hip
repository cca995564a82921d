// Per-CU streaming rate into LDS on MI355X: is LDS-DMA (global_load_lds)
// the ceiling of the decode / prefill GEMM k-loops (~30-40 GB/s per CU)?
// Each workgroup (4 waves) streams NSTEP steps of 24 KiB (6 x 1 KiB
// wave-instructions per wave... 6 x 16 B per thread) through a ring of SLOTS
// LDS slots, D = SLOTS-1 steps in flight, one s_barrier per step -- the
// gemm_ring_kernel structure with the MFMAs removed.
//   MODE 0: LDS-DMA, global_load_lds 16 B per lane
//   MODE 1: global_load_dwordx4 to VGPRs, ds_write_b128 one step later
//   MODE 2: global_load_dwordx4 to VGPRs only (summed; no LDS)
// ROWSTRIDE: 1 KiB wave-instructions as 8 rows x 128 B at a 3200-B pitch
// (a K = 1600 bf16 operand) instead of contiguous.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); std::exit(1); } } while (0)

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void gbl_cvoid;
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int LPS = 6;                  // 16-B loads per thread per step
constexpr int STEP_BYTES = 256 * LPS * 16;  // 24 KiB

constexpr int vmcnt_imm(int n) { return (n & 0xF) | ((n >> 4) << 14) | (0x7 << 4) | (0xF << 8); }

template <bool ROWSTRIDE>
__device__ __forceinline__ const char* src_addr(const char* base, int step, int l) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int inst = w * LPS + l;  // 24 wave-instructions of 1 KiB per step
  if (ROWSTRIDE) {
    // step = 64-k column block; inst -> 8 rows; rows 3200 B apart
    const long row = inst * 8 + (lane >> 3);
    return base + row * 3200 + (long)step * 128 + (lane & 7) * 16;
  }
  return base + (long)step * STEP_BYTES + inst * 1024 + lane * 16;
}

template <int MODE, int SLOTS, bool ROWSTRIDE>
__global__ __launch_bounds__(256) void stream_kernel(const char* data, long per_wg, int nstep, float* sink) {
  constexpr int D = SLOTS - 1;
  __shared__ __attribute__((aligned(16))) char lds[SLOTS * STEP_BYTES];
  const char* base = data + (long)blockIdx.x * per_wg;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  f32x4 reg[D][LPS];
  auto issue = [&](int s, int slot) {
#pragma unroll
    for (int l = 0; l < LPS; ++l) {
      const char* g = src_addr<ROWSTRIDE>(base, s, l);
      if (MODE == 0)
        __builtin_amdgcn_global_load_lds((gbl_cvoid*)g, (lds_void*)(lds + slot * STEP_BYTES + (w * LPS + l) * 1024), 16, 0, 0);
      else
        reg[slot % D][l] = *reinterpret_cast<const f32x4*>(g);
    }
  };
  if (MODE == 0) {
#pragma unroll
    for (int d = 0; d < D; ++d) issue(d, d);
    int slot = 0;
    for (int s = 0; s < nstep; ++s) {
      const int later = min(D - 1, nstep - 1 - s);
      if (later >= 2) __builtin_amdgcn_s_waitcnt(vmcnt_imm(2 * LPS));
      else if (later == 1) __builtin_amdgcn_s_waitcnt(vmcnt_imm(LPS));
      else __builtin_amdgcn_s_waitcnt(vmcnt_imm(0));
      __builtin_amdgcn_s_barrier();
      if (s + D < nstep) issue(s + D, slot == 0 ? SLOTS - 1 : slot - 1);
      acc += *reinterpret_cast<const f32x4*>(lds + slot * STEP_BYTES + threadIdx.x * 16);
      slot = slot == SLOTS - 1 ? 0 : slot + 1;
    }
  } else {
    // register staging: loads for step s+D in flight while step s is written
    // to LDS (MODE 1) or summed (MODE 2)
    for (int s0 = 0; s0 < nstep; s0 += D) {
#pragma unroll
      for (int d = 0; d < D; ++d)
        if (s0 + d < nstep) issue(s0 + d, d);
#pragma unroll
      for (int d = 0; d < D; ++d) {
        if (s0 + d >= nstep) break;
#pragma unroll
        for (int l = 0; l < LPS; ++l) {
          if (MODE == 1)
            *reinterpret_cast<f32x4*>(lds + d * STEP_BYTES + (w * LPS + l) * 1024 + lane * 16) = reg[d][l];
          else
            acc += reg[d][l];
        }
      }
      if (MODE == 1) {
        __syncthreads();
        acc += *reinterpret_cast<const f32x4*>(lds + threadIdx.x * 16);
      }
    }
  }
  if (acc[0] == -1.f) sink[0] = acc[1];
}

template <int MODE, int SLOTS, bool RS>
void run(const char* data, float* sink, int grid, int nstep, const char* name, bool shared = false) {
  const long per_wg = shared ? 0 : RS ? 3200L * 192 : (long)nstep * STEP_BYTES;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(a));
    hipLaunchKernelGGL((stream_kernel<MODE, SLOTS, RS>), dim3(grid), dim3(256), 0, 0, data, per_wg, nstep, sink);
    CK(hipGetLastError());
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    if (rep == 2) {
      const double bytes = (double)grid * nstep * STEP_BYTES;
      std::printf("%-28s grid %3d slots %d: %8.2f us  %6.2f TB/s total  %6.1f GB/s per WG  %5.3f us/step\n", name, grid,
                  SLOTS, ms * 1e3, bytes / ms / 1e9, bytes / grid / ms / 1e6, ms * 1e3 / nstep);
    }
  }
}

int main() {
  const long total = 1L << 30;
  char* data;
  float* sink;
  CK(hipMalloc(&data, total));
  CK(hipMemset(data, 1, total));
  CK(hipMalloc(&sink, 4));
  // every workgroup reads the SAME region (L2-resident after the first pass):
  // the A-operand pattern of a decode GEMM
  for (int grid : {150, 256}) {
    run<0, 3, true>(data, sink, grid, 25, "SHARED lds-dma rowstride", true);
    run<1, 3, true>(data, sink, grid, 25, "SHARED vgpr->ds_write rs", true);
    run<2, 3, true>(data, sink, grid, 25, "SHARED vgpr only rowstride", true);
    run<0, 3, false>(data, sink, grid, 64, "SHARED lds-dma contiguous", true);
    run<2, 3, false>(data, sink, grid, 64, "SHARED vgpr only contig", true);
  }
  for (int grid : {150, 256}) {
    // contiguous: 64 steps x 24 KiB per workgroup (fresh HBM data)
    run<0, 3, false>(data, sink, grid, 64, "lds-dma contiguous");
    run<0, 4, false>(data, sink, grid, 64, "lds-dma contiguous");
    run<1, 3, false>(data, sink, grid, 64, "vgpr->ds_write contiguous");
    run<2, 3, false>(data, sink, grid, 64, "vgpr only contiguous");
    run<2, 5, false>(data, sink, grid, 64, "vgpr only contiguous");
    // row-strided like a K = 1600 operand: 25 k-steps of 128 B per row
    run<0, 3, true>(data, sink, grid, 25, "lds-dma rowstride");
    run<1, 3, true>(data, sink, grid, 25, "vgpr->ds_write rowstride");
    run<2, 3, true>(data, sink, grid, 25, "vgpr only rowstride");
  }
  return 0;
}
