// Grid-barrier cost on MI355X: the building block of a persistent decode
// kernel.  Every workgroup bumps one device-scope counter (release) and
// spins on it (acquire) until all have arrived; the spin is bounded, so a
// grid that is not fully co-resident exits with an error flag instead of
// hanging.  Prints us per barrier for a few grid sizes.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); std::exit(1); } } while (0)

__device__ __forceinline__ void grid_barrier(unsigned* ctr, unsigned target, int* err) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    unsigned spins = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 22)) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

// Two-level: workgroups arrive on one of 8 group counters (blockIdx % 8, the
// XCD of a round-robin dispatch); the last of a group arrives on the top
// counter; the last of those publishes the generation that everyone polls.
template <bool REL = true, bool ACQ = true>
__device__ __forceinline__ void grid_barrier2(unsigned* ctr, unsigned gen, int* err) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned ng = 8, per = gridDim.x / ng;
    unsigned* grp = ctr + 32 * (1 + blockIdx.x % ng);
    unsigned* top = ctr + 32 * 9;
    unsigned* rel = ctr;
    if (REL) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const unsigned o = __hip_atomic_fetch_add(grp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (o == gen * per - 1) {
      const unsigned t = __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (t == gen * ng - 1) __hip_atomic_store(rel, gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    unsigned spins = 0;
    while (__hip_atomic_load(rel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < gen) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 22)) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    if (ACQ) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

// Master: each workgroup stores its generation to its own flag line; wave 0
// of workgroup 0 polls all flags and publishes the generation.
__device__ __forceinline__ void grid_barrier3(unsigned* ctr, unsigned gen, int* err) {
  __syncthreads();
  unsigned* rel = ctr;
  unsigned* flags = ctr + 32 * 16;
  if (threadIdx.x == 0) __hip_atomic_store(flags + 32 * blockIdx.x, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  if (blockIdx.x == 0 && threadIdx.x < 64) {
    unsigned spins = 0;
    for (;;) {
      bool ok = true;
      for (unsigned b = threadIdx.x; b < gridDim.x; b += 64)
        ok &= __hip_atomic_load(flags + 32 * b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= gen;
      if (__all(ok)) break;
      if (++spins > (1u << 22)) {
        if (threadIdx.x == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    if (threadIdx.x == 0) __hip_atomic_store(rel, gen, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (threadIdx.x == 0) {
    unsigned spins = 0;
    while (__hip_atomic_load(rel, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < gen) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 22)) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

template <int KIND>
__global__ __launch_bounds__(256) void bar_kernel2(unsigned* ctr, int nbar, int* err) {
  for (int i = 1; i <= nbar; ++i) {
    if (KIND == 2) grid_barrier2(ctr, (unsigned)i, err);
    else if (KIND == 4) grid_barrier2<false, false>(ctr, (unsigned)i, err);
    else if (KIND == 5) grid_barrier2<true, false>(ctr, (unsigned)i, err);
    else if (KIND == 6) grid_barrier2<false, true>(ctr, (unsigned)i, err);
    else grid_barrier3(ctr, (unsigned)i, err);
  }
}

// WRITE: each barrier is preceded by a 1 KB store per workgroup that the next
// phase's workgroups read back (the activation hand-off of a decode layer).
template <bool WRITE>
__global__ __launch_bounds__(256) void bar_kernel(unsigned* ctr, int nbar, int* err, float* buf, float* sink) {
  float acc = 0.f;
  for (int i = 1; i <= nbar; ++i) {
    if (WRITE) buf[(i & 1) * gridDim.x * 256 + blockIdx.x * 256 + threadIdx.x] = (float)i;
    grid_barrier(ctr, (unsigned)i * gridDim.x, err);
    if (WRITE) acc += buf[(i & 1) * gridDim.x * 256 + ((blockIdx.x + 1) % gridDim.x) * 256 + threadIdx.x];
  }
  if (acc == -1.f) sink[0] = acc;
}

int main() {
  unsigned* ctr;
  int* err;
  float *buf, *sink;
  CK(hipMalloc(&ctr, 4));
  CK(hipMalloc(&err, 4));
  CK(hipMalloc(&buf, 2 * 1024 * 256 * 4));
  CK(hipMalloc(&sink, 4));
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  std::printf("CUs %d\n", p.multiProcessorCount);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int nbar = 2000;
  for (int write = 0; write < 2; ++write)
    for (int grid : {256}) {
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipMemset(ctr, 0, 4));
        CK(hipMemset(err, 0, 4));
        CK(hipEventRecord(a));
        if (write) hipLaunchKernelGGL(bar_kernel<true>, dim3(grid), dim3(256), 0, 0, ctr, nbar, err, buf, sink);
        else hipLaunchKernelGGL(bar_kernel<false>, dim3(grid), dim3(256), 0, 0, ctr, nbar, err, buf, sink);
        CK(hipGetLastError());
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        int e = 0;
        CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
        if (rep == 1) std::printf("write=%d grid=%d: %.3f us per barrier%s\n", write, grid, ms * 1000.f / nbar, e ? "  (TIMEOUT)" : "");
      }
    }
  unsigned* ctr2;
  CK(hipMalloc(&ctr2, 4 * 32 * (16 + 1024)));
  for (int kind = 2; kind <= 6; ++kind)
    for (int grid : {128, 256, 512}) {
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipMemset(ctr2, 0, 4 * 32 * (16 + 1024)));
        CK(hipMemset(err, 0, 4));
        CK(hipEventRecord(a));
        if (kind == 2) hipLaunchKernelGGL(bar_kernel2<2>, dim3(grid), dim3(256), 0, 0, ctr2, nbar, err);
        else if (kind == 3) hipLaunchKernelGGL(bar_kernel2<3>, dim3(grid), dim3(256), 0, 0, ctr2, nbar, err);
        else if (kind == 4) hipLaunchKernelGGL(bar_kernel2<4>, dim3(grid), dim3(256), 0, 0, ctr2, nbar, err);
        else if (kind == 5) hipLaunchKernelGGL(bar_kernel2<5>, dim3(grid), dim3(256), 0, 0, ctr2, nbar, err);
        else hipLaunchKernelGGL(bar_kernel2<6>, dim3(grid), dim3(256), 0, 0, ctr2, nbar, err);
        CK(hipGetLastError());
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        int e = 0;
        CK(hipMemcpy(&e, err, 4, hipMemcpyDeviceToHost));
        if (rep == 1) std::printf("kind=%d grid=%d: %.3f us per barrier%s\n", kind, grid, ms * 1000.f / nbar, e ? "  (TIMEOUT)" : "");
      }
    }
  return 0;
}
