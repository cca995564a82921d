// Memory-pattern probe: one-shot read of a weight-like matrix [N][K] bf16 by
// 4-wave workgroups, each wave issuing all its loads up front, then a wait.
// Patterns: 0 = fragment (16 rows x 64 B per instr), 1 = full line (8 rows x
// 128 B), 2 = contiguous (1 KiB per instr, row-major walk), 3 = fragment with
// 2 k-steps per lane (16 rows x 128 B over 2 instrs, lane-interleaved).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int PAT, int STEPS>
__global__ __launch_bounds__(256) void probe(const char* W, long ldw_bytes, int N, int K2, u32x4* sink, long long* st) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // each block: 64 rows (4 waves x 16 rows) x STEPS*64 B of K
  const int tiles_n = N / 64;
  const int tile = blockIdx.x % tiles_n, ksplit = blockIdx.x / tiles_n;
  const long kbyte0 = (long)ksplit * STEPS * 64;
  u32x4 acc = {0, 0, 0, 0};
  u32x4 v[STEPS];
  if (threadIdx.x == 0) st[blockIdx.x * 2] = __builtin_amdgcn_s_memrealtime();
  const int row0 = tile * 64 + w * 16;
#pragma unroll
  for (int j = 0; j < STEPS; ++j) {
    long off;
    if (PAT == 0) off = (long)(row0 + (lane & 15)) * ldw_bytes + kbyte0 + j * 64 + (lane >> 4) * 16;
    else if (PAT == 1) { int rr = (j & 1) * 8 + (lane >> 3); off = (long)(row0 + rr) * ldw_bytes + kbyte0 + (j >> 1) * 128 + (lane & 7) * 16; }
    else if (PAT == 2) { long lin = (long)j * 1024 + lane * 16; int rr = lin / (STEPS * 64); off = (long)(row0 + rr) * ldw_bytes + kbyte0 + lin % (STEPS * 64); }
    else { off = (long)(row0 + (lane & 15)) * ldw_bytes + kbyte0 + (j >> 1) * 128 + (j & 1) * 16 + (lane >> 4) * 32; }
    v[j] = *reinterpret_cast<const u32x4*>(W + off);
  }
#pragma unroll
  for (int j = 0; j < STEPS; ++j) acc ^= v[j];
  __syncthreads();
  if (threadIdx.x == 0) st[blockIdx.x * 2 + 1] = __builtin_amdgcn_s_memrealtime();
  if (acc[0] == 0x12345678u) sink[threadIdx.x] = acc;
}

int main() {
  const int N = 4800, K = 1600;  // XL QKV
  const long bytes = (long)N * K * 2;
  char* W; hipMalloc(&W, bytes);
  hipMemset(W, 1, bytes);
  char* flush; hipMalloc(&flush, 1L << 30);
  u32x4* sink; hipMalloc(&sink, 4096);
  long long* st; hipMalloc(&st, 1 << 20);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const char* names[] = {"fragment16x64", "fullline8x128", "contig1KB", "frag16x128pair"};
  for (int cold = 1; cold >= 0; --cold)
  for (int steps : {13, 26, 52}) {
    // steps*64 B of K per block: K*2 / (steps*64) splits
    const int splits = (K * 2) / (steps * 64);
    const int blocks = (N / 64) * splits;
    for (int pat = 0; pat < 4; ++pat) {
      float best = 1e9;
      for (int rep = 0; rep < 5; ++rep) {
        if (cold) hipMemsetAsync(flush, rep, 1L << 30, 0);
        hipEventRecord(a, 0);
#define L(P, S) hipLaunchKernelGGL((probe<P, S>), dim3(blocks), dim3(256), 0, 0, W, (long)K * 2, N, K * 2, sink, st)
#define LS(S) if (pat == 0) L(0, S); else if (pat == 1) L(1, S); else if (pat == 2) L(2, S); else L(3, S);
        if (steps == 13) { LS(13) } else if (steps == 26) { LS(26) } else { LS(52) }
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
      }
      printf("%s steps=%d blocks=%d %-16s %7.2f us  %5.2f TB/s\n", cold ? "cold" : "warm", steps, blocks,
             names[pat], best * 1e3, bytes / (best * 1e-3) / 1e12);
    }
  }
  return 0;
}
