#!/bin/bash
# Epilogue store passes with all global reads hoisted before the stores: kernel numerics,
# prefill GEMM timing (kind 4 / 1 vs hipBLASLt), decode ring solo times, bench.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py tests/test_gemv_gpu.py tests/test_numerics_gpu.py tests/test_engine_gpu.py > gpurun_out/t_epi.log 2>&1
rc=$?; tail -3 gpurun_out/t_epi.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_p8.py 4 1 > gpurun_out/bench_epi.log 2>&1 || exit $?  # kind 6 (persistent) was removed
grep -v amdgpu.ids gpurun_out/bench_epi.log
D256_M=256 D256_BASE_R8=2 D256_SHAPES=xl_qkv,xl_fc,xl_proj,xl_proj2,l8_qkv,l8_gu D256_VARIANTS=r8:2:0 \
  timeout -k 10 300 python tools/bench_d256.py > gpurun_out/r3_epi_ring.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r3_epi_ring.log
BENCH_ARGS="--steps 3 --warmup 1" VARIANTS="default;default" bash tools/gpu_ab_env.sh || exit $?
grep -h "^==\|tokens/s" gpurun_out/ab_env.log | sed 's/"config".*//' | cut -c1-250
grep -o '"p50_token_latency_ms": [0-9.]*, "prefill_ms": [0-9.]*' gpurun_out/ab_env.log
