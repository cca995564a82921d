#!/bin/bash
# One-wave-per-SIMD prefill GEMM (kind 7): numerics, then kind 4 vs 7 vs hipBLASLt.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "big_gemm" > gpurun_out/t_w4.log 2>&1
rc=$?; tail -3 gpurun_out/t_w4.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_p8.py 4 10 > gpurun_out/bench_w4.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/bench_w4.log; exit $rc
