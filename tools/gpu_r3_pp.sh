#!/bin/bash
# Persistent prefill GEMM (kind 6): numerics tests first, then kind 4 vs 6 vs hipBLASLt timing.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "persistent or big_gemm" > gpurun_out/t_pp.log 2>&1
rc=$?; tail -3 gpurun_out/t_pp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_p8.py 4 6 > gpurun_out/bench_pp.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/bench_pp.log; exit $rc
