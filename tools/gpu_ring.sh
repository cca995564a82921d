#!/bin/bash
# Ring-GEMM check: numerics tests, microbench (dbuf / ring3 / ring4), bench A/B on slots
cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "ring or big_gemm or two_row or decode_gemm" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ring_test.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/microbench.py tiled3 > gpurun_out/ring_micro.log 2>&1 || exit $?
VARIANTS="${VARIANTS:-default;LSD_RING_SLOTS=4;default;LSD_RING_SLOTS=4}" BENCH_ARGS="${BENCH_ARGS:---steps 3 --warmup 1}" bash tools/gpu_ab_env.sh
