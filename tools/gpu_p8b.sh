#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/p8b.log; : > $L
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py tests/test_gemv_gpu.py >> $L 2>&1 || exit 1
timeout -k 10 300 python tools/microbench.py p8stamps >> $L 2>&1 || exit 1
timeout -k 10 400 python tools/microbench.py p8 >> $L 2>&1
