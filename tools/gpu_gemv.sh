#!/bin/bash
# GEMV numerics + engine GPU tests, then single-stream bench and kernel profile.
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gemv_gpu.py tests/test_engine_gpu.py > gpurun_out/pytest_gemv.log 2>&1 || { echo "pytest rc=$?" >> gpurun_out/pytest_gemv.log; exit 1; }
bash tools/gpu_prof_ss.sh
