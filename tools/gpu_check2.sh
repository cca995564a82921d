#!/bin/bash
# all GPU kernel/engine tests, single-stream profile, headline bench + profile
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests -m gpu > gpurun_out/pytest_all.log 2>&1 || { echo "pytest rc=$?" >> gpurun_out/pytest_all.log; exit 1; }
bash tools/gpu_prof_ss.sh || exit 1
BENCH_ARGS="--steps 3 --warmup 1" bash tools/gpu_prof.sh
