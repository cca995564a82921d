#!/bin/bash
# Kernel GPU tests (TESTS, default the kernel file), then bench configs (SWEEP, ';'-separated env sets).
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest ${TESTS:-tests/test_kernels_gpu.py} -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_k.log 2>&1 || exit $?
: > gpurun_out/sweep.log
IFS=';' read -ra CFGS <<< "$SWEEP"
for c in "${CFGS[@]}"; do
  echo "== $c" >> gpurun_out/sweep.log
  env $c timeout -k 10 300 python bench.py --steps 2 --warmup 1 $BENCH_EXTRA >> gpurun_out/sweep.log 2>&1 || exit $?
done
