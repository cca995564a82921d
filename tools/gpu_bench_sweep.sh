#!/bin/bash
# Run the GPU test suite, then several bench configs (one JSON line each).
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
: > gpurun_out/sweep.log
IFS=';' read -ra CFGS <<< "$SWEEP"
for c in "${CFGS[@]}"; do
  echo "== $c" >> gpurun_out/sweep.log
  env $c timeout -k 10 300 python bench.py --steps 2 --warmup 1 $BENCH_EXTRA >> gpurun_out/sweep.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "rc=$rc" >> gpurun_out/sweep.log; exit $rc; fi
done
