#!/bin/bash
# GPU tests + microbench + flagship bench (each step time-limited; stop on crash codes)
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest ${TEST_ARGS:-tests -m gpu} -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "$MB_ARGS" ]; then
  timeout -k 10 600 python tools/microbench.py ${MB_ARGS} > gpurun_out/micro.log 2>&1
  rc=$?; echo "rc=$rc" >> gpurun_out/micro.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/bench.log
exit $rc
