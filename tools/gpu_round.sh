#!/bin/bash
# Round-end rehearsal: GPU tests, smoke(), default bench (each step time-limited, stop on first failure)
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/bench.log
exit $rc
