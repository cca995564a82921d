#!/bin/bash
# round 5 (late): the whole GPU suite again with this round's additions, smoke(), the default bench x2
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r5_pytest_gpu_full.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/r5_pytest_gpu_full.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_smoke.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > gpurun_out/r5_bench_default.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py >> gpurun_out/r5_bench_default.log 2>&1
