#!/bin/bash
# Every GPU test (no -x: all failures listed), then smoke() and the default bench.
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/pytest_gpu.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc2=$?; echo "rc=$rc2" >> gpurun_out/smoke.log
[ $rc2 -eq 0 ] || exit $rc2
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1
rc3=$?; echo "rc=$rc3" >> gpurun_out/bench.log
exit $((rc + rc3))
