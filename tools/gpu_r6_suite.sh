#!/bin/bash
# round 6: the whole GPU suite (no -x: every failure listed) and smoke()
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6_pytest_gpu_full.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/r6_pytest_gpu_full.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_smoke.log 2>&1 || exit $?
exit $rc
