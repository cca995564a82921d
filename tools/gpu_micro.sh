#!/bin/bash
# GPU tests (kernel numerics) then microbenchmarks; args via MB_ARGS / TEST_ARGS.
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest ${TEST_ARGS:-tests -m gpu} -q -p no:cacheprovider -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python tools/microbench.py ${MB_ARGS} > gpurun_out/micro.log 2>&1
echo "rc=$?" >> gpurun_out/micro.log
