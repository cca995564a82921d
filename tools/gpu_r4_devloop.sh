#!/bin/bash
# Round 4: device loopback channels (graph-captured transfers + native executor
# at P > 1 on one GPU): unit + engine + stall tests, the race checker over the
# devloop engine, then the headline bench once.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_devloop_gpu.py tests/test_racecheck.py tests/test_multigpu.py -m gpu -v -x --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_devloop_tests.log 2>&1
rc=$?; tail -30 gpurun_out/r4_devloop_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/r4_bench1.log 2>&1
rc=$?; tail -3 gpurun_out/r4_bench1.log; exit $rc
