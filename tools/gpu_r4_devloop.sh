#!/bin/bash
# Round 4: device loopback channels (graph-captured transfers + native executor
# at P > 1 on one GPU): unit + engine tests, then the rehearsal of every
# BASELINE config (tools/rehearsal.sh devloop).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_devloop_gpu.py -m gpu -v -x --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_devloop_tests.log 2>&1
rc=$?; tail -25 gpurun_out/r4_devloop_tests.log; exit $rc
