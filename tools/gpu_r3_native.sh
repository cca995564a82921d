#!/bin/bash
# Native stage executor tests + host-issue probe + packed-operand A/B + bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -m gpu -v -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_native_tests.log 2>&1 || exit $?
timeout -k 10 300 python tools/probe_host_issue.py gpt2 1024 4 > gpurun_out/r3_probe_host_gpt2_native.log 2>&1 || exit $?
LSD_NATIVE_EXEC=0 timeout -k 10 300 python tools/probe_host_issue.py gpt2 1024 4 > gpurun_out/r3_probe_host_gpt2_py.log 2>&1 || exit $?
timeout -k 10 300 python tools/bench_ring8_pack.py > gpurun_out/r3_ring8_pack_ab.log 2>&1 || exit $?
for v in 1 0; do
  echo "== LSD_NATIVE_EXEC=$v" >> gpurun_out/r3_native_bench.log
  LSD_NATIVE_EXEC=$v timeout -k 10 300 python bench.py --steps 3 --warmup 1 >> gpurun_out/r3_native_bench.log 2>&1 || exit $?
  LSD_NATIVE_EXEC=$v LSD_HOST_PROFILE=1 timeout -k 10 300 python bench.py --model gpt2 --batch 1024 --microbatches 4 --prompt 64 --gen 64 --steps 2 --warmup 1 >> gpurun_out/r3_native_bench.log 2>&1 || exit $?
done
