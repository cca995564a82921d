#!/bin/bash
# round 5: staged composition-change upload -- tests, issue profile, rehearsal, the default bench
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp LSD_HOST_PROFILE=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py tests/test_devloop_gpu.py tests/test_bench_check.py tests/test_numerics_gpu.py \
  -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_pfgraph3_tests.log 2>&1 || exit $?
PROFILE_STAGES=8 timeout -k 10 400 python -u tools/profile_issue.py > gpurun_out/r5_profile_issue_p8c.log 2>&1 || exit $?
L=gpurun_out/r5_pfgraph3_rehearsal.log; : > $L
run() {
  local lab=$1; shift
  echo "== $lab" >> $L
  timeout -k 10 400 python bench.py --steps 2 --warmup 1 "$@" > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -30 gpurun_out/_r.err >> $L; return 1; }
  grep "^{" gpurun_out/_r.out >> $L
  grep "host per" gpurun_out/_r.err >> $L
}
C="--prompt 64 --gen 64"
run "gpt2 P=1 M=16x256" --model gpt2 --batch 4096 --microbatches 16 $C && \
run "gpt2 P=8 M=16x256 devloop" --model gpt2 --batch 4096 --microbatches 16 --loopback-stages 8 $C && \
run "gpt2 P=1 M=16x256 (2)" --model gpt2 --batch 4096 --microbatches 16 $C && \
run "gpt2 P=8 M=16x256 devloop (2)" --model gpt2 --batch 4096 --microbatches 16 --loopback-stages 8 $C && \
run "xl default" && run "xl default (2)"
