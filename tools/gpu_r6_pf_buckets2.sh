#!/bin/bash
# round 6: bucketed prefill graphs at one stage, re-measured with the bucket graphs captured in an
# unmeasured serving warm-up (the first try paid every capture inside a 7 s run); engine tests first
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
S=gpurun_out/r6_pf_buckets2_tests.log; : > $S
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_engine_gpu.py tests/test_kernels_gpu.py -k "engine or graph or prefill or merged or bucket" >> $S 2>&1 || { tail -40 $S; exit 1; }
tail -1 $S
L=gpurun_out/r6_pf_buckets2.log; : > $L
run() {
  local lab=$1; shift
  echo "== $lab" >> $L
  env "$@" timeout -k 10 400 python -u tools/serve_load.py --requests 4096 --warm-requests 2048 $ARGS > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep "^{" gpurun_out/_r.out >> $L
}
for m in gpt2-xl llama-3-8b gpt2; do
  ARGS="--model $m" run "$m buckets=1" LSD_PF_BUCKETS=1
  ARGS="--model $m" run "$m buckets=0" LSD_PF_BUCKETS=0
done
ARGS="--model gpt2-xl" run "gpt2-xl buckets=1 (2)" LSD_PF_BUCKETS=1
ARGS="--model gpt2-xl" run "gpt2-xl buckets=0 (2)" LSD_PF_BUCKETS=0
grep -o '^== .*\|"tok_s": [0-9.]*\|"per_token_ms_p50": [0-9.]*\|"ttft_ms_p50": [0-9.]*\|"ttft_ms_p90": [0-9.]*' $L | paste -sd' ' | sed 's/ == /\n== /g'
