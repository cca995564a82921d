#!/bin/bash
# round 6: one-stage item order under the serving load: items without prefill chunks issued first
# plus, inside an item, the decode replay before the prefill (LSD_DECODE_FIRST=2) vs 1; engine tests first; warmed serve_load, interleaved
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
S=gpurun_out/r6_decode_first2_tests.log; : > $S
LSD_DECODE_FIRST=2 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_engine_gpu.py >> $S 2>&1 || { tail -40 $S; exit 1; }
tail -1 $S
L=gpurun_out/r6_decode_first2.log; : > $L
run() {
  local lab=$1; shift
  echo "== $lab" >> $L
  env "$@" timeout -k 10 400 python -u tools/serve_load.py --requests 4096 --warm-requests 1024 $ARGS > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep "^{" gpurun_out/_r.out >> $L
}
for r in 1 2; do
  for m in gpt2-xl llama-3-8b gpt2; do
    ARGS="--model $m" run "$m decode_first=2" LSD_DECODE_FIRST=2
    ARGS="--model $m" run "$m decode_first=1" LSD_DECODE_FIRST=1
  done
done
grep -o '^== .*\|"tok_s": [0-9.]*\|"per_token_ms_p50": [0-9.]*\|"ttft_ms_p50": [0-9.]*\|"ttft_ms_p90": [0-9.]*' $L | paste -sd' ' | sed 's/ == /\n== /g'
