#!/bin/bash
# round 6: joiners' prefill on a side stream at one stage (pipeline.py _prefill_side): engine tests,
# then the closed-loop serving load (512 in flight, warmed) with LSD_PF_SIDE=1 vs 0, interleaved
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
S=gpurun_out/r6_pf_side_tests.log; : > $S
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_engine_gpu.py tests/test_devloop_gpu.py >> $S 2>&1 || { tail -40 $S; exit 1; }
tail -1 $S
L=gpurun_out/r6_pf_side.log; : > $L
run() {
  local lab=$1; shift
  echo "== $lab" >> $L
  env "$@" timeout -k 10 400 python -u tools/serve_load.py --requests 4096 --warm-requests 1024 $ARGS > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep "^{" gpurun_out/_r.out >> $L
}
for r in 1 2; do
  for m in gpt2-xl llama-3-8b gpt2; do
    ARGS="--model $m" run "$m side=1" LSD_PF_SIDE=1
    ARGS="--model $m" run "$m side=0" LSD_PF_SIDE=0
  done
done
grep -o '^== .*\|"tok_s": [0-9.]*\|"per_token_ms_p50": [0-9.]*\|"ttft_ms_p50": [0-9.]*\|"ttft_ms_p90": [0-9.]*' $L | paste -sd' ' | sed 's/ == /\n== /g'
