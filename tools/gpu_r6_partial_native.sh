#!/bin/bash
# round 6: one stage, steady decode items of a step with joining groups on the native executor one by one
# (LSD_PARTIAL_NATIVE=1) vs all items through the Python loop; engine tests first; warmed serve_load
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
S=gpurun_out/r6_partial_native_tests.log; : > $S
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_engine_gpu.py tests/test_devloop_gpu.py >> $S 2>&1 || { tail -40 $S; exit 1; }
tail -1 $S
L=gpurun_out/r6_partial_native.log; : > $L
run() {
  local lab=$1; shift
  echo "== $lab" >> $L
  env "$@" timeout -k 10 400 python -u tools/serve_load.py --requests 4096 --warm-requests 1024 $ARGS > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep "^{" gpurun_out/_r.out >> $L
}
for r in 1 2; do
  for m in gpt2-xl llama-3-8b gpt2; do
    ARGS="--model $m" run "$m partial=1" LSD_PARTIAL_NATIVE=1
    ARGS="--model $m" run "$m partial=0" LSD_PARTIAL_NATIVE=0
  done
done
grep -o '^== .*\|"tok_s": [0-9.]*\|"per_token_ms_p50": [0-9.]*\|"ttft_ms_p50": [0-9.]*\|"native_steps": [0-9]*' $L | paste -sd' ' | sed 's/ == /\n== /g'
