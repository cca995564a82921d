#!/bin/bash
# round 6: join policy re-checked on top of the decode-first order and partial native issue (warmed)
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r6_join_sweep2.log; : > $L
run() {
  echo "== $*" >> $L
  timeout -k 10 400 python -u tools/serve_load.py --requests 4096 --warm-requests 1024 "$@" > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep "^{" gpurun_out/_r.out >> $L
}
for m in gpt2-xl llama-3-8b; do
  run --model $m --join-min 32 --join-wait 4
  run --model $m --join-min 1
  run --model $m --join-min 128 --join-wait 8
  run --model $m --join-min 32 --join-wait 4
done
grep -o '^== .*\|"tok_s": [0-9.]*\|"per_token_ms_p50": [0-9.]*\|"ttft_ms_p50": [0-9.]*\|"ttft_ms_p90": [0-9.]*' $L | paste -sd' ' | sed 's/ == /\n== /g'
