#!/bin/bash
# round 6: join policy sweep (join_min / join_max_wait) under the closed-loop serving load
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r6_join_sweep.log; : > $L
run() {
  echo "== $*" >> $L
  timeout -k 10 300 python -u tools/serve_load.py --requests 4096 "$@" > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep "^{" gpurun_out/_r.out >> $L
}
for m in gpt2-xl llama-3-8b; do
  run --model $m --join-min 32 --join-wait 4
  run --model $m --join-min 32 --join-wait 8
  run --model $m --join-min 64 --join-wait 4
  run --model $m --join-min 128 --join-wait 8
  run --model $m --join-min 32 --join-wait 2
done
grep -o '^== .*\|"tok_s": [0-9.]*\|"ttft_ms_p50": [0-9.]*\|"ttft_ms_p90": [0-9.]*' $L | paste -sd' ' | sed 's/ == /\n== /g'
