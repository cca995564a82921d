#!/bin/bash
# round 6: lane stream priorities A/B on the headline and GPT-2 small (interleaved)
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r6_lane_priority.log; : > $L
for rep in 1 2; do
  for pr in "" "-1,0" "0,-1"; do
    for m in gpt2-xl gpt2; do
      echo "== $m LSD_LANE_PRIORITY=$pr (round $rep)" >> $L
      LSD_LANE_PRIORITY=$pr timeout -k 10 300 python -u bench.py --model $m --steps 3 --warmup 1 > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
      grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*\|"prefill_ms": [0-9.]*' gpurun_out/_r.out | tr '\n' ' ' >> $L; echo >> $L
    done
  done
done
