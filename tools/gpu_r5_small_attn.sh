#!/bin/bash
# round 5: GPT-2 small decode attention block shape (LSD_ATTN_LARGE_WAVES 8: V requested with K) A/B, interleaved
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r5_small_attn.log; : > $L
for r in 1 2; do
  for v in 8 4; do
    echo "== gpt2 LSD_ATTN_LARGE_WAVES=$v (round $r)" >> $L
    LSD_ATTN_LARGE_WAVES=$v timeout -k 10 300 python -u bench.py --model gpt2 --steps 3 --warmup 1 > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
    grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*' gpurun_out/_r.out | tr '\n' ' ' >> $L; echo >> $L
  done
done
