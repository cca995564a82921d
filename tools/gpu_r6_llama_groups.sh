#!/bin/bash
# round 6: Llama-3 8B 512 sequences: 1 x 512 (auto) vs 2 x 256 on two lanes
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r6_llama_groups.log; : > $L
for rep in 1 2; do
  for mb in 1 2; do
    echo "== llama-3-8b microbatches=$mb (round $rep)" >> $L
    timeout -k 10 300 python -u bench.py --model llama-3-8b --microbatches $mb --steps 2 --warmup 1 > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
    grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*\|"prefill_ms": [0-9.]*' gpurun_out/_r.out | tr '\n' ' ' >> $L; echo >> $L
  done
done
