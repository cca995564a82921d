#!/bin/bash
# round 6: single-stream decode attention block size (8 vs 16 waves per block)
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r6_small_waves.log; : > $L
for rep in 1 2; do
  for sw in 8 16; do
    for cfg in "--model gpt2-xl --batch 1 --microbatches 1" "--model llama-3-8b --batch 1 --microbatches 1"; do
      echo "== attn_small_waves=$sw $cfg (round $rep)" >> $L
      LSD_ROUTING=attn_small_waves=$sw timeout -k 10 300 python -u bench.py $cfg --steps 2 --warmup 1 > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
      grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*' gpurun_out/_r.out | tr '\n' ' ' >> $L; echo >> $L
    done
  done
done
