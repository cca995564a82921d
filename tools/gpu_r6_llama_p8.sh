#!/bin/bash
# round 6: BASELINE config 5 rehearsal -- Llama-3 8B as an 8-stage pipeline on one MI355X (stage
# threads over device-loopback channels) vs one stage running the same 8 groups of 512 sequences
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r6_llama_p8.log; : > $L
C="--model llama-3-8b --batch 4096 --microbatches 8 --prompt 64 --gen 64"
for r in 1 2; do
  for a in "" "--loopback-stages 8"; do
    echo "== $C $a (round $r)" >> $L
    LSD_MERGE_PREFILL=0 timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 $C $a > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
    grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*\|"prefill_ms": [0-9.]*\|"stage_busy": \[[^]]*\]' gpurun_out/_r.out | tr '\n' ' ' >> $L; echo >> $L
  done
done
