#!/bin/bash
# round 5: Llama-3 8B decode gate_up on hipBLASLt + SiLU*up at 128 / 256 rows -- bench A/B (interleaved)
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r5_llama_small.log; : > $L
for i in 1 2; do
  for m in 64 0; do
    for b in 128 256; do
      echo "== llama-3-8b --batch $b LSD_BLASLT_SILU_MIN_M=$m MAX=256 (round $i)" >> $L
      LSD_BLASLT_SILU_MIN_M=$m LSD_BLASLT_SILU_MAX_M=256 timeout -k 10 400 python -u bench.py --model llama-3-8b --batch $b --steps 2 --warmup 1 >> $L 2>&1 || exit $?
    done
  done
done
