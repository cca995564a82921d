#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/llama_cfg.log; : > $L
for a in "--batch 256" "--batch 128" "--batch 512" "--batch 1 --microbatches 1"; do
  echo "== $a" >> $L
  timeout -k 10 400 python bench.py --model llama-3-8b --steps 2 --warmup 1 $a >> $L 2>&1 || exit 1
done
