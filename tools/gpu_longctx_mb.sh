#!/bin/bash
# Long-context Llama-3 8B: 1 vs 2 microbatch groups.
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/longctx_mb.log; : > $L
for a in "--prompt 4096 --gen 128 --batch 32" "--prompt 2048 --gen 128 --batch 64" "--prompt 1024 --gen 128 --batch 128"; do
  for mb in 1 2; do
    echo "== $a mb=$mb" >> $L
    timeout -k 10 300 python bench.py --model llama-3-8b --steps 1 --warmup 1 --microbatches $mb $a >> $L 2>&1 || exit 1
  done
done
