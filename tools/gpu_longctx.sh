#!/bin/bash
# Long-context benches: Llama-3 8B 4K / 8K prompts, GPT-2 XL at its 1024 cap.
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/longctx.log; : > $L
for a in "--model llama-3-8b --prompt 4096 --gen 128 --batch 32" "--model llama-3-8b --prompt 8000 --gen 128 --batch 8" "--model gpt2-xl --prompt 896 --gen 128 --batch 64"; do
  echo "== $a" >> $L
  timeout -k 10 400 python bench.py --steps 1 --warmup 1 $a >> $L 2>&1 || exit 1
done
