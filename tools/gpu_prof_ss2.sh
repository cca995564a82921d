#!/bin/bash
# Single-stream kernel traces for GPT-2 XL, GPT-2 small, Llama-3 8B (rocprofv3 kernel trace + stats).
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for M in gpt2-xl gpt2 llama-3-8b; do
  timeout -k 10 300 python bench.py --model $M --batch 1 --microbatches 1 --steps 2 --warmup 1 > gpurun_out/ss_bench_$M.log 2>&1 || exit $?
  ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_ss_$M" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --model $M --batch 1 --microbatches 1 --steps 1 --warmup 1 --gen 32 > "$GRAFT_REPO_ROOT/gpurun_out/prof_ss_$M.log" 2>&1 ) || exit $?
done
