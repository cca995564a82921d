#!/bin/bash
# bench.py across the README / BASELINE.md configurations (1 MI355X).
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/configs.log; : > $L
run() {
  echo "== $*" >> $L
  timeout -k 10 400 python bench.py "$@" >> $L 2>&1 || { echo "rc=$?" >> $L; exit 1; }
}
run --steps 3 --warmup 1
run --steps 2 --warmup 1 --greedy
run --steps 2 --warmup 1 --batch 256
run --steps 2 --warmup 1 --batch 384
run --steps 2 --warmup 1 --batch 1024
run --batch 1 --microbatches 1 --steps 2 --warmup 1
run --model gpt2 --steps 3 --warmup 1
run --model gpt2 --batch 1 --microbatches 1 --steps 2 --warmup 1
run --model llama-3-8b --batch 256 --steps 2 --warmup 1
run --model llama-3-8b --batch 128 --steps 2 --warmup 1
run --model llama-3-8b --batch 1 --microbatches 1 --steps 2 --warmup 1
