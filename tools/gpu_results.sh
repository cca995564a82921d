#!/bin/bash
# Headline + other bench configurations for README / BASELINE.md (one JSON line each).
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
: > gpurun_out/results.log
run() {
  echo "== $*" >> gpurun_out/results.log
  timeout -k 10 300 python bench.py "$@" >> gpurun_out/results.log 2>&1 || { echo "rc=$?" >> gpurun_out/results.log; exit 1; }
}
run --steps 3 --warmup 1
run --greedy --steps 2 --warmup 1
run --batch 1024 --steps 2 --warmup 1
run --batch 384 --steps 3 --warmup 1
run --batch 256 --steps 3 --warmup 1
run --batch 1 --microbatches 1 --steps 2 --warmup 1
run --model gpt2 --steps 3 --warmup 1
run --model gpt2 --batch 1 --microbatches 1 --steps 2 --warmup 1
run --model llama-3-8b --batch 512 --steps 2 --warmup 1
run --model llama-3-8b --batch 256 --steps 2 --warmup 1
run --model llama-3-8b --batch 128 --steps 2 --warmup 1
run --model llama-3-8b --batch 1 --microbatches 1 --steps 2 --warmup 1
