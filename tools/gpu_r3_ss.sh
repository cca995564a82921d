#!/bin/bash
# Round 3: GPU tests of the new kernels, then A/Bs: Llama-3 8B 256 sequences
# (auto 256-row kernel vs ring) and single stream (fused attention + out-proj
# vs separate launches) for GPT-2 XL / small / Llama-3 8B.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "oproj or d256 or qkv_kv_append or sampler" > gpurun_out/r3_t4.log 2>&1 || { tail -40 gpurun_out/r3_t4.log; exit 1; }
tail -2 gpurun_out/r3_t4.log
summ() { grep -h "^==\|tokens/s" gpurun_out/ab_env.log | python3 -c "
import sys,json
for l in sys.stdin:
    if l.startswith('=='): print(l.strip()); continue
    d=json.loads(l); print(d['value'], d['p50_token_latency_ms'], d['prefill_ms'])"; }
BENCH_ARGS="--model gpt2-xl --batch 1 --steps 3 --warmup 1" VARIANTS="default;LSD_ATTN_OPROJ_MAX_M=0;default" bash tools/gpu_ab_env.sh || exit 1
echo "## xl single stream"; summ
BENCH_ARGS="--model gpt2 --batch 1 --steps 3 --warmup 1" VARIANTS="default;LSD_ATTN_OPROJ_MAX_M=0;default" bash tools/gpu_ab_env.sh || exit 1
echo "## small single stream"; summ
BENCH_ARGS="--model llama-3-8b --batch 1 --steps 3 --warmup 1" VARIANTS="default;LSD_ATTN_OPROJ_MAX_M=0" bash tools/gpu_ab_env.sh || exit 1
echo "## llama single stream"; summ
BENCH_ARGS="--model llama-3-8b --batch 256 --steps 3 --warmup 1" VARIANTS="default;LSD_D256=0;default;LSD_D256=0" bash tools/gpu_ab_env.sh || exit 1
echo "## llama 256"; summ
