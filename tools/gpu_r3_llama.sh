#!/bin/bash
# Round 3: kernel + numerics tests, then Llama-3 8B (256 sequences) with the
# auto 256-row kernel routing vs the ring everywhere.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_kernels_gpu.py tests/test_numerics_gpu.py \
  > gpurun_out/r3_t3.log 2>&1 || { tail -30 gpurun_out/r3_t3.log; exit 1; }
tail -2 gpurun_out/r3_t3.log
grep -h "llama-3-8b\|gpt2" gpurun_out/r3_t3.log | head -5
BENCH_ARGS="--model llama-3-8b --batch 256 --steps 3 --warmup 1" VARIANTS="default;LSD_D256=0;default;LSD_D256=0" bash tools/gpu_ab_env.sh || exit 1
grep -h "^==\|tokens/s" gpurun_out/ab_env.log | python3 -c "
import sys,json
for l in sys.stdin:
    if l.startswith('=='): print(l.strip()); continue
    d=json.loads(l); print(d['value'], d['p50_token_latency_ms'], d['prefill_ms'])"
