#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
BENCH_ARGS="--steps 4 --warmup 2" VARIANTS="default;LSD_LANE_CU_MASK=split;LSD_LANE_CU_MASK=interleave;LSD_LANE_CU_MASK=interleave LSD_D256=64 LSD_D256_TARGET=1;LSD_LANE_CU_MASK=split LSD_D256=64 LSD_D256_TARGET=1;default" bash tools/gpu_ab_env.sh || exit 1
grep -h "^==\|tokens/s" gpurun_out/ab_env.log | python3 -c "
import sys,json
for l in sys.stdin:
    if l.startswith('=='): print(l.strip()); continue
    d=json.loads(l); print(d['value'], d['p50_token_latency_ms'], d['prefill_ms'])"
