#!/bin/bash
# Control-plane cost at P = 8 (CPU, gloo, 8 ranks): binary plan records vs the
# pickled StepPlan (LSD_PLAN_WIRE=pickle), 16 microbatch groups.  Prints stage
# 0's host time per decode step: plan (build + send) and the send part alone,
# with the bytes rank 0 posts per step.
set -o pipefail
cd "$(dirname "$0")/.."
for wire in pickle binary; do
  echo "== LSD_PLAN_WIRE=$wire"
  LSD_PLAN_WIRE=$wire LSD_HOST_PROFILE=1 OMP_NUM_THREADS=1 timeout 600 python -m torch.distributed.run \
    --nnodes=1 --nproc-per-node=8 --master-addr=127.0.0.1 --master-port=$((29500 + RANDOM % 1000)) \
    bench.py --gpus 8 --device cpu --transport gloo --model gpt2-test --batch 32 --microbatches 16 \
    --prompt 16 --gen 48 --steps 2 --warmup 1 2>&1 | grep -E "^\{|host per" | \
    python -c "import sys,json
for l in sys.stdin:
    if l.startswith('{'): d=json.loads(l); print('  tok/s', d['value'], 'p50', d['p50_token_latency_ms'], 'ms')
    else: print('  ', l.strip())"
done
