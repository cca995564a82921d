#!/bin/bash
# Round 4 A/B: full-batch decode attention blocks of 4 waves (default) vs 8 waves (which also request V
# with K; LSD_ATTN_LARGE_WAVES), headline config, one box, interleaved.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gpurun_out/r4_attn_waves.log; : > $L
for v in 4 8 4 8; do
  echo "== LSD_ATTN_LARGE_WAVES=$v" >> $L
  LSD_ATTN_LARGE_WAVES=$v timeout -k 10 300 python bench.py --steps 3 --warmup 1 2>/dev/null | grep "^{" >> $L || exit 1
done
python3 - <<'PY'
import json
lab=None
for l in open("gpurun_out/r4_attn_waves.log"):
    if l.startswith("=="): lab=l[3:].strip(); continue
    if l.startswith("{"):
        d=json.loads(l); print(f"{lab:26s} {d['value']:10.0f} tok/s p50 {d['p50_token_latency_ms']:.3f} ms prefill {d['prefill_ms']}")
PY
