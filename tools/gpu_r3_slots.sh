#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -f gpurun_out/bench_d256.jsonl
for sl in 2 3 4; do
  D256_SLOTS=$sl D256_SHAPES=xl_qkv,xl_fc,l8_qkv,l8_gu D256_VARIANTS=64:1,64:2,64:3,128:1,128:2 \
    timeout -k 10 300 python -u tools/bench_d256.py > gpurun_out/r3_slots_$sl.log 2>&1 || { tail -20 gpurun_out/r3_slots_$sl.log; exit 1; }
done
for sl in 2 3 4; do echo "== slots $sl"; python3 -c "
import json,sys
for l in open('gpurun_out/r3_slots_$sl.log'):
    if not l.startswith('{'): continue
    r=json.loads(l); print(r['shape'], r['case'], r['us_med'])"; done
