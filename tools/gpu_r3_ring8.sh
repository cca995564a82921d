#!/bin/bash
# A/B: 128x64 decode ring on 4 waves vs 8 waves (loader waves / all compute)
# and ring depth, solo per-call times at 256 rows, then the headline bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
D256_M=256 D256_SHAPES=${SHAPES:-xl_qkv,xl_fc,xl_proj,xl_proj2} D256_VARIANTS=${VARIANTS:-r8:2:3,r8:2:4,r8:2:5} \
  timeout -k 10 300 python tools/bench_d256.py > gpurun_out/r3_ring8_ab.log 2>&1 || exit $?
for s in ${BSLOTS:-3 4 5}; do
  echo "== LSD_RING8=2 slots $s" >> gpurun_out/r3_ring8_bench.log
  LSD_RING8=2 LSD_RING8_SLOTS=$s timeout -k 10 300 python bench.py --steps 3 --warmup 1 >> gpurun_out/r3_ring8_bench.log 2>&1 || exit $?
done
