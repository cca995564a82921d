#!/bin/bash
# A/B of the 8-wave ring's K-start rotation (flag 1) and nt weight staging
# (flag 2): solo per-call times at 256 rows, then the headline bench.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
D256_M=256 D256_BASE_R8=2 D256_SHAPES=xl_qkv,xl_fc,xl_proj,xl_proj2,l8_o D256_VARIANTS=r8:2:1,r8:2:2,r8:2:3 \
  timeout -k 10 300 python tools/bench_d256.py > gpurun_out/r3_ring8_flags_ab.log 2>&1 || exit $?
for f in 0 1 2 3; do
  echo "== LSD_RING8_FLAGS=$f" >> gpurun_out/r3_ring8_flags_bench.log
  LSD_RING8_FLAGS=$f timeout -k 10 300 python bench.py --steps 3 --warmup 1 >> gpurun_out/r3_ring8_flags_bench.log 2>&1 || exit $?
done
