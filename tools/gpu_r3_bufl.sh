#!/bin/bash
# A/B: LDS-DMA staging by buffer_load ... lds (32-bit lane offsets) vs global_load_lds in the
# 8-wave decode ring (LSD_RING8_FLAGS bit 2): solo per-call times at 256 rows, then the bench.
set -o pipefail
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
D256_M=${DM:-256} D256_BASE_R8=2 D256_SHAPES=${SHAPES:-xl_qkv,xl_fc,xl_proj,xl_proj2,l8_qkv,l8_o} D256_VARIANTS=r8:2:4 \
  timeout -k 10 300 python tools/bench_d256.py > gpurun_out/r3_bufl_ab.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r3_bufl_ab.log
BENCH_ARGS="--steps 3 --warmup 1" VARIANTS="default;LSD_RING8_FLAGS=4;default;LSD_RING8_FLAGS=4" bash tools/gpu_ab_env.sh || exit $?
grep -h "^==\|tokens/s" gpurun_out/ab_env.log | sed 's/"config".*//' | cut -c1-250
