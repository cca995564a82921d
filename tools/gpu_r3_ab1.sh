#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "d256 or qkv_kv_append" > gpurun_out/r3_t2.log 2>&1 || { tail -30 gpurun_out/r3_t2.log; exit 1; }
tail -2 gpurun_out/r3_t2.log
BENCH_ARGS="--steps 5 --warmup 2" VARIANTS="default;LSD_D256=64 LSD_D256_TARGET=1;LSD_D256=128 LSD_D256_TARGET=1;LSD_D256=64 LSD_D256_TARGET=150;default" bash tools/gpu_ab_env.sh || exit 1
grep -h "^==\|tokens/s" gpurun_out/ab_env.log | sed 's/"config".*//' | cut -c1-260
