#!/bin/bash
# Round 3: numerics of the 256-row decode GEMM + A/B against the ring kernel.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py \
  -k "d256 or qkv_kv_append or sampler_small or ring_gemm_epilogues or test_linear" > gpurun_out/r3_t1.log 2>&1 || { tail -30 gpurun_out/r3_t1.log; exit 1; }
tail -3 gpurun_out/r3_t1.log
timeout -k 10 600 python -u tools/bench_d256.py > gpurun_out/r3_d256.log 2>&1 || { tail -30 gpurun_out/r3_d256.log; exit 1; }
tail -5 gpurun_out/r3_d256.log
