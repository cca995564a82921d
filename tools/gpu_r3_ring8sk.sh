#!/bin/bash
# 8-wave ring with K splits + in-kernel combine (QKV / MLP-up at 256 rows):
# numerics tests, solo per-call A/B, then the headline bench by workgroup target.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -q -x -k "ring8" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_ring8sk_tests.log 2>&1 || exit $?
D256_M=256 D256_BASE_R8=2 D256_SHAPES=xl_qkv,xl_fc,s_qkv,s_fc,l8_qkv D256_VARIANTS=r8s:2,r8s:3,r8s:4 \
  timeout -k 10 300 python tools/bench_d256.py > gpurun_out/r3_ring8sk_ab.log 2>&1 || exit $?
for t in 0 300 450; do
  echo "== LSD_RING8_SK_TARGET=$t" >> gpurun_out/r3_ring8sk_bench.log
  LSD_RING8_SK_TARGET=$t timeout -k 10 300 python bench.py --steps 3 --warmup 1 >> gpurun_out/r3_ring8sk_bench.log 2>&1 || exit $?
done
