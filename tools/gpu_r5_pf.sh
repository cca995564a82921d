#!/bin/bash
# round 5: 8-wave ring weight-line prefetch -- kernel tests, per-shape A/B
# (cold weights), then the headline bench with and without it, interleaved
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r5_ring8_prefetch.log
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "ring8 or linear_residual or RING8" > gpurun_out/r5_pf_tests.log 2>&1 || exit $?
echo "== per-shape A/B (cold weights, 256 rows)" > $L
D256_BASE_R8=2 D256_SHAPES=xl_qkv,xl_fc,xl_proj,xl_proj2,l8_qkv D256_VARIANTS=pf:2,pf:4,pf:6 \
  timeout -k 10 300 python -u tools/bench_d256.py >> $L 2>&1 || exit $?
for i in 1 2; do
  for pf in 0 4 2; do
    echo "== bench LSD_RING8_PF=$pf (round $i)" >> $L
    LSD_RING8_PF=$pf timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 >> $L 2>&1 || exit $?
  done
done
