#!/bin/bash
# round 5: slab-folding decode norms on the wave-per-row kernel (LSD_NORM_WAVE_SLAB_MIN): tests, then bench
# A/B on GPT-2 XL (headline, 2 x 256 rows) and GPT-2 small (512), interleaved
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r5_normwave_slab.log; : > $L
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "norm" -q --timeout 120 --timeout-method thread -p no:cacheprovider >> $L 2>&1 || exit 1
for r in 1 2; do
  for m in 64 0; do
    for model in gpt2-xl gpt2; do
      echo "== $model LSD_NORM_WAVE_SLAB_MIN=$m (round $r)" >> $L
      LSD_NORM_WAVE_SLAB_MIN=$m timeout -k 10 300 python -u bench.py --model $model --steps 3 --warmup 1 > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
      grep "^{" gpurun_out/_r.out | cut -c1-200 >> $L
      grep -o '"p50_token_latency_ms": [0-9.]*' gpurun_out/_r.out >> $L
    done
  done
done
