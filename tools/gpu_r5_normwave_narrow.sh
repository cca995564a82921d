#!/bin/bash
# round 5: wave-per-row norms for H <= 1024 from 256 rows, slab folds included (LSD_NORM_WAVE_NARROW_MIN):
# norm tests, the pipeline-vs-1-GPU bench checks, then GPT-2 small bench A/B interleaved
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r5_normwave_narrow.log; : > $L
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_bench_check.py -k "norm or token_check" -q --timeout 200 --timeout-method thread -p no:cacheprovider >> $L 2>&1 || exit 1
for r in 1 2; do
  for m in 256 0; do
    echo "== gpt2 LSD_NORM_WAVE_NARROW_MIN=$m (round $r)" >> $L
    LSD_NORM_WAVE_NARROW_MIN=$m timeout -k 10 300 python -u bench.py --model gpt2 --steps 3 --warmup 1 > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
    grep "^{" gpurun_out/_r.out | cut -c1-200 >> $L
    grep -o '"p50_token_latency_ms": [0-9.]*' gpurun_out/_r.out >> $L
  done
done
