#!/bin/bash
# round 5: slab wave norms restricted to H <= 1024, default on from 256 rows: tests + GPT-2 small A/B
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r5_normwave_slab2.log; : > $L
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_numerics_gpu.py -k "norm or gpt2" -q --timeout 200 --timeout-method thread -p no:cacheprovider >> $L 2>&1 || exit 1
for r in 1 2; do
  for m in 256 0; do
    echo "== gpt2 LSD_NORM_WAVE_SLAB_MIN=$m (round $r)" >> $L
    LSD_NORM_WAVE_SLAB_MIN=$m timeout -k 10 300 python -u bench.py --model gpt2 --steps 3 --warmup 1 > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
    grep "^{" gpurun_out/_r.out | cut -c1-200 >> $L
    grep -o '"p50_token_latency_ms": [0-9.]*' gpurun_out/_r.out >> $L
  done
done
