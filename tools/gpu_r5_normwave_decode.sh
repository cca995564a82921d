#!/bin/bash
# round 5: wave-per-row norm for decode-sized no-slab norms (GPT-2 small ln_1 at 128-256 rows):
# LSD_NORM_WAVE_MIN=64 vs the default 4096 (block-per-row kernel below it), bench A/B interleaved
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r5_normwave_decode.log; : > $L
for r in 1 2; do
  for m in 64 4096; do
    for b in 512 256; do
      echo "== gpt2 --batch $b LSD_NORM_WAVE_MIN=$m (round $r)" >> $L
      LSD_NORM_WAVE_MIN=$m timeout -k 10 300 python -u bench.py --model gpt2 --batch $b --steps 3 --warmup 1 > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
      grep "^{" gpurun_out/_r.out | cut -c1-200 >> $L
      grep -o '"p50_token_latency_ms": [0-9.]*' gpurun_out/_r.out >> $L
    done
  done
done
