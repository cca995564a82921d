#!/bin/bash
# round 6: mixed decode + prefill steps (one forward per group and step) -- engine GPU tests, then the
# closed-loop serving load with LSD_MIXED_STEPS=1 / 0 interleaved, then the headline bench (unaffected)
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r6_mixed.log; : > $L
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_engine_gpu.py tests/test_numerics_gpu.py >> $L 2>&1 || { tail -30 $L; exit 1; }
for m in gpt2-xl gpt2 llama-3-8b; do
  for rep in 1 2; do
    for mx in 1 0; do
      echo "== $m LSD_MIXED_STEPS=$mx (round $rep)" >> $L
      LSD_MIXED_STEPS=$mx LSD_HOST_PROFILE=1 timeout -k 10 300 python -u tools/serve_load.py --model $m --concurrency 512 --requests 4096 >> $L 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
    done
  done
done
echo "== headline" >> $L
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 2>/dev/null | grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*' | tr '\n' ' ' >> $L
