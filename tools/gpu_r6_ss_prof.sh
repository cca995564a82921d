#!/bin/bash
# round 6: single-stream kernel statistics after the GEMV segment maxima and the one-round 128-dim attention
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in llama-3-8b gpt2-xl; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ssprof_$m -o run -- python3 -u bench.py --model $m --batch 1 --microbatches 1 --steps 2 --warmup 1 > gpurun_out/_p_$m.out 2> gpurun_out/_p_$m.err || { tail -20 gpurun_out/_p_$m.err; exit 1; }
  find gpurun_out/ssprof_$m -name "*kernel_stats.csv" -exec cp {} gpurun_out/r6_${m}_b1_kernel_stats_v2.csv \;
  rm -rf gpurun_out/ssprof_$m
  grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*' gpurun_out/_p_$m.out | tr '\n' ' '; echo
done
ls gpurun_out/*_v2.csv
