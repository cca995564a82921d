#!/bin/bash
# round 6: GPT-2 small 512-sequence session host phases (LSD_HOST_PROFILE=1), 4 runs: where the
# 4-12 ms spread of session_other_ms comes from
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r6_small_session.log; : > $L
for i in 1 2 3 4; do
  LSD_HOST_PROFILE=1 timeout -k 10 300 python -u bench.py --model gpt2 --steps 5 --warmup 2 > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*\|"prefill_ms": [0-9.]*\|"session_other_ms": [0-9.]*' gpurun_out/_r.out | tr '\n' ' ' >> $L; echo >> $L
  grep "^host per" gpurun_out/_r.err >> $L
done
cat $L
