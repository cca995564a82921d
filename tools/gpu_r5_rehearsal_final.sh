#!/bin/bash
# round 5, final build: one-GPU 8-stage rehearsal (device loopback, threads) of GPT-2 small vs one stage, interleaved
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r5_rehearsal_final.log; : > $L
run() {
  local lab=$1; shift
  echo "== $lab" >> $L
  timeout -k 10 400 python bench.py --steps 2 --warmup 1 "$@" > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -30 gpurun_out/_r.err >> $L; return 1; }
  grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*\|"prefill_ms": [0-9.]*\|"stage_busy": \[[^]]*\]' gpurun_out/_r.out | tr '\n' ' ' >> $L; echo >> $L
}
C="--prompt 64 --gen 64"
run "gpt2 P=1 M=16x256" --model gpt2 --batch 4096 --microbatches 16 $C && \
run "gpt2 P=8 M=16x256 devloop" --model gpt2 --batch 4096 --microbatches 16 --loopback-stages 8 $C && \
run "gpt2 P=1 M=16x256 (2)" --model gpt2 --batch 4096 --microbatches 16 $C && \
run "gpt2 P=8 M=16x256 devloop (2)" --model gpt2 --batch 4096 --microbatches 16 --loopback-stages 8 $C && \
run "gpt2-xl P=1 M=16x256" --batch 4096 --microbatches 16 $C && \
run "gpt2-xl P=8 M=16x256 devloop" --batch 4096 --microbatches 16 --loopback-stages 8 $C
