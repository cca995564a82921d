#!/bin/bash
# round 6: bench.py across the README / BASELINE.md configurations on one MI355X, then the GPT-2
# small 8-stage one-GPU rehearsal (16 x 256, 64 + 64 tokens, merged prefill off on both sides)
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r6_results_bench_configs.log; : > $L
run() {
  echo "== $*" >> $L
  timeout -k 10 400 python -u bench.py "$@" > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep "^{" gpurun_out/_r.out >> $L
}
run --steps 3 --warmup 1
run --steps 2 --warmup 1 --greedy
run --steps 2 --warmup 1 --batch 256
run --steps 2 --warmup 1 --batch 384
run --steps 2 --warmup 1 --batch 1024
run --batch 1 --microbatches 1 --steps 2 --warmup 1
run --model gpt2 --steps 3 --warmup 1
run --model gpt2 --batch 1 --microbatches 1 --steps 2 --warmup 1
run --model llama-3-8b --steps 2 --warmup 1
run --model llama-3-8b --batch 256 --steps 2 --warmup 1
run --model llama-3-8b --batch 128 --steps 2 --warmup 1
run --model llama-3-8b --batch 1 --microbatches 1 --steps 2 --warmup 1
run --steps 3 --warmup 1
L2=gpurun_out/r6_rehearsal_small_p8.log; : > $L2
reh() {
  local lab=$1; shift
  echo "== $lab" >> $L2
  LSD_MERGE_PREFILL=0 timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 "$@" > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L2; exit 1; }
  grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*\|"prefill_ms": [0-9.]*\|"stage_busy": \[[^]]*\]' gpurun_out/_r.out | tr '\n' ' ' >> $L2; echo >> $L2
}
C="--model gpt2 --batch 4096 --microbatches 16 --prompt 64 --gen 64"
for r in 1 2; do
  reh "gpt2 P=1 16x256" $C
  reh "gpt2 P=8 16x256 devloop" $C --loopback-stages 8
done
