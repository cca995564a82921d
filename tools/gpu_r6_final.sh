#!/bin/bash
# round 6 (final build): GPU suite + smoke, then the README / BASELINE bench configurations and the
# 8-stage rehearsals (merged prefill off on both sides of each rehearsal comparison)
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
S=gpurun_out/r6_final_suite.log; : > $S
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/ >> $S 2>&1 || { tail -40 $S; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" >> $S 2>&1 || { tail -20 $S; exit 1; }
tail -4 $S
L=gpurun_out/r6_final_bench_configs.log; : > $L
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
L2=gpurun_out/r6_final_rehearsal.log; : > $L2
reh() {
  local lab=$1; shift
  echo "== $lab" >> $L2
  LSD_MERGE_PREFILL=0 timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 "$@" > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L2; exit 1; }
  grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*\|"prefill_ms": [0-9.]*\|"stage_busy": \[[^]]*\]' gpurun_out/_r.out | tr '\n' ' ' >> $L2; echo >> $L2
}
C="--model gpt2 --batch 4096 --microbatches 16 --prompt 64 --gen 64"
X="--model gpt2-xl --batch 4096 --microbatches 16 --prompt 64 --gen 64"
for r in 1 2; do
  reh "gpt2 P=1 16x256" $C
  reh "gpt2 P=8 16x256 devloop" $C --loopback-stages 8
  reh "gpt2-xl P=1 16x256" $X
  reh "gpt2-xl P=8 16x256 devloop" $X --loopback-stages 8
done
reh "gpt2 P=1 4x256 (config 2)" --model gpt2 --batch 1024 --microbatches 4
reh "gpt2 P=2 4x256 (config 2) devloop" --model gpt2 --batch 1024 --microbatches 4 --loopback-stages 2
