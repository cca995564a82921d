#!/bin/bash
# round 6 (re-entry build): multi-stage rehearsals on one GPU (devloop stage threads), merged prefill off
# on both sides, against one stage running the same groups
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L2=gpurun_out/r6_rehearsal3.log; : > $L2
reh() {
  local lab=$1; shift
  echo "== $lab" >> $L2
  LSD_MERGE_PREFILL=0 timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 "$@" > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L2; exit 1; }
  grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*\|"prefill_ms": [0-9.]*\|"stage_busy": \[[^]]*\]' gpurun_out/_r.out | tr '\n' ' ' >> $L2; echo >> $L2
}
for r in 1 2; do
  reh "gpt2 P=1 4x256 (config 2)" --model gpt2 --batch 1024 --microbatches 4
  reh "gpt2 P=2 4x256 (config 2) devloop" --model gpt2 --batch 1024 --microbatches 4 --loopback-stages 2
done
X="--model gpt2-xl --batch 4096 --microbatches 16 --prompt 64 --gen 64"
reh "gpt2-xl P=1 16x256" $X
reh "gpt2-xl P=8 16x256 devloop" $X --loopback-stages 8
cat $L2
