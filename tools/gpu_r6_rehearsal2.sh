#!/bin/bash
# round 6: one-GPU rehearsals of the multi-GPU schedules at the per-stage shapes of the real
# N-GPU weak-scaling run (2 groups of 256 rows per stage), merged prefill OFF on both sides,
# interleaved: stage threads over the device-loopback data plane (graph-captured edges + native
# executor = the default rccl path's twin) and over the event hand-off (= the torch-nccl
# fallback's twin), against one stage running the same groups.
#   config 2: GPT-2 small, P = 2: 1024 sequences, 4 x 256
#   GPT-2 XL, P = 8: 4096 sequences, 16 x 256, 64 + 64 tokens (KV of 128 + 128 would not fit one GPU)
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r6_rehearsal2.log; : > $L
run() {
  local lab=$1; shift
  echo "== $lab" >> $L
  LSD_MERGE_PREFILL=0 timeout -k 10 400 python -u bench.py "$@" > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep "^{" gpurun_out/_r.out | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    print(d['value'], d['p50_token_latency_ms'], d['prefill_ms'], d.get('transport'), d['config']['parallelism'], d.get('stage_busy'))" >> $L
}
S="--model gpt2 --batch 1024 --microbatches 4 --steps 3 --warmup 1"
for r in 1 2; do
  run "gpt2 P=1 4x256" $S
  run "gpt2 P=2 4x256 devloop" $S --loopback-stages 2
  run "gpt2 P=2 4x256 loopback(event)" $S --loopback-stages 2 --loopback-transport loopback
done
X="--batch 4096 --microbatches 16 --prompt 64 --gen 64 --steps 2 --warmup 1"
for r in 1 2; do
  run "xl P=1 16x256" $X
  run "xl P=8 16x256 devloop" $X --loopback-stages 8
  run "xl P=8 16x256 loopback(event)" $X --loopback-stages 8 --loopback-transport loopback
done
