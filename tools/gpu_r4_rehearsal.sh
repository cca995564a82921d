#!/bin/bash
# Round 4 (verdict r3 item 1): every BASELINE config's multi-stage schedule on ONE GPU through the
# device loopback fabric -- decode graphs carry their own edge receive / send, the native executor
# enqueues whole steps at P > 1 (the --transport rccl code path of an 8-GPU node) -- against P = 1
# at equal microbatch shapes; GPT-2 small P = 8 also with the event hand-off loopback (round 3's
# rehearsal transport) for comparison.  LSD_HOST_PROFILE=1: stage 0's host time per decode step.
set -o pipefail
export TMPDIR=/tmp LSD_HOST_PROFILE=1
mkdir -p gpurun_out
L=gpurun_out/r4_rehearsal.log; : > $L
run() {  # label, args...
  local lab=$1; shift
  echo "== $lab" >> $L
  timeout -k 10 400 python bench.py --steps 2 --warmup 1 "$@" > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -30 gpurun_out/_r.err >> $L; return 1; }
  grep "^{" gpurun_out/_r.out >> $L
  grep "host per" gpurun_out/_r.err >> $L
}
C="--prompt 64 --gen 64"
run "gpt2 P=1 M=16x256"         --model gpt2 --batch 4096 --microbatches 16 $C && \
run "gpt2 P=8 M=16x256 devloop" --model gpt2 --batch 4096 --microbatches 16 --loopback-stages 8 $C && \
run "gpt2 P=8 M=16x256 loopback" --model gpt2 --batch 4096 --microbatches 16 --loopback-stages 8 --loopback-transport loopback $C && \
run "gpt2 P=2 M=4x256 devloop"  --model gpt2 --batch 1024 --microbatches 4 --loopback-stages 2 $C && \
run "gpt2 P=1 M=4x256"          --model gpt2 --batch 1024 --microbatches 4 $C && \
run "xl P=1 M=8x256"            --model gpt2-xl --batch 2048 --microbatches 8 $C && \
run "xl P=4 M=8x256 devloop"    --model gpt2-xl --batch 2048 --microbatches 8 --loopback-stages 4 $C && \
run "xl P=1 M=16x256"           --model gpt2-xl --batch 4096 --microbatches 16 $C && \
run "xl P=8 M=16x256 devloop"   --model gpt2-xl --batch 4096 --microbatches 16 --loopback-stages 8 $C && \
run "llama P=1 M=8x256"         --model llama-3-8b --batch 2048 --microbatches 8 $C && \
run "llama P=8 M=8x256 devloop" --model llama-3-8b --batch 2048 --microbatches 8 --loopback-stages 8 $C
rc=$?
python3 - <<'PY'
lab=None
import json
for l in open("gpurun_out/r4_rehearsal.log"):
    if l.startswith("=="): lab=l[3:].strip(); continue
    if l.startswith("{"):
        d=json.loads(l); print(f"{lab:28s} {d['value']:10.0f} tok/s p50 {d['p50_token_latency_ms']:.3f} ms busy {d.get('stage_busy')}")
    elif l.startswith("host"): print("   ", l.strip())
PY
exit $rc
