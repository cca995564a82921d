#!/bin/bash
# Round 4: (a) verdict r3 item 1's Llama-3 8B row of the 8-stage rehearsal (device loopback
# threads vs P = 1 at equal microbatch shapes); (b) the headline config at 2 / 3 / 4 microbatch
# lanes (BENCH_MB), same box.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gpurun_out/r4_llama_lanes.log; : > $L
run() {  # label, args...
  local lab=$1; shift
  echo "== $lab" >> $L
  timeout -k 10 400 python bench.py "$@" > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -30 gpurun_out/_r.err >> $L; return 1; }
  grep "^{" gpurun_out/_r.out >> $L
}
C="--prompt 64 --gen 64 --steps 2 --warmup 1"
run "llama P=1 M=8x256"         --model llama-3-8b --batch 2048 --microbatches 8 $C && \
run "llama P=8 M=8x256 devloop" --model llama-3-8b --batch 2048 --microbatches 8 --loopback-stages 8 $C && \
run "xl headline MB=2" --steps 3 --warmup 1 --microbatches 2 && \
run "xl headline MB=4" --steps 3 --warmup 1 --microbatches 4 && \
run "xl headline MB=3" --steps 3 --warmup 1 --microbatches 3
rc=$?
python3 - <<'PY'
import json
lab=None
for l in open("gpurun_out/r4_llama_lanes.log"):
    if l.startswith("=="): lab=l[3:].strip(); continue
    if l.startswith("{"):
        d=json.loads(l); print(f"{lab:28s} {d['value']:10.0f} tok/s p50 {d['p50_token_latency_ms']:.3f} ms prefill {d['prefill_ms']} busy {d.get('stage_busy')}")
PY
exit $rc
