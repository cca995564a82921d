#!/bin/bash
# A/B of the GPT-2 small 8-stage devloop rehearsal (threads): where the gap to P = 1 is
# (ring size for the prefill chunks, chunked vs whole-prompt prefill, lanes).
set -o pipefail
export TMPDIR=/tmp LSD_HOST_PROFILE=1
mkdir -p gpurun_out
L=gpurun_out/r4_ab_rehearsal.log; : > $L
C="--model gpt2 --batch 4096 --microbatches 16 --prompt 64 --gen 64 --steps 2 --warmup 1"
run() { local lab=$1; shift; echo "== $lab" >> $L; echo "== $(date +%T) $lab"
  timeout -k 10 300 env "$@" > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; return 1; }
  grep "^{" gpurun_out/_r.out >> $L; grep "host per" gpurun_out/_r.err >> $L; }
run "P=1" python bench.py $C && \
run "P=8 devloop" python bench.py $C --loopback-stages 8 && \
run "P=8 devloop ring 512MB" LSD_LOOP_RING_MB=512 python bench.py $C --loopback-stages 8 && \
run "P=8 devloop no prefill chunks" python bench.py $C --loopback-stages 8 --prefill-chunk 0 && \
run "P=1 prefill chunk 32" python bench.py $C --prefill-chunk 32
rc=$?
python3 - <<'PY'
import json
lab=None
for l in open("gpurun_out/r4_ab_rehearsal.log"):
    if l.startswith("=="): lab=l[3:].strip(); continue
    if l.startswith("{"):
        d=json.loads(l); print(f"{lab:32s} {d['value']:9.0f} tok/s p50 {d['p50_token_latency_ms']:.2f} prefill {d['prefill_ms']:.0f} max {d['max_decode_step_ms']:.0f} ms/step {d['ms_per_step']:.0f}")
    elif l.startswith("host"): print("   ", l.strip()[:160])
PY
exit $rc
