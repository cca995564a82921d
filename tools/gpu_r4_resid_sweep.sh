#!/bin/bash
# Round 4: residual-projection K splits (bf16 slabs: the default since the slab A/B) at 256 rows (LSD_RING_RESID_TARGET: workgroup target of the
# split-K residual GEMMs on the 8-wave ring; 256 default = 3 / 5 splits for GPT-2 XL's K 1600 / 6400).
# Fewer splits = fewer slabs for the next norm to fold and fewer workgroups beside the other lane's
# attention.  Headline config, same box, default run first and last.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gpurun_out/r4_resid_sweep.log; : > $L
run() {  # label, env...
  local lab=$1; shift
  echo "== $lab" >> $L
  env "$@" timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; return 1; }
  grep "^{" gpurun_out/_r.out >> $L
}
run "default" LSD_X=0 && \
run "RESID_TARGET=200 (3 / 4 splits)" LSD_RING_RESID_TARGET=200 && \
run "RESID_TARGET=300 (3 / 6 splits)" LSD_RING_RESID_TARGET=300 && \
run "RESID_TARGET=350 (3 / 7 splits)" LSD_RING_RESID_TARGET=350 && \
run "RESID_TARGET=450 (3 / 9 splits)" LSD_RING_RESID_TARGET=450 && \
run "default (again)" LSD_X=0
rc=$?
python3 - <<'PY'
import json
lab=None
for l in open("gpurun_out/r4_resid_sweep.log"):
    if l.startswith("=="): lab=l[3:].strip(); continue
    if l.startswith("{"):
        d=json.loads(l); print(f"{lab:30s} {d['value']:10.0f} tok/s p50 {d['p50_token_latency_ms']:.3f} ms prefill {d['prefill_ms']}")
PY
exit $rc
