#!/bin/bash
# Round 4: the README's other configurations with bf16 split-K slabs (default) vs fp32 slabs
# (LSD_SLAB_BF16=0), one box: Llama-3 8B 512 sequences, GPT-2 small 512 sequences.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gpurun_out/r4_configs.log; : > $L
run() {  # label, env, args...
  local lab=$1 e=$2; shift 2
  echo "== $lab" >> $L
  env $e timeout -k 10 400 python bench.py --steps 2 --warmup 1 "$@" > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; return 1; }
  grep "^{" gpurun_out/_r.out >> $L
}
run "llama-3-8b 512 bf16 slabs" LSD_SLAB_BF16=1 --model llama-3-8b && \
run "llama-3-8b 512 fp32 slabs" LSD_SLAB_BF16=0 --model llama-3-8b && \
run "gpt2 512 bf16 slabs" LSD_SLAB_BF16=1 --model gpt2 && \
run "gpt2 512 fp32 slabs" LSD_SLAB_BF16=0 --model gpt2
rc=$?
python3 - <<'PY'
import json
lab=None
for l in open("gpurun_out/r4_configs.log"):
    if l.startswith("=="): lab=l[3:].strip(); continue
    if l.startswith("{"):
        d=json.loads(l); print(f"{lab:28s} {d['value']:10.0f} tok/s p50 {d['p50_token_latency_ms']:.3f} ms prefill {d['prefill_ms']}")
PY
exit $rc
