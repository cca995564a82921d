#!/bin/bash
# Round 4 A/B (verdict r3 weak 3, "the slab traffic ... has not been attacked"): residual-projection
# split-K slabs stored bf16 (LSD_SLAB_BF16=1: half the bytes the GEMM writes and the next norm
# reads) vs fp32.  Kernel tests in the default env (the norm's bf16-slab path), the numerics suite
# with bf16 slabs, then the headline bench interleaved fp32 / bf16 / fp32 / bf16 on one box.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gpurun_out/r4_slab_bf16.log; : > $L
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "norm_with_slab" >> $L 2>&1 || exit 1
echo "== numerics with LSD_SLAB_BF16=1" >> $L
LSD_SLAB_BF16=1 timeout -k 10 400 python -u -m pytest -q --timeout 180 --timeout-method thread -m gpu tests/test_numerics_gpu.py tests/test_kernels_gpu.py -k "numerics or residual or golden or depth" >> $L 2>&1
echo "numerics rc=$?" >> $L
run() {  # label, env...
  local lab=$1; shift
  echo "== $lab" >> $L
  env "$@" timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; return 1; }
  grep "^{" gpurun_out/_r.out >> $L
}
run "fp32 slabs" LSD_SLAB_BF16=0 && run "bf16 slabs" LSD_SLAB_BF16=1 && \
run "fp32 slabs (again)" LSD_SLAB_BF16=0 && run "bf16 slabs (again)" LSD_SLAB_BF16=1
rc=$?
python3 - <<'PY'
import json
lab=None
for l in open("gpurun_out/r4_slab_bf16.log"):
    if l.startswith("=="): lab=l[3:].strip(); continue
    if l.startswith("{"):
        d=json.loads(l); print(f"{lab:24s} {d['value']:10.0f} tok/s p50 {d['p50_token_latency_ms']:.3f} ms prefill {d['prefill_ms']}")
PY
exit $rc
