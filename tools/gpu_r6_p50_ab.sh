#!/bin/bash
# round 6: decode p50 regression -- interleaved same-box A/B of the round-4 HEAD (98a0803, built
# in ab/r4) against HEAD, plus HEAD with hipBLASLt routing off.  bench.py --steps 5 --warmup 1.
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r6_p50_ab.log; : > $L
R=$(pwd)
run() {
  local tag=$1 dir=$2; shift 2
  echo "== $tag $*" >> $L
  (cd $dir && env "$@" timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 > $R/gpurun_out/_r.out 2> $R/gpurun_out/_r.err) \
    || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*\|"prefill_ms": [0-9.]*\|"max_decode_step_ms": [0-9.]*' gpurun_out/_r.out | tr '\n' ' ' >> $L; echo >> $L
}
for r in 1 2 3; do
  run r4 ab/r4 LSD_NOOP=1
  run head . LSD_NOOP=1
  run head_noblaslt . LSD_BLASLT_MIN_M=0 LSD_BLASLT_DECODE_GELU_MIN_M=0 LSD_BLASLT_SILU_MIN_M=0 LSD_BLASLT_QKV_MIN_M=0
done
