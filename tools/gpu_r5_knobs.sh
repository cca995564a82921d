#!/bin/bash
# round 5, final build: re-check of the headline's tuning knobs (bench.py --steps 3 --warmup 1, interleaved rounds)
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r5_knobs.log; : > $L
run() {
  echo "== $*" >> $L
  env "$@" timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*\|"prefill_ms": [0-9.]*' gpurun_out/_r.out | tr '\n' ' ' >> $L; echo >> $L
}
for r in 1 2; do
  run LSD_NOOP=1
  run LSD_RING_RESID_TARGET=200
  run LSD_RING_RESID_TARGET=320
  run LSD_ATTN_LARGE_WAVES=8
  run LSD_RING_SLOTS=4
  run LSD_SEGMAX=0
done
