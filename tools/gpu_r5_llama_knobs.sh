#!/bin/bash
# round 5, final build: Llama-3 8B 512-sequence knob re-check (bench.py --steps 2 --warmup 1, interleaved rounds)
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r5_llama_knobs.log; : > $L
run() {
  echo "== $*" >> $L
  env "$@" timeout -k 10 400 python -u bench.py --model llama-3-8b --steps 2 --warmup 1 > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*\|"prefill_ms": [0-9.]*' gpurun_out/_r.out | tr '\n' ' ' >> $L; echo >> $L
}
for r in 1 2; do
  run LSD_NOOP=1
  run LSD_RESID_WG_TARGET=512
  run LSD_RESID_WG_TARGET=2048
  run LSD_BLASLT_SILU_MAX_M=512
done
