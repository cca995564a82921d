#!/bin/bash
# round 6: decode attention block shape in the bench (LSD_ROUTING attn_large_waves 4 / 42 / 2), interleaved
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r6_attn_ab.log; : > $L
run() {  # run ENV=VALUE bench-args...
  echo "== $*" >> $L
  local e=$1; shift
  env "$e" timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 "$@" > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*' gpurun_out/_r.out | tr '\n' ' ' >> $L; echo >> $L
}
for r in 1 2; do
  run LSD_NOOP=1
  run LSD_ROUTING=attn_large_waves=42
  run LSD_ROUTING=attn_large_waves=2
  run LSD_NOOP=1 --model gpt2
  run LSD_ROUTING=attn_large_waves=42 --model gpt2
  run LSD_ROUTING=attn_large_waves=2 --model gpt2
done
