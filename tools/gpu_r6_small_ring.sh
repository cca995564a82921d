#!/bin/bash
# round 6: GPT-2 small 512 sequences: short-K decode GEMM ring tile width (32-wide 4-wave ring by
# default under 128 workgroups; 64-wide tiles run on the 8-wave ring); interleaved
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r6_small_ring.log; : > $L
run() {
  local lab=$1; shift
  echo "== $lab" >> $L
  env "$@" timeout -k 10 300 python -u bench.py --model gpt2 --steps 5 --warmup 2 > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*\|"prefill_ms": [0-9.]*' gpurun_out/_r.out | tr '\n' ' ' >> $L; echo >> $L
}
for r in 1 2; do
  run "default" LSD_ROUTING=
  run "ring_tn=64" LSD_ROUTING=ring_tn=64
  run "ring_fill=64" LSD_ROUTING=ring_fill=64
  run "ring8=0" LSD_ROUTING=ring8=0
done
cat $L
