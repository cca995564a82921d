#!/bin/bash
# round 6: GPT-2 small out-projection (K 768) K splits on the ring: 1 (default, 24 workgroups)
# vs 2 / 3 bf16 slabs folded by the next LayerNorm; interleaved pairs, 512 sequences (2 x 256)
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r6_small_oproj.log; : > $L
run() {
  local lab=$1; shift
  echo "== $lab" >> $L
  env "$@" timeout -k 10 300 python -u bench.py --model gpt2 --steps 5 --warmup 2 > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*\|"prefill_ms": [0-9.]*' gpurun_out/_r.out | tr '\n' ' ' >> $L; echo >> $L
}
for r in 1 2; do
  run "default (512 per split)" LSD_ROUTING=
  run "256 per split (3 slabs)" LSD_ROUTING=resid_short_k_per_split=256
  run "384 per split (2 slabs)" LSD_ROUTING=resid_short_k_per_split=384
done
cat $L
