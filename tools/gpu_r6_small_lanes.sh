#!/bin/bash
# round 6: GPT-2 small 512 sequences: microbatch groups x lanes (streams); interleaved
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r6_small_lanes.log; : > $L
run() {
  local lab=$1; shift
  echo "== $lab" >> $L
  env "$@" timeout -k 10 300 python -u bench.py --model gpt2 --steps 5 --warmup 2 $ARGS > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*\|"prefill_ms": [0-9.]*' gpurun_out/_r.out | tr '\n' ' ' >> $L; echo >> $L
}
for r in 1 2; do
  ARGS="" run "2 x 256, 2 lanes (default)" LSD_LANES=2
  ARGS="--microbatches 4" run "4 x 128, 2 lanes" LSD_LANES=2
  ARGS="--microbatches 4" run "4 x 128, 4 lanes" LSD_LANES=4
  ARGS="--microbatches 3" run "3 x 171, 3 lanes" LSD_LANES=3
  ARGS="--microbatches 4" run "4 x 128, 3 lanes" LSD_LANES=3
done
cat $L
