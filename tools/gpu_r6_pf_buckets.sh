#!/bin/bash
# round 6: bucketed prefill graphs at one stage (parallel/pipeline.py _bucket_graph): engine GPU tests,
# then closed-loop serving (512 in flight, join policy default) with LSD_PF_BUCKETS=1 vs 0, and the
# headline bench (its 65 K-token merged prefill is above the bucket limit: unchanged path)
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
S=gpurun_out/r6_pf_buckets_tests.log; : > $S
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_engine_gpu.py tests/test_kernels_gpu.py -k "engine or graph or prefill or merged or bucket" >> $S 2>&1 || { tail -40 $S; exit 1; }
tail -2 $S
L=gpurun_out/r6_pf_buckets.log; : > $L
run() {
  local lab=$1; shift
  echo "== $lab" >> $L
  env "$@" timeout -k 10 300 python -u tools/serve_load.py --requests 4096 $ARGS > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep "^{" gpurun_out/_r.out >> $L
}
for m in gpt2-xl gpt2 llama-3-8b; do
  ARGS="--model $m" run "$m buckets=1" LSD_PF_BUCKETS=1
  ARGS="--model $m" run "$m buckets=0" LSD_PF_BUCKETS=0
done
ARGS="--model gpt2-xl" run "gpt2-xl buckets=1 (2)" LSD_PF_BUCKETS=1
echo "== headline" >> $L
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*\|"prefill_ms": [0-9.]*' gpurun_out/_r.out | tr '\n' ' ' >> $L
cat $L
