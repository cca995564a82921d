#!/bin/bash
# round 6: single-stream lm_head GEMV writes segment maxima for the sampler; GEMV + sampler kernel
# tests, then single-stream benches (segmax=1 default vs segmax=0, interleaved) and GPT-2 small 512
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
S=gpurun_out/r6_ss_segmax_tests.log; : > $S
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gemv_gpu.py tests/test_kernels_gpu.py -k "gemv or sampler" >> $S 2>&1 || { tail -40 $S; exit 1; }
tail -2 $S
L=gpurun_out/r6_ss_segmax.log; : > $L
run() {
  local lab=$1; shift
  echo "== $lab" >> $L
  env "$@" timeout -k 10 300 python -u bench.py --batch 1 --microbatches 1 --steps 3 --warmup 1 $MODEL > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*' gpurun_out/_r.out | tr '\n' ' ' >> $L; echo >> $L
}
for MODEL in "--model gpt2-xl" "--model llama-3-8b" "--model gpt2"; do
  for r in 1 2; do
    run "$MODEL segmax=1" LSD_ROUTING=
    run "$MODEL segmax=0" LSD_ROUTING=segmax=0
  done
done
echo "== gpt2 512" >> $L
timeout -k 10 300 python -u bench.py --model gpt2 --steps 5 --warmup 2 > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
grep "^{" gpurun_out/_r.out >> $L
cat $L
