#!/bin/bash
# round 6: wave-per-row norm with its weights loaded first; rows per block 4 (default) vs 1 / 2.
# GPT-2 small 512 sequences (decode norms at H 768 take this kernel) and the GPT-2 XL headline
# (its 65 K-row prefill norms do); interleaved
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
S=gpurun_out/r6_normwave_tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_kernels_gpu.py -k "norm" > $S 2>&1 || { tail -30 $S; exit 1; }
grep passed $S
L=gpurun_out/r6_normwave_rpb.log; : > $L
run() {
  local lab=$1; shift
  echo "== $lab" >> $L
  env "$@" timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 $MODEL > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*\|"prefill_ms": [0-9.]*' gpurun_out/_r.out | tr '\n' ' ' >> $L; echo >> $L
}
MODEL="--model gpt2"
for r in 1 2; do
  run "gpt2 rpb=4" LSD_ROUTING=
  run "gpt2 rpb=1" LSD_ROUTING=norm_wave_rpb=1
  run "gpt2 rpb=2" LSD_ROUTING=norm_wave_rpb=2
done
MODEL="--model gpt2-xl"
run "xl rpb=4" LSD_ROUTING=
run "xl rpb=1" LSD_ROUTING=norm_wave_rpb=1
cat $L
