#!/bin/bash
# round 6: single-stream decode attention, 8-wave blocks with 8 keys per wave in flight
# (attn_small_waves=88) vs the default 8 waves x 4 keys; kernel tests, then interleaved benches
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
S=gpurun_out/r6_attn_u8_tests.log; : > $S
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_kernels_gpu.py -k "attention_decode" >> $S 2>&1 || { tail -40 $S; exit 1; }
tail -1 $S
L=gpurun_out/r6_attn_u8.log; : > $L
run() {
  local lab=$1; shift
  echo "== $lab" >> $L
  env "$@" timeout -k 10 300 python -u bench.py --batch 1 --microbatches 1 --steps 3 --warmup 1 $MODEL > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*' gpurun_out/_r.out | tr '\n' ' ' >> $L; echo >> $L
}
for MODEL in "--model llama-3-8b" "--model gpt2-xl"; do
  for r in 1 2; do
    run "$MODEL small_waves=8" LSD_ROUTING=
    run "$MODEL small_waves=88" LSD_ROUTING=attn_small_waves=88
  done
done
MODEL="--model llama-3-8b --batch 4"
run "$MODEL small_waves=8" LSD_ROUTING=
run "$MODEL small_waves=88" LSD_ROUTING=attn_small_waves=88
cat $L
