#!/bin/bash
# round 6: Llama-3 8B 512-row decode QKV on gemm_d256 over two 256-row blocks (routing table):
# numerics gate, bench x2; lm_head tile alternatives (tools/lmhead_routes.py)
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_numerics_gpu.py -k "llama" -q --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r6_pytest_llama_qkv.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/r6_pytest_llama_qkv.log
[ $rc -eq 0 ] || exit $rc
L=gpurun_out/r6_llama_qkv_bench.log; : > $L
run() {
  echo "== $*" >> $L
  env "$@" timeout -k 10 400 python -u bench.py --model llama-3-8b --steps 2 --warmup 1 > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*\|"prefill_ms": [0-9.]*' gpurun_out/_r.out | tr '\n' ' ' >> $L; echo >> $L
}
for r in 1 2; do
  run LSD_NOOP=1
  run LSD_ROUTING=d256_rb_max_m=256
done
timeout -k 10 300 python -u tools/lmhead_routes.py > gpurun_out/r6_lmhead_routes.log 2>&1
