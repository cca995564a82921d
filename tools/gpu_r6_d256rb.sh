#!/bin/bash
# round 6: gemm_d256 over several 256-row blocks (M <= 1024): kernel tests, the Llama-3 8B 512-row
# GEMM tilings (tools/llama512_gemm.py), Llama-3 8B 512 sequences as 1 x 512 and 2 x 256 groups
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "d256 or qkv_kv_append" -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r6_pytest_d256rb.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/r6_pytest_d256rb.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/llama512_gemm.py > gpurun_out/r6_llama512_gemm_v2.log 2>&1 || exit $?
L=gpurun_out/r6_llama_groups.log; : > $L
run() {
  echo "== $*" >> $L
  timeout -k 10 400 python -u bench.py --model llama-3-8b --steps 2 --warmup 1 "$@" > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*\|"prefill_ms": [0-9.]*' gpurun_out/_r.out | tr '\n' ' ' >> $L; echo >> $L
}
run --microbatches 1
run --microbatches 2
