#!/bin/bash
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
S=gpurun_out/r6_attn_u8_check.log; : > $S
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_numerics_gpu.py >> $S 2>&1 || { tail -40 $S; exit 1; }
tail -1 $S
for i in 1 2; do timeout -k 10 300 python -u bench.py --model llama-3-8b --batch 1 --microbatches 1 --steps 3 --warmup 1 2>/dev/null | grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*' | tr '\n' ' ' >> $S; echo >> $S; done
tail -2 $S
