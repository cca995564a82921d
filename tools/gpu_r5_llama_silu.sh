#!/bin/bash
# round 5: Llama decode gate_up on hipBLASLt + SiLU*up pass at >= 512 rows -- tests, then the
# Llama-3 8B 512-sequence bench A/B (interleaved)
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
T=gpurun_out/r5_llama_silu_tests.log
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "silu_mul or blaslt" > $T 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_numerics_gpu.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider -k "blaslt_silu or llama_512" -s >> $T 2>&1 || exit $?
L=gpurun_out/r5_llama_silu.log; : > $L
for i in 1 2; do
  for m in 512 0; do
    echo "== bench llama-3-8b LSD_BLASLT_SILU_MIN_M=$m (round $i)" >> $L
    LSD_BLASLT_SILU_MIN_M=$m timeout -k 10 400 python -u bench.py --model llama-3-8b --steps 2 --warmup 1 >> $L 2>&1 || exit $?
  done
done
