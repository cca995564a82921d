#!/bin/bash
# round 5: Llama-3 8B 512-row decode QKV on hipBLASLt (fp32 out) + the RoPE / cache-append pass
# (LSD_BLASLT_QKV_MIN_M): tests, then the 512-sequence bench A/B, interleaved
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r5_llama_qkv.log; : > $L
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_numerics_gpu.py -k "qkv or llama_512" -q --timeout 200 --timeout-method thread -p no:cacheprovider >> $L 2>&1 || exit 1
for r in 1 2; do
  for m in 512 0; do
    echo "== llama-3-8b LSD_BLASLT_QKV_MIN_M=$m (round $r)" >> $L
    LSD_BLASLT_QKV_MIN_M=$m timeout -k 10 400 python -u bench.py --model llama-3-8b --steps 2 --warmup 1 > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
    grep "^{" gpurun_out/_r.out | cut -c1-420 >> $L
  done
done
