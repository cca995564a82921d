#!/bin/bash
# round 5: refined hipBLASLt routing -- numerics at the headline shape, bench A/B (XL, Llama-3 8B)
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r5_blaslt2.log
timeout -k 10 600 python -u -m pytest tests/test_numerics_gpu.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r5_blaslt2_tests.log 2>&1 || exit $?
: > $L
for i in 1 2; do
  for m in 4096 0; do
    echo "== bench LSD_BLASLT_MIN_M=$m (round $i)" >> $L
    LSD_BLASLT_MIN_M=$m timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 >> $L 2>&1 || exit $?
  done
done
for m in 4096 0; do
  echo "== bench llama-3-8b LSD_BLASLT_MIN_M=$m" >> $L
  LSD_BLASLT_MIN_M=$m timeout -k 10 400 python -u bench.py --model llama-3-8b --steps 2 --warmup 1 >> $L 2>&1 || exit $?
done
