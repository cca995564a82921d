#!/bin/bash
# round 5: wave-per-row prefill norm -- kernel tests, microbench vs the block kernel, bench A/B
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "norm" > gpurun_out/r5_normwave_tests.log 2>&1 || exit $?
L=gpurun_out/r5_normwave.log
echo "== microbench normwave" > $L
timeout -k 10 300 python -u tools/microbench.py normwave >> $L 2>&1 || exit $?
for i in 1 2; do
  for m in 4096 0; do
    echo "== bench LSD_NORM_WAVE_MIN=$m (round $i)" >> $L
    LSD_NORM_WAVE_MIN=$m timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 >> $L 2>&1 || exit $?
  done
done
for m in 4096 0; do
  echo "== bench llama-3-8b LSD_NORM_WAVE_MIN=$m" >> $L
  LSD_NORM_WAVE_MIN=$m timeout -k 10 400 python -u bench.py --model llama-3-8b --steps 2 --warmup 1 >> $L 2>&1 || exit $?
done
