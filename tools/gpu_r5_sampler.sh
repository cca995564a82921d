#!/bin/bash
# round 5: rank-selection sampler + lm_head segment maxima -- kernel tests,
# sampler timing by path, lm_head+sample microbench, headline + GPT-2 small bench A/B
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r5_sampler_final.log
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "sampler or segmax" > gpurun_out/r5_sampler_tests.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_numerics_gpu.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider >> gpurun_out/r5_sampler_tests.log 2>&1 || exit $?
echo "== tools/sample_timing.py" > $L
timeout -k 10 300 python -u tools/sample_timing.py >> $L 2>&1 || exit $?
echo "== microbench lmsample" >> $L
timeout -k 10 300 python -u tools/microbench.py lmsample >> $L 2>&1 || exit $?
for i in 1 2; do
  for sg in 1 0; do
    echo "== bench LSD_SEGMAX=$sg (round $i)" >> $L
    LSD_SEGMAX=$sg timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 >> $L 2>&1 || exit $?
  done
done
for i in 1 2; do
  for sg in 1 0; do
    echo "== bench gpt2 small LSD_SEGMAX=$sg (round $i)" >> $L
    LSD_SEGMAX=$sg timeout -k 10 300 python -u bench.py --model gpt2 --steps 3 --warmup 1 >> $L 2>&1 || exit $?
  done
done
