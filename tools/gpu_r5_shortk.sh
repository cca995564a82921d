#!/bin/bash
# round 5: short-K tiled routing -- engine / numerics tests, GPT-2 small bench A/B (2 x 128, 2 x 256)
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py tests/test_devloop_gpu.py tests/test_numerics_gpu.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_shortk_tests.log 2>&1 || exit $?
L=gpurun_out/r5_shortk.log; : > $L
for i in 1 2; do
  for k in 1024 0; do
    echo "== gpt2 --batch 256 LSD_TILED_SHORT_K=$k (round $i)" >> $L
    LSD_TILED_SHORT_K=$k timeout -k 10 300 python -u bench.py --model gpt2 --batch 256 --steps 3 --warmup 1 >> $L 2>&1 || exit $?
    echo "== gpt2 512 LSD_TILED_SHORT_K=$k (round $i)" >> $L
    LSD_TILED_SHORT_K=$k timeout -k 10 300 python -u bench.py --model gpt2 --steps 3 --warmup 1 >> $L 2>&1 || exit $?
  done
done
