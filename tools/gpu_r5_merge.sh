#!/bin/bash
# round 5: merged prefill at one stage -- test, then the headline bench A/B
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "merged_prefill" > gpurun_out/r5_merge_tests.log 2>&1 || exit $?
L=gpurun_out/r5_merge.log; : > $L
for i in 1 2; do
  for m in 1 0; do
    echo "== bench LSD_MERGE_PREFILL=$m (round $i)" >> $L
    LSD_MERGE_PREFILL=$m timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 >> $L 2>&1 || exit $?
  done
done
for m in 1 0; do
  echo "== bench gpt2 LSD_MERGE_PREFILL=$m" >> $L
  LSD_MERGE_PREFILL=$m timeout -k 10 300 python -u bench.py --model gpt2 --steps 3 --warmup 1 >> $L 2>&1 || exit $?
done
