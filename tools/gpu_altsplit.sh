#!/bin/bash
# Alternating splits: GPU test suite, then the P=8 / P=4 loopback schedules with and without
cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo "tests rc=$?"; exit 1; }
L=gpurun_out/altsplit.log; : > $L
A="--prompt 64 --gen 64 --steps 2 --warmup 1"
for v in 1 0; do
  echo "== P=8 loopback M=16 x 256 LSD_ALT_SPLIT=$v" >> $L
  LSD_ALT_SPLIT=$v timeout -k 10 300 python bench.py --loopback-stages 8 --batch 4096 --microbatches 16 $A >> $L 2>&1 || exit 1
done
echo "== P=1 M=16 x 256" >> $L
timeout -k 10 300 python bench.py --batch 4096 --microbatches 16 $A >> $L 2>&1 || exit 1
