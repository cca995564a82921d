#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/ab_attn.log; : > $L
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py -k attention > gpurun_out/pytest_attn.log 2>&1 || { echo "pytest rc=$?" >> $L; exit 1; }
for sw in 4 8 16 4 8 16; do
  echo "== sw=$sw" >> $L
  LSD_ATTN_SMALL_WAVES=$sw timeout -k 10 200 python bench.py --batch 1 --microbatches 1 --steps 3 --warmup 1 >> $L 2>&1 || exit 1
done
for sw in 4 8; do echo "== llama sw=$sw" >> $L; LSD_ATTN_SMALL_WAVES=$sw timeout -k 10 300 python bench.py --model llama-3-8b --batch 1 --microbatches 1 --steps 2 --warmup 1 >> $L 2>&1 || exit 1; done
