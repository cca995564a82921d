#!/bin/bash
# headline-config variants: microbatch count / rows per group (decode GEMM M)
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/mbsweep.log; : > $L
for a in "--microbatches 1" "--microbatches 2" "--microbatches 4" "--batch 1024 --microbatches 2" "--batch 1024 --microbatches 4"; do
  echo "== $a" >> $L
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 $a >> $L 2>&1 || exit 1
done
