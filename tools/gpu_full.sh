#!/bin/bash
# Full GPU test suite + single-stream and headline bench.
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/full.log; : > $L
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests -m gpu >> $L 2>&1 || exit 1
echo "== single" >> $L
timeout -k 10 200 python bench.py --batch 1 --microbatches 1 --steps 3 --warmup 1 >> $L 2>&1 || exit 1
echo "== headline" >> $L
timeout -k 10 300 python bench.py --steps 3 --warmup 1 >> $L 2>&1 || exit 1
