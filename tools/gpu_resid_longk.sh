#!/bin/bash
# long-K residual split rule at 256 rows: GPU numerics + Llama-3 8B 256-sequence bench A/B
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/resid_longk_ab.log; : > $L
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "resid_splits_above" > gpurun_out/resid_longk_test.log 2>&1 || exit 1
run() { echo "== $*" >> $L; env "$@" timeout -k 10 400 python bench.py --model llama-3-8b --batch 256 --steps 2 --warmup 1 2>&1 | grep metric >> $L; }
run LSD_RESID_LONGK=0 && run LSD_RESID_LONGK=1 && run LSD_RESID_LONGK=0 && run LSD_RESID_LONGK=1
