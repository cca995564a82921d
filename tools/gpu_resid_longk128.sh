#!/bin/bash
# long-K residual split rule extended to 65-128 rows: Llama-3 8B 128-sequence bench A/B
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/resid_longk128_ab.log; : > $L
run() { echo "== $*" >> $L; env "$@" timeout -k 10 400 python bench.py --model llama-3-8b --batch 128 --steps 2 --warmup 1 2>&1 | grep metric >> $L; }
run LSD_RESID_LONGK_MIN_M=128 && run LSD_RESID_LONGK_MIN_M=64 && run LSD_RESID_LONGK_MIN_M=128 && run LSD_RESID_LONGK_MIN_M=64
