#!/bin/bash
# residual split rule at 257-1024 rows: GPU numerics test + bench A/B (Llama-3 8B 512 seqs, GPT-2 XL 1024 seqs, headline)
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/resid512_ab.log; : > $L
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "resid_splits_above" > gpurun_out/resid512_test.log 2>&1 || exit 1
run() { local m=$1; shift; echo "== $m $*" >> $L; env "$@" timeout -k 10 400 python bench.py --model $m --steps 2 --warmup 1 2>&1 | grep metric >> $L; }
run llama-3-8b LSD_RESID_WG_TARGET=0 && run llama-3-8b LSD_RESID_WG_TARGET=1024 && \
run gpt2-xl LSD_RESID_WG_TARGET=0 BENCH_BATCH=1024 && run gpt2-xl LSD_RESID_WG_TARGET=1024 BENCH_BATCH=1024 && \
run gpt2-xl LSD_RESID_WG_TARGET=1024
