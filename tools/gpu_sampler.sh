#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/sampler.log; : > $L
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_kernels_gpu.py -k "sampl or long or engine or graph or chunk or loopback or join or pipeline or stage or greedy or shapes or wide" tests/test_engine_gpu.py tests/test_long_context.py >> $L 2>&1 || exit 1
timeout -k 10 200 python tools/microbench.py sample >> $L 2>&1
echo "== single" >> $L
timeout -k 10 200 python bench.py --batch 1 --microbatches 1 --steps 3 --warmup 1 >> $L 2>&1 || exit 1
echo "== headline" >> $L
timeout -k 10 300 python bench.py --steps 3 --warmup 1 >> $L 2>&1 || exit 1
