#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/bench_cb3.log; : > $L
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_engine_gpu.py tests/test_dist_gpu.py >> $L 2>&1 || exit 1
echo "== single" >> $L
LSD_HOST_PROFILE=1 timeout -k 10 200 python bench.py --batch 1 --microbatches 1 --steps 3 --warmup 1 >> $L 2>&1 || exit 1
echo "== headline" >> $L
LSD_HOST_PROFILE=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 >> $L 2>&1 || exit 1
for P in 2 4 8; do
echo "== loopback P=$P (total 512)" >> $L
timeout -k 10 300 python bench.py --loopback-stages $P --batch 512 --steps 2 --warmup 1 >> $L 2>&1 || exit 1
done
