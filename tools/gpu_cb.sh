#!/bin/bash
# continuous-batching pipeline on the GPU: all GPU tests, then benches
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests -m gpu > gpurun_out/pytest_all.log 2>&1 || { echo "pytest rc=$?" >> gpurun_out/pytest_all.log; exit 1; }
L=gpurun_out/bench_cb.log; : > $L
echo "== headline" >> $L
timeout -k 10 300 python bench.py --steps 3 --warmup 1 >> $L 2>&1 || exit 1
echo "== single" >> $L
timeout -k 10 200 python bench.py --batch 1 --microbatches 1 --steps 3 --warmup 1 >> $L 2>&1 || exit 1
for P in 2 4 8; do
  echo "== loopback P=$P (total 512)" >> $L
  timeout -k 10 300 python bench.py --loopback-stages $P --batch 512 --steps 2 --warmup 1 >> $L 2>&1 || exit 1
done
