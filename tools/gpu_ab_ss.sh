#!/bin/bash
# kernel tests, then single-stream A/B (GEMV nt loads) and the headline bench
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/ab_ss.log; : > $L
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gemv_gpu.py tests/test_kernels_gpu.py -k "gemv or attention" > gpurun_out/pytest_ab.log 2>&1 || { echo "pytest rc=$?" >> $L; exit 1; }
for nt in 0 1 0 1; do
  echo "== nt=$nt" >> $L
  LSD_GEMV_NT=$nt timeout -k 10 200 python bench.py --batch 1 --microbatches 1 --steps 2 --warmup 1 >> $L 2>&1 || exit 1
done
echo "== gpt2 small nt=0/1" >> $L
for nt in 0 1; do LSD_GEMV_NT=$nt timeout -k 10 200 python bench.py --model gpt2 --batch 1 --microbatches 1 --steps 2 --warmup 1 >> $L 2>&1 || exit 1; done
echo "== llama nt=0/1" >> $L
for nt in 0 1; do LSD_GEMV_NT=$nt timeout -k 10 300 python bench.py --model llama-3-8b --batch 1 --microbatches 1 --steps 2 --warmup 1 >> $L 2>&1 || exit 1; done
echo "== headline" >> $L
timeout -k 10 300 python bench.py --steps 3 --warmup 1 >> $L 2>&1
