#!/bin/bash
# round 5: the whole GPU suite (no -x: every failure listed), smoke(), then bench.py across the
# README / BASELINE.md configurations
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r5_pytest_gpu_full.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/r5_pytest_gpu_full.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_smoke.log 2>&1 || exit $?
L=gpurun_out/r5_results_bench_configs.log; : > $L
run() {
  echo "== $*" >> $L
  timeout -k 10 400 python -u bench.py "$@" > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep "^{" gpurun_out/_r.out >> $L
}
run --steps 3 --warmup 1
run --steps 2 --warmup 1 --greedy
run --steps 2 --warmup 1 --batch 256
run --steps 2 --warmup 1 --batch 384
run --steps 2 --warmup 1 --batch 1024
run --batch 1 --microbatches 1 --steps 2 --warmup 1
run --model gpt2 --steps 3 --warmup 1
run --model gpt2 --batch 1 --microbatches 1 --steps 2 --warmup 1
run --model llama-3-8b --steps 2 --warmup 1
run --model llama-3-8b --batch 256 --steps 2 --warmup 1
run --model llama-3-8b --batch 128 --steps 2 --warmup 1
run --model llama-3-8b --batch 1 --microbatches 1 --steps 2 --warmup 1
