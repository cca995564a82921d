#!/bin/bash
# round 6: native composition-change items (apply_rows kernel in exec_items): kernel + engine + devloop tests, benches
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r6_rows.log; : > $L
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_kernels_gpu.py -k "apply_rows" tests/test_engine_gpu.py tests/test_devloop_gpu.py >> $L 2>&1 || { tail -30 $L; exit 1; }
run() {
  echo "== $*" >> $L
  LSD_HOST_PROFILE=1 timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 "$@" > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  cat gpurun_out/_r.out >> $L; grep "^host per" gpurun_out/_r.err >> $L
}
run --model gpt2 --batch 4096 --microbatches 16 --prompt 64 --gen 64
run --model gpt2 --batch 4096 --microbatches 16 --prompt 64 --gen 64 --loopback-stages 8
run
