#!/bin/bash
# round 5: prefill chunk graphs (pipeline.py _prefill_graph) -- engine / devloop / multi-process
# tests, then the 8-stage one-GPU rehearsal with the graphs on (auto: P > 1) and off
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp LSD_HOST_PROFILE=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_engine_gpu.py tests/test_devloop_gpu.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r5_pfgraph_tests.log 2>&1 || exit $?
L=gpurun_out/r5_pfgraph_rehearsal.log; : > $L
run() {  # label, env, args...
  local lab=$1 e=$2; shift 2
  echo "== $lab" >> $L
  env $e timeout -k 10 400 python bench.py --steps 2 --warmup 1 "$@" > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -30 gpurun_out/_r.err >> $L; return 1; }
  grep "^{" gpurun_out/_r.out >> $L
  grep "host per" gpurun_out/_r.err >> $L
}
C="--prompt 64 --gen 64"
run "gpt2 P=1 M=16x256" LSD_PREFILL_GRAPHS=auto --model gpt2 --batch 4096 --microbatches 16 $C && \
run "gpt2 P=8 M=16x256 devloop, prefill graphs" LSD_PREFILL_GRAPHS=auto --model gpt2 --batch 4096 --microbatches 16 --loopback-stages 8 $C && \
run "gpt2 P=8 M=16x256 devloop, eager prefill" LSD_PREFILL_GRAPHS=0 --model gpt2 --batch 4096 --microbatches 16 --loopback-stages 8 $C && \
run "gpt2 P=1 M=16x256 (2)" LSD_PREFILL_GRAPHS=auto --model gpt2 --batch 4096 --microbatches 16 $C && \
run "gpt2 P=8 M=16x256 devloop, prefill graphs (2)" LSD_PREFILL_GRAPHS=auto --model gpt2 --batch 4096 --microbatches 16 --loopback-stages 8 $C && \
run "xl P=1 M=16x256" LSD_PREFILL_GRAPHS=auto --model gpt2-xl --batch 4096 --microbatches 16 $C && \
run "xl P=8 M=16x256 devloop, prefill graphs" LSD_PREFILL_GRAPHS=auto --model gpt2-xl --batch 4096 --microbatches 16 --loopback-stages 8 $C
