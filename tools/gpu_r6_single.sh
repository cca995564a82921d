#!/bin/bash
# round 6: single-stream decode after the GEMV epilogue-operand prefetch (gemv.hip step 0):
# GEMV / engine / numerics tests, bench.py --batch 1 for GPT-2 XL / small / Llama-3 8B (x2,
# interleaved), and rocprofv3 kernel statistics of GPT-2 XL and Llama-3 8B at batch 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemv_gpu.py tests/test_engine_gpu.py tests/test_numerics_gpu.py \
  -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r6_pytest_single.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/r6_pytest_single.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -u tools/probes/prefill_epilogues.py > gpurun_out/r6_prefill_epilogues.log 2>&1 || exit $?
L=gpurun_out/r6_single.log; : > $L
run() {
  echo "== $*" >> $L
  timeout -k 10 300 python -u bench.py --batch 1 --microbatches 1 --steps 3 --warmup 1 "$@" > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*' gpurun_out/_r.out | tr '\n' ' ' >> $L; echo >> $L
}
for r in 1 2; do
  run --model gpt2-xl
  run --model gpt2
  run --model llama-3-8b
done
cd /tmp && export TMPDIR=/tmp
for m in gpt2-xl llama-3-8b; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r6prof_b1_$m" -o run --output-format csv -- \
    python3 "$R/bench.py" --model $m --batch 1 --microbatches 1 --steps 2 --warmup 1 > "$R/gpurun_out/r6prof_b1_$m.log" 2>&1 || exit $?
  rm -f "$R"/gpurun_out/r6prof_b1_$m/*kernel_trace.csv
done
