#!/bin/bash
# round 6: single stream with non-temporal GEMV weight loads (LSD_ROUTING=gemv_nt=1) vs default,
# interleaved; rocprofv3 kernel statistics of Llama-3 8B at 512 sequences (QKV on gemm_d256 row blocks)
export HSA_ENABLE_IPC_MODE_LEGACY=0
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
L=gpurun_out/r6_gemv_nt.log; : > $L
run() {  # run ENV=VALUE bench-args...
  echo "== $*" >> $L
  local e=$1; shift
  env "$e" timeout -k 10 300 python -u bench.py --batch 1 --microbatches 1 --steps 3 --warmup 1 "$@" > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep -o '"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*' gpurun_out/_r.out | tr '\n' ' ' >> $L; echo >> $L
}
for r in 1 2; do
  run LSD_NOOP=1 --model gpt2-xl
  run LSD_ROUTING=gemv_nt=1 --model gpt2-xl
  run LSD_NOOP=1 --model llama-3-8b
  run LSD_ROUTING=gemv_nt=1 --model llama-3-8b
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r6prof_llama_d256" -o run --output-format csv -- \
  python3 "$R/bench.py" --model llama-3-8b --steps 1 --warmup 1 > "$R/gpurun_out/r6prof_llama_d256.log" 2>&1 || exit $?
rm -f "$R"/gpurun_out/r6prof_llama_d256/*kernel_trace.csv
