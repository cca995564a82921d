#!/bin/bash
# round 6 (re-entry, final build): GPU suite + smoke, the README bench configurations, the serving load
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
S=gpurun_out/r6_final2_suite.log; : > $S
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/ >> $S 2>&1 || { tail -40 $S; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" >> $S 2>&1 || { tail -20 $S; exit 1; }
tail -3 $S
L=gpurun_out/r6_final2_bench_configs.log; : > $L
run() {
  echo "== $*" >> $L
  timeout -k 10 400 python -u bench.py "$@" > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep "^{" gpurun_out/_r.out >> $L
}
run --steps 5 --warmup 2
run --steps 3 --warmup 1 --greedy
run --batch 1 --microbatches 1 --steps 2 --warmup 1
run --model gpt2 --steps 5 --warmup 2
run --model gpt2 --batch 1 --microbatches 1 --steps 2 --warmup 1
run --model llama-3-8b --steps 2 --warmup 1
run --model llama-3-8b --batch 1 --microbatches 1 --steps 2 --warmup 1
run --steps 5 --warmup 2
for m in gpt2-xl gpt2 llama-3-8b; do
  echo "== serve_load $m" >> $L
  timeout -k 10 300 python -u tools/serve_load.py --model $m --requests 4096 > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep "^{" gpurun_out/_r.out >> $L
done
grep -o '^== .*\|"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*\|"prefill_ms": [0-9.]*\|"tok_s": [0-9.]*\|"ttft_ms_p50": [0-9.]*' $L | paste -sd' ' | sed 's/ == /\n== /g'
