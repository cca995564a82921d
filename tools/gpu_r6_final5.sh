#!/bin/bash
# round 6 (re-entry, last build + partial native issue): GPU suite + smoke, headline, serving load
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
S=gpurun_out/r6_final5_suite.log; : > $S
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/ >> $S 2>&1 || { tail -40 $S; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" >> $S 2>&1 || { tail -20 $S; exit 1; }
tail -3 $S
L=gpurun_out/r6_final5_bench.log; : > $L
for i in 1 2; do
  echo "== headline" >> $L
  timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep "^{" gpurun_out/_r.out >> $L
done
for m in gpt2-xl gpt2 llama-3-8b; do
  echo "== serve_load $m" >> $L
  timeout -k 10 400 python -u tools/serve_load.py --model $m --requests 4096 --warm-requests 1024 > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep "^{" gpurun_out/_r.out >> $L
done
grep -o '^== .*\|"value": [0-9.]*\|"p50_token_latency_ms": [0-9.]*\|"prefill_ms": [0-9.]*\|"tok_s": [0-9.]*\|"ttft_ms_p50": [0-9.]*' $L | paste -sd' ' | sed 's/ == /\n== /g'
