#!/bin/bash
# round 6 (re-entry): GPU suite + smoke + headline bench on the current HEAD
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
S=gpurun_out/r6_verify_suite.log; : > $S
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/ >> $S 2>&1 || { tail -40 $S; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" >> $S 2>&1 || { tail -20 $S; exit 1; }
tail -4 $S
L=gpurun_out/r6_verify_bench.log; : > $L
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep "^{" gpurun_out/_r.out >> $L
done
cat $L
