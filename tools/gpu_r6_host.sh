#!/bin/bash
# round 6: where a bench step's time goes outside prefill + decode steps (session_other_ms), host
# issue per decode step (LSD_HOST_PROFILE=1)
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r6_host.log; : > $L
for e in LSD_NOOP=1 LSD_HOST_PROFILE=1; do
  echo "== $e" >> $L
  env $e timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  cat gpurun_out/_r.out >> $L; grep "host per decode" gpurun_out/_r.err >> $L
done
