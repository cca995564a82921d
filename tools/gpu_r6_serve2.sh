#!/bin/bash
# round 6: closed-loop serving load with the host profile (where serving loses to the session bench)
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r6_serve_prof.log; : > $L
for m in gpt2-xl gpt2; do
  echo "== $m" >> $L
  LSD_HOST_PROFILE=1 timeout -k 10 300 python -u tools/serve_load.py --model $m --concurrency 512 --requests 4096 >> $L 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
done
