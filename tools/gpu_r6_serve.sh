#!/bin/bash
# round 6: closed-loop serving load (joins / leaves every step), native composition changes on vs off
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r6_serve_load.log; : > $L
for m in gpt2-xl gpt2; do
  for rep in 1 2; do
    for nc in 1 0; do
      echo "== $m LSD_NATIVE_CHANGES=$nc (round $rep)" >> $L
      LSD_NATIVE_CHANGES=$nc timeout -k 10 300 python -u tools/serve_load.py --model $m --concurrency 512 --requests 2048 >> $L 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
    done
  done
done
