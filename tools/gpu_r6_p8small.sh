#!/bin/bash
# round 6: GPT-2 small 8-stage rehearsal, full bench lines (session_other_ms, max step) and host profile
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r6_p8small_detail.log; : > $L
C="--model gpt2 --batch 4096 --microbatches 16 --prompt 64 --gen 64 --steps 2 --warmup 1"
for a in "" "--loopback-stages 8"; do
  echo "== $a" >> $L
  LSD_MERGE_PREFILL=0 LSD_HOST_PROFILE=1 timeout -k 10 400 python -u bench.py $C $a > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  cat gpurun_out/_r.out >> $L; grep "host per decode" gpurun_out/_r.err >> $L
done
