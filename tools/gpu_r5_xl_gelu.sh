#!/bin/bash
# round 5: GPT-2 XL decode MLP-up on hipBLASLt (GELU epilogue) from 384 rows -- bench A/B at 1024 sequences
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r5_xl_gelu.log; : > $L
for i in 1 2; do
  for m in 384 0; do
    echo "== xl --batch 1024 LSD_BLASLT_DECODE_GELU_MIN_M=$m (round $i)" >> $L
    LSD_BLASLT_DECODE_GELU_MIN_M=$m timeout -k 10 400 python -u bench.py --batch 1024 --steps 2 --warmup 1 >> $L 2>&1 || exit $?
  done
done
