#!/bin/bash
# Pipeline machinery on one GPU: P stage threads (loopback transport) vs one
# stage, SAME microbatch shapes (M groups x R rows), so the ratio isolates the
# schedule + transport + host issue cost.
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/loopback.log; : > $L
A="--prompt 64 --gen 64 --steps 2 --warmup 1"
echo "== P=1 M=16 x 256" >> $L
LSD_HOST_PROFILE=1 timeout -k 10 300 python bench.py --batch 4096 --microbatches 16 $A >> $L 2>&1 || exit 1
echo "== P=8 loopback M=16 x 256" >> $L
LSD_HOST_PROFILE=1 timeout -k 10 300 python bench.py --loopback-stages 8 --batch 4096 --microbatches 16 $A >> $L 2>&1 || exit 1
echo "== P=1 M=8 x 256" >> $L
LSD_HOST_PROFILE=1 timeout -k 10 300 python bench.py --batch 2048 --microbatches 8 $A >> $L 2>&1 || exit 1
echo "== P=4 loopback M=8 x 256" >> $L
LSD_HOST_PROFILE=1 timeout -k 10 300 python bench.py --loopback-stages 4 --batch 2048 --microbatches 8 $A >> $L 2>&1 || exit 1
