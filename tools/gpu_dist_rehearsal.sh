#!/bin/bash
# bench.py under torch.distributed.run on ONE GPU: 2 ranks sharing the card over the gloo transport
# (host-staged hops) -- a rehearsal of the driver's multi-GPU command path, not a throughput number.
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/dist_rehearsal.log; : > $L
echo "== 2 ranks, --batch 128" >> $L
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --batch 128 --transport gloo >> $L 2>&1
