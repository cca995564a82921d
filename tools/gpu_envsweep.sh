#!/bin/bash
# bench.py under a list of env settings: SWEEP="A=1 B=2;A=3;..." ARGS="..."
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/envsweep.log; : > $L
IFS=';' read -ra CASES <<< "$SWEEP"
for c in "${CASES[@]}"; do
  echo "== $c" >> $L
  env $c timeout -k 10 300 python bench.py --steps 2 --warmup 1 $ARGS >> $L 2>&1 || exit 1
done
