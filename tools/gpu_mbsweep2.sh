#!/bin/bash
# headline microbatch-group / lane sweep on the current code (batch 512)
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/mbsweep2.log; : > $L
run() { echo "== $*" >> $L; env "$@" timeout -k 10 300 python bench.py --steps 3 --warmup 1 2>&1 | grep metric >> $L; }
run BENCH_MB=2 LSD_LANES=2 && run BENCH_MB=4 LSD_LANES=2 && run BENCH_MB=4 LSD_LANES=4 && \
run BENCH_MB=1 LSD_LANES=1 && run BENCH_MB=2 LSD_LANES=2
