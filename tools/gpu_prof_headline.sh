#!/bin/bash
# Headline bench + rocprofv3 kernel stats (1 timed step).
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/prof_hl
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_hl" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 1 ${BENCH_ARGS} > "$GRAFT_REPO_ROOT/gpurun_out/prof_hl.log" 2>&1
echo "prof rc=$?" >> "$GRAFT_REPO_ROOT/gpurun_out/prof_hl.log"
