#!/bin/bash
# bench + rocprofv3 kernel-trace summary for the bench config in BENCH_ARGS
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/prof
timeout -k 10 400 python bench.py $BENCH_ARGS > gpurun_out/bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" $BENCH_ARGS --steps 1 --warmup 0 > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
echo "prof rc=$?" >> "$GRAFT_REPO_ROOT/gpurun_out/prof.log"
