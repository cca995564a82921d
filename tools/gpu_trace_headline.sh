#!/bin/bash
# Kernel trace of the headline config (1 timed step) for timeline analysis.
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/trace
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/trace" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 1 ${BENCH_ARGS} > "$GRAFT_REPO_ROOT/gpurun_out/trace.log" 2>&1
echo "prof rc=$?" >> "$GRAFT_REPO_ROOT/gpurun_out/trace.log"
cd "$GRAFT_REPO_ROOT" && python tools/timeline.py gpurun_out/trace/run_kernel_trace.csv 0.6 2.0 80 > gpurun_out/trace_timeline.txt 2>&1
