#!/bin/bash
# Single-stream (batch 1) bench + rocprofv3 kernel stats; model via SS_MODEL.
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
M=${SS_MODEL:-gpt2-xl}
mkdir -p gpurun_out/prof_ss
timeout -k 10 300 python bench.py --model $M --batch 1 --microbatches 1 --steps 2 --warmup 1 > gpurun_out/ss_bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_ss" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --model $M --batch 1 --microbatches 1 --steps 1 --warmup 1 --gen 32 > "$GRAFT_REPO_ROOT/gpurun_out/prof_ss.log" 2>&1
echo "prof rc=$?" >> "$GRAFT_REPO_ROOT/gpurun_out/prof_ss.log"
