#!/bin/bash
# round 5: GPT-2 small 512-sequence kernel statistics (rocprofv3, one bench step + warmup)
export HSA_ENABLE_IPC_MODE_LEGACY=0
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/sprof" -o run --output-format csv -- python3 "$R/bench.py" --model gpt2 --steps 1 --warmup 1 > "$R/gpurun_out/sprof.log" 2>&1
