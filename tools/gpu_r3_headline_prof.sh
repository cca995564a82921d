#!/bin/bash
# Headline kernel statistics on the current code: rocprofv3 kernel trace of one bench step
# (GPT-2 XL, 512 sequences, prefill + 127 decode steps; traced lanes serialise: solo times).
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/hprof" -o run --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 1 > "$R/gpurun_out/hprof.log" 2>&1
