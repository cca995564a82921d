#!/bin/bash
# rocprofv3 kernel stats (1 timed step) for GPT-2 small and Llama-3 8B at 512 sequences.
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_small gpurun_out/prof_llama
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_small" -o run --output-format csv -- python3 "$R/bench.py" --model gpt2 --steps 1 --warmup 1 > "$R/gpurun_out/prof_small.log" 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_llama" -o run --output-format csv -- python3 "$R/bench.py" --model llama-3-8b --steps 1 --warmup 1 > "$R/gpurun_out/prof_llama.log" 2>&1
rc=$?
rm -f "$R"/gpurun_out/prof_*/run_kernel_trace.csv
exit $rc
