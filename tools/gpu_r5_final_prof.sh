#!/bin/bash
# round 5, final build: rocprofv3 kernel statistics of the three 512-sequence configurations
# (one bench step + warmup each): GPT-2 XL headline, GPT-2 small, Llama-3 8B; the per-dispatch traces are
# dropped (over the 64 MiB copy-back limit), the statistics kept
export HSA_ENABLE_IPC_MODE_LEGACY=0
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/fprof_xl" -o run --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 1 > "$R/gpurun_out/fprof_xl.log" 2>&1 || exit $?
rm -f "$R"/gpurun_out/fprof_xl/*kernel_trace.csv
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/fprof_s" -o run --output-format csv -- python3 "$R/bench.py" --model gpt2 --steps 1 --warmup 1 > "$R/gpurun_out/fprof_s.log" 2>&1 || exit $?
rm -f "$R"/gpurun_out/fprof_s/*kernel_trace.csv
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/fprof_l8" -o run --output-format csv -- python3 "$R/bench.py" --model llama-3-8b --steps 1 --warmup 1 > "$R/gpurun_out/fprof_l8.log" 2>&1
rc=$?
rm -f "$R"/gpurun_out/fprof_l8/*kernel_trace.csv
exit $rc
