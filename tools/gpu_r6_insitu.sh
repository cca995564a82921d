#!/bin/bash
export HSA_ENABLE_IPC_MODE_LEGACY=0
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/llama_insitu.py > gpurun_out/r6_llama_insitu.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r6prof_insitu" -o run --output-format csv -- \
  python3 "$R/tools/llama_insitu.py" >> "$R/gpurun_out/r6_llama_insitu.log" 2>&1 || exit $?
rm -f "$R"/gpurun_out/r6prof_insitu/*kernel_trace.csv
