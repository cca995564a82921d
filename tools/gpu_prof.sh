#!/bin/bash
# Flagship bench + rocprofv3 kernel trace (per-kernel time summary).
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/prof
ARGS=${BENCH_ARGS:-"--model gpt2-xl --batch 64 --prompt 128 --gen 128 --steps 2 --warmup 1"}
timeout -k 10 300 python -m pytest tests/test_engine_gpu.py -q -p no:cacheprovider -k pipeline > gpurun_out/pytest_pipe.log 2>&1
echo "rc=$?" >> gpurun_out/pytest_pipe.log
timeout -k 10 400 python bench.py $ARGS > gpurun_out/bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" $ARGS --steps 1 --warmup 0 > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
echo "prof rc=$?" >> "$GRAFT_REPO_ROOT/gpurun_out/prof.log"
