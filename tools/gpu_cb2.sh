#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/bench_cb2.log; : > $L
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_engine_gpu.py >> $L 2>&1 || exit 1
echo "== single (host profile)" >> $L
LSD_HOST_PROFILE=1 timeout -k 10 200 python bench.py --batch 1 --microbatches 1 --steps 3 --warmup 1 >> $L 2>&1 || exit 1
echo "== single no timing events" >> $L
echo "== loopback P=8 (total 512)" >> $L
timeout -k 10 300 python bench.py --loopback-stages 8 --batch 512 --steps 2 --warmup 1 >> $L 2>&1 || exit 1
mkdir -p gpurun_out/prof_ss2; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_ss2" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --batch 1 --microbatches 1 --steps 1 --warmup 1 --gen 32 > "$GRAFT_REPO_ROOT/gpurun_out/prof_ss2.log" 2>&1
