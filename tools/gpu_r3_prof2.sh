#!/bin/bash
# (1) p8 loop anatomy (LSD_P8_PROF build of _C.so, built beforehand on the CPU side);
# (2) kernel trace of a short bench run (prefill + 32 decode steps): per-kernel solo times.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 240 python -u tools/microbench.py p8prof > gpurun_out/p8prof2.log 2>&1 || exit $?
grep stamps gpurun_out/p8prof2.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/dprof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --gen 32 --steps 1 --warmup 1 > "$GRAFT_REPO_ROOT/gpurun_out/dprof.log" 2>&1
