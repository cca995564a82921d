#!/bin/bash
# Round 4: HBM-side bytes per kernel class of the headline decode step (GPT-2 XL, 2 x 256 rows),
# two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE: each alone fits the TCC counter budget), on a
# shortened session (--gen 16, no warmup) so the counter-serialised run stays short.
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_fetch" -o run -- python3 "$R/bench.py" --steps 1 --warmup 0 --gen 16 > "$R/gpurun_out/pmc_fetch.log" 2>&1 && \
timeout -s KILL 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/gpurun_out/pmc_write" -o run -- python3 "$R/bench.py" --steps 1 --warmup 0 --gen 16 > "$R/gpurun_out/pmc_write.log" 2>&1
