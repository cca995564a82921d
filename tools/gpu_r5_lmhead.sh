#!/bin/bash
# round 5: decode vocabulary projection (fp32 logits) kernel routing A/B at 256 / 128 rows,
# then the headline kernel statistics (v9) with rocprofv3
export HSA_ENABLE_IPC_MODE_LEGACY=0
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
L="$R/gpurun_out/r5_lmhead_routing.log"
D256_M=256,128 D256_SHAPES=xl_lm,s_lm,l8_lm D256_VARIANTS=knob:big,knob:nop8,knob:r8,64:1,128:1,128:2,64:2 \
  timeout -k 10 400 python -u "$R/tools/bench_d256.py" > "$L" 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/hprof9" -o run --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 1 > "$R/gpurun_out/hprof9.log" 2>&1
