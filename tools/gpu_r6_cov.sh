#!/bin/bash
# round 6: kernel-trace occupancy of the headline bench's last session (GPU idle between kernels)
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
L=$R/gpurun_out/r6_coverage.log; : > $L
cd /tmp && export TMPDIR=/tmp
for m in gpt2-xl gpt2; do
  rm -rf $R/gpurun_out/cov_$m
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/cov_$m -o run -- python3 $R/bench.py --model $m --steps 1 --warmup 1 > $R/gpurun_out/_c.out 2>&1 || { tail -20 $R/gpurun_out/_c.out >> $L; exit 1; }
  f=$(find $R/gpurun_out/cov_$m -name "*kernel_trace.csv" | head -1)
  echo "== $m $(grep '^{' $R/gpurun_out/_c.out | grep -o '"value": [0-9.]*')" >> $L
  python3 $R/tools/kernel_coverage.py $f >> $L
  rm -rf $R/gpurun_out/cov_$m
done
