#!/bin/bash
# A/B of decode-GEMM round length: default build vs -DLSD_SK_ROUND=$R (microbench gemm M=64/128)
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
for R in ${ROUNDS:-default 8}; do
  if [ "$R" = default ]; then unset LSD_HIPCC_FLAGS; else export LSD_HIPCC_FLAGS="-DLSD_SK_ROUND=$R"; fi
  python -c "from llm_sharding_demo_amd.ops import build; build.build()" > gpurun_out/ab_build_$R.log 2>&1 || exit 1
  echo "== round $R" >> gpurun_out/ab.log
  timeout -k 10 300 python tools/microbench.py ${MB_ARGS:-gemm} >> gpurun_out/ab.log 2>&1 || exit $?
  if [ -n "$BENCH" ]; then timeout -k 10 300 python bench.py --steps 2 --warmup 1 >> gpurun_out/ab.log 2>&1 || exit $?; fi
done
