#!/bin/bash
# A/B of compile-time flags: for each entry of FLAGS (';'-separated, "default"
# = none) rebuild the extension with LSD_HIPCC_FLAGS, run the microbench
# cases in MB_ARGS (optional) and bench.py; one block per variant in ab.log.
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
: > gpurun_out/ab.log
IFS=';' read -ra VARIANTS <<< "${FLAGS:-default}"
for f in "${VARIANTS[@]}"; do
  if [ "$f" = default ]; then unset LSD_HIPCC_FLAGS; else export LSD_HIPCC_FLAGS="$f"; fi
  echo "== $f" >> gpurun_out/ab.log
  python -c "from llm_sharding_demo_amd.ops import build; build.build()" > gpurun_out/ab_build.log 2>&1 || exit 1
  if [ -n "$MB_ARGS" ]; then timeout -k 10 300 python tools/microbench.py $MB_ARGS >> gpurun_out/ab.log 2>&1 || exit $?; fi
  timeout -k 10 300 python bench.py $BENCH_ARGS >> gpurun_out/ab.log 2>&1 || exit $?
done
