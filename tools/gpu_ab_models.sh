#!/bin/bash
# Runtime-knob A/B across bench configs: for each config in CONFIGS (';'-separated
# bench args) run every VARIANTS entry; all blocks appended to gpurun_out/ab_models.log
cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out
: > gpurun_out/ab_models.log
IFS=';' read -ra CS <<< "$CONFIGS"
for c in "${CS[@]}"; do
  echo "#### $c" >> gpurun_out/ab_models.log
  VARIANTS="$VARIANTS" BENCH_ARGS="$c" bash tools/gpu_ab_env.sh || exit $?
  cat gpurun_out/ab_env.log >> gpurun_out/ab_models.log
done
