#!/bin/bash
# A/B of runtime env knobs: for each entry of VARIANTS (';'-separated env
# assignments, "default" = none) run bench.py $BENCH_ARGS; one block per
# variant in gpurun_out/ab_env.log.  No rebuild (knobs are read at import).
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
: > gpurun_out/ab_env.log
IFS=';' read -ra VS <<< "${VARIANTS:-default}"
for v in "${VS[@]}"; do
  echo "== $v" >> gpurun_out/ab_env.log
  if [ "$v" = default ]; then
    timeout -k 10 300 python bench.py $BENCH_ARGS >> gpurun_out/ab_env.log 2>&1 || exit $?
  else
    timeout -k 10 300 env $v python bench.py $BENCH_ARGS >> gpurun_out/ab_env.log 2>&1 || exit $?
  fi
done
