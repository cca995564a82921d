#!/bin/bash
# round 6: hand-written kernels only (hipBLASLt off by default, ops/routing.py) + the default N>1
# data plane: the whole GPU suite, bench on the three 512-sequence configurations (default routing
# and the blaslt=1 oracle on the headline), rocprofv3 kernel statistics of the default routing
export HSA_ENABLE_IPC_MODE_LEGACY=0
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
timeout -k 10 600 python -u -m pytest tests -m gpu -v -s --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r6_pytest_gpu.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/r6_pytest_gpu.log
case $rc in 124|134|137|139) exit $rc;; esac
L=gpurun_out/r6_route_bench.log; : > $L
run() {
  echo "== $*" >> $L
  env "$@" timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep "^{" gpurun_out/_r.out >> $L
}
mb() {  # model bench: args after the env
  local m=$1; shift
  echo "== $m $*" >> $L
  timeout -k 10 400 python -u bench.py --model $m --steps 2 --warmup 1 "$@" > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep "^{" gpurun_out/_r.out >> $L
}
run LSD_NOOP=1
run LSD_ROUTING=blaslt=1
run LSD_NOOP=1
mb gpt2
mb llama-3-8b
LSD_ROUTING=blaslt=1 mb llama-3-8b
cd /tmp && export TMPDIR=/tmp
for m in gpt2-xl gpt2 llama-3-8b; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r6prof_$m" -o run --output-format csv -- \
    python3 "$R/bench.py" --model $m --steps 1 --warmup 1 > "$R/gpurun_out/r6prof_$m.log" 2>&1 || exit $?
  rm -f "$R"/gpurun_out/r6prof_$m/*kernel_trace.csv
done
