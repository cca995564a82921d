#!/bin/bash
# Round 4 bundle (two gpurun calls: `tests` then `rehearsal`): devloop tests (threads + processes on one GPU), race checker,
# headline bench, and the multi-stage rehearsals on the rccl code path (tools/gpu_r4_rehearsal.sh
# subset + a torchrun 8-process run on the one GPU).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { echo "== $(date +%T) $*"; }
PHASE=${1:-tests}
if [ "$PHASE" = tests ] || [ "$PHASE" = both ]; then
step tests
timeout -k 10 700 python -u -m pytest tests/test_devloop_gpu.py tests/test_racecheck.py tests/test_multigpu.py -m gpu -v -x --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_devloop_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/r4_devloop_tests.log | tail -40; [ $rc -eq 0 ] || exit $rc
step bench
timeout -k 10 400 python bench.py --steps 5 --warmup 2 > gpurun_out/r4_bench1.log 2>&1 || exit $?
grep "^{" gpurun_out/r4_bench1.log
[ "$PHASE" = both ] || exit 0
fi
export LSD_HOST_PROFILE=1
L=gpurun_out/r4_rehearsal.log; : > $L
run() { local lab=$1; shift; echo "== $lab" >> $L; step "$lab"
  timeout -k 10 400 "$@" > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -30 gpurun_out/_r.err >> $L; return 1; }
  grep "^{" gpurun_out/_r.out >> $L; grep "host per" gpurun_out/_r.err >> $L; tail -2 $L; }
C="--prompt 64 --gen 64 --steps 2 --warmup 1"
run "gpt2 P=1 M=16x256" python bench.py --model gpt2 --batch 4096 --microbatches 16 $C && \
run "gpt2 P=8 M=16x256 devloop threads" python bench.py --model gpt2 --batch 4096 --microbatches 16 --loopback-stages 8 $C && \
run "gpt2 P=8 M=16x256 loopback threads" python bench.py --model gpt2 --batch 4096 --microbatches 16 --loopback-stages 8 --loopback-transport loopback $C && \
run "gpt2 P=8 M=16x256 devloop 8 processes" python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --transport devloop --model gpt2 --batch 512 --microbatches 16 $C && \
run "xl P=1 M=16x256" python bench.py --model gpt2-xl --batch 4096 --microbatches 16 $C && \
run "xl P=8 M=16x256 devloop threads" python bench.py --model gpt2-xl --batch 4096 --microbatches 16 --loopback-stages 8 $C && \
run "xl P=8 M=16x256 devloop 8 processes" python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 8 --transport devloop --model gpt2-xl --batch 512 --microbatches 16 $C
rc=$?
step done
exit $rc
