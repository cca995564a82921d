cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k norm -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_norm.log 2>&1 || exit $?
timeout -k 10 300 python tools/microbench.py norm layer > gpurun_out/micro_norm.log 2>&1 || exit $?
for b in 256 384 512; do
 BENCH_BATCH=$b timeout -k 10 300 python bench.py --steps 2 --warmup 1 >> gpurun_out/bench_batch.log 2>&1 || exit $?
done
