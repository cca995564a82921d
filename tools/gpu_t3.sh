cd "$GRAFT_REPO_ROOT"; export HSA_ENABLE_IPC_MODE_LEGACY=0; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "tiled3 or big_gemm or two_row or decode_gemm" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t3_test.log 2>&1 || exit $?
timeout -k 10 300 env LSD_TILED_MIN_N=6400 python -u tools/microbench.py tiled3 > gpurun_out/t3_micro.log 2>&1 || exit $?
VARIANTS="default;LSD_TILED3_MAX=512;LSD_TILED3_MAX=512 LSD_TILED_MIN_N=4800" BENCH_ARGS="--steps 2 --warmup 1" bash tools/gpu_ab_env.sh
