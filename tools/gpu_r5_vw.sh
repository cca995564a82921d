#!/bin/bash
# round 5: W-to-VGPR decode GEMM (gemm_vw_kernel, launch kind 4) -- numerics, A/B vs the
# production 8-wave ring at 256 rows, then the whole GPU suite and the default bench
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "vw" -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r5_vw_tests.log 2>&1 || exit $?
export D256_BASE_R8=2 D256_SHAPES=xl_qkv,xl_fc,xl_proj,xl_proj2,l8_qkv,l8_o,l8_gu,l8_down,s_qkv,s_fc,s_proj2
export D256_VARIANTS=vw:864,vw:884,vw:843,vw:886,vw:664,vw:684,vw:464,vw:864:2,vw:864:3,vw:864:4,vw:864:6,vw:664:2,vw:664:3,vw:664:4,vw:464:2
timeout -k 10 400 python -u tools/bench_d256.py > gpurun_out/r5_vw_ab.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r5_pytest_gpu.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/r5_pytest_gpu.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 600 python -u bench.py > gpurun_out/r5_bench.log 2>&1
