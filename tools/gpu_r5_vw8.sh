#!/bin/bash
# round 5: 8-wave W-to-VGPR decode GEMM variants (numerics + A/B at 256 rows) and the
# decode-step lane scheduling A/B (tools/lane_schedule_ab.py)
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "vw" -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r5_vw8_tests.log 2>&1 || exit $?
export D256_BASE_R8=2 D256_SHAPES=xl_qkv,xl_fc,xl_proj,xl_proj2,l8_qkv,l8_o,l8_gu
export D256_VARIANTS=vw:664,vw:8464,vw:8484,vw:8443,vw:8864,vw:8884,vw:8464:2,vw:8464:3,vw:8464:4
timeout -k 10 400 python -u tools/bench_d256.py > gpurun_out/r5_vw8_ab.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/lane_schedule_ab.py > gpurun_out/r5_lane_schedule.log 2>&1
