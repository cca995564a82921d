#!/bin/bash
# round 6: decode attention block shapes (tools/attn_blocks.py) + their kernel tests
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attention_decode" -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r6_pytest_attn.log 2>&1
rc=$?; echo "rc=$rc" >> gpurun_out/r6_pytest_attn.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/attn_blocks.py > gpurun_out/r6_attn_blocks.log 2>&1
