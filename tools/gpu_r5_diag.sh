#!/bin/bash
# round 5 diagnostic: production decode GEMM (8-wave ring) at 256 rows, cold (rotating) vs warm (one re-used) weights
set -o pipefail
export D256_SHAPES=xl_qkv,xl_fc,xl_proj,xl_proj2,l8_qkv D256_VARIANTS=r8:2 D256_BASE_R8=2
timeout -k 10 300 python -u tools/bench_d256.py > gpurun_out/r5_diag_cold.log 2>&1 &&
D256_WARM=1 timeout -k 10 300 python -u tools/bench_d256.py > gpurun_out/r5_diag_warm.log 2>&1
