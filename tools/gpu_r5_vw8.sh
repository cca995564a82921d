#!/bin/bash
# round 5: decode-step lane scheduling A/B (tools/lane_schedule_ab.py), headline bench A/B of the
# prefill bf16 residual slabs, 8-wave W-to-VGPR decode GEMM variants (A/B at 256 rows), an
# ordering probe of the W-to-VGPR residual-slab path, and last the lane attention ordering
# (external event nodes in the decode graphs)
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
LANE_MODES=free,free-eager,alt-eager,serial timeout -k 10 300 python -X faulthandler -u tools/lane_schedule_ab.py \
  > gpurun_out/r5_lane_schedule.log 2>&1 || exit $?
for s in 0 1 0 1; do
  echo "== LSD_PREFILL_SLAB=$s" >> gpurun_out/r5_order_slab_bench.log
  LSD_PREFILL_SLAB=$s timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 >> gpurun_out/r5_order_slab_bench.log 2>&1 || exit $?
done
export D256_BASE_R8=2 D256_SHAPES=xl_qkv,xl_fc,xl_proj,xl_proj2,l8_qkv,l8_o,l8_gu
export D256_VARIANTS=vw:664,vw:8464,vw:8484,vw:8443,vw:8864,vw:8884,vw:8464:2,vw:8464:3,vw:8464:4
timeout -k 10 400 python -u tools/bench_d256.py > gpurun_out/r5_vw8_ab.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/vw_race_probe.py 664 864 8464 > gpurun_out/r5_vw_probe.log 2>&1 || exit $?
echo "== LSD_LANE_ORDER=1" >> gpurun_out/r5_order_slab_bench.log
LSD_LANE_ORDER=1 timeout -k 10 300 python -X faulthandler -u bench.py --steps 2 --warmup 1 >> gpurun_out/r5_order_slab_bench.log 2>&1 || exit $?
# the captured form of the alternation last (an earlier build crashed hipStreamEndCapture)
LANE_MODES=free,alt timeout -k 10 300 python -X faulthandler -u tools/lane_schedule_ab.py >> gpurun_out/r5_lane_schedule.log 2>&1
