#!/bin/bash
# round 5: PMC passes over the 256-row decode GEMM variants (tools/pmc_decode_gemm.py):
# the 8-wave LDS ring (production) vs the W-to-VGPR kernel at 96 / 128-row tiles
export HSA_ENABLE_IPC_MODE_LEGACY=0
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/pmc5"
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_WAIT_INST_LDS"
P2="SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE"
P3="TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TA_BUSY_avr TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TC_STALL_sum TD_TD_BUSY_sum"
P4="TCC_HIT_sum TCC_MISS_sum GRBM_COUNT"
for c in ring8 vw664 vw864; do
  i=0
  for P in "$P1" "$P2" "$P3" "$P4"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P -d "$R/gpurun_out/pmc5/$c-$i" -o run --output-format csv \
      -- python3 "$R/tools/pmc_decode_gemm.py" $c > "$R/gpurun_out/pmc5/$c-$i.log" 2>&1 || exit 1
  done
done
