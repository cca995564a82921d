#!/bin/bash
# Kernel trace + PMC passes over the prefill GEMM (gemm_p8_kernel) and hipBLASLt on the
# same shapes (tools/pmc_p8.py): MFMA busy, wave states, LDS, L2 hit rate, TA/TD stalls.
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/pmcp8"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- python3 "$R/tools/pmc_p8.py" > "$O/trace.log" 2>&1 || exit 1
P() {  # pass name, counters...
  local n=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -d "$O/$n" -o run --output-format csv -- python3 "$R/tools/pmc_p8.py" > "$O/$n.log" 2>&1
}
P p1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT || exit 1
P p2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_LDS_DATA_FIFO_FULL TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_DATA_STALLED_BY_TC_CYCLES_sum || exit 1
P p3 TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TD_TC_STALL_sum TD_TD_BUSY_sum SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU || exit 1
echo pmc-done
