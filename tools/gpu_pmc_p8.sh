#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc1 gpurun_out/pmc2
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVES SQ_WAVE_CYCLES -d "$R/gpurun_out/pmc1" -o run --output-format csv -- python3 "$R/tools/pmc_bigemm.py" > "$R/gpurun_out/pmc1.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE TA_BUSY_avr TCC_HIT_sum TCC_MISS_sum -d "$R/gpurun_out/pmc2" -o run --output-format csv -- python3 "$R/tools/pmc_bigemm.py" > "$R/gpurun_out/pmc2.log" 2>&1 || exit 1
