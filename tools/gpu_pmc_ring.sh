#!/bin/bash
# PMC passes over the 256-row decode GEMM on the ring kernel (tools/pmc_ring.py).
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
R="$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmcr1 gpurun_out/pmcr2 gpurun_out/pmcr3 gpurun_out/pmcr0
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/pmcr0" -o run --output-format csv -- python3 "$R/tools/pmc_ring.py" > "$R/gpurun_out/pmcr0.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVES SQ_WAVE_CYCLES -d "$R/gpurun_out/pmcr1" -o run --output-format csv -- python3 "$R/tools/pmc_ring.py" > "$R/gpurun_out/pmcr1.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE TA_BUSY_avr TCC_HIT_sum TCC_MISS_sum -d "$R/gpurun_out/pmcr2" -o run --output-format csv -- python3 "$R/tools/pmc_ring.py" > "$R/gpurun_out/pmcr2.log" 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_SALU SQ_INSTS_VALU -d "$R/gpurun_out/pmcr3" -o run --output-format csv -- python3 "$R/tools/pmc_ring.py" > "$R/gpurun_out/pmcr3.log" 2>&1 || exit 1
