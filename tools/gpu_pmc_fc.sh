#!/bin/bash
# PMC passes over the 256-row MLP-up GEMM variants (tools/microbench.py fc256)
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/pmc
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/kt -o kt -- python3 tools/microbench.py fc256 > gpurun_out/pmc/kt.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_ANY --output-format csv -d gpurun_out/pmc/p1 -o p1 -- python3 tools/microbench.py fc256 > gpurun_out/pmc/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc/p2 -o p2 -- python3 tools/microbench.py fc256 > gpurun_out/pmc/p2.log 2>&1 || exit $?
