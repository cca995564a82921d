#!/bin/bash
# round 6: full GPU suite + smoke
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r6_suite2.log; : > $L
timeout -k 10 1000 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests/ >> $L 2>&1 || { tail -40 $L; exit 1; }
tail -3 $L
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" >> $L 2>&1 && tail -3 $L
