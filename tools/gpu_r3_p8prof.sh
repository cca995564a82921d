#!/bin/bash
# p8 loop anatomy (LSD_P8_PROF diagnostic build of _C.so, built on the CPU side beforehand):
# per-workgroup phase stamps plus wave 0's loop cycles in the vmcnt waits and the two barriers.
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 240 python -u tools/microbench.py p8prof > gpurun_out/p8prof.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/p8prof.log; exit $rc
