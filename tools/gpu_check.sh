#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
python -c "import torch; print(torch.cuda.get_device_name(0))" > gpurun_out/dev.txt 2>&1
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --model gpt2 --batch 16 --prompt 32 --gen 32 --steps 2 --warmup 1 > gpurun_out/bench_small.log 2>&1
rc=$?
echo "bench rc=$rc" >> gpurun_out/bench_small.log
exit $rc
