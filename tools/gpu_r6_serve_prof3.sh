#!/bin/bash
# round 6: where closed-loop serving time goes with the join policy: host phases (LSD_HOST_PROFILE)
# and a rocprofv3 kernel trace of GPT-2 XL serving (512 in flight), last build (decode-first, partial native)
export HSA_ENABLE_IPC_MODE_LEGACY=0
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gpurun_out/r6_serve_prof3.log; : > $L
for m in ${SERVE_MODELS-gpt2-xl gpt2}; do
  echo "== $m" >> $L
  LSD_HOST_PROFILE=1 timeout -k 10 300 python -u tools/serve_load.py --model $m --requests 4096 > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep -v "^/opt" gpurun_out/_r.out >> $L
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/serve_prof -o serve -- python3 -u tools/serve_load.py --model gpt2-xl --requests 2048 --warm-requests 512 > gpurun_out/_p.out 2> gpurun_out/_p.err || { tail -20 gpurun_out/_p.err >> $L; exit 1; }
grep "^{" gpurun_out/_p.out >> $L
find gpurun_out/serve_prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/r6_serve_xl_kernel_stats_v2.csv \;
find gpurun_out/serve_prof -type f ! -name "*kernel_stats.csv" -delete
cat $L
