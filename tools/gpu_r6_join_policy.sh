#!/bin/bash
# round 6: continuous-serving join policy (EngineConfig.join_min / join_max_wait) under the closed-loop
# serving load (tools/serve_load.py, 512 in flight, prompts 16-128, outputs 16-128)
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
L=gpurun_out/r6_join_policy.log; : > $L
run() {
  echo "== $*" >> $L
  timeout -k 10 300 python -u tools/serve_load.py --requests 4096 "$@" > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep "^{" gpurun_out/_r.out >> $L
}
for m in gpt2-xl gpt2; do
  run --model $m --join-min 1
  run --model $m --join-min 16 --join-wait 4
  run --model $m --join-min 32 --join-wait 4
  run --model $m --join-min 64 --join-wait 8
  run --model $m --join-min 1
done
run --model llama-3-8b --join-min 1
run --model llama-3-8b --join-min 32 --join-wait 4
cat $L
