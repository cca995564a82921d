#!/bin/bash
# round 6: (1) Llama-3 8B 512-row decode GEMM tilings (tools/llama512_gemm.py);
# (2) multi-stage rehearsals on ONE MI355X with merged prefill off on both sides:
#     GPT-2 small P=2 (BASELINE config 2) and GPT-2 XL P=8 as stage threads on the device-loopback
#     data plane (graph-captured edges + native executor: the rccl path's twin) and on the event
#     hand-off (the torch-nccl fallback's twin), and GPT-2 small P=2 as two rank PROCESSES with
#     default flags (auto transport -> devloop on a shared GPU);
# (3) GPT-2 small microbatch lanes.
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/llama512_gemm.py > gpurun_out/r6_llama512_gemm.log 2>&1 || exit $?
L=gpurun_out/r6_rehearsal.log; : > $L
run() {
  echo "== $*" >> $L
  env "$@" > gpurun_out/_r.out 2> gpurun_out/_r.err || { tail -20 gpurun_out/_r.err >> $L; exit 1; }
  grep "^{" gpurun_out/_r.out | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    print(d['value'], d['p50_token_latency_ms'], d['prefill_ms'], d.get('transport'), d.get('transport_fallback'),
          d.get('pipeline_matches_1gpu'), d['config']['parallelism'], d.get('stage_busy'))" >> $L
}
B="timeout -k 10 400 python -u bench.py --steps 3 --warmup 1"
for r in 1 2; do
  run LSD_MERGE_PREFILL=0 $B --model gpt2
  run LSD_MERGE_PREFILL=0 $B --model gpt2 --loopback-stages 2
  run LSD_MERGE_PREFILL=0 $B --model gpt2 --loopback-stages 2 --loopback-transport loopback
done
run LSD_MERGE_PREFILL=0 timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --model gpt2 --batch 256 --steps 3 --warmup 1
for r in 1 2; do
  run LSD_MERGE_PREFILL=0 $B
  run LSD_MERGE_PREFILL=0 $B --loopback-stages 8
  run LSD_MERGE_PREFILL=0 $B --loopback-stages 8 --loopback-transport loopback
done
run LSD_LANES=3 $B --model gpt2 --microbatches 3
run LSD_LANES=4 $B --model gpt2 --microbatches 4
run LSD_NOOP=1 $B --model gpt2
