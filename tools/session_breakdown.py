#!/usr/bin/env python3
"""Where a headline bench step (one generation session) spends its wall time:
session wall vs stage 0's event-timed prefill + decode steps, per session.
Same config as bench.py's default (GPT-2 XL, 512 x (128 + 128), 2 lanes)."""
import random
import statistics
import sys
import time

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
import torch  # noqa: E402

from llm_sharding_demo_amd.config import EngineConfig, SamplingParams  # noqa: E402
from llm_sharding_demo_amd.runtime.engine import Engine  # noqa: E402

B, PROMPT, GEN = 512, 128, 128
cfg = EngineConfig(model_id="gpt2-xl", num_stages=1, max_batch=B, prefill_chunk=0,
                   max_seq_len=PROMPT + GEN, device="cuda", num_microbatches=2, seed=0)
eng = Engine(cfg)
rnd = random.Random(0)
V = cfg.model.vocab_size
prompts = [[rnd.randrange(V) for _ in range(PROMPT)] for _ in range(B)]
sp = SamplingParams(greedy=False, temperature=0.6, top_k=40, max_new_tokens=GEN, seed=1234)
for i in range(4):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.generate_ids(prompts, [sp] * B, record_timing=True)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    ls = eng.last_session
    st = ls.step_times_ms
    print(f"session {i}: wall {wall:8.1f} ms | prefill {ls.prefill_ms:6.1f} | {len(st)} steps sum {sum(st):7.1f} "
          f"mean {statistics.mean(st):.3f} p50 {statistics.median(st):.3f} max {max(st):.2f} | "
          f"unaccounted {wall - ls.prefill_ms - sum(st):6.1f} ms | first 3 steps {[round(x, 2) for x in st[:3]]} "
          f"last 3 {[round(x, 2) for x in st[-3:]]}", flush=True)
