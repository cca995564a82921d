#!/usr/bin/env python3
"""Host-side cost of hipGraph replays in the decode loop, and whether the
microbatch lanes overlap on the device (without a profiler attached).

Runs bench-shaped rounds (GPT-2 XL by default) with CUDAGraph.replay wrapped:
host time per replay plus device start/end events around every replay on its
lane stream.  Prints host ms per replay, device ms per replay, and the lane
overlap (sum of replay device spans / union).
usage: python tools/probe_replay.py [batch] [mbs]
"""
from __future__ import annotations

import os
import random
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_demo_amd.config import EngineConfig, SamplingParams  # noqa: E402
from llm_sharding_demo_amd.runtime.engine import Engine  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    M = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    model = os.environ.get("PROBE_MODEL", "gpt2-xl")
    gen = int(os.environ.get("PROBE_GEN", "32"))
    cfg = EngineConfig(model_id=model, num_stages=1, max_batch=B, max_seq_len=128 + gen,
                       device="cuda", num_microbatches=M)
    eng = Engine(cfg)
    rnd = random.Random(0)
    prompts = [[rnd.randrange(cfg.model.vocab_size) for _ in range(128)] for _ in range(B)]
    sp = SamplingParams(temperature=0.6, top_k=40, max_new_tokens=gen, seed=1)
    spec = eng.make_round(prompts, [sp] * B, list(range(B)), microbatches=M, record_timing=True)
    w = eng.workers[0]
    w.run_round(spec)  # warmup + capture
    torch.cuda.synchronize()

    host, evs = [], []
    orig = torch.cuda.CUDAGraph.replay

    def timed(self):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        t = time.perf_counter()
        orig(self)
        host.append(time.perf_counter() - t)
        b.record()
        evs.append((a, b))

    torch.cuda.CUDAGraph.replay = timed
    t0 = time.perf_counter()
    res = w.run_round(spec)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    torch.cuda.CUDAGraph.replay = orig
    r = sorted(host)
    ref = evs[0][0]
    iv = sorted((ref.elapsed_time(a), ref.elapsed_time(b)) for a, b in evs)
    dev = sorted(b - a for a, b in iv)
    union, cur = 0.0, None
    for a, b in iv:
        if cur is None or a > cur[1]:
            if cur:
                union += cur[1] - cur[0]
            cur = [a, b]
        else:
            cur[1] = max(cur[1], b)
    union += cur[1] - cur[0]
    print(f"model {model} B={B} M={M} gen={gen}: wall {wall * 1e3:.1f} ms, replays {len(r)}", flush=True)
    print(f"  host per replay p50 {r[len(r) // 2] * 1e3:.3f} ms max {r[-1] * 1e3:.3f} ms "
          f"sum {sum(r) * 1e3:.1f} ms", flush=True)
    print(f"  device per replay p50 {dev[len(dev) // 2]:.3f} ms; lane overlap "
          f"{sum(dev) / max(union, 1e-9):.2f} (sum {sum(dev):.1f} / union {union:.1f} ms)", flush=True)
    st = sorted(res.step_times_ms)
    print(f"  device step p50 {st[len(st) // 2]:.3f} ms, prefill {res.prefill_ms:.1f} ms", flush=True)


if __name__ == "__main__":
    main()
