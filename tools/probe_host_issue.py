#!/usr/bin/env python3
"""Where stage 0's host time per pipeline item goes (cProfile of one timed
generation session on the driver thread, local mode, one GPU).

usage: python tools/probe_host_issue.py [model] [sequences] [microbatches]
Prints the top functions by own time and by cumulative time, and the
driver-thread CPU seconds per decode item."""
from __future__ import annotations

import cProfile
import os
import pstats
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from llm_sharding_demo_amd import EngineConfig  # noqa: E402
from llm_sharding_demo_amd.runtime.engine import Engine  # noqa: E402
from llm_sharding_demo_amd.runtime.scheduler import SamplingParams  # noqa: E402


def main():
    model = sys.argv[1] if len(sys.argv) > 1 else "gpt2"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    M = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    prompt, gen = 64, 64
    cfg = EngineConfig(model_id=model, num_stages=1, max_batch=B, max_seq_len=prompt + gen,
                       device="cuda", use_graphs=True, num_microbatches=M, seed=0)
    eng = Engine(cfg, mode="local")
    rnd = random.Random(0)
    V = cfg.model.vocab_size
    prompts = [[rnd.randrange(V) for _ in range(prompt)] for _ in range(B)]
    sp = SamplingParams(greedy=False, temperature=0.6, top_k=40, max_new_tokens=gen, seed=1234)
    eng.generate_ids(prompts, [sp] * B)  # warm: graphs captured
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    c0, t0 = time.thread_time(), time.perf_counter()
    pr.enable()
    eng.generate_ids(prompts, [sp] * B)
    pr.disable()
    torch.cuda.synchronize()
    c1, t1 = time.thread_time(), time.perf_counter()
    items = gen * M
    print(f"{model} {B} seqs x {M} groups: wall {1e3 * (t1 - t0):.1f} ms, driver-thread CPU "
          f"{1e3 * (c1 - c0):.1f} ms = {1e6 * (c1 - c0) / items:.1f} us per item ({items} items)")
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)
    st.sort_stats("cumulative").print_stats(30)


if __name__ == "__main__":
    main()
