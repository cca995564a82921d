#!/usr/bin/env python3
"""Host cost of issuing pipeline steps: cProfile of StageWorker.run_step on
every stage thread (per-thread profilers merged), for a generation session of
PROFILE_MODEL with PROFILE_GROUPS x 256 sequences, PROFILE_STAGES stage
threads on one GPU (device loopback; 1 = the plain engine).  Prints the top
functions by internal time over the timed sessions."""
from __future__ import annotations

import cProfile
import io
import os
import pstats
import random
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_demo_amd.config import EngineConfig, SamplingParams  # noqa: E402
from llm_sharding_demo_amd.parallel import pipeline  # noqa: E402
from llm_sharding_demo_amd.runtime.engine import Engine  # noqa: E402

MODEL = os.environ.get("PROFILE_MODEL", "gpt2")
G = int(os.environ.get("PROFILE_GROUPS", "16"))
P = int(os.environ.get("PROFILE_STAGES", "1"))
TRANSPORT = os.environ.get("PROFILE_TRANSPORT", "devloop")

profs = {}
lock = threading.Lock()
active = [False]
orig = pipeline.StageWorker.run_step


def run_step(self, *a, **k):
    if not active[0]:
        return orig(self, *a, **k)
    tid = threading.get_ident()
    with lock:
        pr = profs.setdefault(tid, cProfile.Profile())
    pr.enable()
    try:
        return orig(self, *a, **k)
    finally:
        pr.disable()


pipeline.StageWorker.run_step = run_step


def main():
    B = G * 256
    kw = dict(model_id=MODEL, num_stages=P, max_batch=B, max_seq_len=128 + 1, device="cuda",
              num_microbatches=G, prefill_chunk=0 if P == 1 else 32)
    if P > 1:
        kw["transport"] = TRANSPORT
    eng = Engine(EngineConfig(**kw))
    rnd = random.Random(0)
    prompts = [[rnd.randrange(50257) for _ in range(64)] for _ in range(B)]
    sp = SamplingParams(temperature=0.6, top_k=40, max_new_tokens=64)
    eng.generate_ids(prompts, [sp] * B)  # warm: captures
    eng.generate_ids(prompts, [sp] * B)
    active[0] = True
    t0 = time.perf_counter()
    for _ in range(2):
        eng.generate_ids(prompts, [sp] * B)
    wall = time.perf_counter() - t0
    active[0] = False
    st = None
    for pr in profs.values():
        if st is None:
            st = pstats.Stats(pr)
        else:
            st.add(pr)
    s = io.StringIO()
    st.stream = s
    st.sort_stats("tottime").print_stats(30)
    print(f"model {MODEL} stages {P} groups {G}: 2 sessions in {wall:.3f} s, {len(profs)} profiled threads")
    print(s.getvalue())
    s = io.StringIO()
    st.stream = s
    st.sort_stats("cumulative").print_stats(25)
    print(s.getvalue())


if __name__ == "__main__":
    main()
