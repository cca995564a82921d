#!/usr/bin/env python3
"""Sampler kernel time per launch (256 rows, GPT-2 vocabulary), by path:
greedy argmax, top-k 1 / 40 / 64 fast path, top-k 200 radix path; with and
without lm_head's segment maxima.  hipGraph-replayed, warm logits."""
from __future__ import annotations

import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tools.microbench import timeit  # noqa: E402
from llm_sharding_demo_amd.ops.hip import _load  # noqa: E402

C = _load()
DEV = "cuda"


def main():
    B = int(os.environ.get("SAMPLE_B", "256"))
    V, Vp = 50257, 50304
    lg = torch.randn(B, Vp, device=DEV) * 3
    seg = lg.view(B, Vp // 8, 8).amax(-1).contiguous()
    t = torch.full((B,), 0.6, device=DEV)
    sd = torch.arange(B, dtype=torch.int64, device=DEV)
    st = torch.zeros(B, dtype=torch.int64, device=DEV)
    cases = []
    for name, k, g in (("greedy", 40, 1), ("k1", 1, 0), ("k40", 40, 0), ("k64", 64, 0), ("k200", 200, 0)):
        kk = torch.full((B,), k, dtype=torch.int32, device=DEV)
        gg = torch.full((B,), g, dtype=torch.int32, device=DEV)
        for s in (None, seg):
            cases.append((name + ("+seg" if s is not None else ""),
                          (lambda kk=kk, gg=gg, s=s: C.sample(lg, V, t, kk, gg, sd, st, s))))
    res = {n: [] for n, _ in cases}
    for _ in range(5):
        for n, f in cases:
            res[n].append(timeit(f))
    for n, _ in cases:
        print(json.dumps({"case": n, "B": B, "us": round(statistics.median(res[n]), 2)}), flush=True)


if __name__ == "__main__":
    main()
