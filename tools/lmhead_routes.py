#!/usr/bin/env python3
"""lm_head at decode row counts (fp32 logits + the sampler's 8-logit segment maxima): the
256x256 kernel (default) against the 256-row-block kernel (gemm_d256, 64 / 128-wide tiles)
and the 128x128 kernel, GPT-2 small (K 768) and XL (K 1600), 256 and 128 rows; weights
rotate through > 256 MiB (cold, as in decode)."""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from microbench import C, report, rotating, timeit  # noqa: E402

C.gemm_set_ring8(2)
C.gemm_set_ring_tn(0)
cnt = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
N = 50304


def case(M, K, label, kind=True, splits=1, big_min=160, tiled3=512):
    ws = rotating(lambda: torch.randn(N, K, device="cuda").bfloat16(), N * K * 2)
    a = torch.randn(M, K, device="cuda").bfloat16()
    seg = torch.empty(M, N // 8, device="cuda")
    it = [0]
    C.gemm_set_big_min(big_min)
    C.gemm_set_tiled3_max(tiled3)

    def run():
        w = ws[it[0] % len(ws)]
        it[0] += 1
        C.linear_f32(a, w, kind, splits, cnt, seg)

    us = timeit(run)
    C.gemm_set_big_min(160)
    C.gemm_set_tiled3_max(512)
    report(f"lm_head {label} M={M} N={N} K={K}", us, N * K * 2)


for K in (768, 1600):
    for M in (256, 128):
        case(M, K, "256x256 / ring (default)")
        case(M, K, "d256-128", kind=3)
        case(M, K, "d256-64", kind=2)
        case(M, K, "128x128 tiled", big_min=1 << 30, tiled3=0)
