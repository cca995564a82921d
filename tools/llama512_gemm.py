#!/usr/bin/env python3
"""Llama-3 8B decode GEMMs at 512 rows (the 512-sequence bench, one group):
which hand-written tiling fills the chip.  gate_up (28672 x 4096, SiLU*up
epilogue) runs 224 tiles of 256x256 on gemm_p8 by default (224 workgroups for
256 CUs, 64 k-steps); the 128x128 kernel gives 896 workgroups, two 256-row
launches of gemm_d256 448.  QKV (6144 x 4096) on the 8-wave ring.  torch.matmul
(hipBLASLt, no epilogue) as the yardstick.  Weights rotate through > 256 MiB."""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from microbench import C, report, rotating, timeit  # noqa: E402

C.gemm_set_ring8(2)  # the engine's defaults (ops/routing.py)
C.gemm_set_tiled3_max(512)
C.gemm_set_ring_tn(0)

M, K = 512, 4096
cnt = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
a = torch.randn(M, K, device="cuda").bfloat16()


def case(N, code, label, kind=True, splits=1, halves=False, big_min=160, tiled3=512):
    ws = rotating(lambda: torch.randn(N, K, device="cuda").bfloat16(), N * K * 2)
    it = [0]
    C.gemm_set_big_min(big_min)
    C.gemm_set_tiled3_max(tiled3)

    def run():
        w = ws[it[0] % len(ws)]
        it[0] += 1
        if halves:
            C.linear(a[:256], w, None, code, kind, splits, cnt)
            C.linear(a[256:], w, None, code, kind, splits, cnt)
        else:
            C.linear(a, w, None, code, kind, splits, cnt)

    us = timeit(run)
    C.gemm_set_big_min(160)
    C.gemm_set_tiled3_max(512)
    it[0] = 0

    def tm():
        w = ws[it[0] % len(ws)]
        it[0] += 1
        torch.matmul(a, w.t())

    ut = timeit(tm)
    flop = 2.0 * M * N * K
    report(f"{label} M={M} N={N} K={K}", us, N * K * 2,
           {"PF/s": round(flop / us / 1e9, 3), "hipblaslt_us": round(ut, 2)})


N_GU, N_QKV = 2 * 14336, 6144
case(N_QKV, 0, "qkv-shaped bf16 ring8 (default)")
for kind, bn in ((2, 64), (3, 128)):
    for S in (1, 2, 3, 4):
        case(N_QKV, 0, f"qkv-shaped bf16 d256-{bn} row blocks s{S}", kind=kind, splits=S)
case(N_GU, 2, "gate_up p8 256x256 (default)")
for S in (1, 2):
    case(N_GU, 2, f"gate_up d256-128 row blocks s{S}", kind=3, splits=S)
N_O = 4096
case(N_O, 0, "o-shaped bf16 d256-64 row blocks s2", kind=2, splits=2)
case(N_O, 0, "o-shaped bf16 d256-64 row blocks s4", kind=2, splits=4)
case(N_O, 0, "o-shaped bf16 d256-128 row blocks s4", kind=3, splits=4)
