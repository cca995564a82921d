#!/usr/bin/env python3
"""Llama-3 8B decode projections at 128 / 256 / 512 rows: the engine's routing
(HipBackend, decode) vs hipBLASLt (csrc/blaslt.cpp), rotating weights past
the Infinity Cache, hipGraph-replayed, interleaved rounds; us per call.
gate_up: ours = fused SiLU*up epilogue; blaslt = the bf16 GEMM alone (the
SiLU*up of its output is a separate elementwise pass).  Residual projections:
ours = split-K slabs + the folding norm; blaslt = in-place fp32 accumulate +
the norm without slabs."""
from __future__ import annotations

import json
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_demo_amd.ops import Residual  # noqa: E402
from llm_sharding_demo_amd.ops.hip import HipBackend  # noqa: E402
from tools.bench_d256 import graph_time  # noqa: E402

DEV = "cuda"


def main():
    be = HipBackend()
    be.decode = True
    C = be.C
    be.counters = torch.zeros(1 << 16, dtype=torch.int32, device=DEV)
    shapes = [("gate_up", 28672, 4096, "silu"), ("qkv", 6144, 4096, "plain"),
              ("o", 4096, 4096, "resid"), ("down", 4096, 14336, "resid")]
    for M in [int(m) for m in os.environ.get("LB_M", "512,256,128").split(",")]:
        for name, N, K, kind in shapes:
            nw = max(2, math.ceil((640 << 20) / (N * K * 2)))
            ws = [torch.randn(N, K, device=DEV).mul_(0.02).bfloat16() for _ in range(nw)]
            a = torch.randn(M, K, device=DEV).bfloat16()
            x = torch.randn(M, N, device=DEV)
            g = torch.ones(N, device=DEV).bfloat16()
            it = [0, 0]

            def ours():
                w = ws[it[0] % nw]
                it[0] += 1
                if kind == "silu":
                    return be.linear(a, w, None, act="silu_mul")
                if kind == "plain":
                    return be.linear(a, w, None)
                r = Residual(x)
                be.linear_residual(a, w, None, r)
                return be.rmsnorm(r, g, 1e-5) if hasattr(be, "rmsnorm") else None

            def lt():
                w = ws[it[1] % nw]
                it[1] += 1
                if kind in ("silu", "plain"):
                    return C.blaslt_linear(a, w, None, 0)
                C.blaslt_residual(a, w, None, x)
                return C.norm(x, None, None, g, None, 1e-5, True, None, True)

            t = graph_time([ours, lt], iters=10, rounds=5)
            row = {"M": M, "shape": name, "N": N, "K": K,
                   "ours_us": round(statistics.median(t[0]), 2), "blaslt_us": round(statistics.median(t[1]), 2),
                   "wTB/s_ours": round(N * K * 2 / statistics.median(t[0]) / 1e6, 2),
                   "wTB/s_blaslt": round(N * K * 2 / statistics.median(t[1]) / 1e6, 2)}
            print(json.dumps(row), flush=True)
            del ws
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
