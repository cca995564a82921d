#!/usr/bin/env python3
"""Prefill GEMM kernel vs hipBLASLt (torch.matmul) on random operands, graph-replayed.

Shapes: the GPT-2 XL / Llama-3 8B prefill projections at 64K / 8K tokens and the square
4096^3 / 8192^3 reference points of the guide's 256^2 8-phase template, plain bf16 output
(EPI none) and the fused epilogue each projection runs in the engine.
Usage: python tools/bench_p8.py [kind ...]   (kind: C.gemm_set_big_kind value 0, 1 or 4; default 4)
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_demo_amd.ops.hip import _load  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from microbench import timeit  # noqa: E402

C = _load()
DEV = "cuda"


def case(label, M, N, K, act=0, resid=False, kinds=(1,)):
    a = torch.randn(M, K, device=DEV).bfloat16()
    w = torch.randn(N, K, device=DEV).bfloat16()
    b = torch.randn(N, device=DEV).bfloat16() if act == 1 else None
    x = torch.randn(M, N, device=DEV) if resid else None
    fl = 2.0 * M * N * K
    row = {"case": label, "M": M, "N": N, "K": K}
    C.gemm_set_big_min(1)
    for kind in kinds:
        C.gemm_set_big_kind(kind)
        if resid:
            fn = lambda: C.linear_residual(a, w, None, x, 1, True, None, False)  # noqa: E731
        else:
            fn = lambda: C.linear(a, w, b, act, True, 1, None)  # noqa: E731
        us = timeit(fn, iters=10)
        row[f"k{kind}_us"] = round(us, 1)
        row[f"k{kind}_TF"] = round(fl / us / 1e6, 1)
    C.gemm_set_big_kind(4)
    C.gemm_set_big_min(160)
    ut = timeit(lambda: torch.matmul(a, w.t()), iters=10)
    row["hipblaslt_us"] = round(ut, 1)
    row["hipblaslt_TF"] = round(fl / ut / 1e6, 1)
    print(json.dumps(row), flush=True)


def blaslt_case(label, M, N, K, resid):
    """Engine routing A/B: the hand-written 256x256 kernel with its fused epilogue
    vs hipBLASLt with the library's (csrc/blaslt.cpp), bias included."""
    a = torch.randn(M, K, device=DEV).bfloat16()
    w = torch.randn(N, K, device=DEV).mul_(0.05).bfloat16()
    b = torch.randn(N, device=DEV).mul_(0.1).bfloat16()
    x = torch.randn(M, N, device=DEV)
    fl = 2.0 * M * N * K
    if resid:
        ours = lambda: C.linear_residual(a, w, b, x, 1, True, None, False)  # noqa: E731
        lt = lambda: C.blaslt_residual(a, w, b, x)  # noqa: E731
    else:
        ours = lambda: C.linear(a, w, b, 1, True, 1, None)  # noqa: E731
        lt = lambda: C.blaslt_linear(a, w, b, 1)  # noqa: E731
    row = {"case": label, "M": M, "N": N, "K": K}
    for name, fn in (("p8", ours), ("blaslt", lt)):
        us = min(timeit(fn, iters=10) for _ in range(3))
        row[f"{name}_us"] = round(us, 1)
        row[f"{name}_TF"] = round(fl / us / 1e6, 1)
    print(json.dumps(row), flush=True)


def main():
    if sys.argv[1:] == ["blaslt"]:
        for M in (32768, 65536):
            blaslt_case("xl_fc_gelu", M, 6400, 1600, False)
            blaslt_case("xl_proj_resid", M, 1600, 1600, True)
            blaslt_case("xl_proj2_resid", M, 1600, 6400, True)
        blaslt_case("l8_o_resid", 32768, 4096, 4096, True)
        blaslt_case("l8_down_resid", 32768, 4096, 14336, True)
        return
    kinds = tuple(int(v) for v in sys.argv[1:]) or (1,)
    case("sq4096", 4096, 4096, 4096, kinds=kinds)
    case("sq8192", 8192, 8192, 8192, kinds=kinds)
    case("xl_qkv", 65536, 4800, 1600, kinds=kinds)
    case("xl_fc_gelu", 65536, 6400, 1600, act=1, kinds=kinds)
    case("xl_fc_plain", 65536, 6400, 1600, kinds=kinds)
    case("xl_proj_resid", 65536, 1600, 1600, resid=True, kinds=kinds)
    case("xl_proj2_resid", 65536, 1600, 6400, resid=True, kinds=kinds)
    case("l8_gateup", 8192, 28672, 4096, act=2, kinds=kinds)
    case("l8_down_resid", 8192, 4096, 14336, resid=True, kinds=kinds)


if __name__ == "__main__":
    main()
