#!/usr/bin/env python3
"""Llama-3 8B 512-row MLP half in isolation vs in sequence: the gate_up GEMM (256x256 kernel,
SiLU*up epilogue) replayed alone, and inside the layer's sequence RMSNorm (folding 8 slabs) ->
gate_up -> down (8 K-split bf16 slabs), with cold weights (> 256 MiB rotated).  Run under
rocprofv3 --kernel-trace --stats for the per-kernel times of each phase (the phases use
different kernels' call counts: 40 alone, 40 in sequence)."""
from __future__ import annotations

import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from microbench import C, rotating, timeit  # noqa: E402

from llm_sharding_demo_amd.ops.hip import HipBackend  # noqa: E402

be = HipBackend()
M, H, F = 512, 4096, 14336
cnt = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
wgu = rotating(lambda: (torch.randn(2 * F, H, device="cuda") * 0.02).bfloat16(), 2 * F * H * 2, total=900 << 20)
wdn = rotating(lambda: (torch.randn(H, F, device="cuda") * 0.02).bfloat16(), F * H * 2, total=900 << 20)
x = torch.randn(M, H, device="cuda")
gamma = torch.ones(H, device="cuda").bfloat16()
a = C.norm(x, None, None, gamma, None, 1e-5, True, None, True)
it = [0]
S = be._resid_splits(M, H, F)
tiled_d = be._tiled(M, H)


def alone():
    w = wgu[it[0] % len(wgu)]
    it[0] += 1
    C.linear(a, w, None, 2, True, 1, cnt)


slab = [None]


def layer():
    i = it[0]
    it[0] += 1
    xn = C.norm(x, slab[0], None, gamma, None, 1e-5, True, None, True)
    h = C.linear(xn, wgu[i % len(wgu)], None, 2, True, 1, cnt)
    slab[0] = C.linear_residual(h, wdn[i % len(wdn)], None, x, S, tiled_d, cnt, be.R.defer_resid)


t_alone = timeit(alone, iters=40)
it[0] = 0
t_layer = timeit(layer, iters=40)
print(f"gate_up alone {t_alone:.1f} us; norm + gate_up + down {t_layer:.1f} us per layer (splits {S})", flush=True)
