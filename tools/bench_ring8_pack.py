#!/usr/bin/env python3
"""A/B: the 8-wave 128x64 decode ring reading its operands from k-block
packed layouts (gemm.hip stage_rows_packed: every LDS-DMA instruction reads
1 KiB of consecutive bytes) against the row-strided layouts (8 rows x 128 B
at a K x 2 B pitch).  256 rows, rotating weights past the Infinity Cache,
hipGraph-replayed, interleaved rounds (tools/bench_d256.py graph_time).
pack: 0 none, 1 weights, 2 activations, 3 both.  Prints one JSON line per
(shape, pack) with the max |diff| against the unpacked launch (0 expected:
same k order)."""
from __future__ import annotations

import json
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_demo_amd.ops.hip import HipBackend, _load  # noqa: E402
from tools.bench_d256 import graph_time  # noqa: E402

C = _load()
SHAPES = {"xl_qkv": (4800, 1600), "xl_fc": (6400, 1600), "xl_proj2": (1600, 6400), "l8_o": (4096, 4096),
          "s_qkv": (2304, 768)}


def pack_w(w):
    N, K = w.shape
    return w.view(N // 64, 64, K // 64, 64).permute(0, 2, 1, 3).contiguous().view(N, K)


def pack_a(a):
    M, K = a.shape
    return a.view(M, K // 64, 64).permute(1, 0, 2).contiguous().view(M, K)


def main():
    M = int(os.environ.get("PACK_M", "256"))
    HipBackend()  # routing knobs as in the engine (8-wave ring)
    C.gemm_set_ring8(2)
    cnt = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
    for name in os.environ.get("PACK_SHAPES", ",".join(SHAPES)).split(","):
        N, K = SHAPES[name]
        nw = max(2, math.ceil((640 << 20) / (N * K * 2)))
        ws = [torch.randn(N, K, device="cuda").mul_(0.02).bfloat16() for _ in range(nw)]
        wps = [pack_w(w) for w in ws]
        a = torch.randn(M, K, device="cuda").bfloat16()
        ap = pack_a(a)
        bias = torch.randn(N, device="cuda").mul_(0.1).bfloat16()

        def make(pk):
            it = [0]

            def run():
                C.gemm_set_ring8_pack(pk)  # read at launch (capture) time
                i = it[0] % nw
                it[0] += 1
                return C.linear(ap if pk & 2 else a, wps[i] if pk & 1 else ws[i], bias, 0, True, 1, cnt)
            return run

        outs = []
        for pk in range(4):
            y = make(pk)()
            torch.cuda.synchronize()
            outs.append(y.float())
        times = graph_time([make(pk) for pk in range(4)])
        C.gemm_set_ring8_pack(0)
        for pk, t in enumerate(times):
            row = {"M": M, "shape": name, "N": N, "K": K, "pack": pk, "us_med": round(statistics.median(t), 2),
                   "us_min": round(min(t), 2), "max_diff": float((outs[pk] - outs[0]).abs().max())}
            print(json.dumps(row), flush=True)
        del ws, wps
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
