#!/usr/bin/env python3
"""A/B of the 256-row decode GEMM (gemm_d256_kernel) against the production
routing (128x64 LDS ring) on the bench shapes, one process, interleaved
rounds (guide §5.4 rule 24), rotating weights past the Infinity Cache,
hipGraph-replayed.  Residual projections include the slab-folding norm the
engine pairs them with.  Prints one JSON line per (shape, variant): median /
min us over rounds and the max |diff| against the production path."""
from __future__ import annotations

import json
import math
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_demo_amd.ops.hip import HipBackend, _load  # noqa: E402

C = _load()
DEV = "cuda"
OUT = os.path.join("gpurun_out", "bench_d256.jsonl")

SHAPES = {  # name: (N, K, kind)  kind: act code, or "resid"
    "xl_qkv": (4800, 1600, 0), "xl_fc": (6400, 1600, 1), "xl_proj": (1600, 1600, "resid"),
    "xl_proj2": (1600, 6400, "resid"),
    "l8_qkv": (6144, 4096, 0), "l8_o": (4096, 4096, "resid"), "l8_gu": (28672, 4096, 2),
    "l8_down": (4096, 14336, "resid"),
    "s_qkv": (2304, 768, 0), "s_fc": (3072, 768, 1), "s_proj": (768, 768, "resid"),
    "s_proj2": (768, 3072, "resid"),
    # vocabulary projections (fp32 logits, the decode head)
    "xl_lm": (50304, 1600, "f32"), "s_lm": (50304, 768, "f32"), "l8_lm": (128256, 4096, "f32"),
}

# launch-routing knobs for the f32 (lm_head) variants, read at launch (capture) time
KNOBS = {
    "big": lambda on: C.gemm_set_big_kind(2 if on else 4),          # gemm_big_kernel instead of p8
    "nop8": lambda on: C.gemm_set_big_min((1 << 30) if on else 160),  # no 256x256 kernel: 128-row tiles
    "r8": lambda on: (C.gemm_set_big_min((1 << 30) if on else 160),    # 8-wave 128x64 ring
                      C.gemm_set_tiled3_max((1 << 30) if on else HipBackend.R.tiled3_max)),
}


def graph_time(fns, iters=20, rounds=7):
    """fns: list of callables; returns per-callable list of us per call,
    measured in interleaved rounds."""
    graphs = []
    for fn in fns:
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            for _ in range(3):
                fn()
        torch.cuda.current_stream().wait_stream(st)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(iters):
                fn()
        g.replay()
        graphs.append(g)
    torch.cuda.synchronize()
    res = [[] for _ in fns]
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(rounds):
        for i, g in enumerate(graphs):
            s.record()
            g.replay()
            e.record()
            torch.cuda.synchronize()
            res[i].append(s.elapsed_time(e) * 1e3 / iters)
    return res


def main():
    M_list = [int(x) for x in os.environ.get("D256_M", "256").split(",")]
    names = os.environ.get("D256_SHAPES", ",".join(SHAPES)).split(",")
    variants = os.environ.get("D256_VARIANTS", "64:1,64:2,64:3,64:4,128:1,128:2,128:3,128:4").split(",")
    slots = int(os.environ.get("D256_SLOTS", "3"))
    os.makedirs("gpurun_out", exist_ok=True)
    be = HipBackend()
    cnt = torch.zeros(1 << 16, dtype=torch.int32, device=DEV)
    C.gemm_set_d256_slots(slots)
    for M in M_list:
        for name in names:
            N, K, kind = SHAPES[name]
            nbytes = N * K * 2
            nw = max(2, math.ceil((640 << 20) / nbytes))
            if os.environ.get("D256_WARM"):  # one weight re-used: L2 / MALL-warm W (diagnostic)
                nw = 1
            ws = [torch.randn(N, K, device=DEV).mul_(0.02).bfloat16() for _ in range(nw)]
            a = torch.randn(M, K, device=DEV).bfloat16()
            x0 = torch.randn(M, N, device=DEV)
            bias = torch.randn(N, device=DEV).mul_(0.1).bfloat16()
            resid = kind == "resid"
            f32 = kind == "f32"
            act = 0 if (resid or f32) else kind

            def make(bn, S, r8=0):
                it = [0]
                x = x0.clone()

                kind = 3 if bn == 128 else 2

                def run():
                    if r8 == "tiled":  # force the tiled (ring) routing, one split
                        w = ws[it[0] % nw]
                        it[0] += 1
                        if resid:
                            slab = C.linear_residual(a, w, bias, x, 1, True, cnt, False)
                            return x
                        return C.linear(a, w, bias, act, True, 1, cnt)
                    if r8 == "lt":  # hipBLASLt with its own epilogue (bias / GELU / fp32 accumulate)
                        w = ws[it[0] % nw]
                        it[0] += 1
                        if resid:
                            C.blaslt_residual(a, w, bias, x)
                            C.norm(x, None, None, bias, None, 0.0, True, None, False)
                            return x
                        if f32:  # fp32 output, no epilogue (csrc/blaslt.cpp blaslt_f32)
                            return C.blaslt_f32(a, w)
                        if act == 2:  # SiLU * up: the GEMM, then the elementwise pass
                            return C.silu_mul(C.blaslt_linear(a, w, bias, 0))
                        return C.blaslt_linear(a, w, bias, act)
                    C.gemm_set_ring8(r8 & 15 if not isinstance(r8, str) else HipBackend.R.ring8)  # read at launch
                    C.gemm_set_ring8_flags((r8 >> 4) & 15 if not isinstance(r8, str) else 0)
                    w = ws[it[0] % nw]
                    it[0] += 1
                    if f32:
                        if isinstance(r8, str):
                            KNOBS[r8](True)
                        y = C.linear_f32(a, w, True if bn == 0 else kind, 1 if bn == 0 else S, cnt)
                        if isinstance(r8, str):
                            KNOBS[r8](False)
                        return y
                    if resid:
                        if bn == 0:
                            s2 = be._resid_splits(M, N, K)
                            tiled = be._tiled(M, N)
                            slab = C.linear_residual(a, w, bias, x, s2, tiled, cnt, tiled or be.R.defer_resid)
                        else:
                            slab = C.linear_residual(a, w, bias, x, S, kind, cnt, True)
                        if slab is not None:
                            C.norm(x, slab, bias, None, None, 0.0, True, None, False)
                        return x
                    if bn < 0:  # ring8 split-K
                        return C.linear(a, w, bias, act, 1, -bn, cnt)
                    if bn == 0:
                        tiled, s2 = be._gemm_kw(M, N, K, 2 if act == 2 else 1)
                        return C.linear(a, w, bias, act, tiled, s2, cnt)
                    return C.linear(a, w, bias, act, kind, S, cnt)
                return run

            cases = [("ring", 0, 1, int(os.environ.get("D256_BASE_R8", "0")))]
            for v in variants:
                if v == "tiled":  # the tiled kernels whatever the routing picks
                    cases.append(("tiled", 0, 1, "tiled"))
                    continue
                if v == "lt":  # hipBLASLt (csrc/blaslt.cpp), GELU / bias epilogues
                    cases.append(("blaslt", 0, 1, "lt"))
                    continue
                if v.startswith("knob:"):  # f32 shapes: a launch-routing knob (KNOBS)
                    if f32:
                        cases.append((v[5:], 0, 1, v[5:]))
                    continue
                if v.startswith("r8s:"):  # 8-wave ring, S K splits + in-kernel combine
                    C.gemm_set_ring8(2)
                    if not resid and C.gemm_ring8_tiles(M, N, K, int(v[4:])):
                        cases.append((f"ring8s{v[4:]}", -int(v[4:]), 1, 2))
                    continue
                if v.startswith("r8:"):  # 8-wave ring layouts (gemm_ring8_kernel): r8:VAR[:FLAGS]
                    f = [int(x) for x in v[3:].split(":")]
                    code = f[0] + 16 * (f[1] if len(f) > 1 else 0)
                    cases.append((f"ring8v{f[0]}f{f[1] if len(f) > 1 else 0}", 0, 1, code))
                    continue
                bn, S = map(int, v.split(":"))
                if S > K // 64 // 2 or (bn == 128 and N % 128):
                    continue
                cases.append((f"d{bn}s{S}", bn, S, 0))
            # correctness vs the production path (same weight, fresh residual)
            outs = []
            for _, bn, S, r8 in cases:
                f = make(bn, S, r8)
                y = f()
                torch.cuda.synchronize()
                outs.append((y - x0) if resid else y.float())
            base = outs[0]
            diffs = [float((o - base).abs().max()) for o in outs]
            times = graph_time([make(bn, S, r8) for _, bn, S, r8 in cases])
            C.gemm_set_ring8(0)
            for (lab, bn, S, _), t, d in zip(cases, times, diffs):
                row = {"M": M, "shape": name, "N": N, "K": K, "case": lab,
                       "us_med": round(statistics.median(t), 2), "us_min": round(min(t), 2),
                       "wTB/s": round(nbytes / (statistics.median(t) * 1e-6) / 1e12, 3),
                       "max_diff_vs_ring": round(d, 4)}
                print(json.dumps(row), flush=True)
                with open(OUT, "a") as f:
                    f.write(json.dumps(row) + "\n")
            del ws
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
