#!/usr/bin/env python3
"""Per-kernel microbenchmarks on one MI355X (events, warm L2 excluded where it
matters by rotating through several weight copies > 256 MiB Infinity Cache).

Prints one line per case: time (us), achieved bandwidth (TB/s, weight+KV bytes
streamed), and for GEMMs the torch.matmul (hipBLASLt) time on the same data as
a yardstick.  Output also written as JSON to gpurun_out/microbench.json.
"""
from __future__ import annotations

import json
import math
import statistics
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_demo_amd.ops.hip import _load, prefill_tiles  # noqa: E402
from llm_sharding_demo_amd.runtime.batch import BatchMeta  # noqa: E402

C = _load()
DEV = "cuda"
RESULTS = []


def timeit(fn, iters=50, warm=3, graph=True):
    """Device time per call.  graph=True captures `iters` calls into one
    hipGraph and replays it, so host launch overhead does not bound the
    number (matches how the engine runs decode)."""
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        for _ in range(warm):
            fn()
    torch.cuda.current_stream().wait_stream(st)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if graph:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(iters):
                fn()
        g.replay()
        torch.cuda.synchronize()
        s.record()
        g.replay()
        e.record()
    else:
        s.record()
        for _ in range(iters):
            fn()
        e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters  # us


def rotating(make, nbytes_each, total=640 << 20):
    n = max(2, math.ceil(total / max(nbytes_each, 1)))
    return [make() for _ in range(n)]


def report(name, us, nbytes, extra=None):
    tbs = nbytes / (us * 1e-6) / 1e12
    row = {"case": name, "us": round(us, 2), "TB/s": round(tbs, 3)}
    if extra:
        row.update(extra)
    RESULTS.append(row)
    print(json.dumps(row), flush=True)


def bench_gemm(M, N, K, act=0, resid=False, label="", force_tiled=False):
    ws = rotating(lambda: torch.randn(N, K, device=DEV).bfloat16(), N * K * 2)
    a = torch.randn(M, K, device=DEV).bfloat16()
    x = torch.randn(M, N, device=DEV)
    it = [0]
    be = __import__("llm_sharding_demo_amd.ops.hip", fromlist=["HipBackend"]).HipBackend()

    be.counters = torch.zeros(1 << 16, dtype=torch.int32, device=DEV)
    nw = 2 if act == 2 else 1
    tiled, splits = be._gemm_kw(M, N, K, nw)
    if force_tiled:
        tiled, splits = True, 1
    if resid:
        splits = be._resid_splits(M, N, K)
        if force_tiled:  # the tiled path's own split rule at these M rows
            tiles = math.ceil(M / 128) * math.ceil(N / 128)
            splits = max(1, min(math.ceil(256 / tiles), K // 64 // 2 or 1))

    def run():
        w = ws[it[0] % len(ws)]
        it[0] += 1
        if resid:  # + the combine the engine pairs it with (deferred slabs -> norm)
            slab = C.linear_residual(a, w, None, x, splits, tiled, be.counters, be.R.defer_resid)
            if slab is not None:
                C.norm(x, slab, None, None, None, 0.0, True, None, False)
        else:
            C.linear(a, w, None, act, tiled, splits, be.counters)

    us = timeit(run)
    it[0] = 0

    def tm():
        w = ws[it[0] % len(ws)]
        it[0] += 1
        torch.matmul(a, w.t())

    ut = timeit(tm)
    report(f"gemm{label} M={M} N={N} K={K} S={splits}{' tiled' if tiled else ''}", us, N * K * 2,
           {"hipblaslt_us": round(ut, 2)})


def bench_prefill_gemms(T, H, F, nh, hd, label=""):
    """Prefill-shaped tiled GEMMs with their real fused epilogues (QKV scatter
    into the KV cache, bias+GELU, residual add) vs plain hipBLASLt matmul."""
    nseq = T // 128
    kc = torch.zeros(nseq, nh, 128, hd, device=DEV).bfloat16()
    vc = torch.zeros_like(kc)
    slot = torch.arange(nseq, dtype=torch.int32, device=DEV).repeat_interleave(128)
    pos = torch.arange(128, dtype=torch.int32, device=DEV).repeat(nseq)
    a = torch.randn(T, H, device=DEV).bfloat16()
    af = torch.randn(T, F, device=DEV).bfloat16()
    x = torch.randn(T, H, device=DEV)
    wq = torch.randn(3 * H, H, device=DEV).bfloat16()
    bq = torch.randn(3 * H, device=DEV).bfloat16()
    wf = torch.randn(F, H, device=DEV).bfloat16()
    bf = torch.randn(F, device=DEV).bfloat16()
    wp = torch.randn(H, H, device=DEV).bfloat16()
    wp2 = torch.randn(H, F, device=DEV).bfloat16()
    cases = [
        ("qkv", lambda: C.linear_qkv(a, wq, bq, kc, vc, slot, pos, H, H, hd, None, True, 1, None),
         lambda: torch.matmul(a, wq.t()), 3 * H, H),
        ("fc_gelu", lambda: C.linear(a, wf, bf, 1, True, 1, None), lambda: torch.matmul(a, wf.t()), F, H),
        ("proj_resid", lambda: C.linear_residual(a, wp, None, x, 1, True, None, False),
         lambda: torch.matmul(a, wp.t()), H, H),
        ("proj2_resid", lambda: C.linear_residual(af, wp2, None, x, 1, True, None, False),
         lambda: torch.matmul(af, wp2.t()), H, F),
    ]
    for name, fn, ref, N, K in cases:
        C.gemm_set_big_min(1 << 30)
        u128 = timeit(fn, iters=20)
        C.gemm_set_big_min(1)
        us = timeit(fn, iters=20)
        C.gemm_set_big_min(160)
        ut = timeit(ref, iters=20)
        fl = 2.0 * T * N * K
        report(f"prefill{label}_{name} M={T} N={N} K={K}", us, 0,
               {"TFLOP/s": round(fl / us / 1e6, 1), "tile128_us": round(u128, 2),
                "tile128_TFLOP/s": round(fl / u128 / 1e6, 1), "hipblaslt_us": round(ut, 2),
                "hipblaslt_TFLOP/s": round(fl / ut / 1e6, 1)})


def bench_decode_layer(M, H=1600, F=6400, nh=25, hd=64, ctx=192, slots=256):
    """One GPT-2 XL decode layer's kernels at M rows, in engine order with
    their real epilogues (QKV scatter into a ctx-deep cache, deferred residual
    slabs + norm combine), each timed alone and the chain as one graph, on
    rotating weight copies (cold in the 256 MiB Infinity Cache)."""
    from llm_sharding_demo_amd.ops.hip import HipBackend
    from llm_sharding_demo_amd.ops import Residual

    be = HipBackend()
    be.counters = torch.zeros(1 << 16, dtype=torch.int32, device=DEV)
    nl = 6  # weight copies: 6 x 61 MB > MALL
    W = [dict(wq=torch.randn(3 * H, H, device=DEV).bfloat16() * 0.02,
              bq=torch.zeros(3 * H, device=DEV).bfloat16(),
              wp=torch.randn(H, H, device=DEV).bfloat16() * 0.02,
              wf=torch.randn(F, H, device=DEV).bfloat16() * 0.02,
              bfc=torch.zeros(F, device=DEV).bfloat16(),
              wp2=torch.randn(H, F, device=DEV).bfloat16() * 0.02) for _ in range(nl)]
    g1 = torch.ones(H, device=DEV).bfloat16()
    b1 = torch.zeros(H, device=DEV).bfloat16()
    kc = torch.zeros(slots, nh, ctx + 8, hd, device=DEV).bfloat16()
    vc = torch.zeros_like(kc)
    sl = torch.arange(M, dtype=torch.int32, device=DEV)
    pos = torch.full((M,), ctx, dtype=torch.int32, device=DEV)
    x = torch.randn(M, H, device=DEV)
    it = [0]

    class Meta:
        is_decode, num_seqs, max_ctx = True, M, ctx + 1
        seq_slots, token_pos, token_slots = sl, pos, sl

    def layer(parts):
        w = W[it[0] % nl]
        it[0] += 1
        r = Residual(x)
        xn = be.layernorm(r, g1, b1, 1e-5)
        if "qkv" in parts or "all" in parts:
            q = C.linear_qkv(xn, w["wq"], w["bq"], kc, vc, sl, pos, H, H, hd, None, False,
                             be._sk_splits(M, 3 * H, H), be.counters)
        else:
            q = torch.empty(M, H, device=DEV).bfloat16()
        o = be.attention(q, kc, vc, Meta) if ("attn" in parts or "all" in parts) else q
        be.linear_residual(o, w["wp"], None, r)
        xn = be.layernorm(r, g1, b1, 1e-5)
        h = be.linear(xn, w["wf"], w["bfc"], act="gelu")
        be.linear_residual(h, w["wp2"], None, r)
        be.flush(r)

    us = timeit(lambda: layer(("all",)), iters=12)
    report(f"decode_layer M={M} (norm,qkv,attn,proj,norm,fc,proj2) ctx={ctx}", us, 61e6 + M * ctx * 6400)
    us = timeit(lambda: layer(("attn",)), iters=12)
    report(f"decode_layer_no_qkv M={M}", us, 0)
    us = timeit(lambda: layer(("qkv",)), iters=12)
    report(f"decode_layer_no_attn M={M}", us, 0)


def bench_resid_norm(M, N, K, splits_list, label=""):
    """Residual GEMM + the following LayerNorm, two ways: split-K combined in
    the GEMM (last arriver) vs deferred slabs combined by the norm kernel."""
    ws = rotating(lambda: torch.randn(N, K, device=DEV).bfloat16(), N * K * 2)
    a = torch.randn(M, K, device=DEV).bfloat16()
    x = torch.randn(M, N, device=DEV)
    bias = torch.randn(N, device=DEV).bfloat16()
    g = torch.ones(N, device=DEV).bfloat16()
    cnt = torch.zeros(1 << 16, dtype=torch.int32, device=DEV)
    it = [0]
    for S in splits_list:
        for defer in (False, True):
            def run():
                w = ws[it[0] % len(ws)]
                it[0] += 1
                slab = C.linear_residual(a, w, bias, x, S, False, cnt, defer)
                C.norm(x, slab, bias if slab is not None else None, g, bias, 1e-5, False, None, True)
            us = timeit(run)
            report(f"resid+norm{label} M={M} N={N} K={K} S={S} defer={int(defer)}", us, N * K * 2)


def HipBackendSplits(*a):
    from llm_sharding_demo_amd.ops.hip import HipBackend

    return HipBackend.decode_attn_splits(*a)


def bench_attn_decode(B, nh, n_kv, hd, ctx, slots=None, splits=None):
    slots = slots or B
    S = ctx + 1
    kc = torch.randn(slots, n_kv, S, hd, device=DEV).bfloat16()
    vc = torch.randn(slots, n_kv, S, hd, device=DEV).bfloat16()
    q = torch.randn(B, nh * hd, device=DEV).bfloat16()
    ss = torch.arange(B, dtype=torch.int32, device=DEV)
    pos = torch.full((B,), ctx - 1, dtype=torch.int32, device=DEV)
    if splits is None:
        splits = 1 if B * n_kv >= 512 else min(math.ceil(512 / (B * n_kv)), max(1, math.ceil(ctx / 256)))
    us = timeit(lambda: C.attn_decode(q, kc, vc, ss, pos, nh, splits))
    report(f"attn_decode B={B} nh={nh} kv={n_kv} hd={hd} ctx={ctx} splits={splits}", us,
           B * n_kv * ctx * hd * 2 * 2)


def bench_attn_prefill(nseq, L, nh, n_kv, hd):
    kc = torch.randn(nseq, n_kv, L, hd, device=DEV).bfloat16()
    vc = torch.randn(nseq, n_kv, L, hd, device=DEV).bfloat16()
    meta = BatchMeta.build(list(range(nseq)), [0] * nseq, [L] * nseq, DEV)
    q = torch.randn(meta.num_tokens, nh * hd, device=DEV).bfloat16()
    tiles = prefill_tiles(meta).to(DEV)
    us = timeit(lambda: C.attn_prefill(q, kc, vc, tiles, meta.seq_slots, meta.q_start, meta.cu_q, nh))
    flops = nseq * nh * 2 * 2 * hd * L * L / 2
    report(f"attn_prefill seqs={nseq} L={L} nh={nh} hd={hd}", us, 0, {"TFLOP/s": round(flops / us / 1e6, 1)})


def bench_norm(T, H, splits):
    x = torch.randn(T, H, device=DEV)
    slab = torch.randn(splits, T, H, device=DEV) if splits else None
    w = torch.ones(H, device=DEV).bfloat16()
    b = torch.zeros(H, device=DEV).bfloat16()
    us = timeit(lambda: C.norm(x, slab, None, w, b, 1e-5, False, None, True))
    report(f"norm T={T} H={H} slabs={splits}", us, T * H * 4 * (2 + splits))


def bench_sample(B, V, greedy):
    Vp = (V + 63) // 64 * 64
    lg = torch.randn(B, Vp, device=DEV) * 3
    t = torch.full((B,), 0.6, device=DEV)
    k = torch.full((B,), 40, dtype=torch.int32, device=DEV)
    g = torch.full((B,), int(greedy), dtype=torch.int32, device=DEV)
    sd = torch.arange(B, dtype=torch.int64, device=DEV)
    st = torch.zeros(B, dtype=torch.int64, device=DEV)
    us = timeit(lambda: C.sample(lg, V, t, k, g, sd, st))
    report(f"sample B={B} V={V} greedy={greedy}", us, B * V * 4)


def bench_ring_tn(M, H=1600, F=6400):
    """Decode-sized ring GEMMs: 128x64 vs 128x32 tiles (2 blocks/CU), rotating
    weights; residual projections with their slab combine at several splits."""
    cnt = torch.zeros(1 << 16, dtype=torch.int32, device=DEV)
    C.gemm_set_tiled3_max(512)  # the engine's ring cap (Routing.tiled3_max)
    a = torch.randn(M, H, device=DEV).bfloat16()
    af = torch.randn(M, F, device=DEV).bfloat16()
    x = torch.randn(M, H, device=DEV)
    shapes = {"qkv": (3 * H, H), "fc": (F, H), "proj": (H, H), "proj2": (H, F)}
    ws = {k: rotating(lambda n=n, k_=k_: torch.randn(n, k_, device=DEV).bfloat16(), n * k_ * 2)
          for k, (n, k_) in shapes.items()}
    for tn in (64, 32):
        C.gemm_set_ring_tn(tn)
        for name in ("qkv", "fc"):
            it = [0]
            N, K = shapes[name]

            def run(name=name, it=it):
                w = ws[name][it[0] % len(ws[name])]
                it[0] += 1
                C.linear(a, w, None, 1 if name == "fc" else 0, True, 1, cnt)
            report(f"ring_tn{tn}_{name} M={M} N={N} K={K}", timeit(run), N * K * 2)
        for name in ("proj", "proj2"):
            N, K = shapes[name]
            inp = a if name == "proj" else af
            for S in (2, 3, 5, 8):
                it = [0]

                def run(name=name, it=it, S=S, inp=inp):
                    w = ws[name][it[0] % len(ws[name])]
                    it[0] += 1
                    slab = C.linear_residual(inp, w, None, x, S, True, cnt, True)
                    C.norm(x, slab, None, None, None, 0.0, True, None, False)
                report(f"ring_tn{tn}_{name}+combine M={M} N={N} K={K} S={S}", timeit(run), N * K * 2)
    C.gemm_set_ring_tn(64)


def bench_corun(B=256, H=1600, F=6400, nh=25, hd=64, ctx=192, L=12):
    """Co-running on two streams: an attention chain (HBM-bound) beside a
    decode-GEMM chain (latency-bound), each captured as a graph; wall time
    alone vs together (the overlap a de-phased second microbatch lane can get)."""
    cnt = torch.zeros(2, 1 << 16, dtype=torch.int32, device=DEV)
    C.gemm_set_tiled3_max(512)
    C.gemm_set_ring_tn(0)
    kcs = [torch.randn(B, nh, ctx + 1, hd, device=DEV).bfloat16() for _ in range(L)]
    vcs = [torch.randn(B, nh, ctx + 1, hd, device=DEV).bfloat16() for _ in range(L)]
    q = torch.randn(B, nh * hd, device=DEV).bfloat16()
    ss = torch.arange(B, dtype=torch.int32, device=DEV)
    pos = torch.full((B,), ctx - 1, dtype=torch.int32, device=DEV)
    a = torch.randn(B, H, device=DEV).bfloat16()
    af = torch.randn(B, F, device=DEV).bfloat16()
    x = torch.randn(B, H, device=DEV)
    wq = [torch.randn(3 * H, H, device=DEV).bfloat16() for _ in range(L)]
    wf = [torch.randn(F, H, device=DEV).bfloat16() for _ in range(L)]
    wp = [torch.randn(H, H, device=DEV).bfloat16() for _ in range(L)]
    wp2 = [torch.randn(H, F, device=DEV).bfloat16() for _ in range(L)]

    def attn_chain():
        for i in range(L):
            C.attn_decode(q, kcs[i], vcs[i], ss, pos, nh, 1)

    def gemm_chain():
        for i in range(L):
            C.linear(a, wq[i], None, 0, True, 1, cnt[1])
            s = C.linear_residual(a, wp[i], None, x, 5, True, cnt[1], True)
            C.norm(x, s, None, None, None, 0.0, True, None, False)
            C.linear(a, wf[i], None, 1, True, 1, cnt[1])
            s = C.linear_residual(af, wp2[i], None, x, 5, True, cnt[1], True)
            C.norm(x, s, None, None, None, 0.0, True, None, False)

    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()
    graphs = []
    for fn, st in ((attn_chain, sa), (gemm_chain, sb)):
        with torch.cuda.stream(st):
            fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            fn()
        graphs.append(g)
    ga, gb = graphs

    def wall(run_a, run_b, reps=5):
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            cur = torch.cuda.current_stream()
            s.record(cur)
            sa.wait_stream(cur)
            sb.wait_stream(cur)
            if run_a:
                with torch.cuda.stream(sa):
                    ga.replay()
            if run_b:
                with torch.cuda.stream(sb):
                    gb.replay()
            cur.wait_stream(sa)
            cur.wait_stream(sb)
            e.record(cur)
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e) * 1e3 / L)
        return sorted(ts)[len(ts) // 2]

    ta, tb, tab = wall(True, False), wall(False, True), wall(True, True)
    report(f"corun B={B} ctx={ctx} per layer: attn alone", ta, 0)
    report(f"corun B={B} ctx={ctx} per layer: gemms+norms alone", tb, 0)
    report(f"corun B={B} ctx={ctx} per layer: both on two streams", tab, 0,
           {"sum_us": round(ta + tb, 2), "overlap_saved_us": round(ta + tb - tab, 2)})


def stamps_p8(M=65536, N=6400, K=1600, act=1):
    """Per-workgroup phase timeline of the phase-pipelined prefill GEMM:
    prologue (first K-tiles landed), main loop, epilogue; 100 MHz stamps."""
    a = torch.randn(M, K, device=DEV).bfloat16()
    w = torch.randn(N, K, device=DEV).bfloat16()
    b = torch.randn(N, device=DEV).bfloat16()
    nb = ((M + 255) // 256) * ((N + 255) // 256)
    st = torch.zeros(nb * 8, dtype=torch.int64, device=DEV)
    C.gemm_set_big_min(1)
    for _ in range(2):
        C.linear(a, w, b, act, True, 1, None)
    torch.cuda.synchronize()
    C.set_stamps(st)
    C.linear(a, w, b, act, True, 1, None)
    torch.cuda.synchronize()
    C.set_stamps(None)
    C.gemm_set_big_min(160)
    t = st.view(nb, 8).cpu().double()
    us = lambda x: x * 10 / 1000  # noqa: E731
    q = lambda x: [round(float(x.quantile(v)), 2) for v in (0.0, 0.1, 0.5, 0.9, 1.0)]  # noqa: E731
    row = {"case": f"stamps_p8 M={M} N={N} K={K} blocks={nb}",
           "prologue_us": q(us(t[:, 1] - t[:, 0])), "main_us": q(us(t[:, 2] - t[:, 1])),
           "epilogue_us": q(us(t[:, 3] - t[:, 2])), "block_us": q(us(t[:, 3] - t[:, 0])),
           "span_us": round(float(us(t[:, 3].max() - t[:, 0].min())), 1),
           "sum_block_us_per_cu": round(float(us(t[:, 3] - t[:, 0]).sum()) / 256, 1)}
    if t[:, 4].abs().sum() > 0:  # LSD_P8_PROF build: wave 0's loop cycles and where they went
        lp = t[:, 4]
        row.update({"loop_kcyc": q(lp / 1e3), "vmcnt_wait_frac": q(t[:, 5] / lp),
                    "barrier1_frac": q(t[:, 6] / lp), "barrier2_frac": q(t[:, 7] / lp)})
    RESULTS.append(row)
    print(json.dumps(row), flush=True)


def bench_lmhead_kinds(M=256, N=50304, K=1600):
    """Decode vocab projection at M rows: 256x256 phase-pipelined tiles vs the
    128x128 tiled kernel (2 blocks/CU) vs hipBLASLt; rotating weights."""
    ws = rotating(lambda: torch.randn(N, K, device=DEV).bfloat16(), N * K * 2)
    a = torch.randn(M, K, device=DEV).bfloat16()
    it = [0]

    def run():
        w = ws[it[0] % len(ws)]
        it[0] += 1
        C.linear_f32(a, w, True, 1, None)
    for name, bm in (("p8", 1), ("tiled128", 1 << 30)):
        C.gemm_set_big_min(bm)
        report(f"lmhead_{name} M={M} N={N} K={K}", timeit(run), N * K * 2)
    C.gemm_set_big_min(160)

    def ref():
        w = ws[it[0] % len(ws)]
        it[0] += 1
        torch.matmul(a, w.t())
    report(f"lmhead_hipblaslt M={M} N={N} K={K}", timeit(ref), N * K * 2)


def bench_lmhead_sample(M=256, V=50257, K=1600):
    """Decode head: lm_head (fp32 logits) + the sampler (T 0.6, top-k 40), with
    and without the epilogue's 8-logit segment maxima; rotating weights,
    interleaved rounds; asserts equal draws."""
    Vp = (V + 63) // 64 * 64
    ws = rotating(lambda: torch.randn(Vp, K, device=DEV).mul_(0.05).bfloat16(), Vp * K * 2)
    a = torch.randn(M, K, device=DEV).bfloat16()
    t = torch.full((M,), 0.6, device=DEV)
    k = torch.full((M,), 40, dtype=torch.int32, device=DEV)
    g = torch.zeros(M, dtype=torch.int32, device=DEV)
    sd = torch.arange(M, dtype=torch.int64, device=DEV)
    st = torch.zeros(M, dtype=torch.int64, device=DEV)
    it = [0]
    outs = {}

    def run(seg, sample=True):
        def f():
            w = ws[it[0] % len(ws)]
            it[0] += 1
            sm = torch.empty(M, Vp // 8, device=DEV) if seg else None
            lg = C.linear_f32(a, w, True, 1, None, sm)
            if sample:
                outs[seg] = C.sample(lg, V, t, k, g, sd, st, sm)
        return f
    for seg in (False, True):
        it[0] = 0
        run(seg)()
    torch.cuda.synchronize()
    assert torch.equal(outs[False], outs[True])
    res = {c: [] for c in ("gemm", "gemm+seg", "full", "seg")}
    for _ in range(5):
        res["gemm"].append(timeit(run(False, False)))
        res["gemm+seg"].append(timeit(run(True, False)))
        res["full"].append(timeit(run(False)))
        res["seg"].append(timeit(run(True)))
    for c, v in res.items():
        report(f"lmhead_sample_{c} M={M} V={V} K={K}", statistics.median(v), Vp * K * 2)


def bench_llama_decode_kinds(M=256):
    """Llama-3 8B decode GEMMs at M rows under each tiled-kernel choice:
    128x128 double buffer, LDS ring 128x64 / 128x128, phase-pipelined 256x256."""
    H, F = 4096, 14336
    cnt = torch.zeros(1 << 16, dtype=torch.int32, device=DEV)
    shapes = [("qkv", 6144, H, 0), ("gate_up", 2 * F, H, 2), ("o_proj", H, H, -1), ("down", H, F, -1)]
    for name, N, K, act in shapes:
        ws = rotating(lambda N=N, K=K: torch.randn(N, K, device=DEV).bfloat16(), N * K * 2)
        a = torch.randn(M, K, device=DEV).bfloat16()
        x = torch.randn(M, N, device=DEV)
        for kind, t3, tn, bm in (("dbuf128", 0, 128, 1 << 30), ("ring64", 1 << 30, 64, 1 << 30),
                                 ("ring128", 1 << 30, 128, 1 << 30), ("p8", 0, 64, 1)):
            C.gemm_set_tiled3_max(t3)
            C.gemm_set_ring_tn(tn)
            C.gemm_set_big_min(bm)
            it = [0]

            def run(ws=ws, a=a, x=x, act=act, it=it, N=N):
                w = ws[it[0] % len(ws)]
                it[0] += 1
                if act < 0:
                    C.linear_residual(a, w, None, x, 1, True, cnt, False)
                else:
                    C.linear(a, w, None, act, True, 1, cnt)
            report(f"llama_{name}_{kind} M={M} N={N} K={K}", timeit(run, iters=20), N * K * 2)
    C.gemm_set_tiled3_max(512)
    C.gemm_set_ring_tn(0)
    C.gemm_set_big_min(160)


def bench_llama_sk(M=256):
    """Llama-3 8B decode GEMMs on the split-K decode kernel (W straight to
    VGPRs, last-arriver combine) at several splits."""
    H, F = 4096, 14336
    cnt = torch.zeros(1 << 16, dtype=torch.int32, device=DEV)
    for name, N, K, act in (("qkv", 6144, H, 0), ("gate_up", 2 * F, H, 2), ("o_proj", H, H, 0), ("down", H, F, 0)):
        ws = rotating(lambda N=N, K=K: torch.randn(N, K, device=DEV).bfloat16(), N * K * 2)
        a = torch.randn(M, K, device=DEV).bfloat16()
        for S in (1, 2, 4, 8):
            if K // 32 // S < 2:
                continue
            it = [0]

            def run(ws=ws, a=a, act=act, it=it, S=S):
                w = ws[it[0] % len(ws)]
                it[0] += 1
                C.linear(a, w, None, act, False, S, cnt)
            report(f"llama_{name}_sk M={M} N={N} K={K} S={S}", timeit(run, iters=20), N * K * 2)


def stamps_gemm(M, N, K, splits, act=0, label=""):
    """Per-workgroup phase timeline of one decode-GEMM launch (diagnostic)."""
    w = torch.randn(N, K, device=DEV).bfloat16()
    a = torch.randn(M, K, device=DEV).bfloat16()
    cnt = torch.zeros(1 << 16, dtype=torch.int32, device=DEV)
    nb = (N // 64) * splits
    st = torch.zeros(nb * 8, dtype=torch.int64, device=DEV)
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=DEV)
    for rep in range(3):
        flush.zero_()  # evict W from the Infinity Cache
        torch.cuda.synchronize()
        st.zero_()
        C.set_stamps(st)
        C.linear(a, w, None, act, False, splits, cnt)
        torch.cuda.synchronize()
        C.set_stamps(None)
    t = st.view(nb, 8).cpu().double()
    t0 = t[:, 0].min()
    ph = {}
    ent = (t[:, 0] - t0) * 10 / 1000  # us (100 MHz)
    lat = (t[:, 1] - t[:, 0]) * 10 / 1000
    comp = (t[:, 2] - t[:, 1]) * 10 / 1000
    pub = (t[:, 3] - t[:, 2]) * 10 / 1000
    last = t[:, 5] > 0
    red = (t[last, 4] - t[last, 3]) * 10 / 1000
    epi = (t[last, 5] - t[last, 4]) * 10 / 1000
    end = (t[last, 5] - t0) * 10 / 1000
    q = lambda x: [round(float(x.quantile(v)), 2) for v in (0.0, 0.5, 0.9, 1.0)] if x.numel() else []
    row = {"case": f"stamps{label} M={M} N={N} K={K} S={splits} blocks={nb}",
           "entry_us": q(ent), "load_us": q(lat), "compute_us": q(comp), "publish_us": q(pub),
           "reduce_us": q(red), "epilogue_us": q(epi), "span_us": round(float(end.max()), 2),
           "xcc_hist": torch.bincount(t[:, 7].long(), minlength=8).tolist()}
    RESULTS.append(row)
    print(json.dumps(row), flush=True)


def main():
    which = sys.argv[1:] or ["gemm", "attn", "norm", "sample"]
    if "stamps" in which:
        for M, S in ((16, 1), (16, 4), (64, 1), (64, 4), (64, 8)):
            stamps_gemm(M, 4800, 1600, S, label="_qkv")
        for M, S in ((64, 1), (64, 6), (64, 16)):
            stamps_gemm(M, 1600, 1600, S, label="_proj")
        stamps_gemm(64, 50304, 1600, 1, label="_lmhead")
    H, F, V = 1600, 6400, 50304
    from llm_sharding_demo_amd.ops.hip import HipBackend
    R0 = HipBackend.R

    def route(**kw):  # bench_gemm's HipBackend() reads the class routing table (ops/routing.py)
        HipBackend.R = R0.replace(**kw)

    if "sweep" in which:
        for tgt in (128, 256, 384, 512, 768, 1024):
            route(sk_target=tgt)
            print("sk_target", tgt, flush=True)
            for M in (64, 128):
                bench_gemm(M, 3 * H, H, label="_qkv")
                bench_gemm(M, F, H, act=1, label="_fc")
                bench_gemm(M, H, H, resid=True, label="_proj")
                bench_gemm(M, H, F, resid=True, label="_proj2")
                bench_gemm(M, V, H, label="_lmhead")
        route()
    if "rows" in which:  # decode GEMM: row blocks x split target at M = 128
        for rows in (128, 64):
            for tgt in (256, 384, 512):
                route(sk_rows=rows, sk_target=tgt)
                tag = f"_r{rows}_t{tgt}"
                bench_gemm(128, 3 * H, H, label="_qkv" + tag)
                bench_gemm(128, F, H, act=1, label="_fc" + tag)
                bench_gemm(128, H, H, resid=True, label="_proj" + tag)
                bench_gemm(128, H, F, resid=True, label="_proj2" + tag)
                bench_gemm(128, V, H, label="_lmhead" + tag)
        route()
    if "layer" in which:
        for M in (1, 16, 64, 128):
            bench_decode_layer(M)
    if "lmhead" in which:  # vocab projection: decode kernel vs 128x128 tiled kernel
        for M in (16, 32, 64, 128):
            bench_gemm(M, V, H, label="_lmhead")
            bench_gemm(M, V, H, label="_lmhead_tiled", force_tiled=True)
        bench_gemm(128, 128256, 4096, label="_lmhead_llama")
        bench_gemm(128, 128256, 4096, label="_lmhead_llama_tiled", force_tiled=True)
    if "fc256" in which:  # one shape for PMC passes: MLP-up at 256 rows, ring / dbuf / split-K
        for t3 in (1 << 30, 0):
            route(tiled3_max=t3)
            bench_gemm(256, F, H, act=1, label="_fc_tiled" + ("_ring3" if t3 else "_dbuf"), force_tiled=True)
        route(tiled_min_n=1 << 30, tiled_all_m=1 << 30)
        bench_gemm(256, F, H, act=1, label="_fc_sk")
        route()
    if "tiled3" in which:  # 128x128 kernel: double buffer vs 3-slot LDS ring, decode-sized M
        for M in (128, 256):
            for t3, slots, rtn in ((0, 3, 128), (1 << 30, 3, 128), (1 << 30, 4, 128), (1 << 30, 3, 64)):
                route(tiled3_max=t3, ring_slots=slots, ring_tn=rtn)
                tag = (f"_ring{slots}" + ("_n64" if rtn == 64 else "")) if t3 else "_dbuf"
                if M == 128:
                    bench_gemm(M, V, H, label="_lmhead" + tag, force_tiled=True)
                bench_gemm(M, 3 * H, H, label="_qkv_tiled" + tag, force_tiled=True)
                bench_gemm(M, F, H, act=1, label="_fc_tiled" + tag, force_tiled=True)
                bench_gemm(M, H, F, resid=True, label="_proj2_tiled" + tag, force_tiled=True)
            route(tiled_min_n=1 << 30, tiled_all_m=1 << 30, ring_tn=128)
            bench_gemm(M, 3 * H, H, label="_qkv_sk")
            bench_gemm(M, F, H, act=1, label="_fc_sk")
            bench_gemm(M, H, F, resid=True, label="_proj2_sk")
            route()
    if "tiledsk" in which:  # split-K slabs + norm combine: decode kernel vs 128x128 tiled
        for M in (64, 128):
            for (N, K, nm) in ((3 * H, H, "qkv"), (F, H, "fc"), (H, H, "proj"), (H, F, "proj2")):
                bench_gemm(M, N, K, resid=True, label=f"_resid_{nm}")
                bench_gemm(M, N, K, resid=True, label=f"_resid_{nm}_tiled", force_tiled=True)
    if "gemm" in which:
        for M in (1, 16, 32, 64, 128, 256):
            bench_gemm(M, 3 * H, H, label="_qkv")
            bench_gemm(M, F, H, act=1, label="_fc")
            bench_gemm(M, H, H, resid=True, label="_proj")
            bench_gemm(M, H, F, resid=True, label="_proj2")
        for M in (1, 64):
            bench_gemm(M, V, H, act=0, label="_lmhead")
        bench_gemm(8192, 3 * H, H, label="_prefill_qkv")
    if "resid" in which:
        for M in (64, 128):
            bench_resid_norm(M, H, H, (4, 6, 8, 12, 16), label="_proj")
            bench_resid_norm(M, H, F, (4, 6, 8, 12, 16, 25), label="_proj2")
    if "prefill" in which:
        bench_prefill_gemms(8192, H, F, 25, 64)
        bench_prefill_gemms(4096, 4096, 14336, 32, 128, label="_llama")
    if "attn" in which:
        for B in (1, 16, 64, 128):
            bench_attn_decode(B, 25, 25, 64, 192)
        bench_attn_decode(64, 25, 25, 64, 1024)
        bench_attn_decode(64, 32, 8, 128, 512)
        bench_attn_prefill(64, 128, 25, 25, 64)
        bench_attn_prefill(4, 1024, 25, 25, 64)
        bench_attn_prefill(4, 1024, 32, 8, 128)
    if "norm" in which:
        for s in (0, 4, 8):
            bench_norm(64, H, s)
            bench_norm(128, H, s)
    if "pgroup" in which:  # prefill GEMM tile order: row-panel groups
        for G in (0, 4, 8, 16, 32):
            C.gemm_set_big_group(G)
            bench_prefill_gemms(65536, 1600, 6400, 25, 64, label=f"_xl_G{G}")
        C.gemm_set_big_group(0)
    if "p8" in which:  # large-GEMM kernel: BK=32 ring (0) vs phase-pipelined BK=64 (1)
        for kind in (0, 1):
            C.gemm_set_big_kind(kind)
            bench_prefill_gemms(65536, 1600, 6400, 25, 64, label=f"_xl_kind{kind}")
        C.gemm_set_big_kind(1)
    if "tn32" in which:
        for M in (128, 256):
            bench_ring_tn(M)
    if "corun" in which:
        bench_corun()
    if "p8stamps" in which:
        stamps_p8()
        stamps_p8(N=1600, K=6400, act=0)
    if "p8prof" in which:  # LSD_P8_PROF build: loop cycles split into vmcnt waits and the two barriers
        stamps_p8(act=0)
        stamps_p8(M=4096, N=4096, K=4096, act=0)
    if "normwave" in which:  # prefill norms: block per row vs wave per row
        for T, H in ((8192, 1600), (32768, 1600), (65536, 1600), (8192, 4096), (32768, 768)):
            for wmin in (0, 1):
                C.norm_set_wave_min(wmin)
                bench_norm(T, H, 0)
                print(json.dumps({"norm_wave": wmin}), flush=True)
        C.norm_set_wave_min(0)
    if "lmsample" in which:  # lm_head + sampler, segment maxima on / off
        bench_lmhead_sample(256, 50257, 1600)
        bench_lmhead_sample(256, 50257, 768)
        bench_lmhead_sample(128, 50257, 1600)
        bench_lmhead_sample(256, 128256, 4096)
    if "lmk" in which:
        for M in (256, 512):
            bench_lmhead_kinds(M)
        bench_lmhead_kinds(256, 128256, 4096)
    if "attnm" in which:  # grouped-query decode: MFMA kernel vs VALU kernel
        for B, ctx in ((256, 160), (256, 192), (128, 192), (512, 192), (64, 1024)):
            for mm in (256, 0):
                C.attn_set_mfma_min(mm)
                print("mfma_min", mm, flush=True)
                bench_attn_decode(B, 32, 8, 128, ctx)
        C.attn_set_mfma_min(256)
    if "attnlong" in which:  # long-context grouped-query decode: split MFMA vs VALU
        from llm_sharding_demo_amd.ops.hip import HipBackend
        for B, ctx in ((32, 4224), (8, 8128), (16, 4096), (64, 2048), (32, 320), (4, 8128), (1, 8128)):
            pol = HipBackend.decode_attn_splits(B, 32, 8, 128, ctx)
            print("policy splits", pol, flush=True)
            bench_attn_decode(B, 32, 8, 128, ctx, splits=pol)
            C.attn_set_mfma_min(1 << 30)
            print("VALU (old policy)", flush=True)
            bench_attn_decode(B, 32, 8, 128, ctx)
            C.attn_set_mfma_min(1)
            for sp in (2, 4, 8, 16, 32):
                if sp != pol and B * 8 * sp <= 8192 and ctx // sp >= 128:
                    print("mfma splits", sp, flush=True)
                    bench_attn_decode(B, 32, 8, 128, ctx, splits=sp)
            C.attn_set_mfma_min(256)
    if "attnss" in which:  # single-stream grouped-query decode: VALU vs MFMA over context splits
        for ctx in (192, 320, 1024):
            C.attn_set_mfma_min(1 << 30)
            print("VALU (policy splits)", flush=True)
            bench_attn_decode(1, 32, 8, 128, ctx, splits=HipBackendSplits(1, 32, 8, 128, ctx))
            for sp in (2, 4):
                print("VALU splits", sp, flush=True)
                bench_attn_decode(1, 32, 8, 128, ctx, splits=sp)
            C.attn_set_mfma_min(1)
            for sp in (1, 2, 4, 6, 8, 16):
                if ctx // sp >= 16:
                    print("mfma splits", sp, flush=True)
                    bench_attn_decode(1, 32, 8, 128, ctx, splits=sp)
            C.attn_set_mfma_min(256)
    if "attnw" in which:  # full-batch decode attention: 4 vs 8 waves per block
        for hd, nh, nkv in ((128, 32, 8), (64, 25, 25)):
            for B, ctx in ((256, 160), (256, 192), (128, 192), (512, 192)):
                for wv in (4, 8):
                    C.attn_set_large_waves(hd, wv)
                    print("waves", wv, flush=True)
                    bench_attn_decode(B, nh, nkv, hd, ctx)
            C.attn_set_large_waves(hd, 4)
    if "llamak" in which:
        for M in (256, 128):
            bench_llama_decode_kinds(M)
    if "llamask" in which:
        for M in (256, 128):
            bench_llama_sk(M)
    if "sample" in which:
        for B in (1, 64, 256):
            for g in (True, False):
                bench_sample(B, 50257, g)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/microbench.json", "w") as f:
        json.dump(RESULTS, f, indent=1)


if __name__ == "__main__":
    main()
