"""Kernel routing of the HIP backend: which hand-written kernel (and how many
K splits) every GEMM / norm / attention launch of a forward takes.

One frozen table (`Routing`) holds every tunable with its measured default
and the profile that set it; the decisions are pure functions of the launch
shape and the forward's phase (decode vs prefill, concurrent microbatch
lanes), so `tests/test_routing.py` pins the whole table per (model, GEMM,
rows) on CPU.  Defaults are the production configuration; an A/B run
overrides fields with ONE variable:

    LSD_ROUTING="ring8=0,sk_target=256"      (field=value, comma-separated)

hipBLASLt (csrc/blaslt.cpp) is not on the default hot path: every GEMM runs
on the gfx950 kernels of csrc/kernels.  `blaslt=1` turns the library routes
on for A/B comparisons (the library as an oracle for the hand-written
prefill GEMMs); its thresholds are the `blaslt_*` fields.

Reference: the block's projections these route are `/root/reference/server.py:84-85,99-100`
(GPT2Block c_attn / c_proj / c_fc / c_proj) and the head `server.py:102`.
"""
from __future__ import annotations

import dataclasses
import math
import os
from dataclasses import dataclass


@dataclass(frozen=True)
class Routing:
    # -- single stream / small batches ------------------------------------
    # decode GEMMs of <= gemv_max_m rows on the weight-streaming GEMV
    # (gemv.hip, fused epilogues); <= gemv_norm_max_m rows also fold the
    # preceding LayerNorm / RMSNorm into its prologue (0 disables)
    gemv_max_m: int = 8
    gemv_norm_max_m: int = 2
    gemv_nt: int = 0  # non-temporal weight loads in the GEMV (A/B)
    # -- decode attention --------------------------------------------------
    target_blocks: int = 512  # >> 256 CUs: VALU decode attention splits the context up to this
    split_keys: int = 256      # ... with at least this many keys per split (64 / 128 lose at 1-16
    #                            sequences: the combine launch costs more, r6_split_keys.log)
    # grouped-query decode attention on MFMA (attn_decode_mfma_kernel) at >=
    # attn_mfma_min waves; fewer than attn_mfma_split_below items split the
    # context towards attn_mfma_waves waves, >= 512 keys per split (Llama-3
    # 8B, 2K-8K contexts: 1.3-1.45x the VALU kernel; profiles/r2_long_context.log)
    attn_mfma_min: int = 256
    attn_mfma_split_below: int = 1024
    attn_mfma_waves: int = 1024
    attn_small_waves: int = 8  # waves per small-batch VALU attention block
    # ... for 128-dim heads: 88 = 8 waves with 8 keys per wave in flight (a 256-key
    # context in one round of loads; Llama-3 8B single stream -0.6 %, r6_attn_u8.log)
    attn_small_waves128: int = 88
    # full-batch block: 4 waves; 8 waves 10 % slower (r4_attn_large_waves.log); 42 = 4 waves with 2
    # keys per wave in flight and 2 = 2-wave blocks: faster alone at <= 192 keys, slower in the
    # two-lane bench (XL p50 8.44 -> 8.58-8.63 ms; r6_attn_ab.log)
    attn_large_waves: int = 4
    attn_max_wg: int = 0       # cap the attention grid (A/B; 0 = none)
    # -- decode GEMMs ------------------------------------------------------
    # split-K (last-arriver) kernel up to sk_max_m rows; tiled above
    # tiled_all_m rows at any width, above tiled_min_m rows when >=
    # tiled_min_n wide (GPT-2 XL 2 x 256: split-K 41.2k, all tiled 46.3k tok/s;
    # profiles/r1_ab_tiled_min_n.log, r1_ab_ring_n64.log)
    sk_max_m: int = 256
    tiled_all_m: int = 128
    tiled_min_m: int = 64
    tiled_min_n: int = 4000
    # short-K GEMMs (GPT-2 small K = 768) tiled at any row count above the
    # GEMV: QKV 9.9-15.7 -> 7.6-8.0 us at 8-128 rows (profiles/r5_small_k_routing.log)
    tiled_short_k: int = 1024
    # split-K workgroup target (0: 384 / concurrent lanes) and the k-steps
    # per split; row blocks of sk_rows when the grid is under-filled
    sk_target: int = 0
    sk_min_steps: int = 2
    sk_rows: int = 64
    defer_resid: int = 1  # residual split-K partials as slabs folded by the next norm
    # LDS ring kernels: grids of <= tiled3_max 128x64 tiles (QKV at 256 rows
    # 25.8 -> 20.4 us; profiles/r1_ab_ring_n64.log), ring depth, tile columns
    # (0 = auto: 32-wide below ring_fill 64-wide workgroups; r2_ring_tn32.log)
    tiled3_max: int = 512
    ring_slots: int = 3
    ring_tn: int = 0
    ring_fill: int = 128
    # 8-wave 128x64 ring (2 = 8 computing waves): QKV 16.7 -> 15.2 us at 256
    # rows, bench 48.9k -> 49.7k tok/s (profiles/r3_ring8_ab.log)
    ring8: int = 2
    # residual projections: ring K-split target, 257-1024-row 128x128-tile
    # target (Llama-3 8B down at 512 rows 119.7 -> 81.5 us; r2_resid512_splits.log),
    # 8 splits for K >= 8192 above resid_longk_min_m rows (down at 256 rows 71.9 -> 55.3 us)
    ring_resid_target: int = 256
    resid_wg_target: int = 1024
    resid_longk: int = 1
    resid_longk_min_m: int = 128
    # K per split of a short-K (<= tiled_short_k) residual projection on the
    # ring: GPT-2 small out-proj (K 768) runs unsplit on 24 workgroups at 512
    resid_short_k_per_split: int = 384
    # 129-256-row long-K GEMMs on the 8-wave all-rows kernel (gemm_d256):
    # Llama-3 8B gate/up at 256 rows 84.6 -> 69.0 us (profiles/r3_d256_ab.log)
    d256: int = 1
    d256_min_k: int = 4096
    d256_slots: int = 3
    d256_target: int = 192
    # ... and over 256-row blocks up to d256_rb_max_m rows for long-K GEMMs at
    # most d256_rb_max_n wide: Llama-3 8B QKV at 512 rows 54.6 (8-wave ring)
    # -> 45.2 us (128-wide tiles, 2 K splits; the 28672-wide gate_up stays on
    # the 256x256 kernel: 120 vs 145 us; profiles/r6_llama512_gemm.log)
    d256_rb_max_m: int = 512
    d256_rb_max_n: int = 8192
    # the 256x256 pipelined kernel (gemm_p8) once a tiled launch has this
    # many 256x256 tiles; the 128x128 kernels below (launch_tiled in gemm.hip)
    big_min_blocks: int = 160
    # -- norms / head ------------------------------------------------------
    # one wave per row from norm_wave_min rows (prefill 32 K x 1600 97.7 ->
    # 53.7 us; r5_normwave.log) and from norm_wave_narrow_min rows when H <=
    # 1024 (GPT-2 small decode +0.9 %; r5_normwave_decode.log)
    norm_wave_min: int = 4096
    norm_wave_narrow_min: int = 256
    segmax: int = 1  # lm_head epilogue writes 8-logit segment maxima for the sampler
    # -- hipBLASLt A/B oracle (off: hand-written kernels only) ---------------
    blaslt: int = 0
    blaslt_min_m: int = 4096             # prefill routes at >= this many rows
    blaslt_resid_min_k: int = 4096       # residual projections with K >= this
    blaslt_gelu_min_m: int = 65536       # prefill MLP-up bias + GELU
    blaslt_decode_gelu_min_m: int = 384  # decode MLP-up bias + GELU
    blaslt_silu_min_m: int = 64          # decode gate_up + SiLU*up pass
    blaslt_silu_max_m: int = 128
    blaslt_qkv_min_m: int = 512          # decode QKV (fp32) + RoPE / cache-append pass
    blaslt_qkv_min_k: int = 4096

    @classmethod
    def from_env(cls, spec: str | None = None) -> "Routing":
        spec = os.environ.get("LSD_ROUTING", "") if spec is None else spec
        kw = {}
        names = {f.name for f in dataclasses.fields(cls)}
        for item in filter(None, (s.strip() for s in spec.split(","))):
            k, _, v = item.partition("=")
            k = k.strip()
            if k not in names:
                raise ValueError(f"LSD_ROUTING: unknown field {k!r}")
            kw[k] = int(v, 0)
        return cls(**kw)

    def replace(self, **kw) -> "Routing":
        return dataclasses.replace(self, **kw)

    # ------------------------------------------------------------------
    # decode GEMM decisions (decode: the forward is a decode step; lanes:
    # microbatch lanes running concurrently)
    # ------------------------------------------------------------------
    def tiled(self, M: int, N: int = 0) -> bool:
        return (M > self.sk_max_m or M > self.tiled_all_m
                or (M > self.tiled_min_m and N >= self.tiled_min_n))

    def d256_bn(self, M: int, N: int, K: int) -> int:
        """Tile columns when this GEMM runs on gemm_d256_kernel, else 0
        (mirrors d256_bn() in gemm.hip)."""
        if not self.d256 or K % 64 or N > 32768 or not self.tiled(M, N):
            return 0
        if 256 < M <= self.d256_rb_max_m:  # several 256-row blocks (auto only)
            if self.d256 != 1 or K < self.d256_min_k or N > self.d256_rb_max_n:
                return 0
            return 128 if N % 128 == 0 else 64
        if not (128 < M <= 256):
            return 0
        if self.d256 == 1:  # auto: long-K GEMMs; 128-wide tiles when they alone fill the chip
            if K < self.d256_min_k:
                return 0
            return 128 if N % 128 == 0 and N // 128 >= 128 else 64
        return 128 if self.d256 == 128 and N % 128 == 0 else 64

    @staticmethod
    def d256_kind(bn: int) -> int:  # lsd_gemm launch kind of gemm_d256
        return 3 if bn == 128 else 2

    @staticmethod
    def d256_splits(N: int, K: int, bn: int, target: int, M: int = 256) -> int:
        tiles = math.ceil(N / bn) * math.ceil(M / 256)  # column tiles x 256-row blocks
        return max(1, min(round(target / tiles), K // 64 // 2 or 1, 16))

    def sk_splits(self, M: int, N: int, K: int, lanes: int = 1, nw: int = 1) -> int:
        """nw: 64-column tiles per workgroup (2 for SiLU*up: sk_nw() in gemm.hip)."""
        tiles = math.ceil(N / (64 * nw))  # >= the target: never row-blocked
        target = self.sk_target or max(128, 384 // max(1, lanes))
        return max(1, min(math.ceil(target / tiles), K // 32 // self.sk_min_steps or 1))

    def gemm_kw(self, M: int, N: int, K: int, lanes: int = 1, nw: int = 1):
        """(tiled kind, K splits) of a non-residual GEMM (QKV, MLP-up,
        gate_up, lm_head below vocab width)."""
        bn = self.d256_bn(M, N, K)
        if bn:
            return self.d256_kind(bn), self.d256_splits(N, K, bn, self.d256_target, M)
        if self.tiled(M, N) or (K <= self.tiled_short_k and M <= self.sk_max_m and K % 64 == 0):
            return True, 1
        return False, self.sk_splits(M, N, K, lanes, nw)

    def resid_splits(self, M: int, N: int, K: int, decode: bool = True, lanes: int = 1) -> int:
        """K splits of a residual projection (x += a w^T + b)."""
        if self.tiled(M, N):
            if M <= self.sk_max_m and self.tiled3_max and self.ring_tn in (0, 32, 64):
                # decode rows on the 128x64 ring: as many splits as keep the
                # grid on the ring kernel, at most one per 512 of K (GPT-2 XL
                # out-proj: 3 splits 11.8 us vs 5 splits 12.6 at 256 rows)
                if M > self.resid_longk_min_m and K >= 8192 and self.resid_longk:
                    return min(8, K // 1024)  # leaves the ring for the 128x128 kernel
                tiles = math.ceil(M / 128) * math.ceil(N / 64)
                target = min(self.tiled3_max, self.ring_resid_target or self.tiled3_max)
                kps = self.resid_short_k_per_split if K <= self.tiled_short_k else 512
                return max(1, min(target // tiles, K // kps or 1))
            tiles = math.ceil(M / 128) * math.ceil(N / 128)
            if M <= 1024 and self.resid_wg_target and decode:
                # decode groups of 257-1024 rows: ~resid_wg_target 128x128
                # tiles, at most one split per 1024 of K (at least 2)
                return max(1, min(math.ceil(self.resid_wg_target / tiles), max(2, K // 1024),
                                  K // 64 // 2 or 1))
            return max(1, min(math.ceil(256 / tiles), K // 64 // 2 or 1))
        if self.defer_resid:
            # deferred slabs cost S x M x N x 4 B of writes + norm reads:
            # ~800 k per split, 4..8 splits (tools/microbench.py resid)
            return max(1, min(8, max(4, K // 800), K // 64))
        return self.sk_splits(M, N, K, lanes)

    def logits_kw(self, M: int, N: int, K: int, lanes: int = 1):
        """lm_head: the 128x128 LDS-tiled kernel at vocab width (fills the
        chip without split-K; 41.8 vs 64.2 us at 128 rows, GPT-2 XL)."""
        if N >= 16384 and K % 64 == 0:
            return True, 1
        return self.gemm_kw(M, N, K, lanes)

    # ------------------------------------------------------------------
    # hipBLASLt A/B routes (never taken unless blaslt=1)
    # ------------------------------------------------------------------
    def blaslt_prefill(self, M: int, decode: bool) -> bool:
        return bool(self.blaslt and self.blaslt_min_m) and M >= self.blaslt_min_m and not decode

    def blaslt_gelu(self, M: int, decode: bool) -> bool:
        if not self.blaslt:
            return False
        if decode:
            return bool(self.blaslt_decode_gelu_min_m) and M >= self.blaslt_decode_gelu_min_m
        return self.blaslt_prefill(M, decode) and M >= self.blaslt_gelu_min_m

    def blaslt_silu(self, M: int, N: int, decode: bool) -> bool:
        return (bool(self.blaslt and self.blaslt_silu_min_m) and decode
                and self.blaslt_silu_min_m <= M <= self.blaslt_silu_max_m and N % 32 == 0)

    def blaslt_qkv(self, M: int, K: int, decode: bool) -> bool:
        return (bool(self.blaslt and self.blaslt_qkv_min_m) and decode and M >= self.blaslt_qkv_min_m
                and K >= self.blaslt_qkv_min_k)

    def blaslt_resid(self, M: int, K: int, decode: bool) -> bool:
        return self.blaslt_prefill(M, decode) and K >= self.blaslt_resid_min_k

    # ------------------------------------------------------------------
    def attn_splits(self, B: int, nh: int, n_kv: int, hd: int, max_ctx: int) -> int:
        """Context splits of a decode attention launch (a graph-captured
        property: max_ctx is the captured context bucket)."""
        G, items = nh // n_kv, B * n_kv
        if hd == 128 and G in (2, 4, 8):
            ms = 1
            if items < self.attn_mfma_split_below:
                ms = max(1, min(math.ceil(self.attn_mfma_waves / items), math.ceil(max_ctx / 512), 256))
            if items * ms >= self.attn_mfma_min:
                return ms
        if items < self.target_blocks:
            return min(math.ceil(self.target_blocks / items), max(1, math.ceil(max_ctx / self.split_keys)))
        return 1


def route_table(model: str, rows, routing: Routing | None = None) -> dict:
    """{(gemm, rows, phase): route} of one model's projections: what
    `tests/test_routing.py` pins and `python -m llm_sharding_demo_amd.ops.routing`
    prints.  route = kernel family + K splits, no extension calls."""
    from ..config import get_model_config

    r = routing or Routing.from_env("")
    mc = get_model_config(model)
    H, F = mc.hidden, mc.ffn
    up_n = (2 if mc.arch == "llama" else 1) * F
    shapes = {"qkv": (mc.qkv_size, H, "gemm"), "o": (H, mc.q_size, "resid"),
              "up": (up_n, H, "gemm"), "down": (H, F, "resid"), "lm_head": (mc.vocab_padded, H, "logits")}
    out = {}
    for M in rows:
        for decode in ((True, False) if M >= 256 else (True,)):
            lanes = 2 if decode else 1
            for g, (N, K, kind) in shapes.items():
                if M <= r.gemv_max_m and decode:
                    route = "gemv"
                elif kind == "resid":
                    s = r.resid_splits(M, N, K, decode, lanes)
                    t = r.tiled(M, N)
                    route = f"{'tiled' if t else 'splitk-slab' if r.defer_resid and s > 1 else 'splitk'}/s{s}"
                else:
                    if kind == "logits":
                        t, s = r.logits_kw(M, N, K, lanes)
                    else:
                        t, s = r.gemm_kw(M, N, K, lanes, 2 if (g == "up" and mc.arch == "llama") else 1)
                    route = {False: "splitk", True: "tiled", 2: "d256-64", 3: "d256-128"}[t] + f"/s{s}"
                if r.blaslt and ((g == "up" and (r.blaslt_gelu(M, decode) and mc.arch == "gpt2"
                                                 or mc.arch == "llama" and r.blaslt_silu(M, N, decode)))
                                 or (g == "qkv" and r.blaslt_qkv(M, K, decode))
                                 or (kind == "resid" and r.blaslt_resid(M, K, decode))):
                    route = "hipblaslt"
                out[(g, M, "decode" if decode else "prefill")] = route
    return out


if __name__ == "__main__":
    import sys

    model = sys.argv[1] if len(sys.argv) > 1 else "gpt2-xl"
    rows = [1, 8, 64, 128, 256, 512, 32768, 65536]
    for (g, M, ph), route in sorted(route_table(model, rows).items(), key=lambda x: (x[0][1], x[0][2], x[0][0])):
        print(f"{model:12s} {ph:8s} {M:6d} {g:8s} {route}")
