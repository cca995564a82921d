"""HIP backend: the engine ops on the hand-written gfx950 kernels (_C.so).

There is no fallback: constructing `HipBackend` without the built extension
raises, so a GPU run can never silently execute eager PyTorch math.

Device weight layout (set up once per stage by `prepare_stage`):
  * lm_head rows padded to a multiple of 64 (50257 -> 50304) so the logits
    GEMM tiles evenly; padded logits are never sampled (sampler scans < V).
  * Llama q/k projection rows re-ordered per head so RoPE pairs (i, i+hd/2)
    become adjacent columns (2i, 2i+1): the QKV epilogue then rotates with one
    lane exchange.  Q.K is invariant to a common permutation of head dims, so
    q and the K cache simply live in that order.
  * Llama gate/up rows interleaved in 16-row blocks so one wave holds the gate
    and up value of the same output column (silu(gate)*up fused epilogue).
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch

from . import Backend, Residual
from .routing import Routing

_C = None
_ERR: Optional[BaseException] = None


def _load():
    global _C, _ERR
    if _C is not None:
        return _C
    try:
        from .. import _C as ext  # built in-tree by ops/build.py
    except ImportError as e:  # pragma: no cover
        _ERR = e
        raise RuntimeError(
            "llm_sharding_demo_amd._C (the gfx950 HIP kernels) is not built or failed to load; "
            "run `python -m llm_sharding_demo_amd.ops.build` (or __graft_entry__.build())") from e
    _C = ext
    return _C


def extension_loaded() -> bool:
    try:
        _load()
        return True
    except Exception:
        return False


def rope_pair_permutation(n_heads: int, hd: int) -> torch.Tensor:
    half = hd // 2
    per = []
    for i in range(half):
        per += [i, i + half]
    idx = torch.tensor(per)
    return torch.cat([h * hd + idx for h in range(n_heads)])


def interleave_gate_up(w: torch.Tensor, f: int, blk: int = 16) -> torch.Tensor:
    gate, up = w[:f], w[f:]
    h = w.shape[1]
    return torch.stack([gate.reshape(f // blk, blk, h), up.reshape(f // blk, blk, h)], 1).reshape(2 * f, h)


def rope_table(max_pos: int, hd: int, theta: float, device) -> torch.Tensor:
    inv = 1.0 / (theta ** (torch.arange(0, hd, 2, dtype=torch.float64) / hd))
    ang = torch.arange(max_pos, dtype=torch.float64)[:, None] * inv[None, :]
    return torch.stack([ang.cos(), ang.sin()], -1).float().contiguous().to(device)


def prefill_tiles(meta) -> torch.Tensor:
    """(sequence, query offset) of every 64-query tile of a packed batch."""
    qlens = meta.host_qlens
    tiles = [(i, off) for i, n in enumerate(qlens) for off in range(0, n, 64)]
    return torch.tensor(tiles, dtype=torch.int32).reshape(-1, 2)


class LazyNorm:
    """A norm whose output has not been materialised: at M <= GEMV_NORM_MAX_M
    rows the consuming GEMV (csrc/kernels/gemv.hip) normalises the fp32
    residual rows itself, so the separate norm launch disappears.  Any other
    consumer materialises it through the norm kernel."""

    __slots__ = ("x", "w", "b", "eps", "rms")

    def __init__(self, x, w, b, eps, rms):
        self.x, self.w, self.b, self.eps, self.rms = x, w, b, eps, rms

    @property
    def shape(self):
        return self.x.shape

    @property
    def code(self) -> int:  # gemv norm code: 1 LayerNorm, 2 RMSNorm
        return 2 if self.rms else 1


# gemv epilogue codes (csrc/kernels/gemm.hip Epi)
_EPI = {"none": 0, "gelu": 1, "silu_mul": 2}
EPI_F32, EPI_RESID, EPI_QKV = 3, 4, 6
# longest row the sampler loads once into registers (sample.hip: CH x NT x 4)
SAMPLER_ONE_LOAD = 13 * 1024 * 4


class HipBackend(Backend):
    """The engine ops on the gfx950 kernels.  Every routing decision (which
    kernel, how many K splits) comes from one table, `R` (ops/routing.py;
    `LSD_ROUTING=field=value,...` overrides fields for A/B runs)."""

    name = "hip"
    R: Routing = Routing.from_env()

    def __init__(self):
        self.C = _load()
        R = self.R
        self.C.gemm_set_sk_rows(R.sk_rows)
        self.C.gemm_set_big_min(R.big_min_blocks)
        self.C.gemm_set_nw2_rows(1 << 30)
        self.C.gemm_set_tiled3_max(R.tiled3_max)
        self.C.gemm_set_ring_slots(R.ring_slots)
        self.C.gemm_set_ring_tn(R.ring_tn)
        self.C.gemm_set_ring_fill(R.ring_fill)
        self.C.gemm_set_ring_m96(0)
        self.C.gemm_set_d256_slots(R.d256_slots)
        self.C.gemm_set_ring8(R.ring8)
        self.C.gemm_set_ring8_flags(0)
        self.C.norm_set_wave_min(R.norm_wave_min)
        self.C.norm_set_wave_narrow_min(R.norm_wave_narrow_min)
        self.C.attn_set_max_wg(R.attn_max_wg)
        self.C.gemv_set_nt(R.gemv_nt)
        self.C.attn_set_small_waves(R.attn_small_waves)
        self.C.attn_set_small_waves128(R.attn_small_waves128)
        self.C.attn_set_large_waves(64, R.attn_large_waves)
        self.C.attn_set_large_waves(128, R.attn_large_waves)
        self.counters = None
        self._rope = None
        self.lane = 0  # microbatch lane (stream) currently being issued; see pipeline.py
        self.concurrency = 1  # microbatch lanes running at once (set per round by the pipeline)

    # ------------------------------------------------------------------
    def prepare_stage(self, stage) -> None:
        cfg, w, dev = stage.cfg, stage.w, stage.device
        if stage.last:
            # pad the head IN PLACE: the stage keeps one [vocab_padded, H]
            # tensor and its weight dict points at the first V rows (a
            # contiguous view -- the tied GPT-2 embedding of a 1-stage pipeline
            # reads the same rows), so the unpadded copy is freed
            key = "wte" if cfg.arch == "gpt2" else "lm_head"
            head = w[key]
            if head.shape[0] == cfg.vocab_padded:
                stage._lm_head_padded = head
            else:
                pad = torch.zeros(cfg.vocab_padded, cfg.hidden, dtype=head.dtype, device=dev)
                pad[: cfg.vocab_size] = head
                w[key] = pad[: cfg.vocab_size]
                del head
                stage._lm_head_padded = pad
        if cfg.arch == "llama":
            perm_q = rope_pair_permutation(cfg.n_heads, cfg.head_dim)
            perm_k = rope_pair_permutation(cfg.n_kv_heads, cfg.head_dim) + cfg.q_size
            keep = torch.arange(cfg.q_size + cfg.kv_size, cfg.qkv_size)
            perm = torch.cat([perm_q, perm_k, keep]).to(dev)
            for i in stage.layers:  # a boundary layer may hold only one half here
                p = f"layers.{i}."
                if p + "self_attn.qkv.weight" in w:
                    w[p + "self_attn.qkv.weight"] = w[p + "self_attn.qkv.weight"].index_select(0, perm).contiguous()
                if p + "mlp.gate_up.weight" in w:
                    w[p + "mlp.gate_up.weight"] = interleave_gate_up(w[p + "mlp.gate_up.weight"], cfg.ffn).contiguous()
            stage._rope = rope_table(stage.max_seq, cfg.head_dim, cfg.rope_theta, dev)
        else:
            stage._rope = None
        self._rope = getattr(stage, "_rope", None)
        # split-K ticket counters: zero at rest, re-armed by each tile's last
        # arriver; one row per microbatch lane so concurrent lanes never share one
        self._counters = torch.zeros(8, 1 << 16, dtype=torch.int32, device=dev)
        stage._hip_prepared = True

    @property
    def counters(self):
        return None if self._counters is None else self._counters[self.lane % 8]

    @counters.setter
    def counters(self, value):
        self._counters = None if value is None else value.reshape(-1, 1 << 16)

    # ------------------------------------------------------------------
    # routing (ops/routing.py): this forward's phase and lane count applied
    @classmethod
    def _tiled(cls, M: int, N: int = 0) -> bool:
        return cls.R.tiled(M, N)

    @property
    def _decode(self) -> bool:
        return getattr(self, "decode", True)

    def _gemm_kw(self, M: int, N: int, K: int, nw: int = 1):
        return self.R.gemm_kw(M, N, K, self.concurrency, nw)

    def _resid_splits(self, M: int, N: int, K: int) -> int:
        return self.R.resid_splits(M, N, K, self._decode, getattr(self, "concurrency", 1))

    @classmethod
    def decode_attn_splits(cls, B: int, nh: int, n_kv: int, hd: int, max_ctx: int) -> int:
        return cls.R.attn_splits(B, nh, n_kv, hd, max_ctx)

    # ------------------------------------------------------------------
    def embed(self, ids, pos, wte, wpe):
        return self.C.embed(ids, pos, wte, wpe)

    def _norm(self, r: Residual, w, b, eps, rms: bool):
        if not r.pending and r.x.shape[0] <= self.R.gemv_norm_max_m and r.x.shape[1] % 8 == 0:
            return LazyNorm(r.x, w, b, eps, rms)
        self._flush_extra(r)
        slab, pb = (r.pending[0] if r.pending else (None, None))
        out = self.C.norm(r.x, slab, pb, w, b, eps, rms, None, True)
        r.pending.clear()
        return out

    def _flush_extra(self, r: Residual) -> None:
        while len(r.pending) > 1:
            slab, pb = r.pending.pop(0)
            self.C.norm(r.x, slab, pb, None, None, 0.0, True, None, False)

    def flush(self, r: Residual):
        for slab, pb in r.pending:
            self.C.norm(r.x, slab, pb, None, None, 0.0, True, None, False)
        r.pending.clear()
        return r.x

    def layernorm(self, r, w, b, eps):
        return self._norm(r, w, b, eps, False)

    def rmsnorm(self, r, w, eps):
        return self._norm(r, w, None, eps, True)

    def norm_rows(self, x, w, b, eps, rms: bool, rows=None):
        if rows is None and x.shape[0] <= self.R.gemv_norm_max_m and x.shape[1] % 8 == 0:
            return LazyNorm(x, w, b, eps, rms)
        return self.C.norm(x, None, None, w, b, eps, rms, rows, True)

    def materialize(self, xn):
        if isinstance(xn, LazyNorm):
            return self.C.norm(xn.x, None, None, xn.w, xn.b, xn.eps, xn.rms, None, True)
        return xn

    def _gemv_in(self, xn, K: int, epi: int):
        """(x, norm code, gamma, beta, eps) for a GEMV launch, or None when this
        GEMM does not run on the GEMV (the caller takes the MFMA path)."""
        M = xn.shape[0]
        if M > self.R.gemv_max_m:
            return None
        if isinstance(xn, LazyNorm):
            if self.C.gemv_ok(M, K, epi, xn.code):
                return xn.x, xn.code, xn.w, xn.b, xn.eps
            xn = self.materialize(xn)
        if self.C.gemv_ok(M, K, epi, 0):
            return xn, 0, None, None, 0.0
        return None

    def qkv_kv_append(self, xn, w, b, cache_k, cache_v, meta, mcfg):
        g = self._gemv_in(xn, w.shape[1], EPI_QKV)
        if g is not None:
            x, nc, gw, gb, eps = g
            return self.C.gemv(x, w, b, EPI_QKV, nc, gw, gb, eps, None, cache_k, cache_v,
                               meta.token_slots, meta.token_pos, mcfg.q_size, mcfg.kv_size,
                               mcfg.head_dim, self._rope)
        xn = self.materialize(xn)
        if self.R.blaslt_qkv(xn.shape[0], w.shape[1], getattr(self, "decode", False)) and xn.is_contiguous():
            y = self.C.blaslt_f32(xn, w, self.lane)
            if y is not None:
                return self.C.qkv_post(y, b, cache_k, cache_v, meta.token_slots, meta.token_pos,
                                       mcfg.q_size, mcfg.kv_size, mcfg.head_dim, self._rope)
        tiled, splits = self._gemm_kw(xn.shape[0], w.shape[0], w.shape[1])
        return self.C.linear_qkv(xn, w, b, cache_k, cache_v, meta.token_slots, meta.token_pos,
                                 mcfg.q_size, mcfg.kv_size, mcfg.head_dim, self._rope,
                                 tiled, splits, self.counters)

    def attention(self, q, cache_k, cache_v, meta):
        n_kv, hd = cache_k.shape[1], cache_k.shape[3]
        nh = q.shape[1] // hd
        if meta.is_decode:
            splits = self.decode_attn_splits(meta.num_seqs, nh, n_kv, hd, meta.max_ctx)
            return self.C.attn_decode(q, cache_k, cache_v, meta.seq_slots, meta.token_pos, nh, splits)
        tiles = getattr(meta, "_tiles", None)
        if tiles is None:
            tiles = prefill_tiles(meta).to(q.device)
            meta._tiles = tiles
        return self.C.attn_prefill(q, cache_k, cache_v, tiles, meta.seq_slots, meta.q_start,
                                   meta.cu_q, nh)

    def linear(self, a, w, b=None, act: str = "none"):
        code = _EPI[act]
        g = self._gemv_in(a, w.shape[1], code)
        if g is not None:
            x, nc, gw, gb, eps = g
            return self.C.gemv(x, w, b, code, nc, gw, gb, eps, None, None, None, None, None,
                               0, 0, 0, None)
        a = self.materialize(a)
        dec = getattr(self, "decode", False)
        if code == 1 and self.R.blaslt_gelu(a.shape[0], dec) and a.is_contiguous():
            y = self.C.blaslt_linear(a, w, b, code, self.lane)
            if y is not None:
                return y
        if code == 2 and self.R.blaslt_silu(a.shape[0], w.shape[0], dec) and a.is_contiguous():
            y = self.C.blaslt_linear(a, w, b, 0, self.lane)
            if y is not None:
                return self.C.silu_mul(y)
        tiled, splits = self._gemm_kw(a.shape[0], w.shape[0], w.shape[1], 2 if code == 2 else 1)
        return self.C.linear(a, w, b, code, tiled, splits, self.counters)

    def linear_residual(self, a, w, b, r: Residual) -> None:
        M, K = a.shape
        N = w.shape[0]
        if self._gemv_in(a, K, EPI_RESID) is not None:  # adds straight into r.x
            self.C.gemv(a, w, b, EPI_RESID, 0, None, None, 0.0, r.x, None, None, None, None,
                        0, 0, 0, None)
            return
        if self.R.blaslt_resid(M, K, self._decode) and a.is_contiguous() \
                and self.C.blaslt_residual(a, w, b, r.x, self.lane):
            return
        splits = self._resid_splits(M, N, K)
        tiled = self._tiled(M, N)
        # decode split-K: hand the S partial slabs to the next norm (which
        # reads the rows anyway) instead of a last-arriver reduce in the GEMM
        defer = bool(self.R.defer_resid) and not tiled and splits > 1
        slab = self.C.linear_residual(a, w, b, r.x, splits, tiled, self.counters, defer)
        if slab is not None:
            r.pending.append((slab, b))

    def logits(self, xn, w):
        g = self._gemv_in(xn, w.shape[1], EPI_F32)
        if g is not None:
            x, nc, gw, gb, eps = g
            if not (self.R.segmax and w.shape[0] % 8 == 0 and w.shape[0] > SAMPLER_ONE_LOAD):
                return self.C.gemv(x, w, None, EPI_F32, nc, gw, gb, eps, None, None, None, None,
                                   None, 0, 0, 0, None)
            # one GEMV workgroup = one 8-logit segment: its epilogue writes the
            # segment maxima too, so the single-stream sampler reads ~100
            # candidate segments instead of three passes over a row too long
            # for its one-load path (Llama-3's 128 K vocabulary: sampler 36.4 ->
            # 20.2 us; GPT-2's 50 K rows load once and stay faster without:
            # 15.5 vs 17.2 us; profiles/r6_*_b1_kernel_stats_v2.csv)
            seg = torch.empty(x.shape[0], w.shape[0] // 8, dtype=torch.float32, device=x.device)
            out = self.C.gemv_logits(x, w, nc, gw, gb, eps, seg)
            out._lsd_segmax = seg
            return out
        xn = self.materialize(xn)
        tiled, splits = self.R.logits_kw(xn.shape[0], w.shape[0], w.shape[1], self.concurrency)
        if not (self.R.segmax and tiled and w.shape[0] % 8 == 0):
            return self.C.linear_f32(xn, w, tiled, splits, self.counters)
        # the epilogue also writes each 8-logit segment's maximum; the sampler
        # derives its top-k threshold from them and reads only the segments
        # that reach it (attached to the logits: a slice drops it, and the
        # sampler then scans the full rows)
        seg = torch.empty(xn.shape[0], w.shape[0] // 8, dtype=torch.float32, device=xn.device)
        out = self.C.linear_f32(xn, w, tiled, splits, self.counters, seg)
        out._lsd_segmax = seg
        return out

    def sample(self, logits, samp, vocab: int):
        return self.C.sample(logits, vocab, samp.temperature, samp.top_k, samp.greedy,
                             samp.seeds, samp.step, getattr(logits, "_lsd_segmax", None))

    def sample_into(self, logits, samp, vocab: int, out, meta=None) -> None:
        # one kernel: draw into `out`, advance the per-row sampler counters
        # and (meta given) the decode batch's positions
        self.C.sample_into(logits, vocab, samp.temperature, samp.top_k, samp.greedy,
                           samp.seeds, samp.step, out, getattr(samp, "active", None),
                           meta.token_pos if meta is not None else None,
                           getattr(logits, "_lsd_segmax", None))

    def gather_rows(self, x, idx):
        return x.index_select(0, idx.long())
