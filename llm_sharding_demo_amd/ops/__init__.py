"""Op backends.

The model code (models/stage.py: the GPT-2 and Llama blocks of one pipeline
stage) is written once against the `Backend` interface below.  Two implementations exist:

* `ReferenceBackend` -- plain PyTorch in fp32 (ops/reference.py).  Used on CPU
  (tests, golden numerics, the tiny-gpt2 reference config).
* `HipBackend` (ops/hip.py) -- the hand-written CDNA4 kernels in
  csrc/kernels/*.hip, routed by one table (ops/routing.py).  Used for every
  tensor on a GPU; hipBLASLt only runs when an A/B run asks for it
  (LSD_ROUTING=blaslt=1).  There is no silent fallback: if the extension is
  missing on a GPU box, `get_backend` raises.

Residual stream convention: the residual `x` is fp32 [T, H].  GEMMs whose
epilogue is "add into the residual" may split K across workgroups; their
fp32 partial slabs are parked in `Residual.pending` and folded into `x` by the
next norm (or `flush`).  This keeps the reduction deterministic and costs no
extra kernel launch.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Tuple

import torch

from . import reference as ref


@dataclass
class Residual:
    x: torch.Tensor  # fp32 [T, H]
    pending: List[Tuple[torch.Tensor, Optional[torch.Tensor]]] = field(default_factory=list)


class Backend:
    name = "abstract"

    def prepare_stage(self, stage) -> None:  # optional weight re-layout
        pass


class ReferenceBackend(Backend):
    """fp32 PyTorch implementation of the engine ops (CPU golden path)."""

    name = "reference"

    def embed(self, ids, pos, wte, wpe):
        return ref.embed(ids, pos, wte, wpe)

    def _combine(self, r: Residual) -> None:
        for slabs, bias in r.pending:
            r.x += slabs.sum(0)
            if bias is not None:
                r.x += bias.float()
        r.pending.clear()

    def flush(self, r: Residual) -> torch.Tensor:
        self._combine(r)
        return r.x

    def layernorm(self, r: Residual, w, b, eps):
        self._combine(r)
        return ref.layernorm(r.x, w, b, eps)

    def rmsnorm(self, r: Residual, w, eps):
        self._combine(r)
        return ref.rmsnorm(r.x, w, eps)

    def norm_rows(self, x, w, b, eps, rms: bool, rows=None):
        if rows is not None:
            x = x.index_select(0, rows.long())
        return ref.rmsnorm(x, w, eps) if rms else ref.layernorm(x, w, b, eps)

    def qkv_kv_append(self, xn, w, b, cache_k, cache_v, meta, mcfg):
        """QKV projection; K,V appended to the cache at (slot, pos); returns q [T, nh, hd]."""
        y = ref.linear(xn, w, b)
        T = y.shape[0]
        hd = mcfg.head_dim
        q = y[:, : mcfg.q_size].reshape(T, mcfg.n_heads, hd)
        k = y[:, mcfg.q_size: mcfg.q_size + mcfg.kv_size].reshape(T, mcfg.n_kv_heads, hd)
        v = y[:, mcfg.q_size + mcfg.kv_size:].reshape(T, mcfg.n_kv_heads, hd)
        if mcfg.arch == "llama":
            q = ref.apply_rope(q, meta.token_pos.cpu(), mcfg.rope_theta)
            k = ref.apply_rope(k, meta.token_pos.cpu(), mcfg.rope_theta)
        ref.kv_append(cache_k, cache_v, k, v, meta.token_slots, meta.token_pos)
        return q

    def attention(self, q, cache_k, cache_v, meta):
        o = ref.attention(q, cache_k, cache_v, meta.seq_slots, meta.q_start, meta.cu_q)
        return o.reshape(o.shape[0], -1)

    def linear(self, a, w, b=None, act: str = "none"):
        y = ref.linear(a, w, b)
        if act == "gelu":
            y = ref.gelu_new(y)
        elif act == "silu_mul":
            f = y.shape[1] // 2
            y = ref.silu_mul(y[:, :f], y[:, f:])
        return y

    def linear_residual(self, a, w, b, r: Residual) -> None:
        self._combine(r)
        r.x += ref.linear(a, w, b)

    def logits(self, xn, w):
        return ref.linear(xn, w)

    def sample(self, logits, samp, vocab: int):
        return ref.sample(logits, samp.temperature, samp.top_k, samp.greedy,
                          samp.uniforms(), vocab)

    def sample_into(self, logits, samp, vocab: int, out, meta=None) -> None:
        """Decode step: sampled ids into `out`, then the sampler counters (and,
        given the decode `meta`, its positions) advance."""
        out.copy_(self.sample(logits, samp, vocab))
        samp.advance()
        if meta is not None:
            meta.advance()

    def gather_rows(self, x, idx):
        return x.index_select(0, idx.long())


_REFERENCE = ReferenceBackend()


def hip_available() -> bool:
    try:
        from . import hip  # noqa: F401
        return hip.extension_loaded()
    except Exception:  # pragma: no cover - depends on build
        return False


def get_backend(device) -> Backend:
    dev = torch.device(device)
    if dev.type == "cpu":
        return _REFERENCE
    from .hip import HipBackend  # raises loudly if the extension is missing

    return HipBackend()  # one per stage: owns that stage's split-K counters / tables
