"""One pipeline stage of a GPT-2 or Llama model.

Generalises the reference's two hard-wired shards (`server.py:51-105`):
  * ShardA (`server.py:68-86`): wte + wpe + blocks[0:split]   -> stage 0
  * ShardB (`server.py:90-103`): blocks[split:] + ln_f + lm_head -> stage P-1
to P stages with an arbitrary layer range each.  Differences by design:
  * a stage materialises only its own layers (quirk Q4),
  * the causal mask is explicit in the attention op (quirk Q3),
  * K/V are appended to the shard-local cache, so decode processes one token
    per sequence (quirk Q5),
  * the last stage computes lm_head for the last position of each sequence
    only (quirk Q6) unless `all_logits` is requested (compat /forward_b),
  * a stage boundary may fall between the attention and the MLP half of a
    layer (`units`, parallel/partition.py): unit 2i = attention half of layer
    i, unit 2i+1 = its MLP half.  Only the residual stream crosses either kind
    of boundary; the KV cache of layer i lives with its attention half.
"""
from __future__ import annotations

from typing import Dict, Optional, Sequence, Tuple

import torch

from ..config import ModelConfig
from ..ops import Residual, get_backend
from ..runtime.batch import BatchMeta
from ..runtime.kv_cache import KVCache
from .weights import layer_half, maybe_load


class StageModel:
    def __init__(self, cfg: ModelConfig, layer_start: int, layer_end: int, first: bool,
                 last: bool, device="cpu", dtype: Optional[torch.dtype] = None, seed: int = 0,
                 weights_path: Optional[str] = None, max_slots: int = 8, max_seq: int = 1024,
                 weights: Optional[Dict[str, torch.Tensor]] = None,
                 units: Optional[Tuple[int, int]] = None, backend=None,
                 variants: Optional[Sequence[Tuple[int, int]]] = None):
        self.cfg = cfg
        self.device = torch.device(device)
        if dtype is None:
            dtype = torch.float32 if self.device.type == "cpu" else torch.bfloat16
        self.dtype = dtype
        if units is None:
            units = (2 * layer_start, 2 * layer_end)
        ua, ub = units
        if not 0 <= ua <= ub <= 2 * cfg.n_layers:
            raise ValueError(f"unit range {units} outside [0, {2 * cfg.n_layers}]")
        self.unit_start, self.unit_end = ua, ub
        # alternating splits (parallel/partition.py make_alt_unit_plans): the
        # unit range run for even / odd microbatch groups, both inside `units`
        self.variants = [tuple(v) for v in variants] if variants else [(ua, ub)]
        if any(not (ua <= a <= b <= ub) for a, b in self.variants):
            raise ValueError(f"variant ranges {self.variants} outside the stage's units {units}")
        self.layer_start, self.layer_end = ua // 2, (ub + 1) // 2  # layers touched
        self.first, self.last = first, last
        self.layers = range(self.layer_start, self.layer_end)
        # layers whose attention half (and so whose KV cache) lives here
        self.kv_layers = [i for i in self.layers if ua <= 2 * i < ub]
        self._kv_index = {i: j for j, i in enumerate(self.kv_layers)}
        if weights is None:
            weights = maybe_load(cfg, weights_path, self.layers, first, last, seed, self.device, dtype,
                                 units=units)
        else:
            weights = {k: v.to(device=self.device, dtype=dtype).contiguous() for k, v in weights.items()
                       if self._owns(k)}
        self.w = weights
        self.max_seq = min(max_seq, cfg.max_positions)
        self.kv = KVCache(len(self.kv_layers), max_slots, cfg.n_kv_heads, self.max_seq,
                          cfg.head_dim, dtype, self.device)
        # `backend` overrides the device default: the fp32 golden model runs the
        # plain PyTorch ops (ops/reference.py) on the GPU (utils/golden.py)
        self.backend = backend if backend is not None else get_backend(self.device)
        self.backend.prepare_stage(self)

    def _owns(self, name: str) -> bool:
        """Is tensor `name` used by this stage (its units, embeddings, head)?"""
        lh = layer_half(name)
        if lh is None:
            emb = name in ("wte", "wpe", "embed_tokens")
            head = name in ("ln_f.weight", "ln_f.bias", "norm.weight", "lm_head") or (
                name == "wte" and self.cfg.tie_embeddings)
            return (emb and self.first) or (head and self.last)
        return self.unit_start <= 2 * lh[0] + lh[1] < self.unit_end

    # ------------------------------------------------------------------
    def _lw(self, i: int, name: str) -> torch.Tensor:
        p = "h." if self.cfg.arch == "gpt2" else "layers."
        return self.w[f"{p}{i}.{name}"]

    # [tf5.15] modeling_gpt2.py:262-309 GPT2Block.forward, split at the residual
    def _gpt2_attn(self, li: int, i: int, r: Residual, meta: BatchMeta) -> None:
        be, c, w = self.backend, self.cfg, self._lw
        xn = be.layernorm(r, w(i, "ln_1.weight"), w(i, "ln_1.bias"), c.norm_eps)
        q = be.qkv_kv_append(xn, w(i, "attn.c_attn.weight"), w(i, "attn.c_attn.bias"),
                             self.kv.k(li), self.kv.v(li), meta, c)
        self._attn_out(q, li, meta, w(i, "attn.c_proj.weight"), w(i, "attn.c_proj.bias"), r)

    def _attn_out(self, q, li: int, meta: BatchMeta, wo, bo, r: Residual) -> None:
        """Attention + output projection + residual add: one fused launch when
        the backend has it for this shape (small decode batches), else two."""
        be = self.backend
        dec = getattr(meta, "dec", None)
        if dec is not None:  # mixed step (runtime/batch.py MixedMeta): each part its own kernel
            b = meta.b
            o = torch.cat([be.attention(q[:b], self.kv.k(li), self.kv.v(li), dec),
                           be.attention(q[b:], self.kv.k(li), self.kv.v(li), meta.pf)])
            be.linear_residual(o, wo, bo, r)
            return
        fused = getattr(be, "attention_oproj", None)
        if fused is not None and fused(q, self.kv.k(li), self.kv.v(li), meta, wo, bo, r):
            return
        o = be.attention(q, self.kv.k(li), self.kv.v(li), meta)
        be.linear_residual(o, wo, bo, r)

    def _gpt2_mlp(self, i: int, r: Residual) -> None:
        be, c, w = self.backend, self.cfg, self._lw
        xn = be.layernorm(r, w(i, "ln_2.weight"), w(i, "ln_2.bias"), c.norm_eps)
        h = be.linear(xn, w(i, "mlp.c_fc.weight"), w(i, "mlp.c_fc.bias"), act="gelu")
        be.linear_residual(h, w(i, "mlp.c_proj.weight"), w(i, "mlp.c_proj.bias"), r)

    def _llama_attn(self, li: int, i: int, r: Residual, meta: BatchMeta) -> None:
        be, c, w = self.backend, self.cfg, self._lw
        xn = be.rmsnorm(r, w(i, "input_layernorm.weight"), c.norm_eps)
        q = be.qkv_kv_append(xn, w(i, "self_attn.qkv.weight"), None,
                             self.kv.k(li), self.kv.v(li), meta, c)
        self._attn_out(q, li, meta, w(i, "self_attn.o_proj.weight"), None, r)

    def _llama_mlp(self, i: int, r: Residual) -> None:
        be, c, w = self.backend, self.cfg, self._lw
        xn = be.rmsnorm(r, w(i, "post_attention_layernorm.weight"), c.norm_eps)
        h = be.linear(xn, w(i, "mlp.gate_up.weight"), None, act="silu_mul")
        be.linear_residual(h, w(i, "mlp.down_proj.weight"), None, r)

    # ------------------------------------------------------------------
    def embed(self, ids: torch.Tensor, meta: BatchMeta) -> torch.Tensor:
        if self.cfg.arch == "gpt2":
            return self.backend.embed(ids, meta.token_pos, self.w["wte"], self.w["wpe"])
        return self.backend.embed(ids, meta.token_pos, self.w["embed_tokens"], None)

    def forward(self, meta: BatchMeta, inp: torch.Tensor, all_logits: bool = False,
                head: bool = True, head_rows: Optional[torch.Tensor] = None,
                variant: int = 0) -> torch.Tensor:
        """inp: token ids int32 [T] (first stage) or hidden fp32 [T, H].

        Returns hidden fp32 [T, H] (non-last stage, or `head=False`: a
        non-final prefill chunk only fills the KV cache) or fp32 logits
        [B, vocab_padded] for the last query of each sequence (last stage;
        [T, vocab_padded] with all_logits; the rows `head_rows` of the packed
        batch when given -- e.g. only the prompts whose final chunk this is).
        `variant`: which of the stage's unit ranges to run (the microbatch
        group's parity under alternating splits; 0 otherwise)."""
        x = self.embed(inp, meta) if self.first else inp
        r = Residual(x)
        # decode-only routing rules (ops/hip.py); a mixed step's rows follow them up to 512
        self.backend.decode = getattr(meta, "routing_decode", meta.is_decode) and meta.num_tokens <= 512 \
            if getattr(meta, "dec", None) is not None else meta.is_decode
        gpt2 = self.cfg.arch == "gpt2"
        attn_fn = self._gpt2_attn if gpt2 else self._llama_attn
        mlp_fn = self._gpt2_mlp if gpt2 else self._llama_mlp
        ua, ub = self.variants[variant % len(self.variants)]
        for u in range(ua, ub):
            i = u >> 1
            if u & 1:
                mlp_fn(i, r)
            else:
                attn_fn(self._kv_index[i], i, r, meta)
        x = self.backend.flush(r)
        if not (self.last and head):
            return x
        return self.head(x, meta, all_logits, head_rows)

    def head(self, x: torch.Tensor, meta: BatchMeta, all_logits: bool = False,
             rows: Optional[torch.Tensor] = None) -> torch.Tensor:
        be, c = self.backend, self.cfg
        if rows is None:
            rows = None if (all_logits or meta.is_decode) else meta.last_idx  # last query per sequence
        if c.arch == "gpt2":
            xn = be.norm_rows(x, self.w["ln_f.weight"], self.w["ln_f.bias"], c.norm_eps, False, rows)
        else:
            xn = be.norm_rows(x, self.w["norm.weight"], None, c.norm_eps, True, rows)
        return be.logits(xn, self.lm_head_weight)

    @property
    def lm_head_weight(self) -> torch.Tensor:
        if hasattr(self, "_lm_head_padded"):
            return self._lm_head_padded
        return self.w["wte"] if self.cfg.arch == "gpt2" else self.w["lm_head"]

    def weight_bytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in self.w.values())
