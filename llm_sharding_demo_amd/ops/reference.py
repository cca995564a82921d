"""Pure-PyTorch reference implementations of every op the engine uses.

These are the *semantics* the hand-written HIP kernels in `csrc/kernels/`
must reproduce; they also run the whole engine on CPU (tests, golden
numerics).  They compute in fp32 regardless of input dtype.

Op semantics follow HF GPT-2, which the reference delegates to
(`/root/reference/server.py:79-102`; [tf5.15] models/gpt2/modeling_gpt2.py):
  * LayerNorm eps 1e-5, affine (K4)
  * Conv1D = x @ W + b, with W stored [in, out] by HF; we store W^T [out, in]
  * gelu_new = tanh-approximation GELU (K11, [tf5.15] activations.py:59-66)
  * causal softmax(QK^T / sqrt(hd)) V (K7) -- the causal mask is explicit here
    (the reference gets causality only implicitly through SDPA, quirk Q3).
Llama ops (RMSNorm, RoPE, SwiGLU, GQA) follow [tf5.15] models/llama.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn.functional as F

_GELU_C = math.sqrt(2.0 / math.pi)


def gelu_new(x: torch.Tensor) -> torch.Tensor:
    return 0.5 * x * (1.0 + torch.tanh(_GELU_C * (x + 0.044715 * torch.pow(x, 3.0))))


def embed(ids: torch.Tensor, pos: torch.Tensor, wte: torch.Tensor,
          wpe: Optional[torch.Tensor]) -> torch.Tensor:
    """x[t] = wte[ids[t]] + wpe[pos[t]]  -> fp32 [T, H]."""
    x = wte.index_select(0, ids.long()).float()
    if wpe is not None:
        x = x + wpe.index_select(0, pos.long()).float()
    return x


def layernorm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float) -> torch.Tensor:
    return F.layer_norm(x.float(), (x.shape[-1],), w.float(), b.float(), eps)


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    var = xf.pow(2).mean(-1, keepdim=True)
    return xf * torch.rsqrt(var + eps) * w.float()


def linear(a: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """a [T, K] @ w[N, K]^T (+ bias) in fp32."""
    out = a.float() @ w.float().t()
    if bias is not None:
        out = out + bias.float()
    return out


def silu_mul(gate: torch.Tensor, up: torch.Tensor) -> torch.Tensor:
    g = gate.float()
    return g * torch.sigmoid(g) * up.float()


def rope_cos_sin(pos: torch.Tensor, head_dim: int, theta: float):
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    ang = pos.double()[:, None] * inv[None, :]
    return ang.cos().float(), ang.sin().float()  # [T, hd/2]


def apply_rope(x: torch.Tensor, pos: torch.Tensor, theta: float) -> torch.Tensor:
    """HF rotate_half convention: pairs (i, i + hd/2).  x: [T, nh, hd]."""
    hd = x.shape[-1]
    cos, sin = rope_cos_sin(pos.to(torch.float64), hd, theta)
    cos = cos.to(x.device)[:, None, :]
    sin = sin.to(x.device)[:, None, :]
    x1, x2 = x[..., : hd // 2].float(), x[..., hd // 2:].float()
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1)


def kv_append(k_cache: torch.Tensor, v_cache: torch.Tensor, k: torch.Tensor, v: torch.Tensor,
              slots: torch.Tensor, pos: torch.Tensor) -> None:
    """Cache layout [slots, n_kv, max_seq, hd]; k, v: [T, n_kv, hd]."""
    s, p = slots.long(), pos.long()
    k_cache[s, :, p, :] = k.to(k_cache.dtype)
    v_cache[s, :, p, :] = v.to(v_cache.dtype)


def attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
              seq_slots: torch.Tensor, q_start: torch.Tensor, cu_q: torch.Tensor) -> torch.Tensor:
    """Causal attention of packed queries over the KV cache.

    q: [T, nh, hd] packed; sequence i owns rows cu_q[i]:cu_q[i+1], whose
    positions are q_start[i] + j.  Keys/values for sequence i live at
    k_cache[seq_slots[i], :, 0:q_start[i]+len_i].  GQA: nh % n_kv == 0.
    Returns fp32 [T, nh, hd].
    """
    nh, hd = q.shape[1], q.shape[2]
    n_kv = k_cache.shape[1]
    grp = nh // n_kv
    out = torch.empty(q.shape, dtype=torch.float32, device=q.device)
    scale = 1.0 / math.sqrt(hd)
    for i in range(seq_slots.numel()):
        a, b = int(cu_q[i]), int(cu_q[i + 1])
        if b == a:
            continue
        st = int(q_start[i])
        L = st + (b - a)
        s = int(seq_slots[i])
        kk = k_cache[s, :, :L].float().repeat_interleave(grp, dim=0)  # [nh, L, hd]
        vv = v_cache[s, :, :L].float().repeat_interleave(grp, dim=0)
        qq = q[a:b].float().transpose(0, 1)  # [nh, Lq, hd]
        sc = torch.matmul(qq, kk.transpose(1, 2)) * scale  # [nh, Lq, L]
        qpos = torch.arange(st, L, device=q.device)[:, None]
        kpos = torch.arange(L, device=q.device)[None, :]
        sc = sc.masked_fill(kpos > qpos, float("-inf"))
        p = torch.softmax(sc, dim=-1)
        out[a:b] = torch.matmul(p, vv).transpose(0, 1)
    return out


def sample(logits: torch.Tensor, temperature: torch.Tensor, top_k: torch.Tensor,
           greedy: torch.Tensor, uniforms: torch.Tensor, vocab: int) -> torch.Tensor:
    """Per-row sampler.  Reference semantics (server.py:187-206):
    logits/T -> topk(k) -> softmax over the k values -> draw -> map to vocab id.
    `uniforms` [B] in [0,1) drive the draw (inverse CDF over the top-k sorted
    descending), so the result is a deterministic function of its inputs.
    greedy rows return argmax (lowest index on ties).
    """
    B = logits.shape[0]
    lg = logits[:, :vocab].float()
    out = torch.empty(B, dtype=torch.int32, device=logits.device)
    for r in range(B):
        row = lg[r]
        if bool(greedy[r]):
            out[r] = int(torch.argmax(row))
            continue
        k = int(top_k[r])
        vals, idx = torch.topk(row / float(temperature[r]), k)
        # stable ordering for ties: by value desc then index asc
        order = sorted(range(k), key=lambda j: (-float(vals[j]), int(idx[j])))
        vals, idx = vals[order], idx[order]
        p = torch.softmax(vals, dim=-1)
        c = torch.cumsum(p, 0)
        u = float(uniforms[r]) * float(c[-1])
        j = int(torch.searchsorted(c, torch.tensor([u], dtype=c.dtype)).clamp(max=k - 1))
        out[r] = int(idx[j])
    return out
