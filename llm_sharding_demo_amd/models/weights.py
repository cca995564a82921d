"""Stage-local weight materialisation.

Replaces the reference's "every pod loads the full model from the Hub"
(`server.py:40-42,108`, quirk Q4): a stage materialises ONLY its own layers,
plus the token embedding on the first stage and the final norm + lm_head on
the last stage (`wte` is tied to `lm_head` in GPT-2, so both ends hold a copy;
SURVEY.md §7.4 item 7).

Canonical layout: every projection weight is stored [out_features, in_features]
(K-contiguous), i.e. HF GPT-2 Conv1D weights ([in, out], [tf5.15]
pytorch_utils.py:106-121) are transposed once at load time.  That is the
layout the MFMA kernels want: the B-operand fragment of
`mfma_f32_16x16x32_bf16` is 8 consecutive K elements of one output column,
one 16-byte load.

Random init: each tensor gets its own seed derived from (seed, tensor name),
so any layer partition produces bit-identical weights (the property the
partition-invariance tests rely on).
"""
from __future__ import annotations

import os
import zlib
from typing import Dict, Iterable, Optional, Tuple

import torch

from ..config import ModelConfig


def _seed(seed: int, name: str) -> int:
    return (zlib.crc32(f"{seed}:{name}".encode()) * 2654435761 + seed) % (2 ** 63 - 1)


def _randn(shape, std, seed, name, device, dtype):
    dev = torch.device(device)
    g = torch.Generator(device=dev)
    g.manual_seed(_seed(seed, name))
    t = torch.randn(shape, generator=g, device=dev, dtype=torch.float32) * std
    return t.to(dtype)


def gpt2_layer_names(i: int):
    return [f"h.{i}.{n}" for n in (
        "ln_1.weight", "ln_1.bias", "attn.c_attn.weight", "attn.c_attn.bias",
        "attn.c_proj.weight", "attn.c_proj.bias", "ln_2.weight", "ln_2.bias",
        "mlp.c_fc.weight", "mlp.c_fc.bias", "mlp.c_proj.weight", "mlp.c_proj.bias")]


def _gpt2_shapes(cfg: ModelConfig, i: int) -> Dict[str, tuple]:
    h, f = cfg.hidden, cfg.ffn
    p = f"h.{i}."
    return {
        p + "ln_1.weight": (h,), p + "ln_1.bias": (h,),
        p + "attn.c_attn.weight": (3 * h, h), p + "attn.c_attn.bias": (3 * h,),
        p + "attn.c_proj.weight": (h, h), p + "attn.c_proj.bias": (h,),
        p + "ln_2.weight": (h,), p + "ln_2.bias": (h,),
        p + "mlp.c_fc.weight": (f, h), p + "mlp.c_fc.bias": (f,),
        p + "mlp.c_proj.weight": (h, f), p + "mlp.c_proj.bias": (h,),
    }


def _llama_shapes(cfg: ModelConfig, i: int) -> Dict[str, tuple]:
    h, f = cfg.hidden, cfg.ffn
    p = f"layers.{i}."
    return {
        p + "input_layernorm.weight": (h,),
        p + "self_attn.qkv.weight": (cfg.qkv_size, h),  # q | k | v rows
        p + "self_attn.o_proj.weight": (h, cfg.q_size),
        p + "post_attention_layernorm.weight": (h,),
        p + "mlp.gate_up.weight": (2 * f, h),  # gate rows | up rows
        p + "mlp.down_proj.weight": (h, f),
    }


_ATTN_PARTS = ("ln_1.", "attn.", "input_layernorm.", "self_attn.")
_MLP_PARTS = ("ln_2.", "mlp.", "post_attention_layernorm.")


def layer_half(name: str) -> Optional[Tuple[int, int]]:
    """(layer, 0 = attention half | 1 = MLP half) of a per-layer tensor name,
    None for embeddings / final norm / lm_head (parallel/partition.py units)."""
    for pre in ("h.", "layers."):
        if name.startswith(pre):
            idx, rest = name[len(pre):].split(".", 1)
            if rest.startswith(_ATTN_PARTS):
                return int(idx), 0
            if rest.startswith(_MLP_PARTS):
                return int(idx), 1
            raise ValueError(f"unknown per-layer tensor {name!r}")
    return None


def _filter_units(shapes: Dict[str, tuple], units: Optional[Tuple[int, int]]) -> Dict[str, tuple]:
    if units is None:
        return shapes
    ua, ub = units
    out = {}
    for n, s in shapes.items():
        lh = layer_half(n)
        if lh is None or ua <= 2 * lh[0] + lh[1] < ub:
            out[n] = s
    return out


def stage_tensor_shapes(cfg: ModelConfig, layers: Iterable[int], first: bool, last: bool,
                        units: Optional[Tuple[int, int]] = None):
    """Tensors a stage materialises; with `units` only the halves of the
    boundary layers that the stage runs."""
    return _filter_units(_stage_tensor_shapes(cfg, layers, first, last), units)


def _stage_tensor_shapes(cfg: ModelConfig, layers: Iterable[int], first: bool, last: bool):
    shapes: Dict[str, tuple] = {}
    if cfg.arch == "gpt2":
        if first:
            shapes["wte"] = (cfg.vocab_size, cfg.hidden)
            shapes["wpe"] = (cfg.max_positions, cfg.hidden)
        for i in layers:
            shapes.update(_gpt2_shapes(cfg, i))
        if last:
            shapes["ln_f.weight"] = (cfg.hidden,)
            shapes["ln_f.bias"] = (cfg.hidden,)
            shapes["wte"] = (cfg.vocab_size, cfg.hidden)  # tied lm_head
    else:
        if first:
            shapes["embed_tokens"] = (cfg.vocab_size, cfg.hidden)
        for i in layers:
            shapes.update(_llama_shapes(cfg, i))
        if last:
            shapes["norm.weight"] = (cfg.hidden,)
            shapes["lm_head"] = (cfg.vocab_size, cfg.hidden)
    return shapes


def _init_one(cfg: ModelConfig, name: str, shape, seed: int, device, dtype) -> torch.Tensor:
    base = name.rsplit(".", 1)[-1]
    if name == "embed_tokens":
        # untied (Llama) input embeddings at unit scale (the T5 / muP
        # convention: the residual stream enters at the RMS its norms produce).
        # With HF's 0.02 the first layers' outputs dwarf the stream and random
        # -init depth amplifies bf16 rounding: fp32 vs bf16-emulated logits at
        # 32 layers, H = 2048: 6.6 % -> 1.1 % of the logit std; H = 1024: 3.3 %
        # -> 0.7 % (profiles/r3_llama_init_depth.log).  Residual projections
        # below are depth-scaled (0.02 / sqrt(2L)) as in GPT-2 / Llama training.
        return _randn(shape, 1.0, seed, name, device, dtype)
    if name in ("wte", "lm_head"):
        return _randn(shape, 0.02, seed, name, device, dtype)
    if name == "wpe":
        return _randn(shape, 0.01, seed, name, device, dtype)
    if "norm" in name or "ln_" in name:
        if base == "weight":
            return (1.0 + _randn(shape, 0.05, seed, name, device, torch.float32)).to(dtype)
        return _randn(shape, 0.02, seed, name, device, dtype)
    if base == "bias":
        return _randn(shape, 0.02, seed, name, device, dtype)
    std = 0.02
    if name.endswith("c_proj.weight") or name.endswith("o_proj.weight") or name.endswith("down_proj.weight"):
        std = 0.02 / (2 * cfg.n_layers) ** 0.5
    return _randn(shape, std, seed, name, device, dtype)


def init_stage_weights(cfg: ModelConfig, layers, first: bool, last: bool, seed: int,
                       device, dtype, units=None) -> Dict[str, torch.Tensor]:
    shapes = stage_tensor_shapes(cfg, layers, first, last, units)
    return {n: _init_one(cfg, n, s, seed, device, dtype) for n, s in shapes.items()}


# ---------------------------------------------------------------------------
# Checkpoint loading (safetensors / torch weights_only) -- stage-local slices
# ---------------------------------------------------------------------------

_GPT2_CONV1D = ("attn.c_attn.weight", "attn.c_proj.weight", "mlp.c_fc.weight", "mlp.c_proj.weight")


def _open_checkpoint(path: str):
    """Returns a callable name -> tensor that reads lazily where possible."""
    files = []
    if os.path.isdir(path):
        for fn in sorted(os.listdir(path)):
            if fn.endswith(".safetensors"):
                files.append(os.path.join(path, fn))
        if not files:
            for fn in ("pytorch_model.bin", "model.pt"):
                if os.path.isfile(os.path.join(path, fn)):
                    files.append(os.path.join(path, fn))
    else:
        files = [path]
    if not files:
        raise FileNotFoundError(f"no checkpoint files in {path}")
    if files[0].endswith(".safetensors"):
        from safetensors import safe_open

        index = {}
        handles = [safe_open(f, framework="pt") for f in files]
        for h in handles:
            for k in h.keys():
                index[k] = h
        return lambda k: index[k].get_tensor(k), set(index)
    sd = {}
    for f in files:
        sd.update(torch.load(f, map_location="cpu", weights_only=True))  # never unpickles code
    return lambda k: sd[k], set(sd)


def load_stage_weights(cfg: ModelConfig, path: str, layers, first: bool, last: bool,
                       device, dtype, units=None) -> Dict[str, torch.Tensor]:
    get, keys = _open_checkpoint(path)
    out: Dict[str, torch.Tensor] = {}
    want = stage_tensor_shapes(cfg, layers, first, last, units)

    def find(name):
        for pre in ("", "transformer.", "model."):
            if pre + name in keys:
                return get(pre + name)
        raise KeyError(name)

    for name, shape in want.items():
        if cfg.arch == "gpt2":
            src = {"wte": "wte.weight", "wpe": "wpe.weight"}.get(name, name)
            t = find(src)
            if any(name.endswith(c) for c in _GPT2_CONV1D):
                t = t.t()  # Conv1D [in, out] -> [out, in]
        else:
            if name.endswith("self_attn.qkv.weight"):
                p = name[: -len("qkv.weight")]
                t = torch.cat([find(p + "q_proj.weight"), find(p + "k_proj.weight"),
                               find(p + "v_proj.weight")], 0)
            elif name.endswith("mlp.gate_up.weight"):
                p = name[: -len("gate_up.weight")]
                t = torch.cat([find(p + "gate_proj.weight"), find(p + "up_proj.weight")], 0)
            elif name == "embed_tokens":
                t = find("embed_tokens.weight")
            elif name == "lm_head":
                t = get("lm_head.weight") if "lm_head.weight" in keys else find("embed_tokens.weight")
            else:
                t = find(name)
        if tuple(t.shape) != tuple(shape):
            raise ValueError(f"{name}: checkpoint shape {tuple(t.shape)} != expected {shape}")
        out[name] = t.to(device=device, dtype=dtype).contiguous()
    return out


def hf_state_dict_to_canonical(cfg: ModelConfig, sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """Full HF GPT2LMHeadModel/LlamaForCausalLM state dict -> canonical names (all layers)."""
    import tempfile

    from safetensors.torch import save_file

    with tempfile.TemporaryDirectory() as d:
        tensors = {k: v.detach().contiguous().clone() for k, v in sd.items()}
        if "lm_head.weight" in tensors and cfg.tie_embeddings:
            tensors.pop("lm_head.weight")
        save_file(tensors, os.path.join(d, "model.safetensors"))
        return load_stage_weights(cfg, d, range(cfg.n_layers), True, True, "cpu", torch.float32)


def canonical_to_hf_gpt2(cfg: ModelConfig, w: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """Canonical (all layers) -> HF GPT2LMHeadModel state dict (for golden tests)."""
    sd = {"transformer.wte.weight": w["wte"], "transformer.wpe.weight": w["wpe"],
          "transformer.ln_f.weight": w["ln_f.weight"], "transformer.ln_f.bias": w["ln_f.bias"],
          "lm_head.weight": w["wte"]}
    for i in range(cfg.n_layers):
        for n in gpt2_layer_names(i):
            t = w[n]
            if any(n.endswith(c) for c in _GPT2_CONV1D):
                t = t.t()
            sd["transformer." + n] = t.contiguous()
    return sd


def canonical_to_hf_llama(cfg: ModelConfig, w: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    sd = {"model.embed_tokens.weight": w["embed_tokens"], "model.norm.weight": w["norm.weight"],
          "lm_head.weight": w["lm_head"]}
    q, kv, f = cfg.q_size, cfg.kv_size, cfg.ffn
    for i in range(cfg.n_layers):
        p = f"layers.{i}."
        qkv = w[p + "self_attn.qkv.weight"]
        sd["model." + p + "self_attn.q_proj.weight"] = qkv[:q]
        sd["model." + p + "self_attn.k_proj.weight"] = qkv[q:q + kv]
        sd["model." + p + "self_attn.v_proj.weight"] = qkv[q + kv:]
        sd["model." + p + "self_attn.o_proj.weight"] = w[p + "self_attn.o_proj.weight"]
        gu = w[p + "mlp.gate_up.weight"]
        sd["model." + p + "mlp.gate_proj.weight"] = gu[:f]
        sd["model." + p + "mlp.up_proj.weight"] = gu[f:]
        sd["model." + p + "mlp.down_proj.weight"] = w[p + "mlp.down_proj.weight"]
        sd["model." + p + "input_layernorm.weight"] = w[p + "input_layernorm.weight"]
        sd["model." + p + "post_attention_layernorm.weight"] = w[p + "post_attention_layernorm.weight"]
    return {k: v.contiguous() for k, v in sd.items()}


def maybe_load(cfg: ModelConfig, weights: Optional[str], layers, first, last, seed, device, dtype,
               units=None):
    if weights:
        return load_stage_weights(cfg, weights, layers, first, last, device, dtype, units)
    return init_stage_weights(cfg, layers, first, last, seed, device, dtype, units)
