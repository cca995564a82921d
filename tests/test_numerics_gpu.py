"""Real-dimension numerics on an MI355X: GPT-2 small, GPT-2 XL and Llama-3 8B
(full dims, random init) -- HIP logits vs an fp32 golden of the same weights
computed with the plain PyTorch ops on the same GPU (utils/golden.py), over a
prefill and 8 teacher-forced decode steps.  Covers the shapes the bench runs:
nh = 25, K = 6400, V = 50257 / 128256, the vocab-tiled lm_head, GQA + RoPE.

Tolerance: bf16 weights/activations with fp32 accumulation give per-row
max |error| within a few percent of the golden logits' standard deviation
(measured: GPT-2 small 1.9 %, GPT-2 XL 2.4 %, Llama-3 8B 2.9-3.2 %).  The bounds (BOUNDS) sit at about twice the measurements, and every
test also checks that the same logits with the HIP error tripled FAIL them.

Llama-3 8B at its full 32 layers: with HF's 0.02 embedding init the random
network amplified bf16 rounding with depth (16-21 % after 32 layers, and a
bf16 emulation was as far off: profiles/r2_numerics_llama_depth.log).  The
init now puts the untied input embedding at unit scale (models/weights.py;
profiles/r3_llama_init_depth.log), which is well conditioned, so the full
depth is pinned with the same bounds as the other models.
"""
import dataclasses
import random

import pytest
import torch

from llm_sharding_demo_amd.utils.golden import compare_with_golden

pytestmark = pytest.mark.gpu


# (top-1 floor, max bound, mean bound) per model: about 2x the measured errors
# (round 5, profiles/r5_pytest_gpu_full.log: GPT-2 small max 0.019 / mean 0.017,
# XL 0.024 / 0.018, Llama-3 8B dims at 4 layers 0.029 / 0.024, at full depth
# 0.032 / 0.028; top-1 1.0 everywhere), so a kernel change that doubles the
# error fails the suite instead of hiding under the old 0.15 bound
BOUNDS = {"gpt2": (0.99, 0.05, 0.03), "gpt2-xl": (0.99, 0.05, 0.03), "llama-3-8b": (0.95, 0.07, 0.06)}


def _gate(model, r):
    top1, mx, mean = BOUNDS[model]
    return r["top1_agreement"] >= top1 and r["max_rel_err"] < mx and r["mean_rel_err"] < mean


def _prompts(vocab, lens, seed=3):
    rnd = random.Random(seed)
    return [[rnd.randrange(vocab) for _ in range(n)] for n in lens]


@pytest.mark.parametrize("model,layers,lens", [("gpt2", None, [7, 33, 96]),
                                               ("gpt2-xl", None, [5, 40, 130]),
                                               ("llama-3-8b", 4, [9, 64])])
def test_full_dims_match_fp32_golden(model, layers, lens):
    from llm_sharding_demo_amd.config import get_model_config

    mc = get_model_config(model)
    if layers:
        mc = dataclasses.replace(mc, n_layers=layers)
    prompts = _prompts(mc.vocab_size, lens)
    r, r3 = compare_with_golden(mc, prompts, steps=8, inject=(1.0, 3.0))
    print(model, r)
    assert r["rows"] == 9 * len(lens)
    assert _gate(model, r), r
    # the same logits with the HIP error tripled must fail the gate
    assert not _gate(model, r3), r3
    torch.cuda.empty_cache()


def test_llama3_8b_full_depth_pinned():
    prompts = _prompts(128256, (9, 64))
    r = compare_with_golden("llama-3-8b", prompts, steps=8)
    print("llama-3-8b", r)
    assert _gate("llama-3-8b", r), r
    torch.cuda.empty_cache()


def test_headline_decode_shape_matches_fp32_golden():
    """The bench's decode microbatch: GPT-2 XL, 256 sequences -> 256-row
    decode GEMMs (the 256-row kernels, residual split-K partials in bf16 slabs
    folded by the norm), 128 cached positions, 4 teacher-forced steps.
    Measured at this shape (round 5): top-1 0.998, max 0.026, mean 0.019 of
    the logit std."""
    prompts = _prompts(50257, [128] * 256, seed=11)
    r, r3 = compare_with_golden("gpt2-xl", prompts, steps=4, inject=(1.0, 3.0))
    print("gpt2-xl 256 rows", r)
    gate = lambda x: (x["top1_agreement"] >= 0.99 and x["max_rel_err"] < 0.06  # noqa: E731
                      and x["mean_rel_err"] < 0.04)
    assert gate(r), r
    assert not gate(r3), r3
    torch.cuda.empty_cache()


def test_llama_512_row_decode_matches_fp32_golden():
    """Llama-3 8B dims (4 layers) with 512 sequences: the 512-row decode
    GEMMs of the Llama-3 8B bench (256x256 gate_up kernel with the fused
    SiLU*up epilogue) against the fp32 golden with the Llama bounds.  With
    the hipBLASLt gate_up forced on it measured top-1 0.983, max 0.041, mean
    0.029 (profiles/r5_llama_blaslt.log).  The 512-row decode QKV runs on the
    hand-written ring kernel with the fused RoPE / cache-append epilogue."""
    from llm_sharding_demo_amd.config import get_model_config

    mc = dataclasses.replace(get_model_config("llama-3-8b"), n_layers=4)
    prompts = _prompts(mc.vocab_size, [12] * 512, seed=13)
    r, r3 = compare_with_golden(mc, prompts, steps=3, inject=(1.0, 3.0))
    print("llama-3-8b 512 rows", r)
    assert _gate("llama-3-8b", r), r
    assert not _gate("llama-3-8b", r3), r3
    torch.cuda.empty_cache()
