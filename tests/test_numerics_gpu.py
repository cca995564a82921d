"""Real-dimension numerics on an MI355X: GPT-2 small, GPT-2 XL and Llama-3 8B
(full dims, random init) -- HIP logits vs an fp32 golden of the same weights
computed with the plain PyTorch ops on the same GPU (utils/golden.py), over a
prefill and 8 teacher-forced decode steps.  Covers the shapes the bench runs:
nh = 25, K = 6400, V = 50257 / 128256, the vocab-tiled lm_head, GQA + RoPE.

Tolerance: bf16 weights/activations with fp32 accumulation give per-row
max |error| within a few percent of the golden logits' standard deviation
(measured: GPT-2 small 1.8 %, GPT-2 XL 2.1 %, Llama-3 8B dims at 4 layers
7 %); greedy top-1 agrees on >= 95 % of the rows.

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


@pytest.mark.parametrize("model,layers,lens", [("gpt2", None, [7, 33, 96]),
                                               ("gpt2-xl", None, [5, 40, 130]),
                                               ("llama-3-8b", 4, [9, 64])])
def test_full_dims_match_fp32_golden(model, layers, lens):
    from llm_sharding_demo_amd.config import get_model_config

    mc = get_model_config(model)
    if layers:
        mc = dataclasses.replace(mc, n_layers=layers)
    rnd = random.Random(3)
    prompts = [[rnd.randrange(mc.vocab_size) for _ in range(n)] for n in lens]
    r = compare_with_golden(mc, prompts, steps=8)
    print(model, r)
    assert r["rows"] == 9 * len(lens)
    assert r["top1_agreement"] >= 0.95, r
    assert r["max_rel_err"] < 0.15, r
    assert r["mean_rel_err"] < 0.08, r
    torch.cuda.empty_cache()


def test_llama3_8b_full_depth_pinned():
    rnd = random.Random(3)
    prompts = [[rnd.randrange(128256) for _ in range(n)] for n in (9, 64)]
    r = compare_with_golden("llama-3-8b", prompts, steps=8)
    print("llama-3-8b", r)
    assert r["top1_agreement"] >= 0.95, r
    assert r["max_rel_err"] < 0.15, r
    torch.cuda.empty_cache()
