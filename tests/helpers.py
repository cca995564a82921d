"""Shared test helpers: HF golden models built from our canonical weights."""
from __future__ import annotations

import torch

from llm_sharding_demo_amd.config import ModelConfig
from llm_sharding_demo_amd.models.weights import (canonical_to_hf_gpt2, canonical_to_hf_llama,
                                                  init_stage_weights)


def full_weights(mc: ModelConfig, seed: int = 0, device="cpu", dtype=torch.float32):
    return init_stage_weights(mc, range(mc.n_layers), True, True, seed, device, dtype)


def hf_model(mc: ModelConfig, weights):
    import transformers

    transformers.logging.set_verbosity_error()
    if mc.arch == "gpt2":
        from transformers import GPT2Config, GPT2LMHeadModel

        hc = GPT2Config(vocab_size=mc.vocab_size, n_embd=mc.hidden, n_layer=mc.n_layers,
                        n_head=mc.n_heads, n_positions=mc.max_positions, n_inner=mc.ffn,
                        layer_norm_epsilon=mc.norm_eps, bos_token_id=0, eos_token_id=0)
        m = GPT2LMHeadModel(hc)
        m.load_state_dict(canonical_to_hf_gpt2(mc, weights), strict=True)
    else:
        from transformers import LlamaConfig, LlamaForCausalLM

        hc = LlamaConfig(vocab_size=mc.vocab_size, hidden_size=mc.hidden,
                         intermediate_size=mc.ffn, num_hidden_layers=mc.n_layers,
                         num_attention_heads=mc.n_heads, num_key_value_heads=mc.n_kv_heads,
                         max_position_embeddings=mc.max_positions, rms_norm_eps=mc.norm_eps,
                         rope_theta=mc.rope_theta, tie_word_embeddings=False,
                         bos_token_id=0, eos_token_id=0, pad_token_id=0)
        m = LlamaForCausalLM(hc)
        missing, unexpected = m.load_state_dict(canonical_to_hf_llama(mc, weights), strict=False)
        assert not unexpected and all("rotary" in k for k in missing), (missing, unexpected)
    return m.eval().float()


def hf_greedy(model, prompt, n):
    ids = torch.tensor([prompt])
    with torch.no_grad():
        out = model.generate(ids, max_new_tokens=n, do_sample=False, pad_token_id=0,
                             attention_mask=torch.ones_like(ids))
    return out[0, len(prompt):].tolist()
