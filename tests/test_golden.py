"""Golden numerics: the engine (CPU reference backend) vs HF transformers.

The reference delegates all math to HF GPT-2 (`server.py:41`); these tests pin
our op semantics (LayerNorm, Conv1D transpose, gelu_new, explicit causal
attention, tied lm_head; Llama RMSNorm/RoPE/SwiGLU/GQA) to it.
"""
import pytest
import torch

from llm_sharding_demo_amd.config import EngineConfig, SamplingParams, get_model_config
from llm_sharding_demo_amd.models.stage import StageModel
from llm_sharding_demo_amd.runtime.batch import BatchMeta
from llm_sharding_demo_amd.runtime.engine import Engine

from .helpers import full_weights, hf_greedy, hf_model


@pytest.mark.parametrize("model", ["gpt2-test", "tiny-gpt2", "llama-test"])
def test_full_sequence_logits_match_hf(model):
    mc = get_model_config(model)
    w = full_weights(mc)
    hf = hf_model(mc, w)
    st = StageModel(mc, 0, mc.n_layers, True, True, weights=w, max_slots=2, max_seq=64)
    ids = [3, 17, 5, 99, 42, 7, 1]
    meta = BatchMeta.build([1], [0], [len(ids)], "cpu")
    ours = st.forward(meta, torch.tensor(ids, dtype=torch.int32), all_logits=True)[:, : mc.vocab_size]
    with torch.no_grad():
        theirs = hf(torch.tensor([ids])).logits[0]
    torch.testing.assert_close(ours, theirs, atol=2e-4, rtol=1e-4)


@pytest.mark.parametrize("model", ["gpt2-test", "llama-test"])
def test_greedy_generation_matches_hf(model):
    mc = get_model_config(model)
    w = full_weights(mc)
    hf = hf_model(mc, w)
    eng = Engine(EngineConfig(model_id=model, num_stages=1, max_batch=4, device="cpu"))
    prompts = [[5, 6, 7, 8], [11], [300, 2, 9]]
    outs = eng.generate_ids(prompts, SamplingParams(greedy=True, max_new_tokens=8))
    for p, o in zip(prompts, outs):
        assert o == hf_greedy(hf, p, 8)


def test_kv_cached_decode_equals_full_recompute():
    """Incremental decode through the cache == recomputing the whole sequence
    (what the reference does every step, server.py:169-181)."""
    mc = get_model_config("gpt2-test")
    w = full_weights(mc)
    st = StageModel(mc, 0, mc.n_layers, True, True, weights=w, max_slots=2, max_seq=64)
    seq = [9, 8, 7, 6, 5, 4, 3, 2]
    meta = BatchMeta.build([0], [0], [4], "cpu")
    st.forward(meta, torch.tensor(seq[:4], dtype=torch.int32))
    for t in range(4, len(seq)):
        dm = BatchMeta.decode([0], [t], "cpu", max_ctx=t + 1)
        inc = st.forward(dm, torch.tensor([seq[t]], dtype=torch.int32))
        fm = BatchMeta.build([1], [0], [t + 1], "cpu")
        full = st.forward(fm, torch.tensor(seq[: t + 1], dtype=torch.int32))
        torch.testing.assert_close(inc, full, atol=1e-4, rtol=1e-4)


def test_chunked_prefill_equals_single_prefill():
    mc = get_model_config("llama-test")
    w = full_weights(mc)
    st = StageModel(mc, 0, mc.n_layers, True, True, weights=w, max_slots=2, max_seq=64)
    seq = list(range(20, 33))
    a = st.forward(BatchMeta.build([0], [0], [13], "cpu"), torch.tensor(seq, dtype=torch.int32))
    st.forward(BatchMeta.build([1], [0], [6], "cpu"), torch.tensor(seq[:6], dtype=torch.int32))
    b = st.forward(BatchMeta.build([1], [6], [7], "cpu"), torch.tensor(seq[6:], dtype=torch.int32))
    torch.testing.assert_close(a, b, atol=1e-4, rtol=1e-4)


def test_batched_ragged_prefill_equals_individual():
    mc = get_model_config("gpt2-test")
    w = full_weights(mc)
    st = StageModel(mc, 0, mc.n_layers, True, True, weights=w, max_slots=4, max_seq=64)
    ps = [[1, 2, 3], [4, 5, 6, 7, 8], [9]]
    flat = torch.tensor([t for p in ps for t in p], dtype=torch.int32)
    both = st.forward(BatchMeta.build([0, 1, 2], [0, 0, 0], [3, 5, 1], "cpu"), flat)
    for i, p in enumerate(ps):
        one = st.forward(BatchMeta.build([3], [0], [len(p)], "cpu"), torch.tensor(p, dtype=torch.int32))
        torch.testing.assert_close(both[i:i + 1], one, atol=1e-4, rtol=1e-4)
