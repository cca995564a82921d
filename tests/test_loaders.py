"""Checkpoint loading, tokenizer and reference-compat HTTP coordinator (CPU).

The reference loads real weights and tokenizer from the HF Hub in every role
(`/root/reference/server.py:40-42`) and relays hidden states between shard
pods over HTTP (`server.py:169-206`).  No Hub access here, so parity is pinned
with synthetic fixtures written by these tests: a saved random checkpoint in
HF naming (GPT-2 Conv1D layout, Llama q/k/v + gate/up split), a tiny
byte-level BPE vocabulary, and the HTTP shard loop against in-process
shard apps.
"""
import json

import pytest
import torch

from llm_sharding_demo_amd.config import EngineConfig, SamplingParams, get_model_config
from llm_sharding_demo_amd.models.stage import StageModel
from llm_sharding_demo_amd.models.weights import (canonical_to_hf_gpt2, canonical_to_hf_llama,
                                                  stage_tensor_shapes)
from llm_sharding_demo_amd.runtime.engine import Engine

from .helpers import full_weights


def _save_hf(mc, w, path, fmt="safetensors"):
    sd = canonical_to_hf_gpt2(mc, w) if mc.arch == "gpt2" else canonical_to_hf_llama(mc, w)
    if mc.tie_embeddings:
        sd.pop("lm_head.weight")  # tied to wte, as HF saves GPT-2
    sd = {k: v.contiguous().clone() for k, v in sd.items()}
    if fmt == "safetensors":
        from safetensors.torch import save_file

        save_file(sd, str(path / "model.safetensors"))
    else:
        torch.save(sd, str(path / "pytorch_model.bin"))


@pytest.mark.parametrize("model,units,fmt", [("gpt2-test", (3, 7), "safetensors"),
                                            ("llama-test", (2, 8), "safetensors"),
                                            ("gpt2-test", (0, 8), "bin")])
def test_stage_local_checkpoint_roundtrip(tmp_path, model, units, fmt):
    """A stage loads exactly its own tensors (half-layer boundaries included)
    and they are bit-identical to the weights that were saved."""
    mc = get_model_config(model)
    w = full_weights(mc, seed=11)
    _save_hf(mc, w, tmp_path, fmt)
    a, b = units
    first, last = a == 0, b == 2 * mc.n_layers
    st = StageModel(mc, a // 2, (b + 1) // 2, first, last, weights_path=str(tmp_path),
                    max_slots=2, max_seq=32, units=units)
    want = stage_tensor_shapes(mc, range(a // 2, (b + 1) // 2), first, last, units)
    assert set(st.w) == set(want)
    for name, t in st.w.items():
        assert torch.equal(t, w[name]), name


def test_engine_from_checkpoint_matches_random_init(tmp_path):
    """Engine with WEIGHTS=<dir> over a 2-stage split == the same weights
    initialised in memory (the loader is the only difference)."""
    mc = get_model_config("gpt2-test")
    _save_hf(mc, full_weights(mc, seed=0), tmp_path)
    sp = SamplingParams(greedy=True, max_new_tokens=5)
    prompts = [[5, 6, 7], [1], [40, 41]]
    ref = Engine(EngineConfig(model_id="gpt2-test", max_batch=4, device="cpu", seed=0))
    eng = Engine(EngineConfig(model_id="gpt2-test", num_stages=2, max_batch=4, device="cpu",
                              weights=str(tmp_path)))
    assert eng.generate_ids(prompts, sp) == ref.generate_ids(prompts, sp)


def test_checkpoint_shape_mismatch_is_reported(tmp_path):
    mc = get_model_config("gpt2-test")
    w = full_weights(mc)
    w["h.0.mlp.c_fc.bias"] = w["h.0.mlp.c_fc.bias"][:-1]
    _save_hf(mc, w, tmp_path)
    with pytest.raises(ValueError, match="c_fc.bias"):
        StageModel(mc, 0, 1, True, False, weights_path=str(tmp_path), max_slots=1, max_seq=8)


# ---------------------------------------------------------------------------
# Byte-level BPE (GPT-2 format vocab.json + merges.txt)
# ---------------------------------------------------------------------------

def _tiny_bpe(path):
    from llm_sharding_demo_amd.utils.tokenizer import bytes_to_unicode_order

    order = bytes_to_unicode_order()
    # GPT-2's byte -> unicode map: printable bytes map to themselves, the rest
    # to 256 + n in order of appearance
    n = 0
    vocab = {}
    for i, b in enumerate(order):
        if 33 <= b <= 126 or 161 <= b <= 172 or 174 <= b <= 255:
            vocab[chr(b)] = i
        else:
            vocab[chr(256 + n)] = i
            n += 1
    merges = [("h", "e"), ("l", "l"), ("he", "ll"), ("hell", "o"), ("Ġ", "w")]
    for a, b in merges:
        vocab[a + b] = len(vocab)
    vocab["<|endoftext|>"] = len(vocab)
    (path / "vocab.json").write_text(json.dumps(vocab))
    (path / "merges.txt").write_text("#version: 0.2\n" + "\n".join(f"{a} {b}" for a, b in merges) + "\n")
    return vocab


def test_bpe_fixture_encode_decode(tmp_path):
    from llm_sharding_demo_amd.utils.tokenizer import BPETokenizer, ByteTokenizer, load_tokenizer

    vocab = _tiny_bpe(tmp_path)
    tok = load_tokenizer("gpt2", "gpt2", weights=str(tmp_path))
    assert isinstance(tok, BPETokenizer)
    ids = tok.encode("hello world")
    assert ids[0] == vocab["hello"]           # merges applied
    assert vocab["Ġw"] in ids                 # byte-level space prefix merge
    assert tok.decode(ids) == "hello world"
    eot = vocab["<|endoftext|>"]
    assert tok.decode(ids + [eot], skip_special_tokens=True) == "hello world"
    # single-byte ids agree with the byte fallback (same GPT-2 byte table)
    fb = ByteTokenizer()
    assert tok.encode("xq!") == fb.encode("xq!")


# ---------------------------------------------------------------------------
# Reference-style HTTP coordinator (TRANSPORT=http) over two shard apps
# ---------------------------------------------------------------------------

def test_http_generate_over_shard_apps(monkeypatch):
    """`http_generate` drives shard A and shard B exactly like the reference
    coordinator (full-sequence recompute, hidden states relayed through the
    coordinator); greedy output equals the engine's cached pipeline."""
    from fastapi.testclient import TestClient

    from llm_sharding_demo_amd.serving import server as srv

    base = EngineConfig(model_id="gpt2-test", max_batch=4, device="cpu", split_points=[2],
                        shard_a_service="shard-a", shard_b_service="shard-b", shard_port=5001)
    a = TestClient(srv.create_app(base.replace(role="a"), shard=srv.ShardRunner(base, "a")))
    b = TestClient(srv.create_app(base.replace(role="b"), shard=srv.ShardRunner(base, "b")))
    calls = []

    class _Resp:
        def __init__(self, r):
            self.r = r

        def raise_for_status(self):
            assert self.r.status_code == 200, self.r.text

        def json(self):
            return self.r.json()

    def post(url, json=None, timeout=None):
        calls.append(url)
        host_path = url.split("://", 1)[1]
        host, path = host_path.split("/", 1)
        client = {"shard-a:5001": a, "shard-b:5001": b}[host]
        return _Resp(client.post("/" + path, json=json))

    import requests

    monkeypatch.setattr(requests, "post", post)
    prompt = [5, 6, 7, 8]
    sp = SamplingParams(greedy=True, max_new_tokens=4)
    out = srv.http_generate(base, prompt, sp)
    assert calls[:2] == ["http://shard-a:5001/forward", "http://shard-b:5001/forward_b"]
    assert len(calls) == 8  # two hops per token, like server.py:172-181
    eng = Engine(base.replace(num_stages=2, role="coordinator"))
    assert out == eng.generate_ids([prompt], sp)[0]


def test_kv_slots_follow_hbm_budget():
    from llm_sharding_demo_amd.runtime.kv_cache import KVCache, plan_slots

    per = KVCache.bytes_per_slot(48, 25, 256, 64)
    fake = lambda free: (lambda dev: (free, 288 << 30))  # noqa: E731
    # budget = (free - reserve) * fraction
    assert plan_slots(4096, 48, 25, 256, 64, "cpu", mem_get_info=fake(100 * per), fraction=1.0) == 100
    assert plan_slots(4096, 48, 25, 256, 64, "cpu", mem_get_info=fake(100 * per), fraction=0.5) == 50
    assert plan_slots(4096, 48, 25, 256, 64, "cpu", mem_get_info=fake(100 * per),
                      reserve=40 * per, fraction=1.0) == 60
    assert plan_slots(16, 48, 25, 256, 64, "cpu", mem_get_info=fake(100 * per)) == 16
    assert plan_slots(16, 0, 25, 256, 64, "cpu", mem_get_info=fake(0)) == 16  # no KV layers
    with pytest.raises(MemoryError):
        plan_slots(4, 48, 25, 256, 64, "cpu", mem_get_info=fake(per // 2))
