"""Sampler properties + HTTP API contract tests.

Sampler: reference semantics `server.py:187-206` (T=0.6, top-k=40, softmax
over the k values, multinomial).  Sampling is stochastic, so we test support
(only top-k ids), distribution (matches softmax of the top-k at T), seeded
reproducibility, and greedy determinism.

API: the three reference paths and schemas (`server.py:116-151`), the
role guards that answer HTTP 200 + error (quirk Q8), and the notebook client
contract (`notebook.ipynb:111-120`).
"""
import collections

import pytest
import torch

from llm_sharding_demo_amd.config import EngineConfig, SamplingParams
from llm_sharding_demo_amd.ops import reference as ref
from llm_sharding_demo_amd.runtime.batch import counter_uniform
from llm_sharding_demo_amd.runtime.engine import Engine
from llm_sharding_demo_amd.utils.tokenizer import ByteTokenizer, bytes_to_unicode_order


def _sample(logits, T, k, greedy, seeds, step):
    B = logits.shape[0]
    u = counter_uniform(torch.tensor(seeds), torch.full((B,), step))
    return ref.sample(logits, torch.full((B,), T), torch.full((B,), k, dtype=torch.int32),
                      torch.full((B,), int(greedy), dtype=torch.int32), u, logits.shape[1])


def test_topk_support_and_distribution():
    torch.manual_seed(0)
    logits = torch.randn(1, 500) * 3
    top = set(torch.topk(logits[0], 40).indices.tolist())
    counts = collections.Counter()
    n = 3000
    for s in range(n):
        t = int(_sample(logits, 0.6, 40, False, [1234], s)[0])
        assert t in top
        counts[t] += 1
    vals, idx = torch.topk(logits[0] / 0.6, 40)
    p = torch.softmax(vals, 0)
    for j in range(5):  # the most likely ids appear at ~their probability
        assert abs(counts[int(idx[j])] / n - float(p[j])) < 0.05


def test_greedy_and_seeded_reproducible():
    logits = torch.randn(4, 300)
    g = _sample(logits, 1.0, 10, True, [1, 2, 3, 4], 0)
    assert g.tolist() == logits.argmax(1).tolist()
    a = _sample(logits, 0.7, 20, False, [7, 8, 9, 10], 3)
    b = _sample(logits, 0.7, 20, False, [7, 8, 9, 10], 3)
    assert a.tolist() == b.tolist()


def test_counter_uniform_range():
    u = counter_uniform(torch.arange(1000), torch.arange(1000))
    assert float(u.min()) >= 0 and float(u.max()) < 1
    assert 0.4 < float(u.mean()) < 0.6


def test_engine_seeded_sampling_reproducible_across_stage_counts():
    sp = SamplingParams(temperature=0.6, top_k=40, seed=99, max_new_tokens=6)
    outs = []
    for P in (1, 2, 4):
        eng = Engine(EngineConfig(model_id="gpt2-test", num_stages=P, max_batch=4, device="cpu"))
        outs.append(eng.generate_ids([[1, 2, 3], [4]], [sp, sp]))
    assert outs[0] == outs[1] == outs[2]


def test_byte_tokenizer_roundtrip_and_gpt2_ids():
    tok = ByteTokenizer()
    s = "Hi, ünïcode!"
    ids = tok.encode(s)
    assert tok.decode(ids) == s
    assert tok.encode("!") == [0]  # GPT-2 vocab id of "!" is 0
    assert len(set(bytes_to_unicode_order())) == 256
    assert tok.decode([50256]) == ""  # eos skipped like skip_special_tokens=True


# ---------------------------------------------------------------------------
# HTTP API
# ---------------------------------------------------------------------------

@pytest.fixture(scope="module")
def clients():
    from fastapi.testclient import TestClient

    from llm_sharding_demo_amd.serving.server import ShardRunner, create_app

    base = EngineConfig(model_id="gpt2-test", max_batch=4, device="cpu", split_points=[2])
    coord = create_app(base.replace(role="coordinator", num_stages=2),
                       engine=Engine(base.replace(num_stages=2)))
    a = create_app(base.replace(role="a"), shard=ShardRunner(base, "a"))
    b = create_app(base.replace(role="b"), shard=ShardRunner(base, "b"))
    return TestClient(coord), TestClient(a), TestClient(b)


def test_openapi_paths(clients):
    c, _, _ = clients
    paths = set(c.get("/openapi.json").json()["paths"])
    assert {"/forward", "/forward_b", "/generate"} <= paths


def test_role_guards_return_200_error(clients):
    c, a, b = clients
    r = c.post("/forward", json={"input_ids": [1, 2]})
    assert r.status_code == 200 and r.json() == {"error": "This instance is not shard A."}
    r = a.post("/forward_b", json={"hidden_states": [[[0.0] * 128]]})
    assert r.status_code == 200 and r.json() == {"error": "This instance is not shard B."}
    r = b.post("/generate", json={"prompt": "x"})
    assert r.status_code == 200 and r.json() == {"error": "This instance is not coordinator."}


def test_generate_contract(clients):
    c, _, _ = clients
    r = c.post("/generate", json={"prompt": "Hi, ", "max_new_tokens": 3, "greedy": True})
    assert r.status_code == 200
    assert r.json()["generated"].startswith("Hi, ")
    assert c.post("/generate", json={"prompt": "Hi", "max_new_tokens": 0}).json() == {"generated": "Hi"}
    assert c.post("/generate", json={"max_new_tokens": 3}).status_code == 422  # missing prompt
    assert c.post("/generate", json={"prompt": "", "max_new_tokens": 3}).status_code == 422
    assert c.post("/generate", json={"prompt": "x" * 2000, "max_new_tokens": 3}).status_code == 422


def test_shard_a_then_b_equals_engine_logits(clients):
    """The reference's two-hop path, A then B, over HTTP: logits equal the
    unsplit model's (the engine) -- the split is exact (fixes quirk Q1)."""
    c, a, b = clients
    ids = [5, 6, 7, 8, 9]
    h = a.post("/forward", json={"input_ids": ids}).json()["hidden_states"]
    assert len(h) == 1 and len(h[0]) == len(ids) and len(h[0][0]) == 128
    lg = torch.tensor(b.post("/forward_b", json={"hidden_states": h}).json()["logits"])
    assert lg.shape == (1, len(ids), 1000)
    from llm_sharding_demo_amd.models.stage import StageModel
    from llm_sharding_demo_amd.runtime.batch import BatchMeta
    from llm_sharding_demo_amd.config import get_model_config

    mc = get_model_config("gpt2-test")
    st = StageModel(mc, 0, mc.n_layers, True, True, max_slots=1, max_seq=64)
    full = st.forward(BatchMeta.build([0], [0], [len(ids)], "cpu"),
                      torch.tensor(ids, dtype=torch.int32), all_logits=True)[:, :1000]
    torch.testing.assert_close(lg[0], full, atol=1e-4, rtol=1e-4)


def test_health_and_metrics(clients):
    c, a, _ = clients
    h = c.get("/health").json()
    assert h["status"] == "ok" and h["stages"] == 2
    assert a.get("/health").json()["layers"] == [0, 2]
    c.post("/generate", json={"prompt": "abc", "max_new_tokens": 2})
    m = c.get("/metrics").text
    assert "llmshard_output_tokens_total" in m and "llmshard_kv_slots_total" in m


def test_generate_text_client_contract(monkeypatch):
    import requests

    from llm_sharding_demo_amd.serving import client

    class R:
        def __init__(self, code, body):
            self.status_code, self._b, self.text = code, body, str(body)

        def json(self):
            return self._b

    monkeypatch.setattr(requests, "post", lambda *a, **k: R(200, {"generated": "Hi, x"}))
    assert client.generate_text("Hi, ", max_new_tokens=2) == {"generated": "Hi, x"}
    monkeypatch.setattr(requests, "post", lambda *a, **k: R(500, "boom"))
    assert client.generate_text("Hi, ") == "Error: 500 - boom"

    def raise_(*a, **k):
        raise requests.exceptions.ConnectionError("refused")

    monkeypatch.setattr(requests, "post", raise_)
    assert client.generate_text("Hi, ").startswith("Request failed: ")
