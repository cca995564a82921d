"""Request batching + round watchdog (runtime/scheduler.py), CPU.

Reference behaviour: concurrent /generate calls run
independent decode loops, and a dead shard shows up only as a 30 s HTTP
timeout per hop.  Here concurrent requests must share pipeline rounds with
outputs identical to running them alone, and a hung round must flip /health
and fail requests fast.
"""
import threading
import time

import pytest

from llm_sharding_demo_amd.config import EngineConfig, SamplingParams
from llm_sharding_demo_amd.runtime.engine import Engine
from llm_sharding_demo_amd.runtime.scheduler import RequestBatcher, RequestTimeout, Watchdog

PROMPTS = [[5, 6, 7, 8], [11], [300, 2, 9], [1, 2], [40, 41, 42, 43, 44], [9, 9], [3], [77, 1]]


def _engine(P=2, max_batch=8):
    return Engine(EngineConfig(model_id="gpt2-test", num_stages=P, max_batch=max_batch, device="cpu"))


def test_concurrent_requests_share_rounds_and_match_solo():
    sp = SamplingParams(greedy=True, max_new_tokens=5)
    solo = _engine().generate_ids(PROMPTS, sp)
    eng = _engine()
    b = RequestBatcher(eng, window_ms=200)
    outs = [None] * len(PROMPTS)

    def go(i):
        outs[i] = b.generate(PROMPTS[i], SamplingParams(greedy=True, max_new_tokens=5), timeout=60)

    ts = [threading.Thread(target=go, args=(i,)) for i in range(len(PROMPTS))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    b.close()
    assert outs == solo
    assert b.stats["requests"] == len(PROMPTS)
    assert b.stats["batches"] < len(PROMPTS)  # requests were coalesced
    assert eng.slots.available == eng.slots.capacity


def test_seeded_sampling_independent_of_batching():
    sp = [SamplingParams(temperature=0.8, top_k=20, seed=100 + i, max_new_tokens=6)
          for i in range(len(PROMPTS))]
    solo = [_engine(P=1).generate_ids([p], [s])[0] for p, s in zip(PROMPTS, sp)]
    eng = _engine()
    b = RequestBatcher(eng, window_ms=200)
    reqs = [b.submit(p, s) for p, s in zip(PROMPTS, sp)]
    outs = [r.wait(60) for r in reqs]
    b.close()
    assert outs == solo


def test_length_groups_and_more_requests_than_slots():
    eng = _engine(max_batch=3)
    b = RequestBatcher(eng, window_ms=200)
    lens = [1, 2, 16, 3, 20, 1, 2]
    reqs = [b.submit([1 + i, 2], SamplingParams(greedy=True, max_new_tokens=n)) for i, n in enumerate(lens)]
    outs = [r.wait(60) for r in reqs]
    b.close()
    assert [len(o) for o in outs] == lens
    # a 1-token request never waits for the 20-token round
    assert reqs[0].t_done <= reqs[4].t_done


def test_round_error_fails_group_not_batcher():
    eng = _engine()
    b = RequestBatcher(eng, window_ms=50)
    with pytest.raises(ValueError):
        b.generate([], SamplingParams(greedy=True, max_new_tokens=2), timeout=30)
    eng.healthy = True  # a bad request is not an engine fault
    eng.last_error = None
    assert len(b.generate([1, 2], SamplingParams(greedy=True, max_new_tokens=2), timeout=30)) == 2
    b.close()


class _SlowEngine:
    """Stand-in whose round hangs (a dead RCCL peer)."""

    def __init__(self):
        self.healthy, self.last_error, self.round_started = True, None, None
        self.R = 1
        self.slots = type("S", (), {"capacity": 4})()
        self.release = threading.Event()

    def generate_ids(self, prompts, params, **kw):
        self.round_started = time.monotonic()
        self.release.wait(30)
        self.round_started = None
        return [[0] for _ in prompts]


def test_watchdog_marks_unhealthy_and_requests_fail_fast():
    eng = _SlowEngine()
    wd = Watchdog(eng, round_timeout_s=0.3, poll_s=0.05)
    b = RequestBatcher(eng, window_ms=1)
    req = b.submit([1], SamplingParams(greedy=True, max_new_tokens=1))
    with pytest.raises(RequestTimeout):
        req.wait(timeout=0.8)
    assert not eng.healthy and "deadline" in eng.last_error and wd.fired
    with pytest.raises(RuntimeError, match="unhealthy"):
        b.submit([2], SamplingParams(greedy=True, max_new_tokens=1))
    eng.release.set()
    assert req.wait(5) == [0]
    b.close()
    wd.close()


def test_http_concurrent_generate_batched():
    from fastapi.testclient import TestClient

    from llm_sharding_demo_amd.serving.server import create_app

    cfg = EngineConfig(model_id="gpt2-test", num_stages=2, max_batch=8, device="cpu",
                       batch_window_ms=200)
    eng = Engine(cfg)
    app = create_app(cfg, engine=eng)
    client = TestClient(app)
    res = [None] * 6

    def go(i):
        r = client.post("/generate", json={"prompt": f"hi {i}", "max_new_tokens": 4, "greedy": True})
        res[i] = r.json()

    ts = [threading.Thread(target=go, args=(i,)) for i in range(6)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert all("generated" in r and r["generated"].startswith(f"hi {i}") for i, r in enumerate(res))
    m = client.get("/metrics").text
    assert "llmshard_batched_requests_total 6" in m
    assert "llmshard_stage1_busy_fraction" in m and "llmshard_token_latency_p50_ms" in m
    assert app.state.batcher.stats["batches"] < 6
