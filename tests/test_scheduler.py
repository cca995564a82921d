"""Continuous (iteration-level) batching + progress watchdog
(runtime/scheduler.py, runtime/engine.py), CPU.

Reference behaviour (`server.py:154-155`): concurrent
/generate calls run independent decode loops, so a short request never waits
for a long one, and a dead shard shows up only as a 30 s HTTP timeout per hop.
Here concurrent requests share pipeline steps with outputs identical to
running them alone, a request joins a running batch at the next decode step
and leaves when it has its tokens, and a stalled pipeline flips /health and
fails requests fast.
"""
import threading
import time

import pytest

from llm_sharding_demo_amd.config import EngineConfig, SamplingParams
from llm_sharding_demo_amd.runtime.engine import Engine
from llm_sharding_demo_amd.runtime.scheduler import RequestTimeout, Watchdog

PROMPTS = [[5, 6, 7, 8], [11], [300, 2, 9], [1, 2], [40, 41, 42, 43, 44], [9, 9], [3], [77, 1]]


def _engine(P=2, max_batch=8, **kw):
    return Engine(EngineConfig(model_id="gpt2-test", num_stages=P, max_batch=max_batch,
                               device="cpu", **kw))


def test_concurrent_requests_share_steps_and_match_solo():
    sp = SamplingParams(greedy=True, max_new_tokens=5)
    solo = _engine().generate_ids(PROMPTS, sp)
    eng = _engine()
    eng.start_loop()
    outs = [None] * len(PROMPTS)

    def go(i):
        outs[i] = eng.submit(PROMPTS[i], SamplingParams(greedy=True, max_new_tokens=5)).wait(60)

    ts = [threading.Thread(target=go, args=(i,)) for i in range(len(PROMPTS))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    eng.stop_loop()
    assert outs == solo
    st = eng.scheduler.stats
    assert st["joins"] == len(PROMPTS) and st["leaves"] == len(PROMPTS)
    assert st["max_rows"] > 1  # requests decoded side by side
    assert eng.slots.available == eng.slots.capacity
    eng.shutdown()


def test_short_request_joins_running_batch_and_finishes_first():
    """A 2-token request submitted while a 500-token generation is running
    joins at the next step boundary and completes long before it."""
    eng = _engine(P=2, max_batch=4, max_seq_len=1024)
    eng.start_loop()
    long = eng.submit([1, 2, 3], SamplingParams(greedy=True, max_new_tokens=500))
    while eng.scheduler.stats["steps"] < 20:  # the long one is decoding
        time.sleep(0.005)
    short = eng.submit([7, 8], SamplingParams(greedy=True, max_new_tokens=2))
    assert len(short.wait(60)) == 2
    assert not long.done  # still generating when the short one finished
    assert len(long.wait(120)) == 500
    assert short.t_done < long.t_done
    # the short one reused nothing of the long one's output: same as alone
    assert short.output == _engine(P=1).generate_ids([[7, 8]], SamplingParams(greedy=True,
                                                                              max_new_tokens=2))[0]
    eng.stop_loop()
    eng.shutdown()


def test_seeded_sampling_independent_of_batching():
    sp = [SamplingParams(temperature=0.8, top_k=20, seed=100 + i, max_new_tokens=6)
          for i in range(len(PROMPTS))]
    solo = [_engine(P=1).generate_ids([p], [s])[0] for p, s in zip(PROMPTS, sp)]
    eng = _engine()
    eng.start_loop()
    reqs = []
    for p, s in zip(PROMPTS, sp):  # staggered arrivals: different batch compositions
        reqs.append(eng.submit(p, s))
        time.sleep(0.002)
    outs = [r.wait(60) for r in reqs]
    eng.stop_loop()
    assert outs == solo


def test_more_requests_than_slots_and_mixed_lengths():
    eng = _engine(max_batch=3)
    lens = [1, 2, 16, 3, 20, 1, 2]
    ps = [SamplingParams(greedy=True, max_new_tokens=n) for n in lens]
    outs = eng.generate_ids([[1 + i, 2] for i in range(len(lens))], ps)
    assert [len(o) for o in outs] == lens
    assert eng.slots.available == eng.slots.capacity


def test_eos_stop_leaves_early():
    eng = _engine(P=1)
    base = eng.generate_ids([[5, 6]], SamplingParams(greedy=True, max_new_tokens=12))[0]
    eos = base[3]
    eng.mcfg = type(eng.mcfg)(**{**eng.mcfg.__dict__, "eos_token_id": eos})
    out = eng.generate_ids([[5, 6]], SamplingParams(greedy=True, max_new_tokens=12,
                                                    stop_at_eos=True))[0]
    assert out == base[: base.index(eos) + 1]
    assert eng.slots.available == eng.slots.capacity


def test_bad_request_does_not_hurt_engine():
    eng = _engine()
    eng.start_loop()
    with pytest.raises(ValueError):
        eng.submit([], SamplingParams(greedy=True, max_new_tokens=2))
    assert eng.healthy
    assert len(eng.submit([1, 2], SamplingParams(greedy=True, max_new_tokens=2)).wait(30)) == 2
    eng.stop_loop()


def test_watchdog_marks_unhealthy_and_requests_fail_fast():
    def fault(edge, src, dst, seq):
        return 1.5 if seq >= 2 else None  # the link stalls after two messages

    eng = Engine(EngineConfig(model_id="gpt2-test", num_stages=2, max_batch=4, device="cpu"),
                 fault=fault)
    wd = Watchdog(eng, round_timeout_s=0.3, poll_s=0.05)
    eng.start_loop()
    req = eng.submit([1], SamplingParams(greedy=True, max_new_tokens=20))
    with pytest.raises((RequestTimeout, RuntimeError)):
        req.wait(timeout=10)
    assert not eng.healthy and "progress" in eng.last_error and wd.fired
    with pytest.raises(RuntimeError, match="unhealthy"):
        eng.submit([2], SamplingParams(greedy=True, max_new_tokens=1))
    wd.close()


def test_http_concurrent_generate_and_metrics():
    from fastapi.testclient import TestClient

    from llm_sharding_demo_amd.serving.server import create_app

    cfg = EngineConfig(model_id="gpt2-test", num_stages=2, max_batch=8, device="cpu",
                       metrics_every=1)
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
    assert "# TYPE llmshard_requests_total counter" in m and "llmshard_requests_total 6" in m
    assert "llmshard_output_tokens_total 24" in m
    assert "llmshard_sequence_joins_total 6" in m
    assert "llmshard_stage1_busy_fraction" in m and "llmshard_token_latency_p50_ms" in m
    assert "llmshard_time_to_first_token_p50_s" in m
    h = client.get("/health").json()
    assert h["kv_slots"] == 8 and h["status"] == "ok"
    eng.stop_loop()


def test_metrics_throughput_is_wall_clock():
    """N concurrent requests finishing together: tok/s is tokens over the
    wall-clock span, not over the summed request latencies."""
    from llm_sharding_demo_amd.utils.metrics import Metrics

    m = Metrics()
    t0 = time.monotonic()
    time.sleep(0.2)
    for _ in range(4):  # 4 overlapping requests of 0.2 s, 10 tokens each
        m.observe_request(10, time.monotonic() - t0)
    tps = m.tokens_per_second()
    assert 120 < tps < 220, tps  # ~40 tokens / 0.2 s, not 40 / 0.8 s


def test_watchdog_aborts_data_plane_on_async_error_and_timeout():
    """The watchdog fires on a data-plane async error (polled every tick) and
    on a stalled round, marks the engine unhealthy and aborts the transport
    (the native RCCL transport's abort unblocks kernels waiting on a dead
    peer; tests/test_comm_abort_gpu.py covers that half on the GPU)."""
    import time
    from types import SimpleNamespace

    from llm_sharding_demo_amd.runtime.scheduler import Watchdog

    class FakeTransport:
        def __init__(self, err=None):
            self.err, self.aborts = err, 0

        def check_async(self):
            return self.err

        def abort(self):
            self.aborts += 1

    tr = FakeTransport("RCCL r0fwd0/lane1: remote process exited")
    eng = SimpleNamespace(transport=tr, healthy=True, last_error=None, round_started=None)
    wd = Watchdog(eng, round_timeout_s=60, poll_s=0.02)
    deadline = time.monotonic() + 5
    while eng.healthy and time.monotonic() < deadline:
        time.sleep(0.02)
    wd.close()
    assert not eng.healthy and eng.last_error.startswith("DataPlaneError") and tr.aborts == 1

    tr2 = FakeTransport()
    eng2 = SimpleNamespace(transport=tr2, healthy=True, last_error=None,
                           round_started=time.monotonic())
    wd2 = Watchdog(eng2, round_timeout_s=0.2, poll_s=0.02)
    deadline = time.monotonic() + 5
    while eng2.healthy and time.monotonic() < deadline:
        time.sleep(0.02)
    wd2.close()
    assert not eng2.healthy and eng2.last_error.startswith("WatchdogTimeout") and tr2.aborts == 1


def test_bulk_submit_matches_one_by_one_and_converts_ids():
    """generate_ids admits a batch through Scheduler.submit_many (one pass,
    native push_many / add_many): same tokens as submitting one by one, numpy
    token ids converted, zero-token requests finished at once."""
    import numpy as np

    from llm_sharding_demo_amd.runtime.scheduler import Request

    prompts = [[5, 6, 7], np.array([9, 8], dtype=np.int64), [1] * 7, [4, 4]]
    sps = [SamplingParams(temperature=0.7, top_k=10, seed=s, max_new_tokens=n) for s, n in
           ((1, 5), (2, 3), (3, 0), (4, 6))]
    e = _engine(max_batch=8)
    bulk = e.generate_ids(prompts, sps)
    assert bulk[2] == [] and [len(t) for t in bulk] == [5, 3, 0, 6]
    e2 = _engine(max_batch=8)
    reqs = [e2.submit(list(map(int, p)), sp) for p, sp in zip(prompts, sps)]
    e2.start_loop()
    try:
        assert [r.wait(60) for r in reqs] == bulk
    finally:
        e2.stop_loop()
    reqs = e.scheduler.submit_many([np.array([3, 2], dtype=np.int32)], [sps[0]])
    assert reqs[0].prompt_ids == [3, 2] and all(type(t) is int for t in reqs[0].prompt_ids)
    e.scheduler.fail_all(RuntimeError("drop"))
    with pytest.raises(RuntimeError, match="drop"):
        reqs[0].wait(1)
    # the completion event is made lazily: a waiter blocked before finish() wakes up
    r = Request([1], sps[0])
    threading.Timer(0.05, lambda: r.finish([7])).start()
    assert r.wait(5) == [7] and r.done
    with pytest.raises(RequestTimeout):
        Request([1], sps[0]).wait(0.01)


@pytest.mark.parametrize("greedy", [True, False])
def test_mixed_steps_match_separate_forwards(greedy):
    """One stage: a group that decodes rows AND prefills joining prompts in the
    same step runs one forward over both (pipeline.py _mixed, MixedMeta) --
    same tokens as the decode graph + separate prefill forward, with seeded
    sampling too; requests join a running batch at different steps."""
    import random

    rnd = random.Random(3)
    prompts = [[rnd.randrange(1, 200) for _ in range(rnd.randint(2, 9))] for _ in range(12)]
    sps = [SamplingParams(greedy=greedy, temperature=0.8, top_k=20, seed=100 + i,
                          max_new_tokens=rnd.randint(2, 12)) for i in range(12)]

    def run(mixed: bool):
        e = _engine(P=1, max_batch=16, num_microbatches=2)
        for w in e.workers:
            w.mixed_steps = mixed
        e.start_loop()
        try:
            reqs = []
            for i, (p, sp) in enumerate(zip(prompts, sps)):
                reqs.append(e.submit(p, sp))
                if i % 3 == 2:  # let the running batch advance before more join
                    st = e.scheduler.stats["steps"]
                    while e.scheduler.stats["steps"] < st + 2 and not all(r.done for r in reqs):
                        time.sleep(0.001)
            out = [r.wait(60) for r in reqs]
        finally:
            e.stop_loop()
        return out, sum(w.mixed_items for w in e.workers)

    sep, n_sep = run(False)
    mix, n_mix = run(True)
    assert n_sep == 0 and n_mix > 0
    assert mix == sep
