"""Lockset race detector for the Python runtime (utils/racecheck.py), CPU.

The reference runs concurrent /generate calls in a threadpool over shared globals with
no locks (`server.py:154-155`).  Here the checker is enabled per process by
LSD_RACE_CHECK=1 (read at import), so every case runs in a subprocess:
  * it reports two threads writing a field with no common lock, and stays quiet when a
    tracked lock guards the writes or ownership is handed over explicitly;
  * tracked re-entrant locks work under threading.Condition wait / notify;
  * the multi-stage CPU engine (serving loop + stage threads + concurrent submitters)
    runs clean at 2, 3 and 4 stages.  The checker found one real race there: the
    watchdog heartbeat `round_started` was one slot written by the serving driver AND
    by every stage follower, so a follower's "step done" could clear the driver's
    in-flight start; it is now one slot per thread (engine._round).
"""
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(code: str, timeout: int = 300) -> str:
    env = dict(os.environ, LSD_RACE_CHECK="1", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", textwrap.dedent(code)], env=env, capture_output=True,
                       text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


TOY = """
import threading
from llm_sharding_demo_amd.utils import racecheck as rc
assert rc.ENABLED

class Box(rc.Shared):
    def __init__(self):
        self.n = 0

def hammer(box, lock, k=200):
    def go():
        for _ in range(k):
            if lock is None:
                box.n = box.n + 1
            else:
                with lock:
                    box.n = box.n + 1
    ts = [threading.Thread(target=go) for _ in range(2)]
    [t.start() for t in ts]
    [t.join() for t in ts]
"""


def test_unlocked_writes_from_two_threads_are_reported():
    out = _run(TOY + """
b = Box()
hammer(b, None)
r = rc.reports()
print(len(r), r[0]["object"], r[0]["field"])
""")
    assert out.split() == ["1", "Box", "n"]


def test_common_lock_and_handoff_are_quiet():
    out = _run(TOY + """
b = Box()
hammer(b, rc.Lock("box"))
c = Box()          # written by the main thread ...
c.n = 5
rc.handoff(c)      # ... handed to one worker thread
t = threading.Thread(target=lambda: setattr(c, "n", 6))
t.start(); t.join()
d = Box()          # two different locks: no common one -> reported
l1, l2 = rc.Lock("a"), rc.Lock("b")
def w(l):
    with l:
        d.n = d.n + 1
ts = [threading.Thread(target=w, args=(l,)) for l in (l1, l2)]
[t.start() for t in ts]; [t.join() for t in ts]
print([ (x["object"], x["field"]) for x in rc.reports() ])
""")
    assert out.strip() == "[('Box', 'n')]"  # only the two-lock case


def test_tracked_rlock_condition_wait_notify():
    out = _run("""
import threading, time
from llm_sharding_demo_amd.utils import racecheck as rc

class Q(rc.Shared):
    def __init__(self):
        self.cv = rc.Condition(name="q")
        self.items = 0

q = Q()
got = []
def consumer():
    with q.cv:
        with q.cv:  # re-entrant: wait() must release both levels
            q.cv.wait_for(lambda: q.items >= 3, timeout=30)
            got.append(q.items)
            q.items = 0
t = threading.Thread(target=consumer); t.start()
for _ in range(3):
    time.sleep(0.01)
    with q.cv:
        q.items = q.items + 1
        q.cv.notify_all()
t.join(30)
print(got, len(rc.reports()))
""")
    assert out.strip() == "[3] 0"


@pytest.mark.parametrize("P,transport", [(2, "auto"), (3, "auto"), (4, "auto"), (3, "strict")])
def test_multistage_engine_serving_is_race_free(P, transport):
    out = _run(f"""
import threading
from llm_sharding_demo_amd.utils import racecheck as rc
from llm_sharding_demo_amd.config import EngineConfig, SamplingParams
from llm_sharding_demo_amd.runtime.engine import Engine

PROMPTS = [[5, 6, 7, 8], [11], [300, 2, 9], [1, 2], [40, 41, 42, 43, 44], [9, 9], [3], [77, 1]]
eng = Engine(EngineConfig(model_id="gpt2-test", num_stages={P}, max_batch=8, device="cpu",
                          transport={transport!r}, num_microbatches=2))
solo = eng.generate_ids(PROMPTS, SamplingParams(greedy=True, max_new_tokens=5))
eng.start_loop()
outs = [None] * len(PROMPTS)
def go(i):
    outs[i] = eng.submit(PROMPTS[i], SamplingParams(greedy=True, max_new_tokens=5)).wait(120)
ts = [threading.Thread(target=go, args=(i,), name=f"api{{i}}") for i in range(len(PROMPTS))]
[t.start() for t in ts]; [t.join() for t in ts]
eng.stop_loop(); eng.shutdown()
assert outs == solo
for r in rc.reports():
    print("RACE", r["object"], r["field"], r["thread"], r["held"])
    print(r["stack"])
print("reports", len(rc.reports()))
""")
    assert "reports 0" in out, out


def test_round_started_is_per_thread():
    """The watchdog sees the oldest in-flight step of ANY thread; another thread
    finishing its own step does not clear it."""
    out = _run("""
import threading
from llm_sharding_demo_amd.runtime.engine import Engine
e = Engine.__new__(Engine)
object.__setattr__(e, "_rounds", {})
e._round(100.0)                       # driver thread inside a step since t = 100
t = threading.Thread(target=lambda: (e._round(105.0), e._round(None)))
t.start(); t.join()                   # a follower's step starts and ends
print(e.round_started)
e._round(None)
print(e.round_started)
""")
    assert out.split() == ["100.0", "None"]


@pytest.mark.gpu
@pytest.mark.parametrize("P,transport", [(2, "loopback"), (4, "loopback"), (3, "devloop")])
def test_loopback_gpu_engine_serving_is_race_free(P, transport):
    """The same check on one MI355X: P stage threads with the device-async
    loopback transport, the capture gate shared by the stage threads, graph
    capture and replay, the serving loop and concurrent submitters."""
    out = _run(f"""
import threading
from llm_sharding_demo_amd.utils import racecheck as rc
from llm_sharding_demo_amd.config import EngineConfig, SamplingParams
from llm_sharding_demo_amd.runtime.engine import Engine

PROMPTS = [[i + 1, 2 * i + 3, 5] for i in range(12)]
eng = Engine(EngineConfig(model_id="gpt2-test", num_stages={P}, max_batch=16, device="cuda",
                          num_microbatches=2 * {P}, transport={transport!r}))
eng.start_loop()
outs = [None] * len(PROMPTS)
def go(i):
    outs[i] = eng.submit(PROMPTS[i], SamplingParams(greedy=True, max_new_tokens=8)).wait(120)
ts = [threading.Thread(target=go, args=(i,)) for i in range(len(PROMPTS))]
[t.start() for t in ts]; [t.join() for t in ts]
eng.stop_loop(); eng.shutdown()
assert all(o is not None and len(o) == 8 for o in outs), outs
for r in rc.reports():
    print("RACE", r["object"], r["field"], r["thread"], r["held"])
    print(r["stack"])
print("reports", len(rc.reports()))
""", timeout=110)
    assert "reports 0" in out, out


def test_http_serving_is_race_free():
    """Concurrent /generate calls through the FastAPI app (handler threads), the
    serving loop, 2 stage threads, metrics and /metrics + /health readers."""
    out = _run("""
import threading
from fastapi.testclient import TestClient
from llm_sharding_demo_amd.utils import racecheck as rc
from llm_sharding_demo_amd.config import EngineConfig
from llm_sharding_demo_amd.runtime.engine import Engine
from llm_sharding_demo_amd.serving.server import create_app

cfg = EngineConfig(model_id="gpt2-test", num_stages=2, max_batch=8, device="cpu", metrics_every=1)
eng = Engine(cfg)
client = TestClient(create_app(cfg, engine=eng))
res = [None] * 8
def go(i):
    res[i] = client.post("/generate", json={"prompt": f"hi {i}", "max_new_tokens": 4, "greedy": True}).json()
    client.get("/metrics"); client.get("/health")
ts = [threading.Thread(target=go, args=(i,)) for i in range(8)]
[t.start() for t in ts]; [t.join() for t in ts]
assert all("generated" in r for r in res), res
eng.stop_loop()
for r in rc.reports():
    print("RACE", r["object"], r["field"], r["thread"], r["held"])
    print(r["stack"])
print("reports", len(rc.reports()))
""")
    assert "reports 0" in out, out


def test_finalizer_inside_a_locked_section_does_not_deadlock():
    """A weakref finalizer can run inside any allocation, also one made while
    this thread holds the checker's state lock (note() registers a finalizer
    there, and the collection that allocation triggers may finalize another
    tracked object): _forget only queues the id and never takes the lock."""
    import threading

    from llm_sharding_demo_amd.utils import racecheck

    done = threading.Event()

    def body():
        with racecheck._state_lock:
            racecheck._forget(12345)  # the old _forget re-acquired the lock: self-deadlock
        done.set()

    t = threading.Thread(target=body, daemon=True)
    t.start()
    t.join(5)
    assert done.is_set()
    with racecheck._state_lock:
        racecheck._drop_dead()
    assert 12345 not in racecheck._final
