"""Native continuous-batching core (csrc/runtime/sched_core.h) vs its Python
twin (runtime/scheduler.py PySchedCore): identical plans, readout events and
slot accounting on random workloads (joins at random steps, chunked prefill
under a token budget, EOS stops, several replicas and groups), plus the
engine end to end on each core.  CPU only."""
import random

import pytest

from llm_sharding_demo_amd.config import EngineConfig, SamplingParams
from llm_sharding_demo_amd.runtime.engine import Engine
from llm_sharding_demo_amd.runtime.kv_cache import SlotAllocator as PySlots
from llm_sharding_demo_amd.runtime.scheduler import EV_RELEASE, PySchedCore


def _rt():
    from llm_sharding_demo_amd.runtime.native import build, load

    build()
    rt = load()
    if rt is None or not hasattr(rt, "SchedCore"):
        pytest.skip("native runtime not importable")
    return rt


@pytest.mark.parametrize("policy", [(1, 0), (3, 2), (8, 4)])  # join policy (join_min, max_wait)
@pytest.mark.parametrize("collect", [False, True])
@pytest.mark.parametrize("seed", range(12))
def test_native_core_matches_python_twin(seed, collect, policy):
    rt = _rt()
    rnd = random.Random(seed)
    R, M = rnd.choice([1, 2]), rnd.choice([1, 2, 3])
    cap = rnd.choice([1, 2, 4, 8])
    slots = rnd.choice([cap * M * R, max(1, cap * M * R // 2), 3])
    budget = rnd.choice([0, 0, 5, 16, 64])
    chunk = rnd.choice([0, 0, 3, 8])
    max_seq, eos = 512, 7
    npool = [rt.SlotAllocator(slots) for _ in range(R)]
    ppool = [PySlots(slots) for _ in range(R)]
    nat = rt.SchedCore(R, M, cap, budget, chunk, max_seq, npool)
    py = PySchedCore(R, M, cap, budget, chunk, max_seq, ppool)
    nat.set_join_policy(*policy)
    py.set_join_policy(*policy)
    sid = 0
    pending = []  # (step, rep, g, n_tokens)
    got, fed = {}, {}  # finished token lists (collect) / tokens from plain events
    for step in range(400):
        if step < 150 and rnd.random() < 0.3:
            for _ in range(rnd.randint(1, 4)):
                L, want, stop = rnd.randint(1, 40), rnd.randint(1, 20), rnd.random() < 0.5
                nat.add(sid, L, want, stop)
                py.add(sid, L, want, stop)
                sid += 1
        assert nat.has_work() == py.has_work()
        if not py.has_work() and step >= 150:
            break
        pn, an = nat.plan(step)
        pp, ap = py.plan(step)
        assert an == ap
        assert [[tuple(go[:6]) + ([tuple(c) for c in go[6]], [tuple(r) for r in go[7]]) for go in rep]
                for rep in pn] == [[go[:6] + (go[6], go[7]) for go in rep] for rep in pp], step
        for rep, gos in enumerate(pp):
            for go in gos:
                if go[1]:
                    pending.append((step, rep, go[0], go[1]))
        # read back everything the GPU would have finished (a lag of 0-3 steps)
        lag = rnd.randint(0, 3)
        while pending and pending[0][0] <= step - lag:
            st, rep, g, n = pending.pop(0)
            toks = [rnd.choice([eos, 11, 12, 13]) for _ in range(n)]
            if collect:  # the serving fast path: tokens kept in the core
                import numpy as np

                en, dn = nat.assign_collect(rep, st, g, np.array(toks, dtype=np.int32), eos)
                ep, dp = py.assign_collect(rep, st, g, toks, eos)
                assert [tuple(e) for e in en] == ep and [(a, list(b)) for a, b in dn] == dp
                assert all(e[2] for e in ep)  # plain tokens never come back
                for sid_, tl in dp:
                    got.setdefault(sid_, tl)
            else:
                en = [tuple(e) for e in nat.assign(rep, st, g, toks, eos)]
                ep = py.assign(rep, st, g, toks, eos)
                assert en == ep
                for e in ep:
                    if e[1] >= 0:
                        fed.setdefault(e[0], []).append(e[1])
        assert [p.available for p in npool] == [p.available for p in ppool]
        assert (nat.joins, nat.leaves, nat.max_rows, nat.deferred) == (py.joins, py.leaves, py.max_rows, py.deferred)
    while pending:
        st, rep, g, n = pending.pop(0)
        if collect:
            import numpy as np

            en, dn = nat.assign_collect(rep, st, g, np.full(n, 11, dtype=np.int32), eos)
            ep, dp = py.assign_collect(rep, st, g, [11] * n, eos)
            assert [tuple(e) for e in en] == ep and [(a, list(b)) for a, b in dn] == dp
        else:
            assert [tuple(e) for e in nat.assign(rep, st, g, [11] * n, eos)] == py.assign(rep, st, g, [11] * n, eos)
    assert nat.n_expect == py.n_expect == 0
    # a finished sequence's list holds between 1 and `want` (<= 20) tokens
    for tl in got.values():
        assert 1 <= len(tl) <= 20


def test_native_core_release_and_reset():
    rt = _rt()
    pools = [rt.SlotAllocator(2)]
    c = rt.SchedCore(1, 1, 2, 0, 0, 64, pools)
    c.add(0, 3, 2, False)
    c.add(1, 2, 1, False)
    c.add(2, 2, 1, False)  # waits: no slot
    plans, adm = c.plan(0)
    assert adm == [0, 1] and pools[0].available == 0
    (g, ret, n, b, ctxb, changed, chunks, rows), = plans[0]
    assert [ch[4] for ch in chunks] == [True, True] and ret == 0 and b == 0
    plans, _ = c.plan(1)
    assert plans[0][0][1] == 2  # step 1 reads back the two prefill samples
    ev = [tuple(e) for e in c.assign(0, 1, 0, [5, 6], 50256)]
    assert ev == [(0, 5, 1), (1, 6, 3)]  # seq 1 is complete at its first token
    c.plan(2)  # both leave (every token issued); released at this item's readout
    ev = [tuple(e) for e in c.assign(0, 2, 0, [9, 9], 50256)]
    assert (0, 9, 2) in ev and any(e[0] == 1 and e[2] & EV_RELEASE for e in ev)
    c.reset()
    assert pools[0].available == 2 and not c.has_work()


@pytest.mark.parametrize("py_runtime", ["0", "1"])
def test_engine_on_each_core(monkeypatch, py_runtime):
    """The same generation through the native core and through the Python
    twin (LSD_PY_RUNTIME=1): identical tokens, all slots returned."""
    monkeypatch.setenv("LSD_PY_RUNTIME", py_runtime)
    eng = Engine(EngineConfig(model_id="gpt2-test", num_stages=2, max_batch=4, device="cpu",
                              prefill_chunk=3))
    core = type(eng.scheduler.core).__name__
    assert core == ("PySchedCore" if py_runtime == "1" else "SchedCore")
    prompts = [[1, 2, 3, 4, 5], [6], [7, 8], [9, 10, 11], [12, 13, 14, 15, 16, 17], [3, 3]]
    sp = [SamplingParams(temperature=0.9, top_k=8, seed=40 + i, max_new_tokens=3 + i) for i in range(6)]
    out = eng.generate_ids(prompts, sp, microbatches=2)
    assert [len(o) for o in out] == [3 + i for i in range(6)]
    assert eng.slots.available == eng.slots.capacity
    ref = Engine(EngineConfig(model_id="gpt2-test", max_batch=4, device="cpu"))
    assert out == ref.generate_ids(prompts, sp)


def test_core_stress_under_asan_ubsan(tmp_path):
    """csrc/runtime/tests/sched_core_stress.cpp: 40 random workloads through
    the native core under AddressSanitizer + UBSan (exact token counts, each
    sequence released once, no slot leaks, no pending readouts)."""
    import os
    import shutil
    import subprocess

    if shutil.which("g++") is None:
        pytest.skip("needs g++")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = tmp_path / "scs"
    r = subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined",
                        "-fno-omit-frame-pointer",
                        os.path.join(root, "csrc", "runtime", "tests", "sched_core_stress.cpp"),
                        "-o", str(exe)], capture_output=True, text=True)
    if r.returncode != 0 and "cannot find" in r.stderr:
        pytest.skip(f"sanitizer runtime not available: {r.stderr[-200:]}")
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, UBSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1")
    r = subprocess.run([str(exe), "40"], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert r.stdout.startswith("ok 40")


def test_add_many_matches_add():
    """SchedCore.add_many (bulk admission) == add() one by one, native and
    Python twin: same plans; an empty prompt anywhere rejects the whole batch."""
    rt = _rt()
    seqs = [(i, 1 + (7 * i) % 23, 1 + (5 * i) % 9, i % 2 == 0) for i in range(20)]
    plans = []
    for core in ("native", "py"):
        for bulk in (False, True):
            pool = [rt.SlotAllocator(16)] if core == "native" else [PySlots(16)]
            c = (rt.SchedCore if core == "native" else PySchedCore)(1, 2, 4, 0, 0, 512, pool)
            if bulk:
                c.add_many(*map(list, zip(*seqs)))
                with pytest.raises(ValueError):
                    c.add_many([99, 100], [3, 0], [1, 1], [False, False])
            else:
                for s in seqs:
                    c.add(*s)
            p, adm = c.plan(0)
            plans.append(([[(tuple(go[:6]), [tuple(x) for x in go[6]]) for go in rep] for rep in p], list(adm)))
    assert all(p == plans[0] for p in plans[1:])


@pytest.mark.parametrize("native", [False, True])
def test_join_policy_defers_until_room_or_wait(native):
    """join_min 4 / max_wait 3: a running group with one free row and a long
    queue defers its joins (deferred counts them) until 4 rows are free or it
    has deferred 3 steps; an idle group, or a queue shorter than join_min,
    joins at once -- so the bench's session shape (everything joins at step 0)
    and a lone request are never delayed."""
    if native:
        rt = _rt()
        core = rt.SchedCore(1, 1, 8, 0, 0, 512, [rt.SlotAllocator(64)])
    else:
        core = PySchedCore(1, 1, 8, 0, 0, 512, [PySlots(64)])
    core.set_join_policy(4, 3)
    for sid in range(8):  # idle group: all 8 join at step 0
        core.add(sid, 4, 2 + sid, False)
    _, adm = core.plan(0)
    assert sorted(adm) == list(range(8))
    for sid in range(8, 30):
        core.add(sid, 4, 50, False)
    joined_at = {}
    for step in range(1, 14):
        _, adm = core.plan(step)
        for sid in adm:
            joined_at[sid] = step
    # rows leave one per step from step 2 (want 2 + sid tokens): the first
    # joins wait for 4 free rows or 3 deferred steps, never joining one by one
    steps = sorted(set(joined_at.values()))
    assert steps and all(b - a >= 2 for a, b in zip(steps, steps[1:]))
    assert core.deferred >= 2
    core2 = PySchedCore(1, 1, 8, 0, 0, 512, [PySlots(64)])
    core2.set_join_policy(4, 3)
    core2.add(0, 4, 100, False)
    core2.plan(0)
    core2.add(1, 4, 100, False)  # fewer waiting than join_min: joins at once
    _, adm = core2.plan(1)
    assert adm == [1] and core2.deferred == 0
