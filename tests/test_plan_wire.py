"""Binary control-plane records (runtime/plan.py PlanEncoder / PlanDecoder):
every plan the scheduler can produce round-trips, steady-state decode plans
never pickle, and an unchanged composition costs a REPEAT record."""
import random

from llm_sharding_demo_amd.runtime.plan import (MAGIC_PICKLE, MAGIC_REPEAT, MAGIC_STEADY, Chunk,
                                                GroupPlan, PlanDecoder, PlanEncoder, Row, StepPlan)


def _rt(enc, dec, plan):
    rec, payload = enc.encode(plan)
    out = dec.decode(rec, lambda n: payload[:n])
    return rec, out


def test_round_trip_every_kind():
    enc, dec = PlanEncoder(), PlanDecoder()
    steady = StepPlan(step=7, replica=1, timing=True,
                      groups=[GroupPlan(g, ret=256, n=250, b=256, ctxb=512) for g in range(16)])
    rec, out = _rt(enc, dec, steady)
    assert rec[0] == MAGIC_STEADY and out == steady
    nxt = StepPlan(step=8, replica=1, timing=True,
                   groups=[GroupPlan(g, ret=256, n=250, b=256, ctxb=512) for g in range(16)])
    rec, out = _rt(enc, dec, nxt)
    assert rec[0] == MAGIC_REPEAT and out == nxt
    assert out.groups[0] is not nxt.groups[0]  # fresh objects (receives are keyed by id)
    joined = StepPlan(step=9, groups=[GroupPlan(0, ret=3, n=2, b=2, ctxb=256,
                                                rows=[Row(1, 4, 9, 0.6, 40, False, 3, 1, 0)],
                                                chunks=[Chunk(5, 6, 0, [1, 2, 3], True)])])
    rec, out = _rt(enc, dec, joined)
    assert rec[0] == MAGIC_PICKLE and out == joined
    rec, out = _rt(enc, dec, nxt)  # after a pickle: STEADY again, not REPEAT
    assert rec[0] == MAGIC_STEADY and out == nxt
    for p in (StepPlan(step=-1, end=True, timing=True), StepPlan(step=-1, stop=True),
              StepPlan(step=-2, groups=[GroupPlan(0, kind="fwd_b", fwd_rows=5)])):
        _, out = _rt(enc, dec, p)
        assert out == p


def test_random_plan_streams():
    rnd = random.Random(0)
    enc, dec = PlanEncoder(), PlanDecoder()
    kinds = {MAGIC_PICKLE: 0, MAGIC_REPEAT: 0, MAGIC_STEADY: 0}
    groups = [GroupPlan(g, ret=8, n=8, b=8, ctxb=256) for g in range(6)]
    for step in range(400):
        r = rnd.random()
        if r < 0.1:
            groups = [GroupPlan(g, ret=rnd.randrange(9), n=rnd.randrange(9), b=8,
                                ctxb=256 * rnd.randrange(1, 4)) for g in range(rnd.randrange(1, 7))]
        gs = [GroupPlan(gp.g, ret=gp.ret, n=gp.n, b=gp.b, ctxb=gp.ctxb) for gp in groups]
        if r > 0.95:
            gs[0].chunks = [Chunk(1, 2, 0, [5, 6], True)]
        plan = StepPlan(step=step, groups=gs)
        rec, out = _rt(enc, dec, plan)
        kinds[int(rec[0])] += 1
        assert out == plan
    assert kinds[MAGIC_REPEAT] > kinds[MAGIC_STEADY] > 0 and kinds[MAGIC_PICKLE] > 0


def test_columnar_groups_and_token_ids_only_where_read():
    """Non-steady plans travel with each GroupPlan as columns (runtime/plan.py
    _pack_group): exact round trip of every Chunk / Row field (large seeds,
    fp64 temperatures, greedy flags, rows=[] vs None); an encoder for stages
    that never read prefill token ids (ids=False) sends the chunk lengths only,
    and its payload is several times smaller."""
    rnd = random.Random(5)

    def chunk(i):
        n = rnd.randint(1, 40)
        return Chunk(i, rnd.randrange(4096), rnd.randrange(512), [rnd.randrange(50257) for _ in range(n)],
                     rnd.random() < 0.5, rnd.random() + 0.05, rnd.randint(1, 64), rnd.random() < 0.3,
                     rnd.randrange(1 << 62))

    def row(i):
        return Row(i, rnd.randrange(4096), rnd.randrange(1024), rnd.random() + 0.05, rnd.randint(1, 64),
                   rnd.random() < 0.3, rnd.randrange(1 << 62), rnd.randrange(1 << 40), rnd.randrange(512))

    plan = StepPlan(step=3, replica=1, timing=True, groups=[
        GroupPlan(0, ret=5, n=4, b=8, ctxb=256, chunks=[chunk(i) for i in range(300)], rows=[row(i) for i in range(7)]),
        GroupPlan(1, ret=0, n=0, b=0, ctxb=0, rows=[]),
        GroupPlan(2, ret=2, n=2, b=2, ctxb=256, chunks=[chunk(1000)]),
        GroupPlan(3, kind="fwd_b", fwd_rows=9)])
    rec, out = _rt(PlanEncoder(), PlanDecoder(), plan)
    assert rec[0] == MAGIC_PICKLE and out == plan
    assert out.groups[1].rows == [] and out.groups[2].rows is None
    full = rec[1]
    rec, out = _rt(PlanEncoder(ids=False), PlanDecoder(), plan)
    assert rec[1] * 2 < full
    for a, b in zip(out.groups, plan.groups):
        assert [c.qlen for c in a.chunks] == [c.qlen for c in b.chunks]
        assert [(c.seq, c.slot, c.start, c.final, c.temperature, c.top_k, c.greedy, c.seed) for c in a.chunks] == \
            [(c.seq, c.slot, c.start, c.final, c.temperature, c.top_k, c.greedy, c.seed) for c in b.chunks]
        assert a.rows == b.rows and (a.g, a.ret, a.n, a.b, a.ctxb, a.kind, a.fwd_rows) == \
            (b.g, b.ret, b.n, b.b, b.ctxb, b.kind, b.fwd_rows)
