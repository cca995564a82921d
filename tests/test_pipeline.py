"""Pipeline protocol tests (CPU): partition invariance, microbatching, fake
transport fault injection, and a real multi-process gloo pipeline.

Reference behaviour being generalised: 2-stage split at SPLIT_AT
(`server.py:63-64`), which with the shipped manifests is inconsistent between
the shards (quirk Q1).  Any plan here must reproduce the unsplit model.
"""
import os
import socket
import subprocess
import sys
import textwrap

import pytest
import torch
from hypothesis import given, settings
from hypothesis import strategies as st

from llm_sharding_demo_amd.config import EngineConfig, SamplingParams, get_model_config
from llm_sharding_demo_amd.parallel.comm import TransportError
from llm_sharding_demo_amd.parallel.partition import (auto_partition, make_plan, plan_from_splits,
                                                      stage_costs, validate_plan)
from llm_sharding_demo_amd.runtime.engine import Engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROMPTS = [[5, 6, 7, 8], [11], [300, 2, 9], [1, 2], [40, 41, 42, 43, 44]]


@pytest.fixture(scope="module")
def golden():
    eng = Engine(EngineConfig(model_id="gpt2-test", num_stages=1, max_batch=8, device="cpu"))
    return eng.generate_ids(PROMPTS, SamplingParams(greedy=True, max_new_tokens=6))


def test_plan_validation():
    assert plan_from_splits(4, [1, 3]) == [(0, 1), (1, 3), (3, 4)]
    with pytest.raises(ValueError):
        validate_plan([(0, 2), (1, 4)], 4)  # overlap: the reference's Q1 bug
    with pytest.raises(ValueError):
        validate_plan([(0, 2)], 4)
    with pytest.raises(ValueError):
        make_plan(get_model_config("gpt2-test"), 3, [2])


def test_auto_partition_balances_lm_head():
    mc = get_model_config("gpt2")
    plan = auto_partition(mc, 4)
    costs = stage_costs(mc, plan)
    # last stage carries lm_head (5.4 blocks' worth for GPT-2 small): it gets fewer blocks
    assert plan[-1][1] - plan[-1][0] <= plan[0][1] - plan[0][0]
    even = [(0, 3), (3, 6), (6, 9), (9, 12)]
    assert max(costs) <= max(stage_costs(mc, even)) + 1


@settings(max_examples=6, deadline=None)
@given(st.lists(st.integers(1, 3), min_size=1, max_size=3).filter(lambda xs: sum(xs) < 4))
def test_any_partition_matches_unsplit(golden, cuts):
    splits, acc = [], 0
    for c in cuts:
        acc += c
        splits.append(acc)
    cfg = EngineConfig(model_id="gpt2-test", num_stages=len(splits) + 1, split_points=splits,
                       max_batch=8, device="cpu")
    out = Engine(cfg).generate_ids(PROMPTS, SamplingParams(greedy=True, max_new_tokens=6))
    assert out == golden


@pytest.mark.parametrize("P,M", [(2, 1), (2, 2), (3, 5), (4, 2)])
def test_microbatch_counts(golden, P, M):
    cfg = EngineConfig(model_id="gpt2-test", num_stages=P, max_batch=8, device="cpu")
    out = Engine(cfg).generate_ids(PROMPTS, SamplingParams(greedy=True, max_new_tokens=6),
                                   microbatches=M)
    assert out == golden


def test_per_request_lengths_and_zero_tokens():
    eng = Engine(EngineConfig(model_id="gpt2-test", num_stages=2, max_batch=8, device="cpu"))
    ps = [SamplingParams(greedy=True, max_new_tokens=n) for n in (3, 0, 5)]
    out = eng.generate_ids([[1, 2], [3], [4, 5, 6]], ps)
    assert [len(o) for o in out] == [3, 0, 5]


def test_more_requests_than_slots(golden):
    eng = Engine(EngineConfig(model_id="gpt2-test", num_stages=2, max_batch=2, device="cpu"))
    out = eng.generate_ids(PROMPTS, SamplingParams(greedy=True, max_new_tokens=6))
    assert out == golden
    assert eng.slots.available == 2


def test_fault_injection_fails_cleanly_and_marks_unhealthy():
    def fault(edge, src, dst, seq):
        if edge == "fwd" and seq == 3:
            return "drop"
        return None

    eng = Engine(EngineConfig(model_id="gpt2-test", num_stages=2, max_batch=4, device="cpu"),
                 fault=fault)
    eng.fabric.timeout = 2.0
    with pytest.raises(TransportError):
        eng.generate_ids([[1, 2, 3]], SamplingParams(greedy=True, max_new_tokens=8))
    assert not eng.healthy
    with pytest.raises(RuntimeError, match="unhealthy"):
        eng.generate_ids([[1]], SamplingParams(greedy=True, max_new_tokens=1))


def test_stage_exception_propagates():
    def fault(edge, src, dst, seq):
        return RuntimeError("injected stage failure") if seq == 1 else None

    eng = Engine(EngineConfig(model_id="gpt2-test", num_stages=3, max_batch=4, device="cpu"),
                 fault=fault)
    eng.fabric.timeout = 2.0
    with pytest.raises((RuntimeError, TransportError)):
        eng.generate_ids([[1, 2, 3]], SamplingParams(greedy=True, max_new_tokens=4))
    assert not eng.healthy


def test_delayed_links_still_correct(golden):
    import random

    rnd = random.Random(0)

    def fault(edge, src, dst, seq):
        return rnd.random() * 0.01

    eng = Engine(EngineConfig(model_id="gpt2-test", num_stages=3, max_batch=8, device="cpu"),
                 fault=fault)
    assert eng.generate_ids(PROMPTS, SamplingParams(greedy=True, max_new_tokens=6)) == golden


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,dp,chunk", [(2, 1, 0), (3, 1, 0), (4, 2, 0), (2, 2, 0), (3, 1, 2)])
def test_gloo_multiprocess_pipeline(golden, tmp_path, world, dp, chunk):
    """One process per stage, torch.distributed gloo (the RCCL path's twin);
    dp > 1: `dp` pipeline replicas of world/dp stages share the requests;
    chunk > 0: chunked prefill through a middle stage (bench.py's P >= 2 default)."""
    script = tmp_path / "w.py"
    script.write_text(textwrap.dedent(f"""
        import sys, json, torch
        sys.path.insert(0, {ROOT!r})
        from llm_sharding_demo_amd.config import EngineConfig, SamplingParams
        from llm_sharding_demo_amd.runtime.engine import build_engine
        cfg = EngineConfig(model_id="gpt2-test", max_batch=8, device="cpu", transport="gloo",
                           num_microbatches=2, dp_replicas={dp}, prefill_chunk={chunk})
        eng = build_engine(cfg)
        assert (eng.P, eng.R) == ({world // dp}, {dp})
        if eng.rank != 0:
            eng.worker_loop()
        else:
            out = eng.generate_ids({PROMPTS!r}, SamplingParams(greedy=True, max_new_tokens=6))
            out2 = eng.generate_ids({PROMPTS!r}[:2], SamplingParams(greedy=True, max_new_tokens=6),
                                    record_timing=True)
            stages = eng.last_session.stages
            assert sorted(st["stage"] for st in stages) == sorted(list(range(eng.P)) * {dp}), stages
            eng.shutdown()
            print("RESULT", json.dumps([out, out2]))
    """))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={env['MASTER_PORT']}", str(script)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    import json

    line = [l for l in r.stdout.splitlines() if l.startswith("RESULT")][0]
    out, out2 = json.loads(line[len("RESULT "):])
    assert out == golden
    assert out2 == golden[:2]


def test_gloo_dp_serving_loop_finishes_every_replica(golden, tmp_path):
    """dp = 2 under the serving loop (start_loop): one request lands on each
    replica; replica 1's tokens reach rank 0 over the control plane after
    replica 0's session has nothing left to plan -- every request must still
    finish without any further traffic (readouts kept the session
    alive only when local)."""
    script = tmp_path / "w.py"
    script.write_text(textwrap.dedent(f"""
        import sys, json, time, torch
        sys.path.insert(0, {ROOT!r})
        from llm_sharding_demo_amd.config import EngineConfig, SamplingParams
        from llm_sharding_demo_amd.runtime.engine import build_engine
        cfg = EngineConfig(model_id="gpt2-test", max_batch=4, device="cpu", transport="gloo",
                           num_microbatches=1, dp_replicas=2)
        eng = build_engine(cfg)
        if eng.rank != 0:
            eng.worker_loop()
        else:
            eng.start_loop()
            reqs = [eng.submit(p, SamplingParams(greedy=True, max_new_tokens=6))
                    for p in {PROMPTS!r}[:2]]
            t0 = time.monotonic()
            out = [r.wait(60) for r in reqs]
            dt = time.monotonic() - t0
            eng.shutdown()
            print("RESULT", json.dumps([out, dt]))
    """))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               OMP_NUM_THREADS="1", LSD_TEST_TOK_DELAY_S="0.3")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={env['MASTER_PORT']}", str(script)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    import json

    line = [l for l in r.stdout.splitlines() if l.startswith("RESULT")][0]
    out, dt = json.loads(line[len("RESULT "):])
    assert out == golden[:2]
    assert dt < 30


def test_gloo_compat_forwards_in_dist_mode(tmp_path):
    """/forward and /forward_b served by a torchrun engine (role `all`): stage
    0's output on rank 0, the rest of the pipeline over the pipeline edges;
    equal to the in-process 2-stage engine."""
    script = tmp_path / "w.py"
    script.write_text(textwrap.dedent(f"""
        import sys, json, torch
        sys.path.insert(0, {ROOT!r})
        from llm_sharding_demo_amd.config import EngineConfig, SamplingParams
        from llm_sharding_demo_amd.runtime.engine import Engine, build_engine
        cfg = EngineConfig(model_id="gpt2-test", max_batch=4, device="cpu", transport="gloo")
        eng = build_engine(cfg)
        if eng.rank != 0:
            eng.worker_loop()
        else:
            ids = [5, 6, 7, 8, 9]
            h = eng.forward_a(ids)
            lg = eng.forward_b(h)
            out = eng.generate_ids([ids], SamplingParams(greedy=True, max_new_tokens=3))
            lg2 = eng.forward_b(h)  # again, after a decode session
            loc = Engine(cfg.replace(num_stages=2, transport="auto"))
            hl = loc.forward_a(ids)
            ll = loc.forward_b(hl)
            print("RESULT", json.dumps([float((h - hl).abs().max()), float((lg - ll).abs().max()),
                                        float((lg2 - ll).abs().max()), list(lg.shape), out]))
            eng.shutdown()
    """))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()),
               OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={env['MASTER_PORT']}", str(script)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    import json

    line = [l for l in r.stdout.splitlines() if l.startswith("RESULT")][0]
    dh, dl, dl2, shape, out = json.loads(line[len("RESULT "):])
    assert dh == 0.0 and dl == 0.0 and dl2 == 0.0
    assert shape == [5, 1000] and len(out[0]) == 3


# ---------------------------------------------------------------------------
# Half-layer (unit) partitioning: a stage boundary between a layer's attention
# and MLP halves must reproduce the unsplit model exactly.
# ---------------------------------------------------------------------------
@pytest.fixture(scope="module")
def golden_llama():
    eng = Engine(EngineConfig(model_id="llama-test", num_stages=1, max_batch=8, device="cpu"))
    return eng.generate_ids(PROMPTS, SamplingParams(greedy=True, max_new_tokens=5))


@settings(max_examples=8, deadline=None)
@given(st.lists(st.integers(1, 7), min_size=1, max_size=3, unique=True))
def test_any_half_layer_partition_matches_unsplit(golden, cuts):
    units = sorted(cuts)  # gpt2-test: 4 layers = 8 units, cut points in 1..7
    cfg = EngineConfig(model_id="gpt2-test", num_stages=len(units) + 1, split_units=units,
                       max_batch=8, device="cpu")
    eng = Engine(cfg)
    assert eng.unit_plan[0][0] == 0 and eng.unit_plan[-1][1] == 8
    out = eng.generate_ids(PROMPTS, SamplingParams(greedy=True, max_new_tokens=6))
    assert out == golden


def test_half_layer_partition_llama(golden_llama):
    cfg = EngineConfig(model_id="llama-test", num_stages=3, split_units=[3, 5], max_batch=8,
                       device="cpu")
    eng = Engine(cfg)
    # stage 1 runs layer 1's MLP half and layer 2's attention half
    s1 = eng.stages[1]
    assert (s1.unit_start, s1.unit_end) == (3, 5) and s1.kv_layers == [2]
    assert "layers.1.mlp.gate_up.weight" in s1.w and "layers.1.self_attn.qkv.weight" not in s1.w
    assert "layers.2.self_attn.qkv.weight" in s1.w and "layers.2.mlp.down_proj.weight" not in s1.w
    out = eng.generate_ids(PROMPTS, SamplingParams(greedy=True, max_new_tokens=5))
    assert out == golden_llama


def test_unit_plan_beats_whole_layers_on_xl():
    from llm_sharding_demo_amd.parallel.partition import make_unit_plan, unit_stage_costs

    mc = get_model_config("gpt2-xl")
    for P in (2, 4, 8):
        half = make_unit_plan(mc, P, rows=128, avg_ctx=192)
        whole = make_unit_plan(mc, P, rows=128, avg_ctx=192, half_layers=False)
        assert all(a % 2 == 0 for a, _ in whole)
        ch, cw = unit_stage_costs(mc, half), unit_stage_costs(mc, whole)
        assert max(ch) <= max(cw) + 1e-9
        assert sum(ch) / P / max(ch) > 0.9  # within 10 % of a perfect split
    # SPLIT_AT-style explicit layer splits map to even unit boundaries
    assert make_unit_plan(mc, 2, split_points=[20]) == [(0, 40), (40, 96)]


# ---------------------------------------------------------------------------
# Chunked prefill: the prompt enters the KV cache in end-aligned chunks over
# several pipeline steps; outputs must equal the one-shot prefill.
# ---------------------------------------------------------------------------
def test_prefill_chunks_layout():
    from llm_sharding_demo_amd.parallel.pipeline import prefill_chunks

    ch = prefill_chunks([10, 3, 7], 4)
    assert len(ch) == 3
    # end-aligned: the last chunk holds every sequence's final position
    assert ch[-1] == ([6, 0, 3], [4, 3, 4])
    for i, n in enumerate([10, 3, 7]):
        covered = []
        for starts, qlens in ch:
            covered += list(range(starts[i], starts[i] + qlens[i]))
        assert covered == list(range(n))
    assert prefill_chunks([5, 2], 0) == [([0, 0], [5, 2])]


LONG = [list(range(1, 30)), [5, 6, 7], list(range(100, 117)), [9] * 11, [3]]


@pytest.mark.parametrize("model,P,chunk,M", [("gpt2-test", 1, 4, 1), ("gpt2-test", 2, 5, 2),
                                             ("gpt2-test", 3, 8, 3), ("llama-test", 2, 6, 2)])
def test_chunked_prefill_matches_one_shot(model, P, chunk, M):
    sp = SamplingParams(greedy=True, max_new_tokens=5)
    base = Engine(EngineConfig(model_id=model, num_stages=1, max_batch=8, device="cpu"))
    want = base.generate_ids(LONG, sp)
    eng = Engine(EngineConfig(model_id=model, num_stages=P, max_batch=8, device="cpu",
                              prefill_chunk=chunk))
    assert eng.generate_ids(LONG, sp, microbatches=M) == want
    # sampled decoding is seeded per (request, token): chunking must not change it
    sp2 = SamplingParams(temperature=0.9, top_k=10, seed=3, max_new_tokens=4)
    assert eng.generate_ids(LONG, sp2, microbatches=M) == base.generate_ids(LONG, sp2)


def test_stage_busy_stats_local_and_gloo():
    eng = Engine(EngineConfig(model_id="gpt2-test", num_stages=3, max_batch=8, device="cpu"))
    eng.generate_ids(PROMPTS, SamplingParams(greedy=True, max_new_tokens=4), microbatches=3,
                     record_timing=True)
    st = eng.last_session.stages
    assert [s["stage"] for s in st] == [0, 1, 2]
    assert all(0.0 < s["busy_fraction"] <= 1.0 and s["items"] > 0 for s in st)


def test_alternating_split_plans():
    """Plans A / B (even / odd microbatch groups) cut at most one unit apart,
    each is a valid partition, the stage union holds both, and the mean
    per-stage cost beats the single half-layer plan (GPT-2 XL, 256 rows)."""
    from llm_sharding_demo_amd.parallel.partition import (alt_stage_costs, make_alt_unit_plans,
                                                          make_unit_plan, union_plan,
                                                          unit_stage_costs, validate_unit_plan)

    mc = get_model_config("gpt2-xl")
    for P in (2, 4, 8):
        pa, pb = make_alt_unit_plans(mc, P, rows=256)
        for pl in (pa, pb):
            validate_unit_plan(pl, mc.n_layers)
        assert all(abs(a[1] - b[1]) <= 1 for a, b in zip(pa, pb))
        un = union_plan((pa, pb))
        assert all(u[0] <= min(a[0], b[0]) and max(a[1], b[1]) <= u[1] for u, a, b in zip(un, pa, pb))
        alt = max(alt_stage_costs(mc, (pa, pb), rows=256))
        one = max(unit_stage_costs(mc, make_unit_plan(mc, P, rows=256), rows=256))
        assert alt <= one + 1e-6
    pa, pb = make_alt_unit_plans(mc, 8, rows=256)
    costs = alt_stage_costs(mc, (pa, pb), rows=256)
    assert sum(costs) / 8 / max(costs) > 0.95  # half-layer units alone: ~0.92


@pytest.mark.parametrize("P,M", [(2, 2), (3, 6), (4, 4)])
def test_alternating_split_matches_unsplit(golden, P, M):
    """Even / odd groups on different unit ranges: tokens equal the unsplit
    model; the compat full-sequence path (variant 0) still chains correctly."""
    cfg = EngineConfig(model_id="gpt2-test", num_stages=P, max_batch=8, device="cpu",
                       num_microbatches=M)
    eng = Engine(cfg)
    assert eng.unit_plans is not None and eng.unit_plans[0] != eng.unit_plans[1]
    out = eng.generate_ids(PROMPTS, SamplingParams(greedy=True, max_new_tokens=6))
    assert out == golden
    ref = Engine(EngineConfig(model_id="gpt2-test", num_stages=2, max_batch=8, device="cpu",
                              num_microbatches=1))  # odd group count: one plan
    assert ref.unit_plans is None
    torch.testing.assert_close(eng.forward_b(eng.forward_a([5, 6, 7, 8])),
                               ref.forward_b(ref.forward_a([5, 6, 7, 8])), atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("P", [2, 3])
def test_bf16_wire_is_deterministic_and_close(golden, P):
    """C-CODEC option: hidden states cross stage boundaries as bf16 (half the
    bytes per hop).  The residual stream is rounded at each boundary, so
    tokens need not equal the fp32 wire; they must be deterministic and
    (greedy, random-init model) mostly agree with the unsplit model."""
    cfg = EngineConfig(model_id="gpt2-test", num_stages=P, max_batch=8, device="cpu",
                       wire_dtype="bf16")
    a = Engine(cfg).generate_ids(PROMPTS, SamplingParams(greedy=True, max_new_tokens=6))
    b = Engine(cfg).generate_ids(PROMPTS, SamplingParams(greedy=True, max_new_tokens=6))
    assert a == b
    same = sum(x == y for ra, rg in zip(a, golden) for x, y in zip(ra, rg))
    assert same >= 0.8 * sum(len(r) for r in golden), (a, golden)
    with pytest.raises(ValueError):
        Engine(cfg.replace(wire_dtype="fp16"))
