"""End-to-end engine on an MI355X: HIP path vs the fp32 CPU golden engine,
hipGraph replay vs eager (bit-identical: every kernel is deterministic),
and a multi-stage in-process pipeline vs a single stage (bit-identical: the
boundary hidden state crosses stages in fp32)."""
import pytest
import torch

from llm_sharding_demo_amd.config import EngineConfig, SamplingParams, get_model_config
from llm_sharding_demo_amd.models.stage import StageModel
from llm_sharding_demo_amd.runtime.batch import BatchMeta
from llm_sharding_demo_amd.runtime.engine import Engine

from .helpers import full_weights

pytestmark = pytest.mark.gpu


def _native_loaded():
    import sys

    return "llm_sharding_demo_amd._C" in sys.modules


@pytest.mark.parametrize("model", ["gpt2-test", "llama-test"])
def test_stage_logits_match_cpu_golden(model):
    mc = get_model_config(model)
    w = full_weights(mc)
    cpu = StageModel(mc, 0, mc.n_layers, True, True, weights=w, max_slots=4, max_seq=256)
    gpu = StageModel(mc, 0, mc.n_layers, True, True, device="cuda", weights=w, max_slots=4, max_seq=256)
    assert gpu.backend.name == "hip" and _native_loaded()
    prompts = [[3, 17, 5, 99, 42, 7, 1] * 10, [8, 9], list(range(1, 100))]
    meta_c = BatchMeta.build([0, 1, 2], [0, 0, 0], [len(p) for p in prompts], "cpu")
    meta_g = BatchMeta.build([0, 1, 2], [0, 0, 0], [len(p) for p in prompts], "cuda")
    flat = torch.tensor([t for p in prompts for t in p], dtype=torch.int32)
    lc = cpu.forward(meta_c, flat)[:, : mc.vocab_size]
    lg = gpu.forward(meta_g, flat.cuda())[:, : mc.vocab_size].cpu()
    torch.testing.assert_close(lg, lc, atol=0.05, rtol=0.05)
    # decode steps through the cache
    for step in range(3):
        toks = torch.tensor([5 + step, 6, 7], dtype=torch.int32)
        pos = [len(p) + step for p in prompts]
        dc = cpu.forward(BatchMeta.decode([0, 1, 2], pos, "cpu", max(pos) + 1), toks)[:, : mc.vocab_size]
        dg = gpu.forward(BatchMeta.decode([0, 1, 2], pos, "cuda", max(pos) + 1), toks.cuda())
        torch.testing.assert_close(dg[:, : mc.vocab_size].cpu(), dc, atol=0.05, rtol=0.05)


@pytest.mark.parametrize("model", ["gpt2-test", "llama-test"])
def test_wide_decode_batch_on_ring_gemms_matches_cpu_golden(model):
    """200 decode rows: every decode GEMM (QKV + KV append, MLP, residual
    split-K slabs) leaves the split-K kernel for the 128x64 LDS-ring GEMM."""
    import random

    from llm_sharding_demo_amd.ops.hip import HipBackend

    assert HipBackend._tiled(200, 64) and HipBackend.R.tiled3_max > 0
    mc = get_model_config(model)
    w = full_weights(mc)
    B = 200
    cpu = StageModel(mc, 0, mc.n_layers, True, True, weights=w, max_slots=B, max_seq=64)
    gpu = StageModel(mc, 0, mc.n_layers, True, True, device="cuda", weights=w, max_slots=B, max_seq=64)
    rnd = random.Random(7)
    prompts = [[rnd.randrange(1, 200) for _ in range(rnd.randrange(2, 12))] for _ in range(B)]
    slots = list(range(B))
    flat = torch.tensor([t for p in prompts for t in p], dtype=torch.int32)
    cpu.forward(BatchMeta.build(slots, [0] * B, [len(p) for p in prompts], "cpu"), flat)
    gpu.forward(BatchMeta.build(slots, [0] * B, [len(p) for p in prompts], "cuda"), flat.cuda())
    for step in range(2):
        toks = torch.tensor([rnd.randrange(1, 200) for _ in range(B)], dtype=torch.int32)
        pos = [len(p) + step for p in prompts]
        dc = cpu.forward(BatchMeta.decode(slots, pos, "cpu", max(pos) + 1), toks)[:, : mc.vocab_size]
        dg = gpu.forward(BatchMeta.decode(slots, pos, "cuda", max(pos) + 1), toks.cuda())
        torch.testing.assert_close(dg[:, : mc.vocab_size].cpu(), dc, atol=0.05, rtol=0.05)


def _engine(model, P=1, graphs=True, **kw):
    cfg = EngineConfig(model_id=model, num_stages=P, max_batch=16, device="cuda", use_graphs=graphs,
                       max_seq_len=512, **kw)
    return Engine(cfg, devices=["cuda:0"] * P)


@pytest.mark.parametrize("model", ["gpt2-test", "llama-test"])
def test_graphs_equal_eager(model):
    prompts = [[1, 2, 3, 4], [5, 6], list(range(10, 50))]
    sp = SamplingParams(greedy=True, max_new_tokens=12)
    a = _engine(model, graphs=False).generate_ids(prompts, sp)
    b = _engine(model, graphs=True).generate_ids(prompts, sp)
    assert a == b


def test_graphs_equal_eager_blaslt_silu(monkeypatch):
    """Decode gate_up on hipBLASLt + the SiLU*up pass (the A/B oracle route,
    forced from 1 row) inside captured decode graphs gives the eager tokens."""
    from llm_sharding_demo_amd.ops.hip import HipBackend

    monkeypatch.setattr(HipBackend, "R", HipBackend.R.replace(blaslt=1, blaslt_silu_min_m=1))
    prompts = [[1, 2, 3, 4], [5, 6], list(range(10, 50))]
    sp = SamplingParams(greedy=True, max_new_tokens=12)
    a = _engine("llama-test", graphs=False).generate_ids(prompts, sp)
    e = _engine("llama-test", graphs=True)
    for _ in range(3):  # eager first use, capture, replay
        assert e.generate_ids(prompts, sp) == a


def test_graphs_equal_eager_blaslt_qkv(monkeypatch):
    """Decode QKV on hipBLASLt + the RoPE / cache-append pass (the A/B oracle
    route, forced from 1 row and any K) inside captured decode graphs gives
    the eager tokens."""
    from llm_sharding_demo_amd.ops.hip import HipBackend

    monkeypatch.setattr(HipBackend, "R", HipBackend.R.replace(blaslt=1, blaslt_qkv_min_m=1, blaslt_qkv_min_k=1))
    prompts = [[1, 2, 3, 4], [5, 6], list(range(10, 50))]
    sp = SamplingParams(greedy=True, max_new_tokens=12)
    a = _engine("llama-test", graphs=False).generate_ids(prompts, sp)
    e = _engine("llama-test", graphs=True)
    for _ in range(3):  # eager first use, capture, replay
        assert e.generate_ids(prompts, sp) == a


def test_blaslt_oracle_stages_sharing_a_gpu_match_one_stage(monkeypatch):
    """two pipeline stages on ONE GPU issue hipBLASLt GEMMs
    concurrently from their own lane streams (graph-captured too).  Only
    workspace-free algorithms are accepted, so nothing is shared: with every
    library route forced on (decode QKV / gate_up from 1 row, prefill from 1
    row) the 2-stage pipeline gives the 1-stage tokens."""
    from llm_sharding_demo_amd.ops.hip import HipBackend

    monkeypatch.setattr(HipBackend, "R", HipBackend.R.replace(
        blaslt=1, blaslt_min_m=1, blaslt_resid_min_k=1, blaslt_gelu_min_m=1, blaslt_silu_min_m=1,
        blaslt_silu_max_m=1 << 20, blaslt_qkv_min_m=1, blaslt_qkv_min_k=1))
    prompts = [[1, 2, 3, 4], [5, 6], list(range(10, 50)), [7] * 9]
    sp = SamplingParams(greedy=True, max_new_tokens=10)
    for model in ("llama-test", "gpt2-test"):
        one = _engine(model, merge_prefill=False).generate_ids(prompts, sp, microbatches=2)
        two = _engine(model, P=2).generate_ids(prompts, sp, microbatches=2)
        assert one == two, model


def test_pipeline_stages_bit_identical_on_one_gpu():
    prompts = [[1, 2, 3, 4], [5, 6], list(range(10, 50)), [7] * 9]
    sp = SamplingParams(temperature=0.8, top_k=20, seed=5, max_new_tokens=10)
    one = _engine("gpt2-test", merge_prefill=False).generate_ids(prompts, sp)
    two = _engine("gpt2-test", P=2).generate_ids(prompts, sp, microbatches=2)
    four = _engine("gpt2-test", P=4).generate_ids(prompts, sp, microbatches=4)
    assert one == two == four


def test_greedy_prefix_matches_cpu_golden():
    prompts = [[11, 12, 13, 14, 15]]
    sp = SamplingParams(greedy=True, max_new_tokens=4)
    cpu = Engine(EngineConfig(model_id="gpt2-test", max_batch=4, device="cpu")).generate_ids(prompts, sp)
    gpu = _engine("gpt2-test").generate_ids(prompts, sp)
    assert gpu[0][0] == cpu[0][0]


def test_gpt2_small_shapes_smoke():
    """Real GPT-2 small dims (H=768, 12 heads, vocab 50257) through the engine."""
    e = Engine(EngineConfig(
        model_id="gpt2", max_batch=8, device="cuda", max_seq_len=256))
    out = e.generate_ids([[1, 2, 3]] * 8, SamplingParams(max_new_tokens=8, seed=1))
    assert all(len(o) == 8 and all(0 <= t < 50257 for t in o) for o in out)


@pytest.mark.parametrize("model", ["gpt2-test", "llama-test"])
def test_chunked_prefill_gpu_matches_one_shot(model):
    prompts = [list(range(1, 90)), [5, 6, 7], list(range(100, 160)), [9] * 33]
    sp = SamplingParams(greedy=True, max_new_tokens=8)
    want = _engine(model).generate_ids(prompts, sp)
    got = _engine(model, P=2, prefill_chunk=32).generate_ids(prompts, sp, microbatches=2)
    assert got == want


def test_graphs_cached_across_sessions():
    """Decode graphs live on the stage workers, keyed by (group, bucket rows,
    context bucket): after the first sessions no new captures happen."""
    e = _engine("gpt2-test")
    sp = SamplingParams(greedy=True, max_new_tokens=8)
    prompts = [[1, 2, 3], [4, 5], [6], [7, 8, 9, 10]]
    first = e.generate_ids(prompts, sp)
    e.generate_ids(prompts, sp)
    c = sum(w.captures for w in e.workers)
    assert c > 0
    for _ in range(3):
        assert e.generate_ids(prompts, sp) == first
    assert sum(w.captures for w in e.workers) == c


@pytest.mark.parametrize("chunk", [0, 2, 3, 5])
def test_prefill_chunk_graphs_bit_identical(monkeypatch, chunk):
    """Prefill chunks replayed from captured graphs (pipeline.py
    _prefill_graph, forced on one stage) give the eager path's tokens; the
    chunk index buffer is refilled per replay (slots and starts differ between
    the chunks of one shape), the last stage samples after the replay."""
    from llm_sharding_demo_amd.parallel.pipeline import StageWorker

    sp = SamplingParams(temperature=0.8, top_k=20, seed=5, max_new_tokens=6)
    # chunk 5: the second chunk has one query per sequence (a decode-shaped
    # batch, which stays eager)
    prompts = [[i + 1, 2 * i + 3, 5, 7, i + 9, 11] for i in range(8)]
    monkeypatch.setattr(StageWorker, "PREFILL_GRAPHS", "0")
    want = _engine("gpt2-test", prefill_chunk=chunk).generate_ids(prompts, sp, microbatches=2)
    monkeypatch.setattr(StageWorker, "PREFILL_GRAPHS", "1")
    e = _engine("gpt2-test", prefill_chunk=chunk)
    for _ in range(3):  # eager, capture, replay
        assert e.generate_ids(prompts, sp, microbatches=2) == want
    assert sum(w.pf_replays for w in e.workers) > 0


def test_merged_prefill_equals_per_group(monkeypatch):
    """One stage, every group joining at once: the step's prefill items as one
    forward (pipeline.py _merged_prefill) give the per-group path's greedy
    tokens.  The merged GEMMs have other row counts (other kernels, other
    rounding), so this compares greedy decoding of the small test model,
    whose margins dwarf bf16 rounding; the kernels are deterministic."""
    from llm_sharding_demo_amd.parallel.pipeline import StageWorker

    sp = SamplingParams(greedy=True, max_new_tokens=6)
    prompts = [[i + 1, 2 * i + 3, 5, i % 7 + 1] for i in range(12)]
    monkeypatch.setattr(StageWorker, "MERGE_PREFILL", False)
    want = _engine("gpt2-test").generate_ids(prompts, sp, microbatches=3)
    monkeypatch.setattr(StageWorker, "MERGE_PREFILL", True)
    e = _engine("gpt2-test")
    for _ in range(2):
        assert e.generate_ids(prompts, sp, microbatches=3) == want


def test_prefill_graphs_bounded(monkeypatch):
    """Serving with changing prompt mixes: at most PREFILL_GRAPHS_MAX prefill
    graphs stay captured per group (oldest dropped), tokens unchanged."""
    from llm_sharding_demo_amd.parallel.pipeline import StageWorker

    sp = SamplingParams(greedy=True, max_new_tokens=3)
    mixes = [[[j + 1] * (3 + (k + j) % 4) for j in range(4)] for k in range(6)]
    monkeypatch.setattr(StageWorker, "PREFILL_GRAPHS", "0")
    want = [_engine("gpt2-test").generate_ids(m, sp) for m in mixes]
    monkeypatch.setattr(StageWorker, "PREFILL_GRAPHS", "1")
    monkeypatch.setattr(StageWorker, "PREFILL_GRAPHS_MAX", 2)
    e = _engine("gpt2-test")
    for _ in range(3):
        for m, w in zip(mixes, want):
            assert e.generate_ids(m, sp) == w
    assert sum(w.pf_replays for w in e.workers) > 0
    assert all(len(gs.pf_graphs) <= 2 for w in e.workers for gs in w.groups.values())


@pytest.mark.parametrize("P,chunk", [(2, 0), (4, 0), (3, 2), (4, 1)])
def test_loopback_multi_stage_bit_identical(P, chunk):
    """P stage threads on one GPU with the device-async loopback transport
    (stream waits on events, no host sync) produce the P = 1 tokens; with
    alternating splits (2P groups) and, for chunk > 0, chunked prefill
    through the middle stages (bench.py's multi-stage default)."""
    sp = SamplingParams(temperature=0.8, top_k=20, seed=7, max_new_tokens=10)
    prompts = [[i + 1, 2 * i + 3, 5] for i in range(12)]
    # same microbatch shapes on one stage: a 16-row group would run the
    # split-K GEMM where 4-row groups run the GEMV (equal to bf16 rounding,
    # not bit-equal -- tools/check_m1.py)
    # chunked and one-shot prefill round differently (other GEMM row counts
    # and kernels), so the one-stage reference uses the same chunks
    one = _engine("gpt2-test", num_microbatches=2 * P, prefill_chunk=chunk,
                  merge_prefill=False).generate_ids(prompts, sp)
    e = Engine(EngineConfig(model_id="gpt2-test", num_stages=P, max_batch=16, device="cuda",
                            num_microbatches=2 * P, transport="loopback", prefill_chunk=chunk))
    from llm_sharding_demo_amd.parallel.comm import LoopbackTransport

    assert isinstance(e.workers[1].t, LoopbackTransport)
    assert e.unit_plans is not None  # even / odd groups on different unit ranges
    assert e.generate_ids(prompts, sp) == one
    assert e.generate_ids(prompts, sp) == one  # replayed graphs
    e.shutdown()


def test_join_running_batch_on_gpu():
    """Iteration-level batching on the HIP path: a request joining a running
    batch changes the bucket (new graph) and still matches running alone."""
    import time

    e = _engine("gpt2-test")
    e.start_loop()
    sp_long = SamplingParams(greedy=True, max_new_tokens=60)
    long = e.submit([3, 4, 5], sp_long)
    while e.scheduler.stats["steps"] < 10:
        time.sleep(0.001)
    short = e.submit([9, 8], SamplingParams(greedy=True, max_new_tokens=3))
    s_out, l_out = short.wait(60), long.wait(60)
    e.stop_loop()
    assert short.t_done < long.t_done
    alone = _engine("gpt2-test")
    assert s_out == alone.generate_ids([[9, 8]], SamplingParams(greedy=True, max_new_tokens=3))[0]
    assert l_out == alone.generate_ids([[3, 4, 5]], sp_long)[0]


@pytest.mark.parametrize("timing", [False, True])
def test_native_stage_executor_matches_python_item_loop(monkeypatch, timing):
    """Steady-state decode steps go through the native stage executor
    (csrc/stage_exec.cpp: one C++ call per step -- graph launches, token
    readout copies, busy-timing events) and give the Python item loop's tokens
    bit for bit, with and without per-item timing events; EOS stops and
    sequences leaving mid-session (composition changes) are issued natively
    too: packed row state + apply_rows ahead of the graph."""
    prompts = [[1, 2, 3, 4], [5, 6], list(range(10, 50)), [7] * 9, [3, 3]]
    sps = [SamplingParams(temperature=0.8, top_k=20, seed=5, max_new_tokens=n) for n in (12, 5, 16, 9, 1)]
    monkeypatch.setenv("LSD_NATIVE_EXEC", "0")
    py = _engine("gpt2-test", num_microbatches=2)
    want = py.generate_ids(prompts, sps, record_timing=timing)
    assert sum(w.native_steps for w in py.workers) == 0
    monkeypatch.setenv("LSD_NATIVE_EXEC", "1")
    nat = _engine("gpt2-test", num_microbatches=2)
    assert nat.generate_ids(prompts, sps, record_timing=timing) == want
    got = nat.generate_ids(prompts, sps, record_timing=timing)  # graphs cached: native steps
    assert got == want
    assert sum(w.native_steps for w in nat.workers) > 0
    assert sum(w.native_changes for w in nat.workers) > 0
    if timing:
        assert nat.last_session is not None and 0.0 < nat.last_session.stages[0]["busy_fraction"] <= 1.0
