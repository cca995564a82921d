"""Device loopback channels (csrc/kernels/loopback.hip, csrc/loop_fabric.cpp)
and the graph-I/O pipeline they enable on ONE MI355X.

The 8-GPU data plane (`--transport rccl`) captures each steady-state decode
item's edge receive and send inside the stage's hipGraph, and the native
executor enqueues whole steps from C++.  `DeviceLoopFabric` gives P stage
threads on one GPU the same API and semantics (per-(edge, lane) FIFO
channels, device-side waits, ops enqueued eagerly or captured), so these
tests execute that exact code path -- `_io()`, captured transfers,
`_native_step` / `exec_items` at P > 1 -- and compare its tokens with one
stage.  The stall test checks the failure path: a message that is never
published leaves a receive kernel spinning on the device; the watchdog must
fire, the abort word must drain the lanes and the engine must fail its
requests without hanging.

Reference hop being replaced: shard A -> coordinator -> shard B
(`/root/reference/server.py:169-181`).
"""
import time

import pytest
import torch

from llm_sharding_demo_amd.config import EngineConfig, SamplingParams
from llm_sharding_demo_amd.runtime.engine import Engine

pytestmark = pytest.mark.gpu


def _fabric(P=2, lanes=1, ring=1 << 20, spin_s=10.0, timeout=10.0):
    from llm_sharding_demo_amd.parallel.comm import DeviceLoopFabric

    return DeviceLoopFabric(P, torch.device("cuda", 0), lanes=lanes, ring_bytes=ring,
                            timeout=timeout, spin_limit_s=spin_s)


def test_eager_transfers_in_fifo_order_with_ring_wrap():
    """Many messages of mixed sizes through a small ring (wraps, skips to the
    next lap): every receive gets its message, in order."""
    f = _fabric(ring=256 << 10)
    a, b = f.transport(0), f.transport(1)
    sizes = [1000, 4096, 17, 9000, 3, 16384, 250, 12000] * 6
    srcs = [torch.randn(n, device="cuda") for n in sizes]
    outs = [torch.empty(n, device="cuda") for n in sizes]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for i in range(0, len(sizes), 4):  # sender runs ahead by up to 4 messages
        with torch.cuda.stream(s1):
            for j in range(i, min(i + 4, len(sizes))):
                a.send(srcs[j], 1, "fwd")
        with torch.cuda.stream(s2):
            for j in range(i, min(i + 4, len(sizes))):
                b.irecv(outs[j], 0, "fwd")
    torch.cuda.synchronize()
    assert f.check_async() is None
    for s, o in zip(srcs, outs):
        assert torch.equal(s, o)
    n_send, n_recv, _, _ = f.counts("fwd", 0, 1, 0)
    assert n_send == n_recv == len(sizes)


def test_size_mismatch_is_recorded_on_device():
    """A receive posted with the wrong size records LOOP_ERR_MISMATCH (the
    RCCL op-ordering contract, checked on the device) instead of copying."""
    f = _fabric()
    a, b = f.transport(0), f.transport(1)
    src = torch.arange(16, device="cuda", dtype=torch.float32)
    dst = torch.full((20,), -1.0, device="cuda")
    a.send(src, 1, "fwd")
    b.irecv(dst, 0, "fwd")
    torch.cuda.synchronize()
    err = f.check_async()
    assert err is not None and "op order mismatch" in err, err
    assert torch.all(dst == -1.0)


def test_captured_transfers_replay_with_handshake():
    """Send and receive captured in two hipGraphs (the graph-I/O shape: recv
    -> compute -> send), replayed many times through the I/O-list launch."""
    f = _fabric(P=3)
    t0, t1, t2 = f.transport(0), f.transport(1), f.transport(2)
    x = torch.zeros(256, device="cuda")
    mid = torch.zeros(256, device="cuda")
    y = torch.zeros(256, device="cuda")

    def capture(t, fn):
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        t.begin_capture()
        with torch.cuda.stream(s):
            g.capture_begin()
            fn()
            g.capture_end()
        io = t.end_capture()
        torch.cuda.current_stream().wait_stream(s)
        return g, io

    g0, io0 = capture(t0, lambda: t0.send(x, 1, "fwd"))

    def stage1():
        t1.irecv(mid, 0, "fwd")
        mid.mul_(2.0)
        t1.send(mid, 2, "fwd")
    g1, io1 = capture(t1, stage1)
    g2, io2 = capture(t2, lambda: t2.irecv(y, 1, "fwd"))
    assert io0[0] and io1[0] and io2[0] and len(io1[1]) == 2
    assert f.counts("fwd", 0, 1, 0)[0] == 0  # capturing enqueues nothing
    for k in range(20):
        x.fill_(float(k))
        t0.replay(g0, *io0)
        t1.replay(g1, *io1)
        t2.replay(g2, *io2)
        torch.cuda.synchronize()
        assert torch.all(y == 2.0 * k), (k, y[:4])
    assert f.check_async() is None
    assert f.counts("fwd", 1, 2, 0)[:2] == (20, 20)


def _engine(P, chunk=0, M=None, **kw):
    return Engine(EngineConfig(model_id="gpt2-test", num_stages=P, max_batch=16, device="cuda",
                               num_microbatches=M or 2 * P, transport="devloop",
                               prefill_chunk=chunk, **kw))


@pytest.mark.parametrize("P,chunk", [(2, 0), (3, 2), (4, 0), (4, 1)])
def test_devloop_pipeline_bit_identical_and_native(P, chunk):
    """P stage threads joined by device loopback channels: graph-I/O decode
    graphs and the native executor at P > 1, tokens equal to one stage
    (alternating splits, chunked prefill through the middle stages)."""
    from llm_sharding_demo_amd.parallel.comm import DeviceLoopTransport

    sp = SamplingParams(temperature=0.8, top_k=20, seed=7, max_new_tokens=12)
    prompts = [[i + 1, 2 * i + 3, 5] for i in range(12)]
    one = Engine(EngineConfig(model_id="gpt2-test", num_stages=1, max_batch=16, device="cuda", merge_prefill=False,
                              num_microbatches=2 * P, prefill_chunk=chunk)).generate_ids(prompts, sp)
    e = _engine(P, chunk)
    assert isinstance(e.workers[1].t, DeviceLoopTransport)
    assert all(w.graph_io and w.native_exec for w in e.workers)
    assert e.unit_plans is not None
    for _ in range(3):  # first use eager, then capture, then cached replays
        assert e.generate_ids(prompts, sp) == one
    assert all(w.io_items > 0 for w in e.workers[1:]), [w.io_items for w in e.workers]
    assert all(w.native_steps > 0 for w in e.workers), [w.native_steps for w in e.workers]
    # recurring prefill chunk shapes replay their captured graphs (P > 1: on by
    # default); 1-token chunks are decode-shaped batches and stay eager
    if chunk != 1:
        assert all(w.pf_replays > 0 for w in e.workers), [w.pf_replays for w in e.workers]
    n_io_graphs = sum(len(gs.graph_io) for w in e.workers for gs in w.groups.values())
    assert n_io_graphs > 0
    assert e.fabric.check_async() is None
    # every channel drained: sends == receives
    for (edge, src, dst, lane) in e.fabric.chans:
        n_s, n_r, _, _ = e.fabric.counts(edge, src, dst, lane)
        assert n_s == n_r, (edge, src, dst, lane, n_s, n_r)
    e.shutdown()


def test_devloop_serving_join_and_bf16_wire():
    """Requests joining a running batch (composition changes between graph
    replays) and the bf16 wire (in-graph receive into a bf16 staging row)."""
    sp = SamplingParams(greedy=True, max_new_tokens=16)
    prompts = [[3, 4, 5], [6, 7], [8], [9, 10, 11, 12]]
    for wire in ("fp32", "bf16"):
        # each prompt alone (one row per group: the small-row decode kernels
        # are row-independent, tests/test_engine_gpu.py join test)
        ref = Engine(EngineConfig(model_id="gpt2-test", num_stages=2, max_batch=16, device="cuda",
                                  num_microbatches=4, transport="loopback", wire_dtype=wire))
        want = [ref.generate_ids([p], sp)[0] for p in prompts]
        ref.shutdown()
        e = _engine(2, wire_dtype=wire)
        e.start_loop()
        r1 = [e.submit(p, sp) for p in prompts[:2]]
        time.sleep(0.05)
        r2 = [e.submit(p, sp) for p in prompts[2:]]
        got = [r.wait(120) for r in r1 + r2]
        e.stop_loop()
        assert got == want, wire
        assert e.fabric.check_async() is None
        e.shutdown()


def test_devloop_stall_aborts_spinning_lanes():
    """Stage 0 stops publishing on one channel mid-decode: stage 1's receive
    kernel spins on the device (its host passed the enqueue handshake).  The
    watchdog must fire within round_timeout_s, the abort word must make the
    spinning kernels return, the request must fail and the GPU must drain."""
    e = _engine(2, round_timeout_s=3.0)
    sp = SamplingParams(greedy=True, max_new_tokens=64)
    prompts = [[i + 1, 2] for i in range(8)]
    e.generate_ids(prompts, sp)  # warm: graphs captured, native steps running
    sent = e.fabric.counts("fwd", 0, 1, 0)[0]
    e.fabric.stall("fwd", 0, 1, 0, sent + 6)  # a few steps into the next session
    t0 = time.monotonic()
    with pytest.raises(Exception):
        e.generate_ids(prompts, sp)
    elapsed = time.monotonic() - t0
    assert not e.healthy
    assert e.last_error and ("WatchdogTimeout" in e.last_error or "aborted" in e.last_error), e.last_error
    assert elapsed < 3.0 + 15.0, elapsed
    done = []

    def drain():
        torch.cuda.synchronize()
        done.append(True)
    import threading

    th = threading.Thread(target=drain, daemon=True)
    th.start()
    th.join(20.0)  # well under the kernels' own 30 s spin limit
    assert done, "lanes did not drain after the abort"
    err = e.fabric.C.loop_status(e.fabric.handle)[0]
    assert err == 1, err  # LOOP_ERR_ABORT: a device wait saw the abort word
    with pytest.raises(RuntimeError, match="unhealthy"):
        e.generate_ids([[1]], SamplingParams(greedy=True, max_new_tokens=1))
    # advisor r3: nothing may launch on an aborted data plane -- a cached
    # graph-I/O decode graph is refused, as are the eager ops
    from llm_sharding_demo_amd.parallel.comm import TransportError

    w = e.workers[1]
    cached = [(gs, k) for gs in w.groups.values() for k in gs.graph_io if k in gs.graphs]
    assert cached
    gs, key = cached[0]
    with pytest.raises(TransportError):
        w._replay(gs, key, gs.graphs[key][0])
    with pytest.raises(TransportError):
        w.t.send(torch.zeros(4, device="cuda"), 0, "ret", 0)
