"""Graph-I/O op-ordering contract on CPU (parallel/comm.py StrictLocalTransport).

With the native RCCL transport (and its single-GPU rehearsal, the device
loopback fabric) a steady-state decode item's edge receive and send are
captured INSIDE the stage's decode graph, while prefill chunks, finals and
the stage-0 token-return receive stay eager.  RCCL matches the ops of a
communicator -- one per (edge, lane) -- strictly in issue order, so every
mix of eager and in-graph ops must be issued in the same order at both ends
of each channel.  `StrictLocalTransport` keeps one FIFO per (edge, lane),
makes the worker take the graph-I/O code path (the graph body runs eagerly
on CPU, calling capture_recv / capture_send where a captured graph would),
checks the size and dtype of every receive against the message at its
channel's head and logs every op; these tests drive mixed prefill / decode /
final / join / leave steps through it and compare both ends of every channel.

Reference hop being replaced: shard A -> coordinator -> shard B
(`/root/reference/server.py:169-181`).
"""
from collections import defaultdict

import pytest

from llm_sharding_demo_amd.config import EngineConfig, SamplingParams
from llm_sharding_demo_amd.runtime.engine import Engine

PROMPTS = [[5, 6, 7, 8], [11], [300, 2, 9], [1, 2], [40, 41, 42, 43, 44]]


@pytest.fixture(scope="module")
def golden():
    eng = Engine(EngineConfig(model_id="gpt2-test", num_stages=1, max_batch=8, device="cpu"))
    return eng.generate_ids(PROMPTS, SamplingParams(greedy=True, max_new_tokens=6))


def _check_channels(eng):
    """Per (edge, src, dst, lane): the receiver's op sequence equals the
    sender's (sizes and dtypes), and every sent message was received."""
    sends, recvs = defaultdict(list), defaultdict(list)
    for edge, src, dst, lane, d, nbytes, dt in eng.fabric.oplog:
        (sends if d == "send" else recvs)[(edge, src, dst, lane)].append((nbytes, dt))
    assert sends.keys() == recvs.keys()
    for k in sends:
        assert sends[k] == recvs[k], k
    return sends


@pytest.mark.parametrize("P,M,chunk", [(2, 2, 0), (2, 2, 2), (3, 4, 2), (4, 4, 0), (4, 6, 3)])
def test_graph_io_path_matches_one_stage(golden, P, M, chunk):
    cfg = EngineConfig(model_id="gpt2-test", num_stages=P, max_batch=8, device="cpu",
                       transport="strict", prefill_chunk=chunk, num_microbatches=M)
    eng = Engine(cfg)
    assert all(w.graph_io for w in eng.workers)
    assert eng.unit_plans is not None  # alternating splits (even group counts)
    out = eng.generate_ids(PROMPTS, SamplingParams(greedy=True, max_new_tokens=6))
    assert out == golden
    chans = _check_channels(eng)
    assert sum(w.io_items for w in eng.workers) > 0
    # both lanes carry traffic: the per-(edge, lane) channel split is exercised
    assert {k[3] for k in chans} == {0, 1}


def test_graph_io_joins_leaves_and_sampling(golden):
    """More requests than rows (joins into a running batch), different
    lengths (leaves), seeded sampling: same tokens as one stage, channel
    sequences intact."""
    ps = [SamplingParams(greedy=False, temperature=0.8, top_k=5, seed=11 + i, max_new_tokens=n)
          for i, n in enumerate((6, 2, 5, 1, 4))]
    ref = Engine(EngineConfig(model_id="gpt2-test", num_stages=1, max_batch=2, device="cpu"))
    want = ref.generate_ids(PROMPTS, ps)
    eng = Engine(EngineConfig(model_id="gpt2-test", num_stages=3, max_batch=2, device="cpu",
                              transport="strict", num_microbatches=2, prefill_chunk=2))
    assert eng.generate_ids(PROMPTS, ps) == want
    _check_channels(eng)
    assert eng.generate_ids(PROMPTS[:2], SamplingParams(greedy=True, max_new_tokens=6)) == golden[:2]
    _check_channels(eng)


def test_graph_io_bf16_wire(golden):
    """bf16 wire: the in-graph receive lands in a bf16 staging buffer of the
    same size the sender puts on the channel."""
    eng = Engine(EngineConfig(model_id="gpt2-test", num_stages=2, max_batch=8, device="cpu",
                              transport="strict", wire_dtype="bf16", num_microbatches=2))
    eng.generate_ids(PROMPTS, SamplingParams(greedy=True, max_new_tokens=6))
    chans = _check_channels(eng)
    assert any(dt == "torch.bfloat16" for seq in chans.values() for _, dt in seq)


def test_mismatched_receive_is_detected():
    """A receive posted with the wrong size fails loudly (RCCL would silently
    mis-match or hang)."""
    import torch

    from llm_sharding_demo_amd.parallel.comm import LocalFabric, TransportError

    fab = LocalFabric(2, timeout=2.0)
    a, b = fab.transport(0, "strict"), fab.transport(1, "strict")
    a.send(torch.zeros(4), 1, "fwd", 1)
    with pytest.raises(TransportError, match="op order mismatch"):
        b.irecv(torch.zeros(5), 0, "fwd", 1).wait()
