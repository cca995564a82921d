"""Native RCCL communicator (csrc/comm.cpp) on the GPU.

The pipeline's edges are 2-rank communicators (parallel/comm.py
RcclTransport).  One GPU cannot host a 2-rank RCCL communicator (RCCL
refuses duplicate devices), so these tests drive the same entry points on a
1-rank communicator with grouped self send/recv: unique id, init on the
current device, ncclSend / ncclRecv enqueued on the current stream, a
hipGraph capture of the pair, and teardown.  The 2-rank pipeline path runs in
the multi-GPU scaling bench (`bench.py --transport rccl`).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm():
    from llm_sharding_demo_amd.ops.hip import _load

    C = _load()
    torch.cuda.set_device(0)
    h = C.rccl_comm_init(1, 0, C.rccl_unique_id())
    yield C, h
    torch.cuda.synchronize()
    C.rccl_comm_destroy(h)


@pytest.mark.parametrize("shape,dtype", [((256, 1600), torch.float32), ((7,), torch.int32),
                                         ((3, 50304), torch.bfloat16)])
def test_rccl_self_send_recv(comm, shape, dtype):
    C, h = comm
    src = (torch.randn(shape, device="cuda") * 100).to(dtype)
    dst = torch.zeros_like(src)
    C.rccl_group_start()
    C.rccl_send(h, src, 0)
    C.rccl_recv(h, dst, 0)
    C.rccl_group_end()
    torch.cuda.synchronize()
    assert torch.equal(dst, src)
    assert C.rccl_version() >= 21800


def test_rccl_on_a_side_stream_is_stream_ordered(comm):
    """The pair runs on a comm stream ordered by events, as RcclTransport
    does: the producer kernel, then the transfer, then the consumer."""
    C, h = comm
    x = torch.zeros(1 << 20, device="cuda")
    out = torch.empty_like(x)
    cs = torch.cuda.Stream()
    x.add_(3.0)  # producer on the current stream
    cs.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(cs):
        C.rccl_group_start()
        C.rccl_send(h, x, 0)
        C.rccl_recv(h, out, 0)
        C.rccl_group_end()
        ev = torch.cuda.Event()
        ev.record(cs)
    torch.cuda.current_stream().wait_event(ev)
    y = out * 2  # consumer
    torch.cuda.synchronize()
    assert float(y.min()) == 6.0 and float(y.max()) == 6.0


def test_rccl_pair_captured_in_graph(comm):
    """send/recv inside a hipGraph: replays move the current contents."""
    C, h = comm
    src = torch.zeros(4096, device="cuda")
    dst = torch.zeros_like(src)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        C.rccl_group_start()
        C.rccl_send(h, src, 0)
        C.rccl_recv(h, dst, 0)
        C.rccl_group_end()
    for v in (1.0, 2.5, -4.0):
        src.fill_(v)
        g.replay()
        torch.cuda.synchronize()
        assert float(dst.min()) == v and float(dst.max()) == v
    del g  # release the graph's RCCL resources now, not in a later test's capture
    import gc

    gc.collect()


def test_rccl_rejects_bad_input(comm):
    C, h = comm
    with pytest.raises(RuntimeError):
        C.rccl_send(h, torch.zeros(4, 4, device="cuda").t(), 0)  # not contiguous
    with pytest.raises(RuntimeError):
        C.rccl_send(h, torch.zeros(4), 0)  # host tensor
    with pytest.raises((ValueError, RuntimeError)):
        C.rccl_comm_init(1, 0, b"short")


def test_rccl_comm_init_on_a_helper_thread():
    """RcclTransport runs each blocking ncclCommInitRank on a helper thread
    with a deadline (parallel/comm.py _bounded); the HIP device is per
    thread, so the helper binds the rank's GPU first.  The communicator it
    makes is used from the calling thread."""
    from llm_sharding_demo_amd.ops.hip import _load
    from llm_sharding_demo_amd.parallel.comm import _bounded

    C = _load()
    dev = torch.cuda.current_device()
    uid = C.rccl_unique_id()

    def init():
        torch.cuda.set_device(dev)
        return C.rccl_comm_init(1, 0, uid)

    h, err = _bounded(init, 60.0, "init")
    assert err is None and h
    src = torch.arange(1000, device="cuda", dtype=torch.float32)
    dst = torch.zeros_like(src)
    C.rccl_group_start()
    C.rccl_send(h, src, 0)
    C.rccl_recv(h, dst, 0)
    C.rccl_group_end()
    torch.cuda.synchronize()
    assert torch.equal(dst, src)
    C.rccl_comm_destroy(h)
