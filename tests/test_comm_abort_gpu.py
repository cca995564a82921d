"""Failure handling of the native RCCL data plane on the GPU.

A peer that never sends leaves an ncclRecv spinning on the GPU.  The engine
watchdog (runtime/scheduler.py Watchdog) must notice the stalled round within
round_timeout_s, mark the engine unhealthy and abort the communicators
(ncclCommAbort), after which the transport refuses new work and the device
stays usable.

What one GPU can stage: RCCL refuses two ranks on one device ("Duplicate GPU
detected") and rejects a lone receive from itself on a 1-rank communicator as
invalid usage, so a receive that truly waits for an absent peer needs two
GPUs (the driver's multi-GPU run).  Here the communicator is a real 1-rank
RCCL communicator driven through the same RcclTransport methods the pipeline
uses: a grouped self exchange proves it live, then a round that stops making
progress is left to the watchdog, which must fire within the deadline and
abort that communicator.
"""
import threading
import time
from types import SimpleNamespace

import pytest
import torch

pytestmark = pytest.mark.gpu


def _transport_with(C, h):
    from llm_sharding_demo_amd.parallel.comm import RcclTransport

    t = RcclTransport.__new__(RcclTransport)  # data-plane methods only (no process groups)
    # replica 0, stage 0; the forward edge's communicator is the 1-rank one,
    # registered as member 1 so that its peer (1 - me) is rank 0 = itself
    t.C, t.L, t.aborted, t._lock = C, 1, False, threading.Lock()
    t._issue, t._inflight = threading.Condition(), 0  # the abort gate (advisor r3)
    t.replica, t.rank = 0, 0
    t.comms = {("r0fwd0", 0): (h, 1)}
    return t


def test_stalled_round_aborts_the_rccl_data_plane():
    from llm_sharding_demo_amd.ops.hip import _load
    from llm_sharding_demo_amd.runtime.scheduler import Watchdog

    C = _load()
    torch.cuda.set_device(0)
    h = C.rccl_comm_init(1, 0, C.rccl_unique_id())
    t = _transport_with(C, h)
    src = torch.arange(4096, device="cuda", dtype=torch.float32)
    dst = torch.zeros_like(src)
    C.rccl_group_start()  # live: a self exchange through the transport's methods
    t.send(src, 0, "fwd")
    t.irecv(dst, 0, "fwd")
    C.rccl_group_end()
    torch.cuda.synchronize()
    assert torch.equal(src, dst)
    assert t.check_async() is None

    eng = SimpleNamespace(transport=t, healthy=True, last_error=None, round_started=None)
    timeout = 2.0
    wd = Watchdog(eng, round_timeout_s=timeout, poll_s=0.1)
    try:
        t0 = time.monotonic()
        eng.round_started = t0  # a round begins and never completes
        while not t.aborted:
            assert time.monotonic() - t0 < timeout + 10, "watchdog did not abort the data plane"
            time.sleep(0.05)
        elapsed = time.monotonic() - t0
        assert not eng.healthy and eng.last_error.startswith("WatchdogTimeout"), eng.last_error
        assert timeout <= elapsed < timeout + 10, elapsed
        with pytest.raises(Exception):  # the aborted transport refuses new work
            t.send(src, 0, "fwd")
        assert t.check_async() is None  # aborted communicators are no longer polled
    finally:
        wd.close()
        if not t.aborted:
            t.abort()
    # the device is still usable afterwards
    x = torch.ones(1024, device="cuda")
    assert float((x * 2).sum()) == 2048.0
