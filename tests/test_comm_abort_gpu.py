"""Failure handling of the native RCCL data plane on the GPU.

An unmatched ncclRecv (a peer that never sends: dead or stalled) spins on
the GPU forever.  The engine watchdog (runtime/scheduler.py Watchdog) must
notice the stalled round within round_timeout_s, mark the engine unhealthy
and abort the communicators (ncclCommAbort), after which the stuck kernel
returns and the host wait on its stream completes -- no hang.  One GPU
cannot host a 2-rank communicator, so the stall is an unmatched receive on a
1-rank communicator driven through the same RcclTransport methods the
pipeline uses.
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
    t.C, t.L, t.comms, t.aborted, t._lock = C, 1, {("self", 0): (h, 0)}, False, threading.Lock()
    return t


def test_unmatched_recv_is_aborted_by_the_watchdog():
    from llm_sharding_demo_amd.ops.hip import _load
    from llm_sharding_demo_amd.runtime.scheduler import Watchdog

    C = _load()
    torch.cuda.set_device(0)
    h = C.rccl_comm_init(1, 0, C.rccl_unique_id())
    t = _transport_with(C, h)
    assert t.check_async() is None
    eng = SimpleNamespace(transport=t, healthy=True, last_error=None, round_started=None)
    timeout = 2.0
    wd = Watchdog(eng, round_timeout_s=timeout, poll_s=0.1)
    try:
        s = torch.cuda.Stream()
        buf = torch.zeros(4096, device="cuda")
        t0 = time.monotonic()
        eng.round_started = t0
        with torch.cuda.stream(s):
            t.irecv(buf, 0, "fwd")  # no matching send: the recv kernel waits forever
            ev = torch.cuda.Event()
            ev.record(s)
        while not ev.query():  # the host's readout wait, bounded by the test
            assert time.monotonic() - t0 < 30, "abort did not unblock the stuck receive"
            time.sleep(0.05)
        elapsed = time.monotonic() - t0
        assert not eng.healthy and eng.last_error.startswith("WatchdogTimeout"), eng.last_error
        assert t.aborted
        assert timeout <= elapsed < timeout + 10, elapsed
        with pytest.raises(Exception):  # the aborted transport refuses new work
            t.send(buf, 0, "fwd")
    finally:
        wd.close()
        if not t.aborted:
            t.abort()
    # the device is still usable afterwards
    x = torch.ones(1024, device="cuda")
    assert float((x * 2).sum()) == 2048.0
