"""The one-node control plane's shared-memory broadcast ring
(csrc/runtime/shm_ring.h, parallel/comm.py ShmPlanChannel): every reader sees
every message in order, the producer never overwrites an unread slot, and the
failure modes (oversized message, a reservation /dev/shm cannot hold, a lagging
reader) are exceptions or timeouts, not crashes."""
import multiprocessing as mp
import os
import secrets

import pytest

from llm_sharding_demo_amd.runtime import native

rt = native.load()
pytestmark = pytest.mark.skipif(rt is None or not hasattr(rt, "ShmRing"), reason="native runtime not built")


def _name():
    return f"/lsd-test-{os.getpid()}-{secrets.token_hex(4)}"


def test_broadcast_in_order_to_every_reader():
    name = _name()
    w = rt.ShmRing.create(name, 4, 256, 2)
    try:
        r0, r1 = rt.ShmRing.attach(name, 0), rt.ShmRing.attach(name, 1)
        got0, got1 = [], []
        for i in range(20):  # 5 laps of a 4-slot ring
            assert w.publish(f"m{i}".encode(), 1.0)
            got0.append(r0.read(1.0))
            if i % 2:  # reader 1 drains every other message, two at a time
                got1 += [r1.read(1.0), r1.read(1.0)]
        assert got0 == [f"m{i}".encode() for i in range(20)]
        assert got1 == got0
        assert r0.read(0.01) is None  # nothing new: timeout, no stale slot
    finally:
        w.unlink()


def test_producer_waits_for_the_slowest_reader():
    name = _name()
    w = rt.ShmRing.create(name, 2, 128, 2)
    try:
        r0 = rt.ShmRing.attach(name, 0)
        rt.ShmRing.attach(name, 1)  # never reads
        assert w.publish(b"a", 0.1) and w.publish(b"b", 0.1)
        assert r0.read(0.1) == b"a" and r0.read(0.1) == b"b"
        # reader 1 still holds both slots: a third message would overwrite one
        assert not w.publish(b"c", 0.05)
    finally:
        w.unlink()


def test_bad_sizes_raise():
    name = _name()
    w = rt.ShmRing.create(name, 2, 128, 1)
    try:
        with pytest.raises(Exception):
            w.publish(b"x" * 200, 0.1)  # larger than a slot
    finally:
        w.unlink()
    with pytest.raises(Exception):  # far more than /dev/shm holds: refused up front
        rt.ShmRing.create(_name(), 1 << 20, 1 << 30, 1)
    with pytest.raises(Exception):
        rt.ShmRing.attach(_name(), 0)  # no such segment


def _reader(name, idx, n, q):
    r = rt.ShmRing.attach(name, idx)
    q.put([r.read(10.0) for _ in range(n)])


def test_readers_in_other_processes():
    name = _name()
    n = 200
    w = rt.ShmRing.create(name, 8, 256, 2)
    try:
        ctx = mp.get_context("fork")
        q = ctx.Queue()
        ps = [ctx.Process(target=_reader, args=(name, i, n, q)) for i in range(2)]
        for p in ps:
            p.start()
        for i in range(n):
            assert w.publish(i.to_bytes(4, "little") * (1 + i % 50), 10.0)
        outs = [q.get(timeout=30) for _ in ps]
        for p in ps:
            p.join(30)
        want = [i.to_bytes(4, "little") * (1 + i % 50) for i in range(n)]
        assert outs == [want, want]
    finally:
        w.unlink()


def _create_and_die(name, q):
    w = rt.ShmRing.create(name, 4, 128, 1)
    w.publish(b"last words", 1.0)
    q.put("ok")
    q.close()
    q.join_thread()  # flush the queue's feeder thread before the hard exit
    os._exit(0)  # no close, no unlink: a crashed rank 0


def test_reader_detects_dead_producer_and_close():
    name = _name()
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    p = ctx.Process(target=_create_and_die, args=(name, q))
    p.start()
    assert q.get(timeout=30) == "ok"
    p.join(30)
    r = rt.ShmRing.attach(name, 0)
    try:
        assert r.read(1.0) == b"last words"  # what was published stays readable
        assert r.read(0.01) is None and not r.closed
        assert not r.producer_alive()
    finally:
        os.unlink("/dev/shm" + name)  # a dead producer leaves its segment behind
    # a live producer that closes: readers drain, then see the ring closed
    name2 = _name()
    w = rt.ShmRing.create(name2, 4, 128, 1)
    try:
        r2 = rt.ShmRing.attach(name2, 0)
        assert r2.producer_alive()
        w.publish(b"stop", 1.0)
        w.close()
        assert r2.read(1.0) == b"stop" and r2.read(1.0) is None and r2.closed
    finally:
        w.unlink()
