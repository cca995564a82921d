"""Inter-stage transports.

Reference transport (`server.py:171-181`): per decode step the coordinator
POSTs all token ids to shard A, receives the hidden states as nested JSON
lists, re-POSTs them to shard B and receives [1, S, 50257] fp32 logits as
JSON (8-68 MB per step).  Hidden states are relayed through
the coordinator; A and B never talk directly.

Here stage i sends its boundary hidden state straight to stage i+1 and the
last stage sends the sampled token ids (int32 [B]) back to stage 0:

* `NcclTransport` -- torch.distributed over RCCL (backend "nccl" on ROCm),
  one process per MI355X.  Every pipeline edge i->i+1 and the token-return
  edge P-1->0 gets its OWN communicator (its own process group), so each
  edge has its own RCCL stream and the two directions of a 2-stage ring can
  never serialise behind each other (no cross-edge deadlock).  In an 8x
  MI355X node each edge is one direct xGMI link.  Sends/recvs are async:
  `irecv` for the next microbatch is posted before the current one is
  computed, and `Work.wait()` only makes the compute stream wait on the comm
  stream (no host sync).
* `GlooTransport` -- same protocol over gloo; device tensors are staged
  through host memory.  Used for multi-process CPU tests and for rehearsing
  the multi-rank engine on a single GPU.
* `LocalTransport` -- in-process queues between stage threads (fake
  transport for protocol tests), with optional fault injection.

Ordering contract (what makes it deadlock-free): on every edge the sender
posts sends in (step, microbatch) order and the receiver posts receives in
the same order; no stage ever waits on an edge before posting the ops it
owes on an earlier item.
"""
from __future__ import annotations

import collections
import contextlib
import datetime
import pickle
import queue
import threading
import time
from typing import Dict, List, Optional

import torch

from ..utils import racecheck


class TransportError(RuntimeError):
    pass


class Handle:
    """Result of an async receive: `.wait()` returns the tensor."""

    def __init__(self, tensor: torch.Tensor, work=None, post=None):
        self.tensor, self._work, self._post = tensor, work, post

    def wait(self) -> torch.Tensor:
        if self._work is not None:
            self._work.wait()
            self._work = None
        if self._post is not None:
            self._post()
            self._post = None
        return self.tensor


class SendHandle:
    def __init__(self, work=None):
        self._work = work

    def wait(self) -> None:
        if self._work is not None:
            self._work.wait()
            self._work = None


class Transport:
    rank: int = 0
    world: int = 1

    GRAPH_IO = False  # send / recv may not be captured into a hipGraph

    def send(self, t: torch.Tensor, dst: int, edge: str, lane: int = 0) -> SendHandle:
        raise NotImplementedError

    def irecv(self, out: torch.Tensor, src: int, edge: str, lane: int = 0) -> Handle:
        raise NotImplementedError

    def check_async(self) -> Optional[str]:
        """Asynchronous data-plane error, if the backend reports any."""
        return None

    def abort(self) -> None:
        """Unblock anything waiting on the data plane (native RCCL only)."""

    def issuing(self):
        """Context of a data-plane enqueue that bypasses send / irecv (a graph
        replay with captured transfers, the native executor): the native RCCL
        transport holds its abort gate shared across it."""
        return contextlib.nullcontext()

    def broadcast_object(self, obj, src: int = 0):
        raise NotImplementedError

    def barrier(self) -> None:
        pass

    def close(self) -> None:
        pass


# ---------------------------------------------------------------------------
# torch.distributed transports
# ---------------------------------------------------------------------------

class _DistTransport(Transport):
    """Ranks are laid out replica-major: global rank = replica * P + stage.
    `send`/`irecv` address peers by STAGE index inside this rank's replica;
    every replica has its own per-edge communicators, so replicas never
    share a link or an RCCL stream."""

    EDGE_GROUPS = True  # a torch process group per pipeline edge

    def __init__(self, num_stages: int, replicas: int = 1, timeout_s: Optional[float] = None):
        import torch.distributed as dist

        self.dist = dist
        self.grank = dist.get_rank()
        self.gworld = dist.get_world_size()
        P, R = num_stages, replicas
        if self.gworld != P * R:
            raise TransportError(f"world size {self.gworld} != num_stages {P} x replicas {R}")
        self.P, self.R = P, R
        self.replica, self.rank = divmod(self.grank, P)  # rank = stage index
        self.world = P
        # Groups must be created by every rank in the same order.  Edge and
        # control groups get the engine's round deadline (new_group does not
        # inherit the default group's timeout: gloo would wait 30 min on a
        # dead peer)
        kw = {"timeout": datetime.timedelta(seconds=timeout_s)} if timeout_s else {}
        # the control group carries bring-up collectives (communicator ids,
        # warm-up barriers, KV sizing) and stats: never shorter than 10 min
        ckw = {"timeout": datetime.timedelta(seconds=max(timeout_s, 600.0))} if timeout_s else {}
        self.ctrl = dist.new_group(list(range(P * R)), backend="gloo", **ckw)
        # every rank reaches the edge groups' connect phase together: a rank
        # still importing / binding its GPU must not exhaust a short round
        # deadline there (seen with a 4 s deadline on a loaded host)
        dist.barrier(group=self.ctrl)
        self.groups: Dict[str, object] = {}
        for rep in range(R):
            base = rep * P
            for i in range(P - 1):
                self.groups[f"r{rep}fwd{i}"] = (dist.new_group([base + i, base + i + 1], backend=self._backend(),
                                                               **kw) if self.EDGE_GROUPS else None)
            if P > 1:
                self.groups[f"r{rep}ret"] = (dist.new_group([base + P - 1, base], backend=self._backend(), **kw)
                                             if self.EDGE_GROUPS else None)
        # step plans (rank 0 -> every rank) and DP token readouts (replica
        # stage 0 -> rank 0) travel on their own gloo groups with no practical
        # timeout: an idle server waits on them indefinitely
        idle = datetime.timedelta(days=30)
        self.plan_pg = dist.new_group(list(range(P * R)), backend="gloo", timeout=idle)
        self.tok_pg = dist.new_group(list(range(P * R)), backend="gloo", timeout=idle)

    def _backend(self) -> str:
        raise NotImplementedError

    @property
    def num_comms(self) -> int:
        """Data-plane communicators this rank belongs to (one per edge group)."""
        return sum(1 for name in self.groups if self.grank in self._members(name))

    def _g(self, stage: int) -> int:
        return self.replica * self.P + stage

    def _edge_group(self, edge: str, src: int, dst: int):
        if edge == "fwd":
            return self.groups[f"r{self.replica}fwd{min(src, dst)}"]
        return self.groups[f"r{self.replica}ret"]

    def gather_object(self, obj, dst: int = 0):
        """Gather one picklable object per rank on global rank `dst` (ctrl plane)."""
        out = [None] * self.gworld if self.grank == dst else None
        self.dist.gather_object(obj, out, dst=dst, group=self.ctrl)
        return out

    def broadcast_object(self, obj, src: int = 0):
        lst = [obj]
        self.dist.broadcast_object_list(lst, src=src, group=self.ctrl)
        return lst[0]

    def barrier(self) -> None:
        self.dist.barrier(group=self.ctrl)

    def agree(self, err: Optional[str], what: str) -> None:
        """Every rank learns every rank's outcome of one bring-up step; any
        failure raises the SAME TransportError on all of them, so they leave
        together (to a fallback transport) instead of one rank waiting in a
        communicator init or a transfer on a peer that already left."""
        errs = [None] * self.gworld
        self.dist.all_gather_object(errs, err, group=self.ctrl)
        bad = [e for e in errs if e]
        if bad:
            raise TransportError(f"{what}: " + "; ".join(bad[:4]) + (" ..." if len(bad) > 4 else ""))

    def warmup(self, device) -> None:
        """Eagerly create every edge communicator in a fixed global order so no
        rank blocks in a lazy ncclCommInitRank while its peer waits elsewhere.

        A single isend/irecv does NOT run on a group's collective communicator:
        ProcessGroupNCCL keys it by the peer pair and creates that
        communicator lazily (a blocking init) on the first p2p op.  In the
        pipeline, stage 0 posts its return-edge irecv ahead of its first
        forward send, so a lazy init there would wait for stage P-1 while
        stage P-1 waits for the forward hop: deadlock.  So every edge does one
        blocking p2p exchange here, in the order fwd0, fwd1, ..., ret (the same
        on every rank): rank k joins fwd(k-1) then fwd(k), a chain that
        completes left to right and ends with the return edge."""
        dev = torch.device(device) if self._backend() == "nccl" else torch.device("cpu")
        sync = (lambda: torch.cuda.synchronize(dev)) if dev.type == "cuda" else (lambda: None)
        for name, g in self.groups.items():
            members = self._members(name)
            if self.grank not in members:
                continue
            t = torch.ones(1, device=dev)
            self.dist.all_reduce(t, group=g)  # the group's collective communicator
            src, dst = members  # fwd: lower stage -> higher; ret: P-1 -> 0
            buf = torch.full((1,), float(src), device=dev)
            if self.grank == src:
                self.dist.isend(buf, dst, group=g).wait()
            else:
                self.dist.irecv(buf, src, group=g).wait()
                sync()
                if float(buf.item()) != float(src):
                    raise TransportError(f"warmup p2p on {name}: got {buf.item()}, want {src}")
        sync()
        self.barrier()

    def _members(self, name: str) -> List[int]:
        """Global ranks of group `r{rep}fwd{i}` / `r{rep}ret`."""
        rep, kind = name[1:].split("fwd") if "fwd" in name else (name[1:-3], "ret")
        base = int(rep) * self.P
        if kind == "ret":
            return [base + self.P - 1, base]
        i = int(kind)
        return [base + i, base + i + 1]


class NcclTransport(_DistTransport):
    """RCCL point-to-point over xGMI (backend 'nccl' IS RCCL on ROCm)."""

    def _backend(self) -> str:
        return "nccl"

    def send(self, t, dst, edge, lane=0):
        g = self._edge_group(edge, self.rank, dst)
        if not t.is_contiguous():  # p2p needs a dense buffer (views of padded rows)
            t = t.contiguous()
        return SendHandle(self.dist.isend(t, self._g(dst), group=g))

    def irecv(self, out, src, edge, lane=0):
        g = self._edge_group(edge, src, self.rank)
        if out.is_contiguous():
            return Handle(out, self.dist.irecv(out, self._g(src), group=g))
        tmp = torch.empty(out.shape, dtype=out.dtype, device=out.device)
        return Handle(out, self.dist.irecv(tmp, self._g(src), group=g), post=lambda: out.copy_(tmp))


class GlooTransport(_DistTransport):
    """Same protocol over gloo; device tensors are staged via host memory."""

    def _backend(self) -> str:
        return "gloo"

    def send(self, t, dst, edge, lane=0):
        g = self._edge_group(edge, self.rank, dst)
        host = t.detach().to("cpu", copy=True) if t.device.type != "cpu" else t.detach().clone()
        return SendHandle(self.dist.isend(host, self._g(dst), group=g))

    def irecv(self, out, src, edge, lane=0):
        g = self._edge_group(edge, src, self.rank)
        if out.device.type == "cpu":
            return Handle(out, self.dist.irecv(out, self._g(src), group=g))
        host = torch.empty(out.shape, dtype=out.dtype)
        work = self.dist.irecv(host, self._g(src), group=g)
        return Handle(out, work, post=lambda: out.copy_(host))


class RcclTransport(_DistTransport):
    """Pipeline edges on the native RCCL communicator (csrc/comm.cpp), with
    the decode step's receive and send captured INSIDE the stage's hipGraph.

    Communicators: one 2-rank RCCL communicator per (pipeline edge, lane) --
    edge = stage i -> i+1 or the token return P-1 -> 0, lane = the HIP stream
    a microbatch group runs on (group g -> lane g % L on every stage,
    parallel/pipeline.py).  RCCL requires the operations of a communicator to
    execute in the same order on both ranks; a lane stream executes its items
    in plan order on every rank, so each communicator's ops are totally
    ordered without a dedicated comm stream or any event hop.

    Ops are enqueued on the CURRENT stream: eagerly (the lane stream) or
    during a graph capture (the capture stream -> replayed on the lane).  A
    decode item therefore costs one graph launch: recv -> blocks -> send
    (stage 0: embed -> blocks -> send, after its eager token-return recv;
    stage P-1: recv -> blocks -> lm_head -> sampler -> send).  Sends and
    receives return already-"complete" handles: every later use of the
    buffers is on the same lane stream, so stream order is the
    synchronisation.

    Failure handling: `check_async()` polls every communicator's
    asynchronous error (ncclCommGetAsyncError); `abort()` aborts them all
    (ncclCommAbort), which makes an RCCL kernel blocked on a dead or stalled
    peer return, so the host threads waiting on the lanes wake up and the
    engine fails its requests instead of hanging (runtime/scheduler.py
    Watchdog).

    Bring-up: the unique id of each communicator is made by its first member
    and broadcast over the gloo control group; members join in a fixed global
    order (edge-major, then lane), so the blocking inits complete left to
    right, as in `warmup`.  Every step is bounded and agreed (`agree`): a
    failed or hung init on any rank raises the same TransportError on every
    rank (the engine then falls back to torch's RCCL groups, see
    `open_data_plane`); an init still blocked at its deadline is left on a
    daemon thread."""

    EDGE_GROUPS = False
    GRAPH_IO = True  # the pipeline may capture send / recv into decode graphs

    def _backend(self) -> str:
        return "gloo"  # control plane only; the data plane is native

    def __init__(self, num_stages: int, replicas: int = 1, lanes: int = 2,
                 timeout_s: Optional[float] = None, init_s: float = 120.0):
        super().__init__(num_stages, replicas, timeout_s)
        self.L = max(1, lanes)
        self.comms: Dict[tuple, tuple] = {}  # (edge group name, lane) -> (handle, my index)
        self.aborted = False
        self._lock = threading.Lock()
        # abort gate: every enqueue that touches a communicator runs between
        # _enter / _exit; abort() flips `aborted` (no new enqueue starts), then
        # waits for the enqueues in flight before ncclCommAbort frees the
        # communicators (bounded: an enqueue stuck behind a hung GPU must not
        # keep the abort that would unstick it from running)
        self._issue = threading.Condition()
        self._inflight = 0
        err = None
        dev_idx = 0
        try:
            from ..ops.hip import _load

            self.C = _load()
            self.C.rccl_version()  # resolves librccl and its symbols
            # the bounded init runs on a helper thread, and the current HIP
            # device is per thread: bind it to this rank's GPU there, or every
            # rank's communicators would land on device 0
            dev_idx = torch.cuda.current_device()
        except Exception as e:  # noqa: BLE001 - every rank must learn the outcome
            err = f"rank {self.grank}: {type(e).__name__}: {e}"
        self.agree(err, "native RCCL unavailable")

        def comm_init(me: int, uid: bytes) -> int:
            torch.cuda.set_device(dev_idx)
            return self.C.rccl_comm_init(2, me, uid)

        try:
            for name in self.groups:
                members = self._members(name)
                for lane in range(self.L):
                    uid, err = None, None
                    if self.grank == members[0]:
                        try:
                            uid = self.C.rccl_unique_id()
                        except Exception as e:  # noqa: BLE001
                            err = f"rank {self.grank}: ncclGetUniqueId: {e}"
                    uid = self.broadcast_object(uid, src=members[0])
                    if self.grank in members and err is None and uid is not None:
                        me = members.index(self.grank)
                        h, err = _bounded(lambda: comm_init(me, uid), init_s,
                                          f"rank {self.grank}: ncclCommInitRank {name}/lane{lane}")
                        if h:
                            self.comms[(name, lane)] = (h, me)
                    self.agree(err, f"RCCL communicator {name}/lane{lane}")
        except TransportError:
            self.abort(drain_s=0.0)  # free the communicators made so far
            raise

    @property
    def num_comms(self) -> int:
        return len(self.comms)

    def _edge(self, edge: str, src: int, dst: int, lane: int):
        name = f"r{self.replica}fwd{min(src, dst)}" if edge == "fwd" else f"r{self.replica}ret"
        if self.aborted:
            raise TransportError(f"RCCL communicators aborted; {edge} edge unusable")
        return self.comms[(name, lane % self.L)]

    @contextlib.contextmanager
    def issuing(self):
        with self._issue:
            if self.aborted:
                raise TransportError("RCCL communicators aborted")
            self._inflight += 1
        try:
            yield
        finally:
            with self._issue:
                self._inflight -= 1
                self._issue.notify_all()

    def send(self, t, dst, edge, lane: int = 0):
        if not t.is_contiguous():
            t = t.contiguous()
        with self.issuing():
            h, me = self._edge(edge, self.rank, dst, lane)
            self.C.rccl_send(h, t, 1 - me)
        t.record_stream(torch.cuda.current_stream())
        return SendHandle()

    def irecv(self, out, src, edge, lane: int = 0):
        buf = out if out.is_contiguous() else torch.empty(out.shape, dtype=out.dtype, device=out.device)
        with self.issuing():
            h, me = self._edge(edge, src, self.rank, lane)
            self.C.rccl_recv(h, buf, 1 - me)
        if buf is out:
            return Handle(out)
        return Handle(out, post=lambda: out.copy_(buf))

    def native_recv(self, edge: str, src: int, lane: int) -> tuple:
        """("rccl", communicator, peer) of a receive the native executor enqueues."""
        h, me = self._edge(edge, src, self.rank, lane)
        return ("rccl", h, 1 - me)

    # graph capture: the same enqueue on the capture stream
    capture_send = send
    capture_recv = irecv

    def warmup(self, device) -> None:
        """One exchange per communicator, in the global order (checks the data)."""
        for (name, lane), (h, me) in self.comms.items():
            src = self._members(name)[0]
            kind = "ret" if name.endswith("ret") else "fwd"
            if me == 0:
                buf = torch.full((4,), float(src * self.L + lane), device=device)
                self.send(buf, self._stage_of(self._members(name)[1]), kind, lane)
                torch.cuda.synchronize(device)
            else:
                got = torch.zeros(4, device=device)
                self.irecv(got, self._stage_of(src), kind, lane).wait()
                torch.cuda.synchronize(device)
                if float(got[0].item()) != float(src * self.L + lane):
                    raise TransportError(f"warmup RCCL p2p on {name}/lane{lane}: got {got[0].item()}")
        torch.cuda.synchronize(device)
        self.barrier()

    def _stage_of(self, grank: int) -> int:
        return grank % self.P

    def check_async(self) -> Optional[str]:
        """First asynchronous RCCL error of any communicator, or None."""
        with self._lock:
            if self.aborted or getattr(self, "_comms_aborted", False):
                return None
            for (name, lane), (h, _) in self.comms.items():
                e = self.C.rccl_async_error(h)
                if e not in (0, 7):  # ncclSuccess, ncclInProgress
                    return f"RCCL {name}/lane{lane}: {self.C.rccl_error_string(e)}"
        return None

    def abort(self, drain_s: float = 5.0) -> None:
        """Abort every communicator (unblocks kernels waiting on a peer).
        New enqueues are refused first; enqueues already inside an RCCL call
        get up to `drain_s` to leave it before the communicators are freed."""
        with self._issue:
            self.aborted = True
            deadline = time.monotonic() + drain_s
            while self._inflight and time.monotonic() < deadline:
                self._issue.wait(0.05)
        with self._lock:
            if getattr(self, "_comms_aborted", False):
                return
            self._comms_aborted = True
            for h, _ in self.comms.values():
                try:
                    self.C.rccl_comm_abort(h)
                except RuntimeError:
                    pass

    def close(self) -> None:
        with self._lock:
            if self.aborted:
                self.comms.clear()
                return
            torch.cuda.synchronize()
            for h, _ in self.comms.values():
                self.C.rccl_comm_destroy(h)
            self.comms.clear()


# ---------------------------------------------------------------------------
# Plan channels: stage 0's scheduler -> the other stages (runtime/plan.py)
# ---------------------------------------------------------------------------

class LocalPlanChannel:
    """In-process: one FIFO per follower stage thread."""

    def __init__(self, stages: List[int]):
        self.q = {r: queue.Queue() for r in stages}

    def send(self, dst: int, obj) -> None:
        self.q[dst].put(obj)

    def send_many(self, dsts: List[int], obj) -> None:
        for d in dsts:
            self.q[d].put(obj)

    def recv(self, me: int, timeout: Optional[float] = None):
        return self.q[me].get(timeout=timeout)


class GlooPlanChannel:
    """torch.distributed gloo p2p on a dedicated group.  Step plans use the
    binary record of runtime/plan.py (one fixed-size int32 message per plan in
    steady-state decode; a pickled plan -- our own records, produced by this
    job's rank 0 -- only follows on composition changes, prefill chunks and
    compat forwards).  Other objects (token readouts of DP replicas) are
    pickled as a size message + a byte payload.  Sends are non-blocking
    (isend), so the scheduler never waits on a slow follower; each receiver
    posts blocking receives from its single source in FIFO order.
    `plans=False` selects the plain pickled-object channel."""

    def __init__(self, group, tag: int = 1, plans: bool = True, stages: Optional[int] = None):
        import torch.distributed as dist

        self.dist, self.pg, self.tag = dist, group, tag
        self.plans = plans
        self.P = stages  # pipeline stages per replica (None: send token ids everywhere)
        # posted sends, oldest first; completed ones are dropped from the
        # front (a scan of the whole list per send cost ~2 ms per step at
        # 7 followers x 64 steps of look-ahead: profiles/r4_plan_wire.log)
        self._works: "collections.deque" = collections.deque()
        self._enc: Dict[int, object] = {}
        self._dec: Dict[int, object] = {}
        self.bytes_sent = 0
        self.msgs_sent = 0

    def _isend(self, t: torch.Tensor, dst: int, tag: int):
        self.bytes_sent += t.numel() * t.element_size()
        self.msgs_sent += 1
        return self.dist.isend(t, dst, group=self.pg, tag=tag)

    def send(self, dst: int, obj) -> None:
        if self.plans:
            from ..runtime.plan import PlanEncoder

            enc = self._enc.get(dst)
            if enc is None:
                # token ids only to a replica's first stage
                enc = self._enc[dst] = PlanEncoder(ids=self.P is None or dst % self.P == 0)
            rec, payload = enc.encode(obj)
            hdr = torch.from_numpy(rec)
            works = [self._isend(hdr, dst, self.tag), hdr]
            if payload is not None:
                buf = torch.frombuffer(bytearray(payload), dtype=torch.uint8)
                works += [self._isend(buf, dst, self.tag + 1), buf]
        else:
            data = pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL)
            n = torch.tensor([len(data)], dtype=torch.int64)
            buf = torch.frombuffer(bytearray(data), dtype=torch.uint8)
            works = [self._isend(n, dst, self.tag), n, self._isend(buf, dst, self.tag + 1), buf]
        self._works.append(tuple(works))
        while self._works and all(x.is_completed() for x in self._works[0][0::2]):
            self._works.popleft()

    def send_many(self, dsts: List[int], obj) -> None:
        for d in dsts:
            self.send(d, obj)

    def recv(self, src: int):
        if self.plans:
            from ..runtime.plan import PLAN_WORDS, PlanDecoder

            dec = self._dec.get(src)
            if dec is None:
                dec = self._dec[src] = PlanDecoder()
            hdr = torch.empty(PLAN_WORDS, dtype=torch.int32)
            self.dist.recv(hdr, src, group=self.pg, tag=self.tag)

            def payload(nbytes: int) -> bytes:
                buf = torch.empty(nbytes, dtype=torch.uint8)
                self.dist.recv(buf, src, group=self.pg, tag=self.tag + 1)
                return buf.numpy().tobytes()
            return dec.decode(hdr.numpy(), payload)
        n = torch.empty(1, dtype=torch.int64)
        self.dist.recv(n, src, group=self.pg, tag=self.tag)
        buf = torch.empty(int(n[0]), dtype=torch.uint8)
        self.dist.recv(buf, src, group=self.pg, tag=self.tag + 1)
        return pickle.loads(buf.numpy().tobytes())

    def flush(self) -> None:
        for w in self._works:
            for x in w[0::2]:
                x.wait()
        self._works.clear()


class ShmPlanChannel:
    """One-node control plane: each pipeline replica's step plans go through a
    shared-memory broadcast ring (csrc/runtime/shm_ring.h) that rank 0 writes
    ONCE per step and every follower rank of the replica reads -- instead of
    one gloo message per follower per step (~20 us of rank 0's host time
    each).  Records are runtime/plan.py's binary plans; a pickled plan rides
    inline behind its record when it fits a slot, else over the gloo plan
    group.  Every rank of an 8-GPU MI355X node shares the host, so this is
    the default whenever torchrun reports one node (LOCAL_WORLD_SIZE ==
    WORLD_SIZE); `GlooPlanChannel` otherwise."""

    INLINE, VIA_GLOO = b"I", b"G"

    # 64 x 256 KiB = 16 MiB of /dev/shm per replica, reserved up front; a
    # pickled plan too large for a slot travels over gloo behind its record
    def __init__(self, transport: "_DistTransport", timeout_s: float, slots: int = 64,
                 slot_bytes: int = 256 << 10):
        import secrets

        from ..runtime import native

        rt = native.load()
        if rt is None or not hasattr(rt, "ShmRing"):
            raise TransportError("native runtime with ShmRing not built")
        self.P, self.R, self.grank = transport.P, transport.R, transport.grank
        # round_timeout_s <= 0 means "no watchdog", not "no wait": a publish
        # into a full ring waits for the slowest follower up to 10 min
        self.timeout_s = timeout_s if timeout_s and timeout_s > 0 else 600.0
        token = transport.broadcast_object(secrets.token_hex(6) if self.grank == 0 else None, src=0)
        import os

        prefix = os.environ.get("LSD_SHM_PREFIX", "/lsd-plan")
        names = [f"{prefix}-{token}-r{rep}" for rep in range(self.R)]
        self.readers = [[rep * self.P + s for s in range(self.P) if rep * self.P + s != 0]
                        for rep in range(self.R)]
        self.rings: Dict[int, object] = {}
        self.ring = None
        err = None
        if self.grank == 0:
            try:
                for rep in range(self.R):
                    if self.readers[rep]:
                        self.rings[rep] = rt.ShmRing.create(names[rep], slots, slot_bytes,
                                                            len(self.readers[rep]))
            except Exception as e:  # noqa: BLE001 - every rank must learn the outcome
                err = f"{type(e).__name__}: {e}"
        err = transport.broadcast_object(err, src=0)
        if err is None and self.grank != 0:
            rep = self.grank // self.P
            try:
                self.ring = rt.ShmRing.attach(names[rep], self.readers[rep].index(self.grank))
            except Exception as e:  # noqa: BLE001
                err = f"rank {self.grank}: {type(e).__name__}: {e}"
        errs = transport.gather_object(err, dst=0)
        errs = transport.broadcast_object([e for e in (errs or []) if e], src=0)
        if self.grank == 0:
            for r in self.rings.values():
                r.unlink()  # every reader is attached: the mappings outlive the names
        if err or errs:
            raise TransportError(f"shared-memory plan ring unavailable: {err or errs}")
        from ..runtime.plan import PlanDecoder, PlanEncoder

        # replica 0's stage 0 is rank 0 itself: its followers never read token ids
        self._enc = {rep: PlanEncoder(ids=rep > 0) for rep in self.rings}
        self._dec = PlanDecoder()
        self.fallback = GlooPlanChannel(transport.plan_pg, tag=1, plans=False)
        self.bytes_sent = 0
        self.msgs_sent = 0

    def send_many(self, dsts: List[int], obj) -> None:
        """Publish `obj` (a StepPlan) to the ring whose readers are `dsts`."""
        if not dsts:
            return
        rep = dsts[0] // self.P
        if sorted(dsts) != self.readers[rep]:
            raise ValueError(f"plan destinations {dsts} are not replica {rep}'s followers")
        rec, payload = self._enc[rep].encode(obj)
        ring = self.rings[rep]
        body = rec.tobytes()
        if payload is None or len(payload) + len(body) + 1 <= ring.slot_bytes - 4:
            data = self.INLINE + body + (payload or b"")
            via = False
        else:
            data, via = self.VIA_GLOO + body, True
        if not ring.publish(data, self.timeout_s):
            raise TransportError(f"plan ring of replica {rep}: followers {self.timeout_s:.0f} s behind")
        self.bytes_sent += len(data)
        self.msgs_sent += 1
        if via:
            for d in dsts:
                self.fallback.send(d, payload)

    def send(self, dst: int, obj) -> None:
        raise TypeError("ShmPlanChannel broadcasts per replica: use send_many")

    def recv(self, src: int):
        from ..runtime.plan import PLAN_WORDS

        while True:  # an idle server waits here indefinitely ...
            data = self.ring.read(1.0)
            if data is not None:
                break
            # ... on a live producer: a rank 0 that died (or closed the ring
            # without a stop plan) fails the follower instead of leaving it
            # spinning on a ring nobody will write again
            if self.ring.closed:
                raise TransportError("plan ring closed by rank 0")
            if not self.ring.producer_alive():
                raise TransportError("rank 0 (the plan ring's producer) is gone")
        import numpy as np

        nrec = 4 * PLAN_WORDS
        rec = np.frombuffer(data[1: 1 + nrec], dtype=np.int32)
        if data[:1] == self.INLINE:
            return self._dec.decode(rec, lambda n: data[1 + nrec: 1 + nrec + n])
        return self._dec.decode(rec, lambda n: self.fallback.recv(0))

    def flush(self) -> None:
        self.fallback.flush()

    def close(self) -> None:
        """Rank 0, after the followers' stop plans: end every reader's wait."""
        for r in self.rings.values():
            r.close()


def make_plan_channel(transport: "_DistTransport", timeout_s: float):
    """Shared-memory rings on one node, gloo records otherwise
    (LSD_PLAN_WIRE = shm | binary | pickle)."""
    import os

    import logging

    wire = os.environ.get("LSD_PLAN_WIRE", "shm")
    one_node = os.environ.get("LOCAL_WORLD_SIZE", "") == os.environ.get("WORLD_SIZE", "-")
    if wire == "shm" and one_node:
        try:
            return ShmPlanChannel(transport, timeout_s)
        except TransportError as e:
            # every rank saw the same error list (gathered + broadcast), so
            # all of them fall back together
            logging.getLogger("llm_sharding_demo_amd.comm").warning(
                "shared-memory plan ring unavailable (%s): plans over gloo", e)
    return GlooPlanChannel(transport.plan_pg, tag=1, plans=wire != "pickle", stages=transport.P)


# ---------------------------------------------------------------------------
# In-process fake transport (tests, single-process multi-stage)
# ---------------------------------------------------------------------------

class LocalFabric(racecheck.Shared):
    """Shared mailbox for P in-process stages.  fault: optional callable
    (edge, src, dst, seq) -> None | "drop" | float(delay seconds) | Exception."""

    def __init__(self, num_stages: int, timeout: float = 60.0, fault=None):
        self.P = num_stages
        self.timeout = timeout
        self.fault = fault
        self._q: Dict[tuple, queue.Queue] = {}
        self._lock = racecheck.Lock("fabric")
        self._bcast: Dict[int, queue.Queue] = {r: queue.Queue() for r in range(num_stages)}
        self._seq: Dict[tuple, int] = {}
        self._barrier = threading.Barrier(num_stages)
        self.failed: Optional[BaseException] = None  # a stage thread died: stop waiting on it

    def get(self, key, what: str):
        """Blocking receive from mailbox `key`, bounded by `timeout` and
        abandoned as soon as any stage thread has failed."""
        deadline = time.monotonic() + self.timeout
        q = self.q(key)
        while True:
            if self.failed is not None:
                raise TransportError(f"{what}: a pipeline stage failed: {self.failed}")
            left = deadline - time.monotonic()
            if left <= 0:
                raise TransportError(f"{what}: timed out after {self.timeout}s")
            try:
                return q.get(timeout=min(0.1, left))
            except queue.Empty:
                continue

    def q(self, key) -> queue.Queue:
        with self._lock:
            racecheck.note(self, "_q")
            if key not in self._q:
                self._q[key] = queue.Queue()
            return self._q[key]

    def next_seq(self, key) -> int:
        with self._lock:
            racecheck.note(self, "_seq")
            n = self._seq.get(key, 0)
            self._seq[key] = n + 1
            return n

    def transport(self, rank: int, kind: str = "local") -> Transport:
        if kind == "loopback":
            return LoopbackTransport(self, rank)
        if kind == "strict":
            return StrictLocalTransport(self, rank)
        return LocalTransport(self, rank)


class LoopbackTransport(Transport):
    """Device-async in-process transport: P stage threads on ONE MI355X.

    `send` snapshots the tensor on the sender's stream (an async D2D copy into
    a fresh buffer) and publishes it with a hipEvent; `irecv(...).wait()` makes
    the receiver's stream wait on that event and copies into the receive
    buffer -- no host synchronisation of the device anywhere, unlike
    LocalTransport (whose send synchronises the stream).  This rehearses the
    real RCCL schedule's ordering (stream waits, not host waits) on a single
    GPU: the host threads only hand each other event handles."""

    def __init__(self, fabric: LocalFabric, rank: int):
        self.fabric, self.rank, self.world = fabric, rank, fabric.P

    def send(self, t, dst, edge, lane=0):
        key = (edge, self.rank, dst)
        cur = torch.cuda.current_stream(t.device)
        buf = t.detach().clone()  # enqueued on the sender's stream
        ev = torch.cuda.Event()
        ev.record(cur)
        self.fabric.q(key).put((buf, ev))
        return SendHandle()

    def irecv(self, out, src, edge, lane=0):
        key = (edge, src, self.rank)
        fabric = self.fabric

        def post():
            from .pipeline import GPU_GATE

            buf, ev = fabric.get(key, f"stage {self.rank} waiting on {edge} from stage {src}")
            with GPU_GATE.shared():  # never beside another stage thread's capture
                cur = torch.cuda.current_stream(out.device)
                cur.wait_event(ev)
                buf.record_stream(cur)  # the sender's pool must not recycle it early
                out.copy_(buf, non_blocking=True)

        return Handle(out, None, post=post)

    def broadcast_object(self, obj, src: int = 0):
        return LocalTransport.broadcast_object(self, obj, src)

    def barrier(self) -> None:
        self.fabric._barrier.wait(timeout=self.fabric.timeout)


class DeviceLoopFabric(LocalFabric):
    """P in-process stages on ONE MI355X joined by device loopback channels
    (csrc/kernels/loopback.hip, csrc/loop_fabric.cpp): the single-GPU
    rehearsal of the RCCL data plane, graph I/O included.

    One channel per (edge, lane) -- forward edges i -> i+1 and the token
    return P-1 -> 0, times the L lane streams -- exactly the communicator
    layout of `RcclTransport`, with the same contract: ops of a channel are
    matched in FIFO order, so both ends must issue them in the same order.
    Every receive checks the size of the message at its channel's head on
    the device and records a mismatch instead of copying, so the rehearsal
    verifies RCCL's op-ordering contract on every transfer.

    Ring sizing: a message must fit its channel's ring (`ring_bytes` for the
    forward edges, `ret_bytes` for the token return); both are allocated up
    front, before the KV cache takes its share of HBM."""

    def __init__(self, num_stages: int, device: torch.device, lanes: int, ring_bytes: int,
                 ret_bytes: int = 16 << 20, timeout: float = 60.0, spin_limit_s: float = 30.0):
        super().__init__(num_stages, timeout=timeout)
        from ..ops.hip import _load

        self.C = _load()
        self.L = max(1, lanes)
        self.device = device
        self.handle = self.C.loop_fabric_create(float(timeout))
        self._keep: List[torch.Tensor] = []
        self.chans: Dict[tuple, int] = {}
        nstate = self.C.loop_state_bytes()
        edges = [("fwd", i, i + 1) for i in range(num_stages - 1)]
        if num_stages > 1:
            edges.append(("ret", num_stages - 1, 0))
        with torch.cuda.device(device):
            for edge, src, dst in edges:
                nbytes = ring_bytes if edge == "fwd" else ret_bytes
                nbytes = -(-nbytes // 256) * 256
                for lane in range(self.L):
                    state = torch.zeros(nstate, dtype=torch.uint8, device=device)
                    ring = torch.empty(nbytes, dtype=torch.uint8, device=device)
                    self._keep += [state, ring]
                    self.chans[(edge, src, dst, lane)] = self.C.loop_chan_create(
                        self.handle, state, ring, float(spin_limit_s))
            torch.cuda.synchronize(device)
        self.aborted = False

    def transport(self, rank: int, kind: str = "devloop") -> Transport:
        return DeviceLoopTransport(self, rank)

    def chan(self, edge: str, src: int, dst: int, lane: int) -> int:
        return self.chans[(edge, src, dst, lane % self.L)]

    # data-plane health (runtime/scheduler.py Watchdog)
    def check_async(self) -> Optional[str]:
        err, ch = self.C.loop_status(self.handle)
        if err == 0 or self.aborted:
            return None
        keys = list(self.chans)  # creation order = channel id
        what = {1: "aborted", 2: "device wait timed out",
                3: "receive size != message size (op order mismatch)"}
        key = keys[ch] if 0 <= ch < len(keys) else ch
        return f"loopback channel {key}: {what.get(err, f'error {err}')}"

    def abort(self) -> None:
        """Make every waiting kernel and host handshake give up (the RCCL
        transport's ncclCommAbort)."""
        self.aborted = True
        self.C.loop_abort(self.handle)

    def stall(self, edge: str, src: int, dst: int, lane: int, from_msg: int) -> None:
        """Fault injection: sends number >= from_msg on this channel are never
        published (the receiver's kernel waits on the device)."""
        self.C.loop_stall(self.chan(edge, src, dst, lane), from_msg)

    def counts(self, edge: str, src: int, dst: int, lane: int) -> tuple:
        """(sends enqueued, receives enqueued, send bytes end, recv bytes end)."""
        return tuple(self.C.loop_counts(self.chan(edge, src, dst, lane)))


class _LoopOps:
    """Data-plane ops over device loopback channels (csrc/loop_fabric.cpp),
    with `RcclTransport`'s API: ops enqueued on the current stream, eagerly
    or inside a hipGraph capture; handles already complete in stream order.
    The subclass provides `C`, `_loop_aborted()` and `_chan(edge, src, dst,
    lane)`."""

    GRAPH_IO = True

    def _op(self, ch: int, d: int, t: torch.Tensor) -> None:
        from .pipeline import GPU_GATE

        if self._loop_aborted():
            raise TransportError("loopback data plane aborted")
        nbytes = t.numel() * t.element_size()
        ops = getattr(self._tls, "ops", None)
        if ops is not None and torch.cuda.is_current_stream_capturing():
            (self.C.loop_recv if d else self.C.loop_send)(ch, t, True)
            ops.append((ch, d, nbytes))
            return
        try:
            with GPU_GATE.released():  # the peer may need the gate to reach its enqueue
                self.C.loop_wait([(ch, d, nbytes)])
            with GPU_GATE.shared():
                (self.C.loop_recv if d else self.C.loop_send)(ch, t, False)
        except RuntimeError as e:
            raise TransportError(str(e)) from e

    def send(self, t, dst, edge, lane=0):
        if not t.is_contiguous():
            t = t.contiguous()
        self._op(self._chan(edge, self.rank, dst, lane), 0, t)
        return SendHandle()

    def irecv(self, out, src, edge, lane=0):
        ch = self._chan(edge, src, self.rank, lane)
        if out.is_contiguous():
            self._op(ch, 1, out)
            return Handle(out)
        buf = torch.empty(out.shape, dtype=out.dtype, device=out.device)
        self._op(ch, 1, buf)
        return Handle(out, post=lambda: out.copy_(buf))

    capture_send = send
    capture_recv = irecv

    # -- graph I/O: ops captured inside a decode graph ----------------------
    def begin_capture(self) -> None:
        self._tls.ops = []

    def end_capture(self) -> tuple:
        """(native I/O-list handle or 0, op list) of the capture just ended."""
        ops = self._tls.ops
        self._tls.ops = None
        return (self.C.loop_io_create(ops) if ops else 0), ops

    def prewait(self, ops: List[tuple]) -> None:
        """Enqueue handshake of (chan, dir, bytes) ops about to be issued,
        outside the capture gate (the step's ops in the native executor)."""
        from .pipeline import GPU_GATE

        if self._loop_aborted():
            raise TransportError("loopback data plane aborted")
        if not ops:
            return
        try:
            with GPU_GATE.released():
                self.C.loop_wait(ops)
        except RuntimeError as e:
            raise TransportError(str(e)) from e

    def replay(self, g, io: int, ops: List[tuple]) -> None:
        """Launch a decode graph whose loopback ops are `io` on the current
        stream: handshake (gate released), launch, advance the mirrors."""
        self.prewait(ops)
        try:
            self.C.loop_graph_launch(g.raw_cuda_graph_exec(), io)
        except RuntimeError as e:
            raise TransportError(str(e)) from e

    def native_recv(self, edge: str, src: int, lane: int) -> tuple:
        """("loop", channel) of a receive the native executor enqueues."""
        return ("loop", self._chan(edge, src, self.rank, lane))


class DeviceLoopTransport(_LoopOps, Transport):
    """One stage thread's view of a `DeviceLoopFabric` (P stage threads in
    one process), so the pipeline takes its graph-I/O path and the native
    executor exactly as over RCCL."""

    def __init__(self, fabric: DeviceLoopFabric, rank: int):
        self.fabric, self.rank, self.world = fabric, rank, fabric.P
        self.C = fabric.C
        self._tls = threading.local()

    @property
    def aborted(self) -> bool:
        return self.fabric.aborted

    def _loop_aborted(self) -> bool:
        return self.fabric.aborted

    def _chan(self, edge, src, dst, lane):
        return self.fabric.chan(edge, src, dst, lane)

    def check_async(self) -> Optional[str]:
        return self.fabric.check_async()

    def abort(self) -> None:
        self.fabric.abort()

    def broadcast_object(self, obj, src: int = 0):
        return LocalTransport.broadcast_object(self, obj, src)

    def barrier(self) -> None:
        self.fabric._barrier.wait(timeout=self.fabric.timeout)


class IpcLoopTransport(_LoopOps, _DistTransport):
    """Dist mode (one process per stage, torch.distributed control plane) with
    every rank on the SAME GPU and the pipeline edges on device loopback
    channels shared between the processes: the single-GPU rehearsal of the
    8-GPU `--transport rccl` run -- separate processes (no shared GIL, the
    gloo / shared-memory control plane, worker_loop followers), decode graphs
    with their own edge transfers, the native executor at P > 1.  Only the
    RCCL byte mover itself is replaced (RCCL refuses two ranks on one GPU).

    Channels: one per (replica, edge, lane), as `RcclTransport`'s
    communicators.  The receiving rank allocates a channel's device state and
    ring (hipMalloc) and exports them (hipIpcGetMemHandle); the sending rank
    maps them.  Both ends' enqueue mirrors live in one POSIX shared-memory
    block created by rank 0.  Each process keeps its own pinned abort / error
    word (its watchdog aborts its own waits)."""

    EDGE_GROUPS = False

    def _backend(self) -> str:
        return "gloo"

    def __init__(self, num_stages: int, replicas: int = 1, lanes: int = 2,
                 timeout_s: Optional[float] = None, ring_bytes: int = 64 << 20,
                 ret_bytes: int = 16 << 20, spin_limit_s: float = 30.0):
        import secrets

        super().__init__(num_stages, replicas, timeout_s)
        from ..ops.hip import _load

        self.C = _load()
        self.L = max(1, lanes)
        self._tls = threading.local()
        self.aborted = False
        self.handle = self.C.loop_fabric_create(float(timeout_s or 600.0))
        P, R = self.P, self.R
        table = []  # (replica, edge, src stage, dst stage, lane): channel id = index
        for rep in range(R):
            for i in range(P - 1):
                table += [(rep, "fwd", i, i + 1, l) for l in range(self.L)]
            if P > 1:
                table += [(rep, "ret", P - 1, 0, l) for l in range(self.L)]
        token = self.broadcast_object(secrets.token_hex(6) if self.grank == 0 else None, src=0)
        name = f"/lsd-loop-{token}"
        nmir = max(1, len(table)) * 64
        if self.grank == 0:
            base = self.C.loop_shm_map(name, nmir, True)
        self.barrier()
        if self.grank != 0:
            base = self.C.loop_shm_map(name, nmir, False)
        self.barrier()
        if self.grank == 0:
            self.C.loop_shm_unlink(name)
        nstate = self.C.loop_state_bytes()
        self._own: List[int] = []
        self.chans: Dict[tuple, int] = {}
        exports = {}
        for cid, (rep, edge, src, dst, lane) in enumerate(table):
            if rep * P + dst != self.grank:
                continue
            cap = -(-(ring_bytes if edge == "fwd" else ret_bytes) // 256) * 256
            st, ring = self.C.loop_dev_alloc(nstate), self.C.loop_dev_alloc(cap)
            self._own += [st, ring]
            self.chans[(edge, src, dst, lane)] = self.C.loop_chan_attach(
                self.handle, st, ring, cap, cid, base + 64 * cid, True, float(spin_limit_s))
            exports[cid] = (self.C.loop_ipc_handle(st), self.C.loop_ipc_handle(ring), cap)
        torch.cuda.synchronize()
        allx = self.gather_object(exports, dst=0)
        merged = {}
        for d in (allx or []):
            merged.update(d or {})
        merged = self.broadcast_object(merged, src=0)  # receivers initialised before senders attach
        for cid, (rep, edge, src, dst, lane) in enumerate(table):
            if rep * P + src != self.grank:
                continue
            hs, hr, cap = merged[cid]
            st, ring = self.C.loop_ipc_open(hs), self.C.loop_ipc_open(hr)
            self.chans[(edge, src, dst, lane)] = self.C.loop_chan_attach(
                self.handle, st, ring, cap, cid, base + 64 * cid, False, float(spin_limit_s))
        self.barrier()

    @property
    def num_comms(self) -> int:
        return len(self.chans)

    def _loop_aborted(self) -> bool:
        return self.aborted

    def _chan(self, edge, src, dst, lane):
        return self.chans[(edge, src, dst, lane % self.L)]

    def warmup(self, device) -> None:
        """One exchange per channel in the global order, checking the data."""
        for (edge, src, dst, lane) in sorted(self.chans, key=lambda k: (k[0] != "fwd", k[1], k[3])):
            tag = float(src * self.L + lane + 1)
            if src == self.rank:
                self.send(torch.full((4,), tag, device=device), dst, edge, lane)
            else:
                got = torch.zeros(4, device=device)
                self.irecv(got, src, edge, lane)
                torch.cuda.synchronize(device)
                if float(got[0].item()) != tag:
                    raise TransportError(f"warmup on {edge} {src}->{dst} lane {lane}: got {got[0].item()}")
        torch.cuda.synchronize(device)
        self.barrier()

    def check_async(self) -> Optional[str]:
        if self.aborted:
            return None
        err, ch = self.C.loop_status(self.handle)
        if err == 0:
            return None
        what = {1: "aborted", 2: "device wait timed out",
                3: "receive size != message size (op order mismatch)"}
        return f"loopback channel {ch}: {what.get(err, f'error {err}')}"

    def abort(self) -> None:
        self.aborted = True
        self.C.loop_abort(self.handle)

    def stall(self, edge: str, src: int, dst: int, lane: int, from_msg: int) -> None:
        self.C.loop_stall(self._chan(edge, src, dst, lane), from_msg)


class LocalTransport(Transport):
    def __init__(self, fabric: LocalFabric, rank: int):
        self.fabric, self.rank, self.world = fabric, rank, fabric.P

    def send(self, t, dst, edge, lane=0):
        key = (edge, self.rank, dst)
        seq = self.fabric.next_seq(key)
        payload = t.detach().clone()
        if t.is_cuda:
            torch.cuda.current_stream(t.device).synchronize()
        f = self.fabric.fault(edge, self.rank, dst, seq) if self.fabric.fault else None
        if isinstance(f, Exception):
            raise f
        if f == "drop":
            return SendHandle()
        if isinstance(f, (int, float)) and f > 0:
            time.sleep(f)
        self.fabric.q(key).put(payload)
        return SendHandle()

    def irecv(self, out, src, edge, lane=0):
        key = (edge, src, self.rank)
        fabric = self.fabric

        def post():
            t = fabric.get(key, f"stage {self.rank} waiting on {edge} from stage {src}")
            out.copy_(t)

        return Handle(out, None, post=post)

    def broadcast_object(self, obj, src: int = 0):
        if self.rank == src:
            for r in range(self.world):
                if r != src:
                    self.fabric._bcast[r].put(obj)
            return obj
        return self.fabric._bcast[self.rank].get(timeout=self.fabric.timeout)

    def barrier(self) -> None:
        self.fabric._barrier.wait(timeout=self.fabric.timeout)


class StrictLocalTransport(LocalTransport):
    """CPU twin of the RCCL data plane's matching rule, for protocol tests.

    One FIFO per (edge, src, dst, lane) -- the communicator layout of
    `RcclTransport` / `DeviceLoopFabric` -- and every receive checks that
    the message at its channel's head has the posted size and dtype, raising
    `TransportError` on a mismatch instead of copying.  `GRAPH_IO` makes the
    stage worker take its graph-I/O code path (parallel/pipeline.py `_io`):
    on CPU the decode "graph" body runs eagerly every step, calling
    `capture_recv` / `capture_send` exactly where a captured graph would.
    Every op is appended to `fabric.oplog` as (edge, src, dst, lane, dir,
    bytes, dtype) so tests can compare the two ends of each channel."""

    GRAPH_IO = True
    SIM_GRAPH_IO = True

    def __init__(self, fabric: LocalFabric, rank: int):
        super().__init__(fabric, rank)
        if not hasattr(fabric, "oplog"):
            fabric.oplog = []  # list.append is atomic under the GIL

    def send(self, t, dst, edge, lane=0):
        key = ("strict", edge, self.rank, dst, lane)
        payload = t.detach().clone()
        self.fabric.oplog.append((edge, self.rank, dst, lane, "send",
                                  t.numel() * t.element_size(), str(t.dtype)))
        self.fabric.q(key).put(payload)
        return SendHandle()

    def _take(self, out, src, edge, lane):
        key = ("strict", edge, src, self.rank, lane)
        t = self.fabric.get(key, f"stage {self.rank} waiting on {edge}/lane{lane} from stage {src}")
        nb, ob = t.numel() * t.element_size(), out.numel() * out.element_size()
        self.fabric.oplog.append((edge, src, self.rank, lane, "recv", ob, str(out.dtype)))
        if nb != ob or t.dtype != out.dtype:
            err = TransportError(f"op order mismatch on {edge} {src}->{self.rank} lane {lane}: posted "
                                 f"{ob} B {out.dtype}, head message {nb} B {t.dtype}")
            self.fabric.failed = err
            raise err
        out.copy_(t.view(out.shape))

    def irecv(self, out, src, edge, lane=0):
        return Handle(out, None, post=lambda: self._take(out, src, edge, lane))

    def capture_recv(self, out, src, edge, lane=0):
        self._take(out, src, edge, lane)  # in stream order: complete on return
        return Handle(out)

    capture_send = send


def init_distributed(backend: str, device_type: str, timeout_s: float = 600.0) -> None:
    """Initialise torch.distributed from torchrun env vars (RANK, WORLD_SIZE,
    LOCAL_RANK, MASTER_ADDR/PORT).  Binds the process to its GPU first.

    `timeout_s` bounds every collective / p2p op: with RCCL's async error
    handling a peer that died or hung turns into an exception on the waiting
    ranks after the timeout instead of a silent hang."""
    import datetime
    import os

    import torch.distributed as dist

    if dist.is_initialized():
        return
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    # the default group only carries bring-up (rendezvous, group creation):
    # never shorter than 10 min; data-plane groups get the round deadline
    kw = {"timeout": datetime.timedelta(seconds=max(timeout_s, 600.0))}
    if device_type == "cuda":
        # one rank per GPU; more ranks than GPUs (single-GPU rehearsal over
        # gloo) wrap around.  device_count() does not initialise HIP.
        local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", local)
    dist.init_process_group(backend=backend, **kw)


def make_dist_transport(num_stages: int, kind: str, device, replicas: int = 1,
                        timeout_s: Optional[float] = None, loop_ring_bytes: int = 256 << 20,
                        warmup: bool = True) -> Transport:
    """`loop_ring_bytes`: devloop channel rings, sized by the engine for the
    largest message an edge carries (LSD_LOOP_RING_MB overrides).
    `warmup=False`: no unagreed per-rank exchange (`open_data_plane` runs the
    agreed self-test instead)."""
    import os

    if kind == "rccl":  # native communicator (csrc/comm.cpp), one per (edge, lane)
        t = RcclTransport(num_stages, replicas, lanes=int(os.environ.get("LSD_LANES", "2")),
                          timeout_s=timeout_s, init_s=float(os.environ.get("LSD_RCCL_INIT_S", "120")))
    elif kind == "nccl":
        t = NcclTransport(num_stages, replicas, timeout_s)
    elif kind == "devloop":  # every rank on one GPU: the 1-GPU rehearsal of "rccl"
        t = IpcLoopTransport(num_stages, replicas, lanes=int(os.environ.get("LSD_LANES", "2")),
                             timeout_s=timeout_s,
                             ring_bytes=int(os.environ.get("LSD_LOOP_RING_MB", "0")) << 20 or loop_ring_bytes,
                             spin_limit_s=float(os.environ.get("LSD_LOOP_SPIN_S", "30")))
    elif kind == "gloo":
        t = GlooTransport(num_stages, replicas, timeout_s)  # host-staged, same edge-by-edge bring-up
    else:
        raise ValueError(f"unknown transport {kind!r}")
    if warmup or kind == "nccl":
        # torch's groups create their p2p communicators lazily: the warmup's
        # ordered exchange is what creates them without a cross-edge deadlock
        t.warmup(device)
    return t


# ---------------------------------------------------------------------------
# Data-plane selection: self-test + agreed in-process fallback
# ---------------------------------------------------------------------------

def transport_chain(spec: str, device_type: str, shared_gpu: bool = False) -> List[str]:
    """Data planes to try, in order.  "auto": on GPUs the native RCCL
    communicators with graph-captured edges (the path the one-GPU devloop
    rehearsal exercises: `exec_items`, captured send / recv), falling back to
    torch's RCCL process groups (eager p2p from the Python item loop); rank
    processes sharing ONE GPU (RCCL refuses two ranks on a device) use the
    device loopback channels, falling back to host-staged gloo; on CPU gloo.
    An explicit "a,b" lists the chain itself."""
    if spec in ("", "auto", "local"):
        if device_type != "cuda":
            return ["gloo"]
        return ["devloop", "gloo"] if shared_gpu else ["rccl", "nccl"]
    return [k.strip() for k in spec.split(",") if k.strip()]


def _bounded(fn, timeout_s: float, what: str):
    """(result, None) of fn() run on a daemon thread, or (None, error) when
    it raised or had not returned after `timeout_s` (a blocking communicator
    init whose peer never arrives: the thread is left behind, the caller
    moves on)."""
    box: list = []

    def run():
        try:
            box.append((fn(), None))
        except Exception as e:  # noqa: BLE001
            box.append((None, f"{what}: {type(e).__name__}: {e}"))

    th = threading.Thread(target=run, daemon=True, name="lsd-bounded")
    th.start()
    th.join(timeout_s)
    if not box:
        return None, f"{what}: no result after {timeout_s:.0f} s"
    return box[0]


def _drained(device, deadline: float) -> bool:
    """Wait (bounded) for the work enqueued so far on the current stream."""
    if device.type != "cuda":
        return True
    ev = torch.cuda.Event()
    ev.record()
    while not ev.query():
        if time.monotonic() > deadline:
            return False
        time.sleep(200e-6)
    return True


def _pattern(n: int, tag: float, device) -> torch.Tensor:
    return torch.arange(n, dtype=torch.float32, device=device).mul_(1e-3).add_(tag)


def _edge_list(t) -> List[tuple]:
    """This replica's edges in the global bring-up order: fwd 0..P-2, ret."""
    P = t.P
    out = [("fwd", i, i + 1) for i in range(P - 1)]
    if P > 1:
        out.append(("ret", P - 1, 0))
    return out


def _captured_exchange(t, device, kind, src, dst, lane, tag, deadline) -> Optional[str]:
    """One send / receive captured into a hipGraph on each end, replayed
    twice with fresh data: the decode graphs' edge I/O in miniature."""
    from .pipeline import GPU_GATE

    n = 4096
    buf = torch.zeros(n, dtype=torch.float32, device=device)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(device)
    s.wait_stream(torch.cuda.current_stream(device))
    begin = getattr(t, "begin_capture", None)
    io = (0, [])
    with GPU_GATE.exclusive(), torch.cuda.stream(s):
        if begin is not None:
            begin()
        g.capture_begin(capture_error_mode="thread_local")
        try:
            if t.rank == src:
                t.capture_send(buf, dst, kind, lane)
            else:
                t.capture_recv(buf, src, kind, lane)
        finally:
            g.capture_end()
            if begin is not None:
                io = t.end_capture()
    torch.cuda.current_stream(device).wait_stream(s)
    for k in (1, 2):
        want = _pattern(n, tag + 100.0 * k, device)
        if t.rank == src:
            buf.copy_(want)
        if io[0]:
            t.replay(g, io[0], io[1])
        else:
            with t.issuing():
                g.replay()
        if not _drained(device, deadline):
            return f"captured {kind} {src}->{dst} lane {lane}, replay {k}: not complete by the deadline"
        if t.rank == dst and not torch.equal(buf, want):
            return f"captured {kind} {src}->{dst} lane {lane}, replay {k}: wrong data"
    return None


def selftest_data_plane(t: "_DistTransport", device, deadline_s: float = 60.0) -> Optional[str]:
    """This rank's part of the data-plane self-test, bounded by `deadline_s`:
    on every (edge, lane) it belongs to, in the global order, one eager
    exchange of a small and of a 1 MiB message and -- on transports whose
    decode graphs carry their own transfers -- one exchange captured in a
    hipGraph on both ends and replayed twice; the receiver checks every byte.
    Returns None or this rank's error (the caller agrees on the outcome)."""
    deadline = time.monotonic() + deadline_s
    capture = device.type == "cuda" and getattr(t, "GRAPH_IO", False)
    lanes = getattr(t, "L", 1)
    try:
        for ei, (kind, src, dst) in enumerate(_edge_list(t)):
            if t.rank not in (src, dst):
                continue
            for lane in range(lanes):
                tag = 1000.0 * (ei + 1) + 10.0 * lane
                for n in (1024, 1 << 18):
                    x = _pattern(n, tag, device)
                    if t.rank == src:
                        t.send(x, dst, kind, lane).wait()
                    else:
                        got = torch.zeros_like(x)
                        t.irecv(got, src, kind, lane).wait()
                    if not _drained(device, deadline):
                        return (f"rank {t.grank}: eager {kind} {src}->{dst} lane {lane} ({4 * n} B) "
                                f"not complete after {deadline_s:.0f} s")
                    if t.rank == dst and not torch.equal(got, x):
                        return f"rank {t.grank}: eager {kind} {src}->{dst} lane {lane} ({4 * n} B): wrong data"
                if capture:
                    err = _captured_exchange(t, device, kind, src, dst, lane, tag, deadline)
                    if err:
                        return f"rank {t.grank}: {err}"
    except Exception as e:  # noqa: BLE001
        return f"rank {t.grank}: {type(e).__name__}: {e}"
    return None


def _teardown_failed(t, device, drain_s: float = 30.0) -> None:
    """After a failed self-test: abort the data plane (kernels waiting on a
    peer return) and let this rank's stream drain before the next transport
    is brought up."""
    try:
        t.abort()
    except Exception:  # noqa: BLE001
        pass
    if not _drained(device, time.monotonic() + drain_s):
        raise TransportError("a failed data plane did not drain after its abort; cannot fall back")


def open_data_plane(chain: List[str], num_stages: int, device, replicas: int = 1,
                    timeout_s: Optional[float] = None, loop_ring_bytes: int = 256 << 20):
    """Bring up the first transport of `chain` that passes the self-test on
    EVERY rank: (transport, kind, fallback reason or None).  Each candidate's
    bring-up and self-test outcome is agreed over the gloo control group, so
    all ranks fall back together, in process (no re-exec).  The last
    candidate's failure is raised.  Test hook: LSD_TEST_HOOKS=1 with
    LSD_TEST_SELFTEST_FAIL=<global rank> fails that rank's self-test of the
    first candidate."""
    import os

    reasons: List[str] = []
    for i, kind in enumerate(chain):
        last = i == len(chain) - 1
        try:
            t = make_dist_transport(num_stages, kind, device, replicas, timeout_s, loop_ring_bytes,
                                    warmup=False)
        except TransportError as e:  # agreed: raised on every rank
            if last:
                raise
            reasons.append(f"{kind}: {e}")
            continue
        err = selftest_data_plane(t, device, float(os.environ.get("LSD_SELFTEST_S", "60")))
        if (i == 0 and err is None and os.environ.get("LSD_TEST_HOOKS") == "1"
                and os.environ.get("LSD_TEST_SELFTEST_FAIL") == str(t.grank)):
            err = f"rank {t.grank}: injected self-test failure (LSD_TEST_SELFTEST_FAIL)"
        try:
            t.agree(err, f"{kind} self-test")
        except TransportError as e:
            _teardown_failed(t, device)
            if last:
                raise
            reasons.append(f"{kind}: {e}")
            continue
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        t.barrier()
        return t, kind, ("; ".join(reasons) or None)
    raise TransportError("empty transport chain")
