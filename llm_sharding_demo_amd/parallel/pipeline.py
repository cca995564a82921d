"""Pipeline-parallel stage worker (one per stage / per MI355X).

Replaces the reference's coordinator loop (`server.py:169-206`), which for
every output token runs shard A, relays its hidden state through the
coordinator to shard B, ships all-position logits back and samples on the
host -- strictly sequentially, so one shard is always idle and each token
costs two HTTP round trips.

Here every stage executes the same sequence of `StepPlan`s (runtime/plan.py,
decided by stage 0's scheduler).  A step has one *item* per busy microbatch
group g; the item of group g on stage r does, in order:

    stage 0     receive the token-return vector of g's previous item (from
                stage P-1), rebuild the decode input rows if the group's
                composition changed (rows joined / left)
    all         prefill the joining sequences' prompt chunks (eager)
                decode the group's rows: one hipGraph replay per
                (group, bucket rows, context bucket) -- captured once, cached
                on the worker, replayed across steps and requests
    stage<P-1   send the boundary hidden states to stage r+1 (prefill, decode)
    stage P-1   sample (decode rows + final prefill chunks) and send the token
                ids back to stage 0

With M >= P groups every stage is busy in steady state (stage r works on
group (t - r) mod M at tick t).  Receives of the next item are posted before
the current item's compute when they target different buffers, so the
transfer overlaps compute; `Handle.wait()` only orders the compute stream
behind the comm stream.  Group g runs on HIP stream lanes[g % L], so
independent groups overlap on the GPU.
"""
from __future__ import annotations

import contextlib
import gc
import itertools
import os
import threading
import time
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from ..models.stage import StageModel
from ..runtime.batch import BatchMeta, MixedMeta, SamplingState
from ..runtime.plan import GroupPlan, StepPlan
from ..utils.tracing import trace_range
from ..utils import racecheck
from .comm import Handle, SendHandle, Transport

class _CaptureGate(racecheck.Shared):
    """Stage threads sharing one GPU (local mode) issue work concurrently, but
    HIP rejects a stream capture that overlaps another thread's stream
    operations (hipErrorStreamCaptureIsolation) or a replay during a capture.
    Every GPU-issuing section holds the gate shared; a capture holds it
    exclusively.  Blocking transport waits happen outside the gate, so a
    stage waiting for its input never holds up a capture.  One thread per
    process (dist, P = 1): always uncontended."""

    def __init__(self):
        self._cv = racecheck.Condition(name="capture_gate")
        self._readers = 0
        self._writer = False
        self._waiting = 0
        self._tls = threading.local()  # this thread's shared-hold depth

    def _depth(self) -> int:
        return getattr(self._tls, "depth", 0)

    def _acquire_shared(self) -> None:
        with self._cv:
            while self._writer or self._waiting:
                self._cv.wait()
            self._readers += 1

    def _release_shared(self) -> None:
        with self._cv:
            self._readers -= 1
            if self._readers == 0:
                self._cv.notify_all()

    @contextlib.contextmanager
    def shared(self):
        """Shared hold; re-entrant per thread (a nested hold never waits, so
        a thread inside a GPU section cannot block behind a waiting capture
        that waits for it)."""
        d = self._depth()
        if d == 0:
            self._acquire_shared()
        self._tls.depth = d + 1
        try:
            yield
        finally:
            self._tls.depth = d
            if d == 0:
                self._release_shared()

    @contextlib.contextmanager
    def released(self):
        """Drop this thread's shared hold (if any) around a blocking wait --
        a transport handshake, an exclusive capture -- and take it back
        after."""
        d = self._depth()
        if d == 0:
            yield
            return
        self._tls.depth = 0
        self._release_shared()
        try:
            yield
        finally:
            self._acquire_shared()
            self._tls.depth = d

    @contextlib.contextmanager
    def exclusive(self):
        with self._cv:
            self._waiting += 1
            while self._writer or self._readers:
                self._cv.wait()
            self._waiting -= 1
            self._writer = True
        try:
            yield
        finally:
            with self._cv:
                self._writer = False
                self._cv.notify_all()


GPU_GATE = _CaptureGate()


def wait_event(ev) -> None:
    """Block until `ev` completed without holding GPU_GATE across the wait:
    each query holds the gate (HIP refuses event queries during a sibling
    thread's capture), the sleeps between them do not, so a sibling's
    capture -- and, behind the writer-preferring gate, every other stage's
    issue -- never waits for this thread's GPU wait."""
    pause = 20e-6
    while True:
        with GPU_GATE.shared():
            if ev.query():
                return
        time.sleep(pause)
        pause = min(2 * pause, 200e-6)


def prefill_chunks(lens: List[int], chunk: int) -> List[Tuple[List[int], List[int]]]:
    """(starts, qlens) per prefill chunk for prompts of `lens` tokens, aligned
    to the END of each prompt: the last chunk holds every sequence's final
    position; earlier chunks of a shorter prompt may be empty."""
    top = max(lens)
    if chunk <= 0 or chunk >= top:
        return [([0] * len(lens), list(lens))]
    C = -(-top // chunk)
    out = []
    for c in range(C):
        back_hi, back_lo = (C - c - 1) * chunk, (C - c) * chunk  # distance from the end
        starts = [max(0, n - back_lo) for n in lens]
        ends = [max(0, n - back_hi) for n in lens]
        out.append((starts, [e - s for s, e in zip(starts, ends)]))
    return out


class SamplingView:
    """Sampler parameters of a decode bucket: views of the group's persistent
    per-row tensors (graph-capturable); pad rows never advance."""

    def __init__(self, temperature, top_k, greedy, seeds, step, active):
        self.temperature, self.top_k, self.greedy = temperature, top_k, greedy
        self.seeds, self.step, self.active = seeds, step, active
        self.num_rows = temperature.shape[0]

    def uniforms(self) -> torch.Tensor:
        from ..runtime.batch import counter_uniform

        return counter_uniform(self.seeds, self.step)

    def advance(self) -> None:
        self.step.add_(self.active.to(self.step.dtype))


class GroupState(racecheck.Shared):
    """Persistent per-(stage, group) device state: decode row metadata,
    sampler state, input / output buffers and the group's captured graphs."""

    def __init__(self, w: "StageWorker", g: int, cap: int):
        dev, H = w.device, w.H
        i32 = dict(dtype=torch.int32, device=dev)
        self.g, self.cap = g, cap
        self.slots = torch.full((cap,), w.scratch_slot, **i32)
        self.pos = torch.zeros(cap, **i32)
        self.active = torch.zeros(cap, **i32)
        self.cu = torch.arange(cap + 1, **i32)
        if w.last:
            self.temp = torch.ones(cap, dtype=torch.float32, device=dev)
            self.topk = torch.ones(cap, **i32)
            self.greedy = torch.ones(cap, **i32)
            self.seeds = torch.zeros(cap, dtype=torch.int64, device=dev)
            self.sstep = torch.zeros(cap, dtype=torch.int64, device=dev)
            self.tokret = torch.zeros(cap, **i32)  # [decode rows | final prefill chunks]
        if w.first:
            # decode input ids; with P > 1 also the token-return receive buffer
            self.tin = self.tokret if w.P == 1 else torch.zeros(cap, **i32)
        else:
            self.hd = torch.empty(cap, H, dtype=torch.float32, device=dev)  # decode hidden in/out
        self.hp: Optional[torch.Tensor] = None  # prefill hidden receive buffer (grown)
        self.graphs: Dict[tuple, tuple] = {}
        # loopback graph I/O: key -> (native I/O-list handle, [(chan, dir, bytes)])
        self.graph_io: Dict[tuple, tuple] = {}
        self.seen: set = set()
        # prefill chunks of a recurring shape: (qlens, variant, input buffer)
        # -> (graph, packed index buffer, static meta, output); see _prefill_graph
        self.pf_graphs: Dict[tuple, tuple] = {}
        self.pf_seen: set = set()
        self.pf_pin: List[list] = []  # [pinned int32 staging, event of its last copy] ring
        self.pf_pin_next = 0
        self._metas: Dict[tuple, BatchMeta] = {}
        # composition changes on a GPU (StageWorker._rows_pack): pinned packed
        # row-state ring [pinned int32, event of its last copy, used], the
        # device copy and the apply_rows argument record
        self.rows_pin: List[list] = []
        self.rows_pin_next = 0
        self.rows_dev: Optional[torch.Tensor] = None
        self.rows_args: Optional[torch.Tensor] = None

    def wire_buf(self, w: "StageWorker", b: int) -> Optional[torch.Tensor]:
        """Persistent wire-dtype staging rows of the decode receive (graph I/O)."""
        if w.wire is None or w.first:
            return None
        if getattr(self, "_wire", None) is None:
            self._wire = torch.empty(self.cap, w.H, dtype=w.wire, device=w.device)
        return self._wire[:b]

    def ensure_tokret(self, w: "StageWorker", n: int) -> None:
        """Grow the token-return vector to >= n entries (prefill finals ride
        behind the decode rows).  Growing drops the captured graphs that
        write into it (rare: only when a step finishes more prompts than any
        step before)."""
        buf = self.tokret if w.last else self.tin
        if buf.numel() >= n:
            return
        new = torch.zeros(max(n, 2 * buf.numel()), dtype=torch.int32, device=buf.device)
        new[: buf.numel()].copy_(buf)
        if w.last:
            self.tokret = new
        if w.first:
            self.tin = new
        self.drop_graphs(w)

    def drop_graphs(self, w: "StageWorker") -> None:
        free = getattr(w.t, "C", None)
        for io, _ in self.graph_io.values():
            if io and free is not None:
                free.loop_io_free(io)
        self.graph_io.clear()
        self.graphs.clear()
        self.seen.clear()
        self.pf_graphs.clear()
        self.pf_seen.clear()

    def meta(self, b: int, ctxb: int) -> BatchMeta:
        key = (b, ctxb)
        m = self._metas.get(key)
        if m is None:
            m = BatchMeta(token_slots=self.slots[:b], token_pos=self.pos[:b],
                          seq_slots=self.slots[:b], q_start=self.pos[:b], cu_q=self.cu[: b + 1],
                          last_idx=self.cu[:b], num_tokens=b, num_seqs=b, max_q=1,
                          max_ctx=ctxb, is_decode=True, host_qlens=[1] * b,
                          active=self.active[:b])
            self._metas[key] = m
        return m

    def samp(self, b: int) -> SamplingView:
        return SamplingView(self.temp[:b], self.topk[:b], self.greedy[:b], self.seeds[:b],
                            self.sstep[:b], self.active[:b])


class StepStats:
    """Per-stage busy / bubble accounting over timed steps (hipEvents on the
    GPU, host clocks on CPU)."""

    def __init__(self, dev: torch.device):
        self.dev = dev
        self.marks: List[tuple] = []
        self.t0_ev = None
        self.t_start = time.perf_counter()
        if dev.type == "cuda":
            self.t0_ev = torch.cuda.Event(enable_timing=True)
            self.t0_ev.record()

    def mark(self):
        if self.dev.type == "cuda":
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            return ev
        return time.perf_counter()

    def summary(self, stage: int) -> dict:
        if self.dev.type == "cuda":
            t1 = torch.cuda.Event(enable_timing=True)
            t1.record()
            t1.synchronize()
            iv = sorted((self.t0_ev.elapsed_time(a), self.t0_ev.elapsed_time(b)) for a, b in self.marks)
            wall = self.t0_ev.elapsed_time(t1)
        else:
            iv = sorted(((a - self.t_start) * 1e3, (b - self.t_start) * 1e3) for a, b in self.marks)
            wall = (time.perf_counter() - self.t_start) * 1e3
        busy, cur = 0.0, None
        for a, b in iv:
            if cur is None or a > cur[1]:
                if cur is not None:
                    busy += cur[1] - cur[0]
                cur = [a, b]
            else:
                cur[1] = max(cur[1], b)
        if cur is not None:
            busy += cur[1] - cur[0]
        return {"stage": stage, "wall_ms": round(wall, 3), "busy_ms": round(busy, 3),
                "busy_fraction": round(busy / wall, 4) if wall > 0 else 0.0, "items": len(iv)}


class StageWorker(racecheck.Shared):
    def __init__(self, stage: StageModel, transport: Optional[Transport], stage_idx: int,
                 num_stages: int, scratch_slot: int = 0, compat_slot: int = 0,
                 wire: Optional[torch.dtype] = None):
        self.stage = stage
        # hidden states on the forward edge in this dtype (None: as computed,
        # fp32); converted right before the send / right after the receive
        self.wire = wire
        self.t = transport
        self.r = stage_idx
        self.P = num_stages
        self.device = stage.device
        self.first = stage_idx == 0
        self.last = stage_idx == num_stages - 1
        self.H = stage.cfg.hidden
        self.scratch_slot, self.compat_slot = scratch_slot, compat_slot
        self.use_graphs = True
        # Group "lanes": group g of this stage runs on lanes[g % L], so
        # independent groups overlap on the GPU -- one's latency-bound
        # phases (small GEMMs, split-K tails) run beside another's bandwidth-
        # bound ones (attention over the KV cache).  Each lane has its own
        # split-K ticket counters in the backend.
        n_lanes = int(os.environ.get("LSD_LANES", "2"))
        # lane index of a group, also on CPU (no streams there): transports
        # keep one channel per (edge, lane), as the RCCL communicators do
        self.n_lanes = max(1, n_lanes)
        self.lanes = ([torch.cuda.Stream(self.device) for _ in range(n_lanes)]
                      if self.device.type == "cuda" else [])
        # LSD_LANE_CU_MASK: give each lane its own share of the CUs (spatial
        # partition) instead of letting the lanes' kernels interleave on all
        # of them -- "split" (contiguous halves of the mask numbering) or
        # "interleave" (every n_lanes-th CU)
        cu_mode = os.environ.get("LSD_LANE_CU_MASK", "")
        if cu_mode and self.lanes and n_lanes > 1:
            self.lanes = _cu_masked_lanes(self.device, n_lanes, cu_mode)
        self.groups: Dict[int, GroupState] = {}
        self.cap = 1
        self.send_pending: Dict[int, List[SendHandle]] = {}
        self.recv: Dict[tuple, List[Handle]] = {}
        self.captures = 0          # hipGraph captures so far (cache effectiveness)
        self.pf_replays = 0        # prefill chunk items replayed from a graph (_prefill_graph)
        self.stats: Optional[StepStats] = None
        self.last_stats: Optional[dict] = None
        self.step_events: List[tuple] = []   # stage 0: (step, event) at each step start
        self.readout = None        # stage 0: callable(step, plan, ret_tensor) for token readout
        # stage 0, native executor: callable(plan, gp, pinned host ids, event, release)
        self.readout_native = None
        # Decode graphs that contain their own edge receive and send (native
        # RCCL transport, parallel/comm.py RcclTransport, or its single-GPU
        # rehearsal DeviceLoopTransport): a decode item is then ONE graph
        # launch per stage.  Items carrying prefill chunks keep eager
        # transfers (their sizes vary), as does stage 0's token-return
        # receive (the host reads it back and may re-gather the rows).  On
        # CPU, StrictLocalTransport runs the same code path with the graph
        # body executed eagerly (protocol tests).
        self.graph_io = bool(transport is not None and getattr(transport, "GRAPH_IO", False)
                             and (self.device.type == "cuda" or getattr(transport, "SIM_GRAPH_IO", False))
                             and os.environ.get("LSD_GRAPH_IO", "1") != "0")
        # Native stage executor (csrc/stage_exec.cpp): a step made only of
        # steady-state decode items is enqueued by one C++ call (see
        # _native_step).  Needs lanes and either one stage or graph I/O.
        self.native_exec = (self.device.type == "cuda" and bool(self.lanes)
                            and os.environ.get("LSD_NATIVE_EXEC", "1") != "0"
                            and (num_stages == 1 or self.graph_io))
        self._ev_free: List[torch.cuda.Event] = []   # readout completion events
        self._tev_free: List[torch.cuda.Event] = []  # busy-timing events
        self._tev_used: List[torch.cuda.Event] = []
        self.native_steps = 0
        self.native_changes = 0  # composition-change items issued by exec_items
        self.mixed_items = 0     # decode + prefill items run as one forward (_mixed)
        self.io_items = 0  # decode items whose (graph) body carried its own transfers

    # ------------------------------------------------------------------
    def configure(self, groups: int, cap: int) -> None:
        """(Re)create the persistent group states (engine idle only)."""
        self.sync()
        self.cap = cap
        self.groups = {g: GroupState(self, g, cap) for g in range(groups)}
        self.send_pending.clear()
        self.recv.clear()

    def lane_of(self, g: int) -> int:
        return g % self.n_lanes

    def _io(self, gp: GroupPlan) -> bool:
        """Does this item's decode graph carry its own receive / send?"""
        return (self.graph_io and self.use_graphs and gp.kind != "fwd_b" and gp.b > 0
                and not gp.chunks and self.P > 1)

    def on_lane(self, g: int):
        if not self.lanes:
            return contextlib.nullcontext()
        return torch.cuda.stream(self.lanes[g % len(self.lanes)])

    def sync(self) -> None:
        if self.device.type == "cuda":
            for h in (h for hs in self.send_pending.values() for h in hs):
                h.wait()
            self.send_pending.clear()
            for lane in self.lanes:
                lane.synchronize()

    # ------------------------------------------------------------------
    # timing
    def start_stats(self) -> None:
        self.stats = StepStats(self.device)
        self._tev_free.extend(self._tev_used)
        self._tev_used.clear()

    def end_stats(self) -> Optional[dict]:
        if self.stats is None:
            return None
        self.last_stats = self.stats.summary(self.r)
        self.stats = None
        return self.last_stats

    # ------------------------------------------------------------------
    def begin_session(self) -> None:
        """Order the lanes behind the caller's stream once per session.  Steps
        inside a session add no cross-stream hops: group g always runs on
        lanes[g % L], so its items are ordered by the lane itself (a per-step
        lane <-> stream event round trip costs ~0.2 ms of GPU idle)."""
        # the calling (stage) thread owns this worker and its groups from here on:
        # the hand-over from the constructing thread is ordered by the plan channel,
        # which the lockset checker (utils/racecheck.py) cannot see
        racecheck.handoff(self)
        for gs in (getattr(self, "groups", None) or {}).values():
            racecheck.handoff(gs)
        if not self.lanes:
            return
        with self._gpu():
            cur = torch.cuda.current_stream(self.device)
            for lane in self.lanes:
                lane.wait_stream(cur)

    def end_session(self) -> None:
        if not self.lanes:
            return
        with self._gpu():
            cur = torch.cuda.current_stream(self.device)
            for lane in self.lanes:
                cur.wait_stream(lane)

    def run_step(self, plan: StepPlan, nxt: Optional[StepPlan] = None) -> None:
        """Execute this stage's part of one step (between begin_session and
        end_session).  `nxt` (the following step's plan, when already known)
        lets the last item post the next step's first receive ahead of its
        compute."""
        items = self._items(plan)
        following = self._items(nxt)
        L = max(1, len(self.lanes))
        self.stage.backend.concurrency = max(1, min(L, sum(1 for gp in items if gp.has_work)))
        if self.first and plan.timing and self.device.type == "cuda":
            with self._gpu(), self.on_lane(0):
                ev = torch.cuda.Event(enable_timing=True)
                ev.record()
            self.step_events.append((plan.step, ev))
        if self.native_exec:
            if items and self._native_step(plan, items):
                return
            if self.P == 1 and self.PARTIAL_NATIVE and len(items) > 1:
                # one stage: the steady decode items of a step whose other
                # items join sequences go out natively one by one (in the
                # decode-first order), the rest through the item loop below
                rest = []
                for gp in items:
                    if gp.chunks or not self._native_step(plan, [gp]):
                        rest.append(gp)
                items = rest
                if not items:
                    return
            # the native path posts every receive in stream order itself: no
            # look-ahead posting of the next step's first receive
            following = []
        items = self._merged_prefill(plan, items)
        if self.P == 1 and self.DECODE_FIRST and len(items) > 1:
            # one stage: items without prefill chunks first, so every lane's
            # decode replay is queued before the eager prefill of a joining
            # group holds the issuing thread (the groups are independent)
            items = sorted(items, key=lambda gp: bool(gp.chunks))
        if items:
            self._post(items[0])
        for i, gp in enumerate(items):
            nx = items[i + 1] if i + 1 < len(items) else (following[0] if following else None)
            with self.on_lane(gp.g), trace_range(f"stage{self.r}/step{plan.step}/g{gp.g}"):
                self._item(plan, gp, nx)

    # One stage: the prefill-only items of a step (groups that only join
    # sequences this step: no decode rows, no readout of earlier rows) run as
    # ONE forward over all their chunks on the first such item's lane -- GEMMs
    # of those groups' rows together instead of one per group on concurrent
    # lanes; each group's sampled first tokens go to its own token-return
    # vector and the other lanes wait for the work.  Items with decode rows
    # run as usual after it.  GPT-2 XL headline (every group joins at the
    # session start): prefill 209-210 -> 198 ms, GPT-2 small 21.2 -> 18.8 ms
    # (profiles/r5_merge_prefill.log); LSD_MERGE_PREFILL=0 keeps one item per group.
    MERGE_PREFILL = os.environ.get("LSD_MERGE_PREFILL", "1") == "1"
    DECODE_FIRST = os.environ.get("LSD_DECODE_FIRST", "1") == "1"
    PARTIAL_NATIVE = os.environ.get("LSD_PARTIAL_NATIVE", "1") == "1"

    def _merged_prefill(self, plan: StepPlan, items: List[GroupPlan]) -> List[GroupPlan]:
        """Run the step's prefill-only items merged (>= 2 of them, one stage);
        returns the items still to run."""
        if not (getattr(self, "merge_prefill", self.MERGE_PREFILL) and self.P == 1 and len(items) > 1
                and self.device.type == "cuda"):
            return items
        pure = [gp for gp in items if gp.kind != "fwd_b" and gp.chunks and gp.b == 0 and gp.rows is None
                and gp.ret == 0]
        if len(pure) < 2:
            return items
        rest = [gp for gp in items if not any(gp is q for q in pure)]
        items = pure
        import types

        g0 = items[0].g
        merged = types.SimpleNamespace(chunks=[c for gp in items for c in gp.chunks], g=g0)
        with self.on_lane(g0), trace_range(f"stage{self.r}/step{plan.step}/merged-prefill"), self._gpu():
            self.stage.backend.lane = self.lane_of(g0)
            mark = self.stats.mark() if (self.stats is not None and plan.timing) else None
            ids = self._prefill(merged, self.groups[g0], None)
            off = 0
            for gp in items:
                J = gp.n_final
                if J:
                    gs = self.groups[gp.g]
                    gs.ensure_tokret(self, J)
                    gs.tokret[:J].copy_(ids[off: off + J])
                    off += J
            if mark is not None:
                self.stats.marks.append((mark, self.stats.mark()))
            ev = torch.cuda.Event()
            ev.record()
        for lane in {self.lane_of(gp.g) for gp in items} - {self.lane_of(g0)}:
            self.lanes[lane].wait_event(ev)
        return rest

    def _new_event(self, timing: bool) -> torch.cuda.Event:
        """A created (recorded once) event whose raw handle C++ can record
        (call inside the gate: the first record is a stream operation)."""
        pool = self._tev_free if timing else self._ev_free
        if pool:
            return pool.pop()
        ev = torch.cuda.Event(enable_timing=timing)
        ev.record(self.lanes[0])
        return ev

    def _pinned(self, gs: GroupState, n: int) -> torch.Tensor:
        """Pinned host buffer for one token readout of group gs: a ring per
        group (a slot is reused only after `lag` more readouts of the group,
        long after the scheduler applied it -- Engine._drive blocks on
        readouts older than P + 2 steps)."""
        ring = getattr(gs, "_pin_ring", None)
        if ring is None or ring.shape[1] < n:
            ring = torch.empty(self._PIN_SLOTS, max(n, gs.cap), dtype=torch.int32, pin_memory=True)
            gs._pin_ring, gs._pin_next = ring, 0
        k = gs._pin_next
        gs._pin_next = (k + 1) % self._PIN_SLOTS
        return ring[k, :n]

    _PIN_SLOTS = 64
    # composition-change items (joins activating, leaves) on the native
    # executor; LSD_NATIVE_CHANGES=0 sends them to the Python item loop (A/B,
    # tools/serve_load.py)
    NATIVE_CHANGES = os.environ.get("LSD_NATIVE_CHANGES", "1") == "1"

    def _native_step(self, plan: StepPlan, items: List[GroupPlan]) -> bool:
        """Enqueue this step with one C++ call (csrc/stage_exec.cpp exec_items)
        when every item is a steady-state decode item: a captured graph for
        its (rows, context) bucket, no composition change, no prefill chunk,
        no eager transfer (one stage, or graph I/O).  False = take the
        Python item loop (nothing was issued)."""
        if self.recv or any(self.send_pending.values()):
            return False
        descs = []
        for gp in items:
            if gp.kind == "fwd_b" or gp.chunks or gp.b <= 0 or gp.n_final:
                return False
            if gp.rows is not None and (not self.NATIVE_CHANGES or not hasattr(self.stage.backend, "C")
                                        or gp.n > gp.b):
                return False
            io = self._io(gp)
            if self.P > 1 and not io:
                return False
            gs = self.groups[gp.g]
            key = (gp.b, gp.ctxb, io)
            ent = gs.graphs.get(key)
            if ent is None:
                return False
            ret = gp.ret if self.first else 0
            if ret and (gs.tin.numel() < ret or (self.readout is not None and self.readout_native is None)):
                return False
            descs.append((gp, gs, ent[0], ret, gs.graph_io.get(key)))
        if getattr(self.t, "aborted", False):
            from .comm import TransportError

            raise TransportError("data plane aborted: step not issued")
        timing = plan.timing and self.stats is not None
        C = self.stage.backend.C
        nf = C.exec_fields()
        # loopback channels: the step's whole op sequence passes the enqueue
        # handshake here, outside the gate; exec_items' own checks are then
        # instant (csrc/loop_fabric.cpp)
        pre: List[tuple] = []
        rows, reads, packed = [], [], []
        recv_kind = []
        for gp, gs, g, ret, gio in descs:
            rk = None
            if ret and self.P > 1:  # token-return receive from the last stage
                rk = self.t.native_recv("ret", self.P - 1, self.lane_of(gp.g))
                if rk[0] == "loop":
                    pre.append((rk[1], 1, 4 * ret))
            if gio is not None:
                pre.extend(gio[1])
            recv_kind.append(rk)
        if pre:
            self.t.prewait(pre)
        with self._gpu():
            for (gp, gs, g, ret, gio), rk in zip(descs, recv_kind):
                lane = self.lanes[self.lane_of(gp.g)]
                d = [0] * nf
                d[0] = g.raw_cuda_graph_exec()
                d[1] = lane.cuda_stream
                if rk is not None:
                    if rk[0] == "rccl":
                        d[2], d[5] = rk[1], rk[2]
                    else:
                        d[12] = rk[1]
                    d[3], d[4] = gs.tin.data_ptr(), 4 * ret
                if gio is not None:
                    d[13] = gio[0]
                if timing:
                    t0, t1 = self._new_event(True), self._new_event(True)
                    self._tev_used += (t0, t1)
                    self.stats.marks.append((t0, t1))
                    d[6], d[11] = t0.cuda_event, t1.cuda_event
                if ret and self.readout is not None:
                    host = self._pinned(gs, ret)
                    ev = self._new_event(False)
                    d[7], d[8], d[9], d[10] = gs.tin.data_ptr(), host.data_ptr(), 4 * ret, ev.cuda_event
                    reads.append((gp, host, ev))
                if gp.rows is not None:
                    # composition change: packed row state copied and applied
                    # after the readout, ahead of the graph (csrc/stage_exec.cpp)
                    slot, args = self._rows_pack(gs, gp.rows, gp.b)
                    d[14], d[15], d[16], d[17] = args.data_ptr(), slot[0].data_ptr(), 4 * (10 * gs.cap + 1), gp.b
                    packed.append((slot, lane))
                    self.native_changes += 1
                rows.append(d)
            try:
                with (self.t.issuing() if self.t is not None else contextlib.nullcontext()):
                    C.exec_items(rows)
            except RuntimeError:
                # copies of the items already enqueued may still target the
                # pinned buffers: let them land before the buffers can be reused
                for lane in self.lanes:
                    lane.synchronize()
                raise
            for slot, lane in packed:
                slot[1].record(lane)
                slot[2] = True
        for gp, host, ev in reads:
            self.readout_native(plan, gp, host, ev, self._ev_free.append)
        self.native_steps += 1
        return True

    def _items(self, plan: Optional[StepPlan]) -> List[GroupPlan]:
        if plan is None or plan.end or plan.stop:
            return []
        return [gp for gp in plan.groups if self._touches(gp)]

    def _touches(self, gp: GroupPlan) -> bool:
        if gp.kind == "fwd_b":
            return self.r > 0
        return gp.has_work or (self.first and gp.ret > 0)

    # ------------------------------------------------------------------
    # receives
    def _recv_targets(self, gp: GroupPlan) -> List[Tuple[str, int, torch.Tensor]]:
        """(edge, src stage, buffer) of every receive of item gp, in order."""
        gs = self.groups[gp.g]
        if gp.kind == "fwd_b":
            if self.r == 0:
                return []
            return [("fwd", self.r - 1, self._hp(gs, gp.fwd_rows))]
        if self.first:
            if self.P > 1 and gp.ret > 0:
                gs.ensure_tokret(self, gp.ret)
                return [("ret", self.P - 1, gs.tin[: gp.ret])]
            return []
        out = []
        T = gp.prefill_tokens
        if T > 0:
            out.append(("fwd", self.r - 1, self._hp(gs, T)))
        if gp.b > 0 and not self._io(gp):
            out.append(("fwd", self.r - 1, gs.hd[: gp.b]))
        return out

    def _hp(self, gs: GroupState, T: int) -> torch.Tensor:
        if gs.hp is None or gs.hp.shape[0] < T:
            n = max(T, 2 * gs.hp.shape[0]) if gs.hp is not None else T
            gs.hp = torch.empty(n, self.H, dtype=torch.float32, device=self.device)
        return gs.hp[:T]

    def _post(self, gp: Optional[GroupPlan]) -> None:
        if gp is None or gp.g in {k[0] for k in self.recv}:
            return
        tg = self._recv_targets(gp)
        if not tg:
            return
        with self.on_lane(gp.g):
            # a send of this group's previous item may still read the buffer
            # we are about to receive into (middle stages send their receive
            # buffer: the residual stream is updated in place) -- order the
            # receive behind it (stream-level wait, no host sync)
            for h in self.send_pending.pop(gp.g, []):
                h.wait()
            lane = self.lane_of(gp.g)
            self.recv[(gp.g, id(gp))] = [self._recv(buf, src, edge, lane) for edge, src, buf in tg]

    # wire dtype (C-CODEC): hidden states cross the forward edge as self.wire
    def _recv(self, buf: torch.Tensor, src: int, edge: str, lane: int, stage=None,
              capture: bool = False):
        if self.wire is None or edge != "fwd" or buf.dtype == self.wire:
            return (self.t.capture_recv if capture else self.t.irecv)(buf, src, edge, lane)
        if stage is None:
            stage = torch.empty(buf.shape, dtype=self.wire, device=buf.device)
        if capture:  # inside the graph: receive, then widen in place
            self.t.capture_recv(stage, src, edge, lane)
            buf.copy_(stage)
            return None
        inner = self.t.irecv(stage, src, edge, lane)

        def post():
            inner.wait()
            buf.copy_(stage)
        return Handle(buf, post=post)

    def _send(self, x: torch.Tensor, dst: int, edge: str, lane: int, capture: bool = False):
        if self.wire is not None and edge == "fwd" and x.dtype != self.wire:
            x = x.to(self.wire)
        return (self.t.capture_send if capture else self.t.send)(x, dst, edge, lane)

    def _take_recv(self, gp: GroupPlan) -> List[torch.Tensor]:
        hs = self.recv.pop((gp.g, id(gp)), None)
        if hs is None:
            if self._recv_targets(gp):
                raise RuntimeError(f"stage {self.r}: no receive posted for group {gp.g}")
            return []
        return [h.wait() for h in hs]

    @staticmethod
    def _buffers(tg) -> set:
        return {t[2].untyped_storage().data_ptr() for t in tg}

    # ------------------------------------------------------------------
    def _item(self, plan: StepPlan, gp: GroupPlan, nx: Optional[GroupPlan]) -> None:
        st, gs = self.stage, self.groups[gp.g]
        st.backend.lane = gp.g % max(1, len(self.lanes))
        ins = self._take_recv(gp)
        # post the next item's receives before this compute when they target
        # other buffers (overlap); otherwise after
        early = (nx is not None and nx.g != gp.g
                 and not (self._buffers(self._recv_targets(nx)) & self._buffers(self._recv_targets(gp))))
        if early and self.graph_io and self.lane_of(nx.g) == self.lane_of(gp.g):
            # in-stream transfers: a receive queued on this lane ahead of the
            # current item would hold its compute until the peer's data lands
            early = False
        if early:
            self._post(nx)
        # outputs of this group's previous item must have left before we overwrite them
        for h in self.send_pending.pop(gp.g, []):
            h.wait()
        with self._gpu():
            mark = self.stats.mark() if (self.stats is not None and plan.timing) else None
            if gp.kind == "fwd_b":
                self._fwd_b(gp, ins)
            else:
                self._step_item(plan, gp, gs, ins)
            if mark is not None:
                self.stats.marks.append((mark, self.stats.mark()))
        if not early:
            self._post(nx)

    def _step_item(self, plan: StepPlan, gp: GroupPlan, gs: GroupState, ins) -> None:
        st, be = self.stage, self.stage.backend
        k = 0
        # --- stage 0: the previous item's token-return vector
        if self.first:
            ret = None
            if gp.ret > 0:
                ret = ins[0] if self.P > 1 else gs.tin[: gp.ret]
                k = 1
                if self.readout is not None:
                    self.readout(plan, gp, ret)
        # --- composition change: rewrite the decode rows' state
        if gp.rows is not None:
            self._apply_rows(gp, gs)
        if gp.chunks and gp.b > 0 and self._mixed_ok(gp):
            self._mixed(gp, gs)
            return
        sends: List[torch.Tensor] = []
        finals = None
        # --- prefill chunks of joining sequences (eager)
        if gp.chunks:
            x = self._prefill(gp, gs, ins[k] if not self.first else None)
            if not self.first:
                k += 1
            if self.last:
                finals = x
            elif x is not None:
                sends.append(x)
        # --- decode rows (hipGraph per (bucket, context bucket)); with graph
        # I/O the graph receives its input and sends its output itself
        io = self._io(gp)
        lane = self.lane_of(gp.g)
        if io:
            self.io_items += 1
        if gp.b > 0:
            inp = gs.tin[: gp.b] if self.first else (gs.hd[: gp.b] if io else ins[k])
            out = self._decode(gp, gs, inp, io)
            if not self.last and not io:
                sends.append(out)
        if self.last:
            J = gp.n_final
            nret = gp.b + J
            if J:
                gs.ensure_tokret(self, nret)
                gs.tokret[gp.b: nret].copy_(finals)
            if nret and self.P > 1 and not io:
                self.send_pending.setdefault(gp.g, []).append(self._send(gs.tokret[:nret], 0, "ret", lane))
        else:
            for x in sends:
                self.send_pending.setdefault(gp.g, []).append(self._send(x, self.r + 1, "fwd", lane))

    # Mixed steps (one stage): a group whose step both decodes rows and
    # prefills joining prompts runs ONE eager forward over [decode rows |
    # chunk tokens] (runtime/batch.py MixedMeta) instead of the decode graph
    # plus a second, prefill-only forward -- every weight is read once per
    # step, and the GEMMs see b + T rows.  Continuous serving joins sequences
    # at most steps (tools/serve_load.py); the bench's session shape (every
    # sequence joins at step 0) never mixes.  Opt-in (LSD_MIXED_STEPS=1): the
    # eager mixed forward gives up the decode rows' graph replay, and under
    # the closed-loop serving load it measured slower on GPT-2 XL (34.2-35.5k
    # vs 38.3-38.4k tok/s) and GPT-2 small, +1.4 % on Llama-3 8B
    # (profiles/r6_mixed_steps.log).
    MIXED_STEPS = os.environ.get("LSD_MIXED_STEPS", "0") == "1"

    def _mixed_ok(self, gp: GroupPlan) -> bool:
        return (getattr(self, "mixed_steps", self.MIXED_STEPS) and self.P == 1 and gp.kind == "step"
                and gp.n <= gp.b)

    def _mixed(self, gp: GroupPlan, gs: GroupState) -> None:
        st, be, dev = self.stage, self.stage.backend, self.device
        ch = gp.chunks
        b = gp.b
        pf, ids, _ = self._chunk_meta(gs, ch, tuple(c.qlen for c in ch))
        dec = gs.meta(b, gp.ctxb)
        mm = MixedMeta(token_slots=torch.cat([dec.token_slots, pf.token_slots]),
                       token_pos=torch.cat([dec.token_pos, pf.token_pos]), b=b, dec=dec, pf=pf,
                       num_tokens=b + pf.num_tokens)
        inp = torch.cat([gs.tin[:b], ids])  # a copy: the samplers below overwrite tin (= tokret)
        finals = [i for i, c in enumerate(ch) if c.final]
        J = len(finals)
        rows = torch.arange(b, dtype=torch.int32, device=dev)
        if J:
            fi = torch.tensor(finals, dtype=torch.long, device=dev)
            rows = torch.cat([rows, pf.last_idx.index_select(0, fi) + b])
        logits = st.forward(mm, inp, head=True, head_rows=rows, variant=gp.g & 1)
        gs.ensure_tokret(self, b + J)
        V = st.cfg.vocab_size
        seg = getattr(logits, "_lsd_segmax", None)
        ld = logits[:b]
        if seg is not None:
            ld._lsd_segmax = seg[:b]
        # decode rows: draw, advance their sampler counters and positions (as the graph does)
        be.sample_into(ld, gs.samp(b), V, gs.tokret[:b], dec)
        if J:
            lf = logits[b:]
            if seg is not None:
                lf._lsd_segmax = seg[b:]
            fc = [ch[i] for i in finals]
            samp = SamplingState([c.temperature for c in fc], [c.top_k for c in fc],
                                 [c.greedy for c in fc], [c.seed for c in fc], dev)
            gs.tokret[b: b + J].copy_(be.sample(lf, samp, V))
        self.mixed_items += 1

    def _apply_rows(self, gp: GroupPlan, gs: GroupState) -> None:
        """New composition: rows [0, n) from the plan, pad rows [n, b) idle on
        the scratch slot.  Stage 0 also gathers the rows' input token ids out
        of the token-return vector (kept rows move, joined rows take their
        prefill sample)."""
        dev, rows = self.device, gp.rows
        n, b = gp.n, max(gp.b, gp.n)
        pad = b - n
        sl = [r.slot for r in rows] + [self.scratch_slot] * pad
        pos = [r.pos for r in rows] + [0] * pad
        act = [1] * n + [0] * pad
        if b == 0:
            return
        if dev.type == "cuda":
            if hasattr(self.stage.backend, "C"):
                slot, args = self._rows_pack(gs, rows, b)
                words = 10 * gs.cap + 1
                gs.rows_dev.copy_(slot[0][:words], non_blocking=True)
                self.stage.backend.C.apply_rows(args, b)
                slot[1].record()
                slot[2] = True
                return
            self._apply_rows_staged(gs, rows, b, pad, sl, pos, act)
            return
        gs.slots[:b].copy_(_h2d(sl, torch.int32, dev), non_blocking=True)
        gs.pos[:b].copy_(_h2d(pos, torch.int32, dev), non_blocking=True)
        gs.active[:b].copy_(_h2d(act, torch.int32, dev), non_blocking=True)
        if self.last:
            gs.temp[:b].copy_(_h2d([r.temperature for r in rows] + [1.0] * pad, torch.float32, dev),
                              non_blocking=True)
            gs.topk[:b].copy_(_h2d([r.top_k for r in rows] + [1] * pad, torch.int32, dev),
                              non_blocking=True)
            gs.greedy[:b].copy_(_h2d([1 if r.greedy else 0 for r in rows] + [1] * pad, torch.int32,
                                     dev), non_blocking=True)
            gs.seeds[:b].copy_(_h2d([r.seed for r in rows] + [0] * pad, torch.int64, dev),
                               non_blocking=True)
            gs.sstep[:b].copy_(_h2d([r.step for r in rows] + [0] * pad, torch.int64, dev),
                               non_blocking=True)
        if self.first:
            src = _h2d([r.src for r in rows] + [0] * pad, torch.int64, dev)
            gathered = gs.tin.index_select(0, src.to(dev, non_blocking=True))
            gs.tin[:b].copy_(gathered)

    _ROWS_PIN = 4  # packed row-state buffers per group: reused 4 composition changes later

    def _rows_pack(self, gs: GroupState, rows, b: int):
        """Composition change on a GPU, host side: the new rows' state packed
        into one pinned int32 buffer in the layout of elementwise.hip
        apply_rows_kernel (fixed offsets by the group capacity, so the device
        copy and the kernel depend on the bucket only), and the kernel's
        argument record.  -> (pinned ring slot, CPU int64[12] record); the
        caller enqueues the copy + kernel (eagerly, or in exec_items) and then
        records the slot's event."""
        cap = gs.cap
        words = 10 * cap + 1
        if len(gs.rows_pin) < self._ROWS_PIN:
            gs.rows_pin.append([torch.empty(words, dtype=torch.int32, pin_memory=True), torch.cuda.Event(), False])
        slot = gs.rows_pin[gs.rows_pin_next % len(gs.rows_pin)]
        gs.rows_pin_next += 1
        if slot[2]:
            slot[1].synchronize()  # its previous copy has long landed
        a = slot[0].numpy()
        n = len(rows)
        a[4 * cap] = n
        if n:
            f0 = 4 * cap + 1
            a[f0: f0 + n] = [r.slot for r in rows]
            a[f0 + cap: f0 + cap + n] = [r.pos for r in rows]
            if self.last:
                a[f0 + 2 * cap: f0 + 2 * cap + n] = np.asarray([r.temperature for r in rows], np.float32).view(np.int32)
                a[f0 + 3 * cap: f0 + 3 * cap + n] = [r.top_k for r in rows]
                a[f0 + 4 * cap: f0 + 4 * cap + n] = [1 if r.greedy else 0 for r in rows]
                a64 = a[: 4 * cap].view(np.int64)
                a64[:n] = [r.seed for r in rows]
                a64[cap: cap + n] = [r.step for r in rows]
            if self.first:
                a[f0 + 5 * cap: f0 + 5 * cap + n] = [r.src for r in rows]
        if gs.rows_dev is None:
            gs.rows_dev = torch.empty(words, dtype=torch.int32, device=self.device)
            gs.rows_args = torch.zeros(12, dtype=torch.int64)
        r = gs.rows_args.numpy()
        ptr = lambda t: t.data_ptr()  # noqa: E731
        r[0], r[1], r[2] = cap, self.scratch_slot, ptr(gs.rows_dev)
        r[3], r[4], r[5] = ptr(gs.slots), ptr(gs.pos), ptr(gs.active)
        if self.last:
            r[6], r[7], r[8], r[9], r[10] = ptr(gs.temp), ptr(gs.topk), ptr(gs.greedy), ptr(gs.seeds), ptr(gs.sstep)
        r[11] = ptr(gs.tin) if self.first else 0
        return slot, gs.rows_args

    def _apply_rows_staged(self, gs: GroupState, rows, b: int, pad: int, sl, pos, act) -> None:
        """_apply_rows on a GPU: every per-row field packed into ONE int32
        buffer (float32 temperatures as their bits, int64 seeds / steps as
        int32 pairs at an even offset) uploaded through the group's pinned
        staging ring, then device copies into the row state -- instead of one
        pinned host tensor per field (profiles/r5_profile_issue.log).  The
        int64 fields start at int32 offset 6 b, so their views are aligned."""
        i32 = np.int32
        parts = [np.asarray(sl, i32), np.asarray(pos, i32), np.asarray(act, i32)]
        if self.last:
            parts += [np.asarray([r.temperature for r in rows] + [1.0] * pad, np.float32).view(i32),
                      np.asarray([r.top_k for r in rows] + [1] * pad, i32),
                      np.asarray([1 if r.greedy else 0 for r in rows] + [1] * pad, i32)]
            # the int64 fields start at int32 offset 6 b: 8-byte aligned
            parts += [np.asarray([r.seed for r in rows] + [0] * pad, np.int64).view(i32),
                      np.asarray([r.step for r in rows] + [0] * pad, np.int64).view(i32)]
        if self.first:
            parts.append(np.asarray([r.src for r in rows] + [0] * pad, i32))
        arr = np.concatenate(parts)
        buf = getattr(gs, "_rows_buf", None)
        if buf is None or buf.numel() < arr.size:
            buf = gs._rows_buf = torch.empty(2 * arr.size, dtype=torch.int32, device=self.device)
        self._stage_h2d(gs, arr, buf[: arr.size])
        gs.slots[:b].copy_(buf[:b])
        gs.pos[:b].copy_(buf[b: 2 * b])
        gs.active[:b].copy_(buf[2 * b: 3 * b])
        o = 3 * b
        if self.last:
            gs.temp[:b].copy_(buf[o: o + b].view(torch.float32))
            gs.topk[:b].copy_(buf[o + b: o + 2 * b])
            gs.greedy[:b].copy_(buf[o + 2 * b: o + 3 * b])
            o += 3 * b
            gs.seeds[:b].copy_(buf[o: o + 2 * b].view(torch.int64))
            gs.sstep[:b].copy_(buf[o + 2 * b: o + 4 * b].view(torch.int64))
            o += 4 * b
        if self.first:
            gathered = gs.tin.index_select(0, buf[o: o + b])
            gs.tin[:b].copy_(gathered)

    def _prefill(self, gp: GroupPlan, gs: GroupState, inp: Optional[torch.Tensor]):
        st, be, dev = self.stage, self.stage.backend, self.device
        ch = gp.chunks
        finals = [i for i, c in enumerate(ch) if c.final]
        v = gp.g & 1  # alternating-split variant of this group
        x, meta = self._prefill_graph(gp, gs, inp, v) if self._prefill_graphs() else (None, None)
        if x is None:
            meta, ids, _ = self._chunk_meta(gs, ch, tuple(c.qlen for c in ch))
            if self.first:
                inp = ids
            if not self.last:
                return st.forward(meta, inp, head=False, variant=v)
            if not finals:
                st.forward(meta, inp, head=False, variant=v)  # KV cache only
                return None
            rows = meta.last_idx.index_select(0, torch.tensor(finals, dtype=torch.long, device=dev))
            logits = st.forward(meta, inp, head=True, head_rows=rows, variant=v)
        else:
            if not self.last:
                return x
            if not finals:
                return None
            rows = meta.last_idx.index_select(0, torch.tensor(finals, dtype=torch.long, device=dev))
            be.decode = False
            logits = st.head(x, meta, rows=rows)
        fc = [ch[i] for i in finals]
        samp = SamplingState([c.temperature for c in fc], [c.top_k for c in fc],
                             [c.greedy for c in fc], [c.seed for c in fc], dev)
        return be.sample(logits, samp, st.cfg.vocab_size)

    # Prefill chunks as hipGraphs (the non-steady items):
    # a chunk item whose shape (per-sequence query counts, split variant, input
    # buffer) was seen before replays a captured graph of this stage's forward
    # instead of issuing its ~10 launches per layer from Python.  The graph's
    # index tensors (token slots / positions, sequence slots / starts, and on
    # stage 0 the token ids) are views of ONE device buffer refilled by one
    # host-to-device copy on the lane before each replay; row offsets and
    # attention tiles depend on the query counts only and stay fixed.  The
    # edge transfers stay eager and the last stage's head + sampler run after
    # the replay.  First use of a shape: eager (workspaces, routing); second:
    # capture.  "auto" = on with P > 1 stages (the schedule that chunks prompts:
    # bench.py --prefill-chunk -1), LSD_PREFILL_GRAPHS=1 / 0 forces it.
    PREFILL_GRAPHS = os.environ.get("LSD_PREFILL_GRAPHS", "auto")
    # captured prefill graphs kept per group (each holds its activations'
    # memory pool): serving with varied prompt mixes would otherwise grow them
    # without bound; the oldest is dropped first
    PREFILL_GRAPHS_MAX = int(os.environ.get("LSD_PREFILL_GRAPHS_MAX", "16"))

    def _prefill_graphs(self) -> bool:
        v = self.PREFILL_GRAPHS
        return (self.use_graphs and self.device.type == "cuda"
                and (v == "1" or (v == "auto" and self.P > 1)))

    def _prefill_graph(self, gp: GroupPlan, gs: GroupState, inp: Optional[torch.Tensor], v: int):
        """(hidden out [T, H], static meta) from the chunk's graph, or (None,
        None): first use of the shape, run eagerly."""
        ch = gp.chunks
        qlens = tuple(c.qlen for c in ch)
        if all(n == 1 for n in qlens):
            # one query per sequence: BatchMeta.build makes this a decode batch
            # (decode kernels, attention splits sized by the host context
            # bound) -- eager, as before
            return None, None
        key = (qlens, v, None if self.first else inp.data_ptr())
        ent = gs.pf_graphs.get(key)
        if ent is None and key not in gs.pf_seen:
            if len(gs.pf_seen) >= 64 * self.PREFILL_GRAPHS_MAX:
                gs.pf_seen.clear()  # shapes seen once long ago: forget them
            gs.pf_seen.add(key)
            return None, None
        dev = self.device
        if getattr(self.t, "aborted", False):
            from .comm import TransportError

            raise TransportError("data plane aborted: prefill graph not replayed")
        if ent is None:
            while gs.pf_graphs and len(gs.pf_graphs) >= max(1, self.PREFILL_GRAPHS_MAX):
                # a replay of the oldest graph may still be in flight on this
                # lane: let it finish before its memory pool is released
                torch.cuda.current_stream(dev).synchronize()
                gs.pf_graphs.pop(next(iter(gs.pf_graphs)))
            meta, ids, buf = self._chunk_meta(gs, ch, qlens)
            from ..ops.hip import prefill_tiles

            meta._tiles = prefill_tiles(meta).to(dev)
            x_in = ids if self.first else inp
            g, out, _ = self._capture(lambda: self.stage.forward(meta, x_in, head=False, variant=v))
            ent = gs.pf_graphs[key] = (g, buf, meta, out)
            self.captures += 1
        else:
            self._chunk_meta(gs, ch, qlens, ent[1])
        ent[0].replay()
        self.pf_replays += 1
        return ent[3], ent[2]

    def _chunk_meta(self, gs: GroupState, ch, qlens, buf: Optional[torch.Tensor] = None):
        """(BatchMeta, stage 0's token ids or None, index buffer) of a prefill
        chunk item: every index tensor is a view of ONE device buffer filled by
        one staged host-to-device copy (`buf` given: refill that one).  The
        same values as BatchMeta.build, including a decode-shaped batch (one
        query per sequence)."""
        dev = self.device
        T, B = sum(qlens), len(ch)
        if dev.type != "cuda":
            meta = BatchMeta.build([c.slot for c in ch], [c.start for c in ch], list(qlens), dev)
            ids = (_h2d([t for c in ch for t in c.ids], torch.int32, dev).to(dev) if self.first else None)
            return meta, ids, None
        arr = _chunk_index(ch, qlens, self.first)
        if buf is None:
            buf = torch.empty(arr.size, dtype=torch.int32, device=dev)
        self._stage_h2d(gs, arr, buf)
        o = 2 * T + 2 * B
        dec = all(n == 1 for n in qlens)
        meta = BatchMeta(token_slots=buf[:T], token_pos=buf[T: 2 * T], seq_slots=buf[2 * T: 2 * T + B],
                         q_start=buf[2 * T + B: o], cu_q=buf[o: o + B + 1], last_idx=buf[o + B + 1: o + 2 * B + 1],
                         num_tokens=T, num_seqs=B, max_q=max(qlens, default=0),
                         max_ctx=max((c.start + n for c, n in zip(ch, qlens)), default=0), is_decode=dec,
                         host_qlens=list(qlens))
        return meta, (buf[o + 2 * B + 1:] if self.first else None), buf

    _PF_PIN = 4  # staging buffers per group: a copy's source is reused 4 chunks later

    def _stage_h2d(self, gs: GroupState, arr: np.ndarray, dst: torch.Tensor) -> None:
        """Host int32 array -> dst (device), through a ring of pinned staging
        buffers owned by the group (no per-call pinned allocation: under
        several stage threads, torch's pin_memory took ~1 ms a call,
        profiles/r5_profile_issue.log); a buffer is reused only after the
        copy out of it has completed (its event)."""
        n = arr.size
        if len(gs.pf_pin) < self._PF_PIN:
            gs.pf_pin.append([torch.empty(max(n, 1 << 12), dtype=torch.int32, pin_memory=True),
                              torch.cuda.Event(), False])
        slot = gs.pf_pin[gs.pf_pin_next % len(gs.pf_pin)]
        gs.pf_pin_next += 1
        if slot[2]:
            slot[1].synchronize()
        if slot[0].numel() < n:
            slot[0] = torch.empty(2 * n, dtype=torch.int32, pin_memory=True)
        slot[0].numpy()[:n] = arr
        dst.copy_(slot[0][:n], non_blocking=True)
        slot[1].record()
        slot[2] = True

    def _decode(self, gp: GroupPlan, gs: GroupState, inp: torch.Tensor, io: bool = False) -> torch.Tensor:
        key = (gp.b, gp.ctxb, io)
        lane = self.lane_of(gp.g)

        def body():
            if io and not self.first:  # the edge receive, inside the graph
                self._recv(inp, self.r - 1, "fwd", lane, stage=gs.wire_buf(self, gp.b), capture=True)
            meta = gs.meta(gp.b, gp.ctxb)
            out = self.stage.forward(meta, inp, head=True, variant=gp.g & 1)
            if not self.last:
                meta.advance()
                if io:
                    self._send(out, self.r + 1, "fwd", lane, capture=True)
                return out
            samp = gs.samp(gp.b)
            # the sampler kernel also advances this stage's positions (no add kernel)
            self.stage.backend.sample_into(out, samp, self.stage.cfg.vocab_size, gs.tokret[: gp.b], meta)
            if io:
                self._send(gs.tokret[: gp.b], 0, "ret", lane, capture=True)
            return gs.tokret[: gp.b]

        graphs = self.use_graphs and self.device.type == "cuda"
        if not graphs:
            return body()
        if key in gs.graphs:
            g, out = gs.graphs[key]
            self._replay(gs, key, g)  # inside the item's shared section of GPU_GATE
            return out
        if key not in gs.seen:  # first use: eager (allocates workspaces outside capture)
            gs.seen.add(key)
            return body()
        g, out, io = self._capture(body)
        gs.graphs[key] = (g, out)
        if io[0]:
            gs.graph_io[key] = io
        self.captures += 1
        self._replay(gs, key, g)
        return out

    def _replay(self, gs: GroupState, key: tuple, g) -> None:
        if getattr(self.t, "aborted", False):
            # never replay a graph whose captured transfers use an aborted
            # data plane (freed communicators / abandoned channels)
            from .comm import TransportError

            raise TransportError("data plane aborted: decode graph not replayed")
        io = gs.graph_io.get(key)
        if io is not None:
            self.t.replay(g, io[0], io[1])  # loopback: enqueue handshake around the launch
        elif key[2]:
            with self.t.issuing():  # captured RCCL ops: not beside an abort
                g.replay()
        else:
            g.replay()

    def _fwd_b(self, gp: GroupPlan, ins) -> None:
        """Compat /forward_b on stages 1..P-1: full-sequence forward of the
        hidden rows received from stage 0 on the compat KV slot; the last
        stage returns all-position fp32 logits to stage 0."""
        st = self.stage
        T = gp.fwd_rows
        meta = BatchMeta.build([self.compat_slot], [0], [T], self.device)
        x = ins[0]
        lane = self.lane_of(gp.g)
        if self.last:
            # only the real vocabulary crosses (the HIP lm_head pads it)
            out = st.forward(meta, x, all_logits=True)[:, : st.cfg.vocab_size].contiguous()
            self.send_pending.setdefault(gp.g, []).append(self._send(out, 0, "ret", lane))
        else:
            out = st.forward(meta, x)
            self.send_pending.setdefault(gp.g, []).append(self._send(out, self.r + 1, "fwd", lane))

    # ------------------------------------------------------------------
    def _capture(self, fn):
        """Capture one decode step (this stage's forward for one group bucket,
        plus sampling on the last stage) into a hipGraph."""
        # capture_begin/end directly: torch.cuda.graph() does a device-wide
        # synchronize on entry, which is illegal while a sibling stage thread on
        # the same GPU is capturing.  One capture at a time per process.
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        begin = getattr(self.t, "begin_capture", None)
        io = (0, [])
        with self._gate_released(), GPU_GATE.exclusive():
            # no garbage collection inside the capture: a collected object
            # from an earlier session (a graph, an event, a communicator)
            # would run HIP teardown calls that are illegal mid-capture
            gc.collect()
            was = gc.isenabled()
            gc.disable()
            try:
                with torch.cuda.stream(s):
                    if begin is not None:
                        begin()  # the transport records the ops captured below
                    g.capture_begin(capture_error_mode="thread_local")
                    try:
                        out = fn()
                    finally:
                        g.capture_end()
                        if begin is not None:
                            io = self.t.end_capture()
            finally:
                if was:
                    gc.enable()
        torch.cuda.current_stream(self.device).wait_stream(s)
        return g, out, io

    def _gate_released(self):
        """Drop this thread's shared hold on GPU_GATE (held by the item being
        executed) around an exclusive section, and take it back after."""
        return GPU_GATE.released()

    def _gpu(self):
        """Shared hold on GPU_GATE for a GPU-issuing section of this thread."""
        if self.device.type != "cuda":
            return contextlib.nullcontext()
        return GPU_GATE.shared()


def _cu_masked_lanes(dev: torch.device, n: int, mode: str) -> List[torch.cuda.ExternalStream]:
    from ..ops.hip import _load

    C = _load()
    with torch.cuda.device(dev):
        cus = C.device_cu_count()
        words = (cus + 31) // 32
        lanes = []
        for l in range(n):
            bits = [c for c in range(cus) if ((c % n == l) if mode == "interleave" else (c * n // cus == l))]
            mask = [0] * words
            for c in bits:
                mask[c // 32] |= 1 << (c % 32)
            lanes.append(torch.cuda.ExternalStream(C.stream_with_cu_mask(mask), device=dev))
    return lanes


def _chunk_index(ch, qlens, first: bool) -> np.ndarray:
    """A prefill chunk item's index buffer, int32: token slots [T], token
    positions [T], sequence slots [B], sequence starts [B], row offsets
    [B + 1], last rows [B] (and on stage 0 the token ids [T]) -- vectorised
    (a 256 x 32-token item is 16-24 K values)."""
    B = len(ch)
    q = np.asarray(qlens, dtype=np.int64)
    T = int(q.sum())
    sl = np.fromiter((c.slot for c in ch), dtype=np.int64, count=B)
    st = np.fromiter((c.start for c in ch), dtype=np.int64, count=B)
    cu = np.zeros(B + 1, dtype=np.int64)
    np.cumsum(q, out=cu[1:])
    parts = [np.repeat(sl, q), np.arange(T, dtype=np.int64) + np.repeat(st - cu[:-1], q), sl, st, cu, cu[1:] - 1]
    if first:
        parts.append(np.fromiter(itertools.chain.from_iterable(c.ids for c in ch), dtype=np.int64, count=T))
    return np.concatenate(parts).astype(np.int32)


def _h2d(vals, dtype, dev) -> torch.Tensor:
    """Host tensor for an async copy to `dev` (pinned when `dev` is a GPU;
    the caching host allocator keeps it alive until the copy has run)."""
    t = torch.tensor(vals, dtype=dtype)
    if dev.type == "cuda":
        t = t.pin_memory()
    return t
