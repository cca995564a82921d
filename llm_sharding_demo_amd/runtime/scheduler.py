"""Iteration-level request scheduler (continuous batching) + round watchdog.

Reference behaviour (`server.py:154-210`): every /generate
runs its own decode loop in FastAPI's threadpool; concurrent requests share
nothing and each pays the full per-token HTTP round trips (measured: 4
concurrent requests -> 0.83 tok/s aggregate vs 0.69 for one).

Here one scheduler (on the thread that drives pipeline stage 0) owns every
sequence and decides, at every decode step, a `StepPlan` (runtime/plan.py)
that all stages execute:

  * requests wait in an admission queue (the native `BatchQueue`,
    csrc/runtime/batch_queue.h) and JOIN a microbatch group at the next step
    boundary when the group has a free row and the replica a free KV slot;
    their prompts are prefilled by that step's item (chunked when
    PREFILL_CHUNK is set), and the final chunk's sample is their first token;
  * a sequence LEAVES its group at the step after its last token was
    scheduled (max_new_tokens) or after its EOS was read back (stop_at_eos),
    so a short request never waits behind a long one;
  * decode rows are kept compacted and padded to a power-of-two bucket, so
    the per-(group, bucket) hipGraphs stay valid across steps and requests;
  * sampled token ids come back to the host asynchronously (D2H copy + event
    per item); the scheduler runs at most a few steps ahead of the GPU.

`Watchdog` puts a deadline on pipeline progress: if the
engine makes no progress for `round_timeout_s` (a hung RCCL peer, a dead
stage) it is marked unhealthy with a clear error and waiting requests fail
instead of hanging forever.
"""
from __future__ import annotations

import collections
import itertools
import logging
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Deque, Dict, List, Optional

import torch

from ..config import SamplingParams
from ..utils import racecheck
from .plan import Chunk, GroupPlan, Row, StepPlan

log = logging.getLogger("llm_sharding_demo_amd.scheduler")


class RequestTimeout(RuntimeError):
    pass


_FINISH = threading.Lock()  # orders Request.finish against a waiter creating its event


@dataclass(eq=False)
class Request:
    """One generation request.  Light on purpose: a 4096-sequence session
    creates 4096 of these on the submitting thread, so the completion event
    is made only when someone actually blocks in wait() before the request
    finishes (a threading.Event per request was ~6 us of the ~14 us
    submit cost, profiles/r6_session_host.log)."""
    prompt_ids: List[int]
    params: SamplingParams
    t_submit: float = field(default_factory=time.monotonic)
    t_start: float = 0.0        # joined the pipeline (prefill issued)
    t_first: float = 0.0        # first token read back (TTFT = t_first - t_submit)
    t_done: float = 0.0
    output: Optional[List[int]] = None
    error: Optional[BaseException] = None
    _flag: bool = False
    _ev: Optional[threading.Event] = None

    def wait(self, timeout: Optional[float] = None) -> List[int]:
        if not self._flag:
            with _FINISH:
                if not self._flag and self._ev is None:
                    self._ev = threading.Event()
                ev = self._ev
            if ev is not None and not ev.wait(timeout):
                raise RequestTimeout(f"request not finished after {timeout} s")
        if self.error is not None:
            raise self.error
        return self.output

    @property
    def done(self) -> bool:
        return self._flag

    def finish(self, output=None, error=None) -> None:
        self.output, self.error = output, error
        self.t_done = time.monotonic()
        with _FINISH:
            self._flag = True
            ev = self._ev
        if ev is not None:
            ev.set()


class PyBatchQueue(racecheck.Shared):
    """Pure-Python twin of the native `BatchQueue` (csrc/runtime/batch_queue.h):
    same interface and grouping rule; the reference the tests compare the
    native queue against, and the fallback when _runtime.so is absent."""

    def __init__(self, max_batch: int, length_ratio: float = 4.0):
        if max_batch < 1 or length_ratio < 1.0:
            raise ValueError("max_batch >= 1 and length_ratio >= 1 required")
        self.max_batch, self.ratio = max_batch, length_ratio
        self._cv = racecheck.Condition(name="batch_queue")
        self._q: "collections.deque" = collections.deque()
        self._closed = False
        self.max_seen = 0
        self.pushed = self.popped = 0

    def push(self, id: int, max_new_tokens: int) -> bool:
        with self._cv:
            if self._closed:
                return False
            self._q.append((id, max(1, max_new_tokens)))
            self.pushed += 1
            self._cv.notify()
            return True

    def push_many(self, ids: List[int], max_new_tokens: List[int]) -> bool:
        if len(ids) != len(max_new_tokens):
            raise ValueError("push_many: length mismatch")
        with self._cv:
            if self._closed:
                return False
            self._q.extend((i, max(1, n)) for i, n in zip(ids, max_new_tokens))
            self.pushed += len(ids)
            self._cv.notify_all()
            return True

    def next_groups(self, window_s: float) -> List[List[int]]:
        with self._cv:
            self._cv.wait_for(lambda: self._closed or self._q)
            if self._closed:
                return []
            deadline = time.monotonic() + max(window_s, 0.0)
            batch = []
            while True:
                while self._q and len(batch) < self.max_batch:
                    batch.append(self._q.popleft())
                if len(batch) >= self.max_batch or self._closed:
                    break
                left = deadline - time.monotonic()
                if left <= 0 or not self._cv.wait_for(lambda: self._closed or self._q, left):
                    break
            self.popped += len(batch)
            self.max_seen = max(self.max_seen, len(batch))
        batch.sort(key=lambda it: it[1])
        groups: List[List[int]] = []
        first = 0
        for id_, n in batch:
            if not groups or n > self.ratio * first:
                groups.append([])
                first = n
            groups[-1].append(id_)
        return groups

    def try_pop(self, k: int) -> List[int]:
        """Up to k queued ids in FIFO order, without waiting."""
        with self._cv:
            out = []
            while self._q and len(out) < k:
                out.append(self._q.popleft()[0])
            self.popped += len(out)
            return out

    def wait_nonempty(self, timeout_s: float) -> bool:
        with self._cv:
            return self._cv.wait_for(lambda: self._closed or self._q, timeout_s)

    def close(self) -> None:
        with self._cv:
            self._closed = True
            self._cv.notify_all()

    def drain(self) -> List[int]:
        with self._cv:
            out = [i for i, _ in self._q]
            self._q.clear()
            return out

    @property
    def depth(self) -> int:
        with self._cv:
            return len(self._q)

    @property
    def closed(self) -> bool:
        return self._closed


def make_batch_queue(max_batch: int, length_ratio: float = 4.0, native: bool = True):
    """The native queue (GIL released while the scheduler waits) when
    _runtime.so is built, else the Python twin."""
    if native:
        from .native import load

        R = load()
        if R is not None and hasattr(R, "BatchQueue") and hasattr(R.BatchQueue, "try_pop"):
            return R.BatchQueue(max_batch, length_ratio)
    return PyBatchQueue(max_batch, length_ratio)


# ---------------------------------------------------------------------------
# Scheduler core: the per-step state machine (native csrc/runtime/sched_core.h,
# or this Python twin -- same interface, same plans, compared in
# tests/test_sched_core.py)
# ---------------------------------------------------------------------------

EV_FIRST, EV_FINISH, EV_RELEASE = 1, 2, 4


@dataclass
class _Seq:
    prompt_len: int
    want: int
    stop_at_eos: bool
    rep: int = 0
    g: int = -1
    slot: int = -1
    prefilled: int = 0          # prompt tokens whose chunks have been issued
    issued: int = 0             # output tokens whose production has been issued
    pos: int = 0                # next decode input position
    sstep: int = 1              # sampler counter of the next decode draw
    ntok: int = 0               # tokens read back
    stop: bool = False          # EOS read back (stop_at_eos): leave at the next step
    toks: List[int] = field(default_factory=list)  # assign_collect only
    finished: bool = False


@dataclass
class _Produced:
    """Composition of one item that produced tokens: how to read its
    token-return vector [decode rows (b) | final prefill chunks]."""
    b: int
    rows: List[int]             # seq ids of decode rows [0, n)
    finals: List[int]           # seq ids whose final prefill chunk was sampled
    release: List[int] = field(default_factory=list)  # seqs whose last item this was


@dataclass
class _Group:
    rows: List[int] = field(default_factory=list)
    prefilling: List[int] = field(default_factory=list)
    prev: Optional[_Produced] = None
    waited: int = 0  # consecutive steps this group deferred its joins


def _bucket(n: int, cap: int) -> int:
    if n <= 0:
        return 0
    b = 1
    while b < n:
        b <<= 1
    return min(b, cap)


class PySchedCore:
    """Python twin of lsd_rt::SchedCore (LSD_PY_RUNTIME=1, or no native
    runtime).  plan(step) -> ([per replica: [(g, ret, n, b, ctxb, rows_changed,
    chunks [(sid, slot, start, len, final)], rows [(sid, slot, pos, sstep,
    src)])]], admitted sids); assign(...) -> [(sid, token, flags)]."""

    def __init__(self, replicas: int, groups: int, cap: int, prefill_budget: int, chunk: int,
                 max_seq: int, pools):
        self.R, self.M, self.cap = replicas, groups, cap
        self.budget, self.chunk, self.max_seq = prefill_budget, chunk, max_seq
        self.pools = list(pools)
        self.seqs: Dict[int, _Seq] = {}
        self.waiting: Deque[int] = collections.deque()
        self.groups = [[_Group() for _ in range(groups)] for _ in range(replicas)]
        self.expect: Dict[tuple, _Produced] = {}
        self.joins = self.leaves = self.max_rows = self.steps = 0
        self.join_min, self.max_wait, self.deferred = 1, 0, 0

    def set_join_policy(self, join_min: int, max_wait: int) -> None:
        """lsd_rt::SchedCore::set_join_policy: admit only with room for every
        waiting request or for join_min of them, when the group is idle, or
        after max_wait deferred steps in a row."""
        if join_min < 1 or max_wait < 0:
            raise ValueError("join_min >= 1, max_wait >= 0")
        self.join_min, self.max_wait = join_min, max_wait

    def _join_ok(self, gh: "_Group", room: int, idle: bool) -> bool:
        if not self.waiting or room <= 0:
            gh.waited = 0
            return False
        if idle or room >= min(self.join_min, len(self.waiting)) or gh.waited >= self.max_wait:
            gh.waited = 0
            return True
        gh.waited += 1
        self.deferred += 1
        return False

    def add(self, sid: int, prompt_len: int, want: int, stop_at_eos: bool) -> None:
        if prompt_len <= 0:
            raise ValueError("empty prompt")
        self.seqs[sid] = _Seq(prompt_len, want, stop_at_eos)
        self.waiting.append(sid)

    def add_many(self, sids, prompt_lens, wants, stops) -> None:
        if not len(sids) == len(prompt_lens) == len(wants) == len(stops):
            raise ValueError("add_many: length mismatch")
        if any(n <= 0 for n in prompt_lens):
            raise ValueError("empty prompt")
        for a in zip(sids, prompt_lens, wants, stops):
            self.add(*a)

    def has_work(self) -> bool:
        if self.waiting:
            return True
        return any(g.rows or g.prefilling or g.prev is not None for rep in self.groups for g in rep)

    @property
    def n_waiting(self) -> int:
        return len(self.waiting)

    @property
    def n_seqs(self) -> int:
        return len(self.seqs)

    @property
    def n_expect(self) -> int:
        return len(self.expect)

    def plan(self, step: int):
        admitted: List[int] = []
        out = []
        for rep in range(self.R):
            gs = []
            for g in range(self.M):
                go = self._group_plan(rep, g, step, admitted)
                if go is not None:
                    gs.append(go)
            out.append(gs)
        self.steps += 1
        return out, admitted

    def _admit(self, rep: int, g: int, room: int, admitted: List[int]) -> List[int]:
        pool = self.pools[rep]
        out = []
        while self.waiting and room > 0 and pool.available > 0:
            sid = self.waiting.popleft()
            s = self.seqs[sid]
            s.rep, s.g = rep, g
            s.slot = pool.alloc(1)[0]
            out.append(sid)
            admitted.append(sid)
            room -= 1
            self.joins += 1
        return out

    def _group_plan(self, rep: int, g: int, step: int, admitted: List[int]):
        gh = self.groups[rep][g]
        prev, gh.prev = gh.prev, None
        ret = prev.b + len(prev.finals) if prev is not None else 0
        # leaves: every token scheduled, or EOS read back
        keep = []
        for sid in gh.rows:
            s = self.seqs[sid]
            if s.issued >= s.want or s.stop:
                self.leaves += 1
                if prev is not None:
                    prev.release.append(sid)
            else:
                keep.append(sid)
        new_rows = keep + (list(prev.finals) if prev is not None else [])
        changed = new_rows != gh.rows
        # joins (capacity counts rows + sequences still prefilling)
        room = self.cap - len(new_rows) - len(gh.prefilling)
        if self._join_ok(gh, room, not new_rows and not gh.prefilling):
            gh.prefilling += self._admit(rep, g, room, admitted)
        # prefill chunks (FIFO, one chunk per sequence per step, token budget)
        budget = self.budget or (1 << 62)
        chunks, finals = [], []
        for sid in list(gh.prefilling):
            s = self.seqs[sid]
            L = s.prompt_len
            n = L - s.prefilled if self.chunk <= 0 else min(self.chunk, L - s.prefilled)
            if chunks and n > budget:
                break
            budget -= n
            a = s.prefilled
            final = a + n == L
            chunks.append((sid, s.slot, a, n, final))
            s.prefilled += n
            if final:
                gh.prefilling.remove(sid)
                finals.append(sid)
                s.issued, s.pos, s.sstep = 1, L, 1
        # decode rows
        n = len(new_rows)
        b = _bucket(n, self.cap)
        rows = []
        if changed:
            old_index = {sid: i for i, sid in enumerate(gh.rows)}
            for sid in new_rows:
                s = self.seqs[sid]
                src = old_index[sid] if sid in old_index else prev.b + prev.finals.index(sid)
                rows.append((sid, s.slot, s.pos, s.sstep, src))
        ctxb = 0
        if n:
            top = max(self.seqs[sid].pos for sid in new_rows) + 1
            ctxb = min(-(-top // 256) * 256, self.max_seq)
            for sid in new_rows:  # this step issues one token per decode row
                s = self.seqs[sid]
                s.issued += 1
                s.pos += 1
                s.sstep += 1
        gh.rows = new_rows
        self.max_rows = max(self.max_rows, n)
        if b or finals:
            gh.prev = _Produced(b, list(new_rows), finals)
        if prev is not None:  # its readout comes back in this step's token-return vector
            self.expect[(rep, step, g)] = prev
        if not (ret or b or chunks):
            return None
        return (g, ret, n, b, ctxb, changed, chunks, rows)

    def assign(self, rep: int, step: int, g: int, tokens: List[int], eos: int):
        prod = self.expect.pop((rep, step, g))
        ev = []
        for i, sid in enumerate(prod.rows):
            self._give(sid, tokens[i], eos, ev)
        for j, sid in enumerate(prod.finals):
            self._give(sid, tokens[prod.b + j], eos, ev)
        for sid in prod.release:
            s = self.seqs.pop(sid, None)
            if s is None:
                continue
            if s.slot >= 0:
                self.pools[s.rep].free([s.slot])
            ev.append((sid, -1, EV_RELEASE | (0 if s.finished else EV_FINISH)))
        return ev

    def assign_collect(self, rep: int, step: int, g: int, tokens, eos: int):
        """Twin of SchedCore::assign_collect: only FIRST / FINISH / RELEASE
        events, plus (sid, tokens) of every sequence that finished."""
        prod = self.expect.pop((rep, step, g))
        tokens = [int(t) for t in tokens]
        ev, done = [], []
        for i, sid in enumerate(prod.rows):
            self._give_collect(sid, tokens[i], eos, ev, done)
        for j, sid in enumerate(prod.finals):
            self._give_collect(sid, tokens[prod.b + j], eos, ev, done)
        for sid in prod.release:
            s = self.seqs.pop(sid, None)
            if s is None:
                continue
            if not s.finished:
                done.append((sid, list(s.toks)))
            if s.slot >= 0:
                self.pools[s.rep].free([s.slot])
            ev.append((sid, -1, EV_RELEASE | (0 if s.finished else EV_FINISH)))
        return ev, done

    def _give_collect(self, sid: int, tok: int, eos: int, ev: list, done: list) -> None:
        s = self.seqs.get(sid)
        if s is None or s.finished or s.ntok >= s.want:
            return
        flags = EV_FIRST if s.ntok == 0 else 0
        s.ntok += 1
        s.toks.append(tok)
        if s.stop_at_eos and tok == eos:
            s.stop = True
        if s.ntok >= s.want or s.stop:
            s.finished = True
            flags |= EV_FINISH
            done.append((sid, list(s.toks)))
        if flags:
            ev.append((sid, tok, flags))

    def _give(self, sid: int, tok: int, eos: int, ev: list) -> None:
        s = self.seqs.get(sid)
        if s is None or s.finished or s.ntok >= s.want:
            return
        flags = EV_FIRST if s.ntok == 0 else 0
        s.ntok += 1
        if s.stop_at_eos and tok == eos:
            s.stop = True
        if s.ntok >= s.want or s.stop:
            s.finished = True
            flags |= EV_FINISH
        ev.append((sid, tok, flags))

    def reset(self) -> None:
        for s in self.seqs.values():
            if s.slot >= 0:
                self.pools[s.rep].free([s.slot])
        self.seqs.clear()
        self.waiting.clear()
        self.expect.clear()
        self.groups = [[_Group() for _ in range(self.M)] for _ in range(self.R)]


def make_sched_core(replicas: int, groups: int, cap: int, prefill_budget: int, chunk: int,
                    max_seq: int, pools):
    """The native core when the runtime is built and the slot pools are its
    allocators; the Python twin otherwise (LSD_PY_RUNTIME=1)."""
    from .native import load

    rt = load()
    if rt is not None and hasattr(rt, "SchedCore") and all(isinstance(p, rt.SlotAllocator) for p in pools):
        return rt.SchedCore(replicas, groups, cap, prefill_budget, chunk, max_seq, list(pools))
    return PySchedCore(replicas, groups, cap, prefill_budget, chunk, max_seq, pools)


# ---------------------------------------------------------------------------
# Scheduler
# ---------------------------------------------------------------------------

@dataclass
class _Meta:
    req: Request
    seed: int
    samp: tuple = ()    # (temperature, top_k, greedy, seed): the chunk / row sampling fields
    done: bool = False  # finished by this scheduler (plain flag: the readout loop's hot path)


class Scheduler(racecheck.Shared):
    """Continuous-batching scheduler for one engine (every pipeline replica).

    Runs on the thread that drives stage 0 of replica 0 (`Engine._drive`);
    `submit()` is thread-safe.  The per-step state machine lives in the
    scheduler core (`make_sched_core`); this class owns the request futures,
    the sampling parameters, the plan objects and the GPU readouts."""

    def __init__(self, engine, groups: int, cap: int):
        self.eng = engine
        self.R = engine.R
        self.M, self.cap = groups, cap
        self.queue = make_batch_queue(max(1, cap * groups * self.R))
        self._pending: Dict[int, Request] = {}
        self._ids = itertools.count()
        self._plock = racecheck.Lock("sched.pending")
        self.meta: Dict[int, _Meta] = {}
        self.core = make_sched_core(self.R, groups, cap, engine.cfg.prefill_budget,
                                    engine.cfg.prefill_chunk, engine.max_seq, engine.slot_pools)
        self.core.set_join_policy(max(1, engine.cfg.join_min), max(0, engine.cfg.join_max_wait))
        self.step = 0
        self.readouts: Deque[tuple] = collections.deque()  # (step, ready(), sync(), tokens, key)
        self.lock = racecheck.RLock("sched.driver")         # one driver at a time
        self.timing = False
        self.step_log: List[tuple] = []                     # (step, had_prefill) of timed steps
        self.stats = {"steps": 0, "joins": 0, "leaves": 0, "max_rows": 0, "captures": 0, "deferred": 0}
        self._rng = engine._rng

    # -- admission ---------------------------------------------------------
    def submit(self, prompt_ids: List[int], params: SamplingParams) -> Request:
        req = Request(list(map(int, prompt_ids)), params)
        if params.max_new_tokens == 0:
            req.finish([])
            return req
        rid = next(self._ids)
        with self._plock:
            racecheck.note(self, "_pending")
            self._pending[rid] = req
        if not self.queue.push(rid, params.max_new_tokens):
            with self._plock:
                racecheck.note(self, "_pending")
                self._pending.pop(rid, None)
            raise RuntimeError("scheduler is closed")
        return req

    def submit_many(self, prompts: List[List[int]], params: List[SamplingParams]) -> List[Request]:
        """submit() for a whole batch: one pass under the pending-map lock
        (a 4096-sequence bench session submits everything at once)."""
        now = time.monotonic()
        # a list whose first token is a Python int is taken as a list of ints
        # and only copied (list(map(int, .)) per 64-token prompt was ~4 us,
        # 17 ms of a 4096-prompt session); anything else is converted
        reqs = [Request(list(p) if type(p) is list and p and type(p[0]) is int else list(map(int, p)), sp, now)
                for p, sp in zip(prompts, params)]
        live = []
        for req in reqs:
            if req.params.max_new_tokens == 0:
                req.finish([])
            else:
                live.append((next(self._ids), req))
        with self._plock:
            racecheck.note(self, "_pending")
            self._pending.update(live)
        if not self.queue.push_many([rid for rid, _ in live], [r.params.max_new_tokens for _, r in live]):
            with self._plock:
                racecheck.note(self, "_pending")
                for rid, _ in live:
                    self._pending.pop(rid, None)
            raise RuntimeError("scheduler is closed")
        return reqs

    @property
    def queue_depth(self) -> int:
        return self.queue.depth + self.core.n_waiting

    def _take_new(self) -> None:
        ids = self.queue.try_pop(1 << 20)
        if not ids:
            return
        with self._plock:
            racecheck.note(self, "_pending")
            reqs = [self._pending.pop(i) for i in ids]
        meta, rng = self.meta, self._rng
        lens, wants, stops = [], [], []
        for i, req in zip(ids, reqs):
            p = req.params
            seed = p.seed if p.seed is not None else rng.getrandbits(62)
            meta[i] = _Meta(req, seed, (p.temperature, p.top_k, p.greedy, seed))
            lens.append(len(req.prompt_ids))
            wants.append(p.max_new_tokens)
            stops.append(bool(p.stop_at_eos))
        self.core.add_many(ids, lens, wants, stops)

    def has_work(self) -> bool:
        """Anything left to plan OR to read back: token readouts still queued
        here, or expected by the core (replica > 0 readouts arrive later over
        the control plane), keep a serving session alive until they land."""
        return (bool(self.queue.depth) or self.core.has_work() or bool(self.readouts)
                or self.core.n_expect > 0)

    # -- plan building ---------------------------------------------------------
    def build_step(self) -> Optional[List[StepPlan]]:
        """Plans of the next step for every replica, or None when idle."""
        self._take_new()
        if not self.core.has_work():
            return None
        s = self.step
        self.step += 1
        per_rep, admitted = self.core.plan(s)
        if admitted:
            now = time.monotonic()
            for sid in admitted:
                self.meta[sid].req.t_start = now
        plans = [StepPlan(step=s, groups=[self._group(go) for go in gos], replica=rep,
                          timing=self.timing) for rep, gos in enumerate(per_rep)]
        c = self.core
        self.stats.update(steps=self.stats["steps"] + 1, joins=c.joins, leaves=c.leaves,
                          max_rows=c.max_rows, deferred=c.deferred)
        if self.timing:
            self.step_log.append((s, any(gp.chunks for p in plans for gp in p.groups)))
        return plans

    def _group(self, go) -> GroupPlan:
        g, ret, n, b, ctxb, changed, chunks, rows = go
        gp = GroupPlan(g, ret=ret, n=n, b=b, ctxb=ctxb)
        meta = self.meta
        gp.chunks = [Chunk(sid, slot, start, m.req.prompt_ids[start:start + ln], final, *m.samp)
                     for sid, slot, start, ln, final in chunks for m in (meta[sid],)]
        if changed:
            gp.rows = [Row(sid, slot, pos, *meta[sid].samp, sstep, src)
                       for sid, slot, pos, sstep, src in rows]
        return gp

    # -- token readout -----------------------------------------------------------
    def on_readout(self, plan: StepPlan, gp: GroupPlan, ret: torch.Tensor) -> None:
        """Stage-0 worker callback: the token-return vector of group gp.g's
        previous item is in `ret` (in stream order): copy it to the host."""
        key = (plan.replica, plan.step, gp.g)
        n = gp.ret
        if ret.is_cuda:
            from ..parallel.pipeline import GPU_GATE, wait_event

            host = torch.empty(n, dtype=torch.int32, pin_memory=True)
            host.copy_(ret[:n], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()

            # the coordinator thread polls these beside the stage threads: never
            # in the middle of a sibling's hipGraph capture (HIP refuses event
            # queries then -- hipErrorCapturedEvent -- and invalidates the
            # capture), so each query / wait holds the capture gate shared
            def ready(ev=ev):
                with GPU_GATE.shared():
                    return ev.query()

            def sync(ev=ev):
                wait_event(ev)
            self.readouts.append((plan.step, ready, sync, host, key, None))
        else:
            host = ret[:n].clone()
            self.readouts.append((plan.step, lambda: True, lambda: None, host, key, None))

    def on_readout_native(self, plan: StepPlan, gp: GroupPlan, host: torch.Tensor, ev, release) -> None:
        """Stage-0 native executor callback: the D2H copy of group gp.g's
        previous token-return vector into `host` and its completion event
        `ev` are already enqueued (csrc/stage_exec.cpp); `release(ev)` hands
        the event back to the worker's pool once the readout is applied."""
        from ..parallel.pipeline import GPU_GATE, wait_event

        def ready(ev=ev):
            with GPU_GATE.shared():
                return ev.query()

        def sync(ev=ev):
            wait_event(ev)
        self.readouts.append((plan.step, ready, sync, host, (plan.replica, plan.step, gp.g),
                              lambda ev=ev: release(ev)))

    def push_remote_readout(self, step: int, tokens: List[int], prod_key) -> None:
        """Replica > 0 readouts arrive over the control plane (dist + DP)."""
        host = torch.tensor(tokens, dtype=torch.int32)
        self.readouts.append((step, lambda: True, lambda: None, host, tuple(prod_key), None))

    def poll(self, block_until_step: Optional[int] = None) -> None:
        """Process completed readouts (in order).  With block_until_step,
        wait for every readout of steps <= that one."""
        while self.readouts:
            step, ready, sync, host, key, release = self.readouts[0]
            if not ready():
                if block_until_step is None or step > block_until_step:
                    return
                sync()
            self.readouts.popleft()
            self._assign(host, key)
            if release is not None:
                release()

    def _assign(self, host: torch.Tensor, key) -> None:
        """Apply one group readout.  The core keeps every sequence's tokens
        (assign_collect): a plain token of a running sequence costs nothing
        here, only first tokens (TTFT), finishes and slot releases come back --
        a per-row Python loop at 16 groups x 256 rows per step used to be
        stage 0's largest host cost (profiles/r3_rehearsal_all_configs.log)."""
        rep, step, g = key
        events, done = self.core.assign_collect(rep, step, g, host.numpy(), self.eng.mcfg.eos_token_id)
        if not events:
            return
        now = time.monotonic()
        done = dict(done)
        get = self.meta.get
        for sid, tok, flags in events:
            if flags & EV_RELEASE:
                m = self.meta.pop(sid, None)
                if m is not None and flags & EV_FINISH and not m.done:
                    m.done = True
                    m.req.finish(done.get(sid, []))
                continue
            m = get(sid)
            if m is None or m.done:
                continue
            if flags & EV_FIRST:
                m.req.t_first = now
            if flags & EV_FINISH:
                m.done = True
                m.req.finish(done[sid])

    # -- failure -----------------------------------------------------------------
    def fail_all(self, err: BaseException) -> None:
        for m in self.meta.values():
            if not m.req.done:
                m.done = True
                m.req.finish(error=err)
        self.meta.clear()
        self.core.reset()
        self.readouts.clear()
        with self._plock:
            pend = list(self._pending.values())
            self._pending.clear()
        for rid in self.queue.drain():
            pass
        for req in pend:
            req.finish(error=err)


class Watchdog:
    """Marks the engine unhealthy when the pipeline stops making progress or
    the data plane reports an asynchronous error, and then aborts the data
    plane: with the native RCCL transport a kernel waiting on a dead or
    stalled peer would otherwise spin forever (and every host thread waiting
    on its stream with it); ncclCommAbort makes it return, the waits drain
    and the requests fail instead of hanging (the reference
    fails a request after its 30 s HTTP timeout, server.py:173-174)."""

    def __init__(self, engine, round_timeout_s: float, poll_s: float = 0.25):
        self.engine = engine
        self.timeout = round_timeout_s
        self.poll = poll_s
        self.fired = False
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._loop, name="lsd-watchdog", daemon=True)
        self._thread.start()

    def _loop(self) -> None:
        while not self._stop.wait(self.poll):
            if self.fired:
                continue
            tr = getattr(self.engine, "data_plane", None) or getattr(self.engine, "transport", None)
            try:
                err = tr.check_async() if tr is not None else None
            except Exception as e:  # noqa: BLE001 - a broken communicator is an error too
                err = f"{type(e).__name__}: {e}"
            if err:
                self._fire("DataPlaneError", err)
                continue
            started = getattr(self.engine, "round_started", None)
            if started is None:
                continue
            elapsed = time.monotonic() - started
            if elapsed > self.timeout:
                self._fire("WatchdogTimeout",
                           f"no pipeline progress for {elapsed:.3g} s (deadline {self.timeout:.3g} s)")

    def _fire(self, kind: str, msg: str) -> None:
        self.fired = True
        log.error("watchdog: %s: %s; marking engine unhealthy and aborting the data plane", kind, msg)
        self.engine.healthy = False
        self.engine.last_error = f"{kind}: {msg}"
        tr = getattr(self.engine, "data_plane", None) or getattr(self.engine, "transport", None)
        if tr is not None:
            try:
                tr.abort()
            except Exception as e:  # noqa: BLE001
                log.error("watchdog: data-plane abort failed: %s", e)

    def close(self) -> None:
        self._stop.set()
        self._thread.join(timeout=5)
