"""Per-step execution plans: iteration-level (continuous) batching.

The reference serves every /generate independently in FastAPI's threadpool
(`/root/reference/server.py:154-155`): a short request never waits behind a
long one, but nothing is batched either.  Here the engine keeps M microbatch
*groups* permanently in flight through the pipeline and re-decides their
composition at every decode step:

  * a sequence LEAVES its group as soon as it has its tokens (max_new_tokens,
    or EOS seen), freeing its row and KV slot for the next request;
  * a new request JOINS at the next step boundary: its prompt is prefilled
    (in chunks if PREFILL_CHUNK is set) by the group's item of that step,
    the final chunk's last position is sampled, and from the step after it
    the sequence is a decode row like any other.

A group's decode rows are compacted into rows [0, n) and run as a padded
bucket of b >= n rows (b a power of two, at most the group capacity): the
pad rows point at a scratch KV slot and are masked out of the position /
sampler advance, so one captured hipGraph per (group, b, context bucket) is
replayed for as long as the shapes stay put -- across steps and requests.

Stage 0's scheduler decides a `StepPlan` per step and every other stage
executes the same plan (in-process queue, or the gloo control plane in dist
mode), so all stages agree on shapes without any device->host sync.
"""
from __future__ import annotations

import io
import pickle
from dataclasses import dataclass, field
from typing import List, Optional


@dataclass
class Chunk:
    """One prefill chunk of a joining sequence."""
    seq: int            # scheduler sequence id
    slot: int           # KV slot
    start: int          # first prompt position of the chunk
    ids: List[int]      # the chunk's token ids (consumed by stage 0 only)
    final: bool         # holds the prompt's last token: the last stage samples it
    temperature: float = 0.6
    top_k: int = 40
    greedy: bool = False
    seed: int = 0

    @property
    def qlen(self) -> int:
        return len(self.ids)


@dataclass
class Row:
    """State of one decode row (written to the device when a group's
    composition changes)."""
    seq: int
    slot: int
    pos: int            # position of the row's NEXT input token
    temperature: float
    top_k: int
    greedy: bool
    seed: int
    step: int           # sampler counter of the next draw (prefill draw = 0)
    src: int            # stage 0: index of the row's input token in the previous
                        # item's token-return vector (kept rows: their old row;
                        # newly activated rows: prev_b + final-chunk index)


@dataclass
class GroupPlan:
    g: int                                  # group (microbatch) index
    ret: int = 0                            # stage 0: token-return elements to receive first
    rows: Optional[List[Row]] = None        # new composition (None = unchanged)
    n: int = 0                              # active decode rows
    b: int = 0                              # decode bucket rows (0: no decode this step)
    ctxb: int = 0                           # context bucket of the decode graph
    chunks: List[Chunk] = field(default_factory=list)
    # compat forward (reference /forward_b through stages 1..P-1): hidden rows
    kind: str = "step"                      # "step" | "fwd_b"
    fwd_rows: int = 0

    @property
    def n_final(self) -> int:
        return sum(1 for c in self.chunks if c.final)

    @property
    def prefill_tokens(self) -> int:
        return sum(c.qlen for c in self.chunks)

    @property
    def has_work(self) -> bool:
        """Anything for stages other than 0's token receive."""
        return self.b > 0 or bool(self.chunks) or self.kind != "step"


@dataclass
class StepPlan:
    step: int
    groups: List[GroupPlan] = field(default_factory=list)
    replica: int = 0
    timing: bool = False                    # record per-item compute events
    end: bool = False                       # session end: followers return
    stop: bool = False                      # shut the follower down


# ---------------------------------------------------------------------------
# Binary wire format of the control plane (dist mode: rank 0 -> every rank)
# ---------------------------------------------------------------------------
# A plan travels as ONE fixed-size int32 record of PLAN_WORDS words (a gloo
# message must be received into a buffer of the exact size):
#   REPEAT  [magic, step]                         same groups as the previous
#                                                 plan to this rank, step + 1
#   STEADY  [magic, step, replica, flags, G,      decode-only groups (no
#            (g, ret, n, b, ctxb) x G]            composition change, no chunk)
#   PICKLE  [magic, nbytes]                       a pickled StepPlan follows as
#                                                 a second message (joins,
#                                                 leaves, prefill chunks, compat)
# In steady-state decode every step is REPEAT or STEADY: no pickling, one
# 512-byte message per follower.  The reference's control "plane" is a JSON
# POST per token per shard (`/root/reference/server.py:172-181`).
PLAN_WORDS = 128
MAGIC_REPEAT, MAGIC_STEADY, MAGIC_PICKLE = 0x4C534452, 0x4C534453, 0x4C534450
_MAX_STEADY_GROUPS = (PLAN_WORDS - 5) // 5
_F_TIMING, _F_END, _F_STOP = 1, 2, 4


def _steady_groups(plan: StepPlan):
    """(g, ret, n, b, ctxb) per group when the plan is decode-only, else None."""
    out = []
    for gp in plan.groups:
        if gp.rows is not None or gp.chunks or gp.kind != "step":
            return None
        out.append((gp.g, gp.ret, gp.n, gp.b, gp.ctxb))
    return out if len(out) <= _MAX_STEADY_GROUPS else None


# Non-steady plans (joins, leaves, prefill chunks) are pickled with every
# GroupPlan in a columnar form: one int32 / float64 / int64 column per Chunk
# and Row field instead of one pickled dataclass per sequence.  A step that
# joins 4096 sequences pickled in ~14 ms and unpickled in ~17 ms on every
# follower as objects (631 KB: too big for a plan-ring slot, so it went over
# gloo to each follower); as columns without the token ids -- which only a
# replica's stage 0 reads -- ~6 / ~7 ms and 182 KB, inline in the ring.
def _pack_group(gp: GroupPlan, ids: bool):
    import numpy as np

    ch = None
    if gp.chunks:
        c = gp.chunks
        tok = None
        if ids:
            import itertools

            tok = np.fromiter(itertools.chain.from_iterable(x.ids for x in c), dtype=np.int32,
                              count=sum(len(x.ids) for x in c))
        ch = (np.array([(x.seq, x.slot, x.start, len(x.ids), x.final, x.top_k, x.greedy) for x in c],
                       dtype=np.int64).reshape(-1, 7),
              np.array([x.temperature for x in c], dtype=np.float64),
              np.array([x.seed for x in c], dtype=np.int64), tok)
    rows = None
    if gp.rows is not None:
        r = gp.rows
        rows = (np.array([(x.seq, x.slot, x.pos, x.top_k, x.greedy, x.seed, x.step, x.src) for x in r],
                         dtype=np.int64).reshape(-1, 8),
                np.array([x.temperature for x in r], dtype=np.float64))
    return (gp.g, gp.ret, gp.n, gp.b, gp.ctxb, gp.kind, gp.fwd_rows, ch, rows)


def _unpack_group(g, ret, n, b, ctxb, kind, fwd_rows, ch, rows) -> GroupPlan:
    """Inverse of _pack_group.  Chunks sent without their token ids carry
    range(len) in their place (their stage reads only the lengths)."""
    gp = GroupPlan(g, ret=ret, n=n, b=b, ctxb=ctxb, kind=kind, fwd_rows=fwd_rows)
    if ch is not None:
        ints, temp, seeds, tok = ch
        tok = tok.tolist() if tok is not None else None
        out, o = [], 0
        for (seq, slot, start, ln, final, top_k, greedy), t, sd in zip(ints.tolist(), temp.tolist(),
                                                                      seeds.tolist()):
            out.append(Chunk(seq, slot, start, tok[o: o + ln] if tok is not None else range(ln), bool(final),
                             t, top_k, bool(greedy), sd))
            o += ln
        gp.chunks = out
    if rows is not None:
        ints, temp = rows
        gp.rows = [Row(seq, slot, pos, t, top_k, bool(greedy), seed, step, src)
                   for (seq, slot, pos, top_k, greedy, seed, step, src), t in zip(ints.tolist(), temp.tolist())]
    return gp


class _PlanPickler(pickle.Pickler):
    """Pickles every GroupPlan through _pack_group (ids: with token ids)."""

    def __init__(self, file, ids: bool):
        super().__init__(file, protocol=pickle.HIGHEST_PROTOCOL)
        self.ids = ids

    def reducer_override(self, obj):
        if type(obj) is GroupPlan:
            return _unpack_group, _pack_group(obj, self.ids)
        return NotImplemented


def _plan_dumps(plan: StepPlan, ids: bool) -> bytes:
    buf = io.BytesIO()
    _PlanPickler(buf, ids).dump(plan)
    return buf.getvalue()


class PlanEncoder:
    """Per-destination encoder (remembers what it sent last for REPEAT).
    ids=False: the destination stages never read prefill token ids (every
    stage but a replica's first), so the chunks travel without them."""

    def __init__(self, ids: bool = True):
        self._prev = None  # (step, replica, flags, groups) of the last plan sent
        self.ids = ids

    def encode(self, plan: StepPlan):
        """-> (int32 numpy record, pickle payload bytes or None)."""
        import numpy as np

        rec = np.zeros(PLAN_WORDS, dtype=np.int32)
        flags = (_F_TIMING if plan.timing else 0) | (_F_END if plan.end else 0) | (_F_STOP if plan.stop else 0)
        groups = _steady_groups(plan)
        if groups is None:
            payload = _plan_dumps(plan, self.ids)
            rec[0], rec[1] = MAGIC_PICKLE, len(payload)
            self._prev = None
            return rec, payload
        prev = self._prev
        if (prev is not None and plan.step == prev[0] + 1 and plan.replica == prev[1]
                and flags == prev[2] and groups == prev[3] and groups):
            rec[0], rec[1] = MAGIC_REPEAT, plan.step
        else:
            rec[0], rec[1], rec[2], rec[3], rec[4] = MAGIC_STEADY, plan.step, plan.replica, flags, len(groups)
            if groups:
                rec[5: 5 + 5 * len(groups)] = np.asarray(groups, dtype=np.int32).reshape(-1)
        self._prev = (plan.step, plan.replica, flags, groups)
        return rec, None


class PlanDecoder:
    """Per-source decoder (holds the previous plan's groups for REPEAT)."""

    def __init__(self):
        self._prev = None  # (replica, flags, groups)

    def decode(self, rec, fetch_payload) -> StepPlan:
        """rec: int32 sequence of PLAN_WORDS; fetch_payload(nbytes) -> bytes."""
        magic = int(rec[0])
        if magic == MAGIC_PICKLE:
            self._prev = None
            # our own plan records, produced by this job's rank 0
            return pickle.loads(fetch_payload(int(rec[1])))
        if magic == MAGIC_REPEAT:
            if self._prev is None:
                raise ValueError("plan REPEAT record without a previous plan")
            replica, flags, groups = self._prev
            step = int(rec[1])
        elif magic == MAGIC_STEADY:
            step, replica, flags, G = (int(x) for x in rec[1:5])
            vals = [int(x) for x in rec[5: 5 + 5 * G]]
            groups = [tuple(vals[5 * i: 5 * i + 5]) for i in range(G)]
            self._prev = (replica, flags, groups)
        else:
            raise ValueError(f"bad plan record magic {magic:#x}")
        # fresh GroupPlan objects every step (workers key posted receives by id)
        return StepPlan(step=step, replica=replica, timing=bool(flags & _F_TIMING),
                        end=bool(flags & _F_END), stop=bool(flags & _F_STOP),
                        groups=[GroupPlan(g, ret=r, n=n, b=b, ctxb=c) for g, r, n, b, c in groups])
