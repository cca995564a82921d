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
