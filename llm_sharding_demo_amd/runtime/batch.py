"""Batch metadata + sampling state shared by every stage.

A forward step processes a *packed* set of query tokens (prefill: many per
sequence, decode: one per sequence).  Every stage of the pipeline holds an
identical copy of the metadata for each microbatch, so no metadata crosses
the inter-stage link (only the boundary hidden state does).

In decode, positions advance on the device (`advance()`), which keeps the
step graph-capturable: the hipGraph replays the same kernels, and the kernels
read lengths from these device tensors.

The reference has batch == 1 and recomputes the whole sequence every step
(`server.py:137,169-181`, quirks Q5/Q12); this replaces both.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch


@dataclass
class BatchMeta:
    token_slots: torch.Tensor  # int32 [T]  KV slot of each packed query token
    token_pos: torch.Tensor  # int32 [T]  position of each packed query token
    seq_slots: torch.Tensor  # int32 [B]
    q_start: torch.Tensor  # int32 [B]  position of each sequence's first query
    cu_q: torch.Tensor  # int32 [B+1] packed row offsets
    last_idx: torch.Tensor  # int32 [B]  packed row of each sequence's last query
    num_tokens: int
    num_seqs: int
    max_q: int
    max_ctx: int  # upper bound on q_start + qlen (host-side, for grid sizing)
    is_decode: bool
    host_qlens: Optional[List[int]] = None  # per-sequence query counts (host copy)
    # decode buckets (runtime/plan.py): 1 for real rows, 0 for pad rows, which
    # never advance (they stay on position 0 of the scratch KV slot)
    active: Optional[torch.Tensor] = None

    @staticmethod
    def build(slots: Sequence[int], starts: Sequence[int], qlens: Sequence[int],
              device, max_ctx: Optional[int] = None) -> "BatchMeta":
        tslots: List[int] = []
        tpos: List[int] = []
        cu = [0]
        for s, st, n in zip(slots, starts, qlens):
            tslots += [s] * n
            tpos += list(range(st, st + n))
            cu.append(cu[-1] + n)
        i32 = dict(dtype=torch.int32, device=device)
        T = cu[-1]
        B = len(slots)
        mc = max((st + n for st, n in zip(starts, qlens)), default=0)
        return BatchMeta(
            token_slots=torch.tensor(tslots, **i32),
            token_pos=torch.tensor(tpos, **i32),
            seq_slots=torch.tensor(list(slots), **i32),
            q_start=torch.tensor(list(starts), **i32),
            cu_q=torch.tensor(cu, **i32),
            last_idx=torch.tensor([c - 1 for c in cu[1:]], **i32),
            num_tokens=T, num_seqs=B, max_q=max(qlens, default=0),
            max_ctx=max_ctx if max_ctx is not None else mc,
            is_decode=all(n == 1 for n in qlens), host_qlens=list(qlens))

    @staticmethod
    def decode(slots: Sequence[int], positions: Sequence[int], device,
               max_ctx: int) -> "BatchMeta":
        """Decode batch: one query per sequence.  token_pos IS q_start (shared
        storage), so `advance()` moves both."""
        i32 = dict(dtype=torch.int32, device=device)
        B = len(slots)
        pos = torch.tensor(list(positions), **i32)
        sl = torch.tensor(list(slots), **i32)
        ar = torch.arange(B + 1, **i32)
        return BatchMeta(token_slots=sl, token_pos=pos, seq_slots=sl, q_start=pos,
                         cu_q=ar, last_idx=ar[:B], num_tokens=B, num_seqs=B, max_q=1,
                         max_ctx=max_ctx, is_decode=True, host_qlens=[1] * B)

    def advance(self) -> None:
        """Decode only: every (active) sequence moves one position forward (in place)."""
        assert self.is_decode
        if self.active is None:
            self.token_pos.add_(1)
        else:
            self.token_pos.add_(self.active)


@dataclass
class MixedMeta:
    """One forward over a group's decode rows AND the prefill chunks joining
    it in the same step (parallel/pipeline.py _mixed): rows [0, b) are the
    decode rows (`dec`, the group's captured-bucket meta), rows [b, b + T) the
    chunk tokens (`pf`).  Every row-wise op (norms, GEMMs, the QKV epilogue's
    KV append at `token_slots` / `token_pos`) runs once over all rows, so the
    weights are read once per step instead of once for the decode graph and
    again for the prefill forward; the attention runs per part
    (models/stage.py _attn_out)."""
    token_slots: torch.Tensor  # int32 [b + T]
    token_pos: torch.Tensor    # int32 [b + T]
    b: int
    dec: BatchMeta
    pf: BatchMeta
    num_tokens: int
    is_decode: bool = False
    routing_decode: bool = True  # decode-shaped routing rules while b + T <= 512 rows



class SamplingState:
    """Per-row sampling parameters living on the device of the last stage.

    Random draws use a counter-based generator keyed by (seed, step), so a
    seeded request is reproducible regardless of batching or stage count.
    """

    def __init__(self, temperature, top_k, greedy, seeds, device):
        self.device = torch.device(device)
        B = len(temperature)
        self.temperature = torch.tensor(temperature, dtype=torch.float32, device=device)
        self.top_k = torch.tensor(top_k, dtype=torch.int32, device=device)
        self.greedy = torch.tensor([1 if g else 0 for g in greedy], dtype=torch.int32, device=device)
        self.seeds = torch.tensor(seeds, dtype=torch.int64, device=device)
        self.step = torch.zeros(B, dtype=torch.int64, device=device)
        self.num_rows = B

    def uniforms(self) -> torch.Tensor:
        """U[0,1) per row from (seed, step); host reference of the device hash."""
        return counter_uniform(self.seeds, self.step)

    def advance(self) -> None:
        self.step.add_(1)


def _mix64(z: torch.Tensor) -> torch.Tensor:
    # splitmix64 finalizer in int64 arithmetic (wrap-around); identical to the
    # device implementation in csrc/kernels/sample.hip.
    z = z + (0x9E3779B97F4A7C15 - (1 << 64))
    z = (z ^ _lsr(z, 30)) * (0xBF58476D1CE4E5B9 - (1 << 64))
    z = (z ^ _lsr(z, 27)) * (0x94D049BB133111EB - (1 << 64))
    return z ^ _lsr(z, 31)


def _lsr(z: torch.Tensor, n: int) -> torch.Tensor:
    return (z >> n) & ((1 << (64 - n)) - 1)


def counter_uniform(seeds: torch.Tensor, step: torch.Tensor) -> torch.Tensor:
    z = _mix64(seeds.to(torch.int64) * 0x100000001B3 + step.to(torch.int64))
    return _lsr(z, 40).to(torch.float64).div(float(1 << 24)).to(torch.float32)
