"""Shard-local KV cache + slot allocator.

The reference has no KV cache: every decode step re-sends and recomputes the
whole sequence on both shards (`server.py:169-181`, quirk Q5).  Here each
pipeline stage owns the K/V of ITS layers only, so the only thing that
crosses the inter-stage link per decode step is the boundary hidden state.

Layout (one allocation per stage):
    buf[layer, 0|1 (K|V), slot, kv_head, position, head_dim]   bf16 on GPU
Each (slot, head) row-block is contiguous over positions, so the decode
attention kernel streams K and V for one sequence/head as one linear 1 KiB-
per-wave-instruction read.  Sized for MI355X's 288 GB HBM: the engine asks
`plan_slots` for the slot count that fits the free-memory budget after the
stage's weights (runtime/engine.py `_kv_slots`, reported on /health and
/metrics); two extra slots hold decode pad rows and compat forwards.
"""
from __future__ import annotations

from typing import List

import torch


class KVCache:
    def __init__(self, n_layers: int, slots: int, n_kv: int, max_seq: int, head_dim: int,
                 dtype: torch.dtype, device):
        self.n_layers, self.slots, self.n_kv = n_layers, slots, n_kv
        self.max_seq, self.head_dim = max_seq, head_dim
        shape = (max(n_layers, 1), 2, slots, n_kv, max_seq, head_dim)
        self.buf = torch.zeros(shape, dtype=dtype, device=device)

    def k(self, layer: int) -> torch.Tensor:
        return self.buf[layer, 0]

    def v(self, layer: int) -> torch.Tensor:
        return self.buf[layer, 1]

    @property
    def nbytes(self) -> int:
        return self.buf.numel() * self.buf.element_size()

    @staticmethod
    def bytes_per_slot(n_layers: int, n_kv: int, max_seq: int, head_dim: int, elt: int = 2) -> int:
        return n_layers * 2 * n_kv * max_seq * head_dim * elt


def plan_slots(requested: int, n_layers: int, n_kv: int, max_seq: int, head_dim: int,
               device, fraction: float = 0.85, elt: int = 2, reserve: int = 0,
               mem_get_info=None) -> int:
    """Largest slot count <= requested whose KV fits `fraction` of the free
    device memory left after `reserve` bytes (the stage's weights, loaded
    after this is decided).  `mem_get_info` is injectable for tests."""
    dev = torch.device(device)
    if dev.type != "cuda" and mem_get_info is None:
        return requested
    free, _ = (mem_get_info or torch.cuda.mem_get_info)(dev)
    per = KVCache.bytes_per_slot(n_layers, n_kv, max_seq, head_dim, elt)
    if per == 0:  # a stage without attention halves holds no KV
        return requested
    fit = int(max(0, free - reserve) * fraction) // per
    if fit < 1:
        raise MemoryError(f"KV cache: one slot needs {per / 2**30:.2f} GiB, free {free / 2**30:.2f} GiB")
    return min(requested, fit)


class SlotAllocator:
    """Host-side free list of KV slots (native version: SlotAllocator in
    csrc/runtime/runtime.cpp)."""

    def __init__(self, n: int):
        self._free: List[int] = list(range(n - 1, -1, -1))
        self.capacity = n

    def alloc(self, k: int = 1) -> List[int]:
        if k > len(self._free):
            raise RuntimeError(f"out of KV slots: want {k}, have {len(self._free)}")
        return [self._free.pop() for _ in range(k)]

    def free(self, slots) -> None:
        for s in slots:
            self._free.append(int(s))

    @property
    def available(self) -> int:
        return len(self._free)
