"""Layer partitioner: which blocks go to which pipeline stage.

Reference: a single split point `SPLIT_AT` read independently by every pod
(`server.py:22,63-64,108`).  With the shipped k8s manifests shard A uses 2
and shard B uses 1 (`k8s/shard-a-deployment.yaml:22-23`,
`k8s/shard-b-deployment.yaml:22-23`), so block 1 runs twice (quirk Q1).  Here
the plan has a single owner (the engine) and is validated to cover every
layer exactly once.

Auto partitioning minimises the slowest stage under a decode cost model in
bytes streamed from HBM per step (decode is bandwidth-bound on MI355X):
  block i : weight bytes + KV bytes (batch * avg ctx * per-layer KV)
  + a fixed per-block launch overhead expressed in bytes (~1.3 us/kernel
    boundary * 7 kernels at ~5 TB/s)
  last stage additionally streams lm_head (vocab x hidden; 2.6 blocks' worth
  for GPT-2 XL, 5.4 for GPT-2 small -- SURVEY.md §7.4 item 4).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

from ..config import ModelConfig

Plan = List[Tuple[int, int]]


def plan_from_splits(n_layers: int, splits: Sequence[int]) -> Plan:
    pts = [0] + list(splits) + [n_layers]
    plan = [(pts[i], pts[i + 1]) for i in range(len(pts) - 1)]
    validate_plan(plan, n_layers)
    return plan


def validate_plan(plan: Plan, n_layers: int) -> None:
    if not plan:
        raise ValueError("empty partition plan")
    expect = 0
    for a, b in plan:
        if a != expect or b < a:
            raise ValueError(f"partition {plan} does not tile layers 0..{n_layers} exactly once")
        expect = b
    if expect != n_layers:
        raise ValueError(f"partition {plan} covers {expect} of {n_layers} layers")


def stage_costs(cfg: ModelConfig, plan: Plan, batch: int = 32, avg_ctx: int = 256,
                dtype_bytes: int = 2) -> List[float]:
    blk = cfg.block_params() * dtype_bytes
    kv = batch * avg_ctx * cfg.kv_bytes_per_token_per_layer(dtype_bytes)
    overhead = 7 * 1.3e-6 * 5e12
    head = cfg.lm_head_params() * dtype_bytes + batch * cfg.vocab_padded * 8
    costs = []
    for s, (a, b) in enumerate(plan):
        c = (b - a) * (blk + kv + overhead)
        if s == len(plan) - 1:
            c += head
        costs.append(c)
    return costs


def auto_partition(cfg: ModelConfig, num_stages: int, batch: int = 32, avg_ctx: int = 256) -> Plan:
    """Min-max contiguous partition (exact DP over split points)."""
    L, P = cfg.n_layers, num_stages
    if P < 1:
        raise ValueError("num_stages must be >= 1")
    if P > L:
        raise ValueError(f"cannot split {L} layers into {P} non-empty stages")
    blk = stage_costs(cfg, [(0, 1)], batch, avg_ctx)[0] if L else 0.0
    head = stage_costs(cfg, [(0, 0)], batch, avg_ctx)[0]
    INF = float("inf")
    # best[p][i] = min over partitions of layers[0:i] into p stages of the max stage cost
    best = [[INF] * (L + 1) for _ in range(P + 1)]
    arg = [[0] * (L + 1) for _ in range(P + 1)]
    best[0][0] = 0.0
    for p in range(1, P + 1):
        for i in range(p, L - (P - p) + 1):
            for j in range(p - 1, i):
                c = (i - j) * blk + (head if p == P else 0.0)
                v = max(best[p - 1][j], c)
                if v < best[p][i]:
                    best[p][i], arg[p][i] = v, j
    plan: Plan = []
    i = L
    for p in range(P, 0, -1):
        j = arg[p][i]
        plan.append((j, i))
        i = j
    plan.reverse()
    validate_plan(plan, L)
    return plan


def make_plan(cfg: ModelConfig, num_stages: int, split_points: Optional[Sequence[int]] = None,
              batch: int = 32, avg_ctx: int = 256) -> Plan:
    if split_points:
        plan = plan_from_splits(cfg.n_layers, split_points)
        if len(plan) != num_stages:
            raise ValueError(f"{len(split_points)} split points give {len(plan)} stages, "
                             f"but num_stages={num_stages}")
        return plan
    if num_stages == 1:
        return [(0, cfg.n_layers)]
    return auto_partition(cfg, num_stages, batch, avg_ctx)
