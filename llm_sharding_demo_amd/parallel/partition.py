"""Layer partitioner: which blocks go to which pipeline stage.

Reference: a single split point `SPLIT_AT` read independently by every pod
(`server.py:22,63-64,108`).  With the shipped k8s manifests shard A uses 2
and shard B uses 1 (`k8s/shard-a-deployment.yaml:22-23`,
`k8s/shard-b-deployment.yaml:22-23`), so block 1 runs twice (quirk Q1).  Here
the plan has a single owner (the engine) and is validated to cover every
layer exactly once.

The engine partitions at half-layer granularity (`make_unit_plan`, below):
min-max DP over a per-unit decode time model calibrated on MI355X.  The
whole-layer API (`make_plan` / `auto_partition`, a bytes model) is kept for
explicit SPLIT_AT plans and the compat shard roles:
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


# ---------------------------------------------------------------------------
# Half-layer ("unit") partitioning
# ---------------------------------------------------------------------------
# A transformer block is two residual sub-blocks: unit 2i = attention half of
# layer i (norm, QKV + KV append, attention, output projection + residual),
# unit 2i+1 = MLP half (norm, up projection + activation, down projection +
# residual).  Between the two the residual stream x is the ONLY live state,
# exactly like between layers, so a stage boundary may sit after either half.
# With whole layers the last stage's lm_head + sampler can only be balanced in
# steps of one block: GPT-2 XL on 8 stages has 48 blocks + ~1.2 blocks of head,
# and any whole-layer split leaves a 7-block stage (86 % of ideal); half-layer
# cuts get within a few %.
#
# The cost model is decode time per microbatch per step (us) on MI355X,
# calibrated against the kernel profile and microbenchmarks of the bench
# configs (kernel-trace averages with the other microbatch lane running).
# Up to 64 rows (split-K decode GEMMs; profiles/r1_xl_*_kernel_stats.csv,
# r1_microbench_*):
#   decode GEMM  ~ 5 us + weight bytes / 1.3 TB/s + FLOPs / 2 PF
#   lm_head      ~ 5 us + bytes / 4.4 TB/s (128x128 tiled kernel)
# Above 64 rows (LDS-ring / big tiled GEMMs; profiles/r1_xl_b512_kernel_stats_v5.csv,
# GPT-2 XL 2 x 256: attention half 86.7 us, MLP half 36.5 us, head 138.8 us):
#   decode GEMM  ~ 6 us + FLOPs / 0.45 PF;  lm_head ~ 5 us + FLOPs / 0.55 PF
# Both: QKV + 6 us (KV-cache scatter, RoPE); attention ~ 3 us + KV bytes /
# 6 TB/s; norm 6 us; sampler 8 us + 0.37 us/row up to 128 rows (flat above:
# 57 us at 256 rows); embed 4 us.
UnitPlan = List[Tuple[int, int]]


def _gemm_us(n: int, k: int, rows: int) -> float:
    if rows > 64:
        if n >= 16384:  # vocab projection
            return 5.0 + 2.0 * rows * n * k / 0.55e9
        return 6.0 + 2.0 * rows * n * k / 0.45e9  # FLOPs per us
    if n >= 16384:  # vocab projection on the 128x128 tiled kernel
        return 5.0 + n * k * 2 / 4.4e6
    return 5.0 + n * k * 2 / 1.3e6 + 2.0 * rows * n * k / 2.0e9  # bytes, FLOPs per us


def unit_costs(cfg: ModelConfig, rows: int = 128, avg_ctx: int = 192) -> Tuple[List[float], float, float]:
    """(per-unit decode cost [2L], last-stage head cost, first-stage embed cost) in us."""
    h = cfg.hidden
    norm = 6.0
    attn = 3.0 + rows * avg_ctx * cfg.kv_bytes_per_token_per_layer() / 6.0e6
    if cfg.arch == "gpt2":
        up = _gemm_us(cfg.ffn, h, rows)
    else:
        up = _gemm_us(2 * cfg.ffn, h, rows)
    a = norm + _gemm_us(cfg.qkv_size, h, rows) + 6.0 + attn + _gemm_us(h, cfg.q_size, rows)
    m = norm + up + _gemm_us(h, cfg.ffn, rows)
    head = norm + _gemm_us(cfg.vocab_padded, h, rows) + 8.0 + 0.37 * min(rows, 128)
    embed = 4.0
    return [a, m] * cfg.n_layers, head, embed


def _minmax_dp(costs: Sequence[float], P: int, head: float) -> UnitPlan:
    """Exact min-max contiguous partition of `costs` into P non-empty parts;
    the last part also pays `head` (Python twin of the native runtime's
    partition_minmax)."""
    n = len(costs)
    if not 1 <= P <= n:
        raise ValueError(f"cannot split {n} units into {P} non-empty stages")
    pre = [0.0]
    for c in costs:
        pre.append(pre[-1] + c)
    INF = float("inf")
    best = [[INF] * (n + 1) for _ in range(P + 1)]
    arg = [[0] * (n + 1) for _ in range(P + 1)]
    best[0][0] = 0.0
    for p in range(1, P + 1):
        for i in range(p, n - (P - p) + 1):
            for j in range(p - 1, i):
                c = pre[i] - pre[j] + (head if p == P else 0.0)
                v = max(best[p - 1][j], c)
                if v < best[p][i]:
                    best[p][i], arg[p][i] = v, j
    plan: UnitPlan = []
    i = n
    for p in range(P, 0, -1):
        j = arg[p][i]
        plan.append((j, i))
        i = j
    plan.reverse()
    return plan


def validate_unit_plan(plan: UnitPlan, n_layers: int) -> None:
    validate_plan(plan, 2 * n_layers)
    if any(b <= a for a, b in plan):
        raise ValueError(f"unit plan {plan} has an empty stage")


def unit_stage_costs(cfg: ModelConfig, plan: UnitPlan, rows: int = 128, avg_ctx: int = 192) -> List[float]:
    costs, head, embed = unit_costs(cfg, rows, avg_ctx)
    out = []
    for s, (a, b) in enumerate(plan):
        c = sum(costs[a:b]) + (embed if s == 0 else 0.0) + (head if s == len(plan) - 1 else 0.0)
        out.append(c)
    return out


def make_unit_plan(cfg: ModelConfig, num_stages: int, split_points: Optional[Sequence[int]] = None,
                   split_units: Optional[Sequence[int]] = None, rows: int = 128,
                   avg_ctx: int = 192, half_layers: bool = True) -> UnitPlan:
    """Stage ranges in half-layer units.  Explicit `split_units` (unit
    boundaries) or `split_points` (layer boundaries, SPLIT_AT) win; otherwise
    the min-max DP over the unit cost model, at half-layer granularity unless
    `half_layers` is False (then whole layers only)."""
    L, P = cfg.n_layers, num_stages
    if split_units:
        pts = [0] + list(split_units) + [2 * L]
        plan = [(pts[i], pts[i + 1]) for i in range(len(pts) - 1)]
    elif split_points:
        plan = [(2 * a, 2 * b) for a, b in make_plan(cfg, P, split_points)]
    elif P == 1:
        plan = [(0, 2 * L)]
    else:
        costs, head, embed = unit_costs(cfg, max(1, min(rows, 256)), avg_ctx)
        if half_layers:
            plan = _native_or_python_dp(costs, P, head, embed)
        else:
            layer = [costs[2 * i] + costs[2 * i + 1] for i in range(L)]
            plan = [(2 * a, 2 * b) for a, b in _native_or_python_dp(layer, P, head, embed)]
    if len(plan) != P:
        raise ValueError(f"unit plan {plan} has {len(plan)} stages, but num_stages={P}")
    validate_unit_plan(plan, L)
    return plan


def _native_or_python_dp(costs, P, head, first) -> UnitPlan:
    import os

    from ..runtime import native

    costs = list(costs)
    costs[0] += first  # stage 0 always owns unit 0
    if not 1 <= P <= len(costs):
        raise ValueError(f"cannot split {len(costs)} units into {P} non-empty stages")
    mod = native.load()
    if mod is not None and os.environ.get("LSD_PY_RUNTIME", "0") != "1":
        return [tuple(x) for x in mod.partition_minmax(costs, P, head)]
    return _minmax_dp(costs, P, head)


# ---------------------------------------------------------------------------
# Alternating splits: two unit plans, one per microbatch-group parity
# ---------------------------------------------------------------------------
# Half-layer units are still coarse against a stage's share: GPT-2 XL on 8
# stages (attention half ~83 us, MLP half ~37 us at 256 rows, ~738 us per
# stage) leaves one stage with 7 attention halves, 91 % of an even split.
# Groups of even index run plan A, odd groups plan B; at every boundary the
# two plans cut at most one unit apart, so a stage's work per decode step (the
# sum over its groups) is the MEAN of its two ranges -- quarter-layer
# granularity on average with the same wire protocol (only the fp32 residual
# crosses a boundary).  A stage holds the weights and KV layers of the union
# of its two ranges (at most one extra half-layer per side); a sequence never
# changes group, so each variant's KV cache stays on one stage.
def _alt_dp(costs: Sequence[float], P: int, head: float) -> Tuple[UnitPlan, UnitPlan]:
    """Min-max over the mean of two contiguous partitions.  Position p in
    [0, 2n] cuts plan A at unit p // 2 and plan B at (p + 1) // 2; a stage
    spans positions p1 -> p2 >= p1 + 2 (non-empty in both plans)."""
    n = len(costs)
    if not 1 <= P <= n:
        raise ValueError(f"cannot split {n} units into {P} non-empty stages")
    pre = [0.0]
    for c in costs:
        pre.append(pre[-1] + c)

    def seg(p1: int, p2: int) -> float:
        return 0.5 * ((pre[p2 // 2] - pre[p1 // 2]) + (pre[(p2 + 1) // 2] - pre[(p1 + 1) // 2]))

    N2 = 2 * n
    INF = float("inf")
    best = [[INF] * (N2 + 1) for _ in range(P + 1)]
    arg = [[0] * (N2 + 1) for _ in range(P + 1)]
    best[0][0] = 0.0
    for k in range(1, P + 1):
        lo, hi = 2 * k, N2 - 2 * (P - k)
        for p2 in (range(lo, hi + 1) if k < P else [N2]):
            for p1 in range(2 * (k - 1), p2 - 1):
                if best[k - 1][p1] == INF:
                    continue
                v = max(best[k - 1][p1], seg(p1, p2) + (head if k == P else 0.0))
                if v < best[k][p2]:
                    best[k][p2], arg[k][p2] = v, p1
    cuts = [N2]
    for k in range(P, 0, -1):
        cuts.append(arg[k][cuts[-1]])
    cuts.reverse()
    plan_a = [(cuts[k] // 2, cuts[k + 1] // 2) for k in range(P)]
    plan_b = [((cuts[k] + 1) // 2, (cuts[k + 1] + 1) // 2) for k in range(P)]
    return plan_a, plan_b


def make_alt_unit_plans(cfg: ModelConfig, num_stages: int, rows: int = 128,
                        avg_ctx: int = 192) -> Tuple[UnitPlan, UnitPlan]:
    """(plan A, plan B) for even / odd microbatch groups (see _alt_dp)."""
    P = num_stages
    if P == 1:
        return [(0, 2 * cfg.n_layers)], [(0, 2 * cfg.n_layers)]
    costs, head, embed = unit_costs(cfg, max(1, min(rows, 256)), avg_ctx)
    costs = list(costs)
    costs[0] += embed
    plan_a, plan_b = _alt_dp(costs, P, head)
    for pl in (plan_a, plan_b):
        validate_unit_plan(pl, cfg.n_layers)
    return plan_a, plan_b


def alt_stage_costs(cfg: ModelConfig, plans: Tuple[UnitPlan, UnitPlan], rows: int = 128,
                    avg_ctx: int = 192) -> List[float]:
    """Mean per-stage cost of the two plans (what a decode step pays)."""
    a = unit_stage_costs(cfg, plans[0], rows, avg_ctx)
    b = unit_stage_costs(cfg, plans[1], rows, avg_ctx)
    return [(x + y) / 2 for x, y in zip(a, b)]


def union_plan(plans: Tuple[UnitPlan, UnitPlan]) -> UnitPlan:
    """Per stage, the units either plan runs there (weights, KV layers)."""
    return [(min(a0, a1), max(b0, b1)) for (a0, b0), (a1, b1) in zip(*plans)]


def units_to_layers(plan: UnitPlan) -> Plan:
    """Layers each stage touches (a layer cut in half appears in both stages)."""
    return [(a // 2, (b + 1) // 2) for a, b in plan]
