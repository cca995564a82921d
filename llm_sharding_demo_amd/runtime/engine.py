"""Inference engine: request batching, slot management, round execution.

Plays the reference coordinator's role (`server.py:154-210`: tokenize ->
decode loop -> detokenize), but the decode loop runs inside the stage
workers (parallel/pipeline.py) and only the final token ids come back.

Execution modes
  * local  -- all P stages live in this process.  P == 1 runs inline; P > 1
              runs one thread per stage over the in-memory LocalTransport
              (each stage may sit on its own device).  Used on CPU (tests)
              and for single-GPU runs.
  * dist   -- one process per MI355X under torchrun; rank r owns stage
              r % P of pipeline replica r // P (dp_replicas R, world = P*R).
              Rank 0 is the coordinator and also stage 0 of replica 0; other
              ranks sit in `worker_loop()` and receive per-replica round specs
              over a gloo control group.  Data moves over RCCL p2p
              (NcclTransport), one set of edge communicators per replica.
"""
from __future__ import annotations

import logging
import os
import random
import threading
import time
from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch

from ..config import EngineConfig, SamplingParams
from ..models.stage import StageModel
from ..parallel.comm import LocalFabric, Transport, init_distributed, make_dist_transport
from ..parallel.partition import make_unit_plan, units_to_layers
from ..parallel.pipeline import MicroBatchSpec, RoundResult, RoundSpec, StageWorker
from .kv_cache import SlotAllocator

log = logging.getLogger("llm_sharding_demo_amd.engine")


@dataclass
class GenerationOutput:
    prompt_ids: List[int]
    output_ids: List[int]


def _dtype(name: str, device: torch.device) -> torch.dtype:
    if device.type == "cpu":
        return torch.float32
    return {"bf16": torch.bfloat16, "fp32": torch.float32}[name]


def resolve_device(spec: str) -> torch.device:
    if spec == "auto":
        return torch.device("cuda" if torch.cuda.is_available() else "cpu")
    return torch.device(spec)


class Engine:
    def __init__(self, cfg: EngineConfig, mode: str = "local",
                 devices: Optional[Sequence[str]] = None, fault=None):
        self.cfg = cfg
        self.mcfg = cfg.model
        self.mode = mode
        self.P = cfg.num_stages
        self.R = max(1, cfg.dp_replicas)
        if mode == "local" and self.R != 1:
            raise ValueError("dp_replicas > 1 needs the dist mode (one process per GPU)")
        self.replica, self.stage_idx = 0, 0
        # stage ranges in half-layer units (parallel/partition.py); `plan` is
        # the layer view (a layer cut in half is listed in both stages)
        mb_rows = -(-cfg.max_batch // max(1, cfg.microbatches))
        self.unit_plan = make_unit_plan(self.mcfg, self.P, cfg.split_points, cfg.split_units,
                                        rows=mb_rows, avg_ctx=min(192, cfg.max_seq_len),
                                        half_layers=cfg.half_layer_split)
        self.plan = units_to_layers(self.unit_plan)
        self._rng = random.Random(cfg.seed)
        self.healthy = True
        self.last_error: Optional[str] = None
        self._lock = threading.Lock()
        self.stats = {"requests": 0, "tokens": 0, "rounds": 0, "busy_s": 0.0}
        self.last_round: Optional[RoundResult] = None
        self.round_started: Optional[float] = None  # monotonic start of the running round (watchdog)
        self.max_seq = min(cfg.max_seq_len, self.mcfg.max_positions)

        if mode == "local":
            if devices is None:
                dev = resolve_device(cfg.device)
                devices = [str(dev)] * self.P
            self.devices = [torch.device(d) for d in devices]
            self.stages = [self._build_stage(i, self.devices[i]) for i in range(self.P)]
            self.fabric = LocalFabric(self.P, fault=fault) if self.P > 1 else None
            self.workers = [StageWorker(st, self.fabric.transport(i) if self.fabric else None, i, self.P)
                            for i, st in enumerate(self.stages)]
            self.rank = 0
            self.transport: Optional[Transport] = None
        elif mode == "dist":
            import torch.distributed as dist

            dev = resolve_device(cfg.device)
            kind = cfg.transport if cfg.transport not in ("auto", "local") else (
                "nccl" if dev.type == "cuda" else "gloo")
            init_distributed("nccl" if kind == "nccl" else "gloo", dev.type, cfg.round_timeout_s)
            self.rank = dist.get_rank()
            if dev.type == "cuda":
                dev = torch.device("cuda", torch.cuda.current_device())
            self.devices = [dev]
            self.transport = make_dist_transport(self.P, kind, dev, self.R)
            self.replica, self.stage_idx = self.transport.replica, self.transport.rank
            stage = self._build_stage(self.stage_idx, dev)
            self.stages = [stage]
            self.workers = [StageWorker(stage, self.transport, self.stage_idx, self.P)]
            self.fabric = None
        else:
            raise ValueError(f"unknown mode {mode!r}")
        # one KV-slot pool per pipeline replica (the coordinator allocates for all)
        self.slot_pools = [_make_slot_allocator(self.stages[0].kv.slots) for _ in range(self.R)]
        self.slots = self.slot_pools[0]

    # ------------------------------------------------------------------
    def _build_stage(self, i: int, device: torch.device) -> StageModel:
        a, b = self.plan[i]
        return StageModel(self.mcfg, a, b, first=(i == 0), last=(i == self.P - 1), device=device,
                          dtype=_dtype(self.cfg.dtype, device), seed=self.cfg.seed,
                          weights_path=self.cfg.weights, max_slots=self.cfg.max_batch,
                          max_seq=self.max_seq, units=self.unit_plan[i])

    @property
    def is_coordinator(self) -> bool:
        return self.rank == 0

    # ------------------------------------------------------------------
    def _run_rounds(self, specs: List[Optional[RoundSpec]]) -> List[Optional[RoundResult]]:
        """One round per pipeline replica (None = replica idle this round)."""
        if self.mode != "dist":
            return [self._run_round(specs[0])]
        self.transport.broadcast_object(("round", specs), src=0)
        return self._dist_round(specs)

    def _dist_round(self, specs) -> List[Optional[RoundResult]]:
        spec = specs[self.replica]
        res = self.workers[0].run_round(spec) if spec is not None else None
        if any(sp is not None and sp.record_timing for sp in specs):
            # per-stage busy / bubble figures of every rank, to the coordinator
            stats = self.transport.gather_object(self.workers[0].last_stats if spec else None, dst=0)
            if stats is not None and res is not None:
                res.stages = [dict(st, replica=g // self.P) for g, st in enumerate(stats)
                              if st is not None]
        if self.R == 1:
            return [res]
        # stage 0 of every replica holds its replica's tokens; collect on rank 0
        got = self.transport.gather_object(res if self.stage_idx == 0 else None, dst=0)
        return None if got is None else [got[r * self.P] for r in range(self.R)]

    def _run_round(self, spec: RoundSpec) -> RoundResult:
        if self.mode == "dist":
            return self._run_rounds([spec] + [None] * (self.R - 1))[0]
        if self.P == 1:
            return self.workers[0].run_round(spec)
        results: List[Optional[RoundResult]] = [None] * self.P
        errors: List[BaseException] = []

        def run(i):
            try:
                if self.devices[i].type == "cuda":
                    torch.cuda.set_device(self.devices[i])
                results[i] = self.workers[i].run_round(spec)
            except BaseException as e:  # propagate to caller
                errors.append(e)

        threads = [threading.Thread(target=run, args=(i,), daemon=True) for i in range(self.P)]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        if errors:
            raise errors[0]
        if spec.record_timing:
            results[0].stages = [w.last_stats for w in self.workers if w.last_stats is not None]
        return results[0]

    def worker_loop(self) -> None:
        """Non-coordinator ranks: execute commands until 'stop'."""
        assert self.mode == "dist" and self.rank != 0
        while True:
            cmd = self.transport.broadcast_object(None, src=0)
            if cmd[0] == "round":
                self._dist_round(cmd[1])
            elif cmd[0] == "stop":
                self._close_dist()
                break
            else:
                raise RuntimeError(f"unknown command {cmd[0]!r}")

    def shutdown(self) -> None:
        if self.mode == "dist" and self.rank == 0:
            self.transport.broadcast_object(("stop",), src=0)
            self._close_dist()

    def _close_dist(self) -> None:
        """Orderly teardown: every rank reaches the barrier before any process
        group is destroyed, so no rank exits while a peer still has a gloo /
        RCCL connection open to it."""
        import torch.distributed as dist

        self.transport.barrier()
        if dist.is_initialized():
            dist.destroy_process_group()

    # ------------------------------------------------------------------
    def make_round(self, prompts: List[List[int]], params: List[SamplingParams], slots: List[int],
                   microbatches: Optional[int] = None, use_graphs: Optional[bool] = None,
                   record_timing: bool = False) -> RoundSpec:
        n = len(prompts)
        M = max(1, min(microbatches or self.cfg.microbatches, n))
        steps = max(p.max_new_tokens for p in params)
        bounds = [round(i * n / M) for i in range(M + 1)]
        mbs = []
        for j in range(M):
            a, b = bounds[j], bounds[j + 1]
            ps = params[a:b]
            mbs.append(MicroBatchSpec(
                slots=slots[a:b], prompts=[list(map(int, p)) for p in prompts[a:b]],
                temperature=[p.temperature for p in ps], top_k=[p.top_k for p in ps],
                greedy=[p.greedy for p in ps],
                seeds=[p.seed if p.seed is not None else self._rng.getrandbits(62) for p in ps]))
        g = self.cfg.use_graphs if use_graphs is None else use_graphs
        return RoundSpec(microbatches=mbs, steps=steps, use_graphs=g, record_timing=record_timing,
                         prefill_chunk=self.cfg.prefill_chunk)

    def generate_ids(self, prompts: List[List[int]], params, microbatches: Optional[int] = None,
                     record_timing: bool = False) -> List[List[int]]:
        """Generate continuations for a list of token-id prompts.  Returns the
        generated ids only (not including the prompt)."""
        if isinstance(params, SamplingParams):
            params = [params] * len(prompts)
        for p, sp in zip(prompts, params):
            sp.validate()
            if len(p) == 0:
                raise ValueError("prompt must contain at least one token")
            if len(p) + sp.max_new_tokens > self.max_seq:
                raise ValueError(f"prompt ({len(p)}) + max_new_tokens ({sp.max_new_tokens}) "
                                 f"exceeds the context limit {self.max_seq}")
        outs: List[List[int]] = [[] for _ in prompts]
        todo = [i for i, sp in enumerate(params) if sp.max_new_tokens > 0]
        cap, R = self.slots.capacity, self.R
        with self._lock:
            if not self.healthy:
                raise RuntimeError(f"engine unhealthy: {self.last_error}")
            for c0 in range(0, len(todo), cap * R):
                chunk = todo[c0:c0 + cap * R]
                # contiguous, balanced share per pipeline replica
                parts = [chunk[round(j * len(chunk) / R): round((j + 1) * len(chunk) / R)]
                         for j in range(R)]
                slots = [self.slot_pools[j].alloc(len(part)) if part else []
                         for j, part in enumerate(parts)]
                try:
                    specs = [self.make_round([prompts[i] for i in part], [params[i] for i in part],
                                             slots[j], microbatches, record_timing=record_timing)
                             if part else None for j, part in enumerate(parts)]
                    t0 = time.perf_counter()
                    self.round_started = time.monotonic()
                    try:
                        results = self._run_rounds(specs)
                    finally:
                        self.round_started = None
                    self.stats["busy_s"] += time.perf_counter() - t0
                    self.last_round = results[0]
                except Exception as e:
                    self.healthy = False
                    self.last_error = f"{type(e).__name__}: {e}"
                    raise
                finally:
                    for j, sl in enumerate(slots):
                        if sl:
                            self.slot_pools[j].free(sl)
                for part, res in zip(parts, results):
                    if not part:
                        continue
                    toks = torch.cat([t.t() for t in res.tokens], 0)  # [n, steps]
                    for row, i in enumerate(part):
                        ids = toks[row, : params[i].max_new_tokens].tolist()
                        if params[i].stop_at_eos and self.mcfg.eos_token_id in ids:
                            ids = ids[: ids.index(self.mcfg.eos_token_id) + 1]
                        outs[i] = ids
                self.stats["rounds"] += 1
        self.stats["requests"] += len(prompts)
        self.stats["tokens"] += sum(len(o) for o in outs)
        return outs

    # ------------------------------------------------------------------
    # Compat single-shard forwards (reference /forward and /forward_b)
    # ------------------------------------------------------------------
    def _local_forward_range(self, x, start_stage: int, end_stage: int, ids_len: int,
                             all_logits: bool):
        from .batch import BatchMeta

        slot = self.slots.alloc(1)
        try:
            out = x
            for i in range(start_stage, end_stage):
                st = self.stages[i]
                meta = BatchMeta.build(slot, [0], [ids_len], st.device)
                out = out.to(st.device)
                if st.last:
                    out = st.forward(meta, out, all_logits=all_logits)
                else:
                    out = st.forward(meta, out)
            return out
        finally:
            self.slots.free(slot)

    def forward_a(self, input_ids: List[int]) -> torch.Tensor:
        """Stage-0 output for a full sequence (reference ShardA, server.py:77-86)."""
        if self.mode != "local" or self.P < 2:
            raise RuntimeError("forward_a needs a local engine with >= 2 stages")
        ids = torch.tensor(input_ids, dtype=torch.int32, device=self.stages[0].device)
        return self._local_forward_range(ids, 0, 1, len(input_ids), False)

    def forward_b(self, hidden: torch.Tensor) -> torch.Tensor:
        """Remaining stages + ln_f + lm_head over all positions (ShardB, server.py:98-103)."""
        if self.mode != "local" or self.P < 2:
            raise RuntimeError("forward_b needs a local engine with >= 2 stages")
        h = hidden.reshape(-1, self.mcfg.hidden).float()
        out = self._local_forward_range(h, 1, self.P, h.shape[0], True)
        return out[:, : self.mcfg.vocab_size]


def _make_slot_allocator(n: int):
    """Native (C++) KV-slot allocator when built, Python twin otherwise."""
    from . import native

    mod = native.load()
    if mod is not None and os.environ.get("LSD_PY_RUNTIME", "0") != "1":
        return mod.SlotAllocator(n)
    return SlotAllocator(n)


def build_engine(cfg: EngineConfig, **kw) -> Engine:
    """Pick local vs dist from the environment (torchrun sets WORLD_SIZE)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world > 1:
        R = max(1, cfg.dp_replicas)
        if R == 1 and 1 < cfg.num_stages < world and world % cfg.num_stages == 0:
            R = world // cfg.num_stages  # NUM_STAGES given: the rest is data parallel
        if world % R:
            raise ValueError(f"WORLD_SIZE {world} is not a multiple of dp_replicas {R}")
        cfg = cfg.replace(num_stages=world // R, dp_replicas=R)
        return Engine(cfg, mode="dist", **kw)
    return Engine(cfg, mode="local", **kw)
