"""Inference engine: stages, KV slots, the continuous-batching driver loop.

Plays the reference coordinator's role (`server.py:154-210`: tokenize ->
decode loop -> detokenize), but the decode loop runs inside the stage
workers (parallel/pipeline.py) and only sampled token ids come back.

Execution modes
  * local  -- all P stages live in this process.  Stage 0 runs on the
              driving thread; stages 1..P-1 are persistent worker threads fed
              with step plans through in-process queues, exchanging tensors
              over the in-memory LocalTransport (each stage may sit on its own
              device).  Used on CPU (tests) and for single-GPU runs.
  * dist   -- one process per MI355X under torchrun; rank r owns stage
              r % P of pipeline replica r // P (dp_replicas R, world = P*R).
              Rank 0 runs the scheduler (and stage 0 of replica 0); every
              other rank sits in `worker_loop()` executing the step plans it
              receives on the gloo plan channel.  Data moves over RCCL p2p
              (NcclTransport), one set of edge communicators per replica;
              replica stage-0 ranks ship their sampled ids back to rank 0.

Every request goes through `Scheduler` (runtime/scheduler.py): requests join
and leave microbatch groups at decode-step boundaries (iteration-level
batching), so a short request finishes while a long one keeps decoding.
"""
from __future__ import annotations

import logging
import os
import queue
import random
import statistics
import threading
import gc
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import torch

from ..config import EngineConfig, SamplingParams
from ..utils import racecheck
from ..models.stage import StageModel
from ..parallel.comm import (DeviceLoopFabric, GlooPlanChannel, LocalFabric, LocalPlanChannel,
                             Transport, TransportError, init_distributed, make_plan_channel,
                             open_data_plane, transport_chain)
from ..parallel.partition import make_alt_unit_plans, make_unit_plan, union_plan, units_to_layers
from ..parallel.pipeline import StageWorker
from .kv_cache import KVCache, SlotAllocator, plan_slots
from .plan import GroupPlan, StepPlan
from .scheduler import Request, Scheduler

log = logging.getLogger("llm_sharding_demo_amd.engine")


@dataclass
class SessionStats:
    """Timing of the last timed session (bench, sampled serving steps)."""
    step_times_ms: List[float] = field(default_factory=list)
    prefill_ms: float = 0.0
    stages: List[dict] = field(default_factory=list)


def _dtype(name: str, device: torch.device) -> torch.dtype:
    if device.type == "cpu":
        return torch.float32
    return {"bf16": torch.bfloat16, "fp32": torch.float32}[name]


def resolve_device(spec: str) -> torch.device:
    if spec == "auto":
        return torch.device("cuda" if torch.cuda.is_available() else "cpu")
    return torch.device(spec)


class Engine(racecheck.Shared):
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
        self.M = max(1, cfg.microbatches)                # microbatch groups per replica
        self.group_cap = -(-cfg.max_batch // self.M)     # decode rows per group
        # stage ranges in half-layer units (parallel/partition.py); `plan` is
        # the layer view (a layer cut in half is listed in both stages)
        self.unit_plan = make_unit_plan(self.mcfg, self.P, cfg.split_points, cfg.split_units,
                                        rows=self.group_cap, avg_ctx=min(192, cfg.max_seq_len),
                                        half_layers=cfg.half_layer_split)
        # alternating splits: even / odd microbatch groups run plans A / B,
        # cut at most one unit apart, so each stage pays the mean of two
        # ranges (GPT-2 XL on 8 stages: 92 -> 97 % of an even split); the
        # stage holds the union.  Needs an even group count and the
        # cost-model partition (no explicit split points).
        self.unit_plans = None
        if (self.P > 1 and self.M % 2 == 0 and not cfg.split_points and not cfg.split_units
                and cfg.half_layer_split and os.environ.get("LSD_ALT_SPLIT", "1") != "0"):
            pa, pb = make_alt_unit_plans(self.mcfg, self.P, rows=self.group_cap,
                                         avg_ctx=min(192, cfg.max_seq_len))
            if pa != pb:
                self.unit_plans = (pa, pb)
                self.unit_plan = union_plan(self.unit_plans)
        self.plan = units_to_layers(self.unit_plan)
        self._rng = random.Random(cfg.seed)
        self.healthy = True
        self.last_error: Optional[str] = None
        self._lock = racecheck.RLock("engine")
        # watchdog: per-thread monotonic start of the step each thread is inside (the
        # serving driver and, in local mode, every stage follower); one shared slot
        # let a follower's "done" clear the driver's in-flight start (found by
        # utils/racecheck.py: two writers, no common lock)
        self._rounds: Dict[int, Optional[float]] = {}
        self.max_seq = min(cfg.max_seq_len, self.mcfg.max_positions)
        self.last_session: Optional[SessionStats] = None
        self.loop_thread: Optional[threading.Thread] = None
        self._stop_loop = threading.Event()
        self._wake = threading.Event()  # a request was submitted (serving loop)
        # LSD_HOST_PROFILE=1: host seconds in (plan, issue, readout wait), steps,
        # items, issuing-thread CPU, plan-send seconds, plan bytes sent
        # [plan s, issue s, readout wait s, decode steps, items, issuing CPU s, plan send s, plan bytes,
        #  then steps with prefill chunks: issue s, readout wait s, steps]
        self._hostprof = ([0.0, 0.0, 0.0, 0, 0, 0.0, 0.0, 0, 0.0, 0.0, 0]
                          if os.environ.get("LSD_HOST_PROFILE") == "1" else None)
        # LSD_HOST_PROFILE: host-clock seconds per session phase, summed over sessions
        self._phases: Optional[Dict[str, float]] = {} if self._hostprof is not None else None
        self.kv_slots = 0
        self._stall_after: Optional[int] = None  # test hook, see _test_stall
        # dist mode: the data plane in use and why the preferred one was left
        self.transport_kind: Optional[str] = None
        self.transport_fallback: Optional[str] = None

        if mode == "local":
            if devices is None:
                dev = resolve_device(cfg.device)
                devices = [str(dev)] * self.P
            self.devices = [_with_index(torch.device(d)) for d in devices]
            on_gpu = self.devices[0].type == "cuda"
            # "devloop": device loopback channels with graph I/O and the native
            # executor at P > 1 -- the single-GPU rehearsal of the RCCL data
            # plane (parallel/comm.py DeviceLoopFabric), allocated before the
            # KV cache sizes itself from free HBM.  "loopback": device-async
            # event hand-off between stage threads.  "strict": host queues per
            # (edge, lane) with receive-size checks and the graph-I/O code path
            # (CPU protocol tests).  Else plain host queues.
            kind = {"loopback": "loopback" if on_gpu else "local",
                    "devloop": "devloop" if on_gpu else "strict",
                    "strict": "strict"}.get(cfg.transport, "local")
            self.fabric = None
            if self.P > 1:
                self.fabric = (self._devloop_fabric(self.devices[0]) if kind == "devloop"
                               else LocalFabric(self.P, fault=fault))
            self.kv_slots = self._kv_slots(self.devices)
            self.stages = [self._build_stage(i, self.devices[i]) for i in range(self.P)]
            self.workers = [self._worker(st, self.fabric.transport(i, kind) if self.fabric else None, i)
                            for i, st in enumerate(self.stages)]
            self.rank = 0
            self.transport: Optional[Transport] = None
            self.plan_ch = LocalPlanChannel(list(range(1, self.P)))
            self._follow_err: Optional[BaseException] = None
            self._stats_q: "queue.Queue" = queue.Queue()
            self._followers = [threading.Thread(target=self._local_follower, args=(i,), daemon=True,
                                                name=f"lsd-stage{i}") for i in range(1, self.P)]
            for t in self._followers:
                t.start()
        elif mode == "dist":
            import torch.distributed as dist

            dev = resolve_device(cfg.device)
            # default group: gloo (control plane) unless the chain is torch's
            # RCCL groups alone; a fallback to "nccl" makes its own groups
            pre = transport_chain(cfg.transport, dev.type)
            init_distributed("nccl" if pre == ["nccl"] else "gloo", dev.type, cfg.round_timeout_s)
            self.rank = dist.get_rank()
            if dev.type == "cuda":
                dev = torch.device("cuda", torch.cuda.current_device())
            self.devices = [dev]
            shared = dev.type == "cuda" and _ranks_sharing_device(dev, None) > 1
            chain = transport_chain(cfg.transport, dev.type, shared)
            self.transport, self.transport_kind, self.transport_fallback = open_data_plane(
                chain, self.P, dev, self.R, cfg.round_timeout_s, loop_ring_bytes=self._loop_ring_bytes())
            if self.transport_fallback and self.rank == 0:
                log.warning("data plane %s failed its self-test; running on %s (%s)", chain[0],
                            self.transport_kind, self.transport_fallback)
            self.replica, self.stage_idx = self.transport.replica, self.transport.rank
            if os.environ.get("LSD_TEST_STALL_RANK") == str(self.rank):
                self._stall_after = int(os.environ.get("LSD_TEST_STALL_AFTER", "0"))
            self.kv_slots = self._kv_slots([dev], collective=True)
            stage = self._build_stage(self.stage_idx, dev)
            if os.environ.get("LSD_TEST_HOOKS") == "1" and os.environ.get("LSD_TEST_CORRUPT_RANK") == str(self.rank):
                # test hook (needs LSD_TEST_HOOKS=1): a faulty stage (doubled
                # norm gains) whose output must fail bench.py's token check
                log.warning("LSD_TEST_CORRUPT_RANK: rank %d doubles its norm gains (test hook)", self.rank)
                for k, t in stage.w.items():
                    if k.endswith(("ln_1.weight", "ln_2.weight", "layernorm.weight")):
                        t.mul_(2.0)
            self.stages = [stage]
            self.workers = [self._worker(stage, self.transport, self.stage_idx)]
            self.fabric = None
            # step plans: shared-memory ring per replica on one node, binary
            # gloo records otherwise (LSD_PLAN_WIRE=shm|binary|pickle)
            self.plan_ch = make_plan_channel(self.transport, cfg.round_timeout_s)
            self.tok_ch = GlooPlanChannel(self.transport.tok_pg, tag=3, plans=False)
            self._tok_threads: List[threading.Thread] = []
            if self.rank == 0:
                for rep in range(1, self.R):
                    t = threading.Thread(target=self._tok_receiver, args=(rep,), daemon=True)
                    t.start()
                    self._tok_threads.append(t)
            elif self.stage_idx == 0:
                self._tok_q: "queue.Queue" = queue.Queue()
                t = threading.Thread(target=self._tok_shipper, daemon=True)
                t.start()
                self._tok_threads.append(t)
                self.workers[0].readout = self._ship_readout
        else:
            raise ValueError(f"unknown mode {mode!r}")
        # dist mode: every rank watches its own progress and data plane (a
        # follower stuck behind a dead peer aborts its communicators too);
        # the device-loopback rehearsal has a data plane to abort as well
        self.data_plane = self.transport if mode == "dist" else (
            self.fabric if isinstance(self.fabric, DeviceLoopFabric) else None)
        self.watchdog = None
        if self.data_plane is not None and cfg.round_timeout_s > 0:
            from .scheduler import Watchdog

            self.watchdog = Watchdog(self, cfg.round_timeout_s)
        # one KV-slot pool per pipeline replica (the scheduler allocates for all)
        self.slot_pools = [_make_slot_allocator(self.kv_slots) for _ in range(self.R)]
        self.slots = self.slot_pools[0]
        self.scheduler = Scheduler(self, self.M, self.group_cap)
        if self.rank == 0:
            self.workers[0].readout = self.scheduler.on_readout
            self.workers[0].readout_native = self.scheduler.on_readout_native
        for w in self.workers:
            w.use_graphs = cfg.use_graphs
            w.configure(self.M, self.group_cap)

    # ------------------------------------------------------------------
    def _round(self, t: Optional[float]) -> None:
        self._rounds[threading.get_ident()] = t  # each thread writes only its own key

    @property
    def round_started(self) -> Optional[float]:
        """Start of the oldest step some thread is inside (None: none in flight)."""
        starts = [v for v in list(self._rounds.values()) if v is not None]
        return min(starts) if starts else None

    def _kv_slots(self, devices, collective: bool = False) -> int:
        """KV slots per stage: max_batch, capped by what fits the KV budget of
        free HBM (288 GB per MI355X) after the weights.  In
        dist mode every rank computes its own cap and all take the minimum."""
        want = self.cfg.max_batch
        fits = want
        # stages sharing a device (the 1-GPU loopback rehearsal) share its HBM:
        # sum their weights and their KV layers (every stage holds the same
        # slot count) before sizing the slots against that device's budget
        per_dev: dict = {}
        for i, dev in enumerate(devices):
            if dev.type != "cuda":
                continue
            si = self.stage_idx if collective else i
            a, b = self.unit_plan[si]  # the stage's KV layers: its attention halves
            acc = per_dev.setdefault(str(dev), [dev, 0, 0])
            acc[1] += sum(1 for u in range(a, b) if u % 2 == 0)
            acc[2] += self._weight_bytes(si)
        # dist ranks sharing one GPU (the single-GPU rehearsal of a multi-GPU
        # run): each takes an equal share of the device's memory instead of a
        # fraction of whatever the ranks initialised before it left free
        share = None
        if collective and torch.cuda.is_available() and any(d.type == "cuda" for d in devices):
            per_gpu = self._ranks_sharing_device(devices[0])
            if per_gpu > 1:
                def share(d, n=per_gpu):
                    free, total = torch.cuda.mem_get_info(d)
                    return min(free, int(total * 0.9) // n), total
        for dev, n_kv_layers, w_bytes in per_dev.values():
            fits = min(fits, plan_slots(want + 2, n_kv_layers, self.mcfg.n_kv_heads, self.max_seq,
                                        self.mcfg.head_dim, dev, reserve=w_bytes,
                                        fraction=self.cfg.kv_fraction, mem_get_info=share) - 2)
        if collective:
            import torch.distributed as dist

            t = torch.tensor([fits], dtype=torch.int64)
            dist.all_reduce(t, op=dist.ReduceOp.MIN, group=self.transport.ctrl)
            fits = int(t[0])
        if fits < 1:
            raise MemoryError("KV cache: not even one sequence fits the HBM budget")
        if fits < want:
            log.warning("KV budget: %d of %d requested slots fit", fits, want)
        return fits

    def _ranks_sharing_device(self, dev: torch.device) -> int:
        return _ranks_sharing_device(dev, self.transport.ctrl)

    def _devloop_fabric(self, dev: torch.device) -> DeviceLoopFabric:
        """Loopback channels sized for the largest message an edge carries:
        one item's prefill rows (a group's chunk tokens, fp32) or decode rows;
        eight of them fit each ring (64 MiB - 1 GiB) -- with two, the prefill
        senders of an 8-stage rehearsal waited for ring space (GPT-2 small P=8:
        287k -> 300k tok/s with 512 MiB rings, profiles/r4_ab_rehearsal.log).
        LSD_LOOP_RING_MB overrides."""
        cfg = self.cfg
        return DeviceLoopFabric(self.P, dev, lanes=int(os.environ.get("LSD_LANES", "2")),
                                ring_bytes=self._loop_ring_bytes(),
                                # round_timeout_s <= 0 = no watchdog, not zero-length waits
                                timeout=cfg.round_timeout_s if cfg.round_timeout_s > 0 else 600.0,
                                spin_limit_s=float(os.environ.get("LSD_LOOP_SPIN_S", "30")))

    def _loop_ring_bytes(self) -> int:
        """Device-loopback ring per channel (in-process fabric and the dist-mode
        rehearsal alike): eight of the largest messages an edge carries -- one
        item's prefill rows (a group's chunk tokens, fp32) -- within 64 MiB to
        1 GiB, and never less than one such message plus 1 MiB."""
        per_seq = self.cfg.prefill_chunk if self.cfg.prefill_chunk > 0 else self.max_seq
        big = self.group_cap * min(per_seq, self.max_seq) * self.mcfg.hidden * 4
        ring = int(os.environ.get("LSD_LOOP_RING_MB", "0")) << 20 or min(1 << 30, max(64 << 20, 8 * big))
        return max(ring, big + (1 << 20))

    def _weight_bytes(self, i: int) -> int:
        mc = self.mcfg
        a, b = self.unit_plan[i]
        per_layer = mc.block_params() * 2
        n = per_layer * (b - a) // 2
        if i == 0:
            n += mc.embed_params() * 2
        if i == self.P - 1 and not (i == 0 and mc.tie_embeddings):
            # the head, padded in place (ops/hip.py prepare_stage); a tied
            # GPT-2 head on a 1-stage pipeline is the embedding counted above
            n += mc.lm_head_params() * 2
        return n

    def _build_stage(self, i: int, device: torch.device) -> StageModel:
        a, b = self.plan[i]
        # +2 slots: scratch (pad rows of decode buckets) and compat forwards
        return StageModel(self.mcfg, a, b, first=(i == 0), last=(i == self.P - 1), device=device,
                          dtype=_dtype(self.cfg.dtype, device), seed=self.cfg.seed,
                          weights_path=self.cfg.weights, max_slots=self.kv_slots + 2,
                          max_seq=self.max_seq, units=self.unit_plan[i],
                          variants=[p[i] for p in self.unit_plans] if self.unit_plans else None)

    def _worker(self, st: StageModel, t, i: int) -> StageWorker:
        if self.cfg.wire_dtype not in ("fp32", "bf16"):
            raise ValueError(f"wire_dtype must be fp32 or bf16, got {self.cfg.wire_dtype!r}")
        w = StageWorker(st, t, i, self.P, scratch_slot=self.kv_slots,
                        compat_slot=self.kv_slots + 1,
                        wire=torch.bfloat16 if self.cfg.wire_dtype == "bf16" else None)
        w.merge_prefill = w.MERGE_PREFILL and self.cfg.merge_prefill
        return w

    @property
    def is_coordinator(self) -> bool:
        return self.rank == 0

    def kv_info(self) -> dict:
        st = self.stages[0]
        return {"kv_slots": self.kv_slots, "kv_bytes_stage0": st.kv.nbytes,
                "kv_slots_free": sum(p.available for p in self.slot_pools),
                "group_rows": self.group_cap, "groups": self.M,
                # half-layer unit ranges per stage: one plan, or (even, odd) group plans
                "stage_units": [list(map(list, p)) for p in self.unit_plans] if self.unit_plans
                else [list(map(list, self.unit_plan))]}

    # ------------------------------------------------------------------
    # requests
    # ------------------------------------------------------------------
    def _validate(self, prompt: List[int], sp: SamplingParams) -> None:
        sp.validate()
        if len(prompt) == 0:
            raise ValueError("prompt must contain at least one token")
        if len(prompt) + sp.max_new_tokens > self.max_seq:
            raise ValueError(f"prompt ({len(prompt)}) + max_new_tokens ({sp.max_new_tokens}) "
                             f"exceeds the context limit {self.max_seq}")

    def submit(self, prompt_ids: List[int], params: SamplingParams) -> Request:
        """Thread-safe: queue one request; the driver loop admits it at the
        next decode-step boundary."""
        if self.mode == "dist" and self.rank != 0:
            raise RuntimeError("submit() on a non-coordinator rank")
        if not self.healthy:
            raise RuntimeError(f"engine unhealthy: {self.last_error}")
        self._validate(prompt_ids, params)
        req = self.scheduler.submit(prompt_ids, params)
        self._wake.set()
        return req

    def generate_ids(self, prompts: List[List[int]], params, microbatches: Optional[int] = None,
                     record_timing: bool = False) -> List[List[int]]:
        """Generate continuations for token-id prompts (generated ids only).
        Runs the driver loop on this thread unless the serving loop is up."""
        ph = self._phases
        tp = time.monotonic() if ph is not None else 0.0
        if isinstance(params, SamplingParams):
            params = [params] * len(prompts)
        for p, sp in zip(prompts, params):
            self._validate(p, sp)
        if not self.healthy:
            raise RuntimeError(f"engine unhealthy: {self.last_error}")
        if microbatches and microbatches != self.M and self.loop_thread is None:
            self.set_groups(microbatches)
        reqs = self.scheduler.submit_many(prompts, params)
        if self.loop_thread is not None:
            return [r.wait() for r in reqs]
        if ph is not None:
            self._phase("validate+submit", tp)
        with self._lock:
            self._drive(lambda: all(r.done for r in reqs), timing=record_timing)
        tp = time.monotonic() if ph is not None else 0.0
        out = [r.wait(0) for r in reqs]
        if ph is not None:
            self._phase("collect", tp)
        return out

    def _phase(self, name: str, t0: float) -> float:
        """LSD_HOST_PROFILE: add the host time since t0 to session phase `name`."""
        t = time.monotonic()
        self._phases[name] = self._phases.get(name, 0.0) + (t - t0)
        return t

    def set_groups(self, M: int) -> None:
        """Re-shape the microbatch groups (only between sessions)."""
        with self._lock:
            if self.scheduler.has_work():
                raise RuntimeError("cannot regroup while requests are in flight")
            if self.mode == "dist":
                raise RuntimeError("regrouping needs every rank: set num_microbatches instead")
            self.M = max(1, M)
            self.group_cap = -(-self.cfg.max_batch // self.M)
            self.scheduler = Scheduler(self, self.M, self.group_cap)
            self.workers[0].readout = self.scheduler.on_readout
            self.workers[0].readout_native = self.scheduler.on_readout_native
            for w in self.workers:
                w.configure(self.M, self.group_cap)

    # ------------------------------------------------------------------
    # the driver loop (stage 0 of replica 0 / rank 0)
    # ------------------------------------------------------------------
    def _send_plans(self, plans: Optional[List[StepPlan]], end: bool = False) -> None:
        """Plan of every replica to every rank that executes it."""
        for rep in range(self.R):
            p = plans[rep] if plans is not None else StepPlan(step=-1, replica=rep, end=True,
                                                               timing=self.scheduler.timing)
            dsts = [rep * self.P + r if self.mode == "dist" else r for r in range(self.P)
                    if rep * self.P + r != 0]
            self.plan_ch.send_many(dsts, p)

    def _drive(self, until, timing: bool = False) -> None:
        """Run pipeline steps until `until()` (and no work is left in flight
        that `until` depends on).  One session = plans until idle; followers
        get an `end` marker when it goes idle."""
        sch = self.scheduler
        sch.timing = timing
        w0 = self.workers[0]
        if timing:
            for w in self.workers:
                w.step_events.clear()
            sch.step_log.clear()
            self._start_stats()
        lag = self.P + 2  # steps the host may run ahead of the GPU readouts
        hp = self._hostprof
        ph = self._phases
        tp = time.monotonic()
        ran = False
        try:
            cur = sch.build_step()
            if cur is not None:
                ran = True
                self._send_plans(cur)
                w0.begin_session()
            if ph is not None:
                tp = self._phase("first plan", tp)
            while cur is not None:
                self._check_followers()
                if not self.healthy:
                    raise RuntimeError(self.last_error)
                t0 = time.monotonic()
                self._round(t0)
                nxt = sch.build_step()
                tb = time.monotonic()
                b0 = getattr(self.plan_ch, "bytes_sent", 0)
                self._send_plans(nxt)
                t1 = time.monotonic()
                c1 = time.thread_time() if hp is not None else 0.0
                w0.run_step(cur[0], nxt[0] if nxt is not None else None)
                t2 = time.monotonic()
                c2 = time.thread_time() if hp is not None else 0.0
                sch.poll(block_until_step=cur[0].step - lag)
                if hp is not None and any(gp.chunks for gp in cur[0].groups):
                    t3 = time.monotonic()  # steps with prefill chunks (eager issue)
                    hp[8] += t2 - t1
                    hp[9] += t3 - t2
                    hp[10] += 1
                elif hp is not None:
                    t3 = time.monotonic()  # decode-only steps
                    hp[0] += t1 - t0
                    hp[1] += t2 - t1
                    hp[2] += t3 - t2
                    hp[3] += 1
                    hp[4] += sum(1 for gp in cur[0].groups if gp.has_work)
                    hp[5] += c2 - c1  # CPU time of the issuing thread (no waits)
                    hp[6] += t1 - tb  # encoding + posting the followers' plans
                    hp[7] += getattr(self.plan_ch, "bytes_sent", 0) - b0
                cur = nxt
            if ran:
                w0.end_session()
            if ph is not None:
                tp = self._phase("step loop", tp)
            # everything issued: wait for the outstanding readouts
            while sch.readouts or not until():
                if sch.readouts:
                    sch.poll(block_until_step=1 << 62)
                elif not until():
                    # remote replicas' readouts still on their way
                    self._check_followers()
                    if not self.healthy:
                        raise RuntimeError(self.last_error)
                    time.sleep(0.0005)
                    sch.poll()
            if ph is not None:
                tp = self._phase("drain", tp)
        except BaseException as e:
            self.healthy = False
            self.last_error = f"{type(e).__name__}: {e}"
            sch.fail_all(RuntimeError(f"engine unhealthy: {self.last_error}"))
            raise
        finally:
            self._round(None)
        if timing and ran:
            self._finish_stats()
            if ph is not None:
                self._phase("stats", tp)

    def _check_followers(self) -> None:
        err = getattr(self, "_follow_err", None)
        if err is not None:
            raise err

    # -- timing ------------------------------------------------------------
    def _start_stats(self) -> None:
        self.workers[0].start_stats()

    def _finish_stats(self) -> None:
        from ..parallel.pipeline import GPU_GATE

        w0 = self.workers[0]
        if self.devices[0].type == "cuda":
            with GPU_GATE.shared():
                torch.cuda.synchronize(self.devices[0])
        stats = [w0.end_stats()]
        if self.mode == "local":
            for _ in range(self.P - 1):
                stats.append(self._stats_q.get(timeout=self.cfg.round_timeout_s))
        else:
            got = self.transport.gather_object(stats[0], dst=0)
            stats = [dict(st, replica=g // self.P) for g, st in enumerate(got) if st is not None]
        ss = SessionStats(stages=sorted([s for s in stats if s], key=lambda s: (s.get("replica", 0),
                                                                               s["stage"])))
        ev = w0.step_events
        log_ = dict(self.scheduler.step_log)
        if ev:
            ts = [(ev[k][0], ev[k][1].elapsed_time(ev[k + 1][1])) for k in range(len(ev) - 1)]
            ss.prefill_ms = sum(t for s, t in ts if log_.get(s))
            ss.step_times_ms = [t for s, t in ts if not log_.get(s)]
        self.last_session = ss

    # ------------------------------------------------------------------
    # followers
    # ------------------------------------------------------------------
    def _follow(self, recv, worker: StageWorker) -> bool:
        """Execute plans until the session ends (True) or stop (False)."""
        cur = recv()
        started = False
        began = False
        while True:
            if cur.stop or cur.end:
                if began:
                    worker.end_session()
                if cur.stop:
                    return False
                if started or cur.timing:
                    self._follower_stats(worker, cur)
                return True
            if not began:
                worker.begin_session()
                began = True
            if cur.timing and not started:
                worker.start_stats()
                started = True
            nxt = recv()
            self._round(time.monotonic())  # watchdog: host blocked inside a step
            if self._stall_after is not None:
                self._test_stall()
            worker.run_step(cur, nxt if not nxt.stop else None)
            self._round(None)
            if not self.healthy:
                raise RuntimeError(self.last_error)
            cur = nxt

    def _test_stall(self) -> None:
        """Test hook (LSD_TEST_STALL_RANK / LSD_TEST_STALL_AFTER): this rank
        stops issuing work after that many steps, as a hung peer process
        would; it waits for its own watchdog, then fails."""
        self._stall_after -= 1
        if self._stall_after >= 0:
            return
        log.error("test hook: rank %d stalls", self.rank)
        while self.healthy:
            time.sleep(0.05)
        raise RuntimeError("test stall")

    def _follower_stats(self, worker: StageWorker, end_plan: StepPlan) -> None:
        if not end_plan.timing:
            worker.stats = None
            return
        self._round(time.monotonic())
        worker.sync()
        self._round(None)
        st = worker.end_stats()
        if self.mode == "local":
            self._stats_q.put(st)
        else:
            self.transport.gather_object(st, dst=0)

    def _local_follower(self, i: int) -> None:
        w = self.workers[i]
        try:
            if self.devices[i].type == "cuda":
                torch.cuda.set_device(self.devices[i])
            while self._follow(lambda: self.plan_ch.recv(i), w):
                pass
        except BaseException as e:  # surfaced on the driving thread
            log.error("stage %d failed: %s", i, e)
            self._follow_err = e
            if self.fabric is not None:
                self.fabric.failed = e  # wake stages blocked on this one

    def follow_session(self) -> bool:
        """Dist followers: execute one session's plans (False on stop)."""
        assert self.mode == "dist" and self.rank != 0
        return self._follow(lambda: self.plan_ch.recv(0), self.workers[0])

    def worker_loop(self) -> None:
        """Non-coordinator ranks: execute plans until 'stop'."""
        while self.follow_session():
            pass
        self._close_dist()

    # DP: replica stage-0 ranks ship sampled ids to rank 0 --------------------
    def _ship_readout(self, plan: StepPlan, gp: GroupPlan, ret: torch.Tensor) -> None:
        n = gp.ret
        if ret.is_cuda:
            host = torch.empty(n, dtype=torch.int32, pin_memory=True)
            host.copy_(ret[:n], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        else:
            host, ev = ret[:n].clone(), None
        self._tok_q.put((plan.step, (plan.replica, plan.step, gp.g), host, ev))

    def _tok_shipper(self) -> None:
        # test hook: hold replica readouts back so they land after rank 0's
        # own session has nothing left to plan (tests/test_pipeline.py)
        delay = float(os.environ.get("LSD_TEST_TOK_DELAY_S", "0"))
        while True:
            item = self._tok_q.get()
            if item is None:
                self.tok_ch.send(0, None)
                self.tok_ch.flush()
                return
            step, key, host, ev = item
            if ev is not None:
                from ..parallel.pipeline import wait_event

                wait_event(ev)  # queries gated against a stage thread's capture
            if delay:
                time.sleep(delay)
            self.tok_ch.send(0, (step, key, host.tolist()))

    def _tok_receiver(self, rep: int) -> None:
        src = rep * self.P
        while True:
            msg = self.tok_ch.recv(src)
            if msg is None:
                return
            step, key, toks = msg
            self.scheduler.push_remote_readout(step, toks, key)

    # ------------------------------------------------------------------
    # serving loop (background thread) and shutdown
    # ------------------------------------------------------------------
    def start_loop(self) -> None:
        """Serve submitted requests continuously on a background thread."""
        if self.loop_thread is not None:
            return
        self._stop_loop.clear()
        self.loop_thread = threading.Thread(target=self._serve, name="lsd-engine", daemon=True)
        self.loop_thread.start()

    def _serve(self) -> None:
        sch = self.scheduler
        n = 0
        while not self._stop_loop.is_set():
            if not sch.has_work():
                # Python-side wait: a daemon thread parked inside native code
                # with the GIL released would abort the interpreter at exit
                self._wake.wait(0.05)
                self._wake.clear()
                continue
            # sample the per-stage timing on one session in `metrics_every`
            every = max(0, self.cfg.metrics_every)
            timing = every > 0 and n % every == 0
            n += 1
            try:
                with self._lock:
                    self._drive(lambda: not sch.has_work(), timing=timing)
            except BaseException as e:  # requests already failed by _drive
                log.error("pipeline failed: %s", e)
                if not self.healthy:
                    return

    def stop_loop(self) -> None:
        self._stop_loop.set()
        if self.loop_thread is not None:
            self.loop_thread.join(timeout=30)
            self.loop_thread = None

    def shutdown(self) -> None:
        self.stop_loop()
        if self.mode == "local":
            self.plan_ch.send_many(list(range(1, self.P)), StepPlan(step=-1, stop=True))
            if self.watchdog is not None:
                self.watchdog.close()
            return
        if self.rank == 0:
            for rep in range(self.R):
                self.plan_ch.send_many([g for g in range(rep * self.P, (rep + 1) * self.P) if g],
                                       StepPlan(step=-1, stop=True))
            self.plan_ch.flush()
            if hasattr(self.plan_ch, "close"):
                self.plan_ch.close()  # the stop plans stay readable: readers drain first
            self._close_dist()

    def _close_dist(self) -> None:
        """Orderly teardown: every rank reaches the barrier before any process
        group is destroyed, so no rank exits while a peer still has a gloo /
        RCCL connection open to it."""
        import torch.distributed as dist

        if self.rank != 0 and self.stage_idx == 0 and self.R > 1:
            self._tok_q.put(None)
            for t in self._tok_threads:
                t.join(timeout=30)
        self.transport.barrier()
        if self.rank == 0:
            for t in self._tok_threads:
                t.join(timeout=30)
        if self.watchdog is not None:
            self.watchdog.close()
        self.transport.close()  # native RCCL communicators (no-op for torch groups)
        self.transport.barrier()
        if dist.is_initialized():
            dist.destroy_process_group()

    # ------------------------------------------------------------------
    # Compat single-shard forwards (reference /forward and /forward_b)
    # ------------------------------------------------------------------
    def forward_a(self, input_ids: List[int]) -> torch.Tensor:
        """Stage-0 output for a full sequence (reference ShardA, server.py:77-86):
        embeddings + this pipeline's first stage, on the compat KV slot."""
        from .batch import BatchMeta

        if len(input_ids) > self.max_seq:
            raise ValueError(f"sequence length {len(input_ids)} exceeds {self.max_seq}")
        if self.P < 2:
            raise RuntimeError("forward_a needs >= 2 pipeline stages")
        st = self.stages[0]
        with self._lock:
            ids = torch.tensor(input_ids, dtype=torch.int32, device=st.device)
            meta = BatchMeta.build([self.kv_slots + 1], [0], [len(input_ids)], st.device)
            return st.forward(meta, ids)

    def forward_b(self, hidden: torch.Tensor) -> torch.Tensor:
        """Remaining stages + ln_f + lm_head over all positions (ShardB,
        server.py:98-103).  Local: stage by stage in this process; dist: the
        hidden rows travel stage 1 -> P-1 over the pipeline edges and the
        logits come back on the return edge, between decode sessions."""
        from .batch import BatchMeta

        if self.P < 2:
            raise RuntimeError("forward_b needs >= 2 pipeline stages")
        # a stage updates its input rows in place (the residual stream): copy
        h = hidden.reshape(-1, self.mcfg.hidden).float().clone()
        T = h.shape[0]
        if T > self.max_seq:
            raise ValueError(f"sequence length {T} exceeds {self.max_seq}")
        with self._lock:
            if self.mode == "local":
                out = h
                for st in self.stages[1:]:
                    meta = BatchMeta.build([self.kv_slots + 1], [0], [T], st.device)
                    out = st.forward(meta, out.to(st.device), all_logits=st.last)
                return out[:, : self.mcfg.vocab_size]
            w0 = self.workers[0]
            gp = GroupPlan(0, kind="fwd_b", fwd_rows=T)
            plan = StepPlan(step=-2, groups=[gp])
            self.plan_ch.send_many(list(range(1, self.P)), plan)
            self.plan_ch.send_many(list(range(1, self.P)), StepPlan(step=-1, end=True))
            dev = self.devices[0]
            x = h.to(dev).contiguous()
            w0._send(x, 1, "fwd", 0).wait()  # in the wire dtype stage 1 expects
            out = torch.empty(T, self.mcfg.vocab_size, dtype=torch.float32, device=dev)
            self.transport.irecv(out, self.P - 1, "ret").wait()
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            return out


def _ranks_sharing_device(dev: torch.device, group) -> int:
    """Dist ranks bound to this very GPU (the single-GPU rehearsal puts
    several on one): every rank publishes (host, device identity) on `group`
    (None: the default group) and counts its own key.  Independent of how
    many GPUs each process sees (HIP_VISIBLE_DEVICES) and of the node count."""
    import socket

    import torch.distributed as dist

    props = torch.cuda.get_device_properties(dev)
    ident = str(getattr(props, "uuid", "") or "") or ":".join(
        str(getattr(props, f, "")) for f in ("pci_domain_id", "pci_bus_id", "pci_device_id"))
    key = (socket.gethostname(), ident if ident.strip(":") else str(dev))
    keys = [None] * dist.get_world_size()
    dist.all_gather_object(keys, key, group=group)
    return max(1, sum(1 for k in keys if k == key))


def _with_index(dev: torch.device) -> torch.device:
    if dev.type == "cuda" and dev.index is None:
        return torch.device("cuda", torch.cuda.current_device())
    return dev


def _make_slot_allocator(n: int):
    """Native (C++) KV-slot allocator when built, Python twin otherwise."""
    from . import native

    mod = native.load()
    if mod is not None and os.environ.get("LSD_PY_RUNTIME", "0") != "1":
        return mod.SlotAllocator(n)
    return SlotAllocator(n)


def freeze_gc() -> None:
    """Move every object alive now (model, torch / HIP wrappers, captured
    graphs) out of the cyclic collector's reach (gc.freeze): a 4096-request
    session allocates enough small objects to trigger full collections, and
    each one walked the whole engine (a second session's submit took
    194 ms instead of 61 ms on the CPU, profiles/r6_session_host.log).
    Called once the engine is built and warmed up; objects created later are
    collected as usual."""
    gc.collect()
    gc.freeze()


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
