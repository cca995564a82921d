"""Pipeline-parallel decode scheduler (one worker per stage / per MI355X).

Replaces the reference's coordinator loop (`server.py:169-206`), which for
every output token runs shard A, relays its hidden state through the
coordinator to shard B, ships all-position logits back and samples on the
host -- strictly sequentially, so one shard is always idle and each token
costs two HTTP round trips.

Here a generation *round* is a set of sequences split into M microbatches.
Every stage runs the same static schedule over items (step s, microbatch m):

    steps 0..C-1       prefill chunks (C = 1 unless the round asks for
                       chunked prefill: each chunk carries up to `chunk`
                       prompt tokens per sequence, aligned to the END of the
                       prompt so the last chunk holds every sequence's last
                       position)
    steps C..C+G-2     decode, one token per sequence per step

    for s in steps:
        for m in 0..M-1:
            input  <- prompt chunk s (stage 0, prefill)
                    | sampled ids of (s-1, m) from stage P-1 (stage 0, decode)
                    | boundary hidden of (s, m) from stage r-1
            output <- this stage's units (+ ln_f, lm_head, sampler on P-1 for
                      the last chunk and every decode step)
            send output -> stage r+1   (or token ids -> stage 0 from P-1)

With M >= P microbatches every stage is busy in steady state (stage r works
on microbatch (t - r) mod M at tick t).  Receives for the next item are
posted before the current item's compute is enqueued when they target a
different buffer, so the transfer overlaps compute; `Handle.wait()` only
orders the compute stream behind the comm stream.  Microbatch m runs on
HIP stream lanes[m % L], so independent microbatches overlap on the GPU.
Decode steps after the first replay one hipGraph per microbatch: positions
and sampler counters advance on the device inside the graph.
"""
from __future__ import annotations

import contextlib
import os
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch

from ..models.stage import StageModel
from ..runtime.batch import BatchMeta, SamplingState
from ..utils.tracing import trace_range
from .comm import Handle, SendHandle, Transport


_CAPTURE_LOCK = threading.Lock()


@dataclass
class MicroBatchSpec:
    slots: List[int]
    prompts: List[List[int]]
    temperature: List[float]
    top_k: List[int]
    greedy: List[bool]
    seeds: List[int]

    @property
    def size(self) -> int:
        return len(self.slots)


@dataclass
class RoundSpec:
    microbatches: List[MicroBatchSpec]
    steps: int  # tokens generated per sequence (>= 1)
    use_graphs: bool = True
    record_timing: bool = False
    prefill_chunk: int = 0  # prompt tokens per sequence per prefill step; 0 = whole prompt


@dataclass
class RoundResult:
    tokens: List[torch.Tensor]  # per microbatch: int32 [steps, Bm] (host)
    step_times_ms: List[float] = field(default_factory=list)
    prefill_ms: float = 0.0
    # per stage (record_timing rounds): {"stage", "wall_ms", "busy_ms",
    # "busy_fraction", "items"} -- busy = union of this stage's compute
    # intervals over both lanes; 1 - busy_fraction is the stage's bubble
    stages: List[dict] = field(default_factory=list)


def prefill_chunks(lens: List[int], chunk: int) -> List[Tuple[List[int], List[int]]]:
    """(starts, qlens) per prefill chunk for prompts of `lens` tokens.  Chunks
    are aligned to the end of each prompt: the last chunk holds every
    sequence's final position (its logits are sampled); earlier chunks of a
    shorter prompt may be empty."""
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


class _Round:
    """Buffers, metadata and comm state of one round on one stage."""

    def __init__(self, w: "StageWorker", spec: RoundSpec):
        st, dev = w.stage, w.device
        self.w, self.spec = w, spec
        self.M, self.G = len(spec.microbatches), spec.steps
        if self.G < 1 or self.M < 1:
            raise ValueError("round needs >= 1 step and >= 1 microbatch")
        i32 = dict(dtype=torch.int32, device=dev)
        self.chunk_meta: List[List[BatchMeta]] = []   # [m][c]
        self.chunk_ids: List[List[torch.Tensor]] = []  # stage 0: [m][c] prompt ids
        self.dec_meta, self.samp = [], []
        self.in_pre, self.in_dec, self.tok_in, self.tok_out = [], [], [], []
        per_mb = []
        for mb in spec.microbatches:
            lens = [len(p) for p in mb.prompts]
            if min(lens) < 1:
                raise ValueError("empty prompt")
            if max(lens) + self.G > st.max_seq:
                raise ValueError(f"prompt+generation {max(lens) + self.G} exceeds max_seq {st.max_seq}")
            per_mb.append((lens, prefill_chunks(lens, spec.prefill_chunk)))
        # every microbatch runs the same number of steps: shorter prompts get
        # leading empty chunks
        C = max(len(ch) for _, ch in per_mb)
        for mb, (lens, chunks) in zip(spec.microbatches, per_mb):
            empty = ([0] * mb.size, [0] * mb.size)
            chunks = [empty] * (C - len(chunks)) + chunks
            self.chunk_meta.append([BatchMeta.build(mb.slots, s0, q, dev) for s0, q in chunks])
            self.dec_meta.append(BatchMeta.decode(mb.slots, lens, dev, max_ctx=max(lens) + self.G))
            if w.last:
                self.samp.append(SamplingState(mb.temperature, mb.top_k, mb.greedy, mb.seeds, dev))
            if w.first:
                self.chunk_ids.append([torch.tensor([t for p, a, n in zip(mb.prompts, s0, q)
                                                     for t in p[a:a + n]], **i32)
                                       for s0, q in chunks])
                self.tok_in.append(torch.zeros(mb.size, **i32))
                self.tok_out.append(torch.zeros(self.G, mb.size, **i32))
            else:
                rows = max(sum(q) for _, q in chunks)
                self.in_pre.append(torch.empty(max(rows, 1), w.H, dtype=torch.float32, device=dev))
                self.in_dec.append(torch.empty(mb.size, w.H, dtype=torch.float32, device=dev))
        self.C = C
        self.items = [(s, m) for s in range(C + self.G - 1) for m in range(self.M)]
        self.recv: Dict[tuple, Handle] = {}
        self.send_pending: Dict[int, SendHandle] = {}
        self.graphs: Dict[int, tuple] = {}
        self.step_events: List[torch.cuda.Event] = []
        self.compute_marks: List[tuple] = []  # (start, end) events / host times per item

    def rows(self, s: int, m: int) -> int:
        return self.chunk_meta[m][s].num_tokens if s < self.C else self.spec.microbatches[m].size

    def recv_target(self, s: int, m: int) -> Optional[Tuple[str, int, torch.Tensor]]:
        """(edge, src stage, buffer) the input of item (s, m) arrives in, or None
        when it is local (stage 0 prefill / single-stage decode) or absent."""
        w = self.w
        if w.first:
            if s < self.C or w.P == 1:
                return None
            return ("ret", w.P - 1, self.tok_in[m])
        if s < self.C:
            n = self.rows(s, m)
            return ("fwd", w.r - 1, self.in_pre[m][:n]) if n > 0 else None
        return ("fwd", w.r - 1, self.in_dec[m])

    def post(self, i: int) -> None:
        if i >= len(self.items):
            return
        s, m = self.items[i]
        tgt = self.recv_target(s, m)
        if tgt is not None and (s, m) not in self.recv:
            # posted from m's lane: the comm stream then also waits for the
            # previous reader of this buffer (microbatch m's last compute)
            with self.w.on_lane(m):
                self.recv[(s, m)] = self.w.t.irecv(tgt[2], tgt[1], tgt[0])


def _same_buffer(a: Optional[tuple], b: Optional[tuple]) -> bool:
    return (a is not None and b is not None
            and a[2].untyped_storage().data_ptr() == b[2].untyped_storage().data_ptr())


class StageWorker:
    def __init__(self, stage: StageModel, transport: Optional[Transport], stage_idx: int,
                 num_stages: int):
        self.stage = stage
        self.t = transport
        self.r = stage_idx
        self.P = num_stages
        self.device = stage.device
        self.first = stage_idx == 0
        self.last = stage_idx == num_stages - 1
        self.H = stage.cfg.hidden
        # Each stage worker owns a non-blocking stream: no device-wide syncs, so
        # one stage may capture a hipGraph while another (same GPU) keeps running.
        self.stream = torch.cuda.Stream(self.device) if self.device.type == "cuda" else None
        # Microbatch "lanes": microbatch m of this stage runs on lanes[m % L], so
        # independent microbatches overlap on the GPU -- one's latency-bound
        # phases (small GEMMs, split-K tails) run beside another's bandwidth-
        # bound ones (attention over the KV cache).  Each lane has its own
        # split-K ticket counters in the backend.
        self.last_stats: Optional[dict] = None  # per-stage timing of the last timed round
        n_lanes = int(os.environ.get("LSD_LANES", "2"))
        self.lanes = ([torch.cuda.Stream(self.device) for _ in range(n_lanes)]
                      if self.device.type == "cuda" else [])

    def on_lane(self, m: int):
        if not self.lanes:
            return contextlib.nullcontext()
        return torch.cuda.stream(self.lanes[m % len(self.lanes)])

    # ------------------------------------------------------------------
    def _sync(self) -> None:
        if self.stream is not None:
            self.stream.synchronize()

    def run_round(self, spec: RoundSpec) -> Optional[RoundResult]:
        if self.stream is None:
            return self._run_round(spec)
        self.stream.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.stream):
            res = self._run_round(spec)
        torch.cuda.current_stream(self.device).wait_stream(self.stream)
        return res

    def _run_round(self, spec: RoundSpec) -> Optional[RoundResult]:
        dev, P = self.device, self.P
        R = _Round(self, spec)
        L = max(1, len(self.lanes))
        for lane in self.lanes:
            lane.wait_stream(torch.cuda.current_stream(dev))
        # kernels size their grids for the lanes that actually run side by side
        self.stage.backend.concurrency = min(L, R.M)

        t_start = time.perf_counter()
        timing = spec.record_timing
        t0_ev = None
        if timing and dev.type == "cuda":
            t0_ev = torch.cuda.Event(enable_timing=True)
            t0_ev.record()
        R.post(0)
        for i, (s, m) in enumerate(R.items):
            with self.on_lane(m), trace_range(f"stage{self.r}/step{s}/mb{m}"):
                self._item(R, i, s, m)
        # Stage 0 still owes the receive of the final step's tokens.
        if self.first and P > 1:
            for m in range(R.M):
                with self.on_lane(m):
                    self.t.irecv(R.tok_in[m], P - 1, "ret").wait()
                    R.tok_out[m][R.G - 1].copy_(R.tok_in[m])
        for h in R.send_pending.values():
            h.wait()
        for lane in self.lanes:
            torch.cuda.current_stream(dev).wait_stream(lane)
        if spec.record_timing and self.first and dev.type == "cuda":
            ev = torch.cuda.Event(enable_timing=True)
            with self.on_lane(0):
                ev.record()
            R.step_events.append(ev)
        t1_ev = None
        if t0_ev is not None:
            t1_ev = torch.cuda.Event(enable_timing=True)
            t1_ev.record()
        self._sync()
        elapsed = (time.perf_counter() - t_start) * 1e3
        self.last_stats = self._stage_stats(R, t0_ev, t1_ev, t_start, elapsed) if timing else None
        if not self.first:
            return None
        res = RoundResult(tokens=[t.cpu() for t in R.tok_out])
        ev = R.step_events
        if ev:
            ts = [ev[k].elapsed_time(ev[k + 1]) for k in range(len(ev) - 1)]
            res.prefill_ms = sum(ts[:R.C])
            res.step_times_ms = ts[R.C:]
        else:
            res.prefill_ms = elapsed
        if self.last_stats is not None:
            res.stages = [self.last_stats]
        return res

    def _stage_stats(self, R: _Round, t0_ev, t1_ev, t_start: float, elapsed: float) -> dict:
        if t0_ev is not None:
            iv = sorted((t0_ev.elapsed_time(a), t0_ev.elapsed_time(b)) for a, b in R.compute_marks)
            wall = t0_ev.elapsed_time(t1_ev)
        else:  # CPU: compute is synchronous, host clocks are the compute intervals
            iv = sorted(((a - t_start) * 1e3, (b - t_start) * 1e3) for a, b in R.compute_marks)
            wall = elapsed
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
        return {"stage": self.r, "wall_ms": round(wall, 3), "busy_ms": round(busy, 3),
                "busy_fraction": round(busy / wall, 4) if wall > 0 else 0.0, "items": len(iv)}

    def _body(self, R: _Round, s: int, m: int, inp):
        """Compute of item (s, m); returns what goes downstream (None: nothing)."""
        st = self.stage
        st.backend.lane = m % max(1, len(self.lanes))
        prefill = s < R.C
        if prefill and R.rows(s, m) == 0:  # this microbatch's prompts end before chunk s
            return None
        meta = R.chunk_meta[m][s] if prefill else R.dec_meta[m]
        sample = self.last and (not prefill or s == R.C - 1)
        out = st.forward(meta, inp, head=sample or not self.last)
        if not prefill:
            R.dec_meta[m].advance()
        if sample:
            tok = st.backend.sample(out, R.samp[m], st.cfg.vocab_size)
            R.samp[m].advance()
            return tok
        return None if self.last else out

    def _item(self, R: _Round, i: int, s: int, m: int) -> None:
        """One (step, microbatch) of the static schedule, on microbatch m's lane."""
        P = self.P
        if R.spec.record_timing and m == 0 and self.device.type == "cuda":
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            R.step_events.append(ev)
        # --- input
        if (s, m) in R.recv:
            inp = R.recv.pop((s, m)).wait()
        elif self.first:
            inp = R.chunk_ids[m][s] if s < R.C else R.tok_in[m]
        elif R.recv_target(s, m) is None:
            inp = None  # empty prefill chunk of this microbatch
        else:
            raise RuntimeError(f"stage {self.r}: no input posted for {(s, m)}")
        if self.first and s >= R.C:
            R.tok_out[m][s - R.C].copy_(inp)
        # Post the next receive before enqueueing this compute when it
        # targets a different buffer (overlap); otherwise after.
        cur = R.recv_target(s, m)
        nxt = R.recv_target(*R.items[i + 1]) if i + 1 < len(R.items) else None
        early = nxt is not None and not _same_buffer(cur, nxt)
        if early:
            R.post(i + 1)
        # --- the previous send of this microbatch's static output must be done
        if m in R.send_pending:
            R.send_pending.pop(m).wait()
        # --- compute
        use_graph = R.spec.use_graphs and self.device.type == "cuda" and s >= R.C + 1
        mark = self._mark() if R.spec.record_timing else None
        if use_graph:
            if m not in R.graphs:
                R.graphs[m] = self._capture(lambda s=s, m=m, inp=inp: self._body(R, s, m, inp))
            g, out = R.graphs[m]
            g.replay()
        else:
            out = self._body(R, s, m, inp)
        if mark is not None:
            R.compute_marks.append((mark, self._mark()))
        if not early:
            R.post(i + 1)
        # --- output
        if out is None:
            return
        if self.last:
            if P == 1:
                R.tok_in[m].copy_(out)
                if s == R.C + R.G - 2:
                    R.tok_out[m][R.G - 1].copy_(out)
            else:
                R.send_pending[m] = self.t.send(out, 0, "ret")
        else:
            R.send_pending[m] = self.t.send(out, self.r + 1, "fwd")

    def _mark(self):
        """Timestamp on the current (lane) stream: a timing event on the GPU,
        the host clock on CPU."""
        if self.device.type == "cuda":
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            return ev
        return time.perf_counter()

    # ------------------------------------------------------------------
    def _capture(self, fn):
        """Capture one decode step (this stage's forward for one microbatch,
        plus sampling on the last stage) into a hipGraph."""
        # capture_begin/end directly: torch.cuda.graph() does a device-wide
        # synchronize on entry, which is illegal while a sibling stage thread on
        # the same GPU is capturing.  One capture at a time per process.
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with _CAPTURE_LOCK:
            with torch.cuda.stream(s):
                g.capture_begin(capture_error_mode="thread_local")
                try:
                    out = fn()
                finally:
                    g.capture_end()
        torch.cuda.current_stream(self.device).wait_stream(s)
        return g, out
