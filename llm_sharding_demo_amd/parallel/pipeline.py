"""Pipeline-parallel decode scheduler (one worker per stage / per MI355X).

Replaces the reference's coordinator loop (`server.py:169-206`), which for
every output token runs shard A, relays its hidden state through the
coordinator to shard B, ships all-position logits back and samples on the
host -- strictly sequentially, so one shard is always idle and each token
costs two HTTP round trips.

Here a generation *round* is a set of sequences split into M microbatches.
Every stage runs the same static schedule:

    for step in 0..G-1:            # step 0 = prefill, then one token per step
        for mb in 0..M-1:
            input  <- prompt ids (stage 0, step 0)
                    | sampled ids of (step-1, mb) from stage P-1 (stage 0)
                    | boundary hidden of (step, mb) from stage r-1
            output <- this stage's layers  (+ ln_f, lm_head, sampler on P-1)
            send output -> stage r+1   (or token ids -> stage 0 from P-1)

With M >= P microbatches every stage is busy in steady state (stage r works
on microbatch (t - r) mod M at tick t).  Receives for the next item are
posted before the current item's compute is enqueued, so the transfer
overlaps compute; `Handle.wait()` only orders the compute stream behind the
comm stream.  Decode steps (step >= 2) replay one hipGraph per microbatch:
all positions / sampler counters advance on the device inside the graph.
"""
from __future__ import annotations

import contextlib
import os
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

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


@dataclass
class RoundResult:
    tokens: List[torch.Tensor]  # per microbatch: int32 [steps, Bm] (host)
    step_times_ms: List[float] = field(default_factory=list)
    prefill_ms: float = 0.0


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
        n_lanes = int(os.environ.get("LSD_LANES", "2"))
        self.lanes = ([torch.cuda.Stream(self.device) for _ in range(n_lanes)]
                      if self.device.type == "cuda" else [])

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
        st, dev, P, r = self.stage, self.device, self.P, self.r
        mbs = spec.microbatches
        M, G = len(mbs), spec.steps
        if G < 1 or M < 1:
            raise ValueError("round needs >= 1 step and >= 1 microbatch")
        i32 = dict(dtype=torch.int32, device=dev)
        vocab = st.cfg.vocab_size

        pre_meta, dec_meta, samp = [], [], []
        prompt_ids, in_pre, in_dec, tok_in, tok_out = [], [], [], [], []
        for mb in mbs:
            lens = [len(p) for p in mb.prompts]
            if min(lens) < 1:
                raise ValueError("empty prompt")
            if max(lens) + G > st.max_seq:
                raise ValueError(f"prompt+generation {max(lens) + G} exceeds max_seq {st.max_seq}")
            pre_meta.append(BatchMeta.build(mb.slots, [0] * mb.size, lens, dev))
            dec_meta.append(BatchMeta.decode(mb.slots, lens, dev, max_ctx=max(lens) + G))
            if self.last:
                samp.append(SamplingState(mb.temperature, mb.top_k, mb.greedy, mb.seeds, dev))
            if self.first:
                flat = [t for p in mb.prompts for t in p]
                prompt_ids.append(torch.tensor(flat, **i32))
                tok_in.append(torch.zeros(mb.size, **i32))
                tok_out.append(torch.zeros(G, mb.size, **i32))
            if not self.first:
                in_pre.append(torch.empty(sum(lens), self.H, dtype=torch.float32, device=dev))
                in_dec.append(torch.empty(mb.size, self.H, dtype=torch.float32, device=dev))

        L = max(1, len(self.lanes))
        for lane in self.lanes:
            lane.wait_stream(torch.cuda.current_stream(dev))
        # kernels size their grids for the lanes that actually run side by side
        st.backend.concurrency = min(L, M)

        def on_lane(m):
            if not self.lanes:
                return contextlib.nullcontext()
            return torch.cuda.stream(self.lanes[m % L])

        items = [(s, m) for s in range(G) for m in range(M)]
        recv: Dict[tuple, Handle] = {}
        send_pending: Dict[int, SendHandle] = {}
        graphs: Dict[int, tuple] = {}
        step_events = []

        def recv_key_buf(s, m):
            """(edge, src, buffer) the input of item (s, m) arrives in, or None."""
            if self.first:
                if s == 0 or P == 1:
                    return None
                return ("ret", P - 1, tok_in[m])
            return ("fwd", r - 1, in_pre[m] if s == 0 else in_dec[m])

        def post(i):
            if i >= len(items):
                return
            s, m = items[i]
            kb = recv_key_buf(s, m)
            if kb is not None and (s, m) not in recv:
                # posted from m's lane: the comm stream then also waits for the
                # previous reader of this buffer (microbatch m's last compute)
                with on_lane(m):
                    recv[(s, m)] = self.t.irecv(kb[2], kb[1], kb[0])

        def body(s, m, inp):
            """Compute of item (s, m); returns what goes downstream."""
            meta = pre_meta[m] if s == 0 else dec_meta[m]
            st.backend.lane = m % L
            out = st.forward(meta, inp)
            if s > 0:
                dec_meta[m].advance()
            if self.last:
                tok = st.backend.sample(out, samp[m], vocab)
                samp[m].advance()
                return tok
            return out

        t_start = time.perf_counter()
        post(0)
        for i, (s, m) in enumerate(items):
            with on_lane(m), trace_range(f"stage{r}/step{s}/mb{m}"):
                self._item(i, s, m, items, recv, send_pending, graphs, step_events, spec, post,
                           recv_key_buf, body, prompt_ids, tok_in, tok_out, G, P, r)
        # Stage 0 still owes the receive of the final step's tokens.
        if self.first and P > 1:
            for m in range(M):
                with on_lane(m):
                    self.t.irecv(tok_in[m], P - 1, "ret").wait()
                    tok_out[m][G - 1].copy_(tok_in[m])
        for h in send_pending.values():
            h.wait()
        for lane in self.lanes:
            torch.cuda.current_stream(dev).wait_stream(lane)
        if spec.record_timing and self.first and self.device.type == "cuda":
            ev = torch.cuda.Event(enable_timing=True)
            with on_lane(0):
                ev.record()
            step_events.append(ev)
        self._sync()
        elapsed = (time.perf_counter() - t_start) * 1e3
        if not self.first:
            return None
        res = RoundResult(tokens=[t.cpu() for t in tok_out])
        if step_events:
            ts = [step_events[k].elapsed_time(step_events[k + 1]) for k in range(len(step_events) - 1)]
            res.prefill_ms = ts[0] if ts else 0.0
            res.step_times_ms = ts[1:]
        else:
            res.prefill_ms = elapsed
        return res

    def _item(self, i, s, m, items, recv, send_pending, graphs, step_events, spec, post,
              recv_key_buf, body, prompt_ids, tok_in, tok_out, G, P, r):
        """One (step, microbatch) of the static schedule, on microbatch m's lane."""
        if spec.record_timing and m == 0 and self.device.type == "cuda":
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            step_events.append(ev)
        # --- input
        if (s, m) in recv:
            inp = recv.pop((s, m)).wait()
        elif self.first:
            inp = prompt_ids[m] if s == 0 else tok_in[m]
        else:
            raise RuntimeError(f"stage {r}: no input posted for {(s, m)}")
        if self.first and s > 0:
            tok_out[m][s - 1].copy_(inp)
        # Post the next receive before enqueueing this compute when it
        # targets a different buffer (overlap); otherwise after.
        cur_kb = recv_key_buf(s, m)
        nxt_kb = recv_key_buf(*items[i + 1]) if i + 1 < len(items) else None
        early = nxt_kb is not None and (cur_kb is None or nxt_kb[2] is not cur_kb[2])
        if early:
            post(i + 1)
        # --- the previous send of this microbatch's static output must be done
        if m in send_pending:
            send_pending.pop(m).wait()
        # --- compute
        use_graph = spec.use_graphs and self.device.type == "cuda" and s >= 2
        if use_graph:
            if m not in graphs:
                graphs[m] = self._capture(lambda s=s, m=m, inp=inp: body(s, m, inp))
            g, out = graphs[m]
            g.replay()
        else:
            out = body(s, m, inp)
        if not early:
            post(i + 1)
        # --- output
        if self.last:
            if P == 1:
                tok_in[m].copy_(out)
                if s == G - 1:
                    tok_out[m][s].copy_(out)
            else:
                send_pending[m] = self.t.send(out, 0, "ret")
        else:
            send_pending[m] = self.t.send(out, r + 1, "fwd")

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
