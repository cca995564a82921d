#!/usr/bin/env python3
"""Decode-step lane scheduling A/B (GPT-2 XL, 2 groups x 256 rows, one MI355X).

The headline runs two microbatch lanes whose decode steps overlap one
group's HBM-bound attention with the other's GEMM chain.  Both lanes' steps
are captured here into ONE hipGraph on two streams with different cross-lane
dependencies:
  free   -- no cross-lane edges (what two independent per-lane graphs do);
  alt    -- the attention kernels strictly alternate, A(L) -> B(L) -> A(L+1):
            never two attentions at once, so each one shares the chip with
            the other lane's GEMMs only;
  serial -- one stream (no overlap at all).
Prints one JSON line per mode: ms per decode step (both groups), median of
interleaved rounds.  Weights: random init; KV context fixed at CTX positions.
Round 5 (profiles/r5_lane_schedule.log): free 8.40 ms (graph) / 8.36 (eager),
alternating attentions 8.77 (eager), one stream 10.53 -- the free overlap
already beats enforced anti-phase; kept free.  (External event nodes, which
would order two separately launched per-lane graphs, are disallowed by the
ROCm build of torch.)"""
from __future__ import annotations

import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_demo_amd.config import get_model_config  # noqa: E402
from llm_sharding_demo_amd.models.stage import StageModel  # noqa: E402
from llm_sharding_demo_amd.ops import Residual  # noqa: E402
from llm_sharding_demo_amd.runtime.batch import BatchMeta  # noqa: E402

MODEL = os.environ.get("LANE_MODEL", "gpt2-xl")
ROWS = int(os.environ.get("LANE_ROWS", "256"))
CTX = int(os.environ.get("LANE_CTX", "192"))
# hipGraph-replayed, or issued eagerly (-eager)
MODES = os.environ.get("LANE_MODES", "free,free-eager,alt-eager,alt,serial").split(",")


def main():
    dev = torch.device("cuda")
    print("building the stage", flush=True)
    mc = get_model_config(MODEL)
    L = mc.n_layers
    st = StageModel(mc, 0, L, True, True, device=dev, dtype=torch.bfloat16, max_slots=2 * ROWS + 2,
                    max_seq=CTX + 8)
    be = st.backend
    metas = [BatchMeta.decode(list(range(g * ROWS, (g + 1) * ROWS)), [CTX] * ROWS, dev, CTX + 1)
             for g in range(2)]
    ids = [torch.randint(0, mc.vocab_size, (ROWS,), dtype=torch.int32, device=dev) for _ in range(2)]
    orig_attention = be.attention

    def capture(mode):
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        if mode == "serial":
            streams = [streams[0], streams[0]]
        done = {}  # (lane, layer) -> event recorded after that lane's attention
        keep = []  # every event stays alive: an event destroyed mid-capture (a replaced
        # dict entry) crashed hipStreamEndCapture (round-5 log)

        def lane_attention(g, li):
            def att(q, kc, vc, meta):
                cur = torch.cuda.current_stream()
                if mode.startswith("alt"):
                    prev = done.get((1 - g, li)) if g == 1 else done.get((1, li - 1))
                    if prev is not None:
                        cur.wait_event(prev)
                o = orig_attention(q, kc, vc, meta)
                ev = torch.cuda.Event()
                ev.record(cur)
                done[(g, li)] = ev
                keep.append(ev)
                return o
            return att

        def step():
            main_s = torch.cuda.current_stream()
            for s in streams:
                s.wait_stream(main_s)
            res = []
            for g in range(2):
                with torch.cuda.stream(streams[g]):
                    be.lane, be.decode = g, True
                    res.append(Residual(st.embed(ids[g], metas[g])))
            for u in range(2 * L):  # unit u of both lanes; the edges decide the order on the GPU
                i = u >> 1
                for g in range(2):
                    with torch.cuda.stream(streams[g]):
                        be.lane, be.decode = g, True
                        if u & 1:
                            st._gpt2_mlp(i, res[g])
                        else:
                            be.attention = lane_attention(g, i)
                            st._gpt2_attn(st._kv_index[i], i, res[g], metas[g])
                            be.attention = orig_attention
            for g in range(2):
                with torch.cuda.stream(streams[g]):
                    be.lane = g
                    st.head(be.flush(res[g]), metas[g])
            for s in streams:
                main_s.wait_stream(s)

        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            step()  # warm-up (workspace allocations)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        if mode.endswith("-eager"):
            # eager issue: the host issues the ~670 launches of a step well
            # inside its ~8 ms of GPU time
            return step
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step()
        return g.replay

    print("stage built; capturing", flush=True)
    runs = {}
    for m in MODES:
        runs[m] = capture(m)
        print("ready", m, flush=True)
    for r in runs.values():
        r()
    torch.cuda.synchronize()
    times = {m: [] for m in MODES}
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(7):
        for m, r in runs.items():
            s.record()
            for _ in range(5):
                r()
            e.record()
            torch.cuda.synchronize()
            times[m].append(s.elapsed_time(e) / 5)
    for m in MODES:
        print(json.dumps({"model": MODEL, "rows_per_group": ROWS, "ctx": CTX, "mode": m,
                          "ms_per_step": round(statistics.median(times[m]), 3),
                          "min": round(min(times[m]), 3)}), flush=True)


if __name__ == "__main__":
    main()
