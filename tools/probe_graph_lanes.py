#!/usr/bin/env python3
"""Do two hipGraphs on two streams overlap when replayed from one host thread?

Each graph is N small dependent kernels (in-place adds on its own buffer,
~5 us each).  Patterns, timed over R rounds:
  serial   -- one thread, g0 then g1 each round, both on stream 0
  lanes1t  -- one thread alternating g0 (stream A) / g1 (stream B)
  lanes2t  -- two threads, thread i replays g_i on its own stream
Prints wall ms per round and host ms per replay for each.
usage: python tools/probe_graph_lanes.py [nodes] [rounds]
"""
from __future__ import annotations

import sys
import threading
import time

import torch


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda")
    bufs = [torch.zeros(1 << 20, device=dev) for _ in range(2)]
    streams = [torch.cuda.Stream(dev) for _ in range(2)]
    graphs = []
    for i in range(2):
        g = torch.cuda.CUDAGraph()
        s = streams[i]
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                bufs[i].add_(1.0)
            torch.cuda.synchronize()
            g.capture_begin()
            for _ in range(N):
                bufs[i].add_(1.0)
            g.capture_end()
        graphs.append(g)
    torch.cuda.synchronize()

    def run(name, fn):
        host = []
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn(host)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3 / R
        hs = sorted(host)
        print(f"{name:8s} wall/round {wall:8.3f} ms  host/replay p50 {hs[len(hs) // 2] * 1e3:7.3f} ms "
              f"max {hs[-1] * 1e3:7.3f} ms", flush=True)

    def timed_replay(g, host):
        t = time.perf_counter()
        g.replay()
        host.append(time.perf_counter() - t)

    def serial(host):
        for _ in range(R):
            for g in graphs:
                timed_replay(g, host)

    def lanes1t(host):
        for _ in range(R):
            for i, g in enumerate(graphs):
                with torch.cuda.stream(streams[i]):
                    timed_replay(g, host)

    def lanes2t(host):
        def worker(i):
            with torch.cuda.stream(streams[i]):
                for _ in range(R):
                    timed_replay(graphs[i], host)
        ts = [threading.Thread(target=worker, args=(i,)) for i in range(2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()

    for _ in range(2):
        run("serial", serial)
        run("lanes1t", lanes1t)
        run("lanes2t", lanes2t)


if __name__ == "__main__":
    main()
