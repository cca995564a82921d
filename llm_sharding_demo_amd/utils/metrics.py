"""Serving metrics (Prometheus text exposition).

The reference has no metrics beyond uvicorn's access log and minikube's
metrics-server.  This tracks requests and output tokens
(counters), throughput over wall-clock windows (concurrent requests overlap,
so summing per-request latencies would under-report by the concurrency),
time to first token, request latency, and per-token (decode step) latency
percentiles from the engine's hipEvent step timings.
"""
from __future__ import annotations

import time
from collections import deque
from typing import Dict, Iterable, Optional

from . import racecheck


def percentile(xs, q: float) -> float:
    xs = sorted(xs)
    if not xs:
        return 0.0
    k = (len(xs) - 1) * q
    lo, hi = int(k), min(int(k) + 1, len(xs) - 1)
    return xs[lo] + (xs[hi] - xs[lo]) * (k - lo)


class Metrics(racecheck.Shared):
    def __init__(self, window: int = 4096, rate_window_s: float = 60.0):
        self._lock = racecheck.Lock("metrics")
        self.requests = 0
        self.tokens = 0
        self.t0 = time.monotonic()
        self.rate_window_s = rate_window_s
        self.step_ms = deque(maxlen=window)
        self.request_s = deque(maxlen=window)
        self.ttft_s = deque(maxlen=window)
        self._done = deque()          # (finish time, tokens) inside the rate window
        self._first_done: Optional[float] = None
        self._last_steps_key = None

    def observe_request(self, n_tokens: int, seconds: float, ttft_s: Optional[float] = None) -> None:
        now = time.monotonic()
        with self._lock:
            racecheck.note(self, "_done")
            self.requests += 1
            self.tokens += n_tokens
            self.request_s.append(seconds)
            if ttft_s is not None:
                self.ttft_s.append(ttft_s)
            self._done.append((now, n_tokens, now - seconds))
            while self._done and self._done[0][0] < now - self.rate_window_s:
                self._done.popleft()
            if self._first_done is None:
                self._first_done = now - seconds

    def observe_steps(self, steps_ms: Iterable[float], key=None) -> None:
        with self._lock:
            if key is not None and key == self._last_steps_key:
                return  # the same session's steps are only counted once
            self._last_steps_key = key
            racecheck.note(self, "step_ms")
            self.step_ms.extend(steps_ms)

    def tokens_per_second(self) -> float:
        """Output tokens finished in the rate window / wall-clock span of the
        window (from the earliest start of a request in it to now)."""
        now = time.monotonic()
        with self._lock:
            if not self._done:
                return 0.0
            start = min(s for _, _, s in self._done)
            span = max(now - start, 1e-9)
            return sum(n for _, n, _ in self._done) / span

    def snapshot(self) -> Dict[str, Dict[str, float]]:
        tps = self.tokens_per_second()
        with self._lock:
            st = list(self.step_ms)
            return {
                "counter": {
                    "requests_total": self.requests,
                    "output_tokens_total": self.tokens,
                },
                "gauge": {
                    "output_tokens_per_second": tps,
                    "token_latency_p50_ms": percentile(st, 0.5),
                    "token_latency_p90_ms": percentile(st, 0.9),
                    "time_to_first_token_p50_s": percentile(list(self.ttft_s), 0.5),
                    "time_to_first_token_p90_s": percentile(list(self.ttft_s), 0.9),
                    "request_latency_p50_s": percentile(list(self.request_s), 0.5),
                    "uptime_seconds": time.monotonic() - self.t0,
                },
            }

    def render(self, gauges: Dict[str, float] = None, counters: Dict[str, float] = None) -> str:
        snap = self.snapshot()
        snap["gauge"].update(gauges or {})
        snap["counter"].update(counters or {})
        lines = []
        for typ in ("counter", "gauge"):
            for k, v in snap[typ].items():
                lines.append(f"# TYPE llmshard_{k} {typ}")
                lines.append(f"llmshard_{k} {float(v):.6g}")
        return "\n".join(lines) + "\n"
