"""Serving metrics (Prometheus text exposition).

The reference has no metrics beyond uvicorn's access log and minikube's
metrics-server.  This tracks requests, output tokens,
aggregate tok/s and per-token latency percentiles (from the engine's per-step
hipEvent timings).
"""
from __future__ import annotations

import threading
import time
from collections import deque
from typing import Dict, Iterable


def percentile(xs, q: float) -> float:
    xs = sorted(xs)
    if not xs:
        return 0.0
    k = (len(xs) - 1) * q
    lo, hi = int(k), min(int(k) + 1, len(xs) - 1)
    return xs[lo] + (xs[hi] - xs[lo]) * (k - lo)


class Metrics:
    def __init__(self, window: int = 4096):
        self._lock = threading.Lock()
        self.requests = 0
        self.tokens = 0
        self.busy_s = 0.0
        self.t0 = time.time()
        self.step_ms = deque(maxlen=window)
        self.request_s = deque(maxlen=window)

    def observe_request(self, n_tokens: int, seconds: float) -> None:
        with self._lock:
            self.requests += 1
            self.tokens += n_tokens
            self.busy_s += seconds
            self.request_s.append(seconds)

    def observe_steps(self, steps_ms: Iterable[float]) -> None:
        with self._lock:
            self.step_ms.extend(steps_ms)

    def snapshot(self) -> Dict[str, float]:
        with self._lock:
            st = list(self.step_ms)
            return {
                "requests_total": self.requests,
                "output_tokens_total": self.tokens,
                "output_tokens_per_second": self.tokens / self.busy_s if self.busy_s else 0.0,
                "token_latency_p50_ms": percentile(st, 0.5),
                "token_latency_p90_ms": percentile(st, 0.9),
                "request_latency_p50_s": percentile(list(self.request_s), 0.5),
                "uptime_seconds": time.time() - self.t0,
            }

    def render(self, extra: Dict[str, float] = None) -> str:
        snap = self.snapshot()
        snap.update(extra or {})
        lines = []
        for k, v in snap.items():
            lines.append(f"# TYPE llmshard_{k} gauge")
            lines.append(f"llmshard_{k} {float(v):.6g}")
        return "\n".join(lines) + "\n"
