"""roctx trace ranges (rocprofv3 --marker-trace shows them on the timeline).

The reference has no tracing (`time` is imported and unused, `server.py:3`).
Ranges are opened around each stage's forward and each inter-stage transfer
when LSD_TRACE=1; torch.cuda.nvtx maps to roctx on ROCm builds.  Off by
default: a range push/pop is a host call per op.
"""
from __future__ import annotations

import contextlib
import os

ENABLED = os.environ.get("LSD_TRACE", "0") == "1"


@contextlib.contextmanager
def trace_range(name: str):
    if not ENABLED:
        yield
        return
    import torch

    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()
