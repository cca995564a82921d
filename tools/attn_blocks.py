#!/usr/bin/env python3
"""Decode attention block shape at full batches (attn_decode_kernel): 4 waves with 4 keys per
wave in flight (default), 8 waves, 4 waves with 2 in flight (fewer registers, more blocks per CU)
and 2-wave blocks -- GPT-2 small (12 heads) and XL (25 heads) at 256 sequences, 128-256 keys;
Llama-3 8B (GQA, 8 kv heads x 128) for reference."""
from __future__ import annotations

import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from microbench import C, bench_attn_decode  # noqa: E402

for lw in (4, 8, 42, 2):
    C.attn_set_large_waves(64, lw)
    C.attn_set_large_waves(128, lw)
    print("large_waves", lw, flush=True)
    for ctx in (128, 192, 256):
        bench_attn_decode(256, 12, 12, 64, ctx)
        bench_attn_decode(256, 25, 25, 64, ctx)
    bench_attn_decode(128, 32, 32, 128, 192)
C.attn_set_large_waves(64, 4)
C.attn_set_large_waves(128, 4)
