"""Per-workgroup timeline of the 256x256 prefill GEMM (gemm_p8) at the GPT-2 XL
prefill shapes (65 K rows): prologue / main loop / epilogue per block and the
per-CU sum against the span (the gap = dispatch between consecutive blocks)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import microbench as mb  # noqa: E402

for N, K, act in ((6400, 1600, 1), (4800, 1600, 0), (1600, 1600, 0), (1600, 6400, 0)):
    mb.stamps_p8(65536, N, K, act)
