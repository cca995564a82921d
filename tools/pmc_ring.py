"""Decode-shaped GEMMs (GPT-2 XL, 256 rows) on the ring kernel, a few
launches each: a short program for rocprofv3 --pmc passes.
usage: pmc_ring.py [N K]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_sharding_demo_amd.ops.hip import _load  # noqa: E402

C = _load()
N, K = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (4800, 1600)
M = 256
C.gemm_set_tiled3_max(512)
C.gemm_set_ring_tn(0)
a = torch.randn(M, K, device="cuda").bfloat16()
w = torch.randn(N, K, device="cuda").bfloat16()
b = torch.randn(N, device="cuda").bfloat16()
for _ in range(5):
    C.linear(a, w, b, 0, True, 1, None)
torch.cuda.synchronize()
print("done")
