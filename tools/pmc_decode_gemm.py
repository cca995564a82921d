"""A short program for rocprofv3 --pmc passes over ONE decode GEMM variant at
256 rows (GPT-2 XL QKV shape by default): 20 launches over rotating weights
(cold, like the model's weight stream).
usage: pmc_decode_gemm.py CASE [N K]   CASE = ring8 | ring
(the round-5 passes also ran the W-to-VGPR kernel, since removed: git history)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_sharding_demo_amd.ops.hip import HipBackend, _load  # noqa: E402

C = _load()
HipBackend()  # production GEMM routing knobs (8-wave ring, tiled3 caps)
case = sys.argv[1]
N, K = (int(sys.argv[2]), int(sys.argv[3])) if len(sys.argv) > 3 else (4800, 1600)
M = 256
a = torch.randn(M, K, device="cuda").bfloat16()
ws = [torch.randn(N, K, device="cuda").mul_(0.02).bfloat16() for _ in range(max(2, (640 << 20) // (N * K * 2)))]
b = torch.randn(N, device="cuda").bfloat16()
kind = 1
if case == "ring":
    C.gemm_set_ring8(0)
for i in range(20):
    C.linear(a, ws[i % len(ws)], b, 0, kind, 1, None)
torch.cuda.synchronize()
print("done", case, N, K)
