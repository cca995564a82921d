"""One prefill-shaped GEMM per large-GEMM kernel kind, a few launches each
(a short program for rocprofv3 --pmc passes).  usage: pmc_bigemm.py [N K]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_sharding_demo_amd.ops.hip import _load  # noqa: E402

C = _load()
N, K = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (6400, 1600)
M = 65536
a = torch.randn(M, K, device="cuda").bfloat16()
w = torch.randn(N, K, device="cuda").bfloat16()
b = torch.randn(N, device="cuda").bfloat16()
C.gemm_set_big_min(1)
for kind in (0, 1):
    C.gemm_set_big_kind(kind)
    for _ in range(3):
        C.linear(a, w, b, 1, True, 1, None)
torch.cuda.synchronize()
print("done")
