"""Prefill GEMM kernel (gemm_p8_kernel) and hipBLASLt on the same operands, a few
launches each: a short program for rocprofv3 --kernel-trace / --pmc passes
(tools/gpu_r3_pmc_p8.sh).  The hipBLASLt kernel name carries its macro tile."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_sharding_demo_amd.ops.hip import _load  # noqa: E402

C = _load()
shapes = [(65536, 6400, 1600), (4096, 4096, 4096)]
if len(sys.argv) > 3:
    shapes = [tuple(int(v) for v in sys.argv[1:4])]
C.gemm_set_big_min(1)
for M, N, K in shapes:
    a = torch.randn(M, K, device="cuda").bfloat16()
    w = torch.randn(N, K, device="cuda").bfloat16()
    for _ in range(3):
        C.linear(a, w, None, 0, True, 1, None)
    for _ in range(3):
        torch.matmul(a, w.t())
    torch.cuda.synchronize()
print("done")
