"""GPT-2 XL QKV at 256 rows on the 8-wave decode ring (gemm_ring8_kernel),
a few launches over rotating weights (cold, as in the decode step): a short
program for rocprofv3 --pmc passes (tools/gpu_r3_pmc_ring8.sh)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_sharding_demo_amd.ops.hip import HipBackend, _load  # noqa: E402

C = _load()
HipBackend()  # engine routing (8-wave ring)
N, K = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (4800, 1600)
M = 256
ws = [torch.randn(N, K, device="cuda").mul_(0.02).bfloat16() for _ in range(24)]
a = torch.randn(M, K, device="cuda").bfloat16()
b = torch.randn(N, device="cuda").bfloat16()
for i in range(24):
    C.linear(a, ws[i], b, 0, True, 1, None)
torch.cuda.synchronize()
print("done")
