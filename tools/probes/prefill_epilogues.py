"""Probe: what each fused epilogue of the 256x256 prefill kernel (gemm_p8) costs on the GPT-2 XL
65 K-row prefill shapes -- the same GEMM with a plain bf16 store against QKV (paged-cache scatter),
bias + GELU and the fp32 residual read-modify-write; hipBLASLt's bare matmul as the yardstick."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_demo_amd.ops.hip import _load  # noqa: E402
from microbench import timeit  # noqa: E402

C = _load()
DEV = "cuda"
M, H, F, nh, hd = 65536, 1600, 6400, 25, 64
a = torch.randn(M, H, device=DEV).bfloat16()
a4 = torch.randn(M, F, device=DEV).bfloat16()
seqs, L = M // 128, 128
kc = torch.zeros(seqs, nh, 256, hd, dtype=torch.bfloat16, device=DEV)
vc = torch.zeros_like(kc)
tslot = torch.arange(seqs, device=DEV, dtype=torch.int32).repeat_interleave(L)
tpos = torch.arange(L, device=DEV, dtype=torch.int32).repeat(seqs)
x = torch.randn(M, H, device=DEV)


def row(case, N, K, t, t_lt):
    fl = 2.0 * M * N * K
    print(json.dumps({"case": case, "M": M, "N": N, "K": K, "us": round(t, 1), "TF": round(fl / t / 1e6),
                      "hipblaslt_us": round(t_lt, 1)}), flush=True)


for case, N, K, A in (("qkv", 3 * H, H, a), ("fc", F, H, a), ("proj", H, H, a), ("proj2", H, F, a4)):
    w = (torch.randn(N, K, device=DEV) * 0.02).bfloat16()
    b = (torch.randn(N, device=DEV) * 0.1).bfloat16()
    t_lt = timeit(lambda: torch.matmul(A, w.t()), iters=10)
    row(f"{case} plain bf16", N, K, timeit(lambda: C.linear(A, w, b, 0, True, 1, None), iters=10), t_lt)
    if case == "qkv":
        row("qkv fused (cache scatter)", N, K, timeit(lambda: C.linear_qkv(A, w, b, kc, vc, tslot, tpos, H, H, hd,
                                                                         None, True, 1, None), iters=10), t_lt)
    if case == "fc":
        row("fc bias+gelu_new", N, K, timeit(lambda: C.linear(A, w, b, 1, True, 1, None), iters=10), t_lt)
    if case.startswith("proj"):
        row(f"{case} fp32 residual RMW", N, K,
            timeit(lambda: C.linear_residual(A, w, b, x, 1, True, None, False), iters=10), t_lt)
