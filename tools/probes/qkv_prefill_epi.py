"""Probe: cost of the fused QKV epilogue (RoPE + paged-cache scatter) in the 256x256 prefill kernel --
plain bf16 output vs EPI_QKV on the same shapes, hipBLASLt bare matmul as the yardstick."""
import json, os, sys
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_demo_amd.ops.hip import _load, rope_table  # noqa: E402
from microbench import timeit  # noqa: E402
C = _load()
DEV = "cuda"
for label, M, nh, n_kv, hd, H, rope in (("xl", 65536, 25, 25, 64, 1600, False), ("l8", 32768, 32, 8, 128, 4096, True)):
    qs, kvs = nh * hd, n_kv * hd
    N = qs + 2 * kvs
    a = torch.randn(M, H, device=DEV).bfloat16()
    w = (torch.randn(N, H, device=DEV) * 0.02).bfloat16()
    b = None if rope else (torch.randn(N, device=DEV) * 0.1).bfloat16()
    seqs, L = M // 128, 128
    kc = torch.zeros(seqs, n_kv, 256, hd, dtype=torch.bfloat16, device=DEV)
    vc = torch.zeros_like(kc)
    tslot = torch.arange(seqs, device=DEV, dtype=torch.int32).repeat_interleave(L)
    tpos = torch.arange(L, device=DEV, dtype=torch.int32).repeat(seqs)
    table = rope_table(256, hd, 10000.0, DEV) if rope else None
    fl = 2.0 * M * N * H
    t_plain = timeit(lambda: C.linear(a, w, b, 0, True, 1, None), iters=10)
    t_qkv = timeit(lambda: C.linear_qkv(a, w, b, kc, vc, tslot, tpos, qs, kvs, hd, table, True, 1, None), iters=10)
    t_lt = timeit(lambda: torch.matmul(a, w.t()), iters=10)
    print(json.dumps({"case": label, "M": M, "N": N, "K": H, "plain_us": round(t_plain, 1), "qkv_us": round(t_qkv, 1),
                      "hipblaslt_us": round(t_lt, 1), "plain_TF": round(fl / t_plain / 1e6), "qkv_TF": round(fl / t_qkv / 1e6),
                      "hipblaslt_TF": round(fl / t_lt / 1e6)}), flush=True)
