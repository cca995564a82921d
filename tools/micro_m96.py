import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo") + "/tools")
sys.argv = ["microbench.py", "none"]
import microbench as mb
import torch
C, DEV = mb.C, mb.DEV
cnt = torch.zeros(1 << 16, dtype=torch.int32, device=DEV)
C.gemm_set_tiled3_max(512); C.gemm_set_ring_tn(0)
for M in (256, 192, 160):
    for name, N, K, act in (("qkv", 4800, 1600, 0), ("fc", 6400, 1600, 1), ("small_qkv", 2304, 768, 0), ("small_fc", 3072, 768, 1)):
        a = torch.randn(M, K, device=DEV).bfloat16()
        ws = mb.rotating(lambda: torch.randn(N, K, device=DEV).bfloat16(), N * K * 2)
        for m96 in (0, 256):
            C.gemm_set_ring_m96(m96)
            it = [0]
            def run(it=it):
                w = ws[it[0] % len(ws)]; it[0] += 1
                C.linear(a, w, None, act, True, 1, cnt)
            mb.report(f"{name} M={M} N={N} K={K} m96={m96}", mb.timeit(run), N * K * 2)
