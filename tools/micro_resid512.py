"""Residual projections at 512 decode rows: K-split count (2 = current
routing, 128x64 ring; >= 5 puts the grid on the 256x256 p8 kernel) timed
together with the norm that folds the slabs in.  us per (GEMM + norm)."""
import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo") + "/tools")
sys.argv = ["microbench.py", "none"]
import microbench as mb
import torch
C, DEV = mb.C, mb.DEV
cnt = torch.zeros(1 << 16, dtype=torch.int32, device=DEV)
M = 512
for name, N, K, rms in (("llama_down", 4096, 14336, True), ("llama_o", 4096, 4096, True),
                        ("xl_down", 1600, 6400, False), ("xl_o", 1600, 1600, False)):
    a = torch.randn(M, K, device=DEV).bfloat16()
    x = torch.randn(M, N, device=DEV)
    g = torch.ones(N, device=DEV).bfloat16()
    b = None if rms else torch.zeros(N, device=DEV).bfloat16()
    ws = mb.rotating(lambda: (torch.randn(N, K, device=DEV) * 0.02).bfloat16(), N * K * 2)
    for s in (2, 4, 6, 8, 12, 16):
        if K // 64 < s:
            continue
        it = [0]
        def run(it=it, s=s):
            w = ws[it[0] % len(ws)]; it[0] += 1
            slab = C.linear_residual(a, w, None, x, s, True, cnt, True)
            C.norm(x, slab, None, g, b, 1e-5, rms, None, True)
        mb.report(f"{name} M={M} N={N} K={K} splits={s}", mb.timeit(run), N * K * 2)
