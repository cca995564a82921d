"""Residual projections at 256 decode rows: K splits x kernel (tiled3_max 512
= 128x64 ring as routed today; 0 = the 2-blocks/CU 128x128 tiled kernel),
GEMM + slab-folding norm, us."""
import sys, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo") + "/tools")
sys.argv = ["microbench.py", "none"]
import microbench as mb
import torch
C, DEV = mb.C, mb.DEV
cnt = torch.zeros(1 << 16, dtype=torch.int32, device=DEV)
C.gemm_set_ring_tn(0)
M = 256
for name, N, K, rms in (("xl_down", 1600, 6400, False), ("xl_o", 1600, 1600, False),
                        ("llama_down", 4096, 14336, True), ("llama_o", 4096, 4096, True)):
    a = torch.randn(M, K, device=DEV).bfloat16()
    x = torch.randn(M, N, device=DEV)
    g = torch.ones(N, device=DEV).bfloat16()
    b = None if rms else torch.zeros(N, device=DEV).bfloat16()
    ws = mb.rotating(lambda: (torch.randn(N, K, device=DEV) * 0.02).bfloat16(), N * K * 2)
    for t3 in (512, 0):
        C.gemm_set_tiled3_max(t3)
        for s in (2, 3, 5, 8, 12):
            it = [0]
            def run(it=it, s=s):
                w = ws[it[0] % len(ws)]; it[0] += 1
                slab = C.linear_residual(a, w, None, x, s, True, cnt, True)
                C.norm(x, slab, None, g, b, 1e-5, rms, None, True)
            mb.report(f"{name} M={M} K={K} t3={t3} splits={s}", mb.timeit(run), N * K * 2)
C.gemm_set_tiled3_max(512)
