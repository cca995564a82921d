"""Repeat one W-to-VGPR GEMM config (residual slabs, 256 rows) against the fp32
reference and count mismatching launches -- a numerics probe for an
intermittent ordering bug, not a fault test."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_demo_amd.ops.hip import _load  # noqa: E402
from llm_sharding_demo_amd.ops import reference as ref  # noqa: E402

C = _load()
C.gemm_set_slab_bf16(0)
for code in [int(c) for c in sys.argv[1:]] or [664]:
    C.gemm_set_vw(code)
    for (M, K, S) in [(256, 640, 2), (256, 1600, 1), (200, 384, 3)]:
        g = torch.Generator(device="cuda").manual_seed(1)
        a = (torch.randn(M, K, generator=g, device="cuda")).bfloat16()
        w = (torch.randn(320, K, generator=g, device="cuda") * 0.05).bfloat16()
        y_ref = ref.linear(a, w, None)
        bad = 0
        worst = 0.0
        for it in range(40):
            if S > 1:
                slab = C.linear_residual(a, w, None, torch.zeros(M, 320, device="cuda"), S, 4, None, False)
                y = slab.float().sum(0)
            else:
                y = C.linear_f32(a, w, 4, 1, None)
            d = float((y - y_ref).abs().max())
            worst = max(worst, d)
            bad += d > 2e-3 * 50
        print(f"vw{code} M={M} K={K} S={S}: bad launches {bad}/40, worst |diff| {worst:.4g}", flush=True)
