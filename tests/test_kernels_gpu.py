"""HIP kernel numerics on an MI355X, each vs a plain PyTorch fp32 reference
(ops/reference.py) of the same op.  bf16 inputs, fp32 accumulation.
"""
import math

import pytest
import torch

from llm_sharding_demo_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

DEV = "cuda"


@pytest.fixture(scope="module")
def C():
    from llm_sharding_demo_amd.ops.hip import _load

    return _load()


def bf(*shape, scale=1.0, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return (torch.randn(*shape, generator=g, device=DEV) * scale).to(torch.bfloat16)


def close(a, b, atol, rtol=2e-2):
    torch.testing.assert_close(a.float().cpu(), b.float().cpu(), atol=atol, rtol=rtol)


def test_embed(C):
    V, H, P, T = 1000, 256, 64, 37
    wte, wpe = bf(V, H, seed=1), bf(P, H, seed=2)
    ids = torch.randint(0, V, (T,), dtype=torch.int32, device=DEV)
    pos = torch.randint(0, P, (T,), dtype=torch.int32, device=DEV)
    close(C.embed(ids, pos, wte, wpe), ref.embed(ids, pos, wte, wpe), 1e-6)
    close(C.embed(ids, pos, wte, None), ref.embed(ids, pos, wte, None), 1e-6)


@pytest.mark.parametrize("H", [128, 768, 1600, 4096, 8192])
@pytest.mark.parametrize("rms", [False, True])
@pytest.mark.parametrize("S", [1, 3, 8, 12])  # exact-count unrolled slabs (<= 8) and runtime loop
@pytest.mark.parametrize("sdt", [torch.float32, torch.bfloat16])  # LSD_SLAB_BF16 slabs
def test_norm_with_slab_combine(C, H, rms, S, sdt):
    T = 19
    x = torch.randn(T, H, device=DEV)
    slab = (torch.randn(S, T, H, device=DEV) * 0.1).to(sdt)
    pb = bf(H, scale=0.1, seed=3)
    w, b = (1 + 0.1 * torch.randn(H, device=DEV)).bfloat16(), bf(H, scale=0.1, seed=4)
    x_ref = x + slab.float().sum(0) + pb.float()
    y_ref = ref.rmsnorm(x_ref, w, 1e-5) if rms else ref.layernorm(x_ref, w, b, 1e-5)
    y = C.norm(x, slab, pb, w, None if rms else b, 1e-5, rms, None, True)
    close(x, x_ref, 1e-5)
    close(y, y_ref, 2e-2)
    rows = torch.tensor([3, 0, 18], dtype=torch.int32, device=DEV)
    y2 = C.norm(x, None, None, w, None if rms else b, 1e-5, rms, rows, True)
    close(y2, y_ref[rows.long()], 2e-2)


@pytest.mark.parametrize("H", [768, 1024, 516, 1600])  # 1600: the block kernel (narrow threshold: H <= 1024)
@pytest.mark.parametrize("rms", [False, True])
@pytest.mark.parametrize("S", [1, 3, 6, 8, 12])  # 12: folded by the block kernel first, then the wave kernel
@pytest.mark.parametrize("sdt", [torch.float32, torch.bfloat16])
def test_norm_wave_with_slabs(C, H, rms, S, sdt):
    """Norms that fold split-K slabs on the wave-per-row kernel (H <= 1024 from
    lsd_norm_set_wave_narrow_min rows, forced from 1 row here): the folded
    residual is bit-equal to the block kernel's (same add order), the output
    matches the fp32 reference and the block kernel; 258 rows leave a partial
    last block of 4."""
    T = 258
    x0 = torch.randn(T, H, device=DEV)
    slab = (torch.randn(S, T, H, device=DEV) * 0.1).to(sdt)
    pb = bf(H, scale=0.1, seed=3)
    w, b = (1 + 0.1 * torch.randn(H, device=DEV)).bfloat16(), bf(H, scale=0.1, seed=4)
    x_ref = x0 + slab.float().sum(0) + pb.float()
    y_ref = ref.rmsnorm(x_ref, w, 1e-5) if rms else ref.layernorm(x_ref, w, b, 1e-5)
    C.norm_set_wave_min(0)
    C.norm_set_wave_narrow_min(0)
    xb = x0.clone()
    yb = C.norm(xb, slab, pb, w, None if rms else b, 1e-5, rms, None, True)  # block kernel
    C.norm_set_wave_narrow_min(1)
    try:
        x = x0.clone()
        y = C.norm(x, slab, pb, w, None if rms else b, 1e-5, rms, None, True)
    finally:
        _norm_defaults(C)
    assert torch.equal(x, xb)
    close(x, x_ref, 1e-5)
    close(y, y_ref, 2e-2)
    close(y, yb, 2e-2)


def _norm_defaults(C):
    from llm_sharding_demo_amd.ops.hip import HipBackend

    C.norm_set_wave_min(HipBackend.R.norm_wave_min)
    C.norm_set_wave_narrow_min(HipBackend.R.norm_wave_narrow_min)


@pytest.mark.parametrize("T,H", [(258, 768), (258, 1600), (4099, 768), (4099, 1600), (100, 768)])
@pytest.mark.parametrize("S", [3, 6, 12])
def test_norm_slab_fold_equals_flush_then_norm(C, T, H, S):
    """The engine's kernel choice for a norm depends on (rows, H) only: a norm
    that folds pending slabs and the same norm after a separate fold (what a
    pipeline stage boundary does) give bit-identical residuals and outputs at
    the default thresholds -- the property that keeps a P-stage pipeline
    equal to one stage."""
    _norm_defaults(C)
    x0 = torch.randn(T, H, device=DEV)
    slab = (torch.randn(S, T, H, device=DEV) * 0.1).bfloat16()
    pb = bf(H, scale=0.1, seed=3)
    w, b = (1 + 0.1 * torch.randn(H, device=DEV)).bfloat16(), bf(H, scale=0.1, seed=4)
    x1, x2 = x0.clone(), x0.clone()
    y1 = C.norm(x1, slab, pb, w, b, 1e-5, False, None, True)
    C.norm(x2, slab, pb, None, None, 0.0, True, None, False)  # fold only (stage-boundary flush)
    y2 = C.norm(x2, None, None, w, b, 1e-5, False, None, True)
    assert torch.equal(x1, x2)
    assert torch.equal(y1, y2)


@pytest.mark.parametrize("H", [768, 1600, 4096, 1036])
@pytest.mark.parametrize("rms", [False, True])
@pytest.mark.parametrize("T", [5, 4099])
def test_norm_wave_per_row(C, H, rms, T):
    """Prefill norms at >= lsd_norm_set_wave_min rows run one wave per row
    (norm.hip norm_wave_kernel; forced on here from 1 row): against the fp32
    reference, odd row counts (a partial last block of 4 rows) and an H whose
    16-byte chunks do not fill the lanes evenly; x is left untouched."""
    C.norm_set_wave_min(1)
    try:
        x = torch.randn(T, H, device=DEV) * 2 + 0.5
        x0 = x.clone()
        w, b = (1 + 0.1 * torch.randn(H, device=DEV)).bfloat16(), bf(H, scale=0.1, seed=5)
        y = C.norm(x, None, None, w, None if rms else b, 1e-5, rms, None, True)
        y_ref = ref.rmsnorm(x, w, 1e-5) if rms else ref.layernorm(x, w, b, 1e-5)
        close(y, y_ref, 2e-2)
        assert torch.equal(x, x0)
    finally:
        _norm_defaults(C)


@pytest.fixture(scope="module")
def CNT():
    return torch.zeros(1 << 16, dtype=torch.int32, device=DEV)


@pytest.fixture(autouse=True)
def _fp32_slabs(C):
    """The GEMM tests below check split-K residual slabs at fp32 precision; the
    bf16 slabs of production decode (LSD_SLAB_BF16) have their own test."""
    prev = C.gemm_slab_bf16()
    C.gemm_set_slab_bf16(0)
    yield
    C.gemm_set_slab_bf16(int(prev))


# 8-wave decode ring (256 / 130 rows), split-K decode kernel (64 rows, deferred) and the
# 256x256 prefill-class kernel (1024 rows x 6 splits = 168 tiles)
@pytest.mark.parametrize("tiled,M,splits", [(True, 256, 3), (True, 256, 5), (True, 130, 3), (False, 64, 5),
                                            (True, 1024, 6), (True, 1024, 1), (True, 3000, 1)])
def test_linear_residual_bf16_slabs(C, CNT, tiled, M, splits):
    """bf16 partial slabs: each split's partial rounded once to bf16 (a bf16
    GEMM output's precision), folded into the fp32 residual by the norm.  One
    split with defer: the prefill form (the GEMM writes one bf16 slab instead
    of a read-modify-write of the fp32 residual)."""
    C.gemm_set_slab_bf16(1)
    N, K = 1600, 1600
    a, w, bias = bf(M, K, seed=8), bf(N, K, scale=0.05, seed=9), bf(N, scale=0.1, seed=10)
    x = torch.randn(M, N, device=DEV)
    y = ref.linear(a, w, bias)
    x_ref = x + y
    slab = C.linear_residual(a, w, bias, x, splits, tiled, CNT, not tiled or splits == 1)
    assert slab is not None and slab.dtype == torch.bfloat16 and slab.shape == (splits, M, N)
    C.norm(x, slab, bias, None, None, 0.0, True, None, False)
    # error of S bf16 roundings of partials of |y| / sqrt(S)-ish size
    err = (x - x_ref).abs()
    assert float(err.max()) <= 2.0 ** -8 * float(y.abs().max()) * splits, float(err.max())
    assert float(err.mean()) <= 2.0 ** -9 * float(y.abs().mean()) * 2, float(err.mean())


@pytest.mark.parametrize("M", [1, 5, 16, 33, 64, 65, 100, 128, 200])
@pytest.mark.parametrize("act", ["none", "gelu", "silu_mul"])
@pytest.mark.parametrize("splits", [1, 3, 7])
def test_linear(C, CNT, M, act, splits):
    from llm_sharding_demo_amd.ops.hip import interleave_gate_up

    N, K = 384, 640
    a, w, bias = bf(M, K, seed=5), bf(N, K, scale=0.05, seed=6), bf(N, scale=0.1, seed=7)
    tiled = M > 128
    sp = 1 if tiled else splits
    if act == "silu_mul":
        N = 256
        w = w[:N].contiguous()
        y = C.linear(a, interleave_gate_up(w, N // 2).contiguous(), None, 2, tiled, sp, CNT)
        y_ref = ref.silu_mul(*ref.linear(a, w).split(N // 2, 1))
    else:
        y = C.linear(a, w, bias, 1 if act == "gelu" else 0, tiled, sp, CNT)
        y_ref = ref.linear(a, w, bias)
        if act == "gelu":
            y_ref = ref.gelu_new(y_ref)
    close(y, y_ref, 3e-2)
    assert int(CNT.abs().sum()) == 0  # every ticket counter re-armed


@pytest.mark.parametrize("M,splits", [(3, 1), (16, 4), (64, 5), (64, 16), (100, 1), (128, 5), (130, 3)])
@pytest.mark.parametrize("defer", [False, True])
def test_linear_residual_and_f32(C, CNT, M, splits, defer):
    N, K = 256, 1024
    a, w, bias = bf(M, K, seed=8), bf(N, K, scale=0.05, seed=9), bf(N, scale=0.1, seed=10)
    tiled = M > 128
    x = torch.randn(M, N, device=DEV)
    x_ref = x + ref.linear(a, w, bias)
    slab = C.linear_residual(a, w, bias, x, splits, tiled, CNT, defer)
    assert (slab is not None) == ((tiled or defer) and splits > 1)
    if slab is not None:
        C.norm(x, slab, bias, None, None, 0.0, True, None, False)
    close(x, x_ref, 2e-3, 1e-3)
    close(C.linear_f32(a, w, tiled, 1 if tiled else splits, CNT), ref.linear(a, w), 2e-3, 1e-3)


@pytest.mark.parametrize("M", [1, 40, 128])
def test_decode_gemm_wide_partial_tiles(C, CNT, M):
    """128-column decode tiles (NW = 2) with a masked partial last tile
    (N = 320 = 2.5 tiles): plain, GELU, split-K residual and fp32 epilogues."""
    C.gemm_set_nw2_rows(0)
    try:
        N, K = 320, 512
        a, w, bias = bf(M, K, seed=40), bf(N, K, scale=0.05, seed=41), bf(N, scale=0.1, seed=42)
        assert C.gemm_sk_nw(M, 0) == 2
        for sp in (1, 3):
            close(C.linear(a, w, bias, 1, False, sp, CNT), ref.gelu_new(ref.linear(a, w, bias)), 3e-2)
            close(C.linear_f32(a, w, False, sp, CNT), ref.linear(a, w), 2e-3, 1e-3)
            x = torch.randn(M, N, device=DEV)
            x_ref = x + ref.linear(a, w, bias)
            C.linear_residual(a, w, bias, x, sp, False, CNT, False)
            close(x, x_ref, 2e-3, 1e-3)
        assert int(CNT.abs().sum()) == 0
    finally:
        C.gemm_set_nw2_rows(1 << 30)


@pytest.mark.parametrize("M", [129, 200, 256])
@pytest.mark.parametrize("splits", [1, 3])
def test_decode_gemm_two_row_blocks(C, CNT, M, splits):
    """Decode GEMM above 128 rows runs as >= 2 row blocks of <= 128 (grid z)
    sharing each W tile: plain / GELU / SiLU-mul / fp32 / residual epilogues."""
    from llm_sharding_demo_amd.ops.hip import interleave_gate_up

    N, K = 384, 640
    a, w, bias = bf(M, K, seed=50), bf(N, K, scale=0.05, seed=51), bf(N, scale=0.1, seed=52)
    assert C.gemm_sk_rblocks(M, N, splits) >= 2
    close(C.linear(a, w, bias, 0, False, splits, CNT), ref.linear(a, w, bias), 3e-2)
    close(C.linear(a, w, bias, 1, False, splits, CNT), ref.gelu_new(ref.linear(a, w, bias)), 3e-2)
    close(C.linear_f32(a, w, False, splits, CNT), ref.linear(a, w), 2e-3, 1e-3)
    w2 = w[:256].contiguous()
    y = C.linear(a, interleave_gate_up(w2, 128).contiguous(), None, 2, False, splits, CNT)
    close(y, ref.silu_mul(*ref.linear(a, w2).split(128, 1)), 3e-2)
    for defer in (False, True):
        x = torch.randn(M, N, device=DEV)
        x_ref = x + ref.linear(a, w, bias)
        slab = C.linear_residual(a, w, bias, x, splits, False, CNT, defer)
        if slab is not None:
            C.norm(x, slab, bias, None, None, 0.0, True, None, False)
        close(x, x_ref, 2e-3, 1e-3)
    assert int(CNT.abs().sum()) == 0


def test_split_k_deterministic(C, CNT):
    a, w = bf(64, 1600, seed=30), bf(4800, 1600, scale=0.03, seed=31)
    y1 = C.linear(a, w, None, 0, False, 7, CNT)
    for _ in range(5):
        assert torch.equal(C.linear(a, w, None, 0, False, 7, CNT), y1)


def test_gemm_large_prefill_shape(C, CNT):
    M, N, K = 1000, 4800, 1600
    a, w = bf(M, K, seed=11), bf(N, K, scale=0.03, seed=12)
    close(C.linear(a, w, None, 0, True, 1, CNT), ref.linear(a, w), 3e-2)


@pytest.fixture(params=[(3, 128), (4, 128), (3, 64), (3, 32), (3, 0)])
def RING(C, request):
    """Route every tiled launch to the LDS ring variant: 3 or 4 slots of
    128x128 tiles, or 3 slots of 128x64 / 128x32 tiles (0: auto width)."""
    slots, tn = request.param
    C.gemm_set_tiled3_max(1 << 30)
    C.gemm_set_ring_slots(slots)
    C.gemm_set_ring_tn(tn)
    yield C
    C.gemm_set_tiled3_max(0)
    C.gemm_set_ring_slots(3)
    C.gemm_set_ring_tn(128)


@pytest.mark.parametrize("M", [100, 256, 300])
@pytest.mark.parametrize("K", [64, 128, 192, 256, 640])
def test_ring_gemm_epilogues(RING, CNT, M, K):
    """Ring 128x128 kernel: every epilogue, M/N tails, 1, 2, 3, 4 and 10
    k-steps (fewer than, equal to and more than the ring), split-K slabs."""
    from llm_sharding_demo_amd.ops.hip import interleave_gate_up

    C = RING
    N = 352  # 2.75 tiles of 128 columns, 5.5 of 64: a partial last tile either way
    a, w, bias = bf(M, K, seed=60), bf(N, K, scale=0.05, seed=61), bf(N, scale=0.1, seed=62)
    y_ref = ref.linear(a, w, bias)
    close(C.linear(a, w, bias, 0, True, 1, CNT), y_ref, 3e-2)
    close(C.linear(a, w, bias, 1, True, 1, CNT), ref.gelu_new(y_ref), 3e-2)
    w2 = w[:256].contiguous()
    y = C.linear(a, interleave_gate_up(w2, 128).contiguous(), None, 2, True, 1, CNT)
    close(y, ref.silu_mul(*ref.linear(a, w2).split(128, 1)), 3e-2)
    close(C.linear_f32(a, w, True, 1, CNT), ref.linear(a, w), 2e-3, 1e-3)
    x = torch.randn(M, N, device=DEV)
    x_ref = x + y_ref
    assert C.linear_residual(a, w, bias, x, 1, True, CNT, False) is None
    close(x, x_ref, 2e-3, 1e-3)
    if K >= 128:
        x = torch.randn(M, N, device=DEV)
        x_ref = x + y_ref
        slab = C.linear_residual(a, w, bias, x, 2, True, CNT, False)
        C.norm(x, slab, bias, None, None, 0.0, True, None, False)
        close(x, x_ref, 2e-3, 1e-3)


@pytest.mark.parametrize("M", [129, 200, 256, 300])
@pytest.mark.parametrize("K", [64, 192, 640])
def test_ring_gemm_96_row_tiles(C, CNT, M, K):
    """Ring kernel with 96-row tiles (3 MFMA row tiles per wave): every
    epilogue, partial row / column tiles, k-steps fewer than and beyond the ring."""
    from llm_sharding_demo_amd.ops.hip import interleave_gate_up

    C.gemm_set_tiled3_max(1 << 30)
    C.gemm_set_ring_tn(64)
    C.gemm_set_ring_m96(1 << 30)
    try:
        N = 352
        a, w, bias = bf(M, K, seed=66), bf(N, K, scale=0.05, seed=67), bf(N, scale=0.1, seed=68)
        y_ref = ref.linear(a, w, bias)
        close(C.linear(a, w, bias, 0, True, 1, CNT), y_ref, 3e-2)
        close(C.linear(a, w, bias, 1, True, 1, CNT), ref.gelu_new(y_ref), 3e-2)
        w2 = w[:256].contiguous()
        y = C.linear(a, interleave_gate_up(w2, 128).contiguous(), None, 2, True, 1, CNT)
        close(y, ref.silu_mul(*ref.linear(a, w2).split(128, 1)), 3e-2)
        close(C.linear_f32(a, w, True, 1, CNT), ref.linear(a, w), 2e-3, 1e-3)
        x = torch.randn(M, N, device=DEV)
        x_ref = x + y_ref
        assert C.linear_residual(a, w, bias, x, 1, True, CNT, False) is None
        close(x, x_ref, 2e-3, 1e-3)
    finally:
        C.gemm_set_ring_m96(0)
        C.gemm_set_tiled3_max(0)
        C.gemm_set_ring_tn(128)


@pytest.fixture(params=[(1, 0), (2, 0), (2, 1), (2, 2)])
def RING8(C, request):
    """128x64 decode ring on 8 waves (gemm_ring8_kernel): (layout, A/B flags)
    -- 1 = 4 computing + 4 loader waves, 2 = 8 computing waves; flag 1 =
    rotated K start per tile, 2 = nt weight staging."""
    var, flags = request.param
    C.gemm_set_tiled3_max(1 << 30)
    C.gemm_set_ring_tn(64)
    C.gemm_set_ring8(var)
    C.gemm_set_ring8_flags(flags)
    yield C, var
    C.gemm_set_ring8(0)
    C.gemm_set_ring8_flags(0)
    C.gemm_set_tiled3_max(0)
    C.gemm_set_ring_tn(128)


@pytest.mark.parametrize("M", [100, 200, 256])
@pytest.mark.parametrize("K,splits", [(64, 1), (192, 1), (640, 1), (640, 2), (1600, 1), (1600, 3), (1600, 4)])
def test_ring8_gemm_epilogues(RING8, CNT, M, K, splits):
    """8-wave decode ring: every epilogue, M / N tails, 1 to 25 k-steps,
    in-kernel split-K combine (8 computing waves) bit-stable across launches
    that reuse the re-armed ticket counters, residual slabs folded by the norm."""
    from llm_sharding_demo_amd.ops.hip import interleave_gate_up

    C, var = RING8
    if splits > 1 and var != 2:
        pytest.skip("the split-K combine is built for the 8-computing-wave layout")
    N = 352  # 5.5 tiles of 64 columns: a partial last tile
    a, w, bias = bf(M, K, seed=90), bf(N, K, scale=0.05, seed=91), bf(N, scale=0.1, seed=92)
    y_ref = ref.linear(a, w, bias)
    y1 = C.linear(a, w, bias, 0, True, splits, CNT)
    close(y1, y_ref, 3e-2)
    assert torch.equal(C.linear(a, w, bias, 0, True, splits, CNT), y1)
    close(C.linear(a, w, bias, 1, True, splits, CNT), ref.gelu_new(y_ref), 3e-2)
    w2 = w[:256].contiguous()
    y = C.linear(a, interleave_gate_up(w2, 128).contiguous(), None, 2, True, splits, CNT)
    close(y, ref.silu_mul(*ref.linear(a, w2).split(128, 1)), 3e-2)
    close(C.linear_f32(a, w, True, splits, CNT), ref.linear(a, w), 2e-3, 1e-3)
    x = torch.randn(M, N, device=DEV)
    x_ref = x + y_ref
    slab = C.linear_residual(a, w, bias, x, splits, True, CNT, False)
    if splits > 1:
        C.norm(x, slab, bias, None, None, 0.0, True, None, False)
    close(x, x_ref, 2e-3, 1e-3)


@pytest.fixture(params=[(2, 3), (3, 3), (2, 2), (2, 4), (3, 2)])
def D256(C, request):
    """(launch kind, ring slots) of the 8-wave all-rows kernel gemm_d256:
    kind 2 = 64-column tiles, 3 = 128-column tiles."""
    kind, slots = request.param
    C.gemm_set_d256_slots(slots)
    yield C, kind
    C.gemm_set_d256_slots(3)


@pytest.mark.parametrize("M", [1, 100, 129, 200, 256, 300, 512, 700])
@pytest.mark.parametrize("K,splits", [(64, 1), (192, 1), (192, 3), (640, 2), (640, 5), (1600, 3), (1600, 1)])
def test_d256_gemm_epilogues(D256, CNT, M, K, splits):
    """256-row decode kernel: every epilogue, row tails (1 to 256 rows), rows
    in several 256-row blocks (300 / 512 / 700: a partial last block), a
    partial last column tile, 1 to 25 k-steps (fewer than, equal to and more
    than the ring), split-K with the in-kernel last-arriver combine and the
    residual slabs folded by the norm; repeated launches reuse the re-armed
    ticket counters."""
    from llm_sharding_demo_amd.ops.hip import interleave_gate_up

    C, kind = D256
    N = 384 if kind == 3 else 352  # 352: a partial last 64-wide tile
    a, w, bias = bf(M, K, seed=80), bf(N, K, scale=0.05, seed=81), bf(N, scale=0.1, seed=82)
    y_ref = ref.linear(a, w, bias)
    for _ in range(2):
        close(C.linear(a, w, bias, 0, kind, splits, CNT), y_ref, 3e-2)
    close(C.linear(a, w, bias, 1, kind, splits, CNT), ref.gelu_new(y_ref), 3e-2)
    w2 = w[:256].contiguous()
    y = C.linear(a, interleave_gate_up(w2, 128).contiguous(), None, 2, kind, splits, CNT)
    close(y, ref.silu_mul(*ref.linear(a, w2).split(128, 1)), 3e-2)
    close(C.linear_f32(a, w, kind, splits, CNT), ref.linear(a, w), 2e-3, 1e-3)
    x = torch.randn(M, N, device=DEV)
    x_ref = x + y_ref
    slab = C.linear_residual(a, w, bias, x, splits, kind, CNT, False)
    if splits > 1:
        assert slab is not None and slab.shape == (splits, M, N)
        C.norm(x, slab, bias, None, None, 0.0, True, None, False)
    else:
        assert slab is None
    close(x, x_ref, 2e-3, 1e-3)
    # split-K combine order is fixed: bit-identical on a second launch
    if splits > 1:
        assert torch.equal(C.linear(a, w, bias, 0, kind, splits, CNT),
                           C.linear(a, w, bias, 0, kind, splits, CNT))
    assert int(CNT.abs().sum()) == 0  # every ticket re-armed


@pytest.fixture
def BIG(C):
    """Force the pipelined 256x256 kernel for every tiled launch with M >= 256."""
    C.gemm_set_big_min(1)
    yield C
    C.gemm_set_big_min(160)


@pytest.fixture(params=[4, 1, 0])
def BIGK(BIG, request):
    """The 256x256 kernel kinds: 4 = phase-pipelined BK=64 with buffer_load ... lds staging
    (default), 1 = the same with global_load_lds, 0 = the BK=32 4-slot ring."""
    BIG.gemm_set_big_kind(request.param)
    yield BIG
    BIG.gemm_set_big_kind(4)


@pytest.mark.parametrize("M", [256, 300, 777, 1300])
@pytest.mark.parametrize("K", [64, 128, 384])
def test_big_gemm_epilogues(BIGK, CNT, M, K):
    """256x256 ring-pipelined kernel: every epilogue, M/N tails, K of 2, 4 and 12
    k-steps (fewer than, equal to and more than the ring depth)."""
    from llm_sharding_demo_amd.ops.hip import interleave_gate_up

    C = BIGK
    N = 320  # second column tile is a 64-wide tail
    a, w, bias = bf(M, K, seed=40), bf(N, K, scale=0.05, seed=41), bf(N, scale=0.1, seed=42)
    y_ref = ref.linear(a, w, bias)
    close(C.linear(a, w, bias, 0, True, 1, CNT), y_ref, 3e-2)
    close(C.linear(a, w, bias, 1, True, 1, CNT), ref.gelu_new(y_ref), 3e-2)
    w2 = w[:256].contiguous()
    y = C.linear(a, interleave_gate_up(w2, 128).contiguous(), None, 2, True, 1, CNT)
    close(y, ref.silu_mul(*ref.linear(a, w2).split(128, 1)), 3e-2)
    close(C.linear_f32(a, w, True, 1, CNT), ref.linear(a, w), 2e-3, 1e-3)
    x = torch.randn(M, N, device=DEV)
    x_ref = x + y_ref
    assert C.linear_residual(a, w, bias, x, 1, True, CNT, False) is None
    close(x, x_ref, 2e-3, 1e-3)
    if K >= 128:
        x = torch.randn(M, N, device=DEV)
        x_ref = x + y_ref
        slab = C.linear_residual(a, w, bias, x, 2, True, CNT, False)
        C.norm(x, slab, bias, None, None, 0.0, True, None, False)
        close(x, x_ref, 2e-3, 1e-3)


@pytest.mark.parametrize("M,N,K", [(512, 1600, 6400), (512, 4096, 4096), (384, 1600, 1600), (256, 1024, 8192)])
@pytest.mark.parametrize("splits", [2, 4, 6, 8])
def test_resid_splits_above_256_rows(C, CNT, M, N, K, splits):
    """Residual projections of 257-1024-row decode groups with the K-split
    counts _resid_splits now picks (default routing: 128x64 ring, 128x128
    tiled or the 256x256 p8 kernel, depending on the grid), slabs folded by
    the norm, against the fp32 reference."""
    a, w, bias = bf(M, K, seed=70), bf(N, K, scale=0.02, seed=71), bf(N, scale=0.1, seed=72)
    C.gemm_set_tiled3_max(512)  # the engine's routing (HipBackend defaults)
    C.gemm_set_ring_tn(0)
    try:
        x = torch.randn(M, N, device=DEV)
        x_ref = x + ref.linear(a, w, bias)
        slab = C.linear_residual(a, w, bias, x, splits, True, CNT, True)
        assert slab is not None and slab.shape == (splits, M, N)
        C.norm(x, slab, bias, None, None, 0.0, True, None, False)
        close(x, x_ref, 3e-3, 2e-3)
    finally:
        C.gemm_set_tiled3_max(0)
        C.gemm_set_ring_tn(128)


def _cache(slots, n_kv, S, hd):
    return (torch.zeros(slots, n_kv, S, hd, dtype=torch.bfloat16, device=DEV),
            torch.zeros(slots, n_kv, S, hd, dtype=torch.bfloat16, device=DEV))


@pytest.mark.parametrize("rope", [False, True])
@pytest.mark.parametrize("mode", ["decode1", "decode4", "tiled", "big", "d256", "d256s3", "d256rb"])
def test_qkv_kv_append(C, CNT, rope, mode):
    from llm_sharding_demo_amd.ops.hip import rope_pair_permutation, rope_table

    nh, n_kv, hd, H = 4, 2, 64, 256
    qs, kvs = nh * hd, n_kv * hd
    tiled = mode in ("tiled", "big", "d256", "d256s3", "d256rb")
    splits = 4 if mode == "decode4" else (3 if mode == "d256s3" else (2 if mode == "d256rb" else 1))
    # decode: 10 tokens of 2 sequences; tiled: 2 sequences of 150 tokens;
    # d256: 200 decode-like rows (100 + 100) on the 256-row kernel (kind 2);
    # d256rb: 400 rows in two 256-row blocks, split-K combine
    n0, n1 = (4, 6) if not tiled else ((100, 100) if mode in ("d256", "d256s3") else
                                       ((200, 200) if mode == "d256rb" else (150, 150)))
    if mode.startswith("d256"):
        tiled = 2
    T, slots, S = n0 + n1, 3, 320
    a, w, bias = bf(T, H, seed=13), bf(qs + 2 * kvs, H, scale=0.05, seed=14), bf(qs + 2 * kvs, scale=0.1, seed=15)
    tslot = torch.tensor([0] * n0 + [2] * n1, dtype=torch.int32, device=DEV)
    tpos = torch.tensor(list(range(n0)) + list(range(5, 5 + n1)), dtype=torch.int32, device=DEV)
    if mode == "big":
        C.gemm_set_big_min(1)
    kc, vc = _cache(slots, n_kv, S, hd)
    kr, vr = _cache(slots, n_kv, S, hd)
    y = ref.linear(a, w, bias)
    q_ref = y[:, :qs].reshape(T, nh, hd)
    k_ref = y[:, qs:qs + kvs].reshape(T, n_kv, hd)
    v_ref = y[:, qs + kvs:].reshape(T, n_kv, hd)
    if rope:
        q_ref = ref.apply_rope(q_ref, tpos.cpu(), 10000.0)
        k_ref = ref.apply_rope(k_ref, tpos.cpu(), 10000.0)
        perm = torch.cat([rope_pair_permutation(nh, hd), rope_pair_permutation(n_kv, hd) + qs,
                          torch.arange(qs + kvs, qs + 2 * kvs)]).to(DEV)
        w, bias = w[perm].contiguous(), bias[perm].contiguous()
        table = rope_table(S, hd, 10000.0, DEV)
        q = C.linear_qkv(a, w, bias, kc, vc, tslot, tpos, qs, kvs, hd, table, tiled, splits, CNT)
        # un-permute the pair-interleaved head dims for comparison
        p1 = rope_pair_permutation(1, hd)
        inv = torch.argsort(p1).to(DEV)
        q = q.reshape(T, nh, hd)[:, :, inv]
        kc = kc[..., inv]
    else:
        q = C.linear_qkv(a, w, bias, kc, vc, tslot, tpos, qs, kvs, hd, None, tiled, splits, CNT).reshape(T, nh, hd)
    C.gemm_set_big_min(160)
    ref.kv_append(kr, vr, k_ref, v_ref, tslot, tpos)
    close(q, q_ref, 3e-2)
    close(kc, kr, 3e-2)
    close(vc, vr, 3e-2)


@pytest.mark.parametrize("hd,nh,n_kv", [(64, 4, 4), (64, 8, 2), (128, 8, 2), (128, 32, 8)])
@pytest.mark.parametrize("splits", [1, 3])
@pytest.mark.parametrize("max_wg", [0, 3])
@pytest.mark.parametrize("B,small_waves", [(5, 8), (5, 16), (5, 4), (5, 88), (70, 8)])
def test_attention_decode(C, hd, nh, n_kv, splits, max_wg, B, small_waves):
    """max_wg > 0: capped grid, each block loops over (sequence, head) items.
    B = 5: the small-batch blocks (8 / 16 / 4 waves; 88 = 8 waves with 8 keys
    per wave in flight); B = 70: 4-wave blocks."""
    from llm_sharding_demo_amd.ops.hip import HipBackend

    C.attn_set_max_wg(max_wg)
    C.attn_set_small_waves(small_waves)
    C.attn_set_small_waves128(small_waves)
    try:
        _attention_decode_case(C, hd, nh, n_kv, splits, B)
    finally:
        C.attn_set_max_wg(0)
        C.attn_set_small_waves(HipBackend.R.attn_small_waves)
        C.attn_set_small_waves128(HipBackend.R.attn_small_waves128)


@pytest.mark.parametrize("hd,nh,n_kv", [(64, 12, 12), (128, 8, 2)])
@pytest.mark.parametrize("lw", [8, 42, 2])
def test_attention_decode_full_batch_blocks(C, hd, nh, n_kv, lw):
    """Full-batch block shapes of the VALU decode kernel (A/B variants of the
    4-wave default): 8 waves, 4 waves with 2 keys per wave in flight, 2 waves."""
    C.attn_set_large_waves(hd, lw)
    try:
        _attention_decode_case(C, hd, nh, n_kv, 1, 70)
        _attention_decode_case(C, hd, nh, n_kv, 3, 70)
    finally:
        C.attn_set_large_waves(hd, 4)


def _attention_decode_case(C, hd, nh, n_kv, splits, B=5):
    slots, S = max(6, B), 300
    kc, vc = bf(slots, n_kv, S, hd, seed=16), bf(slots, n_kv, S, hd, seed=17)
    q = bf(B, nh * hd, seed=18)
    if B == 5:
        seq_slots = torch.tensor([5, 0, 2, 3, 1], dtype=torch.int32, device=DEV)
        pos = torch.tensor([0, 17, 63, 140, 299], dtype=torch.int32, device=DEV)
    else:
        g = torch.Generator().manual_seed(B)
        seq_slots = torch.randperm(slots, generator=g)[:B].int().to(DEV)
        pos = torch.randint(0, S, (B,), generator=g).int().to(DEV)
    o = C.attn_decode(q, kc, vc, seq_slots, pos, nh, splits)
    cu = torch.arange(B + 1, dtype=torch.int32)
    o_ref = ref.attention(q.reshape(B, nh, hd).cpu(), kc.cpu(), vc.cpu(), seq_slots.cpu(), pos.cpu(), cu)
    close(o.reshape(B, nh, hd), o_ref, 2e-2)


@pytest.mark.parametrize("nh,n_kv", [(32, 8), (16, 8), (64, 8)])
@pytest.mark.parametrize("B", [40, 3])
def test_attention_decode_mfma_grouped(C, nh, n_kv, B):
    """Grouped-query decode on MFMA (HD 128, G = 2 / 4 / 8 query heads per kv
    head), forced on for any batch: positions at 32-key tile edges, against
    the fp32 reference and the VALU kernel."""
    hd, slots, S = 128, max(B, 8), 300
    kc, vc = bf(slots, n_kv, S, hd, seed=26), bf(slots, n_kv, S, hd, seed=27)
    q = bf(B, nh * hd, seed=28)
    g = torch.Generator().manual_seed(B + nh)
    seq_slots = torch.randperm(slots, generator=g)[:B].int().to(DEV)
    edge = [0, 30, 31, 32, 63, 64, 95, 299]
    pos = torch.tensor([edge[i] if i < len(edge) else int(torch.randint(0, S, (1,), generator=g))
                        for i in range(B)], dtype=torch.int32, device=DEV)
    cu = torch.arange(B + 1, dtype=torch.int32)
    o_ref = ref.attention(q.reshape(B, nh, hd).cpu(), kc.cpu(), vc.cpu(), seq_slots.cpu(), pos.cpu(), cu)
    C.attn_set_mfma_min(1)
    try:
        o = C.attn_decode(q, kc, vc, seq_slots, pos, nh, 1)
    finally:
        C.attn_set_mfma_min(256)
    close(o.reshape(B, nh, hd), o_ref, 2e-2)
    C.attn_set_mfma_min(0)
    try:
        o_valu = C.attn_decode(q, kc, vc, seq_slots, pos, nh, 1)
    finally:
        C.attn_set_mfma_min(256)
    close(o, o_valu, 2e-2)


@pytest.mark.parametrize("splits", [2, 5, 16])
def test_attention_decode_mfma_context_splits(C, splits):
    """The MFMA decode kernel over context splits (long contexts, few
    sequences): per-split partials merged by the combine kernel, including
    splits past a short sequence's end (empty ranges) and split boundaries
    that are not 32-key aligned."""
    B, nh, n_kv, hd, S = 6, 32, 8, 128, 1100
    kc, vc = bf(B + 2, n_kv, S, hd, seed=36), bf(B + 2, n_kv, S, hd, seed=37)
    q = bf(B, nh * hd, seed=38)
    seq_slots = torch.tensor([7, 0, 3, 5, 1, 2], dtype=torch.int32, device=DEV)
    pos = torch.tensor([1099, 0, 7, 517, 1023, 64], dtype=torch.int32, device=DEV)
    cu = torch.arange(B + 1, dtype=torch.int32)
    o_ref = ref.attention(q.reshape(B, nh, hd).cpu(), kc.cpu(), vc.cpu(), seq_slots.cpu(), pos.cpu(), cu)
    C.attn_set_mfma_min(1)
    try:
        o = C.attn_decode(q, kc, vc, seq_slots, pos, nh, splits)
    finally:
        C.attn_set_mfma_min(256)
    assert torch.isfinite(o.float()).all()
    close(o.reshape(B, nh, hd), o_ref, 2e-2)


def test_decode_attn_split_policy():
    """Long contexts with few sequences take the MFMA kernel with context
    splits; the headline batches stay unsplit."""
    from llm_sharding_demo_amd.ops.hip import HipBackend as H

    assert H.decode_attn_splits(256, 32, 8, 128, 400) == 1  # 2048 items
    assert H.decode_attn_splits(32, 32, 8, 128, 4224) == 4  # 256 items -> 1024 waves
    assert H.decode_attn_splits(8, 32, 8, 128, 8128) == 16  # 64 items -> 1024 waves
    assert H.decode_attn_splits(4, 32, 8, 128, 8128) == 16  # >= 512 keys per split
    assert H.decode_attn_splits(1, 32, 8, 128, 300) == 2  # VALU split rule
    assert H.decode_attn_splits(64, 25, 25, 64, 300) == 1  # GPT-2 XL: VALU


@pytest.mark.parametrize("hd,nh,n_kv", [(64, 4, 4), (128, 8, 2)])
def test_attention_prefill_ragged_chunked(C, hd, nh, n_kv):
    from llm_sharding_demo_amd.ops.hip import prefill_tiles
    from llm_sharding_demo_amd.runtime.batch import BatchMeta

    slots, S = 4, 400
    kc, vc = bf(slots, n_kv, S, hd, seed=19), bf(slots, n_kv, S, hd, seed=20)
    # seq 0: fresh 130 tokens; seq 1: 1 token; seq 2: chunk of 70 after 200 cached; seq 3: 64
    meta = BatchMeta.build([1, 0, 3, 2], [0, 0, 200, 5], [130, 1, 70, 64], DEV)
    q = bf(meta.num_tokens, nh * hd, seed=21)
    o = C.attn_prefill(q, kc, vc, prefill_tiles(meta).to(DEV), meta.seq_slots, meta.q_start,
                       meta.cu_q, nh)
    o_ref = ref.attention(q.reshape(-1, nh, hd).cpu(), kc.cpu(), vc.cpu(), meta.seq_slots.cpu(),
                          meta.q_start.cpu(), meta.cu_q.cpu())
    close(o.reshape(-1, nh, hd), o_ref, 2e-2)


def test_attention_prefill_large_logits_stable(C):
    """Spiky scores force the online-softmax rescale path (guide rule 26)."""
    from llm_sharding_demo_amd.ops.hip import prefill_tiles
    from llm_sharding_demo_amd.runtime.batch import BatchMeta

    hd, nh = 64, 2
    kc, vc = bf(1, nh, 256, hd, scale=3.0, seed=22), bf(1, nh, 256, hd, seed=23)
    kc[0, :, 200] *= 8  # one late key dominates
    meta = BatchMeta.build([0], [0], [256], DEV)
    q = bf(256, nh * hd, scale=3.0, seed=24)
    o = C.attn_prefill(q, kc, vc, prefill_tiles(meta).to(DEV), meta.seq_slots, meta.q_start,
                       meta.cu_q, nh)
    o_ref = ref.attention(q.reshape(-1, nh, hd).cpu(), kc.cpu(), vc.cpu(), meta.seq_slots.cpu(),
                          meta.q_start.cpu(), meta.cu_q.cpu())
    assert torch.isfinite(o.float()).all()
    close(o.reshape(-1, nh, hd), o_ref, 3e-2)


@pytest.mark.parametrize("M,N,K,kind,splits", [(1, 1040, 128, 1, 1), (64, 1040, 640, 1, 1),
                                                (200, 1040, 640, 1, 1), (256, 50304, 1600, 1, 1),
                                                (512, 4096, 256, 1, 1), (256, 4800, 1600, 2, 2),
                                                (100, 352, 640, 3, 3)])
def test_linear_f32_segmax(C, CNT, M, N, K, kind, splits):
    """lm_head epilogue: fp32 logits plus the max of every 8-column segment,
    bit-equal to the maximum of the stored logits, on every tiled kernel the
    grid size routes to (ring, 8-wave ring, 256^2, 256-row split-K)."""
    a, w = bf(M, K, seed=90), bf(N, K, scale=0.05, seed=91)
    seg = torch.full((M, N // 8), float("nan"), device=DEV)
    out = C.linear_f32(a, w, kind, splits, CNT, seg)
    close(out, ref.linear(a, w), 2e-3, 1e-3)
    assert torch.equal(seg, out.view(M, N // 8, 8).amax(-1))


@pytest.mark.parametrize("M,N,K", [(4096, 1600, 1600), (4100, 6400, 1600), (8192, 768, 3072)])
def test_blaslt_prefill_projections(C, M, N, K):
    """hipBLASLt prefill projections (csrc/blaslt.cpp, the opt-in A/B oracle):
    bf16 out with bias and bias + GELU epilogues, and the fp32 residual
    accumulate (beta = 1, C = D = x) -- against the fp32 reference; the
    library's GELU against GPT-2's tanh-approximated gelu_new at bf16
    resolution.  Only workspace-free algorithms are accepted: a shape the
    library then declines is reported (None) and skipped here."""
    a, w, bias = bf(M, K, seed=95), bf(N, K, scale=0.05, seed=96), bf(N, scale=0.1, seed=97)
    y_ref = ref.linear(a, w, bias)
    y = C.blaslt_linear(a, w, bias, 0)
    if y is None:
        pytest.skip("hipBLASLt has no workspace-free algorithm for this shape")
    close(y, y_ref, 3e-2)
    close(C.blaslt_linear(a, w, bias, 1), ref.gelu_new(y_ref), 3e-2)
    close(C.blaslt_linear(a, w, None, 1), ref.gelu_new(ref.linear(a, w)), 3e-2)
    for b in (bias, None):
        x = torch.randn(M, N, device=DEV)
        x_ref = x + ref.linear(a, w, b)
        assert C.blaslt_residual(a, w, b, x)
        close(x, x_ref, 2e-3, 1e-3)


@pytest.mark.parametrize("M", [512, 100])
def test_silu_mul_after_blaslt(C, CNT, M):
    """Decode gate_up at >= 512 rows: the hipBLASLt GEMM over the
    gate/up-interleaved weight, then the SiLU*up pass (elementwise.hip) --
    against the fp32 reference and the fused-epilogue kernel."""
    from llm_sharding_demo_amd.ops.hip import interleave_gate_up

    F, K = 1024, 512
    a, w = bf(M, K, seed=98), bf(2 * F, K, scale=0.05, seed=99)
    wi = interleave_gate_up(w, F).contiguous()
    y = C.blaslt_linear(a, wi, None, 0)
    assert y is not None
    out = C.silu_mul(y)
    ref_out = ref.silu_mul(*ref.linear(a, w).split(F, 1))
    close(out, ref_out, 3e-2)
    close(out, C.linear(a, wi, None, 2, True, 1, CNT), 3e-2)


@pytest.mark.parametrize("rope", [False, True])
def test_qkv_post_after_blaslt(C, CNT, rope):
    """Decode QKV on hipBLASLt (fp32 out) + the RoPE / cache-append pass
    (elementwise.hip qkv_post): q and both caches against the fp32 reference
    and against the fused-epilogue kernel (linear_qkv), padding rows on the
    scratch slot included."""
    from llm_sharding_demo_amd.ops.hip import rope_pair_permutation, rope_table

    nh, n_kv, hd, H = 8, 2, 128, 512
    qs, kvs = nh * hd, n_kv * hd
    T, slots, S = 96, 5, 200
    a, w, bias = bf(T, H, seed=113), bf(qs + 2 * kvs, H, scale=0.05, seed=114), bf(qs + 2 * kvs, scale=0.1, seed=115)
    g = torch.Generator().manual_seed(7)
    tslot = torch.randint(0, slots, (T,), generator=g).int().to(DEV)
    tpos = torch.randperm(S, generator=g)[:T].int().to(DEV)  # distinct (slot, pos): no write races
    y_ref = ref.linear(a, w, bias)
    q_ref = y_ref[:, :qs].reshape(T, nh, hd)
    k_ref = y_ref[:, qs:qs + kvs].reshape(T, n_kv, hd)
    v_ref = y_ref[:, qs + kvs:].reshape(T, n_kv, hd)
    table = None
    if rope:
        q_ref = ref.apply_rope(q_ref, tpos.cpu(), 10000.0)
        k_ref = ref.apply_rope(k_ref, tpos.cpu(), 10000.0)
        perm = torch.cat([rope_pair_permutation(nh, hd), rope_pair_permutation(n_kv, hd) + qs,
                          torch.arange(qs + kvs, qs + 2 * kvs)]).to(DEV)
        w, bias = w[perm].contiguous(), bias[perm].contiguous()
        table = rope_table(S, hd, 10000.0, DEV)
    kc, vc = _cache(slots, n_kv, S, hd)
    kf, vf = _cache(slots, n_kv, S, hd)
    y = C.blaslt_f32(a, w)
    assert y is not None and y.dtype == torch.float32
    q = C.qkv_post(y, bias, kc, vc, tslot, tpos, qs, kvs, hd, table)
    qf = C.linear_qkv(a, w, bias, kf, vf, tslot, tpos, qs, kvs, hd, table, True, 1, CNT)
    close(q, qf, 2e-2)
    close(kc, kf, 2e-2)
    close(vc, vf, 2e-2)
    if rope:  # un-permute the pair-interleaved head dims for the reference
        inv = torch.argsort(rope_pair_permutation(1, hd)).to(DEV)
        q = q.reshape(T, nh, hd)[:, :, inv]
        kc = kc[..., inv]
    kr, vr = _cache(slots, n_kv, S, hd)
    ref.kv_append(kr, vr, k_ref, v_ref, tslot, tpos)
    close(q.reshape(T, nh, hd), q_ref, 3e-2)
    close(kc, kr, 3e-2)
    close(vc, vr, 3e-2)


def _segmax(logits):
    """What linear_f32 writes beside these logits (padding columns included)."""
    B, Vp = logits.shape
    return logits.view(B, Vp // 8, 8).amax(-1).contiguous()


def test_sampler(C):
    from llm_sharding_demo_amd.runtime.batch import counter_uniform

    B, V, Vp = 6, 50257, 50304
    logits = torch.randn(B, Vp, device=DEV) * 3
    logits[:, V:] = 100.0  # padding must never be selected
    temp = torch.tensor([1.0, 0.6, 0.6, 2.0, 1.0, 0.6], device=DEV)
    topk = torch.tensor([1, 40, 40, 5, 1024, 40], dtype=torch.int32, device=DEV)
    greedy = torch.tensor([1, 0, 0, 0, 0, 1], dtype=torch.int32, device=DEV)
    seeds = torch.arange(B, dtype=torch.int64, device=DEV) * 7919
    step = torch.full((B,), 3, dtype=torch.int64, device=DEV)
    out = C.sample(logits, V, temp, topk, greedy, seeds, step)
    exp = ref.sample(logits.cpu(), temp.cpu(), topk.cpu(), greedy.cpu(),
                     counter_uniform(seeds.cpu(), step.cpu()), V)
    assert out.cpu().tolist() == exp.tolist()
    # decode-step form: same draw written into a slice, counters advanced in-kernel
    buf = torch.full((B + 3,), -1, dtype=torch.int32, device=DEV)
    st2 = step.clone()
    C.sample_into(logits, V, temp, topk, greedy, seeds, st2, buf[:B], None)
    assert buf[:B].cpu().tolist() == exp.tolist() and buf[B:].cpu().tolist() == [-1] * 3
    assert torch.equal(st2, step + 1)
    act = (torch.arange(B, device=DEV) % 3 != 0).int()  # pad rows (0) keep their counter
    st3 = step.clone()
    C.sample_into(logits, V, temp, topk, greedy, seeds, st3, buf[:B], act)
    assert buf[:B].cpu().tolist() == exp.tolist() and torch.equal(st3, step + act)
    # the last stage's decode positions advance in the same kernel
    pos = torch.arange(B, dtype=torch.int32, device=DEV) + 100
    st4 = step.clone()
    C.sample_into(logits, V, temp, topk, greedy, seeds, st4, buf[:B], act, pos)
    assert torch.equal(st4, step + act) and torch.equal(pos, torch.arange(B, device=DEV).int() + 100 + act)
    for r in range(B):
        k = 1 if greedy[r] else int(topk[r])
        assert int(out[r]) in set(torch.topk(logits[r, :V], k).indices.tolist())


@pytest.mark.parametrize("seg", [False, True])
@pytest.mark.parametrize("case", ["random", "ties", "flat", "quantized", "llama_vocab"])
def test_sampler_fast_path_and_ties(C, case, seg):
    """top-k <= 64 takes the threshold/filter path (seg: its threshold from
    lm_head's 8-logit segment maxima, reading only the segments that reach
    it; the partial last segment's maximum includes the padding); flat logits
    (more candidates than fit) fall back to the radix path; ties are broken
    by the lowest index in both -- bit-equal to the host reference either way."""
    from llm_sharding_demo_amd.runtime.batch import counter_uniform

    B, V, Vp = (12, 128256, 128256) if case == "llama_vocab" else (12, 50257, 50304)
    g = torch.Generator(device=DEV).manual_seed(5)
    logits = torch.randn(B, Vp, device=DEV, generator=g) * 2
    if case == "ties":  # many exact duplicates around the top
        logits = (logits * 4).round() / 4
    elif case == "flat":
        logits[:6] = 0.25
    elif case == "quantized":
        logits = (logits * 16).round() / 16
    logits[:, V:] = 100.0
    temp = torch.linspace(0.5, 1.5, B, device=DEV)
    topk = torch.tensor([1, 2, 5, 16, 40, 63, 64, 65, 40, 40, 200, 40], dtype=torch.int32, device=DEV)
    greedy = torch.tensor([0] * 11 + [1], dtype=torch.int32, device=DEV)
    seeds = torch.arange(B, dtype=torch.int64, device=DEV) * 104729 + 11
    step = torch.arange(B, dtype=torch.int64, device=DEV)
    sm = _segmax(logits) if seg else None
    out = C.sample(logits, V, temp, topk, greedy, seeds, step, sm)
    exp = ref.sample(logits.cpu(), temp.cpu(), topk.cpu(), greedy.cpu(),
                     counter_uniform(seeds.cpu(), step.cpu()), V)
    assert out.cpu().tolist() == exp.tolist()
    # decode-step form: same draw written into a slice, counters advanced in-kernel
    buf = torch.full((B + 3,), -1, dtype=torch.int32, device=DEV)
    st2 = step.clone()
    C.sample_into(logits, V, temp, topk, greedy, seeds, st2, buf[:B], None, None, sm)
    assert buf[:B].cpu().tolist() == exp.tolist() and buf[B:].cpu().tolist() == [-1] * 3
    assert torch.equal(st2, step + 1)
    act = (torch.arange(B, device=DEV) % 3 != 0).int()  # pad rows (0) keep their counter
    st3 = step.clone()
    C.sample_into(logits, V, temp, topk, greedy, seeds, st3, buf[:B], act, None, sm)
    assert buf[:B].cpu().tolist() == exp.tolist() and torch.equal(st3, step + act)


@pytest.mark.parametrize("seg", [False, True])
@pytest.mark.parametrize("V,Vp", [(1000, 1024), (1000, 1000), (3000, 3008), (2997, 3008)])
def test_sampler_small_vocab(C, V, Vp, seg):
    """V < 4096 (the test presets): fewer than k of the 64 segments hold real
    logits, so the fast path's threshold is -inf -- padding past V must never
    become a candidate (its index lies past the row).  The rows sit
    at the very end of their allocation so an over-read would leave it."""
    from llm_sharding_demo_amd.runtime.batch import counter_uniform

    B = 4
    g = torch.Generator(device=DEV).manual_seed(9)
    store = torch.empty(B * Vp, device=DEV)  # exact size: nothing after the last row
    logits = store.view(B, Vp)
    logits.copy_(torch.randn(B, Vp, device=DEV, generator=g) * 2)
    logits[:, V:] = 100.0
    temp = torch.tensor([0.6, 1.0, 0.6, 1.0], device=DEV)
    topk = torch.tensor([20, 40, 64, 40], dtype=torch.int32, device=DEV)
    greedy = torch.zeros(B, dtype=torch.int32, device=DEV)
    seeds = torch.arange(B, dtype=torch.int64, device=DEV) * 31 + 1
    step = torch.arange(B, dtype=torch.int64, device=DEV)
    out = C.sample(logits, V, temp, topk, greedy, seeds, step, _segmax(logits) if seg else None)
    exp = ref.sample(logits.cpu(), temp.cpu(), topk.cpu(), greedy.cpu(),
                     counter_uniform(seeds.cpu(), step.cpu()), V)
    assert out.cpu().tolist() == exp.tolist()
    assert all(0 <= t < V for t in out.cpu().tolist())


@pytest.mark.parametrize("hd,nh,n_kv,N", [(64, 25, 25, 1600), (64, 12, 12, 768), (128, 32, 8, 4096),
                                          (128, 8, 2, 320), (128, 16, 2, 256), (128, 8, 8, 1024)])
@pytest.mark.parametrize("B", [1, 2, 4])
@pytest.mark.parametrize("nc", [16, 160, 0])
def test_attention_oproj_fused(C, CNT, hd, nh, n_kv, N, B, nc):
    """Fused decode attention + output projection + residual add (small
    batches): x += attention(q) @ W^T + b, against the fp32 reference of the
    two separate ops; column chunks of 16 / 160 / the engine's choice (0),
    contexts 1..300, deterministic across launches (fixed kv-head order)."""
    from llm_sharding_demo_amd.ops.hip import HipBackend  # noqa: F401

    slots, S = 6, 300
    kc, vc = bf(slots, n_kv, S, hd, seed=96), bf(slots, n_kv, S, hd, seed=97)
    q = bf(B, nh * hd, seed=98)
    w, bias = bf(N, nh * hd, scale=0.03, seed=99), bf(N, scale=0.1, seed=100)
    g = torch.Generator().manual_seed(B + N)
    seq_slots = torch.randperm(slots, generator=g)[:B].int().to(DEV)
    pos = torch.tensor([0, 299, 17, 150][:B], dtype=torch.int32, device=DEV)
    if nc == 0:
        C_ = max(1, -(-256 // n_kv))
        nc = -(-(-(-N // C_)) // 16) * 16
    cu = torch.arange(B + 1, dtype=torch.int32)
    o_ref = ref.attention(q.reshape(B, nh, hd).cpu(), kc.cpu(), vc.cpu(), seq_slots.cpu(), pos.cpu(), cu)
    y_ref = o_ref.reshape(B, nh * hd).float() @ w.float().cpu().t() + bias.float().cpu()
    x0 = torch.randn(B, N, device=DEV)
    x = x0.clone()
    C.attn_oproj(q, kc, vc, seq_slots, pos, nh, w, bias, x, nc, CNT)
    close(x - x0, y_ref, 2e-2)
    x2 = x0.clone()
    C.attn_oproj(q, kc, vc, seq_slots, pos, nh, w, bias, x2, nc, CNT)
    assert torch.equal(x, x2)
    x3 = x0.clone()
    C.attn_oproj(q, kc, vc, seq_slots, pos, nh, w, None, x3, nc, CNT)  # no bias
    close(x3 - x0, y_ref - bias.float().cpu(), 2e-2)
    assert int(CNT.abs().sum()) == 0


@pytest.mark.parametrize("cap,b,n,first,last", [(256, 256, 256, True, True), (256, 128, 77, True, True),
                                                (300, 64, 0, True, False), (2048, 2048, 1500, False, True),
                                                (8, 8, 3, False, False)])
def test_apply_rows(C, cap, b, n, first, last):
    """Composition change of a decode group (elementwise.hip apply_rows_kernel):
    the packed row state scattered into the row vectors, pad rows [n, b) idle
    on the scratch slot, stage 0's in-place token gather (sources anywhere in
    the previous return vector, including rows this launch overwrites) -- vs
    the same fields written from Python lists."""
    import numpy as np

    g = torch.Generator().manual_seed(cap + b + n)
    scratch = 12345
    ri = lambda lo, hi, k: torch.randint(lo, hi, (k,), generator=g)  # noqa: E731
    slot, pos, topk, greedy, src = ri(0, 10000, n), ri(0, 4096, n), ri(1, 64, n), ri(0, 2, n), ri(0, cap, n)
    temp = torch.rand(n, generator=g) + 0.1
    seed, step = ri(0, 1 << 62, n), ri(0, 1 << 40, n)
    a = np.zeros(10 * cap + 1, np.int32)
    a[: 4 * cap].view(np.int64)[:n] = seed.numpy()
    a[: 4 * cap].view(np.int64)[cap: cap + n] = step.numpy()
    a[4 * cap] = n
    f0 = 4 * cap + 1
    for k, v in enumerate((slot, pos, None, topk, greedy, src)):
        if v is not None:
            a[f0 + k * cap: f0 + k * cap + n] = v.numpy()
    a[f0 + 2 * cap: f0 + 2 * cap + n] = temp.numpy().astype(np.float32).view(np.int32)
    i32 = dict(dtype=torch.int32, device=DEV)
    buf = torch.from_numpy(a).to(DEV)
    t = dict(slots=torch.full((cap,), -1, **i32), pos=torch.full((cap,), -1, **i32), act=torch.full((cap,), -1, **i32))
    if last:
        t.update(temp=torch.zeros(cap, device=DEV), topk=torch.zeros(cap, **i32), greedy=torch.zeros(cap, **i32),
                 seeds=torch.full((cap,), -1, dtype=torch.int64, device=DEV),
                 sstep=torch.full((cap,), -1, dtype=torch.int64, device=DEV))
    tin0 = ri(0, 50000, cap).to(torch.int32)
    tin = tin0.to(DEV)
    ptr = lambda k: t[k].data_ptr() if k in t else 0  # noqa: E731
    args = torch.tensor([cap, scratch, buf.data_ptr(), ptr("slots"), ptr("pos"), ptr("act"), ptr("temp"), ptr("topk"),
                         ptr("greedy"), ptr("seeds"), ptr("sstep"), tin.data_ptr() if first else 0], dtype=torch.int64)
    C.apply_rows(args, b)
    torch.cuda.synchronize()
    pad = b - n
    cat = lambda v, fill: torch.cat([v.to(torch.int64), torch.full((pad,), fill, dtype=torch.int64)])  # noqa: E731
    assert torch.equal(t["slots"][:b].cpu().long(), cat(slot, scratch))
    assert torch.equal(t["pos"][:b].cpu().long(), cat(pos, 0))
    assert torch.equal(t["act"][:b].cpu().long(), cat(torch.ones(n, dtype=torch.int64), 0))
    assert (t["slots"][b:] == -1).all()  # rows past the bucket untouched
    if last:
        assert torch.equal(t["temp"][:b].cpu(), torch.cat([temp.float(), torch.ones(pad)]))
        assert torch.equal(t["topk"][:b].cpu().long(), cat(topk, 1))
        assert torch.equal(t["greedy"][:b].cpu().long(), cat(greedy, 1))
        assert torch.equal(t["seeds"][:b].cpu(), cat(seed, 0))
        assert torch.equal(t["sstep"][:b].cpu(), cat(step, 0))
    want = tin0.clone()
    if first:
        want[:b] = tin0[cat(src, 0)]
    assert torch.equal(tin.cpu(), want)
