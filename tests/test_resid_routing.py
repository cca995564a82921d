"""Decode GEMM routing rule for residual projections (CPU: the rule only,
no extension calls).  The kernels it routes to are checked on the GPU by
tests/test_kernels_gpu.py::test_resid_splits_above_256_rows."""


def test_resid_split_rule_above_256_rows():
    from llm_sharding_demo_amd.ops.hip import HipBackend
    b = HipBackend.__new__(HipBackend)  # routing rule only: no extension calls
    assert b._resid_splits(512, 4096, 14336) == 8   # Llama-3 8B down
    assert b._resid_splits(512, 4096, 4096) == 4    # Llama-3 8B o-proj
    assert b._resid_splits(512, 1600, 6400) == 6    # GPT-2 XL MLP-down
    assert b._resid_splits(512, 1600, 1600) == 2    # GPT-2 XL out-proj
    assert b._resid_splits(65536, 1600, 6400) == 1  # prefill keeps the old rule


def test_resid_split_rule_long_k_256_rows():
    from llm_sharding_demo_amd.ops.hip import HipBackend
    b = HipBackend.__new__(HipBackend)
    assert b._resid_splits(256, 4096, 14336) == 8   # Llama-3 8B down: off the ring
    assert b._resid_splits(256, 4096, 4096) == 2    # o-proj stays on the ring rule
    assert b._resid_splits(256, 1600, 6400) == 5    # GPT-2 XL MLP-down unchanged
    assert b._resid_splits(256, 1600, 1600) == 3    # GPT-2 XL out-proj unchanged
    assert b._resid_splits(128, 4096, 14336) == 4   # 128 rows unchanged


def test_resid_rule_prefill_chunks_keep_prefill_rule():
    """the 257-1024-row decode target must not re-route prefill
    chunks of that size (the backend learns decode vs prefill per forward)."""
    from llm_sharding_demo_amd.ops.hip import HipBackend
    b = HipBackend.__new__(HipBackend)
    b.decode = True
    dec = b._resid_splits(512, 1600, 6400)
    b.decode = False
    pre = b._resid_splits(512, 1600, 6400)
    assert dec == 6 and pre == max(1, min(-(-256 // 52), 6400 // 64 // 2))


def test_gemv_ok_matches_dispatch():
    """lsd_gemv_ok must accept exactly the (epilogue, norm) pairs lsd_gemv
    instantiates: BF16+LN etc. read 'not ok' so the caller
    materialises the norm instead of failing at launch."""
    import pytest
    try:
        from llm_sharding_demo_amd import _C
    except Exception as e:  # pragma: no cover - extension not built here
        pytest.skip(f"_C not importable: {e}")
    dispatched = {(0, 0), (1, 0), (1, 1), (2, 0), (2, 2), (3, 0), (3, 1), (3, 2), (4, 0),
                  (6, 0), (6, 1), (6, 2)}
    for epi in (0, 1, 2, 3, 4, 5, 6):
        for norm in (0, 1, 2):
            ok = bool(_C.gemv_ok(1, 1600, epi, norm))
            assert ok == ((epi, norm) in dispatched), (epi, norm)
