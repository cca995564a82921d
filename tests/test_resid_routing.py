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
