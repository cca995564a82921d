"""Small-M GEMV (csrc/kernels/gemv.hip) vs plain PyTorch fp32 references of
the same op: every epilogue, fused LayerNorm / RMSNorm prologue, M = 1..8,
K from 768 to 14336 (tail chunks not a multiple of 512), N not a multiple of
the 8-column workgroup tile."""
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


def norm_ref(x, g, b, rms):
    return ref.rmsnorm(x, g, 1e-5) if rms else ref.layernorm(x, g, b, 1e-5)


@pytest.mark.parametrize("M", [1, 2, 3, 4, 5, 8])
@pytest.mark.parametrize("K", [768, 1600, 4096, 6400])
@pytest.mark.parametrize("act", [0, 1])
def test_gemv_bf16_gelu(C, M, K, act):
    if not C.gemv_ok(M, K, act, 0):
        pytest.skip("shape not on the GEMV")
    N = 1000  # 125 workgroups of 8 columns; the last one partial
    a, w, bias = bf(M, K, seed=1), bf(N, K, scale=0.05, seed=2), bf(N, scale=0.1, seed=3)
    y = C.gemv(a, w, bias, act, 0, None, None, 0.0, None, None, None, None, None, 0, 0, 0, None)
    y_ref = ref.linear(a, w, bias)
    if act == 1:
        y_ref = ref.gelu_new(y_ref)
    close(y, y_ref, 3e-2)


@pytest.mark.parametrize("M", [1, 2, 4, 7])
@pytest.mark.parametrize("K", [1600, 6400, 14336])
def test_gemv_residual_and_f32(C, M, K):
    if not C.gemv_ok(M, K, 4, 0):
        pytest.skip("shape not on the GEMV")
    N = 1600
    a, w, bias = bf(M, K, seed=4), bf(N, K, scale=0.03, seed=5), bf(N, scale=0.1, seed=6)
    x = torch.randn(M, N, device=DEV)
    x_ref = x + ref.linear(a, w, bias)
    assert C.gemv(a, w, bias, 4, 0, None, None, 0.0, x, None, None, None, None, 0, 0, 0, None) is None
    close(x, x_ref, 2e-3, 1e-3)
    y = C.gemv(a, w, None, 3, 0, None, None, 0.0, None, None, None, None, None, 0, 0, 0, None)
    close(y, ref.linear(a, w), 2e-3, 1e-3)


@pytest.mark.parametrize("M", [1, 2, 4])
@pytest.mark.parametrize("K", [768, 1600, 4096])
@pytest.mark.parametrize("rms", [False, True])
def test_gemv_fused_norm(C, M, K, rms):
    """norm(x) computed inside the GEMV == the norm kernel's bf16 output fed
    to the plain reference GEMM (fp32 logits and GELU epilogues)."""
    code = 2 if rms else 1
    if not C.gemv_ok(M, K, 3, code):
        pytest.skip("shape not on the fused-norm GEMV")
    N = 520
    x = torch.randn(M, K, device=DEV) * 2 + 0.5
    g, b = (1 + 0.1 * torch.randn(K, device=DEV)).bfloat16(), bf(K, scale=0.1, seed=7)
    w = bf(N, K, scale=0.05, seed=8)
    xn = norm_ref(x, g, b, rms).bfloat16()
    y = C.gemv(x, w, None, 3, code, g, None if rms else b, 1e-5, None, None, None, None, None,
               0, 0, 0, None)
    close(y, ref.linear(xn, w), 2e-2, 2e-2)
    if not rms:
        bias = bf(N, scale=0.1, seed=9)
        y = C.gemv(x, w, bias, 1, code, g, b, 1e-5, None, None, None, None, None, 0, 0, 0, None)
        close(y, ref.gelu_new(ref.linear(xn, w, bias)), 3e-2)


@pytest.mark.parametrize("M", [1, 3, 8])
@pytest.mark.parametrize("norm", [0, 2])
def test_gemv_silu_mul(C, M, norm):
    from llm_sharding_demo_amd.ops.hip import interleave_gate_up

    K, F = 1024, 352  # 2F = 704 W rows: 22 interleaved 32-row blocks
    if not C.gemv_ok(M, K, 2, norm):
        pytest.skip("shape not on the GEMV")
    w = bf(2 * F, K, scale=0.05, seed=10)
    wi = interleave_gate_up(w, F).contiguous()
    if norm:
        x = torch.randn(M, K, device=DEV)
        g = (1 + 0.1 * torch.randn(K, device=DEV)).bfloat16()
        a = ref.rmsnorm(x, g, 1e-5).bfloat16()
        y = C.gemv(x, wi, None, 2, 2, g, None, 1e-5, None, None, None, None, None, 0, 0, 0, None)
    else:
        a = bf(M, K, seed=11)
        y = C.gemv(a, wi, None, 2, 0, None, None, 0.0, None, None, None, None, None, 0, 0, 0, None)
    y_ref = ref.silu_mul(*ref.linear(a, w).split(F, 1))
    close(y, y_ref, 3e-2)


@pytest.mark.parametrize("arch", ["gpt2", "llama"])
@pytest.mark.parametrize("M", [1, 2, 5])
def test_gemv_qkv_kv_append(C, arch, M):
    """QKV epilogue: q out, k/v scattered into the cache at (slot, pos), RoPE
    on the pair-permuted q/k rows (Llama), fused norm when M <= 2."""
    from llm_sharding_demo_amd.ops.hip import rope_pair_permutation, rope_table

    hd, nh, nkv = (64, 6, 6) if arch == "gpt2" else (128, 8, 2)
    H = 768 if arch == "gpt2" else 1024
    q_size, kv_size = nh * hd, nkv * hd
    N = q_size + 2 * kv_size
    slots, max_seq = 6, 96
    w, bias = bf(N, H, scale=0.05, seed=12), (bf(N, scale=0.1, seed=13) if arch == "gpt2" else None)
    x = torch.randn(M, H, device=DEV)
    g = (1 + 0.1 * torch.randn(H, device=DEV)).bfloat16()
    b = bf(H, scale=0.1, seed=14) if arch == "gpt2" else None
    rms = arch == "llama"
    xn = norm_ref(x, g, b, rms).bfloat16()
    tslot = torch.randperm(slots, device=DEV)[:M].int()
    tpos = torch.randint(0, max_seq, (M,), device=DEV).int()
    y = ref.linear(xn, w, bias)
    q = y[:, :q_size].reshape(M, nh, hd)
    k = y[:, q_size:q_size + kv_size].reshape(M, nkv, hd)
    v = y[:, q_size + kv_size:].reshape(M, nkv, hd)
    rope = None
    wk = w
    if arch == "llama":
        q = ref.apply_rope(q.cpu(), tpos.cpu(), 500000.0).to(DEV)
        k = ref.apply_rope(k.cpu(), tpos.cpu(), 500000.0).to(DEV)
        perm = torch.cat([rope_pair_permutation(nh, hd), rope_pair_permutation(nkv, hd) + q_size,
                          torch.arange(q_size + kv_size, N)]).to(DEV)
        wk = w.index_select(0, perm).contiguous()
        rope = rope_table(max_seq, hd, 500000.0, DEV)
        # the kernel writes q and K in the pair-permuted head-dim order
        hp = rope_pair_permutation(1, hd).to(DEV)
        q, k = q[..., hp], k[..., hp]
    for norm in ([0, 2 if rms else 1] if M <= 2 else [0]):
        kc = torch.zeros(slots, nkv, max_seq, hd, dtype=torch.bfloat16, device=DEV)
        vc = torch.zeros_like(kc)
        if norm:
            out = C.gemv(x, wk, bias, 6, norm, g, b, 1e-5, None, kc, vc, tslot, tpos,
                         q_size, kv_size, hd, rope)
        else:
            out = C.gemv(xn, wk, bias, 6, 0, None, None, 0.0, None, kc, vc, tslot, tpos,
                         q_size, kv_size, hd, rope)
        close(out, q.reshape(M, -1), 3e-2)
        sl, ps = tslot.long(), tpos.long()
        close(kc[sl, :, ps], k, 3e-2)
        close(vc[sl, :, ps], v, 3e-2)
        assert int((kc != 0).sum()) == M * nkv * hd  # nothing else written


def test_gemv_rejects_unsupported(C):
    assert not C.gemv_ok(9, 1600, 0, 0)       # more than 8 rows
    assert not C.gemv_ok(8, 6400, 0, 0)       # LDS image over 64 KiB
    assert not C.gemv_ok(8, 1600, 0, 1)       # fused norm: at most 4 rows x 2048 of K
    assert not C.gemv_ok(2, 6400, 0, 2)
    assert not C.gemv_ok(1, 1600, 5, 0)       # no split-K slab epilogue


@pytest.mark.parametrize("M", [1, 2, 5, 8])
@pytest.mark.parametrize("norm", [0, 1, 2])
@pytest.mark.parametrize("K,N", [(1600, 50304), (4096, 128256), (768, 1000)])
def test_gemv_logits_segmax(C, M, norm, K, N):
    """The lm_head GEMV's segment maxima (one workgroup = one 8-logit
    segment) equal a max over the fp32 logits it stores, the logits equal the
    plain fp32 GEMV's, and the sampler draws the same tokens from them as from
    the full rows (bit-equal to the host reference)."""
    from llm_sharding_demo_amd.runtime.batch import counter_uniform

    if not C.gemv_ok(M, K, 3, norm):
        pytest.skip("shape not on the GEMV")
    g = torch.Generator(device=DEV).manual_seed(M * 7 + norm)
    if norm:
        x = torch.randn(M, K, device=DEV, generator=g) * 2 + 0.3
        gm, b = (1 + 0.1 * torch.randn(K, device=DEV, generator=g)).bfloat16(), bf(K, scale=0.1, seed=3)
        args = (norm, gm, b if norm == 1 else None, 1e-5)
    else:
        x = bf(M, K, seed=2)
        args = (0, None, None, 0.0)
    w = bf(N, K, scale=0.05, seed=11)
    seg = torch.full((M, N // 8), float("nan"), device=DEV)
    y = C.gemv_logits(x, w, *args, seg)
    y0 = C.gemv(x, w, None, 3, *args, None, None, None, None, None, 0, 0, 0, None)
    assert torch.equal(y, y0)
    assert torch.equal(seg, y.view(M, N // 8, 8).amax(-1))
    V = N - 7 if N % 64 == 0 else N  # a partial last segment past the real vocabulary
    y[:, V:] = 100.0  # padding: never drawn (the sampler rescans the partial last segment)
    temp = torch.full((M,), 0.6, device=DEV)
    topk = torch.full((M,), 40, dtype=torch.int32, device=DEV)
    greedy = torch.zeros(M, dtype=torch.int32, device=DEV)
    seeds = torch.arange(M, dtype=torch.int64, device=DEV) * 31 + 5
    step = torch.arange(M, dtype=torch.int64, device=DEV)
    out = C.sample(y, V, temp, topk, greedy, seeds, step, seg)
    exp = ref.sample(y.cpu(), temp.cpu(), topk.cpu(), greedy.cpu(), counter_uniform(seeds.cpu(), step.cpu()), V)
    assert out.cpu().tolist() == exp.tolist()
