"""Long context: positions up to the model's cap.

The reference recomputes the full sequence every token and is bounded only by
GPT-2's 1024 positions (`/root/reference/server.py:169-181`).  Here the
shard-local KV cache, chunked prefill and the split-K decode attention must
hold up to the cap: GPT-2 1024 positions, the Llama test config 2048.
CPU tests run the fp32 reference path; the GPU tests compare the HIP path
(prefill flash attention over long ragged rows, decode attention with many
KV splits) against the fp32 golden of the same weights.
"""
import pytest
import torch

from llm_sharding_demo_amd.config import EngineConfig, SamplingParams, get_model_config
from llm_sharding_demo_amd.models.stage import StageModel
from llm_sharding_demo_amd.runtime.batch import BatchMeta
from llm_sharding_demo_amd.runtime.engine import Engine

from .helpers import full_weights


def _prompts(n_pos, vocab, seed=0):
    g = torch.Generator().manual_seed(seed)
    return [torch.randint(1, vocab, (n,), generator=g).tolist() for n in n_pos]


@pytest.mark.parametrize("model,lens,chunk", [("gpt2-test", (1000, 517, 3), 128),
                                              ("llama-test", (2000, 1023), 256)])
def test_long_prompt_chunked_prefill_cpu(model, lens, chunk):
    """Prompts close to the position cap: chunked prefill through a 2-stage
    pipeline == one-shot prefill on one stage, decode continues to the cap."""
    mc = get_model_config(model)
    prompts = _prompts(lens, mc.vocab_size)
    gen = mc.max_positions - max(lens)  # fill every position up to the cap
    sp = SamplingParams(greedy=True, max_new_tokens=gen)
    base = Engine(EngineConfig(model_id=model, max_batch=4, device="cpu", max_seq_len=mc.max_positions))
    want = base.generate_ids(prompts, sp)
    eng = Engine(EngineConfig(model_id=model, num_stages=2, max_batch=4, device="cpu",
                              max_seq_len=mc.max_positions, prefill_chunk=chunk))
    got = eng.generate_ids(prompts, sp, microbatches=2)
    assert got == want
    assert [len(o) for o in got] == [gen] * len(prompts)


def test_prompt_over_cap_is_rejected():
    mc = get_model_config("gpt2-test")
    eng = Engine(EngineConfig(model_id="gpt2-test", max_batch=2, device="cpu", max_seq_len=mc.max_positions))
    with pytest.raises(ValueError):
        eng.generate_ids([[1] * (mc.max_positions + 1)], SamplingParams(greedy=True, max_new_tokens=1))


@pytest.mark.gpu
@pytest.mark.parametrize("model,lens", [("gpt2-test", (1000, 300, 777)), ("llama-test", (2000, 1500, 64))])
def test_long_context_hip_matches_fp32_golden(model, lens):
    """HIP prefill + 6 decode steps at up to 2000 cached positions vs the fp32
    CPU stage on the same weights (bf16 tolerance as the short-context test)."""
    mc = get_model_config(model)
    w = full_weights(mc)
    max_seq = mc.max_positions
    cpu = StageModel(mc, 0, mc.n_layers, True, True, weights=w, max_slots=4, max_seq=max_seq)
    gpu = StageModel(mc, 0, mc.n_layers, True, True, device="cuda", weights=w, max_slots=4, max_seq=max_seq)
    prompts = _prompts(lens, mc.vocab_size, seed=1)
    n = len(prompts)
    flat = torch.tensor([t for p in prompts for t in p], dtype=torch.int32)
    lc = cpu.forward(BatchMeta.build(list(range(n)), [0] * n, list(lens), "cpu"), flat)[:, : mc.vocab_size]
    lg = gpu.forward(BatchMeta.build(list(range(n)), [0] * n, list(lens), "cuda"), flat.cuda())
    torch.testing.assert_close(lg[:, : mc.vocab_size].cpu(), lc, atol=0.05, rtol=0.05)
    for step in range(6):
        toks = torch.tensor([(7 * step + i) % mc.vocab_size + 1 for i in range(n)], dtype=torch.int32)
        pos = [L + step for L in lens]
        dc = cpu.forward(BatchMeta.decode(list(range(n)), pos, "cpu", max(pos) + 1), toks)[:, : mc.vocab_size]
        dg = gpu.forward(BatchMeta.decode(list(range(n)), pos, "cuda", max(pos) + 1), toks.cuda())
        torch.testing.assert_close(dg[:, : mc.vocab_size].cpu(), dc, atol=0.05, rtol=0.05)


@pytest.mark.gpu
def test_long_context_chunked_prefill_hip_matches_one_shot():
    """HIP path, 1900 + 1200 + 5-token prompts: prefill in 256-token chunks
    through the KV cache == one-shot prefill, to bf16 tolerance (the GEMM
    split choice depends on the chunk's rows, so the two are not bit-equal),
    and the engine's chunked 2-stage pipeline generates to the 2048 cap."""
    mc = get_model_config("llama-test")
    w = full_weights(mc)
    lens = [1900, 1200, 5]
    prompts = _prompts(lens, mc.vocab_size, seed=2)
    n, max_seq = len(lens), mc.max_positions
    one = StageModel(mc, 0, mc.n_layers, True, True, device="cuda", weights=w, max_slots=4, max_seq=max_seq)
    chk = StageModel(mc, 0, mc.n_layers, True, True, device="cuda", weights=w, max_slots=4, max_seq=max_seq)
    flat = torch.tensor([t for p in prompts for t in p], dtype=torch.int32)
    want = one.forward(BatchMeta.build(list(range(n)), [0] * n, lens, "cuda"), flat.cuda())[:, : mc.vocab_size]
    got = [None] * n
    for start in range(0, max(lens), 256):
        rows = [i for i in range(n) if start < lens[i]]
        q = [min(256, lens[i] - start) for i in rows]
        ids = torch.tensor([t for i, m in zip(rows, q) for t in prompts[i][start:start + m]], dtype=torch.int32)
        out = chk.forward(BatchMeta.build(rows, [start] * len(rows), q, "cuda"), ids.cuda())
        for j, i in enumerate(rows):
            if start + q[j] == lens[i]:
                got[i] = out[j, : mc.vocab_size]
    torch.testing.assert_close(torch.stack(got).cpu(), want.cpu(), atol=0.05, rtol=0.05)

    sp = SamplingParams(greedy=True, max_new_tokens=max_seq - 1900)
    eng = Engine(EngineConfig(model_id="llama-test", num_stages=2, max_batch=4, device="cuda",
                              max_seq_len=max_seq, prefill_chunk=256), devices=["cuda:0"] * 2)
    ref = Engine(EngineConfig(model_id="llama-test", max_batch=4, device="cuda", max_seq_len=max_seq))
    a, b = eng.generate_ids(prompts, sp, microbatches=2), ref.generate_ids(prompts, sp)
    assert [len(o) for o in a] == [sp.max_new_tokens] * n
    assert [o[0] for o in a] == [o[0] for o in b]  # first token: same prefill logits' argmax
