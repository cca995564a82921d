import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from llm_sharding_demo_amd.ops.hip import _load
C = _load()
torch.manual_seed(0)
cnt = torch.zeros(1 << 16, dtype=torch.int32, device="cuda")
for (N, K) in [(1000, 128), (384, 128), (128, 512), (512, 128), (50304, 1600)]:
    w = (torch.randn(N, K, device="cuda") * 0.05).bfloat16()
    x = torch.randn(16, K, device="cuda").bfloat16()
    for epi in (0, 1):
        outs = {}
        for M in (1, 2, 3, 4, 8):
            if C.gemv_ok(M, K, epi, 0):
                outs[M] = C.gemv(x[:M].contiguous(), w, None, epi, 0, None, None, 0.0, None, None, None, None, None, 0, 0, 0, None)
        base = outs.get(1)
        print(N, K, "epi", epi, {M: bool(torch.equal(o[:1].float(), base[:1].float())) for M, o in outs.items()})
    # split-K decode GEMM at MT=1 (9 rows) vs MT=2 (18 rows)
    if N % 64:
        continue
    a = torch.randn(18, K, device="cuda").bfloat16()
    y18 = C.linear(a, w, None, 0, False, 2, cnt)
    y9 = C.linear(a[:9].contiguous(), w, None, 0, False, 2, cnt)
    print("  sk 9 vs 18 rows equal:", bool(torch.equal(y18[:9], y9)))
    # prefill attention + the rest of a full stage: batch composition of a forward
from llm_sharding_demo_amd.config import get_model_config
from llm_sharding_demo_amd.models.stage import StageModel
from llm_sharding_demo_amd.runtime.batch import BatchMeta
import importlib.util, pathlib
spec = importlib.util.spec_from_file_location("helpers", pathlib.Path(__file__).parent.parent / "tests" / "helpers.py")
h = importlib.util.module_from_spec(spec); spec.loader.exec_module(h)
mc = get_model_config("gpt2-test")
w = h.full_weights(mc)
for nseq in (3, 6):
    st = StageModel(mc, 0, mc.n_layers, True, True, device="cuda", weights=w, max_slots=16, max_seq=64)
    prompts = [[i + 1, 2 * i + 3, 5] for i in range(nseq)]
    flat = torch.tensor([t for p in prompts for t in p], dtype=torch.int32, device="cuda")
    lg = st.forward(BatchMeta.build(list(range(nseq)), [0] * nseq, [3] * nseq, "cuda"), flat)
    toks = torch.tensor([7] * nseq, dtype=torch.int32, device="cuda")
    dg = st.forward(BatchMeta.decode(list(range(nseq)), [3] * nseq, "cuda", 4), toks)
    if nseq == 3:
        p3, d3 = lg.clone(), dg.clone()
    else:
        print("stage prefill rows 0-2 equal (3 vs 6 seqs):", bool(torch.equal(p3, lg[:3])),
              "decode:", bool(torch.equal(d3, dg[:3])))
