"""Do pad rows (scratch slot, pos 0) change a real row's decode logits?"""
import importlib.util
import os
import pathlib
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

torch.use_deterministic_algorithms(True, warn_only=True)
torch.utils.deterministic.fill_uninitialized_memory = True
from llm_sharding_demo_amd.config import get_model_config  # noqa: E402
from llm_sharding_demo_amd.models.stage import StageModel  # noqa: E402
from llm_sharding_demo_amd.runtime.batch import BatchMeta  # noqa: E402

spec = importlib.util.spec_from_file_location("helpers", pathlib.Path(__file__).parent.parent / "tests" / "helpers.py")
h = importlib.util.module_from_spec(spec)
spec.loader.exec_module(h)
mc = get_model_config("gpt2-test")
w = h.full_weights(mc)
res = {}
for b, n in ((12, 12), (16, 12), (16, 16)):
    st = StageModel(mc, 0, mc.n_layers, True, True, device="cuda", weights=w, max_slots=20, max_seq=64)
    prompts = [[i + 1, 2 * i + 3, 5] for i in range(12)]
    flat = torch.tensor([t for p in prompts for t in p], dtype=torch.int32, device="cuda")
    st.forward(BatchMeta.build(list(range(12)), [0] * 12, [3] * 12, "cuda"), flat)
    outs = []
    for step in range(9):
        slots = list(range(12)) + [19] * (b - 12)
        pos = [3 + step] * 12 + [0] * (b - 12)
        meta = BatchMeta.decode(slots, pos, "cuda", 3 + step + 1)
        toks = torch.tensor([7 + step] * b, dtype=torch.int32, device="cuda")
        outs.append(st.forward(meta, toks)[:12, : mc.vocab_size].clone())
    res[(b, n)] = outs
for k in res:
    print(k, [bool(torch.equal(a, b)) for a, b in zip(res[(12, 12)], res[k])], flush=True)
