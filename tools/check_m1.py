"""P=1: one 16-row group (4 pad rows) vs two groups -- per-step row-0 sampler inputs."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_sharding_demo_amd.config import EngineConfig, SamplingParams  # noqa: E402
from llm_sharding_demo_amd.ops.hip import HipBackend  # noqa: E402
from llm_sharding_demo_amd.runtime.engine import Engine  # noqa: E402

rec = []
orig = HipBackend.sample


def spy(self, logits, samp, vocab):
    out = orig(self, logits, samp, vocab)
    torch.cuda.synchronize()
    rec.append((logits.shape[0], logits[0, :vocab].float().cpu().clone(), float(samp.temperature[0]),
                int(samp.top_k[0]), int(samp.greedy[0]), int(samp.seeds[0]), int(samp.step[0]), int(out[0])))
    return out


HipBackend.sample = spy
sp = SamplingParams(temperature=0.8, top_k=20, seed=7, max_new_tokens=10)
prompts = [[i + 1, 2 * i + 3, 5] for i in range(12)]
runs = {}
for M in (1, 2):
    rec.clear()
    e = Engine(EngineConfig(model_id="gpt2-test", num_stages=1, max_batch=16, device="cuda", max_seq_len=512,
                            num_microbatches=M, use_graphs=False))
    out = e.generate_ids(prompts, sp)
    runs[M] = (out[0], list(rec))
    print("M", M, "seq0", out[0], flush=True)
a, b = runs[1][1], runs[2][1]
# row 0 of group 0 is seq 0 in both layouts: compare the group-0 sample calls in order
ga = [r for r in a]
gb = [r for r in b if r[0] in (8,) or True]
for i, r in enumerate(a):
    print("M1 call", i, "rows", r[0], "T", r[2], "k", r[3], "greedy", r[4], "seed", r[5], "step", r[6], "tok", r[7])
for i, r in enumerate(b):
    print("M2 call", i, "rows", r[0], "T", r[2], "k", r[3], "greedy", r[4], "seed", r[5], "step", r[6], "tok", r[7])
