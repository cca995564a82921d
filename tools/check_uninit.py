"""Loopback / multi-stage comparison with every torch.empty filled with
NaN / INT_MAX (torch deterministic fill): an engine read of uninitialised
device memory shows up as a token mismatch or an error."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

torch.use_deterministic_algorithms(True, warn_only=True)
torch.utils.deterministic.fill_uninitialized_memory = True
from llm_sharding_demo_amd.config import EngineConfig, SamplingParams  # noqa: E402
from llm_sharding_demo_amd.runtime.engine import Engine  # noqa: E402

sp = SamplingParams(temperature=0.8, top_k=20, seed=7, max_new_tokens=10)
prompts = [[i + 1, 2 * i + 3, 5] for i in range(12)]
one = Engine(EngineConfig(model_id="gpt2-test", num_stages=1, max_batch=16, device="cuda",
                          max_seq_len=512)).generate_ids(prompts, sp)
print("P=1", one[0], flush=True)
for P in (2, 4):
    e = Engine(EngineConfig(model_id="gpt2-test", num_stages=P, max_batch=16, device="cuda",
                            num_microbatches=2 * P, transport="loopback"))
    got = e.generate_ids(prompts, sp)
    diff = [(i, j) for i, (a, b) in enumerate(zip(got, one)) for j, (x, y) in enumerate(zip(a, b)) if x != y]
    print("P", P, got == one, diff[:8], flush=True)
    e.shutdown()
