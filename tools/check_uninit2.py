"""Which P=1 configuration reads uninitialised memory (torch.empty filled)?"""
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
for name, kw in [("graphs M=2", dict(num_microbatches=2)), ("eager M=2", dict(num_microbatches=2, use_graphs=False)),
                 ("graphs M=1", dict(num_microbatches=1)), ("graphs M=4", dict(num_microbatches=4)),
                 ("graphs M=2 again", dict(num_microbatches=2))]:
    e = Engine(EngineConfig(model_id="gpt2-test", num_stages=1, max_batch=16, device="cuda", max_seq_len=512, **kw))
    out = e.generate_ids(prompts, sp)
    out2 = e.generate_ids(prompts, sp)
    print(name, [o[9] for o in out], "second session", [o[9] for o in out2], flush=True)
