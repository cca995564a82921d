"""Repeat the loopback P=2 vs P=1 comparison (flakiness probe)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_demo_amd.config import EngineConfig, SamplingParams  # noqa: E402
from llm_sharding_demo_amd.runtime.engine import Engine  # noqa: E402

sp = SamplingParams(temperature=0.8, top_k=20, seed=7, max_new_tokens=10)
prompts = [[i + 1, 2 * i + 3, 5] for i in range(12)]
M = int(sys.argv[1]) if len(sys.argv) > 1 else 2
one_e = Engine(EngineConfig(model_id="gpt2-test", num_stages=1, max_batch=16, device="cuda",
                            max_seq_len=512, num_microbatches=M))
one = one_e.generate_ids(prompts, sp)
for rep in range(3):
    again = one_e.generate_ids(prompts, sp)
    print("P=1 repeat", rep, again == one, flush=True)
for P in (2, 4):
    e = Engine(EngineConfig(model_id="gpt2-test", num_stages=P, max_batch=16, device="cuda",
                            num_microbatches=2 * P, transport="loopback"))
    for rep in range(3):
        got = e.generate_ids(prompts, sp)
        diff = [(i, j) for i, (a, b) in enumerate(zip(got, one)) for j, (x, y) in enumerate(zip(a, b)) if x != y]
        print("P", P, "rep", rep, got == one, diff[:5], flush=True)
    e.shutdown()
    l = Engine(EngineConfig(model_id="gpt2-test", num_stages=P, max_batch=16, device="cuda",
                            num_microbatches=2 * P), devices=["cuda:0"] * P)
    got = l.generate_ids(prompts, sp)
    print("P", P, "local-transport", got == one, flush=True)
    l.shutdown()
