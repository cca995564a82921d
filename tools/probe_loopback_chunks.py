"""Which loopback configurations reproduce the P = 1 tokens (same prefill
chunk) : stages x prefill chunk x alternating splits (LSD_ALT_SPLIT read at
Engine construction).  Chunked vs one-shot prefill is NOT bit-identical (other
GEMM row counts / kernels round differently), so the reference uses the same
chunk."""
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from llm_sharding_demo_amd.config import EngineConfig, SamplingParams  # noqa: E402
from llm_sharding_demo_amd.runtime.engine import Engine  # noqa: E402

sp = SamplingParams(temperature=0.8, top_k=20, seed=7, max_new_tokens=10)
prompts = [[i + 1, 2 * i + 3, 5] for i in range(12)]
cases = [(2, 2, "1"), (3, 0, "1"), (3, 2, "1"), (3, 2, "0"), (2, 2, "0"), (3, 1, "0"), (4, 1, "0")]
for P, chunk, alt in cases:
    os.environ["LSD_ALT_SPLIT"] = alt
    one = Engine(EngineConfig(model_id="gpt2-test", num_stages=1, max_batch=16, device="cuda",
                              num_microbatches=2 * P, prefill_chunk=chunk)).generate_ids(prompts, sp)
    for transport in ("loopback", "local"):
        e = Engine(EngineConfig(model_id="gpt2-test", num_stages=P, max_batch=16, device="cuda",
                                num_microbatches=2 * P, transport=transport, prefill_chunk=chunk))
        got = e.generate_ids(prompts, sp)
        bad = [i for i in range(len(prompts)) if got[i] != one[i]]
        print(f"P={P} chunk={chunk} alt={alt} {transport}: alt_plans={e.unit_plans is not None} "
              f"mismatching sequences {bad}", flush=True)
        e.shutdown()
