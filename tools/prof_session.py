import cProfile, pstats, random, time
from llm_sharding_demo_amd.config import EngineConfig, SamplingParams
from llm_sharding_demo_amd.runtime.engine import Engine
B = 4096
cfg = EngineConfig(model_id="gpt2-test", num_stages=1, max_batch=B, device="cpu", num_microbatches=16, max_seq_len=32)
eng = Engine(cfg)
rnd = random.Random(0)
prompts = [[rnd.randrange(100) for _ in range(6)] for _ in range(B)]
sp = SamplingParams(temperature=0.6, top_k=40, max_new_tokens=3, seed=1234)
eng.generate_ids(prompts, [sp] * B)
t0 = time.perf_counter(); eng.generate_ids(prompts, [sp] * B); print("session s", time.perf_counter() - t0)
pr = cProfile.Profile(); pr.enable(); eng.generate_ids(prompts, [sp] * B); pr.disable()
st = pstats.Stats(pr); st.sort_stats("cumulative").print_stats("scheduler|engine.py|plan.py|batch.py|native|pipeline.py", 40)
