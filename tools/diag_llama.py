"""HIP vs fp32 golden vs bf16 emulation, Llama-3 8B dims at several depths."""
import dataclasses
import random
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from llm_sharding_demo_amd.config import get_model_config
from llm_sharding_demo_amd.utils.golden import compare_three_way

rnd = random.Random(3)
for name, L in [("llama-3-8b", 1), ("llama-3-8b", 4), ("llama-3-8b", 32), ("gpt2-xl", 48)]:
    mc = dataclasses.replace(get_model_config(name), n_layers=L)
    prompts = [[rnd.randrange(mc.vocab_size) for _ in range(n)] for n in (9, 40)]
    print(name, L, compare_three_way(mc, prompts, steps=3), flush=True)
    torch.cuda.empty_cache()
