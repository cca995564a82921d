#!/usr/bin/env python3
"""Whole-model numerics at the headline's decode shape: GPT-2 XL, 256 sequences (256-row
decode GEMMs on the 8-wave ring with split-K slabs folded by the norm), HIP logits vs the
fp32 golden of the same weights over a 32-token prefill and 6 teacher-forced decode steps.
Run once per slab dtype (LSD_SLAB_BF16 is read once per process)."""
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_demo_amd.utils.golden import compare_with_golden  # noqa: E402

rnd = random.Random(7)
model = sys.argv[1] if len(sys.argv) > 1 else "gpt2-xl"
prompts = [[rnd.randrange(50257) for _ in range(32)] for _ in range(256)]
r = compare_with_golden(model, prompts, steps=6)
print(f"{model} LSD_SLAB_BF16={os.environ.get('LSD_SLAB_BF16', '0')}: "
      f"top1 {r['top1_agreement']:.4f} max_rel {r['max_rel_err']:.4f} mean_rel {r['mean_rel_err']:.4f} rows {r['rows']}",
      flush=True)
