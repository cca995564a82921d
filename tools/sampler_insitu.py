#!/usr/bin/env python3
"""The sampler on the headline model's own logits: GPT-2 XL (random init), one
256-row decode step at 128 cached positions -> fp32 logits + segment maxima,
then the sampler (T 0.6, top-k 40) timed on them and the number of threshold
candidates per row (the fast path's superset: elements >= the k-th largest of
the 64 group maxima, emulated on the host).  hipGraph-replayed."""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_sharding_demo_amd.config import get_model_config  # noqa: E402
from llm_sharding_demo_amd.models.stage import StageModel  # noqa: E402
from llm_sharding_demo_amd.runtime.batch import BatchMeta, SamplingState  # noqa: E402
from tools.microbench import timeit  # noqa: E402


def main():
    dev = torch.device("cuda")
    mc = get_model_config(os.environ.get("SI_MODEL", "gpt2-xl"))
    R, CTX = 256, 128
    st = StageModel(mc, 0, mc.n_layers, True, True, device=dev, dtype=torch.bfloat16, max_slots=R + 2,
                    max_seq=CTX + 8)
    be = st.backend
    meta = BatchMeta.decode(list(range(R)), [CTX] * R, dev, CTX + 1)
    ids = torch.randint(0, mc.vocab_size, (R,), dtype=torch.int32, device=dev)
    with torch.no_grad():
        lg = st.forward(meta, ids, head=True)
    seg = getattr(lg, "_lsd_segmax", None)
    V = mc.vocab_size
    samp = SamplingState([0.6] * R, [40] * R, [False] * R, list(range(R)), dev)
    C = be.C
    t_seg = timeit(lambda: C.sample(lg, V, samp.temperature, samp.top_k, samp.greedy, samp.seeds, samp.step, seg))
    t_full = timeit(lambda: C.sample(lg, V, samp.temperature, samp.top_k, samp.greedy, samp.seeds, samp.step))
    x = lg[:, :V].float()
    # host emulation of the fast path's threshold: 64 groups of the row (contiguous ranges)
    groups = torch.tensor_split(x, 64, dim=1)
    gmax = torch.stack([g.amax(1) for g in groups], 1)
    tau = gmax.topk(40, dim=1).values[:, -1:]
    cand = (x >= tau).sum(1).float()
    std = x.std(1)
    print(json.dumps({"model": mc.name if hasattr(mc, "name") else "", "rows": R, "sample_us_seg": round(t_seg, 2),
                      "sample_us_full": round(t_full, 2), "cand_mean": round(float(cand.mean()), 1),
                      "cand_max": int(cand.max()), "rows_over_256": int((cand > 256).sum()),
                      "rows_over_1024": int((cand > 1024).sum()), "logit_std_mean": round(float(std.mean()), 4),
                      "distinct_top40_frac": round(float(torch.stack([r.topk(40).values.unique().numel() / 40.0
                                                                       for r in torch.unbind(x[:8])]).mean()) if False else 0, 3)}),
          flush=True)


if __name__ == "__main__":
    main()
