#!/usr/bin/env python3
"""Quickstart (the reference's notebook.ipynb, minus minikube).

1. In-process: build the engine on this machine's GPUs (or CPU) and generate.
2. HTTP: start the server, then call generate_text() exactly like the
   reference notebook (notebook.ipynb:111-126).

    # single GPU
    python -m llm_sharding_demo_amd serve --model-id gpt2 &
    # 8 x MI355X, one pipeline stage per GPU (rank 0 serves HTTP)
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        -m llm_sharding_demo_amd serve --model-id gpt2-xl
"""
import sys

from llm_sharding_demo_amd import LLM, EngineConfig, generate_text


def in_process():
    import torch

    dev = "cuda" if torch.cuda.is_available() else "cpu"
    llm = LLM(EngineConfig(model_id="gpt2" if dev == "cuda" else "gpt2-test", device=dev,
                           max_batch=8, max_seq_len=256))
    print(llm.generate_text("Hi, ", max_new_tokens=8))                      # reference sampler
    print(llm.generate_text("Hi, ", max_new_tokens=8, greedy=True))         # argmax
    print(llm.generate_text("Hi, ", max_new_tokens=8, seed=1234))           # reproducible


def over_http(url="http://127.0.0.1:5000/generate"):
    # identical call and return contract to the reference notebook
    print(generate_text("Hi, ", max_new_tokens=2, url=url))


if __name__ == "__main__":
    over_http() if "--http" in sys.argv else in_process()
