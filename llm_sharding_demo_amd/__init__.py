"""MI355X-native pipeline-sharded LLM inference.

Same capabilities/API as kanchan-rihan/llm-sharding-demo (coordinator /
shard-A / shard-B roles, /generate /forward /forward_b, generate_text), but
the shards are pipeline stages pinned one per MI355X, linked by RCCL p2p over
xGMI, with a shard-local KV cache, hipGraph-captured decode steps and
hand-written CDNA4 HIP kernels for the whole forward pass.
"""
from __future__ import annotations

from typing import Optional

from .config import MODEL_PRESETS, EngineConfig, ModelConfig, SamplingParams, get_model_config

__all__ = ["EngineConfig", "ModelConfig", "SamplingParams", "MODEL_PRESETS", "get_model_config",
           "Engine", "LLM", "generate_text"]
__version__ = "0.1.0"


def __getattr__(name):
    if name == "Engine":
        from .runtime.engine import Engine
        return Engine
    raise AttributeError(name)


class LLM:
    """In-process front-end: engine + tokenizer.

    >>> llm = LLM(EngineConfig(model_id="gpt2", num_stages=1))
    >>> llm.generate_text("Hi, ", max_new_tokens=2)
    {'generated': 'Hi, ...'}
    """

    def __init__(self, cfg: Optional[EngineConfig] = None, **kw):
        from .runtime.engine import build_engine
        from .utils.tokenizer import load_tokenizer

        cfg = cfg or EngineConfig.from_env()
        self.engine = build_engine(cfg, **kw)
        mc = cfg.model
        self.tokenizer = load_tokenizer(cfg.model_id, mc.arch, cfg.weights, mc.eos_token_id)

    def generate_text(self, prompt: str, max_new_tokens: int = 20, **sampling) -> dict:
        """Same return contract as the reference /generate: prompt + continuation."""
        ids = self.tokenizer.encode(prompt)
        sp = SamplingParams(max_new_tokens=max_new_tokens, **sampling)
        if max_new_tokens == 0:
            return {"generated": self.tokenizer.decode(ids, skip_special_tokens=True)}
        out = self.engine.generate_ids([ids], [sp])[0]
        return {"generated": self.tokenizer.decode(ids + out, skip_special_tokens=True)}

    def generate(self, prompts, max_new_tokens: int = 20, **sampling):
        ids = [self.tokenizer.encode(p) for p in prompts]
        sp = [SamplingParams(max_new_tokens=max_new_tokens, **sampling) for _ in prompts]
        outs = self.engine.generate_ids(ids, sp)
        return [self.tokenizer.decode(i + o) for i, o in zip(ids, outs)]


def generate_text(prompt: str, max_new_tokens: int = 20, url: Optional[str] = None, **kw):
    """HTTP client helper with the notebook's contract (notebook.ipynb:111-120)."""
    from .serving.client import generate_text as _gt

    return _gt(prompt, max_new_tokens, url=url, **kw)
