"""Configuration: model presets, engine settings, env-var compatibility.

The reference configures itself only through six environment variables
(`/root/reference/server.py:20-25`): MODEL_ID, SHARD_ROLE, SPLIT_AT,
SHARD_A_SERVICE, SHARD_B_SERVICE, SHARD_PORT.  Those names are kept here with
the same defaults; everything else the MI355X engine needs (stage count,
microbatching, KV budget, sampling defaults) is a dataclass field that can be
set from CLI > env > defaults.

Sampling defaults match the reference's hard-coded sampler
(`server.py:187-188`: temperature 0.6, top-k 40, multinomial).
"""
from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass, field
from typing import Optional, Sequence


# ---------------------------------------------------------------------------
# Model presets
# ---------------------------------------------------------------------------

@dataclass(frozen=True)
class ModelConfig:
    """Architecture description shared by the GPT-2 and Llama families."""

    name: str
    arch: str  # "gpt2" | "llama"
    vocab_size: int
    hidden: int
    n_layers: int
    n_heads: int
    n_kv_heads: int
    ffn: int
    max_positions: int
    norm_eps: float
    tie_embeddings: bool
    rope_theta: float = 0.0
    bos_token_id: int = 50256
    eos_token_id: int = 50256

    @property
    def head_dim(self) -> int:
        return self.hidden // self.n_heads

    @property
    def q_size(self) -> int:
        return self.n_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.n_kv_heads * self.head_dim

    @property
    def qkv_size(self) -> int:
        return self.q_size + 2 * self.kv_size

    @property
    def vocab_padded(self) -> int:
        """Vocab rounded up to a multiple of 64 so lm_head tiles evenly."""
        return (self.vocab_size + 63) // 64 * 64

    def block_params(self) -> int:
        h, f = self.hidden, self.ffn
        if self.arch == "gpt2":
            return 12 * h * h + 13 * h  # qkv+proj+fc+proj weights/biases + 2 LN
        return h * self.qkv_size + self.q_size * h + 3 * h * f + 2 * h

    def embed_params(self) -> int:
        n = self.vocab_size * self.hidden
        if self.arch == "gpt2":
            n += self.max_positions * self.hidden
        return n

    def lm_head_params(self) -> int:
        return self.vocab_size * self.hidden

    def kv_bytes_per_token_per_layer(self, dtype_bytes: int = 2) -> int:
        return 2 * self.kv_size * dtype_bytes


def _gpt2(name: str, h: int, l: int, nh: int, vocab: int = 50257) -> ModelConfig:
    return ModelConfig(
        name=name, arch="gpt2", vocab_size=vocab, hidden=h, n_layers=l,
        n_heads=nh, n_kv_heads=nh, ffn=4 * h, max_positions=1024,
        norm_eps=1e-5, tie_embeddings=True)


# Dims from [tf5.15] models/gpt2/configuration_gpt2.py and SURVEY.md §2.5.
MODEL_PRESETS = {
    # sshleifer/tiny-gpt2: the reference default MODEL_ID (server.py:20)
    "tiny-gpt2": _gpt2("tiny-gpt2", 2, 2, 2),
    "gpt2": _gpt2("gpt2", 768, 12, 12),
    "gpt2-medium": _gpt2("gpt2-medium", 1024, 24, 16),
    "gpt2-large": _gpt2("gpt2-large", 1280, 36, 20),
    "gpt2-xl": _gpt2("gpt2-xl", 1600, 48, 25),
    # Small GPT-2 shapes used by kernel / pipeline tests (hd = 64 like real GPT-2).
    "gpt2-test": _gpt2("gpt2-test", 128, 4, 2, vocab=1000),
    "llama-3-8b": ModelConfig(
        name="llama-3-8b", arch="llama", vocab_size=128256, hidden=4096,
        n_layers=32, n_heads=32, n_kv_heads=8, ffn=14336, max_positions=8192,
        norm_eps=1e-5, tie_embeddings=False, rope_theta=500000.0,
        bos_token_id=128000, eos_token_id=128001),
    "llama-test": ModelConfig(
        name="llama-test", arch="llama", vocab_size=1000, hidden=256,
        n_layers=4, n_heads=4, n_kv_heads=2, ffn=512, max_positions=2048,
        norm_eps=1e-5, tie_embeddings=False, rope_theta=10000.0,
        bos_token_id=1, eos_token_id=2),
}

_ALIASES = {
    "sshleifer/tiny-gpt2": "tiny-gpt2",
    "openai-community/gpt2": "gpt2",
    "gpt2-small": "gpt2",
    "openai-community/gpt2-medium": "gpt2-medium",
    "openai-community/gpt2-large": "gpt2-large",
    "openai-community/gpt2-xl": "gpt2-xl",
    "meta-llama/Meta-Llama-3-8B": "llama-3-8b",
    "meta-llama/Llama-3.1-8B": "llama-3-8b",
    "llama3-8b": "llama-3-8b",
}


def get_model_config(model_id: str) -> ModelConfig:
    """Resolve a preset name or HF-style id to a ModelConfig."""
    key = _ALIASES.get(model_id, model_id)
    if key in MODEL_PRESETS:
        return MODEL_PRESETS[key]
    # A local HF directory with a config.json: read the dims from it.
    cfg_path = os.path.join(model_id, "config.json")
    if os.path.isfile(cfg_path):
        return model_config_from_hf_json(cfg_path)
    raise KeyError(f"unknown model {model_id!r}; presets: {sorted(MODEL_PRESETS)}")


def model_config_from_hf_json(path: str) -> ModelConfig:
    import json

    with open(path) as f:
        c = json.load(f)
    mt = c.get("model_type", "gpt2")
    if mt == "gpt2":
        h = c["n_embd"]
        return ModelConfig(
            name=os.path.basename(os.path.dirname(path)) or "gpt2", arch="gpt2",
            vocab_size=c["vocab_size"], hidden=h, n_layers=c["n_layer"],
            n_heads=c["n_head"], n_kv_heads=c["n_head"],
            ffn=c.get("n_inner") or 4 * h, max_positions=c["n_positions"],
            norm_eps=c.get("layer_norm_epsilon", 1e-5), tie_embeddings=True,
            bos_token_id=c.get("bos_token_id", 50256),
            eos_token_id=c.get("eos_token_id", 50256))
    if mt == "llama":
        eos = c.get("eos_token_id", 2)
        if isinstance(eos, list):
            eos = eos[0]
        return ModelConfig(
            name=os.path.basename(os.path.dirname(path)) or "llama", arch="llama",
            vocab_size=c["vocab_size"], hidden=c["hidden_size"],
            n_layers=c["num_hidden_layers"], n_heads=c["num_attention_heads"],
            n_kv_heads=c.get("num_key_value_heads", c["num_attention_heads"]),
            ffn=c["intermediate_size"], max_positions=c.get("max_position_embeddings", 8192),
            norm_eps=c.get("rms_norm_eps", 1e-5),
            tie_embeddings=c.get("tie_word_embeddings", False),
            rope_theta=c.get("rope_theta", 10000.0),
            bos_token_id=c.get("bos_token_id", 1), eos_token_id=eos)
    raise ValueError(f"unsupported model_type {mt!r} in {path}")


# ---------------------------------------------------------------------------
# Sampling
# ---------------------------------------------------------------------------

@dataclass
class SamplingParams:
    """Per-request sampling.  Defaults reproduce `server.py:187-205`."""

    temperature: float = 0.6
    top_k: int = 40
    greedy: bool = False
    seed: Optional[int] = None
    max_new_tokens: int = 20
    stop_at_eos: bool = False  # reference never stops early (quirk Q10)

    def validate(self) -> None:
        if self.max_new_tokens < 0:
            raise ValueError("max_new_tokens must be >= 0")
        if not self.greedy:
            if self.temperature <= 0:
                raise ValueError("temperature must be > 0 (use greedy=True for argmax)")
            if not (1 <= self.top_k <= 1024):
                raise ValueError("top_k must be in [1, 1024]")


# ---------------------------------------------------------------------------
# Engine config
# ---------------------------------------------------------------------------

def _env(name: str, default: str) -> str:
    return os.environ.get(name, default)


@dataclass
class EngineConfig:
    model_id: str = "sshleifer/tiny-gpt2"
    # Pipeline: number of stages (= GPUs, one rank per GPU) and the layer split.
    num_stages: int = 1
    # Data parallelism over whole pipelines: world = num_stages x dp_replicas
    # ranks; replica r owns ranks [r*P, (r+1)*P).  Requests are spread over
    # the replicas (SURVEY.md §2.2 "DP -- request-level replicas").
    dp_replicas: int = 1
    # Explicit split points (len num_stages-1), e.g. SPLIT_AT=2 -> [2].  None = cost model.
    split_points: Optional[Sequence[int]] = None
    # Explicit split points in half-layer units: a stage starts at unit u, where
    # u = 2i is layer i's attention half and u = 2i + 1 its MLP half, e.g.
    # [13] cuts layer 6 between attention and MLP.
    split_units: Optional[Sequence[int]] = None
    # Auto partition may cut between a layer's attention and MLP halves
    # (finer balance of the last stage's lm_head + sampler).
    half_layer_split: bool = True
    dtype: str = "bf16"  # compute / storage dtype on GPU; CPU golden runs in fp32
    device: str = "auto"  # "auto" -> cuda if available else cpu
    max_batch: int = 64  # max concurrent sequences (KV slots)
    max_seq_len: int = 1024
    num_microbatches: int = 0  # 0 -> num_stages (1 when single stage)
    use_graphs: bool = True  # hipGraph-capture decode steps
    seed: int = 0
    weights: Optional[str] = None  # safetensors / HF dir; None -> random init
    sampling: SamplingParams = field(default_factory=SamplingParams)
    # Compat roles (reference server.py:21): "coordinator" | "a" | "b" | "engine".
    role: str = "coordinator"
    shard_a_service: str = "llm-shard-a"
    shard_b_service: str = "llm-shard-b"
    shard_port: int = 5000
    # auto | nccl | rccl | gloo | local | http | loopback (P stage threads on
    # one GPU, device-async event hand-off) | devloop (P stage threads on one
    # GPU joined by device loopback channels with graph-captured transfers:
    # the single-GPU rehearsal of the rccl data plane) | strict (host queues
    # per (edge, lane) with receive-size checks: CPU protocol tests)
    transport: str = "auto"
    # Boundary hidden states on the wire: "fp32" (the residual stream as is:
    # bit-identical to one stage) or "bf16" (half the bytes per hop; the
    # stream is rounded to bf16 at each stage boundary).  The reference ships
    # them as JSON floats (server.py:140,148).
    wire_dtype: str = "fp32"
    # Serving (runtime/scheduler.py): concurrent /generate requests arriving
    # within batch_window_ms share one pipeline round; a round running longer
    # than round_timeout_s marks the engine unhealthy; an HTTP request waits at
    # most request_timeout_s.
    batch_window_ms: float = 2.0
    # Chunked prefill: prompts are prefilled in steps of at most this many
    # tokens per sequence (0 = whole prompt in one step).  Bounds prefill
    # activation memory for long contexts and lets chunks of different
    # microbatches pipeline across stages.
    prefill_chunk: int = 0
    round_timeout_s: float = 600.0
    request_timeout_s: float = 900.0
    # Prefill tokens per microbatch group per step when requests join a
    # running batch (0 = unlimited: every waiting prompt joins at once).
    prefill_budget: int = 0
    # Join policy (runtime/sched_core.h set_join_policy): a running group
    # admits waiting requests only when it has room for all of them or for
    # join_min of them, when idle, or after deferring join_max_wait steps --
    # larger, rarer prefill items (1: admit whatever fits at every step).  Closed-loop serving, 512
    # in flight (profiles/r6_join_policy.log), 1 -> 32 / 4: GPT-2 XL 37.4-38.2k
    # -> 41.4k tok/s, GPT-2 small 156-164k -> 209k, Llama-3 8B 20.1k -> 21.6k,
    # TTFT p50 lower, p90 unchanged.
    join_min: int = 32
    join_max_wait: int = 4
    # One stage: a step's prefill items of groups that all only join
    # sequences run as one forward (parallel/pipeline.py _merged_prefill).
    # Off for references that must match a multi-stage pipeline bit for bit
    # (other GEMM row counts round differently).
    merge_prefill: bool = True
    # Fraction of the HBM left after the weights that the KV cache may use.
    kv_fraction: float = 0.85
    # Serving: record per-stage busy / bubble timing on one pipeline session
    # in this many (0 = never) -- it costs a control-plane gather per session.
    metrics_every: int = 16

    @property
    def model(self) -> ModelConfig:
        return get_model_config(self.model_id)

    @classmethod
    def from_env(cls, **overrides) -> "EngineConfig":
        """Build from the reference's env vars (server.py:20-25) plus extras."""
        split = _env("SPLIT_AT", "")
        cfg = cls(
            model_id=_env("MODEL_ID", "sshleifer/tiny-gpt2"),
            role=_env("SHARD_ROLE", "coordinator").lower(),
            split_points=[int(s) for s in split.split(",") if s.strip()] or None,
            shard_a_service=_env("SHARD_A_SERVICE", "llm-shard-a"),
            shard_b_service=_env("SHARD_B_SERVICE", "llm-shard-b"),
            shard_port=int(_env("SHARD_PORT", "5000")),
            num_stages=int(_env("NUM_STAGES", "0") or 0) or 1,
            max_batch=int(_env("MAX_BATCH", "64")),
            max_seq_len=int(_env("MAX_SEQ_LEN", "1024")),
            dtype=_env("DTYPE", "bf16"),
            weights=os.environ.get("WEIGHTS") or None,
            transport=_env("TRANSPORT", "auto"),
            wire_dtype=_env("WIRE_DTYPE", "fp32"),
            dp_replicas=int(_env("DP_REPLICAS", "1") or 1),
            batch_window_ms=float(_env("BATCH_WINDOW_MS", "2.0")),
            prefill_chunk=int(_env("PREFILL_CHUNK", "0")),
            round_timeout_s=float(_env("ROUND_TIMEOUT_S", "600")),
            request_timeout_s=float(_env("REQUEST_TIMEOUT_S", "900")),
            prefill_budget=int(_env("PREFILL_BUDGET", "0")),
            join_min=int(_env("JOIN_MIN", "32")),
            join_max_wait=int(_env("JOIN_MAX_WAIT", "4")),
            kv_fraction=float(_env("KV_FRACTION", "0.85")),
            metrics_every=int(_env("METRICS_EVERY", "16")),
        )
        if cfg.split_points and cfg.num_stages == 1:
            cfg.num_stages = len(cfg.split_points) + 1
        for k, v in overrides.items():
            if not hasattr(cfg, k):
                raise AttributeError(f"EngineConfig has no field {k!r}")
            setattr(cfg, k, v)
        return cfg

    def replace(self, **kw) -> "EngineConfig":
        return dataclasses.replace(self, **kw)

    @property
    def microbatches(self) -> int:
        return self.num_microbatches or self.num_stages
