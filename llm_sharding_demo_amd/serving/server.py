"""HTTP API -- wire-compatible with the reference FastAPI app.

Reference contract (`/root/reference/server.py:116-210`):
  POST /generate   {prompt, max_new_tokens=20}  -> {"generated": prompt + continuation}
  POST /forward    {input_ids: [int]}           -> {"hidden_states": [1][S][H]}   (shard A)
  POST /forward_b  {hidden_states: [B][S][H]}   -> {"logits": [B][S][V]}          (shard B)
  wrong role -> HTTP 200 {"error": "This instance is not shard A." | "...shard B." |
  "...coordinator."}  (kept for compat, quirk Q8)

Roles (env SHARD_ROLE, `server.py:21`):
  coordinator  /generate through the MI355X engine (local or torchrun pipeline);
               with TRANSPORT=http it instead drives remote a/b shards over
               HTTP exactly like the reference (compat / multi-node mode).
  a            stage 0 = embeddings + blocks[0:SPLIT_AT]          -> /forward
  b            blocks[SPLIT_AT:] + ln_f + lm_head                 -> /forward_b
  all          one process answers every endpoint (debug)
Additions: optional sampling fields on /generate (temperature, top_k, greedy,
seed, stop_at_eos; defaults = reference sampler), 422 on empty/over-long
prompts (instead of the reference's 500, quirk Q9), GET /health, GET /metrics
(Prometheus text).  Concurrent /generate calls are batched at decode-step
granularity by the engine's continuous-batching scheduler
(runtime/scheduler.py): a request joins the running batch at the next step
and leaves as soon as it has its tokens; a progress watchdog turns a hung
pipeline into 503s instead of hanging requests.
"""
from __future__ import annotations

import logging
import time
from typing import List, Optional

import torch
from pydantic import BaseModel

from ..config import EngineConfig, SamplingParams
from ..utils import racecheck
from ..utils.metrics import Metrics
from ..utils.tokenizer import load_tokenizer

log = logging.getLogger("llm_sharding_demo_amd.server")


# Wire schemas -- `server.py:116-124`, plus optional sampling fields.
class InputIDs(BaseModel):
    input_ids: List[int]


class HiddenStates(BaseModel):
    hidden_states: list  # nested lists (batch, seq, hidden_dim)


class GenerateReq(BaseModel):
    prompt: str
    max_new_tokens: int = 20
    temperature: float = 0.6
    top_k: int = 40
    greedy: bool = False
    seed: Optional[int] = None
    stop_at_eos: bool = False


class ShardRunner:
    """A single shard process (role a or b): one StageModel over a layer range."""

    def __init__(self, cfg: EngineConfig, role: str, device=None):
        from ..models.stage import StageModel
        from ..runtime.engine import _dtype, resolve_device

        mc = cfg.model
        split = (cfg.split_points or [1])[0]
        if not 0 <= split <= mc.n_layers:
            raise ValueError(f"SPLIT_AT={split} outside [0, {mc.n_layers}]")
        dev = resolve_device(device or cfg.device)
        a, b = (0, split) if role == "a" else (split, mc.n_layers)
        self.stage = StageModel(mc, a, b, first=(role == "a"), last=(role == "b"), device=dev,
                                dtype=_dtype(cfg.dtype, dev), seed=cfg.seed,
                                weights_path=cfg.weights, max_slots=1,
                                max_seq=min(cfg.max_seq_len, mc.max_positions))
        self.role = role
        self.lock = racecheck.Lock("shard_runner")

    def run(self, x: torch.Tensor, seq_len: int) -> torch.Tensor:
        from ..runtime.batch import BatchMeta

        st = self.stage
        if seq_len > st.max_seq:
            raise ValueError(f"sequence length {seq_len} exceeds {st.max_seq}")
        with self.lock:
            meta = BatchMeta.build([0], [0], [seq_len], st.device)
            out = st.forward(meta, x.to(st.device), all_logits=True)
        return out


def create_app(cfg: EngineConfig, engine=None, shard: Optional[ShardRunner] = None):
    from fastapi import FastAPI, HTTPException
    from fastapi.responses import PlainTextResponse

    role = cfg.role
    mc = cfg.model
    tok = load_tokenizer(cfg.model_id, mc.arch, cfg.weights, mc.eos_token_id)
    metrics = Metrics()
    app = FastAPI(title="llm-sharding-demo (MI355X)")
    app.state.engine, app.state.shard, app.state.metrics = engine, shard, metrics
    watchdog = None
    if engine is not None:
        from ..runtime.scheduler import Watchdog

        engine.start_loop()
        # dist engines run their own (every rank); local ones get one here
        watchdog = getattr(engine, "watchdog", None) or Watchdog(engine, cfg.round_timeout_s)
    app.state.watchdog = watchdog

    def _role_is(*roles):
        return role in roles or role == "all"

    @app.post("/forward")
    def forward_a(req: InputIDs):
        if not _role_is("a"):
            return {"error": "This instance is not shard A."}
        if not req.input_ids:
            raise HTTPException(422, "input_ids must be non-empty")
        ids = torch.tensor(req.input_ids, dtype=torch.int32)
        try:
            if shard is not None:
                h = shard.run(ids, len(req.input_ids))
            else:
                h = engine.forward_a(req.input_ids)
        except ValueError as e:
            raise HTTPException(422, str(e))
        except RuntimeError as e:  # e.g. a single-stage engine has no shard A / B split
            raise HTTPException(400, str(e))
        return {"hidden_states": h.float().cpu().unsqueeze(0).tolist()}

    @app.post("/forward_b")
    def forward_b(req: HiddenStates):
        if not _role_is("b"):
            return {"error": "This instance is not shard B."}
        hidden = torch.tensor(req.hidden_states, dtype=torch.float32)
        if hidden.dim() != 3 or hidden.shape[-1] != mc.hidden:
            raise HTTPException(422, f"hidden_states must be [B][S][{mc.hidden}]")
        B, S, H = hidden.shape
        outs = []
        try:
            for b in range(B):
                if shard is not None:
                    lg = shard.run(hidden[b], S)[:, : mc.vocab_size]
                else:
                    lg = engine.forward_b(hidden[b])
                outs.append(lg.float().cpu())
        except ValueError as e:
            raise HTTPException(422, str(e))
        except RuntimeError as e:
            raise HTTPException(400, str(e))
        return {"logits": torch.stack(outs).tolist()}

    @app.post("/generate")
    def generate(req: GenerateReq):
        if not _role_is("coordinator"):
            return {"error": "This instance is not coordinator."}
        ids = tok.encode(req.prompt)
        sp = SamplingParams(temperature=req.temperature, top_k=req.top_k, greedy=req.greedy,
                            seed=req.seed, max_new_tokens=req.max_new_tokens,
                            stop_at_eos=req.stop_at_eos)
        if req.max_new_tokens == 0:
            return {"generated": tok.decode(ids, skip_special_tokens=True)}
        if not ids:
            raise HTTPException(422, "prompt must encode to at least one token")
        t0 = time.perf_counter()
        from ..runtime.scheduler import RequestTimeout

        try:
            sp.validate()
            if engine is not None:
                if len(ids) + sp.max_new_tokens > engine.max_seq:
                    raise ValueError(f"prompt ({len(ids)}) + max_new_tokens ({sp.max_new_tokens}) "
                                     f"exceeds the context limit {engine.max_seq}")
                req_ = engine.submit(ids, sp)
                out = req_.wait(timeout=cfg.request_timeout_s)
                metrics.observe_request(len(out), time.perf_counter() - t0,
                                        ttft_s=(req_.t_first - req_.t_submit) if req_.t_first else None)
            else:
                out = http_generate(cfg, ids, sp)
                metrics.observe_request(len(out), time.perf_counter() - t0)
        except ValueError as e:
            raise HTTPException(422, str(e))
        except RequestTimeout as e:
            raise HTTPException(504, str(e))
        except RuntimeError as e:
            if engine is not None and not engine.healthy:
                raise HTTPException(503, f"engine unhealthy: {engine.last_error}")
            raise
        return {"generated": tok.decode(ids + out, skip_special_tokens=True)}

    @app.get("/health")
    def health():
        ok = engine.healthy if engine is not None else True
        body = {"status": "ok" if ok else "unhealthy", "role": role, "model": mc.name}
        if engine is not None:
            body.update(stages=engine.P, plan=engine.plan, unit_plan=engine.unit_plan, mode=engine.mode,
                        devices=[str(d) for d in engine.devices], **engine.kv_info())
            if not ok:
                body["error"] = engine.last_error
        if shard is not None:
            body.update(layers=[shard.stage.layer_start, shard.stage.layer_end],
                        device=str(shard.stage.device))
        return body

    @app.get("/metrics", response_class=PlainTextResponse)
    def prom():
        gauges, counters = {}, {}
        if engine is not None:
            sch = engine.scheduler
            kv = engine.kv_info()
            gauges = {"engine_healthy": 1 if engine.healthy else 0,
                      "engine_stages": engine.P,
                      "kv_slots_free": kv["kv_slots_free"],
                      "kv_slots_total": kv["kv_slots"] * engine.R,
                      "kv_cache_bytes_stage0": kv["kv_bytes_stage0"],
                      "queue_depth": sch.queue_depth,
                      "max_batch_rows_seen": sch.stats["max_rows"]}
            counters = {"pipeline_steps_total": sch.stats["steps"],
                        "sequence_joins_total": sch.stats["joins"],
                        "sequence_leaves_total": sch.stats["leaves"],
                        "hipgraph_captures_total": sum(w.captures for w in engine.workers)}
            ls = engine.last_session
            if ls is not None:
                if ls.step_times_ms:
                    metrics.observe_steps(ls.step_times_ms, key=id(ls))
                for st in ls.stages:
                    tag = f"stage{st['stage']}" + (f"_replica{st['replica']}" if st.get("replica") else "")
                    gauges[f"{tag}_busy_fraction"] = st["busy_fraction"]
                    gauges[f"{tag}_bubble_fraction"] = 1.0 - st["busy_fraction"]
        return metrics.render(gauges, counters)

    return app


def http_generate(cfg: EngineConfig, ids: List[int], sp: SamplingParams) -> List[int]:
    """Reference-style coordinator loop over remote shards (`server.py:169-206`):
    full-sequence recompute on every step, hidden states relayed through here.
    Kept for deployments where the shards are separate hosts without xGMI."""
    import requests

    from ..ops import reference as ref
    from ..runtime.batch import counter_uniform

    seed = sp.seed if sp.seed is not None else int.from_bytes(__import__("os").urandom(7), "little")
    vocab = cfg.model.vocab_size
    out: List[int] = []
    seq = list(ids)
    url_a = f"http://{cfg.shard_a_service}:{cfg.shard_port}/forward"
    url_b = f"http://{cfg.shard_b_service}:{cfg.shard_port}/forward_b"
    for step in range(sp.max_new_tokens):
        r = requests.post(url_a, json={"input_ids": seq}, timeout=30)
        r.raise_for_status()
        hidden = r.json()["hidden_states"]
        r2 = requests.post(url_b, json={"hidden_states": hidden}, timeout=30)
        r2.raise_for_status()
        logits = torch.tensor(r2.json()["logits"], dtype=torch.float32)[0, -1:]
        u = counter_uniform(torch.tensor([seed]), torch.tensor([step]))
        nxt = int(ref.sample(logits, torch.tensor([sp.temperature]), torch.tensor([sp.top_k]),
                             torch.tensor([1 if sp.greedy else 0]), u, vocab)[0])
        seq.append(nxt)
        out.append(nxt)
    return out
