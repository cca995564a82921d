"""Command line: `python -m llm_sharding_demo_amd {serve,generate}`.

The reference's only entry point is `uvicorn server:app` with the role picked
by env vars (`Dockerfile:19`, `server.py:20-25`).  `serve` does the same (env
vars are honoured; flags override), and also runs under torchrun for the
multi-GPU pipeline: rank 0 serves HTTP, the other ranks are stage workers.
"""
from __future__ import annotations

import argparse
import logging
import os
import sys

from .config import EngineConfig


def _cfg(args) -> EngineConfig:
    over = {}
    for k in ("model_id", "num_stages", "max_batch", "max_seq_len", "device", "dtype",
              "weights", "transport", "role", "num_microbatches"):
        v = getattr(args, k, None)
        if v is not None:
            over[k] = v
    if getattr(args, "split_at", None):
        over["split_points"] = [int(s) for s in args.split_at.split(",")]
    if getattr(args, "no_graphs", False):
        over["use_graphs"] = False
    cfg = EngineConfig.from_env(**over)
    if "split_points" in over and "num_stages" not in over and cfg.role not in ("a", "b"):
        cfg.num_stages = len(cfg.split_points) + 1
    return cfg


def main(argv=None) -> int:
    p = argparse.ArgumentParser(prog="llm_sharding_demo_amd")
    sub = p.add_subparsers(dest="cmd", required=True)
    for name in ("serve", "generate"):
        s = sub.add_parser(name)
        s.add_argument("--model-id", dest="model_id")
        s.add_argument("--num-stages", dest="num_stages", type=int)
        s.add_argument("--split-at", dest="split_at")
        s.add_argument("--max-batch", dest="max_batch", type=int)
        s.add_argument("--max-seq-len", dest="max_seq_len", type=int)
        s.add_argument("--microbatches", dest="num_microbatches", type=int)
        s.add_argument("--device")
        s.add_argument("--dtype")
        s.add_argument("--weights")
        s.add_argument("--transport")
        s.add_argument("--no-graphs", action="store_true")
    sub.choices["serve"].add_argument("--role")
    sub.choices["serve"].add_argument("--host", default="0.0.0.0")
    sub.choices["serve"].add_argument("--port", type=int,
                                      default=int(os.environ.get("PORT", os.environ.get("SHARD_PORT", "5000"))))
    g = sub.choices["generate"]
    g.add_argument("prompt")
    g.add_argument("--max-new-tokens", type=int, default=20)
    g.add_argument("--greedy", action="store_true")
    g.add_argument("--temperature", type=float, default=0.6)
    g.add_argument("--top-k", type=int, default=40)
    g.add_argument("--seed", type=int)
    args = p.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(name)s %(levelname)s %(message)s")
    cfg = _cfg(args)
    log = logging.getLogger("llm_sharding_demo_amd")

    if args.cmd == "generate":
        from . import LLM

        llm = LLM(cfg)
        if llm.engine.mode == "dist" and llm.engine.rank != 0:
            llm.engine.worker_loop()
            return 0
        out = llm.generate_text(args.prompt, args.max_new_tokens, greedy=args.greedy,
                                temperature=args.temperature, top_k=args.top_k, seed=args.seed)
        print(out)
        llm.engine.shutdown()
        return 0

    import uvicorn

    from .serving.server import ShardRunner, create_app

    log.info("Starting server role: %s model: %s", cfg.role, cfg.model_id)  # server.py:27
    if cfg.role in ("a", "b"):
        app = create_app(cfg, shard=ShardRunner(cfg, cfg.role))
    elif cfg.transport == "http":  # reference-style coordinator over remote shards
        app = create_app(cfg)
    else:
        from .runtime.engine import build_engine, freeze_gc

        engine = build_engine(cfg)
        freeze_gc()
        if engine.mode == "dist" and engine.rank != 0:
            engine.worker_loop()
            return 0
        app = create_app(cfg, engine=engine if cfg.transport != "http" else None)
    uvicorn.run(app, host=args.host, port=args.port, log_level="info")
    return 0


if __name__ == "__main__":
    sys.exit(main())
