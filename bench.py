#!/usr/bin/env python3
"""Headline benchmark: output tokens/s + p50 per-token latency of the GPT-2
pipeline at N stages = N MI355X (BASELINE.json "metric").

One step = one complete generation round, end to end: prefill of every
prompt, then `--gen` decode steps, for a global batch of N x --batch
sequences split into 2N microbatches that flow through the N-stage pipeline
(one stage per GPU, RCCL p2p between stages; each stage keeps two
microbatches in flight on two HIP streams).  `--dp R` instead runs R
replicas of an N/R-stage pipeline (hybrid PP x DP).  Weak scaling: each GPU holds
1/N of the layers and the global batch grows with N.  Nothing is skipped in
the timed region: prefill, every layer, lm_head and the sampler (reference
sampler: T=0.6, top-k=40; --greedy for argmax) run for every token.

Data: synthetic random prompts, random-init weights of the named architecture
(no network in this environment).

Usage:  python bench.py [--gpus N --steps K --warmup W]
        python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import random
import statistics
import sys
import time

# Reference measurements (reference server.py path on CPU): tok/s
REFERENCE_TOK_S = {"gpt2": 0.69, "tiny-gpt2": 0.69, "gpt2-xl": 0.42}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--model", default="gpt2-xl")
    p.add_argument("--batch", type=int, default=int(os.environ.get("BENCH_BATCH", "512")),
                   help="sequences per GPU")
    p.add_argument("--prompt", type=int, default=128)
    p.add_argument("--gen", type=int, default=128)
    p.add_argument("--microbatches", type=int, default=int(os.environ.get("BENCH_MB", "0")),
                   help="0 -> auto: 2 groups per stage when decode reads more KV than weights "
                        "(two lanes overlap one group's attention with the other's GEMMs), "
                        "else 1 (weights read once per step)")
    p.add_argument("--dp", type=int, default=int(os.environ.get("BENCH_DP", "1")),
                   help="pipeline replicas: N GPUs = (N/dp)-stage pipeline x dp (default 1: ppN)")
    p.add_argument("--transport", default=os.environ.get("BENCH_TRANSPORT", "auto"),
                   help="auto (default: on GPUs the native RCCL communicators with graph-captured edges, "
                        "self-tested at startup, falling back in process to torch's RCCL groups; ranks "
                        "sharing one GPU: devloop, then gloo) | rccl | nccl (RCCL via torch.distributed) | "
                        "gloo (host-staged, for rehearsals) | devloop (every rank on ONE GPU: device loopback "
                        "channels between the rank processes, the rccl code path's rehearsal) | a,b (an "
                        "explicit chain: a, falling back to b)")
    p.add_argument("--loopback-stages", type=int, default=0,
                   help="rehearsal: run this many pipeline stages as threads on ONE GPU; "
                        "--batch is then the total batch")
    p.add_argument("--loopback-transport", default=os.environ.get("BENCH_LOOPBACK", "devloop"),
                   help="devloop (device loopback channels: graph-captured transfers + the native "
                        "executor, the rccl data plane's code path) | loopback (event hand-off)")
    p.add_argument("--prefill-chunk", type=int, default=int(os.environ.get("BENCH_PREFILL_CHUNK", "-1")),
                   help="prompt tokens per prefill chunk (0: whole prompts); -1 -> auto: whole prompts on "
                        "one stage, prompt/4 (>= 32) on P >= 2 stages.  Chunks shorten the pipeline fill "
                        "(the last stage idles (P-1) x one group's prefill time per session) and cost "
                        "nothing measurable on one stage or in the 2/4-stage loopback rehearsal "
                        "(profiles/r2_prefill_chunk.log)")
    p.add_argument("--device", default="cuda",
                   help="cuda (MI355X); cpu only to rehearse the multi-rank contract with gloo")
    p.add_argument("--greedy", action="store_true")
    p.add_argument("--no-graphs", action="store_true")
    p.add_argument("--seed", type=int, default=0)
    return p.parse_args()


def auto_groups(args, P: int) -> int:
    """Microbatch groups per replica: 2 per stage when a decode step reads more
    KV cache than weights AND the attention runs on the VALU decode kernel
    (GPT-2 XL at 512 x 192 positions: 629 vs 61 MB per layer -- the two lanes
    overlap one group's attention with the other's GEMMs: 46.5k vs 44.9k
    tok/s), otherwise 1 per stage so the weights are read once per step
    (Llama-3 8B, 256 sequences: 201 vs 436 MB per layer, 21.4k vs 18.9k tok/s;
    profiles/r2_llama_microbatches.log).  Grouped-query attention on MFMA
    (head_dim 128, 2-8 query heads per kv head) streams the KV at the HBM
    roofline, so there is nothing to overlap: Llama-3 8B at 32 x 4K positions
    (545 vs 436 MB per layer) 1405 vs 1272 tok/s on 1 group
    (profiles/r2_long_context.log)."""
    from llm_sharding_demo_amd.config import get_model_config

    mc = get_model_config(args.model)
    if mc.head_dim == 128 and mc.n_heads // mc.n_kv_heads in (2, 4, 8):
        return P
    ctx = args.prompt + args.gen // 2
    kv = P * args.batch * ctx * mc.kv_bytes_per_token_per_layer()
    weights = 2 * mc.block_params()
    return 2 * P if kv > weights else P


def main() -> int:
    args = parse()
    import torch

    from llm_sharding_demo_amd.config import EngineConfig, SamplingParams
    from llm_sharding_demo_amd.runtime.engine import Engine, freeze_gc

    N = args.gpus
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != N:
        raise SystemExit(f"--gpus {N} but WORLD_SIZE={world}: launch N>1 with torch.distributed.run")
    R = args.dp
    if N % R:
        raise SystemExit(f"--gpus {N} is not a multiple of --dp {R}")
    P = N // R                      # pipeline stages per replica
    M = args.microbatches or auto_groups(args, P)  # microbatch groups per replica
    B = N * args.batch              # global batch (weak scaling: fixed per GPU)
    Br = P * args.batch             # sequences per replica
    transport = args.transport
    if args.loopback_stages:
        if N != 1:
            raise SystemExit("--loopback-stages runs on one GPU")
        P = args.loopback_stages
        M = args.microbatches or auto_groups(args, P)
        transport = args.loopback_transport
    chunk = args.prefill_chunk
    if chunk < 0:
        chunk = 0 if P == 1 else max(32, args.prompt // 4)
        chunk = 0 if chunk >= args.prompt else chunk
    cfg = EngineConfig(model_id=args.model, num_stages=P, dp_replicas=R, max_batch=Br,
                       prefill_chunk=chunk,
                       max_seq_len=args.prompt + args.gen, device=args.device,
                       use_graphs=not args.no_graphs, num_microbatches=M, seed=args.seed,
                       transport=transport)
    eng = Engine(cfg, mode="dist" if N > 1 else "local")
    rank = eng.rank

    vocab = cfg.model.vocab_size
    sp = SamplingParams(greedy=args.greedy, temperature=0.6, top_k=40,
                        max_new_tokens=args.gen, seed=1234)
    rnd = random.Random(args.seed)
    prompts = [[rnd.randrange(vocab) for _ in range(args.prompt)] for _ in range(B)]

    def barrier():
        if N > 1:
            eng.transport.barrier()

    def sync():
        if args.device != "cpu":
            torch.cuda.synchronize()

    last_out = [None]

    def session(timing: bool):
        """One bench step = one generation session of the whole global batch:
        every sequence joins at step 0 (prefill), decodes, and leaves."""
        if rank == 0:
            last_out[0] = eng.generate_ids(prompts, [sp] * B, record_timing=timing)
        else:
            eng.follow_session()

    for _ in range(args.warmup):
        session(False)
    if os.environ.get("BENCH_GC_FREEZE", "1") == "1":
        freeze_gc()  # as the server does after start-up (engine.freeze_gc)
    sync()
    barrier()
    sync()
    if getattr(eng, "_phases", None):
        eng._phases.clear()
        eng._hostprof[:] = [0.0] * len(eng._hostprof)
    t0 = time.perf_counter()
    step_ms, prefill_ms, max_step, decode_sum = [], [], [], []
    for _ in range(args.steps):
        session(True)
        if rank == 0 and eng.last_session is not None:
            ls = eng.last_session
            step_ms += ls.step_times_ms
            prefill_ms.append(ls.prefill_ms)
            max_step.append(max(ls.step_times_ms, default=0.0))
            decode_sum.append(sum(ls.step_times_ms))
    sync()
    barrier()
    sync()
    elapsed = time.perf_counter() - t0
    ranks = None
    if N > 1:
        import torch.distributed as dist

        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=eng.transport.ctrl)
        elapsed = float(t[0])
        # data-plane evidence from every rank: what the process group and the
        # transport saw (world size, device, communicators this rank joined)
        me = {"rank": eng.rank, "replica": eng.replica, "stage": eng.stage_idx,
              "device": str(eng.devices[0]), "pg_world": dist.get_world_size(),
              "comms": eng.transport.num_comms}
        ranks = eng.transport.gather_object(me, dst=0)
    if rank == 0:
        ms_per_step = elapsed * 1e3 / args.steps
        tokens = B * args.gen * args.steps
        value = tokens / elapsed
        p50 = statistics.median(step_ms) if step_ms else None
        base = REFERENCE_TOK_S.get(args.model)
        out = {
            "metric": "output tokens/sec + p50 per-token latency, "
                      + ("GPT-2" if args.model.startswith(("gpt2", "tiny-gpt2")) else args.model)
                      + " pipeline at N MI355X",
            "value": round(value, 2), "unit": "tokens/s", "n_gpus": N, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": round(value / base, 1) if base else None,
            "vs_baseline_note": "vs the reference's own CPU fp32 HTTP code path (survey-measured, "
                                "BASELINE.md); the reference publishes no number: not a like-for-like speedup",
            "dtype": "bf16" if args.device != "cpu" else "fp32",
            "data": "synthetic prompts, random-init weights",
            "p50_token_latency_ms": round(p50, 4) if p50 is not None else None,
            # stage-0 clock, mean per timed step: prefill (TTFT of the batch)
            # and the slowest decode step (graphs are cached across sessions)
            "prefill_ms": round(statistics.mean(prefill_ms), 3) if prefill_ms else None,
            "max_decode_step_ms": round(statistics.mean(max_step), 3) if max_step else None,
            # the rest of a step on the host clock: session setup / drain and the
            # last decode step (the stage-0 events time the steps between starts)
            "session_other_ms": (round(ms_per_step - statistics.mean(prefill_ms) - statistics.mean(decode_sum), 3)
                                 if prefill_ms and decode_sum else None),
            "config": {"model": args.model, "global_batch": B, "seq_len": args.prompt + args.gen,
                       "prompt_len": args.prompt, "gen_tokens": args.gen, "microbatches": M,
                       "prefill_chunk": chunk,
                       "parallelism": f"pp{P}" + (f"xdp{R}" if R > 1 else "")
                       + ("-loopback-1gpu" if args.loopback_stages else "")
                       + ("-ranks-on-1gpu" if eng.transport_kind == "devloop" and N > 1 else ""),
                       "sampler": "greedy" if args.greedy else "T0.6/top-k40",
                       "hipgraphs": not args.no_graphs},
        }
        C = getattr(getattr(eng.stages[0], "backend", None), "C", None) if eng.stages else None
        if C is not None and hasattr(C, "gemm_slab_bf16"):
            # precision of the residual projections' split-K partials (bf16 = one
            # rounding per partial before the fp32 residual add; LSD_SLAB_BF16=0: fp32)
            out["split_k_slabs"] = "bf16" if C.gemm_slab_bf16() else "fp32"
        if (args.loopback_stages or N > 1) and eng.last_session is not None:
            out["stage_busy"] = [st["busy_fraction"] for st in eng.last_session.stages]
        if args.loopback_stages:
            out["transport"] = transport
        if N > 1:
            # the data plane that ran, and why the preferred one was left (or null)
            out["transport"] = eng.transport_kind
            out["transport_fallback"] = eng.transport_fallback
        if ranks is not None:
            out["pg_world_size"] = ranks[0]["pg_world"]
            out["data_plane_comms"] = sum(r["comms"] for r in ranks)
            out["rank_devices"] = [r["device"] for r in ranks]
        rc = 0
        if N > 1 and os.environ.get("BENCH_CHECK", "1") != "0":
            # outside the timed region: the pipeline's tokens of the last timed
            # session against a 1-stage engine on this rank's own GPU
            chk = check_against_one_gpu(cfg, eng, prompts, sp, last_out[0])
            out.update(chk)
            if not chk["pipeline_matches_1gpu"]:
                rc = 3
        print(json.dumps(out), flush=True)
        hp = getattr(eng, "_hostprof", None)
        if hp is not None and hp[3]:
            print(f"host per decode step: plan {hp[0] / hp[3] * 1e6:.1f} us (of which plan send "
              f"{hp[6] / hp[3] * 1e6:.1f} us, {hp[7] / hp[3]:.0f} B), issue {hp[1] / hp[3] * 1e6:.1f} us "
                  f"({hp[1] / max(hp[4], 1) * 1e6:.1f} us per item; issuing-thread CPU "
                  f"{hp[5] / max(hp[4], 1) * 1e6:.1f} us per item), readout wait "
                  f"{hp[2] / hp[3] * 1e6:.1f} us over {hp[3]} steps", file=sys.stderr)
            print("host per session (ms): " + ", ".join(f"{k} {v * 1e3 / args.steps:.2f}"
                                                        for k, v in eng._phases.items()), file=sys.stderr)
    if N > 1:
        if rank == 0:
            eng.shutdown()  # stop the followers, barrier, tear the groups down in order
        else:
            eng.worker_loop()
    return rc if rank == 0 else 0


def check_against_one_gpu(cfg, eng, prompts, sp, got) -> dict:
    """Token-for-token check of a multi-rank run (rank 0, after the timed
    region): the first BENCH_CHECK_SEQS (default 512) sequences of replica 0
    -- whole microbatch groups, in the scheduler's admission order -- are
    generated again by a 1-stage engine on rank 0's own device with the same
    weights (seeded per layer), group rows, prefill chunking and sampling
    (seeded counter-based draws keyed by (seed, step), not by slot or rank).
    The same GEMM shapes per group and an fp32 residual on the wire make the
    pipeline bit-identical to one stage, so any difference is a data-plane
    fault.  This replaces the reference's relay (`/root/reference/server.py:171-181`),
    which nothing checks either."""
    import dataclasses

    from llm_sharding_demo_amd.runtime.engine import Engine

    rows = eng.group_cap
    want_seqs = int(os.environ.get("BENCH_CHECK_SEQS", "512"))
    groups = max(1, min(eng.M, want_seqs // rows))
    n = min(groups * rows, len(prompts), len(got))
    t0 = time.perf_counter()
    # merge_prefill off: the pipeline prefills each group separately, and a
    # merged prefill's GEMMs (other row counts) would round differently
    ref_cfg = dataclasses.replace(cfg, num_stages=1, dp_replicas=1, max_batch=groups * rows,
                                  num_microbatches=groups, transport="auto",
                                  device=str(eng.devices[0]), merge_prefill=False)
    ref = Engine(ref_cfg, mode="local")
    try:
        want = ref.generate_ids(prompts[:n], [sp] * n)
    finally:
        ref.shutdown()
    bad = [i for i in range(n) if want[i] != got[i]]
    res = {"pipeline_matches_1gpu": not bad, "check_seqs": n, "check_groups": groups,
           "check_s": round(time.perf_counter() - t0, 2)}
    if bad:
        res["check_mismatched_seqs"] = len(bad)
        print(f"pipeline/1-GPU token mismatch in {len(bad)} of {n} sequences (first: {bad[0]})",
              file=sys.stderr, flush=True)
    del ref
    return res


if __name__ == "__main__":
    try:
        rc = main()
    except BaseException:  # noqa: BLE001
        # a failed run may leave stage threads parked in native code (a
        # data-plane wait, a stream synchronize); interpreter finalization
        # would then abort the process -- report and leave without it
        import traceback

        traceback.print_exc()
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(1)
    sys.exit(rc)
