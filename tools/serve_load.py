"""Closed-loop serving load on one engine: C requests in flight, each finished
request replaced by a new one, varied prompt and output lengths -- sequences
join and leave at every step (continuous batching), unlike bench.py's session
where the whole batch joins at step 0 and leaves together.  Prints one JSON
line: output tok/s, per-token latency and TTFT percentiles, steps and how many
items the native executor issued (steady / composition changes).

  python tools/serve_load.py --model gpt2-xl --concurrency 512 --requests 2048
"""
import argparse
import json
import os
import random
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from llm_sharding_demo_amd.config import EngineConfig, SamplingParams  # noqa: E402
from llm_sharding_demo_amd.runtime.engine import Engine, freeze_gc  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--model", default="gpt2-xl")
    p.add_argument("--concurrency", type=int, default=512)
    p.add_argument("--requests", type=int, default=2048)
    p.add_argument("--prompt", default="16,128", help="min,max prompt tokens")
    p.add_argument("--gen", default="16,128", help="min,max new tokens")
    p.add_argument("--microbatches", type=int, default=2)
    p.add_argument("--device", default="cuda")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--join-min", type=int, default=32, help="EngineConfig.join_min (join policy)")
    p.add_argument("--join-wait", type=int, default=4, help="EngineConfig.join_max_wait")
    p.add_argument("--warm-requests", type=int, default=0,
                   help="an unmeasured closed-loop phase of this many requests first (serving-shaped "
                        "graphs captured before the clock starts)")
    a = p.parse_args()
    pl, ph = map(int, a.prompt.split(","))
    gl, gh = map(int, a.gen.split(","))
    C = a.concurrency
    cfg = EngineConfig(model_id=a.model, num_stages=1, max_batch=C, max_seq_len=ph + gh,
                       num_microbatches=a.microbatches, device=a.device, seed=a.seed,
                       metrics_every=1, join_min=a.join_min, join_max_wait=a.join_wait)  # per-stage busy fraction of the serving session
    eng = Engine(cfg)
    rnd = random.Random(a.seed)
    V = eng.mcfg.vocab_size

    def make():
        n = rnd.randint(pl, ph)
        return ([rnd.randrange(V) for _ in range(n)],
                SamplingParams(temperature=0.6, top_k=40, max_new_tokens=rnd.randint(gl, gh),
                               seed=rnd.randrange(1 << 30)))

    # warm-up: every bucket / context graph the run can meet is captured once
    warm = [make() for _ in range(C)]
    eng.generate_ids([w[0] for w in warm], [w[1] for w in warm])
    freeze_gc()
    if getattr(eng, "_hostprof", None) is not None:
        eng._hostprof[:] = [0.0] * len(eng._hostprof)
    eng.start_loop()

    def closed_loop(n):
        live = [eng.submit(*make()) for _ in range(min(C, n))]
        sent, done = len(live), []
        while live:
            keep = []
            for r in live:
                if r.done:
                    done.append(r)
                    if sent < n:
                        keep.append(eng.submit(*make()))
                        sent += 1
                else:
                    keep.append(r)
            live = keep
            time.sleep(0.0005)
        return done

    if a.warm_requests:
        closed_loop(a.warm_requests)
    st0 = eng.scheduler.stats["steps"]
    n0 = sum(w.native_steps for w in eng.workers), sum(w.native_changes for w in eng.workers)
    t0 = time.monotonic()
    done = closed_loop(a.requests)
    el = time.monotonic() - t0
    eng.stop_loop()
    toks = sum(len(r.output) for r in done)
    tpot = [(r.t_done - r.t_first) / (len(r.output) - 1) * 1e3 for r in done if len(r.output) > 1]
    ttft = sorted((r.t_first - r.t_submit) * 1e3 for r in done)
    q = lambda v, f: v[min(len(v) - 1, int(f * len(v)))]  # noqa: E731
    print(json.dumps({
        "model": a.model, "concurrency": C, "requests": len(done), "prompt": a.prompt, "gen": a.gen,
        "tok_s": round(toks / el, 1), "elapsed_s": round(el, 3),
        "per_token_ms_p50": round(statistics.median(tpot), 3), "ttft_ms_p50": round(q(ttft, 0.5), 2),
        "ttft_ms_p90": round(q(ttft, 0.9), 2), "steps": eng.scheduler.stats["steps"] - st0,
        "native_steps": sum(w.native_steps for w in eng.workers) - n0[0],
        "native_changes": sum(w.native_changes for w in eng.workers) - n0[1],
        "native_changes_env": os.environ.get("LSD_NATIVE_CHANGES", "1"),
        "join_min": a.join_min, "join_wait": a.join_wait, "deferred_joins": eng.scheduler.stats.get("deferred"),
        "stage0_busy": (eng.last_session.stages[0]["busy_fraction"] if eng.last_session is not None
                        and eng.last_session.stages else None)}), flush=True)
    hp = getattr(eng, "_hostprof", None)
    if hp is not None and hp[3]:
        print(f"host per decode-only step: plan {hp[0] / hp[3] * 1e6:.1f} us, issue {hp[1] / hp[3] * 1e6:.1f} us, "
              f"readout wait {hp[2] / hp[3] * 1e6:.1f} us over {hp[3]} steps", flush=True)
    if hp is not None and hp[10]:
        print(f"host per step with prefill chunks: issue {hp[8] / hp[10] * 1e6:.1f} us, readout wait "
              f"{hp[9] / hp[10] * 1e6:.1f} us over {hp[10]} steps", flush=True)
    eng.shutdown()


if __name__ == "__main__":
    main()
