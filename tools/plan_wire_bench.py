"""Control-plane microbenchmark (verdict r3 item 5): rank 0 posts one step
plan per follower per step over the gloo plan channel, as Engine._send_plans
does; followers receive and decode.  No model: the cost isolated is encoding
+ posting on rank 0 (and decoding on the followers), per step, for
steady-state decode plans of G groups -- binary records vs pickled StepPlans.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \
        tools/plan_wire_bench.py [groups] [steps]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch.distributed as dist  # noqa: E402

from llm_sharding_demo_amd.parallel.comm import GlooPlanChannel  # noqa: E402
from llm_sharding_demo_amd.runtime.plan import GroupPlan, StepPlan  # noqa: E402


def main():
    G = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    pg = dist.new_group(list(range(world)), backend="gloo")
    for wire in ("pickle", "binary"):
        ch = GlooPlanChannel(pg, tag=1, plans=True) if wire == "binary" else GlooPlanChannel(pg, tag=1, plans=False)
        dist.barrier()
        if rank == 0:
            t_send, b0 = 0.0, ch.bytes_sent
            for s in range(steps):
                # what the scheduler builds in steady state: fresh objects each step
                plan = StepPlan(step=s, groups=[GroupPlan(g, ret=256, n=256, b=256, ctxb=256)
                                                for g in range(G)])
                t0 = time.perf_counter()
                for r in range(1, world):
                    ch.send(r, plan)
                t_send += time.perf_counter() - t0
                if s % 64 == 63:
                    ch.flush()  # keep rank 0 at most 64 steps ahead (the engine's readout lag)
            ch.send_stop = None
            for r in range(1, world):
                ch.send(r, StepPlan(step=-1, stop=True))
            ch.flush()
            print(f"{wire:6s} G={G} world={world}: send {t_send / steps * 1e6:7.1f} us/step "
                  f"({(ch.bytes_sent - b0) / (steps + 1):.0f} B/step to {world - 1} followers)", flush=True)
        else:
            t_dec, n = 0.0, 0
            while True:
                t0 = time.perf_counter()
                p = ch.recv(0)
                t_dec += time.perf_counter() - t0
                n += 1
                if p.stop:
                    break
        dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
