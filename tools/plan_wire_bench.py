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

from llm_sharding_demo_amd.parallel.comm import GlooPlanChannel, ShmPlanChannel  # noqa: E402
from llm_sharding_demo_amd.runtime.plan import GroupPlan, StepPlan  # noqa: E402


def main():
    G = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    pg = dist.new_group(list(range(world)), backend="gloo")
    pg2 = dist.new_group(list(range(world)), backend="gloo")
    class T:  # the transport surface ShmPlanChannel uses
        P, R, grank, plan_pg = world, 1, rank, pg

        @staticmethod
        def broadcast_object(o, src=0):
            lst = [o]
            dist.broadcast_object_list(lst, src=src)
            return lst[0]

        @staticmethod
        def gather_object(o, dst=0):
            out = [None] * world if rank == dst else None
            dist.gather_object(o, out, dst=dst)
            return out

    for wire in ("pickle", "binary", "shm"):
        if wire == "shm":
            ch = ShmPlanChannel(T, 60.0)
        else:
            ch = GlooPlanChannel(pg, tag=1, plans=wire == "binary")
        dist.barrier()
        if rank == 0:
            t_send, b0 = 0.0, ch.bytes_sent
            for s in range(steps):
                # what the scheduler builds in steady state: fresh objects each step
                plan = StepPlan(step=s, groups=[GroupPlan(g, ret=256, n=256, b=256, ctxb=256)
                                                for g in range(G)])
                t0 = time.perf_counter()
                ch.send_many(list(range(1, world)), plan)
                t_send += time.perf_counter() - t0
                if s % 32 == 31:
                    ch.flush()  # keep rank 0 at most 32 steps ahead (the engine's readout lag)
                    dist.barrier(group=pg2)
            ch.send_many(list(range(1, world)), StepPlan(step=-1, stop=True))
            ch.flush()
            print(f"{wire:6s} G={G} world={world}: send {t_send / steps * 1e6:7.1f} us/step "
                  f"({(ch.bytes_sent - b0) / (steps + 1):.0f} B/step to {world - 1} followers)", flush=True)
        else:
            n = 0
            while True:
                p = ch.recv(0)
                if p.stop:
                    break
                n += 1
                if n % 32 == 0:
                    dist.barrier(group=pg2)
        dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
