"""Multi-process engine on the GPU: 2 torchrun ranks (one pipeline stage
each) on the box's GPU, linked by the gloo transport (device tensors staged
through host memory).  Exercises the whole dist path -- process groups,
control-plane broadcast, per-rank stages, token return edge -- with the HIP
kernels; only the RCCL byte-mover itself is substituted (RCCL refuses two
ranks on one GPU)."""
import json
import os
import socket
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("dp", [1, 2])
def test_two_rank_pipeline_matches_single_gpu(tmp_path, dp):
    """dp=1: one 2-stage pipeline; dp=2: two 1-stage replicas sharing the requests."""
    prompts = [[1, 2, 3, 4], [5, 6], list(range(10, 40)), [7] * 9]
    script = tmp_path / "w.py"
    script.write_text(textwrap.dedent(f"""
        import sys, json
        sys.path.insert(0, {ROOT!r})
        from llm_sharding_demo_amd.config import EngineConfig, SamplingParams
        from llm_sharding_demo_amd.runtime.engine import build_engine
        cfg = EngineConfig(model_id="gpt2-test", max_batch=8, device="cuda", transport="gloo",
                           num_microbatches=2, max_seq_len=128, dp_replicas={dp})
        eng = build_engine(cfg)
        if eng.rank != 0:
            eng.worker_loop()
        else:
            sp = SamplingParams(temperature=0.8, top_k=20, seed=5, max_new_tokens=10)
            out = eng.generate_ids({prompts!r}, sp)
            eng.shutdown()
            print("RESULT", json.dumps(out))
    """))
    port = _port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}", str(script)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-4000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("RESULT")][0]
    dist_out = json.loads(line[len("RESULT "):])

    from llm_sharding_demo_amd.config import EngineConfig, SamplingParams
    from llm_sharding_demo_amd.runtime.engine import Engine

    one = Engine(EngineConfig(model_id="gpt2-test", num_stages=1, max_batch=8, device="cuda",
                              max_seq_len=128, merge_prefill=False))
    ref = one.generate_ids(prompts, SamplingParams(temperature=0.8, top_k=20, seed=5,
                                                   max_new_tokens=10))
    assert dist_out == ref
