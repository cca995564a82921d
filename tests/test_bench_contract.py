"""bench.py driver contract, rehearsed on CPU: one JSON line from rank 0 with
the required fields, N>1 under torch.distributed.run (gloo), incl. PP x DP."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
        "scaling", "vs_baseline", "dtype", "data", "config"}


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("n,dp", [(1, 1), (2, 1), (4, 2), (8, 1)])
def test_bench_json_contract(n, dp):
    args = ["--gpus", str(n), "--dp", str(dp), "--device", "cpu", "--transport", "gloo",
            "--model", "gpt2-test", "--batch", "2", "--prompt", "4", "--gen", "3",
            "--steps", "2", "--warmup", "1"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    if n == 1:
        cmd = [sys.executable, os.path.join(ROOT, "bench.py")] + args
    else:
        port = str(_port())
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py")] + args
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only, exactly one line
    d = json.loads(lines[0])
    assert KEYS <= set(d)
    assert d["n_gpus"] == n and d["steps"] == 2 and d["warmup"] == 1
    assert d["scaling"] == "weak" and d["higher_is_better"] is True
    assert d["config"]["global_batch"] == 2 * n
    assert d["config"]["parallelism"] == f"pp{n // dp}" + (f"xdp{dp}" if dp > 1 else "")
    # value is the whole-job token rate over the timed steps
    toks = d["config"]["global_batch"] * d["config"]["gen_tokens"]
    assert d["value"] == pytest.approx(toks / (d["ms_per_step"] / 1e3), rel=0.02)
    if n > 1:  # the data plane's own evidence (verdict r2: a SCALE line must show N ranks)
        assert d["transport"] == "gloo" and d["pg_world_size"] == n
        assert len(d["rank_devices"]) == n and len(d["stage_busy"]) == n
        # every rank is on 2 edge groups (fwd in / fwd out or the return edge), P = 1 on none
        P = n // dp
        assert d["data_plane_comms"] == (2 * n if P > 1 else 0)


def test_auto_microbatch_groups():
    """bench.py default groups: 2 per stage when a decode step reads more KV
    than weights on the VALU attention kernel (GPT-2 XL headline), 1 per
    stage otherwise (Llama-3 8B: grouped-query attention on MFMA)."""
    import importlib.util
    import types

    spec = importlib.util.spec_from_file_location("bench", os.path.join(ROOT, "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    a = lambda m, n: types.SimpleNamespace(model=m, batch=n, prompt=128, gen=128)  # noqa: E731
    assert b.auto_groups(a("gpt2-xl", 512), 1) == 2
    assert b.auto_groups(a("gpt2-xl", 512), 8) == 16
    assert b.auto_groups(a("gpt2-xl", 1), 1) == 1
    assert b.auto_groups(a("llama-3-8b", 256), 1) == 1
    assert b.auto_groups(a("llama-3-8b", 256), 4) == 4  # KV-bound, but MFMA attention is at roofline
    assert b.auto_groups(types.SimpleNamespace(model="llama-3-8b", batch=32, prompt=4096, gen=128), 1) == 1
