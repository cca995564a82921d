"""bench.py at N > 1 checks its own tokens: after the timed region rank 0
re-generates the first groups of the last session on a 1-stage engine on its
own device and reports `pipeline_matches_1gpu`; a mismatch exits non-zero.
The driver's multi-GPU scaling run is the only hardware execution the RCCL
path gets, so a pipeline producing wrong tokens must not print a number and
pass (the hop it replaces, `/root/reference/server.py:171-181`, checks
nothing).  CPU: gloo ranks; GPU: rank processes on one MI355X (devloop)."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench(world, extra, env_extra=None, timeout=400):
    port = _port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="1")
    env.update(env_extra or {})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"),
           "--gpus", str(world), "--steps", "1", "--warmup", "0"] + extra
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    return r, (json.loads(lines[-1]) if lines else None)


CPU = ["--model", "gpt2-test", "--batch", "8", "--prompt", "6", "--gen", "5", "--device", "cpu",
       "--transport", "gloo"]


@pytest.mark.parametrize("world", [2, 8])
def test_gloo_bench_reports_token_check(world):
    r, out = _bench(world, CPU)
    assert r.returncode == 0 and out is not None, r.stderr[-3000:]
    assert out["pipeline_matches_1gpu"] is True, out
    assert out["check_seqs"] > 0 and out["pg_world_size"] == world, out


def test_gloo_bench_corrupted_stage_fails():
    r, out = _bench(2, CPU, env_extra={"LSD_TEST_HOOKS": "1", "LSD_TEST_CORRUPT_RANK": "1"})
    assert r.returncode != 0, r.stdout[-2000:]
    assert out is not None and out["pipeline_matches_1gpu"] is False, out
    assert out["check_mismatched_seqs"] > 0


def test_gloo_selftest_failure_falls_back_in_process():
    """The data plane's startup self-test fails on one rank (injected): every
    rank agrees, tears the first transport down and brings up the next one of
    the chain in the same processes; the run then reports the transport it
    used, why it left the first, and its tokens still match one stage."""
    cpu = [a for a in CPU if a != "gloo"]
    cpu[cpu.index("--transport") + 1:cpu.index("--transport") + 1] = ["gloo,gloo"]
    r, out = _bench(2, cpu, env_extra={"LSD_TEST_HOOKS": "1", "LSD_TEST_SELFTEST_FAIL": "1"})
    assert r.returncode == 0 and out is not None, r.stderr[-3000:]
    assert out["transport"] == "gloo" and "injected" in (out["transport_fallback"] or ""), out
    assert out["pipeline_matches_1gpu"] is True, out


def test_gloo_selftest_pass_reports_no_fallback():
    r, out = _bench(2, CPU)
    assert r.returncode == 0 and out is not None, r.stderr[-3000:]
    assert out["transport"] == "gloo" and out["transport_fallback"] is None, out


def test_transport_chain_defaults():
    from llm_sharding_demo_amd.parallel.comm import transport_chain

    assert transport_chain("auto", "cuda") == ["rccl", "nccl"]
    assert transport_chain("auto", "cuda", shared_gpu=True) == ["devloop", "gloo"]
    assert transport_chain("auto", "cpu") == ["gloo"]
    assert transport_chain("rccl,nccl", "cuda") == ["rccl", "nccl"]
    assert transport_chain("nccl", "cuda") == ["nccl"]


@pytest.mark.gpu
def test_devloop_selftest_failure_falls_back_to_gloo():
    """Two rank processes on one MI355X: the device-loopback data plane
    passes its own eager + graph-captured self-test, a failure injected on
    rank 1 makes both ranks abort it and fall back to host-staged gloo in
    process; tokens still match one GPU."""
    r, out = _bench(2, ["--model", "gpt2", "--batch", "16", "--prompt", "16", "--gen", "8",
                        "--transport", "devloop,gloo"],
                    env_extra={"LSD_LOOP_RING_MB": "16", "LSD_TEST_HOOKS": "1", "LSD_TEST_SELFTEST_FAIL": "1"})
    assert r.returncode == 0 and out is not None, (r.stdout[-2000:], r.stderr[-3000:])
    assert out["transport"] == "gloo" and "injected" in (out["transport_fallback"] or ""), out
    assert out["pipeline_matches_1gpu"] is True, out


@pytest.mark.gpu
def test_auto_transport_ranks_on_one_gpu_take_devloop():
    """Default flags with two ranks on one GPU: the auto chain detects the
    shared device and runs the device loopback plane (self-test passed)."""
    r, out = _bench(2, ["--model", "gpt2", "--batch", "16", "--prompt", "16", "--gen", "8"],
                    env_extra={"LSD_LOOP_RING_MB": "16"})
    assert r.returncode == 0 and out is not None, (r.stdout[-2000:], r.stderr[-3000:])
    assert out["transport"] == "devloop" and out["transport_fallback"] is None, out
    assert out["pipeline_matches_1gpu"] is True, out


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_devloop_bench_reports_token_check(world):
    """Rank processes sharing one MI355X over the device-loopback data plane
    (the rccl code path's rehearsal), GPT-2 small, 2 groups per stage."""
    r, out = _bench(world, ["--model", "gpt2", "--batch", "16", "--prompt", "16", "--gen", "8",
                            "--transport", "devloop"], env_extra={"LSD_LOOP_RING_MB": "16"})
    assert r.returncode == 0 and out is not None, (r.stdout[-2000:], r.stderr[-3000:])
    assert out["pipeline_matches_1gpu"] is True and out["transport"] == "devloop", out


def test_bounded_reports_a_hang_and_an_error():
    """The bring-up helper for blocking communicator inits: a call that does
    not return by the deadline and a call that raises both come back as an
    error string (the caller agrees on it with every rank), never a hang."""
    import time

    from llm_sharding_demo_amd.parallel.comm import _bounded

    r, err = _bounded(lambda: time.sleep(5), 0.2, "stuck init")
    assert r is None and "no result after" in err
    r, err = _bounded(lambda: 1 // 0, 5.0, "bad init")
    assert r is None and "ZeroDivisionError" in err
    assert _bounded(lambda: 7, 5.0, "ok") == (7, None)


def test_native_rccl_unavailable_falls_back_on_every_rank():
    """The real RcclTransport bring-up on a box without GPUs: every rank fails
    its first step (no HIP device), the failure is agreed over the gloo
    control group, and both ranks bring up the next transport of the chain
    in process; the run reports why and still matches one stage."""
    cpu = [a for a in CPU if a != "gloo"]
    cpu[cpu.index("--transport") + 1:cpu.index("--transport") + 1] = ["rccl,gloo"]
    r, out = _bench(2, cpu)
    assert r.returncode == 0 and out is not None, r.stderr[-3000:]
    assert out["transport"] == "gloo" and "native RCCL unavailable" in (out["transport_fallback"] or ""), out
    assert out["pipeline_matches_1gpu"] is True, out
