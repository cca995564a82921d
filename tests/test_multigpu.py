"""Real multi-GPU pipelines: one process per MI355X under torch.distributed.run,
RCCL point-to-point between the stages -- through torch.distributed
(`--transport nccl`) and through the native communicator with transfers
captured in the decode graphs (`--transport rccl`) -- compared token for
token with one GPU.  These run only where the box has >= 2 GPUs (the
driver's 8-GPU node); on one GPU they skip.  Their CPU twins (same worker
script, gloo, world 2 / 4) run in `pytest -m "not gpu"`.

The stall test is the failure path of the reference's two-hop relay
(`/root/reference/server.py:171-181`, where a dead shard surfaces as a 500
after the 30 s HTTP timeout): one rank stops issuing mid-session, the peer
waiting on it must fail its requests within the round deadline -- over RCCL
through ncclCommAbort returning the blocked ncclRecv, over gloo through the
process group's timeout.
"""
import json
import os
import socket
import subprocess
import sys
import textwrap

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROMPTS = [[1, 2, 3, 4], [5, 6], list(range(10, 40)), [7] * 9, [3, 1, 4, 1, 5], [9, 2, 6]]


def _ngpu() -> int:
    return torch.cuda.device_count() if torch.cuda.is_available() else 0


needs_2gpu = pytest.mark.skipif(_ngpu() < 2, reason="needs >= 2 GPUs (one rank per MI355X)")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(tmp_path, world, device, transport, dp=1, greedy=True, env_extra=None, timeout=600,
         round_timeout=120.0, chunk=0):
    """Launch `world` ranks; rank 0 prints RESULT {tokens, evidence per rank}."""
    M = 2 * (world // dp)
    script = tmp_path / f"w_{transport}_{world}_{dp}.py"
    script.write_text(textwrap.dedent(f"""
        import sys, json, os, time
        sys.path.insert(0, {ROOT!r})
        from llm_sharding_demo_amd.config import EngineConfig, SamplingParams
        from llm_sharding_demo_amd.runtime.engine import build_engine
        cfg = EngineConfig(model_id="gpt2-test", max_batch=12, device={device!r}, transport={transport!r},
                           num_microbatches={M}, max_seq_len=128, dp_replicas={dp},
                           round_timeout_s={round_timeout}, prefill_chunk={chunk})
        code = 0
        try:
            eng = build_engine(cfg)
            sp = SamplingParams(greedy={greedy}, temperature=0.8, top_k=20, seed=5, max_new_tokens=10)
            if eng.rank != 0:
                try:
                    eng.worker_loop()
                finally:
                    w = eng.workers[0]
                    # one write per line: ranks share the pipe, print() writes text and newline separately
                    os.write(1, ("EVID " + json.dumps(dict(rank=eng.rank, native=w.native_steps, io=w.io_items,
                                                            graph_io=w.graph_io, comms=eng.transport.num_comms))
                                 + "\\n").encode())
            else:
                t0 = time.monotonic()
                err = None
                try:
                    out = eng.generate_ids({PROMPTS!r}, sp)
                    out2 = eng.generate_ids({PROMPTS!r}, sp)  # graphs cached: captured transfers replay
                except Exception as e:
                    out = out2 = None
                    err = f"{{type(e).__name__}}: {{e}}"
                w = eng.workers[0]
                os.write(1, ("RESULT " + json.dumps(dict(out=out, out2=out2, err=err, healthy=eng.healthy,
                                                          elapsed=time.monotonic() - t0, native=w.native_steps,
                                                          graph_io=w.graph_io, world=eng.transport.gworld,
                                                          comms=eng.transport.num_comms)) + "\\n").encode())
                if err is None:
                    eng.shutdown()
        except Exception as e:
            print("FAIL", type(e).__name__, e, flush=True)
            # a follower whose data plane failed in a stall test exits 0: a
            # non-zero exit makes torchrun kill rank 0 before it prints RESULT;
            # in a healthy run any follower failure (or an engine that could
            # not even be built) fails the job
            stall = bool(os.environ.get("LSD_TEST_STALL_RANK"))
            code = 0 if ("eng" in dir() and stall) else 3
        sys.stdout.flush()
        os._exit(code)  # a stalled peer must not hold the teardown
    """))
    port = _port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="1")
    env.update(env_extra or {})
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={port}", str(script)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout)
    res = [l[l.index("RESULT"):] for l in r.stdout.splitlines() if "RESULT {" in l]
    if not res:  # keep the lines that say what went wrong (the tail is mostly torchrun's summary)
        keep = [l for l in (r.stdout + r.stderr).splitlines()
                if any(k in l for k in ("FAIL", "Error", "error", "Traceback", "line ", "raise"))]
        raise AssertionError(f"rc {r.returncode}\n" + "\n".join(keep[-60:]))
    import re

    evid = [json.loads(m) for m in re.findall(r"EVID (\{[^{}]*\})", r.stdout)]
    return json.loads(res[0][len("RESULT "):]), evid, r


def _one_stage(device, dp_groups, greedy=True):
    from llm_sharding_demo_amd.config import EngineConfig, SamplingParams
    from llm_sharding_demo_amd.runtime.engine import Engine

    eng = Engine(EngineConfig(model_id="gpt2-test", num_stages=1, max_batch=12, device=device,
                              num_microbatches=dp_groups, max_seq_len=128, merge_prefill=False))
    sp = SamplingParams(greedy=greedy, temperature=0.8, top_k=20, seed=5, max_new_tokens=10)
    out = eng.generate_ids(PROMPTS, sp)
    eng.shutdown()
    return out


# ---------------------------------------------------------------------------
# >= 2 GPUs: RCCL between processes
# ---------------------------------------------------------------------------
def _gpu_worlds():
    n = min(8, _ngpu())
    return sorted({2, n}) if n >= 2 else [2]


@pytest.mark.gpu
@needs_2gpu
@pytest.mark.parametrize("transport", ["nccl", "rccl"])
@pytest.mark.parametrize("world", _gpu_worlds())
@pytest.mark.parametrize("greedy", [True, False])
def test_rccl_pipeline_matches_one_gpu(tmp_path, transport, world, greedy):
    res, evid, r = _run(tmp_path, world, "cuda", transport, greedy=greedy)
    assert res["err"] is None, (res, r.stderr[-4000:])
    assert res["world"] == world and res["healthy"]
    want = _one_stage("cuda", 2 * world, greedy)
    assert res["out"] == want and res["out2"] == want
    if transport == "rccl":
        # graph-captured ncclRecv / ncclSend and the native executor ran
        assert res["graph_io"] and res["native"] > 0, res
        assert all(e["graph_io"] and e["native"] > 0 for e in evid), evid
        assert all(e["io"] > 0 for e in evid), evid
        assert res["comms"] == 2 * 2  # (fwd0, ret) x 2 lanes on stage 0


@pytest.mark.gpu
@pytest.mark.skipif(_ngpu() < 4, reason="needs >= 4 GPUs (2 replicas x 2 stages)")
@pytest.mark.parametrize("transport", ["nccl", "rccl"])
def test_rccl_dp2_pipelines_match_one_gpu(tmp_path, transport):
    world = min(8, _ngpu()) // 2 * 2
    res, evid, r = _run(tmp_path, world, "cuda", transport, dp=2)
    assert res["err"] is None, (res, r.stderr[-4000:])
    assert res["out"] == _one_stage("cuda", world)  # 2 replicas x (world/2 stages x 2 groups)


@pytest.mark.gpu
@needs_2gpu
def test_rccl_stall_abort_unblocks_recv(tmp_path):
    """Rank 1 (the last stage) stops issuing after a few steps: rank 0's
    token-return ncclRecv is blocked on the device; its watchdog must fire,
    ncclCommAbort must return the receive, and the request must fail within
    the deadline."""
    res, evid, r = _run(tmp_path, 2, "cuda", "rccl", round_timeout=8.0, timeout=300,
                        env_extra={"LSD_TEST_STALL_RANK": "1", "LSD_TEST_STALL_AFTER": "8"})
    assert res["err"] is not None and not res["healthy"], res
    assert "WatchdogTimeout" in res["err"] or "abort" in res["err"], res["err"]
    assert res["elapsed"] < 8.0 + 30.0, res


# ---------------------------------------------------------------------------
# CPU twins: the same worker script over gloo
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("world,dp,chunk", [(2, 1, 0), (4, 1, 2), (4, 2, 0), (8, 1, 2), (8, 2, 0)])
def test_gloo_twin_matches_one_stage(tmp_path, world, dp, chunk):
    res, evid, r = _run(tmp_path, world, "cpu", "gloo", dp=dp, greedy=False, chunk=chunk, timeout=300)
    assert res["err"] is None, (res, r.stderr[-4000:])
    assert res["world"] == world
    want = _one_stage("cpu", 1, greedy=False)  # the CPU path is batch-invariant
    assert res["out"] == want and res["out2"] == want


def test_gloo_twin_stall_fails_within_deadline(tmp_path):
    res, evid, r = _run(tmp_path, 2, "cpu", "gloo", round_timeout=4.0, timeout=200,
                        env_extra={"LSD_TEST_STALL_RANK": "1", "LSD_TEST_STALL_AFTER": "5"})
    assert res["err"] is not None and not res["healthy"], res
    assert res["elapsed"] < 4.0 + 30.0, res


def test_gloo_twin_plan_ring_failure_falls_back(tmp_path):
    """A node without usable shared memory (here: an invalid segment name)
    falls back to the gloo plan records on every rank together."""
    res, evid, r = _run(tmp_path, 2, "cpu", "gloo", greedy=False, timeout=300,
                        env_extra={"LSD_SHM_PREFIX": "/no/such/dir"})
    assert res["err"] is None, (res, r.stderr[-4000:])
    assert "plans over gloo" in r.stderr
    want = _one_stage("cpu", 1, greedy=False)
    assert res["out"] == want


# ---------------------------------------------------------------------------
# One GPU, several processes: the dist-mode rehearsal of the rccl data plane
# (parallel/comm.py IpcLoopTransport: device loopback channels shared between
# the rank processes, graph-captured transfers, native executor at P > 1)
# ---------------------------------------------------------------------------
@pytest.mark.gpu
@pytest.mark.parametrize("world,dp", [(2, 1), (3, 1), (4, 2)])
def test_devloop_processes_on_one_gpu_match_one_gpu(tmp_path, world, dp):
    res, evid, r = _run(tmp_path, world, "cuda", "devloop", dp=dp, greedy=False, timeout=400,
                        env_extra={"LSD_LOOP_RING_MB": "16"})
    assert res["err"] is None, (res, r.stderr[-4000:])
    assert res["world"] == world and res["healthy"]
    assert res["out"] == _one_stage("cuda", 2 * world // dp, greedy=False) == res["out2"]
    # every rank of replica 0 ran captured edge transfers and native steps (the
    # scheduler may place all six requests on replica 0)
    P = world // dp
    assert res["graph_io"] and res["native"] > 0, res
    assert all(e["graph_io"] for e in evid), evid
    assert all(e["native"] > 0 and e["io"] > 0 for e in evid if e["rank"] < P), evid


@pytest.mark.gpu
def test_devloop_processes_stall_fails_within_deadline(tmp_path):
    res, evid, r = _run(tmp_path, 2, "cuda", "devloop", round_timeout=6.0, timeout=300,
                        env_extra={"LSD_LOOP_RING_MB": "16", "LSD_TEST_STALL_RANK": "1",
                                   "LSD_TEST_STALL_AFTER": "8"})
    assert res["err"] is not None and not res["healthy"], res
    assert res["elapsed"] < 6.0 + 30.0, res
