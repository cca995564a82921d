"""Sanitizer stress drivers for the host concurrency protocols of the
multi-rank control and data planes:
  * csrc/runtime/loop_handshake.h -- the per-channel enqueue handshake of the
    device loopback channels (csrc/loop_fabric.cpp), sender / receiver
    threads on shared mirrors, wraparound, cumulative I/O lists, abort and
    timeout (csrc/runtime/tests/loop_handshake_stress.cpp);
  * csrc/runtime/shm_ring.h -- the shared-memory plan ring (parallel/comm.py
    ShmPlanChannel): one producer, several readers with their own mappings,
    a slow reader, timeouts, close (csrc/runtime/tests/shm_ring_stress.cpp).
Both run under ThreadSanitizer and under AddressSanitizer + UBSan.  The
reference's handlers share module globals across threads with no locks and
no checker at all (`/root/reference/server.py:153-210`)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
@pytest.mark.parametrize("driver,args,expect", [
    ("loop_handshake_stress.cpp", ["4", "2000"], "ok 4 channels"),
    ("shm_ring_stress.cpp", ["4", "6000"], "ok 4 readers"),
])
def test_protocol_under_sanitizer(tmp_path, san, driver, args, expect):
    if shutil.which("g++") is None:
        pytest.skip("needs g++")
    exe = tmp_path / driver.replace(".cpp", "")
    r = subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-pthread", f"-fsanitize={san}",
                        "-fno-omit-frame-pointer", os.path.join(ROOT, "csrc", "runtime", "tests", driver),
                        "-o", str(exe), "-lrt"], capture_output=True, text=True)
    if r.returncode != 0 and "cannot find" in r.stderr:
        pytest.skip(f"sanitizer runtime not available: {r.stderr[-200:]}")
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1",
               UBSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1")
    r = subprocess.run([str(exe)] + args, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr[-4000:]
    assert r.stdout.startswith(expect), r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr, r.stderr[-4000:]
