"""Build/load the native host runtime (csrc/runtime/runtime.cpp -> _runtime.so).

Pure C++17 + pybind11 (no HIP, no torch), so it also builds and runs on the
CPU-only dev box.  The Python engine uses it when present (slot allocation,
microbatch planning, partition DP); the pure-Python twins in kv_cache.py /
partition.py remain as the reference implementation the tests compare to.
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sysconfig

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROOT = os.path.dirname(PKG)
SRC = os.path.join(ROOT, "csrc", "runtime", "runtime.cpp")
HDR = os.path.join(ROOT, "csrc", "runtime", "batch_queue.h")
CORE = os.path.join(ROOT, "csrc", "runtime", "sched_core.h")
SHM = os.path.join(ROOT, "csrc", "runtime", "shm_ring.h")


def build(force: bool = False) -> str:
    import pybind11

    so = os.path.join(PKG, "_runtime.so")
    stamp = os.path.join(ROOT, "build", "native", "_runtime.sha")
    os.makedirs(os.path.dirname(stamp), exist_ok=True)
    flags = ["-O2", "-std=c++17", "-fPIC", "-shared", f"-I{pybind11.get_include()}",
             f"-I{sysconfig.get_paths()['include']}"]
    h = hashlib.sha1(" ".join(flags).encode())
    for src in (SRC, HDR, CORE, SHM):
        with open(src, "rb") as f:
            h.update(f.read())
    sig = h.hexdigest()
    if not force and os.path.exists(so) and os.path.exists(stamp) and open(stamp).read() == sig:
        return so
    tmp = so + ".tmp"
    r = subprocess.run(["g++"] + flags + [SRC, "-o", tmp, "-lrt"], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"runtime build failed:\n{r.stderr}")
    os.replace(tmp, so)
    with open(stamp, "w") as f:
        f.write(sig)
    return so


def load():
    try:
        from .. import _runtime

        return _runtime
    except ImportError:
        return None
