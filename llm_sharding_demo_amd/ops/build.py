"""In-tree native build: CDNA4 kernels + bindings -> llm_sharding_demo_amd/_C.so.

No torch.utils.cpp_extension JIT and no hipify: every .hip file is compiled
directly for gfx950 with hipcc, the pybind11 bindings with g++ against the
torch headers, and the result is linked into a .so inside the package so it
travels with the repo snapshot to the GPU box (a JIT cache under ~/.cache
would not).  The extension links libamdhip64.so.7 by SONAME, so in-process it
binds to the HIP runtime torch already loaded (one runtime per process;
SURVEY.md §5.8 hazard).

Incremental: objects are rebuilt only when a source/header or the flags change.
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from typing import List

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "native")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

KERNELS = ["gemm.hip", "gemv.hip", "norm.hip", "attention.hip", "sample.hip", "loopback.hip", "elementwise.hip"]
# host code of the extension: kernel bindings, native RCCL communicator, native stage
# executor, device loopback channels (single-GPU rehearsal of the RCCL edges),
# hipBLASLt prefill projections
HOST_SOURCES = ["bindings.cpp", "comm.cpp", "stage_exec.cpp", "loop_fabric.cpp", "blaslt.cpp"]
EXT_NAME = "_C"


def _torch_flags():
    import torch
    from torch.utils.cpp_extension import include_paths

    inc = [f"-I{p}" for p in include_paths("cuda")] + [f"-I{sysconfig.get_paths()['include']}",
                                                       "-I/opt/rocm/include"]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    lib = os.path.join(os.path.dirname(torch.__file__), "lib")
    return inc, abi, lib


def _hash(paths: List[str], extra: str) -> str:
    h = hashlib.sha1(extra.encode())
    for p in paths:
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _run(cmd: List[str], verbose: bool) -> None:
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def headers() -> List[str]:
    out = []
    for d in (os.path.join(CSRC, "kernels"), CSRC, os.path.join(CSRC, "runtime")):
        for fn in sorted(os.listdir(d)):
            if fn.endswith(".h"):
                out.append(os.path.join(d, fn))
    return out


def build(verbose: bool = False, force: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    inc, abi, torch_lib = _torch_flags()
    hdrs = headers()
    kflags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
              "-Wno-unused-result"] + os.environ.get("LSD_HIPCC_FLAGS", "").split()  # tuning A/B
    jobs = []
    objs = []
    for k in KERNELS:
        src = os.path.join(CSRC, "kernels", k)
        obj = os.path.join(BUILD, k.replace(".hip", ".o"))
        stamp = obj + ".sha"
        sig = _hash([src] + hdrs, " ".join(kflags))
        objs.append(obj)
        if force or not os.path.exists(obj) or not os.path.exists(stamp) or open(stamp).read() != sig:
            jobs.append(([HIPCC] + kflags + ["-c", src, "-o", obj], stamp, sig))
    bflags = ["-O2", "-std=c++17", "-fPIC", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
              f"-D_GLIBCXX_USE_CXX11_ABI={abi}", f"-DTORCH_EXTENSION_NAME={EXT_NAME}",
              "-DTORCH_API_INCLUDE_EXTENSION_H", "-Wno-deprecated-declarations"] + inc
    for host_src in HOST_SOURCES:  # torch-extension host code (g++)
        bsrc = os.path.join(CSRC, host_src)
        bobj = os.path.join(BUILD, host_src.replace(".cpp", ".o"))
        bsig = _hash([bsrc] + hdrs, " ".join(bflags))
        bstamp = bobj + ".sha"
        if force or not os.path.exists(bobj) or not os.path.exists(bstamp) or open(bstamp).read() != bsig:
            jobs.append((["g++"] + bflags + ["-c", bsrc, "-o", bobj], bstamp, bsig))
        objs.append(bobj)

    def do(job):
        cmd, stamp, sig = job
        _run(cmd, verbose)
        with open(stamp, "w") as f:
            f.write(sig)

    workers = min(len(jobs), int(os.environ.get("MAX_JOBS", "8")), 8) or 1
    with ThreadPoolExecutor(workers) as ex:
        list(ex.map(do, jobs))
    so = os.path.join(PKG, EXT_NAME + ".so")
    if jobs or force or not os.path.exists(so):
        tmp = so + ".tmp"
        _run([HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}"] + objs +
             ["-o", tmp, f"-L{torch_lib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
              "-ltorch_python", "-ltorch_hip", "-lhipblaslt", "-ldl", f"-Wl,-rpath,{torch_lib}"], verbose)
        os.replace(tmp, so)
    return so


if __name__ == "__main__":
    print(build(verbose="-v" in sys.argv, force="-f" in sys.argv))
