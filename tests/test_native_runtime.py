"""Native host runtime (csrc/runtime/runtime.cpp): equivalence with the
Python twins, pipeline-schedule simulation properties, and a host-side
ASan/UBSan run (GPU sanitizers are not available on this pool)."""
import os
import shutil
import subprocess
import sys
import textwrap

import pytest

from llm_sharding_demo_amd.config import get_model_config
from llm_sharding_demo_amd.parallel.partition import auto_partition, stage_costs
from llm_sharding_demo_amd.runtime import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def R():
    native.build()
    mod = native.load()
    assert mod is not None
    return mod


def test_partition_dp_matches_python(R):
    for name in ("gpt2", "gpt2-xl", "llama-3-8b"):
        mc = get_model_config(name)
        for P in (2, 4, 8):
            py = auto_partition(mc, P, batch=64, avg_ctx=192)
            blk = stage_costs(mc, [(0, 1)], 64, 192)[0]
            head = stage_costs(mc, [(0, 0)], 64, 192)[0]
            cc = R.partition_minmax([blk] * mc.n_layers, P, head)
            cost = lambda plan: max(stage_costs(mc, plan, 64, 192))
            assert abs(cost(cc) - cost(py)) < 1e-6 * cost(py)


def test_slot_allocator(R):
    a = R.SlotAllocator(4)
    s = a.alloc(3)
    assert sorted(s) == [0, 1, 2] and a.available == 1
    with pytest.raises(RuntimeError):
        a.alloc(2)
    a.free(s)
    with pytest.raises(RuntimeError):
        a.free([0])  # double free detected


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_runtime_under_asan_ubsan(tmp_path):
    import pybind11
    import sysconfig

    libasan = subprocess.run(["g++", "-print-file-name=libasan.so"], capture_output=True,
                             text=True).stdout.strip()
    if not os.path.isfile(libasan):
        pytest.skip("libasan not available")
    so = tmp_path / "_runtime.so"
    r = subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-fPIC", "-shared",
                        "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                        f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}",
                        os.path.join(ROOT, "csrc", "runtime", "runtime.cpp"), "-o", str(so)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    script = tmp_path / "run.py"
    script.write_text(textwrap.dedent(f"""
        import sys; sys.path.insert(0, {str(tmp_path)!r})
        import _runtime as R
        a = R.SlotAllocator(64)
        for _ in range(200):
            s = a.alloc(7); a.free(s)
        R.partition_minmax([1.0] * 48, 8, 2.6)
        q = R.BatchQueue(8, 4.0)
        for i in range(20):
            q.push(i, 1 + i % 5)
        got = q.try_pop(5) + [x for g in q.next_groups(0.0) for x in g]
        print(len(got), float(sorted(got)[2]))
    """))
    env = dict(os.environ, LD_PRELOAD=libasan, ASAN_OPTIONS="detect_leaks=0",
               UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([sys.executable, str(script)], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.strip().endswith("2.0")
