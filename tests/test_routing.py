"""The HIP backend's kernel routing table (ops/routing.py), pinned on CPU.

Every GEMM of GPT-2 small / XL and Llama-3 8B at the row counts the benches
and serving run (single stream, 8-512-row decode groups, 65 K-row merged
prefill) routes to a hand-written gfx950 kernel family with a fixed K split;
`tests/data/routing_table.json` is that table.  A routing change must update
it deliberately (regenerate with `route_table`), and the default table never
names hipBLASLt (the library is an opt-in A/B oracle, `LSD_ROUTING=blaslt=1`).
The block projections routed here are the reference's GPT2Block c_attn /
c_proj / c_fc / c_proj and lm_head (`/root/reference/server.py:84-85,99-102`)."""
import json
import os

import pytest

from llm_sharding_demo_amd.ops.routing import Routing, route_table

ROWS = [1, 8, 64, 128, 256, 512, 65536]
TABLE = os.path.join(os.path.dirname(__file__), "data", "routing_table.json")


def _table(r: Routing) -> dict:
    out = {}
    for m in ["gpt2", "gpt2-xl", "llama-3-8b"]:
        for (g, M, ph), route in route_table(m, ROWS, r).items():
            out[f"{m}|{ph}|{M}|{g}"] = route
    return out


def test_default_routing_matches_pinned_table():
    want = json.load(open(TABLE))
    got = _table(Routing())
    diff = {k: (want.get(k), got.get(k)) for k in set(want) | set(got) if want.get(k) != got.get(k)}
    assert not diff, diff


def test_default_routing_is_hand_written_only():
    assert all(r != "hipblaslt" for r in _table(Routing()).values())
    assert Routing().blaslt == 0


def test_blaslt_oracle_routes_when_asked():
    t = _table(Routing(blaslt=1))
    assert t["gpt2-xl|prefill|65536|up"] == "hipblaslt"       # bias + GELU epilogue
    assert t["gpt2-xl|prefill|65536|down"] == "hipblaslt"     # K 6400 residual
    assert t["gpt2-xl|prefill|65536|o"].startswith("tiled")   # K 1600 stays hand-written
    assert t["llama-3-8b|decode|512|qkv"] == "hipblaslt"
    assert t["llama-3-8b|decode|128|up"] == "hipblaslt"
    assert t["gpt2-xl|decode|256|up"].startswith("tiled")


def test_single_stream_on_gemv_and_key_shapes():
    t = _table(Routing())
    for m in ["gpt2", "gpt2-xl", "llama-3-8b"]:
        for g in ["qkv", "o", "up", "down", "lm_head"]:
            assert t[f"{m}|decode|1|{g}"] == "gemv"
    assert t["gpt2-xl|decode|256|qkv"] == "tiled/s1"           # 8-wave LDS ring
    assert t["gpt2-xl|decode|256|down"] == "tiled/s5"          # residual slabs folded by the norm
    assert t["llama-3-8b|decode|256|up"].startswith("d256")    # all-rows kernel for long K


def test_routing_env_override():
    r = Routing.from_env("ring8=0, sk_target=256")
    assert r.ring8 == 0 and r.sk_target == 256 and r.tiled3_max == Routing().tiled3_max
    with pytest.raises(ValueError):
        Routing.from_env("no_such_knob=1")


def test_attention_splits_policy():
    r = Routing()
    assert r.attn_splits(1, 32, 8, 128, 192) >= 1
    assert r.attn_splits(512, 25, 25, 64, 256) == 1      # full batch: no split
    assert r.attn_splits(1, 25, 25, 64, 1024) > 1        # single stream long context splits
