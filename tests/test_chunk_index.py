"""The prefill items' packed index buffer (parallel/pipeline.py _chunk_index):
the same token slots / positions, sequence slots / starts, row offsets, last
rows and token ids as BatchMeta.build and the chunk lists, for random chunk
mixes (decode-shaped ones included)."""
import random

import pytest

from llm_sharding_demo_amd.parallel.pipeline import _chunk_index
from llm_sharding_demo_amd.runtime.batch import BatchMeta
from llm_sharding_demo_amd.runtime.plan import Chunk


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("first", [True, False])
def test_chunk_index_matches_batchmeta(seed, first):
    rnd = random.Random(seed)
    B = rnd.randrange(1, 40)
    one = seed % 3 == 0  # decode-shaped: one query per sequence
    ch = [Chunk(seq=i, slot=rnd.randrange(1000), start=rnd.randrange(500),
                ids=[rnd.randrange(50257) for _ in range(1 if one else rnd.randrange(1, 70))],
                final=rnd.random() < 0.5) for i in range(B)]
    q = tuple(c.qlen for c in ch)
    a = _chunk_index(ch, q, first).tolist()
    m = BatchMeta.build([c.slot for c in ch], [c.start for c in ch], list(q), "cpu")
    T = sum(q)
    o = 2 * T + 2 * B
    assert a[:T] == m.token_slots.tolist()
    assert a[T: 2 * T] == m.token_pos.tolist()
    assert a[2 * T: 2 * T + B] == m.seq_slots.tolist()
    assert a[2 * T + B: o] == m.q_start.tolist()
    assert a[o: o + B + 1] == m.cu_q.tolist()
    assert a[o + B + 1: o + 2 * B + 1] == m.last_idx.tolist()
    assert a[o + 2 * B + 1:] == ([t for c in ch for t in c.ids] if first else [])
