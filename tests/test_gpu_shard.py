"""Multi-GPU sharding on one box: one host thread + one context per device, each
decoding its contiguous block of row groups (shard.decode_sharded).  On a one-GPU box the devices
are [0, 0]: two contexts and two threads on the same card, which exercises the same code path."""
import numpy as np
import pytest

import fixtures
from oracle import oracle as O
from parity import assert_chunk, oracle_chunk

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("ndev", [2, 3])
def test_decode_sharded_contexts(pq, ndev):
    data = fixtures.flat_c2_like(n=40000, v2=True)
    f = pq.native.File(data)
    ncols = len(f.columns())
    nrg = f.num_row_groups
    out = pq.shard.decode_sharded(data, [0] * ndev)
    fr = O.FileReader(data)
    pos = 0
    for dev, rg0, rg1, res in out:
        assert rg0 == pos
        pos = rg1
        assert len(res) == (rg1 - rg0) * ncols
        for k, col in enumerate(res):
            rg, ci = rg0 + k // ncols, k % ncols
            assert_chunk(col, oracle_chunk(fr, rg, ci), where=f"dev{dev} rg{rg} c{ci}")
    assert pos == nrg
    blocks = [(rg0, rg1, sum(f.row_group_num_rows(g) for g in range(rg0, rg1)), 0) for _, rg0, rg1, _ in out]
    assert pq.shard.check_cover(blocks, nrg, f.num_rows)
