"""The end-to-end streaming ring (reader.RowGroupStream): a file several times
larger than the ring's pinned staging, read range by range -- host walk into a slot's pinned block,
H2D and decode in order on the slot's one stream, `slots` ranges in flight -- and every
chunk compared with the seeded input it was written from (datasets.mixed: north_star's mixed file
at a smaller size), two row groups with the oracle bit for bit.  The pinned memory stays bounded
by the slots, pass after pass."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("threaded", [False, True])
def test_row_group_stream_ring(pq, threaded):
    from oracle import oracle as O
    from parity import assert_chunk, oracle_chunk
    from parquet_go_amd import datasets

    rows, nrg, per_range, slots = 3_200_000, 32, 2, 2
    data = datasets.mixed(rows=rows, row_groups=nrg)
    sizes = datasets.mixed_sizes(rows, nrg)
    f = pq.native.File(data)
    ncols = len(f.columns())
    cols = f.columns()
    fr = O.FileReader(data)
    st = pq.reader.RowGroupStream(f, list(range(ncols)), per_range=per_range, slots=slots,
                                    threaded=threaded)
    try:
        for a, b, batch, hb in st:  # a pass abandoned after its first range releases every slot
            break
        biggest = 0
        for rnd in range(2):
            seen, total = [], 0
            for a, b, batch, hb in st:
                seen.append((a, b))
                biggest = max(biggest, hb.payload_bytes)
                total += hb.payload_bytes
                ctx = batch.ctx
                for rg in range(a, b):
                    for ci, (name, col, _) in enumerate(datasets.mixed_row_group(rg, sizes[rg])):
                        o = batch.chunk_out((rg - a) * ncols + ci)
                        assert o.status == pq.native.OK, (rg, name, o.status)
                        n, nn = sizes[rg], sizes[rg]
                        if col.def_levels is not None:
                            assert np.array_equal(ctx.d2h_array(o.def_levels, n), col.def_levels), (rg, name)
                            nn = int(np.count_nonzero(col.def_levels))
                        assert o.num_non_null == nn, (rg, name)
                        got = ctx.d2h_array(o.values, nn * o.value_size)
                        assert np.array_equal(got, col.data[:nn * o.value_size]), (rg, name, "values")
                    if rg in (0, nrg - 1):
                        for ci in range(ncols):
                            cd = pq.reader.ColumnData(cols[ci][0], cols[ci][1:], batch.chunk_out((rg - a) * ncols + ci), [], ctx)
                            assert_chunk(cd, oracle_chunk(fr, rg, ci), where=f"rg{rg} c{ci}")
            assert seen == [(r, r + per_range) for r in range(0, nrg, per_range)]
            # one pinned payload block per slot (1/8 headroom, 2 MiB granules) + one 2 MiB block of
            # plan tables, however many ranges passed
            bound = slots * (((biggest + biggest // 8 + (2 << 20) - 1) // (2 << 20)) * (2 << 20) + (2 << 20))
            assert 0 < st.pinned_bytes() <= bound, (st.pinned_bytes(), bound)
            assert total >= 4 * st.pinned_bytes(), (total, st.pinned_bytes())  # the file is several rings
    finally:
        st.close()
        f.close()
