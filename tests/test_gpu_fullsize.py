"""Full-size round trips at the BASELINE.json configurations: the generator's
seeded column data is written in the reference writer's layout, decoded on the GPU in one batch,
and every decoded chunk must equal the slice of the input it was written from -- values, definition
levels, byte-array offsets and bytes, bit for bit.  The oracle checks the decoders at sizes it
finishes in seconds (test_gpu_parity.py); these check the same kernels at the sizes the bench runs.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(pq):
    return pq.native.Context(0)


def _decode(pq, ctx, data):
    f = pq.native.File(data)
    ncols = len(f.columns())
    hb = f.load(0, f.num_row_groups, list(range(ncols)))
    b = pq.native.Batch.from_host(ctx, hb)
    b.run()
    b.sync()
    rows = [f.row_group_num_rows(rg) for rg in range(f.num_row_groups)]
    return f, hb, b, ncols, rows


def _fixed_chunks(pq, ctx, b, ncols, rows, ci, col, size):
    """Compare column ci chunk by chunk with the written Column (fixed-width values)."""
    vstart = sstart = 0
    for rg, n in enumerate(rows):
        o = b.chunk_out(rg * ncols + ci)
        assert o.status == pq.native.OK, (ci, rg, o.status)
        if col.def_levels is not None:
            want_def = col.def_levels[sstart:sstart + n]
            got_def = ctx.d2h_array(o.def_levels, n)
            assert np.array_equal(got_def, want_def), (ci, rg, "def levels")
            nn = int(np.count_nonzero(want_def))
        else:
            nn = n
        assert o.num_non_null == nn and o.value_size == size, (ci, rg)
        got = ctx.d2h_array(o.values, nn * size)
        assert np.array_equal(got, col.data[vstart * size:(vstart + nn) * size]), (ci, rg, "values")
        vstart += nn
        sstart += n


def test_c1_full(pq, ctx):
    """C1 (BASELINE configs[0]) at full size: 10M required INT32 dictionary values (K = 4096, index
    width bits.Len(4096) = 13, page_v1.go:184-191), reference-writer V1 pages of ~258k values whose
    index stream is ONE bit-packed run (hybrid_encoder.go:55-70) spanning many tiles.  Every chunk
    must equal the oracle's decode bit for bit, and the seeded input."""
    import numpy as np

    from oracle import oracle as O
    from parquet_go_amd import datasets

    rows = 10_000_000
    data = datasets.c1(rows=rows, seed=1)
    f, hb, b, ncols, rg_rows = _decode(pq, ctx, data)
    assert ncols == 1 and sum(rg_rows) == rows
    pages = hb.pages()
    big = [p for p in pages if p.page_type != O.DICTIONARY_PAGE]
    assert max(p.num_values for p in big) > 200_000  # the reference writer's 1 MiB page estimate
    rng = np.random.default_rng(1)
    dictionary = rng.integers(-2**31, 2**31 - 1, 4096).astype(np.int32)
    want_all = dictionary[np.random.default_rng(2).integers(0, 4096, rows)]
    fr = O.FileReader(data)
    start = 0
    for rg, n in enumerate(rg_rows):
        o = b.chunk_out(rg)
        assert o.status == pq.native.OK and o.num_non_null == n, rg
        got = ctx.d2h_array(o.values, n * 4)
        res = O.decode_chunk(fr.read_chunk(rg, 0))
        assert all(r.status == 0 for r in res)
        assert got.tobytes() == b"".join(r.values for r in res), (rg, "oracle")
        assert np.array_equal(got.view(np.int32), want_all[start:start + n]), (rg, "input")
        start += n
    b.close()
    hb.close()


def test_c1_pyarrow_variant(pq, ctx):
    """The pyarrow-written C1 variant: dictionary indices of width 12 in mixed
    RLE / bit-packed runs, 10M rows, V1 pages."""
    import io

    import numpy as np
    import pyarrow as pa
    import pyarrow.parquet as pqa

    rows = 10_000_000
    rng = np.random.default_rng(5)
    dictionary = rng.integers(-2**31, 2**31 - 1, 4000).astype(np.int32)
    idx = rng.integers(0, 4000, rows)
    idx[rng.random(rows) < 0.3] = 7  # runs of repeats -> RLE runs between bit-packed ones
    idx = np.where(np.repeat(rng.random(rows // 100) < 0.2, 100)[:rows], 11, idx)
    vals = dictionary[idx]
    buf = io.BytesIO()
    pqa.write_table(pa.table({"v": vals}), buf, row_group_size=2_500_000, data_page_version="1.0",
                    compression="NONE", use_dictionary=True)
    f, hb, b, ncols, rg_rows = _decode(pq, ctx, buf.getvalue())
    start = 0
    for rg, n in enumerate(rg_rows):
        o = b.chunk_out(rg)
        assert o.status == pq.native.OK and o.num_non_null == n, (rg, o.status)
        got = ctx.d2h_array(o.values, n * 4).view(np.int32)
        assert np.array_equal(got, vals[start:start + n]), rg
        start += n
    assert start == rows
    b.close()
    hb.close()


def test_c2_full(pq, ctx):
    """C2: 100M rows x 6 columns, V2, 16 row groups (the bench's default workload)."""
    from parquet_go_amd import datasets, writer as W

    rows = 100_000_000
    cols = datasets.c2_columns(rows, 10)
    data = W.flat(cols, -(-rows // 16), v2=True, as_array=True)
    f, hb, b, ncols, rg_rows = _decode(pq, ctx, data)
    assert f.num_row_groups == 16 and sum(rg_rows) == rows
    for ci, (_, col, _) in enumerate(cols):
        size = 16 if col.ptype == W.FIXED_LEN_BYTE_ARRAY else col.data.itemsize * len(col.data) // max(1, col.num_values)
        _fixed_chunks(pq, ctx, b, ncols, rg_rows, ci, col, size)
    b.close()
    hb.close()


def test_c3_full(pq, ctx):
    """C3: 1,000,000,000 INT64 timestamps, DELTA_BINARY_PACKED 128/4, 128 row groups."""
    from parquet_go_amd import datasets, writer as W

    rows = 1_000_000_000
    ts = datasets.c3_values(rows, 20)
    data = W.flat([("ts", W.Column(W.INT64, ts, encoding=W.DELTA_BINARY_PACKED, use_dict=False), W.REQUIRED)],
                  7_812_500, v2=False, as_array=True)
    f, hb, b, ncols, rg_rows = _decode(pq, ctx, data)
    assert f.num_row_groups == 128
    start = 0
    for rg, n in enumerate(rg_rows):
        o = b.chunk_out(rg)
        assert o.status == pq.native.OK and o.num_non_null == n, rg
        got = ctx.d2h_array(o.values, n, np.int64)
        assert np.array_equal(got, ts[start:start + n]), rg
        start += n
    b.close()
    hb.close()


def test_c5_full(pq, ctx):
    """C5: 50M strings, dictionary pages then DELTA_LENGTH fallback, SNAPPY, 8 row groups."""
    from parquet_go_amd import datasets, writer as W

    rows = 50_000_000
    sdata, soff = datasets.c5_strings(rows, 40)
    col = W.Column(W.BYTE_ARRAY, (sdata, soff), encoding=W.DELTA_LENGTH_BYTE_ARRAY, dict_page_limit=1 << 20)
    data = W.flat([("s", col, W.REQUIRED)], -(-rows // 8), v2=False, codec=W.SNAPPY, as_array=True)
    f, hb, b, ncols, rg_rows = _decode(pq, ctx, data)
    start = 0
    for rg, n in enumerate(rg_rows):
        o = b.chunk_out(rg)
        assert o.status == pq.native.OK and o.num_non_null == n, rg
        offs = ctx.d2h_array(o.offsets, n + 1, np.int64)
        want = soff[start:start + n + 1] - soff[start]
        assert np.array_equal(offs, want), (rg, "offsets")
        got = ctx.d2h_array(o.bytes, int(offs[-1]))
        assert np.array_equal(got, sdata[soff[start]:soff[start + n]]), (rg, "bytes")
        start += n
    b.close()
    hb.close()


@pytest.mark.parametrize("v2", [False, True])
def test_c4_full(pq, ctx, v2):
    """C4: 20M rows of LIST<optional int64> + MAP<string, optional int32>, 4 row groups, data pages
    V1 and V2: levels, values and key strings of every chunk equal the written
    columns."""
    from parquet_go_amd import datasets, writer as W

    rows, rgs = 20_000_000, 4
    schema, cols = datasets.c4_columns(rows, 30)
    per = -(-rows // rgs)
    data = W.write(schema, cols, [min(per, rows - i * per) for i in range(rgs)], v2=v2, as_array=True)
    f, hb, b, ncols, rg_rows = _decode(pq, ctx, data)
    max_def = [3, 2, 3]
    for ci, col in enumerate(cols):
        row_starts = np.flatnonzero(col.rep_levels == 0)
        bounds = list(row_starts[::per]) + [len(col.rep_levels)]
        vstart = 0
        for rg in range(rgs):
            s0, s1 = int(bounds[rg]), int(bounds[rg + 1])
            o = b.chunk_out(rg * ncols + ci)
            assert o.status == pq.native.OK and o.num_values == s1 - s0, (ci, rg)
            d = col.def_levels[s0:s1]
            assert np.array_equal(ctx.d2h_array(o.def_levels, s1 - s0), d), (ci, rg, "def")
            assert np.array_equal(ctx.d2h_array(o.rep_levels, s1 - s0), col.rep_levels[s0:s1]), (ci, rg, "rep")
            nn = int(np.count_nonzero(d == max_def[ci]))
            assert o.num_non_null == nn, (ci, rg)
            if col.offsets is None:
                size = 8 if col.ptype == W.INT64 else 4
                got = ctx.d2h_array(o.values, nn * size)
                assert np.array_equal(got, col.data[vstart * size:(vstart + nn) * size]), (ci, rg, "values")
            else:
                offs = ctx.d2h_array(o.offsets, nn + 1, np.int64)
                assert np.array_equal(offs, col.offsets[vstart:vstart + nn + 1] - col.offsets[vstart]), (ci, rg)
                got = ctx.d2h_array(o.bytes, int(offs[-1]))
                assert np.array_equal(got, col.data[col.offsets[vstart]:col.offsets[vstart + nn]]), (ci, rg, "bytes")
            vstart += nn
    b.close()
    hb.close()


def test_mixed_1b_full(pq, ctx):
    """north_star's target file: ONE 1,000,000,000-row mixed-encoding file -- C2's six columns
    (int32 / float dictionaries, int64 / double / FLBA(16) / boolean PLAIN, the double optional) plus
    C3's DELTA_BINARY_PACKED timestamps, V2 pages, 128 row groups (datasets.mixed, the reference
    writer's layout) -- decoded in ONE HBM-resident batch.  Every chunk equals the seeded input it
    was written from (values, definition levels), and row groups 0, 64 and 127 equal the oracle's
    decode bit for bit."""
    from oracle import oracle as O
    from parity import assert_chunk, oracle_chunk
    from parquet_go_amd import datasets

    data = datasets.mixed()
    f = pq.native.File(data)
    ncols = len(f.columns())
    assert f.num_row_groups == 128 and f.num_rows == 1_000_000_000 and ncols == 7
    hb = f.load(0, f.num_row_groups, list(range(ncols)))
    b = pq.native.Batch.from_host(ctx, hb)
    hb.close()
    b.run()
    b.sync()
    for rg, n in enumerate(datasets.mixed_sizes()):
        for ci, (name, col, _) in enumerate(datasets.mixed_row_group(rg, n)):
            o = b.chunk_out(rg * ncols + ci)
            assert o.status == pq.native.OK, (rg, name, o.status)
            nn = n
            if col.def_levels is not None:
                assert np.array_equal(ctx.d2h_array(o.def_levels, n), col.def_levels), (rg, name, "def levels")
                nn = int(np.count_nonzero(col.def_levels))
            assert o.num_non_null == nn, (rg, name)
            got = ctx.d2h_array(o.values, nn * o.value_size)
            assert np.array_equal(got, col.data[:nn * o.value_size]), (rg, name, "values")
    fr = O.FileReader(data)
    cols = f.columns()
    for rg in (0, 64, 127):
        for ci in range(ncols):
            cd = pq.reader.ColumnData(cols[ci][0], cols[ci][1:], b.chunk_out(rg * ncols + ci), [], ctx)
            assert_chunk(cd, oracle_chunk(fr, rg, ci), where=f"mixed rg{rg} c{ci}")
    b.close()
    f.close()
