"""The input generator (libpqgen, tooling): its bulk paths and its streaming writer produce the same
bytes as its general page-cut loop and one-shot write, and the mixed workload's row groups
regenerate exactly -- so the full-size tests and the bench decode files in the reference writer's
layout and can check every chunk against the seeded input."""
import numpy as np
import pytest

from test_records import _pkg


def _flat_cases():
    pq = _pkg()
    W, D = pq.writer, pq.datasets
    rng = np.random.default_rng(5)
    n = 300_001
    yield "c2", D.c2_columns(n, 10), 70_000, {}
    yield "c3", [("ts", W.Column(W.INT64, D.c3_values(n, 20), encoding=W.DELTA_BINARY_PACKED, use_dict=False),
                  W.REQUIRED)], 100_000, {}
    # DELTA int32 pages whose size estimate lands on (n - 1) % 128 == 0 (one more value), small pages
    for page in (129 * 4, 257 * 4, 1000):
        v = rng.integers(-2**31, 2**31 - 1, 50_000).astype(np.int32)
        yield f"delta32-{page}", [("d", W.Column(W.INT32, v, encoding=W.DELTA_BINARY_PACKED, use_dict=False),
                                   W.REQUIRED)], 20_000, {"max_page_size": page}
    yield "flba-int96", [("f", W.Column(W.FIXED_LEN_BYTE_ARRAY, rng.integers(0, 256, (n, 7), dtype=np.uint8),
                                        type_length=7, use_dict=False), W.REQUIRED),
                         ("t", W.Column(W.INT96, rng.integers(0, 256, (n, 12), dtype=np.uint8), use_dict=False),
                          W.REQUIRED)], 150_000, {"max_page_size": 64 * 1024}


@pytest.mark.parametrize("name", [c[0] for c in _flat_cases()])
@pytest.mark.parametrize("v2", [False, True])
def test_fast_paths_match_page_cut_loop(name, v2):
    W = _pkg().writer
    _, cols, per, kw = next(c for c in _flat_cases() if c[0] == name)
    n = cols[0][1].num_slots
    rg = [min(per, n - i) for i in range(0, n, per)]
    schema = W.flat_schema(cols)
    fast = W.write(schema, [c for _, c, _ in cols], rg, v2=v2, as_array=True, **kw)
    slow = W.write(schema, [c for _, c, _ in cols], rg, v2=v2, as_array=True, fast_paths=False, **kw)
    assert np.array_equal(fast, slow)


def test_stream_writer_equals_write():
    pq = _pkg()
    W, D = pq.writer, pq.datasets
    rows, rgs = 1_000_003, 6
    data = D.mixed(rows=rows, row_groups=rgs, batch=4)
    per = -(-rows // rgs)
    sizes = [min(per, rows - g * per) for g in range(rgs)]
    parts = [D.mixed_row_group(g, n) for g, n in enumerate(sizes)]
    merged = []
    for ci in range(7):
        cs = [p[ci][1] for p in parts]
        c0 = cs[0]
        raw = np.concatenate([c.data for c in cs])
        vals = raw.reshape(-1, 16) if c0.ptype == W.FIXED_LEN_BYTE_ARRAY else \
            raw.view({W.INT32: np.int32, W.INT64: np.int64, W.FLOAT: np.float32, W.DOUBLE: np.float64}.get(c0.ptype, np.uint8))
        dl = np.concatenate([c.def_levels for c in cs]) if c0.def_levels is not None else None
        merged.append(W.Column(c0.ptype, vals, def_levels=dl, encoding=c0.encoding, use_dict=c0.use_dict,
                               type_length=c0.type_length))
    whole = W.write(W.flat_schema(parts[0]), merged, sizes, v2=True, as_array=True)
    assert np.array_equal(whole, data)


def test_mixed_row_groups_regenerate():
    D = _pkg().datasets
    a = D.mixed_row_group(7, 200_000, threads=1)
    b = D.mixed_row_group(7, 200_000, threads=8)
    c = D.mixed_row_group(7, 150_000, threads=3)  # a prefix of the row group: the same values
    for (na, ca, _), (_, cb, _), (_, cc, _) in zip(a, b, c):
        assert np.array_equal(ca.data, cb.data), na
        if ca.def_levels is not None:
            assert np.array_equal(ca.def_levels, cb.def_levels)
            nn = int(cc.def_levels.sum())
            assert np.array_equal(cc.data, ca.data[:len(cc.data)]) and len(cc.data) == nn * 8
        else:
            assert np.array_equal(cc.data, ca.data[:len(cc.data)]), na
    ts = a[6][1].data.view(np.int64)
    assert np.all(np.diff(ts) >= 1_000_000) and np.all(np.diff(ts) < 1_000_000 + 4096)
    assert 0.005 < 1 - a[3][1].def_levels.mean() < 0.015  # ~1% nulls


def test_mixed_file_reads_in_pyarrow():
    """The mixed workload file is a valid Parquet file: pyarrow (an independent reader) returns the
    seeded columns of every row group."""
    import pyarrow as pa
    import pyarrow.parquet as pqa

    D = _pkg().datasets
    rows = 300_000
    data = D.mixed(rows=rows, row_groups=6, batch=4)
    pf = pqa.ParquetFile(pa.BufferReader(pa.py_buffer(data.tobytes())))
    assert pf.metadata.num_row_groups == 6 and pf.metadata.num_rows == rows
    for rg, n in enumerate(D.mixed_sizes(rows, 6)):
        t = pf.read_row_group(rg)
        for name, col, _ in D.mixed_row_group(rg, n):
            got = t.column(name).combine_chunks()
            if name == "c_uuid":
                assert np.frombuffer(got.buffers()[1], np.uint8)[:16 * n].tobytes() == col.data.tobytes()
            elif name == "c_double":
                valid = col.def_levels.astype(bool)
                assert np.array_equal(np.asarray(got.is_valid()), valid)
                assert np.array_equal(got.drop_null().to_numpy(), col.data.view(np.float64))
            elif name == "c_bool":
                assert np.array_equal(got.to_numpy(zero_copy_only=False).astype(np.uint8), col.data)
            else:
                assert got.to_numpy().tobytes() == col.data.tobytes(), name
