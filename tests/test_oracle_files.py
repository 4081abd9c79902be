"""Pin the oracle on whole files (CPU only): oracle decode == pyarrow 25 (independent decoder) on
spec-conforming files, == the generator's inputs, and reproduces the reference's documented
quirks."""
import io

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc
import pyarrow.parquet as pqa
import pytest

import fixtures
from oracle import oracle as O
from parity import oracle_chunk

W = fixtures.W


def _pa_values(arr, path):
    """Non-null leaf values of a pyarrow column, in order."""
    arr = arr.combine_chunks() if hasattr(arr, "combine_chunks") else arr
    parts = path.split(".")
    if pa.types.is_map(arr.type):
        arr = arr.keys if parts[-1] == "key" else arr.items
    elif pa.types.is_list(arr.type):
        arr = pc.list_flatten(arr)
    return arr.filter(arr.is_valid())


def _compare(col_phys, exp, vals):
    if col_phys in (O.INT32, O.INT64, O.FLOAT, O.DOUBLE):
        dt = {O.INT32: np.int32, O.INT64: np.int64, O.FLOAT: np.float32, O.DOUBLE: np.float64}[col_phys]
        got = np.frombuffer(exp.values, dtype=dt)
        want = np.asarray(vals.to_numpy(zero_copy_only=False), dtype=dt)
        assert got.tobytes() == want.tobytes()
    elif col_phys == O.BOOLEAN:
        assert np.frombuffer(exp.values, np.uint8).tolist() == [int(b) for b in vals.to_pylist()]
    elif col_phys == O.FIXED_LEN_BYTE_ARRAY:
        want = b"".join(vals.to_pylist())
        assert exp.values + exp.data == want  # (data: chunks with DELTA_BYTE_ARRAY pages)
    elif col_phys == O.BYTE_ARRAY:
        want = [v if isinstance(v, bytes) else v.encode() for v in vals.to_pylist()]
        got = [exp.data[exp.offsets[i]:exp.offsets[i + 1]] for i in range(len(exp.offsets) - 1)]
        assert got == want


def _check_file(data):
    fr = O.FileReader(data)
    tbl = pqa.read_table(io.BytesIO(data))
    checked = 0
    for ci, col in enumerate(fr.columns):
        if col.physical_type == O.INT96:
            continue
        top = col.path.split(".")[0]
        per_rg = []
        for rg in range(len(fr.row_groups)):
            e = oracle_chunk(fr, rg, ci)
            if e.status:
                per_rg = None
                break
            per_rg.append(e)
        if per_rg is None:
            continue
        merged = per_rg[0]
        for e in per_rg[1:]:
            merged.values += e.values
            if e.offsets is not None:
                merged.offsets = np.concatenate([merged.offsets, e.offsets[1:] + len(merged.data)])
                merged.data += e.data
        _compare(col.physical_type, merged, _pa_values(tbl[top], col.path))
        checked += 1
    return checked


@pytest.mark.parametrize("v2", [False, True])
@pytest.mark.parametrize("codec", [0, 1, 2])
def test_oracle_vs_pyarrow_generated(v2, codec):
    data = fixtures.flat_all_types(n=8000, v2=v2, codec=codec, page=16 * 1024, rows_per_group=3000)
    assert _check_file(data) >= 15


@pytest.mark.parametrize("version", ["1.0", "2.0"])
@pytest.mark.parametrize("compression", ["NONE", "GZIP"])
def test_oracle_vs_pyarrow_written(version, compression):
    data = fixtures.pyarrow_file(n=6000, version=version, compression=compression)
    # V2 + codec: pyarrow marks incompressible pages is_compressed=false -> the reference fails them
    assert _check_file(data) >= (8 if version == "1.0" or compression == "NONE" else 2)


def test_oracle_nested():
    data = fixtures.nested_list_map(n=3000)
    assert _check_file(data) == 3


def test_oracle_int96_vs_input():
    rng = np.random.default_rng(3)
    v = rng.integers(0, 256, (1000, 12), dtype=np.uint8)
    data = W.flat([("t", W.Column(W.INT96, v, use_dict=False), W.REQUIRED)], 1000)
    e = oracle_chunk(O.FileReader(data), 0, 0)
    assert e.status == 0 and e.values == v.tobytes()


def test_oracle_hybrid_roundtrip():
    """hybrid_test.go:34-61 shape: encoder->decoder round trip at every width."""
    rng = np.random.default_rng(5)
    for w in range(0, 33):
        hi = 2**w if w < 31 else 2**31
        vals = rng.integers(0, hi, 8 * 1024 + 5).astype(np.int64).astype(np.int32) if w else np.zeros(8197, np.int32)
        enc = W.hybrid_encode(w, vals)
        st, out = O.hybrid_decode(w, enc, len(vals))
        assert st == 0 and np.array_equal(out, vals), w


def test_oracle_delta_roundtrip():
    """deltabp_test.go:21-52 shape (8197 random int32) plus int64."""
    rng = np.random.default_rng(6)
    v32 = rng.integers(-2**31, 2**31 - 1, 8197).astype(np.int32)
    st, out, vc = O.delta_decode(W.delta_encode(v32, 32), len(v32), 32)
    assert st == 0 and vc == len(v32) and np.array_equal(out, v32)
    v64 = rng.integers(-2**62, 2**62, 8197)
    st, out, vc = O.delta_decode(W.delta_encode(v64, 64), len(v64), 64)
    assert st == 0 and np.array_equal(out, v64)


@pytest.mark.parametrize("n,ok", [(1, True), (2, True), (128, True), (129, False), (130, True), (257, False),
                                  (300, True)])
def test_oracle_delta_readahead_quirk(n, ok):
    """the decoder reads delta[n-1]; at (n-1) % 128 == 0 that needs a block
    header the writer never emits -> the reference fails (deltabp_decoder.go:124-128)."""
    v = np.arange(n, dtype=np.int64) * 3 + 11
    st, out, _ = O.delta_decode(W.delta_encode(v, 64), n, 64)
    if ok:
        assert st == 0 and np.array_equal(out, v)
    else:
        assert st == 1 and len(out) == n - 1  # io.EOF at position n-1


def test_oracle_v2_is_compressed_ignored():
    """page_v2.go:125: pyarrow writes is_compressed=false for incompressible V2 pages; the
    reference decompresses them anyway and fails the chunk."""
    rng = np.random.default_rng(1)
    tbl = pa.table({"i": pa.array(rng.integers(0, 300, 20000).astype(np.int32))})
    buf = io.BytesIO()
    pqa.write_table(tbl, buf, data_page_version="2.0", compression="SNAPPY", data_page_size=4096)
    fr = O.FileReader(buf.getvalue())
    assert fr.read_chunk(0, 0).status == O.ERR_DECOMPRESS
