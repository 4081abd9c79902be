"""The C-ABI library (CPU only, no compute calls): it loads, exports every function declared in
include/pqhip.h, and its host-side page walker (thrift, CRC, codecs) matches the oracle walker
page for page, byte for byte."""
import ctypes
import os
import re

import numpy as np
import pytest

import fixtures
from conftest import ROOT
from oracle import oracle as O


def _declared_functions():
    text = open(os.path.join(ROOT, "include", "pqhip.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(pqh_[a-z0-9_]+)\s*\(", text)))


def test_exports_every_declared_symbol(pq):
    from parquet_go_amd import _lib

    L = ctypes.CDLL(_lib.hip_path())
    names = _declared_functions()
    assert len(names) >= 35
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    bound = {p[0] for p in pq.native.PROTOTYPES}
    assert set(names) == bound, set(names) ^ bound


def test_abi_version_and_devices(pq):
    L = pq._lib.hip()
    assert L.pqh_abi_version() == pq.native.ABI_VERSION == 8
    n = pq.native.device_count()
    assert n >= 0


def test_no_device_context_raises(pq):
    if pq.native.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(pq.native.PqhError):
        pq.native.Context(0)


def _walk_compare(pq, data, crc=False):
    f = pq.native.File(data)
    fr = O.FileReader(data)
    assert f.num_row_groups == len(fr.row_groups)
    assert f.num_rows == fr.num_rows
    cols = f.columns()
    assert [c[0] for c in cols] == [c.path for c in fr.columns]
    assert [(c[3], c[4]) for c in cols] == [(c.max_def, c.max_rep) for c in fr.columns]
    hb = f.load(0, f.num_row_groups, list(range(len(cols))), validate_crc=crc)
    payload = hb.payload()
    pages = hb.pages()
    for k, ch in enumerate(hb.chunks()):
        rg, ci = divmod(k, len(cols))
        och = fr.read_chunk(rg, ci, validate_crc=crc)
        assert (ch.host_status != 0) == (och.status != 0), (rg, ci, ch.host_status, och.status)
        if och.status:
            continue
        mine = [pages[p] for p in range(ch.first_page, ch.first_page + ch.num_pages)]
        want = ([("dict", och.dict_page)] if och.dict_page is not None else []) + [("data", p) for p in och.pages]
        assert len(mine) == len(want), (rg, ci)
        for pg, (kind, w) in zip(mine, want):
            img = payload[pg.image_offset: pg.image_offset + pg.image_len].tobytes()
            if kind == "dict":
                assert pg.page_type == O.DICTIONARY_PAGE
                continue
            assert pg.page_type == w.page_type and pg.num_values == w.num_values and pg.encoding == w.encoding
            assert (pg.def_levels_byte_length, pg.rep_levels_byte_length) == (w.def_len, w.rep_len)
            assert img == w.image
    return hb


@pytest.mark.parametrize("v2", [False, True])
@pytest.mark.parametrize("codec", [0, 1, 2])
def test_host_walker_generated(pq, v2, codec):
    data = fixtures.flat_all_types(n=6000, v2=v2, codec=codec, page=16 * 1024, rows_per_group=2500, crc=True)
    hb = _walk_compare(pq, data, crc=True)
    assert hb.num_pages > 40


@pytest.mark.parametrize("version", ["1.0", "2.0"])
@pytest.mark.parametrize("compression", ["NONE", "SNAPPY", "GZIP"])
def test_host_walker_pyarrow(pq, version, compression):
    _walk_compare(pq, fixtures.pyarrow_file(n=5000, version=version, compression=compression))


def test_host_walker_nested(pq):
    _walk_compare(pq, fixtures.nested_list_map(n=2000, v2=True))


def test_host_crc_mismatch(pq):
    data = bytearray(fixtures.flat_c2_like(n=3000, v2=False))
    # flip a byte inside the first data page's payload: CRC is not written by default -> no error
    f = pq.native.File(bytes(data))
    hb = f.load(0, 1, [1], validate_crc=True)
    assert hb.chunks()[0].host_status == 0


def test_snappy_roundtrip_against_pyarrow(pq):
    """Our SNAPPY compressor output is decodable by pyarrow's snappy and vice versa (the codec
    is outside the reference's tests: compress_test.go:11-32 is a round trip only)."""
    import pyarrow as pa

    rng = np.random.default_rng(0)
    blob = bytes(rng.integers(0, 8, 200000).astype(np.uint8)) + b"abc" * 10000
    data = fixtures.W.flat([("s", fixtures.W.Column(fixtures.W.BYTE_ARRAY, [blob[i:i + 50] for i in range(0, 60000, 50)],
                                                    use_dict=False), 0)], 1000, codec=1)
    fr = O.FileReader(data)
    assert fr.read_chunk(0, 0).status == 0  # pyarrow decompressed our snappy
    comp = pa.compress(blob, codec="snappy", asbytes=True)
    assert len(comp) < len(blob)


@pytest.mark.parametrize("depth", [1, 9, 17, 32])
def test_deep_schema_rep_def(pq, depth):
    """readColumnSchema / readGroupSchema's levels (schema.go:893-990) for chains of repeated groups
    up to PQH_MAX_NEST deep: max_def, max_rep and every repeated node's definition level (what the
    nesting outputs need) equal the oracle's schema walk."""
    data, D = fixtures.deep_repeated(n=40, depth=depth, seed=depth)
    fr = O.FileReader(data)
    f = pq.native.File(data)
    c = fr.columns[0]
    assert c.rep_def == tuple(D) and c.max_rep == depth
    assert f.columns()[0][3:] == (c.max_def, c.max_rep)
    assert f.rep_def(0) == tuple(D)
    _walk_compare(pq, data)
