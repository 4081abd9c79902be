"""The reference's own corrupt / foreign-writer files (tests/golden/fuzz, extracted by
tests/golden/make_fuzz_fixtures.py from the byte-string literals of fuzz_test.go:11-47,
type_dict_test.go:33-177, packed_array_test.go:61, deltabp_decoder_test.go:5-297,
chunk_reader_test.go:5-22, page_v1_test.go:5, type_bytearray_test.go:14-36, schema_test.go:162,241).

The reference's tests assert only that reading them does not panic (readAllData,
schema_test.go:388-403).  Here they pin the host boundary and the state machines against the
oracle: NewFileReader fails or succeeds alike (thrift footer, schema), every chunk ends with the
same (status, phase, index) -- walker, codec, page-load and readValues errors in the reference's
order -- and NextRow produces the same rows and errors call by call."""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O
from parity import assert_chunk, oracle_chunk

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fuzz")
MANIFEST = json.load(open(os.path.join(HERE, "manifest.json")))["fixtures"]
IDS = [m["test"] for m in MANIFEST]


def _data(m):
    if "data" in m:  # (mutants from test_host_fuzz)
        return m["data"]
    d = open(os.path.join(HERE, m["file"]), "rb").read()
    assert len(d) == m["length"]
    return d


def _open_both(pq, data):
    """(oracle FileReader or None, product File or None): both must accept or both reject."""
    try:
        fr = O.FileReader(data)
    except O.FileError:
        fr = None
    try:
        f = pq.native.File(data)
    except pq.native.PqhError:
        f = None
    assert (fr is None) == (f is None), f"NewFileReader: oracle {'fails' if fr is None else 'opens'}, product differs"
    return fr, f


@pytest.mark.parametrize("m", MANIFEST, ids=IDS)
def test_fixture_footer_schema_and_walk(pq, m):
    """CPU: the footer / schema outcome, the column list with its levels, the row groups, the column
    checks of readRowGroupData and the host page walk agree with the oracle (no crash either way)."""
    data = _data(m)
    fr, f = _open_both(pq, data)
    if fr is None:
        return
    cols = f.columns()
    assert [(c[0], c[1], c[3], c[4]) for c in cols] == \
        [(c.path, c.physical_type, c.max_def, c.max_rep) for c in fr.columns]
    assert f.num_row_groups == len(fr.row_groups) and f.num_rows == fr.num_rows
    for rg in range(f.num_row_groups):
        assert f.row_group_num_rows(rg) == fr.row_group_num_rows(rg)
        for ci in range(len(cols)):
            for sel in (True, False):
                assert f.chunk_check(rg, ci, sel) == fr.chunk_check(rg, ci, sel), (rg, ci, sel)
    hb = f.load(0, f.num_row_groups, list(range(len(cols))))
    for k, ch in enumerate(hb.chunks()):
        och = fr.read_chunk(*divmod(k, len(cols)))
        data_pages = [p for p in hb.pages()[ch.first_page:ch.first_page + ch.num_pages] if p.page_type != O.DICTIONARY_PAGE]
        if ch.host_status == pq.native.UNSUPPORTED_CODEC:
            # a registered codec the library does not decode (ZSTD): handed back before any page, the
            # shim's reference readChunk gives the oracle's outcome (test_codec_registry.py)
            codec = fr.row_groups[k // len(cols)][1][k % len(cols)][3][4]
            assert codec in O.DEFAULT_CODECS and codec not in (0, 1, 2) and ch.num_pages == 0, (k, codec)
            continue
        if ch.host_status:  # the walk stopped at a page the oracle cannot read either (or earlier)
            assert och.status != 0 and len(och.pages) <= len(data_pages), (k, ch.host_status, och.status)
            if len(och.pages) == len(data_pages):  # stopped at the same page: the same error
                assert och.status == ch.host_status, (k, ch.host_status, och.status)
        if och.status == 0:
            assert ch.host_status == 0 and len(data_pages) == len(och.pages)
    hb.close()
    f.close()


@pytest.fixture(scope="module")
def ctx(pq):
    return pq.native.Context(0)


@pytest.mark.gpu
@pytest.mark.parametrize("m", MANIFEST, ids=IDS)
def test_fixture_decode_parity(pq, ctx, m):
    """GPU: every chunk's result equals the oracle's -- the exact (status, phase, index) of its first
    error in the reference's order, or its values and levels bit for bit."""
    data = _data(m)
    fr, f = _open_both(pq, data)
    if fr is None:
        return
    ncols = len(f.columns())
    res = pq.reader.decode_chunks(ctx, f, 0, f.num_row_groups, list(range(ncols)))
    for k, col in enumerate(res):
        rg, ci = divmod(k, ncols)
        assert col.status != pq.native.NOT_IMPLEMENTED
        assert_chunk(col, oracle_chunk(fr, rg, ci), where=f"{m['test']} rg{rg} {col.path}")
    f.close()


@pytest.mark.gpu
@pytest.mark.parametrize("m", MANIFEST, ids=IDS)
def test_fixture_next_row(pq, ctx, m):
    """GPU: reading every row as readAllData does (NextRow until the file's row count or an error)
    never crashes, and every NextRow call returns the row or error status the oracle-driven
    assembly returns (test_records.oracle_next_rows)."""
    from test_records import _norm, error_outcome, oracle_next_rows

    data = _data(m)
    fr, f = _open_both(pq, data)
    if fr is None:
        return
    f.close()
    want = oracle_next_rows(data)
    r = pq.reader.FileReader(data, ctx=ctx)
    got = []
    while len(got) < len(want) + 1:
        try:
            got.append(r.NextRow())
        except EOFError:
            break
        except (pq.reader.DecodeError, pq.records.RecordError) as e:
            got.append(error_outcome(e))
    r.close()
    assert [_norm(g) for g in got] == [_norm(w) for w in want]
