"""INTEGRATION.md's cgo shim (gpuPageReader) inside the reference's page walk, on the CPU.

readPages (chunk_reader.go:182-263) reads each PageHeader from the same reader the page readers
read their blocks from, so a shim `read` must consume exactly CompressedPageSize bytes (what
readPageBlock consumes, chunk_reader.go:161-180, page_v1.go:96) and its `index` must name the i-th
DATA page of the chunk in the batch (the dictionary page, read by the reference's dictPageReader,
comes first).  tests/shim_adapter.py restates the walk over an offset reader; here the shim adapter
(readValues from the host batch's page images, decoded by the oracle) must walk every chunk exactly
as the oracle's dataPageReaderV1/V2 do -- same pages, same readValues results call by call, same
error at the same page -- on multi-page V1 / V2 / dictionary / SNAPPY / GZIP / nested / pyarrow
chunks and on corrupted files.  The GPU variant (readValues = pqh_batch_page_read) is in
test_gpu_compat.py."""
import numpy as np
import pytest

import fixtures
from oracle import oracle as O
from shim_adapter import OraclePage, Shim, ShimPage, read_pages


def files():
    yield "v1-dict", fixtures.flat_all_types(n=4000, v2=False, page=4 * 1024, rows_per_group=2000)
    yield "v2-dict", fixtures.flat_all_types(n=4000, v2=True, page=4 * 1024, rows_per_group=2000)
    yield "v2-snappy", fixtures.flat_all_types(n=4000, v2=True, codec=O.SNAPPY, page=4 * 1024, rows_per_group=4000)
    yield "v1-gzip", fixtures.flat_all_types(n=3000, v2=False, codec=O.GZIP, page=4 * 1024, rows_per_group=3000)
    yield "nested", fixtures.nested_list_map(n=1500, v2=False)
    yield "pyarrow-1.0", fixtures.pyarrow_file(n=6000, version="1.0", compression="SNAPPY", page=2048)
    yield "pyarrow-2.0", fixtures.pyarrow_file(n=6000, version="2.0", compression="NONE", page=2048)


SIZES = (7, 100, 1 << 30)


def _raw(x):  # bytes as they are (np.asarray(b"") would be a one-byte S1 array), arrays by their bytes
    return bytes(x) if isinstance(x, (bytes, bytearray)) else np.ascontiguousarray(x).tobytes()  # readValues(size) calls per page: the page read in three calls


def _as_arrays(v, desc):
    """Byte-array values as (offsets, bytes).  A FIXED_LEN_BYTE_ARRAY chunk with DELTA_BYTE_ARRAY
    pages comes off the device as offsets + bytes for all its pages (its dictionary pages too); the
    oracle gives such a page's fixed-width values as they are -- the same []byte values either way."""
    if isinstance(v, tuple):
        return np.asarray(v[0], np.int64), _raw(v[1])
    raw = _raw(v)
    w = desc[1]  # type_length
    return np.arange(0, len(raw) + 1, w, dtype=np.int64), raw


def walk_both(pq, data, backend="host", batch_for=None, crc=False):
    """Returns the number of data pages compared."""
    fr = O.FileReader(data)
    f = pq.native.File(data)
    ncols = len(f.columns())
    hb = f.load(0, f.num_row_groups, list(range(ncols)), validate_crc=crc)
    batch = batch_for(hb) if batch_for else None
    compared = 0
    for k in range(len(hb.chunks())):
        rg, ci = divmod(k, ncols)
        desc = fr.columns[ci].desc()
        want, wdict, werr = read_pages(data, fr, rg, ci, lambda i, d: OraclePage(desc, d), validate_crc=crc)
        shim = Shim(hb, k, desc, backend=backend, batch=batch)
        got, gdict, gerr = read_pages(data, fr, rg, ci, lambda i, d: ShimPage(shim, i), validate_crc=crc)
        where = f"rg {rg} col {ci}"
        assert len(got) == len(want), f"{where}: {len(got)} pages vs {len(want)}"
        assert (gerr is None) == (werr is None), f"{where}: {gerr} vs {werr}"
        if werr is not None:
            assert (gerr.status, gerr.page) == (werr.status, werr.page), f"{where}: {gerr} vs {werr}"
            continue  # readChunk failed: the row group fails, no page is read (chunk_reader.go:394-400)
        for i, (g, w) in enumerate(zip(got, want)):
            assert g.num_values() == w.num_values(), f"{where} page {i}"
            for size in SIZES:
                a, b = g.read_values(size), w.read_values(size)
                assert a[:2] == b[:2], f"{where} page {i}: status {a[:2]} vs {b[:2]}"
                if a[0]:
                    break
                for x, y in zip(a[2:], b[2:]):
                    if isinstance(x, tuple) or isinstance(y, tuple):
                        x, y = _as_arrays(x, desc), _as_arrays(y, desc)
                        assert np.array_equal(x[0], y[0]) and bytes(x[1]) == bytes(y[1]), f"{where} page {i}"
                    elif x is None or y is None:
                        assert x is None and y is None, f"{where} page {i}"
                    elif isinstance(x, list) or isinstance(y, list):  # boxed with nil INT96 values
                        assert x == y, f"{where} page {i}"
                    else:
                        assert _raw(x) == _raw(y), f"{where} page {i}"
            compared += 1
    hb.close()
    f.close()
    return compared


@pytest.mark.parametrize("name", [n for n, _ in files()])
def test_shim_walk_matches_reference_pages(pq, name):
    data = dict(files())[name]
    assert walk_both(pq, data) > 8


def test_shim_walk_corrupt_files(pq):
    """Bytes flipped inside chunks (headers, levels, values, compressed blocks): the walk fails at
    the same page with the same status, or reads the same pages and values."""
    rng = np.random.default_rng(17)
    base = fixtures.flat_all_types(n=3000, v2=True, codec=O.SNAPPY, page=4 * 1024, rows_per_group=3000, crc=True)
    fr = O.FileReader(base)
    errors = 0
    for trial in range(24):
        buf = bytearray(base)
        ci = trial % len(fr.columns)
        md = fr.row_groups[0][1][ci][3]
        lo = md.get(11, md[9])
        for _ in range(int(rng.integers(1, 3))):
            buf[lo + int(rng.integers(0, md[7]))] ^= 1 << int(rng.integers(0, 8))
        try:
            O.FileReader(bytes(buf))
        except O.FileError:
            continue
        walk_both(pq, bytes(buf), crc=bool(trial & 1))
        fr2 = O.FileReader(bytes(buf))
        errors += fr2.read_chunk(0, ci, validate_crc=bool(trial & 1)).status != 0
    assert errors >= 4


def test_consuming_nothing_desynchronises_the_walk(pq):
    """The r03 shim's read consumed nothing from r: the next readThrift then parses page-body bytes
    as a header, so a multi-page chunk cannot walk (the bug the byte accounting fixes)."""

    class NoConsume(ShimPage):
        def read(self, r, ph, codec, crc):
            return self.shim.load_error(self.ordinal)

    data = fixtures.flat_all_types(n=4000, v2=False, page=4 * 1024, rows_per_group=4000)
    fr = O.FileReader(data)
    f = pq.native.File(data)
    hb = f.load(0, 1, list(range(len(fr.columns))))
    broken = multi = 0
    for ci in range(len(fr.columns)):
        desc = fr.columns[ci].desc()
        want, _, werr = read_pages(data, fr, 0, ci, lambda i, d: OraclePage(desc, d))
        assert werr is None
        if len(want) < 2:
            continue
        multi += 1
        shim = Shim(hb, ci, desc)
        got, _, gerr = read_pages(data, fr, 0, ci, lambda i, d: NoConsume(shim, i))
        broken += gerr is not None or len(got) != len(want)
    assert broken == multi >= 4
