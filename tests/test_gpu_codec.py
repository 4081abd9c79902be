"""Device SNAPPY and GZIP (k_snappy / k_gzip) against the oracle.

* pqh_decompress_pages on its own: hand-built blocks covering every element kind, bulk literals,
  batch-cap boundaries and long chains of tiny overlapping copies; pyarrow-compressed data of
  several kinds; and a seeded mutation fuzzer -- the device's status and bytes must equal
  oracle.snappy_decode (golang/snappy decode.go restated), ErrCorrupt <-> PQH_ERR_DECOMPRESS.
* whole files decoded with the pages of SNAPPY chunks decompressed on the device (plain batches and
  staged end-to-end batches) must equal the oracle's decode chunk by chunk, bit for bit.
* a chunk whose compressed page is corrupt reports PQH_ERR_DECOMPRESS, as the host walker does.
* GZIP: every stream of tests/gzip_blocks.py (valid zlib streams of every level / strategy / flush,
  multistream, header fields, hand-built blocks, each error class, seeded mutants) through k_gzip
  against oracle.gzip_decode (Go's compress/gzip reader restated, compress.go:64-77), status and
  bytes; whole GZIP files decoded with device_gzip against the oracle chunk by chunk.
"""
import numpy as np
import pyarrow as pa
import pytest

import fixtures
from oracle import oracle as O
from parity import assert_chunk, oracle_chunk
from snappy_blocks import edge_blocks, far_copy_block, sample_blocks, uvarint_header_cases

pytestmark = pytest.mark.gpu

DECOMPRESS = 23


@pytest.fixture(scope="module")
def ctx(pq):
    return pq.native.Context(0)


@pytest.fixture(autouse=True)
def every_page_on_the_device(monkeypatch, request):
    """These tests exercise the device codecs on every page of a device-codec chunk, barely
    compressible ones included (the walker's default keeps pages whose values compress to >= 0.95
    of their size on the host route: test_device_codec_skips_incompressible_pages)."""
    if request.node.name.startswith("test_device_codec_skips"):
        return
    monkeypatch.setenv("PQH_DEVICE_CODEC_MAX_RATIO", "0")


@pytest.mark.parametrize("codec", [O.SNAPPY, O.GZIP])
def test_device_codec_skips_incompressible_pages(pq, ctx, codec):
    """Default routing: with device codecs requested, pages whose compressed
    values are >= 0.95 of their size travel decompressed (the host decodes them; the device copies
    the image: codec page codec 0) and the others travel compressed; strings of random bytes are all
    of the first kind (for SNAPPY, C5's random letters too), URL-like strings of the second.  Every chunk equals the oracle either way."""
    W = pq.writer
    rng = np.random.default_rng(11)
    rand = [bytes(rng.integers(0, 256, int(k)).astype(np.uint8)) for k in rng.integers(8, 40, 6000)]
    urls = [b"https://www.example.com/news-%d/item%d?id=%d" % (i % 40, i % 500, i) for i in range(6000)]
    cols = [("r", W.Column(W.BYTE_ARRAY, rand, encoding=W.DELTA_LENGTH_BYTE_ARRAY, use_dict=False), W.REQUIRED),
            ("u", W.Column(W.BYTE_ARRAY, urls, encoding=W.DELTA_LENGTH_BYTE_ARRAY, use_dict=False), W.REQUIRED)]
    data = W.flat(cols, 3000, codec=codec, max_page_size=16 * 1024)
    f = pq.native.File(data)
    hb = f.load(0, f.num_row_groups, [0, 1], device_snappy=True, device_gzip=True)
    kinds = {}
    for cp in hb.codec_pages():
        kinds.setdefault(cp.chunk % 2, set()).add(cp.codec)
    assert kinds[0] == {0} and kinds[1] == {codec}, kinds
    hb.close()
    res = pq.reader.decode_chunks(ctx, f, 0, f.num_row_groups, [0, 1], device_snappy=True, device_gzip=True)
    fr = O.FileReader(data)
    for k, col in enumerate(res):
        assert_chunk(col, oracle_chunk(fr, *divmod(k, 2)), where=f"chunk {k}")
    f.close()


def _device_decompress(pq, ctx, blocks, sizes, codec=O.SNAPPY):
    """Every block as one codec page; returns [(status, bytes)]."""
    N = pq.native
    src, pages, soff, ioff = [], [], 0, 0
    for blk, size in zip(blocks, sizes):
        pad = (-soff) % 64
        src.append(b"\0" * pad + blk)
        soff += pad
        ioff = (ioff + 63) & ~63
        pages.append(N.CodecPage(soff, ioff, len(blk), size, 0, codec, 0, 0))
        soff += len(blk)
        ioff += size
    s = np.frombuffer(b"".join(src) + b"\0" * N.PAYLOAD_PAD, np.uint8).copy()
    ds, dd = ctx.malloc(len(s)), ctx.malloc(ioff + N.PAYLOAD_PAD)
    try:
        ctx.h2d(ds, s.ctypes.data, len(s))
        st = ctx.decompress_pages(pages, ds, dd)
        img = ctx.d2h_array(dd, ioff) if ioff else np.zeros(0, np.uint8)
    finally:
        ctx.free(ds)
        ctx.free(dd)
    return [(st[i], img[p.image_offset:p.image_offset + p.image_len].tobytes()) for i, p in enumerate(pages)]


def _expect(blk, size):
    try:
        raw = O.snappy_decode(blk)
    except O.SnappyCorrupt:
        return DECOMPRESS, None
    return (0, raw) if len(raw) == size else (DECOMPRESS, None)


def _check(pq, ctx, blocks, sizes):
    got = _device_decompress(pq, ctx, blocks, sizes)
    bad = 0
    for i, (blk, size) in enumerate(zip(blocks, sizes)):
        st, raw = _expect(blk, size)
        assert got[i][0] == st, f"block {i}: device status {got[i][0]} vs oracle {st}"
        if st == 0:
            assert got[i][1] == raw, f"block {i}: bytes differ"
        bad += st != 0
    return bad


def test_snappy_edge_blocks(pq, ctx):
    cases = edge_blocks()
    assert _check(pq, ctx, [c[0] for c in cases], [len(c[1]) for c in cases]) == 0


def test_snappy_uvarint_headers(pq, ctx):
    """decodedLen = binary.Uvarint (golang/snappy decode.go:32-36) on the device: 10-byte headers
    with a 10th byte > 1, 11-byte headers and lengths > 2^32 - 1 are ErrCorrupt, non-minimal ones
    valid -- status and bytes equal to the oracle's (and the host walker's, test_codec_oracle.py)."""
    cases = uvarint_header_cases()
    bad = _check(pq, ctx, [c[1] for c in cases], [c[2] for c in cases])
    assert bad == sum(1 for _, b, s in cases if _expect(b, s)[0]) and bad >= 6


def test_snappy_far_copy_offsets(pq, ctx):
    """A 16.2 MiB block whose copy4 offsets reach 2^24 and beyond (k_snap_emit packs
    offsets in 24 bits; such blocks go to k_snappy, which keeps 31): bytes equal to the oracle's,
    beside a small multi-workgroup block in the same launch."""
    blk, raw = far_copy_block()
    assert len(raw) > (1 << 24) + 64
    small = edge_blocks()[1]
    got = _device_decompress(pq, ctx, [blk, small[0]], [len(raw), len(small[1])])
    assert got[0][0] == 0 and got[0][1] == raw
    assert got[1][0] == 0 and got[1][1] == small[1]


def test_snappy_pyarrow_blocks(pq, ctx):
    raws = sample_blocks()
    blocks = [pa.compress(r, codec="snappy", asbytes=True) for r in raws]
    assert _check(pq, ctx, blocks, [len(r) for r in raws]) == 0


def test_snappy_mutation_fuzz(pq, ctx):
    rng = np.random.default_rng(97)
    raws = sample_blocks(seed=9) + [c[1] for c in edge_blocks()]
    blocks, sizes = [], []
    for r in raws:
        comp = pa.compress(r, codec="snappy", asbytes=True) if len(r) else b"\0"
        for k in range(12):
            b = bytearray(comp)
            mode = k % 4
            if mode == 0 and len(b) > 1:
                for _ in range(int(rng.integers(1, 4))):
                    b[int(rng.integers(1, len(b)))] = int(rng.integers(0, 256))
            elif mode == 1:
                b = b[:int(rng.integers(0, len(b) + 1))]
            elif mode == 2 and len(b) > 1:
                i = int(rng.integers(1, len(b)))
                b[i] ^= 1 << int(rng.integers(0, 8))
            blocks.append(bytes(b))
            sizes.append(len(r) + (int(rng.integers(-2, 3)) if mode == 3 else 0))
    bad = _check(pq, ctx, blocks, [max(0, s) for s in sizes])
    assert bad > 20


def test_snappy_page_mode_everywhere(pq, monkeypatch):
    """PQH_SNAPPY_PAGE=1 sends every SNAPPY page to k_snappy's one-workgroup-per-page decoder (the
    path barely compressible pages take anyway): the edge blocks, pyarrow blocks and a mutated subset
    give the oracle's status and bytes there too."""
    monkeypatch.setenv("PQH_SNAPPY_PAGE", "1")
    ctx = pq.native.Context(0)
    cases = edge_blocks()
    assert _check(pq, ctx, [c[0] for c in cases], [len(c[1]) for c in cases]) == 0
    raws = sample_blocks()
    assert _check(pq, ctx, [pa.compress(r, codec="snappy", asbytes=True) for r in raws], [len(r) for r in raws]) == 0
    rng = np.random.default_rng(5)
    blocks, sizes = [], []
    for r in [r for r in raws if len(r) > 64][:6]:
        comp = bytearray(pa.compress(r, codec="snappy", asbytes=True))
        for _ in range(6):
            b = bytearray(comp)
            b[int(rng.integers(1, len(b)))] ^= 1 << int(rng.integers(0, 8))
            blocks.append(bytes(b))
            sizes.append(len(r))
    _check(pq, ctx, blocks, sizes)
    ctx.close()


def _files():
    yield "writer-v1", fixtures.flat_all_types(n=8000, v2=False, codec=O.SNAPPY, page=16 * 1024, rows_per_group=4000)
    yield "writer-v2", fixtures.flat_all_types(n=8000, v2=True, codec=O.SNAPPY, page=16 * 1024, rows_per_group=4000)
    yield "pyarrow-v1", fixtures.pyarrow_file(n=20000, version="1.0", compression="SNAPPY")
    yield "pyarrow-v2", fixtures.pyarrow_file(n=20000, version="2.0", compression="SNAPPY")


@pytest.mark.parametrize("staged", [False, True])
def test_device_snappy_files(pq, ctx, staged):
    checked = 0
    for name, data in _files():
        f = pq.native.File(data)
        ncols = len(f.columns())
        res = pq.reader.decode_chunks(ctx, f, 0, f.num_row_groups, list(range(ncols)), device_snappy=True,
                                      staged_runs=2 if staged else 0)
        fr = O.FileReader(data)
        for k, col in enumerate(res):
            rg, ci = divmod(k, ncols)
            assert col.status != pq.native.NOT_IMPLEMENTED, f"{name} rg{rg} {col.path}: NOT_IMPLEMENTED"
            assert_chunk(col, oracle_chunk(fr, rg, ci), where=f"{name} rg{rg} {col.path}")
            checked += 1
    assert checked > 40


def test_device_snappy_corrupt_page_fails_its_chunk(pq, ctx):
    """A corrupt compressed page (announced length intact): the chunk fails with DECOMPRESS on the
    device exactly when the host decoder (and golang/snappy) rejects the block."""
    W = pq.writer
    rng = np.random.default_rng(3)
    vals = np.repeat(rng.integers(0, 1 << 40, 3000), 8)
    data = W.flat([("v", W.Column(W.INT64, vals, use_dict=False), W.REQUIRED),
                   ("w", W.Column(W.INT64, vals[::-1].copy(), use_dict=False), W.REQUIRED)], len(vals),
                  codec=O.SNAPPY, max_page_size=8 * 1024)
    f = pq.native.File(data)
    failed = ok = 0
    for trial in range(12):
        hb = f.load(0, 1, [0, 1], device_snappy=True)
        cps = hb.codec_pages()
        src = hb.payload()  # writable view of the host batch's source bytes
        victim = cps[int(rng.integers(0, len(cps)))]
        lo = victim.src_offset + victim.raw_len + 3  # past the announced length
        i = int(rng.integers(lo, victim.src_offset + victim.src_len))
        src[i] ^= 1 << int(rng.integers(0, 8))
        blk = bytes(src[victim.src_offset + victim.raw_len:victim.src_offset + victim.src_len])
        st, _ = _expect(blk, victim.image_len - victim.raw_len)
        b = pq.native.Batch.from_host(ctx, hb)
        b.run()
        b.sync()
        out = b.chunk_out(victim.chunk)
        if st:
            assert out.status == DECOMPRESS, f"trial {trial}: device status {out.status}"
            failed += 1
        else:
            ok += 1
        other = b.chunk_out(1 - victim.chunk)
        assert other.status == 0
        b.close()
        hb.close()
    assert failed >= 3, (failed, ok)


def _gzip_check(pq, ctx, cases):
    import test_gzip_codec as TG

    got = _device_decompress(pq, ctx, [c[1] for c in cases], [c[2] for c in cases], codec=O.GZIP)
    ok = bad = 0
    for (name, s, size), (st, raw) in zip(cases, got):
        est, eraw = TG.expected(s, size)
        assert st == est, f"{name}: device status {st} vs oracle {est}"
        if est == 0:
            assert raw == eraw, f"{name}: bytes differ"
        ok += est == 0
        bad += est != 0
    return ok, bad


def test_gzip_valid_streams(pq, ctx):
    import test_gzip_codec as TG

    cases = [c for c in TG.all_cases() if "mut" not in c[0]]
    ok, bad = _gzip_check(pq, ctx, cases)
    assert ok > 60 and bad > 25, (ok, bad)


def test_gzip_mutants(pq, ctx):
    import gzip_blocks as G

    valid = [(n, s, len(O.gzip_decode(s))) for n, s, _ in G.valid_cases()]
    ok, bad = _gzip_check(pq, ctx, G.mutants(valid, seed=11, per=9))
    assert bad > 100, (ok, bad)


def _gzip_files():
    yield "writer-v1", fixtures.flat_all_types(n=8000, v2=False, codec=O.GZIP, page=16 * 1024, rows_per_group=4000)
    yield "writer-v2", fixtures.flat_all_types(n=8000, v2=True, codec=O.GZIP, page=16 * 1024, rows_per_group=4000)
    yield "nested", fixtures.nested_list_map(n=3000, v2=True, codec=O.GZIP)
    yield "pyarrow-v1", fixtures.pyarrow_file(n=20000, version="1.0", compression="GZIP")
    yield "pyarrow-v2", fixtures.pyarrow_file(n=20000, version="2.0", compression="GZIP")


@pytest.mark.parametrize("staged", [False, True])
def test_device_gzip_files(pq, ctx, staged):
    checked = gz = 0
    for name, data in _gzip_files():
        f = pq.native.File(data)
        ncols = len(f.columns())
        hb = f.load(0, f.num_row_groups, list(range(ncols)), device_gzip=True)
        gz += sum(c.codec == O.GZIP for c in hb.codec_pages())
        hb.close()
        res = pq.reader.decode_chunks(ctx, f, 0, f.num_row_groups, list(range(ncols)), device_gzip=True,
                                      staged_runs=2 if staged else 0)
        fr = O.FileReader(data)
        for k, col in enumerate(res):
            rg, ci = divmod(k, ncols)
            assert_chunk(col, oracle_chunk(fr, rg, ci), where=f"{name} rg{rg} {col.path}")
            checked += 1
    assert checked > 40 and gz > 50, (checked, gz)


def test_device_gzip_corrupt_page_fails_its_chunk(pq, ctx):
    """A corrupted GZIP page fails its chunk with DECOMPRESS on the device exactly when the
    reference's reader rejects the block; the other chunk decodes."""
    import test_gzip_codec as TG

    W = pq.writer
    rng = np.random.default_rng(4)
    vals = np.repeat(rng.integers(0, 1 << 40, 3000), 8)
    data = W.flat([("v", W.Column(W.INT64, vals, use_dict=False), W.REQUIRED),
                   ("w", W.Column(W.INT64, vals[::-1].copy(), use_dict=False), W.REQUIRED)], len(vals),
                  codec=O.GZIP, max_page_size=8 * 1024)
    f = pq.native.File(data)
    failed = ok = 0
    for trial in range(12):
        hb = f.load(0, 1, [0, 1], device_gzip=True)
        cps = hb.codec_pages()
        src = hb.payload()
        victim = cps[int(rng.integers(0, len(cps)))]
        i = int(rng.integers(victim.src_offset + 10, victim.src_offset + victim.src_len))
        src[i] ^= 1 << int(rng.integers(0, 8))
        blk = bytes(src[victim.src_offset:victim.src_offset + victim.src_len])
        st, _ = TG.expected(blk, victim.image_len)
        b = pq.native.Batch.from_host(ctx, hb)
        b.run()
        b.sync()
        out = b.chunk_out(victim.chunk)
        if st:
            assert out.status == DECOMPRESS, f"trial {trial}: device status {out.status}"
            failed += 1
        else:
            ok += 1
        assert b.chunk_out(1 - victim.chunk).status == 0
        b.close()
        hb.close()
    assert failed >= 6, (failed, ok)


@pytest.mark.parametrize("codec", ["snappy", "gzip"])
def test_device_codec_url_pages_repeat(pq, ctx, codec):
    """URL-like DELTA_LENGTH pages of ~1 MiB (many 64 KiB emit units per SNAPPY page, windows stitched
    across long pages): decoded with device decompression in plain and staged batches, run several
    times back to back; every run equals the oracle's decode bit for bit."""
    from parquet_go_amd import datasets

    W = pq.writer
    data = datasets.c5z(rows=400_000, row_groups=2, seed=7, codec=W.GZIP if codec == "gzip" else W.SNAPPY).tobytes()
    f = pq.native.File(data)
    fr = O.FileReader(data)
    expect = [oracle_chunk(fr, rg, 0) for rg in range(f.num_row_groups)]
    dev = dict(device_snappy=codec == "snappy", device_gzip=codec == "gzip")
    for staged in (False, True):
        hb = f.load(0, f.num_row_groups, [0], ctx=ctx if staged else None, **dev)
        units = sum(-(-(c.image_len - c.raw_len) // 65536) for c in hb.codec_pages())
        assert units > 2 * len(hb.codec_pages())
        b = pq.native.Batch.staged(ctx, hb) if staged else pq.native.Batch.from_host(ctx, hb)
        for run in range(3):
            for _ in range(2):  # back to back, no sync in between
                b.run_staged() if staged else b.run()
            b.sync()
            res = b.page_results(hb.num_pages)
            pages = hb.pages()
            path, pt, tl, md, mr = f.columns()[0]
            for rg, ch in enumerate(hb.chunks()):
                span = range(ch.first_page, ch.first_page + ch.num_pages)
                info = [(pages[p].page_type, pages[p].num_values, res[p]) for p in span]
                col = pq.reader.ColumnData(path, (pt, tl, md, mr), b.chunk_out(rg), [res[p] for p in span], ctx, None, info)
                assert_chunk(col, expect[rg], where=f"{codec} staged={staged} run {run} rg{rg}")
        b.close()
        hb.close()
