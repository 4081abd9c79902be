"""GPU parity: the HIP decode through the C-ABI vs the CPU oracle, bit for bit.

Covers every page layout the reference decodes (V1/V2, dictionary + fallback, PLAIN fixed / INT96
/ FLBA / booleans PLAIN + RLE, optional and repeated levels), reference-writer-shaped streams (one
bit-packed run) and pyarrow-shaped streams (many RLE + bit-packed runs), codecs decompressed on
the host, and a seeded mutation fuzzer whose per-page status / first-error position / outputs must
match the oracle's.
"""
import numpy as np
import pytest

import fixtures
from oracle import oracle as O
from parity import assert_chunk, oracle_chunk

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(pq):
    return pq.native.Context(0)


@pytest.fixture(params=["tiles", "streams", "split"])
def delta_mode(request, monkeypatch):
    """Every DELTA decode path: per-tile sums + page scan + tile expands; one workgroup per stream
    (k_delta_fused + k_delta_page), which the planner picks for batches of >= 256 delta streams; and
    the opt-in windowed heads (k_delta_split, PQH_DELTA_SPLIT=1) in page mode."""
    monkeypatch.setenv("PQH_DELTA_PAGE_MODE", "0" if request.param == "tiles" else "1")
    monkeypatch.setenv("PQH_DELTA_SPLIT", "1" if request.param == "split" else "0")
    return request.param


def _run_file(pq, ctx, data):
    f = pq.native.File(data)
    ncols = len(f.columns())
    cols = list(range(ncols))
    res = pq.reader.decode_chunks(ctx, f, 0, f.num_row_groups, cols)
    fr = O.FileReader(data)
    checked = skipped = 0
    for k, col in enumerate(res):
        rg, ci = divmod(k, ncols)
        # every (type, encoding) pair getValuesDecoder accepts (chunk_reader.go:106-159) decodes
        # on the device: NOT_IMPLEMENTED is a failure, never a skip
        assert col.status != pq.native.NOT_IMPLEMENTED, f"rg{rg} {col.path}: NOT_IMPLEMENTED"
        assert_chunk(col, oracle_chunk(fr, rg, ci), where=f"rg{rg} {col.path}")
        checked += 1
    return checked, skipped


@pytest.mark.parametrize("v2", [False, True])
@pytest.mark.parametrize("codec", [0, 1, 2])
def test_all_types(pq, ctx, v2, codec):
    data = fixtures.flat_all_types(n=20000, v2=v2, codec=codec, page=32 * 1024, rows_per_group=7000)
    checked, skipped = _run_file(pq, ctx, data)
    assert checked >= 3 * 10


@pytest.mark.parametrize("v2", [False, True])
def test_c2_schema(pq, ctx, v2):
    checked, skipped = _run_file(pq, ctx, fixtures.flat_c2_like(n=40000, v2=v2))
    assert checked == 4 * 6


def test_staged_end_to_end(pq, ctx):
    """End-to-end mode: one staged batch per row group (pinned page images, H2D on the copy stream,
    decode on the compute stream), all enqueued before one sync, each run three times so repeat
    copies must wait for the previous decode of the same batch."""
    data = fixtures.flat_c2_like(n=40000, v2=True)
    f = pq.native.File(data)
    ncols = len(f.columns())
    fr = O.FileReader(data)
    # odd row groups: the payload written straight into pinned memory (pqh_file_load_pinned), adopted
    # by the staged batch without a copy; the host batch is closed first (the block stays shared)
    hbs = [f.load(rg, rg + 1, list(range(ncols)), ctx=ctx if rg % 2 else None) for rg in range(f.num_row_groups)]
    batches = [pq.native.Batch.staged(ctx, hb) for hb in hbs]
    for rg in range(1, f.num_row_groups, 2):
        hbs[rg].close()
        hbs[rg] = f.load(rg, rg + 1, list(range(ncols)))  # (tables only, for the chunk list below)
    for _ in range(3):
        for b in batches:
            b.run_staged()
    for rg, (hb, b) in enumerate(zip(hbs, batches)):
        b.sync()
        for ci, ch in enumerate(hb.chunks()):
            col = pq.reader.ColumnData(f.columns()[ci][0], f.columns()[ci][1:], b.chunk_out(ci), [], ctx, None)
            assert_chunk(col, oracle_chunk(fr, rg, ci), where=f"staged rg{rg} c{ci}")
        b.close()
        hb.close()
    assert f.num_row_groups == 4
    res = pq.reader.decode_chunks(ctx, f, 1, 3, [0, 3, 5], staged_runs=2)
    for k, col in enumerate(res):
        rg, ci = 1 + k // 3, [0, 3, 5][k % 3]
        assert_chunk(col, oracle_chunk(fr, rg, ci), where=f"staged multi-rg rg{rg} c{ci}")


@pytest.mark.parametrize("version", ["1.0", "2.0"])
@pytest.mark.parametrize("compression", ["NONE", "SNAPPY", "GZIP"])
def test_pyarrow_files(pq, ctx, version, compression):
    _run_file(pq, ctx, fixtures.pyarrow_file(n=20000, version=version, compression=compression))


@pytest.mark.parametrize("v2", [False, True])
def test_nested_levels(pq, ctx, v2):
    _run_file(pq, ctx, fixtures.nested_list_map(n=6000, v2=v2))


def test_large_pages_single_run(pq, ctx):
    """Reference-writer pages spanning many tiles (1 MiB page estimate, one bit-packed run)."""
    W = fixtures.W
    rng = np.random.default_rng(9)
    n = 600000
    cols = [("d", W.Column(W.INT32, rng.integers(0, 4096, n).astype(np.int32)), W.REQUIRED),
            ("o", W.optional(W.INT64, rng.integers(0, 2**60, n), rng.random(n) < 0.3, use_dict=False), W.OPTIONAL),
            ("b", W.Column(W.BOOLEAN, (rng.random(n) < 0.5).astype(np.uint8)), W.REQUIRED)]
    checked, _ = _run_file(pq, ctx, W.flat(cols, n))
    assert checked == 3


# ---------------------------------------------------------------------------------------------
# mutation fuzzing at the page level (pqh_batch_create with explicit page tables)
# ---------------------------------------------------------------------------------------------
def _page_sets(pq, data):
    """(column, dictionary image or None, [data pages]) for every chunk of a file (host walker)."""
    f = pq.native.File(data)
    cols = f.columns()
    hb = f.load(0, f.num_row_groups, list(range(len(cols))))
    payload = hb.payload()
    pages = hb.pages()
    out = []
    for k, ch in enumerate(hb.chunks()):
        col = cols[k % len(cols)]
        dict_img, dpages = None, []
        for p in range(ch.first_page, ch.first_page + ch.num_pages):
            pg = pages[p]
            img = payload[pg.image_offset: pg.image_offset + pg.image_len].tobytes()
            if pg.page_type == O.DICTIONARY_PAGE:
                dict_img = (pg.num_values, pg.encoding, img)
            else:
                dpages.append((pg.page_type, pg.num_values, pg.encoding, pg.def_levels_byte_length,
                               pg.rep_levels_byte_length, img))
        out.append((col, dict_img, dpages))
    return out


def _mutate(rng, img):
    b = bytearray(img)
    if not b:
        return bytes(b)
    kind = rng.integers(0, 5)
    if kind == 0:  # flip bytes near the start (headers / widths / run headers)
        for _ in range(int(rng.integers(1, 4))):
            i = int(rng.integers(0, min(len(b), 24)))
            b[i] = int(rng.integers(0, 256))
    elif kind == 1:  # truncate
        b = b[: int(rng.integers(0, len(b)))]
    elif kind == 2:  # random byte anywhere
        i = int(rng.integers(0, len(b)))
        b[i] ^= 1 << int(rng.integers(0, 8))
    elif kind == 3:  # zero a window
        i = int(rng.integers(0, len(b)))
        b[i:i + 8] = bytes(len(b[i:i + 8]))
    else:  # set a byte to 0xff
        b[int(rng.integers(0, len(b)))] = 0xFF
    return bytes(b)


def _fuzz(pq, ctx, data, seed, per_page=3):
    return _run_cases(pq, ctx, _fuzz_cases(pq, data, seed, per_page))


def _fuzz_cases(pq, data, seed, per_page=3):
    rng = np.random.default_rng(seed)
    cases = []
    for (path, pt, tl, md, mr), dict_img, dpages in _page_sets(pq, data):
        col = (pt, tl, md, mr)
        for pg in dpages:
            for _ in range(per_page):
                ptype, nv, enc, dl, rl, img = pg
                img2 = _mutate(rng, img)
                if ptype == O.DATA_PAGE_V2 and rl + dl > len(img2):
                    continue  # the host walker rejects such headers before the device sees them
                cases.append((col, dict_img, (ptype, nv, enc, dl, rl, img2)))
    return cases


def _run_cases(pq, ctx, cases, stats=None, runs=1, hints=None):
    """Decode `cases` = [(column, dictionary (num_values, encoding, image) or None, data page)] in ONE
    batch (every case its own chunk) and compare each against the oracle's decode_page.  stats: a
    dict that gets the batch's kernel launch counts by name (profiled contexts).  runs: decodes of
    the batch before its one sync (each must leave the batch's device counters as it found them)."""
    N = pq.native
    # every case is its own chunk (dictionary page first when present)
    blobs, chunks, pages = [], [], []
    off = 0

    def add(img):
        nonlocal off
        base = (off + 63) & ~63
        blobs.append(b"\0" * (base - off) + img)
        off = base + len(img)
        return base

    for ci, (col, dict_img, (ptype, nv, enc, dl, rl, img)) in enumerate(cases):
        first = len(pages)
        if dict_img is not None:
            o = add(dict_img[2])
            pages.append(N.Page(o, len(dict_img[2]), O.DICTIONARY_PAGE, dict_img[0], dict_img[1], 0, 0, len(chunks), 0))
        o = add(img)
        # (hints: the V2 header's num_nulls per case -- k_flat's speculative notNull; 0 otherwise)
        pages.append(N.Page(o, len(img), ptype, nv, enc, dl, rl, len(chunks), hints[ci] if hints else 0))
        chunks.append(N.Chunk(N.Column(*col), first, len(pages) - first, 0, 0))
    payload = b"".join(blobs) + b"\0" * N.PAYLOAD_PAD
    arr = np.frombuffer(payload, dtype=np.uint8).copy()
    d = ctx.malloc(len(arr))
    try:
        ctx.h2d(d, arr.ctypes.data, len(arr))
        ctx.sync()
        b = N.Batch.from_tables(ctx, chunks, pages, d, off)
        for _ in range(runs):
            b.run()
        b.sync()
        compared = errors = 0
        for i, (col, dict_img, (ptype, nv, enc, dl, rl, img)) in enumerate(cases):
            o = b.chunk_out(i)
            assert o.status != N.NOT_IMPLEMENTED, f"case {i}: NOT_IMPLEMENTED"
            cd = pq.reader.ColumnData("fuzz", col, o, [], ctx)
            od = O.decode_dict_page(col, dict_img[0], dict_img[1], dict_img[2]) if dict_img else None
            if od is not None and od.status:  # the dictionary page itself fails
                assert cd.status != 0
                compared += 1
                errors += 1
                continue
            r = O.decode_page(col, ptype, nv, enc, dl, rl, img, od)
            from parity import Expected

            e = Expected()
            e.status, e.phase, e.index = r.status, r.phase, r.index
            e.nn, e.values, e.def_levels, e.rep_levels = r.nn, r.values, r.def_levels, r.rep_levels
            e.nil = r.nil
            if r.offsets is not None:
                e.offsets, e.data = r.offsets, r.values
            assert_chunk(cd, e, where=f"case {i} col {col} enc {enc} type {ptype}")
            compared += 1
            errors += r.status != 0
        if stats is not None:
            stats.update({k.name.decode(): k.launches for k in b.kernel_stats()})
        b.close()
        return compared, errors
    finally:
        ctx.free(d)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_fuzz_generated_pages(pq, ctx, seed):
    data = fixtures.flat_all_types(n=3000, v2=bool(seed % 2), page=8 * 1024, rows_per_group=3000)
    compared, errors = _fuzz(pq, ctx, data, seed)
    assert compared > 20 and errors > 5


@pytest.mark.parametrize("seed", [4, 5])
def test_fuzz_pyarrow_pages(pq, ctx, seed):
    data = fixtures.pyarrow_file(n=4000, version="1.0" if seed == 4 else "2.0")
    compared, errors = _fuzz(pq, ctx, data, seed)
    assert compared > 20 and errors > 5


def test_fuzz_nested_pages(pq, ctx):
    compared, errors = _fuzz(pq, ctx, fixtures.nested_list_map(n=1500), 6)
    assert compared > 5


def _required_flat(n, v2, seed=21):
    """Required flat fixed-width columns of every kind k_flat takes (dictionary, PLAIN, INT96, FLBA,
    PLAIN booleans), reference-writer pages."""
    W = fixtures.W
    rng = np.random.default_rng(seed)
    cols = [("i32_dict", W.Column(W.INT32, rng.integers(-2**31, 2**31 - 1, 4096).astype(np.int32)[rng.integers(0, 4096, n)]), W.REQUIRED),
            ("i64", W.Column(W.INT64, rng.integers(-2**62, 2**62, n), use_dict=False), W.REQUIRED),
            ("f32_dict", W.Column(W.FLOAT, rng.standard_normal(7).astype(np.float32)[rng.integers(0, 7, n)]), W.REQUIRED),
            ("bool", W.Column(W.BOOLEAN, (rng.random(n) < 0.5).astype(np.uint8)), W.REQUIRED),
            ("flba", W.Column(W.FIXED_LEN_BYTE_ARRAY, rng.integers(0, 256, (n, 16), dtype=np.uint8), type_length=16,
                              use_dict=False), W.REQUIRED),
            ("i96_dict", W.Column(W.INT96, rng.integers(0, 256, (40, 12), dtype=np.uint8)[rng.integers(0, 40, n)]),
             W.REQUIRED),
            ("d_const", W.Column(W.DOUBLE, np.full(n, 2.5)), W.REQUIRED)]  # one-entry dictionary: width 0
    return W.flat(cols, n // 2, v2=v2, max_page_size=48 * 1024)


@pytest.mark.parametrize("flat", ["one_launch", "three_kernels"])
def test_flat_one_launch(pq, monkeypatch, flat):
    """Small batches of required flat fixed-width columns decode in ONE launch, k_flat: every tile
    decodes from its page's speculative state (clean page, one bit-packed run, enough bytes) and the
    host's value bases, and the page checks (k_prologue's body) compare; with PQH_FLAT=0 through
    k_prologue / k_scan / k_expand.  Clean pages stay on k_flat; the mutation fuzzer's pages (errors,
    limits, failed dictionaries, keys out of range) and pyarrow-style streams (many runs) fail the
    speculation, and the batch is decoded again by the three kernels: the reference's results
    either way.  Each batch is run three times before its sync."""
    W = fixtures.W
    monkeypatch.setenv("PQH_FLAT", "1" if flat == "one_launch" else "0")
    ctx = pq.native.Context(0, profile=True)
    for v2 in (False, True):
        data = _required_flat(60000, v2)
        checked, _ = _run_file(pq, ctx, data)
        assert checked == 2 * 7
        # dictionary pages of the file start at value bases that are not multiples of 4 (k_flat's
        # 16-byte streaming stores of gathered INT32 values are then only 4-byte aligned)
        fr = O.FileReader(data)
        bases = [int(b) for ci in range(len(fr.columns)) if fr.columns[ci].physical_type == W.INT32
                 for b in np.cumsum([r.num_values for r in O.decode_chunk(fr.read_chunk(0, ci))])[:-1]]
        assert any(b % 4 for b in bases), bases
        # the same pages as explicit cases (each its own chunk): clean, then with mutants among them
        clean = _page_sets_cases(pq, data)
        stats = {}
        compared, errors = _run_cases(pq, ctx, clean, stats, runs=3)
        assert compared == len(clean) and errors == 0
        want = {"k_flat": 3, "k_expand": 0} if flat == "one_launch" else {"k_flat": 0, "k_expand": 3}
        assert {k: stats.get(k, 0) for k in want} == want, stats
        mutants = _fuzz_cases(pq, data, 13 + v2, per_page=2)
        stats = {}
        compared, errors = _run_cases(pq, ctx, clean[:20] + mutants[:200] + clean[20:], stats, runs=3)
        assert compared == len(clean) + min(len(mutants), 200) and errors > 10, (compared, errors)
        # (k_flat's runs are dropped with its speculation; the rerun is the three kernels')
        assert stats.get("k_expand", 0) == (1 if flat == "one_launch" else 3), stats
    # the fixture's required fixed-width pages (V1 / V2), mutated
    for seed, v2 in ((11, False), (12, True)):
        data = fixtures.flat_all_types(n=3000, v2=v2, page=8 * 1024, rows_per_group=3000)
        skip = (W.DELTA_BINARY_PACKED, W.DELTA_LENGTH_BYTE_ARRAY, W.DELTA_BYTE_ARRAY)
        cases = [c for c in _fuzz_cases(pq, data, seed, per_page=6)
                 if c[0][0] != W.BYTE_ARRAY and c[0][2] == 0 and c[2][2] not in skip]
        compared, errors = _run_cases(pq, ctx, cases[:300], runs=3)
        assert compared == min(len(cases), 300) and compared > 100 and errors > 20, (compared, errors)
    ctx.close()
    # unprofiled: the runs replay a captured graph, which the fallback drops and captures again
    ctx = pq.native.Context(0)
    data = _required_flat(20000, True, seed=5)
    clean = _page_sets_cases(pq, data)
    compared, errors = _run_cases(pq, ctx, clean, runs=3)
    assert compared == len(clean) and errors == 0
    compared, errors = _run_cases(pq, ctx, clean + _fuzz_cases(pq, data, 17, per_page=2)[:100], runs=3)
    assert compared > len(clean) and errors > 5, (compared, errors)
    ctx.close()


def _nullable_flat(n, seed=23, null_frac=0.01):
    """Nullable (max_def 1) flat fixed-width columns, V2 pages (reference-writer levels: one
    bit-packed run of width 1), plus a required column: the mixed workload's shape."""
    W = fixtures.W
    rng = np.random.default_rng(seed)

    def defs():
        return (rng.random(n) >= null_frac).astype(np.uint8)

    d0, d1, d2 = defs(), defs(), defs()
    cols = [("f64", W.Column(W.DOUBLE, rng.standard_normal(int(d0.sum())), def_levels=d0, use_dict=False), W.OPTIONAL),
            ("i32_dict", W.Column(W.INT32, rng.integers(0, 900, int(d1.sum())).astype(np.int32), def_levels=d1),
             W.OPTIONAL),
            ("flba", W.Column(W.FIXED_LEN_BYTE_ARRAY, rng.integers(0, 256, (int(d2.sum()), 16), dtype=np.uint8),
                              def_levels=d2, type_length=16, use_dict=False), W.OPTIONAL),
            ("i64", W.Column(W.INT64, rng.integers(-2**62, 2**62, n), use_dict=False), W.REQUIRED)]
    return W.flat(cols, n // 2, v2=True, max_page_size=48 * 1024)


@pytest.mark.parametrize("flat", ["one_launch", "three_kernels"])
def test_flat_nullable_v2(pq, monkeypatch, flat):
    """Nullable flat columns with V2 pages decode in k_flat's one launch too: the speculative
    notNull is the header's num_values - num_nulls, the definition levels (one bit-packed run) are
    expanded by level tiles of the same launch, and the page checks count the levels.  A page whose
    num_nulls hint is wrong (the explicit cases below carry 0) fails the speculation and the batch is
    decoded again by the three kernels: the reference's results either way."""
    monkeypatch.setenv("PQH_FLAT", "1" if flat == "one_launch" else "0")
    ctx = pq.native.Context(0, profile=True)
    for null_frac in (0.01, 0.5, 0.0, 1.0):
        data = _nullable_flat(30000, null_frac=null_frac)
        f = pq.native.File(data)
        res, b, hb = pq.reader.decode_chunks(ctx, f, 0, f.num_row_groups, list(range(4)), return_batch=True)
        paths = b.paths()
        stats = {s.name.decode(): s.launches for s in b.kernel_stats() if s.launches}
        assert paths["flat_fallbacks"] == 0, (null_frac, paths)
        want = {"k_flat": 1, "k_expand": 0} if flat == "one_launch" else {"k_flat": 0, "k_expand": 1}
        assert {k: stats.get(k, 0) for k in want} == want, (null_frac, stats)
        fr = O.FileReader(data)
        for k, col in enumerate(res):
            rg, ci = divmod(k, 4)
            assert_chunk(col, oracle_chunk(fr, rg, ci), where=f"nulls {null_frac} rg{rg} {col.path}")
        assert sum(1 for c in res if c.def_levels is not None and (c.def_levels == 0).any()) == \
            (0 if null_frac == 0.0 else 6)
        b.close()
        hb.close()
    # the same pages as explicit cases: num_nulls hint 0 on pages that hold nulls
    data = _nullable_flat(20000)
    clean = _page_sets_cases(pq, data)
    stats = {}
    compared, errors = _run_cases(pq, ctx, clean, stats, runs=3)
    assert compared == len(clean) and errors == 0
    assert stats.get("k_expand", 0) == (1 if flat == "one_launch" else 3), stats
    # with their true hints they stay in one launch; mutants (levels, values, truncation) with the
    # unmutated page's hint: those whose speculation still holds decode in k_flat, the others fall
    # back -- the oracle's results and first errors either way
    hints = _v2_null_hints(pq, data)
    stats = {}
    compared, errors = _run_cases(pq, ctx, clean, stats, runs=3, hints=hints)
    assert compared == len(clean) and errors == 0
    assert stats.get("k_expand", 0) == (0 if flat == "one_launch" else 3), stats
    rng = np.random.default_rng(29)
    mut, mh = [], []
    for (col, dimg, pg), h in zip(clean, hints):
        for _ in range(6):
            img2 = _mutate(rng, pg[5])
            if pg[3] + pg[4] > len(img2):
                continue  # (the host walker rejects such headers before the device sees them)
            mut.append((col, dimg, pg[:5] + (img2,)))
            mh.append(h)
    compared, errors = _run_cases(pq, ctx, clean[:10] + mut, runs=3, hints=hints[:10] + mh)
    assert compared == 10 + len(mut) and errors >= 5, (compared, errors)  # (each case vs the oracle)
    ctx.close()


def _v2_null_hints(pq, data):
    """num_nulls of every data page of `data`, in _page_sets_cases order (the host walker's V2
    header field)."""
    f = pq.native.File(data)
    hb = f.load(0, f.num_row_groups, list(range(len(f.columns()))))
    pages = hb.pages()
    out = []
    for ch in hb.chunks():
        for p in range(ch.first_page, ch.first_page + ch.num_pages):
            if pages[p].page_type != O.DICTIONARY_PAGE:
                out.append(pages[p].num_nulls)
    hb.close()
    f.close()
    return out


def _page_sets_cases(pq, data):
    """Every data page of `data` as an unmutated case."""
    out = []
    for (path, pt, tl, md, mr), dict_img, dpages in _page_sets(pq, data):
        for pg in dpages:
            out.append(((pt, tl, md, mr), dict_img, pg))
    return out


# ---------------------------------------------------------------------------------------------
# DELTA_BINARY_PACKED: every block geometry the reference decoder accepts
# ---------------------------------------------------------------------------------------------
DELTA_GEOMETRIES = [(128, 4), (128, 1), (256, 8), (512, 4), (1024, 8), (2048, 4), (2048, 1),  # device fast path
                    (64, 2), (128, 16), (96, 3), (24, 3), (12, 3), (4096, 4), (32, 1)]     # serial decoder


def _delta_cases(rng, sizes, kinds, mutate):
    import delta_streams as DS
    W = fixtures.W
    cases = []
    for bs, mbc in DELTA_GEOMETRIES:
        for bits in (32, 64):
            col = (W.INT32 if bits == 32 else W.INT64, 0, 0, 0)
            for n in sizes:
                kind = kinds[int(rng.integers(0, len(kinds)))]
                finish = "omit" if rng.random() < 0.5 else "full"
                vals = DS.random_values(rng, n, bits, kind)
                img = DS.encode(vals, bits, bs, mbc, finish)
                cases.append((col, None, (O.DATA_PAGE, n, W.DELTA_BINARY_PACKED, 0, 0, img)))
                if not mutate:
                    continue
                # page claims more values than the stream holds; header count below the page's
                cases.append((col, None, (O.DATA_PAGE, n + int(rng.integers(1, 20)), W.DELTA_BINARY_PACKED, 0, 0, img)))
                img2 = DS.encode(vals, bits, bs, mbc, finish, total=max(0, n - int(rng.integers(1, 10))))
                cases.append((col, None, (O.DATA_PAGE, n, W.DELTA_BINARY_PACKED, 0, 0, img2)))
                # truncated anywhere, or a corrupted byte
                cut = int(rng.integers(0, len(img) + 1))
                cases.append((col, None, (O.DATA_PAGE, n, W.DELTA_BINARY_PACKED, 0, 0, img[:cut])))
                cases.append((col, None, (O.DATA_PAGE, n, W.DELTA_BINARY_PACKED, 0, 0, _mutate(rng, img))))
    return cases


def test_delta_geometries(pq, ctx, delta_mode):
    rng = np.random.default_rng(31)
    cases = _delta_cases(rng, [1, 2, 8, 9, 33, 129, 257, 1000, 2049, 4097], ["const", "mono", "small", "full", "mixed"],
                         mutate=True)
    compared, errors = _run_cases(pq, ctx, cases)
    assert compared == len(cases) and errors > 50


def test_delta_width_edges(pq, ctx, delta_mode):
    """Miniblock widths around the 32-bit scan limit of the int64 expansion (kNarrowWidth = 22:
    a 1024-value row of packed deltas must fit in 32 bits) and at 32/64; every tile either narrow,
    wide or alternating.  Deltas are 0 or all-ones in the width, so the row sums are the largest
    the width allows."""
    import delta_streams as DS
    W = fixtures.W
    rng = np.random.default_rng(35)
    cases = []
    for bits, widths in ((64, (21, 22, 23, 31, 32, 33, 63, 64)), (32, (22, 23, 31, 32))):
        col = (W.INT32 if bits == 32 else W.INT64, 0, 0, 0)
        for bs, mbc in ((128, 4), (1024, 8), (2048, 1)):
            for w in widths:
                n = 20000
                top = (1 << w) - 1
                # one 0 per 64 deltas keeps minDelta at the base, so the packed deltas reach `top`
                deltas = np.where(np.arange(n) % 64 == 0, 0, top).astype(object)
                if w >= 23:  # alternate blocks of width w with narrow ones
                    narrow = (np.arange(n) // (bs * 8)) % 2 == 1
                    deltas = np.where(narrow, np.arange(n) % 5, deltas)
                base = int(rng.integers(-1000, 1000))
                vals = [base]
                for dlt in deltas[1:]:
                    vals.append(vals[-1] + int(dlt) - (1 << (w - 1) if w == bits else 0))
                img = DS.encode(vals, bits, bs, mbc, "omit")
                cases.append((col, None, (O.DATA_PAGE, n, W.DELTA_BINARY_PACKED, 0, 0, img)))
    compared, errors = _run_cases(pq, ctx, cases)
    assert compared == len(cases) and errors == 0


def test_edge_pages(pq, ctx, delta_mode):
    """Edge cases the reference decoders meet at the boundaries: pages with no values, all-null
    optional pages, single values, ragged counts (not a multiple of 8), dictionary index widths 0,
    1, 32 and 33 (> 32 fails at init, type_dict.go:23-30), one-entry and empty dictionaries, DELTA
    streams of 0/1/2 values and constant runs."""
    import delta_streams as DS
    W = fixtures.W
    rng = np.random.default_rng(50)
    cases = []

    def v1_defs(defs):  # V1 page: u32 length + hybrid definition levels (maxD 1)
        h = W.hybrid_encode(1, np.asarray(defs, np.int32))
        return len(h).to_bytes(4, "little") + h

    for ptype, size in ((W.INT32, 4), (W.INT64, 8), (W.FLOAT, 4), (W.DOUBLE, 8), (W.BOOLEAN, 0),
                        (W.FIXED_LEN_BYTE_ARRAY, 16), (W.BYTE_ARRAY, 0)):
        tl = 16 if ptype == W.FIXED_LEN_BYTE_ARRAY else 0
        cases.append(((ptype, tl, 0, 0), None, (O.DATA_PAGE, 0, W.PLAIN, 0, 0, b"")))
        cases.append(((ptype, tl, 1, 0), None, (O.DATA_PAGE, 37, W.PLAIN, 0, 0, v1_defs([0] * 37))))
        one = (b"\x05\x00\x00\x00hello" if ptype == W.BYTE_ARRAY else
               bytes([1]) if ptype == W.BOOLEAN else rng.bytes(size))
        cases.append(((ptype, tl, 1, 0), None, (O.DATA_PAGE, 1, W.PLAIN, 0, 0, v1_defs([1]) + one)))
        cases.append(((ptype, tl, 1, 0), None, (O.DATA_PAGE, 3, W.PLAIN, 0, 0, v1_defs([0, 1, 0]) + one)))
    for n in (1, 7, 9, 63, 65, 1023):  # ragged boolean and level counts
        bits = rng.integers(0, 2, n).astype(np.uint8)
        cases.append(((W.BOOLEAN, 0, 0, 0), None,
                      (O.DATA_PAGE, n, W.PLAIN, 0, 0, np.packbits(bits, bitorder="little").tobytes())))
        defs = rng.integers(0, 2, n)
        vals = rng.integers(-9, 9, int(defs.sum())).astype(np.int32).tobytes()
        cases.append(((W.INT32, 0, 1, 0), None, (O.DATA_PAGE, n, W.PLAIN, 0, 0, v1_defs(defs) + vals)))
    d5 = np.arange(10, 15, dtype=np.int32).tobytes()
    idx = rng.integers(0, 5, 200).astype(np.int32)
    for w, body in ((0, b""), (1, W.hybrid_encode(1, idx % 2)), (3, W.hybrid_encode(3, idx)),
                    (32, W.hybrid_encode(32, idx)), (33, W.hybrid_encode(3, idx))):
        cases.append(((W.INT32, 0, 0, 0), (5, W.PLAIN, d5), (O.DATA_PAGE, 200, W.RLE_DICTIONARY, 0, 0, bytes([w]) + body)))
    cases.append(((W.INT64, 0, 0, 0), (1, W.PLAIN, (7).to_bytes(8, "little")),
                  (O.DATA_PAGE, 1000, W.RLE_DICTIONARY, 0, 0, bytes([1]) + W.hybrid_encode(1, np.zeros(1000, np.int32)))))
    cases.append(((W.INT32, 0, 0, 0), (0, W.PLAIN, b""),
                  (O.DATA_PAGE, 3, W.RLE_DICTIONARY, 0, 0, bytes([1]) + W.hybrid_encode(1, np.zeros(3, np.int32)))))
    cases.append(((W.INT32, 0, 0, 0), (5, W.PLAIN, d5), (O.DATA_PAGE, 0, W.RLE_DICTIONARY, 0, 0, b"")))
    for bits in (32, 64):
        col = (W.INT32 if bits == 32 else W.INT64, 0, 0, 0)
        for vals in ([], [5], [5, -3], [7] * 300, list(range(0, 3000, 3))):
            img = DS.encode(vals, bits, 128, 4, "full")
            cases.append((col, None, (O.DATA_PAGE, len(vals), W.DELTA_BINARY_PACKED, 0, 0, img)))
    compared, errors = _run_cases(pq, ctx, cases)
    assert compared == len(cases) and errors >= 2


def test_delta_multi_tile_pages(pq, ctx, delta_mode):
    """Pages spanning several 8192-value delta tiles (tile sums + page scan)."""
    rng = np.random.default_rng(32)
    cases = _delta_cases(rng, [8193, 30001], ["small", "mixed", "full"], mutate=False)
    compared, _ = _run_cases(pq, ctx, cases)
    assert compared == len(cases)


def _regimes(rng, n, bits):
    """Runs of constant, narrow and full-width deltas: blocks of 5 bytes next to blocks of 1-2 KiB."""
    lo, hi = -(1 << (bits - 1)), (1 << (bits - 1)) - 1
    d = np.zeros(n, np.int64)
    i = 0
    while i < n:
        span = int(rng.integers(1, 3000))
        kind = int(rng.integers(0, 3))
        if kind == 1:
            d[i:i + span] = rng.integers(-8, 8, min(span, n - i))
        elif kind == 2:
            d[i:i + span] = rng.integers(lo, hi, min(span, n - i), dtype=np.int64, endpoint=True)
        i += span
    v = np.cumsum(d.astype(np.uint64)).astype(np.int64) if bits == 64 else np.cumsum(d).astype(np.int32)
    return v


def test_delta_chain_speculation(pq, ctx, delta_mode):
    """Large reference-writer pages (128/4 blocks) whose block chains the walk finds with per-lane
    speculative segment walks: constant deltas (5-byte blocks), full-width deltas (2 KiB blocks),
    regime changes, timestamps; plus corrupted bytes and cuts anywhere in them (the stitched chain
    must hand over to the exact walk at the first bad header)."""
    W = fixtures.W
    rng = np.random.default_rng(36)
    cases = []
    for bits in (32, 64):
        col = (W.INT32 if bits == 32 else W.INT64, 0, 0, 0)
        dt = np.int32 if bits == 32 else np.int64
        for n in (131072, 50001):
            series = [np.full(n, 7, dt),
                      rng.integers(-(1 << (bits - 1)), (1 << (bits - 1)) - 1, n, dtype=np.int64).astype(dt),
                      _regimes(rng, n, bits),
                      (np.cumsum(1_000_000 + rng.integers(0, 4096, n)) % (1 << 31)).astype(dt)]
            for vals in series:
                img = W.delta_encode(vals, bits)
                cases.append((col, None, (O.DATA_PAGE, n, W.DELTA_BINARY_PACKED, 0, 0, img)))
                for _ in range(2):
                    cases.append((col, None, (O.DATA_PAGE, n, W.DELTA_BINARY_PACKED, 0, 0, _mutate(rng, img))))
                cut = int(rng.integers(len(img) // 4, len(img)))
                cases.append((col, None, (O.DATA_PAGE, n, W.DELTA_BINARY_PACKED, 0, 0, img[:cut])))
    compared, errors = _run_cases(pq, ctx, cases)
    assert compared == len(cases) and errors > 0


def test_delta_optional_v2(pq, ctx, delta_mode):
    """DELTA values behind definition levels (notNull < num_values) on V2 pages."""
    import delta_streams as DS
    W = fixtures.W
    rng = np.random.default_rng(33)
    cases = []
    for bits in (32, 64):
        for n in (1, 100, 129, 5000, 20000):
            mask = rng.random(n) < 0.7
            dl = W.hybrid_encode(1, mask.astype(np.int32))
            nn = int(mask.sum())
            img = DS.encode(DS.random_values(rng, nn, bits, "mixed"), bits, 128, 4, "omit") if nn else DS.encode([], bits)
            col = (W.INT32 if bits == 32 else W.INT64, 0, 1, 0)
            cases.append((col, None, (O.DATA_PAGE_V2, n, W.DELTA_BINARY_PACKED, len(dl), 0, dl + img)))
    compared, _ = _run_cases(pq, ctx, cases)
    assert compared == len(cases)


def test_delta_writer_pages(pq, ctx, delta_mode):
    """Reference-writer delta columns (128/4 blocks) in files: required, optional, large pages."""
    W = fixtures.W
    rng = np.random.default_rng(34)
    n = 300000
    cols = [("a", W.Column(W.INT64, np.cumsum(rng.integers(-5, 100, n)), encoding=W.DELTA_BINARY_PACKED), W.REQUIRED),
            ("b", W.Column(W.INT32, rng.integers(-2**31, 2**31 - 1, n, dtype=np.int64).astype(np.int32),
                           encoding=W.DELTA_BINARY_PACKED), W.REQUIRED),
            ("c", W.optional(W.INT64, rng.integers(0, 2**40, n), rng.random(n) < 0.2, encoding=W.DELTA_BINARY_PACKED,
                             use_dict=False), W.OPTIONAL)]
    for v2 in (False, True):
        checked, _ = _run_file(pq, ctx, W.flat(cols, n // 2, v2=v2))
        assert checked == 6


# ---------------------------------------------------------------------------------------------
# Byte arrays (byte-array dictionaries of a6/a11)
# ---------------------------------------------------------------------------------------------
def _plain_chain(strs):
    return b"".join(len(x).to_bytes(4, "little") + x for x in strs)


def _ba_cases(rng):
    import delta_streams as DS
    W = fixtures.W
    col = (W.BYTE_ARRAY, 0, 0, 0)
    cases = []
    for n in (0, 1, 7, 100, 129, 2049, 5000):
        strs = [rng.bytes(int(rng.integers(0, 40))) for _ in range(n)]
        plain = _plain_chain(strs)
        dlba = DS.encode([len(x) for x in strs], 32, 128, 4, "omit") + b"".join(strs)
        for enc, img in ((W.PLAIN, plain), (W.DELTA_LENGTH_BYTE_ARRAY, dlba)):
            cases.append((col, None, (O.DATA_PAGE, n, enc, 0, 0, img)))
            cases.append((col, None, (O.DATA_PAGE, n, enc, 0, 0, img[: int(rng.integers(0, len(img) + 1))])))
            cases.append((col, None, (O.DATA_PAGE, n + 3, enc, 0, 0, img)))
            cases.append((col, None, (O.DATA_PAGE, n, enc, 0, 0, _mutate(rng, img))))
        if n > 2:
            k = int(rng.integers(0, n))
            bad = list(strs)
            neg = _plain_chain(bad[:k]) + b"\xff\xff\xff\xff" + _plain_chain(bad[k:])
            cases.append((col, None, (O.DATA_PAGE, n, W.PLAIN, 0, 0, neg)))
            lens = [len(x) for x in strs]
            lens[k] = -int(rng.integers(1, 5))
            cases.append((col, None, (O.DATA_PAGE, n, W.DELTA_LENGTH_BYTE_ARRAY, 0, 0,
                                      DS.encode(lens, 32, 128, 4, "omit") + b"".join(strs))))
            lens = [len(x) for x in strs]
            lens[k] += 1000  # bytes run past the page
            cases.append((col, None, (O.DATA_PAGE, n, W.DELTA_LENGTH_BYTE_ARRAY, 0, 0,
                                      DS.encode(lens, 32, 128, 4, "omit") + b"".join(strs))))
    # byte-array dictionaries: PLAIN chain dictionary page + hybrid index pages
    for K in (1, 37, 3000):
        dstrs = [rng.bytes(int(rng.integers(0, 30))) for _ in range(K)]
        dimg = _plain_chain(dstrs)
        w = max(1, int(K - 1).bit_length())
        for n in (1, 500, 20000):
            idx = rng.integers(0, K, n).astype(np.int32)
            img = bytes([w]) + W.hybrid_encode(w, idx)
            cases.append((col, (K, W.PLAIN, dimg), (O.DATA_PAGE, n, W.RLE_DICTIONARY, 0, 0, img)))
            idx2 = idx.copy()
            idx2[int(rng.integers(0, n))] = min(K + 3, (1 << w) - 1)  # out of range (when representable)
            img2 = bytes([w]) + W.hybrid_encode(w, idx2)
            cases.append((col, (K, W.PLAIN, dimg), (O.DATA_PAGE, n, W.RLE_DICTIONARY, 0, 0, img2)))
        cases.append((col, (K + 2, W.PLAIN, dimg), (O.DATA_PAGE, 10, W.RLE_DICTIONARY, 0, 0,
                                                      bytes([w]) + W.hybrid_encode(w, np.zeros(10, np.int32)))))
        cases.append((col, (K, W.PLAIN, dimg[: len(dimg) // 2]), (O.DATA_PAGE, 10, W.RLE_DICTIONARY, 0, 0,
                                                                   bytes([w]) + W.hybrid_encode(w, np.zeros(10, np.int32)))))
    return cases


def test_byte_array_pages(pq, ctx):
    cases = _ba_cases(np.random.default_rng(41))
    compared, errors = _run_cases(pq, ctx, cases)
    assert compared == len(cases) and errors > 20


def test_byte_array_files(pq, ctx):
    """Reference-writer string columns: PLAIN, DELTA_LENGTH, dictionary (+ nulls), V1/V2, codecs."""
    W = fixtures.W
    rng = np.random.default_rng(42)
    n = 60000
    s = [rng.bytes(int(rng.integers(8, 41))) for _ in range(n)]
    mask = rng.random(n) < 0.1
    cols = [("p", W.Column(W.BYTE_ARRAY, s, use_dict=False), W.REQUIRED),
            ("l", W.Column(W.BYTE_ARRAY, s, encoding=W.DELTA_LENGTH_BYTE_ARRAY, use_dict=False), W.REQUIRED),
            ("d", W.Column(W.BYTE_ARRAY, [s[k % 4000] for k in range(n)]), W.REQUIRED),
            ("o", W.optional(W.BYTE_ARRAY, [s[k % 300] for k in range(n)], mask), W.OPTIONAL)]
    for v2, codec in ((False, 0), (True, 1), (True, 2)):
        checked, _ = _run_file(pq, ctx, W.flat(cols, 25000, v2=v2, codec=codec))
        assert checked == 3 * 4


def test_c5_dictionary_fallback(pq, ctx, delta_mode):
    """C5 layout: RLE_DICTIONARY pages (dictionary page <= 1 MiB) then DELTA_LENGTH fallback, SNAPPY."""
    from parquet_go_amd import datasets

    data = datasets.c5(rows=600_000, row_groups=2)
    checked, _ = _run_file(pq, ctx, data)
    assert checked == 2


# ---------------------------------------------------------------------------------------------
# Nesting: levels -> list offsets / presence per level + leaf validity
# ---------------------------------------------------------------------------------------------
def _check_nesting(pq, ctx, data):
    f = pq.native.File(data)
    ncols = len(f.columns())
    res = pq.reader.decode_chunks(ctx, f, 0, f.num_row_groups, list(range(ncols)))
    fr = O.FileReader(data)
    checked = 0
    for k, col in enumerate(res):
        rg, ci = divmod(k, ncols)
        c = fr.columns[ci]
        if c.max_rep == 0:
            continue
        e = oracle_chunk(fr, rg, ci)
        assert e.status == 0 and col.status == 0, (rg, c.path)
        want_levels, want_leaf = O.nest_levels(e.def_levels, e.rep_levels, c.max_def, c.rep_def)
        got_levels, got_leaf = col.nesting
        assert len(got_levels) == len(want_levels) == c.max_rep
        for lvl, ((o, v), (wo, wv)) in enumerate(zip(got_levels, want_levels)):
            np.testing.assert_array_equal(o, wo, err_msg=f"rg{rg} {c.path} level {lvl + 1} offsets")
            np.testing.assert_array_equal(v, wv, err_msg=f"rg{rg} {c.path} level {lvl + 1} validity")
        np.testing.assert_array_equal(got_leaf, want_leaf, err_msg=f"rg{rg} {c.path} leaf validity")
        assert int(got_leaf.sum()) == col.num_non_null
        checked += 1
    return checked


@pytest.mark.parametrize("v2", [False, True])
def test_nesting_list_map(pq, ctx, v2):
    assert _check_nesting(pq, ctx, fixtures.nested_list_map(n=6000, v2=v2)) == 6


def test_nesting_c4_multi_tile(pq, ctx):
    from parquet_go_amd import datasets

    assert _check_nesting(pq, ctx, datasets.c4(rows=150_000, row_groups=2)) == 6


def test_nesting_sparse_lists(pq, ctx):
    """Mostly null / empty lists: nest tiles starting more than half a tile of lists (the list
    offsets are staged in parts), for one and two repetition levels."""
    import io

    import pyarrow as pa
    import pyarrow.parquet as pqa

    rng = np.random.default_rng(11)
    n = 40000

    def row():
        u = rng.random()
        if u < 0.45:
            return None
        if u < 0.9:
            return []
        return [int(rng.integers(0, 1000)) for _ in range(rng.poisson(2))]

    a = [row() for _ in range(n)]
    b = [None if rng.random() < 0.5 else [row() for _ in range(rng.poisson(0.5))] for _ in range(n)]
    t = pa.table({"a": pa.array(a, pa.list_(pa.int64())), "b": pa.array(b, pa.list_(pa.list_(pa.int64())))})
    buf = io.BytesIO()
    pqa.write_table(t, buf, row_group_size=n, data_page_size=1 << 20, use_dictionary=False)
    assert _check_nesting(pq, ctx, buf.getvalue()) == 2


def test_nesting_deep_lists(pq, ctx):
    """list<list<int32>> and list<struct<list<string>>> from pyarrow (max_rep 2)."""
    import io

    import pyarrow as pa
    import pyarrow.parquet as pqa

    rng = np.random.default_rng(7)

    def inner(p_null):
        if rng.random() < 0.1:
            return None
        return [None if rng.random() < p_null else int(rng.integers(0, 1000)) for _ in range(rng.poisson(2))]

    a = [None if rng.random() < 0.1 else [inner(0.1) for _ in range(rng.poisson(3))] for _ in range(20000)]
    b = [None if rng.random() < 0.1 else [{"s": None if rng.random() < 0.2 else
                                           [str(rng.integers(0, 99)) for _ in range(rng.poisson(1.5))]}
                                          for _ in range(rng.poisson(2))] for _ in range(20000)]
    t = pa.table({"a": pa.array(a, pa.list_(pa.list_(pa.int32()))),
                  "b": pa.array(b, pa.list_(pa.struct([("s", pa.list_(pa.string()))])))})
    buf = io.BytesIO()
    pqa.write_table(t, buf, row_group_size=7000, data_page_size=8192, use_dictionary=False)
    assert _check_nesting(pq, ctx, buf.getvalue()) == 6


@pytest.mark.parametrize("depth,rows", [(9, 3000), (10, 3000), (17, 600), (32, 40)])
def test_nesting_deeper_than_a_window(pq, ctx, depth, rows):
    """Chains of up to 32 repeated groups (schema.go:893-990 takes any depth): the nesting outputs
    come in windows of 8 levels (one count / scan / write set per window, DevNest.lbase), every
    level's offsets and presence and the leaf validity equal oracle.nest_levels."""
    data, _ = fixtures.deep_repeated(n=rows, depth=depth, seed=depth)
    assert _check_nesting(pq, ctx, data) == 2


def test_plain_chain_layouts(pq, ctx):
    """PLAIN byte-array chains that stress the parallel chain resolution: runs of empty strings
    (every offset looks like a record start), zero bytes inside strings, strings longer than a
    segment (256 B) and than a window (64 KiB), pages spanning many windows, and dictionary pages."""
    W = fixtures.W
    rng = np.random.default_rng(43)
    col = (W.BYTE_ARRAY, 0, 0, 0)
    cases = []

    def strings(n, kind):
        out = []
        for _ in range(n):
            u = rng.random()
            if kind == "empty_runs":
                out.append(b"" if u < 0.7 else bytes(int(rng.integers(0, 3))))
            elif kind == "zeros":
                out.append(bytes(rng.integers(0, 2, int(rng.integers(0, 12))).astype(np.uint8)))
            elif kind == "long":
                out.append(rng.bytes(int(rng.integers(200, 3000))) if u < 0.8 else b"")
            elif kind == "huge":
                out.append(rng.bytes(int(rng.integers(60000, 140000))) if u < 0.3 else rng.bytes(5))
            elif kind == "lookalike":  # strings of small little-endian u32s: most offsets parse as records
                k = int(rng.integers(0, 6))
                out.append(b"".join(int(rng.integers(0, 24)).to_bytes(4, "little") for _ in range(k)))
            else:
                out.append(bytes(rng.integers(97, 123, int(rng.integers(8, 41))).astype(np.uint8)))
        return out

    for kind, n in (("empty_runs", 40000), ("zeros", 30000), ("long", 400), ("huge", 12), ("ascii", 60000),
                    ("lookalike", 50000)):
        s = strings(n, kind)
        img = _plain_chain(s)
        cases.append((col, None, (O.DATA_PAGE, n, W.PLAIN, 0, 0, img)))
        cases.append((col, None, (O.DATA_PAGE, n, W.PLAIN, 0, 0, img[: len(img) * 2 // 3])))
        cases.append((col, None, (O.DATA_PAGE, max(1, n // 2), W.PLAIN, 0, 0, img)))  # stops early
        k = int(rng.integers(0, n))
        cases.append((col, None, (O.DATA_PAGE, n, W.PLAIN, 0, 0,
                                  _plain_chain(s[:k]) + b"\x00\x00\x00\x80" + _plain_chain(s[k:]))))
        d = s[: min(n, 30000)]  # dictionary pages of several chain windows
        idx = rng.integers(0, len(d), 5000).astype(np.int32)
        w = max(1, int(len(d) - 1).bit_length())
        cases.append((col, (len(d), W.PLAIN, _plain_chain(d)),
                      (O.DATA_PAGE, 5000, W.RLE_DICTIONARY, 0, 0, bytes([w]) + W.hybrid_encode(w, idx))))
    compared, errors = _run_cases(pq, ctx, cases)
    assert compared == len(cases) and errors >= 10


def test_fused_plain_chains(pq):
    """Chunks of PLAIN byte-array pages only take the fused k_ba_chain (one read of the page bytes,
    byte bases from the page sizes, look-back between windows): the layouts of
    test_plain_chain_layouts, several pages per chunk, in one batch that decodes without the scratch
    path.  Then each defect alone in an otherwise clean batch -- a page whose chain has records past
    notNull (trailing bytes), one that ends early, an invalid length, a page with fewer bytes than
    4 * notNull -- sends the batch back to the scratch path, with the reference's results."""
    W = fixtures.W
    rng = np.random.default_rng(47)
    col = (W.BYTE_ARRAY, 0, 0, 0)
    ctx = pq.native.Context(0, profile=True)

    def strings(n, kind):
        out = []
        for _ in range(n):
            u = rng.random()
            if kind == "empty_runs":
                out.append(b"" if u < 0.7 else bytes(int(rng.integers(0, 3))))
            elif kind == "long":
                out.append(rng.bytes(int(rng.integers(200, 3000))) if u < 0.8 else b"")
            elif kind == "huge":
                out.append(rng.bytes(int(rng.integers(60000, 140000))) if u < 0.3 else rng.bytes(5))
            elif kind == "lookalike":
                k = int(rng.integers(0, 6))
                out.append(b"".join(int(rng.integers(0, 24)).to_bytes(4, "little") for _ in range(k)))
            else:
                out.append(bytes(rng.integers(97, 123, int(rng.integers(0, 41))).astype(np.uint8)))
        return out

    clean = []
    for kind, n in (("empty_runs", 40000), ("long", 400), ("huge", 12), ("ascii", 60000), ("lookalike", 50000),
                    ("ascii", 1), ("ascii", 0)):
        s = strings(n, kind)
        clean.append((col, None, (O.DATA_PAGE, n, W.PLAIN, 0, 0, _plain_chain(s))))
    stats = {}
    compared, errors = _run_cases(pq, ctx, clean, stats)
    assert compared == len(clean) and errors == 0
    assert stats.get("k_ba_chain", 0) == 1 and stats.get("k_ba_wspec", 0) == 0 and stats.get("k_ba_wcopy", 0) == 0

    # multi-page chunks through the file path (value / byte bases across pages, pages of many windows)
    words = [bytes(rng.integers(97, 123, int(k), dtype=np.uint8)) for k in rng.integers(0, 60, 200000)]
    data = W.flat([("p", W.Column(W.BYTE_ARRAY, words, use_dict=False), W.REQUIRED),
                   ("q", W.optional(W.BYTE_ARRAY, words[::-1], rng.random(200000) < 0.2, use_dict=False), W.OPTIONAL)],
                  70000, max_page_size=96 * 1024)
    checked, skipped = _run_file(pq, ctx, data)
    assert checked == 6 and skipped == 0

    s = strings(30000, "ascii")
    img = _plain_chain(s)
    defects = {
        "trailing records": (O.DATA_PAGE, 20000, W.PLAIN, 0, 0, img),
        "ends early": (O.DATA_PAGE, 30000, W.PLAIN, 0, 0, img[: len(img) * 2 // 3]),
        "negative length": (O.DATA_PAGE, 30000, W.PLAIN, 0, 0,
                            _plain_chain(s[:17000]) + b"\x00\x00\x00\x80" + _plain_chain(s[17000:])),
        "fewer bytes than lengths": (O.DATA_PAGE, 30000, W.PLAIN, 0, 0, img[:100000]),
        "trailing garbage": (O.DATA_PAGE, 30000, W.PLAIN, 0, 0, img + b"\x07\x00"),
    }
    for name, page in defects.items():
        stats = {}
        compared, _ = _run_cases(pq, ctx, clean[:3] + [(col, None, page)] + clean[3:], stats)
        assert compared == len(clean) + 1, name
        assert stats.get("k_ba_wspec", 0) == 1 and stats.get("k_ba_wcopy", 0) == 1, (name, stats)
    ctx.close()


def _dba_page(strs, total=None, plens=None, slens=None, geom=(128, 4)):
    """DELTA_BYTE_ARRAY image: prefix lengths, suffix lengths (DELTA_BINARY_PACKED), suffixes."""
    import delta_streams as DS
    pl, sl, data, prev = [], [], [], b""
    for x in strs:
        p = 0
        while p < len(prev) and p < len(x) and prev[p] == x[p]:
            p += 1
        pl.append(p)
        sl.append(len(x) - p)
        data.append(x[p:])
        prev = x
    pl = plens if plens is not None else pl
    sl = slens if slens is not None else sl
    return (DS.encode(pl, 32, geom[0], geom[1], "omit", total=total) +
            DS.encode(sl, 32, geom[0], geom[1], "omit") + b"".join(data))


def test_delta_byte_array_pages(pq, ctx, delta_mode):
    """DELTA_BYTE_ARRAY (type_bytearray.go:189-240): sorted and random strings, long shared
    prefixes, every error of decodeValues in the reference's order, count mismatch at init."""
    W = fixtures.W
    rng = np.random.default_rng(44)
    col = (W.BYTE_ARRAY, 0, 0, 0)
    cases = []
    for n in (1, 2, 9, 300, 4097, 20000):
        base = [bytes(rng.integers(97, 100, int(rng.integers(0, 30))).astype(np.uint8)) for _ in range(n)]
        for strs in (sorted(base), base, [b"common/prefix/" * 3 + x for x in sorted(base)]):
            img = _dba_page(strs)
            cases.append((col, None, (O.DATA_PAGE, n, W.DELTA_BYTE_ARRAY, 0, 0, img)))
            cases.append((col, None, (O.DATA_PAGE, n, W.DELTA_BYTE_ARRAY, 0, 0, img[: int(rng.integers(0, len(img)))])))
            cases.append((col, None, (O.DATA_PAGE, n + 2, W.DELTA_BYTE_ARRAY, 0, 0, img)))
        if n > 3:
            strs = sorted(base)
            k = int(rng.integers(1, n))
            pl = [0] * n
            pl[k] = 1000  # longer than the previous value
            cases.append((col, None, (O.DATA_PAGE, n, W.DELTA_BYTE_ARRAY, 0, 0, _dba_page(strs, plens=pl))))
            sl = [len(x) for x in strs]
            sl[k] = -3
            cases.append((col, None, (O.DATA_PAGE, n, W.DELTA_BYTE_ARRAY, 0, 0,
                                      _dba_page(strs, plens=[0] * n, slens=sl))))
            pl = [0] * n
            pl[k] = -50  # negative total
            cases.append((col, None, (O.DATA_PAGE, n, W.DELTA_BYTE_ARRAY, 0, 0,
                                      _dba_page(strs, plens=pl, slens=[len(x) for x in strs]))))
            cases.append((col, None, (O.DATA_PAGE, n, W.DELTA_BYTE_ARRAY, 0, 0, _dba_page(strs, total=n + 1))))
            cases.append((col, None, (O.DATA_PAGE, n, W.DELTA_BYTE_ARRAY, 0, 0, _dba_page(strs, geom=(96, 3)))))
    # FIXED_LEN_BYTE_ARRAY + DELTA_BYTE_ARRAY (chunk_reader.go:67-78): byteArrayDeltaDecoder yields
    # variable-length []byte whatever type_length says (no length check): values of the declared
    # length, shorter, longer and empty ones all come out as offsets + bytes
    for tl in (16, 4):
        for n in (1, 300, 5000):
            fixed = [bytes(rng.integers(97, 100, tl).astype(np.uint8)) for _ in range(n)]
            ragged = [bytes(rng.integers(97, 100, int(rng.integers(0, 2 * tl))).astype(np.uint8)) for _ in range(n)]
            for strs in (sorted(fixed), ragged):
                img = _dba_page(strs)
                col = (W.FIXED_LEN_BYTE_ARRAY, tl, 0, 0)
                cases.append((col, None, (O.DATA_PAGE, n, W.DELTA_BYTE_ARRAY, 0, 0, img)))
                cases.append((col, None, (O.DATA_PAGE, n, W.DELTA_BYTE_ARRAY, 0, 0, img[: int(rng.integers(0, len(img)))])))
    compared, errors = _run_cases(pq, ctx, cases)
    assert compared == len(cases) and errors > 15


def test_flba_mixed_chunks(pq, ctx, delta_mode):
    """FIXED_LEN_BYTE_ARRAY chunks that mix fixed-width pages (PLAIN, dictionary) with
    DELTA_BYTE_ARRAY pages (the reference decodes each page with its own decoder,
    chunk_reader.go:249-251): the whole chunk comes out as offsets + bytes, the fixed pages'
    values at their declared length, in page order; plus optional V2 pages and failing pages."""
    W = fixtures.W
    N = pq.native
    rng = np.random.default_rng(45)
    L = 16
    dict_vals = [bytes(rng.integers(0, 256, L).astype(np.uint8)) for _ in range(40)]
    dimg = b"".join(dict_vals)

    def plain_page(n):
        return (O.DATA_PAGE, n, W.PLAIN, 0, 0, rng.integers(0, 256, n * L).astype(np.uint8).tobytes())

    def dict_page(n, bad=False):
        idx = rng.integers(0, len(dict_vals), n).astype(np.int32)
        if bad:
            idx[n // 2] = 63
        return (O.DATA_PAGE, n, W.RLE_DICTIONARY, 0, 0, bytes([6]) + W.hybrid_encode(6, idx))

    def dba_page(n, ragged=False):
        strs = sorted(bytes(rng.integers(97, 99, int(rng.integers(0, 2 * L)) if ragged else L).astype(np.uint8))
                      for _ in range(n))
        return (O.DATA_PAGE, n, W.DELTA_BYTE_ARRAY, 0, 0, _dba_page(strs))

    col = (W.FIXED_LEN_BYTE_ARRAY, L, 0, 0)
    chunks = [
        (col, (len(dict_vals), W.PLAIN, dimg), [dict_page(3000), dba_page(2500), dict_page(100), dba_page(7, True)]),
        (col, None, [plain_page(5000), dba_page(3000, True), plain_page(1), plain_page(0), plain_page(2100)]),
        (col, (len(dict_vals), W.PLAIN, dimg), [plain_page(900), dict_page(4000), dba_page(4100)]),
        (col, (len(dict_vals), W.PLAIN, dimg), [dict_page(300), dba_page(600), dict_page(500, bad=True)]),
        (col, None, [plain_page(50), dba_page(70)[:5] + (dba_page(70)[5][:40],), plain_page(10)]),
    ]
    # optional column, V2 pages: levels raw before the values
    ocol = (W.FIXED_LEN_BYTE_ARRAY, L, 1, 0)
    opages = []
    for kind in ("plain", "dba", "plain"):
        n = 3000
        defs = (rng.random(n) < 0.9).astype(np.int32)
        nn = int(defs.sum())
        lv = W.hybrid_encode(1, defs)
        body = plain_page(nn)[5] if kind == "plain" else dba_page(nn)[5]
        opages.append((O.DATA_PAGE_V2, n, W.PLAIN if kind == "plain" else W.DELTA_BYTE_ARRAY, len(lv), 0, lv + body))
    chunks.append((ocol, None, opages))
    blobs, tchunks, tpages = [], [], []
    off = 0

    def add(img):
        nonlocal off
        base = (off + 63) & ~63
        blobs.append(b"\0" * (base - off) + img)
        off = base + len(img)
        return base

    for c, d, pgs in chunks:
        first = len(tpages)
        if d is not None:
            o = add(d[2])
            tpages.append(N.Page(o, len(d[2]), O.DICTIONARY_PAGE, d[0], d[1], 0, 0, len(tchunks), 0))
        for (ptype, nv, enc, dl, rl, img) in pgs:
            o = add(img)
            tpages.append(N.Page(o, len(img), ptype, nv, enc, dl, rl, len(tchunks), 0))
        tchunks.append(N.Chunk(N.Column(*c), first, len(tpages) - first, 0, 0))
    arr = np.frombuffer(b"".join(blobs) + b"\0" * N.PAYLOAD_PAD, dtype=np.uint8).copy()
    dptr = ctx.malloc(len(arr))
    try:
        ctx.h2d(dptr, arr.ctypes.data, len(arr))
        ctx.sync()
        b = N.Batch.from_tables(ctx, tchunks, tpages, dptr, off)
        b.run()
        b.sync()
        from parity import Expected

        failed = 0
        for i, (c, d, pgs) in enumerate(chunks):
            od = O.decode_dict_page(c, d[0], d[1], d[2]) if d else None
            e = Expected()
            offs, data, defs = [np.zeros(1, np.int64)], [], []
            base = 0
            for k, pg in enumerate(pgs):
                r = O.decode_page(c, *pg, od)
                if r.status and e.status == 0:
                    e.status, e.phase, e.index = r.status, r.phase, r.index
                e.nn += r.nn
                o = r.offsets if r.offsets is not None else np.arange(len(r.values) // L + 1, dtype=np.int64) * L
                offs.append(o[1:] + base)
                base += len(r.values)
                data.append(r.values)
                if r.def_levels is not None:
                    defs.append(r.def_levels)
            e.offsets, e.data = np.concatenate(offs), b"".join(data)
            e.def_levels = np.concatenate(defs) if defs else None
            cd = pq.reader.ColumnData("flba", c, b.chunk_out(i), [], ctx)
            assert cd.value_size == 0, f"chunk {i}: not laid out as byte arrays"
            assert_chunk(cd, e, where=f"flba chunk {i}")
            failed += e.status != 0
        b.close()
        assert 2 <= failed < len(chunks), failed
    finally:
        ctx.free(dptr)


@pytest.mark.parametrize("mode", ["graph", "direct", "one_stream", "profiled", "gather_serial"])
def test_launch_modes(pq, mode, monkeypatch):
    """Every launch mode decodes the same bytes: graph replay and direct launches with the side-stream
    branches (PLAIN byte-array chain beside k_scan / k_expand, nesting beside the byte-array copies),
    everything on one stream (PQH_FORK=0), and profiled runs (per-kernel events, one stream).  The
    flat file joins the chain branch before k_expand (byte-array dictionary keys need the dictionary
    sizes); the nested one joins it before the byte sums.  The C5-shaped file (dictionary pages, then
    DELTA_LENGTH fallback pages, no other branch open) runs k_ba_gather beside k_ba_expand on the
    third side stream in the graph / direct modes and after it with PQH_BA_GATHER_SERIAL=1."""
    W = pq.writer
    if mode == "direct":
        monkeypatch.setenv("PQH_GRAPH", "0")
    if mode == "one_stream":
        monkeypatch.setenv("PQH_FORK", "0")
    if mode == "gather_serial":
        monkeypatch.setenv("PQH_BA_GATHER_SERIAL", "1")
    c = pq.native.Context(0, profile=(mode == "profiled"))
    rng = np.random.default_rng(7)
    n = 30000
    words = [b"w%05d" % (i % 700) + b"x" * (i % 11) for i in rng.integers(0, 10**6, n)]
    plain = [bytes(rng.integers(97, 123, int(k), dtype=np.uint8)) for k in rng.integers(0, 40, n)]
    flat = W.flat([("d", W.Column(W.BYTE_ARRAY, words), W.REQUIRED),
                   ("p", W.Column(W.BYTE_ARRAY, plain, use_dict=False), W.REQUIRED),
                   ("i", W.Column(W.INT64, rng.integers(-2**40, 2**40, n), use_dict=False), W.REQUIRED)],
                  12000, max_page_size=48 * 1024)
    for data in (flat, pq.datasets.c4(rows=40_000, row_groups=2), pq.datasets.c5(rows=400_000, row_groups=2)):
        for _ in range(2):  # a re-run of the same batch (graph replay) too
            checked, skipped = _run_file(pq, c, data)
            assert checked > 0 and skipped == 0
    c.close()


def test_float_bit_patterns(pq, ctx):
    """NaN payloads (quiet, signalling, negative), +-0, +-inf and subnormals keep their bits through
    PLAIN and dictionary pages, V1 and V2, required and optional columns (the reference's NaN
    round trip, readwrite_test.go:1354-1432): the decoded bytes equal the written bit patterns and the
    oracle's."""
    W = fixtures.W
    rng = np.random.default_rng(3)
    f32_bits = np.array([0x7fc00000, 0x7fc00001, 0xffc00000, 0x7f800001, 0xff800001, 0x7fbfffff, 0x00000000,
                         0x80000000, 0x7f800000, 0xff800000, 0x00000001, 0x807fffff, 0x3f800000], np.uint32)
    f64_bits = np.array([0x7ff8000000000000, 0x7ff8000000000001, 0xfff8000000000000, 0x7ff0000000000001,
                         0xfff0000000000001, 0x7ff7ffffffffffff, 0, 0x8000000000000000, 0x7ff0000000000000,
                         0xfff0000000000000, 1, 0x800fffffffffffff, 0x3ff0000000000000], np.uint64)
    n = 6000
    a = f32_bits[rng.integers(0, len(f32_bits), n)]
    b = f64_bits[rng.integers(0, len(f64_bits), n)]
    d = (rng.random(n) < 0.9).astype(np.uint8)
    for v2 in (False, True):
        for use_dict in (False, True):
            cols = [("f", W.Column(W.FLOAT, a.view(np.float32), use_dict=use_dict), W.REQUIRED),
                    ("d", W.Column(W.DOUBLE, b.view(np.float64), use_dict=use_dict), W.REQUIRED),
                    ("od", W.Column(W.DOUBLE, b[d.astype(bool)].view(np.float64), def_levels=d, use_dict=use_dict),
                     W.OPTIONAL)]
            data = W.flat(cols, n // 2, v2=v2)
            checked, _ = _run_file(pq, ctx, data)
            assert checked == 2 * 3
            f = pq.native.File(data)
            res = pq.reader.decode_chunks(ctx, f, 0, f.num_row_groups, [0, 1, 2])
            for ci, want in ((0, a), (1, b), (2, b[d.astype(bool)])):
                got = np.concatenate([res[k].values.view(want.dtype) for k in range(ci, len(res), 3)])
                assert np.array_equal(got, want), (v2, use_dict, ci)


@pytest.mark.parametrize("v2", [False, True])
def test_tiny_snappy_pages(pq, ctx, v2):
    """1 KiB SNAPPY pages of every type and encoding (the reference's multi-page snappy round trip,
    readwrite_test.go:1291-1352): hundreds of pages per chunk through the host codec and through the
    device codecs, every chunk equal to the oracle's."""
    data = fixtures.flat_all_types(n=6000, v2=v2, codec=O.SNAPPY, page=1024, rows_per_group=3000)
    fr = O.FileReader(data)
    f = pq.native.File(data)
    ncols = len(f.columns())
    for dev in (False, True):
        res = pq.reader.decode_chunks(ctx, f, 0, f.num_row_groups, list(range(ncols)), device_snappy=dev)
        for k, col in enumerate(res):
            rg, ci = divmod(k, ncols)
            assert_chunk(col, oracle_chunk(fr, rg, ci), where=f"device={dev} rg{rg} {col.path}")
    hb = f.load(0, f.num_row_groups, list(range(ncols)))
    assert hb.num_pages > 20 * ncols  # (many pages per chunk)
    hb.close()
