"""The compat path of the drop-in boundary: pqh_batch_page_read, the host
materialisation of one page's pageReader.readValues(size) result (reference interfaces.go:11-18,
page_v1.go:33-63, page_v2.go:31-60) that a cgo shim boxes into []interface{} + packedArray levels
(INTEGRATION.md).  Page by page through ctypes against oracle.decode_page, including pages whose
value stream ends early (the reference's "need N value read M" partial-count error), corrupted
pages, and readValues split into several calls."""
import numpy as np
import pytest

import fixtures
from oracle import oracle as O
from test_gpu_parity import _mutate, _page_sets

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(pq):
    return pq.native.Context(0)


def _batch(pq, ctx, cases):
    """One batch, every case its own chunk (dictionary page first); returns (batch, device payload,
    data-page index of every case)."""
    N = pq.native
    blobs, chunks, pages, data_page = [], [], [], []
    off = 0

    def add(img):
        nonlocal off
        base = (off + 63) & ~63
        blobs.append(b"\0" * (base - off) + img)
        off = base + len(img)
        return base

    for col, dict_img, (ptype, nv, enc, dl, rl, img) in cases:
        first = len(pages)
        if dict_img is not None:
            o = add(dict_img[2])
            pages.append(N.Page(o, len(dict_img[2]), O.DICTIONARY_PAGE, dict_img[0], dict_img[1], 0, 0, len(chunks), 0))
        o = add(img)
        data_page.append(len(pages))
        pages.append(N.Page(o, len(img), ptype, nv, enc, dl, rl, len(chunks), 0))
        chunks.append(N.Chunk(N.Column(*col), first, len(pages) - first, 0, 0))
    arr = np.frombuffer(b"".join(blobs) + b"\0" * N.PAYLOAD_PAD, dtype=np.uint8).copy()
    d = ctx.malloc(len(arr))
    ctx.h2d(d, arr.ctypes.data, len(arr))
    b = N.Batch.from_tables(ctx, chunks, pages, d, off)
    b.run()
    b.sync()
    return b, d, data_page


def _cases(pq):
    W = fixtures.W
    rng = np.random.default_rng(61)
    cases = []
    files = [fixtures.flat_all_types(n=3000, v2=False, page=8 * 1024, rows_per_group=3000),
             fixtures.flat_all_types(n=3000, v2=True, page=8 * 1024, rows_per_group=3000),
             fixtures.nested_list_map(n=1500)]
    for data in files:
        for (path, pt, tl, md, mr), dict_img, dpages in _page_sets(pq, data):
            col = (pt, tl, md, mr)
            for pg in dpages[:3]:
                ptype, nv, enc, dl, rl, img = pg
                cases.append((col, dict_img, pg))
                # value stream cut short: readValues fails after a partial count
                cut = max(rl + dl, len(img) - int(rng.integers(1, 40)))
                cases.append((col, dict_img, (ptype, nv, enc, dl, rl, img[:cut])))
                img2 = _mutate(rng, img)
                if not (ptype == O.DATA_PAGE_V2 and rl + dl > len(img2)):
                    cases.append((col, dict_img, (ptype, nv, enc, dl, rl, img2)))
                if ptype == O.DATA_PAGE and md > 0 and mr == 0:
                    # V1 definition levels cut to half their length: the level stream ends mid-page
                    half = int.from_bytes(img[:4], "little") // 2
                    cases.append((col, dict_img, (ptype, nv, enc, dl, rl, half.to_bytes(4, "little") + img[4:])))
    # PLAIN int64 / strings whose value section is short by whole values
    vals = rng.integers(-2**40, 2**40, 500).astype(np.int64).tobytes()
    cases.append(((W.INT64, 0, 0, 0), None, (O.DATA_PAGE, 500, W.PLAIN, 0, 0, vals[:8 * 321])))
    strs = b"".join(len(x).to_bytes(4, "little") + x for x in (rng.bytes(int(rng.integers(0, 20))) for _ in range(300)))
    cases.append(((W.BYTE_ARRAY, 0, 0, 0), None, (O.DATA_PAGE, 300, W.PLAIN, 0, 0, strs[: len(strs) // 2])))
    return cases


def pq_status(name):
    from conftest import load_package

    return {v: k for k, v in load_package().native.STATUS.items()}[name]


def _check_whole(pv, got, d, r, col, exp, where):
    pt, tl, md, mr = col
    if exp.status:
        assert pv.status != 0, f"{where}: oracle fails ({exp.status}) but readValues succeeded"
        assert (pv.status, pv.phase, pv.index) == (exp.status, exp.phase, exp.index), \
            f"{where}: {(pv.status, pv.phase, pv.index)} vs {(exp.status, exp.phase, exp.index)}"
        if exp.phase == 3:  # "need %d value read %d" (page_v1.go:56-58)
            zero = exp.status in (pq_status("DICT_INDEX"), pq_status("DBA_PREFIX"))
            assert pv.values_read == (0 if zero else exp.index), f"{where}: partial count"
        return False
    assert pv.status == 0, f"{where}: status {pv.status} phase {pv.phase} index {pv.index}"
    assert pv.num_non_null == exp.nn, where
    if pv.value_size > 0:
        assert got.tobytes() == bytes(exp.values), f"{where}: values"
    else:
        offs, data = got
        assert np.array_equal(offs, exp.offsets), f"{where}: offsets"
        assert data.tobytes() == bytes(exp.values), f"{where}: bytes"
    if md > 0:
        assert np.array_equal(d, exp.def_levels), f"{where}: def levels"
    if mr > 0:
        assert np.array_equal(r, exp.rep_levels), f"{where}: rep levels"
    return True


def test_page_read_matches_read_values(pq, ctx):
    cases = _cases(pq)
    b, d, data_page = _batch(pq, ctx, cases)
    try:
        ok = failed = partial = level_ranged = 0
        for i, (col, dict_img, (ptype, nv, enc, dl, rl, img)) in enumerate(cases):
            od = O.decode_dict_page(col, dict_img[0], dict_img[1], dict_img[2]) if dict_img else None
            if od is not None and od.status:
                continue
            exp = O.decode_page(col, ptype, nv, enc, dl, rl, img, od)
            pv, got, dd, rr = b.page_read(data_page[i])
            assert pv.status != pq.native.NOT_IMPLEMENTED, f"case {i}: NOT_IMPLEMENTED"
            assert pv.num_slots == max(0, nv)
            good = _check_whole(pv, got, dd, rr, col, exp, f"case {i} col {col} enc {enc}")
            ok += good
            failed += not good
            if not good and exp.phase in (O.PHASE_REP, O.PHASE_DEF) and exp.index >= 2:
                # a ranged call ending before the failing level slot: the device decoded no values of
                # this page, so the call reports the page's error (documented divergence: the
                # reference would return the range); it never reads another page's values
                pr, _, _, _ = b.page_read(data_page[i], 0, exp.index // 2)
                assert (pr.status, pr.phase, pr.index) == (exp.status, exp.phase, exp.index), f"case {i}: ranged"
                level_ranged += 1
            partial += (not good) and exp.phase == 3 and exp.index > 0
            if good and nv > 2:
                # readValues(size) in three calls: the concatenation is the whole-page result
                cuts = [0, nv // 3, 2 * nv // 3, nv]
                parts = [b.page_read(data_page[i], cuts[k], cuts[k + 1] - cuts[k]) for k in range(3)]
                assert all(p[0].status == 0 for p in parts)
                assert sum(p[0].num_slots for p in parts) == nv
                if pv.value_size > 0:
                    assert b"".join(p[1].tobytes() for p in parts) == got.tobytes(), f"case {i}: split values"
                else:
                    assert b"".join(p[1][1].tobytes() for p in parts) == got[1].tobytes(), f"case {i}: split bytes"
                if col[2] > 0:
                    assert np.array_equal(np.concatenate([p[2] for p in parts]), dd), f"case {i}: split def"
        assert ok > 30 and failed > 10 and partial > 3 and level_ranged > 0, (ok, failed, partial, level_ranged)
    finally:
        b.close()
        ctx.free(d)


def test_shim_walk_device(pq, ctx):
    """INTEGRATION.md's gpuPageReader inside the reference's readPages (tests/shim_adapter.py):
    `read` consumes CompressedPageSize bytes and reports the batch's load error for its page,
    readValues(size) is pqh_batch_page_read of the chunk's i-th data page -- every chunk of
    multi-page V1 / V2 / dictionary / SNAPPY / nested / pyarrow files walks like the oracle's
    dataPageReaderV1/V2, three readValues calls per page compared value for value, level for level."""
    import test_shim_walk as TS

    batches = []

    def batch_for(hb):
        b = pq.native.Batch.from_host(ctx, hb)
        b.run()
        b.sync()
        batches.append(b)
        return b

    n = 0
    for name, data in TS.files():
        n += TS.walk_both(pq, data, backend="device", batch_for=batch_for)
    for b in batches:
        b.close()
    assert n > 100
