"""The reference's nil INT96 values (type_int96.go:21-42, type_dict.go:40-60).

int96PlainDecoder.decodeValues reads 12 bytes per slot with a plain Read, not ReadFull: when the
page's values end inside a value, that Read returns the few bytes left with a nil error, the value is
dropped and the loop goes on.  Before the last slot the next Read returns io.EOF (an error); at the
LAST slot the loop simply ends and decodeValues returns (len(dst), nil) with dst[nn-1] never
assigned -- readValues succeeds and hands a nil interface{} up.  A dictionary page decodes its
entries the same way, so its last entry can be that nil, and dictDecoder.decodeValues copies it to
every value whose key indexes it.  The record assembly then leaves a nil value of a non-repeated
leaf out of the row (getNextData: data == nil), and panics on a repeated one (int96Store.append's
type assertion, a runtime.Error that FileReader.recover re-panics, file_reader.go:177-184).

Oracle (oracle/refdecode.c) and product (pqh_chunk_out.value_nil, pqh_page_result.num_nil,
pqh_batch_page_read's value_nil) carry these as 12 zero bytes plus a nil mark; the shim boxes them as
nil.  CPU tests pin the oracle on crafted pages and files; GPU tests compare the device with it.
"""
import numpy as np
import pytest

import pqcraft
from oracle import oracle as O
from test_records import _pkg, error_outcome, oracle_next_rows

ERR_EOF = 1  # PQH_ERR_EOF (include/pqhip.h)
COL_REQ = (O.INT96, 0, 0, 0)
COL_OPT = (O.INT96, 0, 1, 0)
PLAIN, RLE_DICTIONARY = 0, 8


def _vals(rng, n):
    return rng.integers(0, 256, (n, 12), dtype=np.uint8)


def _plain_cases(rng):
    """(column, dictionary, page) cases + what the oracle must say: PLAIN INT96 pages of nn values
    whose values section holds 12 * (nn - 1) + k bytes for k = 0..11, and 12 * (nn - 2) + k."""
    W = _pkg().writer
    cases = []
    for nn in (1, 2, 7, 300):
        v = _vals(rng, nn).tobytes()
        for k in range(12):
            for short in (1, 2):
                if nn - short < 0:
                    continue
                blk = v[:12 * (nn - short) + k]
                # nil slot: exactly the last value short; anything else fails (io.EOF)
                want = "nil" if short == 1 and k else "error"
                if nn - short == 0 and k == 0 and short == 1:
                    want = "error"
                for opt in (False, True):
                    if opt:  # an optional column: nulls among the slots, the same values section
                        d = np.ones(nn + 3, np.uint8)
                        d[rng.choice(nn + 3, 3, replace=False)] = 0  # three nulls among nn values
                        lv = W.hybrid_encode(1, d)
                        for v2 in (False, True):
                            if v2:
                                cases.append((COL_OPT, None, (O.DATA_PAGE_V2, len(d), PLAIN, len(lv), 0, lv + blk), want))
                            else:
                                img = len(lv).to_bytes(4, "little") + lv + blk
                                cases.append((COL_OPT, None, (O.DATA_PAGE, len(d), PLAIN, 0, 0, img), want))
                    else:
                        cases.append((COL_REQ, None, (O.DATA_PAGE, nn, PLAIN, 0, 0, blk), want))
    return cases


def _dict_cases(rng):
    """Dictionary pages of K INT96 entries whose image ends inside the last entry (nil entry) or an
    earlier one (error), with data pages whose keys do / do not reach the last entry."""
    W = _pkg().writer
    cases = []
    for K in (1, 2, 5, 40):
        dv = _vals(rng, K).tobytes()
        w = max(1, int(K - 1).bit_length()) if K > 1 else 0
        for k in (1, 5, 11):
            for n in (1, 9, 1000):
                keys = rng.integers(0, K, n).astype(np.int32)
                if n > 3:
                    keys[rng.integers(0, n, 3)] = K - 1
                img = bytes([w]) + W.hybrid_encode(w, keys)
                cases.append((COL_REQ, (K, PLAIN, dv[:12 * (K - 1) + k]), (O.DATA_PAGE, n, RLE_DICTIONARY, 0, 0, img),
                              "nil" if (keys == K - 1).any() else "ok"))
                if K >= 2:
                    cases.append((COL_REQ, (K, PLAIN, dv[:12 * (K - 2) + k]), (O.DATA_PAGE, n, RLE_DICTIONARY, 0, 0, img),
                                  "dict_error"))
                low = np.minimum(keys, max(0, K - 2)) if K >= 2 else None
                if low is not None:  # keys below the nil entry: no nil value at all
                    img2 = bytes([w]) + W.hybrid_encode(w, low)
                    cases.append((COL_REQ, (K, PLAIN, dv[:12 * (K - 1) + k]),
                                  (O.DATA_PAGE, n, RLE_DICTIONARY, 0, 0, img2), "ok"))
    return cases


def _oracle(case):
    col, dict_img, (ptype, nv, enc, dl, rl, img), _ = case
    od = O.decode_dict_page(col, dict_img[0], dict_img[1], dict_img[2]) if dict_img else None
    if od is not None and od.status:
        return od, None
    return od, O.decode_page(col, ptype, nv, enc, dl, rl, img, od)


def test_oracle_plain_short_values():
    rng = np.random.default_rng(96)
    cases = _plain_cases(rng)
    nils = 0
    for case in cases:
        _, r = _oracle(case)
        col, _, (ptype, nv, enc, dl, rl, img), want = case
        if want == "nil":
            assert r.status == O.OK and r.nil is not None, case[2][:3]
            assert r.nil.tolist() == [0] * (r.nn - 1) + [1]
            assert len(r.values) == 12 * r.nn and r.values[-12:] == b"\0" * 12
            # the values section is the image's tail: 12 * (nn - 1) full values + the short one
            full = 12 * (r.nn - 1)
            section = img[len(img) - full - len(img) % 12:] if col == COL_REQ else None
            if section is not None:
                assert r.values[:-12] == section[:full]
            nils += 1
        else:
            assert r.status == ERR_EOF and r.nil is None, (case[2][:3], r.status)
    assert nils >= 40


def test_oracle_dictionary_nil_entry():
    rng = np.random.default_rng(97)
    seen = set()
    for case in _dict_cases(rng):
        od, r = _oracle(case)
        col, (K, _, dimg), (ptype, nv, enc, dl, rl, img), want = case
        seen.add(want)
        if want == "dict_error":
            assert od.status == ERR_EOF
            continue
        assert od.status == O.OK and od.nil_last and od.num_values == K
        assert od.values[-12:] == b"\0" * 12
        keys = O.hybrid_decode(img[0], img[1:], nv)[1]
        assert r.status == O.OK
        if want == "nil":
            assert r.nil is not None and np.array_equal(r.nil, (keys == K - 1).astype(np.uint8))
            got = np.frombuffer(r.values, np.uint8).reshape(-1, 12)
            assert not got[keys == K - 1].any()
        else:
            assert r.nil is None
    assert seen == {"nil", "ok", "dict_error"}


def _nil_files(rng):
    """Crafted files (name, data, repetition): required / optional / repeated INT96 columns whose
    pages end inside their last value, a dictionary with a nil last entry, and clean row groups
    around them."""
    _pkg()
    v = _vals(rng, 64).tobytes()
    req = pqcraft.int96_file([
        (None, [(v[:12 * 10], 10, PLAIN, None, None), (v[:12 * 6 + 5], 7, PLAIN, None, None)]),
        (None, [(v[:12 * 3 + 11], 4, PLAIN, None, None)]),
        ((v[:12 * 4 + 2], 5), [(bytes([3]) + _pkg().writer.hybrid_encode(3, np.array([0, 4, 1, 4, 2, 3], np.int32)),
                                6, RLE_DICTIONARY, None, None)]),
    ])
    d = np.array([1, 0, 1, 1, 0, 1], np.uint8)
    opt = pqcraft.int96_file([(None, [(v[:12 * 3 + 4], 6, PLAIN, d, None)]),
                              (None, [(v[:12 * 4], 6, PLAIN, d, None)])], repetition=pqcraft.OPTIONAL)
    r = np.array([0, 1, 1, 0, 1], np.uint8)
    rep = pqcraft.int96_file([(None, [(v[:12 * 5], 5, PLAIN, np.ones(5, np.uint8), r)]),
                              (None, [(v[:12 * 4 + 7], 5, PLAIN, np.ones(5, np.uint8), r)])],
                             repetition=pqcraft.REPEATED)
    return [("required", req), ("optional", opt), ("repeated", rep)]


def test_oracle_records_with_nil_values():
    """The assembly over the oracle's pages: a nil value of a required / optional leaf is absent
    from its row; a repeated leaf's nil panics (the reference's process would crash)."""
    rng = np.random.default_rng(98)
    files = dict(_nil_files(rng))
    rows = oracle_next_rows(files["required"])
    assert len(rows) == 10 + 7 + 4 + 6
    assert rows[16] == {} and rows[20] == {} and all("t" in rows[i] for i in range(16))
    assert [("t" in x) for x in rows[21:]] == [True, False, True, False, True, True]  # keys 4 = nil entry
    rows = oracle_next_rows(files["optional"])
    assert [("t" in x) for x in rows[:6]] == [True, False, True, True, False, False]
    rows = oracle_next_rows(files["repeated"])
    assert rows[:2] == [{"t": [x for x in rows[0]["t"]]}, rows[1]] and len(rows[0]["t"]) == 3
    assert ("panic",) in rows


def test_shim_walk_int96_nil_host():
    """INTEGRATION.md's readPages walk over the crafted files with the host-side page results (CPU)."""
    from test_shim_walk import walk_both

    for name, data in _nil_files(np.random.default_rng(99)):
        assert walk_both(_pkg(), data) >= 2, name


# ---------------------------------------------------------------------------------------------
# the device
# ---------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def ctx(pq):
    return pq.native.Context(0)


@pytest.mark.gpu
def test_gpu_int96_nil_pages(pq, ctx):
    """Crafted PLAIN / dictionary INT96 pages through one batch: status, values (zeros at nil
    slots) and the nil marks equal the oracle's, case by case."""
    from test_gpu_parity import _run_cases

    rng = np.random.default_rng(100)
    cases = _plain_cases(rng) + _dict_cases(rng)
    compared, errors = _run_cases(pq, ctx, [c[:3] for c in cases])
    assert compared == len(cases)
    assert errors == sum(c[3] in ("error", "dict_error") for c in cases)


@pytest.mark.gpu
def test_gpu_int96_nil_files(pq, ctx):
    """The crafted files through FileReader.NextRow (GPU decode, value-by-value assembly of the row
    groups with nil values), the shim's device walk (pqh_batch_page_read's value_nil) and the
    chunk outputs' nil counts."""
    from test_records import _read_batches
    from test_shim_walk import walk_both

    for name, data in _nil_files(np.random.default_rng(98)):
        want = oracle_next_rows(data)
        fr = pq.reader.FileReader(data, ctx=ctx)
        got = []
        while True:
            try:
                got.append(fr.NextRow())
            except EOFError:
                break
            except (pq.reader.DecodeError, pq.records.RecordError) as e:
                got.append(error_outcome(e))
            assert len(got) <= len(want) + 1
        fr.close()
        assert got == want, name
        assert _read_batches(pq, ctx, data, 4) == want, name
        assert walk_both(pq, data, backend="device", batch_for=lambda hb: _batch(pq, ctx, hb)) >= 2, name
        f = pq.native.File(data)
        hb = f.load(0, f.num_row_groups, [0])
        b = pq.native.Batch.from_host(ctx, hb)
        b.run()
        b.sync()
        res = b.page_results(hb.num_pages)
        fro = O.FileReader(data)
        for rg in range(f.num_row_groups):
            o = b.chunk_out(rg)
            exp = [r for r in O.decode_chunk(fro.read_chunk(rg, 0))]
            want_nil = sum(int(r.nil.sum()) for r in exp if r.nil is not None)
            assert o.num_nil == want_nil, (name, rg)
            assert (o.value_nil is not None and o.value_nil != 0) or want_nil == 0
        assert sum(r.num_nil for r in res) == sum(b.chunk_out(rg).num_nil for rg in range(f.num_row_groups))
        b.close()
        hb.close()
        f.close()


def _batch(pq, ctx, hb):
    b = pq.native.Batch.from_host(ctx, hb)
    b.run()
    b.sync()
    return b


@pytest.mark.gpu
def test_gpu_int96_plain_on_flat(pq, ctx):
    """PLAIN INT96 chunks stay on the one-launch k_flat path: a clean file decodes
    there (paths()['flat_active'], no fallback) bit for bit as the oracle; a page whose short last
    value is the reference's nil fails k_flat's speculation, and the three-kernel decode marks the
    nil (zeros, value_nil, num_nil) as the oracle does."""
    rng = np.random.default_rng(101)
    v = _vals(rng, 64).tobytes()
    clean = pqcraft.int96_file([(None, [(v[:12 * 20], 20, PLAIN, None, None), (v[:12 * 9], 9, PLAIN, None, None)]),
                                (None, [(v[:12 * 33], 33, PLAIN, None, None)])])
    short = pqcraft.int96_file([(None, [(v[:12 * 20], 20, PLAIN, None, None), (v[:12 * 8 + 3], 9, PLAIN, None, None)])])
    for data, nil in ((clean, 0), (short, 1)):
        f = pq.native.File(data)
        hb = f.load(0, f.num_row_groups, [0])
        b = pq.native.Batch.from_host(ctx, hb)
        b.run()
        b.sync()
        paths = b.paths()
        if nil:
            assert paths["flat_fallbacks"] == 1 and not paths["flat_active"], paths
        else:
            assert paths["flat_active"] == 1 and paths["flat_fallbacks"] == 0, paths
        fro = O.FileReader(data)
        for rg in range(f.num_row_groups):
            o = b.chunk_out(rg)
            exp = O.decode_chunk(fro.read_chunk(rg, 0))
            assert all(r.status == 0 for r in exp)
            want = b"".join(r.values for r in exp)
            assert ctx.d2h_array(o.values, o.num_non_null * 12).tobytes() == want
            assert o.num_nil == sum(int(r.nil.sum()) for r in exp if r.nil is not None)
        assert sum(b.chunk_out(rg).num_nil for rg in range(f.num_row_groups)) == nil
        b.close()
        hb.close()
        f.close()


@pytest.mark.gpu
def test_gpu_int96_nil_entry_with_bad_key(pq, ctx):
    """A dictionary whose last entry is the reference's nil, and a data page that indexes it before
    an out-of-range key: the page fails with DICT_INDEX and returns 0 values (type_dict.go:52-54), so
    no nil counts for it (num_nil only over the values the reference returns); the
    page before it keeps its nils."""
    W = _pkg().writer
    rng = np.random.default_rng(102)
    v = _vals(rng, 8).tobytes()
    dpage = (v[:12 * 4 + 2], 5)  # entries 0..3, then the short nil entry 4
    good = bytes([3]) + W.hybrid_encode(3, np.array([4, 0, 4, 1], np.int32))
    bad = bytes([4]) + W.hybrid_encode(4, np.array([4, 1, 4, 9, 0], np.int32))  # key 9 >= 5
    data = pqcraft.int96_file([(dpage, [(good, 4, RLE_DICTIONARY, None, None), (bad, 5, RLE_DICTIONARY, None, None)])])
    f = pq.native.File(data)
    hb = f.load(0, 1, [0])
    b = pq.native.Batch.from_host(ctx, hb)
    b.run()
    b.sync()
    res = b.page_results(hb.num_pages)
    exp = O.decode_chunk(O.FileReader(data).read_chunk(0, 0))
    data_res = [r for r, p in zip(res, hb.pages()) if p.page_type != O.DICTIONARY_PAGE]
    assert [r.status for r in data_res] == [e.status for e in exp] == [0, 10]
    assert [r.num_nil for r in data_res] == [2, 0]
    assert b.chunk_out(0).num_nil == 2
    b.close()
    hb.close()
    f.close()
