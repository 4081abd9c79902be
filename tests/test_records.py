"""Row materialisation: FileReader.NextRow's records, pinned to the reference's
record-shredding known answers (tests/golden/dremel_kat.json, from data_store_test.go:18-497: the
rows the reference shreds and reads back unchanged).

CPU: the assembly (records.RowAssembler, a restatement of Column.getData / ColumnStore.get,
schema.go:216-312 / data_store.go:262-309) over the KAT levels, and over the oracle's decode of the
KAT rows written to a file.  GPU: the same files read row by row through reader.FileReader.NextRow
(device decode + host assembly), and multi-page / multi-row-group files whose records must equal the
assembly over the oracle's per-page readValues results."""
import json
import os
import struct

import numpy as np
import pytest

import fixtures
from oracle import oracle as O

KATS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "dremel_kat.json")))


def _pkg():
    from conftest import load_package

    return load_package()


def kat_file(kat, **kw):
    """The KAT's rows as a file: schema from the flat (path, repetition) list, one INT64 leaf column
    per KAT leaf with its asserted levels and values."""
    W = _pkg().writer
    reps = {"REQUIRED": W.REQUIRED, "OPTIONAL": W.OPTIONAL, "REPEATED": W.REPEATED}
    paths = [p for p, _ in kat["schema"]]
    leaves = {lf["path"]: lf for lf in kat["leaves"]}

    def kids(prefix):
        depth = prefix.count(".") + 1 if prefix else 0
        return [p for p in paths if p.count(".") == depth and (not prefix or p.startswith(prefix + "."))]

    schema = [W.element("schema", repetition=-1, num_children=len(kids("")))]
    cols = []

    def walk(path, rep):
        ch = kids(path)
        name = path.rsplit(".", 1)[-1]
        if not ch:
            lf = leaves[path]
            schema.append(W.element(name, W.INT64, reps[rep]))
            cols.append(W.Column(W.INT64, np.array(lf["values"], np.int64),
                                 def_levels=lf["def"] if lf["max_def"] else None,
                                 rep_levels=lf["rep"] if lf["max_rep"] else None, **kw))
            return
        schema.append(W.element(name, repetition=reps[rep], num_children=len(ch)))
        for c in ch:
            walk(c, dict(kat["schema"])[c])

    for p in kids(""):
        walk(p, dict(kat["schema"])[p])
    return W.write(schema, cols, [len(kat["rows"])])


class _El:
    def __init__(self, column, max_def, max_rep, repetition, num_children):
        self.column, self.max_def, self.max_rep = column, max_def, max_rep
        self.repetition, self.num_children = repetition, num_children


def _oracle_schema(fr):
    """The flat schema list (name, element) of a file from the oracle's footer parse, with the
    levels readColumnSchema derives (schema.go:893-990)."""
    els = fr.meta[2]
    out = []
    pos = [0]
    leaf = [0]

    def walk(d, r):
        e = els[pos[0]]
        pos[0] += 1
        rep = e.get(3, -1)
        nd = d + (1 if rep in (1, 2) else 0)
        nr = r + (1 if rep == 2 else 0)
        n = e.get(5, 0)
        name = e.get(4, b"")
        name = name.decode("utf-8", "surrogateescape") if isinstance(name, bytes) else name
        if n == 0:
            out.append((name, _El(leaf[0], nd, nr, rep, 0)))
            leaf[0] += 1
            return
        out.append((name, _El(-1, nd, nr, rep, n)))
        for _ in range(n):
            walk(nd, nr)

    root = els[0]
    pos[0] = 1
    out.append((root.get(4, b"schema"), _El(-1, 0, 0, -1, root.get(5, 0))))
    while pos[0] < len(els):  # readSchema: top-level children until the list ends (schema.go:992-1015)
        walk(0, 0)
    return out


def _go_values(r, col):
    """One oracle page's dense values as the reference's Go values."""
    pt = col.physical_type
    if r.offsets is not None:
        return [r.values[r.offsets[i]:r.offsets[i + 1]] for i in range(len(r.offsets) - 1)]
    np_t = {O_INT32: np.int32, O_INT64: np.int64, O_FLOAT: np.float32, O_DOUBLE: np.float64}.get(pt)
    if pt == O_BOOLEAN:
        return [bool(b) for b in r.values]
    if np_t is not None:
        return np.frombuffer(r.values, np_t).tolist()
    size = r.value_size
    vals = [r.values[i:i + size] for i in range(0, len(r.values), size)]
    if r.nil is not None:  # the reference's nil INT96 values (type_int96.go:21-42)
        vals = [None if r.nil[i] else v for i, v in enumerate(vals)]
    return vals


O_BOOLEAN, O_INT32, O_INT64, O_INT96, O_FLOAT, O_DOUBLE = range(6)


def oracle_rows(data):
    """Every record of a file, assembled over the oracle's per-page readValues results."""
    R = _pkg().records
    fr = O.FileReader(data)
    schema = _oracle_schema(fr)
    rows = []
    for rg in range(len(fr.row_groups)):
        stores = {}
        for ci, col in enumerate(fr.columns):
            ch = fr.read_chunk(rg, ci)
            assert ch.status == 0
            pages = []
            for r in O.decode_chunk(ch):
                assert r.status == 0
                n = r.num_values
                d = r.def_levels if r.def_levels is not None else np.zeros(n, np.uint8)
                rp = r.rep_levels if r.rep_levels is not None else np.zeros(n, np.uint8)
                pages.append((R.PAGE_OK, n, d, rp, lambda r=r, col=col: _go_values(r, col)))
            el = [e for _, e in schema if e.num_children == 0][ci]
            stores[ci] = R.LeafStore(None, col.path, el.repetition, col.max_def, col.max_rep, pages)
        asm = R.RowAssembler(schema, None, fr.row_group_num_rows(rg), stores=stores)
        rows.extend(asm.next_row() for _ in range(fr.row_group_num_rows(rg)))
    return rows


def _norm(v):
    """bytes -> str so KAT rows (JSON) and Go []byte values compare; floats by bit pattern."""
    if isinstance(v, dict):
        return {k: _norm(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_norm(x) for x in v]
    if isinstance(v, (bytes, bytearray)):
        return bytes(v).decode("latin-1")
    if isinstance(v, float):  # NaN != NaN: compare float values by their bits
        return ("f64", struct.pack("<d", v))
    return v


@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_assembly_matches_reference_records(kat):
    """The assembly over the KAT's asserted levels reads back the KAT's rows (the reference's
    AddData -> getData round trip, data_store_test.go)."""
    R = _pkg().records
    reps = {"REQUIRED": 0, "OPTIONAL": 1, "REPEATED": 2}
    data = kat_file(kat)
    fr = O.FileReader(data)
    schema = _oracle_schema(fr)
    by_path = {lf["path"]: lf for lf in kat["leaves"]}
    stores = {}
    for ci, col in enumerate(fr.columns):
        lf = by_path[col.path]
        n = len(lf["def"])
        page = (R.PAGE_OK, n, np.array(lf["def"], np.uint8), np.array(lf["rep"], np.uint8), lambda lf=lf: list(lf["values"]))
        stores[ci] = R.LeafStore(None, col.path, reps[dict(kat["schema"])[col.path]], lf["max_def"], lf["max_rep"],
                                 [page])
    asm = R.RowAssembler(schema, None, len(kat["rows"]), stores=stores)
    got = [asm.next_row() for _ in kat["rows"]]
    assert got == kat["rows"]


@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_oracle_file_records_match_reference(kat):
    """KAT rows -> file (reference-writer layout) -> oracle readValues -> assembly == KAT rows."""
    assert oracle_rows(kat_file(kat)) == kat["rows"]


def _read_all(pq, ctx, data, *columns, columnar=True, stats=None):
    fr = pq.reader.FileReader(data, *columns, ctx=ctx, columnar=columnar)
    rows = []
    while True:
        try:
            rows.append(fr.NextRow())
        except EOFError:
            break
    fr.close()
    if stats is not None:
        for k, v in fr.assembled.items():
            stats[k] = stats.get(k, 0) + v
    return rows


def error_outcome(e):
    """A failing NextRow call as recorded by the tests: ("error", status) when a row group fails to
    load (reader.DecodeError; the oracle side records its status), ("error", status, phase, index,
    page) when the assembly reaches a page that failed to decode (records.RecordError: the same
    attributes from the columnar and the value-by-value assembly)."""
    if isinstance(e, _pkg().records.ReferencePanic):  # (the reference would crash here)
        return ("panic",)
    if isinstance(e, _pkg().records.RecordError):
        return ("error", e.status, e.phase, e.index, e.page)
    return ("error", e.status)


def _read_batches(pq, ctx, data, n):
    """NextBatch(n) until the end, errors recorded as NextRow's are (error_outcome)."""
    fr = pq.reader.FileReader(data, ctx=ctx)
    out = []
    while True:
        try:
            b = fr.NextBatch(n)
        except (pq.reader.DecodeError, pq.records.RecordError) as e:
            out.append(error_outcome(e))
            continue
        if not b:
            break
        assert len(b) <= n
        out.extend(b)
    fr.close()
    return out


@pytest.fixture(scope="module")
def ctx():
    return _pkg().native.Context(0)


@pytest.mark.gpu
@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_next_row_matches_reference_records(pq, ctx, kat):
    """NextRow over the GPU decode of the KAT file returns exactly the reference's rows, then EOF."""
    stats = {}
    for use_dict in (True, False):
        data = kat_file(kat, use_dict=use_dict)
        assert _read_all(pq, ctx, data, stats=stats) == kat["rows"], f"use_dict={use_dict}"
        assert _read_batches(pq, ctx, data, 3) == kat["rows"]
    assert stats["columnar"] >= 1  # the device's nesting outputs assembled the rows


@pytest.mark.gpu
@pytest.mark.parametrize("v2", [False, True])
def test_next_row_multi_page(pq, ctx, v2):
    """Nested LIST / MAP columns over many pages and two row groups, and the flat all-types file:
    NextRow (GPU) == assembly over the oracle's pages, row by row."""
    for data in (fixtures.nested_list_map(n=3000, v2=v2), fixtures.flat_all_types(n=4000, v2=v2)):
        want = oracle_rows(data)
        stats = {}
        got = _read_all(pq, ctx, data, stats=stats)
        assert stats == {"columnar": len(O.FileReader(data).row_groups), "value_by_value": 0}
        assert len(got) == len(want) == O.FileReader(data).num_rows
        for i, (g, w) in enumerate(zip(got, want)):
            assert _norm(g) == _norm(w), f"row {i}: {g} vs {w}"
        assert [_norm(x) for x in _read_batches(pq, ctx, data, 700)] == [_norm(w) for w in want]


@pytest.mark.gpu
def test_next_row_columnar_vs_value_by_value(pq, ctx):
    """Deep chains (value-by-value where getFirstRDLevel's quirk applies) and a columnar-only file:
    FileReader's two assembly paths over the same GPU decode give identical rows."""
    for data in (fixtures.deep_repeated(n=400, depth=10)[0], fixtures.deep_repeated(n=1500, depth=4, seed=2)[0],
                 fixtures.nested_list_map(n=2000)):
        want = oracle_rows(data)
        for columnar in (True, False):
            got = _read_all(pq, ctx, data, columnar=columnar)
            assert [_norm(g) for g in got] == [_norm(w) for w in want], columnar


@pytest.mark.gpu
def test_next_row_selected_columns_and_cursor(pq, ctx):
    """WithColumns: unselected leaves are skipped (absent from the rows); SeekToRowGroup is 1-based
    as in the reference (file_reader.go:193-198) and SkipRowGroup moves NextRow to the next group."""
    data = fixtures.nested_list_map(n=2000)
    want = oracle_rows(data)
    nrg0 = O.FileReader(data).row_group_num_rows(0)
    got = _read_all(pq, ctx, data, "m")
    assert [_norm(r) for r in got] == [{k: v for k, v in _norm(w).items() if k == "m"} for w in want]
    fr = pq.reader.FileReader(data, ctx=ctx)
    fr.SeekToRowGroup(2)
    assert _norm(fr.NextRow()) == _norm(want[nrg0])
    with pytest.raises(IndexError):
        fr.SeekToRowGroup(0)
    fr2 = pq.reader.FileReader(data, ctx=ctx)
    assert _norm(fr2.NextRow()) == _norm(want[0])
    fr2.SkipRowGroup()
    assert _norm(fr2.NextRow()) == _norm(want[nrg0])
    fr2.SkipRowGroup()
    with pytest.raises(EOFError):
        fr2.NextRow()
    fr.close()
    fr2.close()


# ---------------------------------------------------------------------------------------------
# Error timing (chunk_reader.go:364-404, data_store.go:236-269): a row group fails only on
# readChunk errors; a readValues error surfaces at the row that reaches the failing page
# ---------------------------------------------------------------------------------------------
def oracle_next_rows(data):
    """Every NextRow outcome of a file (a row dict, or ("error", status)), from the oracle's pages:
    readRowGroupData fails at the first column whose readChunk fails (walker / codec / page load,
    phase 0) -- one failing NextRow, then the next row group; otherwise each NextRow assembles a row,
    and a page whose readValues failed raises when the assembly reaches it (rows before it are
    returned).  Page 0's first readValues error is swallowed at load (chunk_reader.go:368-370) and
    raised by the first get; the reference re-runs readValues on the partly consumed decoders there,
    the restatement raises the first attempt's error (documented divergence)."""
    R = _pkg().records
    fr = O.FileReader(data)
    schema = _oracle_schema(fr)
    out = []
    for rg in range(len(fr.row_groups)):
        stores, rg_err = {}, None
        for ci, col in enumerate(fr.columns):
            ch = fr.read_chunk(rg, ci)
            if ch.status:
                rg_err = ch.status
                break
            res = O.decode_chunk(ch)
            load = [r for r in res if r.status and r.phase == O.PHASE_LOAD]
            if load:
                rg_err = load[0].status
                break
            pages = []
            for r in res:
                n = r.num_values
                d = r.def_levels if r.def_levels is not None else np.zeros(n, np.uint8)
                rp = r.rep_levels if r.rep_levels is not None else np.zeros(n, np.uint8)
                pages.append((R.PageResult(r.status, r.phase, r.index), n, d, rp,
                              lambda r=r, col=col: _go_values(r, col)))
            el = [e for _, e in schema if e.num_children == 0][ci]
            stores[ci] = R.LeafStore(None, col.path, el.repetition, col.max_def, col.max_rep, pages)
        if rg_err is not None:
            out.append(("error", rg_err))
            continue
        asm = R.RowAssembler(schema, None, fr.row_group_num_rows(rg), stores=stores)
        for _ in range(fr.row_group_num_rows(rg)):
            try:
                out.append(asm.next_row())
            except R.RecordError as e:
                out.append(error_outcome(e))
    return out


def _page_blocks(data, rg, ci):
    """File offsets of a chunk's page blocks: [(page_type, start, length)] (the readPages walk)."""
    fr = O.FileReader(data)
    md = fr.row_groups[rg][1][ci][3]
    pos = md.get(11, md.get(9))
    end = pos + md[7]
    out = []
    while pos < end:
        rd = O.CompactReader(fr.data, pos)
        ph = rd.struct()
        pos = rd.pos
        out.append((ph[1], pos, ph[3]))
        pos += ph[3]
    return out


def _error_file():
    """3 row groups x (dictionary INT64, optional DOUBLE, dictionary strings), V1, small pages."""
    W = _pkg().writer
    rng = np.random.default_rng(71)
    n = 9000
    a = rng.integers(0, 100, n) * 1000
    b = rng.normal(size=n)
    bmask = rng.random(n) < 0.2
    c = [b"s%03d" % k for k in rng.integers(0, 300, n)]
    cols = [("a", W.Column(W.INT64, a), W.REQUIRED), ("b", W.optional(W.DOUBLE, b, bmask, use_dict=False), W.OPTIONAL),
            ("c", W.Column(W.BYTE_ARRAY, c), W.REQUIRED)]
    return W.flat(cols, 3000, max_page_size=4 * 1024)


def _corrupt(data, edits):
    """edits: [(rg, column, data page k, fn(bytearray block) -> None)]."""
    buf = bytearray(data)
    for rg, ci, k, fn in edits:
        blocks = [b for b in _page_blocks(data, rg, ci) if b[0] != O.DICTIONARY_PAGE]
        _, s, ln = blocks[k]
        blk = bytearray(buf[s:s + ln])
        fn(blk)
        assert len(blk) == ln
        buf[s:s + ln] = blk
    return bytes(buf)


def _bad_key(blk):  # dictionary indices (after the width byte): a run of all-ones keys, out of range
    blk[len(blk) // 2: len(blk) // 2 + 4] = b"\xff" * 4


def _short_levels(blk):  # V1 definition levels' length prefix cut to one byte: the level stream ends early
    blk[0:4] = (1).to_bytes(4, "little")


def _bad_width(blk):  # dictionary bit width 33: dictDecoder.init fails (type_dict.go:23-30), a load error
    blk[0] = 33


ERROR_CASES = {
    "dict_index_page2": [(0, 0, 2, _bad_key)],
    "def_levels_page0": [(1, 1, 0, _short_levels)],
    "load_error_rg0": [(0, 2, 1, _bad_width)],
    "mixed": [(0, 1, 3, _short_levels), (1, 2, 0, _bad_width), (2, 0, 1, _bad_key), (2, 2, 4, _bad_key)],
}


@pytest.mark.parametrize("case", sorted(ERROR_CASES))
def test_oracle_error_timing(case):
    """The restated error timing over the corrupted files: every case produces its errors, and the
    rows before a failing page are still returned."""
    data = _corrupt(_error_file(), ERROR_CASES[case])
    out = oracle_next_rows(data)
    errs = [o for o in out if isinstance(o, tuple)]
    rows = [o for o in out if not isinstance(o, tuple)]
    assert errs and rows
    if case == "dict_index_page2":  # the first two pages of column a decode: their rows come first
        assert not isinstance(out[0], tuple) and isinstance(out[2999], tuple)
    if case == "load_error_rg0":  # row group 0 fails as a whole: one error, then row group 1
        assert isinstance(out[0], tuple) and len(out) == 1 + 6000


@pytest.mark.gpu
@pytest.mark.parametrize("case", sorted(ERROR_CASES))
def test_next_row_error_timing(pq, ctx, case):
    """NextRow over the GPU decode of a file with corrupted pages: exactly the rows and errors (with
    the same status) that the assembly over the oracle's pages produces, call by call; after a failed
    row group the cursor moves on (skipRowGroup, file_reader.go:228-232)."""
    data = _corrupt(_error_file(), ERROR_CASES[case])
    want = oracle_next_rows(data)
    assert [_norm(x) for x in _read_batches(pq, ctx, data, 1000)] == [_norm(w) for w in want]
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
    assert fr.assembled["columnar"] >= 1
    assert len(got) == len(want)
    for i, (g, w) in enumerate(zip(got, want)):
        assert _norm(g) == _norm(w), f"call {i}: {g} vs {w}"


@pytest.mark.gpu
def test_next_batch_pending_error_cleared_by_seek(pq, ctx):
    """NextBatch stops before a failing row and keeps its error for the next call; moving the cursor
    (SeekToRowGroup / SkipRowGroup) leaves that row group, so its error is dropped with it -- the
    reference keeps no such state.  NextBatch(n <= 0) returns no rows and consumes none."""
    data = _corrupt(_error_file(), ERROR_CASES["dict_index_page2"])
    want = oracle_next_rows(data)
    first_err = next(i for i, w in enumerate(want) if isinstance(w, tuple))
    nrg0 = O.FileReader(data).row_group_num_rows(0)
    assert 0 < first_err < nrg0
    for move in ("seek", "skip"):
        fr = pq.reader.FileReader(data, ctx=ctx)
        assert fr.NextBatch(0) == [] and fr.NextBatch(-3) == []
        got = fr.NextBatch(nrg0)
        assert [_norm(g) for g in got] == [_norm(w) for w in want[:first_err]]
        if move == "seek":
            fr.SeekToRowGroup(2)
        else:
            fr.SkipRowGroup()
        assert _norm(fr.NextRow()) == _norm(want[nrg0])
        fr.close()
    # without a move the kept error is raised by the next call, as NextRow would have raised it
    fr = pq.reader.FileReader(data, ctx=ctx)
    fr.NextBatch(nrg0)
    with pytest.raises(pq.records.RecordError) as ei:
        fr.NextBatch(10)
    assert error_outcome(ei.value) == want[first_err]
    fr.close()


def _read_arrow(pq, data):
    """Every outcome of ReadRowGroupArrow until the end: rows (drop_absent of the tables' to_pylist)
    and errors (error_outcome), in order, plus the assembly paths used."""
    A = pq.assemble
    fr = pq.reader.FileReader(data, ctx=pq.native.Context(0))
    out = []
    while True:
        try:
            t = fr.ReadRowGroupArrow()
        except (pq.reader.DecodeError, pq.records.RecordError) as e:
            out.append(error_outcome(e))
            continue
        if t is None:
            break
        out.extend(A.drop_absent(r) for r in t.to_pylist())
    paths = dict(fr.assembled)
    fr.close()
    return out, paths


@pytest.mark.gpu
def test_read_row_group_arrow(pq, ctx):
    """The Arrow export of the columnar assembly (assemble.ColumnarAssembler.arrow: ListArray /
    StructArray over the device's list offsets, presence and leaf validity, the dense values taken
    through the leaf validity) gives NextRow's records: the Dremel KATs, nested LIST / MAP files over
    many pages, the flat all-types file, a C4-shaped file, and the corrupted files of the
    error-timing tests (rows before a failing row, then its error, then the next row group)."""
    for kat in KATS:
        got, paths = _read_arrow(pq, kat_file(kat))
        assert [_norm(g) for g in got] == [_norm(r) for r in kat["rows"]], kat["name"]
    files = [fixtures.nested_list_map(n=3000, v2=True), fixtures.flat_all_types(n=4000, v2=False),
             pq.datasets.c4(rows=30_000, row_groups=2)]
    for data in files:
        want = oracle_rows(data)
        got, paths = _read_arrow(pq, data)
        assert paths.get("arrow", 0) == len(O.FileReader(data).row_groups), paths
        assert len(got) == len(want) and all(_norm(g) == _norm(w) for g, w in zip(got, want))
    for case in sorted(ERROR_CASES):
        data = _corrupt(_error_file(), ERROR_CASES[case])
        want = oracle_next_rows(data)
        got, _ = _read_arrow(pq, data)
        # (a row group's rows before its failing row come as one table, then one error per call for
        # each row left, as NextRow raises them; then the next row group)
        assert [_norm(g) for g in got] == [_norm(w) for w in want], case


@pytest.mark.gpu
def test_read_row_group_arrow_lazy_fallback(pq, ctx):
    """ReadRowGroupArrow on a row group whose columnar assembly fails only in its lazy checks (two
    leaves disagreeing on their group's presence, fixtures.disagreeing_group): the Arrow export
    raises NotColumnar inside ReadRowGroupArrow, which then goes value by value (as NextRow does)
    instead of raising -- the same records as NextRow and the oracle's assembly."""
    data = fixtures.disagreeing_group()
    want = [_norm(w) for w in oracle_next_rows(data)]
    got, paths = _read_arrow(pq, data)
    assert [_norm(g) for g in got] == want
    assert paths.get("value_by_value", 0) == 1 and paths.get("arrow", 0) == 1, paths


@pytest.mark.gpu
def test_next_row_many_small_row_groups(pq, ctx):
    """A row group every 100 rows (the reference's column-selection file, filereader_test.go:13-247):
    100 row groups of the all-types file and of a nested LIST / MAP file, NextRow with every column and
    with a selection, equal call by call to the assembly over the oracle's pages; ReadRowGroupArrow the
    same.  In 4 of the all-types file's row groups the FLBA column's DELTA_BYTE_ARRAY fallback page
    holds ONE value, so its length streams hit the reference's DELTA read-ahead failure ((n - 1) % 128
    == 0, deltabp_decoder.go) when the decoder initialises: those row groups fail
    whole, on the GPU as in the reference (pyarrow, without that quirk, reads them)."""
    def next_rows(data, *cols):
        fr = pq.reader.FileReader(data, *cols, ctx=ctx)
        out = []
        while True:
            try:
                out.append(fr.NextRow())
            except EOFError:
                break
            except (pq.reader.DecodeError, pq.records.RecordError) as e:
                out.append(error_outcome(e))
        fr.close()
        return out

    for data, sel in ((fixtures.flat_all_types(n=10_000, v2=True, rows_per_group=100), None),
                      (fixtures.nested_list_map(n=10_000, rows_per_group=100), "m")):
        assert len(O.FileReader(data).row_groups) == 100
        want = [_norm(w) for w in oracle_next_rows(data)]
        assert [_norm(g) for g in next_rows(data)] == want
        arrow, _ = _read_arrow(pq, data)
        assert [_norm(g) for g in arrow] == want
        if sel:
            got = next_rows(data, sel)
            assert [_norm(r) for r in got] == [{k: v for k, v in w.items() if k == sel} for w in want]
