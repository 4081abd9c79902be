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
        name = name.decode() if isinstance(name, bytes) else name
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
    for _ in range(root.get(5, 0)):
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
    return [r.values[i:i + size] for i in range(0, len(r.values), size)]


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
                pages.append((0, n, d, rp, lambda r=r, col=col: _go_values(r, col)))
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
        page = (0, n, np.array(lf["def"], np.uint8), np.array(lf["rep"], np.uint8), lambda lf=lf: list(lf["values"]))
        stores[ci] = R.LeafStore(None, col.path, reps[dict(kat["schema"])[col.path]], lf["max_def"], lf["max_rep"],
                                 [page])
    asm = R.RowAssembler(schema, None, len(kat["rows"]), stores=stores)
    got = [asm.next_row() for _ in kat["rows"]]
    assert got == kat["rows"]


@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_oracle_file_records_match_reference(kat):
    """KAT rows -> file (reference-writer layout) -> oracle readValues -> assembly == KAT rows."""
    assert oracle_rows(kat_file(kat)) == kat["rows"]


def _read_all(pq, ctx, data, *columns):
    fr = pq.reader.FileReader(data, *columns, ctx=ctx)
    rows = []
    while True:
        try:
            rows.append(fr.NextRow())
        except EOFError:
            break
    fr.close()
    return rows


@pytest.fixture(scope="module")
def ctx():
    return _pkg().native.Context(0)


@pytest.mark.gpu
@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_next_row_matches_reference_records(pq, ctx, kat):
    """NextRow over the GPU decode of the KAT file returns exactly the reference's rows, then EOF."""
    for use_dict in (True, False):
        data = kat_file(kat, use_dict=use_dict)
        assert _read_all(pq, ctx, data) == kat["rows"], f"use_dict={use_dict}"


@pytest.mark.gpu
@pytest.mark.parametrize("v2", [False, True])
def test_next_row_multi_page(pq, ctx, v2):
    """Nested LIST / MAP columns over many pages and two row groups, and the flat all-types file:
    NextRow (GPU) == assembly over the oracle's pages, row by row."""
    for data in (fixtures.nested_list_map(n=3000, v2=v2), fixtures.flat_all_types(n=4000, v2=v2)):
        want = oracle_rows(data)
        got = _read_all(pq, ctx, data)
        assert len(got) == len(want) == O.FileReader(data).num_rows
        for i, (g, w) in enumerate(zip(got, want)):
            assert _norm(g) == _norm(w), f"row {i}: {g} vs {w}"


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
