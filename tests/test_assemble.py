"""The columnar record assembly (assemble.py, §8(f)1) against the value-by-value restatement of the
reference's record assembly (records.py: Column.getData / ColumnStore.get, schema.go:216-312,
data_store.go:262-309), on the CPU: the leaves' inputs are the oracle's page results and the
nesting outputs of oracle.nest_levels (the device's pqh_batch_nesting is pinned to it by
test_gpu_parity.py).  Same rows and the same errors call by call: the reference's Dremel KATs
(data_store_test.go), nested / flat / deep / pyarrow files, column selections, and the corrupted
files of the error-timing tests.  The GPU path (FileReader.NextRow / NextBatch over the device's
nesting outputs) is checked in test_records.py."""
import numpy as np
import pytest

import fixtures
from oracle import oracle as O
from test_records import ERROR_CASES, KATS, _corrupt, _error_file, _go_values, _norm, _oracle_schema, _pkg, \
    error_outcome, kat_file, oracle_next_rows


def _pa():
    import pyarrow

    return pyarrow


def columnar_next_rows(data, columns=None, stats=None):
    """oracle_next_rows' outcomes through assemble.ColumnarAssembler (records.RowAssembler where a
    row group breaks a precondition; counted in stats)."""
    A = _pkg().assemble
    R = _pkg().records
    fr = O.FileReader(data)
    schema = _oracle_schema(fr)
    sel = list(range(len(fr.columns))) if columns is None else columns
    leaf_el = [e for _, e in schema if e.num_children == 0]
    out = []
    for rg in range(len(fr.row_groups)):
        leaves, stores, rg_err, nil_values = {}, {}, None, False
        for ci in sel:
            col = fr.columns[ci]
            ch = fr.read_chunk(rg, ci)
            if ch.status:
                rg_err = ch.status
                break
            res = O.decode_chunk(ch)
            load = [r for r in res if r.status and r.phase == O.PHASE_LOAD]
            if load:
                rg_err = load[0].status
                break
            nil_values = nil_values or any(r.nil is not None for r in res)
            n = sum(r.num_values for r in res)
            cat = lambda a: np.concatenate([np.asarray(getattr(r, a) if getattr(r, a) is not None else  # noqa: E731
                                                       np.zeros(r.num_values, np.uint8), np.uint8)[:r.num_values]
                                            for r in res]) if res else np.zeros(0, np.uint8)
            d = cat("def_levels") if col.max_def else None
            rr = cat("rep_levels") if col.max_rep else None
            firsts = np.cumsum([0] + [r.num_values for r in res])[:-1].tolist()
            pages = [(f, r.status, r.phase, r.index) for f, r in zip(firsts, res)]
            levels, leaf = None, None
            if col.max_rep:
                levels, leaf = O.nest_levels(d, rr, col.max_def, col.rep_def)
            vals = [v for r in res for v in _go_values(r, col)] if all(r.status == 0 for r in res) else None
            if vals is None:  # values of the pages before the first failing one
                vals = []
                for r in res:
                    if r.status:
                        break
                    vals += _go_values(r, col)
            leaves[ci] = A.Leaf(col.path, col.max_def, col.max_rep, col.rep_def, d, rr, levels, leaf,
                                lambda vals=vals: vals, pages, n,
                                arrow=lambda vals=vals, col=col: _pa().array(
                                    vals, type=A.arrow_type(col.physical_type, col.type_length or 0)))
            el = leaf_el[ci]
            spages = []
            for r in res:
                nv = r.num_values
                spages.append((R.PageResult(r.status, r.phase, r.index), nv,
                               r.def_levels if r.def_levels is not None else np.zeros(nv, np.uint8),
                               r.rep_levels if r.rep_levels is not None else np.zeros(nv, np.uint8),
                               lambda r=r, col=col: _go_values(r, col)))
            stores[ci] = R.LeafStore(None, col.path, el.repetition, col.max_def, col.max_rep, spages)
        if rg_err is not None:
            out.append(("error", rg_err))
            continue
        nrows = fr.row_group_num_rows(rg)
        try:
            if nil_values:  # reader.FileReader assembles these value by value (Go nil values)
                raise A.NotColumnar("nil INT96 values")
            asm = A.ColumnarAssembler(schema, leaves, nrows)
            rows = asm.rows()
        except A.NotColumnar:
            if stats is not None:
                stats["fallback"] = stats.get("fallback", 0) + 1
            for ci in range(len(fr.columns)):
                if ci not in stores:
                    stores[ci] = R.LeafStore(None, fr.columns[ci].path, leaf_el[ci].repetition, 0, 0, skipped=True)
            ra = R.RowAssembler(schema, None, nrows, stores=stores)
            for _ in range(nrows):
                try:
                    out.append(ra.next_row())
                except R.RecordError as e:
                    out.append(error_outcome(e))
            continue
        if stats is not None:
            stats["columnar"] = stats.get("columnar", 0) + 1
        # the same records through the Arrow export (no per-row objects until to_pylist)
        t = asm.arrow()
        arows = [A.drop_absent(r) for r in t.to_pylist()] if t.num_columns else [{}] * len(rows)
        assert len(arows) == len(rows) and all(_norm(a) == _norm(b) for a, b in zip(arows, rows)), "arrow export"
        out.extend(rows)
        # (status, phase, index, page) as records.RecordError carries them: reader.NextRow raises these
        out.extend(("error", e[1], e[2], e[3], e[5]) for e in asm.errors())
    return out


def _selected_oracle(data, columns):
    """oracle_next_rows with unselected leaves skipped (WithColumns)."""
    R = _pkg().records
    fr = O.FileReader(data)
    schema = _oracle_schema(fr)
    out = []
    leaf_el = [e for _, e in schema if e.num_children == 0]
    for rg in range(len(fr.row_groups)):
        stores = {}
        for ci, col in enumerate(fr.columns):
            if ci not in columns:
                stores[ci] = R.LeafStore(None, col.path, leaf_el[ci].repetition, 0, 0, skipped=True)
                continue
            pages = []
            for r in O.decode_chunk(fr.read_chunk(rg, ci)):
                nv = r.num_values
                pages.append((R.PAGE_OK, nv, r.def_levels if r.def_levels is not None else np.zeros(nv, np.uint8),
                              r.rep_levels if r.rep_levels is not None else np.zeros(nv, np.uint8),
                              lambda r=r, col=col: _go_values(r, col)))
            stores[ci] = R.LeafStore(None, col.path, leaf_el[ci].repetition, col.max_def, col.max_rep, pages)
        asm = R.RowAssembler(schema, None, fr.row_group_num_rows(rg), stores=stores)
        out.extend(asm.next_row() for _ in range(fr.row_group_num_rows(rg)))
    return out


def _same(got, want):
    assert len(got) == len(want)
    for i, (g, w) in enumerate(zip(got, want)):
        assert _norm(g) == _norm(w), f"call {i}: {g} vs {w}"


@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_columnar_kat_rows(kat):
    """The reference's record-shredding KATs (data_store_test.go:18-497) through the columnar
    assembly: exactly the KAT rows."""
    stats = {}
    for use_dict in (True, False):
        got = columnar_next_rows(kat_file(kat, use_dict=use_dict), stats=stats)
        assert [_norm(g) for g in got] == [_norm(w) for w in kat["rows"]]
    assert stats.get("columnar", 0) >= 1


def _files():
    yield "nested-v1", fixtures.nested_list_map(n=3000, v2=False)
    yield "nested-v2", fixtures.nested_list_map(n=3000, v2=True)
    yield "flat", fixtures.flat_all_types(n=4000)
    yield "deep10", fixtures.deep_repeated(n=500, depth=10)[0]
    yield "deep3-nowrap", fixtures.deep_repeated(n=2000, depth=3, wrap=[False] * 3, seed=3)[0]


@pytest.mark.parametrize("name", [n for n, _ in _files()])
def test_columnar_matches_value_by_value(name):
    data = dict(_files())[name]
    stats = {}
    _same(columnar_next_rows(data, stats=stats), oracle_next_rows(data))
    if name.startswith("deep"):
        # chains of repeated groups whose only child is repeated: an element followed by an empty
        # inner list makes getFirstRDLevel return -1 and the reference ends the outer list there
        # (schema.go:260-312) -- those row groups take the value-by-value assembly
        assert stats.get("fallback")
    else:
        assert stats.get("columnar", 0) == len(O.FileReader(data).row_groups) and not stats.get("fallback")


def test_columnar_pyarrow_nested():
    """pyarrow-written lists of lists / structs of lists (page boundaries at row boundaries).  (With
    null or empty inner lists, or inner lists starting with a null, the outer list's continuation
    finds no decisive child -- getFirstRDLevel returns -1 and the reference ends the outer list
    early; such row groups fall back, test_columnar_matches_value_by_value[deep*].)"""
    import io

    import pyarrow as pa
    import pyarrow.parquet as pqa

    rng = np.random.default_rng(7)

    def inner():  # an empty / null inner list, or one starting with a null, would end the outer list
        return [int(rng.integers(0, 99))] + [None if rng.random() < 0.1 else int(rng.integers(0, 99))
                                             for _ in range(rng.poisson(2))]

    a = [None if rng.random() < 0.1 else [inner() for _ in range(rng.poisson(2))] for _ in range(3000)]
    b = [None if rng.random() < 0.1 else {"x": int(rng.integers(0, 9)), "s": None if rng.random() < 0.2 else
                                          [str(rng.integers(0, 99)) for _ in range(rng.poisson(1.5))]}
         for _ in range(3000)]
    t = pa.table({"a": pa.array(a, pa.list_(pa.list_(pa.int32()))),
                  "b": pa.array(b, pa.struct([("x", pa.int64()), ("s", pa.list_(pa.string()))]))})
    buf = io.BytesIO()
    pqa.write_table(t, buf, row_group_size=1000, data_page_size=4096, use_dictionary=False)
    data = buf.getvalue()
    stats = {}
    _same(columnar_next_rows(data, stats=stats), oracle_next_rows(data))
    assert stats.get("columnar", 0) >= 1


@pytest.mark.parametrize("case", sorted(ERROR_CASES))
def test_columnar_error_timing(case):
    """Corrupted pages: the rows before the first failing row, then the errors call by call, as the
    value-by-value assembly produces them."""
    data = _corrupt(_error_file(), ERROR_CASES[case])
    stats = {}
    _same(columnar_next_rows(data, stats=stats), oracle_next_rows(data))
    assert stats.get("columnar", 0) >= 1


def test_columnar_selected_columns():
    """WithColumns: a skipped leaf first in a repeated group would end its lists early in the
    reference (getFirstRDLevel reads a skipped store as the end): such row groups fall back to the
    value-by-value assembly; the others assemble columnar.  Rows equal either way."""
    data = fixtures.nested_list_map(n=2000)
    for cols in ([0], [1, 2], [2], [0, 2]):
        stats = {}
        got = columnar_next_rows(data, columns=cols, stats=stats)
        _same(got, _selected_oracle(data, cols))
        if cols == [2]:  # the map's key leaf (first child of key_value) is skipped
            assert stats.get("fallback")
        if cols in ([0], [1, 2]):
            assert not stats.get("fallback")


def test_lazy_not_columnar_row_group():
    """A row group the columnar assembler accepts at construction but whose lazy presence check
    rejects (two leaves disagreeing on their group's presence): rows() and arrow() both raise
    NotColumnar (so reader.FileReader's NextRow and ReadRowGroupArrow go value by value), and the
    assembled rows equal the value-by-value restatement's; the consistent row group stays columnar."""
    A = _pkg().assemble
    data = fixtures.disagreeing_group()
    lazy = []

    class Probe(A.ColumnarAssembler):
        def arrow(self):
            try:
                return super().arrow()
            except A.NotColumnar as e:
                lazy.append(str(e))
                raise

    orig = A.ColumnarAssembler
    A.ColumnarAssembler = Probe
    try:
        stats = {}
        _same(columnar_next_rows(data, stats=stats), oracle_next_rows(data))
    finally:
        A.ColumnarAssembler = orig
    assert stats == {"fallback": 1, "columnar": 1}, stats
    # (rows() raised first for the first row group; the second one's arrow() ran clean)
    fr = O.FileReader(data)
    assert len(fr.row_groups) == 2 and not lazy


def test_records_table_fallback():
    """ReadRowGroupArrow's table for non-columnar row groups (assemble.records_table): every
    top-level field any record holds becomes a column, not just the first record's (records omit
    absent fields), and records with no field keep the row count."""
    A = _pkg().assemble
    rows = [{"a": {"list": [{"element": 1}, {}]}}, {}, {"c": {"list": [{"element": {"s": {}}}]}, "m": {}},
            {"b": {"list": [{"element": {"list": [{"element": -3}]}}]}, "a": {}}]
    t = A.records_table(rows)
    assert sorted(t.column_names) == ["a", "b", "c", "m"] and t.num_rows == 4
    assert [A.drop_absent(r) for r in t.to_pylist()] == rows
    t = A.records_table([{}, {}, {}])
    assert t.num_rows == 3 and [A.drop_absent(r) for r in t.to_pylist()] == [{}, {}, {}]
