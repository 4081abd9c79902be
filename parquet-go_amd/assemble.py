"""Columnar record assembly: FileReader.NextRow / NextBatch rows built from the
device's nesting outputs, not from per-value level walks.

The reference assembles one record at a time (Column.getData / ColumnStore.get, schema.go:216-312,
data_store.go:262-309; restated value by value in records.py).  On well-formed data its result has a
columnar description, which this module evaluates node by node over whole row groups:

  * k(X) = the repeated nodes on the path root..X (= X's max repetition level).  A non-repeated node
    X has one instance per level-k(X) element (per row when k = 0); a repeated node X has one list
    per level-(k(X)-1) element: pqh_batch_nesting's level-k offsets give each list's elements.
  * leaf instance: the dense value when the leaf slot is valid (pqh_nest_out.leaf_validity, i.e.
    d == max_def), else absent (ColumnStore.get: d < maxD is a null);
  * repeated node: absent when its list is empty (an absent or empty list: its first element is nil,
    Column.getData returns nil), else the list of its element instances;
  * group instance: present iff the definition level at its first slot reaches the group's max_def
    (getNextData's not-nil count: a child defined, or null exactly one level below), then the dict of
    its present children -- {} when every child is absent;
  * row: the root's dict, {} when empty (schema.getData never returns nil).

Preconditions (checked per row group; otherwise the caller uses records.RowAssembler, the exact
value-by-value restatement): every selected leaf's pages start at row boundaries (the reference's
level cursors are page-local, so a list crossing a page would be cut); leaves under one group agree
on its instances and their presence; no repeated group can end early on getFirstRDLevel's -1 / skipped
leaf quirk (schema.go:260-312).

Errors (data_store.go:236-269): a leaf's failing page fails the first row that reaches it; rows before
it are returned.  After that, every NextRow of the row group fails with the first leaf (in traversal
order) whose failing page is reached -- leaves before the stuck one keep advancing, as the reference's
cursors do.
"""
import numpy as np

REQUIRED, OPTIONAL, REPEATED = 0, 1, 2
BOOLEAN, INT32, INT64, INT96, FLOAT, DOUBLE, BYTE_ARRAY, FIXED_LEN_BYTE_ARRAY = range(8)


class NotColumnar(Exception):
    """The row group breaks a precondition of the columnar assembly (use records.RowAssembler)."""


class Leaf:
    """One selected leaf column of a row group.
    d, r: level bytes per slot (None when the max level is 0); levels: [(offsets int32, validity u8)]
    per repetition level (pqh_batch_nesting; absent for max_rep 0); leaf_valid: u8 per leaf slot;
    values(): the dense values as Go-like Python values; pages: [(first slot, status, phase, index)] of
    the chunk's data pages."""

    def __init__(self, path, max_d, max_r, rep_def, d, r, levels, leaf_valid, values, pages, n, arrow=None):
        self.path, self.max_d, self.max_r, self.rep_def = path, max_d, max_r, tuple(rep_def)
        self._arrow = arrow  # () -> the dense values as a pyarrow Array (ColumnarAssembler.arrow)
        self.n = n
        self.d = d if d is not None else np.zeros(n, np.uint8)
        self.r = r if r is not None else np.zeros(n, np.uint8)
        self.levels = levels or []
        self.leaf_valid = leaf_valid if leaf_valid is not None else (self.d == max_d).astype(np.uint8)
        self._values = values
        self._vals = None
        self.pages = pages

    def values(self):
        if self._vals is None:
            self._vals = self._values()
        return self._vals


def arrow_type(ptype, type_length):
    """The Arrow type of a leaf's values (the Go values' types: []byte for byte arrays, FLBA and the
    12-byte INT96)."""
    import pyarrow as pa

    return {BOOLEAN: pa.bool_(), INT32: pa.int32(), INT64: pa.int64(), FLOAT: pa.float32(), DOUBLE: pa.float64(),
            BYTE_ARRAY: pa.large_binary(), INT96: pa.binary(12)}.get(ptype) or pa.binary(int(type_length))


def arrow_dense(col, ptype):
    """The dense values of a decoded chunk (reader.ColumnData) as a pyarrow Array, zero-copy over the
    host copies of the device outputs where Arrow's layout allows (fixed width, offsets + bytes)."""
    import pyarrow as pa

    t = arrow_type(ptype, col.type_length)
    if col.values is not None:
        v = col.values
        if ptype == BOOLEAN:
            return pa.array(v.astype(bool), type=t)
        if v.ndim == 2:
            return pa.Array.from_buffers(t, len(v), [None, pa.py_buffer(np.ascontiguousarray(v))])
        return pa.array(v, type=t)
    if col.offsets is None:
        return pa.array([], type=t)
    # (int64 offsets + bytes: large_binary as is; a FIXED_LEN_BYTE_ARRAY chunk of DELTA_BYTE_ARRAY
    # pages comes out this way too)
    n = len(col.offsets) - 1
    return pa.Array.from_buffers(pa.large_binary(), n, [None, pa.py_buffer(col.offsets), pa.py_buffer(col.data)])


def dense_values(col, ptype):
    """All dense values of a decoded chunk (reader.ColumnData) as the reference's Go values."""
    if col.values is not None:
        v = col.values
        if ptype == BOOLEAN:
            return v.astype(bool).tolist()
        if v.ndim == 2:
            b = v.tobytes()
            w = v.shape[1]
            return [b[i:i + w] for i in range(0, len(b), w)]
        return v.tolist()
    if col.offsets is None:
        return []
    d = col.data.tobytes()
    o = col.offsets.tolist()
    return [d[a:b] for a, b in zip(o[:-1], o[1:])]


class _Node:
    __slots__ = ("name", "rep", "max_d", "max_r", "children", "column")

    def __init__(self, name, rep, max_d, max_r, children=None, column=-1):
        self.name, self.rep, self.max_d, self.max_r = name, rep, max_d, max_r
        self.children, self.column = children, column


def _tree(schema):
    """The schema tree (readSchema: elements after the root are top-level children until the list
    ends, schema.go:992-1015)."""
    pos = [1]

    def node(i):
        name, e = schema[i]
        if e.num_children == 0:
            return _Node(name, e.repetition, e.max_def, e.max_rep, column=e.column)
        kids = []
        for _ in range(e.num_children):
            j = pos[0]
            pos[0] += 1
            kids.append(node(j))
        return _Node(name, e.repetition, e.max_def, e.max_rep, children=kids)

    kids = []
    while pos[0] < len(schema):
        j = pos[0]
        pos[0] += 1
        kids.append(node(j))
    return _Node(schema[0][0], REQUIRED, 0, 0, children=kids)


class ColumnarAssembler:
    """The records of one loaded row group from its selected leaves {column index: Leaf}."""

    def __init__(self, schema, leaves, num_rows):
        self.root = _tree(schema)
        self.leaves = leaves
        self.num_rows = num_rows
        self._order = []  # selected leaves in traversal order (getData visits children in order)
        self._walk(self.root)
        self._check_quirks(self.root)
        for lf in leaves.values():
            self._check_pages(lf)
        self._plan_errors()
        self._rows = None
        self.current = 0

    # ------------------------------------------------------------------ preconditions
    def _walk(self, x):
        if x.children is None:
            if x.column in self.leaves:
                self._order.append(x.column)
            return
        for c in x.children:
            self._walk(c)

    def _first_rd(self, x):
        """What getFirstRDLevel (schema.go:260-281) meets first below x at a continuation element of
        its repeated ancestor: "always" (a selected non-repeated leaf: rl == the ancestor's level),
        "last" (a skipped leaf: its empty level arrays read as the end), or "maybe" (only repeated
        children: decided by their definition levels)."""
        if x.children is None:
            if x.column not in self.leaves:
                return "last"
            return "maybe" if x.rep == REPEATED else "always"
        for c in x.children:
            s = self._first_rd(c)
            if s == "last":
                return "last"
            if s == "always" and c.rep != REPEATED:
                return "always"
        return "maybe"

    def _check_quirks(self, x):
        if x.children is None:
            return
        if x.rep == REPEATED and any(c in self.leaves for c in self._columns(x)):
            # getData's loop continues while getFirstRDLevel returns rl >= max_r; a skipped first
            # leaf (last) or children that all return -1 (only repeated ones, with empty lists) end
            # the list early.  Statically safe when a selected non-repeated leaf decides first;
            # otherwise checked at every continuation element of x (_frd).
            first = None
            for c in x.children:
                s = self._first_rd(c)
                if s == "last" or (s == "always" and c.rep != REPEATED):
                    first = s
                    break
            if first != "always":
                self._check_continuations(x)
        for c in x.children:
            self._check_quirks(c)

    def _check_continuations(self, x):
        R = x.max_r
        lf = self._rep_leaf(x)
        st = self._starts(lf, R, None)
        cont = lf.r[st] == R  # the elements after the first of each list: where getData's loop asks
        m = int(np.count_nonzero(cont))
        if m == 0:
            return
        ret, last, _ = self._frd_group(x, R, m)
        if not np.all(ret & ~last):
            raise NotColumnar(f"repeated group {x.name}: getFirstRDLevel ends a list early")

    def _frd(self, c, R, m):
        """getFirstRDLevel of node c at the continuation elements of its level-R repeated ancestor:
        (returned, last, dl) arrays of length m (returned False = the -1 result)."""
        if c.children is None:
            if c.column not in self.leaves:  # skipped store: (0, 0, last)
                return np.ones(m, bool), np.ones(m, bool), np.zeros(m, np.int32)
            lf = self.leaves[c.column]
            st = self._starts(lf, R, None)
            st = st[lf.r[st] == R]
            if len(st) != m:
                raise NotColumnar(f"{c.name}: continuation elements disagree")
            return np.ones(m, bool), np.zeros(m, bool), lf.d[st].astype(np.int32)
        return self._frd_group(c, R, m)

    def _frd_group(self, g, R, m):
        ret = np.zeros(m, bool)
        last = np.zeros(m, bool)
        dl = np.full(m, -1, np.int32)
        undecided = np.ones(m, bool)
        for cc in g.children:
            r2, l2, d2 = self._frd(cc, R, m)
            take = undecided & r2 & (l2 | (R >= cc.max_r) | (d2 >= cc.max_d))
            ret |= take
            last |= take & l2
            dl = np.where(take, d2, dl)
            undecided &= ~take
        return ret, last, dl

    def _columns(self, x):
        if x.children is None:
            return [x.column]
        return [c for k in x.children for c in self._columns(k)]

    def _check_pages(self, lf):
        if lf.max_r == 0:
            return
        for first, *_ in lf.pages:
            if first < lf.n and lf.r[first] != 0:
                raise NotColumnar(f"{lf.path}: a page starts inside a row (page-local level cursors)")

    # ------------------------------------------------------------------ error timing
    def _plan_errors(self):
        """fail_row[c] = the row that reads leaf c's first failing page (rows before it assemble)."""
        self.fail = {}
        for c in self._order:
            lf = self.leaves[c]
            for page, (first, status, phase, index) in enumerate(lf.pages):
                if status:  # (page = the data page's position in the chunk, as records.LeafStore counts)
                    row = int(np.count_nonzero(lf.r[:first] == 0)) if lf.max_r else first
                    self.fail[c] = (row, status, phase, index, lf.path, page)
                    break
        self.ok_rows = min([f[0] for f in self.fail.values()] + [self.num_rows])

    def errors(self):
        """The errors of NextRow calls ok_rows, ok_rows + 1, ... num_rows - 1, in order: per call the
        reference's traversal visits the leaves in order; a leaf at its failing row raises (it never
        advances again, and the leaves after it are not visited in that call), the others advance
        one row."""
        k = {c: self.ok_rows for c in self._order}
        out = []
        for _ in range(self.ok_rows, self.num_rows):
            err = None
            for c in self._order:
                f = self.fail.get(c)
                if f is not None and k[c] >= f[0]:
                    err = f
                    break
                k[c] += 1
            out.append(err)
        return out

    # ------------------------------------------------------------------ assembly
    def _starts(self, lf, k, rows):
        """Slot index of every level-k element (rows when k == 0) of leaf lf within the first `rows`
        rows."""
        key = ("starts", k)
        cache = lf.__dict__.setdefault("_cache", {})
        if key not in cache:
            if k == 0:
                s = np.flatnonzero(lf.r == 0) if lf.max_r else np.arange(lf.n)
            else:
                s = np.flatnonzero((lf.r <= k) & (lf.d >= lf.rep_def[k - 1]))
            cache[key] = s
        return cache[key]

    def _count(self, lf, k, rows):
        """Elements of level k in the first `rows` rows (chained through the nesting offsets)."""
        n = rows
        for l in range(1, k + 1):
            n = int(lf.levels[l - 1][0][n])
        return n

    def _rep_leaf(self, x):
        for c in self._columns(x):
            if c in self.leaves:
                return self.leaves[c]
        return None

    def _values(self, x, k, rows):
        """x's instances (x non-repeated at level k, or x's lists per level-k element when x is
        repeated) over the first `rows` rows: (list of values, absent mask) -- the mask a numpy bool
        array (True = absent), or None for a node without a selected leaf (skipped everywhere, as a
        skipped ColumnStore's get returns nil)."""
        lf = self._rep_leaf(x)
        if lf is None:
            return None
        if x.rep == REPEATED:
            n_inst = self._count(lf, k, rows)
            kk = k + 1
            off = lf.levels[kk - 1][0][:n_inst + 1]
            elems, emask = self._element_values(x, kk, rows)
            if emask.any():  # a nil element inside a list (Column.getData appends it as nil)
                if x.children is None:  # ColumnStore.get would read a value for it: not columnar
                    raise NotColumnar(f"{x.name}: a repeated leaf slot without a value inside a list")
                for i in np.flatnonzero(emask).tolist():
                    elems[i] = None
            o = off.tolist()
            return [elems[a:b] for a, b in zip(o[:-1], o[1:])], np.diff(off) == 0  # empty list: nil
        return self._element_values(x, k, rows)

    def _element_values(self, x, k, rows):
        """x as an element instance at level k (one per level-k element): (values, absent mask)."""
        if x.children is None:
            lf = self.leaves[x.column]
            n = self._count(lf, k, rows)  # leaf slots of the first `rows` rows
            valid = lf.leaf_valid[:n].astype(bool)
            vals = lf.values()
            nv = int(np.count_nonzero(valid))
            if nv == n:
                return vals[:n], ~valid
            out = [None] * n
            for i, v in zip(np.flatnonzero(valid).tolist(), vals[:nv]):
                out[i] = v
            return out, ~valid
        lf = self._rep_leaf(x)
        n = self._count(lf, k, rows)
        kids = []
        for c in x.children:
            v = self._values(c, k, rows)
            if v is not None:
                if len(v[0]) != n:
                    raise NotColumnar(f"{c.name}: {len(v[0])} instances under {x.name}, expected {n}")
                kids.append((c.name, v[0], v[1]))
        return _dicts(kids, n), ~self._presence(x, lf, k, rows, n)

    def _presence(self, x, lf, k, rows, n):
        """Group x's presence per level-k instance (d at its first slot >= x's max_d); every selected
        leaf below x must agree."""
        starts = self._starts(lf, k, rows)[:n]
        present = lf.d[starts] >= x.max_d
        for c in self._columns(x):
            o = self.leaves.get(c)
            if o is not None and o is not lf and x.max_d > 0:
                s2 = self._starts(o, k, rows)[:n]
                if len(s2) != n or not np.array_equal(o.d[s2] >= x.max_d, present):
                    raise NotColumnar(f"{x.name}: leaves disagree on its instances")
        return present

    def rows(self):
        """Every row this row group returns before its first error (cached).  The cyclic garbage
        collector is paused while the containers are built (they form no cycles; its passes over
        the growing object graph would otherwise dominate)."""
        if self._rows is None:
            import gc

            was = gc.isenabled()
            gc.disable()
            try:
                self._rows = self._build()
            finally:
                if was:
                    gc.enable()
        return self._rows

    # ------------------------------------------------------------------ Arrow export
    def arrow(self):
        """The rows() records as a pyarrow Table, built column by column from the same columnar
        description without any per-row Python object: a repeated node is a ListArray over its
        level offsets (an empty list is null: the reference's nil), a group a StructArray whose
        validity is its presence, a leaf the dense values taken through its leaf validity (nulls at
        the null slots).  Table.to_pylist() equals rows() once absent fields (None in a struct) are
        dropped, as the reference's records omit them.  A native consumer of the device's columnar
        outputs: no value passes through the interpreter."""
        import pyarrow as pa

        n = self.ok_rows
        arrays, names = [], []
        for c in self.root.children:
            v = self._arrow_values(c, 0, n)
            if v is not None:
                if len(v[0]) != n:
                    raise NotColumnar(f"{c.name}: {len(v[0])} rows, expected {n}")
                arrays.append(v[0])
                names.append(c.name)
        return pa.Table.from_arrays(arrays, names=names)

    def _arrow_values(self, x, k, rows):
        import pyarrow as pa

        lf = self._rep_leaf(x)
        if lf is None:
            return None
        if x.rep == REPEATED:
            n_inst = self._count(lf, k, rows)
            kk = k + 1
            off = np.ascontiguousarray(lf.levels[kk - 1][0][:n_inst + 1], np.int32)
            elems, emask = self._arrow_element(x, kk, rows)
            if x.children is None and emask.any():
                raise NotColumnar(f"{x.name}: a repeated leaf slot without a value inside a list")
            empty = np.diff(off) == 0
            arr = pa.ListArray.from_arrays(pa.array(off), elems, mask=pa.array(empty))
            return arr, empty
        return self._arrow_element(x, k, rows)

    def _arrow_element(self, x, k, rows):
        import pyarrow as pa

        if x.children is None:
            lf = self.leaves[x.column]
            if lf._arrow is None:
                raise NotColumnar(f"{x.name}: no Arrow values")
            n = self._count(lf, k, rows)
            valid = lf.leaf_valid[:n].astype(bool)
            dense = lf._arrow()
            if valid.all():
                return dense.slice(0, n), ~valid
            if not valid.any():
                return pa.nulls(n, type=dense.type), ~valid
            idx = np.maximum(np.cumsum(valid, dtype=np.int64) - 1, 0)
            return dense.take(pa.array(idx, mask=~valid)), ~valid
        lf = self._rep_leaf(x)
        n = self._count(lf, k, rows)
        arrays, names = [], []
        for c in x.children:
            v = self._arrow_values(c, k, rows)
            if v is not None:
                if len(v[0]) != n:
                    raise NotColumnar(f"{c.name}: {len(v[0])} instances under {x.name}, expected {n}")
                arrays.append(v[0])
                names.append(c.name)
        present = self._presence(x, lf, k, rows, n)
        return pa.StructArray.from_arrays(arrays, names=names, mask=pa.array(~present)), ~present

    def _build(self):
        n = self.ok_rows
        kids = []
        for c in self.root.children:
            v = self._values(c, 0, n)
            if v is not None:
                if len(v[0]) != n:
                    raise NotColumnar(f"{c.name}: {len(v[0])} rows, expected {n}")
                kids.append((c.name, v[0], v[1]))
        return _dicts(kids, n)


def drop_absent(x):
    """A record of Table.to_pylist() in the reference's form: struct fields that are None (absent)
    dropped, at every depth (list elements keep their None: a nil element)."""
    if isinstance(x, dict):
        return {k: drop_absent(v) for k, v in x.items() if v is not None}
    if isinstance(x, list):
        return [drop_absent(v) for v in x]
    return x


def _dicts(kids, n):
    """n dicts of the present children: kids = [(name, values, absent mask)].  All-present rows are
    built by one comprehension; rows with an absent child are rebuilt without it."""
    names = [k[0] for k in kids]
    cols = [k[1] for k in kids]
    if len(kids) == 0:
        return [{} for _ in range(n)]
    if len(kids) == 1:
        n0 = names[0]
        out = [{n0: a} for a in cols[0]]
    elif len(kids) == 2:
        n0, n1 = names
        out = [{n0: a, n1: b} for a, b in zip(cols[0], cols[1])]
    else:
        out = [dict(zip(names, t)) for t in zip(*cols)]
    any_absent = np.zeros(n, bool)
    for k in kids:
        any_absent |= k[2]
    for i in np.flatnonzero(any_absent).tolist():
        out[i] = {nm: c[i] for nm, c, m in kids if not m[i]}
    return out


def records_table(rows):
    """Records (NextBatch's dicts) as a Table, for ReadRowGroupArrow's non-columnar row groups: a
    column per top-level field any row holds, its type inferred over all rows (pyarrow unions the
    keys of nested dicts; a field a record omits is null), so drop_absent of to_pylist() gives the
    records back.  Rows that hold no field at all keep their count (a zero-field struct batch), which
    Table.from_pylist -- names from the first row only -- loses."""
    import pyarrow as pa

    names = list(dict.fromkeys(k for r in rows for k in r))
    if not names:
        return pa.Table.from_batches([pa.RecordBatch.from_struct_array(pa.array([{}] * len(rows), pa.struct([])))])
    return pa.table({k: pa.array([r.get(k) for r in rows]) for k in names})
