"""Row materialisation: FileReader.NextRow's records from the GPU-decoded
columns.

A restatement of the reference's record assembly over the columnar outputs of the device decode
(per page: definition / repetition levels and the dense not-null values):

  ColumnStore.get / getRDLevelAt / readNextPage   data_store.go:193-309  -> LeafStore
  Column.getNextData / getFirstRDLevel / getData  schema.go:216-312      -> Node
  schema.getData (root, never nil)                schema.go:790-800      -> RowAssembler.next_row

Records are dicts keyed by field name; a repeated leaf yields a list of its values, a repeated
group a list of dicts, a group a dict; null / empty fields are absent, exactly as the reference's
map[string]interface{} rows.  Level cursors are page-local as in the reference (readNextPage resets
them), so the assembly sees the same page boundaries.
"""
from collections import namedtuple

import numpy as np

REQUIRED, OPTIONAL, REPEATED = 0, 1, 2
# readValues outcome of one page: status 0 or the first error's (status, phase, index)
PageResult = namedtuple("PageResult", "status phase index")
PAGE_OK = PageResult(0, 0, 0)
BOOLEAN, INT32, INT64, INT96, FLOAT, DOUBLE, BYTE_ARRAY, FIXED_LEN_BYTE_ARRAY = range(8)


class RecordError(RuntimeError):
    """An error of the row assembly; for a page that failed to decode, its (status, phase, index)
    and the page's position in the chunk."""

    def __init__(self, msg, status=0, phase=0, index=0, page=-1):
        super().__init__(msg)
        self.status, self.phase, self.index, self.page = status, phase, index, page


class ReferencePanic(RecordError):
    """Where the reference's record assembly panics with a runtime.Error, which FileReader.recover
    re-panics (file_reader.go:177-184): the process would crash; here the call raises this."""


def page_values(ptype, col, v0, nn):
    """Dense values [v0, v0 + nn) of a decoded chunk as the reference's Go values (int32/int64 ->
    int, float32/float64 -> float, bool, []byte / [12]byte -> bytes; the nil interface{} of a short
    INT96 value, col.value_nil, -> None)."""
    if nn == 0:
        return []
    if col.values is not None:
        v = col.values[v0:v0 + nn]
        if ptype == BOOLEAN:
            return [bool(x) for x in v]
        if v.ndim == 2:
            nil = getattr(col, "value_nil", None)
            if nil is not None:
                return [None if nil[v0 + i] else bytes(r) for i, r in enumerate(v)]
            return [bytes(r) for r in v]
        return v.tolist()
    d = col.data.tobytes()
    o = col.offsets
    return [d[o[i]:o[i + 1]] for i in range(v0, v0 + nn)]


class LeafStore:
    """ColumnStore (data_store.go): the levels and values of one leaf column chunk, page by page."""

    def __init__(self, col, path, rep_typ, max_d, max_r, pages=None, skipped=False):
        self.col = col
        self.path = path
        self.rep_typ = rep_typ
        self.max_d, self.max_r = max_d, max_r
        self.skipped = skipped
        self.pages = pages or []  # [(result, n, def, rep, values())] of the chunk's data pages
        self.page_idx = 0
        self.read_pos = 0
        self.d = self.r = np.zeros(0, np.uint8)
        self.vals, self.vpos = [], 0

    @classmethod
    def from_column(cls, col, ptype, path, rep_typ):
        """Pages of a GPU-decoded chunk (reader.ColumnData with its page results)."""
        pages = []
        if col.load_error is None:  # (a chunk whose readChunk failed never gets here: its row group fails)
            for pt, n, res in col.page_info:
                if pt == 2:  # the dictionary page is consumed at chunk load
                    continue
                lo = res.level_offset
                d = col.def_levels[lo:lo + n] if col.def_levels is not None else np.zeros(n, np.uint8)
                r = col.rep_levels[lo:lo + n] if col.rep_levels is not None else np.zeros(n, np.uint8)
                pages.append((res, n, d, r,
                              lambda v0=res.value_offset, nn=res.num_non_null: page_values(ptype, col, v0, nn)))
        return cls(col, path, rep_typ, col.max_def, col.max_rep, pages)

    def _read_next_page(self):  # readNextPage (data_store.go:236-260)
        if self.page_idx >= len(self.pages):
            raise RecordError(f"{self.path}: out of range: requested page index = {self.page_idx} "
                              f"total number of pages = {len(self.pages)}")
        res, n, d, r, vals = self.pages[self.page_idx]
        if res.status:  # readValues fails: the error surfaces here, page_idx stays (every later call fails too)
            raise RecordError(f"{self.path}: page {self.page_idx} failed to decode (status {res.status}, phase "
                              f"{res.phase}, index {res.index})", res.status, res.phase, res.index, self.page_idx)
        self.page_idx += 1
        self.read_pos = 0
        self.d, self.r = d, r
        self.vals = vals()
        self.vpos = 0

    def rd_level_at(self, pos=-1):  # getRDLevelAt (data_store.go:193-210)
        if pos < 0:
            pos = self.read_pos
        if pos >= len(self.r) or pos >= len(self.d):
            return 0, 0, True
        return int(self.r[pos]), int(self.d[pos]), False

    def _next(self):  # getNext -> dictStore.getNextValue
        if self.vpos >= len(self.vals):
            raise RecordError(f"{self.path}: out of range: no more values")
        v = self.vals[self.vpos]
        self.vpos += 1
        return v

    def get(self, max_d, max_r):  # ColumnStore.get (data_store.go:262-309)
        if self.skipped:
            return None, 0
        if self.read_pos >= len(self.r) or self.read_pos >= len(self.d):
            self._read_next_page()
        dl = int(self.d[self.read_pos])
        if dl < max_d:  # a null at depth dl
            self.read_pos += 1
            return None, dl
        v = self._next()
        if self.rep_typ != REPEATED:
            self.read_pos += 1
            return v, max_d
        ret = [self._append(v)]
        while True:
            self.read_pos += 1
            rl, _, last = self.rd_level_at(self.read_pos)
            if last or rl < max_r:
                return ret, max_d
            ret.append(self._append(self._next()))

    def _append(self, v):
        """typedColumnStore.append: a nil value of a repeated leaf (a short INT96 value,
        type_int96.go:21-42) fails int96Store.append's type assertion value.([12]byte)
        (type_int96.go:113-118) -- a runtime panic the reference re-panics."""
        if v is None:
            raise ReferencePanic(f"{self.path}: panic: interface conversion: interface {{}} is nil, not [12]uint8")
        return v


class Node:
    """Column (schema.go): a group with children, or a leaf with its store."""

    def __init__(self, name, rep, max_d, max_r, children=None, store=None):
        self.name, self.rep, self.max_d, self.max_r = name, rep, max_d, max_r
        self.children = children
        self.store = store

    def get_next_data(self):  # getNextData (schema.go:216-258)
        ret = {}
        not_nil = 0
        max_d = 0
        for c in self.children:
            data, dl = c.get_data()
            if dl > max_d:
                max_d = dl
            if data is not None:
                ret[c.name] = data
                not_nil += 1
            diff = 1 if c.rep != REQUIRED else 0
            if dl == c.max_d - diff:  # null one level below: the parent is there
                not_nil += 1
        if not_nil == 0:
            return None, max_d
        return ret, self.max_d

    def first_rd_level(self):  # getFirstRDLevel (schema.go:260-281)
        if self.store is not None:
            return self.store.rd_level_at(-1)
        for c in self.children:
            rl, dl, last = c.first_rd_level()
            if last:
                return rl, dl, last
            if rl >= c.max_r or dl >= c.max_d:
                return rl, dl, last
        return -1, -1, False

    def get_data(self):  # getData (schema.go:283-312)
        if self.children is not None:
            data, max_d = self.get_next_data()
            if self.rep != REPEATED or data is None:
                return data, max_d
            ret = [data]
            while True:
                rl, _, last = self.first_rd_level()
                if last or rl < self.max_r or rl == 0:
                    return ret, max_d
                data, _ = self.get_next_data()
                ret.append(data)
        return self.store.get(self.max_d, self.max_r)


def build_tree(schema, stores):
    """The Column tree from the flat schema list [(name, pqh_schema_element)] (DFS, root first);
    stores[column index] = the leaf's LeafStore (a skipped store for unselected columns)."""
    pos = [1]

    def node(i):
        name, e = schema[i]
        if e.num_children == 0:
            return Node(name, e.repetition, e.max_def, e.max_rep, store=stores[e.column])
        kids = []
        for _ in range(e.num_children):
            j = pos[0]
            pos[0] += 1
            kids.append(node(j))
        return Node(name, e.repetition, e.max_def, e.max_rep, children=kids)

    # readSchema (schema.go:992-1015): every element after the root is read as a top-level child
    # until the list ends (the root's num_children is not consulted)
    root_name, root = schema[0]
    kids = []
    while pos[0] < len(schema):
        j = pos[0]
        pos[0] += 1
        kids.append(node(j))
    return Node(root_name, REQUIRED, 0, 0, children=kids)


class RowAssembler:
    """The records of one loaded row group (schemaReader after readRowGroupData)."""

    def __init__(self, schema, columns, num_rows, stores=None):
        """columns: {column index: (reader.ColumnData, physical type, path)} of the selected leaves;
        or stores: {column index: LeafStore} built by the caller (unlisted leaves are skipped)."""
        given = stores or {}
        stores = {}
        for name, e in schema:
            if e.num_children == 0:
                if e.column in given:
                    stores[e.column] = given[e.column]
                elif columns and e.column in columns:
                    col, ptype, path = columns[e.column]
                    stores[e.column] = LeafStore.from_column(col, ptype, path, e.repetition)
                else:
                    stores[e.column] = LeafStore(None, name, e.repetition, e.max_def, e.max_rep, skipped=True)
        self.root = build_tree(schema, stores)
        self.num_rows = num_rows
        self.current = 0

    def next_row(self):  # schema.getData (schema.go:790-800)
        d, _ = self.root.get_data()
        self.current += 1
        return {} if d is None else d
