"""Python front of libpqgen: files laid out like the reference WRITER produces them.

Tooling for tests and the benchmark (inputs only); decoding never goes through here.
"""
import ctypes
import os

import numpy as np

from . import _lib

BOOLEAN, INT32, INT64, INT96, FLOAT, DOUBLE, BYTE_ARRAY, FIXED_LEN_BYTE_ARRAY = range(8)
PLAIN, PLAIN_DICTIONARY, RLE, BIT_PACKED, DELTA_BINARY_PACKED, DELTA_LENGTH_BYTE_ARRAY, DELTA_BYTE_ARRAY, \
    RLE_DICTIONARY = 0, 2, 3, 4, 5, 6, 7, 8
REQUIRED, OPTIONAL, REPEATED = 0, 1, 2
UNCOMPRESSED, SNAPPY, GZIP = 0, 1, 2

_NP = {INT32: np.int32, INT64: np.int64, FLOAT: np.float32, DOUBLE: np.float64, BOOLEAN: np.uint8}


class SchemaElement(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("type", ctypes.c_int32), ("type_length", ctypes.c_int32),
                ("repetition", ctypes.c_int32), ("num_children", ctypes.c_int32), ("converted_type", ctypes.c_int32)]


class ColumnData(ctypes.Structure):
    _fields_ = [("encoding", ctypes.c_int32), ("use_dict", ctypes.c_int32),
                ("values", ctypes.c_void_p), ("offsets", ctypes.c_void_p), ("num_values", ctypes.c_int64),
                ("def_levels", ctypes.c_void_p), ("rep_levels", ctypes.c_void_p), ("num_slots", ctypes.c_int64),
                ("dict_page_limit", ctypes.c_int64)]


class Options(ctypes.Structure):
    _fields_ = [("data_page_v2", ctypes.c_int32), ("codec", ctypes.c_int32), ("max_page_size", ctypes.c_int64),
                ("enable_crc", ctypes.c_int32), ("num_threads", ctypes.c_int32), ("no_fast_paths", ctypes.c_int32)]


def element(name, ptype=-1, repetition=REQUIRED, num_children=0, type_length=0, converted_type=-1):
    return (name, ptype, type_length, repetition, num_children, converted_type)


class Column:
    """Leaf data: not-null values in order plus optional def/rep levels for every slot."""

    def __init__(self, ptype, values, def_levels=None, rep_levels=None, encoding=PLAIN, use_dict=True,
                 type_length=0, dict_page_limit=0):
        self.ptype = ptype
        self.dict_page_limit = dict_page_limit
        self.encoding = encoding
        self.use_dict = bool(use_dict) and ptype != BOOLEAN
        self.type_length = type_length
        if ptype == BYTE_ARRAY:
            if isinstance(values, tuple):
                self.data, self.offsets = values
            else:
                lens = np.fromiter((len(v) for v in values), dtype=np.int64, count=len(values))
                self.offsets = np.zeros(len(values) + 1, dtype=np.int64)
                np.cumsum(lens, out=self.offsets[1:])
                self.data = np.frombuffer(b"".join(values) + b"\0", dtype=np.uint8)
            self.num_values = len(self.offsets) - 1
        else:
            if ptype in _NP:
                arr = np.ascontiguousarray(values, dtype=_NP[ptype])
                self.data = arr.view(np.uint8).reshape(-1)
                self.num_values = len(arr)
            else:
                size = 12 if ptype == INT96 else type_length
                if isinstance(values, np.ndarray):
                    arr = np.ascontiguousarray(values, dtype=np.uint8).reshape(-1)
                else:
                    arr = np.frombuffer(b"".join(values), dtype=np.uint8)
                self.data = arr
                self.num_values = len(arr) // size
            self.offsets = None
        self.def_levels = None if def_levels is None else np.ascontiguousarray(def_levels, dtype=np.uint8)
        self.rep_levels = None if rep_levels is None else np.ascontiguousarray(rep_levels, dtype=np.uint8)
        self.num_slots = len(self.def_levels) if self.def_levels is not None else (
            len(self.rep_levels) if self.rep_levels is not None else self.num_values)

    def cstruct(self):
        c = ColumnData()
        c.encoding = self.encoding
        c.use_dict = int(self.use_dict)
        c.values = self.data.ctypes.data if len(self.data) else None
        c.offsets = self.offsets.ctypes.data if self.offsets is not None else None
        c.num_values = self.num_values
        c.def_levels = self.def_levels.ctypes.data if self.def_levels is not None else None
        c.rep_levels = self.rep_levels.ctypes.data if self.rep_levels is not None else None
        c.num_slots = self.num_slots
        c.dict_page_limit = self.dict_page_limit
        return c


def write(schema, columns, rg_rows, v2=False, codec=UNCOMPRESSED, max_page_size=0, crc=False, threads=0,
          as_array=False, fast_paths=True):
    """Write a file to bytes (or a uint8 numpy array with as_array=True, for multi-GB files).
    schema: list of element(...) tuples, root first, DFS order."""
    L = _lib.gen()
    names = [s[0].encode() for s in schema]
    els = (SchemaElement * len(schema))()
    for i, s in enumerate(schema):
        els[i] = SchemaElement(names[i], s[1], s[2], s[3], s[4], s[5])
    cols = (ColumnData * len(columns))()
    for i, c in enumerate(columns):
        cols[i] = c.cstruct()
    rows = np.ascontiguousarray(rg_rows, dtype=np.int64)
    opt = Options(int(v2), codec, max_page_size, int(crc), threads, int(not fast_paths))
    out = ctypes.POINTER(ctypes.c_uint8)()
    out_len = ctypes.c_int64()
    err = ctypes.create_string_buffer(512)
    rc = L.pqg_write(els, len(schema), cols, len(columns), rows.ctypes.data, len(rows), ctypes.byref(opt),
                     ctypes.byref(out), ctypes.byref(out_len), err, 512)
    if rc != 0:
        raise ValueError("pqg_write: " + err.value.decode())
    try:
        arr = np.empty(out_len.value, dtype=np.uint8)
        ctypes.memmove(arr.ctypes.data, out, out_len.value)
        return arr if as_array else arr.tobytes()
    finally:
        L.pqg_free(out)


class StreamWriter:
    """A file written row-group batch by row-group batch into one preallocated buffer (pqg_stream_*):
    for files larger than the columns of all their rows should be in memory at once.  `capacity`
    is an upper bound of the file size (the buffer is np.empty: pages never written are never
    touched).  The result equals write() of the same rows, byte for byte."""

    def __init__(self, schema, capacity, v2=False, codec=UNCOMPRESSED, max_page_size=0, crc=False, threads=0, buf=None):
        L = _lib.gen()
        self.L = L
        self._names = [x[0].encode() for x in schema]
        self._els = (SchemaElement * len(schema))()
        for i, x in enumerate(schema):
            self._els[i] = SchemaElement(self._names[i], x[1], x[2], x[3], x[4], x[5])
        self._opt = Options(int(v2), codec, max_page_size, int(crc), threads, 0)
        err = ctypes.create_string_buffer(512)
        self.h = L.pqg_stream_open(self._els, len(schema), ctypes.byref(self._opt), err, 512)
        if not self.h:
            raise ValueError("pqg_stream_open: " + err.value.decode())
        # (buf: a caller's uint8 buffer of >= capacity bytes, e.g. an np.memmap of a file, which the
        # pages are written into in place)
        self.buf = np.empty(int(capacity), dtype=np.uint8) if buf is None else buf
        self.pos = ctypes.c_int64(0)

    def write(self, columns, rg_rows):
        """Append row groups rg_rows (records each) whose data `columns` (Column list, schema leaf
        order) hold exactly."""
        cols = (ColumnData * len(columns))()
        for i, c in enumerate(columns):
            cols[i] = c.cstruct()
        rows = np.ascontiguousarray(rg_rows, dtype=np.int64)
        err = ctypes.create_string_buffer(512)
        rc = self.L.pqg_stream_write(self.h, cols, len(columns), rows.ctypes.data, len(rows), self.buf.ctypes.data,
                                     len(self.buf), ctypes.byref(self.pos), err, 512)
        if rc != 0:
            raise ValueError("pqg_stream_write: " + err.value.decode())

    def finish(self):
        """The file: a view of the buffer's first bytes."""
        err = ctypes.create_string_buffer(512)
        rc = self.L.pqg_stream_finish(self.h, self.buf.ctypes.data, len(self.buf), ctypes.byref(self.pos), err, 512)
        self.L.pqg_stream_close(self.h)
        self.h = None
        if rc != 0:
            raise ValueError("pqg_stream_finish: " + err.value.decode())
        return self.buf[:self.pos.value]


def flat_schema(columns):
    """The schema list of a flat file.  columns: list of (name, Column, repetition)."""
    schema = [element("schema", num_children=len(columns), repetition=-1)]
    for name, col, rep in columns:
        schema.append(element(name, col.ptype, rep, type_length=col.type_length))
    return schema


def flat(columns, rows_per_group, **kw):
    """Flat schema helper.  columns: list of (name, Column, repetition)."""
    schema = flat_schema(columns)
    n = columns[0][1].num_slots
    rg = []
    left = n
    while left > 0:
        rg.append(min(rows_per_group, left))
        left -= rg[-1]
    return write(schema, [c for _, c, _ in columns], rg or [0], **kw)


def optional(ptype, values, null_mask, **kw):
    """An OPTIONAL flat column from full-length values and a null mask (True = null)."""
    null_mask = np.asarray(null_mask, dtype=bool)
    deflv = (~null_mask).astype(np.uint8)
    if ptype == BYTE_ARRAY or isinstance(values, list):
        vals = [v for v, m in zip(values, null_mask) if not m]
    else:
        vals = np.asarray(values)[~null_mask]
    return Column(ptype, vals, def_levels=deflv, **kw)


def hybrid_encode(width, values):
    v = np.ascontiguousarray(values, dtype=np.int32)
    cap = 16 + (len(v) + 8) * max(width, 1)
    buf = np.zeros(cap, dtype=np.uint8)
    n = _lib.gen().pqg_hybrid_encode(width, v.ctypes.data, len(v), buf.ctypes.data, cap)
    assert n >= 0
    return buf[:n].tobytes()


def delta_encode(values, bits=64):
    v = np.ascontiguousarray(values, dtype=np.int64 if bits == 64 else np.int32)
    cap = 64 + len(v) * 10
    buf = np.zeros(cap, dtype=np.uint8)
    f = _lib.gen().pqg_delta_encode64 if bits == 64 else _lib.gen().pqg_delta_encode32
    n = f(v.ctypes.data, len(v), buf.ctypes.data, cap)
    assert n >= 0
    return buf[:n].tobytes()
