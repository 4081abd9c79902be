"""CPU ORACLE — test infrastructure only (never imported by the product path).

Python side of the oracle:
  * a pure-Python thrift compact-protocol reader for FileMetaData / PageHeader
    (restating reference helpers.go:103-109 + parquet/parquet.go generated readers),
  * a page walker restating FileReader.readChunk/readPages (chunk_reader.go:182-362) with
    readPageBlock / newBlockReader (chunk_reader.go:161-180, compress.go:131-152); codecs come
    from the Python stdlib (gzip) and pyarrow (snappy/zstd), independent of the product's C++,
  * ctypes bindings to oracle/build/liborcl.so (refdecode.c), the C restatement of the value and
    level decoders.

Parity pinning: see refdecode.h and DESIGN.md "Oracle".  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline may use this module.
"""
import ctypes
import gzip
import os
import struct
import subprocess
import zlib

import numpy as np

try:
    from .thrift_spec import SPEC
except ImportError:  # imported as a top-level module (oracle/ on sys.path)
    from thrift_spec import SPEC

HERE = os.path.dirname(os.path.abspath(__file__))
# ORC_LIB: another build of the oracle library (the sanitizer variant build/san/liborcl.so)
LIB_PATH = os.environ.get("ORC_LIB") or os.path.join(HERE, "build", "liborcl.so")

# parquet enums (parquet/parquet.thrift)
BOOLEAN, INT32, INT64, INT96, FLOAT, DOUBLE, BYTE_ARRAY, FIXED_LEN_BYTE_ARRAY = range(8)
DATA_PAGE, INDEX_PAGE, DICTIONARY_PAGE, DATA_PAGE_V2 = range(4)
UNCOMPRESSED, SNAPPY, GZIP, ZSTD = 0, 1, 2, 6
PHASE_LOAD, PHASE_REP, PHASE_DEF, PHASE_VALUES = range(4)

# status codes shared with include/pqhip.h
OK = 0
ERR_PAGE_HEADER = 22
ERR_DECOMPRESS = 23
ERR_CRC = 24
ERR_THRIFT = 25
ERR_SCHEMA = 30
ERR_DICT_PAGE = 31
ERR_UNSUPPORTED = 21


def build():
    """Compile refdecode.c (gcc) into oracle/build/liborcl.so."""
    subprocess.check_call(["make", "-s", "-C", HERE])


# ------------------------------------------------------------------------------------------------
# ctypes binding
# ------------------------------------------------------------------------------------------------
class OrcColumn(ctypes.Structure):
    _fields_ = [("physical_type", ctypes.c_int32), ("type_length", ctypes.c_int32),
                ("max_def", ctypes.c_int32), ("max_rep", ctypes.c_int32)]


class OrcPage(ctypes.Structure):
    _fields_ = [("page_type", ctypes.c_int32), ("num_values", ctypes.c_int32),
                ("encoding", ctypes.c_int32), ("def_levels_byte_length", ctypes.c_int32),
                ("rep_levels_byte_length", ctypes.c_int32)]


class OrcDict(ctypes.Structure):
    _fields_ = [("num_values", ctypes.c_int32), ("value_size", ctypes.c_int32),
                ("values", ctypes.POINTER(ctypes.c_uint8)), ("offsets", ctypes.POINTER(ctypes.c_int64)),
                ("num_bytes", ctypes.c_int64), ("nil_last", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class OrcOut(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int32), ("phase", ctypes.c_int32), ("index", ctypes.c_int64),
                ("num_values", ctypes.c_int32), ("nn", ctypes.c_int32),
                ("def_", ctypes.POINTER(ctypes.c_uint8)), ("rep", ctypes.POINTER(ctypes.c_uint8)),
                ("value_size", ctypes.c_int32), ("values", ctypes.POINTER(ctypes.c_uint8)),
                ("values_bytes", ctypes.c_int64), ("offsets", ctypes.POINTER(ctypes.c_int64)),
                ("num_offsets", ctypes.c_int64), ("nil", ctypes.POINTER(ctypes.c_uint8)),
                ("num_nil", ctypes.c_int64)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.orc_unpack8_int32.argtypes = [ctypes.c_int32, u8p, ctypes.POINTER(ctypes.c_int32)]
        L.orc_unpack8_int64.argtypes = [ctypes.c_int32, u8p, ctypes.POINTER(ctypes.c_int64)]
        L.orc_pack8_int32.argtypes = [ctypes.c_int32, ctypes.POINTER(ctypes.c_int32), u8p]
        L.orc_pack8_int64.argtypes = [ctypes.c_int32, ctypes.POINTER(ctypes.c_int64), u8p]
        L.orc_hybrid_decode.argtypes = [ctypes.c_int32, u8p, ctypes.c_int64, ctypes.c_int32,
                                        ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]
        L.orc_delta_decode32.argtypes = [u8p, ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32),
                                         ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]
        L.orc_delta_decode64.argtypes = [u8p, ctypes.c_int64, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64),
                                         ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]
        L.orc_decode_dict_page.argtypes = [ctypes.POINTER(OrcColumn), ctypes.c_int32, ctypes.c_int32, u8p,
                                           ctypes.c_int64, ctypes.POINTER(OrcDict)]
        L.orc_decode_dict_page_ex.argtypes = [ctypes.POINTER(OrcColumn), ctypes.c_int32, ctypes.c_int32, u8p,
                                              ctypes.c_int64, ctypes.POINTER(OrcDict), ctypes.POINTER(ctypes.c_int64)]
        L.orc_dict_free.argtypes = [ctypes.POINTER(OrcDict)]
        L.orc_select.argtypes = [ctypes.POINTER(OrcColumn), ctypes.c_int32]
        L.orc_decode_page.argtypes = [ctypes.POINTER(OrcColumn), ctypes.POINTER(OrcPage), u8p, ctypes.c_int64,
                                      ctypes.POINTER(OrcDict), ctypes.POINTER(OrcOut)]
        L.orc_out_free.argtypes = [ctypes.POINTER(OrcOut)]
        _lib = L
    return _lib


def _u8(buf):
    arr = np.frombuffer(buf, dtype=np.uint8) if not isinstance(buf, np.ndarray) else buf
    arr = np.ascontiguousarray(arr, dtype=np.uint8)
    return arr, arr.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def unpack8(width, data, bits=32):
    arr, p = _u8(bytes(data) + b"\0" * 64)
    if bits == 32:
        out = (ctypes.c_int32 * 8)()
        lib().orc_unpack8_int32(width, p, out)
    else:
        out = (ctypes.c_int64 * 8)()
        lib().orc_unpack8_int64(width, p, out)
    return list(out)


def pack8(width, values, bits=32):
    buf = (ctypes.c_uint8 * max(width, 1))()
    if bits == 32:
        lib().orc_pack8_int32(width, (ctypes.c_int32 * 8)(*values), buf)
    else:
        lib().orc_pack8_int64(width, (ctypes.c_int64 * 8)(*values), buf)
    return bytes(buf)[:width]


def hybrid_decode(width, data, n):
    arr, p = _u8(data)
    out = np.zeros(max(n, 1), dtype=np.int32)
    dec = ctypes.c_int32()
    st = lib().orc_hybrid_decode(width, p, len(arr), n, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                 ctypes.byref(dec))
    return st, out[: dec.value]


def delta_decode(data, n, bits=64):
    arr, p = _u8(data)
    dec = ctypes.c_int32()
    vc = ctypes.c_int32()
    if bits == 64:
        out = np.zeros(max(n, 1), dtype=np.int64)
        st = lib().orc_delta_decode64(p, len(arr), n, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                      ctypes.byref(dec), ctypes.byref(vc))
    else:
        out = np.zeros(max(n, 1), dtype=np.int32)
        st = lib().orc_delta_decode32(p, len(arr), n, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                      ctypes.byref(dec), ctypes.byref(vc))
    return st, out[: dec.value], vc.value


class Dictionary:
    def __init__(self, status, num_values=0, value_size=0, values=b"", offsets=None, index=0, nil_last=False):
        self.status = status
        self.index = index  # the values read before the failing one
        self.num_values = num_values
        self.value_size = value_size
        self.values = values
        self.offsets = offsets
        # the last entry is the reference's nil (INT96 dictionary page whose last value is short,
        # type_int96.go:21-42); its bytes in `values` are zeros
        self.nil_last = nil_last


def decode_dict_page(col, num_values, encoding, image):
    arr, p = _u8(image)
    c = OrcColumn(*col)
    d = OrcDict()
    ei = ctypes.c_int64()
    st = lib().orc_decode_dict_page_ex(ctypes.byref(c), num_values, encoding, p, len(arr), ctypes.byref(d),
                                       ctypes.byref(ei))
    if st:
        return Dictionary(st, index=ei.value)
    vals = ctypes.string_at(d.values, d.num_bytes) if d.num_bytes else b""
    offs = None
    if d.value_size == 0:
        offs = np.ctypeslib.as_array(d.offsets, shape=(d.num_values + 1,)).copy()
    res = Dictionary(OK, d.num_values, d.value_size, vals, offs, nil_last=bool(d.nil_last))
    lib().orc_dict_free(ctypes.byref(d))
    return res


class PageResult:
    """readValues(numValues) of one page: values, dLevel, rLevel, notNull, and the first error."""

    def __init__(self):
        self.status = OK
        self.phase = 0
        self.index = 0
        self.num_values = 0
        self.nn = 0
        self.def_levels = None
        self.rep_levels = None
        self.value_size = 0
        self.values = b""
        self.offsets = None
        # None, or a uint8 array of nn: 1 = the value slot is the reference's nil (an INT96 value
        # left unassigned by a short read, type_int96.go:21-42); its bytes in `values` are zeros
        self.nil = None


def _to_cdict(d):
    if d is None or d.status != OK:
        return None, None
    keep = []
    cd = OrcDict()
    cd.num_values = d.num_values
    cd.value_size = d.value_size
    va = np.frombuffer(d.values + b"\0", dtype=np.uint8).copy()
    keep.append(va)
    cd.values = va.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))
    cd.num_bytes = len(d.values)
    cd.nil_last = int(getattr(d, "nil_last", False))
    if d.offsets is not None:
        oa = np.ascontiguousarray(d.offsets, dtype=np.int64)
        keep.append(oa)
        cd.offsets = oa.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))
    return cd, keep


def select(col, encoding):
    """getValuesDecoder (chunk_reader.go:106-159): OK or ERR_UNSUPPORTED."""
    c = OrcColumn(*col)
    return lib().orc_select(ctypes.byref(c), encoding)


def decode_page(col, page_type, num_values, encoding, def_len, rep_len, image, dictionary=None):
    arr, p = _u8(image if len(image) else b"\0")
    c = OrcColumn(*col)
    pg = OrcPage(page_type, num_values, encoding, def_len, rep_len)
    cd, keep = _to_cdict(dictionary)
    o = OrcOut()
    lib().orc_decode_page(ctypes.byref(c), ctypes.byref(pg), p, len(image), ctypes.byref(cd) if cd else None,
                          ctypes.byref(o))
    r = PageResult()
    r.status, r.phase, r.index = o.status, o.phase, o.index
    r.num_values, r.nn, r.value_size = o.num_values, o.nn, o.value_size
    if o.def_:
        r.def_levels = np.ctypeslib.as_array(o.def_, shape=(o.num_values,)).copy()
    if o.rep:
        r.rep_levels = np.ctypeslib.as_array(o.rep, shape=(o.num_values,)).copy()
    if o.values_bytes:
        r.values = ctypes.string_at(o.values, o.values_bytes)
    if o.offsets and o.num_offsets:
        r.offsets = np.ctypeslib.as_array(o.offsets, shape=(o.num_offsets,)).copy()
    if o.nil:
        r.nil = np.ctypeslib.as_array(o.nil, shape=(o.nn,)).copy()
    lib().orc_out_free(ctypes.byref(o))
    return r


# ------------------------------------------------------------------------------------------------
# Thrift compact protocol, restated from the reference's thrift library (vendored apache/thrift
# v0.16.0: lib/go/thrift/compact_protocol.go ReadFieldBegin :429-468, ReadListBegin :505-529,
# ReadMapBegin :475-497, ReadBool :546-553, ReadI16/I32/I64 :565-588, ReadString :601-622,
# readVarint64 :747-762, getTType :802-830; protocol.go Skip :92-182; configuration.go
# checkSizeForProtocol :305-319) and the generated struct readers (parquet/parquet.go, their field
# ids / accepted wire types / required fields as the table oracle/thrift_spec.py).
# ------------------------------------------------------------------------------------------------
class ThriftError(Exception):
    pass


MAX_SIZE = 100 * 1024 * 1024  # DEFAULT_MAX_MESSAGE_SIZE
MAX_DEPTH = 64                # DEFAULT_RECURSION_DEPTH


def _i32(u):
    u &= 0xFFFFFFFF
    return u - (1 << 32) if u >> 31 else u


def _i64(u):
    u &= (1 << 64) - 1
    return u - (1 << 64) if u >> 63 else u


class CompactReader:
    """A TCompactProtocol over buf[pos:end] (StreamTransport: reads past `end` fail)."""

    def __init__(self, buf, pos=0, end=None):
        self.buf = buf
        self.pos = pos
        self.end = len(buf) if end is None else end
        self.bool_pending = None

    def byte(self):
        if self.pos >= self.end:
            raise ThriftError("EOF")
        b = self.buf[self.pos]
        self.pos += 1
        return b

    def varint64(self):  # no length limit; bits past 63 vanish
        x, s = 0, 0
        while True:
            b = self.byte()
            if s < 64:
                x |= (b & 0x7F) << s
            if not b & 0x80:
                return _i64(x)
            s += 7

    def varint32(self):
        return _i32(self.varint64())

    def i32(self):
        u = self.varint32() & 0xFFFFFFFF
        return _i32((u >> 1) ^ -(u & 1))

    def i16(self):
        v = self.i32() & 0xFFFF
        return v - 0x10000 if v >> 15 else v

    def i64(self):
        u = self.varint64() & ((1 << 64) - 1)
        return _i64((u >> 1) ^ -(u & 1))

    def double(self):
        if self.end - self.pos < 8:
            raise ThriftError("EOF in double")
        v = struct.unpack_from("<d", self.buf, self.pos)[0]
        self.pos += 8
        return v

    def string(self):
        n = self.varint32()
        if n < 0 or n > MAX_SIZE:
            raise ThriftError("bad size")
        if self.end - self.pos < n:
            raise ThriftError("EOF in binary")
        v = bytes(self.buf[self.pos:self.pos + n])
        self.pos += n
        return v

    @staticmethod
    def wire(nib):
        """getTType: 0 STOP, 1 bool (compact 1 / 2), 3..12, None for 13..15."""
        nib &= 0x0F
        if nib == 2:
            return 1
        return nib if nib <= 12 else None

    def field(self, last):
        """(id, wire type) or None at STOP."""
        h = self.byte()
        if h & 0x0F == 0:
            return None
        d = h >> 4
        fid = self.i16() if d == 0 else ((last + d + 0x8000) & 0xFFFF) - 0x8000
        t = self.wire(h)
        if t is None:
            raise ThriftError(f"unknown type {h & 0x0F}")
        if t == 1:
            self.bool_pending = (h & 0x0F) == 1
        return fid, t

    def read_bool(self):
        if self.bool_pending is not None:
            v, self.bool_pending = self.bool_pending, None
            return v
        return self.byte() == 1

    def list_begin(self):
        h = self.byte()
        n = h >> 4
        if n == 15:
            n = self.varint32()
        et = self.wire(h)
        if n < 0 or n > MAX_SIZE or et is None:
            raise ThriftError("bad list header")
        return et, n

    def skip(self, t, depth=MAX_DEPTH):
        if depth <= 0:
            raise ThriftError("depth limit")
        if t == 1:
            self.read_bool()
        elif t == 3:
            self.byte()
        elif t in (4, 5):
            self.varint32()
        elif t == 6:
            self.varint64()
        elif t == 7:
            self.double()
        elif t == 8:
            self.string()
        elif t in (9, 10):
            et, n = self.list_begin()
            for _ in range(n):
                self.skip(et, depth - 1)
        elif t == 11:
            n = self.varint32()
            if n < 0 or n > MAX_SIZE:
                raise ThriftError("bad map size")
            kv = self.byte() if n else 0
            kt, vt = self.wire(kv >> 4) or 0, self.wire(kv & 0x0F) or 0
            for _ in range(n):
                self.skip(kt, depth - 1)
                self.skip(vt, depth - 1)
        elif t == 12:
            last = 0
            while True:
                f = self.field(last)
                if f is None:
                    return
                last = f[0]
                self.skip(f[1], depth - 1)
        else:
            raise ThriftError(f"unknown data type {t}")

    def _elem(self, t, sub):
        if t == 1:
            return self.read_bool()
        if t == 3:
            b = self.byte()
            return b - 256 if b > 127 else b
        if t == 4:
            return self.i16()
        if t == 5:
            return self.i32()
        if t == 6:
            return self.i64()
        if t == 7:
            return self.double()
        if t == 8:
            return self.string()
        if t == 12:
            return self.read(sub)
        raise ThriftError(f"bad element type {t}")

    def read(self, name):
        """The generated Go reader of struct `name`: {field id: value} of the fields whose id and wire
        type match (others skipped; a repeated field keeps its last value); required fields checked."""
        spec = SPEC[name]
        out = {}
        last = 0
        while True:
            f = self.field(last)
            if f is None:
                break
            fid, t = f
            last = fid
            sp = spec.get(fid)
            if sp is None or sp[1] != t:
                self.skip(t)
                continue
            _, wt, et, sub, _ = sp
            if wt == 9:
                _, n = self.list_begin()
                out[fid] = [self._elem(et, sub) for _ in range(n)]
            else:
                out[fid] = self._elem(wt, sub)
        for fid, sp in spec.items():
            if sp[4] and fid not in out:
                raise ThriftError(f"required field {name}.{sp[0]} is not set")
        return out

    def struct(self, name="PageHeader"):
        return self.read(name)


# ------------------------------------------------------------------------------------------------
# File reader restatement
# ------------------------------------------------------------------------------------------------
class Column:
    def __init__(self, path, element, max_def, max_rep, rep_def=()):
        self.path = path
        self.physical_type = element.get(1)
        self.type_length = element.get(2, 0)
        self.max_def = max_def
        self.max_rep = max_rep
        self.rep_def = tuple(rep_def)  # definition level of each REPEATED node on the path, outermost first

    def desc(self):
        return (self.physical_type, self.type_length or 0, self.max_def, self.max_rep)


class SchemaError(ValueError):
    pass


def _name(s):
    return s.get(4, b"").decode("utf-8", "surrogateescape")


def read_schema(schema):
    """makeSchema + readSchema (schema.go:1048-1079, :992-1015): the elements after the root are read
    as top-level groups / columns until the list ends; readGroupSchema / readColumnSchema
    (:893-990) and getValuesStore (data_store.go:328-362) checks.  Leaves in DFS order."""
    if len(schema) < 1:
        raise SchemaError("no schema element found")
    els = schema[1:]
    leaves = []

    def column(idx, path, d, r, rd):
        s = els[idx]
        if not s.get(4):
            raise SchemaError("name in schema is empty")
        rep = s.get(3)
        if rep is None:
            raise SchemaError("field RepetitionType is nil")
        if rep != 0:
            d += 1
        if rep == 2:
            r += 1
            rd = rd + [d]
        t = s.get(1)
        if t < 0 or t > FIXED_LEN_BYTE_ARRAY:
            raise SchemaError("unsupported type")
        if t == FIXED_LEN_BYTE_ARRAY and s.get(2) is None:
            raise SchemaError("type with nil type length")
        leaves.append(Column(".".join(path + [_name(s)]), s, d, r, rd))
        return idx + 1

    def group(idx, path, d, r, rd):
        if len(els) <= idx:
            raise SchemaError("schema index out of bound")
        s = els[idx]
        if s.get(1) is not None:
            raise SchemaError("field Type is not nil")
        n = s.get(5)
        if n is None:
            raise SchemaError("the field NumChildren is invalid")
        if n <= 0:
            raise SchemaError("the field NumChildren is zero")
        if len(els) <= idx + n:
            raise SchemaError("not enough element in the schema list")
        rep = s.get(3)
        if rep is not None and rep != 0:
            d += 1
        if rep is not None and rep == 2:
            r += 1
            rd = rd + [d]
        p = path + [_name(s)]
        idx += 1
        for _ in range(n):
            if len(els) <= idx:
                raise SchemaError("schema index is out of bounds")
            idx = group(idx, p, d, r, rd) if els[idx].get(1) is None else column(idx, p, d, r, rd)
        return idx

    idx = 0
    while idx < len(els):
        idx = group(idx, [], 0, 0, []) if els[idx].get(1) is None else column(idx, [], 0, 0, [])
    return leaves


# The codecs the reference registers at init (compress.go:182-187).
DEFAULT_CODECS = (UNCOMPRESSED, GZIP, SNAPPY, ZSTD)


def decompress(codec, data, uncompressed_size):
    if codec == UNCOMPRESSED:
        return bytes(data)
    if codec == GZIP:
        return gzip_decode(data)
    if codec == SNAPPY:
        return snappy_decode(data)
    import pyarrow as pa

    name = {ZSTD: "zstd"}.get(codec)
    if name is None:
        raise ValueError(f"codec {codec} not supported")
    return pa.decompress(bytes(data), decompressed_size=uncompressed_size, codec=name, asbytes=True)


class GzipCorrupt(Exception):
    pass


def gzip_decode(src):
    """The reference's GZIP codec (gzipCompressor.DecompressBlock, compress.go:64-77):
    gzip.NewReader + ioutil.ReadAll of Go's compress/gzip (gunzip.go, the standard library; not
    vendored in /root/reference), restated member by member:
      header  = 10 bytes (io.ReadFull: fewer is an error; none at all is io.EOF, an error for the
                first member and the end of the stream after a later one), ID1 0x1f ID2 0x8b CM 8
                (ErrHeader; reserved flag bits are ignored), FEXTRA (2-byte LE length + data, short
                reads fail), FNAME / FCOMMENT (NUL-terminated within 512 bytes, else ErrHeader),
                FHCRC (uint16 of the CRC-32 of the header bytes before it, else ErrHeader);
      body    = one raw DEFLATE stream (RFC 1951) -> zlib raw inflate (identical to Go's
                compress/flate on every valid stream; any error fails the block);
      trailer = CRC-32 and ISIZE (output length mod 2^32) of the member, 8 bytes LE (short:
                ErrUnexpectedEOF; mismatch: ErrChecksum);
    then the next member (multistream, the Reader's default) until the input ends.  Python's
    gzip.decompress differs (it skips zero padding after a member), so it is not used here.
    Raises GzipCorrupt."""
    data = bytes(src)
    out = bytearray()
    pos, first = 0, True
    while True:
        if pos == len(data) and not first:
            break
        if len(data) - pos < 10:
            raise GzipCorrupt("header")
        h = data[pos:pos + 10]
        if h[0] != 0x1F or h[1] != 0x8B or h[2] != 8:
            raise GzipCorrupt("ErrHeader")
        flg, q = h[3], pos + 10
        if flg & 4:  # FEXTRA
            if len(data) - q < 2:
                raise GzipCorrupt("extra length")
            xlen = int.from_bytes(data[q:q + 2], "little")
            q += 2
            if len(data) - q < xlen:
                raise GzipCorrupt("extra")
            q += xlen
        for bit in (8, 16):  # FNAME, FCOMMENT: readString
            if flg & bit:
                i = 0
                while True:
                    if i >= 512:
                        raise GzipCorrupt("ErrHeader: string")
                    if q + i >= len(data):
                        raise GzipCorrupt("string EOF")
                    if data[q + i] == 0:
                        break
                    i += 1
                q += i + 1
        if flg & 2:  # FHCRC
            if len(data) - q < 2:
                raise GzipCorrupt("header crc")
            if (zlib.crc32(data[pos:q]) & 0xFFFF) != int.from_bytes(data[q:q + 2], "little"):
                raise GzipCorrupt("ErrHeader: crc")
            q += 2
        d = zlib.decompressobj(-15)
        try:
            member = d.decompress(data[q:])
        except zlib.error as e:
            raise GzipCorrupt(f"flate: {e}") from None
        if not d.eof:
            raise GzipCorrupt("flate: unexpected EOF")
        t = len(data) - len(d.unused_data)
        if len(data) - t < 8:
            raise GzipCorrupt("trailer")
        crc = int.from_bytes(data[t:t + 4], "little")
        isize = int.from_bytes(data[t + 4:t + 8], "little")
        if crc != (zlib.crc32(member) & 0xFFFFFFFF) or isize != (len(member) & 0xFFFFFFFF):
            raise GzipCorrupt("ErrChecksum")
        out += member
        pos, first = t + 8, False
    return bytes(out)


class SnappyCorrupt(Exception):
    pass


def snappy_decode(src):
    """github.com/golang/snappy v0.0.4 Decode, restated from the copy vendored in the reference:
    vendor/github.com/golang/snappy/decode.go:32-55 (decodedLen), :57-76 (Decode) and
    decode_other.go:14-101 (decode: tagLiteral :18-58, tagCopy1/2/4 :60-83, the offset / length
    check :85; the amd64 / arm64 assembly implements the same loop) — the reference's SNAPPY codec
    (compress.go:43-49).  Returns the block or raises SnappyCorrupt
    (ErrCorrupt / ErrTooLarge).  Pinned against pyarrow's snappy on valid blocks
    (tests/test_codec_oracle.py)."""
    src = bytes(src)
    # decodedLen: binary.Uvarint (n <= 0 on a missing terminator or a 64-bit overflow)
    v, shift, n = 0, 0, 0
    for i, c in enumerate(src[:10]):
        if i == 9 and c > 1:
            raise SnappyCorrupt("uvarint overflow")
        v |= (c & 0x7F) << shift
        shift += 7
        if c < 0x80:
            n = i + 1
            break
    if n == 0 or v > 0xFFFFFFFF:
        raise SnappyCorrupt("decodedLen")
    dst = bytearray(v)
    d, s = 0, n
    while s < len(src):
        tag = src[s]
        kind = tag & 3
        if kind == 0:
            x = tag >> 2
            if x < 60:
                s += 1
            else:
                k = x - 59
                s += 1 + k
                if s > len(src):
                    raise SnappyCorrupt("literal header")
                x = int.from_bytes(src[s - k:s], "little")
            length = x + 1
            if length > len(dst) - d or length > len(src) - s:
                raise SnappyCorrupt("literal")
            dst[d:d + length] = src[s:s + length]
            d += length
            s += length
            continue
        if kind == 1:
            s += 2
            if s > len(src):
                raise SnappyCorrupt("copy1 header")
            length = 4 + ((tag >> 2) & 7)
            offset = ((tag & 0xE0) << 3) | src[s - 1]
        elif kind == 2:
            s += 3
            if s > len(src):
                raise SnappyCorrupt("copy2 header")
            length = 1 + (tag >> 2)
            offset = src[s - 2] | (src[s - 1] << 8)
        else:
            s += 5
            if s > len(src):
                raise SnappyCorrupt("copy4 header")
            length = 1 + (tag >> 2)
            offset = int.from_bytes(src[s - 4:s], "little")
        if offset <= 0 or d < offset or length > len(dst) - d:
            raise SnappyCorrupt("copy")
        for i in range(length):  # forward, overlap-safe
            dst[d + i] = dst[d + i - offset]
        d += length
    if d != len(dst):
        raise SnappyCorrupt("short")
    return bytes(dst)


class Page:
    def __init__(self, page_type, num_values, encoding, def_len, rep_len, image):
        self.page_type = page_type
        self.num_values = num_values
        self.encoding = encoding
        self.def_len = def_len
        self.rep_len = rep_len
        self.image = image


class Chunk:
    def __init__(self, column):
        self.column = column
        self.pages = []   # data pages (Page) read before the walk ended
        self.dict_page = None
        self.status = OK  # readChunk's error: (status, index) of the first page it could not load
        self.index = 0
        self.page = -1    # data pages read before that page


class FileError(ValueError):
    pass


ERR_IO = 26
PLAIN_ENC, PLAIN_DICTIONARY_ENC, RLE_ENC = 0, 2, 3


class FileReader:
    """The oracle's NewFileReader over a bytes object: ReadFileMetaData(r, extraValidation = true)
    (file_meta.go:23-73) + makeSchema (schema.go:1048-1079).  Raises FileError where the reference's
    NewFileReader returns an error."""

    def __init__(self, data, codecs=DEFAULT_CODECS):
        # the reference's compressors registry (compress.go:16-33,160-187): its init registers
        # UNCOMPRESSED, GZIP, SNAPPY and ZSTD; decompressBlock fails "method not supported" for others
        self.codecs = frozenset(codecs)
        # (bytes as given; anything else -- a numpy array, an mmap -- read in place through a
        # memoryview: a 36 GB file is not copied; page blocks are copied as they are read)
        self.data = data if isinstance(data, bytes) else memoryview(data).cast("B")
        d = self.data
        if len(d) < 4 or d[:4] != b"PAR1":
            raise FileError("invalid parquet file header")
        if d[-4:] != b"PAR1":
            raise FileError("invalid parquet file footer")
        if len(d) < 8:
            raise FileError("seek for the footer len failed")
        flen = struct.unpack_from("<i", d, len(d) - 8)[0]
        if flen <= 0:
            raise FileError(f"invalid footer len {flen}")
        if flen > len(d) - 8:
            raise FileError("seek file meta data failed")
        try:
            meta = CompactReader(d, len(d) - 8 - flen, len(d) - 8).read("FileMetaData")
        except ThriftError as e:
            raise FileError(f"read file meta failed: {e}")
        self.meta = meta
        try:
            self.columns = read_schema(meta[2])
        except SchemaError as e:
            raise FileError(f"creating schema failed: {e}")
        self.row_groups = meta[4]
        self.num_rows = meta[3]

    def row_group_num_rows(self, rg):
        return self.row_groups[rg][3]

    def chunk_check(self, rg, ci, selected=True):
        """readRowGroupData's checks of column ci before its pages (chunk_reader.go:381-393; readChunk
        :299-324 when selected, skipChunk :271-297 when not): OK / ERR_SCHEMA / ERR_IO."""
        cols = self.row_groups[rg][1]
        if len(cols) <= ci:
            return ERR_SCHEMA
        cc = cols[ci]
        if 1 in cc:
            return ERR_IO
        md = cc.get(3)
        if md is None:
            return ERR_SCHEMA
        if md[1] != self.columns[ci].physical_type:
            return ERR_SCHEMA
        off = md.get(11, md[9])
        if (off if selected else off + md[7]) < 0:
            return ERR_IO
        return OK

    def read_chunk(self, rg, ci, validate_crc=False):
        """readChunk + readPages (chunk_reader.go:182-362) in the reference's order of checks: every
        page is read and its decoders initialised (pageReader.read) before the next header; the walk
        stops at the first page that fails (ch.status, ch.index = the load step / values read).
        Returns the decompressed page images of the pages before it."""
        col = self.columns[ci]
        ch = Chunk(col)

        def fail(status, index=0):
            ch.status, ch.index, ch.page = status, index, len(ch.pages)
            return ch

        st = self.chunk_check(rg, ci)
        if st:
            return fail(st)
        md = self.row_groups[rg][1][ci][3]
        desc = col.desc()
        pos = md.get(11, md[9])
        total, codec = md[7], md[4]
        count = 0
        d = self.data
        while total - count > 0:
            try:
                rd = CompactReader(d, min(pos, len(d)))
                ph = rd.read("PageHeader")
            except ThriftError:
                return fail(ERR_THRIFT)
            count += rd.pos - min(pos, len(d))
            pos = rd.pos
            ptype = ph[1]
            usize, csize = ph[2], ph[3]
            block = None

            def read_block():  # readPageBlock (:161-180)
                nonlocal pos, count, block
                if csize < 0 or usize < 0:
                    return ERR_PAGE_HEADER
                block = bytes(d[pos:pos + csize])
                pos += len(block)
                count += len(block)
                if validate_crc and 4 in ph and (zlib.crc32(block) & 0xFFFFFFFF) != (ph[4] & 0xFFFFFFFF):
                    return ERR_CRC
                return OK

            def inflate(blk, csz, usz):  # newBlockReader (compress.go:131-152)
                if csz < 0 or usz < 0:
                    return None, ERR_PAGE_HEADER
                if len(blk) != csz:
                    return None, ERR_DECOMPRESS
                if codec not in self.codecs:  # decompressBlock: "method %q is not supported" (:119-129)
                    return None, ERR_DECOMPRESS
                try:
                    img = decompress(codec, blk, usz)
                except Exception:
                    return None, ERR_DECOMPRESS
                return (img, OK) if len(img) == usz else (None, ERR_DECOMPRESS)

            if ptype == DICTIONARY_PAGE:
                if ch.dict_page is not None:
                    return fail(ERR_DICT_PAGE)
                if col.physical_type == BOOLEAN:  # getDictValuesDecoder (:17-39)
                    return fail(ERR_UNSUPPORTED)
                dh = ph.get(7)  # dictPageReader.read (page_dict.go:35-72)
                if dh is None or dh[1] < 0:
                    return fail(ERR_PAGE_HEADER)
                if dh[2] not in (PLAIN_ENC, PLAIN_DICTIONARY_ENC):
                    return fail(ERR_DICT_PAGE)
                st = read_block()
                if st:
                    return fail(st)
                img, st = inflate(block, csize, usize)
                if st:
                    return fail(st)
                dic = decode_dict_page(desc, dh[1], dh[2], img)
                if dic.status != OK:
                    return fail(dic.status, dic.index)
                ch.dict_page = dic
                if 11 in md and md[11] != pos:  # back to DataPageOffset
                    if md[9] < 0:
                        return fail(ERR_IO)
                    count += md[9] - pos
                    pos = md[9]
                continue
            if ptype == DATA_PAGE:
                h = ph.get(5)  # dataPageReaderV1.init (page_v1.go:65-85), then .read (:87-122)
                if h is None:
                    return fail(ERR_PAGE_HEADER)
                if (col.max_rep > 0 and h[4] != RLE_ENC) or (col.max_def > 0 and h[3] != RLE_ENC):
                    return fail(ERR_UNSUPPORTED)
                if h[1] < 0:
                    return fail(ERR_PAGE_HEADER)
                st = read_block()
                if st:
                    return fail(st)
                img, st = inflate(block, csize, usize)
                if st:
                    return fail(st)
                page = Page(DATA_PAGE, h[1], h[2], 0, 0, img)
            elif ptype == DATA_PAGE_V2:
                h = ph.get(8)  # dataPageReaderV2.read (page_v2.go:79-131)
                if h is None:
                    return fail(ERR_PAGE_HEADER)
                dl, rl = h[5], h[6]
                if h[1] < 0 or rl < 0 or dl < 0:
                    return fail(ERR_PAGE_HEADER)
                if select(desc, h[4]) != OK:  # getValuesDecoder before the block (:107-112)
                    return fail(ERR_UNSUPPORTED)
                st = read_block()
                if st:
                    return fail(st)
                if rl + dl > len(block):  # the level slices: a runtime panic in the reference
                    return fail(ERR_PAGE_HEADER)
                vals, st = inflate(block[rl + dl:], csize - rl - dl, usize - rl - dl)
                if st:
                    return fail(st)
                page = Page(DATA_PAGE_V2, h[1], h[4], dl, rl, block[: rl + dl] + vals)
            else:
                return fail(ERR_PAGE_HEADER)
            # the page's decoders: getValuesDecoder, initSize / init (phase 0 of the page decode)
            r = decode_page(desc, page.page_type, page.num_values, page.encoding, page.def_len, page.rep_len,
                            page.image, ch.dict_page)
            if r.status and r.phase == PHASE_LOAD:
                return fail(r.status, r.index)
            ch.pages.append(page)
        return ch


def decode_chunk(ch):
    """readValues(numValues) for every data page of a chunk (data_store.go:236-260)."""
    if ch.status != OK:
        return []
    return [decode_page(ch.column.desc(), p.page_type, p.num_values, p.encoding, p.def_len, p.rep_len,
                        p.image, ch.dict_page) for p in ch.pages]


# ---------------------------------------------------------------------------------------------
# Nesting: levels -> per repetition level list offsets / validity + leaf validity
# ---------------------------------------------------------------------------------------------
def nest_levels(def_levels, rep_levels, max_def, rep_def):
    """Columnar form of the reference's record assembly for one leaf column
    (ColumnStore.get data_store.go:262-309: d < maxD is a null at depth d, a repeated value collects
    while the next r >= maxR; Column.getNextData / getData schema.go:216-312: a group exists when a
    child is defined at its depth, a repeated group collects while r >= its maxR).

    rep_def[l-1] = definition level D_l of the l-th REPEATED node on the path.  For level l:
      a list starts at slot i when r_i <= l-1 and (l == 1 or d_i >= D_{l-1}): one list per row at
      level 1, one per element of the enclosing level otherwise;
      an element of level l starts at slot i when r_i <= l and d_i >= D_l;
      the list is present (possibly empty) when d >= D_l - 1 at its first slot.
    Leaf slots are the elements of the innermost level (every slot when max_rep == 0); a leaf value
    is non-null when d == max_def.
    Returns ([(offsets int32[lists+1], validity u8[lists]) per level], leaf_validity u8)."""
    d = np.asarray(def_levels, dtype=np.int32)
    r = np.asarray(rep_levels, dtype=np.int32) if rep_levels is not None else np.zeros_like(d)
    levels = []
    for l in range(1, len(rep_def) + 1):
        D = rep_def[l - 1]
        start = (r <= l - 1) & ((d >= rep_def[l - 2]) if l >= 2 else True)
        elem = (r <= l) & (d >= D)
        before = np.concatenate([[0], np.cumsum(elem)])  # elements before each slot
        idx = np.nonzero(start)[0]
        offsets = np.concatenate([before[idx], [before[-1]]]).astype(np.int32)
        validity = (d[idx] >= D - 1).astype(np.uint8)
        levels.append((offsets, validity))
    leaf = d >= rep_def[-1] if len(rep_def) else np.ones(len(d), bool)
    leaf_valid = (d[leaf] == max_def).astype(np.uint8)
    return levels, leaf_valid
