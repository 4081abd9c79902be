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

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liborcl.so")

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
                ("num_bytes", ctypes.c_int64)]


class OrcOut(ctypes.Structure):
    _fields_ = [("status", ctypes.c_int32), ("phase", ctypes.c_int32), ("index", ctypes.c_int64),
                ("num_values", ctypes.c_int32), ("nn", ctypes.c_int32),
                ("def_", ctypes.POINTER(ctypes.c_uint8)), ("rep", ctypes.POINTER(ctypes.c_uint8)),
                ("value_size", ctypes.c_int32), ("values", ctypes.POINTER(ctypes.c_uint8)),
                ("values_bytes", ctypes.c_int64), ("offsets", ctypes.POINTER(ctypes.c_int64))]


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
        L.orc_dict_free.argtypes = [ctypes.POINTER(OrcDict)]
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
    def __init__(self, status, num_values=0, value_size=0, values=b"", offsets=None):
        self.status = status
        self.num_values = num_values
        self.value_size = value_size
        self.values = values
        self.offsets = offsets


def decode_dict_page(col, num_values, encoding, image):
    arr, p = _u8(image)
    c = OrcColumn(*col)
    d = OrcDict()
    st = lib().orc_decode_dict_page(ctypes.byref(c), num_values, encoding, p, len(arr), ctypes.byref(d))
    if st:
        return Dictionary(st)
    vals = ctypes.string_at(d.values, d.num_bytes) if d.num_bytes else b""
    offs = None
    if d.value_size == 0:
        offs = np.ctypeslib.as_array(d.offsets, shape=(d.num_values + 1,)).copy()
    res = Dictionary(OK, d.num_values, d.value_size, vals, offs)
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
    if d.offsets is not None:
        oa = np.ascontiguousarray(d.offsets, dtype=np.int64)
        keep.append(oa)
        cd.offsets = oa.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))
    return cd, keep


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
    if o.offsets:
        r.offsets = np.ctypeslib.as_array(o.offsets, shape=(o.nn + 1,)).copy()
    lib().orc_out_free(ctypes.byref(o))
    return r


# ------------------------------------------------------------------------------------------------
# Thrift compact protocol (generic reader: struct -> {field id: value})
# ------------------------------------------------------------------------------------------------
class ThriftError(Exception):
    pass


class CompactReader:
    def __init__(self, buf, pos=0):
        self.buf = buf
        self.pos = pos

    def byte(self):
        if self.pos >= len(self.buf):
            raise ThriftError("EOF")
        b = self.buf[self.pos]
        self.pos += 1
        return b

    def uvarint(self):
        x = 0
        s = 0
        while True:
            b = self.byte()
            x |= (b & 0x7F) << s
            if b < 0x80:
                return x
            s += 7
            if s > 63:
                raise ThriftError("varint overflow")

    def zigzag(self):
        u = self.uvarint()
        return (u >> 1) ^ -(u & 1)

    def binary(self):
        n = self.uvarint()
        if self.pos + n > len(self.buf):
            raise ThriftError("EOF in binary")
        v = bytes(self.buf[self.pos:self.pos + n])
        self.pos += n
        return v

    def value(self, t):
        if t in (1, 2):
            return t == 1
        if t == 3:
            b = self.byte()
            return b - 256 if b > 127 else b
        if t in (4, 5, 6):
            return self.zigzag()
        if t == 7:
            if self.pos + 8 > len(self.buf):
                raise ThriftError("EOF in double")
            v = struct.unpack_from("<d", self.buf, self.pos)[0]
            self.pos += 8
            return v
        if t == 8:
            return self.binary()
        if t in (9, 10):
            h = self.byte()
            n = h >> 4
            et = h & 0x0F
            if n == 15:
                n = self.uvarint()
            out = []
            for _ in range(n):
                if et in (1, 2):
                    out.append(self.byte() == 1)
                else:
                    out.append(self.value(et))
            return out
        if t == 11:
            n = self.uvarint()
            if n == 0:
                return {}
            kv = self.byte()
            return {self.value(kv >> 4): self.value(kv & 0x0F) for _ in range(n)}
        if t == 12:
            return self.struct()
        raise ThriftError(f"bad type {t}")

    def struct(self):
        out = {}
        last = 0
        while True:
            h = self.byte()
            if h == 0:
                return out
            t = h & 0x0F
            d = h >> 4
            fid = last + d if d else self.zigzag()
            last = fid
            out[fid] = self.value(t)


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


def read_schema(schema):
    """readSchema / readGroupSchema / readColumnSchema (schema.go:893-1015): leaves in DFS order."""
    leaves = []

    def walk(idx, path, d, r, rd, is_root):
        s = schema[idx]
        rep = s.get(3)
        if not is_root and rep is not None and rep != 0:
            d += 1
        if not is_root and rep == 2:
            r += 1
            rd = rd + [d]
        name = s.get(4, b"").decode()
        p = path + ([name] if not is_root else [])
        if s.get(1) is not None and not is_root:
            leaves.append(Column(".".join(p), s, d, r, rd))
            return idx + 1
        idx += 1
        for _ in range(s.get(5, 0)):
            idx = walk(idx, p, d, r, rd, False)
        return idx

    walk(0, [], 0, 0, [], True)
    return leaves


def decompress(codec, data, uncompressed_size):
    if codec == UNCOMPRESSED:
        return bytes(data)
    if codec == GZIP:
        return gzip.decompress(bytes(data))
    import pyarrow as pa

    name = {SNAPPY: "snappy", ZSTD: "zstd"}.get(codec)
    if name is None:
        raise ValueError(f"codec {codec} not supported")
    return pa.decompress(bytes(data), decompressed_size=uncompressed_size, codec=name, asbytes=True)


class SnappyCorrupt(Exception):
    pass


def snappy_decode(src):
    """github.com/golang/snappy v0.0.4 Decode (decode.go: decodedLen + decode), restated: the
    reference's SNAPPY codec (compress.go:43-49).  Returns the block or raises SnappyCorrupt
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
        self.pages = []   # data pages (Page)
        self.dict_page = None
        self.status = OK


class FileReader:
    """The oracle's NewFileReader: footer + schema + page walker over a bytes object."""

    def __init__(self, data):
        self.data = data.tobytes() if hasattr(data, "tobytes") else bytes(data)
        if len(self.data) < 12 or self.data[:4] != b"PAR1" or self.data[-4:] != b"PAR1":
            raise ValueError("not a parquet file")
        flen = struct.unpack_from("<I", self.data, len(self.data) - 8)[0]
        meta = CompactReader(self.data, len(self.data) - 8 - flen).struct()
        self.meta = meta
        self.columns = read_schema(meta[2])
        self.row_groups = meta.get(4, [])
        self.num_rows = meta.get(3, 0)

    def row_group_num_rows(self, rg):
        return self.row_groups[rg].get(3, 0)

    def read_chunk(self, rg, ci, validate_crc=False):
        """readChunk + readPages (chunk_reader.go:182-362); decompressed page images."""
        col = self.columns[ci]
        ch = Chunk(col)
        cc = self.row_groups[rg][1][ci]
        md = cc.get(3)
        if md is None or md.get(1) != col.physical_type:
            ch.status = ERR_SCHEMA
            return ch
        offset = md.get(11, md.get(9))
        total = md.get(7)
        codec = md.get(4, 0)
        pos = offset
        count = 0
        while total - count > 0:
            try:
                rd = CompactReader(self.data, pos)
                ph = rd.struct()
            except ThriftError:
                ch.status = ERR_THRIFT
                return ch
            count += rd.pos - pos
            pos = rd.pos
            ptype = ph.get(1)
            usize, csize = ph.get(2, 0), ph.get(3, 0)
            if csize < 0 or usize < 0:
                ch.status = ERR_PAGE_HEADER
                return ch
            block = self.data[pos:pos + csize]
            pos += len(block)
            count += len(block)
            if validate_crc and 4 in ph and (zlib.crc32(block) & 0xFFFFFFFF) != (ph[4] & 0xFFFFFFFF):
                ch.status = ERR_CRC
                return ch
            if ptype == DICTIONARY_PAGE:
                if ch.dict_page is not None:
                    ch.status = ERR_DICT_PAGE
                    return ch
                dh = ph.get(7)
                if dh is None:
                    ch.status = ERR_PAGE_HEADER
                    return ch
                try:
                    img = decompress(codec, block, usize)
                except Exception:
                    ch.status = ERR_DECOMPRESS
                    return ch
                if len(block) != csize or len(img) != usize:
                    ch.status = ERR_DECOMPRESS
                    return ch
                d = decode_dict_page(col.desc(), dh.get(1, 0), dh.get(2, 0), img)
                if d.status != OK:
                    ch.status = d.status
                    return ch
                ch.dict_page = d
                if 11 in md and md[11] != pos:
                    count += md[9] - pos
                    pos = md[9]
                continue
            if ptype == DATA_PAGE:
                h = ph.get(5)
                if h is None:
                    ch.status = ERR_PAGE_HEADER
                    return ch
                try:
                    img = decompress(codec, block, usize)
                except Exception:
                    ch.status = ERR_DECOMPRESS
                    return ch
                if len(block) != csize or len(img) != usize:
                    ch.status = ERR_DECOMPRESS
                    return ch
                ch.pages.append(Page(DATA_PAGE, h.get(1, 0), h.get(2, 0), 0, 0, img))
            elif ptype == DATA_PAGE_V2:
                h = ph.get(8)
                if h is None:
                    ch.status = ERR_PAGE_HEADER
                    return ch
                dl, rl = h.get(5, 0), h.get(6, 0)
                if dl < 0 or rl < 0 or h.get(1, 0) < 0 or dl + rl > len(block):
                    ch.status = ERR_PAGE_HEADER
                    return ch
                lv = block[: rl + dl]
                try:
                    vals = decompress(codec, block[rl + dl:], usize - rl - dl)
                except Exception:
                    ch.status = ERR_DECOMPRESS
                    return ch
                if len(vals) != usize - rl - dl:
                    ch.status = ERR_DECOMPRESS
                    return ch
                ch.pages.append(Page(DATA_PAGE_V2, h.get(1, 0), h.get(4, 0), dl, rl, lv + vals))
            else:
                ch.status = ERR_PAGE_HEADER
                return ch
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
