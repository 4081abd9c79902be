"""ctypes declaration of the C-ABI in include/pqhip.h (libpqhip.so) and thin RAII wrappers.

Every symbol bound here is declared in include/pqhip.h; tests/test_abi.py checks the library
exports all of them.  There is no CPU fallback: constructing a Context without a HIP device
raises, and the decode always runs through the HIP kernels.
"""
import ctypes

import numpy as np

from . import _lib

i32, i64, u32, f64 = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32, ctypes.c_double
vp, cp = ctypes.c_void_p, ctypes.c_char_p

# status codes (pqh_status)
STATUS = {
    0: "OK", 1: "EOF", 2: "UNEXPECTED_EOF", 3: "VARINT_OVERFLOW", 4: "INT32_RANGE", 5: "EMPTY_BP_RUN",
    6: "EMPTY_RLE_RUN", 7: "RLE_VALUE_TOO_LARGE", 8: "READER_NOT_INITIALIZED", 9: "DICT_BIT_WIDTH",
    10: "DICT_INDEX", 11: "DELTA_BLOCK_SIZE", 12: "DELTA_MINIBLOCKS", 13: "DELTA_VALUE_COUNT",
    14: "DELTA_BIT_WIDTH", 15: "DELTA_STREAM", 16: "NEGATIVE_LENGTH", 17: "NEGATIVE_DLBA_LENGTH",
    18: "DBA_PREFIX", 19: "DBA_COUNT", 20: "INT96_SHORT", 21: "UNSUPPORTED", 22: "PAGE_HEADER",
    23: "DECOMPRESS", 24: "CRC", 25: "THRIFT", 26: "IO", 27: "ARG", 28: "HIP", 29: "NOMEM", 30: "SCHEMA",
    31: "DICT_PAGE", 32: "NO_DEVICE", 33: "NOT_IMPLEMENTED", 34: "INTERNAL", 35: "UNSUPPORTED_CODEC",
}
OK = 0
NOT_IMPLEMENTED = 33
INTERNAL = 34
UNSUPPORTED_CODEC = 35  # the chunk's codec is not decoded here: the caller routes it to the reference
# error phases (pqh_phase): page load (readChunk), repetition levels, definition levels, values
PHASE_LOAD, PHASE_REP, PHASE_DEF, PHASE_VALUES = range(4)
CTX_PROFILE = 1
CTX_STREAMING = 2  # one slot of a streaming ring (reader.RowGroupStream)
PAYLOAD_PAD = 256
MAX_NEST = 32  # include/pqhip.h PQH_MAX_NEST


class Column(ctypes.Structure):
    _fields_ = [("physical_type", i32), ("type_length", i32), ("max_def", i32), ("max_rep", i32),
                ("rep_def", i32 * MAX_NEST)]


class Page(ctypes.Structure):
    _fields_ = [("image_offset", i64), ("image_len", i32), ("page_type", i32), ("num_values", i32),
                ("encoding", i32), ("def_levels_byte_length", i32), ("rep_levels_byte_length", i32),
                ("chunk", i32), ("num_nulls", i32)]


class Chunk(ctypes.Structure):
    _fields_ = [("column", Column), ("first_page", i32), ("num_pages", i32), ("host_status", i32),
                ("reserved", i32)]


class ChunkOut(ctypes.Structure):
    _fields_ = [("num_values", i64), ("num_non_null", i64), ("value_size", i32), ("status", i32),
                ("error_page", i32), ("error_phase", i32), ("error_index", i64), ("values", vp),
                ("offsets", vp), ("bytes", vp), ("num_bytes", i64), ("def_levels", vp), ("rep_levels", vp),
                ("value_nil", vp), ("num_nil", i64)]


class NestLevel(ctypes.Structure):
    _fields_ = [("def_level", i32), ("reserved", i32), ("num_lists", i64), ("offsets", vp), ("validity", vp)]


class NestOut(ctypes.Structure):
    _fields_ = [("num_levels", i32), ("status", i32), ("num_leaf_slots", i64), ("leaf_validity", vp),
                ("levels", NestLevel * MAX_NEST)]


class PageResult(ctypes.Structure):
    _fields_ = [("status", i32), ("phase", i32), ("index", i64), ("num_non_null", i32), ("num_nil", i32),
                ("value_offset", i64), ("level_offset", i64)]


class CodecPage(ctypes.Structure):
    _fields_ = [("src_offset", i64), ("image_offset", i64), ("src_len", i32), ("image_len", i32),
                ("raw_len", i32), ("codec", i32), ("chunk", i32), ("reserved", i32)]


LOAD_DEVICE_SNAPPY = 1
LOAD_DEVICE_GZIP = 2


class SchemaElement(ctypes.Structure):
    _fields_ = [("physical_type", i32), ("type_length", i32), ("repetition", i32), ("num_children", i32),
                ("column", i32), ("max_def", i32), ("max_rep", i32), ("reserved", i32)]


class PageValues(ctypes.Structure):
    _fields_ = [("status", i32), ("phase", i32), ("index", i64), ("num_slots", i64), ("num_non_null", i64),
                ("values_read", i64), ("num_bytes", i64), ("value_size", i32), ("num_nil", i32)]


class KernelStat(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 32), ("launches", i32), ("work_items", i32), ("total_ms", f64),
                ("bytes_read", f64), ("bytes_written", f64)]


class BatchPaths(ctypes.Structure):
    _fields_ = [("flat_active", i32), ("flat_fallbacks", i32), ("ba_fuse_active", i32), ("ba_fuse_fallbacks", i32),
                ("regrows", i32), ("graph_replay", i32), ("reserved", i32 * 2)]


# (name, restype, argtypes) for every function of include/pqhip.h
ABI_VERSION = 8  # include/pqhip.h PQH_ABI_VERSION

PROTOTYPES = [
    ("pqh_abi_version", ctypes.c_int, []),
    ("pqh_build_id", cp, []),
    ("pqh_device_count", ctypes.c_int, [ctypes.POINTER(i32)]),
    ("pqh_ctx_create", ctypes.c_int, [i32, u32, ctypes.POINTER(vp)]),
    ("pqh_ctx_destroy", None, [vp]),
    ("pqh_ctx_set_flags", ctypes.c_int, [vp, u32]),
    ("pqh_last_error", cp, [vp]),
    ("pqh_ctx_stream", vp, [vp]),
    ("pqh_ctx_pinned_bytes", i64, [vp]),
    ("pqh_malloc", ctypes.c_int, [vp, ctypes.POINTER(vp), ctypes.c_size_t]),
    ("pqh_free", ctypes.c_int, [vp, vp]),
    ("pqh_host_alloc", ctypes.c_int, [vp, ctypes.POINTER(vp), ctypes.c_size_t]),
    ("pqh_host_free", ctypes.c_int, [vp, vp]),
    ("pqh_memcpy_h2d", ctypes.c_int, [vp, vp, vp, ctypes.c_size_t]),
    ("pqh_memcpy_d2h", ctypes.c_int, [vp, vp, vp, ctypes.c_size_t]),
    ("pqh_memcpy_h2d_pinned_async", ctypes.c_int, [vp, vp, vp, ctypes.c_size_t]),
    ("pqh_sync", ctypes.c_int, [vp]),
    ("pqh_batch_create", ctypes.c_int, [vp, ctypes.POINTER(Chunk), i32, ctypes.POINTER(Page), i32, vp, i64,
                                        ctypes.POINTER(vp)]),
    ("pqh_batch_run", ctypes.c_int, [vp]),
    ("pqh_batch_sync", ctypes.c_int, [vp]),
    ("pqh_batch_chunk_out", ctypes.c_int, [vp, i32, ctypes.POINTER(ChunkOut)]),
    ("pqh_batch_nesting", ctypes.c_int, [vp, i32, ctypes.POINTER(NestOut)]),
    ("pqh_batch_page_results", ctypes.c_int, [vp, ctypes.POINTER(PageResult), i32]),
    ("pqh_batch_page_read", ctypes.c_int, [vp, i32, i64, i64, vp, i64, vp, i64, vp, i64, vp, vp, vp, i64,
                                           ctypes.POINTER(PageValues)]),
    ("pqh_batch_kernel_stats", ctypes.c_int, [vp, ctypes.POINTER(KernelStat), i32, ctypes.POINTER(i32)]),
    ("pqh_batch_path_info", ctypes.c_int, [vp, ctypes.POINTER(BatchPaths)]),
    ("pqh_batch_reset_stats", ctypes.c_int, [vp]),
    ("pqh_batch_traffic", ctypes.c_int, [vp, ctypes.POINTER(f64), ctypes.POINTER(f64)]),
    ("pqh_batch_destroy", None, [vp]),
    ("pqh_file_open", ctypes.c_int, [cp, ctypes.POINTER(vp)]),
    ("pqh_file_open_memory", ctypes.c_int, [vp, i64, ctypes.POINTER(vp)]),
    ("pqh_file_close", None, [vp]),
    ("pqh_file_error", cp, [vp]),
    ("pqh_file_num_row_groups", i32, [vp]),
    ("pqh_file_num_rows", i64, [vp]),
    ("pqh_file_row_group_num_rows", i64, [vp, i32]),
    ("pqh_file_num_columns", i32, [vp]),
    ("pqh_file_column", ctypes.c_int, [vp, i32, ctypes.POINTER(Column), ctypes.c_char_p, i32]),
    ("pqh_file_chunk_check", ctypes.c_int, [vp, i32, i32, i32]),
    ("pqh_file_set_codecs", ctypes.c_int, [vp, ctypes.POINTER(i32), i32]),
    ("pqh_file_column_path", i32, [vp, i32, ctypes.c_char_p, i32]),
    ("pqh_file_schema_name", i32, [vp, i32, ctypes.c_char_p, i32]),
    ("pqh_file_num_schema_elements", i32, [vp]),
    ("pqh_file_schema_element", ctypes.c_int, [vp, i32, ctypes.POINTER(SchemaElement), ctypes.c_char_p, i32]),
    ("pqh_file_load", ctypes.c_int, [vp, i32, i32, ctypes.POINTER(i32), i32, i32, ctypes.POINTER(vp)]),
    ("pqh_file_load_ex", ctypes.c_int, [vp, i32, i32, ctypes.POINTER(i32), i32, i32, ctypes.c_uint32,
                                        ctypes.POINTER(vp)]),
    ("pqh_file_load_pinned", ctypes.c_int, [vp, vp, i32, i32, ctypes.POINTER(i32), i32, i32, ctypes.c_uint32,
                                            ctypes.POINTER(vp)]),
    ("pqh_host_batch_num_codec_pages", i32, [vp]),
    ("pqh_host_batch_codec_pages", ctypes.POINTER(CodecPage), [vp]),
    ("pqh_host_batch_image_bytes", i64, [vp]),
    ("pqh_decompress_pages", ctypes.c_int, [vp, ctypes.POINTER(CodecPage), i32, vp, vp, ctypes.POINTER(i32)]),
    ("pqh_hybrid_decode", ctypes.c_int, [vp, vp, i64, i32, i64, i32, vp, ctypes.POINTER(i32), ctypes.POINTER(i64)]),
    ("pqh_host_batch_num_chunks", i32, [vp]),
    ("pqh_host_batch_num_pages", i32, [vp]),
    ("pqh_host_batch_chunks", ctypes.POINTER(Chunk), [vp]),
    ("pqh_host_batch_pages", ctypes.POINTER(Page), [vp]),
    ("pqh_host_batch_payload", ctypes.POINTER(ctypes.c_uint8), [vp]),
    ("pqh_host_batch_payload_bytes", i64, [vp]),
    ("pqh_host_batch_decompress_seconds", f64, [vp]),
    ("pqh_host_batch_free", None, [vp]),
    ("pqh_batch_create_from_host", ctypes.c_int, [vp, vp, ctypes.POINTER(vp)]),
    ("pqh_batch_create_staged", ctypes.c_int, [vp, vp, ctypes.POINTER(vp)]),
    ("pqh_batch_run_staged", ctypes.c_int, [vp]),
]


def bind(L):
    if L.pqh_abi_version() != ABI_VERSION:
        raise RuntimeError(f"libpqhip ABI {L.pqh_abi_version()} != {ABI_VERSION}: rebuild (python parquet-go_amd/build.py)")
    for name, res, args in PROTOTYPES:
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    return L


class PqhError(RuntimeError):
    def __init__(self, status, msg=""):
        self.status = status
        super().__init__(f"{STATUS.get(status, status)}: {msg}")


def _check(rc, msg=""):
    if rc != OK:
        raise PqhError(rc, msg)


def build_info():
    """{"source_hash", "git_head"} of the loaded libpqhip: the hash compiled into it (pqh_build_id)
    and the commit build.py recorded beside it (lib/*.buildinfo.json; None when it does not match)."""
    import json
    import os

    h = (_lib.hip().pqh_build_id() or b"").decode()
    info = {"source_hash": h, "git_head": None}
    try:
        with open(_lib.hip_path() + ".buildinfo.json") as fh:
            bi = json.load(fh)
        if bi.get("source_hash") == h:
            info["git_head"] = bi.get("git_head")
            if bi.get("hipflags"):
                info["hipflags"] = bi["hipflags"]
    except (OSError, ValueError):
        pass
    return info


def device_count():
    n = i32()
    _lib.hip().pqh_device_count(ctypes.byref(n))
    return n.value


class Context:
    """One HIP device + stream (pqh_ctx)."""

    def __init__(self, device=0, profile=False, streaming=False):
        L = _lib.hip()
        self.L = L
        h = vp()
        rc = L.pqh_ctx_create(device, (CTX_PROFILE if profile else 0) | (CTX_STREAMING if streaming else 0),
                              ctypes.byref(h))
        if rc != OK:
            raise PqhError(rc, (L.pqh_last_error(None) or b"").decode())
        self.h = h
        self.device = device

    def error(self):
        return (self.L.pqh_last_error(self.h) or b"").decode()

    def check(self, rc):
        _check(rc, self.error())

    def sync(self):
        self.check(self.L.pqh_sync(self.h))

    def pinned_bytes(self):
        """Pinned host bytes the context's payload pool holds (in use + kept for reuse)."""
        return int(self.L.pqh_ctx_pinned_bytes(self.h))

    def set_profile(self, on):
        """Per-kernel HIP-event timing on (direct launches) or off (graph replay)."""
        self.check(self.L.pqh_ctx_set_flags(self.h, CTX_PROFILE if on else 0))

    def malloc(self, n):
        p = vp()
        self.check(self.L.pqh_malloc(self.h, ctypes.byref(p), n))
        return p.value

    def free(self, p):
        if p:
            self.L.pqh_free(self.h, p)

    def h2d(self, dst, src_ptr, n):
        """Synchronous copy from pageable (or pinned) host memory."""
        self.check(self.L.pqh_memcpy_h2d(self.h, dst, src_ptr, n))

    def h2d_pinned_async(self, dst, pinned_ptr, n):
        """Asynchronous copy on the context stream from pqh_host_alloc memory."""
        self.check(self.L.pqh_memcpy_h2d_pinned_async(self.h, dst, pinned_ptr, n))

    def decompress_pages(self, pages, d_src, d_dst):
        """The device codecs on their own (k_snappy, k_gzip): rebuild `pages` (CodecPage list) from
        d_src into d_dst; statuses."""
        arr = (CodecPage * max(1, len(pages)))(*pages)
        st = (i32 * max(1, len(pages)))()
        self.check(self.L.pqh_decompress_pages(self.h, arr, len(pages), d_src, d_dst, st))
        return [st[i] for i in range(len(pages))]

    def hybrid_decode(self, stream, width, n, group=8):
        """The device's hybrid (RLE / bit-packing) decoder on one stream (host bytes): (status,
        values decoded before the first error, uint32 values) (pqh_hybrid_decode)."""
        arr = np.frombuffer(bytes(stream) + b"\0" * PAYLOAD_PAD, dtype=np.uint8).copy()
        d = self.malloc(len(arr))
        o = self.malloc(max(4 * n, 16))
        try:
            self.h2d(d, arr.ctypes.data, len(arr))
            st, nv = i32(), i64()
            self.check(self.L.pqh_hybrid_decode(self.h, d, len(stream), width, n, group, o, ctypes.byref(st),
                                                ctypes.byref(nv)))
            return st.value, nv.value, self.d2h_array(o, nv.value, np.uint32)
        finally:
            self.free(o)
            self.free(d)

    def d2h_array(self, src, n, dtype=np.uint8):
        out = np.empty(n, dtype=dtype)
        nbytes = out.nbytes
        if nbytes:
            self.check(self.L.pqh_memcpy_d2h(self.h, out.ctypes.data, src, nbytes))
            self.sync()
        return out

    def close(self):
        if self.h:
            self.L.pqh_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HostBatch:
    """Result of the host page walker (pqh_file_load)."""

    def __init__(self, L, h):
        self.L = L
        self.h = h

    @property
    def num_chunks(self):
        return self.L.pqh_host_batch_num_chunks(self.h)

    @property
    def num_pages(self):
        return self.L.pqh_host_batch_num_pages(self.h)

    def chunks(self):
        p = self.L.pqh_host_batch_chunks(self.h)
        return [p[i] for i in range(self.num_chunks)]

    def pages(self):
        p = self.L.pqh_host_batch_pages(self.h)
        return [p[i] for i in range(self.num_pages)]

    def codec_pages(self):
        n = self.L.pqh_host_batch_num_codec_pages(self.h)
        p = self.L.pqh_host_batch_codec_pages(self.h)
        return [p[i] for i in range(n)]

    @property
    def image_bytes(self):
        """Device codecs: bytes of the page images the source payload decompresses to (else 0)."""
        return self.L.pqh_host_batch_image_bytes(self.h)

    def payload(self):
        n = self.L.pqh_host_batch_payload_bytes(self.h)
        return np.ctypeslib.as_array(self.L.pqh_host_batch_payload(self.h), shape=(n + PAYLOAD_PAD,))

    @property
    def payload_bytes(self):
        return self.L.pqh_host_batch_payload_bytes(self.h)

    @property
    def decompress_seconds(self):
        return self.L.pqh_host_batch_decompress_seconds(self.h)

    def close(self):
        if self.h:
            self.L.pqh_host_batch_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class File:
    """Footer + page walker (pqh_file_*): no GPU needed."""

    def __init__(self, source):
        L = _lib.hip()
        self.L = L
        h = vp()
        if isinstance(source, np.ndarray):
            self._buf = np.ascontiguousarray(source, dtype=np.uint8)
            rc = L.pqh_file_open_memory(self._buf.ctypes.data, len(self._buf), ctypes.byref(h))
        elif isinstance(source, (bytes, bytearray, memoryview)):
            self._buf = np.frombuffer(bytes(source), dtype=np.uint8)
            rc = L.pqh_file_open_memory(self._buf.ctypes.data, len(self._buf), ctypes.byref(h))
        else:
            rc = L.pqh_file_open(str(source).encode(), ctypes.byref(h))
        self.h = h
        if rc != OK:
            msg = (L.pqh_file_error(h) or b"").decode() if h else ""
            self.close()
            raise PqhError(rc, msg)

    @property
    def num_row_groups(self):
        return self.L.pqh_file_num_row_groups(self.h)

    @property
    def num_rows(self):
        return self.L.pqh_file_num_rows(self.h)

    def row_group_num_rows(self, rg):
        return self.L.pqh_file_row_group_num_rows(self.h, rg)

    def columns(self):
        out = []
        for i in range(self.L.pqh_file_num_columns(self.h)):
            c = Column()
            _check(self.L.pqh_file_column(self.h, i, ctypes.byref(c), None, 0))
            out.append((self._text(self.L.pqh_file_column_path, i), c.physical_type, c.type_length, c.max_def,
                        c.max_rep))
        return out

    def rep_def(self, i):
        """pqh_column.rep_def of column i: the definition level of each REPEATED node on its path."""
        c = Column()
        _check(self.L.pqh_file_column(self.h, i, ctypes.byref(c), None, 0))
        return tuple(c.rep_def[k] for k in range(min(c.max_rep, MAX_NEST)))

    def schema(self):
        """[(name, SchemaElement)] in DFS order, root first."""
        out = []
        for i in range(self.L.pqh_file_num_schema_elements(self.h)):
            e = SchemaElement()
            _check(self.L.pqh_file_schema_element(self.h, i, ctypes.byref(e), None, 0))
            out.append((self._text(self.L.pqh_file_schema_name, i), e))
        return out

    def _text(self, fn, i):
        """A path / name of any bytes (Go strings), as str with undecodable bytes escaped."""
        n = fn(self.h, i, None, 0)
        buf = ctypes.create_string_buffer(max(n, 1))
        fn(self.h, i, buf, n)
        return buf.raw[:n].decode("utf-8", "surrogateescape")

    def set_codecs(self, codecs):
        """The caller's codec registry (pqh_file_set_codecs; default UNCOMPRESSED / GZIP / SNAPPY /
        ZSTD, compress.go:182-187): registered codecs this library does not decode fail their chunks
        with UNSUPPORTED_CODEC at load, unregistered ones as the reference fails them."""
        arr = (i32 * max(len(codecs), 1))(*codecs)
        _check(self.L.pqh_file_set_codecs(self.h, arr, len(codecs)))

    def chunk_check(self, rg, column, selected=True):
        """readRowGroupData's checks of a column before its pages (pqh_file_chunk_check): a status."""
        return self.L.pqh_file_chunk_check(self.h, rg, column, int(selected))

    def load(self, rg_begin, rg_end, columns, validate_crc=False, device_snappy=False, ctx=None,
             device_gzip=False):
        """Walk the pages of `columns` in row groups [rg_begin, rg_end).  device_snappy /
        device_gzip: SNAPPY / GZIP pages stay compressed (the batch decompresses them on the
        device, k_snappy / k_gzip).  ctx: the
        payload is written into pinned memory from the context's pool (pqh_file_load_pinned), which
        Batch.staged adopts without a copy."""
        cols = (i32 * len(columns))(*columns)
        h = vp()
        flags = (LOAD_DEVICE_SNAPPY if device_snappy else 0) | (LOAD_DEVICE_GZIP if device_gzip else 0)
        if ctx is not None:
            rc = self.L.pqh_file_load_pinned(ctx.h, self.h, rg_begin, rg_end, cols, len(columns), int(validate_crc),
                                             flags, ctypes.byref(h))
        else:
            rc = self.L.pqh_file_load_ex(self.h, rg_begin, rg_end, cols, len(columns), int(validate_crc), flags,
                                         ctypes.byref(h))
        if rc != OK:
            raise PqhError(rc, (self.L.pqh_file_error(self.h) or b"").decode())
        return HostBatch(self.L, h)

    def close(self):
        if getattr(self, "h", None):
            self.L.pqh_file_close(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Batch:
    """A planned device decode of a set of chunks (pqh_batch)."""

    def __init__(self, ctx, h, owned=None):
        self.ctx = ctx
        self.L = ctx.L
        self.h = h
        self._owned = owned  # device payload owned by the caller wrapper

    @classmethod
    def from_host(cls, ctx, hb):
        h = vp()
        ctx.check(ctx.L.pqh_batch_create_from_host(ctx.h, hb.h, ctypes.byref(h)))
        return cls(ctx, h)

    @classmethod
    def staged(cls, ctx, hb):
        """End-to-end batch: pinned host copy of hb's page images, copied to HBM on every run_staged
        (copy stream) ahead of the decode (compute stream)."""
        h = vp()
        ctx.check(ctx.L.pqh_batch_create_staged(ctx.h, hb.h, ctypes.byref(h)))
        return cls(ctx, h)

    @classmethod
    def from_tables(cls, ctx, chunks, pages, d_payload, payload_bytes):
        ch = (Chunk * len(chunks))(*chunks)
        pg = (Page * len(pages))(*pages)
        h = vp()
        ctx.check(ctx.L.pqh_batch_create(ctx.h, ch, len(chunks), pg, len(pages), d_payload, payload_bytes,
                                         ctypes.byref(h)))
        return cls(ctx, h)

    def run(self):
        self.ctx.check(self.L.pqh_batch_run(self.h))

    def run_staged(self):
        self.ctx.check(self.L.pqh_batch_run_staged(self.h))

    def sync(self):
        self.ctx.check(self.L.pqh_batch_sync(self.h))

    def chunk_out(self, i):
        o = ChunkOut()
        self.ctx.check(self.L.pqh_batch_chunk_out(self.h, i, ctypes.byref(o)))
        return o

    def nesting(self, i):
        o = NestOut()
        self.ctx.check(self.L.pqh_batch_nesting(self.h, i, ctypes.byref(o)))
        return o

    def page_results(self, n):
        arr = (PageResult * max(n, 1))()
        self.ctx.check(self.L.pqh_batch_page_results(self.h, arr, n))
        return [arr[i] for i in range(n)]

    def page_read(self, page, first=0, count=None, nil=None):
        """readValues(count) of one page from level slot `first` (the compat path of the cgo shim):
        (PageValues, values or (offsets, data), def levels or None, rep levels or None) as host
        numpy arrays; values are None when the call fails.  nil: a list that receives the returned
        values' nil mask (uint8 per value, 1 = the reference's nil INT96 value) when pv.num_nil."""
        if count is None:
            count = 1 << 62
        pv = PageValues()
        self.ctx.check(self.L.pqh_batch_page_read(self.h, page, first, count, None, 0, None, 0, None, 0, None, None,
                                                  None, 0, ctypes.byref(pv)))
        ns = pv.num_slots
        d = np.empty(ns, np.uint8)
        r = np.empty(ns, np.uint8)
        vals = offs = data = None
        if pv.status == OK:
            if pv.value_size > 0:
                vals = np.empty(pv.num_non_null * pv.value_size, np.uint8)
            else:
                offs = np.empty(pv.num_non_null + 1, np.int64)
                data = np.empty(max(pv.num_bytes, 1), np.uint8)
        m = np.zeros(max(pv.num_non_null, 1), np.uint8) if pv.status == OK else None
        p = lambda a: a.ctypes.data if a is not None else None  # noqa: E731
        self.ctx.check(self.L.pqh_batch_page_read(
            self.h, page, first, count, p(vals), 0 if vals is None else vals.nbytes, p(offs),
            0 if offs is None else len(offs), p(data), 0 if data is None else data.nbytes, p(d), p(r), p(m),
            0 if m is None else len(m), ctypes.byref(pv)))
        if data is not None:
            data = data[:pv.num_bytes]
        if nil is not None and m is not None:
            nil.append(m[:pv.num_non_null])
        return pv, (vals if pv.value_size > 0 else (offs, data)), d, r

    def kernel_stats(self):
        arr = (KernelStat * 64)()
        n = i32()
        self.ctx.check(self.L.pqh_batch_kernel_stats(self.h, arr, 64, ctypes.byref(n)))
        return [arr[i] for i in range(n.value)]

    def paths(self):
        """{flat_active, flat_fallbacks, ba_fuse_active, ba_fuse_fallbacks, regrows, graph_replay}:
        the decode paths the batch takes now and the fallbacks pqh_batch_sync made."""
        p = BatchPaths()
        self.ctx.check(self.L.pqh_batch_path_info(self.h, ctypes.byref(p)))
        return {k: getattr(p, k) for k, _ in BatchPaths._fields_ if k != "reserved"}

    def reset_stats(self):
        self.L.pqh_batch_reset_stats(self.h)

    def traffic(self):
        r, w = f64(), f64()
        self.ctx.check(self.L.pqh_batch_traffic(self.h, ctypes.byref(r), ctypes.byref(w)))
        return r.value, w.value

    def close(self):
        if self.h:
            self.L.pqh_batch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
