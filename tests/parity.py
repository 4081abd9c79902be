"""Chunk-level comparison of the product (C-ABI / HIP) against the CPU oracle."""
import numpy as np

from oracle import oracle as O

DELTA_BYTE_ARRAY = 7  # parquet.thrift Encoding
UNSUPPORTED_CODEC = 35  # PQH_ERR_UNSUPPORTED_CODEC (include/pqhip.h)


class Expected:
    def __init__(self):
        self.status = 0
        self.phase = 0
        self.index = 0
        self.page = -1
        self.host_error = False
        self.values = b""
        self.offsets = None
        self.data = b""
        self.def_levels = None
        self.rep_levels = None
        self.nn = 0
        self.n = 0
        self.nil = None  # uint8 per value: the reference's nil INT96 values, None when there are none
        # the chunk's codec is registered but not decoded by libpqhip (ZSTD): the product hands it back
        # at load (PQH_ERR_UNSUPPORTED_CODEC) and the shim's reference readChunk decodes it
        self.routed = False


def oracle_chunk(fr, rg, ci):
    """readChunk + readValues for every page (oracle)."""
    e = Expected()
    if fr.chunk_check(rg, ci) == 0:
        codec = fr.row_groups[rg][1][ci][3][4]
        e.routed = codec in fr.codecs and codec not in (O.UNCOMPRESSED, O.SNAPPY, O.GZIP)
    ch = fr.read_chunk(rg, ci)
    if ch.status:  # readChunk failed (walker, codec or a page's load step): exact (status, phase 0, index)
        e.status, e.phase, e.index = ch.status, O.PHASE_LOAD, ch.index
        return e
    col = ch.column
    res = O.decode_chunk(ch)
    vals, defs, reps, offs, data, nils = [], [], [], [], [], []
    base = 0
    # FIXED_LEN_BYTE_ARRAY pages with DELTA_BYTE_ARRAY yield variable-length []byte
    # (type_bytearray.go:189-240): the product lays such a chunk out as offsets + bytes throughout
    flba_var = col.physical_type == O.FIXED_LEN_BYTE_ARRAY and col.type_length > 0 and \
        any(p.encoding == DELTA_BYTE_ARRAY for p in ch.pages)
    for i, r in enumerate(res):
        if flba_var and r.offsets is None:
            L = col.type_length
            r.offsets = np.arange(len(r.values) // L + 1, dtype=np.int64) * L
        if r.status and e.status == 0:
            e.status, e.phase, e.index, e.page = r.status, r.phase, r.index, i
        e.n += r.num_values
        e.nn += r.nn
        if r.def_levels is not None:
            defs.append(r.def_levels)
        elif col.max_def > 0:
            defs.append(np.zeros(0, np.uint8))
        if r.rep_levels is not None:
            reps.append(r.rep_levels)
        if r.offsets is not None:
            offs.append(r.offsets[1:] + base)
            base += len(r.values)
            data.append(r.values)
        else:
            vals.append(r.values)
        nils.append(r.nil if r.nil is not None else np.zeros(r.nn if not r.status else 0, np.uint8))
    e.values = b"".join(vals)
    if any(r.nil is not None for r in res):
        e.nil = np.concatenate(nils)
    e.data = b"".join(data)
    if offs:
        e.offsets = np.concatenate([np.zeros(1, np.int64)] + offs)
    e.def_levels = np.concatenate(defs) if defs else None
    e.rep_levels = np.concatenate(reps) if reps else None
    return e


def assert_chunk(gpu, exp, where=""):
    """Bit-exact comparison of one decoded chunk; error status must agree."""
    if exp.routed:
        assert gpu.status == UNSUPPORTED_CODEC, f"{where}: a ZSTD chunk must come back as UNSUPPORTED_CODEC"
        return
    if exp.status:
        assert gpu.status != 0, f"{where}: oracle fails with {exp.status} but the GPU decoded the chunk"
        if not exp.host_error:
            assert (gpu.status, gpu.error_phase, gpu.error_index) == (exp.status, exp.phase, exp.index), \
                f"{where}: first error differs gpu={(gpu.status, gpu.error_phase, gpu.error_index)} " \
                f"oracle={(exp.status, exp.phase, exp.index)}"
        return
    assert gpu.status == 0, f"{where}: GPU status {gpu.status} phase {gpu.error_phase} idx {gpu.error_index}"
    assert gpu.num_non_null == exp.nn, where
    if gpu.values is not None:
        got = gpu.values.view(np.uint8).tobytes()
        assert got == exp.values, f"{where}: values differ (len {len(got)} vs {len(exp.values)})"
    else:  # byte arrays: a chunk without values still has offsets [0]
        exp_offsets = exp.offsets if exp.offsets is not None else np.zeros(1, np.int64)
        assert np.array_equal(gpu.offsets, exp_offsets), f"{where}: offsets differ"
        assert gpu.data.tobytes() == exp.data, f"{where}: byte data differs"
    got_nil = getattr(gpu, "value_nil", None)
    assert (got_nil is None) == (exp.nil is None), f"{where}: nil values {got_nil is not None} vs {exp.nil is not None}"
    if exp.nil is not None:
        assert np.array_equal(got_nil, exp.nil), f"{where}: nil value marks differ"
    if exp.def_levels is not None:
        assert np.array_equal(gpu.def_levels, exp.def_levels), f"{where}: def levels differ"
    if exp.rep_levels is not None:
        assert np.array_equal(gpu.rep_levels, exp.rep_levels), f"{where}: rep levels differ"
