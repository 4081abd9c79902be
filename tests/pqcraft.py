"""A minimal Parquet file builder for crafted page blocks (test infrastructure): one REQUIRED INT32
column "v", one row group per chunk, V1 data pages whose compressed blocks are given verbatim.
Thrift compact protocol written by hand (the structures of parquet.thrift the reference reads in
file_meta.go / chunk_reader.go: PageHeader, FileMetaData, RowGroup, ColumnChunk,
ColumnMetaData)."""
import struct

I32, I64, BINARY, LIST, STRUCT = 5, 6, 8, 9, 12


def _uvarint(x):
    out = bytearray()
    while True:
        b = x & 0x7F
        x >>= 7
        if x:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _zz(x):
    return (x << 1) ^ (x >> 63)


def _value(t, v):
    if t in (I32, I64):
        return _uvarint(_zz(v) & ((1 << 64) - 1))
    if t == BINARY:
        return _uvarint(len(v)) + v
    if t == STRUCT:
        return struct_(v)
    if t == LIST:
        et, items = v
        h = bytes([(len(items) << 4) | et]) if len(items) < 15 else bytes([0xF0 | et]) + _uvarint(len(items))
        return h + b"".join(_value(et, x) for x in items)
    raise ValueError(t)


def struct_(fields):
    """fields: [(id, type, value)] in increasing id order."""
    out, last = bytearray(), 0
    for fid, t, v in fields:
        d = fid - last
        out += bytes([(d << 4) | t]) if 0 < d <= 15 else bytes([t]) + _uvarint(_zz(fid))
        out += _value(t, v)
        last = fid
    out.append(0)
    return bytes(out)


def page_header(csize, usize, num_values):
    dph = [(1, I32, num_values), (2, I32, 0), (3, I32, 3), (4, I32, 3)]
    return struct_([(1, I32, 0), (2, I32, usize), (3, I32, csize), (5, STRUCT, dph)])


def file_with_blocks(chunks, codec):
    """chunks: [[(block bytes, uncompressed size, num_values), ...] per row group]."""
    out = bytearray(b"PAR1")
    rgs = []
    for pages in chunks:
        start = len(out)
        tot_c = tot_u = nv = 0
        for blk, usize, n in pages:
            h = page_header(len(blk), usize, n)
            out += h + blk
            tot_c += len(h) + len(blk)
            tot_u += len(h) + usize
            nv += n
        md = [(1, I32, 1), (2, LIST, (I32, [0])), (3, LIST, (BINARY, [b"v"])), (4, I32, codec), (5, I64, nv),
              (6, I64, tot_u), (7, I64, tot_c), (9, I64, start)]
        cc = [(2, I64, start), (3, STRUCT, md)]
        rgs.append([(1, LIST, (STRUCT, [cc])), (2, I64, tot_u), (3, I64, nv)])
    schema = [[(4, BINARY, b"schema"), (5, I32, 1)], [(1, I32, 1), (3, I32, 0), (4, BINARY, b"v")]]
    nrows = sum(r[2][2] for r in rgs)
    meta = struct_([(1, I32, 1), (2, LIST, (STRUCT, schema)), (3, I64, nrows), (4, LIST, (STRUCT, rgs))])
    out += meta + struct.pack("<I", len(meta)) + b"PAR1"
    return bytes(out)


INT96 = 3
REQUIRED, OPTIONAL, REPEATED = 0, 1, 2


def _hybrid_levels(levels, width):
    """V1 level stream: u32 length + one bit-packed run (the reference writer's layout)."""
    from parquet_go_amd import writer as W  # (tests put the package on the path as parquet_go_amd)

    enc = W.hybrid_encode(width, levels)
    return struct.pack("<I", len(enc)) + enc


def int96_file(row_groups, repetition=REQUIRED):
    """One INT96 column "t" (REQUIRED, OPTIONAL or REPEATED directly under the root), V1 pages,
    UNCOMPRESSED.  row_groups: [(dictionary or None, [page, ...])] with dictionary = (values block,
    num_values) and page = (values block, num_values, encoding, def levels or None, rep levels or
    None); the level streams are prepended to the page block as the reference writer lays them out.
    Page blocks are taken verbatim, so a block may end inside a value (the short INT96 reads of
    type_int96.go:21-42)."""
    out = bytearray(b"PAR1")
    rgs, nrows_total = [], 0
    for dictionary, pages in row_groups:
        start = len(out)
        dict_off = None
        tot = nv_total = 0
        if dictionary is not None:
            blk, n = dictionary
            h = struct_([(1, I32, 2), (2, I32, len(blk)), (3, I32, len(blk)),
                         (7, STRUCT, [(1, I32, n), (2, I32, 0)])])
            dict_off = len(out)
            out += h + blk
            tot += len(h) + len(blk)
        data_off = len(out)
        rows = 0
        for blk, n, enc, d, r in pages:
            lv = b""
            if r is not None:
                lv += _hybrid_levels(r, 1)
                rows += sum(1 for x in r if x == 0)
            else:
                rows += n
            if d is not None:
                lv += _hybrid_levels(d, 1)
            body = lv + blk
            dph = [(1, I32, n), (2, I32, enc), (3, I32, 3), (4, I32, 3)]
            h = struct_([(1, I32, 0), (2, I32, len(body)), (3, I32, len(body)), (5, STRUCT, dph)])
            out += h + body
            tot += len(h) + len(body)
            nv_total += n
        encs = [3, 0] + ([8] if dictionary is not None else [])
        md = [(1, I32, INT96), (2, LIST, (I32, encs)), (3, LIST, (BINARY, [b"t"])), (4, I32, 0), (5, I64, nv_total),
              (6, I64, tot), (7, I64, tot), (9, I64, data_off)]
        if dict_off is not None:
            md.append((11, I64, dict_off))
        cc = [(2, I64, start), (3, STRUCT, md)]
        rgs.append([(1, LIST, (STRUCT, [cc])), (2, I64, tot), (3, I64, rows)])
        nrows_total += rows
    schema = [[(4, BINARY, b"schema"), (5, I32, 1)], [(1, I32, INT96), (3, I32, repetition), (4, BINARY, b"t")]]
    meta = struct_([(1, I32, 1), (2, LIST, (STRUCT, schema)), (3, I64, nrows_total), (4, LIST, (STRUCT, rgs))])
    out += meta + struct.pack("<I", len(meta)) + b"PAR1"
    return bytes(out)
