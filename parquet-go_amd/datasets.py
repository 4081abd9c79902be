"""Seeded synthetic inputs for the BASELINE.json configs, written in the
reference writer's layout by libpqgen.  Used by bench.py and the tests; nothing here decodes.

  C1  configs[0]: required INT32, dictionary K=4096 (index width 13), UNCOMPRESSED, V1
  C2  configs[1]: 6 flat columns (int32 dict K=1000, int64 PLAIN, float dict K=256, optional double
                  PLAIN 1% nulls, boolean PLAIN, FLBA(16) PLAIN), V2 pages, 16 row groups
  C3  configs[2]: INT64 timestamps DELTA_BINARY_PACKED 128/4, row groups of 7,812,500 rows
  C4  configs[3]: optional LIST<optional int64> + optional MAP<string, optional int32>, V1 or V2,
                  UNCOMPRESSED (levels -> list offsets / validity)
  C5  configs[4]: required BYTE_ARRAY strings, length U[8,40], ~half unique; each chunk starts with
                  RLE_DICTIONARY pages (dictionary page <= 1 MiB) and falls back to
                  DELTA_LENGTH_BYTE_ARRAY; SNAPPY
"""
import os

import numpy as np

from . import writer as W


def c1(rows=10_000_000, seed=1):
    rng = np.random.default_rng(seed)
    dictionary = rng.integers(-2**31, 2**31 - 1, 4096).astype(np.int32)
    idx = np.random.default_rng(seed + 1).integers(0, 4096, rows)
    vals = dictionary[idx]
    return W.flat([("v", W.Column(W.INT32, vals), W.REQUIRED)], rows, v2=False, as_array=True)


def c2_columns(rows, seed=10):
    r = [np.random.default_rng(seed + k) for k in range(6)]
    d_i32 = r[0].integers(-2**31, 2**31 - 1, 1000).astype(np.int32)
    c_i32 = d_i32[r[0].integers(0, 1000, rows)]
    c_i64 = r[1].integers(-2**63, 2**63 - 1, rows, dtype=np.int64)
    d_f32 = r[2].standard_normal(256).astype(np.float32)
    c_f32 = d_f32[r[2].integers(0, 256, rows)]
    c_f64 = r[3].standard_normal(rows)
    nulls = r[3].random(rows) < 0.01
    c_bool = (r[4].random(rows) < 0.5).astype(np.uint8)
    c_uuid = r[5].integers(0, 256, (rows, 16), dtype=np.uint8)
    return [
        ("c_int32", W.Column(W.INT32, c_i32), W.REQUIRED),
        ("c_int64", W.Column(W.INT64, c_i64, use_dict=False), W.REQUIRED),
        ("c_float", W.Column(W.FLOAT, c_f32), W.REQUIRED),
        ("c_double", W.optional(W.DOUBLE, c_f64, nulls, use_dict=False), W.OPTIONAL),
        ("c_bool", W.Column(W.BOOLEAN, c_bool), W.REQUIRED),
        ("c_uuid", W.Column(W.FIXED_LEN_BYTE_ARRAY, c_uuid, type_length=16, use_dict=False), W.REQUIRED),
    ]


def c2(rows=100_000_000, row_groups=16, seed=10):
    per = -(-rows // row_groups)
    return W.flat(c2_columns(rows, seed), per, v2=True, as_array=True)


def c3_values(rows=1_000_000_000, seed=20):
    rng = np.random.default_rng(seed)
    return np.cumsum(1_000_000 + rng.integers(0, 4096, rows), dtype=np.int64) + 1_700_000_000_000_000_000


def c3(rows=1_000_000_000, rows_per_group=None, seed=20, row_groups=128):
    """BASELINE configs[2]: 128 row groups (7,812,500 rows each at 1B rows) unless rows_per_group."""
    if rows_per_group is None:
        rows_per_group = -(-rows // row_groups)
    ts = c3_values(rows, seed)
    return W.flat([("ts", W.Column(W.INT64, ts, encoding=W.DELTA_BINARY_PACKED, use_dict=False), W.REQUIRED)],
                  rows_per_group, v2=False, as_array=True)


def _repeated_levels(rng, rows, mean, p_null, p_empty, p_null_elem, max_d):
    """Levels of one repeated leaf under an optional group (max_d = 3 with an optional leaf):
    per row a null group (d 0), an empty group (d 1) or Poisson(mean) >= 1 entries (d max_d, or
    max_d - 1 for a null leaf); r = 0 at each row's first slot."""
    u = rng.random(rows)
    k = np.maximum(1, rng.poisson(mean, rows))
    k[u < p_null + p_empty] = 1
    starts = np.zeros(rows + 1, np.int64)
    np.cumsum(k, out=starts[1:])
    n = int(starts[-1])
    rep = np.ones(n, np.uint8)
    rep[starts[:-1]] = 0
    d = np.full(n, max_d, np.uint8)
    if p_null_elem > 0:
        d[rng.random(n) < p_null_elem] = max_d - 1
    d[starts[:-1][u < p_null]] = 0
    d[starts[:-1][(u >= p_null) & (u < p_null + p_empty)]] = 1
    return d, rep


def c4(rows=20_000_000, row_groups=4, v2=False, seed=30):
    schema, cols = c4_columns(rows, seed)
    per = -(-rows // row_groups)
    rg = [min(per, rows - i * per) for i in range(row_groups)]
    return W.write(schema, cols, rg, v2=v2, as_array=True)


def c4_columns(rows, seed=30):
    rng = np.random.default_rng(seed)
    ld, lr = _repeated_levels(rng, rows, 4.0, 0.05, 0.05, 0.05, 3)
    lv = rng.integers(-2**40, 2**40, int((ld == 3).sum()))
    rng = np.random.default_rng(seed + 1)
    kd, kr = _repeated_levels(rng, rows, 3.0, 0.0, 0.05, 0.0, 2)
    nk = int((kd == 2).sum())
    klen = rng.integers(4, 13, nk).astype(np.int64)
    koff = np.zeros(nk + 1, np.int64)
    np.cumsum(klen, out=koff[1:])
    kdata = np.concatenate([rng.integers(97, 123, int(koff[-1]), dtype=np.uint8), np.zeros(1, np.uint8)])
    vd = kd.copy()
    vd[vd == 2] = 3
    vd[(vd == 3) & (rng.random(len(vd)) < 0.05)] = 2
    vv = rng.integers(-2**31, 2**31 - 1, int((vd == 3).sum())).astype(np.int32)
    schema = [
        W.element("schema", repetition=-1, num_children=2),
        W.element("l", repetition=W.OPTIONAL, num_children=1, converted_type=3),
        W.element("list", repetition=W.REPEATED, num_children=1),
        W.element("element", W.INT64, W.OPTIONAL),
        W.element("m", repetition=W.OPTIONAL, num_children=1, converted_type=1),
        W.element("key_value", repetition=W.REPEATED, num_children=2),
        W.element("key", W.BYTE_ARRAY, W.REQUIRED, converted_type=0),
        W.element("value", W.INT32, W.OPTIONAL),
    ]
    cols = [W.Column(W.INT64, lv, def_levels=ld, rep_levels=lr, use_dict=False),
            W.Column(W.BYTE_ARRAY, (kdata, koff), def_levels=kd, rep_levels=kr, use_dict=False),
            W.Column(W.INT32, vv, def_levels=vd, rep_levels=kr, use_dict=False)]
    return schema, cols


def c5_strings(rows, seed=40, chunk=4_000_000):
    """(data, offsets) of `rows` strings drawn from a pool of rows/2 random lowercase strings of
    length U[8,40] (about 43% of the rows distinct)."""
    rng = np.random.default_rng(seed)
    pool_n = max(1, rows // 2)
    plen = rng.integers(8, 41, pool_n).astype(np.int64)
    poff = np.zeros(pool_n + 1, np.int64)
    np.cumsum(plen, out=poff[1:])
    pool = rng.integers(97, 123, int(poff[-1]), dtype=np.uint8)
    idx = rng.integers(0, pool_n, rows)
    lens = plen[idx]
    offsets = np.zeros(rows + 1, np.int64)
    np.cumsum(lens, out=offsets[1:])
    data = np.empty(int(offsets[-1]) + 1, np.uint8)
    for a in range(0, rows, chunk):  # gather pool bytes chunk by chunk (bounded index arrays)
        b = min(rows, a + chunk)
        ln = lens[a:b]
        starts = np.repeat(poff[idx[a:b]] - offsets[a:b], ln)
        pos = np.arange(offsets[a], offsets[b], dtype=np.int64)
        data[offsets[a]:offsets[b]] = pool[pos + starts]
    return data, offsets


def c5(rows=50_000_000, row_groups=8, seed=40, codec=W.SNAPPY):
    per = -(-rows // row_groups)
    col = W.Column(W.BYTE_ARRAY, c5_strings(rows, seed), encoding=W.DELTA_LENGTH_BYTE_ARRAY,
                   dict_page_limit=1 << 20)
    return W.flat([("s", col, W.REQUIRED)], per, v2=False, codec=codec, as_array=True)

def c5z_strings(rows, seed=41, chunk=2_000_000):
    """(data, offsets) of `rows` URL-like strings "https://<host>/<section>/<item>?id=<n>": a few
    hundred hosts / sections, sequential ids -- text that SNAPPY compresses (unlike C5's random
    letters), for the device-SNAPPY end-to-end measurement."""
    rng = np.random.default_rng(seed)
    hosts = [f"www.{w}.example.com".encode() for w in ("alpha", "bravo", "charlie", "delta", "echo", "foxtrot")]
    sections = [f"{a}-{b}".encode() for a in ("news", "shop", "blog", "docs", "media") for b in range(40)]
    parts, lens = [], []
    for a in range(0, rows, chunk):
        n = min(chunk, rows - a)
        h = rng.integers(0, len(hosts), n)
        sc = rng.integers(0, len(sections), n)
        it = rng.integers(0, 5000, n)
        for i in range(n):
            s = b"https://" + hosts[h[i]] + b"/" + sections[sc[i]] + b"/item" + str(it[i]).encode() + \
                b"?id=" + str(a + i).encode()
            parts.append(s)
            lens.append(len(s))
    offsets = np.zeros(rows + 1, np.int64)
    np.cumsum(np.array(lens, np.int64), out=offsets[1:])
    return np.frombuffer(b"".join(parts) + b"\0", np.uint8), offsets


def c5z(rows=10_000_000, row_groups=8, seed=41, codec=W.SNAPPY):
    """Supplementary (not a BASELINE config): compressible strings, DELTA_LENGTH_BYTE_ARRAY, SNAPPY."""
    per = -(-rows // row_groups)
    col = W.Column(W.BYTE_ARRAY, c5z_strings(rows, seed), encoding=W.DELTA_LENGTH_BYTE_ARRAY, use_dict=False)
    return W.flat([("url", col, W.REQUIRED)], per, v2=False, codec=codec, as_array=True)


MIXED_ROWS, MIXED_ROW_GROUPS = 1_000_000_000, 128


def _mixed_arrays(rows):
    return {"i32": np.empty(rows, np.int32), "i64": np.empty(rows, np.int64), "f32": np.empty(rows, np.float32),
            "f64": np.empty(rows, np.float64), "d64": np.empty(rows, np.uint8), "b": np.empty(rows, np.uint8),
            "uuid": np.empty((rows, 16), np.uint8), "ts": np.empty(rows, np.int64)}


def _mixed_fill(A, r0, f0, g, rows, seed, threads):
    """Row group g into the arrays A at row r0 (compacted doubles at f0); returns its non-null
    double count."""
    L = W._lib.gen()
    at = lambda a, o: a.ctypes.data + o * a.strides[0]  # noqa: E731
    return L.pqg_mixed_row_group(seed, g, rows, at(A["i32"], r0), at(A["i64"], r0), at(A["f32"], r0),
                                 at(A["f64"], f0), at(A["d64"], r0), at(A["b"], r0), at(A["uuid"], r0),
                                 at(A["ts"], r0), threads)


def _mixed_columns(A, rows, nn):
    return [
        ("c_int32", W.Column(W.INT32, A["i32"][:rows]), W.REQUIRED),
        ("c_int64", W.Column(W.INT64, A["i64"][:rows], use_dict=False), W.REQUIRED),
        ("c_float", W.Column(W.FLOAT, A["f32"][:rows]), W.REQUIRED),
        ("c_double", W.Column(W.DOUBLE, A["f64"][:nn], def_levels=A["d64"][:rows], use_dict=False), W.OPTIONAL),
        ("c_bool", W.Column(W.BOOLEAN, A["b"][:rows]), W.REQUIRED),
        ("c_uuid", W.Column(W.FIXED_LEN_BYTE_ARRAY, A["uuid"][:rows], type_length=16, use_dict=False), W.REQUIRED),
        ("ts", W.Column(W.INT64, A["ts"][:rows], encoding=W.DELTA_BINARY_PACKED, use_dict=False), W.REQUIRED),
    ]


def mixed_row_group(g, rows, seed=50, threads=0):
    """Row group g of the mixed workload (north_star's target file): the columns as
    [(name, Column, repetition)] -- C2's six (int32 dictionary K=1000, int64 PLAIN, float
    dictionary K=256, optional double PLAIN 1% null, boolean PLAIN, FLBA(16) PLAIN) and C3's
    timestamps (INT64 DELTA_BINARY_PACKED 128/4), generated by libpqgen from a counter-based hash
    (pqg_mixed_row_group), so any row group is regenerated exactly for checking."""
    A = _mixed_arrays(rows)
    nn = _mixed_fill(A, 0, 0, g, rows, seed, threads)
    return _mixed_columns(A, rows, nn)


def mixed_sizes(rows=MIXED_ROWS, row_groups=MIXED_ROW_GROUPS):
    per = -(-rows // row_groups)
    return [min(per, rows - g * per) for g in range(row_groups) if rows - g * per > 0]


def mixed(rows=MIXED_ROWS, row_groups=MIXED_ROW_GROUPS, seed=50, batch=4, threads=0, path=None):
    """The mixed-encoding workload file (BASELINE north_star: "a 1B-row mixed-encoding Parquet
    file"): `row_groups` row groups of ceil(rows / row_groups) records, V2 pages, UNCOMPRESSED, in
    the reference writer's layout, streamed `batch` row groups at a time into one buffer (the
    columns of all 1B rows never exist at once).  Returns the file as a uint8 array; with `path`,
    the pages are written in place into that file (memory-mapped, e.g. under /dev/shm for ranks that
    share it), which is cut to the file's size, and the path is returned."""
    sizes = mixed_sizes(rows, row_groups)
    schema = W.flat_schema(mixed_row_group(0, 0, seed))
    # upper bound: 57 bytes per row of values + levels + page / chunk overheads
    cap = 57 * rows + (64 << 20)
    buf = np.memmap(path, dtype=np.uint8, mode="w+", shape=(cap,)) if path else None  # (sparse until written)
    sw = W.StreamWriter(schema, cap, v2=True, threads=threads, buf=buf)
    A = _mixed_arrays(sum(sizes[:batch]))
    for g0 in range(0, len(sizes), batch):
        part = sizes[g0:g0 + batch]
        r0 = nn = 0
        for k, n in enumerate(part):  # the batch's row groups generated in place, one after another
            nn += _mixed_fill(A, r0, nn, g0 + k, n, seed, threads)
            r0 += n
        sw.write([c for _, c, _ in _mixed_columns(A, r0, nn)], part)
    out = sw.finish()
    if path is None:
        return out
    n = len(out)
    del out, sw
    buf.flush()
    del buf
    os.truncate(path, n)
    return path


WORKLOADS = {
    "c1": ("C1: 10M rows, required INT32 dictionary K=4096 (width 13), UNCOMPRESSED, data page V1", c1),
    "c2": ("C2: 100M rows x 6 columns (int32 dict / int64 PLAIN / float dict / optional double PLAIN "
           "1% null / boolean PLAIN / FLBA(16) PLAIN), data page V2, 16 row groups", c2),
    "c3": ("C3: INT64 timestamps DELTA_BINARY_PACKED 128/4, 128 row groups (7,812,500 rows each at 1B rows)", c3),
    "c4": ("C4: optional LIST<optional int64> + optional MAP<string, optional int32>, 20M rows, V1, "
           "UNCOMPRESSED", c4),
    "c5": ("C5: required BYTE_ARRAY strings U[8,40] ~half unique, RLE_DICTIONARY (dict page <= 1 MiB) "
           "then DELTA_LENGTH_BYTE_ARRAY fallback, SNAPPY, 8 row groups", c5),
    "c5z": ("C5z (supplementary, not a BASELINE config): 10M URL-like strings, DELTA_LENGTH_BYTE_ARRAY, "
            "SNAPPY-compressible, 8 row groups", c5z),
    "mixed": ("mixed (north_star's target file): 1B rows x 7 columns -- C2's six (int32 dict / int64 PLAIN / "
              "float dict / optional double PLAIN 1% null / boolean PLAIN / FLBA(16) PLAIN) + C3's INT64 "
              "timestamps DELTA_BINARY_PACKED -- data page V2, 128 row groups", mixed),
}
