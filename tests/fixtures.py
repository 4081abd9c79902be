"""Seeded test inputs: reference-writer-shaped files (libpqgen) and pyarrow-written files.

Each builder returns (file bytes, {column path: expected python values or None}).  Sizes are
small so the oracle (and pure-Python walker) finish in seconds.
"""
import io

import numpy as np

from conftest import load_package

pq = load_package()
W = pq.writer


def _strings(rng, n, lo=8, hi=40, alphabet=(97, 123)):
    return [bytes(rng.integers(alphabet[0], alphabet[1], int(k)).astype(np.uint8)) for k in rng.integers(lo, hi, n)]


def flat_all_types(n=30000, v2=False, codec=0, page=64 * 1024, rows_per_group=12000, seed=7, crc=False):
    """Every physical type and value encoding of the reference, flat schema."""
    rng = np.random.default_rng(seed)
    i32 = rng.integers(0, 1000, n).astype(np.int32)
    i64 = rng.integers(-2**50, 2**50, n)
    f32 = (rng.integers(0, 256, n).astype(np.float32) * 0.25)
    f32[::97] = np.float32(np.nan)
    dbl = rng.normal(size=n)
    dmask = rng.random(n) < 0.05
    bo = (rng.random(n) < 0.5).astype(np.uint8)
    bo2 = (rng.random(n) < 0.1).astype(np.uint8)
    fl = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    i96 = rng.integers(0, 256, (n, 12), dtype=np.uint8)
    ts = (1_700_000_000_000_000_000 + np.cumsum(1_000_000 + rng.integers(0, 4096, n))).astype(np.int64)
    d32 = rng.integers(-2**31, 2**31 - 1, n).astype(np.int32)
    s = _strings(rng, n)
    smask = rng.random(n) < 0.1
    fl_sorted = fl[np.lexsort(fl.T[::-1])]
    fl6 = rng.integers(97, 101, (n, 6), dtype=np.uint8)[np.minimum(rng.geometric(0.002, n), n - 1)]
    fl6_mask = rng.random(n) < 0.05
    cols = [
        ("i32_dict", W.Column(W.INT32, i32), W.REQUIRED),
        ("i64_plain", W.Column(W.INT64, i64, use_dict=False), W.REQUIRED),
        ("f32_dict", W.Column(W.FLOAT, f32), W.REQUIRED),
        ("f64_opt", W.optional(W.DOUBLE, dbl, dmask, use_dict=False), W.OPTIONAL),
        ("f64_opt_dict", W.optional(W.DOUBLE, np.round(dbl, 1), dmask), W.OPTIONAL),
        ("bool_plain", W.Column(W.BOOLEAN, bo), W.REQUIRED),
        ("bool_rle", W.Column(W.BOOLEAN, bo2, encoding=W.RLE), W.REQUIRED),
        ("flba16", W.Column(W.FIXED_LEN_BYTE_ARRAY, fl, type_length=16, use_dict=False), W.REQUIRED),
        ("flba16_dict", W.Column(W.FIXED_LEN_BYTE_ARRAY, fl[rng.integers(0, 50, n)], type_length=16), W.REQUIRED),
        ("i96", W.Column(W.INT96, i96, use_dict=False), W.REQUIRED),
        ("i96_dict", W.Column(W.INT96, i96[rng.integers(0, 20, n)]), W.REQUIRED),
        ("i64_delta", W.Column(W.INT64, ts, encoding=W.DELTA_BINARY_PACKED, use_dict=False), W.REQUIRED),
        ("i32_delta", W.Column(W.INT32, d32, encoding=W.DELTA_BINARY_PACKED, use_dict=False), W.REQUIRED),
        ("str_plain", W.Column(W.BYTE_ARRAY, s, use_dict=False), W.REQUIRED),
        ("str_dict_opt", W.optional(W.BYTE_ARRAY, [s[k % 500] for k in range(n)], smask), W.OPTIONAL),
        ("str_dlba", W.Column(W.BYTE_ARRAY, s, encoding=W.DELTA_LENGTH_BYTE_ARRAY, use_dict=False), W.REQUIRED),
        ("str_dba", W.Column(W.BYTE_ARRAY, sorted(s), encoding=W.DELTA_BYTE_ARRAY, use_dict=False), W.REQUIRED),
        # FIXED_LEN_BYTE_ARRAY + DELTA_BYTE_ARRAY (chunk_reader.go:71-72): sorted rows share prefixes
        ("flba16_dba", W.Column(W.FIXED_LEN_BYTE_ARRAY, fl_sorted, type_length=16, encoding=W.DELTA_BYTE_ARRAY,
                                use_dict=False), W.REQUIRED),
        # dictionary pages until the dictionary page would pass 2 KiB, then DELTA_BYTE_ARRAY pages in
        # the same chunk (fixed-width dictionary values and variable-length DBA values in one chunk)
        ("flba6_dict_dba", W.optional(W.FIXED_LEN_BYTE_ARRAY, fl6, fl6_mask, type_length=6,
                                      encoding=W.DELTA_BYTE_ARRAY, dict_page_limit=2048), W.OPTIONAL),
    ]
    data = W.flat(cols, rows_per_group, v2=v2, codec=codec, max_page_size=page, crc=crc)
    return data


def flat_c2_like(n=40000, v2=True, seed=11):
    """The BASELINE configs[1] schema (C2) at test size."""
    rng = np.random.default_rng(seed)
    i32 = rng.integers(0, 1000, n).astype(np.int32)
    i64 = rng.integers(-2**62, 2**62, n)
    f32 = rng.integers(0, 256, n).astype(np.float32) / 7
    dbl = rng.normal(size=n)
    dmask = rng.random(n) < 0.01
    bo = (rng.random(n) < 0.5).astype(np.uint8)
    fl = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    cols = [
        ("c_int32", W.Column(W.INT32, i32), W.REQUIRED),
        ("c_int64", W.Column(W.INT64, i64, use_dict=False), W.REQUIRED),
        ("c_float", W.Column(W.FLOAT, f32), W.REQUIRED),
        ("c_double", W.optional(W.DOUBLE, dbl, dmask, use_dict=False), W.OPTIONAL),
        ("c_bool", W.Column(W.BOOLEAN, bo), W.REQUIRED),
        ("c_uuid", W.Column(W.FIXED_LEN_BYTE_ARRAY, fl, type_length=16, use_dict=False), W.REQUIRED),
    ]
    return W.flat(cols, 10000, v2=v2, max_page_size=32 * 1024)


def nested_list_map(n=5000, v2=False, seed=30, codec=0, rows_per_group=None):
    """optional LIST<optional int64> + optional MAP<string, optional int32> (C4 shape); two row groups,
    or row groups of rows_per_group rows."""
    rng = np.random.default_rng(seed)
    # LIST: levels for path l.list.element: maxD 3, maxR 1
    ld, lr, lv = [], [], []
    md_k, mr_k, mk = [], [], []
    md_v, mv = [], []
    for r in range(n):
        u = rng.random()
        if u < 0.05:
            ld.append(0); lr.append(0)
        elif u < 0.10:
            ld.append(1); lr.append(0)
        else:
            k = max(1, rng.poisson(4))
            for j in range(k):
                lr.append(0 if j == 0 else 1)
                if rng.random() < 0.05:
                    ld.append(2)
                else:
                    ld.append(3); lv.append(int(rng.integers(-2**40, 2**40)))
        u = rng.random()
        if u < 0.05:
            md_k.append(0); mr_k.append(0); md_v.append(0)
        elif u < 0.10:
            md_k.append(1); mr_k.append(0); md_v.append(1)
        else:
            k = max(1, rng.poisson(3))
            for j in range(k):
                mr_k.append(0 if j == 0 else 1)
                md_k.append(2)
                mk.append(bytes(rng.integers(97, 123, int(rng.integers(4, 13))).astype(np.uint8)))
                if rng.random() < 0.05:
                    md_v.append(2)
                else:
                    md_v.append(3); mv.append(int(rng.integers(-2**31, 2**31 - 1)))
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
    cols = [
        W.Column(W.INT64, np.array(lv, dtype=np.int64), def_levels=ld, rep_levels=lr, use_dict=False),
        W.Column(W.BYTE_ARRAY, mk, def_levels=md_k, rep_levels=mr_k, use_dict=False),
        W.Column(W.INT32, np.array(mv, dtype=np.int32), def_levels=md_v, rep_levels=mr_k, use_dict=False),
    ]
    rg = [n // 2, n - n // 2] if rows_per_group is None else \
        [min(rows_per_group, n - i) for i in range(0, n, rows_per_group)]
    return W.write(schema, cols, rg, v2=v2, codec=codec, max_page_size=16 * 1024)


def pyarrow_file(n=20000, version="1.0", compression="NONE", seed=1, page=4096):
    """Multi-run hybrid streams, fallback-to-PLAIN dictionaries, nested lists (spec cross-check)."""
    import pyarrow as pa
    import pyarrow.parquet as pqa

    rng = np.random.default_rng(seed)
    tbl = pa.table({
        "i32": pa.array(rng.integers(0, 300, n).astype(np.int32)),
        "i32_runs": pa.array(np.repeat(rng.integers(0, 50, n // 100 + 1), 100)[:n].astype(np.int32)),
        "i64": pa.array(rng.integers(-2**40, 2**40, n)),
        "f": pa.array(rng.random(n).astype(np.float32), mask=rng.random(n) < 0.1),
        "d": pa.array(rng.random(n)),
        "b": pa.array(rng.random(n) < 0.3),
        "b_opt": pa.array(rng.random(n) < 0.3, mask=rng.random(n) < 0.2),
        "s": pa.array([("x" * int(k)) for k in rng.integers(0, 20, n)], mask=rng.random(n) < 0.05),
        "l": pa.array([[1, 2, None] if k % 3 == 0 else ([] if k % 3 == 1 else None) for k in range(n)],
                      pa.list_(pa.int64())),
    })
    buf = io.BytesIO()
    pqa.write_table(tbl, buf, data_page_version=version, compression=compression, row_group_size=n // 2 + 3,
                    data_page_size=page)
    return buf.getvalue()


def deep_repeated(n=3000, depth=10, seed=5, wrap=None, v2=False):
    """A chain of `depth` REPEATED groups (an OPTIONAL group before level l where wrap[l-1]) ending in
    an OPTIONAL INT32 leaf: max_rep = depth, rep_def[l-1] = D_l.  Rows are random nested lists (null
    wrappers, empty lists, null leaves), shredded with the Dremel rules the reference's writer follows
    (data_store.go / schema.go): an element after the first of its list at level l has r = l; a
    missing wrapper at level l has d = D_{l-1}, an empty list d = D_l - 1, a null leaf d = D_L."""
    rng = np.random.default_rng(seed)
    wrap = list(wrap) if wrap is not None else [l % 3 == 1 for l in range(depth)]
    D, d = [], 0
    for l in range(depth):
        d += 2 if wrap[l] else 1
        D.append(d)
    dl, rl, vals = [], [], []

    def shred(x, l, r):  # x = the content of level l (1-based)
        base = D[l - 2] if l >= 2 else 0
        if wrap[l - 1] and x is None:
            dl.append(base); rl.append(r)
            return
        if not x:
            dl.append(D[l - 1] - 1); rl.append(r)
            return
        for i, e in enumerate(x):
            rr = r if i == 0 else l
            if l == depth:
                dl.append(D[-1] + (e is not None)); rl.append(rr)
                if e is not None:
                    vals.append(e)
            else:
                shred(e, l + 1, rr)

    def gen(l):
        if wrap[l - 1] and rng.random() < 0.08:
            return None
        k = int(rng.poisson(1.3 if l < depth else 2.0))
        if l == depth:
            return [None if rng.random() < 0.1 else int(rng.integers(-2**31, 2**31 - 1)) for _ in range(k)]
        return [gen(l + 1) for _ in range(k)]

    for _ in range(n):
        shred(gen(1), 1, 0)
    schema = [W.element("schema", repetition=-1, num_children=1)]
    for l in range(depth):
        if wrap[l]:
            schema.append(W.element(f"o{l + 1}", repetition=W.OPTIONAL, num_children=1))
        schema.append(W.element(f"r{l + 1}", repetition=W.REPEATED, num_children=1))
    schema[-1] = W.element(f"r{depth}", repetition=W.REPEATED, num_children=1)
    schema.append(W.element("v", W.INT32, W.OPTIONAL))
    col = W.Column(W.INT32, np.array(vals, dtype=np.int32), def_levels=np.array(dl, np.uint8),
                   rep_levels=np.array(rl, np.uint8), use_dict=False)
    return W.write(schema, [col], [n // 2, n - n // 2], v2=v2, max_page_size=8 * 1024), D


def disagreeing_group(n=4000, seed=9):
    """optional group g {optional int32 a; optional int32 b} whose two leaves disagree on g's presence
    in some rows (a writes d = 0 where b writes g present): a file the columnar assembly accepts at
    construction but whose lazy presence check (assemble.ColumnarAssembler._presence) rejects, so
    NextRow and ReadRowGroupArrow assemble it value by value.  Two row groups, the second consistent."""
    rng = np.random.default_rng(seed)
    da = rng.integers(0, 3, n).astype(np.uint8)
    db = np.where(da == 0, 0, rng.integers(1, 3, n)).astype(np.uint8)  # mostly consistent ...
    flip = rng.random(n // 2) < 0.05
    db[:n // 2][flip & (da[:n // 2] == 0)] = 2  # ... except some rows of the first row group
    schema = [W.element("schema", repetition=-1, num_children=1),
              W.element("g", repetition=W.OPTIONAL, num_children=2),
              W.element("a", W.INT32, W.OPTIONAL), W.element("b", W.INT32, W.OPTIONAL)]
    cols = [W.Column(W.INT32, rng.integers(-99, 99, int((da == 2).sum())).astype(np.int32), def_levels=da, use_dict=False),
            W.Column(W.INT32, rng.integers(-99, 99, int((db == 2).sum())).astype(np.int32), def_levels=db, use_dict=False)]
    return W.write(schema, cols, [n // 2, n - n // 2], max_page_size=4 * 1024)
