"""Seeded synthetic inputs for the BASELINE.json configs, written in the
reference writer's layout by libpqgen.  Used by bench.py and the tests; nothing here decodes.

  C1  configs[0]: required INT32, dictionary K=4096 (index width 13), UNCOMPRESSED, V1
  C2  configs[1]: 6 flat columns (int32 dict K=1000, int64 PLAIN, float dict K=256, optional double
                  PLAIN 1% nulls, boolean PLAIN, FLBA(16) PLAIN), V2 pages, 16 row groups
  C3  configs[2]: INT64 timestamps DELTA_BINARY_PACKED 128/4, row groups of 7,812,500 rows
"""
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


def c3(rows=1_000_000_000, rows_per_group=7_812_500, seed=20):
    rng = np.random.default_rng(seed)
    ts = np.cumsum(1_000_000 + rng.integers(0, 4096, rows), dtype=np.int64) + 1_700_000_000_000_000_000
    return W.flat([("ts", W.Column(W.INT64, ts, encoding=W.DELTA_BINARY_PACKED, use_dict=False), W.REQUIRED)],
                  rows_per_group, v2=False, as_array=True)


WORKLOADS = {
    "c1": ("C1: 10M rows, required INT32 dictionary K=4096 (width 13), UNCOMPRESSED, data page V1", c1),
    "c2": ("C2: 100M rows x 6 columns (int32 dict / int64 PLAIN / float dict / optional double PLAIN "
           "1% null / boolean PLAIN / FLBA(16) PLAIN), data page V2, 16 row groups", c2),
    "c3": ("C3: INT64 timestamps DELTA_BINARY_PACKED 128/4, 7,812,500-row row groups", c3),
}
