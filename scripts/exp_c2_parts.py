"""Experiment: k_expand time and algorithmic GB/s per C2 column group (each group decoded alone)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge

ge._package()
from parquet_go_amd import datasets, native, writer as W

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000_000
cols = datasets.c2_columns(rows, 10)
groups = {"copy(int64,double,flba)": [cols[1], cols[3], cols[5]], "dict(int32,float)": [cols[0], cols[2]],
          "bool": [cols[4]], "all": cols}
ctx = native.Context(0, profile=True)
for name, cs in groups.items():
    data = W.flat(cs, -(-rows // 8), v2=True, as_array=True)
    f = native.File(data)
    hb = f.load(0, f.num_row_groups, list(range(len(f.columns()))))
    b = native.Batch.from_host(ctx, hb)
    for _ in range(3):
        b.run()
    b.sync()
    b.reset_stats()
    for _ in range(10):
        b.run()
    b.sync()
    for s in b.kernel_stats():
        if s.launches and s.name.decode() == "k_expand":
            ms = s.total_ms / s.launches
            print(f"{name:28s} k_expand {ms:.3f} ms  {(s.bytes_read + s.bytes_written) / ms / 1e6:.0f} GB/s "
                  f"(read {s.bytes_read / 1e9:.2f} GB, written {s.bytes_written / 1e9:.2f} GB, tiles {s.work_items})",
                  flush=True)
    b.close()
    hb.close()
