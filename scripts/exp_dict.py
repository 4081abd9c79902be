"""Experiment: the C2 dictionary columns (int32 K=1000, float K=256) alone, 10 decode passes (for
rocprofv3 counter runs on k_expand's dictionary tiles)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge

ge._package()
from parquet_go_amd import datasets, native, writer as W

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 50_000_000
cols = datasets.c2_columns(rows, 10)
data = W.flat([cols[0], cols[2]], -(-rows // 8), v2=True, as_array=True)
ctx = native.Context(0, profile=True)
f = native.File(data)
hb = f.load(0, f.num_row_groups, list(range(len(f.columns()))))
b = native.Batch.from_host(ctx, hb)
for _ in range(10):
    b.run()
b.sync()
for s in b.kernel_stats():
    if s.launches:
        print(s.name.decode(), round(s.total_ms / s.launches, 4), s.work_items)
