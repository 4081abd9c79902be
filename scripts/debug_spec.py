"""Decode C3 / C5 files once (debug builds print per-page walk statistics)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge
pkg = ge._package()
from parquet_go_amd import datasets, native, reader
ctx = native.Context(0)
which = sys.argv[1] if len(sys.argv) > 1 else "c3"
rows = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
data = datasets.c3(rows=rows) if which == "c3" else datasets.c5(rows=rows, row_groups=1)
f = native.File(data)
res = reader.decode_chunks(ctx, f, 0, f.num_row_groups, list(range(len(f.columns()))))
for c in res:
    c.raise_for_status()
print("ok", len(res))
