import ctypes, numpy as np, sys, os
sys.path.insert(0, '/root/repo')
import __graft_entry__ as ge; ge._package()
from parquet_go_amd import datasets, native, _lib
data = datasets.c3()
ctx = native.Context(0, profile=True)
f = native.File(data)
hb = f.load(0, f.num_row_groups, [0])
b = native.Batch.from_host(ctx, hb)
for _ in range(3):
    b.run(); b.sync()
buf = np.zeros((16384, 6), np.uint64)
_lib.hip().pqh_debug_ftrace(ctypes.c_void_p(buf.ctypes.data))
n = int((buf[:, 0] > 0).sum())
t = buf[:n].astype(np.float64) / 100.0
tiles = (buf[:n, 5] >> 32).astype(np.int64)
print("streams", n, "tiles/stream", tiles.mean())
for k, lab in enumerate(["total", "stage", "chase", "tables", "expand"]):
    print(f"  {lab:7s} mean {t[:, k].mean():8.2f} us  per tile {(t[:, k] / np.maximum(tiles, 1)).mean():7.2f}")
print({s.name.decode(): round(s.total_ms / max(1, s.launches), 4) for s in b.kernel_stats() if s.launches})
