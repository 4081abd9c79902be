"""Where the streaming ring's time goes (reader.RowGroupStream over north_star's mixed file):
per (slots, row groups per range) the pass time, payload GB/s and the host-side time of each step
(walk, batch creation, run submission, sync wait, close).  usage: python scripts/stream_probe.py [rows]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

pq = ge._package()
from parquet_go_amd import datasets, native, reader  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else datasets.MIXED_ROWS
t0 = time.perf_counter()
data = datasets.mixed(rows=rows)
print(f"generated {rows} rows, {len(data) / 1e9:.2f} GB in {time.perf_counter() - t0:.1f}s", flush=True)
f = native.File(data)
ncols = len(f.columns())
CONFIGS = [tuple(int(x) for x in c.split(",")) for c in os.environ.get("PROBE_CONFIGS", "1,3,4;1,4,4;1,3,8;0,3,4").split(";")]
for threaded, slots, per in CONFIGS:
    st = reader.RowGroupStream(f, list(range(ncols)), per_range=per, slots=slots, threaded=threaded)
    for p in range(2):
        for k in st.times:
            st.times[k] = 0.0
        payload = 0
        t0 = time.perf_counter()
        for a, b, batch, hb in st:
            payload += hb.payload_bytes
        el = time.perf_counter() - t0
    print(f"{'threaded' if threaded else 'inline'} slots {slots} x {per} rg: {el:.3f}s {payload / el / 1e9:.1f} GB/s pinned {st.pinned_bytes() / 1e9:.2f} GB "
          + " ".join(f"{k} {v:.3f}" for k, v in st.times.items()), flush=True)
    st.close()
