"""C1 launch-rate probe: host submission time of batch.run() vs the GPU's step time.

  python scripts/c1_launch_probe.py [runs]

Prints, for the C1 batch: the loop's submit-only time per run (no sync inside), the synced time per
run, and the same for a loop of bare hipGraph replays timed by HIP events on the decode stream.
If submit ~= synced, the step is host-bound.
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import __graft_entry__ as G  # noqa: E402

pkg = G._package()
from parquet_go_amd import datasets, native  # noqa: E402

runs = int(sys.argv[1]) if len(sys.argv) > 1 else 200
data = datasets.c1(seed=1)
ctx = native.Context(0, profile=False)
f = native.File(data)
hb = f.load(0, f.num_row_groups, list(range(len(f.columns()))), ctx=ctx)
b = native.Batch.from_host(ctx, hb)
for _ in range(5):
    b.run()
b.sync()
for rep in range(3):
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(runs):
        b.run()
    t1 = time.perf_counter()
    ctx.sync()
    t2 = time.perf_counter()
    print(f"flat={os.environ.get('PQH_FLAT', '1')} runs {runs}: submit {1e6 * (t1 - t0) / runs:.2f} us/run, "
          f"synced {1e6 * (t2 - t0) / runs:.2f} us/run", flush=True)
b.sync()
b.close()
hb.close()
