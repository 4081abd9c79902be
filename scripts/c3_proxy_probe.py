#!/usr/bin/env python3
"""C3 strong-scaling proxy probe: step time and per-kernel times of blocks of
the 128-row-group C3 file, for a range of block sizes, in both DELTA decode modes (page mode: one
workgroup per stream; tile mode: tile sums + page scan + tile expands).  Prints one JSON line per
(block, mode).

  python scripts/c3_proxy_probe.py [--rgs 8,16,24,32,48,64,128] [--modes 1,0] [--steps 10]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rgs", default="8,12,16,20,24,28,32,40,48,64,96,128")
    ap.add_argument("--modes", default="1,0")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rows", type=int, default=1_000_000_000)
    args = ap.parse_args()
    import __graft_entry__ as ge

    ge._package()
    from parquet_go_amd import datasets, native

    data = datasets.c3(rows=args.rows, seed=20)
    f = native.File(data)
    ctx = native.Context(0)
    for mode in args.modes.split(","):
        os.environ["PQH_DELTA_PAGE_MODE"] = mode
        for n in [int(x) for x in args.rgs.split(",")]:
            hb = f.load(0, n, [0], ctx=ctx)
            b = native.Batch.from_host(ctx, hb)
            b.run()
            b.sync()
            rd, wr = b.traffic()
            for _ in range(3):
                b.run()
            b.sync()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                b.run()
            b.sync()
            el = (time.perf_counter() - t0) / args.steps
            ctx.set_profile(True)
            b.reset_stats()
            for _ in range(args.steps):
                b.run()
            b.sync()
            ks = {s.name.decode(): [round(s.total_ms / s.launches, 4), s.work_items] for s in b.kernel_stats() if s.launches}
            ctx.set_profile(False)
            print(json.dumps({"mode": "page" if mode == "1" else "tile", "row_groups": n, "pages": hb.num_pages,
                              "ms": round(el * 1e3, 4), "gbps": round(wr / el / 1e9, 1), "kernels": ks}), flush=True)
            b.close()
            hb.close()
    ctx.close()
    f.close()


if __name__ == "__main__":
    main()
