"""Device-codec repeatability check: the C5z file (SNAPPY or GZIP pages decompressed on the device)
decoded N times as one batch, plain runs and staged end-to-end runs, every run's chunk statuses and
output checksums compared with the first run's.  A race in a codec kernel shows up as a status or
checksum that changes between runs.

    python scripts/codec_stress.py [snappy|gzip] [runs]
"""
import os
import sys
import zlib

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    codec = sys.argv[1] if len(sys.argv) > 1 else "gzip"
    runs = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    import __graft_entry__ as ge

    pq = ge._package()
    from parquet_go_amd import datasets, native
    from parquet_go_amd import writer as W

    _, builder = datasets.WORKLOADS["c5z"]
    kw = {"codec": W.GZIP} if codec == "gzip" else {}
    data = builder(seed=41, **kw)
    f = native.File(data)
    ncols = len(f.columns())
    ctx = native.Context(0)
    dev = dict(device_snappy=codec == "snappy", device_gzip=codec == "gzip")

    def digest(b, nchunks):
        st, sums = [], []
        for c in range(nchunks):
            o = b.chunk_out(c)
            st.append(o.status)
            crc = 0
            if o.status == native.OK:
                if o.value_size > 0:
                    crc = zlib.crc32(ctx.d2h_array(o.values, o.num_non_null * o.value_size).tobytes())
                else:
                    crc = zlib.crc32(ctx.d2h_array(o.offsets, o.num_non_null + 1, np.int64).tobytes())
                    crc = zlib.crc32(ctx.d2h_array(o.bytes, o.num_bytes).tobytes(), crc)
            sums.append(crc)
        return st, sums

    for mode in ("plain", "staged"):
        hb = f.load(0, f.num_row_groups, list(range(ncols)), ctx=ctx if mode == "staged" else None, **dev)
        nch = hb.num_chunks
        b = native.Batch.staged(ctx, hb) if mode == "staged" else native.Batch.from_host(ctx, hb)
        ref = None
        bad = 0
        for r in range(runs):
            if mode == "staged":
                b.run_staged()
            else:
                b.run()
            b.sync()
            d = digest(b, nch)
            if ref is None:
                ref = d
                print(f"{codec} {mode}: {nch} chunks, statuses {sorted(set(d[0]))}", flush=True)
            elif d != ref:
                bad += 1
                print(f"{codec} {mode}: run {r} differs: statuses {d[0]} vs {ref[0]}", flush=True)
        # back-to-back runs without a sync in between (the bench's timed loop), then one check
        for r in range(runs):
            if mode == "staged":
                b.run_staged()
            else:
                b.run()
        b.sync()
        if digest(b, nch) != ref:
            bad += 1
            print(f"{codec} {mode}: back-to-back runs differ", flush=True)
        print(f"{codec} {mode}: {runs} + {runs} runs, {bad} mismatches", flush=True)
        b.close()
        hb.close()


if __name__ == "__main__":
    main()
