"""Device SNAPPY timing probe (multi-workgroup pipeline "mw" and k_snappy "page"): one page vs many copies of it, per kind of block (bulk literals,
copy-heavy runs, URL-like text, random letters).  Prints ms per launch and decompressed GB/s."""
import os
import sys
import time

import numpy as np
import pyarrow as pa

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import __graft_entry__ as ge

    pq = ge._package()
    N = pq.native
    from parquet_go_amd import datasets

    ctx = N.Context(0)
    rng = np.random.default_rng(1)
    data, offs = datasets.c5z_strings(40000)
    url = data[:int(offs[-1])].tobytes()[:1 << 20]
    cases = {
        "literal_1MiB": rng.bytes(1 << 20),
        "runs_1MiB": np.repeat(rng.integers(0, 4, 20000, dtype=np.uint8), 53)[:1 << 20].tobytes(),
        "url_1MiB": url,
        "letters_1MiB": bytes(rng.integers(97, 123, 1 << 20, dtype=np.uint8)),
    }
    modes = os.environ.get("PROBE_MODES", "mw,page").split(",")
    sel = os.environ.get("PROBE_CASES")
    for name, raw in cases.items():
        if sel and name not in sel.split(","):
            continue
        blk = pa.compress(raw, codec="snappy", asbytes=True)
        for mode, copies in [(m, c) for m in modes for c in [int(x) for x in os.environ.get("PROBE_COPIES", "1,512").split(",")]]:
            os.environ["PQH_SNAPPY_PAGE"] = "1" if mode == "page" else "0"  # k_snappy vs k_snap_* pipeline
            soff = (len(blk) + 63) & ~63
            ioff = (len(raw) + 63) & ~63
            pages = [N.CodecPage(i * soff, i * ioff, len(blk), len(raw), 0, 1, 0, 0) for i in range(copies)]
            src = np.zeros(soff * copies + 4096, np.uint8)
            for i in range(copies):
                src[i * soff:i * soff + len(blk)] = np.frombuffer(blk, np.uint8)
            ds, dd = ctx.malloc(len(src)), ctx.malloc(ioff * copies + 4096)
            ctx.h2d(ds, src.ctypes.data, len(src))
            st = ctx.decompress_pages(pages, ds, dd)
            assert all(x == 0 for x in st), st[:4]
            t0 = time.perf_counter()
            reps = 3
            for _ in range(reps):
                ctx.decompress_pages(pages, ds, dd)
            ms = (time.perf_counter() - t0) / reps * 1e3
            chk = ctx.d2h_array(dd, len(raw)).tobytes() == raw
            print(f"{mode:4s} {name:14s} ratio {len(raw) / len(blk):5.2f} pages {copies:4d}: {ms:8.3f} ms "
                  f"{len(raw) * copies / ms / 1e6:8.2f} GB/s ok={chk}", flush=True)
            ctx.free(ds)
            ctx.free(dd)


if __name__ == "__main__":
    main()
