"""k_gzip timing probe: one page vs many copies of it, per kind of data (URL-like text as C5z,
random letters as C5, repetitive runs, zeros).  Prints ms per launch and decompressed GB/s.
PQH_HIP_LIB selects a variant build (PQH_HIPFLAGS=-DPQH_GZIP_PARSE_ONLY / -DPQH_GZIP_NO_CRC)."""
import os
import sys
import time
import zlib

import numpy as np

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
        "url_1MiB": url,
        "letters_1MiB": bytes(rng.integers(97, 123, 1 << 20, dtype=np.uint8)),
        "runs_1MiB": np.repeat(rng.integers(0, 4, 20000, dtype=np.uint8), 53)[:1 << 20].tobytes(),
        "zeros_1MiB": bytes(1 << 20),
    }
    for name, raw in cases.items():
        c = zlib.compressobj(6, zlib.DEFLATED, 31)
        blk = c.compress(raw) + c.flush()
        for copies in [int(x) for x in os.environ.get("PROBE_COPIES", "1,256,1024").split(",")]:
            soff = (len(blk) + 63) & ~63
            ioff = (len(raw) + 63) & ~63
            pages = [N.CodecPage(i * soff, i * ioff, len(blk), len(raw), 0, 2, 0, 0) for i in range(copies)]
            src = np.zeros(soff * copies + 4096, np.uint8)
            for i in range(copies):
                src[i * soff:i * soff + len(blk)] = np.frombuffer(blk, np.uint8)
            ds, dd = ctx.malloc(len(src)), ctx.malloc(ioff * copies + 4096)
            ctx.h2d(ds, src.ctypes.data, len(src))
            st = ctx.decompress_pages(pages, ds, dd)
            t0 = time.perf_counter()
            reps = 2
            for _ in range(reps):
                ctx.decompress_pages(pages, ds, dd)
            ms = (time.perf_counter() - t0) / reps * 1e3
            chk = ctx.d2h_array(dd, len(raw)).tobytes() == raw
            print(f"{name:14s} ratio {len(raw) / len(blk):6.2f} pages {copies:4d}: {ms:9.3f} ms "
                  f"{len(raw) * copies / ms / 1e6:8.2f} GB/s status={st[0]} ok={chk}", flush=True)
            ctx.free(ds)
            ctx.free(dd)


if __name__ == "__main__":
    main()
