#!/usr/bin/env python3
"""Parity stress on the GPU: the mutation fuzzer of tests/test_gpu_parity.py (_fuzz_cases /
_run_cases: every mutated page its own chunk, status / first error / outputs vs the oracle) over
many seeds and fixtures, with PQH_FLAT on and off.  Prints one line per (fixture, seed); exits 1 on
the first mismatch (the assertion names the case).

  python scripts/fuzz_stress.py [--seeds 40]
  python scripts/fuzz_stress.py --codecs N | --chains N | --delta N | --nest N | --flat N | --records N | --files N
(one mode per run; the logs of the round-5 runs are under profiles/r05/fuzz_*.log)
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=40)
    ap.add_argument("--codecs", type=int, default=0, help="seeds of the SNAPPY / GZIP mutation fuzz instead")
    ap.add_argument("--chains", type=int, default=0, help="seeds of random PLAIN byte-array chains instead")
    ap.add_argument("--delta", type=int, default=0, help="seeds of the DELTA_BINARY_PACKED geometry fuzz instead")
    ap.add_argument("--nest", type=int, default=0, help="seeds of random nested files (nesting outputs) instead")
    ap.add_argument("--records", type=int, default=0, help="seeds of random nested files read by NextRow / Arrow")
    ap.add_argument("--files", type=int, default=0, help="seeds of random flat pyarrow files (types x encodings)")
    ap.add_argument("--flat", type=int, default=0, help="seeds of random nullable / required k_flat batches instead")
    args = ap.parse_args()
    if args.codecs:
        return codecs(args.codecs)
    if args.chains:
        return chains(args.chains)
    if args.delta:
        return delta(args.delta)
    if args.nest:
        return nest(args.nest)
    if args.flat:
        return flat(args.flat)
    if args.records:
        return records(args.records)
    if args.files:
        return pyarrow_files(args.files)
    import __graft_entry__ as ge

    pq = ge._package()
    import fixtures
    import test_gpu_parity as T

    files = {
        "all_types_v1": fixtures.flat_all_types(n=3000, v2=False, page=8 * 1024, rows_per_group=3000),
        "all_types_v2": fixtures.flat_all_types(n=3000, v2=True, page=8 * 1024, rows_per_group=3000),
        "nested_v2": fixtures.nested_list_map(n=1500, v2=True),
        "pyarrow_v2": fixtures.pyarrow_file(n=4000, version="2.0"),
        "nullable_flat": T._nullable_flat(6000),
    }
    ctx = pq.native.Context(0)
    total = 0
    for name, data in files.items():
        for seed in range(1000, 1000 + args.seeds):
            os.environ["PQH_FLAT"] = "1" if seed % 2 else "0"
            cases = T._fuzz_cases(pq, data, seed, per_page=2)[:400]
            t0 = time.perf_counter()
            compared, errors = T._run_cases(pq, ctx, cases, runs=1 + seed % 2)
            total += compared
            print(f"{name} seed {seed}: {compared} cases, {errors} errors, {time.perf_counter() - t0:.2f}s", flush=True)
    print(f"ok: {total} mutated pages equal to the oracle", flush=True)


def codecs(nseeds):
    """The device codecs' mutation fuzz (tests/test_gpu_codec.py) over many seeds: SNAPPY blocks
    (pyarrow-compressed samples and edge blocks, byte flips / truncations / size changes) and GZIP
    streams (gzip_blocks.mutants), each page's status and bytes vs the oracle's codecs."""
    import numpy as np
    import pyarrow as pa

    import __graft_entry__ as ge

    pq = ge._package()
    import gzip_blocks as G
    import test_gpu_codec as TC
    from oracle import oracle as O
    from snappy_blocks import edge_blocks, sample_blocks

    ctx = pq.native.Context(0)
    raws = sample_blocks(seed=9) + [c[1] for c in edge_blocks()]
    comps = [pa.compress(r, codec="snappy", asbytes=True) if len(r) else b"\0" for r in raws]
    valid = [(n, s, len(O.gzip_decode(s))) for n, s, _ in G.valid_cases()]
    total = 0
    for seed in range(2000, 2000 + nseeds):
        rng = np.random.default_rng(seed)
        blocks, sizes = [], []
        for r, comp in zip(raws, comps):
            for k in range(6):
                b = bytearray(comp)
                mode = k % 4
                if mode == 0 and len(b) > 1:
                    for _ in range(int(rng.integers(1, 4))):
                        b[int(rng.integers(1, len(b)))] = int(rng.integers(0, 256))
                elif mode == 1:
                    b = b[:int(rng.integers(0, len(b) + 1))]
                elif mode == 2 and len(b) > 1:
                    b[int(rng.integers(1, len(b)))] ^= 1 << int(rng.integers(0, 8))
                blocks.append(bytes(b))
                sizes.append(max(0, len(r) + (int(rng.integers(-2, 3)) if mode == 3 else 0)))
        bad = TC._check(pq, ctx, blocks, sizes)
        ok, gbad = TC._gzip_check(pq, ctx, G.mutants(valid, seed=seed, per=3))
        total += len(blocks) + ok + gbad
        print(f"seed {seed}: snappy {len(blocks)} blocks ({bad} corrupt), gzip {ok + gbad} streams ({gbad} corrupt)",
              flush=True)
    print(f"ok: {total} mutated codec pages equal to the oracle", flush=True)


def chains(nseeds):
    """PLAIN byte-array pages of random string-length mixes (empty runs, 4-12 byte keys, long
    strings, records that look like length fields, strings of 60-140 KiB) through the fused chain
    (k_ba_chain: every chunk one PLAIN page, no dictionary), clean and with a truncated / trailing /
    corrupted page among them (the batch falls back to the scratch path): every case vs the oracle."""
    import numpy as np

    import __graft_entry__ as ge

    pq = ge._package()
    import fixtures
    import test_gpu_parity as T
    from oracle import oracle as O

    W = fixtures.W
    col = (W.BYTE_ARRAY, 0, 0, 0)
    ctx = pq.native.Context(0, profile=True)

    def strings(rng, n):
        kind = int(rng.integers(0, 6))
        out = []
        for _ in range(n):
            u = rng.random()
            if kind == 0:
                out.append(b"" if u < 0.6 else bytes(int(rng.integers(0, 4))))
            elif kind == 1:
                out.append(bytes(rng.integers(97, 123, int(rng.integers(4, 13))).astype(np.uint8)))
            elif kind == 2:
                out.append(rng.bytes(int(rng.integers(100, 4000))) if u < 0.7 else b"")
            elif kind == 3:
                out.append(b"".join(int(rng.integers(0, 40)).to_bytes(4, "little") for _ in range(int(rng.integers(0, 5)))))
            elif kind == 4:
                out.append(rng.bytes(int(rng.integers(60000, 140000))) if u < 0.05 else rng.bytes(int(rng.integers(0, 9))))
            else:
                out.append(rng.bytes(int(rng.integers(0, 64))))
        return out

    total = fused = 0
    for seed in range(3000, 3000 + nseeds):
        rng = np.random.default_rng(seed)
        cases = []
        for _ in range(int(rng.integers(4, 10))):
            n = int(rng.integers(0, 30000))
            cases.append((col, None, (O.DATA_PAGE, n, W.PLAIN, 0, 0, T._plain_chain(strings(rng, n)))))
        stats = {}
        compared, errors = T._run_cases(pq, ctx, cases, stats)
        fused += stats.get("k_ba_chain", 0) > 0
        # one defect among the clean pages: trailing bytes, a short chain, a cut, a flipped byte
        k = int(rng.integers(0, len(cases)))
        c, d, (pt, n, enc, dl, rl, img) = cases[k]
        defect = int(rng.integers(0, 4))
        if defect == 0:
            img = img + rng.bytes(int(rng.integers(1, 9)))
        elif defect == 1:
            n = n + int(rng.integers(1, 5))
        elif defect == 2 and img:
            img = img[:int(rng.integers(0, len(img)))]
        elif img:
            b = bytearray(img)
            b[int(rng.integers(0, len(b)))] ^= 1 << int(rng.integers(0, 8))
            img = bytes(b)
        bad = cases[:k] + [(c, d, (pt, n, enc, dl, rl, img))] + cases[k + 1:]
        compared2, errors2 = T._run_cases(pq, ctx, bad, {})
        total += compared + compared2
        print(f"seed {seed}: {len(cases)} pages clean ({errors} errors, fused {stats.get('k_ba_chain', 0)}), "
              f"defect {defect} ({errors2} errors)", flush=True)
    print(f"ok: {total} byte-array pages equal to the oracle; {fused} of {nseeds} clean batches on the fused chain",
          flush=True)


def delta(nseeds):
    """DELTA_BINARY_PACKED streams of every block geometry the reference accepts (14 geometries,
    int32 / int64, random sizes and value regimes, with the test suite's mutations: counts above /
    below the stream's, truncations, flipped bytes) over many seeds, in turn in tile mode, page mode
    (k_delta_fused) and split page mode (k_delta_split), with one stream of 8K-60K values per size
    set so that pages span several fused tiles (the stage kept across tiles for narrow blocks):
    every case vs the oracle."""
    import numpy as np

    import __graft_entry__ as ge

    pq = ge._package()
    import test_gpu_parity as T

    ctx = pq.native.Context(0)
    total = 0
    for seed in range(4000, 4000 + nseeds):
        rng = np.random.default_rng(seed)
        mode = ("tile", "page", "split")[seed % 3]
        os.environ["PQH_DELTA_PAGE_MODE"] = "0" if mode == "tile" else "1"
        os.environ["PQH_DELTA_SPLIT"] = "1" if mode == "split" else "0"
        sizes = sorted({int(x) for x in rng.integers(1, 5000, 4)} | {int(rng.integers(1, 130))}
                       | {int(rng.integers(8000, 60000))})
        cases = T._delta_cases(rng, sizes, ["const", "mono", "small", "full", "mixed"], mutate=True)
        compared, errors = T._run_cases(pq, ctx, cases)
        total += compared
        print(f"seed {seed} ({mode} mode): {compared} streams, {errors} errors", flush=True)
    print(f"ok: {total} DELTA streams equal to the oracle", flush=True)


def _nested_file(seed, n_lo=500, n_hi=8000):
    """A random nested file written by pyarrow (seeded): list<int64>, list<list<int32>>,
    list<struct<list<string>>>, map<string, int64>; random null / empty / length mixes, row group and
    page sizes, V1 / V2 pages.  Returns (bytes, rows, p_null, p_empty, mean, the generator)."""
    import io

    import numpy as np
    import pyarrow as pa
    import pyarrow.parquet as pqa

    rng = np.random.default_rng(seed)
    p_null, p_empty, mean = float(rng.uniform(0, 0.5)), float(rng.uniform(0, 0.5)), float(rng.uniform(0.3, 5))

    def lst(f):
        u = rng.random()
        if u < p_null:
            return None
        if u < p_null + p_empty:
            return []
        return [f() for _ in range(rng.poisson(mean))]

    n = int(rng.integers(n_lo, n_hi))
    leaf = lambda: None if rng.random() < p_null else int(rng.integers(-1000, 1000))  # noqa: E731
    a = [lst(leaf) for _ in range(n)]
    b = [lst(lambda: lst(leaf)) for _ in range(n)]
    c = [lst(lambda: {"s": lst(lambda: None if rng.random() < p_null else str(rng.integers(0, 99)))})
         for _ in range(n)]
    m = [None if rng.random() < p_null else [(str(rng.integers(0, 50)), leaf()) for _ in range(rng.poisson(mean))]
         for _ in range(n)]
    t = pa.table({"a": pa.array(a, pa.list_(pa.int64())), "b": pa.array(b, pa.list_(pa.list_(pa.int32()))),
                  "c": pa.array(c, pa.list_(pa.struct([("s", pa.list_(pa.string()))]))),
                  "m": pa.array(m, pa.map_(pa.string(), pa.int64()))})
    buf = io.BytesIO()
    pqa.write_table(t, buf, row_group_size=int(rng.integers(min(200, n), n + 1)),
                    data_page_size=int(rng.choice([1024, 8192, 1 << 20])), use_dictionary=bool(seed % 3 == 0),
                    data_page_version="2.0" if seed % 2 else "1.0",
                    # (pyarrow marks V2 pages with few values uncompressed; the reference decompresses
                    # every V2 page regardless -- SURVEY.md A.5 -- so SNAPPY V2 files fail there)
                    compression="NONE" if seed % 2 else "SNAPPY")
    return buf.getvalue(), n, p_null, p_empty, mean, rng


def nest(nseeds):
    """Random nested files written by pyarrow (lists of lists, lists of structs of lists, maps;
    random null / empty / length mixes, V1 / V2 pages, small pages) and the writer's deep repeated
    chains (depth 1-20): every chunk's list offsets, presence per level and leaf validity vs
    oracle.nest_levels (the Dremel-KAT-pinned restatement)."""
    import __graft_entry__ as ge

    pq = ge._package()
    import fixtures
    import test_gpu_parity as T

    ctx = pq.native.Context(0)
    total = 0
    for seed in range(5000, 5000 + nseeds):
        data, n, p_null, p_empty, mean, rng = _nested_file(seed)
        checked = T._check_nesting(pq, ctx, data)
        depth = int(rng.integers(1, 21))
        deep, _ = fixtures.deep_repeated(n=int(rng.integers(20, 800)), depth=depth, seed=seed)
        checked += T._check_nesting(pq, ctx, deep)
        total += checked
        print(f"seed {seed}: {n} rows, nulls {p_null:.2f} empty {p_empty:.2f} mean {mean:.1f}; depth {depth}: "
              f"{checked} nested chunks", flush=True)
    print(f"ok: {total} nested chunks equal to oracle.nest_levels", flush=True)




def flat(nseeds):
    """k_flat's one-launch path (PQH_FLAT=1) on random small batches: nullable V2 columns (random
    null fractions, including none and all) must decode in the one launch with no fallback, required
    V1 / V2 columns beside them; then the same pages as explicit cases with their true num_nulls
    hints, with wrong hints (the speculation fails, the batch falls back), and mutated: every chunk
    and case vs the oracle."""
    import numpy as np

    import __graft_entry__ as ge

    pq = ge._package()
    import test_gpu_parity as T
    from parity import assert_chunk, oracle_chunk
    from oracle import oracle as O

    os.environ["PQH_FLAT"] = "1"
    ctx = pq.native.Context(0, profile=True)
    total = one_launch = 0
    for seed in range(6000, 6000 + nseeds):
        rng = np.random.default_rng(seed)
        nf = [0.0, 1e-3, float(rng.uniform(0, 1)), 1.0][seed % 4]
        n = int(rng.integers(2000, 40000))
        for data in (T._nullable_flat(n, seed=seed, null_frac=nf), T._required_flat(n, bool(seed % 2), seed=seed)):
            f = pq.native.File(data)
            nc = len(f.columns())
            res, b, hb = pq.reader.decode_chunks(ctx, f, 0, f.num_row_groups, list(range(nc)), return_batch=True)
            paths = b.paths()
            stats = {s.name.decode(): s.launches for s in b.kernel_stats() if s.launches}
            assert paths["flat_fallbacks"] == 0 and stats.get("k_flat", 0) == 1 and "k_expand" not in stats, \
                (seed, paths, stats)
            one_launch += 1
            fr = O.FileReader(data)
            for k, col in enumerate(res):
                rg, ci = divmod(k, nc)
                assert_chunk(col, oracle_chunk(fr, rg, ci), where=f"seed {seed} rg{rg} {col.path}")
            total += len(res)
            b.close()
            hb.close()
            f.close()
        data = T._nullable_flat(n, seed=seed, null_frac=nf)
        clean = T._page_sets_cases(pq, data)
        hints = T._v2_null_hints(pq, data)
        wrong = [h + int(rng.integers(1, 4)) if rng.random() < 0.3 else h for h in hints]
        mut, mh = [], []
        for (col, dimg, pg), h in zip(clean, hints):
            for _ in range(3):
                img2 = T._mutate(rng, pg[5])
                if pg[3] + pg[4] <= len(img2):
                    mut.append((col, dimg, pg[:5] + (img2,)))
                    mh.append(h)
        c1, e1 = T._run_cases(pq, ctx, clean, runs=2, hints=hints)
        c2, e2 = T._run_cases(pq, ctx, clean, runs=1, hints=wrong)
        c3, e3 = T._run_cases(pq, ctx, mut, runs=1 + seed % 2, hints=mh)
        assert e1 == e2 == 0, (seed, e1, e2)
        total += c1 + c2 + c3
        print(f"seed {seed}: n {n} nulls {nf:.3f}: 2 files in one launch; {c1} + {c2} hinted / wrong-hint "
              f"pages, {c3} mutants ({e3} errors)", flush=True)
    print(f"ok: {one_launch} batches in k_flat's one launch, {total} chunks and cases equal to the oracle", flush=True)

def records(nseeds):
    """The record API over random nested files (_nested_file, smaller; some with one corrupted page
    block): every NextRow outcome -- row, load error, or the page error at the row that reaches it --
    and every ReadRowGroupArrow table equal, call by call, to the assembly over the oracle's pages
    (tests/test_records.py oracle_next_rows)."""
    import numpy as np

    import __graft_entry__ as ge

    pq = ge._package()
    import test_records as R
    from oracle import oracle as O

    ctx = pq.native.Context(0)
    total = rows = errs = 0
    for seed in range(7000, 7000 + nseeds):
        data, n, *_ = _nested_file(seed, 100, 1500)
        rng = np.random.default_rng(seed + 1)
        if seed % 3 == 0:  # one byte flipped inside a random page block
            fr = O.FileReader(data)
            rg, ci = int(rng.integers(0, len(fr.row_groups))), int(rng.integers(0, len(fr.columns)))
            blocks = R._page_blocks(data, rg, ci)
            _, start, length = blocks[int(rng.integers(0, len(blocks)))]
            pos = start + int(rng.integers(0, min(24, length) if rng.random() < 0.5 else length))  # (header or body)
            data = data[:pos] + bytes([data[pos] ^ (1 << int(rng.integers(0, 8)))]) + data[pos + 1:]
        want = [R._norm(w) for w in R.oracle_next_rows(data)]
        fr = pq.reader.FileReader(data, ctx=ctx)
        got = []
        while True:
            try:
                got.append(R._norm(fr.NextRow()))
            except EOFError:
                break
            except (pq.reader.DecodeError, pq.records.RecordError) as e:
                got.append(R._norm(R.error_outcome(e)))
        fr.close()
        assert got == want, (seed, next(i for i, (g, w) in enumerate(zip(got + [None], want)) if g != w))
        arrow, paths = R._read_arrow(pq, data)
        assert [R._norm(g) for g in arrow] == want, seed
        e = sum(1 for w in want if isinstance(w, tuple))
        total += 1
        rows += len(want) - e
        errs += e
        print(f"seed {seed}: {n} rows{' (corrupted)' if seed % 3 == 0 else ''}: {len(want) - e} rows, {e} errors; "
              f"NextRow and ReadRowGroupArrow equal to the oracle {paths}", flush=True)
    print(f"ok: {total} files, {rows} rows and {errs} error outcomes equal to the oracle's records", flush=True)

def _flat_file(seed):
    """A random flat file written by pyarrow (seeded): 4-9 columns of random types (INT32 / INT64 /
    FLOAT / DOUBLE / BOOLEAN / BYTE_ARRAY / FIXED_LEN_BYTE_ARRAY / INT96 timestamps), each required or
    nullable at a random null fraction, each dictionary / PLAIN / a DELTA encoding / BYTE_STREAM_SPLIT
    as the type allows; random row group and page sizes; V1 pages UNCOMPRESSED / SNAPPY / GZIP, V2
    pages uncompressed.  Returns (bytes, rows, description)."""
    import io

    import numpy as np
    import pyarrow as pa
    import pyarrow.parquet as pqa

    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 60000))
    kinds = ["i32", "i64", "f32", "f64", "bool", "str", "bin", "flba", "ts96"]
    cols, enc, dict_cols, desc = {}, {}, [], []
    for k in range(int(rng.integers(4, 10))):
        kind = kinds[int(rng.integers(0, len(kinds)))]
        name = f"{kind}_{k}"
        card = int(rng.choice([1, 7, 300, 1 << 20]))
        if kind in ("i32", "i64"):
            hi = int(rng.choice([2, 1000, 2**31 - 1]))
            v = pa.array(rng.integers(-hi, hi, n) % card if card < 1000 else rng.integers(-hi, hi, n),
                         pa.int32() if kind == "i32" else pa.int64())
            choices = ["dict", "PLAIN", "DELTA_BINARY_PACKED"]
        elif kind in ("f32", "f64"):
            v = pa.array(rng.standard_normal(n)[rng.integers(0, min(card, n), n)] if card < n else rng.standard_normal(n),
                         pa.float32() if kind == "f32" else pa.float64())
            choices = ["dict", "PLAIN", "BYTE_STREAM_SPLIT"]
        elif kind == "bool":
            v = pa.array(rng.random(n) < rng.random())
            choices = ["PLAIN"]
        elif kind in ("str", "bin"):
            lens = rng.integers(0, int(rng.choice([1, 8, 40, 300])), n)
            pool = [rng.bytes(int(x)) for x in lens[:min(card, n)]]
            raw = [pool[int(i)] for i in rng.integers(0, len(pool), n)] if card < n else [rng.bytes(int(x)) for x in lens]
            v = pa.array([r.hex() for r in raw]) if kind == "str" else pa.array(raw, pa.binary())
            choices = ["dict", "PLAIN", "DELTA_LENGTH_BYTE_ARRAY", "DELTA_BYTE_ARRAY"]
        elif kind == "flba":
            v = pa.array([bytes(r) for r in rng.integers(0, 256, (n, 16), dtype=np.uint8)[rng.integers(0, min(card, n), n)]],
                         pa.binary(16))
            choices = ["dict", "PLAIN", "DELTA_BYTE_ARRAY"]
        else:
            v = pa.array(rng.integers(0, 2**62, n) % (10**18), pa.timestamp("ns"))
            choices = ["dict", "PLAIN"]
        if rng.random() < 0.5:
            nf = float(rng.choice([0.0, 0.01, rng.random(), 1.0]))
            v = pa.array(v.to_pylist(), v.type, mask=rng.random(n) < nf)
        else:
            nf = None
        e = choices[int(rng.integers(0, len(choices)))]
        if e == "dict":
            dict_cols.append(name)
        else:
            enc[name] = e
        cols[name] = v
        desc.append(f"{name}:{e}" + ("" if nf is None else f"/nulls {nf:.2f}"))
    t = pa.table(cols)
    schema = pa.schema([pa.field(k, c.type, nullable=(k in cols and cols[k].null_count > 0) or rng.random() < 0.5)
                        for k, c in cols.items()])
    t = t.cast(schema)
    v2 = bool(seed % 2)
    comp = "NONE" if v2 else str(rng.choice(["NONE", "SNAPPY", "GZIP"]))
    buf = io.BytesIO()
    pqa.write_table(t, buf, row_group_size=int(rng.integers(max(1, n // 8), n + 1)),
                    data_page_size=int(rng.choice([1024, 16384, 1 << 20])), use_dictionary=dict_cols or False,
                    column_encoding=enc or None, data_page_version="2.0" if v2 else "1.0", compression=comp,
                    use_deprecated_int96_timestamps=True, store_schema=False)
    return buf.getvalue(), n, f"{'V2' if v2 else 'V1'} {comp}: " + " ".join(desc)


def pyarrow_files(nseeds):
    """Random flat pyarrow files (_flat_file) through decode_chunks: every chunk's status, first
    error, levels and values vs the oracle (tests/test_gpu_parity.py _run_file; a type / encoding pair
    the reference rejects must fail the same way, NOT_IMPLEMENTED never)."""
    import __graft_entry__ as ge

    pq = ge._package()
    import test_gpu_parity as T

    ctx = pq.native.Context(0)
    total = 0
    for seed in range(8000, 8000 + nseeds):
        data, n, desc = _flat_file(seed)
        checked, _ = T._run_file(pq, ctx, data)
        total += checked
        print(f"seed {seed}: {n} rows, {checked} chunks: {desc}", flush=True)
    print(f"ok: {total} chunks of random pyarrow files equal to the oracle", flush=True)


if __name__ == "__main__":
    main()
