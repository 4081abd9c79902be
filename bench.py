#!/usr/bin/env python3
"""Benchmark: decoded output GB/s of the HIP page decoder + HBM roofline fraction.

A "step" is one full decode pass (every page of every chunk of the rank's row groups) over
HBM-resident page images: k_prologue -> (delta / byte-array walks) -> k_scan -> k_expand (levels,
PLAIN copies, booleans, dictionaries) / k_delta_* / k_ba_* / k_nest_*.
Default workload = BASELINE.json configs[1] (C2): 100M rows x 6 columns, data page V2, 16 row
groups, at EVERY N: each rank decodes its own C2 file ("scaling": "weak"), so the driver's N=1 and
N>1 lines measure the same per-GPU work.  Every line also carries `c3_strong`, BASELINE.json
configs[2] (C3: ONE 1B-row file of 128 row groups): at N>1 the row groups are sharded in contiguous
blocks over the N GPUs and timed as strong scaling; at N=1 the whole file is timed, and so is rank
0's share of it at N = 2, 4, 8 (shard.row_group_block) on the one GPU -- the single-GPU proxy of the
1->8 curve, with its predicted efficiency.  (--workload c3 makes the strong-scaling C3 run the main
line.)  One process per GPU, no data-path collective: the only collectives are the measurement
reductions and one all-gather of the blocks.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c1|c2|c3|c4|c5|c5z] [--rows R] [--no-c3]

--gpus N without a launcher (WORLD_SIZE unset): bench.py starts the N rank processes itself (before
anything touches the GPU), rendezvous at 127.0.0.1; under torchrun it is one of the ranks.
--dry-run (tests): no GPU -- each rank decodes its shard with the CPU oracle over gloo, to check the
launcher, the shard plan and the reductions.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
MALL_BYTES = 256 << 20  # Infinity Cache (MALL) capacity: a working set below it stays resident between steps
METRIC = "decoded output GB/s (per GPU and whole node) + fraction of HBM roofline"


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def package():
    import __graft_entry__ as ge

    return ge._package()


def cpu_baseline(data, seconds, threads=1, verify=None):
    """The oracle (plain-C restatement of the reference decoders) on a bounded sample of the same
    file: whole row groups until `seconds` of single-thread decode work (walk excluded).  With
    threads > 1 the same sample is decoded again chunk-parallel on a thread pool (the C decoder runs
    without the GIL) -- SURVEY.md §8(d): "1 core and all host cores (page-parallel)".
    verify(rg, ci, results): called outside the timed region with the oracle's page results of every
    sampled chunk, to check the GPU's outputs of the same chunk against them."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import oracle as O

    fr = O.FileReader(data)
    ncols = len(fr.columns)

    def run(ch):
        res = O.decode_chunk(ch)
        n = 0
        for r in res:
            if r.status:
                raise RuntimeError(f"oracle failed: status {r.status}")
            n += len(r.values) + (0 if r.def_levels is None else len(r.def_levels)) + \
                (0 if r.rep_levels is None else len(r.rep_levels))
        return n, res

    def decode(ch):
        return run(ch)[0]

    out_bytes = 0
    spent = 0.0
    sample = []
    for rg in range(len(fr.row_groups)):
        chunks = [fr.read_chunk(rg, ci) for ci in range(ncols)]
        for ci, ch in enumerate(chunks):
            t0 = time.perf_counter()
            n, res = run(ch)
            spent += time.perf_counter() - t0
            out_bytes += n
            if verify is not None:
                verify(rg, ci, res)
            del res
        sample.append(chunks)
        if spent >= seconds:
            break
    rgs = len(sample)
    cpu_baseline.row_groups = rgs
    res = {"value": round(out_bytes / spent / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": "port",
           "sample": f"{rgs} of {len(fr.row_groups)} row groups ({out_bytes / 1e9:.3f} GB decoded) by oracle/refdecode.c "
                     f"(C restatement of the reference Go decoders), single thread, {spent:.1f} s"}
    multi = None
    if threads > 1:
        flat = [ch for chunks in sample for ch in chunks]
        rg = rgs
        while len(flat) < 2 * threads and rg < len(fr.row_groups):  # enough chunks to occupy the pool
            flat += [fr.read_chunk(rg, ci) for ci in range(ncols)]
            rg += 1
        with ThreadPoolExecutor(threads) as ex:
            t0 = time.perf_counter()
            got = sum(ex.map(decode, flat))
            el = time.perf_counter() - t0
        multi = {"value": round(got / el / 1e9, 4), "unit": "GB/s", "cores": threads, "kind": "port",
                 "sample": f"{rg} row groups ({len(flat)} chunks) decoded chunk-parallel on {threads} threads, "
                           f"{el:.2f} s"}
    return res, multi


def cpu_comparator_pyarrow(data, rgs, bytes_per_row, threads):
    """pyarrow's C++ Parquet reader (an industry CPU comparator, NOT the reference)
    reading the oracle sample's row groups of the same in-memory file into Arrow tables on `threads`
    host cores; best of 3.  Decoded bytes are counted with this bench's formula for the same rows."""
    try:
        import pyarrow as pa
        import pyarrow.parquet as pq

        pa.set_cpu_count(threads)
        pf = pq.ParquetFile(pa.BufferReader(pa.py_buffer(data)))
        best, rows = None, 0
        for _ in range(3):
            t0 = time.perf_counter()
            t = pf.read_row_groups(list(range(rgs)), use_threads=threads > 1)
            el = time.perf_counter() - t0
            rows = t.num_rows
            best = el if best is None else min(best, el)
            del t
        return {"value": round(bytes_per_row * rows / best / 1e9, 4), "unit": "GB/s", "cores": threads,
                "kind": f"pyarrow {pa.__version__} C++ reader (comparator, not the reference)",
                "sample": f"{rgs} row groups ({rows} rows) read into Arrow tables, best of 3: {best:.3f} s"}
    except Exception as e:  # a file layout pyarrow refuses: reported, never fatal
        return {"value": None, "error": f"{type(e).__name__}: {str(e)[:160]}"}


def pmc_traffic(kernel, workload, rows):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary of the same
    workload (profiles/*/pmc_summary.json, written by scripts/pmc_summary.py from FETCH_SIZE x2 +
    WRITE_SIZE passes of this bench) that was measured on THIS build: its stamped source hash must
    equal the loaded library's (pqh_build_id).  Returns (bytes or None, source or the reason there
    is none).  bench.py cannot collect PMC counters itself."""
    from parquet_go_amd import native

    mine = native.build_info()["source_hash"]
    prof = os.path.join(ROOT, "profiles")
    if not os.path.isdir(prof):
        return None, "no profiles/ directory"
    stale = []
    for tag in sorted(os.listdir(prof), reverse=True):
        p = os.path.join(prof, tag, "pmc_summary.json")
        if not os.path.exists(p):
            continue
        try:
            s = json.load(open(p))
        except Exception:
            continue
        lines = s.get("bench_lines") or []
        if not lines:
            continue
        keys = {(lines[0]["config"]["workload"], lines[0]["config"]["rows_per_gpu"])}
        if lines[0].get("c1_x10"):  # (a --workload c1 run: its c1_x10 sub-record's kernels are its own)
            keys.add(("c1_x10", 100_000_000))
        if (workload, rows) not in keys:
            continue
        if s.get("variant"):  # an experiment's profile (a non-default switch), not this build's path
            continue
        k = s["kernels"].get(kernel) or {}
        if not k.get("hbm_traffic_bytes_per_launch"):
            continue
        theirs = (s.get("build") or {}).get("source_hash")
        if theirs != mine:
            stale.append(f"profiles/{tag} ({theirs or 'unstamped'})")
            continue
        return k["hbm_traffic_bytes_per_launch"], f"profiles/{tag}/pmc_summary.json (build {mine})"
    return None, (f"no PMC summary of this build ({mine}) for this workload"
                  + (f"; refused, measured on other builds: {', '.join(stale[:3])}" if stale else ""))


def check_chunk(ctx, batch, chunk, res, np):
    """The GPU's outputs of one chunk equal the oracle's page results (values, byte-array offsets
    and bytes, definition / repetition levels), bit for bit."""
    o = batch.chunk_out(chunk)
    if o.status != 0:
        raise RuntimeError(f"chunk {chunk}: GPU status {o.status}")
    want_vals = b"".join(r.values for r in res)
    if o.value_size > 0:
        got = ctx.d2h_array(o.values, o.num_non_null * o.value_size)
        ok = got.tobytes() == want_vals
    else:
        offs = ctx.d2h_array(o.offsets, o.num_non_null + 1, np.int64)
        lens = np.concatenate([np.diff(r.offsets) for r in res if r.offsets is not None] or [np.zeros(0, np.int64)])
        ok = np.array_equal(np.diff(offs), lens) and ctx.d2h_array(o.bytes, int(offs[-1])).tobytes() == want_vals
    for ptr, attr in ((o.def_levels, "def_levels"), (o.rep_levels, "rep_levels")):
        if ptr:
            want = np.concatenate([getattr(r, attr) for r in res])
            ok = ok and np.array_equal(ctx.d2h_array(ptr, o.num_values), want)
    if not ok:
        raise RuntimeError(f"chunk {chunk}: GPU output differs from the oracle")


def check_statuses(batch, num_chunks, native, where):
    """Every chunk of the batch's LAST run decoded without error (a guard that fired during the timed
    passes -- PQH_ERR_INTERNAL, or any decode error -- fails the bench instead of passing unseen)."""
    for c in range(num_chunks):
        o = batch.chunk_out(c)
        if o.status != native.OK:
            raise RuntimeError(f"{where}: chunk {c} failed: {native.STATUS.get(o.status, o.status)} "
                               f"page {o.error_page} phase {o.error_phase}")


def timed_block(ctx, native, f, rg0, rg1, steps, warmup, barrier_sync, pinned=True, verify=None):
    """Load row groups [rg0, rg1) of f into one HBM-resident batch and time `steps` decode runs
    (graph replays) between barriers; statuses checked before and after the timed runs.
    pinned: the walk writes the page images into the context's pinned pool (False: pageable host
    memory, for blocks of tens of GB).  verify(batch): called after the timed runs (outside them).
    Returns (seconds, decoded bytes per run, algorithmic bytes read per run, pages)."""
    ncols = len(f.columns())
    hb = f.load(rg0, rg1, list(range(ncols)), ctx=ctx if pinned else None)
    b = native.Batch.from_host(ctx, hb)
    try:
        b.run()
        b.sync()
        check_statuses(b, hb.num_chunks, native, f"row groups [{rg0}, {rg1})")
        rd, wr = b.traffic()
        for _ in range(warmup):
            b.run()
        barrier_sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            b.run()
        barrier_sync()
        el = time.perf_counter() - t0
        b.sync()
        check_statuses(b, hb.num_chunks, native, f"row groups [{rg0}, {rg1}) after the timed runs")
        if verify is not None:
            verify(b)
        return el, wr, rd, hb.num_pages
    finally:
        b.close()
        hb.close()


def kernel_table(stats, workload, rows):
    """Per-kernel averages of profiled runs (HIP events on the decode stream) and the roofline of the
    dominant kernel = the longest one that moves algorithmic bytes (walks that only read headers
    carry none).  Returns (kernels, roofline, kernel ms of one profiled step)."""
    kernels = {}
    dom = None
    nsteps = 0
    for s in stats:
        if s.launches == 0:
            continue
        avg_ms = s.total_ms / s.launches
        algo = s.bytes_read + s.bytes_written
        kernels[s.name.decode()] = {"avg_ms": round(avg_ms, 4), "launches": s.launches, "work_items": s.work_items,
                                    "algo_bytes": algo,
                                    "gbps": round(algo / (avg_ms * 1e-3) / 1e9, 1) if avg_ms > 0 else None}
        if algo > 0 and (dom is None or s.total_ms > dom.total_ms):
            dom = s
        nsteps = max(nsteps, s.launches)
    roof = None
    if dom is not None:
        avg_ms = dom.total_ms / dom.launches
        ach = (dom.bytes_read + dom.bytes_written) / (avg_ms * 1e-3) / 1e9
        traffic, src = pmc_traffic(dom.name.decode(), workload, rows)
        roof = {"bound": "hbm", "kernel": dom.name.decode(), "achieved": round(ach, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(ach / HBM_PEAK_GBS, 4),
                "traffic": round(traffic) if traffic else None, "traffic_source": src,
                "algo_bytes_per_launch": dom.bytes_read + dom.bytes_written,
                "frac_of_measured_copy_ceiling": round(ach / 6290.0, 4)}
    all_ms = sum(s.total_ms for s in stats) / max(1, nsteps)
    return kernels, roof, all_ms


def mixed_strong_record(args, ctx, native, pkg, datasets, world, rank, local, dist, barrier_sync):
    """N > 1: north_star's 1B-row mixed file as strong scaling over the ranks ("near-linear
    row-group scaling to 8 GPUs"; chunk_reader.go:375-404 readRowGroupData per row group,
    file_reader.go:187-198 SeekToRowGroup addresses any of them).  Rank 0 writes the file once into
    /dev/shm (in place, datasets.mixed(path=...)); every rank memory-maps it and decodes its block
    shard.row_group_block(128, N, rank) HBM-resident; whole-node GB/s = the decoded bytes of all
    ranks / the slowest rank's time; the blocks are checked to tile the file; each rank's first and
    last row group (every chunk) is compared with the oracle after its timed runs."""
    import numpy as np

    from oracle import oracle as O

    rows = args.mixed_rows or datasets.MIXED_ROWS
    desc = datasets.WORKLOADS["mixed"][0]
    steps = max(3, min(args.steps, 10))
    warm = max(1, min(args.warmup, 2))
    shm = "/dev/shm" if os.path.isdir("/dev/shm") else "/tmp"
    path = os.path.join(shm, f"pqh_bench_mixed_50_{os.environ.get('MASTER_PORT', '0')}.parquet")
    t0 = time.perf_counter()
    if rank == 0:
        datasets.mixed(rows=rows, path=path + ".part")
        os.replace(path + ".part", path)
    dist.barrier()
    gen_s = time.perf_counter() - t0
    f = native.File(path)
    try:
        nrg, ncols = f.num_row_groups, len(f.columns())
        rg0, rg1 = pkg.shard.row_group_block(nrg, world, rank)
        dev = f"cuda:{local}"
        checked = []

        def verify(b):  # the rank's first and last row group, every chunk, vs the oracle (untimed)
            fr = O.FileReader(np.memmap(path, dtype=np.uint8, mode="r"))
            for rg in sorted({rg0, rg1 - 1}):
                for ci in range(ncols):
                    check_chunk(ctx, b, (rg - rg0) * ncols + ci, O.decode_chunk(fr.read_chunk(rg, ci)), np)
                checked.append(rg)

        el, wr, rd, pages = timed_block(ctx, native, f, rg0, rg1, steps, warm, barrier_sync, pinned=False,
                                        verify=verify)
        my_rows = sum(f.row_group_num_rows(g) for g in range(rg0, rg1))
        el, total = pkg.shard.reduce_step(el, wr, device=dev)
        blocks = pkg.shard.gather_blocks(rg0, rg1, my_rows, wr, device=dev)
        pkg.shard.check_cover(blocks, nrg, f.num_rows)
        t = el / steps
        e2e = None
        if not args.no_e2e:
            e2e = mixed_stream_e2e(ctx, native, pkg, f, ncols, rg_begin=rg0, rg_end=rg1, barrier_sync=barrier_sync,
                                   device=dev)
        rec = {"workload": desc, "scaling": "strong", "n_gpus": world, "rows_total": f.num_rows,
                "row_groups": nrg, "file_bytes": os.path.getsize(path), "steps": steps,
                "ms_per_step": round(t * 1e3, 4), "value": round(total / t / 1e9, 2),
                "unit": "GB/s (decoded output, whole node)",
                "per_gpu_gbps_rank0": round(wr / t / 1e9, 2), "pages_rank0": pages,
                "step_roofline_rank0": {"bound": "hbm", "achieved": round((rd + wr) / t / 1e9, 1), "peak": HBM_PEAK_GBS,
                                        "unit": "GB/s", "frac": round((rd + wr) / t / 1e9 / HBM_PEAK_GBS, 4),
                                        "note": "rank 0's algorithmic bytes / the slowest rank's step time"},
                "shards": [{"rank": r, "row_groups": [b[0], b[1]], "rows": b[2], "decoded_bytes": b[3]}
                           for r, b in enumerate(blocks)],
                "verified": f"rank 0: row groups {checked}: {len(checked) * ncols} chunks bit-exact vs the oracle "
                            "(every rank checks its first and last row group)",
                "generate_s": round(gen_s, 2)}
        if e2e is not None:
            rec["e2e"] = e2e
        return rec
    finally:
        f.close()
        dist.barrier()
        if rank == 0:
            os.unlink(path)


def mixed_stream_e2e(ctx, native, pkg, f, ncols, per_range=4, slots=4, passes=2, rg_begin=0, rg_end=None,
                     barrier_sync=None, device=None):
    """End-to-end over the whole 1B-row file through a bounded ring (reader.RowGroupStream): ranges
    of `per_range` row groups walked on the host (thrift headers, page images) straight into pinned
    slot blocks, copied to HBM and decoded in order on each slot's one stream, `slots`
    ranges in flight, so the host walk of the next range overlaps the H2D and decode of the ones
    before it.  Every range's chunks are status-checked as the ring hands them out.  The first pass
    pins the slots' blocks; the second (reported) reuses them.  Host decompression: none (the file
    is UNCOMPRESSED; the walk copies the page images).  N > 1: every rank streams its own block
    [rg_begin, rg_end) through its own ring (its own host threads, pinned blocks and PCIe link),
    each pass between barriers; whole-node payload GB/s = the payload of all ranks / the slowest
    rank's pass."""
    ceiling = pinned_h2d_rate(ctx, native)
    st = pkg.reader.RowGroupStream(f, list(range(ncols)), rg_begin=rg_begin, rg_end=rg_end, per_range=per_range,
                                   slots=slots)
    try:
        out = None
        for k in range(passes):
            st.walk_s = 0.0
            for key in st.times:
                st.times[key] = 0.0
            payload = written = 0
            nr = 0
            if barrier_sync:
                barrier_sync()
            t0 = time.perf_counter()
            for a, b, batch, hb in st:
                check_statuses(batch, hb.num_chunks, native, f"stream e2e: row groups [{a}, {b})")
                payload += hb.payload_bytes
                written += batch.traffic()[1]
                nr += 1
            el = time.perf_counter() - t0
            el_max, payload_all = pkg.shard.reduce_step(el, payload, device=device)
            _, written_all = pkg.shard.reduce_step(el, written, device=device)
            out = {"mode": "streaming ring (reader.RowGroupStream): a walker thread walks each range into its slot's "
                           "pinned block, a submitter thread creates its batch (slot arena) and starts the H2D on the "
                           "slot's stream with the decode behind it, the caller waits for decoded "
                           "ranges; %d slots of %d row groups; the host walk is inside the timed pass; host "
                           "decompression: none (UNCOMPRESSED file)"
                           % (slots, per_range),
                   "pass": k, "ranges": nr, "seconds": round(el_max, 3), "payload_bytes": int(payload_all),
                   "payload_h2d_gbps": round(payload_all / el_max / 1e9, 2),
                   "decoded_gbps": round(written_all / el_max / 1e9, 2),
                   "rank0_payload_h2d_gbps": round(payload / el / 1e9, 2),
                   "host_walk_s": round(st.walk_s, 3),
                   "host_seconds": {k: round(v, 3) for k, v in st.times.items()},
                   "pinned_h2d_ceiling_gbps": ceiling,
                   "payload_frac_of_pinned_ceiling": round(payload / el / 1e9 / ceiling, 3) if ceiling else None,
                   "frac_note": "rank 0's payload rate / rank 0's pinned-copy ceiling (one GPU's PCIe link)",
                   "pinned_bytes": st.pinned_bytes(),
                   "pinned_bound_note": f"{slots} pinned blocks (one per slot, reused range after range)"}
        return out
    finally:
        st.close()


def mixed_record(args, ctx, native, pkg, datasets, barrier_sync):
    """north_star's headline workload: ONE 1B-row mixed-encoding file (C2's six columns -- int32 and
    float dictionaries, int64 / double / FLBA(16) / boolean PLAIN, an optional column -- plus C3's
    DELTA_BINARY_PACKED timestamps; V2 pages, 128 row groups; datasets.mixed) decoded HBM-resident
    on this GPU: step time, decoded GB/s, the whole step against the HBM roofline (algorithmic bytes
    read + written / step time / 8 TB/s) and the dominant kernel's.  Row groups 0 and 127 (every
    chunk) are checked against the oracle outside the timed region.  Then rank 0's block of
    shard.row_group_block(128, N, 0) for N = 2, 4, 8 timed alone: the 1->8 proxy on this file."""
    import numpy as np

    from oracle import oracle as O

    rows = args.mixed_rows or datasets.MIXED_ROWS
    desc = datasets.WORKLOADS["mixed"][0]
    steps = max(3, min(args.steps, 10))
    warm = max(1, min(args.warmup, 2))
    t0 = time.perf_counter()
    data = datasets.mixed(rows=rows)
    gen_s = time.perf_counter() - t0
    log(f"mixed: generated {rows} rows ({len(data) / 1e9:.2f} GB file) in {gen_s:.1f}s")
    f = native.File(data)
    try:
        nrg, ncols = f.num_row_groups, len(f.columns())
        t0 = time.perf_counter()
        hb = f.load(0, nrg, list(range(ncols)))
        walk_s = time.perf_counter() - t0
        t0 = time.perf_counter()
        b = native.Batch.from_host(ctx, hb)
        h2d_s = time.perf_counter() - t0
        payload, pages, nch = hb.payload_bytes, hb.num_pages, hb.num_chunks
        hb.close()
        try:
            b.run()
            b.sync()
            check_statuses(b, nch, native, "mixed: first run")
            rd, wr = b.traffic()
            for _ in range(warm):
                b.run()
            barrier_sync()
            t0 = time.perf_counter()
            for _ in range(steps):
                b.run()
            barrier_sync()
            el = time.perf_counter() - t0
            b.sync()
            check_statuses(b, nch, native, "mixed: after the timed steps")
            paths = b.paths()
            ctx.set_profile(True)
            b.reset_stats()
            for _ in range(3):
                b.run()
            b.sync()
            check_statuses(b, nch, native, "mixed: after the profiled steps")
            kernels, roof, all_ms = kernel_table(b.kernel_stats(), desc, rows)
            ctx.set_profile(False)
            # bit-exact sample vs the oracle (outside every timed region)
            fr = O.FileReader(data)
            sample = sorted({0, nrg - 1})
            for rg in sample:
                for ci in range(ncols):
                    check_chunk(ctx, b, rg * ncols + ci, O.decode_chunk(fr.read_chunk(rg, ci)), np)
            del fr
        finally:
            b.close()
        t1 = el / steps
        rec = {"workload": desc, "rows_total": f.num_rows, "row_groups": nrg, "pages": pages,
               "file_bytes": len(data), "payload_bytes": payload, "steps": steps, "ms_per_step": round(t1 * 1e3, 4),
               "value": round(wr / t1 / 1e9, 2), "unit": "GB/s (decoded output)",
               "algo_read_bytes_per_step": rd, "decoded_bytes_per_step": wr,
               "step_roofline": {"bound": "hbm", "achieved": round((rd + wr) / t1 / 1e9, 1), "peak": HBM_PEAK_GBS,
                                 "unit": "GB/s", "frac": round((rd + wr) / t1 / 1e9 / HBM_PEAK_GBS, 4),
                                 "note": "algorithmic bytes of the whole step (page bytes read once + decoded "
                                         "bytes written) / graph-replay step time"},
               "roofline": roof, "kernels": kernels,
               "profiled_kernel_ms_per_step": round(all_ms, 4), "paths": paths,
               "verified": f"row groups {sample}: {len(sample) * ncols} chunks bit-exact vs the oracle",
               "host": {"generate_s": round(gen_s, 2), "walk_s": round(walk_s, 2), "h2d_s": round(h2d_s, 2)},
               "proxy": []}
        for n in (2, 4, 8):
            a, bb = pkg.shard.row_group_block(nrg, n, 0)
            eln, wrn, _, _ = timed_block(ctx, native, f, a, bb, steps, warm, barrier_sync, pinned=False)
            tn = eln / steps
            rec["proxy"].append({"n_gpus": n, "rank0_row_groups": [a, bb], "rank0_ms_per_step": round(tn * 1e3, 4),
                                 "predicted_whole_node_gbps": round(wr / tn / 1e9, 2),
                                 "predicted_efficiency": round(t1 / (n * tn), 4)})
        rec["proxy_method"] = ("rank 0's block of shard.row_group_block(128, N, 0) decoded alone on this one GPU: "
                               "predicted whole-node GB/s = the file's decoded bytes / that time")
        if not args.no_e2e:
            rec["e2e"] = mixed_stream_e2e(ctx, native, pkg, f, ncols)
        return rec
    finally:
        f.close()


def c1_x10_record(args, ctx, native, datasets, barrier_sync):
    """C1's decode on a working set larger than the Infinity Cache: 10 row groups of C1's 10M rows
    (560 MB of page images + output), one batch.  The C1 line itself fits the 256 MiB MALL, so its
    roofline fraction is not HBM evidence; this one is.  (Past k_flat's batch limits, so the three
    kernels run.)"""
    import numpy as np

    W = datasets.W
    rng = np.random.default_rng(1)
    dictionary = rng.integers(-2**31, 2**31 - 1, 4096).astype(np.int32)
    vals = dictionary[np.random.default_rng(2).integers(0, 4096, 100_000_000)]
    data = W.flat([("v", W.Column(W.INT32, vals), W.REQUIRED)], 10_000_000, v2=False, as_array=True)
    del vals
    f = native.File(data)
    try:
        steps = max(3, min(args.steps, 20))
        hb = f.load(0, f.num_row_groups, [0])
        b = native.Batch.from_host(ctx, hb)
        hb.close()
        try:
            b.run()
            b.sync()
            check_statuses(b, f.num_row_groups, native, "c1_x10")
            rd, wr = b.traffic()
            for _ in range(2):
                b.run()
            barrier_sync()
            t0 = time.perf_counter()
            for _ in range(steps):
                b.run()
            barrier_sync()
            el = (time.perf_counter() - t0) / steps
            ctx.set_profile(True)
            b.reset_stats()
            for _ in range(steps):
                b.run()
            b.sync()
            kernels, roof, _ = kernel_table(b.kernel_stats(), "c1_x10", 100_000_000)
            ctx.set_profile(False)
        finally:
            b.close()
        return {"workload": "C1 x10: 100M rows (10 row groups of C1's 10M), required INT32 dictionary K=4096, V1",
                "ms_per_step": round(el * 1e3, 4), "value": round(wr / el / 1e9, 2), "unit": "GB/s",
                "working_set_bytes": rd + wr, "roofline": roof, "kernels": kernels}
    finally:
        f.close()


def c3_strong_record(args, ctx, native, pkg, datasets, world, rank, local, dist, barrier_sync, log):
    """BASELINE.json configs[2] (C3, 128 row groups of one 1B-row file) as strong scaling.
    N>1: every rank opens the SAME file (generated once into /dev/shm) and decodes its contiguous
    block; whole-node GB/s = sum of decoded bytes / max rank time.  N=1: the whole file on the one
    GPU, plus rank 0's block at N = 2, 4, 8 timed alone on the one GPU: the proxy of the 1->8 curve,
    predicted efficiency(N) = T(128 row groups) / (N x T(rank 0's block))."""
    desc, builder = datasets.WORKLOADS["c3"]
    steps = max(3, min(args.steps, 10))
    warm = max(1, min(args.warmup, 2))
    t0 = time.perf_counter()
    shm = "/dev/shm" if os.path.isdir("/dev/shm") else "/tmp"
    path = os.path.join(shm, f"pqh_bench_c3_20_{os.environ.get('MASTER_PORT', '0')}_{os.getpid() if world == 1 else 0}.parquet")
    if rank == 0:
        builder(seed=20, **({"rows": args.c3_rows} if args.c3_rows else {})).tofile(path + ".part")
        os.replace(path + ".part", path)
    if world > 1:
        dist.barrier()
    gen_s = time.perf_counter() - t0
    f = native.File(path)
    try:
        nrg = f.num_row_groups
        dev = f"cuda:{local}" if world > 1 else None
        if world > 1:
            rg0, rg1 = pkg.shard.row_group_block(nrg, world, rank)
            el, wr, _, pages = timed_block(ctx, native, f, rg0, rg1, steps, warm, barrier_sync)
            rows = sum(f.row_group_num_rows(g) for g in range(rg0, rg1))
            el, total = pkg.shard.reduce_step(el, wr, device=dev)
            blocks = pkg.shard.gather_blocks(rg0, rg1, rows, wr, device=dev)
            pkg.shard.check_cover(blocks, nrg, f.num_rows)
            rec = {"workload": desc, "scaling": "strong", "n_gpus": world, "rows_total": f.num_rows,
                   "row_groups": nrg, "steps": steps, "ms_per_step": round(el / steps * 1e3, 4),
                   "value": round(total * steps / el / 1e9, 2), "unit": "GB/s",
                   "shards": [{"rank": r, "row_groups": [b[0], b[1]], "rows": b[2], "decoded_bytes": b[3]}
                              for r, b in enumerate(blocks)]}
        else:
            el1, wr1, _, pages = timed_block(ctx, native, f, 0, nrg, steps, warm, barrier_sync)
            t1 = el1 / steps
            rec = {"workload": desc, "scaling": "strong", "n_gpus": 1, "rows_total": f.num_rows, "row_groups": nrg,
                   "steps": steps, "ms_per_step": round(t1 * 1e3, 4), "value": round(wr1 / t1 / 1e9, 2), "unit": "GB/s",
                   "proxy": []}
            for n in (2, 4, 8):
                a, b = pkg.shard.row_group_block(nrg, n, 0)
                el, wr, _, _ = timed_block(ctx, native, f, a, b, steps, warm, barrier_sync)
                tn = el / steps
                rec["proxy"].append({"n_gpus": n, "rank0_row_groups": [a, b], "rank0_ms_per_step": round(tn * 1e3, 4),
                                     "predicted_whole_node_gbps": round(wr1 / tn / 1e9, 2),
                                     "predicted_efficiency": round(t1 / (n * tn), 4)})
            rec["proxy_method"] = ("rank 0's block of shard.row_group_block(128, N, 0) decoded alone on this one GPU "
                                   "(each rank owns a GPU, an HBM and a host link; no collective in the timed region): "
                                   "predicted whole-node GB/s = the file's decoded bytes / that time")
        rec["generate_s"] = round(gen_s, 2)
        return rec
    finally:
        f.close()
        if world > 1:
            dist.barrier()
        if rank == 0:
            os.unlink(path)


def next_row_record(ctx, pkg, rows=100_000):
    """FileReader.NextRow throughput on a C4-shaped file (LIST<optional int64> +
    MAP<string, optional int32>, 2 row groups): records/s through the GPU decode + the columnar
    assembly over the device's nesting outputs (NextBatch), the GPU decode + the value-by-value
    restatement (records.RowAssembler), and the oracle's decode + the value-by-value assembly (the
    CPU path the reference's algorithm implies).  Rows are compared across the three."""
    import numpy as np

    from oracle import oracle as O
    from parquet_go_amd import datasets, reader, records

    data = datasets.c4(rows=rows, row_groups=2)
    out = {"workload": f"C4 shape, {rows} rows, 2 row groups (NextRow records as dicts)"}

    def gpu(columnar):
        t0 = time.perf_counter()
        fr = reader.FileReader(data, ctx=ctx, columnar=columnar)
        got = []
        while True:
            b = fr.NextBatch(1 << 20)
            if not b:
                break
            got.extend(b)
        el = time.perf_counter() - t0
        paths = dict(fr.assembled)
        fr.close()
        return got, el, paths

    got_c, el_c, paths = gpu(True)
    got_v, el_v, _ = gpu(False)
    # the oracle's decode + value-by-value assembly
    t0 = time.perf_counter()
    fr = O.FileReader(data)
    f = pkg.native.File(data)
    schema = f.schema()
    leaf_el = [e for _, e in schema if e.num_children == 0]
    ref = []
    for rg in range(len(fr.row_groups)):
        stores = {}
        for ci, col in enumerate(fr.columns):
            pages = []
            for r in O.decode_chunk(fr.read_chunk(rg, ci)):
                if r.status:
                    raise RuntimeError(f"oracle failed: {r.status}")
                nv = r.num_values
                if r.offsets is not None:
                    vals = [r.values[a:b] for a, b in zip(r.offsets[:-1].tolist(), r.offsets[1:].tolist())]
                else:
                    vals = np.frombuffer(r.values, np.int64 if col.physical_type == 2 else np.int32).tolist()
                pages.append((records.PAGE_OK, nv, r.def_levels, r.rep_levels, lambda v=vals: v))
            stores[ci] = records.LeafStore(None, col.path, leaf_el[ci].repetition, col.max_def, col.max_rep, pages)
        asm = records.RowAssembler(schema, None, fr.row_group_num_rows(rg), stores=stores)
        ref.extend(asm.next_row() for _ in range(fr.row_group_num_rows(rg)))
    el_o = time.perf_counter() - t0
    f.close()
    if not (got_c == got_v == ref):
        raise RuntimeError("NextRow records differ between the assembly paths")

    import pyarrow  # noqa: F401  (imported before the clock: the first import takes ~1 s)

    def arrow_read(blob):
        """The whole file through ReadRowGroupArrow: (tables, seconds, export seconds)."""
        t0 = time.perf_counter()
        fr = reader.FileReader(blob, ctx=ctx)
        tables, ex = [], 0.0
        while True:
            if fr.row_group_position < fr.RowGroupCount():
                fr.PreLoad()  # (walk + decode of the next row group, outside the export's time)
            e0 = time.perf_counter()
            t = fr.ReadRowGroupArrow()
            if t is None:
                break
            ex += time.perf_counter() - e0
            tables.append(t)
        el = time.perf_counter() - t0
        fr.close()
        return tables, el, ex

    arrow_read(data)  # (warm: pyarrow's compute kernels initialise on their first call)
    tabs, el_a, ex_a = arrow_read(data)
    from parquet_go_amd import assemble
    if [assemble.drop_absent(r) for t in tabs for r in t.to_pylist()] != ref:
        raise RuntimeError("the Arrow export differs from NextRow's records")
    big_rows = 20_000_000
    big = datasets.c4(rows=big_rows, row_groups=4)
    tabs_b, el_b, ex_b = arrow_read(big)
    nb = sum(t.num_rows for t in tabs_b)
    del big, tabs_b
    out.update({"rows": len(ref), "verified": "identical records from the three paths and the Arrow export",
                "gpu_columnar_rows_per_s": round(len(ref) / el_c), "gpu_columnar_s": round(el_c, 3),
                "assembly_paths": paths,
                "gpu_value_by_value_rows_per_s": round(len(ref) / el_v), "gpu_value_by_value_s": round(el_v, 3),
                "oracle_value_by_value_rows_per_s": round(len(ref) / el_o), "oracle_value_by_value_s": round(el_o, 3),
                "gpu_arrow_rows_per_s": round(len(ref) / el_a), "gpu_arrow_s": round(el_a, 3),
                "arrow_c4_full": {"rows": nb, "rows_per_s": round(nb / el_b), "s": round(el_b, 3),
                                  "export_rows_per_s": round(nb / ex_b), "export_s": round(ex_b, 3),
                                  "note": "C4 at BASELINE size (20M rows, 4 row groups): host walk + GPU decode + "
                                          "the Arrow export (ReadRowGroupArrow); export = the Arrow build alone"},
                "note": "each time covers the whole read: host page walk, decode, assembly into Python dicts "
                        "(NextRow paths) or into pyarrow Tables from the device's columnar outputs (arrow: "
                        "ListArray / StructArray over list offsets, presence and leaf validity, no per-row "
                        "Python objects)"})
    return out


def pinned_h2d_rate(ctx, native, nbytes=256 << 20, reps=4):
    """Plain pinned host -> HBM copy rate on this box (the PCIe bound of the end-to-end mode)."""
    import ctypes

    h = ctypes.c_void_p()
    ctx.check(ctx.L.pqh_host_alloc(ctx.h, ctypes.byref(h), nbytes))
    d = ctx.malloc(nbytes)
    try:
        ctx.h2d_pinned_async(d, h.value, nbytes)
        ctx.sync()
        t0 = time.perf_counter()
        for _ in range(reps):
            ctx.h2d_pinned_async(d, h.value, nbytes)
        ctx.sync()
        return round(nbytes * reps / (time.perf_counter() - t0) / 1e9, 2)
    finally:
        ctx.free(d)
        ctx.L.pqh_host_free(ctx.h, h.value)


def launch_ranks(n):
    """`--gpus N` without a launcher: start N copies of this script as ranks 0..N-1 (one per GPU,
    LOCAL_RANK = rank) with a 127.0.0.1 rendezvous, wait for all of them and return the worst exit
    status.  Runs before anything in this process touches the GPU (children are started, never
    exec'd into).  Rank 0's stdout carries the JSON line."""
    import signal
    import socket
    import subprocess

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], env=env))
    log(f"launched {n} ranks (pids {[p.pid for p in procs]}), rendezvous 127.0.0.1:{port}")
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            r = p.poll()
            if r is None:
                continue
            pending.remove(p)
            if r != 0 and rc == 0:
                rc = r if r > 0 else 128 - r
                for q in pending:  # a failed rank: the others would wait at a barrier forever
                    q.send_signal(signal.SIGTERM)
        time.sleep(0.05)
    return rc


def dry_run(args, world, rank, dist, pkg, datasets, builder, kw, seed, strong, desc):
    """--dry-run: the rank plan and the reductions without a GPU (CPU oracle decode of the shard) --
    the main line's shape (weak: a file per rank; strong: blocks of one file) and the c3_strong
    sub-record's (blocks of one C3 file at N > 1; at N = 1 the proxy blocks for N = 2, 4, 8)."""
    from oracle import oracle as O

    def decode(fr, rg0, rg1):
        written = 0
        for rg in range(rg0, rg1):
            for ci in range(len(fr.columns)):
                for r in O.decode_chunk(fr.read_chunk(rg, ci)):
                    written += len(r.values) + (0 if r.def_levels is None else len(r.def_levels))
        return written

    def sharded(fr, strong_):
        nrg = len(fr.row_groups)
        rg0, rg1 = pkg.shard.row_group_block(nrg, world, rank) if strong_ else (0, nrg)
        rows = sum(fr.row_group_num_rows(g) for g in range(rg0, rg1))
        t0 = time.perf_counter()
        written = decode(fr, rg0, rg1)
        el, total = pkg.shard.reduce_step(time.perf_counter() - t0, written)
        blocks = pkg.shard.gather_blocks(rg0, rg1, rows, written)
        if strong_:
            pkg.shard.check_cover(blocks, nrg, fr.num_rows)
        return el, total, [{"rank": r, "row_groups": [b[0], b[1]], "rows": b[2], "decoded_bytes": b[3]}
                           for r, b in enumerate(blocks)]

    fr = O.FileReader(builder(seed=seed, **kw))
    el, total, shards = sharded(fr, strong)
    c3 = None
    if not strong and not args.no_c3:
        c3desc, c3b = datasets.WORKLOADS["c3"]
        fr3 = O.FileReader(c3b(seed=20, **({"rows": args.c3_rows} if args.c3_rows else {})))
        nrg = len(fr3.row_groups)
        if world > 1:
            el3, total3, shards3 = sharded(fr3, True)
            c3 = {"workload": c3desc, "scaling": "strong", "n_gpus": world, "rows_total": fr3.num_rows,
                  "row_groups": nrg, "decoded_bytes_total": total3, "max_rank_s": el3, "shards": shards3}
        else:
            full = decode(fr3, 0, nrg)
            proxy = []
            for n in (2, 4, 8):
                a, b = pkg.shard.row_group_block(nrg, n, 0)
                proxy.append({"n_gpus": n, "rank0_row_groups": [a, b], "rank0_decoded_bytes": decode(fr3, a, b)})
            c3 = {"workload": c3desc, "scaling": "strong", "n_gpus": 1, "rows_total": fr3.num_rows, "row_groups": nrg,
                  "decoded_bytes_total": full, "proxy": proxy}
    mixed = None
    if world > 1 and not args.no_mixed and args.workload != "mixed" and args.mixed_rows:
        # mixed_strong_record's plan: rank 0 writes the file in place into a shared path, every rank
        # maps it and decodes its block of row_group_block(128, N, rank)
        import numpy as np

        shm = "/dev/shm" if os.path.isdir("/dev/shm") else "/tmp"
        mpath = os.path.join(shm, f"pqh_dry_mixed_{os.environ.get('MASTER_PORT', '0')}.parquet")
        if rank == 0:
            datasets.mixed(rows=args.mixed_rows, path=mpath + ".part")
            os.replace(mpath + ".part", mpath)
        dist.barrier()
        frm = O.FileReader(np.memmap(mpath, dtype=np.uint8, mode="r"))
        elm, totalm, shardsm = sharded(frm, True)
        mixed = {"workload": datasets.WORKLOADS["mixed"][0], "scaling": "strong", "n_gpus": world,
                 "rows_total": frm.num_rows, "row_groups": len(frm.row_groups), "decoded_bytes_total": totalm,
                 "max_rank_s": elm, "shards": shardsm}
        del frm
        dist.barrier()
        if rank == 0:
            os.unlink(mpath)
    if rank == 0:
        print(json.dumps({"dry_run": True, "metric": METRIC, "n_gpus": world, "scaling": "strong" if strong else "weak",
                          "config": {"workload": desc, "rows_total": fr.num_rows if strong else fr.num_rows * world},
                          "decoded_bytes_total": total, "max_rank_s": el, "shards": shards, "c3_strong": c3,
                          "mixed_1b": mixed}),
              flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c2", choices=["c1", "c2", "c3", "c4", "c5", "c5z", "mixed"],
                    help="default: c2 (weak scaling: a C2 file per GPU) at every N; c3 / mixed = strong scaling "
                         "of one file")
    ap.add_argument("--rows", type=int, default=0, help="override rows per GPU (default: the config's)")
    ap.add_argument("--codec", default=None, choices=["snappy", "gzip"],
                    help="c5 / c5z: the page codec (default SNAPPY, as configs[4] names)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end (pinned H2D + decode) pass")
    ap.add_argument("--no-c3", action="store_true", help="skip the c3_strong sub-record")
    ap.add_argument("--no-mixed", action="store_true", help="skip the mixed_1b sub-record (N=1: the file on one GPU "
                    "+ the rank-0 proxy; N>1: strong scaling of the file over the ranks)")
    ap.add_argument("--mixed-rows", type=int, default=0, help=argparse.SUPPRESS)  # tests: a smaller mixed file
    ap.add_argument("--e2e-dev-ranges", type=int, default=4,
                    help="end-to-end with device codecs: staged batches (H2D of one overlaps the codec of the last)")
    ap.add_argument("--no-next-row", action="store_true", help="skip the NextRow records/s sub-record")
    ap.add_argument("--next-row-rows", type=int, default=100_000)
    ap.add_argument("--c3-rows", type=int, default=0, help=argparse.SUPPRESS)  # tests: a smaller C3 file
    ap.add_argument("--dry-run", action="store_true", help=argparse.SUPPRESS)
    # rehearsal of the N > 1 path on a box with fewer GPUs than ranks: ranks share the visible GPUs
    # (LOCAL_RANK modulo their count) and reduce over gloo (RCCL refuses two ranks on one GPU)
    ap.add_argument("--share-gpu", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"WORLD_SIZE={world} (launcher) overrides --gpus {args.gpus}")
    torch = dist = None
    try:
        import torch  # noqa: F811
        import torch.distributed as dist  # noqa: F811
    except Exception:
        torch = None
    if world > 1:
        if args.share_gpu:
            local %= max(1, torch.cuda.device_count())
            os.environ["LOCAL_RANK"] = str(local)
        if not args.dry_run:
            torch.cuda.set_device(local)
        dist.init_process_group("gloo" if args.dry_run or args.share_gpu else "nccl")

    pkg = package()
    from parquet_go_amd import datasets, native

    desc, builder = datasets.WORKLOADS[args.workload]
    kw = {}
    if args.rows:
        kw["rows"] = args.rows
    if args.codec == "gzip" and args.workload in ("c5", "c5z"):
        from parquet_go_amd import writer as W

        kw["codec"] = W.GZIP
        desc = desc.replace("SNAPPY", "GZIP") + " (--codec gzip)"
    # C3 (BASELINE configs[2]: 128 row groups of ONE file sharded across 1/2/4/8 GPUs) is strong
    # scaling: every rank opens the same file and decodes its contiguous block of row groups
    # (shard.row_group_block).  The other workloads give every rank its own file (weak scaling).
    strong = args.workload in ("c3", "mixed")
    seed_kw = {"c1": 1, "c2": 10, "c3": 20, "c4": 30, "c5": 40, "c5z": 41, "mixed": 50}[args.workload] + \
        (0 if strong else 1000 * rank)
    if args.workload == "mixed" and args.mixed_rows:
        kw["rows"] = args.mixed_rows
    if args.dry_run:
        return dry_run(args, world, rank, dist, pkg, datasets, builder, kw, seed_kw, strong, desc)
    t0 = time.perf_counter()
    path = None
    if strong and world > 1:
        # generated once (rank 0) into a shared file that every rank memory-maps
        shm = "/dev/shm" if os.path.isdir("/dev/shm") else "/tmp"
        path = os.path.join(shm, f"pqh_bench_{args.workload}_{seed_kw}_{os.environ.get('MASTER_PORT', '0')}.parquet")
        if rank == 0:
            if args.workload == "mixed":  # (36 GB: written in place, never held in this process)
                builder(seed=seed_kw, path=path + ".part", **kw)
            else:
                builder(seed=seed_kw, **kw).tofile(path + ".part")
            os.replace(path + ".part", path)
        dist.barrier()
        data = None
    else:
        data = builder(seed=seed_kw, **kw)
    gen_s = time.perf_counter() - t0
    log(f"rank {rank}: {'opened' if data is None else 'generated'} the {args.workload} file in {gen_s:.1f}s")

    # timed steps replay each batch's captured hipGraph (unprofiled); per-kernel HIP-event timing for
    # the roofline comes from separate profiled passes of the same batch
    ctx = native.Context(local, profile=False)
    f = native.File(data if data is not None else path)
    ncols = len(f.columns())
    rg0, rg1 = pkg.shard.row_group_block(f.num_row_groups, world, rank) if strong else (0, f.num_row_groups)
    my_rows = sum(f.row_group_num_rows(rg) for rg in range(rg0, rg1))
    t0 = time.perf_counter()
    hb = f.load(rg0, rg1, list(range(ncols)), ctx=ctx)
    walk_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    batch = native.Batch.from_host(ctx, hb)
    h2d_s = time.perf_counter() - t0
    log(f"rank {rank}: row groups [{rg0}, {rg1}) of {f.num_row_groups}: walked {hb.num_pages} pages / "
        f"{hb.num_chunks} chunks in {walk_s:.2f}s, payload {hb.payload_bytes / 1e9:.2f} GB uploaded in {h2d_s:.2f}s")

    batch.run()
    batch.sync()
    check_statuses(batch, hb.num_chunks, native, "first run")
    bytes_read, bytes_written = batch.traffic()
    pages_per_gpu, payload_bytes = hb.num_pages, hb.payload_bytes
    for _ in range(args.warmup):
        batch.run()
    batch.sync()
    batch.reset_stats()

    def barrier_sync():
        if world > 1:
            dist.barrier()
        ctx.sync()
        if torch is not None and torch.cuda.is_available():
            torch.cuda.synchronize()

    barrier_sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        batch.run()
    barrier_sync()
    elapsed = time.perf_counter() - t0
    batch.sync()
    check_statuses(batch, hb.num_chunks, native, "after the timed steps")
    # whole job: max step time over ranks, sum of decoded bytes (shard.py; RCCL for N > 1)
    dev = f"cuda:{local}" if world > 1 else None
    elapsed, total_written = pkg.shard.reduce_step(elapsed, bytes_written, device=dev)
    # the sharded decode's one exchange: every rank's block, checked to tile the file (strong mode)
    blocks = pkg.shard.gather_blocks(rg0, rg1, my_rows, bytes_written, device=dev)
    if strong:
        pkg.shard.check_cover(blocks, f.num_row_groups, f.num_rows)
    batch.sync()
    # profiled passes: every kernel between HIP events on the decode stream
    ctx.set_profile(True)
    batch.reset_stats()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        batch.run()
    batch.sync()
    prof_ms = (time.perf_counter() - t0) / args.steps * 1e3
    check_statuses(batch, hb.num_chunks, native, "after the profiled steps")
    stats = batch.kernel_stats()
    ctx.set_profile(False)
    ms_per_step = elapsed / args.steps * 1e3
    value = total_written * args.steps / elapsed / 1e9

    kernels, roof, all_ms = kernel_table(stats, desc, my_rows)
    if roof and roof["algo_bytes_per_launch"] < MALL_BYTES:
        # the dominant kernel's whole working set fits the 256 MiB Infinity Cache and stays resident
        # from step to step (MI355X_MICROARCH.md): its rate is an upper bound, not HBM evidence
        roof["mall_resident"] = True
        roof["note"] = (f"working set {roof['algo_bytes_per_launch'] / 1e6:.0f} MB < 256 MiB: resident in the Infinity "
                        "Cache across steps, so this fraction is not an HBM roofline measurement (see c1_x10)")
    cpu = cpu_mt = cpu_pa = None
    verified = None
    if rank == 0 and world == 1 and not args.no_cpu:
        import numpy as np

        log("timing the CPU baseline (oracle) and checking the GPU outputs of its sample ...")
        nchk = [0]

        def verify(rg, ci, res):
            check_chunk(ctx, batch, rg * ncols + ci, res, np)
            nchk[0] += 1

        # the GPU box grants this job 16 host cores (os.cpu_count() reports the whole machine)
        cpu, cpu_mt = cpu_baseline(data, args.cpu_seconds, threads=min(16, os.cpu_count() or 1), verify=verify)
        verified = f"{nchk[0]} of {hb.num_chunks} chunks (the CPU sample) bit-exact vs the oracle"
        cpu_pa = cpu_comparator_pyarrow(data, cpu_baseline.row_groups, bytes_written / max(1, my_rows),
                                        min(16, os.cpu_count() or 1))
    batch.close()

    # End-to-end: one staged batch per row-group range holding its decompressed
    # page images in pinned host memory; every pass copies each range to HBM on the copy stream
    # while the previous range decodes on the compute stream.  Host decompression excluded.
    # device codecs: the ranges hold the pages of SNAPPY / GZIP chunks still
    # compressed, so H2D moves compressed bytes and every decode starts with k_snappy / k_gzip.
    def e2e_pass(device_snappy, ranges=None):
        # at most 16 staged batches (contiguous row-group ranges): pipeline depth 16, copies of
        # >= 1/16 of the payload each
        nrg = rg1 - rg0
        # device codecs: --e2e-dev-ranges staged batches (default 4): a range's compressed H2D
        # overlaps the previous range's codec + decode, and every range pays the per-page latency
        # of k_snap_stitch / k_gzip once (a launch takes its slowest page's sequential walk); r04,
        # C5z: 72.4 GB/s with 4 ranges vs 59.6 with 1 (host-decompressed e2e 56-60)
        groups = min(nrg, ranges or (max(1, args.e2e_dev_ranges) if device_snappy else 16))
        cuts = [nrg * g // groups for g in range(groups + 1)]

        def load_all():
            # the walker threads write every page image straight into pinned memory from the
            # context's pool (pqh_file_load_pinned); the staged batches adopt it without a copy
            staged, payload, images, walk = [], 0, 0, 0.0
            for g in range(groups):
                t0 = time.perf_counter()
                hbr = f.load(rg0 + cuts[g], rg0 + cuts[g + 1], list(range(ncols)), device_snappy=device_snappy,
                             device_gzip=device_snappy, ctx=ctx)
                walk += time.perf_counter() - t0
                payload += hbr.payload_bytes
                images += hbr.image_bytes or hbr.payload_bytes
                staged.append(native.Batch.staged(ctx, hbr))
                hbr.close()
            return staged, payload, images, walk

        # a first load pins the pool's blocks (one-time cost per process), the second reuses them
        staged, _, _, walk_cold = load_all()
        for sb in staged:
            sb.close()
        staged, payload, images, walk = load_all()
        written = 0.0
        for sb in staged:
            sb.run_staged()
        for g, sb in enumerate(staged):
            sb.sync()
            written += sb.traffic()[1]
            for c in range(ncols * (cuts[g + 1] - cuts[g])):
                if sb.chunk_out(c).status != native.OK:
                    raise RuntimeError("staged decode failed")
        steps = max(1, min(args.steps, 10))
        barrier_sync()
        t0 = time.perf_counter()
        for _ in range(steps):
            for sb in staged:
                sb.run_staged()
        barrier_sync()
        el = time.perf_counter() - t0
        for g, sb in enumerate(staged):  # the last timed pass decoded every chunk without error
            sb.sync()
            for c in range(ncols * (cuts[g + 1] - cuts[g])):
                if sb.chunk_out(c).status != native.OK:
                    raise RuntimeError(f"staged decode failed after the timed passes: range {g} chunk {c} "
                                       f"{native.STATUS.get(sb.chunk_out(c).status)}")
        el, total = pkg.shard.reduce_step(el, written, device=f"cuda:{local}" if world > 1 else None)
        out = {"mode": ("pinned H2D of the COMPRESSED pages, then k_snappy / k_gzip + decode of all of them in one batch"
                        if device_snappy else
                        "pinned H2D on a copy stream, overlapped per row group with decode; host decompression excluded"),
               "payload_bytes_per_gpu": payload, "image_bytes_per_gpu": images, "staged_batches": groups,
               "steps": steps, "ms_per_step": round(el / steps * 1e3, 3),
               "gbps": round(total * steps / el / 1e9, 2),
               "per_gpu_gbps": round(written * steps / el / 1e9, 2),
               "payload_h2d_gbps_per_gpu": round(payload * steps / el / 1e9, 2),
               # one pass over the file with the host's page walk (and, without device SNAPPY, its
               # decompression on the host's chunk threads) counted too
               "host_walk_s": round(walk, 3),
               "host_walk_cold_s": round(walk_cold, 3),
               "host_walk_gbps": round(images / walk / 1e9, 2) if walk > 0 else None,
               "per_gpu_gbps_incl_host_walk": round(written / (walk + el / steps) / 1e9, 2)}
        for sb in staged:
            sb.close()
        return out

    e2e = e2e_dev = None
    if not args.no_e2e:
        e2e = e2e_pass(False)
        e2e["unstaged_h2d_s"] = round(h2d_s, 4)
        e2e["pinned_h2d_ceiling_gbps"] = pinned_h2d_rate(ctx, native)
        probe = f.load(rg0, rg0 + 1, list(range(ncols)), device_snappy=True, device_gzip=True)
        dev_codecs = {c.codec for c in probe.codec_pages()} - {0}
        probe.close()
        dev_kernel = "k_gzip" if 2 in dev_codecs else "k_snappy"
        # compressed at all?  the same probe with every page eligible for the device codecs
        keep = os.environ.get("PQH_DEVICE_CODEC_MAX_RATIO")
        os.environ["PQH_DEVICE_CODEC_MAX_RATIO"] = "0"
        try:
            every = f.load(rg0, rg0 + 1, list(range(ncols)), device_snappy=True, device_gzip=True)
            compressed = len(every.codec_pages()) > 0
            every.close()
        finally:
            if keep is None:
                del os.environ["PQH_DEVICE_CODEC_MAX_RATIO"]
            else:
                os.environ["PQH_DEVICE_CODEC_MAX_RATIO"] = keep
        if compressed and not dev_codecs:
            # every page compresses to >= PQH_DEVICE_CODEC_MAX_RATIO of its image (C5's random letters):
            # the device-codec load keeps them all on the host route, so its end-to-end pass is the
            # host-decompressed one -- measured, not assumed
            e2e_dev = e2e_pass(True, ranges=16)  # (the host path's ranges: nothing for a codec to overlap)
            e2e_dev["device_codec"] = {"pages_on_device": 0,
                                       "note": "no page compresses below PQH_DEVICE_CODEC_MAX_RATIO (0.95) of its image: "
                                               "all stay on the host-decompressed route (no PCIe bytes to save)"}
        if dev_codecs:
            e2e_dev = e2e_pass(True)
            # the codec kernel alone: HBM-resident batch of the rank's row groups, profiled runs
            hd = f.load(rg0, rg1, list(range(ncols)), device_snappy=True, device_gzip=True)
            bd = native.Batch.from_host(ctx, hd)
            bd.run()
            bd.sync()
            ctx.set_profile(True)
            bd.reset_stats()
            for _ in range(3):
                bd.run()
            bd.sync()
            check_statuses(bd, hd.num_chunks, native, f"{dev_kernel} profiled runs")
            codec_kernels = ("k_gzip",) if dev_kernel == "k_gzip" else \
                ("k_snappy", "k_snap_spec", "k_snap_stitch", "k_snap_emit", "k_snap_fixup")
            ks = [s for s in bd.kernel_stats() if s.name.decode() in codec_kernels and s.launches]
            ctx.set_profile(False)
            if ks:
                parts = {s.name.decode(): {"avg_ms": round(s.total_ms / s.launches, 4), "work_items": s.work_items}
                         for s in ks}
                ms = sum(p["avg_ms"] for p in parts.values())
                e2e_dev["device_codec"] = {"kernels": parts, "avg_ms": round(ms, 4),
                                           "compressed_bytes": hd.payload_bytes, "image_bytes": hd.image_bytes,
                                           "decompressed_gbps": round(hd.image_bytes / (ms * 1e-3) / 1e9, 1)}
            bd.close()
            hd.close()
    next_row = None
    if rank == 0 and world == 1 and not args.no_next_row:
        next_row = next_row_record(ctx, pkg, rows=args.next_row_rows)
    c3 = mixed = None
    if not args.no_c3 and args.workload not in ("c3", "mixed"):
        hb.close()
        hb = None
        c3 = c3_strong_record(args, ctx, native, pkg, datasets, world, rank, local, dist, barrier_sync, log)
    c1_x10 = None
    if world == 1 and args.workload == "c1":
        c1_x10 = c1_x10_record(args, ctx, native, datasets, barrier_sync)
    if not args.no_mixed and args.workload != "mixed":
        if hb is not None:
            hb.close()
            hb = None
        data = None  # (the main file: its memory back before the 1B-row file is built)
        if world > 1:
            mixed = mixed_strong_record(args, ctx, native, pkg, datasets, world, rank, local, dist, barrier_sync)
        else:
            mixed = mixed_record(args, ctx, native, pkg, datasets, barrier_sync)
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "launch": ("direct launch of the one kernel (k_flat) per step" if "k_flat" in kernels else
                       "hipGraph replay per step") + " (profiled direct launches: %.4f ms/step)" % prof_ms,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "int32/int64/f32/f64/bool/flba16 (bit-exact integer/byte decode)" if args.workload == "c2"
            else "int32" if args.workload == "c1" else "bytes (int64 offsets + string bytes)" if args.workload in ("c5", "c5z")
            else "int64/int32/bytes + u8 levels + int32 list offsets" if args.workload == "c4" else "int64",
            "data": "synthetic, seeded, written in the reference writer's layout (libpqgen)",
            "build": native.build_info(),
            "config": {"workload": desc, "rows_total": f.num_rows if strong else f.num_rows * world,
                       "rows_per_gpu": my_rows, "row_groups_per_gpu": rg1 - rg0,
                       "pages_per_gpu": pages_per_gpu,
                       "parallelism": (f"row groups of one file sharded in contiguous blocks over {world} GPU(s)"
                                       if strong else f"one file of {f.num_row_groups} row groups per GPU x{world}")
                       + "; no data-path collective",
                       "mode": "HBM-resident"},
            "shards": [{"rank": r, "row_groups": [b[0], b[1]], "rows": b[2], "decoded_bytes": b[3]}
                       for r, b in enumerate(blocks)],
            "per_gpu_gbps": round(bytes_written * args.steps / elapsed / 1e9, 2),
            "per_gpu_gbps_mean": round(total_written / world * args.steps / elapsed / 1e9, 2),
            "algo_read_bytes_per_step": bytes_read,
            "decoded_bytes_per_step": bytes_written,
            "algo_gbps_all_kernels": round((bytes_read + bytes_written) / (all_ms * 1e-3) / 1e9, 1) if all_ms else None,
            "roofline": roof,
            "kernels": kernels,
            "host": {"generate_s": round(gen_s, 2), "walk_decompress_s": round(walk_s, 2), "h2d_s": round(h2d_s, 3),
                     "h2d_gbps": round(payload_bytes / h2d_s / 1e9, 2)},
            "e2e": e2e,
            ("e2e_device_gzip" if args.codec == "gzip" else "e2e_device_snappy"): e2e_dev,
            "c3_strong": c3,
            "mixed_1b": mixed,
            "c1_x10": c1_x10,
            "next_row": next_row,
            "cpu_baseline": cpu,
            "cpu_baseline_multicore": cpu_mt,
            "cpu_comparator_pyarrow": cpu_pa,
            "verified": verified,
        }
        print(json.dumps(line), flush=True)
    if hb is not None:
        hb.close()
    f.close()
    ctx.close()
    if world > 1:
        dist.barrier()
        if path and rank == 0:
            os.unlink(path)
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
