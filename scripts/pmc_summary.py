#!/usr/bin/env python3
"""Summarise rocprofv3 outputs (gpurun_out/prof_*) into profiles/<tag>/:

  kernel_stats.csv       rocprofv3 --kernel-trace --stats summary (copied)
  pmc_summary.json       per-kernel average duration, FETCH_SIZE / WRITE_SIZE per launch, HBM traffic

HBM traffic per launch = FETCH_SIZE x 2 + WRITE_SIZE (KB -> bytes): on gfx950 FETCH_SIZE reports
half the bytes of wide coalesced streaming reads (MI355X_MICROARCH.md §HBM); every read of the
decode kernels is a 16-byte-per-lane coalesced load (copies, LDS staging) or an 8-byte load.

usage: python scripts/pmc_summary.py <tag> [gpurun_out] [prefix (default prof)]
"""
import csv
import json
import os
import shutil
import sys


def per_kernel(path, value_col="Counter_Value"):
    agg = {}
    if not os.path.exists(path):
        return agg
    for r in csv.DictReader(open(path)):
        agg.setdefault(r["Kernel_Name"], []).append(float(r[value_col]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def durations(path):
    agg = {}
    if not os.path.exists(path):
        return agg
    for r in csv.DictReader(open(path)):
        agg.setdefault(r["Kernel_Name"], []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return {k: sum(v) / len(v) / 1e6 for k, v in agg.items()}


def main():
    tag = sys.argv[1]
    src = sys.argv[2] if len(sys.argv) > 2 else "gpurun_out"
    pre = sys.argv[3] if len(sys.argv) > 3 else "prof"
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = os.path.join(root, "profiles", tag)
    os.makedirs(out, exist_ok=True)
    stats = os.path.join(src, pre + "_trace", "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(out, "kernel_stats.csv"))
    fetch = per_kernel(os.path.join(src, pre + "_fetch", "run_counter_collection.csv"))
    write = per_kernel(os.path.join(src, pre + "_write", "run_counter_collection.csv"))
    dur = durations(os.path.join(src, pre + "_trace", "run_kernel_trace.csv"))
    kernels = {}
    for k in sorted(set(fetch) | set(write) | set(dur)):
        f = fetch.get(k)
        w = write.get(k)
        traffic = (f * 2 + w) * 1024 if f is not None and w is not None else None
        kernels[k] = {"avg_ms": dur.get(k), "fetch_size_kb": f, "write_size_kb": w,
                      "hbm_read_bytes_corrected": f * 2 * 1024 if f is not None else None,
                      "hbm_write_bytes": w * 1024 if w is not None else None,
                      "hbm_traffic_bytes_per_launch": traffic}
    summary = {"source": "rocprofv3 --kernel-trace --stats; --pmc FETCH_SIZE; --pmc WRITE_SIZE (separate passes)",
               "correction": "FETCH_SIZE x2 on gfx950 (MI355X_MICROARCH.md §HBM)", "kernels": kernels}
    # the bench line of the profiled run itself (its workload keys the summary); a plain bench.log
    # only when the trace pass left none
    for name in (pre + "_trace.log", "bench.log"):
        p = os.path.join(src, name)
        if os.path.exists(p):
            for line in open(p):
                if line.startswith("{"):
                    summary.setdefault("bench_lines", []).append(json.loads(line))
        if summary.get("bench_lines"):
            break
    # the build the counters measured: the bench line's (pqh_build_id of the library that ran), else
    # the build record beside the in-tree library.  bench.py quotes a summary only for this build.
    builds = [ln.get("build") for ln in summary.get("bench_lines", []) if ln.get("build")]
    if builds:
        summary["build"] = builds[0]
    else:
        bi = os.path.join(root, "parquet-go_amd", "lib", "libpqhip.so.buildinfo.json")
        if os.path.exists(bi):
            summary["build"] = json.load(open(bi))
    json.dump(summary, open(os.path.join(out, "pmc_summary.json"), "w"), indent=1)
    print(json.dumps({k: v["hbm_traffic_bytes_per_launch"] for k, v in kernels.items()}, indent=1))


if __name__ == "__main__":
    main()
