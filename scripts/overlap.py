#!/usr/bin/env python3
"""Per-step kernel timeline of a rocprofv3 kernel trace (run_kernel_trace.csv): the steps are cut at
each k_prologue launch; for every kernel its start / end relative to the step's first kernel, its
queue, and how much of its span overlaps other kernels of the step.  Used to see whether the side
streams' kernels (k_ba_chain, the nesting passes, the DELTA pages) really run beside k_expand under
graph replay.

usage: python scripts/overlap.py <run_kernel_trace.csv> [--steps a:b] [--first-kernel k_prologue]
"""
import argparse
import csv
import statistics


def load(path):
    rows = []
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("pqhip::", "")
        if name.startswith("__amd"):
            continue
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, int(r["Queue_Id"])))
    rows.sort()
    return rows


def steps_of(rows, first):
    out, cur = [], None
    for r in rows:
        if r[2].startswith(first):
            cur = []
            out.append(cur)
        if cur is not None:
            cur.append(r)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", default=None, help="a:b slice of the steps to summarise")
    ap.add_argument("--first-kernel", default="k_prologue")
    a = ap.parse_args()
    steps = steps_of(load(a.trace), a.first_kernel)
    if a.steps:
        lo, hi = (int(x) if x else None for x in a.steps.split(":"))
        steps = steps[lo:hi]
    print(f"{len(steps)} steps")
    table = {}
    spans = []
    for st in steps:
        t0 = st[0][0]
        t1 = max(e for _, e, _, _ in st)
        spans.append((t1 - t0) / 1e6)
        busy = sum(e - s for s, e, _, _ in st)
        for s, e, n, q in st:
            ov = 0
            for s2, e2, n2, _ in st:
                if (s2, e2, n2) != (s, e, n):
                    ov = max(ov, min(e, e2) - max(s, s2))
            table.setdefault(n, []).append(((s - t0) / 1e6, (e - t0) / 1e6, (e - s) / 1e6, ov / 1e6, q))
        table.setdefault("_busy", []).append(busy / 1e6)
    print(f"step span (first start -> last end): median {statistics.median(spans):.4f} ms, "
          f"min {min(spans):.4f}, max {max(spans):.4f}")
    print(f"sum of kernel durations per step: median {statistics.median(table.pop('_busy')):.4f} ms")
    print(f"{'kernel':<16} {'queue':>5} {'start':>8} {'end':>8} {'dur':>8} {'max overlap':>11}  (ms, medians)")
    for n, v in sorted(table.items(), key=lambda kv: statistics.median(x[0] for x in kv[1])):
        med = lambda i: statistics.median(x[i] for x in v)  # noqa: E731
        print(f"{n:<16} {v[0][4]:>5} {med(0):8.4f} {med(1):8.4f} {med(2):8.4f} {med(3):11.4f}")


if __name__ == "__main__":
    main()
