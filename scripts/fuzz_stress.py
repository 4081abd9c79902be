#!/usr/bin/env python3
"""Parity stress on the GPU: the mutation fuzzer of tests/test_gpu_parity.py (_fuzz_cases /
_run_cases: every mutated page its own chunk, status / first error / outputs vs the oracle) over
many seeds and fixtures, with PQH_FLAT on and off.  Prints one line per (fixture, seed); exits 1 on
the first mismatch (the assertion names the case).

  python scripts/fuzz_stress.py [--seeds 40]
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
    args = ap.parse_args()
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


if __name__ == "__main__":
    main()
