"""bench.py's roofline.traffic comes from the committed rocprofv3 PMC summaries (profiles/*/
pmc_summary.json, shipped to the GPU box): the headline C2 workload must find one, and its HBM
traffic per k_expand launch must stay close to the algorithmic bytes (no wasted re-reads)."""
import importlib.util
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    argv = sys.argv
    sys.argv = ["bench.py"]
    try:
        spec.loader.exec_module(m)
    finally:
        sys.argv = argv
    return m


def test_c2_traffic_summary_found():
    m = _bench()
    src = None
    for tag in sorted(os.listdir(os.path.join(ROOT, "profiles")), reverse=True):
        p = os.path.join(ROOT, "profiles", tag, "pmc_summary.json")
        if os.path.exists(p):
            s = json.load(open(p))
            lines = s.get("bench_lines") or []
            if lines and lines[0]["config"]["workload"].startswith("C2:"):
                src = lines[0]
                break
    assert src is not None, "no C2 PMC summary under profiles/"
    traffic, where = m.pmc_traffic("k_expand", src["config"]["workload"], src["config"]["rows_per_gpu"])
    assert traffic and where.endswith("pmc_summary.json")
    algo = src["roofline"]["algo_bytes_per_launch"]
    assert 0.95 * algo <= traffic <= 1.10 * algo
