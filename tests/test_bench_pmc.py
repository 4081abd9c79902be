"""bench.py's roofline.traffic comes from the committed rocprofv3 PMC summaries (profiles/*/
pmc_summary.json, shipped to the GPU box), and only from a summary measured on THIS build: each
summary is stamped with the source hash of the library that ran (pqh_build_id), and a summary of
any other build is refused (traffic null, with the reason)."""
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
    m.package()
    return m


def _summary(tmp, tag, workload, rows, traffic, source_hash):
    d = tmp / "profiles" / tag
    d.mkdir(parents=True)
    s = {"kernels": {"k_expand": {"hbm_traffic_bytes_per_launch": traffic}},
         "bench_lines": [{"config": {"workload": workload, "rows_per_gpu": rows}}]}
    if source_hash is not None:
        s["build"] = {"source_hash": source_hash}
    (d / "pmc_summary.json").write_text(json.dumps(s))


def test_build_id_is_the_source_hash():
    m = _bench()
    from parquet_go_amd import build, native

    info = native.build_info()
    assert info["source_hash"] == build.source_hash() and len(info["source_hash"]) == 16
    assert m is not None


def test_traffic_only_from_this_build(tmp_path):
    m = _bench()
    from parquet_go_amd import native

    mine = native.build_info()["source_hash"]
    m.ROOT = str(tmp_path)
    _summary(tmp_path, "r09_new", "W", 10, 111, "0123456789abcdef")  # newer, another build
    _summary(tmp_path, "r08_unstamped", "W", 10, 222, None)
    traffic, why = m.pmc_traffic("k_expand", "W", 10)
    assert traffic is None and "refused" in why and "r09_new" in why and "unstamped" in why
    _summary(tmp_path, "r07_this_build", "W", 10, 333, mine)
    traffic, src = m.pmc_traffic("k_expand", "W", 10)
    assert traffic == 333 and src.startswith("profiles/r07_this_build/") and mine in src
    assert m.pmc_traffic("k_expand", "W", 11)[0] is None  # another workload size


def test_committed_summaries_are_stamped_or_refused():
    """Every committed C2 summary either carries a build stamp or is refused as unstamped."""
    m = _bench()
    for tag in sorted(os.listdir(os.path.join(ROOT, "profiles"))):
        p = os.path.join(ROOT, "profiles", tag, "pmc_summary.json")
        if not os.path.exists(p):
            continue
        s = json.load(open(p))
        lines = s.get("bench_lines") or []
        if not lines or not lines[0]["config"]["workload"].startswith("C2:"):
            continue
        traffic, where = m.pmc_traffic("k_expand", lines[0]["config"]["workload"], lines[0]["config"]["rows_per_gpu"])
        if traffic is None:
            assert "no PMC summary of this build" in where
        else:
            assert where.endswith(")") and "pmc_summary.json" in where
