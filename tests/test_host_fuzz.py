"""Mutation fuzzing of whole files through the host boundary (CPU): footer, schema, page headers
and page walk of the product (libpqhip's C++ walker) against the oracle's restatement.  Random byte
edits land in the thrift footer, the page headers and the page data; for every mutant both
implementations must agree on NewFileReader failing or not, on the columns and row groups, on
readRowGroupData's column checks and on where each chunk's walk ends (test_fuzz_fixtures rules).
Run under ASan + UBSan by scripts/run_sanitized.sh."""
import numpy as np
import pytest

import fixtures
from test_fuzz_fixtures import test_fixture_footer_schema_and_walk as _compare


def _mutants(data, rng, n):
    d = np.frombuffer(data, dtype=np.uint8)
    flen = int.from_bytes(data[-8:-4], "little")
    foot0 = max(4, len(data) - 8 - flen)
    for _ in range(n):
        m = d.copy()
        for _ in range(int(rng.integers(1, 4))):
            where = rng.random()
            if where < 0.5:  # the footer (thrift FileMetaData)
                i = int(rng.integers(foot0, len(data) - 8))
            elif where < 0.6:  # the footer length / magics
                i = int(rng.choice([0, 1, 2, 3, len(data) - 8, len(data) - 7, len(data) - 5, len(data) - 1]))
            else:  # anywhere in the pages (headers and data)
                i = int(rng.integers(4, foot0))
            m[i] = rng.integers(0, 256) if rng.random() < 0.7 else m[i] ^ (1 << int(rng.integers(0, 8)))
        yield m.tobytes()


@pytest.mark.parametrize("case", ["v1", "v2-snappy", "gzip", "nested"])
def test_host_walk_mutations(pq, case):
    rng = np.random.default_rng({"v1": 101, "v2-snappy": 102, "gzip": 103, "nested": 104}[case])
    if case == "nested":
        data = fixtures.nested_list_map(n=600)
    else:
        data = fixtures.flat_all_types(n=1500, v2=case == "v2-snappy", codec={"v1": 0, "v2-snappy": 1, "gzip": 2}[case],
                                       page=4 * 1024, rows_per_group=800)
    opened = 0
    for k, m in enumerate(_mutants(data, rng, 150)):
        _compare(pq, {"file": None, "length": len(m), "data": m})
        opened += 1
    assert opened == 150
