"""Every decode path through a streaming ring (reader.RowGroupStream over PQH_CTX_STREAMING
contexts): one stream per slot (no side-stream branches: the PLAIN chains, nesting and DELTA pages
run in order on it), buffers packed in the slot's arena (conftest turns on the guard-gap check, so
a kernel writing past any buffer fails here), plan tables copied by pqh_batch_run_staged.  One row
group per range and two slots, so each slot's arena is reset and refilled by batches of different
shapes; every chunk compared with the oracle (values, offsets and bytes, levels, first error)."""
import pytest

import fixtures
from oracle import oracle as O
from parity import assert_chunk, oracle_chunk

pytestmark = pytest.mark.gpu

FILES = {
    "all_types_v1_plain": lambda: fixtures.flat_all_types(n=12000, v2=False, codec=0, page=16 * 1024, rows_per_group=3000),
    "all_types_v2_snappy": lambda: fixtures.flat_all_types(n=12000, v2=True, codec=1, page=16 * 1024, rows_per_group=3000),
    "all_types_v1_gzip": lambda: fixtures.flat_all_types(n=12000, v2=False, codec=2, page=16 * 1024, rows_per_group=3000),
    "c2_like": lambda: fixtures.flat_c2_like(n=40000, v2=True),
    "nested_list_map": lambda: fixtures.nested_list_map(n=6000, rows_per_group=1500),
    "deep_repeated": lambda: fixtures.deep_repeated(n=2000, depth=10)[0],
    "pyarrow_snappy": lambda: fixtures.pyarrow_file(n=20000, version="2.0", compression="SNAPPY"),
    "disagreeing_group": lambda: fixtures.disagreeing_group(),
}


@pytest.mark.parametrize("threaded", [False, True])
@pytest.mark.parametrize("device_codecs", [False, True])
@pytest.mark.parametrize("name", sorted(FILES))
def test_stream_every_path(pq, monkeypatch, name, device_codecs, threaded):
    if device_codecs:  # every SNAPPY / GZIP page to the device codecs, however compressible
        monkeypatch.setenv("PQH_DEVICE_CODEC_MAX_RATIO", "0")
    data = FILES[name]()
    f = pq.native.File(data)
    ncols = len(f.columns())
    fr = O.FileReader(data)
    st = pq.reader.RowGroupStream(f, list(range(ncols)), per_range=1, slots=2, threaded=threaded,
                                  device_snappy=device_codecs, device_gzip=device_codecs)
    try:
        seen = 0
        for a, b, batch, hb in st:
            for k, col in enumerate(st.column_data(batch, hb)):
                rg, ci = a + k // ncols, k % ncols
                assert col.status != pq.native.NOT_IMPLEMENTED, f"{name} rg{rg} {col.path}"
                assert_chunk(col, oracle_chunk(fr, rg, ci), where=f"{name} rg{rg} {col.path}")
                seen += 1
        assert seen == f.num_row_groups * ncols and f.num_row_groups >= 2, (seen, f.num_row_groups)
    finally:
        st.close()
        f.close()
