"""The test-side DELTA_BINARY_PACKED builder (tests/delta_streams.py) against the oracle's
restatement of deltaBitPackDecoder32/64 (deltabp_decoder.go:13-333): every geometry the device
parity tests use must round-trip, except the reference's read-ahead failure when the last block is
exactly full ((n-1) % blockSize == 0), which must fail at index n-1."""
import numpy as np
import pytest

import delta_streams as DS
from oracle import oracle as O

GEOMS = [(128, 4), (128, 1), (256, 8), (2048, 4), (64, 2), (128, 16), (96, 3), (24, 3), (12, 3), (32, 1)]


@pytest.mark.parametrize("bs,mbc", GEOMS)
@pytest.mark.parametrize("bits", [32, 64])
def test_roundtrip(bs, mbc, bits):
    rng = np.random.default_rng(bs * 31 + mbc + bits)
    for n in (1, 2, 8, 9, 100, 257, 1500):
        for kind in ("const", "small", "full", "mixed"):
            for finish in ("omit", "full"):
                vals = DS.random_values(rng, n, bits, kind)
                st, out, vc = O.delta_decode(DS.encode(vals, bits, bs, mbc, finish), n, bits)
                assert vc == n
                mask = (1 << bits) - 1
                want = np.array([DS._signed(int(v) & mask, bits) for v in vals],
                                dtype=np.int64 if bits == 64 else np.int32)
                if (bs // mbc) % 8:
                    continue  # miniblocks of < 8 values: the padding skip reads past them (invalid stream)
                if (n - 1) % bs == 0:
                    assert st != 0 and len(out) == n - 1, (n, bs, st, len(out))
                    np.testing.assert_array_equal(out, want[: n - 1])
                else:
                    assert st == 0, (n, bs, mbc, kind, finish, st)
                    np.testing.assert_array_equal(out, want)


def test_matches_writer_layout():
    """(128, 4) 'omit' decodes identically to the generator's reference-writer layout."""
    from conftest import load_package

    W = load_package().writer
    rng = np.random.default_rng(5)
    vals = np.cumsum(rng.integers(-100, 100, 5000)).astype(np.int64)
    a = O.delta_decode(DS.encode(list(vals), 64, 128, 4, "omit"), 5000, 64)
    b = O.delta_decode(W.delta_encode(vals, 64), 5000, 64)
    assert a[0] == b[0] == 0
    np.testing.assert_array_equal(a[1], b[1])
