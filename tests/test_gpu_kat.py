"""The reference's bit-packing known answers (tests/golden/bitpack{32,64}_kat.json, from
bitpacking32_test.go:25-654 and bitpacking64_test.go:25-1744: width, packed bytes, the 8 values)
fed straight through the DEVICE unpack, compared with the KAT values themselves (not the oracle):

  * widths 0..32: hybrid bit-packed runs (hybridDecoder.readBitPackedRun, hybrid_decoder.go:132-140)
    through pqh_hybrid_decode -- the prologue's run walk + k_expand's unpack -- as a one-group run,
    after an RLE run (the run-list path), and all vectors of a width in one many-group run (the
    LDS-staged path), with the 8-value (levels) and 4-value (dictionary) groupings;
  * widths 0..64 (int64) and 0..32 (int32): DELTA_BINARY_PACKED miniblocks (deltabp_decoder.go:
    88-174) of a one-miniblock geometry holding the KAT group, decoded as INT64 / INT32 pages by the
    delta kernels in both modes: the values are the KAT values' running sums."""
import json
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
KAT32 = json.load(open(os.path.join(GOLD, "bitpack32_kat.json")))["vectors"]
KAT64 = json.load(open(os.path.join(GOLD, "bitpack64_kat.json")))["vectors"]


def uvarint(x):
    out = bytearray()
    while x >= 0x80:
        out.append((x & 0x7F) | 0x80)
        x >>= 7
    out.append(x)
    return bytes(out)


def zigzag(v):
    return uvarint((v << 1) ^ (v >> 63) if v >= 0 else ((-v) << 1) - 1)


@pytest.fixture(scope="module")
def ctx(pq):
    return pq.native.Context(0)


@pytest.mark.parametrize("group", [8, 4])
def test_hybrid_unpack_kat32(pq, ctx, group):
    checked = 0
    by_w = {}
    for k in KAT32:
        w, data = k["width"], bytes(k["data"])
        want = np.array(k["values"], dtype=np.int64).astype(np.uint32)
        by_w.setdefault(w, []).append((data, want))
        # one bit-packed group
        st, n, got = ctx.hybrid_decode(uvarint(3) + data, w, 8, group)
        assert st == 0 and n == 8 and np.array_equal(got, want), (w, got, want)
        # after an RLE run of 5 zeros: the tile's run list (decode8 / bp_value)
        st, n, got = ctx.hybrid_decode(uvarint(5 << 1) + b"\0" * ((w + 7) // 8) + uvarint(3) + data, w, 13, group)
        assert st == 0 and n == 13 and np.array_equal(got[5:], want) and not got[:5].any(), (w, got)
        checked += 1
    for w, vecs in by_w.items():  # every vector of a width in one run, repeated past a tile
        reps = 1500
        data = b"".join(d for d, _ in vecs) * reps
        want = np.concatenate([v for _, v in vecs] * reps)
        st, n, got = ctx.hybrid_decode(uvarint((len(vecs) * reps) << 1 | 1) + data, w, len(want), group)
        assert st == 0 and n == len(want) and np.array_equal(got, want), w
    assert checked == len(KAT32) and sorted(by_w) == list(range(33))


def _delta_page(w, data, bits):
    """blockSize 8, one miniblock: [header][block: minDelta 0, width w, the KAT bytes][block 2: all
    zero deltas] -- 9 values, so the read-ahead of the ninth delta finds block 2."""
    return (uvarint(8) + uvarint(1) + uvarint(9) + zigzag(0) + zigzag(0) + bytes([w]) + data + zigzag(0) + bytes([0]))


@pytest.mark.parametrize("mode", ["tiles", "streams", "split"])
@pytest.mark.parametrize("bits", [64, 32])
def test_delta_miniblock_kat(pq, ctx, bits, mode, monkeypatch):
    monkeypatch.setenv("PQH_DELTA_PAGE_MODE", "0" if mode == "tiles" else "1")
    monkeypatch.setenv("PQH_DELTA_SPLIT", "1" if mode == "split" else "0")
    N = pq.native
    kat = KAT64 if bits == 64 else KAT32
    col = (O.INT64 if bits == 64 else O.INT32, 0, 0, 0)
    blobs, chunks, pages, off = [], [], [], 0
    for k in kat:
        img = _delta_page(k["width"], bytes(k["data"]), bits)
        base = (off + 63) & ~63
        blobs.append(b"\0" * (base - off) + img)
        off = base + len(img)
        pages.append(N.Page(base, len(img), O.DATA_PAGE, 9, 5, 0, 0, len(chunks), 0))
        chunks.append(N.Chunk(N.Column(*col), len(pages) - 1, 1, 0, 0))
    arr = np.frombuffer(b"".join(blobs) + b"\0" * N.PAYLOAD_PAD, dtype=np.uint8).copy()
    d = ctx.malloc(len(arr))
    try:
        ctx.h2d(d, arr.ctypes.data, len(arr))
        ctx.sync()
        b = N.Batch.from_tables(ctx, chunks, pages, d, off)
        b.run()
        b.sync()
        mask = (1 << bits) - 1
        for i, k in enumerate(kat):
            o = b.chunk_out(i)
            assert o.status == 0, (k["width"], o.status, o.error_phase, o.error_index)
            got = ctx.d2h_array(o.values, 9 * bits // 8).view(np.uint64 if bits == 64 else np.uint32)
            acc, want = 0, [0]
            for v in k["values"]:  # value[i+1] = value[i] + delta[i] + minDelta, wrapping
                acc = (acc + v) & mask
                want.append(acc)
            assert got.tolist() == want, (k["width"], got.tolist(), want)
            r = O.decode_page(col, O.DATA_PAGE, 9, 5, 0, 0, pages_img(arr, pages[i]), None)
            assert r.status == 0 and r.values == got.tobytes()
        b.close()
    finally:
        ctx.free(d)


def pages_img(arr, pg):
    return arr[pg.image_offset:pg.image_offset + pg.image_len].tobytes()
