"""Device-codec groundwork on the CPU.

* oracle.snappy_decode (a restatement of github.com/golang/snappy v0.0.4 decode.go, the
  reference's SNAPPY codec at compress.go:43-49) pinned against pyarrow's snappy on valid blocks,
  and its corruption rules on hand-built blocks;
* the host walker's device-codec layout (pqh_file_load_ex + PQH_LOAD_DEVICE_SNAPPY): every page's
  source bytes rebuild exactly the image the host-decompressing walker produces, and the checks the
  walker still makes itself (announced length, impossible expansion) fail the chunk as before.
"""
import numpy as np
import pyarrow as pa
import pytest

import fixtures
from oracle import oracle as O
from snappy_blocks import literal, copy1, copy2, copy4, block, sample_blocks



@pytest.fixture(autouse=True)
def every_page_on_the_device(monkeypatch):
    """The layout tests put every page of a device-codec chunk on the device (the walker's default
    keeps barely compressible pages on the host route; test_gpu_codec.py tests that rule)."""
    monkeypatch.setenv("PQH_DEVICE_CODEC_MAX_RATIO", "0")

def test_snappy_oracle_matches_pyarrow():
    for raw in sample_blocks():
        comp = pa.compress(raw, codec="snappy", asbytes=True)
        assert O.snappy_decode(comp) == raw


def test_snappy_oracle_hand_built():
    # literals of every length-header size, copies of every kind, overlapping copies
    raw = b"abcdefgh" * 3
    blk = block(len(raw) + 8 + 70000 + 5, literal(raw) + copy1(8, 8) + literal(b"z" * 70000) + copy2(5, 1))
    out = O.snappy_decode(blk)
    assert out == raw + raw[-8:] + b"z" * 70000 + b"z" * 5
    assert O.snappy_decode(block(10, literal(b"ab") + copy4(8, 2))) == b"ab" * 5
    for bad in (block(5, literal(b"abc")),                  # short output
                block(3, literal(b"abcd")),                 # literal past the output
                block(6, literal(b"ab") + copy2(4, 3)),     # offset before the output start
                block(6, literal(b"ab") + copy2(4, 0)),     # offset 0
                block(4, literal(b"ab"))[:-1],              # literal past the input
                b"\xff" * 11,                               # uvarint without a terminator
                b"\x80\x80\x80\x80\x80\x80\x80\x80\x80\x02"):  # 64-bit overflow
        with pytest.raises(O.SnappyCorrupt):
            O.snappy_decode(bad)
    # a non-canonical (padded) uvarint is accepted by binary.Uvarint
    assert O.snappy_decode(b"\x83\x80\x00" + literal(b"xyz")) == b"xyz"


@pytest.mark.parametrize("v2", [False, True])
def test_device_codec_layout(pq, v2):
    data = fixtures.flat_all_types(n=6000, v2=v2, codec=O.SNAPPY, page=16 * 1024, rows_per_group=3000)
    f = pq.native.File(data)
    cols = list(range(len(f.columns())))
    host = f.load(0, f.num_row_groups, cols)
    dev = f.load(0, f.num_row_groups, cols, device_snappy=True)
    hp, dp, cps = host.pages(), dev.pages(), dev.codec_pages()
    assert len(hp) == len(dp) == len(cps) and dev.image_bytes > 0
    hpay, src = host.payload(), dev.payload()
    snappy_pages = 0
    for a, b, c in zip(hp, dp, cps):
        assert (a.page_type, a.num_values, a.encoding, a.image_len) == (b.page_type, b.num_values, b.encoding, b.image_len)
        assert (c.image_offset, c.image_len) == (b.image_offset, b.image_len) and b.image_offset % 64 == 0
        want = bytes(hpay[a.image_offset:a.image_offset + a.image_len])
        s = bytes(src[c.src_offset:c.src_offset + c.src_len])
        if c.codec == O.SNAPPY:
            got = s[:c.raw_len] + O.snappy_decode(s[c.raw_len:])
            snappy_pages += 1
        else:
            got = s
        assert got == want
    assert snappy_pages == len(cps)


def test_device_codec_plain_files_keep_the_host_layout(pq):
    data = fixtures.flat_all_types(n=3000, codec=O.UNCOMPRESSED)
    f = pq.native.File(data)
    hb = f.load(0, f.num_row_groups, [0, 1], device_snappy=True)
    assert hb.codec_pages() == [] and hb.image_bytes == 0


def test_device_codec_walker_checks(pq):
    """Announced lengths that cannot match fail the chunk on the host, as decoding would."""
    W = pq.writer
    vals = np.arange(5000, dtype=np.int64)
    data = bytearray(W.flat([("v", W.Column(W.INT64, vals, use_dict=False), W.REQUIRED)], 5000, codec=O.SNAPPY))
    f = pq.native.File(bytes(data))
    hb = f.load(0, 1, [0], device_snappy=True)
    cp = hb.codec_pages()[0]
    assert hb.chunks()[0].host_status == 0
    # find the page's compressed block in the file and break its announced length
    blk = bytes(hb.payload()[cp.src_offset:cp.src_offset + cp.src_len])
    pos = bytes(data).find(blk)
    assert pos > 0
    data[pos] ^= 0x01
    for dev in (False, True):
        f2 = pq.native.File(bytes(data))
        hb2 = f2.load(0, 1, [0], device_snappy=dev)
        assert hb2.chunks()[0].host_status == {v: k for k, v in pq.native.STATUS.items()}["DECOMPRESS"]


def test_snappy_uvarint_header_parity(pq):
    """golang/snappy's decodedLen (binary.Uvarint, decode.go:32-36) on crafted page blocks: the host
    walker (codec.cpp, both the host-decompressing and the device-codec layout) fails or decodes
    every page exactly as the oracle does -- incl. the 10-byte header `88 80x8 02`, whose overflow
    bit a plain 7-bit-shift loop drops (decoded length 8 instead of ErrCorrupt).  The device codecs
    are checked against the same cases in test_gpu_codec.py."""
    import pqcraft
    from snappy_blocks import uvarint_header_cases

    cases = uvarint_header_cases()
    data = pqcraft.file_with_blocks([[(blk, size, size // 4)] for _, blk, size in cases], O.SNAPPY)
    fr = O.FileReader(data)
    f = pq.native.File(data)
    host = f.load(0, f.num_row_groups, [0])
    dev = f.load(0, f.num_row_groups, [0], device_snappy=True)
    hch, hpages, hpay = host.chunks(), host.pages(), host.payload()
    seen = set()
    for i, (name, blk, size) in enumerate(cases):
        och = fr.read_chunk(i, 0)
        assert hch[i].host_status == och.status, f"{name}: host {hch[i].host_status} vs oracle {och.status}"
        assert dev.chunks()[i].host_status == och.status, f"{name}: device-codec walker"
        if och.status == 0:
            p = hpages[hch[i].first_page]
            assert hpay[p.image_offset:p.image_offset + p.image_len].tobytes() == och.pages[0].image, name
        seen.add(och.status)
    assert seen == {0, O.ERR_DECOMPRESS}
    assert fr.read_chunk(4, 0).status == O.ERR_DECOMPRESS  # the 88 80x8 02 page


def test_host_crc_mismatch_validated(pq):
    """readPageBlock's CRC32 check (chunk_reader.go:173-177) under WithCRC32Validation
    (file_reader.go:134-139): one flipped bit in a CRC'd page fails its chunk with PQH_ERR_CRC on the
    host exactly when (and where) the oracle's walker does; without validation the flip only reaches
    the decoders, and unflipped chunks stay OK."""
    data = fixtures.flat_all_types(n=4000, v2=False, codec=O.UNCOMPRESSED, page=8 * 1024, rows_per_group=4000, crc=True)
    fr = O.FileReader(data)
    f = pq.native.File(data)
    ncols = len(f.columns())
    CRC = {v: k for k, v in pq.native.STATUS.items()}["CRC"]
    assert CRC == O.ERR_CRC
    rng = np.random.default_rng(8)
    flipped = 0
    for trial in range(8):
        ci = trial % ncols
        md = fr.row_groups[0][1][ci][3]
        lo, span = md.get(11, md[9]), md[7]
        buf = bytearray(data)
        pos = lo + span // 2 + int(rng.integers(-span // 4, span // 4 + 1))
        buf[pos] ^= 1 << int(rng.integers(0, 8))
        fr2, f2 = O.FileReader(bytes(buf)), pq.native.File(bytes(buf))
        hb = f2.load(0, 1, list(range(ncols)), validate_crc=True)
        for c, ch in enumerate(hb.chunks()):
            och = fr2.read_chunk(0, c, validate_crc=True)
            assert ch.host_status == och.status, (trial, c, ch.host_status, och.status)
            if c != ci:
                assert och.status == 0
        flipped += fr2.read_chunk(0, ci, validate_crc=True).status == O.ERR_CRC
    assert flipped >= 4, flipped
