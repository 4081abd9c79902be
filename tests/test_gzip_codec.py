"""GZIP, the reference's codec at compress.go:64-77 (Go compress/gzip, multistream), on the CPU:

* the oracle's restatement (oracle.gzip_decode: Go's member / header / trailer rules around a raw
  DEFLATE inflate) equals Python's gzip module on every valid stream, and rejects what Go rejects
  where Python's module differs (zero padding after a member);
* the host walker's GZIP path (codec.cpp gzip_into, the reference's readPageBlock) decodes or
  fails every crafted page exactly as the oracle does, bytes included (tests/gzip_blocks.py:
  zlib streams of every level / strategy / flush mode, multistream, every header field, hand-built
  DEFLATE blocks, each error class, seeded mutants);
* with PQH_LOAD_DEVICE_GZIP the walker leaves GZIP pages compressed in the device-codec layout.
The device decoder (k_gzip) is checked against the same cases in test_gpu_codec.py."""
import gzip

import pytest

import gzip_blocks as G
import pqcraft
from oracle import oracle as O

DECOMPRESS = 23



@pytest.fixture(autouse=True)
def every_page_on_the_device(monkeypatch):
    """The layout tests put every page of a device-codec chunk on the device (the walker's default
    keeps barely compressible pages on the host route; test_gpu_codec.py tests that rule)."""
    monkeypatch.setenv("PQH_DEVICE_CODEC_MAX_RATIO", "0")

def expected(stream, size):
    """(status, bytes) the reference's readPageBlock gives a page of `size` bytes."""
    try:
        raw = O.gzip_decode(stream)
    except O.GzipCorrupt:
        return DECOMPRESS, None
    if size is not None and len(raw) != size:
        return DECOMPRESS, None
    return 0, raw


def all_cases():
    valid = [(n, s, len(O.gzip_decode(s))) for n, s, _ in G.valid_cases()]
    return valid + G.error_cases() + G.mutants(valid[::3], per=6)


def test_oracle_matches_python_gzip_on_valid_streams():
    cases = G.valid_cases()
    assert len(cases) > 60
    for name, s, _ in cases:
        assert O.gzip_decode(s) == gzip.decompress(s), name


def test_oracle_error_classes():
    for name, s, size in G.error_cases():
        st, _ = expected(s, size)
        assert st == DECOMPRESS, name
    good = G.gz(b"hello world")
    # Python's gzip module skips zero padding after a member; Go's reader does not
    assert gzip.decompress(good + b"\0") == b"hello world"
    with pytest.raises(O.GzipCorrupt):
        O.gzip_decode(good + b"\0")


def _load(pq, cases, **kw):
    chunks = [[(s, size, 0)] for _, s, size in cases]
    data = pqcraft.file_with_blocks(chunks, O.GZIP)
    f = pq.native.File(data)
    return f, f.load(0, f.num_row_groups, [0], **kw)


def test_host_gzip_pages_match_oracle(pq):
    cases = all_cases()
    f, hb = _load(pq, cases)
    try:
        chunks, pages, payload = hb.chunks(), hb.pages(), hb.payload()
        assert len(chunks) == len(cases)
        ok = bad = 0
        for i, (name, s, size) in enumerate(cases):
            st, raw = expected(s, size)
            c = chunks[i]
            if st:
                assert c.host_status == DECOMPRESS and c.num_pages == 0, f"{name}: {c.host_status}"
                bad += 1
                continue
            assert c.host_status == 0 and c.num_pages == 1, f"{name}: {c.host_status}"
            p = pages[c.first_page]
            assert payload[p.image_offset:p.image_offset + p.image_len].tobytes() == raw, name
            ok += 1
        assert ok > 60 and bad > 40, (ok, bad)
    finally:
        hb.close()
        f.close()


def test_device_gzip_layout(pq):
    cases = [(n, s, len(O.gzip_decode(s))) for n, s, _ in G.valid_cases()[:12]]
    f, hb = _load(pq, cases, device_gzip=True)
    try:
        cps, pages, payload = hb.codec_pages(), hb.pages(), hb.payload()
        assert len(cps) == len(cases) == len(pages)
        for (name, s, size), cp, p in zip(cases, cps, pages):
            assert cp.codec == O.GZIP and cp.raw_len == 0, name
            assert cp.src_len == len(s) and cp.image_len == size == p.image_len, name
            assert payload[cp.src_offset:cp.src_offset + cp.src_len].tobytes() == s, name
            assert cp.image_offset == p.image_offset
        assert hb.image_bytes >= sum(c[2] for c in cases)
    finally:
        hb.close()
        f.close()
    # device_snappy alone keeps GZIP chunks on the host
    f, hb = _load(pq, cases, device_snappy=True)
    try:
        assert hb.codec_pages() == [] and hb.image_bytes == 0
    finally:
        hb.close()
        f.close()
