"""GZIP streams for the device-codec tests (k_gzip vs oracle.gzip_decode, the restatement of the
reference's codec at compress.go:64-77): valid members from zlib at every level / strategy /
flush mode, multistream concatenations, every optional header field, and hand-built DEFLATE
blocks and malformed members covering each error class.  Each case is (name, stream, size) where
size is the page's uncompressed size the decoder must reach (the size check of newBlockReader,
compress.go:131-152); None = the true decoded size."""
import struct
import zlib

import numpy as np


def gz(data, level=6, strategy=zlib.Z_DEFAULT_STRATEGY, mem=8, flushes=()):
    """One gzip member from zlib (wbits 31: gzip wrapper).  flushes: [(offset, mode)] flush points."""
    c = zlib.compressobj(level, zlib.DEFLATED, 31, mem, strategy)
    out, pos = [], 0
    for off, mode in sorted(flushes):
        out.append(c.compress(data[pos:off]))
        out.append(c.flush(mode))
        pos = off
    out.append(c.compress(data[pos:]))
    out.append(c.flush())
    return b"".join(out)


class Bits:
    """DEFLATE bit writer: fields LSB first, Huffman codes MSB first (RFC 1951 §3.1.1)."""

    def __init__(self):
        self.v, self.n = 0, 0

    def put(self, x, k):
        self.v |= (x & ((1 << k) - 1)) << self.n
        self.n += k

    def huff(self, code, k):
        self.put(int(format(code, f"0{k}b")[::-1], 2), k)

    def align(self):
        self.n = (self.n + 7) & ~7

    def bytes(self):
        return self.v.to_bytes((self.n + 7) // 8, "little")


def fixed_lit(b, s):
    if s < 144:
        b.huff(0x30 + s, 8)
    elif s < 256:
        b.huff(0x190 + s - 144, 9)
    elif s < 280:
        b.huff(s - 256, 7)
    else:
        b.huff(0xC0 + s - 280, 8)


LBASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195,
         227, 258]
LEXT = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DBASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073,
         4097, 6145, 8193, 12289, 16385, 24577]
DEXT = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13]


def fixed_match(b, length, dist):
    i = max(k for k in range(29) if LBASE[k] <= length)
    if length == 258:
        i = 28
    fixed_lit(b, 257 + i)
    b.put(length - LBASE[i], LEXT[i])
    j = max(k for k in range(30) if DBASE[k] <= dist)
    b.huff(j, 5)
    b.put(dist - DBASE[j], DEXT[j])


def fixed_block(symbols, final=True, b=None):
    """symbols: ints (literals / 256 = end) or (length, distance) pairs; returns raw DEFLATE."""
    b = b or Bits()
    b.put(1 if final else 0, 1)
    b.put(1, 2)
    for s in symbols:
        if isinstance(s, tuple):
            fixed_match(b, *s)
        else:
            fixed_lit(b, s)
    return b


def member(raw_deflate, data=None, crc=None, size=None, flg=0, extra=b"", name=None, comment=None, hcrc=None):
    """A gzip member around raw DEFLATE bytes; the trailer from `data` unless crc / size given."""
    h = bytearray(b"\x1f\x8b\x08" + bytes([flg]) + b"\0\0\0\0\0\xff")
    if flg & 4:
        h += struct.pack("<H", len(extra)) + extra
    if flg & 8:
        h += name if name is not None else b"name\0"
    if flg & 16:
        h += comment if comment is not None else b"comment\0"
    if flg & 2:
        h += struct.pack("<H", (zlib.crc32(bytes(h)) & 0xFFFF) if hcrc is None else hcrc)
    data = data if data is not None else b""
    c = zlib.crc32(data) & 0xFFFFFFFF if crc is None else crc
    s = len(data) & 0xFFFFFFFF if size is None else size
    return bytes(h) + raw_deflate + struct.pack("<II", c, s)


def raw(data, level=6, strategy=zlib.Z_DEFAULT_STRATEGY):
    c = zlib.compressobj(level, zlib.DEFLATED, -15, 8, strategy)
    return c.compress(data) + c.flush()


def _text(rng, n):
    words = [bytes(rng.integers(97, 123, int(rng.integers(2, 10))).astype(np.uint8)) for _ in range(400)]
    out, k = bytearray(), 0
    while len(out) < n:
        out += words[int(rng.integers(0, len(words)))] + b" "
        k += 1
        if k % 13 == 0:
            out += b"%d," % int(rng.integers(0, 10 ** 6))
    return bytes(out[:n])


def payloads(seed=5):
    rng = np.random.default_rng(seed)
    return [
        ("empty", b""),
        ("one", b"x"),
        ("text1k", _text(rng, 1000)),
        ("text200k", _text(rng, 200_000)),
        ("random64k", rng.bytes(65_536)),
        ("random300k", rng.bytes(300_000)),
        ("zeros1m", bytes(1 << 20)),
        ("ints", rng.integers(0, 1000, 50_000).astype(np.int32).tobytes()),
        ("repeat", (b"abcdefghij" * 30_000)[:299_999]),
        ("far", rng.bytes(20_000) + rng.bytes(5_000) + bytes(100) + rng.bytes(40_000)),
    ]


def valid_cases(seed=5):
    """Valid streams: (name, stream, None)."""
    out = []
    pl = payloads(seed)
    for name, data in pl:
        for level in (0, 1, 6, 9):
            out.append((f"{name}-l{level}", gz(data, level), None))
        if len(data) > 10:
            out.append((f"{name}-huffonly", gz(data, 6, zlib.Z_HUFFMAN_ONLY), None))
            out.append((f"{name}-rle", gz(data, 6, zlib.Z_RLE), None))
            out.append((f"{name}-fixed", gz(data, 6, zlib.Z_FIXED), None))
            out.append((f"{name}-mem1", gz(data, 9, mem=1), None))
            cut = len(data) // 3
            out.append((f"{name}-sync", gz(data, 6, flushes=[(cut, zlib.Z_SYNC_FLUSH), (2 * cut, zlib.Z_FULL_FLUSH)]), None))
    d = dict(pl)
    # multistream: members back to back (one with no output at all)
    out.append(("multi2", gz(d["text1k"]) + gz(d["ints"], 1), None))
    out.append(("multi-empty-mid", gz(d["text1k"]) + gz(b"") + gz(d["repeat"], 0), None))
    out.append(("multi5", b"".join(gz(d["text200k"][i * 1000:(i + 1) * 7000], [0, 1, 6, 9, 6][i]) for i in range(5)), None))
    # every optional header field (reserved flag bits are ignored by Go's reader)
    txt = d["text1k"]
    r6 = raw(txt)
    out.append(("hdr-name", member(r6, txt, flg=8), None))
    out.append(("hdr-comment", member(r6, txt, flg=16), None))
    out.append(("hdr-extra", member(r6, txt, flg=4, extra=b"ab\x04\x00wxyz"), None))
    out.append(("hdr-extra-big", member(r6, txt, flg=4, extra=bytes(range(256)) * 40), None))
    out.append(("hdr-all", member(r6, txt, flg=2 | 4 | 8 | 16, extra=b"e"), None))
    out.append(("hdr-reserved", member(r6, txt, flg=0xE0), None))
    out.append(("hdr-name511", member(r6, txt, flg=8, name=b"n" * 511 + b"\0"), None))
    # hand-built fixed blocks: overlapping copies, maximum length / distance
    data = b"ab" + b"ab" * 200
    blk = fixed_block([97, 98, (258, 2), (142, 2), 256]).bytes()
    out.append(("fixed-overlap", member(blk, data), None))
    big = rng_bytes(32768, 3)
    blk = raw(big, 0) + b""  # a stored stream of 32 KiB ...
    b2 = Bits()
    b2.put(0, 1)
    b2.put(0, 2)
    b2.align()
    b2.put(len(big), 16)
    b2.put(~len(big) & 0xFFFF, 16)
    stored = b2.bytes() + big
    tail = fixed_block([(258, 32768), (3, 32768), 256]).bytes()
    out.append(("max-distance", member(stored + tail, big + big[:258] + big[258:261]), None))
    return out + stored_mix_cases()


def stored_block(data, final=False):
    """A byte-aligned stored block (BFINAL, BTYPE 00, LEN, NLEN, bytes)."""
    return bytes([1 if final else 0]) + struct.pack("<HH", len(data), ~len(data) & 0xFFFF) + data


def stored_mix_cases(seed=8):
    """Streams whose stored bytes lie outside k_gzip's 8 KiB stage within one serial batch (the
    HBM `src` read-back path of gz_batch): runs of empty stored blocks that carry the input ahead
    without output, then stored data starting near the stage's end; many tiny stored blocks (the
    1024-token batch spans more input than the stage); Huffman segments (full flushes) between
    them.  (name, stream, None)."""
    rng = np.random.default_rng(seed)
    out = []
    for empties, ln in ((1400, 8000), (1500, 8191), (1510, 5000), (1000, 8192), (1509, 1), (700, 20000)):
        data = rng.bytes(ln)
        raw_ = stored_block(b"") * empties + stored_block(data) + stored_block(b"", final=True)
        out.append((f"stored-after-{empties}-empty-{ln}", member(raw_, data), None))
    for sizes in ((1, 16), (4, 9), (0, 3)):
        chunks = [rng.bytes(int(rng.integers(sizes[0], sizes[1] + 1))) for _ in range(3000)]
        data = b"".join(chunks)
        raw_ = b"".join(stored_block(c) for c in chunks) + stored_block(b"", final=True)
        out.append((f"stored-tiny-{sizes[0]}-{sizes[1]}", member(raw_, data), None))
    # Huffman segments (each its own compressor, ended by a full flush: byte aligned, no reference
    # into earlier segments), empty stored blocks and stored data, interleaved
    parts, data = [], b""
    for k in range(12):
        t = _text(rng, int(rng.integers(100, 30000)))
        c = zlib.compressobj(int(rng.integers(1, 10)), zlib.DEFLATED, -15)
        parts.append(c.compress(t) + c.flush(zlib.Z_FULL_FLUSH))
        d2 = rng.bytes(int(rng.integers(1, 12000)))
        parts.append(stored_block(b"") * int(rng.integers(0, 1600)) + stored_block(d2))
        data += t + d2
    out.append(("stored-huffman-mix", member(b"".join(parts) + stored_block(b"", final=True), data), None))
    return out


def rng_bytes(n, seed):
    return np.random.default_rng(seed).bytes(n)


def error_cases(seed=6):
    """Malformed streams (and valid ones at a wrong page size): (name, stream, size)."""
    rng = np.random.default_rng(seed)
    txt = _text(rng, 5000)
    good = gz(txt)
    r6 = raw(txt)
    out = [
        ("empty-input", b"", 0),
        ("short-header", good[:9], len(txt)),
        ("bad-magic", b"\x1f\x8c" + good[2:], len(txt)),
        ("bad-method", good[:2] + b"\x07" + good[3:], len(txt)),
        ("truncated-body", good[:len(good) // 2], len(txt)),
        ("truncated-trailer", good[:-3], len(txt)),
        ("no-trailer", good[:-8], len(txt)),
        ("bad-crc", good[:-8] + struct.pack("<I", (zlib.crc32(txt) ^ 1) & 0xFFFFFFFF) + good[-4:], len(txt)),
        ("bad-isize", good[:-4] + struct.pack("<I", len(txt) + 1), len(txt)),
        ("trailing-zero", good + b"\0", len(txt)),
        ("trailing-zeros10", good + bytes(10), len(txt)),
        ("trailing-garbage", good + b"garbage!!!!!", len(txt)),
        ("size-short", good, len(txt) - 1),
        ("size-long", good, len(txt) + 1),
        ("size-zero", good, 0),
        ("name-no-nul", member(r6, txt, flg=8, name=b"abc"), len(txt)),
        ("name-512", member(r6, txt, flg=8, name=b"n" * 512 + b"\0"), len(txt)),
        ("extra-short", (member(r6, txt, flg=4, extra=b"abcdef"))[:14], len(txt)),
        ("hcrc-bad", member(r6, txt, flg=2, hcrc=0x1234), len(txt)),
        ("second-member-bad", good + b"\x1f\x8b\x08\x00" + bytes(6) + b"\x07", len(txt)),
    ]
    b = Bits()
    b.put(1, 1)
    b.put(3, 2)  # block type 3
    out.append(("btype3", member(b.bytes() + bytes(4), b""), 0))
    b = Bits()
    b.put(1, 1)
    b.put(0, 2)
    b.align()
    b.put(5, 16)
    b.put(5, 16)  # NLEN != ~LEN
    out.append(("stored-nlen", member(b.bytes() + b"hello", b"hello"), 5))
    out.append(("too-far", member(fixed_block([97, (3, 2), 256]).bytes(), b"aaaa"), 4))
    out.append(("too-far-member", gz(b"xyz") + member(fixed_block([97, (3, 4), 256]).bytes(), b"aaaa"), 7))
    out.append(("bad-dist-code", member(_fixed_with_dist_code(30), b"aaaa"), 4))
    out.append(("bad-len-code", member(_fixed_with_len_code(286), b"a"), 1))
    out.append(("hlit-287", member(_dyn_header(30, 0, 15), b""), 0))
    out.append(("hdist-31", member(_dyn_header(0, 30, 15), b""), 0))
    out.append(("no-final", member(fixed_block([97, 256], final=False).bytes(), b"a"), 1))
    # a valid member whose trailer is followed by an incomplete second member
    out.append(("second-truncated", good + gz(txt)[:30], 2 * len(txt)))
    return out


def _fixed_with_dist_code(code):
    b = Bits()
    b.put(1, 1)
    b.put(1, 2)
    fixed_lit(b, 97)
    fixed_lit(b, 257)  # length 3
    b.huff(code, 5)  # distance code 30 / 31: invalid
    fixed_lit(b, 256)
    return b.bytes()


def _fixed_with_len_code(code):
    b = Bits()
    b.put(1, 1)
    b.put(1, 2)
    fixed_lit(b, 97)
    fixed_lit(b, code)  # 286 / 287: invalid
    b.huff(0, 5)
    fixed_lit(b, 256)
    return b.bytes()


def _dyn_header(hlit, hdist, hclen):
    b = Bits()
    b.put(1, 1)
    b.put(2, 2)
    b.put(hlit, 5)
    b.put(hdist, 5)
    b.put(hclen, 4)
    for _ in range(hclen + 4):
        b.put(4, 3)
    return b.bytes() + bytes(64)


def mutants(streams, seed=7, per=6):
    """Seeded corruptions of valid streams: byte sets, truncations, bit flips (page size kept)."""
    rng = np.random.default_rng(seed)
    out = []
    for name, s, size in streams:
        true = size
        for k in range(per):
            b = bytearray(s)
            mode = k % 3
            if mode == 0 and len(b) > 10:
                for _ in range(int(rng.integers(1, 4))):
                    b[int(rng.integers(10, len(b)))] = int(rng.integers(0, 256))
            elif mode == 1:
                b = b[:int(rng.integers(0, len(b) + 1))]
            elif len(b) > 10:
                i = int(rng.integers(10, len(b)))
                b[i] ^= 1 << int(rng.integers(0, 8))
            out.append((f"{name}-mut{k}", bytes(b), true))
    return out
