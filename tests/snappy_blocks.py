"""Hand-built snappy blocks (test-side encoder of the block format, golang/snappy decode.go):
elements of every kind and length-header size, and sample data for the codec tests."""
import numpy as np


def uvarint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def literal(data):
    n = len(data) - 1
    if n < 60:
        return bytes([n << 2]) + data
    k = 1 if n < 1 << 8 else 2 if n < 1 << 16 else 3 if n < 1 << 24 else 4
    return bytes([(59 + k) << 2]) + n.to_bytes(k, "little") + data


def copy1(length, offset):
    assert 4 <= length <= 11 and offset < 2048
    return bytes([1 | ((length - 4) << 2) | ((offset >> 8) << 5), offset & 0xFF])


def copy2(length, offset):
    assert 1 <= length <= 64 and offset < 65536
    return bytes([2 | ((length - 1) << 2)]) + offset.to_bytes(2, "little")


def copy4(length, offset):
    assert 1 <= length <= 64
    return bytes([3 | ((length - 1) << 2)]) + offset.to_bytes(4, "little")


def block(decoded_len, elements):
    return uvarint(decoded_len) + elements


def sample_blocks(seed=5):
    """Raw data of several kinds: random, runs, repeated words, small-alphabet text, empty."""
    rng = np.random.default_rng(seed)
    out = [b"", b"a", rng.bytes(100), rng.bytes(70000), bytes(100000), b"ab" * 20000]
    words = [rng.bytes(int(rng.integers(3, 12))) for _ in range(200)]
    out.append(b"".join(words[int(i)] for i in rng.integers(0, 200, 20000)))
    out.append(bytes(rng.integers(97, 101, 50000, dtype=np.uint8)))
    out.append(np.repeat(rng.integers(0, 256, 3000, dtype=np.uint8), rng.integers(1, 40, 3000)).tobytes())
    return out


def edge_blocks():
    """(block, raw or None if corrupt) exercising the decoder's paths: long literals (bulk copies),
    batches ending exactly at their output cap, overlapping copies of every offset, 4-byte offsets."""
    cases = []
    lit = bytes(range(256)) * 40  # 10240 bytes: a literal longer than a batch
    cases.append((block(len(lit), literal(lit)), lit))
    pre = b"0123456789abcdef"
    e = literal(pre)
    raw = bytearray(pre)
    for off in range(1, 17):
        for ln in (1, 4, 11, 33, 64):
            e += copy2(ln, off)
            for _ in range(ln):
                raw.append(raw[-off])
    cases.append((block(len(raw), e), bytes(raw)))
    e2 = literal(b"x" * 4095) + copy1(4, 1) + literal(b"y" * 5000) + copy4(64, 4000)
    r2 = bytearray(b"x" * 4095 + b"xxxx" + b"y" * 5000)
    for _ in range(64):
        r2.append(r2[-4000])
    cases.append((block(len(r2), e2), bytes(r2)))
    # many tiny elements (long chains per 64-byte window)
    from oracle import oracle as O

    e3, n3 = literal(b"q"), 1
    for i in range(5000):
        ln = 4 + i % 8
        e3 += copy1(ln, 1 + i % min(n3, 2000))
        n3 += ln
    cases.append((block(n3, e3), O.snappy_decode(block(n3, e3))))
    cases.append((block(20, literal(b"ab") + copy2(18, 2)), b"ab" * 10))
    cases.append((block(0, b""), b""))
    cases += multi_unit_blocks()
    return cases


def _decode(blk):
    from oracle import oracle as O

    return O.snappy_decode(blk)


def multi_unit_blocks():
    """Blocks for the multi-workgroup decoder (k_snap_spec / stitch / emit / fixup): 4 KiB input
    windows, 64 KiB output units.  Literals spanning many windows and straddling units, copies
    straddling units, copies reaching into earlier units (each unit depending on the one before:
    the in-order fixup), and a literal whose body is a run of valid-looking copy tags across a
    window start (the window's guessed entry is wrong: the stitch parses it again)."""
    rng = np.random.default_rng(21)
    cases = []
    # 1. one literal of 150 KiB (37 windows, three units)
    lit = rng.bytes(150000)
    cases.append(block(len(lit), literal(lit)))
    # 2. short elements, then a literal and a copy straddling the 64 KiB unit boundary
    e, n = literal(rng.bytes(1000)), 1000
    while n < 65536 - 300:
        e += copy2(64, 900)
        n += 64
    e += literal(rng.bytes(65536 - n + 200))
    n = 65536 + 200
    e += copy2(64, 3000) + literal(rng.bytes(5)) + copy1(11, 7)
    cases.append(block(n + 64 + 5 + 11, e))
    # 3. a copy straddling the unit boundary (starts 10 bytes before it)
    e, n = literal(rng.bytes(2000)), 2000
    while n + 64 <= 65536 - 10:
        e += copy2(64, 1999)
        n += 64
    e += literal(rng.bytes(65536 - 10 - n))
    n = 65536 - 10
    e += copy2(40, 65000) + copy1(5, 3)
    cases.append(block(n + 45, e))
    # 4. copies 70000 back: every unit after the first reads the unit before it (fixup chain)
    e, n = literal(rng.bytes(70000)), 70000
    while n < 260000:
        e += copy4(64, 70000) + literal(rng.bytes(3))
        n += 67
    cases.append(block(n, e))
    # 5. a literal of copy1 tags across the window start at 4096 (the guessed entry is a false chain)
    e = literal(rng.bytes(3700))
    fake = bytes([1, 0]) * 300
    e += literal(fake) + copy2(30, 100) + literal(rng.bytes(9000)) + copy2(64, 5000)
    cases.append(block(3700 + 600 + 30 + 9000 + 64, e))
    # 6. the same trick at every window start of a long block
    e, n = b"", 0
    for _ in range(40):
        body = bytes([1, 0]) * 200 + rng.bytes(3000)
        e += literal(body) + copy2(17, 333) + copy1(9, 1)
        n += len(body) + 26
    cases.append(block(n, e))
    # 7. random short elements over 300 KiB of output (many units, many windows)
    e, n = literal(rng.bytes(64)), 64
    while n < 300000:
        k = int(rng.integers(0, 4))
        if k == 0:
            ln = int(rng.integers(1, 80))
            e += literal(rng.bytes(ln))
        elif k == 1:
            ln = int(rng.integers(4, 12))
            e += copy1(ln, int(rng.integers(1, min(n, 2047) + 1)))
        elif k == 2:
            ln = int(rng.integers(1, 65))
            e += copy2(ln, int(rng.integers(1, min(n, 65535) + 1)))
        else:
            ln = int(rng.integers(1, 65))
            e += copy4(ln, int(rng.integers(1, n + 1)))
        n += ln
    cases.append(block(n, e))
    return [(b, _decode(b)) for b in cases]


def uvarint_header_cases():
    """(name, block, page size) around golang/snappy's decodedLen = encoding/binary.Uvarint
    (vendor/github.com/golang/snappy/decode.go:32-36): non-minimal and 10-byte headers are valid
    while their 10th byte is 0 or 1; a 10th byte > 1 overflows 64 bits and an 11th byte is never read
    -- both ErrCorrupt, whatever the low bits say.  Body: one 8-byte literal."""
    body = literal(b"abcdefgh")
    cont = b"\x80"
    return [
        ("minimal", b"\x08" + body, 8),
        ("3-byte", b"\x88\x80\x00" + body, 8),
        ("10-byte, last 0", b"\x88" + cont * 8 + b"\x00" + body, 8),
        ("10-byte, last 1 (> 2^32)", b"\x88" + cont * 8 + b"\x01" + body, 8),
        ("10-byte, last 2 (overflow, low bits 8)", b"\x88" + cont * 8 + b"\x02" + body, 8),
        ("10-byte, last 0x7f (overflow)", b"\x88" + cont * 8 + b"\x7f" + body, 8),
        ("11-byte", b"\x88" + cont * 9 + b"\x00" + body, 8),
        ("10 continuation bytes", b"\x88" + cont * 9 + b"\x80" + body, 8),
        ("5-byte 2^32 - 1", b"\xff\xff\xff\xff\x0f" + body, 8),
        ("5-byte 2^32", b"\x80\x80\x80\x80\x10" + body, 8),
        ("truncated header", b"\x88\x80", 8),
    ]


def far_copy_block(far=(1 << 24) + 777, tail=200_000, seed=31):
    """A valid block of more than 16 MiB whose copy4 elements reach 2^24 bytes back and further
    (golang/snappy accepts any offset up to 2^32 within the output, decode_other.go:75-85; Go and C++
    encoders never emit one, other encoders may).  Returns (block, raw)."""
    rng = np.random.default_rng(seed)
    head = rng.bytes(far + 64)
    e = bytearray(literal(head))
    raw = bytearray(head)
    n = len(raw)
    while n < far + 64 + tail:
        for off in (far, far + 13, (1 << 24), (1 << 24) - 1, 5):
            ln = int(rng.integers(1, 65))
            e += copy4(ln, off)
            for _ in range(ln):
                raw.append(raw[-off])
            n += ln
        lit = rng.bytes(int(rng.integers(1, 300)))
        e += literal(lit)
        raw += lit
        n += len(lit)
    return block(len(raw), bytes(e)), bytes(raw)
