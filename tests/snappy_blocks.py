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
    return cases
