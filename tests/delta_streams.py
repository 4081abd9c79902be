"""Test-side DELTA_BINARY_PACKED stream builder with arbitrary geometry.

The reference writer always emits blocks of 128 values in 4 miniblocks (deltabp_encoder.go); the
reference DECODER (deltabp_decoder.go:13-333) accepts any block size / miniblock count, so the
parity tests also feed it layouts the writer never produces: other block sizes, 1..16 miniblocks,
miniblocks of fewer than 8 values, and two ways of finishing the last block ("full": every miniblock
of the last block carries data, "omit": miniblocks past the last delta get width 0 and no data),
plus mutations (truncation, header counts that disagree with the page).

Format (parquet spec, as read by readBlockHeader / readMiniBlockHeader):
  uvarint blockSize, uvarint miniBlockCount, uvarint totalValueCount, zigzag firstValue,
  per block: zigzag minDelta, miniBlockCount width bytes, miniblock data (LSB-first bit packing).
"""
import numpy as np


def _uvarint(x):
    out = bytearray()
    x = int(x)
    while True:
        b = x & 0x7F
        x >>= 7
        if x:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _zigzag(x, bits):
    x = int(x)
    return ((x << 1) ^ (x >> (bits - 1))) & ((1 << bits) - 1) if bits == 32 else ((x << 1) ^ (x >> 63)) & ((1 << 64) - 1)


def _signed(x, bits):
    x &= (1 << bits) - 1
    return x - (1 << bits) if x >> (bits - 1) else x


def _pack(vals, w):
    """LSB-first bit packing of len(vals) (multiple of 8) values of w bits."""
    if w == 0:
        return b""
    bits = np.zeros(len(vals) * w, dtype=np.uint8)
    v = np.array([int(x) for x in vals], dtype=object)
    for k in range(w):
        bits[k::w] = np.array([(int(x) >> k) & 1 for x in v], dtype=np.uint8)
    return np.packbits(bits, bitorder="little").tobytes()


def encode(values, bits=32, block_size=128, mb_count=4, finish="omit", total=None):
    """Encode `values` (python ints, taken mod 2^bits).  `total` overrides the header's value count."""
    mask = (1 << bits) - 1
    vals = [int(x) & mask for x in values]
    n = len(vals)
    out = bytearray()
    out += _uvarint(block_size) + _uvarint(mb_count) + _uvarint(n if total is None else total)
    first = _signed(vals[0], bits) if n else 0
    out += _uvarint(_zigzag(first, bits))
    deltas = [_signed(vals[i + 1] - vals[i], bits) for i in range(n - 1)]
    mbvc = block_size // mb_count
    for b0 in range(0, len(deltas), block_size):
        blk = deltas[b0:b0 + block_size]
        md = min(blk)
        out += _uvarint(_zigzag(md, bits))
        rel = [(d - md) & mask for d in blk]
        widths, datas = [], []
        for m in range(mb_count):
            part = rel[m * mbvc:(m + 1) * mbvc]
            if not part and finish == "omit":
                widths.append(0)
                datas.append(b"")
                continue
            w = max(x.bit_length() for x in part) if part else 0
            part = part + [0] * (mbvc - len(part))
            padded = part + [0] * ((-len(part)) % 8)
            widths.append(w)
            datas.append(_pack(padded, w))
        out += bytes(widths)
        for d in datas:
            out += d
    return bytes(out)


def random_values(rng, n, bits, kind):
    """Value distributions that exercise widths 0..bits."""
    lo, hi = -(1 << (bits - 1)), (1 << (bits - 1)) - 1
    if kind == "const":
        return [int(rng.integers(-1000, 1000))] * n
    if kind == "mono":
        return list(np.cumsum(rng.integers(0, 50, n)).astype(np.int64))
    if kind == "small":
        return list(rng.integers(-300, 300, n))
    if kind == "full":
        return [int(x) for x in rng.integers(lo, hi, n, dtype=np.int64, endpoint=True)]
    if kind == "mixed":  # runs of narrow and wide deltas
        v, cur = [], 0
        while len(v) < n:
            span = int(rng.integers(1, 400))
            wide = rng.random() < 0.3
            for _ in range(span):
                cur += int(rng.integers(lo, hi, dtype=np.int64)) if wide else int(rng.integers(-8, 8))
                v.append(cur)
        return v[:n]
    raise ValueError(kind)
