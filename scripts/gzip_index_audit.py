#!/usr/bin/env python3
"""Host build of k_gzip's index arithmetic (gzip_impl.h).

Emulates, thread by thread and phase by phase, the part of k_gzip whose tables the speculative pass
fills before they are verified -- gz_huff_stage (per-thread bit ranges, 96-bit warm-up, fixpoint
rounds, exclusive scans of output bytes / back-references, batch cuts) and the token tables it
hands gz_batch -- together with the serial states (gz_serial: member header, block headers, stored
runs, trailer) that feed the same batches.  For every output byte of every batch it evaluates the
index gz_batch would read from HBM:
    from == 1 (a back-reference before the batch):  ga = d + eout[e] - o + (rel % o | rel)  in [0, d)
    from == 2 (a stored byte outside the stage):    ga = esrc[e] + rel                      in [0, n)
and checks the range, and it rebuilds the page image from the emulated batches and compares it
with zlib's.  Decoding tables are canonical Huffman codes (RFC 1951); a symbol at any bit position
decodes from the 8 KiB + 96-byte stage exactly as gz_sym does (bytes past the input read as 0).

Usage: python scripts/gzip_index_audit.py [--pages N] [--mutants M]
"""
import argparse
import os
import sys
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

STAGE, MAXE, OUT, BLOCK, WARM = 8192, 1024, 8192, 256, 96
LBASE = [3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258]
LEXT = [0] * 8 + [1] * 4 + [2] * 4 + [3] * 4 + [4] * 4 + [5] * 4 + [0]
DBASE = [1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769, 1025, 1537, 2049, 3073,
         4097, 6145, 8193, 12289, 16385, 24577]
DEXT = [0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13]
ORDER = [16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15]


class Corrupt(Exception):
    pass


class Huff:
    """Canonical code (puff's count / symbol tables): decode from an LSB-first bit source."""

    def __init__(self, lens):
        self.count = [0] * 16
        for l in lens:
            self.count[l] += 1
        self.count[0] = 0
        left = 1
        for l in range(1, 16):
            left = (left << 1) - self.count[l]
            if left < 0:
                raise Corrupt("over-subscribed")
        self.incomplete = left > 0
        offs = [0] * 16
        for l in range(1, 15):
            offs[l + 1] = offs[l] + self.count[l]
        self.sym = [0] * len(lens)
        for s, l in enumerate(lens):
            if l:
                self.sym[offs[l]] = s
                offs[l] += 1

    def decode(self, bits):
        """bits: int (LSB-first).  (symbol, length) or (None, 1) for a code that is not in the set."""
        code = first = index = 0
        for l in range(1, 16):
            code |= bits & 1
            bits >>= 1
            c = self.count[l]
            if code - c < first:
                return self.sym[index + code - first], l
            index += c
            first = (first + c) << 1
            code <<= 1
        return None, 1


def table_ok(lens, kind):
    """gz_table_wave's acceptance: over-subscribed fails; incomplete fails unless a single 1-bit code
    (kind 1 / 2); the code-length code must be complete."""
    count = [0] * 16
    for l in lens:
        count[l] += 1
    mx = max([l for l in range(16) if count[l] and l] or [0])
    if mx == 0:
        return True
    left = 1
    for l in range(1, 16):
        left = (left << 1) - count[l]
        if left < 0:
            return False
    return not (left > 0 and (kind == 0 or mx != 1))


class Page:
    """k_gzip over one GZIP stream src (bytes) into a `total`-byte image."""

    def __init__(self, src, total):
        self.src, self.n, self.total = src, len(src), total
        self.dst = bytearray(total)
        self.reads = {"dst": [0, 0, None, None], "src": [0, 0, None, None]}  # count, oob, min, max
        self.oob = []
        # the write side: batches (gz_batch: [d, d + T)) and bulk stored copies ([d, d + left)), the
        # highest byte each writes, and how many would end past the page (what the pre-177f91c kernel,
        # without gz_batch's d + T > total guard, would have stored out of bounds)
        self.writes = {"batches": 0, "bulk": 0, "bytes": 0, "max_end": 0, "past_page": 0}

    # ---- the stage: bytes [a0, a0 + STAGE + 96) of src, past the input end read as 0
    def stage(self, a0):
        self.a0 = a0
        b = self.src[max(0, a0):a0 + STAGE + 96]
        self.stg = (b"\0" * (-a0 if a0 < 0 else 0)) + b + b"\0" * (STAGE + 96 + 16)
        self.stint = int.from_bytes(self.stg[:STAGE + 112], "little")

    def bits(self, pos, k=64):
        o = pos - 8 * self.a0
        return (self.stint >> o) & ((1 << k) - 1)

    # ---- gz_sym at bit pos: (kind, L, olen, x)
    def sym(self, pos):
        w = self.bits(pos, 64)
        s, u = self.lit.decode(w)
        if s is None or s >= 286 or (self.lit_single and s is None):
            return 3, u, 0, 0
        if s < 256:
            return 0, u, 1, s
        if s == 256:
            return 2, u, 0, 0
        i = s - 257
        ne = LEXT[i]
        ln = LBASE[i] + ((w >> u) & ((1 << ne) - 1))
        w2 = w >> (u + ne)
        ds, v = self.dist.decode(w2) if self.dist is not None else (None, 1)
        if ds is None or ds >= 30:
            return 3, u, 0, 0
        nd = DEXT[ds]
        return 1, u + ne + v + nd, ln, DBASE[ds] + ((w2 >> v) & ((1 << nd) - 1))

    def run(self, start, count_from, end):
        """gz_run: (f, x, o, k, st)."""
        f, o, k = -1, 0, 0
        pos = start
        while pos < end:
            kind, L, olen, _ = self.sym(pos)
            if pos < count_from:
                pos = count_from if kind >= 2 else pos + L
                continue
            if f < 0:
                f = pos
            if kind == 3:
                return f, pos, o, k, 2
            if kind == 2:
                return f, pos + L, o, k, 1
            o += olen
            k += kind == 1
            pos += L
        return (pos if f < 0 else f), pos, o, k, 0

    # ---- one batch of T bytes (tokens 1..nE-1) at page offset d: gz_batch's reads, checked
    def write(self, d, n, kind):
        w = self.writes
        w[kind] += 1
        w["bytes"] += n
        w["max_end"] = max(w["max_end"], d + n)
        w["past_page"] += d + n > self.total

    def batch(self, T, tokens, litb, d):
        self.write(d, T, "batches")
        if T < 0 or T > OUT or not (1 <= len(tokens) + 1 <= MAXE) or d + T > self.total:
            raise Corrupt("internal: batch geometry")  # gz_batch's first guard
        emap = [0] * T
        for e, (eo, typ, esrc, elen) in enumerate(tokens, 1):
            if not 0 <= eo < T:
                raise Corrupt(f"internal: token output {eo} outside the batch of {T}")
            emap[eo] = e
        cur = 0
        out = bytearray(T)
        s_lo, s_hi = self.a0, self.a0 + STAGE + 96
        for b in range(T):
            cur = max(cur, emap[b])
            if cur == 0:
                out[b] = litb[b]
                continue
            eo, typ, esrc, elen = tokens[cur - 1]
            rel = b - eo
            if rel >= elen:
                out[b] = litb[b]
            elif typ == 2:
                sp = esrc + rel
                if s_lo <= sp < s_hi:
                    out[b] = self.stg[sp - s_lo]
                else:
                    out[b] = self.read("src", sp, self.n, self.src)
            else:
                o = esrc
                sabs = d + eo - o + (rel % o if o < elen else rel)
                if sabs >= d:
                    out[b] = out[sabs - d]
                else:
                    out[b] = self.read("dst", sabs, d, self.dst)
        self.dst[d:d + T] = out

    def read(self, which, ga, bound, buf):
        r = self.reads[which]
        r[0] += 1
        r[2] = ga if r[2] is None else min(r[2], ga)
        r[3] = ga if r[3] is None else max(r[3], ga)
        if not 0 <= ga < bound:
            r[1] += 1
            self.oob.append((which, ga, bound))
            return 0
        return buf[ga]

    # ---- gz_huff_stage
    def huff_stage(self, d, ms):
        nbits = self.n * 8
        P0 = self.pbit
        Pend = min((self.a0 + STAGE) * 8, nbits)
        if P0 >= Pend:
            raise Corrupt("input ends inside the block")
        S = (Pend - P0 + BLOCK - 1) // BLOCK
        lo = [min(P0 + S * t, Pend) for t in range(BLOCK)]
        hi = [min(P0 + S * (t + 1), Pend) for t in range(BLOCK)]
        res = [self.run(P0 if t == 0 else max(lo[t] - WARM, P0), lo[t], hi[t]) for t in range(BLOCK)]
        for _ in range(BLOCK + 1):
            redo = [t > 0 and res[t - 1][4] == 0 and res[t - 1][1] != res[t][0] for t in range(BLOCK)]
            if not any(redo):
                break
            res = [self.run(res[t - 1][1], res[t - 1][1], hi[t]) if redo[t] else res[t] for t in range(BLOCK)]
        else:
            raise Corrupt("no fixpoint")
        e = next((t for t in range(BLOCK) if res[t][4]), BLOCK)
        if e < BLOCK and res[e][4] == 2:
            raise Corrupt("invalid code")
        last = e if e < BLOCK else BLOCK - 1
        O, K, acc_o, acc_k = [0] * BLOCK, [0] * BLOCK, 0, 0
        for t in range(BLOCK):
            O[t], K[t] = acc_o, acc_k
            if t <= last:
                acc_o += res[t][2]
                acc_k += res[t][3]
        Ototal, Ktotal = acc_o, acc_k
        bt, bo, bk, bp = 0, 0, 0, P0
        while True:
            lim_o, lim_k = bo + OUT, bk + MAXE - 1
            tokens = {}
            litb = bytearray(OUT)
            cut = None
            for t in range(bt, last + 1):
                p = bp if t == bt else res[t][0]
                out = bo if t == bt else O[t]
                tok = bk if t == bt else K[t]
                if not (out <= lim_o and tok <= lim_k):
                    continue
                pos = p
                while pos < hi[t]:
                    kind, L, olen, x = self.sym(pos)
                    if kind == 3 or pos + L > nbits:
                        raise Corrupt("bad symbol")
                    if kind == 2:
                        break
                    copy = kind == 1
                    if out + olen > lim_o or (copy and tok >= lim_k):
                        if cut is not None:
                            raise Corrupt("internal: two cuts")
                        cut = (t, pos, out, tok)
                        break
                    if d + out + olen > self.total:
                        raise Corrupt("past the page")
                    if copy:
                        if x > d + out - ms:
                            raise Corrupt("distance too far")
                        tokens[1 + tok - bk] = (out - bo, 1, x, olen)
                        tok += 1
                    else:
                        litb[out - bo] = x
                    out += olen
                    pos += L
            end_o = cut[2] if cut else Ototal
            end_k = cut[3] if cut else Ktotal
            T = end_o - bo
            if T > 0:
                nE = 1 + end_k - bk
                missing = [i for i in range(1, nE) if i not in tokens]
                if missing:
                    raise Corrupt(f"internal: {len(missing)} stale tokens")
                self.batch(T, [tokens[i] for i in range(1, nE)], litb, d + bo)
            if cut is None:
                break
            bt, bp, bo, bk = cut[0], cut[1], end_o, end_k
        d += Ototal
        if e < BLOCK:
            self.pbit = res[e][1]
            self.mode = "trailer" if self.final else "block"
        else:
            self.pbit = res[BLOCK - 1][1]
        return d

    # ---- the serial states (gz_serial): header, block header (tables), stored runs, trailer
    def header(self, p):
        s, n = self.src, self.n
        if n - p < 10 or s[p] != 0x1F or s[p + 1] != 0x8B or s[p + 2] != 8:
            raise Corrupt("header")
        flg, q = s[p + 3], p + 10
        if flg & 4:
            if n - q < 2:
                raise Corrupt("extra")
            xl = s[q] | (s[q + 1] << 8)
            q += 2
            if n - q < xl:
                raise Corrupt("extra")
            q += xl
        for bit in (8, 16):
            if flg & bit:
                i = 0
                while True:
                    if i >= 512 or q + i >= n:
                        raise Corrupt("string")
                    if s[q + i] == 0:
                        break
                    i += 1
                q += i + 1
        if flg & 2:
            if n - q < 2 or (zlib.crc32(s[p:q]) & 0xFFFF) != (s[q] | (s[q + 1] << 8)):
                raise Corrupt("hcrc")
            q += 2
        return q

    def block_header(self):
        pos = self.pbit
        w = self.bits(pos, 64)
        self.final = w & 1
        typ = (w >> 1) & 3
        pos += 3
        if typ == 0:
            pos = (pos + 7) & ~7
            w = self.bits(pos, 32)
            ln, nln = w & 0xFFFF, (w >> 16) & 0xFFFF
            if ln != (~nln & 0xFFFF):
                raise Corrupt("stored length")
            self.stored_left = ln
            self.mode = "stored"
            self.pbit = pos + 32
        elif typ == 1:
            lens = [8] * 144 + [9] * 112 + [7] * 24 + [8] * 8
            self.lit, self.dist, self.lit_single = Huff(lens), Huff([5] * 32), False
            self.mode = "huff"
            self.pbit = pos
        elif typ == 2:
            w = self.bits(pos, 14)
            nlen, ndist, ncode = (w & 31) + 257, ((w >> 5) & 31) + 1, ((w >> 10) & 15) + 4
            pos += 14
            if nlen > 286 or ndist > 30:
                raise Corrupt("too many symbols")
            cl = [0] * 19
            for i in range(ncode):
                cl[ORDER[i]] = self.bits(pos, 3)
                pos += 3
            if not table_ok(cl, 0):
                raise Corrupt("code lengths")
            ch = Huff(cl)
            lens = []
            while len(lens) < nlen + ndist:
                sym, u = ch.decode(self.bits(pos, 16))
                if sym is None:
                    raise Corrupt("code length symbol")
                pos += u
                if sym < 16:
                    lens.append(sym)
                    continue
                if sym == 16:
                    if not lens:
                        raise Corrupt("repeat")
                    v, rep = lens[-1], 3 + self.bits(pos, 2)
                    pos += 2
                elif sym == 17:
                    v, rep = 0, 3 + self.bits(pos, 3)
                    pos += 3
                else:
                    v, rep = 0, 11 + self.bits(pos, 7)
                    pos += 7
                if len(lens) + rep > nlen + ndist:
                    raise Corrupt("repeat past")
                lens += [v] * rep
            if lens[256] == 0:
                raise Corrupt("no end of block")
            ll, dl = lens[:nlen], lens[nlen:]
            if not (table_ok(ll, 1) and table_ok(dl, 2)):
                raise Corrupt("tables")
            self.lit = Huff(ll)
            self.dist = Huff(dl) if any(dl) else None
            self.lit_single = False
            self.mode = "huff"
            self.pbit = pos
        else:
            raise Corrupt("block type 3")
        if self.pbit > self.n * 8:
            raise Corrupt("past input")

    def decode(self):
        """gzip_stream: (status, image); status 0 / 'corrupt' / 'internal: ...'."""
        self.pbit, self.mode, members, d, ms = 0, "header", 0, 0, 0
        while True:
            p = self.pbit >> 3
            self.stage(p - (p & 15))
            if self.mode == "huff":
                d = self.huff_stage(d, ms)
                continue
            # serial batch: stored runs up to OUT bytes / MAXE tokens, or one transition
            lim = self.a0 + STAGE
            T, tokens = 0, []
            while self.mode != "huff":
                if self.mode == "header":
                    if members and p == self.n:
                        return d
                    body = self.header(self.pbit >> 3)
                    ms = d + T
                    self.mode = "block"
                    self.pbit = body * 8
                    if body > lim - 640:
                        break
                elif self.mode == "block":
                    if (self.pbit >> 3) > lim - 640:
                        break
                    self.block_header()
                elif self.mode == "stored":
                    q = self.pbit >> 3
                    left = self.stored_left
                    if left == 0:
                        self.mode = "trailer" if self.final else "block"
                        continue
                    if T == 0 and not tokens and left >= OUT:  # bulk copy
                        if q + left > self.n or d + left > self.total:
                            raise Corrupt("stored past")
                        self.write(d, left, "bulk")
                        self.dst[d:d + left] = self.src[q:q + left]
                        d += left
                        self.stored_left = 0
                        self.mode = "trailer" if self.final else "block"
                        self.pbit = (q + left) * 8
                        break
                    m = min(left, OUT - T)
                    if m == 0 or len(tokens) + 1 >= MAXE:
                        break
                    if q + m > self.n or d + T + m > self.total:
                        raise Corrupt("stored past")
                    tokens.append((T, 2, q, m))
                    T += m
                    self.stored_left = left - m
                    self.pbit = (q + m) * 8
                else:  # trailer
                    q = (self.pbit + 7) >> 3
                    if q + 8 > self.n:
                        raise Corrupt("trailer")
                    crc = int.from_bytes(self.src[q:q + 4], "little")
                    size = int.from_bytes(self.src[q + 4:q + 8], "little")
                    if T:
                        self.batch(T, tokens, bytearray(OUT), d)
                        d += T
                        T, tokens = 0, []
                    if (zlib.crc32(self.dst[ms:d]) & 0xFFFFFFFF) != crc or (d - ms) & 0xFFFFFFFF != size:
                        raise Corrupt("checksum")
                    members += 1
                    self.mode = "header"
                    self.pbit = (q + 8) * 8
                    break
            if T:
                self.batch(T, tokens, bytearray(OUT), d)
                d += T


def audit(name, stream, size, stats):
    from oracle import oracle as O

    try:
        want = O.gzip_decode(stream)
        if size is not None and len(want) != size:
            want = None
    except O.GzipCorrupt:
        want = None
    total = size if size is not None else (len(want) if want is not None else 0)
    pg = Page(stream, total)
    try:
        d = pg.decode()
        got = bytes(pg.dst) if d == total else None
        st = "ok" if got is not None else "corrupt"
    except Corrupt as e:
        got, st = None, ("internal" if str(e).startswith("internal") else "corrupt")
        if st == "internal":
            stats["internal"].append((name, str(e)))
    stats["pages"] += 1
    stats["match"] += (got == want) if want is not None else (got is None)
    if (got is None) != (want is None) or (got is not None and got != want):
        stats["mismatch"].append(name)
    for k in ("dst", "src"):
        r, a = stats[k], pg.reads[k]
        r[0] += a[0]
        r[1] += a[1]
    stats["oob"] += pg.oob[:5]
    w = stats["writes"]
    for k in ("batches", "bulk", "bytes", "past_page"):
        w[k] += pg.writes[k]
    if pg.writes["past_page"]:
        stats["oob"].append(("write past the page", name, pg.writes["max_end"], total))
    if pg.writes["max_end"] > total:
        w["pages_past"] += 1
    if st == "ok":
        w["ok_pages_ending_at_size"] += pg.writes["max_end"] == total or total == 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pages", type=int, default=12, help="C5z --codec gzip pages to emulate")
    ap.add_argument("--mutants", type=int, default=4, help="mutants per crafted valid stream")
    args = ap.parse_args()
    import gzip_blocks as G
    from conftest import load_package
    from oracle import oracle as O

    load_package()
    from parquet_go_amd import datasets
    from parquet_go_amd import writer as W

    stats = {"pages": 0, "match": 0, "mismatch": [], "internal": [], "oob": [], "dst": [0, 0], "src": [0, 0],
             "writes": {"batches": 0, "bulk": 0, "bytes": 0, "past_page": 0, "pages_past": 0,
                        "ok_pages_ending_at_size": 0}}
    # 1. the C5z --codec gzip pages (the workload of the r03 fault): the walker's compressed blocks
    data = datasets.c5z(rows=400_000, row_groups=1, codec=W.GZIP)
    fr = O.FileReader(data)
    md = fr.row_groups[0][1][0][3]
    pos, end, k = md.get(11, md[9]), md.get(11, md[9]) + md[7], 0
    while pos < end and k < args.pages:
        rd = O.CompactReader(fr.data, pos)
        ph = rd.struct()
        pos = rd.pos
        blk = bytes(fr.data[pos:pos + ph[3]])
        audit(f"c5z page {k}", blk, ph[2], stats)
        pos += ph[3]
        k += 1
    n_c5z = stats["pages"]
    # 2. every crafted valid stream and error class of the device-codec tests (valid_cases includes the
    # stored-block streams whose stored bytes lie past the 8 KiB stage: gz_batch's `src` read-backs),
    # plus seeded mutants of the valid ones and of the stored-block streams
    valid = [(n, s, len(O.gzip_decode(s))) for n, s, _ in G.valid_cases()]
    stored = [(n, s, len(O.gzip_decode(s))) for n, s, _ in G.stored_mix_cases()]
    for name, s, size in valid + G.error_cases() + G.mutants(valid[::2] + stored, per=args.mutants):
        audit(name, s, size, stats)
    print(f"pages emulated: {stats['pages']} ({n_c5z} C5z gzip pages of 1 MiB, {stats['pages'] - n_c5z} crafted "
          f"streams and mutants)")
    print(f"status and bytes equal to the oracle (Go's gzip reader restated): {stats['match']} / {stats['pages']}")
    print(f"HBM read-backs: dst (back-references before the batch) {stats['dst'][0]}, out of [0, d): "
          f"{stats['dst'][1]}; src (stored bytes outside the stage) {stats['src'][0]}, out of [0, n): "
          f"{stats['src'][1]}")
    w = stats["writes"]
    print(f"writes: {w['batches']} batches + {w['bulk']} bulk stored copies, {w['bytes']} bytes; ending past the "
          f"page's size: {w['past_page']} (pages: {w['pages_past']}); decoded pages whose last write ends exactly "
          f"at their size: {w['ok_pages_ending_at_size']}")
    print(f"internal inconsistencies (stale tokens, token outside its batch, two cuts): {len(stats['internal'])}")
    for x in stats["mismatch"][:10] + stats["internal"][:10] + stats["oob"][:10]:
        print("  ", x)
    return 0 if not (stats["mismatch"] or stats["internal"] or stats["oob"]) else 1


if __name__ == "__main__":
    sys.exit(main())
