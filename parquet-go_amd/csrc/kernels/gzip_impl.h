// gzip_impl.h — GZIP page decompression on the device (included by decode.hip
// after snappy_impl.h, whose batch resolution it shares).
//
// The reference decompresses GZIP page blocks on the host: gzipCompressor.DecompressBlock
// (compress.go:64-77) = Go's compress/gzip Reader (multistream) read to the end, then
// newBlockReader's exact-size check (compress.go:131-152).  k_gzip rebuilds each page image in HBM
// from the compressed bytes instead:
//
//   member  = header (gunzip.go readHeader: ID 1f 8b, CM 8, FEXTRA, FNAME / FCOMMENT within 512
//             bytes, FHCRC; reserved flag bits ignored), raw DEFLATE blocks (RFC 1951: stored,
//             fixed and dynamic Huffman), trailer CRC-32 + ISIZE; members repeat until the input
//             ends (a first member is required; a short header / trailer is an error);
//   errors  = any malformed header, block, code set, symbol or distance, output past the page's
//             uncompressed size, a checksum mismatch, or a short output -> PQH_ERR_DECOMPRESS.
//
// DEFLATE symbols are bit-serial, so one lane (thread 0) walks them: a 64-bit bit buffer refilled
// from an LDS stage of the compressed input, two-level decoding tables in LDS (the canonical
// construction zlib's inftrees.c uses: 9 root bits for literal/length codes, 6 for distances,
// sub-tables for longer codes).  It emits tokens — runs of literals (bytes kept in LDS at their
// output position), stored runs (source positions) and back-references — for up to kSnapOut output
// bytes; the whole workgroup then produces the batch's bytes with k_snappy's resolution (element
// map + pointer jumping, back-references before the batch read back from HBM).  At a member's end
// the workgroup computes the CRC-32 of the member's output (slice-by-4 per thread, combined across
// threads with GF(2) polynomial arithmetic) and checks the trailer.  Stored blocks of a batch or
// more are copied in bulk.
#pragma once

constexpr int kGzStage = 8192;    // compressed bytes staged in LDS per batch
constexpr int kGzMaxE = 1024;     // tokens per batch
constexpr int kGzEnoughL = 852;   // largest literal/length table with 9 root bits (RFC 1951 codes)
constexpr int kGzEnoughD = 592;   // largest distance table with 6 root bits
constexpr int kGzHdrRoom = 640;   // bytes a dynamic block header may need (14 + 19*3 + 316*14 bits)
constexpr uint32_t kCrcPoly = 0xedb88320u;  // CRC-32 (IEEE), reflected

// RFC 1951 §3.2.5: length / distance base values and extra bits.  The op byte of a table entry is
// 16 + extra bits for a length or distance base, 0 for a literal, 96 for end-of-block, 64 for an
// invalid code (lengths 286/287, distances 30/31), 1..15 for a link to a sub-table of that many bits.
__constant__ uint16_t kGzLBase[31] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27, 31,
                                      35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258, 0, 0};
__constant__ uint8_t kGzLOp[31] = {16, 16, 16, 16, 16, 16, 16, 16, 17, 17, 17, 17, 18, 18, 18, 18,
                                   19, 19, 19, 19, 20, 20, 20, 20, 21, 21, 21, 21, 16, 64, 64};
__constant__ uint16_t kGzDBase[32] = {1,    2,    3,    4,    5,    7,     9,     13,    17,  25,   33,
                                      49,   65,   97,   129,  193,  257,   385,   513,   769, 1025, 1537,
                                      2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577, 0,   0};
__constant__ uint8_t kGzDOp[32] = {16, 16, 16, 16, 17, 17, 18, 18, 19, 19, 20, 20, 21, 21, 22, 22,
                                   23, 23, 24, 24, 25, 25, 26, 26, 27, 27, 28, 28, 29, 29, 64, 64};
__constant__ uint8_t kGzClOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

struct __attribute__((aligned(16))) GzLds {
  uint8_t in[kGzStage + 96];      // the stage: input bytes [a0, a0 + kGzStage + 96)
  uint16_t emap[kSnapOut];        // batch resolution (batch_emap / batch_jump_store)
  uint8_t out[kSnapOut];
  uint8_t litb[kSnapOut];         // Huffman literals at their batch output position
  int32_t eout[kGzMaxE + 1];      // token output start, batch-relative; eout[nE] = the batch size
  int32_t esrc[kGzMaxE];          // back-reference: distance; stored run: input position
  int32_t elen[kGzMaxE];
  uint8_t etyp[kGzMaxE];          // 0 literal run, 1 back-reference, 2 stored run
  uint32_t lcode[kGzEnoughL];     // literal/length table (also the code-length table while a
  uint32_t dcode[kGzEnoughD];     //   dynamic header is read); distance table
  uint32_t crc[4][256];           // slice-by-4 CRC-32 tables
  uint32_t x2n[32];               // x^(2^k) mod P(x)
  uint32_t part_crc[kBlock];
  int32_t part_len[kBlock];
  uint16_t lens[320];             // code lengths of the current dynamic block
  uint16_t work[320];             // symbols sorted by code length (table construction)
  uint16_t cnt[16], offs[16];
  int32_t wmax[4];
  // decoder state between batches (thread 0 writes, everyone reads after a barrier)
  int64_t pbit;                   // input bit position of the next symbol / header
  int32_t mode, final_blk, stored_left, members, lbits, dbits, ms, fixed_ready;
  uint32_t tcrc, tsize;
  int32_t nE, bend, bad, bulk_len, bulk_src, member_end, done, progress;
};

__device__ __forceinline__ uint32_t gz_entry(uint32_t op, uint32_t bits, uint32_t val) {
  return op | (bits << 8) | (val << 16);
}

// The canonical Huffman decoding table for `codes` code lengths (RFC 1951 §3.2.2), built the way
// zlib's inflate_table does: a root table of *bits index bits (lowered to the longest code,
// raised to the shortest), codes longer than the root in sub-tables sized to what they need.
// type 0 = code-length code, 1 = literal/length, 2 = distance.  False on an over-subscribed code,
// or an incomplete one other than a single 1-bit code (code-length codes must be complete).  No
// codes at all: a table whose every entry is invalid (an error only if a symbol is decoded).
// Thread 0 only.
__device__ bool gz_table(GzLds& E, int type, const uint16_t* lens, int codes, uint32_t* table, int32_t* bits) {
  uint16_t* count = E.cnt;
  uint16_t* offs = E.offs;
  for (int l = 0; l < 16; l++) count[l] = 0;
  for (int s = 0; s < codes; s++) count[lens[s]]++;
  int root = *bits, max = 15;
  while (max >= 1 && count[max] == 0) max--;
  if (root > max) root = max;
  if (max == 0) {
    table[0] = table[1] = gz_entry(64, 1, 0);
    *bits = 1;
    return true;
  }
  int min = 1;
  while (min < max && count[min] == 0) min++;
  if (root < min) root = min;
  int left = 1;
  for (int l = 1; l <= 15; l++) {
    left = (left << 1) - count[l];
    if (left < 0) return false;  // over-subscribed
  }
  if (left > 0 && (type == 0 || max != 1)) return false;  // incomplete
  offs[1] = 0;
  for (int l = 1; l < 15; l++) offs[l + 1] = uint16_t(offs[l] + count[l]);
  for (int s = 0; s < codes; s++)
    if (lens[s] != 0) E.work[offs[lens[s]]++] = uint16_t(s);
  const uint16_t* base = type == 1 ? kGzLBase : kGzDBase;
  const uint8_t* ops = type == 1 ? kGzLOp : kGzDOp;
  const int match = type == 0 ? 20 : (type == 1 ? 257 : 0);
  uint32_t huff = 0;  // the current code, bit-reversed
  int sym = 0, len = min, curr = root, drop = 0, used = 1 << root;
  uint32_t low = 0xffffffffu;
  const uint32_t mask = uint32_t(used) - 1;
  const int enough = type == 1 ? kGzEnoughL : kGzEnoughD;
  if (type != 0 && used > enough) return false;
  uint32_t* next = table;
  for (;;) {
    const int w = E.work[sym];
    uint32_t here;
    if (w + 1 < match) here = gz_entry(0, uint32_t(len - drop), uint32_t(w));
    else if (w >= match) here = gz_entry(ops[w - match], uint32_t(len - drop), base[w - match]);
    else here = gz_entry(96, uint32_t(len - drop), 0);  // end of block
    // replicate over every index whose low (len - drop) bits are this code
    const int incr = 1 << (len - drop);
    int fill = 1 << curr;
    const int tsize = fill;
    do {
      fill -= incr;
      next[(huff >> drop) + uint32_t(fill)] = here;
    } while (fill != 0);
    // the next code of this length: increment huff in bit-reversed order
    uint32_t inc = 1u << (len - 1);
    while (huff & inc) inc >>= 1;
    huff = inc ? (huff & (inc - 1)) + inc : 0;
    sym++;
    if (--count[len] == 0) {
      if (len == max) break;
      len = lens[E.work[sym]];
    }
    if (len > root && (huff & mask) != low) {  // a new sub-table
      if (drop == 0) drop = root;
      next += tsize;
      curr = len - drop;
      int lft = 1 << curr;
      while (curr + drop < max) {
        lft -= count[curr + drop];
        if (lft <= 0) break;
        curr++;
        lft <<= 1;
      }
      used += 1 << curr;
      if (type != 0 && used > enough) return false;
      low = huff & mask;
      table[low] = gz_entry(uint32_t(curr), uint32_t(root), uint32_t(next - table));
    }
  }
  if (huff != 0) next[huff] = gz_entry(64, uint32_t(len - drop), 0);  // the one slot of an incomplete code
  *bits = root;
  return true;
}

// zlib's multmodp / x2nmodp (crc32.c), restated: GF(2) polynomials modulo the reflected CRC-32
// polynomial; crc(A || B) = (crc(A) * x^(8 |B|)) ^ crc(B).
__device__ __forceinline__ uint32_t gz_multmodp(uint32_t a, uint32_t b) {
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = (b & 1) ? (b >> 1) ^ kCrcPoly : b >> 1;
  }
  return p;
}

__device__ __forceinline__ uint32_t gz_crc_combine(const GzLds& E, uint32_t crc1, uint32_t crc2, uint32_t len2) {
  uint32_t p = 1u << 31;  // x^0
  for (int k = 3; len2; len2 >>= 1, k++)
    if (len2 & 1) p = gz_multmodp(E.x2n[k & 31], p);
  return gz_multmodp(p, crc1) ^ crc2;
}

// A gzip member header at src[p] (gunzip.go readHeader); *body = its first DEFLATE byte.
__device__ bool gz_header(const GzLds& E, const uint8_t* src, int32_t n, int32_t p, int32_t* body) {
  if (n - p < 10) return false;
  if (src[p] != 0x1f || src[p + 1] != 0x8b || src[p + 2] != 8) return false;
  const uint32_t flg = src[p + 3];
  int32_t q = p + 10;
  if (flg & 4) {  // FEXTRA
    if (n - q < 2) return false;
    const int32_t xlen = int32_t(src[q]) | (int32_t(src[q + 1]) << 8);
    q += 2;
    if (n - q < xlen) return false;
    q += xlen;
  }
  for (uint32_t bit = 8; bit <= 16; bit <<= 1) {  // FNAME, FCOMMENT: NUL within 512 bytes
    if (!(flg & bit)) continue;
    int32_t i = 0;
    for (;; i++) {
      if (i >= 512 || q + i >= n) return false;
      if (src[q + i] == 0) break;
    }
    q += i + 1;
  }
  if (flg & 2) {  // FHCRC: low 16 bits of the header's CRC-32
    if (n - q < 2) return false;
    uint32_t c = 0xffffffffu;
    for (int32_t j = p; j < q; j++) c = E.crc[0][(c ^ src[j]) & 0xff] ^ (c >> 8);
    c = ~c;
    if ((c & 0xffff) != (uint32_t(src[q]) | (uint32_t(src[q + 1]) << 8))) return false;
    q += 2;
  }
  *body = q;
  return true;
}

// The bit reader of thread 0 over the stage: hold has nb valid bits; bp = the next input byte to
// load (absolute).  Refill keeps 56..63 bits (the bytes above nb are the same bytes the next refill
// loads, so OR-ing them again is harmless).
struct GzBits {
  uint64_t hold;
  int32_t nb, bp;
};

__device__ __forceinline__ uint64_t gz_load64(const GzLds& E, int32_t o) {
  const uint32_t* in32 = reinterpret_cast<const uint32_t*>(E.in);
  const int32_t i = o >> 2, sh = 8 * (o & 3);
  const uint64_t lo = (uint64_t(in32[i + 1]) << 32) | in32[i];
  const uint64_t hi = in32[i + 2];
  return sh ? (lo >> sh) | (hi << (64 - sh)) : lo;
}

__device__ __forceinline__ void gz_refill(const GzLds& E, GzBits& R, int32_t a0) {
  R.hold |= gz_load64(E, R.bp - a0) << R.nb;
  R.bp += (63 - R.nb) >> 3;
  R.nb |= 56;
}

__device__ __forceinline__ void gz_drop(GzBits& R, int k) {
  R.hold >>= k;
  R.nb -= k;
}

__device__ __forceinline__ void gz_seek(const GzLds& E, GzBits& R, int64_t bit, int32_t a0) {
  R.bp = int32_t(bit >> 3);
  R.hold = 0;
  R.nb = 0;
  gz_refill(E, R, a0);
  gz_drop(R, int(bit & 7));
}

__device__ __forceinline__ int64_t gz_pos(const GzBits& R) { return int64_t(R.bp) * 8 - R.nb; }

// A table entry for the bits in hold: the root entry, or the sub-table entry it links to.
// *used = the code's length.
__device__ __forceinline__ uint32_t gz_decode(const uint32_t* tab, int32_t rbits, uint64_t hold, int* used) {
  uint32_t e = tab[uint32_t(hold) & ((1u << rbits) - 1)];
  uint32_t op = e & 0xff;
  int u = int((e >> 8) & 0xff);
  if (op != 0 && (op & 0xf0) == 0) {
    e = tab[(e >> 16) + (uint32_t(hold >> u) & ((1u << op) - 1))];
    u += int((e >> 8) & 0xff);
  }
  *used = u;
  return e;
}

// A dynamic block's header (RFC 1951 §3.2.7): the code-length code, then the literal/length and
// distance code lengths, then both tables.  False where zlib reports "too many length or distance
// symbols", "invalid code lengths set", "invalid bit length repeat", "missing end-of-block",
// "invalid literal/lengths set" or "invalid distances set".
__device__ bool gz_dynamic(GzLds& E, GzBits& R, int32_t a0) {
  gz_refill(E, R, a0);
  const int nlen = int(R.hold & 31) + 257, ndist = int((R.hold >> 5) & 31) + 1, ncode = int((R.hold >> 10) & 15) + 4;
  gz_drop(R, 14);
  if (nlen > 286 || ndist > 30) return false;
  for (int i = 0; i < 19; i++) {
    uint16_t l = 0;
    if (i < ncode) {
      gz_refill(E, R, a0);
      l = uint16_t(R.hold & 7);
      gz_drop(R, 3);
    }
    E.lens[kGzClOrder[i]] = l;
  }
  int32_t cb = 7;
  if (!gz_table(E, 0, E.lens, 19, E.lcode, &cb)) return false;
  const int total = nlen + ndist;
  int i = 0;
  while (i < total) {
    gz_refill(E, R, a0);
    int u;
    const uint32_t e = gz_decode(E.lcode, cb, R.hold, &u);
    if ((e & 0xff) != 0) return false;  // (a complete code never reaches an invalid entry)
    gz_drop(R, u);
    const int sym = int(e >> 16);
    if (sym < 16) {
      E.lens[i++] = uint16_t(sym);
      continue;
    }
    uint16_t v = 0;
    int rep;
    if (sym == 16) {
      if (i == 0) return false;
      v = E.lens[i - 1];
      rep = 3 + int(R.hold & 3);
      gz_drop(R, 2);
    } else if (sym == 17) {
      rep = 3 + int(R.hold & 7);
      gz_drop(R, 3);
    } else {
      rep = 11 + int(R.hold & 127);
      gz_drop(R, 7);
    }
    if (i + rep > total) return false;
    while (rep--) E.lens[i++] = v;
  }
  if (E.lens[256] == 0) return false;
  E.lbits = 9;
  if (!gz_table(E, 1, E.lens, nlen, E.lcode, &E.lbits)) return false;
  E.dbits = 6;
  if (!gz_table(E, 2, E.lens + nlen, ndist, E.dcode, &E.dbits)) return false;
  E.fixed_ready = 0;
  return true;
}

__device__ bool gz_fixed(GzLds& E) {
  if (E.fixed_ready) return true;
  for (int s = 0; s < 288; s++) E.lens[s] = uint16_t(s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8);
  E.lbits = 9;
  if (!gz_table(E, 1, E.lens, 288, E.lcode, &E.lbits)) return false;
  for (int s = 0; s < 32; s++) E.lens[s] = 5;
  E.dbits = 5;
  if (!gz_table(E, 2, E.lens, 32, E.dcode, &E.dbits)) return false;
  E.fixed_ready = 1;
  return true;
}

enum : int32_t { kGzHeader = 0, kGzBlock = 1, kGzHuff = 2, kGzStored = 3, kGzTrailer = 4 };

// Thread 0: the tokens of one batch from the state in E (input staged from a0), output from d.
__device__ void gz_parse(GzLds& E, const uint8_t* src, int32_t n, int32_t a0, int32_t d, int32_t total) {
  const int64_t nbits = int64_t(n) * 8;
  const int32_t lim = a0 + kGzStage;  // the reader's next byte stays at or below this
  int32_t mode = E.mode, k = 0, T = 0, bulk_len = 0, bulk_src = 0;
  bool bad = false, member_end = false, done = false;
  int64_t jump = -1;  // >= 0: the next batch starts at this bit (a position outside the stage)
  const int64_t start = E.pbit;
  GzBits R;
  R.hold = 0;
  R.nb = 0;
  R.bp = 0;
  bool live = false;  // R holds the position
  if (mode == kGzHeader) {
    jump = start;
  } else {
    gz_seek(E, R, start, a0);
    live = true;
  }
  int32_t run0 = -1;  // the open literal run's output start
  auto close_run = [&]() {
    if (run0 >= 0) {
      E.eout[k] = run0;
      E.elen[k] = T - run0;
      E.etyp[k] = 0;
      k++;
      run0 = -1;
    }
  };
  for (;;) {
    if (mode == kGzHeader) {
      const int32_t p = int32_t(jump >> 3);  // byte aligned
      if (E.members > 0 && p == n) {
        done = true;
        break;
      }
      int32_t body;
      if (!gz_header(E, src, n, p, &body)) {
        bad = true;
        break;
      }
      E.ms = d + T;
      mode = kGzBlock;
      jump = int64_t(body) * 8;
      if (body > lim - kGzHdrRoom) break;  // restage at the first block
      gz_seek(E, R, jump, a0);
      live = true;
      jump = -1;
      continue;
    }
    if (mode == kGzBlock) {
      if (R.bp > lim - kGzHdrRoom) break;  // restage: a dynamic header must fit the stage
      gz_refill(E, R, a0);
      E.final_blk = int32_t(R.hold & 1);
      const int type = int((R.hold >> 1) & 3);
      gz_drop(R, 3);
      if (type == 0) {
        gz_drop(R, R.nb & 7);  // to a byte boundary
        gz_refill(E, R, a0);
        const uint32_t len = uint32_t(R.hold & 0xffff), nlen = uint32_t((R.hold >> 16) & 0xffff);
        gz_drop(R, 32);
        if (len != (~nlen & 0xffff)) bad = true;
        E.stored_left = int32_t(len);
        mode = kGzStored;
      } else if (type == 1) {
        if (!gz_fixed(E)) bad = true;
        mode = kGzHuff;
      } else if (type == 2) {
        if (!gz_dynamic(E, R, a0)) bad = true;
        mode = kGzHuff;
      } else {
        bad = true;
      }
      if (bad || gz_pos(R) > nbits) {
        bad = true;
        break;
      }
      continue;
    }
    if (mode == kGzHuff) {
      const uint32_t* lc = E.lcode;
      const uint32_t* dc = E.dcode;
      const int32_t lb = E.lbits, db = E.dbits;
      const int32_t ms = E.ms;
      bool eob = false;
      for (;;) {
        if (T > kSnapOut - 258 || k >= kGzMaxE - 2 || R.bp > lim) break;
        gz_refill(E, R, a0);
        int u;
        const uint32_t e = gz_decode(lc, lb, R.hold, &u);
        gz_drop(R, u);
        const uint32_t op = e & 0xff;
        if (op == 0) {  // literal
          if (d + T >= total) {
            bad = true;
            break;
          }
          if (run0 < 0) run0 = T;
          E.litb[T++] = uint8_t(e >> 16);
        } else if (op & 16) {  // length, then a distance
          const int32_t len = int32_t(e >> 16) + int32_t(uint32_t(R.hold) & ((1u << (op & 15)) - 1));
          gz_drop(R, int(op & 15));
          int v;
          const uint32_t f = gz_decode(dc, db, R.hold, &v);
          gz_drop(R, v);
          const uint32_t dop = f & 0xff;
          if (!(dop & 16)) {  // invalid distance code
            bad = true;
            break;
          }
          const int32_t dist = int32_t(f >> 16) + int32_t(uint32_t(R.hold) & ((1u << (dop & 15)) - 1));
          gz_drop(R, int(dop & 15));
          if (dist > d + T - ms || d + T + len > total) {  // too far back / past the page size
            bad = true;
            break;
          }
          close_run();
          E.eout[k] = T;
          E.elen[k] = len;
          E.esrc[k] = dist;
          E.etyp[k] = 1;
          k++;
          T += len;
        } else if (op & 32) {  // end of block
          eob = true;
          break;
        } else {  // invalid code
          bad = true;
          break;
        }
      }
      if (!bad && gz_pos(R) > nbits) bad = true;  // the input ended inside a symbol
      if (bad || !eob) break;
      mode = E.final_blk ? kGzTrailer : kGzBlock;
      continue;
    }
    if (mode == kGzStored) {
      const int64_t here = live ? gz_pos(R) : jump;  // byte aligned
      const int32_t q = int32_t(here >> 3);
      const int32_t left = E.stored_left;
      if (left == 0) {
        mode = E.final_blk ? kGzTrailer : kGzBlock;
        if (!live) {
          if (q > lim - kGzHdrRoom) break;
          gz_seek(E, R, here, a0);
          live = true;
          jump = -1;
        }
        continue;
      }
      close_run();
      if (T == 0 && k == 0 && left >= kSnapOut) {  // a batch or more: bulk copy
        if (q + int64_t(left) > n || d + int64_t(left) > total) {
          bad = true;
          break;
        }
        bulk_len = left;
        bulk_src = q;
        E.stored_left = 0;
        mode = E.final_blk ? kGzTrailer : kGzBlock;
        jump = int64_t(q + left) * 8;
        live = false;
        break;
      }
      const int32_t m = left < kSnapOut - T ? left : kSnapOut - T;
      if (m == 0 || k >= kGzMaxE - 2) {
        jump = here;
        live = false;
        break;
      }
      if (q + int64_t(m) > n || d + T + int64_t(m) > total) {
        bad = true;
        break;
      }
      E.eout[k] = T;
      E.elen[k] = m;
      E.esrc[k] = q;
      E.etyp[k] = 2;
      k++;
      T += m;
      E.stored_left = left - m;
      jump = int64_t(q + m) * 8;
      live = false;
      continue;
    }
    // kGzTrailer: CRC-32 and ISIZE at the next byte boundary
    {
      const int64_t here = live ? gz_pos(R) : jump;
      const int32_t q = int32_t((here + 7) >> 3);
      if (int64_t(q) + 8 > n) {
        bad = true;
        break;
      }
      E.tcrc = uint32_t(src[q]) | (uint32_t(src[q + 1]) << 8) | (uint32_t(src[q + 2]) << 16) | (uint32_t(src[q + 3]) << 24);
      E.tsize = uint32_t(src[q + 4]) | (uint32_t(src[q + 5]) << 8) | (uint32_t(src[q + 6]) << 16) |
                (uint32_t(src[q + 7]) << 24);
      E.members += 1;
      member_end = true;
      mode = kGzHeader;
      jump = int64_t(q + 8) * 8;
      live = false;
      break;
    }
  }
  close_run();
  E.eout[k] = T;
  const int64_t next = live ? gz_pos(R) : jump;
  E.pbit = next;
  E.mode = mode;
  E.nE = k;
  E.bend = T;
  E.bad = bad;
  E.bulk_len = bulk_len;
  E.bulk_src = bulk_src;
  E.member_end = member_end;
  E.done = done;
  E.progress = T > 0 || bulk_len > 0 || member_end || done || next != start;
}

// Decode one gzip stream src[0, n) into dst[0, expected).  Whole workgroup; returns PQH_OK or
// PQH_ERR_DECOMPRESS (uniform).
__device__ int gzip_stream(const uint8_t* src, int64_t n64, uint8_t* dst, int64_t expected, GzLds& E) {
  const int tid = threadIdx.x;
  if (n64 > 0x7fffffff - kGzStage || expected > 0x7fffffff) return PQH_ERR_DECOMPRESS;
  for (int i = tid; i < 256; i += kBlock) {
    uint32_t c = uint32_t(i);
    for (int j = 0; j < 8; j++) c = (c & 1) ? (c >> 1) ^ kCrcPoly : c >> 1;
    E.crc[0][i] = c;
  }
  __syncthreads();
  for (int i = tid; i < 256; i += kBlock)
    for (int t = 1; t < 4; t++) E.crc[t][i] = (E.crc[t - 1][i] >> 8) ^ E.crc[0][E.crc[t - 1][i] & 0xff];
  if (tid == 0) {
    uint32_t p = 1u << 30;  // x^1
    E.x2n[0] = p;
    for (int k = 1; k < 32; k++) E.x2n[k] = p = gz_multmodp(p, p);
    E.pbit = 0;
    E.mode = kGzHeader;
    E.members = 0;
    E.fixed_ready = 0;
    E.final_blk = 0;
    E.stored_left = 0;
    E.ms = 0;
  }
  const int32_t n = uni(int32_t(n64)), total = uni(int32_t(expected));
  int32_t d = 0;
  for (;;) {
    __syncthreads();  // the previous batch's readers of the stage and the state are done
    const int32_t p = uni(int32_t(E.pbit >> 3));
    const int32_t a0 = uni(p - int32_t((reinterpret_cast<uintptr_t>(src) + uintptr_t(p)) & 15));
    {  // up to the input's end rounded to 16 bytes (inside the payload pad)
      const uint4* sp = reinterpret_cast<const uint4*>(src + a0);
      uint4* lp = reinterpret_cast<uint4*>(E.in);
      const int32_t avail = (n - a0 + 15) >> 4;
      const int nu = avail < (kGzStage + 96) / 16 ? avail : (kGzStage + 96) / 16;
      for (int u = tid; u < nu; u += kBlock) lp[u] = sp[u];
    }
    __syncthreads();
    if (tid == 0) gz_parse(E, src, n, a0, d, total);
    __syncthreads();
    if (uni(E.bad) || !uni(E.progress)) return PQH_ERR_DECOMPRESS;
    const int32_t nE = uni(E.nE), T = uni(E.bend);
    if (nE == 0) {
      const int32_t bl = uni(E.bulk_len);
      if (bl > 0) {
        snap_copy(dst + d, src + uni(E.bulk_src), bl);
        d += bl;
      }
    } else {
      batch_emap(E, nE);
      const int32_t s_lo = a0, s_hi = a0 + kGzStage + 96;
      int16_t ptr[kPer];
      uint8_t val[kPer];
#pragma unroll
      for (int i0 = 0; i0 < kPer; i0 += 8) {
        int32_t ga[8];
        uint8_t from[8];  // 0 resolved / in-batch pointer, 1 dst (an earlier batch), 2 src (stored bytes outside the stage)
#pragma unroll
        for (int j = 0; j < 8; j++) {
          const int32_t b = (i0 + j) * kBlock + tid;
          from[j] = 0;
          ga[j] = 0;
          val[i0 + j] = 0;
          ptr[i0 + j] = -1;
          if (b >= T) continue;
          const int e = E.emap[b];
          const int32_t rel = b - E.eout[e];
          const int typ = E.etyp[e];
          if (typ == 0) {
            val[i0 + j] = E.litb[b];
          } else if (typ == 2) {
            const int32_t sp = E.esrc[e] + rel;
            if (sp >= s_lo && sp < s_hi) {
              val[i0 + j] = E.in[sp - s_lo];
            } else {
              from[j] = 2;
              ga[j] = sp;
            }
          } else {
            const int32_t o = E.esrc[e];
            const int32_t sabs = d + E.eout[e] - o + (o < E.elen[e] ? rel % o : rel);  // overlapping copies repeat
            if (sabs >= d) {
              ptr[i0 + j] = int16_t(sabs - d);
            } else {
              from[j] = 1;
              ga[j] = sabs;
            }
          }
        }
#pragma unroll
        for (int j = 0; j < 8; j++)
          if (from[j]) val[i0 + j] = from[j] == 1 ? dst[ga[j]] : src[ga[j]];
      }
      batch_jump_store(E, T, ptr, val, dst + d);
      d += T;
    }
    __syncthreads();  // this batch's bytes are visible to the next batches' reads and the CRC
    if (uni(E.member_end)) {
      // CRC-32 of the member's output [ms, d): a slice of whole words per thread, then a tree of
      // crc32_combine steps
      const int32_t ms = uni(E.ms), len = d - ms;
      const int32_t seg = ((len + kBlock - 1) / kBlock + 3) & ~3;
      const int32_t b0 = ms + (tid * seg < len ? tid * seg : len);
      const int32_t b1 = ms + ((tid + 1) * seg < len ? (tid + 1) * seg : len);
      uint32_t c = 0xffffffffu;
      int32_t x = b0;
      for (; x + 4 <= b1; x += 4) {
        c ^= uint32_t(dst[x]) | (uint32_t(dst[x + 1]) << 8) | (uint32_t(dst[x + 2]) << 16) | (uint32_t(dst[x + 3]) << 24);
        c = E.crc[3][c & 0xff] ^ E.crc[2][(c >> 8) & 0xff] ^ E.crc[1][(c >> 16) & 0xff] ^ E.crc[0][c >> 24];
      }
      for (; x < b1; x++) c = E.crc[0][(c ^ dst[x]) & 0xff] ^ (c >> 8);
      E.part_crc[tid] = ~c;
      E.part_len[tid] = b1 - b0;
      for (int s = 1; s < kBlock; s <<= 1) {
        __syncthreads();
        if ((tid & (2 * s - 1)) == 0) {
          E.part_crc[tid] = gz_crc_combine(E, E.part_crc[tid], E.part_crc[tid + s], uint32_t(E.part_len[tid + s]));
          E.part_len[tid] += E.part_len[tid + s];
        }
      }
      __syncthreads();
      if (uint32_t(uni(int32_t(E.part_crc[0]))) != uint32_t(uni(int32_t(E.tcrc))) ||
          uint32_t(len) != uint32_t(uni(int32_t(E.tsize))))
        return PQH_ERR_DECOMPRESS;
    }
    if (uni(E.done)) break;
  }
  return d == total ? PQH_OK : PQH_ERR_DECOMPRESS;
}

// One workgroup per GZIP page (other codecs: k_snappy): its image rebuilt at image_offset.
__global__ __launch_bounds__(256) void k_gzip(const pqh_codec_page* cps, const uint8_t* src_all, uint8_t* dst_all,
                                              int32_t* status) {
  __shared__ GzLds E;
  const pqh_codec_page cp = cps[blockIdx.x];
  if (cp.codec != PQH_CODEC_GZIP) return;
  const uint8_t* src = src_all + cp.src_offset;
  uint8_t* dst = dst_all + cp.image_offset;
  int rc;
  const int32_t raw = cp.raw_len < cp.src_len ? cp.raw_len : cp.src_len;
  snap_copy(dst, src, raw < cp.image_len ? raw : cp.image_len);  // DataPageV2 levels: never compressed
  if (raw > cp.image_len) rc = PQH_ERR_DECOMPRESS;
  else rc = gzip_stream(src + raw, cp.src_len - raw, dst + raw, int64_t(cp.image_len) - raw, E);
  if (threadIdx.x == 0) status[blockIdx.x] = rc;
}
