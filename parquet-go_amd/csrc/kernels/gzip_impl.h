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
  int32_t tnext[16], toffs[17];   // canonical first code / sorted offset per length (gz_table_wave)
  uint16_t gofs[320];             // long-code sub-tables (gz_table_wave): offset and index bits per group
  uint8_t gbits[320];
  int32_t nlen, ndist, tab_kind;
  int32_t wmax[4];
  // decoder state between batches (thread 0 writes, everyone reads after a barrier)
  int64_t pbit;                   // input bit position of the next symbol / header
  int32_t mode, final_blk, stored_left, members, lbits, dbits, ms, fixed_ready;
  uint32_t tcrc, tsize;
  int32_t nE, bend, bad, bulk_len, bulk_src, member_end, done, progress;
  // Huffman stage (gz_huff_stage): per thread its entry / exit bit, output bytes, back-references,
  // state (0 ok, 1 end of block, 2 invalid code); the first ended thread; the batch cut
  int64_t hf[kBlock], hx[kBlock];
  int32_t ho[kBlock], hk[kBlock];
  uint8_t hst[kBlock];
  int32_t wsum[8];
  int32_t hend, hcut, hcut_out, hcut_tok;
  int64_t hcut_pos;
#ifdef PQH_GZIP_PROF  // timing experiments: clock64() per phase (wave 0), printed for page 0
  uint64_t prof[12];
#endif
};
#ifdef PQH_GZIP_PROF
#define GZ_CLK(v) const uint64_t v = clock64()
#define GZ_ADD(i, x) (E.prof[i] += (x))
#else
#define GZ_CLK(v)
#define GZ_ADD(i, x)
#endif

__device__ __forceinline__ uint32_t gz_entry(uint32_t op, uint32_t bits, uint32_t val) {
  return op | (bits << 8) | (val << 16);
}

// The canonical Huffman decoding table for `codes` code lengths (RFC 1951 §3.2.2), built the way
// zlib's inflate_table (inftrees.c) does -- a restatement of that routine; zlib is (C) 1995-2024
// Jean-loup Gailly and Mark Adler under the zlib license ("This software is provided 'as-is' ...
// Permission is granted to anyone to use this software for any purpose, including commercial
// applications, and to alter it and redistribute it freely", with its three conditions: no
// misrepresented origin, altered versions plainly marked, the notice kept).  gz_multmodp below
// restates zlib's multmodp (crc32.c) under the same license.  The build's own wave-parallel
// construction, gz_table_wave, builds the literal/length and distance tables; gz_table serves only
// the 19-symbol code-length code.  zlib's inflate_table does: a root table of *bits index bits (lowered to the longest code,
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

// A dynamic block's header (RFC 1951 §3.2.7), lane 0: the code-length code, then the
// literal/length and distance code lengths into E.lens (E.nlen, E.ndist); the wave then builds both
// tables (gz_build_tables: "invalid literal/lengths set", "invalid distances set").  False where
// zlib reports "too many length or distance symbols", "invalid code lengths set", "invalid bit
// length repeat" or "missing end-of-block".
__device__ __forceinline__ bool gz_dynamic(GzLds& E, GzBits& R, int32_t a0) {
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
  E.nlen = nlen;
  E.ndist = ndist;
  return true;
}

__device__ __forceinline__ uint32_t gz_sym_entry(int type, int s, uint32_t bits) {
  if (type == 0) return gz_entry(0, bits, uint32_t(s));
  if (type == 1) {
    if (s < 256) return gz_entry(0, bits, uint32_t(s));
    if (s == 256) return gz_entry(96, bits, 0);
    return gz_entry(kGzLOp[s - 257], bits, kGzLBase[s - 257]);
  }
  return gz_entry(kGzDOp[s], bits, kGzDBase[s]);
}

// A long code's canonical value, and its root-prefix key, from its sorted position i.
__device__ __forceinline__ uint32_t gz_long_code(const GzLds& E, const uint16_t* lens, int i, int* len) {
  const int l = lens[E.work[i]];
  *len = l;
  return uint32_t(E.tnext[l] + (i - E.toffs[l]));
}

__device__ __forceinline__ uint32_t gz_long_key(const GzLds& E, const uint16_t* lens, int i, int root) {
  int l;
  const uint32_t c = gz_long_code(E, lens, i, &l);
  return c >> (l - root);
}

// gz_table's tables built by wave 0 in parallel: the same validity rules and the same decoding.  A
// canonical code's long codes sharing a root prefix are contiguous in (length, symbol) order and
// exactly fill a sub-table of (their longest length - root) index bits — the size zlib's
// construction picks for a complete code.  Ranks by ballots; each short code replicated over the
// root table by its own lane; sub-table offsets by a scan over the groups of long codes.
__device__ bool gz_table_wave(GzLds& E, int type, const uint16_t* lens, int codes, uint32_t* table, int32_t root_req,
                              int32_t* bits_out) {
  const int lane = threadIdx.x & 63;
  const uint64_t below = (1ull << lane) - 1, upto = below | (1ull << lane);
  const int nch = (codes + 63) >> 6;
  int32_t cnt[16];
#pragma unroll
  for (int l = 0; l < 16; l++) cnt[l] = 0;
  for (int c = 0; c < nch; c++) {
    const int s = c * 64 + lane;
    const int l = s < codes ? lens[s] : 0;
#pragma unroll
    for (int L = 1; L < 16; L++) cnt[L] += __popcll(__ballot(l == L));
  }
  int max = 15;
  while (max >= 1 && cnt[max] == 0) max--;
  int root = root_req > max ? max : root_req;
  if (max == 0) {  // no codes: every entry invalid
    if (lane == 0) {
      table[0] = table[1] = gz_entry(64, 1, 0);
      *bits_out = 1;
    }
    return true;
  }
  int min = 1;
  while (min < max && cnt[min] == 0) min++;
  if (root < min) root = min;
  int left = 1;
  for (int l = 1; l <= 15; l++) {
    left = (left << 1) - cnt[l];
    if (left < 0) return false;  // over-subscribed
  }
  if (left > 0 && (type == 0 || max != 1)) return false;  // incomplete
  if (left > 0 && lane == 0) table[0] = table[1] = gz_entry(64, 1, 0);  // the single 1-bit code: one slot invalid
  int32_t offs[17], next[16];
  offs[0] = offs[1] = 0;
  next[0] = 0;
  int code = 0;
#pragma unroll
  for (int l = 1; l < 16; l++) {
    offs[l + 1] = offs[l] + cnt[l];
    code = (code + cnt[l - 1]) << 1;
    next[l] = code;
  }
  if (lane < 16) {  // the same values for the dynamically indexed long-code passes
    int32_t nv = 0, ov = 0;
#pragma unroll
    for (int l = 0; l < 16; l++)
      if (lane == l) {
        nv = next[l];
        ov = offs[l];
      }
    E.tnext[lane] = nv;
    E.toffs[lane] = ov;
  }
  // ranks, canonical codes, sorted order; short codes fill the root table
  int32_t run[16];
#pragma unroll
  for (int l = 0; l < 16; l++) run[l] = 0;
  const uint32_t rsize = 1u << root;
  for (int c = 0; c < nch; c++) {
    const int s = c * 64 + lane;
    const int l = s < codes ? lens[s] : 0;
    int rank = 0, nx = 0, of = 0;
#pragma unroll
    for (int L = 1; L < 16; L++) {
      const uint64_t m = __ballot(l == L);
      if (l == L) {
        rank = run[L] + __popcll(m & below);
        nx = next[L];
        of = offs[L];
      }
      run[L] += __popcll(m);
    }
    if (l > 0) {
      E.work[of + rank] = uint16_t(s);
      if (l <= root) {
        const uint32_t rev = __builtin_bitreverse32(uint32_t(nx + rank)) >> (32 - l);
        const uint32_t ent = gz_sym_entry(type, s, uint32_t(l));
        for (uint32_t j = rev; j < rsize; j += 1u << l) table[j] = ent;
      }
    }
  }
  if (max > root) {
    // long codes: the sorted tail work[first, last); pass 1: groups' index bits and offsets
    const int first = offs[root + 1], last = offs[16];
    int gbase = 0, used = int(rsize);
    for (int i0 = first; i0 < last; i0 += 64) {
      const int i = i0 + lane;
      const bool on = i < last;
      bool start = false, end = false;
      int l = 0;
      if (on) {
        const uint32_t key = gz_long_key(E, lens, i, root);
        l = lens[E.work[i]];
        start = i == first || gz_long_key(E, lens, i - 1, root) != key;
        end = i == last - 1 || gz_long_key(E, lens, i + 1, root) != key;
      }
      const uint64_t sm = __ballot(start);
      const int g = gbase + __popcll(sm & upto) - 1;
      const uint32_t size = end ? (1u << (l - root)) : 0u;
      const uint32_t incl = wave_incl_scan32(size);
      if (end) {
        E.gbits[g] = uint8_t(l - root);
        E.gofs[g] = uint16_t(used + int(incl - size));
      }
      used += __builtin_amdgcn_readlane(int32_t(incl), 63);
      gbase += __popcll(sm);
    }
    const int enough = type == 1 ? kGzEnoughL : kGzEnoughD;
    if (type != 0 && used > enough) return false;
    // pass 2: root links and sub-table entries
    gbase = 0;
    for (int i0 = first; i0 < last; i0 += 64) {
      const int i = i0 + lane;
      const bool on = i < last;
      bool start = false;
      int s = 0, l = 0;
      uint32_t cv = 0;
      if (on) {
        s = E.work[i];
        cv = gz_long_code(E, lens, i, &l);
        start = i == first || gz_long_key(E, lens, i - 1, root) != (cv >> (l - root));
      }
      const uint64_t sm = __ballot(start);
      const int g = gbase + __popcll(sm & upto) - 1;
      gbase += __popcll(sm);
      if (on) {
        const uint32_t rev = __builtin_bitreverse32(cv) >> (32 - l);
        const uint32_t sub = E.gbits[g], base = E.gofs[g];
        if (start) table[rev & (rsize - 1)] = gz_entry(sub, uint32_t(root), base);
        const uint32_t ent = gz_sym_entry(type, s, uint32_t(l - root));
        for (uint32_t j = rev >> root; j < (1u << sub); j += 1u << (l - root)) table[base + j] = ent;
      }
    }
  }
  if (lane == 0) *bits_out = root;
  return true;
}

// Wave 0: the tables of the block whose header lane 0 just read (E.tab_kind 1 fixed, 2 dynamic).
__device__ bool gz_build_tables(GzLds& E) {
  const int lane = threadIdx.x & 63;
  if (uni(E.tab_kind) == 1) {
    if (uni(E.fixed_ready)) return true;
    for (int s = lane; s < 320; s += 64) E.lens[s] = uint16_t(s >= 288 ? 5 : s < 144 ? 8 : s < 256 ? 9 : s < 280 ? 7 : 8);
    const bool ok = gz_table_wave(E, 1, E.lens, 288, E.lcode, 9, &E.lbits) &&
                    gz_table_wave(E, 2, E.lens + 288, 32, E.dcode, 6, &E.dbits);
    if (lane == 0) E.fixed_ready = ok;
    return ok;
  }
  const int32_t nlen = uni(E.nlen), ndist = uni(E.ndist);
  if (lane == 0) E.fixed_ready = 0;
  return gz_table_wave(E, 1, E.lens, nlen, E.lcode, 9, &E.lbits) &&
         gz_table_wave(E, 2, E.lens + nlen, ndist, E.dcode, 6, &E.dbits);
}

enum : int32_t { kGzHeader = 0, kGzBlock = 1, kGzHuff = 2, kGzStored = 3, kGzTrailer = 4 };

constexpr uint32_t kGzStop = 1, kGzBad = 2, kGzMemberEnd = 4, kGzDone = 8, kGzTables = 16;

// Lane 0: one transition of the non-Huffman states (member header, block header, stored data,
// trailer).  pos = the input bit position (byte aligned in the header / stored / trailer states);
// T / k = the batch's output bytes / next token index (tokens start at 1).  Sets kGzStop to end the
// batch here (restage, batch full, bulk copy), kGzBad on an error.
__device__ void gz_serial(GzLds& E, const uint8_t* src, int32_t n, int32_t a0, int32_t d, int32_t total, int32_t& mode,
                          int64_t& pos, int32_t& T, int32_t& k, uint32_t& flags, int32_t& bulk_len, int32_t& bulk_src) {
  const int64_t nbits = int64_t(n) * 8;
  const int32_t lim = a0 + kGzStage;
  if (mode == kGzHeader) {
    const int32_t p = int32_t(pos >> 3);
    if (E.members > 0 && p == n) {
      flags |= kGzDone;
      return;
    }
    int32_t body;
    if (!gz_header(E, src, n, p, &body)) {
      flags |= kGzBad;
      return;
    }
    E.ms = d + T;
    mode = kGzBlock;
    pos = int64_t(body) * 8;
    if (body > lim - kGzHdrRoom) flags |= kGzStop;  // restage at the first block
    return;
  }
  if (mode == kGzBlock) {
    if ((pos >> 3) > lim - kGzHdrRoom) {  // restage: a dynamic header must fit the stage
      flags |= kGzStop;
      return;
    }
    GzBits R;
    gz_seek(E, R, pos, a0);
    gz_refill(E, R, a0);
    E.final_blk = int32_t(R.hold & 1);
    const int type = int((R.hold >> 1) & 3);
    gz_drop(R, 3);
    bool ok = true;
    if (type == 0) {
      gz_drop(R, R.nb & 7);  // to a byte boundary
      gz_refill(E, R, a0);
      const uint32_t len = uint32_t(R.hold & 0xffff), nlen = uint32_t((R.hold >> 16) & 0xffff);
      gz_drop(R, 32);
      ok = len == (~nlen & 0xffff);
      E.stored_left = int32_t(len);
      mode = kGzStored;
    } else if (type == 1) {
      E.tab_kind = 1;
      flags |= kGzTables;
      mode = kGzHuff;
    } else if (type == 2) {
      ok = gz_dynamic(E, R, a0);
      E.tab_kind = 2;
      flags |= kGzTables;
      mode = kGzHuff;
    } else {
      ok = false;
    }
    pos = gz_pos(R);
    if (!ok || pos > nbits) flags |= kGzBad;
    return;
  }
  if (mode == kGzStored) {
    const int32_t q = int32_t(pos >> 3);
    const int32_t left = E.stored_left;
    if (left == 0) {
      mode = E.final_blk ? kGzTrailer : kGzBlock;
      return;
    }
    if (T == 0 && k == 1 && left >= kSnapOut) {  // a batch or more: bulk copy
      if (q + int64_t(left) > n || d + int64_t(left) > total) {
        flags |= kGzBad;
        return;
      }
      bulk_len = left;
      bulk_src = q;
      E.stored_left = 0;
      mode = E.final_blk ? kGzTrailer : kGzBlock;
      pos = int64_t(q + left) * 8;
      flags |= kGzStop;
      return;
    }
    const int32_t m = left < kSnapOut - T ? left : kSnapOut - T;
    if (m == 0 || k >= kGzMaxE) {
      flags |= kGzStop;
      return;
    }
    if (q + int64_t(m) > n || d + T + int64_t(m) > total) {
      flags |= kGzBad;
      return;
    }
    E.eout[k] = T;
    E.elen[k] = m;
    E.esrc[k] = q;
    E.etyp[k] = 2;
    k++;
    T += m;
    E.stored_left = left - m;
    pos = int64_t(q + m) * 8;
    return;
  }
  // kGzTrailer: CRC-32 and ISIZE at the next byte boundary
  const int32_t q = int32_t((pos + 7) >> 3);
  if (int64_t(q) + 8 > n) {
    flags |= kGzBad;
    return;
  }
  E.tcrc = uint32_t(src[q]) | (uint32_t(src[q + 1]) << 8) | (uint32_t(src[q + 2]) << 16) | (uint32_t(src[q + 3]) << 24);
  E.tsize = uint32_t(src[q + 4]) | (uint32_t(src[q + 5]) << 8) | (uint32_t(src[q + 6]) << 16) | (uint32_t(src[q + 7]) << 24);
  E.members += 1;
  mode = kGzHeader;
  pos = int64_t(q + 8) * 8;
  flags |= kGzMemberEnd;
}

// (uni64: bytearray_impl.h)
// Wave 0: the non-Huffman states of one batch (lane 0's transitions, broadcast), until the stream
// reaches Huffman-coded data (gz_huff_stage's), the batch ends, or the member / stream ends.
__device__ void gz_parse(GzLds& E, const uint8_t* src, int32_t n, int32_t a0, int32_t d, int32_t total) {
  const int lane = threadIdx.x & 63;
  int32_t mode = uni(E.mode);
  const int32_t mode0 = mode;
  int64_t pos = uni64(E.pbit);
  const int64_t start = pos;
  int32_t k = 1, T = 0, bulk_len = 0, bulk_src = 0;
  uint32_t flags = 0;
  while (mode != kGzHuff) {
    int32_t s_mode = mode, s_T = T, s_k = k, s_bl = 0, s_bs = 0;
    int64_t s_pos = pos;
    uint32_t s_flags = 0;
    if (lane == 0) gz_serial(E, src, n, a0, d, total, s_mode, s_pos, s_T, s_k, s_flags, s_bl, s_bs);
    mode = uni(s_mode);
    pos = uni64(s_pos);
    T = uni(s_T);
    k = uni(s_k);
    flags = uint32_t(uni(int32_t(s_flags)));
    bulk_len = uni(s_bl);
    bulk_src = uni(s_bs);
    if (flags & kGzTables) {  // a Huffman block's header was read: the wave builds its tables
      flags &= ~kGzTables;
      if (!(flags & kGzBad) && !gz_build_tables(E)) flags |= kGzBad;
    }
    if (flags) break;
  }
  if (lane == 0) {
    E.pbit = pos;
    E.mode = mode;
    E.nE = k;
    E.bend = T;
    E.bad = (flags & kGzBad) != 0;
    E.bulk_len = bulk_len;
    E.bulk_src = bulk_src;
    E.member_end = (flags & kGzMemberEnd) != 0;
    E.done = (flags & kGzDone) != 0;
    E.progress = T > 0 || bulk_len > 0 || (flags & (kGzMemberEnd | kGzDone)) || pos != start || mode != mode0;
  }
}

// One Huffman-coded symbol at bit pos: kind 0 literal (x = byte), 1 length + distance (olen =
// length, x = distance), 2 end of block, 3 invalid code; L = its bits.
struct GzSym {
  uint32_t kind, L, olen, x;
};

__device__ __forceinline__ GzSym gz_sym(const GzLds& E, int64_t pos, int32_t lb, int32_t db, int32_t a0) {
  const uint64_t w = gz_load64(E, int32_t(pos >> 3) - a0) >> (pos & 7);  // >= 56 valid bits
  int u;
  const uint32_t e = gz_decode(E.lcode, lb, w, &u);
  const uint32_t op = e & 0xff;
  GzSym s;
  s.kind = 3;
  s.L = u > 0 ? uint32_t(u) : 1u;
  s.olen = 0;
  s.x = 0;
  if (op == 0) {
    s.kind = 0;
    s.olen = 1;
    s.x = e >> 16;
  } else if (op & 16) {
    const int ne = int(op & 15);
    const uint32_t len = (e >> 16) + (uint32_t(w >> u) & ((1u << ne) - 1));
    const uint64_t w2 = w >> (u + ne);
    int v;
    const uint32_t f = gz_decode(E.dcode, db, w2, &v);
    const uint32_t dop = f & 0xff;
    if (dop & 16) {
      const int nd = int(dop & 15);
      s.kind = 1;
      s.olen = len;
      s.x = (f >> 16) + (uint32_t(w2 >> v) & ((1u << nd) - 1));
      s.L = uint32_t(u + ne + v + nd);
    }
  } else if (op & 32) {
    s.kind = 2;
  }
  return s;
}

constexpr int64_t kGzWarm = 96;  // bits a speculative decode runs before its range to synchronise

struct GzRun {
  int64_t f, x;  // first symbol at or after count_from; the first symbol position at or after `end`
  int32_t o, k, st;
};

// Decode from `start` while symbols start before `end`, counting (output bytes, back-references)
// the symbols from count_from on.  An end-of-block or invalid code stops the walk (st 1 / 2; x = the
// bit after the end of block).  Before count_from (the warm-up) such a symbol restarts the walk at
// count_from.
__device__ GzRun gz_run(const GzLds& E, int64_t start, int64_t count_from, int64_t end, int32_t lb, int32_t db,
                        int32_t a0) {
  GzRun R;
  R.f = -1;
  R.o = 0;
  R.k = 0;
  R.st = 0;
  int64_t pos = start;
  while (pos < end) {
    const GzSym s = gz_sym(E, pos, lb, db, a0);
    if (pos < count_from) {
      pos = s.kind >= 2 ? count_from : pos + s.L;
      continue;
    }
    if (R.f < 0) R.f = pos;
    if (s.kind == 3) {
      R.st = 2;
      R.x = pos;
      return R;
    }
    if (s.kind == 2) {
      R.st = 1;
      R.x = pos + s.L;
      return R;
    }
    R.o += int32_t(s.olen);
    R.k += s.kind == 1;
    pos += s.L;
  }
  R.x = pos;
  if (R.f < 0) R.f = pos;
  return R;
}

enum : int { kGzEmitDone = 0, kGzEmitCut = 1, kGzEmitBad = 2 };

// A thread's symbols from `pos` (stage output `out`, back-reference count `tok`) into the batch
// [bo, lim_o) x token indices [1 + tok - bk ...]: literals to litb, back-references to the token
// arrays, with the reference's checks; stops at the first symbol past the batch (the cut).
__device__ int gz_emit(GzLds& E, int64_t pos, int64_t end, int32_t out, int32_t tok, int32_t bo, int32_t bk, int32_t lim_o,
                       int32_t lim_k, int32_t dbase, int32_t ms, int32_t total, int64_t nbits, int32_t lb, int32_t db,
                       int32_t a0, int64_t* cpos, int32_t* cout, int32_t* ctok) {
  while (pos < end) {
    const GzSym s = gz_sym(E, pos, lb, db, a0);
    if (s.kind == 3 || pos + s.L > nbits) return kGzEmitBad;
    if (s.kind == 2) return kGzEmitDone;
    const bool copy = s.kind == 1;
    if (out + int32_t(s.olen) > lim_o || (copy && tok >= lim_k)) {
      *cpos = pos;
      *cout = out;
      *ctok = tok;
      return kGzEmitCut;
    }
    if (int64_t(dbase) + out + s.olen > total) return kGzEmitBad;  // past the page's size
    if (copy) {
      if (int64_t(s.x) > int64_t(dbase) + out - ms) return kGzEmitBad;  // distance too far back
      const int32_t i = 1 + tok - bk;
      E.eout[i] = out - bo;
      E.elen[i] = int32_t(s.olen);
      E.esrc[i] = int32_t(s.x);
      E.etyp[i] = 1;
      tok++;
    } else {
      E.litb[out - bo] = uint8_t(s.x);
    }
    out += int32_t(s.olen);
    pos += s.L;
  }
  return kGzEmitDone;
}

__device__ __forceinline__ int32_t block_excl_scan(GzLds& E, int32_t x, int32_t* total) {
  const int tid = threadIdx.x;
  const uint32_t incl = wave_incl_scan32(uint32_t(x));
  if ((tid & 63) == 63) E.wsum[tid >> 6] = int32_t(incl);
  __syncthreads();
  int32_t base = 0, all = 0;
#pragma unroll
  for (int w = 0; w < kBlock / 64; w++) {
    const int32_t v = E.wsum[w];
    if (w < (tid >> 6)) base += v;
    all += v;
  }
  __syncthreads();  // wsum is reused
  *total = all;
  return base + int32_t(incl) - x;
}

// Resolve a batch of T output bytes (tokens 1..nE-1; literal bytes in litb) and store it at
// dst + d.  Whole workgroup.
// Every HBM read is bounds-checked (a back-reference inside [0, d), a stored byte inside [0, n)) and
// the batch must end inside the page (total): false, with nothing read or written out of bounds, when
// the batch's tables are inconsistent.  gz_emit / gz_serial validate every token against the input
// and the page before it is stored, so a failing guard is an internal inconsistency of the kernel,
// never a corrupt page: the callers report PQH_ERR_INTERNAL (the r03 GZIP fault).
__device__ bool gz_batch(GzLds& E, int32_t T, int32_t nE, int32_t d, int32_t a0, const uint8_t* src, uint8_t* dst,
                         int32_t n, int32_t total) {
  const int tid = threadIdx.x;
  if (T < 0 || T > kSnapOut || nE < 1 || nE > kGzMaxE || int64_t(d) + T > total) {
#ifdef PQH_GZIP_DEBUG
    if (tid == 0) printf("gz_batch guard: page %d T %d nE %d d %d total %d\n", int(blockIdx.x), T, nE, d, total);
#endif
    return false;
  }
  bool oob = false;
  batch_emap(E, nE, 1);
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
      if (e == 0 || rel >= E.elen[e]) {  // a literal
        val[i0 + j] = E.litb[b];
      } else if (E.etyp[e] == 2) {
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
    for (int j = 0; j < 8; j++) {
      if (!from[j]) continue;
      if (ga[j] < 0 || ga[j] >= (from[j] == 1 ? d : n)) {
#ifdef PQH_GZIP_DEBUG
        printf("gz_batch guard: page %d from %d ga %d d %d n %d\n", int(blockIdx.x), int(from[j]), ga[j], d, n);
#endif
        oob = true;
        continue;
      }
      val[i0 + j] = from[j] == 1 ? dst[ga[j]] : src[ga[j]];
    }
  }
  if (__syncthreads_or(oob)) return false;
  batch_jump_store(E, T, ptr, val, dst + d);
  return true;
}

// The Huffman-coded data of the current block from E.pbit to the end of the stage (or the block's
// end of block), by the whole workgroup.  The bit range is cut into kBlock equal parts; thread t
// decodes its part speculatively, starting kGzWarm bits early so that its walk (almost always)
// falls into step with the true symbol chain before its part begins (Huffman codes resynchronise
// within a few symbols).  Rounds then re-decode every part whose first symbol differs from the
// previous part's exit, from that exit, until nothing changes: thread 0 starts on the chain, so
// after round r parts 0..r are exact and the fixpoint is the true decode.  A scan places the parts'
// output; batches of at most kSnapOut bytes / kGzMaxE - 1 back-references are then emitted (each
// part re-decoded from its true entry) and resolved with gz_batch.  Returns PQH_OK,
// PQH_ERR_DECOMPRESS (the stream is corrupt) or PQH_ERR_INTERNAL (a gz_batch guard fired); uniform.
__device__ int gz_huff_stage(GzLds& E, const uint8_t* src, int32_t n, int32_t a0, int32_t& d, int32_t total,
                              uint8_t* dst) {
  const int tid = threadIdx.x;
  const int64_t nbits = int64_t(n) * 8;
  const int64_t P0 = uni64(E.pbit);
  const int64_t stage_end = int64_t(a0 + kGzStage) * 8;
  const int64_t Pend = stage_end < nbits ? stage_end : nbits;
  if (P0 >= Pend) return PQH_ERR_DECOMPRESS;  // the input ends inside the block
  const int32_t lb = uni(E.lbits), db = uni(E.dbits), ms = uni(E.ms);
  const int64_t S = (Pend - P0 + kBlock - 1) / kBlock;
  const int64_t lo = P0 + S * tid < Pend ? P0 + S * tid : Pend;
  const int64_t hi = P0 + S * (tid + 1) < Pend ? P0 + S * (tid + 1) : Pend;
  GZ_CLK(h0);
  {
    const int64_t warm = tid == 0 ? P0 : (lo - kGzWarm > P0 ? lo - kGzWarm : P0);
    const GzRun R = gz_run(E, warm, lo, hi, lb, db, a0);
    E.hf[tid] = R.f;
    E.hx[tid] = R.x;
    E.ho[tid] = R.o;
    E.hk[tid] = R.k;
    E.hst[tid] = uint8_t(R.st);
  }
  bool converged = false;
  for (int round = 0; round <= kBlock; round++) {
    __syncthreads();
    const bool redo = tid > 0 && E.hst[tid - 1] == 0 && E.hx[tid - 1] != E.hf[tid];
    const int64_t entry = redo ? E.hx[tid - 1] : 0;
    __syncthreads();  // every thread has read the previous round
    if (redo) {
      const GzRun R = gz_run(E, entry, entry, hi, lb, db, a0);
      E.hf[tid] = R.f;
      E.hx[tid] = R.x;
      E.ho[tid] = R.o;
      E.hk[tid] = R.k;
      E.hst[tid] = uint8_t(R.st);
    }
#ifdef PQH_GZIP_PROF
    if (tid == 0) GZ_ADD(1, 1);
#endif
    if (!__syncthreads_or(redo)) {
      converged = true;
      break;
    }
  }
  if (!converged) return PQH_ERR_DECOMPRESS;  // (cannot happen: round r fixes part r)
#ifdef PQH_GZIP_PROF
  {
    GZ_CLK(h1);
    if (tid == 0) GZ_ADD(0, h1 - h0);
  }
#endif
  // the first part that ended (end of block) or failed; the parts after it are not in this block
  if (tid == 0) E.hend = kBlock;
  __syncthreads();
  if (E.hst[tid]) atomicMin(&E.hend, tid);
  __syncthreads();
  const int32_t e = uni(E.hend);
  if (e < kBlock && E.hst[e] == 2) return PQH_ERR_DECOMPRESS;  // an invalid code on the chain
  const int32_t last = e < kBlock ? e : kBlock - 1;
  const bool mine = tid <= last;
  int32_t Ototal, Ktotal;
  const int32_t O = block_excl_scan(E, mine ? E.ho[tid] : 0, &Ototal);
  const int32_t K = block_excl_scan(E, mine ? E.hk[tid] : 0, &Ktotal);
  const int64_t my_f = E.hf[tid];
  // ---- batches
  int32_t bt = 0, bo = 0, bk = 0;
  int64_t bp = P0;
  for (;;) {
    const int32_t lim_o = bo + kSnapOut, lim_k = bk + kGzMaxE - 1;
    if (tid == 0) E.hcut = -1;
    __syncthreads();
    int r = kGzEmitDone;
    GZ_CLK(h2);
    if (mine && tid >= bt) {
      const int64_t p = tid == bt ? bp : my_f;
      const int32_t out = tid == bt ? bo : O, tok = tid == bt ? bk : K;
      if (out <= lim_o && tok <= lim_k) {
        int64_t cp;
        int32_t co, ck;
        r = gz_emit(E, p, hi, out, tok, bo, bk, lim_o, lim_k, d, ms, total, nbits, lb, db, a0, &cp, &co, &ck);
        if (r == kGzEmitCut) {  // exactly one part holds the first symbol past the batch
          E.hcut = tid;
          E.hcut_pos = cp;
          E.hcut_out = co;
          E.hcut_tok = ck;
        }
      }
    }
    if (__syncthreads_or(r == kGzEmitBad)) return PQH_ERR_DECOMPRESS;
    const int32_t cut = uni(E.hcut);
    const int32_t end_o = cut >= 0 ? uni(E.hcut_out) : Ototal;
    const int32_t end_k = cut >= 0 ? uni(E.hcut_tok) : Ktotal;
    const int32_t T = end_o - bo;
    GZ_CLK(h3);
    if (T > 0) {
      if (!gz_batch(E, T, 1 + end_k - bk, d + bo, a0, src, dst, n, total)) return PQH_ERR_INTERNAL;
      __syncthreads();  // the batch's bytes are visible to later batches
    }
#ifdef PQH_GZIP_PROF
    {
      GZ_CLK(h4);
      if (tid == 0) {
        GZ_ADD(2, h3 - h2);
        GZ_ADD(4, h4 - h3);
        GZ_ADD(10, 1);
      }
    }
#endif
    if (cut < 0) break;
    bt = cut;
    bp = uni64(E.hcut_pos);
    bo = end_o;
    bk = end_k;
  }
  d += Ototal;
  __syncthreads();
  if (tid == 0) {
    if (e < kBlock) {
      E.pbit = E.hx[e];
      E.mode = E.final_blk ? kGzTrailer : kGzBlock;
    } else {
      E.pbit = E.hx[kBlock - 1];
    }
  }
  return PQH_OK;
}

// Decode one gzip stream src[0, n) into dst[0, expected).  Whole workgroup; returns PQH_OK,
// PQH_ERR_DECOMPRESS or PQH_ERR_INTERNAL (uniform).
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
    E.eout[0] = 0;  // token 0: the "literal" every byte before the first token maps to
    E.elen[0] = 0;
    E.etyp[0] = 0;
    E.esrc[0] = 0;
#ifdef PQH_GZIP_PROF
    for (int i = 0; i < 12; i++) E.prof[i] = 0;
#endif
  }
  const int32_t n = uni(int32_t(n64)), total = uni(int32_t(expected));
  int32_t d = 0;
  for (;;) {
    __syncthreads();  // the previous batch's readers of the stage and the state are done
    GZ_CLK(t0);
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
    GZ_CLK(t1);
#ifdef PQH_GZIP_PROF
    if (tid == 0) GZ_ADD(6, t1 - t0);
#endif
    if (uni(E.mode) == kGzHuff) {
      const int hs = gz_huff_stage(E, src, n, a0, d, total, dst);
#ifdef PQH_GZIP_PROF
      GZ_CLK(t2);
      if (tid == 0) {
        GZ_ADD(7, t2 - t1);
        GZ_ADD(3, 1);
      }
#endif
      if (hs != PQH_OK) return hs;
      continue;
    }
    if (tid < 64) gz_parse(E, src, n, a0, d, total);
    __syncthreads();
    if (uni(E.bad) || !uni(E.progress)) return PQH_ERR_DECOMPRESS;
    const int32_t nE = uni(E.nE), T = uni(E.bend);
    const int32_t bl = uni(E.bulk_len);
    if (bl > 0) {
      const int32_t bs = uni(E.bulk_src);
      if (int64_t(d) + bl > total || bs < 0 || int64_t(bs) + bl > n) return PQH_ERR_INTERNAL;  // (validated by gz_serial)
      snap_copy(dst + d, src + bs, bl);
      d += bl;
    } else if (T > 0) {
      if (!gz_batch(E, T, nE, d, a0, src, dst, n, total)) return PQH_ERR_INTERNAL;
      d += T;
    }
    __syncthreads();  // this batch's bytes are visible to the next batches' reads and the CRC
#ifdef PQH_GZIP_PROF
    {
      GZ_CLK(t3);
      if (tid == 0) {
        GZ_ADD(9, t3 - t1);
        GZ_ADD(8, 1);
      }
    }
#endif
#ifndef PQH_GZIP_NO_CRC  // timing experiments: without the trailer check
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
#endif
    if (uni(E.done)) break;
  }
#ifdef PQH_GZIP_PROF
  if (tid == 0 && blockIdx.x == 0)
    printf("gzprof huffman stages %lu (rounds %lu, batches %lu) serial batches %lu | cycles: stage loads %lu huffman %lu "
           "(decode+rounds %lu emit %lu resolve %lu) serial+batches %lu\n",
           E.prof[3], E.prof[1], E.prof[10], E.prof[8], E.prof[6], E.prof[7], E.prof[0], E.prof[2], E.prof[4], E.prof[9]);
#endif
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
