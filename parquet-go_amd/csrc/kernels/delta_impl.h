// delta_impl.h — DELTA_BINARY_PACKED on the device (included by decode.hip).
//
// Reference: deltaBitPackDecoder32/64 (deltabp_decoder.go:13-333).  The stream is a chain of
// blocks whose byte length depends on their own header (varint minDelta + miniblock widths), so
// it is walked sequentially, once per page, by one wave64 reading the page through an LDS window
// (k_delta_walk).  The walk replays next()'s exact read pattern — eager block + first miniblock
// header at init, the one-delta read-ahead, the padding skip at position+8 >= valuesCount with its
// currentMiniBlock index quirk (:149-164) — and records, per block, minDelta, widths and the data
// offset.  Decoding is then data parallel: per-tile delta sums (k_delta_sum) -> per-page exclusive
// scan seeded with the first value (k_delta_scan) -> per tile: unpack from LDS, block-wide scan,
// store (TK_DELTA in k_expand).  Streams outside the fast-path geometry (miniblock count > 8,
// miniblock values not a multiple of 8, block size not dividing 2048) are decoded by an exact
// sequential restatement (TK_DELTA_SERIAL).
#pragma once

constexpr int kWin = 8192;  // LDS window per wave for the block walk

struct Win {
  const uint8_t* img;
  int64_t e;     // end of the stream (image offset)
  uint8_t* buf;  // LDS, kWin bytes
  int64_t lo, hi;
};

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Refill the window so that it starts at (16-byte aligned) pos.  Bytes at or past `e` are never
// interpreted (every read checks pos < e); the 16-byte loads stay inside the payload pad.
__device__ __forceinline__ void win_load(Win& w, int64_t pos, int lane) {
  const int64_t lo = pos - int64_t((reinterpret_cast<uintptr_t>(w.img) + uintptr_t(pos)) & 15);
  constexpr int kPer = kWin / 16 / 64, kHalf = kPer / 2;
  wave_lds_sync();
  // loads in flight four at a time (addresses past the stream clamp to `lo`)
  for (int h = 0; h < kPer; h += kHalf) {
    uint4 x[kHalf];
#pragma unroll
    for (int k = 0; k < kHalf; k++) {
      const int64_t o = lo + 16 * int64_t(lane + 64 * (h + k));
      x[k] = *reinterpret_cast<const uint4*>(w.img + (o < w.e ? o : lo));
    }
#pragma unroll
    for (int k = 0; k < kHalf; k++) {
      const int64_t o = lo + 16 * int64_t(lane + 64 * (h + k));
      reinterpret_cast<uint4*>(w.buf)[lane + 64 * (h + k)] = o < w.e ? x[k] : make_uint4(0, 0, 0, 0);
    }
  }
  wave_lds_sync();
  w.lo = lo;
  w.hi = lo + kWin;
}

__device__ __forceinline__ void win_ensure(Win& w, int64_t pos, int need, int lane) {
  if (pos < w.lo || pos + need > w.hi) win_load(w, pos, lane);
}

// binary.ReadUvarint through the window.
__device__ int win_uvarint(Win& w, int64_t& pos, uint64_t& v, int lane) {
  win_ensure(w, pos, 10, lane);
  uint64_t x = 0;
  int s = 0;
  for (int i = 0; i < 10; i++) {
    if (pos >= w.e) return i ? PQH_ERR_UNEXPECTED_EOF : PQH_ERR_EOF;
    const uint32_t c = w.buf[pos - w.lo];
    pos++;
    if (c < 0x80) {
      if (i == 9 && c > 1) return PQH_ERR_VARINT_OVERFLOW;
      v = x | (uint64_t(c) << s);
      return PQH_OK;
    }
    x |= uint64_t(c & 0x7f) << s;
    s += 7;
  }
  return PQH_ERR_VARINT_OVERFLOW;
}

// readUVariant32 (helpers.go:151-167)
__device__ __forceinline__ int win_uvar32(Win& w, int64_t& pos, int32_t& out, int lane) {
  uint64_t v;
  int st = win_uvarint(w, pos, v, lane);
  if (st) return st;
  if (v > 0x7fffffffull) return PQH_ERR_INT32_RANGE;
  out = int32_t(v);
  return PQH_OK;
}

// readVariant32 / readVariant64 (helpers.go:169-208) as uint64 bits
__device__ __forceinline__ int win_varint(Win& w, int64_t& pos, bool is64, uint64_t& out, int lane) {
  uint64_t u;
  int st = win_uvarint(w, pos, u, lane);
  if (st) return st;
  const int64_t x = int64_t(u >> 1) ^ -int64_t(u & 1);
  if (!is64 && (x > 2147483647ll || x < -2147483648ll)) return PQH_ERR_INT32_RANGE;
  out = uint64_t(x);
  return PQH_OK;
}

// readMiniBlockHeader (:88-111 / :247-270): minDelta + mb_count width bytes (mb_count <= 8).
__device__ __forceinline__ int win_miniblock_header(Win& w, int64_t& pos, bool is64, int mbc, uint64_t& min_delta,
                                                    uint64_t& widths, int lane) {
  int st = win_varint(w, pos, is64, min_delta, lane);
  if (st) return st;
  const int64_t avail = w.e - pos;
  if (avail <= 0) return PQH_ERR_EOF;
  if (avail < mbc) return PQH_ERR_UNEXPECTED_EOF;
  win_ensure(w, pos, 8, lane);
  widths = 0;
  for (int i = 0; i < mbc; i++) {
    const uint32_t wb = w.buf[pos - w.lo + i];
    if (wb > (is64 ? 64u : 32u)) return PQH_ERR_DELTA_BIT_WIDTH;
    widths |= uint64_t(wb) << (8 * i);
  }
  pos += mbc;
  return PQH_OK;
}

__device__ __forceinline__ int mb_width(uint64_t widths, int m) { return int((widths >> (8 * m)) & 0xff); }

__device__ __forceinline__ uint64_t rfl64(uint64_t x) {
  return uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(x))))) |
         (uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(int(uint32_t(x >> 32))))) << 32);
}

// Bytes [pos, pos + 16) of the window as two little-endian words (window holds pos + 24).
__device__ __forceinline__ void win_bytes16(const Win& w, int64_t pos, uint64_t& a, uint64_t& b) {
  const int64_t off = pos - w.lo;
  const uint64_t* q = reinterpret_cast<const uint64_t*>(w.buf) + (off >> 3);
  // the walk is wave-uniform: move the words to SGPRs so the header arithmetic runs on the SALU
  const uint64_t x0 = rfl64(q[0]), x1 = rfl64(q[1]), x2 = rfl64(q[2]);
  const int sh = int(off & 7) * 8;
  a = sh ? (x0 >> sh) | (x1 << (64 - sh)) : x0;
  b = sh ? (x1 >> sh) | (x2 << (64 - sh)) : x1;
}

// Common case of readMiniBlockHeader: a varint of <= 8 bytes followed by the widths, all well inside
// the stream, values in range.  One LDS round trip; anything else returns false and the exact
// byte-by-byte reader produces the reference's error.
__device__ __forceinline__ bool fast_block_header(Win& w, int64_t& pos, bool is64, int mbc, uint64_t& md,
                                                  uint64_t& widths, int lane) {
  if (w.e - pos < 24) return false;
  win_ensure(w, pos, 24, lane);
  uint64_t a, b;
  win_bytes16(w, pos, a, b);
  const uint64_t stop = ~a & 0x8080808080808080ull;
  if (!stop) return false;
  const int len = (__builtin_ctzll(stop) >> 3) + 1;
  uint64_t u = 0;
#pragma unroll
  for (int i = 0; i < 8; i++)
    if (i < len) u |= ((a >> (8 * i)) & 0x7f) << (7 * i);
  const int64_t x = int64_t(u >> 1) ^ -int64_t(u & 1);
  if (!is64 && (x > 2147483647ll || x < -2147483648ll)) return false;
  const int sh = len * 8;
  uint64_t wd = sh == 64 ? b : (a >> sh) | (b << (64 - sh));
  if (mbc < 8) wd &= (1ull << (8 * mbc)) - 1;
  const uint32_t lim = is64 ? 64u : 32u;
  bool ok = true;
#pragma unroll
  for (int m = 0; m < 8; m++) ok = ok && ((wd >> (8 * m)) & 0xff) <= lim;
  if (!ok) return false;
  md = uint64_t(x);
  widths = wd;
  pos += len + mbc;
  return true;
}

__device__ __forceinline__ int64_t block_data_bytes(uint64_t widths, int mbvc) {
  int64_t sum = 0;
#pragma unroll
  for (int m = 0; m < 8; m++) sum += int64_t((widths >> (8 * m)) & 0xff);
  return sum * (mbvc / 8);
}

// ------------------------------------------------------------------------------------------------
// Speculative lane-parallel block chain.  Walking the chain one block at a time costs the wave a
// dependent round trip plus ~150 wave-uniform instructions per block, for 1024 blocks per
// reference-writer page.  Instead the 64 lanes each take one byte segment of the stream, find a
// plausible header in it (two consecutive headers that parse), and walk their own chain through
// L2 until they leave the segment.  The segments are then stitched in order: from the true header
// that enters a segment, the chain is deterministic, so a lane's list is kept from that header on.
// A segment whose walk never meets the true chain, or outgrows its list, ends the speculation
// there and the exact sequential walk takes over from the last verified header.
// ------------------------------------------------------------------------------------------------
constexpr int kSpecCap = kWin / (64 * 4);



// The common-case readMiniBlockHeader over 16 bytes (a = bytes 0-7, b = 8-15): varint minDelta of
// <= 8 bytes, value in range, mbc width bytes <= the limit.  Returns the header length or 0.
__device__ __forceinline__ int parse_hdr16(uint64_t a, uint64_t b, bool is64, int mbc, uint64_t& md, uint64_t& wd) {
  const uint64_t stop = ~a & 0x8080808080808080ull;
  if (!stop) return 0;
  const int len = (__builtin_ctzll(stop) >> 3) + 1;
  // the len 7-bit groups, packed (SWAR: 8x7 -> 4x14 -> 2x28 -> 56 bits)
  const int sh = len * 8;
  uint64_t u = (sh == 64 ? a : a & ((1ull << sh) - 1)) & 0x7f7f7f7f7f7f7f7full;
  u = (u & 0x007f007f007f007full) | ((u & 0x7f007f007f007f00ull) >> 1);
  u = (u & 0x00003fff00003fffull) | ((u & 0x3fff00003fff0000ull) >> 2);
  u = (u & 0x000000000fffffffull) | ((u & 0x0fffffff00000000ull) >> 4);
  const int64_t x = int64_t(u >> 1) ^ -int64_t(u & 1);
  if (!is64 && (x > 2147483647ll || x < -2147483648ll)) return 0;
  uint64_t w = sh == 64 ? b : (a >> sh) | (b << (64 - sh));
  if (mbc < 8) w &= (1ull << (8 * mbc)) - 1;
  // any byte > lim: high bit set, or low 7 bits + (127 - lim) carries into bit 7 (no cross-byte carry)
  const uint64_t lim = is64 ? 64 : 32;
  const uint64_t bad = (((w & 0x7f7f7f7f7f7f7f7full) + (0x7f - lim) * 0x0101010101010101ull) | w) &
                       0x8080808080808080ull;
  if (bad) return 0;
  md = uint64_t(x);
  wd = w;
  return len + mbc;
}

__device__ __forceinline__ int64_t widths_sum(uint64_t w) {
  const uint64_t m = 0x00ff00ff00ff00ffull;
  uint64_t t = (w & m) + ((w >> 8) & m);  // 4 x 16-bit sums
  t += t >> 16;
  t += t >> 32;
  return int64_t(t & 0xffff);
}

typedef const __attribute__((address_space(1))) uint64_t* gptr64;

// The 16 bytes at image offset p (image 8-byte aligned) as two little-endian words.
__device__ __forceinline__ void bytes16_global(const uint8_t* img, int64_t p, uint64_t& a, uint64_t& b) {
  const gptr64 q = (gptr64)(img + (p & ~int64_t(7)));
  const uint64_t x0 = q[0], x1 = q[1], x2 = q[2];
  const uint32_t sh = uint32_t(p & 7) * 8;
  a = sh ? (x0 >> sh) | (x1 << (64 - sh)) : x0;
  b = sh ? (x1 >> sh) | (x2 << (64 - sh)) : x1;
}

typedef uint4 uint4_a8 __attribute__((aligned(8)));

// Per lane, through L2: the header at image offset p.  dat = its data, nxt = the next header; false
// unless the common-case parse applies and the whole block lies inside the stream.  One 16-byte load
// (8-byte aligned) covers headers of up to 9 - p % 8 bytes; longer ones load the next 8 bytes.
__device__ __forceinline__ bool hdr_global(const uint8_t* img, int64_t p, int64_t e, bool is64, int mbc, int gbytes,
                                           uint64_t& md, uint64_t& wd, int64_t& dat, int64_t& nxt) {
  if (e - p < 24) return false;
  const uint8_t* q = img + (p & ~int64_t(7));
  const uint4 v = *reinterpret_cast<const uint4_a8*>(q);
  const uint64_t x0 = uint64_t(v.x) | (uint64_t(v.y) << 32), x1 = uint64_t(v.z) | (uint64_t(v.w) << 32);
  const uint32_t sh = uint32_t(p & 7) * 8;
  const uint64_t a = sh ? (x0 >> sh) | (x1 << (64 - sh)) : x0;
  uint64_t b = sh ? x1 >> sh : x1;
  // header bytes past q + 16: varint terminator at byte len - 1 of a, then mbc width bytes
  const uint64_t stop = ~a & 0x8080808080808080ull;
  const int len = stop ? (__builtin_ctzll(stop) >> 3) + 1 : 8;
  if (sh && int(sh / 8) + len + mbc > 16) b |= ((gptr64)q)[2] << (64 - sh);
  const int hl = parse_hdr16(a, b, is64, mbc, md, wd);
  if (!hl) return false;
  dat = p + hl;
  nxt = dat + widths_sum(wd) * gbytes;
  return nxt <= e;
}

// A block record written by the speculative walk holds only its header position (pad == 1): the
// consumer parses the header (already validated by the walk) when it loads the record.
__device__ __forceinline__ DeltaBlock load_block(const DeltaBlock* recs, int64_t i, const uint8_t* img, bool is64,
                                                 int mbc) {
  DeltaBlock r = recs[i];
  if (r.pad) {
    uint64_t a, b, md = 0, wd = 0;
    bytes16_global(img, r.data_off, a, b);
    r.data_off += parse_hdr16(a, b, is64, mbc, md, wd);
    r.min_delta = md;
    r.widths = wd;
    r.pad = 0;
  }
  return r;
}

__device__ __forceinline__ int64_t readlane64(int64_t x, int i) {
  return int64_t(uint64_t(uint32_t(__builtin_amdgcn_readlane(int(uint32_t(uint64_t(x))), i))) |
                 (uint64_t(uint32_t(__builtin_amdgcn_readlane(int(uint32_t(uint64_t(x) >> 32)), i))) << 32));
}

// Per byte of x: MSB set where the byte is <= lim (lim < 128; no carries cross bytes).
__device__ __forceinline__ uint64_t small_bytes(uint64_t x, uint64_t lim) {
  return ~(((x & 0x7f7f7f7f7f7f7f7full) + (0x7f - lim) * 0x0101010101010101ull) | x) & 0x8080808080808080ull;
}

// Per lane: the first position in [s0, s1) whose header parses (s1 if none).  32 positions per
// step: a byte-parallel filter keeps the positions p whose byte is a varint terminator (< 0x80)
// followed by mbc bytes <= the width limit, and only those get a full parse (L1-hot).  A header
// whose varint ends at byte p has the same widths and successor as the 1-byte varint at p, so p
// stands for every start of that varint (the stitch resolves which one is true).
__device__ int64_t spec_sync(const uint8_t* img, int64_t s0, int64_t s1, int64_t e, bool is64, int mbc,
                                          int gbytes) {
  const uint64_t lim = is64 ? 64 : 32;
  const int64_t se = s1 < e - 24 ? s1 : e - 24;  // headers need 24 bytes before the stream end
  for (int64_t base = s0 & ~int64_t(15); base < se; base += 32) {
    uint64_t cand[4];
    {
      // bytes past the stream end are read from the following image or the payload pad (>= 256
      // zero bytes after the last image) and never accepted: hdr_global wants 24 bytes before e
      const uint4* q4 = reinterpret_cast<const uint4*>(img + base);
      const uint4 c0 = q4[0], c1 = q4[1], c2 = q4[2];
      const uint64_t x[5] = {uint64_t(c0.x) | (uint64_t(c0.y) << 32), uint64_t(c0.z) | (uint64_t(c0.w) << 32),
                             uint64_t(c1.x) | (uint64_t(c1.y) << 32), uint64_t(c1.z) | (uint64_t(c1.w) << 32),
                             uint64_t(c2.x) | (uint64_t(c2.y) << 32)};
      uint64_t x0 = x[0], S0 = small_bytes(x0, lim);
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint64_t x1 = x[j + 1], S1 = small_bytes(x1, lim);
        uint64_t c = ~x0 & 0x8080808080808080ull;
        for (int k = 1; k <= mbc; k++) c &= k == 8 ? S1 : (S0 >> (8 * k)) | (S1 << (64 - 8 * k));
        cand[j] = c;
        x0 = x1;
        S0 = S1;
      }
    }
    for (int j = 0; j < 4; j++) {
      uint64_t c = cand[j];
      const int64_t w0 = base + 8 * j;
      if (s0 > w0) c &= s0 - w0 >= 8 ? 0 : ~0ull << (8 * (s0 - w0));
      if (se - w0 < 8) c &= se <= w0 ? 0 : (1ull << (8 * (se - w0))) - 1;
      while (c) {
        const int64_t p = w0 + (__builtin_ctzll(c) >> 3);
        c &= c - 1;
        uint64_t md, wd;
        int64_t dat, n1;
        if (hdr_global(img, p, e, is64, mbc, gbytes, md, wd, dat, n1)) return p;
      }
    }
  }
  return s1;
}

// Headers of the whole blocks [1, kmax) starting at h1 (block 1's header): records written, returns
// r = blocks recorded including block 0 (1 <= r <= kmax) and *hr = the header of block r.  Rounds:
// the span of the blocks still missing is estimated from the bytes per block so far and split over
// the lanes; every round advances at least through lane 0's segment unless the true chain reaches
// a header the fast parse rejects (the exact walk takes over there).
__device__ int spec_chain(const uint8_t* img, int64_t h1, int64_t e, bool is64, int mbc, int gbytes, int bs,
                          int kmax, int64_t blk0_bytes, DeltaBlock* recs, int32_t* lst, int lane, int64_t& hr) {
  int64_t T = h1, bytes_done = blk0_bytes;
  int nb = 1;
  while (nb < kmax) {
    const int64_t avg = bytes_done / nb > 0 ? bytes_done / nb : 1;
    int64_t span = int64_t(kmax - nb) * avg;
    span += span / 8 + 64;
    if (span > e - T) span = e - T;
    int64_t seg = (span + 63) / 64;
    if (seg < 32) seg = 32;
    const int64_t s0 = T + seg * lane, s1 = s0 + seg;
    int cnt = 0;
    bool dead = false;
    int64_t p = s0, x2 = -1;
    wave_lds_sync();  // the previous round's readers of the lists are done
    if (s0 < e) {
      uint64_t md, wd;
      int64_t dat, n1;
      if (lane > 0) p = spec_sync(img, s0, s1, e, is64, mbc, gbytes);
      while (p < s1 && cnt < kSpecCap - 1) {
        lst[cnt * 64 + lane] = int32_t(p);
        cnt++;
        if (!hdr_global(img, p, e, is64, mbc, gbytes, md, wd, dat, n1)) {
          if (cnt == 2 && lane > 0) {  // the synchronisation point's successor does not parse: scan on
            cnt = 0;
            p = spec_sync(img, int64_t(lst[lane]) + 1, s1, e, is64, mbc, gbytes);
            continue;
          }
          dead = true;
          break;
        }
        p = n1;
      }
      // one block past the segment: the exit header (list slot cnt, not counted) and its successor
      if (!dead && p >= s1 && p < e) {
        lst[cnt * 64 + lane] = int32_t(p);
        if (hdr_global(img, p, e, is64, mbc, gbytes, md, wd, dat, n1)) x2 = n1;
      }
    }
    const bool full = !dead && p < s1;
    wave_lds_sync();
    // ---- stitch.  In parallel: where the left neighbour's exit header (and its successor) sit in
    // my list; the true chain runs through every lane linked to its left neighbour that way.
    const int64_t T0 = T;
    const int nb0 = nb;
    const int nseg = int((e - T0 + seg - 1) / seg) < 64 ? int((e - T0 + seg - 1) / seg) : 64;
    const bool exit_ok = s0 < e && !dead && !full && p < e;
    const int64_t xl = __shfl_up(p, 1, 64), x2l = __shfl_up(x2, 1, 64);
    const bool left_ok = __shfl_up(int(exit_ok), 1, 64) != 0 && xl >= s0 && xl < s1;
    int jd = -1, j2 = -1;
    if (lane > 0 && left_ok) {
      for (int k = 0; k < cnt; k++) {
        const int32_t q = lst[k * 64 + lane];
        if (jd < 0 && q == int32_t(xl)) jd = k;
        if (j2 < 0 && x2l >= 0 && q == int32_t(x2l)) j2 = k;
      }
      // the left neighbour's exit is my segment's only true header: its successor is my exit
      if (jd < 0 && j2 < 0 && exit_ok && x2l == p) j2 = cnt;
    }
    const bool link = lane < nseg && (lane == 0 || (left_ok && (jd >= 0 || j2 >= 0)));
    int j = lane == 0 ? 0 : (jd >= 0 ? jd : j2);
    // lane i synchronised just before T (the previous block's last data bytes continuing into T's
    // varint) or on T's varint terminator and joined the true chain one block later: its left
    // neighbour parsed T as its exit header (list slot cnt) and records it
    const bool extra = lane > 0 && link && jd < 0;
    const uint64_t linkm = __ballot(link);
    const int k_bad = linkm == ~0ull ? 64 : __builtin_ctzll(~linkm);
    const uint64_t deadm = __ballot(dead && lane < nseg) & (k_bad >= 64 ? ~0ull : (1ull << k_bad) - 1);
    const int last = deadm ? __builtin_ctzll(deadm) : k_bad - 1;
    const bool valid = lane <= last;
    const bool extra_r = __shfl_down(int(extra), 1, 64) != 0 && lane + 1 <= last && lane < 63;
    const int n_all = valid ? cnt - j - (dead ? 1 : 0) + (extra_r ? 1 : 0) : 0;
    int incl = n_all;
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(incl, off, 64);
      if (lane >= off) incl += y;
    }
    const int base = nb + incl - n_all;
    const int total = __builtin_amdgcn_readlane(incl, 63);
    int my_j = j, my_base = base;
    int my_n = base + n_all > kmax ? (kmax - base > 0 ? kmax - base : 0) : n_all;
    bool stop = false;
    int i_next = last + 1;
    if (nb + total >= kmax) {
      // block kmax's header: the entry after the last kept one
      const bool hit = valid && base <= kmax && kmax < base + n_all;
      const uint64_t hm = __ballot(hit);
      const int32_t q = hit ? lst[(j + (kmax - base)) * 64 + lane] : 0;
      T = hm ? int64_t(__builtin_amdgcn_readlane(q, __builtin_ctzll(hm))) : readlane64(p, last);
      nb = kmax;
      stop = true;
    } else {
      nb += total;
      if (deadm) {  // the true chain reached a header the fast parse rejects
        const int32_t q = lst[(cnt > 0 ? cnt - 1 : 0) * 64 + lane];
        T = int64_t(__builtin_amdgcn_readlane(q, last));
        stop = true;
      } else if (last >= 0) {
        T = readlane64(p, last);
      }
    }
    // the rare cases, one segment at a time (wave-uniform): a block longer than a segment, a lane
    // whose walk joined the true chain late or never, a lane that outgrew its list
    for (int i = i_next; i < nseg && nb < kmax && !stop; i++) {
      const int64_t seg_end = T0 + seg * (i + 1);
      if (T >= seg_end) continue;  // no true header in segment i
      const int ci = __builtin_amdgcn_readlane(cnt, i);
      const bool di = __builtin_amdgcn_readlane(int(dead), i) != 0;
      const bool fi = __builtin_amdgcn_readlane(int(full), i) != 0;
      const int64_t xi = readlane64(p, i);
      uint64_t m = __ballot(lane < ci && lst[lane * 64 + i] == int32_t(T));
      // follow the true chain a few blocks by hand until it meets lane i's walk
      for (int t = 0; t < 3 && !m && nb < kmax && T < seg_end; t++) {
        uint64_t md, wd;
        int64_t dat, nx;
        if (!hdr_global(img, T, e, is64, mbc, gbytes, md, wd, dat, nx)) {
          stop = true;
          break;
        }
        if (lane == 0) recs[nb] = DeltaBlock{md, int32_t(dat), int32_t(T), wd, 0};
        nb++;
        T = nx;
        m = __ballot(lane < ci && lst[lane * 64 + i] == int32_t(T));
      }
      if (stop || nb >= kmax) break;
      if (T >= seg_end) continue;
      if (!m) break;  // lane i's walk never met the true chain: next round from T
      const int jj = __builtin_ctzll(m);
      int n = ci - jj - (di ? 1 : 0);
      if (nb + n > kmax) n = kmax - nb;
      if (lane == i) {
        my_j = jj;
        my_n = n;
        my_base = nb;
      }
      nb += n;
      T = jj + n < ci ? int64_t(__builtin_amdgcn_readfirstlane(lst[(jj + n) * 64 + i])) : xi;
      if (di) stop = true;
      if (di || fi) break;
    }
    // records: header positions only (pad = 1), parsed by their consumers
    for (int k = 0; k < my_n; k++) {
      const int b = my_base + k;
      const int32_t h = lst[(my_j + k) * 64 + lane];
      recs[b] = DeltaBlock{0, h, h, 0, 1};
    }
    if (nb == nb0 || stop) break;
    bytes_done += T - T0;
  }
  wave_lds_sync();
  hr = T;
  return nb;
}

// deltaBitPackDecoder.init (page load, phase 0 step 3): readBlockHeader + the first
// readMiniBlockHeader.  D.mode = DM_FAST (geometry of the data-parallel path; pos = block 0's data),
// DM_SERIAL (other geometries: the exact sequential decoder redoes the page) or an error key.
__device__ uint64_t delta_init(Win& w, int64_t& pos, bool is64, DeltaState& D, int32_t& vc, uint64_t& md,
                               uint64_t& widths, int lane, int64_t* hdr0 = nullptr) {
  int st;
  int32_t bs, mbc;
  if ((st = win_uvar32(w, pos, bs, lane))) return err_key(0, 3, st);
  if ((st = win_uvar32(w, pos, mbc, lane))) return err_key(0, 3, st);
  if (mbc <= 0 || bs % mbc != 0) return err_key(0, 3, PQH_ERR_DELTA_MINIBLOCKS);
  const int32_t mbvc = bs / mbc;
  if (mbvc == 0) return err_key(0, 3, PQH_ERR_DELTA_MINIBLOCKS);
  if ((st = win_uvar32(w, pos, vc, lane))) return err_key(0, 3, st);
  uint64_t first;
  if ((st = win_varint(w, pos, is64, first, lane))) return err_key(0, 3, st);
  D.block_size = bs;
  D.mb_count = mbc;
  D.mbvc = mbvc;
  D.first = first;
  const bool fast = mbc <= 8 && (mbvc & 7) == 0 && bs >= kDeltaBlockMin && (2048 % bs) == 0;
  if (!fast) {
    D.mode = DM_SERIAL;
    return kNoError;
  }
  if (hdr0) *hdr0 = pos;
  if ((st = win_miniblock_header(w, pos, is64, mbc, md, widths, lane))) return err_key(0, 3, st);
  D.mode = DM_FAST;
  return kNoError;
}

// Whole blocks [0, kmax): every group read of blocks before the padding-skip group and the last
// reachable position succeeds when the block lies inside the stream.
__device__ __forceinline__ int64_t delta_whole_blocks(int64_t nn, int32_t vc, int32_t bs, int32_t cap) {
  const int64_t L = nn < vc ? nn : vc;
  const int64_t pstar = vc <= 8 ? 0 : ((int64_t(vc) - 8 + 7) / 8) * 8;
  const int64_t lp = L < pstar ? L : pstar;
  return lp / bs < cap ? lp / bs : cap;
}

// The block walk of one page (whole wave, uniform).  Returns the first error key.
// init_all: byteArrayDeltaLengthDecoder.init (type_bytearray.go:104-116) decodes ALL valuesCount
// lengths at page load: every error is a load error (phase 0, step 3) and nn is ignored.
__device__ uint64_t delta_walk(Win& w, int64_t vs, bool is64, int64_t nn, DeltaBlock* recs, int32_t cap,
                               DeltaState& D, int lane, bool init_all, int spec_r = 0, int64_t spec_hr = 0) {
  D.mode = DM_NONE;
  D.nblocks = 0;
  D.limit = 0;
  D.first = 0;
  D.end_pos = vs;
  D.rec_base = 0;
  D.head_blocks = 0;
  D.head_carry = 0;
  D.head_neg = INT64_MAX;
  int64_t pos = vs;
  int st;
  int32_t vc;
  uint64_t md, widths;
  int64_t hpos = pos;  // header of the block being read
  const uint64_t ik = delta_init(w, pos, is64, D, vc, md, widths, lane, &hpos);
  if (ik != kNoError || D.mode != DM_FAST) return ik;
  const int32_t bs = D.block_size, mbc = D.mb_count, mbvc = D.mbvc;
  // ---- readValues: positions [0, nn) (phase 3) ----
  if (init_all) nn = vc;
  const int64_t L = nn < vc ? nn : vc;                                 // reachable positions
  const int64_t pstar = vc <= 8 ? 0 : ((int64_t(vc) - 8 + 7) / 8) * 8;  // padding-skip group
  const int64_t gbytes = mbvc / 8;
  uint64_t err = kNoError;
  int64_t limit = nn;
  bool padded = false;
  int64_t b_start = 0;
  if (spec_r >= 1 && spec_r <= delta_whole_blocks(nn, vc, bs, cap)) {
    // blocks [1, spec_r) recorded by k_delta_spec, or [0, spec_r) decoded by k_delta_fused; resume
    // at block spec_r's header
    if (lane == 0) recs[0] = DeltaBlock{md, int32_t(pos), int32_t(hpos), widths, 0};
    D.nblocks = spec_r;
    b_start = spec_r;
    pos = spec_hr;
  }
  for (int64_t b = b_start; int64_t(b) * bs < L && !padded && err == kNoError; b++) {
    const int64_t p0 = b * bs;
    if (b > 0) hpos = pos;
    if (b > 0 && !fast_block_header(w, pos, is64, mbc, md, widths, lane) &&
        (st = win_miniblock_header(w, pos, is64, mbc, md, widths, lane))) {
      err = init_all ? err_key(0, 3, st) : err_key(3, p0, st);
      limit = p0;
      break;
    }
    if (D.nblocks >= cap) {
      D.mode = DM_SERIAL;
      return kNoError;
    }
    if (lane == 0) recs[D.nblocks] = DeltaBlock{md, int32_t(pos), int32_t(hpos), widths, 0};
    D.nblocks++;
    // a whole block before the padding group and the last reachable position, inside the stream:
    // every group read succeeds
    if (p0 + bs <= L && p0 + bs <= pstar) {
      const int64_t nb = block_data_bytes(widths, mbvc);
      if (pos + nb <= w.e) {
        pos += nb;
        continue;
      }
    }
    for (int m = 0; m < mbc; m++) {
      const int64_t pm = p0 + int64_t(m) * mbvc;
      if (pm >= L) break;
      const int wm = mb_width(widths, m);
      const int64_t pend = pm + mbvc < L ? pm + mbvc : L;
      const bool has_pad = pstar >= pm && pstar < pend;
      const int64_t ng = has_pad ? (pstar - pm) / 8 + 1 : (pend - pm + 7) / 8;  // group reads
      if (wm > 0 && pos + ng * wm > w.e) {  // io.ReadFull(w bytes) per group: the first group past the end fails
        const int64_t avail = w.e - pos > 0 ? w.e - pos : 0;
        const int64_t gf = avail / wm;
        if (gf < ng) {
          const int code = avail - gf * wm <= 0 ? PQH_ERR_EOF : PQH_ERR_UNEXPECTED_EOF;
          err = init_all ? err_key(0, 3, code) : err_key(3, pm + 8 * gf, code);
          limit = pm + 8 * gf;
          break;
        }
      }
      pos += ng * wm;
      if (has_pad) {  // skip the rest of this miniblock, then (sic) widths[currentMiniBlock] per miniblock left
        const int64_t l = gbytes * wm - ng * wm;
        pos = pos + l < w.e ? pos + l : (pos > w.e ? pos : w.e);
        if (m + 1 < mbc) {
          const int w2 = mb_width(widths, m + 1);
          for (int i = m + 1; i < mbc; i++)
            if (w2 != 0) pos = pos + gbytes * w2 < w.e ? pos + gbytes * w2 : (pos > w.e ? pos : w.e);
        }
        padded = true;
        break;
      }
    }
  }
  if (err == kNoError && nn > vc) {  // next() at position >= valuesCount -> io.EOF
    err = err_key(3, vc, PQH_ERR_EOF);
    limit = vc;
  }
  D.limit = int32_t(limit);
  D.end_pos = pos;
  return err;
}

// One wave per delta page.
// k_delta_spec: one wave per delta page, before k_delta_walk.  The page's init (as delta_walk), then
// the speculative chain of its whole blocks [1, kmax): records written, (blocks found, header of the
// next block) left in dstates[p].nblocks / end_pos for the walk to resume from.  DELTA_BYTE_ARRAY
// suffix streams start where the prefix stream ends and are walked by k_delta_walk alone.
__global__ __launch_bounds__(256) void k_delta_spec(DevBatch b, const int32_t* delta_pages, int32_t n) {
  __shared__ __attribute__((aligned(16))) uint8_t win_all[4][kWin];
  const int lane = threadIdx.x & 63;
  const int wv = int(threadIdx.x >> 6);
  const int idx = __builtin_amdgcn_readfirstlane(int(blockIdx.x) * 4 + wv);
  if (idx >= n) return;
  const int p = delta_pages[idx];
  const DevPage P = b.pages[p];
  const PageState S = b.states[p];
  int r = 0;
  int64_t hr = 0;
  const bool load_ok = S.err == kNoError || (S.err >> 56) > 0;
  if (P.host_err == kNoError && load_ok) {
    Win w{b.payload + P.image_off, S.val_e, win_all[wv], 0, 0};
    win_load(w, S.val_s, lane);
    const bool is64 = P.kind == K_DELTA64;
    const bool before_values = S.err != kNoError && (S.err >> 56) <= 2;
    DeltaState D;
    int32_t vc;
    uint64_t md, widths;
    int64_t pos = S.val_s;
    if (delta_init(w, pos, is64, D, vc, md, widths, lane) == kNoError && D.mode == DM_FAST) {
      const int64_t nn = P.kind == K_DLBA || P.kind == K_DBA ? vc : (before_values ? 0 : S.nn);
      const int64_t kmax = delta_whole_blocks(nn, vc, D.block_size, P.dblk_cap);
      const int64_t h1 = pos + block_data_bytes(widths, D.mbvc);
      if (kmax >= 2 && h1 <= w.e)
        r = spec_chain(w.img, h1, w.e, is64, D.mb_count, D.mbvc / 8, D.block_size, int(kmax), h1 - S.val_s,
                       b.dblocks + P.dblk_base, reinterpret_cast<int32_t*>(w.buf), lane, hr);
    }
  }
  if (lane == 0) {
    b.dstates[p].nblocks = r;
    b.dstates[p].end_pos = hr;
    b.dstates[p].head_blocks = 0;
  }
}

// One wave per delta page.
__global__ __launch_bounds__(256) void k_delta_walk(DevBatch b, const int32_t* delta_pages, int32_t n) {
  __shared__ __attribute__((aligned(16))) uint8_t win_all[4][kWin];
  const int lane = threadIdx.x & 63;
  const int wv = int(threadIdx.x >> 6);
  const int idx = __builtin_amdgcn_readfirstlane(int(blockIdx.x) * 4 + wv);
  if (idx >= n) return;
  const int p = delta_pages[idx];
  const DevPage P = b.pages[p];
  const PageState S = b.states[p];
  const int spec_r = __builtin_amdgcn_readfirstlane(b.dstates[p].nblocks);
  const int64_t spec_hr = rfl64(uint64_t(b.dstates[p].end_pos));
  const int head_in = __builtin_amdgcn_readfirstlane(b.dstates[p].head_blocks);
  const uint64_t carry_in = rfl64(b.dstates[p].head_carry);
  const int64_t neg_in = int64_t(rfl64(uint64_t(b.dstates[p].head_neg)));
  DeltaState D, D1;
  D.mode = D1.mode = DM_NONE;
  D.block_size = D.mb_count = D.mbvc = D.nblocks = D.limit = D.rec_base = D.head_blocks = 0;
  D.head_carry = 0;
  D.head_neg = INT64_MAX;
  D.first = 0;
  D.end_pos = 0;
  D1 = D;
  uint64_t err = kNoError;
  const bool dba = P.kind == K_DBA;
  // A page whose earlier load steps failed never initialises its values decoder.
  const bool load_ok = S.err == kNoError || (S.err >> 56) > 0;
  if (P.host_err == kNoError && load_ok) {
    Win w{b.payload + P.image_off, S.val_e, win_all[wv], 0, 0};
    win_load(w, S.val_s, lane);
    const bool before_values = S.err != kNoError && (S.err >> 56) <= 2;
    DeltaBlock* recs = b.dblocks + P.dblk_base;
    err = delta_walk(w, S.val_s, P.kind == K_DELTA64, before_values ? 0 : S.nn, recs, P.dblk_cap, D, lane,
                     P.kind == K_DLBA || dba, spec_r, spec_hr);
    if (dba && err == kNoError) {
      // byteArrayDeltaDecoder.init (type_bytearray.go:195-211): prefix lengths, then the
      // DELTA_LENGTH suffix decoder on the rest; both decode every length at load
      if (D.mode == DM_FAST) {
        err = delta_walk(w, D.end_pos, false, 0, recs + D.nblocks, P.dblk_cap - D.nblocks, D1, lane, true);
        D1.rec_base = D.nblocks;
        if (err == kNoError && D1.mode == DM_FAST && D.limit != D1.limit)
          err = err_key(0, 3, PQH_ERR_DBA_COUNT);
        if (D1.mode == DM_SERIAL) D.mode = DM_SERIAL;  // the serial tile redoes both streams
      } else {
        D1.mode = DM_SERIAL;
      }
    }
  }
  // blocks decoded by k_delta_fused count only if the walk resumed right after them
  if (head_in > 0 && D.mode == DM_FAST && D.nblocks >= head_in && spec_r == head_in) {
    D.head_blocks = head_in;
    D.head_carry = carry_in;
    D.head_neg = neg_in;
  }
  if (lane == 0) {
    b.dstates[p] = D;
    if (dba) b.dstates[b.num_pages + p] = D1;
    if (err != kNoError) atomicMin(&b.states[p].err, (unsigned long long)err);
  }
}

// ------------------------------------------------------------------------------------------------
// Tile work: deltas of values [c0, c1) staged in LDS block by block.
// ------------------------------------------------------------------------------------------------
struct DeltaLds {
  int32_t mboff[16][8];  // byte offset of each miniblock's data relative to the stage start
  uint8_t mbw[16][8];
  uint64_t md[16];
  uint64_t wsum[4];
  int32_t lead;          // bytes between the 16-aligned stage start and the first data byte
  int32_t pad;
};

__device__ __forceinline__ uint64_t extract64(const uint32_t* stage, uint32_t bit, int w) {
  if (w == 0) return 0;
  const uint32_t k = bit >> 5, s = bit & 31;
  const uint64_t lo = uint64_t(stage[k]) | (uint64_t(stage[k + 1]) << 32);
  uint64_t v = s ? ((lo >> s) | (uint64_t(stage[k + 2]) << (64 - s))) : lo;
  return w >= 64 ? v : (v & ((1ull << w) - 1));
}

// n values of width w <= 32 starting at `bit`: one funnel shift each (v_alignbit) from the two
// dwords holding it; w == 0 gives zeros.
template <int N>
__device__ __forceinline__ void extract32n(const uint32_t* stage, uint32_t bit, int w, uint64_t md, uint64_t* d) {
  const uint32_t mask = w >= 32 ? ~0u : (1u << w) - 1;
#pragma unroll
  for (int j = 0; j < N; j++) {
    const uint32_t bj = bit + uint32_t(j * w), k = bj >> 5;
    d[j] = uint64_t(__builtin_amdgcn_alignbit(stage[k + 1], stage[k], bj & 31) & mask) + md;
  }
}

// Inclusive block-wide scan of one uint64 per thread; returns the exclusive prefix, *total set.
__device__ __forceinline__ uint64_t block_exclusive_scan(uint64_t x, uint64_t* wsum, uint64_t* total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t incl = x;
  for (int off = 1; off < 64; off <<= 1) {
    const uint64_t y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  if (lane == 63) wsum[wv] = incl;
  __syncthreads();
  uint64_t before = 0;
  for (int k = 0; k < wv; k++) before += wsum[k];
  *total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  __syncthreads();
  return before + incl - x;
}

// Process values [v0, v1) of a DM_FAST delta page: sum (store == false) or store values.
// Returns the sum of (delta + minDelta) over positions [v0, v1).  Sub-chunks of 256*VPT positions
// are staged in LDS from the byte holding the first position's bits (at most 8 KiB of deltas plus
// the headers of <= 16 blocks); VPT consecutive positions per thread always share one miniblock.
template <bool IS64>
__device__ uint64_t delta_tile(const DevBatch& b, const DevPage& P, const DeltaState& D, int64_t v0, int64_t v1,
                               uint64_t base, bool store, uint8_t* out, uint32_t* stage, DeltaLds& DL) {
  constexpr int VPT = IS64 ? 4 : 8;
  constexpr int SUB = kBlock * VPT;
  const uint8_t* img = b.payload + P.image_off;
  const DeltaBlock* recs = b.dblocks + P.dblk_base + D.rec_base;
  const int bs = D.block_size, mbvc = D.mbvc, mbc = D.mb_count;
  uint64_t carry = base, total_all = 0;
  for (int64_t c0 = v0; c0 < v1; c0 += SUB) {
    const int64_t c1 = c0 + SUB < v1 ? c0 + SUB : v1;
    const int bb0 = int(int32_t(c0) / bs), nb = int(int32_t(c1 - 1) / bs) - bb0 + 1;
    __syncthreads();
    if (threadIdx.x < nb) {  // per-block miniblock data offsets (image offsets)
      const DeltaBlock r = load_block(recs, bb0 + threadIdx.x, img, P.kind == K_DELTA64, mbc);
      int32_t off = r.data_off;
      for (int m = 0; m < 8; m++) {
        const int wm = m < mbc ? mb_width(r.widths, m) : 0;
        DL.mboff[threadIdx.x][m] = off;
        DL.mbw[threadIdx.x][m] = uint8_t(wm);
        off += (mbvc / 8) * wm;
      }
      DL.md[threadIdx.x] = r.min_delta;
    }
    __syncthreads();
    // exact byte range holding the bits of positions [c0, c1)
    const int32_t r0 = int32_t(c0) % bs, r1 = int32_t(c1 - 1) % bs;
    const int m0 = r0 / mbvc, j0 = r0 % mbvc;
    const int64_t q = c1 - 1;
    const int bl = int(int32_t(q) / bs) - bb0, m1 = r1 / mbvc, j1 = r1 % mbvc;
    const int64_t start = DL.mboff[0][m0] + (int64_t(j0) * DL.mbw[0][m0]) / 8;
    const int64_t end = DL.mboff[bl][m1] + (int64_t(j1 + 1) * DL.mbw[bl][m1] + 7) / 8;
    const int64_t a0 = start - int64_t((reinterpret_cast<uintptr_t>(img) + uintptr_t(start)) & 15);
    const int64_t nvec = end > a0 ? (end - a0 + 15) >> 4 : 0;
    const int64_t e = P.image_len;  // never past the page image (+pad)
    stage_copy(reinterpret_cast<uint4*>(stage), img + a0, nvec, e - a0);
    if (threadIdx.x == 0) {
      stage[nvec * 4] = 0;
      stage[nvec * 4 + 1] = 0;
    }
    __syncthreads();
    const int64_t p = c0 + VPT * int64_t(threadIdx.x);
    uint64_t d[VPT];
    uint64_t tsum = 0;
#pragma unroll
    for (int j = 0; j < VPT; j++) d[j] = 0;
    if (p < c1) {
      const int32_t rp = int32_t(p) % bs;
      const int blk = int(int32_t(p) / bs) - bb0;
      const int m = rp / mbvc;
      const int wm = DL.mbw[blk][m];
      const uint32_t bit0 = uint32_t(DL.mboff[blk][m] - a0) * 8 + uint32_t(rp % mbvc) * uint32_t(wm);
      const uint64_t md = DL.md[blk];
#pragma unroll
      for (int j = 0; j < VPT; j++) {
        const uint64_t x = p + j < c1 ? extract64(stage, bit0 + uint32_t(j * wm), wm) + md : 0;
        d[j] = x;
        tsum += x;
      }
    }
    uint64_t tot;
    const uint64_t excl = block_exclusive_scan(tsum, DL.wsum, &tot);
    if (store && p < c1) {
      uint64_t v = carry + excl;
      using T = typename std::conditional<IS64, uint64_t, uint32_t>::type;
      T vals[VPT];
#pragma unroll
      for (int j = 0; j < VPT; j++) {
        vals[j] = T(v);
        v += d[j];
      }
      T* o = reinterpret_cast<T*>(out) + p;
      if (p + VPT <= c1) {
        __builtin_memcpy(o, vals, sizeof(vals));
      } else {
#pragma unroll
        for (int j = 0; j < VPT; j++)
          if (p + j < c1) o[j] = vals[j];
      }
    }
    carry += tot;
    total_all += tot;
  }
  return total_all;
}

// ------------------------------------------------------------------------------------------------
// k_delta_expand: single pass over the packed deltas with a decoupled look-back across the tiles of
// a page (Merrill & Garland's single-pass scan).  Tiles take tickets in start order, so a tile's
// predecessor always started before it.  Per tile: unpack + sum (aggregate published), look back
// for the exclusive prefix (inclusive prefix published), unpack again from L2 and store
// value[i] = prefix + sum of the deltas before i.  Tile 0 of a page starts from the first value.
// ------------------------------------------------------------------------------------------------
// Whole-tile staging (the common case: a tile's packed deltas fit kTileStage bytes): the block
// table of the tile's <= 64 blocks and all of its bytes are loaded once; both phases read LDS only.
// Values are assigned in rows of 256 consecutive positions (thread t owns position row*256 + t), so
// every store is coalesced; each row is one block-wide scan.  Block and miniblock sizes are powers
// of two on the fast path (the block size divides 2048, the miniblock count divides it).
constexpr int kTileStage = 32768;
constexpr int kTileBlocks = kDeltaTile / kDeltaBlockMin;  // 64

struct TileStageLds {
  uint32_t data[(kTileStage + 64) / 4];
  int32_t mbbit[kTileBlocks][8];  // first bit of each miniblock's data in `data`
  uint8_t mbw[kTileBlocks][8];
  uint64_t md[kTileBlocks];
  uint64_t wtot[2][4];
  uint64_t wtot2[2][4];
  uint64_t mdb[kTileBlocks];  // expand_rows: minDelta sum of the tile's blocks before each block
  int32_t narrow;             // expand_rows: every miniblock width <= kNarrowWidth
  int32_t fits;
};

// Stage the tile; returns false (uniformly) when its bytes exceed kTileStage.
__device__ bool stage_tile(const DevBatch& b, const DevPage& P, const DeltaState& D, int64_t v0, int64_t v1,
                           TileStageLds& T) {
  const uint8_t* img = b.payload + P.image_off;
  const DeltaBlock* recs = b.dblocks + P.dblk_base + D.rec_base;
  const int lbs = __builtin_ctz(uint32_t(D.block_size));
  const int bb0 = int(v0 >> lbs), nb = int(((v1 - 1) >> lbs)) - bb0 + 1;
  const int mbc = D.mb_count, gbytes = D.mbvc / 8;
  if (nb > kTileBlocks || bb0 + nb > D.nblocks) return false;  // (uniform) not stageable
  __shared__ int64_t s_start, s_end;
  if (threadIdx.x < nb) {
    const DeltaBlock r = load_block(recs, bb0 + threadIdx.x, img, P.kind == K_DELTA64, mbc);
    int32_t off = r.data_off;
    for (int m = 0; m < 8; m++) {
      const int wm = m < mbc ? mb_width(r.widths, m) : 0;
      T.mbbit[threadIdx.x][m] = off;  // byte offset for now
      T.mbw[threadIdx.x][m] = uint8_t(wm);
      off += gbytes * wm;
    }
    T.md[threadIdx.x] = r.min_delta;
    if (threadIdx.x == 0) s_start = r.data_off;
    if (threadIdx.x == nb - 1) s_end = off;
  }
  __syncthreads();
  const int64_t start = s_start, end = s_end;
  // the blocks' data must lie inside the page image (records are offsets into it)
  if (start < 0 || end < start || end > int64_t(P.image_len)) return false;
  const int64_t a0 = start - int64_t((reinterpret_cast<uintptr_t>(img) + uintptr_t(start)) & 15);
  const int64_t nvec = (end - a0 + 15) >> 4;
  if (nvec * 16 > kTileStage) return false;
  if (threadIdx.x < nb)
    for (int m = 0; m < 8; m++) T.mbbit[threadIdx.x][m] = int32_t(T.mbbit[threadIdx.x][m] - a0) * 8;
  const int64_t e = P.image_len;
  stage_copy(reinterpret_cast<uint4*>(T.data), img + a0, nvec, e - a0);
  if (threadIdx.x < 4) T.data[nvec * 4 + threadIdx.x] = 0;
  __syncthreads();
  return true;
}

// delta(p) + minDelta of the staged tile (p relative to the page).
__device__ __forceinline__ uint64_t staged_delta(const TileStageLds& T, int64_t p, int bb0, int lbs, int lmb) {
  const int32_t q = int32_t(p);
  const int blk = (q >> lbs) - bb0;
  const int r = q & ((1 << lbs) - 1);
  const int m = r >> lmb;
  const int wm = T.mbw[blk][m];
  const uint32_t bit = uint32_t(T.mbbit[blk][m]) + uint32_t(r & ((1 << lmb) - 1)) * uint32_t(wm);
  return extract64(T.data, bit, wm) + T.md[blk];
}

// Delta tiles: the page-level prefix of the deltas is a three-step scan with kernel boundaries as
// the only synchronisation (a single-pass decoupled look-back would need agent-scope release /
// acquire per tile, i.e. L2 write-back / invalidate across the XCDs):
//   k_delta_sum    per tile: stage it, sum of (delta + minDelta) over its positions
//   k_delta_scan   per page stream: exclusive scan of its tile sums seeded with the first value
//   k_delta_expand per tile: stage it again, rows of 256 positions with block scans, coalesced stores
struct DeltaTileCtx {
  DevPage P;
  PageState S;
  DeltaState D;
  int64_t v0, v1;
  int64_t me;  // index of this (page, stream, tile) in dsums
  int stream;
  bool ok;
};

__device__ __forceinline__ DeltaTileCtx delta_tile_ctx(const DevBatch& b, const Tile& t) {
  DeltaTileCtx c;
  c.P = b.pages[t.page];
  c.S = b.states[t.page];
  c.stream = t.kind;  // DELTA_BYTE_ARRAY: 0 prefix lengths, 1 suffix lengths
  c.D = b.dstates[c.stream ? b.num_pages + t.page : t.page];
  c.v0 = int64_t(t.k) * kDeltaTile;
  c.v1 = c.v0 + kDeltaTile;
  if (c.v1 > c.D.limit) c.v1 = c.D.limit;
  const bool lens = c.P.kind == K_DLBA || c.P.kind == K_DBA;
  if (lens && c.v1 > c.S.nn) c.v1 = c.S.nn;
  c.me = int64_t(c.P.dtile_base) + int64_t(c.stream) * c.P.dtile_n + t.k;
  c.ok = !page_failed_before_values(c.S) && c.D.mode == DM_FAST && c.v0 < c.v1;
  return c;
}

// delta + minDelta of the 4 positions p..p+3 (p % 4 == 0: one miniblock, miniblocks hold >= 8).
template <class L>
__device__ __forceinline__ void staged_delta4(const L& T, int64_t p, int bb0, int lbs, int lmb, uint64_t d[4]) {
  const int32_t q = int32_t(p);
  const int blk = (q >> lbs) - bb0;
  const int r = q & ((1 << lbs) - 1);
  const int m = r >> lmb;
  const int wm = T.mbw[blk][m];
  const uint64_t md = T.md[blk];
  const uint32_t bit = uint32_t(T.mbbit[blk][m]) + uint32_t(r & ((1 << lmb) - 1)) * uint32_t(wm);
  if (wm <= 32) {
    extract32n<4>(T.data, bit, wm, md, d);
  } else {
#pragma unroll
    for (int j = 0; j < 4; j++) d[j] = extract64(T.data, bit + uint32_t(j * wm), wm) + md;
  }
}

__global__ __launch_bounds__(256) void k_delta_sum(DevBatch b, const Tile* tiles) {
  __shared__ TileStageLds T;
  __shared__ DeltaLds DL;
  const Tile t = tiles[blockIdx.x];
  const DeltaTileCtx c = delta_tile_ctx(b, t);
  if (!c.ok) return;
  const int lbs = __builtin_ctz(uint32_t(c.D.block_size)), lmb = __builtin_ctz(uint32_t(c.D.mbvc));
  uint64_t agg;
  if (stage_tile(b, c.P, c.D, c.v0, c.v1, T)) {
    const int bb0 = int(c.v0 >> lbs);
    uint64_t s = 0;
    for (int64_t p = c.v0 + 4 * int64_t(threadIdx.x); p < c.v1; p += 4 * kBlock) {
      uint64_t d[4];
      staged_delta4(T, p, bb0, lbs, lmb, d);
#pragma unroll
      for (int j = 0; j < 4; j++) s += p + j < c.v1 ? d[j] : 0;
    }
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if ((threadIdx.x & 63) == 0) T.wtot[0][threadIdx.x >> 6] = s;
    __syncthreads();
    agg = T.wtot[0][0] + T.wtot[0][1] + T.wtot[0][2] + T.wtot[0][3];
  } else {
    agg = c.P.kind == K_DELTA64
              ? delta_tile<true>(b, c.P, c.D, c.v0, c.v1, 0, false, nullptr, reinterpret_cast<uint32_t*>(T.data), DL)
              : delta_tile<false>(b, c.P, c.D, c.v0, c.v1, 0, false, nullptr, reinterpret_cast<uint32_t*>(T.data), DL);
  }
  if (threadIdx.x == 0) b.dsums[c.me] = agg;
}

// One thread per delta page: both streams of a DELTA_BYTE_ARRAY page.
__global__ __launch_bounds__(256) void k_delta_scan(DevBatch b, const int32_t* delta_pages, int32_t n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int p = delta_pages[i];
  const DevPage P = b.pages[p];
  const int streams = P.kind == K_DBA ? 2 : 1;
  for (int st = 0; st < streams; st++) {
    const DeltaState D = b.dstates[st ? b.num_pages + p : p];
    if (D.mode != DM_FAST) continue;
    uint64_t run = D.first;
    const int64_t base = int64_t(P.dtile_base) + int64_t(st) * P.dtile_n;
    const int64_t nt = (int64_t(D.limit) + kDeltaTile - 1) / kDeltaTile;  // tiles with positions
    for (int64_t k = 0; k < nt && k < P.dtile_n; k++) {
      const uint64_t s = b.dsums[base + k];
      b.dsums[base + k] = run;
      run += s;
    }
  }
}

// DPP move of both halves of a 64-bit value (lanes without a source read 0).
template <int CTRL, int ROWS>
__device__ __forceinline__ uint64_t dpp64(uint64_t x) {
  const int lo = __builtin_amdgcn_update_dpp(0, int(uint32_t(x)), CTRL, ROWS, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, int(uint32_t(x >> 32)), CTRL, ROWS, 0xf, false);
  return uint64_t(uint32_t(lo)) | (uint64_t(uint32_t(hi)) << 32);
}

// Inclusive wave64 scan (wrapping uint64): row_shr 1/2/4/8 inside each row of 16 lanes, then
// row_bcast:15 / row_bcast:31 carry the row totals across (GFX9 DPP, no LDS round trips).
__device__ __forceinline__ uint64_t wave_incl_scan(uint64_t x) {
  x += dpp64<0x111, 0xf>(x);
  x += dpp64<0x112, 0xf>(x);
  x += dpp64<0x114, 0xf>(x);
  x += dpp64<0x118, 0xf>(x);
  x += dpp64<0x142, 0xa>(x);
  x += dpp64<0x143, 0xc>(x);
  return x;
}

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2)));

// Inclusive wave64 scan of 32-bit values (wrapping), same DPP pattern as wave_incl_scan.
__device__ __forceinline__ uint32_t wave_incl_scan32(uint32_t x) {
  x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x111, 0xf, 0xf, false));
  x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x112, 0xf, 0xf, false));
  x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x114, 0xf, 0xf, false));
  x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x118, 0xf, 0xf, false));
  x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x142, 0xa, 0xf, false));
  x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x143, 0xc, 0xf, false));
  return x;
}

// Packed deltas (without minDelta) of the N positions q.. of one miniblock whose width is <= 32;
// md = the block's minDelta, blk = its tile-relative block.
template <int N, class L>
__device__ __forceinline__ void staged_u32(const L& T, int32_t q, int bb0, int lbs, int lmb, uint32_t* u, uint64_t& md,
                                           int& blk) {
  blk = (q >> lbs) - bb0;
  const int r = q & ((1 << lbs) - 1);
  const int m = r >> lmb;
  const int wm = T.mbw[blk][m];
  md = T.md[blk];
  const uint32_t bit = uint32_t(T.mbbit[blk][m]) + uint32_t(r & ((1 << lmb) - 1)) * uint32_t(wm);
  const uint32_t mask = wm >= 32 ? ~0u : (1u << wm) - 1;
#pragma unroll
  for (int j = 0; j < N; j++) {
    const uint32_t bj = bit + uint32_t(j * wm), k = bj >> 5;
    u[j] = __builtin_amdgcn_alignbit(T.data[k + 1], T.data[k], bj & 31) & mask;
  }
}

// Widths up to this keep a row's (1024 values) sum of packed deltas inside 32 bits.
constexpr int kNarrowWidth = 22;

// delta + minDelta of the 2 positions p, p+1 (p even: one miniblock).
template <class L>
__device__ __forceinline__ void staged_delta2(const L& T, int64_t p, int bb0, int lbs, int lmb, uint64_t d[2]) {
  const int32_t q = int32_t(p);
  const int blk = (q >> lbs) - bb0;
  const int r = q & ((1 << lbs) - 1);
  const int m = r >> lmb;
  const int wm = T.mbw[blk][m];
  const uint64_t md = T.md[blk];
  const uint32_t bit = uint32_t(T.mbbit[blk][m]) + uint32_t(r & ((1 << lmb) - 1)) * uint32_t(wm);
  if (wm <= 32) {
    extract32n<2>(T.data, bit, wm, md, d);
  } else {
    d[0] = extract64(T.data, bit, wm) + md;
    d[1] = extract64(T.data, bit + uint32_t(wm), wm) + md;
  }
}

// DELTA_LENGTH_BYTE_ARRAY lengths: the byte sum of every kBaTile tile of the page accumulated while
// the lengths are in registers (what k_ba_sum would re-read), and the first negative length
// (make([]byte, negative) panics, file_reader.go:179-181).  Positions >= lim are not counted.
struct LenSums {
  int64_t* tsum;  // basums + the page's batile_base (atomic adds; zeroed before the first producer)
  int64_t lim;
  int64_t neg;    // first negative length seen (INT64_MAX: none)
};

// One wave's partial sums of tile `tile` into tsum (one atomic per wave and tile).
__device__ __forceinline__ void flush_tile_sum(int64_t* tsum, int64_t tile, uint64_t acc) {
  const uint64_t tot = wave_incl_scan(acc);
  if ((threadIdx.x & 63) == 63 && tot) atomicAdd(reinterpret_cast<unsigned long long*>(tsum + tile), tot);
}

// Running kBaTile sums of one wave (call with the whole wave): lane x at position pos, the wave's
// positions [wfirst, wlast] (wave-uniform, ascending from call to call by less than a tile).  A lane
// keeps the sum of the wave's current tile `tacc` in `acc`; the wave flushes it when it moves on.
struct WaveTileSum {
  int64_t tacc;
  uint64_t acc;
};
__device__ __forceinline__ void wave_tile_add(WaveTileSum& w, int64_t* tsum, int64_t wfirst, int64_t wlast, int64_t pos,
                                              uint64_t x) {
  const int64_t t0 = wfirst / kBaTile;
  if (t0 != w.tacc) {
    flush_tile_sum(tsum, w.tacc, w.acc);
    w.acc = 0;
    w.tacc = t0;
  }
  if (wlast / kBaTile != t0) {  // the wave's positions cross into tile t0 + 1
    const bool lo = pos < (t0 + 1) * kBaTile;
    flush_tile_sum(tsum, t0, w.acc + (lo ? x : 0));
    w.acc = lo ? 0 : x;
    w.tacc = t0 + 1;
  } else {
    w.acc += x;
  }
}

// Rows of 1024 positions of a staged tile, one block scan each (wave totals double-buffered by row
// parity).  Every store instruction writes 16 contiguous bytes per lane, 1 KiB per wave: int32
// values 4 consecutive per thread; int64 values 2 consecutive per thread in each half row (two
// independent scans).  Returns the carry after the tile.  kSum (int32 DELTA_LENGTH lengths): each
// lane also sums its lengths of the wave's current kBaTile tile in a register, flushed (one wave
// reduction + one atomic) when the wave moves on to the next tile.
template <bool kSum = false, int kRows32 = 1, class L>
__device__ __forceinline__ uint64_t expand_rows(L& T, int64_t v0, int64_t v1, int lbs, int lmb, uint8_t* out,
                                                bool is64, uint64_t carry, LenSums* ls = nullptr) {
  const int bb0 = int(v0 >> lbs);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  int row = 0;
  if (is64) {
    // Narrow tiles (every width <= kNarrowWidth, the common case): the packed deltas are scanned in
    // 32 bits and the minDelta part is added per value from the blocks' running minDelta sums
    // (mdb), which cuts the 64-bit DPP scans and adds.  Wrapping 64-bit arithmetic gives the same
    // sums in any grouping, so both paths produce identical values.
    const int nblk = int(((v1 - 1) >> lbs) - bb0) + 1;
    if (threadIdx.x < 64) {
      bool wide = (v0 & ((int64_t(1) << lbs) - 1)) != 0;
      uint64_t m = 0;
      if (lane < nblk) {
#pragma unroll
        for (int k = 0; k < 8; k++) wide |= T.mbw[lane][k] > kNarrowWidth;
        m = T.md[lane] << lbs;
      }
      const uint64_t incl = wave_incl_scan(m);
      if (lane < nblk) T.mdb[lane] = incl - m;
      const uint64_t wm = __ballot(wide);
      if (lane == 0) T.narrow = wm == 0;
    }
    __syncthreads();
    uint64_t* o64 = reinterpret_cast<uint64_t*>(out);
    if (T.narrow) {
      uint64_t cu = carry;  // carry + packed deltas of the rows so far
      for (int64_t r0 = v0; r0 < v1; r0 += 4 * kBlock, row ^= 1) {
        const int64_t pa = r0 + 2 * int64_t(threadIdx.x), pb = pa + 2 * kBlock;
        uint32_t a[2] = {0, 0}, c[2] = {0, 0};
        uint64_t mda = 0, mdc = 0;
        int ba = 0, bc = 0;
        if (pa < v1) staged_u32<2>(T, int32_t(pa), bb0, lbs, lmb, a, mda, ba);
        if (pb < v1) staged_u32<2>(T, int32_t(pb), bb0, lbs, lmb, c, mdc, bc);
        a[1] = pa + 1 < v1 ? a[1] : 0;
        c[1] = pb + 1 < v1 ? c[1] : 0;
        const uint32_t sa = a[0] + a[1], sb = c[0] + c[1];
        const uint32_t ia = wave_incl_scan32(sa), ib = wave_incl_scan32(sb);
        if (lane == 63) {
          T.wtot[row][wv] = ia;
          T.wtot2[row][wv] = ib;
        }
        __syncthreads();
        const uint32_t ta = uint32_t(T.wtot[row][0] + T.wtot[row][1] + T.wtot[row][2] + T.wtot[row][3]);
        uint32_t ua = ia - sa, ub = ta + ib - sb;
        for (int k = 0; k < wv; k++) {
          ua += uint32_t(T.wtot[row][k]);
          ub += uint32_t(T.wtot2[row][k]);
        }
        if (pa < v1) {
          const uint64_t va = cu + ua + T.mdb[ba] + uint64_t(uint32_t(pa) & ((1u << lbs) - 1)) * mda;
          if (pa + 2 <= v1) __builtin_nontemporal_store(u64x2{va, va + a[0] + mda}, reinterpret_cast<u64x2*>(o64 + pa));
          else o64[pa] = va;
        }
        if (pb < v1) {
          const uint64_t vb = cu + ub + T.mdb[bc] + uint64_t(uint32_t(pb) & ((1u << lbs) - 1)) * mdc;
          if (pb + 2 <= v1) __builtin_nontemporal_store(u64x2{vb, vb + c[0] + mdc}, reinterpret_cast<u64x2*>(o64 + pb));
          else o64[pb] = vb;
        }
        cu += uint64_t(ta) + uint32_t(T.wtot2[row][0] + T.wtot2[row][1] + T.wtot2[row][2] + T.wtot2[row][3]);
      }
      // the value at v1: packed deltas + minDelta of every position in [v0, v1)
      const int64_t t1 = v1 - v0;
      const int bl = int((t1 - 1) >> lbs);
      return cu + T.mdb[bl] + uint64_t(t1 - (int64_t(bl) << lbs)) * T.md[bl];
    }
    for (int64_t r0 = v0; r0 < v1; r0 += 4 * kBlock, row ^= 1) {
      const int64_t pa = r0 + 2 * int64_t(threadIdx.x), pb = pa + 2 * kBlock;
      uint64_t a[2] = {0, 0}, c[2] = {0, 0};
      if (pa < v1) staged_delta2(T, pa, bb0, lbs, lmb, a);
      if (pb < v1) staged_delta2(T, pb, bb0, lbs, lmb, c);
      a[1] = pa + 1 < v1 ? a[1] : 0;
      c[0] = pb < v1 ? c[0] : 0;
      c[1] = pb + 1 < v1 ? c[1] : 0;
      const uint64_t sa = a[0] + a[1], sb = c[0] + c[1];
      const uint64_t ia = wave_incl_scan(sa), ib = wave_incl_scan(sb);
      if (lane == 63) {
        T.wtot[row][wv] = ia;
        T.wtot2[row][wv] = ib;
      }
      __syncthreads();
      const uint64_t ta = T.wtot[row][0] + T.wtot[row][1] + T.wtot[row][2] + T.wtot[row][3];
      uint64_t va = carry + ia - sa, vb = carry + ta + ib - sb;
      for (int k = 0; k < wv; k++) {
        va += T.wtot[row][k];
        vb += T.wtot2[row][k];
      }
      if (pa + 2 <= v1) {
        __builtin_nontemporal_store(u64x2{va, va + a[0]}, reinterpret_cast<u64x2*>(o64 + pa));
      } else if (pa < v1) {
        o64[pa] = va;
      }
      if (pb + 2 <= v1) {
        __builtin_nontemporal_store(u64x2{vb, vb + c[0]}, reinterpret_cast<u64x2*>(o64 + pb));
      } else if (pb < v1) {
        o64[pb] = vb;
      }
      carry += ta + T.wtot2[row][0] + T.wtot2[row][1] + T.wtot2[row][2] + T.wtot2[row][3];
    }
    return carry;
  }
  // 32-bit values: every sum wraps modulo 2^32 (the int32 decoder's arithmetic), so the whole
  // expansion runs in 32 bits (widths of 32-bit streams are <= 32)
  uint32_t* o32 = reinterpret_cast<uint32_t*>(out);
  uint32_t c32 = uint32_t(carry);
  WaveTileSum wts{(v0 + 4 * 64 * wv) / kBaTile, 0};
  const int64_t lim_e = kSum ? (v1 < ls->lim ? v1 : ls->lim) : 0;
  if constexpr (kRows32 > 1) {
    // kRows32 rows per barrier: every row's LDS reads and wave scan are independent of the other
    // rows', so they overlap; one barrier publishes the wave totals of all of them (the lengths
    // kernel runs ~3 workgroups per CU, where each row's dependent LDS reads + scan + barrier set
    // the time, not HBM)
    for (int64_t g0 = v0; g0 < v1; g0 += kRows32 * 4 * kBlock, row ^= 1) {
      uint32_t d[kRows32][4], ts[kRows32], inc[kRows32];
#pragma unroll
      for (int rr = 0; rr < kRows32; rr++) {
        const int64_t p = g0 + rr * 4 * kBlock + 4 * int64_t(threadIdx.x);
        d[rr][0] = d[rr][1] = d[rr][2] = d[rr][3] = 0;
        if (p < v1) {
          uint64_t md;
          int bk;
          staged_u32<4>(T, int32_t(p), bb0, lbs, lmb, d[rr], md, bk);
#pragma unroll
          for (int j = 0; j < 4; j++) d[rr][j] = p + j < v1 ? d[rr][j] + uint32_t(md) : 0;
        }
        ts[rr] = d[rr][0] + d[rr][1] + d[rr][2] + d[rr][3];
      }
#pragma unroll
      for (int rr = 0; rr < kRows32; rr++) inc[rr] = wave_incl_scan32(ts[rr]);
      if (lane == 63) {
#pragma unroll
        for (int rr = 0; rr < kRows32; rr++) T.wt32[row][rr][wv] = inc[rr];
      }
      __syncthreads();
#pragma unroll
      for (int rr = 0; rr < kRows32; rr++) {
        const int64_t r0 = g0 + rr * 4 * kBlock;
        if (r0 >= v1) break;
        const int64_t p = r0 + 4 * int64_t(threadIdx.x);
        const uint32_t w0 = T.wt32[row][rr][0], w1 = T.wt32[row][rr][1], w2 = T.wt32[row][rr][2],
                       w3 = T.wt32[row][rr][3];
        const uint32_t v = c32 + inc[rr] - ts[rr] + (wv > 0 ? w0 : 0) + (wv > 1 ? w1 : 0) + (wv > 2 ? w2 : 0);
        const uint32_t o4[4] = {v, v + d[rr][0], v + d[rr][0] + d[rr][1], v + d[rr][0] + d[rr][1] + d[rr][2]};
        if (p + 4 <= v1) {
          __builtin_memcpy(o32 + p, o4, 16);
        } else {
#pragma unroll
          for (int j = 0; j < 4; j++)
            if (p + j < v1) o32[p + j] = o4[j];
        }
        if constexpr (kSum) {
          uint64_t rs;
          if (p + 4 <= lim_e && ((o4[0] | o4[1] | o4[2] | o4[3]) >> 31) == 0) {
            rs = uint64_t(o4[0] + o4[1]) + uint64_t(o4[2] + o4[3]);
          } else {
            rs = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) {
              if (p + j >= lim_e) break;
              if (int32_t(o4[j]) < 0) ls->neg = p + j < ls->neg ? p + j : ls->neg;
              else rs += o4[j];
            }
          }
          const int64_t wp = r0 + 4 * 64 * wv;
          wave_tile_add(wts, ls->tsum, wp, wp + 255, p, rs);
        }
        c32 += w0 + w1 + w2 + w3;
      }
    }
    if constexpr (kSum) flush_tile_sum(ls->tsum, wts.tacc, wts.acc);
    return c32;
  }
  for (int64_t r0 = v0; r0 < v1; r0 += 4 * kBlock, row ^= 1) {
    const int64_t p = r0 + 4 * int64_t(threadIdx.x);
    uint32_t d[4] = {0, 0, 0, 0};
    if (p < v1) {
      uint64_t md;
      int bk;
      staged_u32<4>(T, int32_t(p), bb0, lbs, lmb, d, md, bk);
#pragma unroll
      for (int j = 0; j < 4; j++) d[j] = p + j < v1 ? d[j] + uint32_t(md) : 0;
    }
    const uint32_t tsum = d[0] + d[1] + d[2] + d[3];
    const uint32_t incl = wave_incl_scan32(tsum);
    if (lane == 63) T.wtot[row][wv] = incl;
    __syncthreads();
    uint32_t v = c32 + incl - tsum;
    for (int k = 0; k < wv; k++) v += uint32_t(T.wtot[row][k]);
    const uint32_t o4[4] = {v, v + d[0], v + d[0] + d[1], v + d[0] + d[1] + d[2]};
    if (p + 4 <= v1) {
      __builtin_memcpy(o32 + p, o4, 16);
    } else {
#pragma unroll
      for (int j = 0; j < 4; j++)
        if (p + j < v1) o32[p + j] = o4[j];
    }
    if constexpr (kSum) {
      // the lane's 4 lengths: non-negative int32 pairs add without overflow in 32 bits
      uint64_t rs;
      if (p + 4 <= lim_e && ((o4[0] | o4[1] | o4[2] | o4[3]) >> 31) == 0) {
        rs = uint64_t(o4[0] + o4[1]) + uint64_t(o4[2] + o4[3]);
      } else {
        rs = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
          if (p + j >= lim_e) break;
          if (int32_t(o4[j]) < 0) ls->neg = p + j < ls->neg ? p + j : ls->neg;
          else rs += o4[j];
        }
      }
      const int64_t w0 = r0 + 4 * 64 * wv;  // the wave's 256 positions of this row
      wave_tile_add(wts, ls->tsum, w0, w0 + 255, p, rs);
    }
    c32 += uint32_t(T.wtot[row][0] + T.wtot[row][1] + T.wtot[row][2] + T.wtot[row][3]);
  }
  if constexpr (kSum) flush_tile_sum(ls->tsum, wts.tacc, wts.acc);
  return c32;
}




__device__ __forceinline__ uint8_t* delta_out(const DevBatch& b, const DeltaTileCtx& c) {
  const DevChunk C = b.chunks[c.P.chunk];
  const bool lens = c.P.kind == K_DLBA || c.P.kind == K_DBA;  // int32 lengths into aux / aux2
  int32_t* lp = c.P.kind == K_DBA && c.stream == 0 ? C.aux2 : C.aux;
  return lens ? reinterpret_cast<uint8_t*>(lp + c.S.value_base) : C.values + c.S.value_base * c.P.value_size;
}

__global__ __launch_bounds__(256) void k_delta_expand(DevBatch b, const Tile* tiles) {
  __shared__ TileStageLds T;
  __shared__ DeltaLds DL;
  const Tile t = tiles[blockIdx.x];
  const DeltaTileCtx c = delta_tile_ctx(b, t);
  if (!c.ok) return;
  const bool is64 = c.P.kind == K_DELTA64;
  uint8_t* out = delta_out(b, c);
  const uint64_t base = b.dsums[c.me];
  if (!stage_tile(b, c.P, c.D, c.v0, c.v1, T)) {
    if (is64) delta_tile<true>(b, c.P, c.D, c.v0, c.v1, base, true, out, reinterpret_cast<uint32_t*>(T.data), DL);
    else delta_tile<false>(b, c.P, c.D, c.v0, c.v1, base, true, out, reinterpret_cast<uint32_t*>(T.data), DL);
    return;
  }
  expand_rows(T, c.v0, c.v1, __builtin_ctz(uint32_t(c.D.block_size)), __builtin_ctz(uint32_t(c.D.mbvc)), out, is64,
              base);
}

// k_delta_page: one workgroup per (page, stream) decodes the stream's blocks in order with a running
// carry seeded by the first value: no tile sums, no page scan, the packed deltas are read once.
// Used when a batch has enough delta streams to fill the GPU with one workgroup each.  Tiles are cut
// by bytes: as many blocks (<= 64) as fit a 16 KiB stage, so that several workgroups share a CU.
constexpr int kPageStage = 16384 + 64;  // >= one block of 2048 64-bit deltas + alignment lead

template <int kStage>
struct PageTileLdsT {
  static constexpr int kStageBytes = kStage;
  uint32_t data[kStage / 4 + 4];
  int32_t mbbit[kTileBlocks][8];  // first bit of each miniblock's data in `data`
  uint8_t mbw[kTileBlocks][8];
  uint64_t md[kTileBlocks];
  union {
    struct {
      uint64_t wtot[2][4];
      uint64_t wtot2[2][4];
    };
    uint32_t wt32[2][4][4];  // 32-bit rows, kRows32 per barrier: [parity][row][wave]
  };
  uint64_t mdb[kTileBlocks];
  int64_t a0;
  int32_t nfit;
  int32_t end;
  int32_t narrow;
  int32_t pad;
};
using PageTileLds = PageTileLdsT<kPageStage>;

// k_delta_fused's stage: 14.5 KiB, so that its LDS (20448 B) and registers (64 VGPRs, 8 waves per
// SIMD) let 8 workgroups share a CU (2048 streams in flight instead of 1536: C3 32 row groups
// k_delta_fused 0.504 -> 0.461 ms, 128 row groups 1.649 -> 1.605 ms, same box,
// profiles/r05_exp/c3_probe_*.log).  A block whose bytes do not fit the stage (2048 values wider than
// ~57 bits) ends the fused head; k_delta_walk / k_delta_page (16 KiB stage) take the rest.
constexpr int kFusedStage = 14848;
// DELTA_LENGTH lengths (k_delta_fused_lens, k_delta_page): 1024-value rows expanded per barrier
#ifndef PQH_LENS_ROWS
#define PQH_LENS_ROWS 4
#endif
#define PQH_FUSED_ATTR __attribute__((amdgpu_waves_per_eu(8)))

__global__ __launch_bounds__(256) void k_delta_page(DevBatch b, const Tile* streams) {
  __shared__ PageTileLds T;
  const DeltaTileCtx c = delta_tile_ctx(b, streams[blockIdx.x]);
  if (!c.ok) return;
  const bool is64 = c.P.kind == K_DELTA64;
  uint8_t* out = delta_out(b, c);
  int64_t vlim = c.D.limit;
  if ((c.P.kind == K_DLBA || c.P.kind == K_DBA) && vlim > c.S.nn) vlim = c.S.nn;
  const int lbs = __builtin_ctz(uint32_t(c.D.block_size)), lmb = __builtin_ctz(uint32_t(c.D.mbvc));
  const int mbc = c.D.mb_count, gbytes = c.D.mbvc / 8;
  const uint8_t* img = b.payload + c.P.image_off;
  const DeltaBlock* recs = b.dblocks + c.P.dblk_base + c.D.rec_base;
  const int64_t nblk = (vlim + c.D.block_size - 1) >> lbs;
  const int64_t e = c.P.image_len;
  const int tid = threadIdx.x;
  // DELTA_LENGTH: the tile byte sums of the page (k_delta_fused added the head's when the walk
  // accepted it; otherwise they start again from zero) and the first negative length
  __shared__ unsigned long long s_neg;
  const bool sums = c.P.kind == K_DLBA;
  LenSums ls{b.basums + c.P.batile_base, vlim < c.S.val_limit ? vlim : c.S.val_limit, INT64_MAX};
  if (sums) {
    if (c.D.head_blocks == 0)
      for (int k = tid; k < c.P.batile_n; k += kBlock) ls.tsum[k] = 0;
    if (tid == 0) s_neg = uint64_t(c.D.head_neg);
    __syncthreads();
  }
  // blocks [0, head_blocks) were decoded by k_delta_fused
  uint64_t carry = c.D.head_blocks ? c.D.head_carry : c.D.first;
  for (int64_t blk0 = c.D.head_blocks; blk0 < nblk;) {
    __syncthreads();  // the previous tile's readers of T are done
    // block table of the next <= 64 blocks; the blocks whose bytes fit the stage form the tile
    if (tid < 64) {
      const bool have = blk0 + tid < nblk;
      int32_t start = 0, end = 0;
      if (have) {
        const DeltaBlock r = load_block(recs, blk0 + tid, img, is64, mbc);
        int32_t off = r.data_off;
        start = off;
        for (int m = 0; m < 8; m++) {
          const int wm = m < mbc ? mb_width(r.widths, m) : 0;
          T.mbbit[tid][m] = off;  // byte offset for now
          T.mbw[tid][m] = uint8_t(wm);
          off += gbytes * wm;
        }
        T.md[tid] = r.min_delta;
        end = off;
      }
      const int32_t s0 = __builtin_amdgcn_readfirstlane(start);
      const int64_t a0 = s0 - int64_t((reinterpret_cast<uintptr_t>(img) + uintptr_t(s0)) & 15);
      const uint64_t fit = __ballot(have && int64_t(end) - a0 <= kPageStage - 16);
      const int nfit = fit == ~0ull ? 64 : __builtin_ctzll(~fit);  // >= 1: a block never exceeds the stage
      const int32_t end_last = __builtin_amdgcn_readlane(end, nfit - 1);
      if (tid == 0) {
        T.nfit = nfit;
        T.a0 = a0;
        T.end = end_last;
      }
    }
    __syncthreads();
    const int nfit = T.nfit;
    const int64_t a0 = T.a0, end = T.end;  // the tile's bytes run to the end of its last block's data
    if (tid < nfit)
      for (int m = 0; m < 8; m++) T.mbbit[tid][m] = int32_t(T.mbbit[tid][m] - a0) * 8;
    const int64_t nvec = (end - a0 + 15) >> 4;
    stage_copy(reinterpret_cast<uint4*>(T.data), img + a0, nvec, e - a0);
    if (tid < 4) T.data[nvec * 4 + tid] = 0;
    __syncthreads();
    const int64_t v0 = blk0 << lbs;
    int64_t v1 = (blk0 + nfit) << lbs;
    if (v1 > vlim) v1 = vlim;
    if (sums) carry = expand_rows<true, PQH_LENS_ROWS>(T, v0, v1, lbs, lmb, out, false, carry, &ls);
    else carry = expand_rows(T, v0, v1, lbs, lmb, out, is64, carry);
    blk0 += nfit;
  }
  if (sums) {
    if (ls.neg != INT64_MAX) atomicMin(&s_neg, (unsigned long long)ls.neg);
    __syncthreads();
    if (tid == 0) {
      if (s_neg != (~0ull >> 1))  // make([]byte, negative) panics (re-panicked, file_reader.go:179-181)
        atomicMin(&b.states[streams[blockIdx.x].page].err,
                  (unsigned long long)err_key(3, int64_t(s_neg), PQH_ERR_NEGATIVE_DLBA_LENGTH));
      b.states[streams[blockIdx.x].page].ba_summed = 1;
    }
  }
}

// TK_DELTA_SERIAL: exact sequential restatement of deltaBitPackDecoder.init + next for streams
// outside the fast-path geometry.  One thread; the rest of the workgroup idles (rare layouts only).
// init_all (DELTA_LENGTH / DELTA_BYTE_ARRAY lengths): all valuesCount values are decoded at load and
// every error is a load error; the first `nvals` values are kept.  Returns the first error key.
__device__ uint64_t serial_stream(const uint8_t* img, int64_t& pos, int64_t e, bool is64, uint8_t* out,
                                  int64_t nvals, bool init_all, int32_t& vc_out) {
  auto uvar = [&](uint64_t& v) { return read_uvarint(img, pos, e, v); };
  auto uvar32 = [&](int32_t& o) {
    uint64_t v;
    int st = uvar(v);
    if (st) return st;
    if (v > 0x7fffffffull) return int(PQH_ERR_INT32_RANGE);
    o = int32_t(v);
    return int(PQH_OK);
  };
  auto var = [&](uint64_t& o) {
    uint64_t u;
    int st = uvar(u);
    if (st) return st;
    const int64_t x = int64_t(u >> 1) ^ -int64_t(u & 1);
    if (!is64 && (x > 2147483647ll || x < -2147483648ll)) return int(PQH_ERR_INT32_RANGE);
    o = uint64_t(x);
    return int(PQH_OK);
  };
  auto read_full_skip = [&](int64_t nbytes) {  // io.ReadFull, errors ignored
    if (nbytes <= 0) return;
    pos = pos + nbytes < e ? pos + nbytes : (pos > e ? pos : e);
  };
  int32_t bs = 0, mbc = 0, vc = 0, mbvc = 0;
  uint64_t prev = 0, md = 0;
  int64_t widths_pos = 0;  // widths live in the image at widths_pos (mbc bytes)
  int st;
  vc_out = 0;
  // ---- init: readBlockHeader + readMiniBlockHeader (deltabp_decoder.go:37-111) ----
  if ((st = uvar32(bs)) || (st = uvar32(mbc))) return err_key(0, 3, st);
  if (mbc <= 0 || bs % mbc != 0) return err_key(0, 3, PQH_ERR_DELTA_MINIBLOCKS);
  mbvc = bs / mbc;
  if (mbvc == 0) return err_key(0, 3, PQH_ERR_DELTA_MINIBLOCKS);
  if ((st = uvar32(vc))) return err_key(0, 3, st);
  if ((st = var(prev))) return err_key(0, 3, st);
  auto mini_header = [&]() -> int {
    int s2 = var(md);
    if (s2) return s2;
    const int64_t avail = e - pos;
    if (avail <= 0) return PQH_ERR_EOF;
    if (avail < mbc) {
      pos = e;
      return PQH_ERR_UNEXPECTED_EOF;
    }
    widths_pos = pos;
    for (int32_t i = 0; i < mbc; i++)
      if (img[pos + i] > (is64 ? 64 : 32)) return PQH_ERR_DELTA_BIT_WIDTH;
    pos += mbc;
    return PQH_OK;
  };
  if ((st = mini_header())) return err_key(0, 3, st);
  vc_out = vc;
  // ---- next() x nn (deltabp_decoder.go:113-170) ----
  const int64_t nn = init_all ? vc : nvals;
  auto verr = [&](int64_t position, int code) { return init_all ? err_key(0, 3, code) : err_key(3, position, code); };
  int32_t cur_mb = 0, cur_w = 0, mb_pos = 0;
  int64_t gpos = 0;  // byte offset of the current group of 8 deltas
  for (int64_t position = 0; position < nn; position++) {
    if (position >= vc) return err_key(3, position, PQH_ERR_EOF);
    if (position % 8 == 0) {
      if (position % mbvc == 0) {
        if (cur_mb >= mbc) {
          if ((st = mini_header())) return verr(position, st);
          cur_mb = 0;
        }
        cur_w = img[widths_pos + cur_mb];
        mb_pos = 0;
        cur_mb++;
      }
      const int32_t w = cur_w;
      if (w > 0) {
        const int64_t avail = e - pos;
        if (avail < w) return verr(position, avail <= 0 ? PQH_ERR_EOF : PQH_ERR_UNEXPECTED_EOF);
      }
      gpos = pos;
      pos += w;
      mb_pos += w;
      if (position + 8 >= vc) {
        const int64_t l = int64_t(mbvc / 8) * w - mb_pos;
        if (l < 0) return verr(position, PQH_ERR_DELTA_STREAM);
        read_full_skip(l);
        for (int32_t i = cur_mb; i < mbc; i++) {
          const int32_t w2 = img[widths_pos + cur_mb];
          if (w2 != 0) read_full_skip(int64_t(mbvc / 8) * w2);
        }
      }
    }
    if (position < nvals) {
      if (is64) reinterpret_cast<uint64_t*>(out)[position] = prev;
      else reinterpret_cast<uint32_t*>(out)[position] = uint32_t(prev);
    }
    uint64_t delta = 0;  // unpack8 (LSB first) of this position's w bits
    for (int k2 = 0; k2 < cur_w; k2++) {
      const int64_t bit = int64_t(position % 8) * cur_w + k2;
      delta |= uint64_t((img[gpos + (bit >> 3)] >> (bit & 7)) & 1) << k2;
    }
    prev += delta + md;
  }
  return kNoError;
}

// k_delta_serial: one wave per delta page; pages the walk marked DM_SERIAL are decoded by lane 0:
// plain delta values, DELTA_LENGTH lengths, or both DELTA_BYTE_ARRAY length streams (then the
// count check of type_bytearray.go:206-208).
__global__ __launch_bounds__(64) void k_delta_serial(DevBatch b, const int32_t* delta_pages) {
  const Tile t{delta_pages[blockIdx.x], 0, TK_DELTA_SERIAL, 1};
  const DevPage P = b.pages[t.page];
  const PageState S = b.states[t.page];
  const DeltaState D0 = b.dstates[t.page];
  if (D0.mode != DM_SERIAL || threadIdx.x != 0) return;
  const uint8_t* img = b.payload + P.image_off;
  const bool before_values = S.err != kNoError && (S.err >> 56) <= 2;
  const int64_t nvals = before_values ? 0 : S.nn;
  const DevChunk C = b.chunks[P.chunk];
  int64_t pos = S.val_s;
  int32_t vc = 0;
  uint64_t err;
  if (P.kind == K_DLBA) {
    err = serial_stream(img, pos, S.val_e, false, reinterpret_cast<uint8_t*>(C.aux + S.value_base), nvals, true, vc);
    b.dstates[t.page].end_pos = pos;
    b.dstates[t.page].limit = err == kNoError ? vc : 0;
  } else if (P.kind == K_DBA) {
    err = serial_stream(img, pos, S.val_e, false, reinterpret_cast<uint8_t*>(C.aux2 + S.value_base), nvals, true, vc);
    int32_t vc1 = 0;
    if (err == kNoError) {
      err = serial_stream(img, pos, S.val_e, false, reinterpret_cast<uint8_t*>(C.aux + S.value_base), nvals, true, vc1);
      if (err == kNoError && vc != vc1) err = err_key(0, 3, PQH_ERR_DBA_COUNT);
    }
    b.dstates[t.page].limit = err == kNoError ? vc : 0;
    b.dstates[b.num_pages + t.page].end_pos = pos;
    b.dstates[b.num_pages + t.page].limit = err == kNoError ? vc1 : 0;
  } else {
    err = serial_stream(img, pos, S.val_e, P.kind == K_DELTA64, C.values + S.value_base * P.value_size, nvals, false, vc);
  }
  if (err != kNoError) atomicMin(&b.states[t.page].err, (unsigned long long)err);
}

// ------------------------------------------------------------------------------------------------
// Lane-parallel chase of the block headers inside a staged window (k_delta_fused): the speculative
// segment walk of spec_chain, with LDS instead of L2 as the byte source and at most 64 blocks (one
// tile) per call.  Lane i takes the byte segment [loc0 + i*S, loc0 + (i+1)*S) with S the mean block
// span (so about one header per lane), synchronises on its first plausible header, walks to the
// segment's exit header and parses that one's successor; lanes are linked to their left neighbour
// when its exit header (or the exit's successor) is in their list.  A block is usable when its data
// ends inside the window (dlim) and the stream (eloc).
// ------------------------------------------------------------------------------------------------
constexpr int kChaseCap = 8;  // chain entries per lane

// Per lane: the header at local offset loc of the staged window.  Returns its data end (-1 if the
// common-case parse fails), *dat / *md / *wd.
__device__ __forceinline__ int32_t lds_hdr(const uint32_t* data, int32_t loc, bool is64, int mbc, int gbytes,
                                           int32_t& dat, uint64_t& md, uint64_t& wd) {
  const uint64_t* w64 = reinterpret_cast<const uint64_t*>(data);
  const int32_t q = loc >> 3;
  const uint64_t x0 = w64[q], x1 = w64[q + 1], x2 = w64[q + 2];
  const uint32_t sh = uint32_t(loc & 7) * 8;
  const uint64_t lo = sh ? (x0 >> sh) | (x1 << (64 - sh)) : x0;
  const uint64_t hi = sh ? (x1 >> sh) | (x2 << (64 - sh)) : x1;
  const int hl = parse_hdr16(lo, hi, is64, mbc, md, wd);
  if (!hl) return -1;
  dat = loc + hl;
  return dat + int32_t(widths_sum(wd)) * gbytes;
}

// Usable header at loc: parses, its block ends inside the window and the stream.
__device__ __forceinline__ bool lds_block(const uint32_t* data, int32_t loc, int32_t eloc, int32_t plim,
                                          int32_t dlim, bool is64, int mbc, int gbytes, int32_t& dend) {
  if (loc >= plim || loc + 24 > eloc) return false;
  int32_t dat;
  uint64_t md, wd;
  dend = lds_hdr(data, loc, is64, mbc, gbytes, dat, md, wd);
  return dend >= 0 && dend <= dlim && dend <= eloc;
}

__device__ void lds_chase(const uint32_t* data, int32_t loc0, int32_t eloc, int32_t est, int nmax, bool is64, int mbc,
                          int gbytes, int16_t (*lst)[64], int32_t* blkbit, uint64_t* blkw, uint64_t* mdt, int lane,
                          int& n_out, int32_t& next_out, bool& stop_out, int32_t stage = kPageStage) {
  const int32_t plim = stage - 32, dlim = stage - 16;
  const uint64_t lim = is64 ? 64 : 32;
  if (est <= 0) {  // first tile: the span of block 0
    int32_t d0 = -1;
    est = lds_block(data, loc0, eloc, plim, dlim, is64, mbc, gbytes, d0) ? d0 - loc0 : 64;
  }
  {
    // uniform spans (reference-writer streams of steady data): lane i parses the header predicted
    // at loc0 + i*est; lanes 0..m-1 whose block is usable and ends exactly at the next prediction
    // are the chain (by induction from lane 0, which sits on the true header loc0).  Taken when it
    // covers nmax blocks or stops only because the next block runs past the window; anything else
    // goes through the segment chase below.
    const int32_t g = loc0 + est * lane;
    int32_t dat = 0, dend = -1;
    uint64_t md = 0, wd = 0;
    const bool parsed = g < plim && g + 24 <= eloc && (dend = lds_hdr(data, g, is64, mbc, gbytes, dat, md, wd)) >= 0;
    const bool usable = parsed && dend <= dlim && dend <= eloc;
    const uint64_t cm = __ballot(usable && dend == g + est);
    const int m = cm == ~0ull ? 64 : __builtin_ctzll(~cm);
    bool take = m >= nmax;
    if (!take && m > 0) {  // lane m: the true next header; accept if its block only overflows the window
      const int ok = __builtin_amdgcn_readlane(int(parsed && dend > dlim && dend <= eloc), m);
      take = ok != 0;
    }
    if (take && est > 0) {
      const int n = m < nmax ? m : nmax;
      if (lane < n) {
        blkbit[lane] = dat * 8;
        blkw[lane] = wd;
        mdt[lane] = md;
      }
      n_out = n;
      next_out = loc0 + est * n;
      stop_out = false;
      return;
    }
  }
  const int32_t S = est < 16 ? 16 : est;
  const int32_t s0 = loc0 + S * lane, s1 = s0 + S;
  int cnt = 0;
  bool dead = false, bad = false;  // bad: the chain reached a header the exact walk must handle
  int32_t p = s0, x2 = -1;
  if (s0 < plim) {
    if (lane > 0) {  // synchronise: first plausible header in [s0, s1)
      p = s1;
      for (int32_t base = s0 & ~7; base < s1 && base < plim && p == s1; base += 32) {
        const uint64_t* w64 = reinterpret_cast<const uint64_t*>(data) + (base >> 3);
        uint64_t x0 = w64[0], S0 = small_bytes(x0, lim);
        for (int j = 0; j < 4 && p == s1; j++) {
          const uint64_t x1 = w64[j + 1], S1 = small_bytes(x1, lim);
          uint64_t c = ~x0 & 0x8080808080808080ull;
          for (int k = 1; k <= mbc; k++) c &= k == 8 ? S1 : (S0 >> (8 * k)) | (S1 << (64 - 8 * k));
          const int32_t w0 = base + 8 * j;
          if (s0 > w0) c &= s0 - w0 >= 8 ? 0 : ~0ull << (8 * (s0 - w0));
          if (s1 - w0 < 8) c &= s1 <= w0 ? 0 : (1ull << (8 * (s1 - w0))) - 1;
          while (c) {
            const int32_t q = w0 + (__builtin_ctzll(c) >> 3);
            c &= c - 1;
            int32_t d;
            if (lds_block(data, q, eloc, plim, dlim, is64, mbc, gbytes, d)) {
              p = q;
              break;
            }
          }
          x0 = x1;
          S0 = S1;
        }
      }
    }
    while (p < s1 && cnt < kChaseCap) {
      lst[cnt][lane] = int16_t(p);
      cnt++;
      int32_t d;
      if (!lds_block(data, p, eloc, plim, dlim, is64, mbc, gbytes, d)) {
        dead = true;
        // the true chain stops here for good unless the block merely runs past the window
        int32_t dat;
        uint64_t md, wd;
        const int32_t de = p < plim ? lds_hdr(data, p, is64, mbc, gbytes, dat, md, wd) : 0;
        bad = p + 24 > eloc || (p < plim && (de < 0 || de > eloc));
        break;
      }
      p = d;
    }
    if (!dead && p >= s1 && cnt < kChaseCap) {  // exit header (slot cnt, not counted) and its successor
      lst[cnt][lane] = int16_t(p);
      int32_t d;
      if (lds_block(data, p, eloc, plim, dlim, is64, mbc, gbytes, d)) x2 = d;
    }
  }
  const bool full = !dead && p < s1;
  // ---- stitch (as spec_chain): link to the left neighbour through its exit header or its successor
  const int32_t xl = __shfl_up(p, 1, 64), x2l = __shfl_up(x2, 1, 64);
  const bool exit_ok = s0 < plim && !dead && !full && cnt < kChaseCap;
  const bool left_ok = __shfl_up(int(exit_ok), 1, 64) != 0 && xl >= s0 && xl < s1;
  int jd = -1, j2 = -1;
  if (lane > 0 && left_ok) {
    for (int k = 0; k < cnt; k++) {
      const int32_t q = lst[k][lane];
      if (jd < 0 && q == xl) jd = k;
      if (j2 < 0 && x2l >= 0 && q == x2l) j2 = k;
    }
    // the left neighbour's exit is my segment's only true header: its successor is my exit
    if (jd < 0 && j2 < 0 && exit_ok && x2l == p) j2 = cnt;
  }
  const bool active = s0 < plim;
  const bool link = active && (lane == 0 || (left_ok && (jd >= 0 || j2 >= 0)));
  const int j = lane == 0 ? 0 : (jd >= 0 ? jd : j2);
  const bool extra = lane > 0 && link && jd < 0;  // the left neighbour records its exit header
  const uint64_t linkm = __ballot(link);
  const int k_bad = linkm == ~0ull ? 64 : __builtin_ctzll(~linkm);
  const uint64_t deadm = __ballot(dead) & (k_bad >= 64 ? ~0ull : (1ull << k_bad) - 1);
  const int last = deadm ? __builtin_ctzll(deadm) : k_bad - 1;  // >= 0: lane 0 always links
  const bool valid = lane <= last;
  const bool extra_r = __shfl_down(int(extra), 1, 64) != 0 && lane + 1 <= last && lane < 63;
  const int n_all = valid ? cnt - j - (dead ? 1 : 0) + (extra_r ? 1 : 0) : 0;
  int incl = n_all;
  for (int off = 1; off < 64; off <<= 1) {
    const int y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  const int base = incl - n_all;
  const int total = __builtin_amdgcn_readlane(incl, 63);
  const int my_n = base + n_all > nmax ? (nmax - base > 0 ? nmax - base : 0) : n_all;
  for (int k = 0; k < my_n; k++) {  // tables of the kept blocks
    const int32_t q = lst[j + k][lane];
    int32_t dat;
    uint64_t md, wd;
    lds_hdr(data, q, is64, mbc, gbytes, dat, md, wd);
    blkbit[base + k] = dat * 8;
    blkw[base + k] = wd;
    mdt[base + k] = md;
  }
  int32_t nxt;
  bool stop = false;
  if (total > nmax) {  // the header after the last kept block
    const bool hit = valid && base <= nmax && nmax < base + n_all;
    const uint64_t hm = __ballot(hit);
    const int32_t q = hit ? lst[j + (nmax - base)][lane] : 0;
    nxt = __builtin_amdgcn_readlane(q, __builtin_ctzll(hm));
  } else if (deadm) {
    nxt = __builtin_amdgcn_readlane(int32_t(lst[cnt > 0 ? cnt - 1 : 0][lane]), last);
    stop = __builtin_amdgcn_readlane(int(bad), last) != 0;
  } else {
    nxt = __builtin_amdgcn_readlane(p, last);
  }
  int n = total < nmax ? total : nmax;
  // A chain cut short by a lane that synchronised on a false header (low-entropy packed data reads
  // as plausible headers) ends on a true header: continue from it serially inside the same window
  // (one LDS header parse per block) instead of restaging the window for the next few blocks.
  while (!stop && n < nmax) {  // (one header parse per block: lds_block's test on the same parse)
    int32_t dat = 0, dend = -1;
    uint64_t md = 0, wd = 0;
    const bool in_reach = nxt < plim && nxt + 24 <= eloc;
    if (in_reach) dend = lds_hdr(data, nxt, is64, mbc, gbytes, dat, md, wd);
    if (!in_reach || dend < 0 || dend > dlim || dend > eloc) {
      stop = nxt + 24 > eloc || (nxt < plim && (dend < 0 || dend > eloc));
      break;
    }
    if (lane == 0) {
      blkbit[n] = dat * 8;
      blkw[n] = wd;
      mdt[n] = md;
    }
    n++;
    nxt = dend;
  }
  n_out = n;
  next_out = nxt;
  stop_out = stop;
}

// k_delta_fused (page mode): one workgroup per DELTA_BINARY_PACKED / DELTA_LENGTH stream (and the
// prefix-length stream of DELTA_BYTE_ARRAY pages).  The stream is staged 16 KiB at a time from the
// next block header; wave 0 chases the block headers in LDS (wave-uniform, scalar), and the whole
// blocks [0, kmax) are decoded with a running carry: the packed deltas are read from HBM once and
// no block records are written.  The chase stops at the first header the common-case parse rejects
// or a block that runs past the stream; k_delta_walk resumes there with the exact semantics (and the
// records of the remaining blocks) and k_delta_page decodes the rest.
// kLens: the DELTA_LENGTH streams' launch (tile byte sums in the row loop); the other streams run
// the instantiation without them, which keeps its register budget (occupancy) unchanged.
#ifdef PQH_FUSED_PROF
// (-DPQH_FUSED_PROF experiments) per phase wall-clock ticks summed over workgroups:
// [0] init, [1] stage, [2] chase, [3] tables, [4] expand, [5] tiles, [6] workgroups, [7] whole body
__device__ unsigned long long g_fprof[2][8];
#define FPROF_T(v) const uint64_t v = wall_clock64()
#define FPROF_ADD(k, x) prof[k] += (x)
#else
#define FPROF_T(v)
#define FPROF_ADD(k, x)
#endif

template <bool kLens>
__device__ __forceinline__ void delta_fused_body(DevBatch b, const Tile* streams) {
#ifdef PQH_FUSED_PROF
  uint64_t prof[8] = {0, 0, 0, 0, 0, 0, 1, 0};
  const uint64_t t_begin = wall_clock64();
#endif
  __shared__ PageTileLdsT<kLens ? kPageStage : kFusedStage> T;
  __shared__ int32_t s_blkbit[kTileBlocks];
  __shared__ uint64_t s_blkw[kTileBlocks];
  __shared__ int64_t s_h;
  __shared__ uint64_t s_first;
  __shared__ int32_t s_geo[5];  // kmax (0 = nothing to do), block size, miniblocks, values per miniblock, vc
  __shared__ int32_t s_n, s_stop;
  __shared__ int16_t s_lst[kChaseCap][64];
  __shared__ unsigned long long s_neg;
  const Tile t = streams[blockIdx.x];
  if (t.kind != 0) return;  // DELTA_BYTE_ARRAY suffix lengths: k_delta_walk + k_delta_page
  const int p = t.page;
  const DevPage P = b.pages[p];
  const PageState S = b.states[p];
  const int tid = threadIdx.x, lane = tid & 63;
  const uint8_t* img = b.payload + P.image_off;
  const bool is64 = P.kind == K_DELTA64;
  const bool lens = P.kind == K_DLBA || P.kind == K_DBA;
  const int64_t e = S.val_e;
  if (tid < 64) {
    int32_t kmax = 0;
    const bool load_ok = S.err == kNoError || (S.err >> 56) > 0;
    if (P.host_err == kNoError && load_ok) {
      Win w{img, e, reinterpret_cast<uint8_t*>(T.data), 0, 0};
      win_load(w, S.val_s, lane);
      const bool before_values = S.err != kNoError && (S.err >> 56) <= 2;
      DeltaState D;
      int32_t vc;
      uint64_t md, widths;
      int64_t pos = S.val_s, h0 = pos;
      if (delta_init(w, pos, is64, D, vc, md, widths, lane, &h0) == kNoError && D.mode == DM_FAST) {
        const int64_t nn = lens ? vc : (before_values ? 0 : S.nn);
        kmax = int32_t(delta_whole_blocks(nn, vc, D.block_size, P.dblk_cap));
        if (tid == 0) {
          s_geo[1] = D.block_size;
          s_geo[2] = D.mb_count;
          s_geo[3] = D.mbvc;
          s_first = D.first;
          s_h = h0;
          s_geo[4] = vc;
        }
      }
    }
    if (tid == 0) {
      s_geo[0] = kmax;
      s_neg = ~0ull >> 1;
    }
  }
  __syncthreads();
  const int kmax = s_geo[0];
#ifdef PQH_FUSED_PROF
  uint64_t t_ph = wall_clock64();
  FPROF_ADD(0, t_ph - t_begin);
#endif
  // DELTA_LENGTH: tile byte sums + first negative length of the head (k_delta_init zeroed the sums)
  const bool sums = kLens && P.kind == K_DLBA && kmax > 0;
  LenSums ls{b.basums + P.batile_base, sums ? (S.val_limit < s_geo[4] ? S.val_limit : s_geo[4]) : 0, INT64_MAX};
  int r = 0;
  int64_t h = s_h;
  uint64_t carry = s_first;
  if (kmax > 0) {
    const int bs = s_geo[1], mbc = s_geo[2], mbvc = s_geo[3], gbytes = mbvc / 8;
    const int lbs = __builtin_ctz(uint32_t(bs)), lmb = __builtin_ctz(uint32_t(mbvc));
    const DevChunk C = b.chunks[P.chunk];
    int32_t* lp = P.kind == K_DBA ? C.aux2 : C.aux;
    uint8_t* out = lens ? reinterpret_cast<uint8_t*>(lp + S.value_base) : C.values + S.value_base * P.value_size;
    const bool before_values = S.err != kNoError && (S.err >> 56) <= 2;
    const int64_t vcap = lens ? (before_values ? 0 : int64_t(S.nn)) : int64_t(kmax) << lbs;  // values to emit
    const int64_t img_len = P.image_len;
    int32_t est = 0;  // 0: the first tile measures block 0
    int64_t a0 = -1;  // the stage's base
    for (;;) {
      __syncthreads();  // the previous tile's readers of T are done
      // restage from the next header unless the stage still holds a whole tile's worth of blocks
      // after it (narrow streams -- DELTA_LENGTH lengths of ~100 bytes per block -- fit 2-6 tiles in
      // one stage: one HBM round trip instead of one per tile)
      if (a0 < 0 || h - a0 + int64_t(est) * kTileBlocks + 512 > T.kStageBytes - 64) {
        a0 = h - int64_t((reinterpret_cast<uintptr_t>(img) + uintptr_t(h)) & 15);
        stage_copy(reinterpret_cast<uint4*>(T.data), img + a0, T.kStageBytes / 16, img_len - a0);
        __syncthreads();
      }
#ifdef PQH_FUSED_PROF
      { FPROF_T(t); FPROF_ADD(1, t - t_ph); t_ph = t; FPROF_ADD(5, 1); }
#endif
      if (tid < 64) {
        int n;
        int32_t nxt;
        bool stop;
        const int nmax = kmax - r < kTileBlocks ? kmax - r : kTileBlocks;
        lds_chase(T.data, int32_t(h - a0), int32_t(e - a0), est, nmax, is64, mbc,
                  gbytes, s_lst, s_blkbit, s_blkw, T.md, lane, n, nxt, stop, T.kStageBytes);
        if (tid == 0) {
          s_n = n;
          s_stop = stop;
          s_h = a0 + nxt;
        }
      }
      __syncthreads();
      const int n = s_n;
#ifdef PQH_FUSED_PROF
      { FPROF_T(t); FPROF_ADD(2, t - t_ph); t_ph = t; }
#endif
      if (n == 0) break;
      for (int i = tid; i < n * 8; i += kBlock) {  // miniblock tables
        const int blk = i >> 3, m = i & 7;
        const uint64_t wd = s_blkw[blk];
        const int wm = m < mbc ? int((wd >> (8 * m)) & 0xff) : 0;
        const uint64_t below = m ? wd & ((1ull << (8 * m)) - 1) : 0;
        T.mbbit[blk][m] = s_blkbit[blk] + int32_t(widths_sum(below)) * mbvc;
        T.mbw[blk][m] = uint8_t(wm);
      }
      __syncthreads();
#ifdef PQH_FUSED_PROF
      { FPROF_T(t); FPROF_ADD(3, t - t_ph); t_ph = t; }
#endif
      const int64_t v0 = int64_t(r) << lbs;
      int64_t v1 = int64_t(r + n) << lbs;
      if (v1 > vcap) v1 = vcap;
      if (v0 < v1) {
        if constexpr (kLens) {
          if (sums) carry = expand_rows<true, PQH_LENS_ROWS>(T, v0, v1, lbs, lmb, out, false, carry, &ls);
          else carry = expand_rows(T, v0, v1, lbs, lmb, out, is64, carry);
        } else {
          carry = expand_rows(T, v0, v1, lbs, lmb, out, is64, carry);
        }
      }
#ifdef PQH_FUSED_PROF
      __syncthreads();
      { FPROF_T(t); FPROF_ADD(4, t - t_ph); t_ph = t; }
#endif
      est = int32_t((s_h - h) / n);  // mean block span so far: the next tile's lane segments
      r += n;
      h = s_h;
      if (s_stop || r >= kmax || v1 >= vcap) break;
    }
  }
  if (sums && ls.neg != INT64_MAX) atomicMin(&s_neg, (unsigned long long)ls.neg);
  __syncthreads();
  if (tid == 0) {
    b.dstates[p].nblocks = r;
    b.dstates[p].end_pos = h;
    b.dstates[p].head_blocks = r;
    b.dstates[p].head_carry = carry;
    b.dstates[p].head_neg = int64_t(s_neg);  // counts only if k_delta_walk accepts the head
  }
#ifdef PQH_FUSED_PROF
  prof[7] = wall_clock64() - t_begin;
  if (tid == 0)
    for (int k = 0; k < 8; k++) atomicAdd(&g_fprof[kLens ? 1 : 0][k], (unsigned long long)prof[k]);
#endif
}

__global__ __launch_bounds__(256) PQH_FUSED_ATTR void k_delta_fused(DevBatch b, const Tile* streams) {
  delta_fused_body<false>(b, streams);
}
__global__ __launch_bounds__(256) void k_delta_fused_lens(DevBatch b, const Tile* streams) {
  delta_fused_body<true>(b, streams);
}

// ------------------------------------------------------------------------------------------------
// k_delta_split (page mode): the head of every DELTA stream decoded by many workgroups per page
// instead of one (k_delta_fused), so that a page's ~0.16 ms dependent chain of stage -> chase ->
// expand no longer sets the time of a small shard (C3's N = 8 block: 960 pages for 2048 slots).
// Reference: deltaBitPackDecoder.next (deltabp_decoder.go:113-174), value[i + 1] = value[i] +
// delta[i] + minDelta over the chain of blocks (:51-111); byteArrayDeltaLengthDecoder's lengths
// (type_bytearray.go:98-140).
//   * a page's stream is cut into windows of kSplitStride bytes from block 0's header h0: window w
//     owns the blocks whose header lies in [B_w, B_w+1), B_w = h0 + w * kSplitStride;
//   * one workgroup per window, by ticket window-major (every page's window 0, then every window 1,
//     ...), stages its bytes (kSplitStage: the stride + room for the block that crosses its end),
//     takes its entry -- window 0: h0; w > 0: the first position >= B_w where three consecutive
//     headers parse (a guess) -- and chases its blocks with lds_chase; their sum of delta + minDelta
//     (the window's aggregate) is computed from the staged bytes;
//   * decoupled look-back over three 64-bit words per window (relaxed agent-scope atomics, each of
//     the two carry words tagged with the status word's high half, so that a reader takes only a
//     consistent triple -- no fence, no L2 write-back): PARTIAL = (blocks, guessed entry, exit,
//     aggregate), FINAL = (blocks through the window, exit, value after it, ended).  The nearest
//     FINAL plus the PARTIALs after it give a window its first block and carry when every PARTIAL's
//     guessed entry is its predecessor's exit; otherwise it waits for its predecessor's FINAL.  A
//     wrong guess of its own is chased again from the true entry (the bytes are still staged);
//   * the page's head is the whole blocks [0, R) that k_delta_fused would decode (R from
//     delta_whole_blocks and the positions to emit); a chain that stops earlier (a header the
//     common-case parse rejects, the stream end, a block wider than the stage's slack, more than
//     kSplitMaxBlocks blocks in a window) ends the head there.  The window that ends the head writes
//     (nblocks, end_pos, head_blocks, head_carry) -- exactly what k_delta_fused leaves -- and
//     k_delta_walk / k_delta_page continue from it with the reference's exact semantics.
// ------------------------------------------------------------------------------------------------
constexpr int kSplitStage = kFusedStage;  // 14848: the stride + 2.5 KiB for the block crossing its end
constexpr int kSplitMaxBlocks = 1024;     // a window with more blocks (near-constant data) ends the head
constexpr int kSplitSpinCap = 1 << 22;
constexpr uint64_t kSpPartial = 1ull << 62, kSpFinal = 2ull << 62, kSpEnded = 1ull << 61;

// The sum of delta + minDelta over the whole blocks [v0, v1) of the staged table (block-aligned v0;
// wrapping: the 32-bit streams use its low half).  Whole workgroup; every thread gets the total.
template <class L>
__device__ uint64_t split_sum(const L& T, int64_t v0, int64_t v1, int lbs, int lmb, uint64_t* wsum) {
  const int bb0 = int(v0 >> lbs);
  uint64_t acc = 0;
  for (int64_t p = v0 + 4 * int64_t(threadIdx.x); p < v1; p += 4 * kBlock) {
    const int blk = int(p >> lbs) - bb0;
    const int m = int(p & ((int64_t(1) << lbs) - 1)) >> lmb;
    if (T.mbw[blk][m] <= 32) {
      uint32_t u[4];
      uint64_t md;
      int bk;
      staged_u32<4>(T, int32_t(p), bb0, lbs, lmb, u, md, bk);
      acc += uint64_t(u[0]) + u[1] + u[2] + u[3] + 4 * md;
    } else {
      uint64_t d[2], d2[2];
      staged_delta2(T, p, bb0, lbs, lmb, d);
      staged_delta2(T, p + 2, bb0, lbs, lmb, d2);
      acc += d[0] + d[1] + d2[0] + d2[1];
    }
  }
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) wsum[threadIdx.x >> 6] = acc;
  __syncthreads();
  return wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

struct SplitLds {
  PageTileLdsT<kSplitStage> T;
  int16_t hdr[kSplitMaxBlocks + 1];  // stage-relative header offsets of the window's chain
  int32_t blkbit[kTileBlocks];
  uint64_t blkw[kTileBlocks];
  int16_t lst[kChaseCap][64];
  uint64_t wsum[4];
  int64_t sh[8];
  int32_t si[8];
  unsigned long long neg;
};

// Wave 0: the first position in [loc, lim) where a header and its two successors parse inside the
// stage (or the chain reaches the stream's end exactly); lim if none.
__device__ __forceinline__ int32_t split_guess(const uint32_t* data, int32_t loc, int32_t lim, int32_t eloc, bool is64,
                                               int mbc, int gbytes) {
  const int lane = threadIdx.x & 63;
  const int32_t plim = kSplitStage - 32, dlim = kSplitStage - 16;
  for (int32_t x0 = loc; x0 < lim; x0 += 64) {
    const int32_t x = x0 + lane;
    int32_t d1 = -1, d2 = -1, d3 = -1;
    bool ok = x < lim && lds_block(data, x, eloc, plim, dlim, is64, mbc, gbytes, d1);
    ok = ok && (d1 == eloc || lds_block(data, d1, eloc, plim, dlim, is64, mbc, gbytes, d2));
    ok = ok && (d1 == eloc || d2 == eloc || lds_block(data, d2, eloc, plim, dlim, is64, mbc, gbytes, d3));
    const uint64_t m = __ballot(ok);
    if (m) return x0 + __builtin_ctzll(m);
  }
  return lim;
}

// Chase the window's chain from `entry` (stage-relative): headers into S.hdr, the aggregate, the
// exit (the first header >= wend, or where the chain stops).  Whole workgroup.  Returns the number
// of blocks; *stop = the chain ends inside the window (*exit is then where it stops).
__device__ int split_chain(SplitLds& S, int32_t entry, int32_t wend, int32_t eloc, bool is64, int mbc, int mbvc,
                           int lbs, int lmb, uint64_t* agg, int32_t* exit, bool* stop) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int gbytes = mbvc / 8;
  int count = 0;
  uint64_t sum = 0;
  int32_t loc = entry;
  int32_t est = 0;
  bool stopped = false;
  for (;;) {
    if (loc >= wend) break;
    if (count >= kSplitMaxBlocks) {
      stopped = true;
      break;
    }
    if (tid < 64) {
      int n;
      int32_t nxt;
      bool st;
      const int nmax = kSplitMaxBlocks - count < kTileBlocks ? kSplitMaxBlocks - count : kTileBlocks;
      lds_chase(S.T.data, loc, eloc, est, nmax, is64, mbc, gbytes, S.lst, S.blkbit, S.blkw, S.T.md, lane, n, nxt, st,
                kSplitStage);
      // headers of the chased blocks; keep those that start before wend
      int32_t h = -1;
      if (lane < n) h = lane == 0 ? loc : 0;
      if (lane >= 1 && lane <= n) {  // header k = the data end of block k - 1
        h = S.blkbit[lane - 1] / 8 + int32_t(widths_sum(S.blkw[lane - 1])) * gbytes;
      }
      const uint64_t inside = __ballot(lane < n && h < wend);
      const int keep = inside == ~0ull ? 64 : __builtin_ctzll(~inside);  // (headers ascend)
      if (lane < keep) S.hdr[count + lane] = int16_t(h);
      int32_t next = keep < n ? __builtin_amdgcn_readlane(h, keep) : nxt;
      bool stp = keep < n ? false : st;
      // a block ending past the stage (not a parse failure): the head ends at it
      if (keep == n && !st && n < nmax && next < wend) stp = true;
      if (tid == 0) {
        S.si[0] = keep;
        S.si[1] = next;
        S.si[2] = stp;
      }
    }
    __syncthreads();
    const int keep = S.si[0];
    const int32_t next = S.si[1];
    if (keep > 0) {
      for (int i = tid; i < keep * 8; i += kBlock) {  // miniblock tables of the kept blocks
        const int blk = i >> 3, m = i & 7;
        const uint64_t wd = S.blkw[blk];
        const uint64_t below = m ? wd & ((1ull << (8 * m)) - 1) : 0;
        S.T.mbbit[blk][m] = S.blkbit[blk] + int32_t(widths_sum(below)) * mbvc;
        S.T.mbw[blk][m] = uint8_t(m < mbc ? int((wd >> (8 * m)) & 0xff) : 0);
      }
      __syncthreads();
      const int64_t v0 = int64_t(count) << lbs;
      sum += split_sum(S.T, v0, v0 + (int64_t(keep) << lbs), lbs, lmb, S.wsum);
      est = (next - loc) / keep;
    }
    count += keep;
    loc = next;
    const bool stp = S.si[2] != 0;
    __syncthreads();  // (S.si / tables read by every thread before the next round rewrites them)
    if (stp) {
      stopped = true;
      break;
    }
    if (keep == 0) break;
  }
  *agg = sum;
  *exit = loc;
  *stop = stopped;
  return count;
}

// Tables of the window's blocks [k0, k0 + n) (n <= 64) from their headers (stage-relative).
__device__ __forceinline__ void split_tables(SplitLds& S, int k0, int n, bool is64, int mbc, int mbvc) {
  const int tid = threadIdx.x;
  if (tid < n) {
    int32_t dat;
    uint64_t md, wd;
    lds_hdr(S.T.data, S.hdr[k0 + tid], is64, mbc, mbvc / 8, dat, md, wd);
    S.T.md[tid] = md;
    S.blkbit[tid] = dat * 8;
    S.blkw[tid] = wd;
  }
  __syncthreads();
  for (int i = tid; i < n * 8; i += kBlock) {
    const int blk = i >> 3, m = i & 7;
    const uint64_t wd = S.blkw[blk];
    const uint64_t below = m ? wd & ((1ull << (8 * m)) - 1) : 0;
    S.T.mbbit[blk][m] = S.blkbit[blk] + int32_t(widths_sum(below)) * mbvc;
    S.T.mbw[blk][m] = uint8_t(m < mbc ? int((wd >> (8 * m)) & 0xff) : 0);
  }
  __syncthreads();
}

__device__ __forceinline__ void split_publish(uint64_t* words, int t, uint64_t w0, uint64_t carry) {
  const uint64_t tag = w0 & 0xffffffff00000000ull;
  __hip_atomic_store(words + 3 * int64_t(t) + 1, tag | (carry & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(words + 3 * int64_t(t) + 2, tag | (carry >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(words + 3 * int64_t(t), w0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// A consistent (status, carry) of window j, or status 0 when not (yet) published.
__device__ __forceinline__ uint64_t split_read(const uint64_t* words, int64_t j, uint64_t* carry) {
  const uint64_t w0 = __hip_atomic_load(words + 3 * j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if ((w0 >> 62) == 0) return 0;
  const uint64_t w1 = __hip_atomic_load(words + 3 * j + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t w2 = __hip_atomic_load(words + 3 * j + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t tag = w0 & 0xffffffff00000000ull;
  if ((w1 & 0xffffffff00000000ull) != tag || (w2 & 0xffffffff00000000ull) != tag) return 0;
  *carry = (w1 & 0xffffffffull) | (w2 << 32);
  return w0;
}

// Wave 0: window t (page window w >= 1, the page's window 0 at t - w).  Returns false when the
// look-back is not decisive (wait for window t - 1's FINAL); otherwise the blocks and the value
// before window t, the exit of window t - 1 and whether the head already ended.
__device__ bool split_lookback(const uint64_t* words, int t, int w, int64_t h0, int64_t* pblk, uint64_t* pcarry,
                               int64_t* pexit, bool* pended, bool* timeout) {
  const int lane = threadIdx.x & 63;
  const int first = t - w;
  int hi = t - 1;
  int64_t cnt = 0, need = -1, exit1 = -1;
  uint64_t acc = 0;
  bool ended1 = false;
  for (bool round0 = true;; round0 = false) {
    const int j = hi - lane;
    const bool in = j >= first;
    uint64_t v = 0, c = 0;
    for (int spin = 0;; spin++) {
      if (in && v == 0) v = split_read(words, j, &c);
      if (__ballot(in && v == 0) == 0) break;
      if (spin > kSplitSpinCap) {
        *timeout = true;
        return true;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    const bool fin = in && (v >> 62) == 2;
    const uint64_t fm = __ballot(fin);
    const int f = fm ? __builtin_ctzll(fm) : 64;
    const int64_t ex = int64_t(uint32_t(v));
    const bool end = (v & kSpEnded) != 0;
    // the PARTIAL's guessed entry: its window base + the 16-bit offset
    const int64_t ent = h0 + int64_t(w - (t - j)) * kSplitStride + int64_t((v >> 45) & 0xffff);
    int64_t nxt = __shfl_up(ent, 1, 64);  // the entry the next newer window guessed
    if (lane == 0) nxt = need;
    if (round0) {
      exit1 = __shfl(ex, 0, 64);
      ended1 = __shfl(int(end), 0, 64) != 0;
    }
    // a FINAL that ended the head: everything after it is past the head
    if (f < 64 && __shfl(int(end), f, 64)) {
      // (consistency of the PARTIALs after it is irrelevant: no window after an ended head writes)
      const uint64_t vf = __shfl(v, f, 64);
      *pblk = int64_t((vf >> 32) & 0x1fffffff);
      *pcarry = 0;
      *pexit = int64_t(uint32_t(vf));
      *pended = true;
      return true;
    }
    const bool lead = round0 && lane == 0;
    // lanes before the FINAL: each exit meets its successor's guess; only window t - 1 may end
    const bool ok = !in || lane > f || ((nxt < 0 || ex == nxt) && (!end || lead));
    if (__ballot(!ok)) return false;
    uint64_t a = (in && lane < f) ? c : 0;
    int64_t k = (in && lane < f) ? int64_t((v >> 32) & 0x1fff) : 0;
    for (int off = 32; off > 0; off >>= 1) {
      a += __shfl_xor(a, off, 64);
      k += __shfl_xor(k, off, 64);
    }
    if (f < 64) {
      const uint64_t vf = __shfl(v, f, 64);
      const uint64_t cf = __shfl(c, f, 64);
      *pblk = int64_t((vf >> 32) & 0x1fffffff) + cnt + k;
      *pcarry = cf + acc + a;
      *pexit = exit1;
      *pended = ended1;
      return true;
    }
    acc += a;
    cnt += k;
    need = __shfl(ent, 63, 64);
    hi -= 64;
  }
}

template <bool kLens>
__device__ __forceinline__ void delta_split_body(DevBatch b, const int2* wins, const int32_t* order, int32_t nwin,
                                                 uint32_t* ticket) {
  __shared__ SplitLds S;
  const int tid = threadIdx.x, lane = tid & 63;
  // (ticket == nullptr: the dispatch order itself, blockIdx.x -- no contended atomic per window)
  if (tid == 0) S.sh[0] = ticket ? atomicAdd(ticket, 1u) : blockIdx.x;
  __syncthreads();
  if (int(S.sh[0]) >= nwin) return;
  const int t = order[S.sh[0]];
  const int2 pw = wins[t];
  const int p = pw.x, w = pw.y;
  const DeltaSplit Q = b.dsplit[p];
  if (Q.R <= 0) return;
  const int64_t Bw = Q.h0 + int64_t(w) * kSplitStride;
  if (Bw >= Q.e) return;  // no header starts here (nor in the page's later windows)
  const DevPage P = b.pages[p];
  const uint8_t* img = b.payload + P.image_off;
  const bool is64 = P.kind == K_DELTA64;
  const int bs = Q.bs, mbc = Q.mbc, mbvc = Q.mbvc;
  const int lbs = __builtin_ctz(uint32_t(bs)), lmb = __builtin_ctz(uint32_t(mbvc));
  const int64_t a0 = Bw - int64_t((reinterpret_cast<uintptr_t>(img) + uintptr_t(Bw)) & 15);
  stage_copy(reinterpret_cast<uint4*>(S.T.data), img + a0, kSplitStage / 16, Q.e - a0);
  if (tid < 4) S.T.data[kSplitStage / 4 + tid] = 0;
  __syncthreads();
  const int32_t eloc = int32_t(Q.e - a0 < kSplitStage ? Q.e - a0 : kSplitStage + 64);  // (past the stage: never reached)
  const int32_t wend = int32_t(Bw - a0) + kSplitStride;
  int32_t entry = int32_t(Q.h0 - a0);
  if (w > 0) {
    if (tid < 64) {
      const int32_t g = split_guess(S.T.data, int32_t(Bw - a0), wend, eloc, is64, mbc, mbvc / 8);
      if (tid == 0) S.si[3] = g;
    }
    __syncthreads();
    entry = S.si[3];
  }
  uint64_t agg;
  int32_t ex;
  bool stop;
  int n = entry < wend ? split_chain(S, entry, wend, eloc, is64, mbc, mbvc, lbs, lmb, &agg, &ex, &stop) : 0;
  if (entry >= wend) {
    agg = 0;
    ex = entry;
    stop = false;
  }
  uint64_t* words = b.dwords;
  int64_t pblk = 0;
  uint64_t carry = Q.first;
  bool pended = false;
  if (w > 0) {
    if (tid == 0)  // PARTIAL
      split_publish(words, t, kSpPartial | (stop ? kSpEnded : 0) | (uint64_t(entry - int32_t(Bw - a0)) << 45) |
                                  (uint64_t(n) << 32) | uint64_t(uint32_t(a0 + ex)),
                    agg);
    if (tid < 64) {
      int64_t pb = 0, pe = 0;
      uint64_t pc = 0;
      bool en = false, to = false;
      if (!split_lookback(words, t, w, Q.h0, &pb, &pc, &pe, &en, &to)) {
        uint64_t v = 0, c = 0;
        for (int spin = 0;; spin++) {  // the predecessor's FINAL
          if (tid == 0) v = split_read(words, t - 1, &c);
          v = __shfl(v, 0, 64);
          if ((v >> 62) == 2) break;
          if (spin > kSplitSpinCap) {
            to = true;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
        c = __shfl(c, 0, 64);
        pb = int64_t((v >> 32) & 0x1fffffff);
        pc = c;
        pe = int64_t(uint32_t(v));
        en = (v & kSpEnded) != 0;
      }
      if (tid == 0) {
        if (to) {  // never expected: the page errs instead of hanging (PQH_ERR_INTERNAL)
          atomicMin(&b.states[p].err, (unsigned long long)err_key(3, 0, PQH_ERR_INTERNAL));
          en = true;
        }
        S.sh[1] = pb;
        S.sh[2] = int64_t(pc);
        S.sh[3] = pe;
        S.sh[4] = en;
      }
    }
    __syncthreads();
    pblk = S.sh[1];
    carry = uint64_t(S.sh[2]);
    const int64_t pexit = S.sh[3];
    pended = S.sh[4] != 0;
    if (!pended && pexit != a0 + entry) {
      // a wrong guess: the true entry is the predecessor's exit (>= B_w)
      const int32_t te = int32_t(pexit - a0);
      if (te < wend) {
        n = split_chain(S, te, wend, eloc, is64, mbc, mbvc, lbs, lmb, &agg, &ex, &stop);
      } else {
        n = 0;
        agg = 0;
        ex = te;
        stop = false;
      }
    }
  }
  if (pended) {
    if (tid == 0) split_publish(words, t, kSpFinal | kSpEnded | (uint64_t(pblk & 0x1fffffff) << 32), 0);
    return;
  }
  // the head: whole blocks [0, R)
  const int64_t R = Q.R;
  const int use = int(pblk + n <= R ? n : (R - pblk > 0 ? R - pblk : 0));
  bool ended = stop || pblk + use >= R;
  int64_t hexit = a0 + ex;  // the header after this window's blocks of the head
  uint64_t after = carry + agg;
  if (use < n) {
    hexit = a0 + S.hdr[use];
    ended = true;
  }
  // tables of the blocks in use (the chase left those of its last round: rebuilt unless that round
  // covered them all), the exact value after them when the head ends inside the window, expansion
  // FINAL before the expansion, so that the windows after this one need not wait for it (its carry
  // counts only while the head goes on: when the head ends here, the value after it is computed
  // below for k_delta_walk / k_delta_page)
  if (tid == 0)
    split_publish(words, t, kSpFinal | (ended ? kSpEnded : 0) | (uint64_t((pblk + use) & 0x1fffffff) << 32) |
                                uint64_t(uint32_t(hexit)),
                  after);
  const int64_t vcap = Q.vcap;
  LenSums ls{b.basums + P.batile_base, Q.lim, INT64_MAX};
  const DevChunk C = b.chunks[P.chunk];
  const bool lens = P.kind == K_DLBA || P.kind == K_DBA;
  int32_t* lp = P.kind == K_DBA ? C.aux2 : C.aux;
  const PageState PS = b.states[p];
  uint8_t* out = lens ? reinterpret_cast<uint8_t*>(lp + PS.value_base) : C.values + PS.value_base * P.value_size;
  uint64_t c = carry;
  uint64_t partial = 0;  // the sum over the blocks in use (only needed when use < n)
  for (int k0 = 0; k0 < use; k0 += kTileBlocks) {
    const int nb = use - k0 < kTileBlocks ? use - k0 : kTileBlocks;
    __syncthreads();
    split_tables(S, k0, nb, is64, mbc, mbvc);
    const int64_t v0 = (pblk + k0) << lbs;
    if (use < n) partial += split_sum(S.T, v0, v0 + (int64_t(nb) << lbs), lbs, lmb, S.wsum);
    int64_t v1 = (pblk + k0 + nb) << lbs;
    if (v1 > vcap) v1 = vcap;
    if (v0 < v1) {
      if constexpr (kLens) c = expand_rows<true>(S.T, v0, v1, lbs, lmb, out, false, c, &ls);
      else c = expand_rows(S.T, v0, v1, lbs, lmb, out, is64, c);
    }
  }
  if (use < n) after = carry + partial;
  if constexpr (kLens) {
    if (ls.neg != INT64_MAX) atomicMin(reinterpret_cast<unsigned long long*>(&b.dstates[p].head_neg),
                                       (unsigned long long)ls.neg);
  }
  // the head ends in this window when it ends here and began before it (pblk >= R: the head ended
  // exactly where this window starts, and the window that reached R wrote it)
  if (ended && pblk < R && tid == 0) {  // what k_delta_fused leaves for k_delta_walk / k_delta_page
    b.dstates[p].nblocks = int32_t(pblk + use);
    b.dstates[p].end_pos = hexit;
    b.dstates[p].head_blocks = int32_t(pblk + use);
    b.dstates[p].head_carry = after;
  }
}

__global__ __launch_bounds__(256) void k_delta_split(DevBatch b, const int2* wins, const int32_t* order, int32_t nwin,
                                                     int32_t use_ticket) {
  delta_split_body<false>(b, wins, order, nwin, use_ticket ? b.dticket : nullptr);
}
__global__ __launch_bounds__(256) void k_delta_split_lens(DevBatch b, const int2* wins, const int32_t* order,
                                                          int32_t nwin, int32_t use_ticket) {
  delta_split_body<true>(b, wins, order, nwin, use_ticket ? b.dticket + 1 : nullptr);
}

// k_delta_init (page mode, before k_scan): deltaBitPackDecoder.init of every DELTA_BINARY_PACKED
// page, so that its load errors (phase 0) are known to the value-offset scan before k_delta_fused
// decodes into the chunk outputs.  k_delta_walk repeats the init later and finds the same keys.
__global__ __launch_bounds__(256) void k_delta_init(DevBatch b, const int32_t* delta_pages, int32_t n) {
  __shared__ __attribute__((aligned(16))) uint8_t win_all[4][kWin];
  const int lane = threadIdx.x & 63;
  const int wv = int(threadIdx.x >> 6);
  const int idx = __builtin_amdgcn_readfirstlane(int(blockIdx.x) * 4 + wv);
  if (idx >= n) return;
  const int p = delta_pages[idx];
  const DevPage P = b.pages[p];
  const PageState S = b.states[p];
  DeltaSplit Q;  // k_delta_split's view of the page (R = 0: nothing for it)
  Q.h0 = Q.e = Q.vcap = Q.lim = 0;
  Q.first = 0;
  Q.R = Q.bs = Q.mbc = Q.mbvc = 0;
  if (lane == 0 && b.dsplit) {  // no head until a k_delta_fused / k_delta_split window writes one
    b.dstates[p].nblocks = 0;
    b.dstates[p].end_pos = 0;
    b.dstates[p].head_blocks = 0;
    b.dstates[p].head_carry = 0;
    b.dstates[p].head_neg = INT64_MAX;
  }
  const bool load_ok = S.err == kNoError || (S.err >> 56) > 0;
  if (P.host_err == kNoError && load_ok) {
    if (P.kind == K_DLBA)  // k_delta_fused / k_delta_page add the tile byte sums of its lengths
      for (int k = lane; k < P.batile_n; k += 64) b.basums[P.batile_base + k] = 0;
    Win w{b.payload + P.image_off, S.val_e, win_all[wv], 0, 0};
    win_load(w, S.val_s, lane);
    DeltaState D;
    int32_t vc;
    uint64_t md, widths;
    int64_t pos = S.val_s, h0 = pos;
    const uint64_t err = delta_init(w, pos, P.kind == K_DELTA64, D, vc, md, widths, lane, &h0);
    if (lane == 0 && err != kNoError) atomicMin(&b.states[p].err, (unsigned long long)err);
    if (err == kNoError && D.mode == DM_FAST) {  // k_delta_fused's head, as whole blocks [0, R)
      const bool lens = P.kind == K_DLBA || P.kind == K_DBA;
      const bool before_values = S.err != kNoError && (S.err >> 56) <= 2;
      const int64_t nn = lens ? vc : (before_values ? 0 : S.nn);
      const int64_t kmax = delta_whole_blocks(nn, vc, D.block_size, P.dblk_cap);
      const int lbs = __builtin_ctz(uint32_t(D.block_size));
      const int64_t vcap = lens ? (before_values ? 0 : int64_t(S.nn)) : kmax << lbs;
      const int64_t need = (vcap + D.block_size - 1) >> lbs;
      Q.R = int32_t(kmax < need ? kmax : need);
      Q.h0 = h0;
      Q.e = S.val_e;
      Q.vcap = vcap;
      Q.lim = P.kind == K_DLBA ? (S.val_limit < vc ? S.val_limit : vc) : 0;
      Q.first = D.first;
      Q.bs = D.block_size;
      Q.mbc = D.mb_count;
      Q.mbvc = D.mbvc;
    }
  }
  if (lane == 0 && b.dsplit) b.dsplit[p] = Q;
}
