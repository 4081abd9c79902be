// snappy_impl.h — page decompression on the device (included by decode.hip).
//
// The reference decompresses every page block on the host with github.com/golang/snappy v0.0.4
// (snappy.Decode, compress.go:43-49) inside readPageBlock / newBlockReader, which then checks the
// exact uncompressed size (compress.go:131-152).  Here the pages of SNAPPY chunks travel to HBM
// compressed and k_snappy rebuilds each page image in place of the host's decompressed copy:
//
//   block  = uvarint(decoded length) then elements (golang snappy decode.go):
//            tag & 3 == 0 literal  len-1 in tag>>2, or in the 1..4 bytes after it (tag>>2 = 60..63)
//                       1 copy     len 4 + ((tag>>2) & 7), offset ((tag>>5) << 8) | next byte
//                       2 copy     len 1 + (tag>>2), 16-bit LE offset
//                       3 copy     len 1 + (tag>>2), 32-bit LE offset
//   errors = ErrCorrupt: a malformed / > 0xffffffff length, an element past the input or the
//            output, a copy offset of 0 or before the output start, a short output; plus the
//            reference's size check against the page header -> PQH_ERR_DECOMPRESS.
//
// One wave per page.  The element chain is sequential by definition; it is resolved 64 input bytes
// at a time: every lane decodes the element that WOULD start at its byte, the wave then follows
// the true chain from the window's first element with readlane steps, and a wave scan places the
// chain's elements in the output.  The batch's output bytes are then produced lane-parallel: a
// byte of a literal comes from the input; a byte of a copy maps to an earlier output position
// (periodically for overlapping copies) which is either written by an earlier batch (read back
// from HBM) or resolved again inside this batch.  Literals longer than one batch are copied in
// bulk.  DataPageV2 pages copy their uncompressed level prefix first (page_v2.go:116-125).
#pragma once

constexpr int kSnapBatch = 4096;  // output bytes resolved per batch (literals beyond: bulk copy)

struct SnapLds {
  int32_t out[65];  // element output start (stream-relative); out[m] = the batch's end
  int32_t src[64];  // literal: input position of its bytes; copy: offset
  int32_t len[64];
  uint8_t lit[64];
};

// n bytes from src to dst by one wave (any alignment): 16-byte stores once dst is aligned, each fed
// by an unaligned 16-byte load (the source payload keeps PQH_PAYLOAD_PAD readable bytes past it).
__device__ __forceinline__ void wave_copy(uint8_t* dst, const uint8_t* src, int64_t n) {
  const int lane = threadIdx.x & 63;
  const int64_t head0 = int64_t((16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15);
  const int64_t head = head0 < n ? head0 : n;
  if (lane < head) dst[lane] = src[lane];
  typedef uint4 uint4_u __attribute__((aligned(1)));
  const int64_t units = (n - head) >> 4;
  const uint4_u* sp = reinterpret_cast<const uint4_u*>(src + head);
  uint4* dp = reinterpret_cast<uint4*>(dst + head);
  for (int64_t u = lane; u < units; u += 64) dp[u] = sp[u];
  const int64_t done = head + units * 16;
  if (lane < n - done) dst[done + lane] = src[done + lane];
}

__device__ __forceinline__ int64_t wave_excl_scan64(int64_t x) {
  const int lane = threadIdx.x & 63;
  int64_t incl = x;
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t y = __shfl_up(incl, off, 64);
    if (lane >= off) incl += y;
  }
  return incl - x;
}

// Decode one snappy block src[0, n) into dst[0, expected).  Whole wave; returns PQH_OK or
// PQH_ERR_DECOMPRESS (uniform).
__device__ int snappy_block(const uint8_t* src, int64_t n, uint8_t* dst, int64_t expected, SnapLds& E) {
  const int lane = threadIdx.x & 63;
  // decodedLen: binary.Uvarint, at most 10 bytes; > 0xffffffff is ErrCorrupt
  uint64_t v = 0;
  int hl = 0;
  {
    bool done = false;
    for (int i = 0; i < 10 && i < n && !done; i++) {
      const uint8_t c = src[i];
      if (i == 9 && c > 1) return PQH_ERR_DECOMPRESS;  // overflows 64 bits
      v |= uint64_t(c & 0x7f) << (7 * i);
      hl = i + 1;
      done = c < 0x80;
    }
    if (!done || v > 0xffffffffull || int64_t(v) != expected) return PQH_ERR_DECOMPRESS;
  }
  const int32_t total = int32_t(v);
  int32_t p = hl, d = 0;
  while (p < n) {
    // ---- every lane: the element that would start at byte q
    const int32_t q = p + lane;
    uint64_t w = 0;
    __builtin_memcpy(&w, src + q, 8);  // in the page's bytes or the payload pad
    const uint32_t tag = uint32_t(w & 0xff);
    int32_t hdr, off = 0;
    int64_t len;
    bool lit = (tag & 3) == 0;
    if (lit) {
      const uint32_t x = tag >> 2;
      if (x < 60) {
        hdr = 1;
        len = int64_t(x) + 1;
      } else {
        const int k = int(x) - 59;
        hdr = 1 + k;
        len = int64_t((w >> 8) & (k == 4 ? 0xffffffffull : ((1ull << (8 * k)) - 1))) + 1;
      }
    } else if ((tag & 3) == 1) {
      hdr = 2;
      len = 4 + ((tag >> 2) & 7);
      off = int32_t(((tag >> 5) << 8) | ((w >> 8) & 0xff));
    } else if ((tag & 3) == 2) {
      hdr = 3;
      len = 1 + (tag >> 2);
      off = int32_t((w >> 8) & 0xffff);
    } else {
      hdr = 5;
      len = 1 + (tag >> 2);
      const uint64_t o = (w >> 8) & 0xffffffffull;
      off = o > 0x7fffffffull ? 0x7fffffff : int32_t(o);  // beyond any output position: invalid
    }
    const bool hdr_ok = int64_t(q) + hdr <= n;
    const int64_t nx64 = int64_t(q) + hdr + (lit ? len : 0);
    const int32_t nxt = nx64 > n ? int32_t(n) + 1 : int32_t(nx64);  // past the input: invalid below
    // ---- the true chain from p (the window's first element), wave-uniform
    uint64_t chain = 0;
    bool bad = false;
    for (int32_t pos = p; pos < p + 64 && pos < n;) {
      const int l = pos - p;
      chain |= 1ull << l;
      if (!__builtin_amdgcn_readlane(int(hdr_ok), l)) {
        bad = true;
        break;
      }
      pos = __builtin_amdgcn_readlane(nxt, l);
    }
    if (bad) return PQH_ERR_DECOMPRESS;
    const bool on = (chain >> lane) & 1;
    const int idx = __popcll(chain & ((1ull << lane) - 1));
    // ---- output positions of the chain's elements; checks of every element (decode.go order: all
    // of them fail as ErrCorrupt, so which one does not matter)
    const int64_t excl = wave_excl_scan64(on ? len : 0);
    const int64_t eo = int64_t(d) + excl;
    bool ebad = false;
    if (on) {
      if (lit) ebad = nx64 > n || eo + len > total;
      else ebad = off == 0 || off > eo || eo + len > total;
    }
    if (__ballot(ebad)) return PQH_ERR_DECOMPRESS;
    // every chain element now lies inside the output: lengths and positions fit 32 bits
    const int32_t ln32 = int32_t(len);
    // ---- batch: the chain's first m elements whose output fits kSnapBatch (copies are <= 64 bytes)
    const uint64_t fit = __ballot(on && excl + len <= kSnapBatch);
    const int m = __popcll(fit);
    if (m == 0) {  // a literal longer than a batch (the chain's first element, lane 0): bulk copy
      const int32_t l0 = __builtin_amdgcn_readfirstlane(ln32);
      const int32_t h0 = __builtin_amdgcn_readfirstlane(hdr);
      wave_copy(dst + d, src + p + h0, l0);
      __syncthreads();
      d += l0;
      p = __builtin_amdgcn_readfirstlane(nxt);
      continue;
    }
    const int last = 63 - __builtin_clzll(fit);  // lane of element m-1 (fit is a prefix of the chain)
    const int32_t p_next = __builtin_amdgcn_readlane(nxt, last);
    const int32_t bend = d + __builtin_amdgcn_readlane(int32_t(excl) + ln32, last);
    if (on && idx < m) {
      E.out[idx] = int32_t(eo);
      E.len[idx] = ln32;
      E.lit[idx] = lit;
      E.src[idx] = lit ? q + hdr : off;
    }
    if (lane == 0) E.out[m] = bend;
    __syncthreads();
    // ---- the batch's output bytes, lane-parallel
    for (int32_t b = d + lane; b < bend; b += 64) {
      int32_t pos = b;
      uint8_t val;
      for (;;) {
        int lo = 0, hi = m;  // E.out[lo] <= pos < E.out[hi]
        while (hi - lo > 1) {
          const int mid = (lo + hi) >> 1;
          if (E.out[mid] <= pos) lo = mid;
          else hi = mid;
        }
        const int32_t rel = pos - E.out[lo];
        if (E.lit[lo]) {
          val = src[E.src[lo] + rel];
          break;
        }
        const int32_t o = E.src[lo];
        const int32_t s = E.out[lo] - o + (o < E.len[lo] ? rel % o : rel);  // overlapping copies repeat
        if (s < d) {  // written by an earlier batch
          val = dst[s];
          break;
        }
        pos = s;
      }
      dst[b] = val;
    }
    __syncthreads();  // this batch's bytes are visible to the next batches' reads
    d = bend;
    p = p_next;
  }
  return d == total ? PQH_OK : PQH_ERR_DECOMPRESS;
}

// One wave per page: its image rebuilt at image_offset from its source bytes (codec 0: copied).
__global__ __launch_bounds__(64) void k_snappy(const pqh_codec_page* cps, const uint8_t* src_all, uint8_t* dst_all,
                                               int32_t* status) {
  __shared__ SnapLds E;
  const pqh_codec_page cp = cps[blockIdx.x];
  const uint8_t* src = src_all + cp.src_offset;
  uint8_t* dst = dst_all + cp.image_offset;
  int rc = PQH_OK;
  if (cp.codec != PQH_CODEC_SNAPPY) {
    wave_copy(dst, src, cp.src_len < cp.image_len ? cp.src_len : cp.image_len);
    if (cp.src_len != cp.image_len) rc = PQH_ERR_DECOMPRESS;
  } else {
    const int32_t raw = cp.raw_len < cp.src_len ? cp.raw_len : cp.src_len;
    wave_copy(dst, src, raw < cp.image_len ? raw : cp.image_len);  // DataPageV2 levels: never compressed
    if (raw > cp.image_len) rc = PQH_ERR_DECOMPRESS;
    else rc = snappy_block(src + raw, cp.src_len - raw, dst + raw, int64_t(cp.image_len) - raw, E);
  }
  if (threadIdx.x == 0) status[blockIdx.x] = rc;
}
