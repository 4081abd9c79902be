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
// One workgroup per page.  The element chain is sequential by definition; it is resolved 64 input
// bytes at a time by wave 0 from an LDS stage of the compressed input: every lane decodes the
// element that WOULD start at its byte, the wave follows the true chain from the window's first
// element with readlane steps, and a wave scan places the chain's elements in the output.  Up to
// kSnapOut output bytes (kSnapMaxE elements) form a batch; all 256 threads then produce the batch's
// bytes: an output byte -> element map (max-scan of the elements' start markers) finds each byte's
// element; a literal byte comes from the stage (or HBM), a copy byte maps to an earlier output
// position (periodically for overlapping copies) that is resolved again inside the batch or read
// back from HBM, written by an earlier batch.  Literals longer than a batch are copied in bulk.
// DataPageV2 pages copy their uncompressed level prefix first (page_v2.go:116-125).
#pragma once

constexpr int kSnapStage = 8192;  // compressed input bytes staged in LDS per batch
constexpr int kSnapOut = 8192;    // output bytes per batch (a longer literal: bulk copy)
constexpr int kSnapMaxE = 1024;   // elements per batch

struct __attribute__((aligned(16))) SnapLds {
  uint8_t in[kSnapStage + 96];    // the stage: block bytes [a0, a0 + kSnapStage + 96)
  uint16_t emap[kSnapOut];        // batch output byte -> element; then (as int16) the byte's pointer
  uint8_t out[kSnapOut];          // the batch's output bytes
  int32_t eout[kSnapMaxE + 1];    // element output start, batch-relative; eout[nE] = the batch's size
  int32_t esrc[kSnapMaxE];        // literal: block position of its bytes; copy: offset
  int32_t elen[kSnapMaxE];
  uint8_t elit[kSnapMaxE];
  int32_t wmax[4];
  int32_t nE, bend, p_next, bad, bulk_len, bulk_src;
};

// n bytes from src to dst by the workgroup (any alignment): 16-byte stores once dst is aligned,
// each fed by an unaligned 16-byte load (the source payload keeps PQH_PAYLOAD_PAD readable bytes).
__device__ __forceinline__ void snap_copy(uint8_t* dst, const uint8_t* src, int64_t n) {
  const int tid = threadIdx.x;
  const int64_t head0 = int64_t((16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15);
  const int64_t head = head0 < n ? head0 : n;
  if (tid < head) dst[tid] = src[tid];
  typedef uint4 uint4_u __attribute__((aligned(1)));
  const int64_t units = (n - head) >> 4;
  const uint4_u* sp = reinterpret_cast<const uint4_u*>(src + head);
  uint4* dp = reinterpret_cast<uint4*>(dst + head);
  int64_t u = tid;
  for (; u + 3 * kBlock < units; u += 4 * kBlock) {  // four loads in flight
    const uint4 x0 = sp[u], x1 = sp[u + kBlock], x2 = sp[u + 2 * kBlock], x3 = sp[u + 3 * kBlock];
    dp[u] = x0;
    dp[u + kBlock] = x1;
    dp[u + 2 * kBlock] = x2;
    dp[u + 3 * kBlock] = x3;
  }
  for (; u < units; u += kBlock) dp[u] = sp[u];
  const int64_t done = head + units * 16;
  if (tid < n - done) dst[done + tid] = src[done + tid];
}

// (wave_excl_scan64: bytearray_impl.h)

// ---- Batch resolution shared by the device codecs (k_snappy, k_gzip).  A batch is up to kSnapOut
// output bytes made of elements (eout[e] = start, batch-relative; eout[nE] = the batch size).
constexpr int kPer = kSnapOut / kBlock;  // 32 output bytes per thread: b = i * kBlock + tid

// Output byte -> element: start markers of elements e0..nE-1, then a max-scan (element ids rise
// with output; bytes before the first marker map to 0).
template <class L>
__device__ __forceinline__ void batch_emap(L& E, int32_t nE, int32_t e0 = 0) {
  const int tid = threadIdx.x;
  {  // every thread owns 32 consecutive entries (64 bytes: four 16-byte LDS accesses)
    uint4* m4 = reinterpret_cast<uint4*>(E.emap) + tid * 4;
#pragma unroll
    for (int k = 0; k < 4; k++) m4[k] = make_uint4(0, 0, 0, 0);
  }
  __syncthreads();
  for (int e = e0 + tid; e < nE; e += kBlock) E.emap[E.eout[e]] = uint16_t(e);
  __syncthreads();
  {
    uint4* m4 = reinterpret_cast<uint4*>(E.emap) + tid * 4;
    uint32_t wv[16];
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint4 x = m4[k];
      wv[4 * k] = x.x;
      wv[4 * k + 1] = x.y;
      wv[4 * k + 2] = x.z;
      wv[4 * k + 3] = x.w;
    }
    uint32_t mx = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      const uint32_t a = wv[k] & 0xffff, c = wv[k] >> 16;
      mx = a > mx ? a : mx;
      mx = c > mx ? c : mx;
    }
    int32_t incl = int32_t(mx);  // inclusive max over the threads before
    for (int o = 1; o < 64; o <<= 1) {
      const int32_t y = __shfl_up(incl, o, 64);
      if ((tid & 63) >= o) incl = y > incl ? y : incl;
    }
    if ((tid & 63) == 63) E.wmax[tid >> 6] = incl;
    __syncthreads();
    int32_t runv = __shfl_up(incl, 1, 64);
    if ((tid & 63) == 0) runv = 0;
    for (int w8 = 0; w8 < (tid >> 6); w8++) runv = E.wmax[w8] > runv ? E.wmax[w8] : runv;
    uint32_t run = uint32_t(runv);
#pragma unroll
    for (int k = 0; k < 16; k++) {
      uint32_t a = wv[k] & 0xffff, c = wv[k] >> 16;
      run = a > run ? a : run;
      a = run;
      run = c > run ? c : run;
      c = run;
      wv[k] = a | (c << 16);
    }
#pragma unroll
    for (int k = 0; k < 4; k++) m4[k] = make_uint4(wv[4 * k], wv[4 * k + 1], wv[4 * k + 2], wv[4 * k + 3]);
  }
  __syncthreads();
}

// Pointer jumping over the batch (ptr[i] >= 0: byte b points at an earlier byte of the batch;
// val[i]: the byte when known), then the batch to HBM at o: bytes until o is 16-byte aligned, then
// 16-byte stores.
template <class L>
__device__ __forceinline__ void batch_jump_store(L& E, int32_t T, int16_t (&ptr)[kPer], uint8_t (&val)[kPer], uint8_t* o) {
  const int tid = threadIdx.x;
  __syncthreads();  // emap no longer read: it becomes the pointer array
  int16_t* P = reinterpret_cast<int16_t*>(E.emap);
#pragma unroll
  for (int i = 0; i < kPer; i++) {
    const int32_t b = i * kBlock + tid;
    if (b < T) {
      P[b] = ptr[i];
      E.out[b] = val[i];
    }
  }
  __syncthreads();
  for (;;) {
    // read half: a pointer to a resolved byte takes its value, otherwise jumps to its target's pointer
    int pending = 0;
#pragma unroll
    for (int i = 0; i < kPer; i++) {
      if (ptr[i] < 0) continue;
      const int16_t q = P[ptr[i]];
      if (q < 0) val[i] = E.out[ptr[i]];
      else pending = 1;
      ptr[i] = q;
    }
    const int more = __syncthreads_or(pending);
    // write half
#pragma unroll
    for (int i = 0; i < kPer; i++) {
      const int32_t b = i * kBlock + tid;
      if (b < T) {
        P[b] = ptr[i];
        E.out[b] = val[i];
      }
    }
    __syncthreads();
    if (!more) break;
  }
  // ---- the batch to HBM: bytes until dst is 16-byte aligned, then 16-byte stores
  {
    const int32_t head0 = int32_t((16 - (reinterpret_cast<uintptr_t>(o) & 15)) & 15);
    const int32_t head = head0 < T ? head0 : T;
    if (tid < head) o[tid] = E.out[tid];
    const int32_t units = (T - head) >> 4;
    for (int32_t u = tid; u < units; u += kBlock) {
      uint32_t w[4];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int32_t x = head + 16 * u + 4 * q;
        w[q] = uint32_t(E.out[x]) | (uint32_t(E.out[x + 1]) << 8) | (uint32_t(E.out[x + 2]) << 16) |
               (uint32_t(E.out[x + 3]) << 24);
      }
      *reinterpret_cast<uint4*>(o + head + 16 * u) = make_uint4(w[0], w[1], w[2], w[3]);
    }
    const int32_t done = head + units * 16;
    if (tid < T - done) o[done + tid] = E.out[done + tid];
  }
}

// Wave 0: the elements of one batch from block position p (the stage holds [a0, ...)), output
// starting at d.  Results in E (nE, bend, p_next, bad, bulk_*).
// Every position / count here is wave-uniform; readfirstlane makes that visible to the compiler so
// that the readlane chain steps take their lane index from an SGPR (a lane index it believes
// divergent turns each readlane into a loop over the wave).
__device__ __forceinline__ int32_t uni(int32_t x) { return __builtin_amdgcn_readfirstlane(x); }

__device__ __forceinline__ void snappy_parse(SnapLds& E, int32_t n_, int32_t p, int32_t a0_, int32_t d_, int32_t total_) {
  const int lane = threadIdx.x & 63;
  const int32_t n = uni(n_), a0 = uni(a0_), d = uni(d_), total = uni(total_);
  int32_t pos = uni(p), k = 0, T = 0, bulk_len = 0, bulk_src = 0;
  bool bad = false;
  for (;;) {
    pos = uni(pos);
    if (pos >= n || pos - a0 > kSnapStage - 64) break;  // done, or the stage is used up
    // ---- every lane: the element that would start at byte q
    const int32_t q = pos + lane;
    const int32_t o8 = int32_t(q - a0);
    // bytes q..q+4 from two aligned LDS dwords
    const uint32_t* in32 = reinterpret_cast<const uint32_t*>(E.in);
    const uint64_t w = ((uint64_t(in32[(o8 >> 2) + 1]) << 32) | in32[o8 >> 2]) >> (8 * (o8 & 3));
    const uint32_t tag = uint32_t(w & 0xff);
    int32_t hdr, off = 0;
    int64_t len;
    const bool lit = (tag & 3) == 0;
    if (lit) {
      const uint32_t x = tag >> 2;
      if (x < 60) {
        hdr = 1;
        len = int64_t(x) + 1;
      } else {
        const int kb = int(x) - 59;
        hdr = 1 + kb;
        len = int64_t((w >> 8) & (kb == 4 ? 0xffffffffull : ((1ull << (8 * kb)) - 1))) + 1;
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
      const uint64_t ov = (w >> 8) & 0xffffffffull;
      off = ov > 0x7fffffffull ? 0x7fffffff : int32_t(ov);  // beyond any output position: invalid
    }
    const bool hdr_ok = int64_t(q) + hdr <= n;
    const int64_t nx64 = int64_t(q) + hdr + (lit ? len : 0);
    const int32_t nxt = nx64 > n ? int32_t(n) + 1 : int32_t(nx64);  // past the input: invalid below
    // ---- the true chain from pos: pointer doubling over the window's lanes.  R = lanes on the path
    // from this lane within 2^k steps, J = the lane 2^k steps on (64: the path left the window).
    const bool here = q < n;
    uint64_t R = here ? 1ull << lane : 0;
    int32_t J = here ? (nxt - pos < 64 ? nxt - pos : 64) : 64;
#pragma unroll
    for (int r = 0; r < 6; r++) {
      const int32_t src_lane = J < 64 ? J : lane;
      const uint64_t Rn = __shfl(R, src_lane, 64);
      const int32_t Jn = __shfl(J, src_lane, 64);
      if (J < 64) {
        R |= Rn;
        J = Jn;
      }
    }
    const uint64_t chain = (uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(R >> 32)))) << 32) |
                           uint32_t(__builtin_amdgcn_readfirstlane(uint32_t(R)));  // lane 0's path
    const bool on = (chain >> lane) & 1;
    if (__ballot(on && !hdr_ok)) {  // an element header past the input
      bad = true;
      break;
    }
    const int32_t exitp = uni(__builtin_amdgcn_readlane(nxt, 63 - __builtin_clzll(chain)));
    const int idx = __popcll(chain & ((1ull << lane) - 1));
    // output positions: a 32-bit DPP scan unless some element is 16 MiB or longer
    int64_t excl;
    if (__ballot(on && len >= (1 << 24)) == 0) {
      const uint32_t x = on ? uint32_t(len) : 0u;
      excl = int64_t(wave_incl_scan32(x) - x);
    } else {
      excl = wave_excl_scan64(on ? len : 0);
    }
    const int64_t eo = int64_t(d) + T + excl;  // stream output position
    bool ebad = false;
    if (on) {
      if (lit) ebad = nx64 > n || eo + len > total;
      else ebad = off == 0 || off > eo || eo + len > total;
    }
    if (__ballot(ebad)) {
      bad = true;
      break;
    }
    // every chain element now lies inside the output: lengths and positions fit 32 bits
    const uint64_t fit = __ballot(on && T + excl + len <= kSnapOut && k + idx < kSnapMaxE);
    const int m = __popcll(fit);
    if (m == 0) {
      if (k == 0) {  // a literal longer than a batch (the window's first element, lane 0): bulk copy
        bulk_len = __builtin_amdgcn_readfirstlane(int32_t(len));
        bulk_src = pos + __builtin_amdgcn_readfirstlane(hdr);
        pos = __builtin_amdgcn_readfirstlane(nxt);
      }
      break;
    }
    if (on && idx < m) {
      E.eout[k + idx] = T + int32_t(excl);
      E.elen[k + idx] = int32_t(len);
      E.elit[k + idx] = lit;
      E.esrc[k + idx] = lit ? q + hdr : off;
    }
    const int last = uni(63 - __builtin_clzll(fit));  // lane of the last element taken
    T = uni(T + __builtin_amdgcn_readlane(int32_t(excl + len), last));
    k = uni(k + m);
    if (m < __popcll(chain)) {  // batch full: the next batch starts at the first element not taken
      const uint64_t rest = chain & ~fit;
      pos += __builtin_ctzll(rest);
      break;
    }
    pos = exitp;
  }
  if (lane == 0) {
    E.nE = k;
    E.bend = T;
    E.eout[k] = T;
    E.p_next = pos;
    E.bad = bad;
    E.bulk_len = bulk_len;
    E.bulk_src = bulk_src;
  }
}

// Decode one snappy block src[0, n) into dst[0, expected).  Whole workgroup; returns PQH_OK or
// PQH_ERR_DECOMPRESS (uniform).
__device__ int snappy_block(const uint8_t* src, int64_t n, uint8_t* dst, int64_t expected, SnapLds& E) {
  const int tid = threadIdx.x;
  // decodedLen: binary.Uvarint, at most 10 bytes; > 0xffffffff is ErrCorrupt
  uint64_t v = 0;
  int hl = 0;
  {
    bool done = false;
    for (int i = 0; i < 10 && i < n && !done; i++) {
      const uint8_t c = uint8_t(uni(src[i]));
      if (i == 9 && c > 1) return PQH_ERR_DECOMPRESS;  // overflows 64 bits
      v |= uint64_t(c & 0x7f) << (7 * i);
      hl = i + 1;
      done = c < 0x80;
    }
    if (!done || v > 0xffffffffull || int64_t(v) != expected) return PQH_ERR_DECOMPRESS;
  }
  const int32_t total = uni(int32_t(v));
  int32_t p = uni(hl), d = 0;
  const int32_t n32 = uni(int32_t(n));
  while (p < n32) {
    p = uni(p);
    d = uni(d);
    // ---- stage the compressed bytes from p (16-byte aligned start; the source payload is padded)
    const int32_t a0 = uni(p - int32_t((reinterpret_cast<uintptr_t>(src) + uintptr_t(p)) & 15));
    __syncthreads();  // the previous batch's readers of the stage are done
    {  // up to the block's end rounded to 16 bytes (inside the payload pad): bytes past it never
       // decide a valid element
      const uint4* sp = reinterpret_cast<const uint4*>(src + a0);
      uint4* lp = reinterpret_cast<uint4*>(E.in);
      const int64_t avail = (n - a0 + 15) >> 4;
      const int nu = avail < (kSnapStage + 96) / 16 ? int(avail) : (kSnapStage + 96) / 16;
      for (int u = tid; u < nu; u += kBlock) lp[u] = sp[u];
    }
    __syncthreads();
    if (tid < 64) snappy_parse(E, n32, p, a0, d, total);
    __syncthreads();
    if (uni(E.bad)) return PQH_ERR_DECOMPRESS;
    const int32_t nE = uni(E.nE), T = uni(E.bend);
    if (nE == 0) {
      const int32_t bl = uni(E.bulk_len);
      if (bl > 0) {
        snap_copy(dst + d, src + uni(E.bulk_src), bl);
        d += bl;
      }
      p = uni(E.p_next);
      __syncthreads();  // the bulk bytes are visible to the next batches' reads
      continue;
    }
#ifdef PQH_SNAPPY_PARSE_ONLY  // timing experiments: the element parse alone
    d += T;
    p = uni(E.p_next);
    continue;
#endif
    batch_emap(E, nE);
    // ---- the batch's bytes.  Each byte is either known at once (a literal byte: from the stage or
    // HBM; a copy byte whose source precedes the batch: read back from HBM) or points at an earlier
    // byte of the batch; pointer jumping then resolves every chain in O(log length) rounds.
    const int32_t s_lo = a0, s_hi = a0 + kSnapStage + 96;
    int16_t ptr[kPer];
    uint8_t val[kPer];
#pragma unroll
    for (int i0 = 0; i0 < kPer; i0 += 8) {
      int32_t ga[8];
      uint8_t from[8];  // 0 resolved / in-batch pointer, 1 dst (an earlier batch), 2 src (literal outside the stage)
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
        if (E.elit[e]) {
          const int32_t sp = E.esrc[e] + rel;
          if (sp >= s_lo && sp < s_hi) {
            val[i0 + j] = E.in[sp - s_lo];
          } else {
            from[j] = 2;
            ga[j] = sp;
          }
          continue;
        }
        const int32_t o = E.esrc[e];
        const int32_t sabs = d + E.eout[e] - o + (o < E.elen[e] ? rel % o : rel);  // overlapping copies repeat
        if (sabs >= d) {
          ptr[i0 + j] = int16_t(sabs - d);
        } else {
          from[j] = 1;
          ga[j] = sabs;
        }
      }
#pragma unroll
      for (int j = 0; j < 8; j++)  // the HBM reads of 8 bytes in flight together
        if (from[j]) val[i0 + j] = from[j] == 1 ? dst[ga[j]] : src[ga[j]];
    }
    batch_jump_store(E, T, ptr, val, dst + d);
    __syncthreads();  // this batch's bytes are visible to the next batches' reads
    d += T;
    p = uni(E.p_next);
  }
  return d == total ? PQH_OK : PQH_ERR_DECOMPRESS;
}

// One workgroup per page: its image rebuilt at image_offset from its source bytes (codec 0: copied;
// GZIP pages: k_gzip).
__global__ __launch_bounds__(256) void k_snappy(const pqh_codec_page* cps, const uint8_t* src_all, uint8_t* dst_all,
                                                int32_t* status, const int32_t* only) {
  __shared__ SnapLds E;
  if (only && !only[blockIdx.x]) return;  // (the multi-workgroup pipeline's page)
  const pqh_codec_page cp = cps[blockIdx.x];
  if (cp.codec == PQH_CODEC_GZIP) return;  // k_gzip's
  const uint8_t* src = src_all + cp.src_offset;
  uint8_t* dst = dst_all + cp.image_offset;
  int rc = PQH_OK;
  if (cp.codec != PQH_CODEC_SNAPPY) {
    snap_copy(dst, src, cp.src_len < cp.image_len ? cp.src_len : cp.image_len);
    if (cp.src_len != cp.image_len) rc = PQH_ERR_DECOMPRESS;
  } else {
    const int32_t raw = cp.raw_len < cp.src_len ? cp.raw_len : cp.src_len;
    snap_copy(dst, src, raw < cp.image_len ? raw : cp.image_len);  // DataPageV2 levels: never compressed
    if (raw > cp.image_len) rc = PQH_ERR_DECOMPRESS;
    else rc = snappy_block(src + raw, cp.src_len - raw, dst + raw, int64_t(cp.image_len) - raw, E);
  }
  if (threadIdx.x == 0) status[blockIdx.x] = rc;
}
