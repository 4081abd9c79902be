// bytearray_impl.h — BYTE_ARRAY values on the device (included by decode.hip).
//
// Output per chunk: int64 offsets[notNull + 1] + the concatenated bytes (Arrow-style) — what
// decodeValues fills into []interface{} of []byte (type_bytearray.go).  Three producers of
// per-value lengths feed one offsets/copy pipeline:
//   PLAIN       byteArrayPlainDecoder.next (type_bytearray.go:24-45): a [u32 len][bytes] chain,
//               resolved by one workgroup per page (k_ba_walk) -> lengths in aux + the first error;
//   DELTA_LEN   byteArrayDeltaLengthDecoder (type_bytearray.go:98-140): the lengths are a
//               DELTA_BINARY_PACKED stream decoded by the delta pipeline into aux (init decodes
//               all valuesCount lengths: delta_walk init_all); the string bytes follow the stream;
//   DICTIONARY  dictDecoder over a byte-array dictionary page (type_dict.go:40-60): the
//               dictionary page's PLAIN chain is walked into a cumulative-bytes table (dcum) and
//               the index stream is expanded into aux (keys, KeySink in decode.hip).
// Then per kBaTile tile: byte sums (k_ba_sum) -> per-chunk exclusive scan (k_ba_scan) -> block
// scan, offsets, byte copy (k_ba_expand).
#pragma once

// ------------------------------------------------------------------------------------------------
// PLAIN byte-array chains (data pages and byte-array dictionary pages).  The chain [u32 len][len
// bytes] (byteArrayPlainDecoder.next, type_bytearray.go:24-45) is sequential by definition; it is
// resolved in parallel and exactly, over many workgroups per page:
//   * a page's bytes are cut into windows: window w holds the records whose start lies in
//     [B_w, B_w+1), B_w = entry + w * kChainStride;
//   * k_ba_wspec (one workgroup per window): window w's entry (the first record start >= B_w) is
//     guessed (window 0: the known entry), then resolved inside the window: each thread owns a
//     124-byte segment and walks it from a speculative start (the shortest plausible record among
//     four neighbouring offsets), the walks are checked in parallel against their predecessor's
//     exit and the first mismatch re-walked from its true entry until all agree; the window's
//     records (lengths, or bytes before each record for dictionary pages), count, byte sum, exit and
//     first invalid record go to scratch;
//   * k_ba_wstitch (one workgroup per page): window w's entry must be window w-1's exit; a window
//     whose guess was wrong is resolved again from the true entry (rare); window bases = running
//     record / byte counts; the page's error (the first invalid record on the chain before `count`
//     records) and limits;
//   * k_ba_wemit (one workgroup per window): the window's records copied out at its base: lengths
//     (data page -> aux) or cumulative offsets (dictionary page -> dcum).
// ------------------------------------------------------------------------------------------------
// 124-byte segments: neighbouring lanes' segments start 31 dwords apart, so their LDS reads fall in
// different banks (a power-of-two stride would put a whole wave on one bank)

struct ChainLds {
  uint32_t win[(kChainWin + 64) / 4];
  // segment j's record-start marks as 32-bit words, word-major (mask[k][j]): the 64 lanes of a wave
  // touch 64 consecutive dwords, one per bank, on every mark / clear / read (a [j][k] layout of 64-bit
  // words put lanes j, j + 16, j + 32, j + 48 in one bank: 4-way conflicts on each record's mark)
  uint32_t mask[2 * kChainWords][kBlock];
  int32_t exitv[kBlock];
  uint8_t exitbad[kBlock];
  int32_t first_bad;
  int32_t stop;
  int32_t guess;
  int32_t pad;
  uint64_t wsum[4];
};

__device__ __forceinline__ uint64_t seg_mask(const ChainLds& C, int j, int k) {
  return uint64_t(C.mask[2 * k][j]) | (uint64_t(C.mask[2 * k + 1][j]) << 32);
}

__device__ __forceinline__ void seg_clear(ChainLds& C, int j) {
#pragma unroll
  for (int k = 0; k < 2 * kChainWords; k++) C.mask[k][j] = 0;
}

// Workgroup sum (every thread gets it).
__device__ __forceinline__ int64_t block_sum64(int64_t x, int64_t* wsum) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
  __syncthreads();
  if (lane == 0) wsum[wv] = x;
  __syncthreads();
  return wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

// Every position below is a byte offset in the page image (32 bits: pages are < 2 GiB); wb is the
// window's stage base, e0 the end of the page's value bytes.
// One record at page offset p: 0 and the next offset, or the error code.
__device__ __forceinline__ int chain_step(const ChainLds& C, int32_t wb, int32_t e0, int32_t p, int32_t& next,
                                          int32_t& len) {
  const int32_t avail = e0 - p;
  if (avail < 4) return avail <= 0 ? PQH_ERR_EOF : PQH_ERR_UNEXPECTED_EOF;  // binary.Read(u32)
  const int32_t o = p - wb;
  const uint32_t w0 = C.win[o >> 2], w1 = C.win[(o >> 2) + 1];
  len = int32_t(__builtin_amdgcn_alignbit(w1, w0, uint32_t(o & 3) * 8));
  if (len < 0) return PQH_ERR_NEGATIVE_LENGTH;
  if (len > 0 && avail - 4 < len) return avail - 4 <= 0 ? PQH_ERR_EOF : PQH_ERR_UNEXPECTED_EOF;  // ReadFull
  next = p + 4 + len;
  return PQH_OK;
}

// chain_step's validity test without its error codes (branch-free: the walks' inner loops):
// avail >= 4 and 0 <= len <= avail - 4  <=>  avail >= 4 and unsigned(len) <= unsigned(avail - 4).
__device__ __forceinline__ bool chain_ok(const ChainLds& C, int32_t wb, int32_t e0, int32_t p, int32_t& next,
                                         int32_t& len) {
  const int32_t avail = e0 - p;
  const int32_t o = p - wb;
  const uint32_t w0 = C.win[o >> 2], w1 = C.win[(o >> 2) + 1];
  len = int32_t(__builtin_amdgcn_alignbit(w1, w0, uint32_t(o & 3) * 8));
  next = p + 4 + len;
  return (avail >= 4) & (uint32_t(len) <= uint32_t(avail - 4));  // (bitwise: no branch)
}

__device__ __forceinline__ int32_t seg_end(int j, int32_t wb, int32_t wend) {
  const int32_t s1 = wb + (j + 1) * kChainSeg;
  return s1 < wend ? s1 : wend;
}

// Walk segment j [s0, s1) from `start` (must lie in the segment): marks + exit.  The marks go
// straight to the segment's LDS words by one fire-and-forget OR per record (the thread's own words);
// the error code of the record that stops the walk is taken once, after the loop.
__device__ void chain_walk(ChainLds& C, int j, int32_t wb, int32_t wend, int32_t e0, int32_t start) {
  const int32_t s0 = wb + j * kChainSeg, s1 = seg_end(j, wb, wend);
  seg_clear(C, j);
  int32_t p = start;
  bool stop = false;
  while (p < s1) {
    int32_t nx, l;
    if (!chain_ok(C, wb, e0, p, nx, l)) {
      stop = true;
      break;
    }
    const int q = p - s0;
    atomicOr(&C.mask[q >> 5][j], 1u << (q & 31));
    p = nx;
  }
  uint8_t bad = 0;
  if (stop) {
    int32_t nx, l;
    bad = uint8_t(chain_step(C, wb, e0, p, nx, l));
  }
  C.exitv[j] = p;
  C.exitbad[j] = bad;
}

__device__ __forceinline__ bool chain_has(const ChainLds& C, int j, int q) {
  return (C.mask[q >> 5][j] >> (q & 31)) & 1;
}

// Is segment j's stored result right for its true entry (the previous segment's exit)?  By
// induction from segment 0 (whose start is the window entry), when every segment passes, all
// segments up to the first invalid exit are exact and that exit is the true end of the chain.
__device__ __forceinline__ bool chain_good(const ChainLds& C, int j, int32_t wb, int32_t wend, int32_t entry) {
  const int32_t s0 = wb + j * kChainSeg, s1 = seg_end(j, wb, wend);
  int32_t T = entry;
  uint8_t pbad = 0;
  if (j > 0) {
    T = C.exitv[j - 1];
    pbad = C.exitbad[j - 1];
  }
  bool empty = true;
#pragma unroll
  for (int k = 0; k < 2 * kChainWords; k++) empty = empty && C.mask[k][j] == 0;
  if (pbad) return true;  // the chain ended before j (exactly, if j-1 is right): nothing here counts
  if (T >= s1) return empty && !C.exitbad[j] && C.exitv[j] == T;  // skipped by a long record
  if (empty && C.exitbad[j] && C.exitv[j] == T) return true;       // the record at T itself is invalid
  return chain_has(C, j, T - s0);
}

// Make segment j right for the entry T (pbad: the chain already ended before it).
__device__ void chain_fix(ChainLds& C, int j, int32_t wb, int32_t wend, int32_t e0, int32_t T, uint8_t pbad) {
  const int32_t s0 = wb + j * kChainSeg;
  if (pbad || T >= seg_end(j, wb, wend)) {
    seg_clear(C, j);
    C.exitv[j] = T;
    C.exitbad[j] = pbad;
  } else if (!chain_has(C, j, T - s0)) {
    chain_walk(C, j, wb, wend, e0, T);
  }
}

// The record starts <= 3 bytes apart at x..x+3 that look like records (valid, and followed inside
// the window by another valid one): the shortest wins.  The last byte of a string followed by a
// small length field reads as a record ~256x longer than the true one a byte later.
__device__ __forceinline__ int32_t chain_guess(const ChainLds& C, int32_t wb, int32_t e0, int32_t s0, int32_t s1,
                                               int32_t staged_end) {
  auto plausible = [&](int32_t x, int32_t& l) {
    int32_t nx, nx2, l2;
    if (!chain_ok(C, wb, e0, x, nx, l)) return false;
    return nx + 4 <= staged_end && (nx >= e0 || chain_ok(C, wb, e0, nx, nx2, l2));
  };
  // scan 16 positions per step from 5 dwords loaded together (independent LDS reads; the length at
  // each byte offset is a funnel shift of two of them): a mask of the positions whose own record is
  // valid, then the full test on those in order
  const int32_t lim = s1 < e0 ? s1 : e0;
  int32_t x = -1;
  for (int32_t base = wb + ((s0 - wb) & ~3); base < lim && x < 0; base += 16) {
    const int k = (base - wb) >> 2;
    uint32_t w[5];
#pragma unroll
    for (int i = 0; i < 5; i++) w[i] = C.win[k + i];
    const int32_t rel = e0 - base;  // bytes left at base
    const int32_t lo = s0 > base ? s0 - base : 0, hi = lim - base < 16 ? lim - base : 16;
    uint32_t cand = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) {  // chain_ok's test, one compare per position (a position with
                                    // fewer than 4 bytes left is masked below)
      const uint32_t len = __builtin_amdgcn_alignbit(w[(i >> 2) + 1], w[i >> 2], uint32_t(i & 3) * 8);
      cand |= uint32_t(len <= uint32_t(rel - i - 4)) << i;
    }
    const int32_t n4 = rel - 3;  // positions i < n4 have 4 bytes or more left
    const uint32_t m4 = n4 >= 16 ? 0xffffu : (n4 <= 0 ? 0u : (1u << n4) - 1);
    cand &= m4 & ((1u << hi) - 1) & ~((1u << lo) - 1);  // (0 <= lo < hi <= 16)
    for (; cand; cand &= cand - 1) {
      int32_t l;
      const int32_t p = base + __builtin_ctz(cand);
      if (plausible(p, l)) {
        x = p;
        break;
      }
    }
  }
  if (x >= 0) {
    int32_t l;
    plausible(x, l);
    int32_t start = x;
    // only a long record can be the false start (a string's last byte + a small length field)
    for (int d = 1; d <= 3 && x + d < s1 && l >= 256; d++) {
      int32_t l2;
      if (plausible(x + d, l2) && l2 < l) {
        start = x + d;
        l = l2;
      }
    }
    return start;
  }
  return -1;
}

// Resolve the chain of the window [wb, wend) from `entry` (whole workgroup; C.win staged from wb).
// Afterwards segment j's marks hold the true record starts in it, C.first_bad = the first segment
// whose walk ended on an invalid record (kBlock if none).
__device__ void chain_resolve(ChainLds& C, int32_t wb, int32_t wend, int32_t e0, int32_t entry) {
  const int j = threadIdx.x;
  {
    const int32_t s0 = wb + j * kChainSeg, s1 = seg_end(j, wb, wend);
    int32_t start = -1;
    if (s0 <= entry) start = entry;  // the segment holding the entry (segments before it stay empty)
    else if (s0 < s1) start = chain_guess(C, wb, e0, s0, s1, wb + kChainWin);
    if (s1 <= entry) {
      seg_clear(C, j);
      C.exitv[j] = entry;
      C.exitbad[j] = 0;
    } else if (start >= 0) {
      chain_walk(C, j, wb, wend, e0, start);
    } else if (s0 >= e0 && s0 < s1) {
      // past the end of the bytes: what a walk from s0 gives (EOF at s0), so that the segments after
      // the chain's end agree at once instead of being fixed one per round
      seg_clear(C, j);
      C.exitv[j] = s0;
      C.exitbad[j] = uint8_t(PQH_ERR_EOF);
    } else {
      seg_clear(C, j);
      C.exitv[j] = s1 > s0 ? s1 : s0;
      C.exitbad[j] = 0;
    }
  }
  __syncthreads();
  // the first segment whose walk misses its true entry has an exact predecessor: re-walk it; repeat
  for (;;) {
    if (j == 0) C.stop = kBlock;
    __syncthreads();
    if (!chain_good(C, j, wb, wend, entry)) atomicMin(&C.stop, j);
    __syncthreads();
    const int sg = C.stop;
    if (sg >= kBlock) break;
    if (j == sg) chain_fix(C, sg, wb, wend, e0, sg == 0 ? entry : C.exitv[sg - 1], sg == 0 ? 0 : C.exitbad[sg - 1]);
    __syncthreads();
  }
  if (j == 0) C.first_bad = kBlock;
  __syncthreads();
  if (C.exitbad[j]) atomicMin(&C.first_bad, j);  // segments before the chain's end are exact
  __syncthreads();
}

// Segment j's marks on the true chain (starts before its true entry dropped; none past the end).
__device__ __forceinline__ int chain_marks(const ChainLds& C, int j, int32_t wb, int32_t entry, int fb,
                                           uint64_t m[kChainWords]) {
  const int32_t s0 = wb + j * kChainSeg;
  const int32_t T = j == 0 ? entry : C.exitv[j - 1];
  const bool live = j <= fb;
  int cnt = 0;
#pragma unroll
  for (int k = 0; k < kChainWords; k++) {
    m[k] = live ? seg_mask(C, j, k) : 0;
    const int32_t lo = T - s0 - 64 * k;
    if (lo > 0) m[k] = lo >= 64 ? 0 : m[k] & ~((1ull << lo) - 1);
    cnt += __popcll(m[k]);
  }
  return cnt;
}

struct BaPageCtx {
  bool ok, dict;
  int64_t count, entry, e0;
  const uint8_t* img;
};

__device__ __forceinline__ BaPageCtx ba_page_ctx(const DevBatch& b, int p) {
  BaPageCtx c;
  const DevPage P = b.pages[p];
  const PageState S = b.states[p];
  c.dict = P.page_type == PQH_DICTIONARY_PAGE;
  c.ok = !(S.err != kNoError && (c.dict || page_failed_before_values(S)));
  c.count = c.dict ? P.num_values : S.nn;
  c.entry = c.dict ? 0 : S.val_s;
  c.e0 = c.dict ? P.image_len : S.val_e;
  c.img = b.payload + P.image_off;
  return c;
}

// Window w is staged from B_w = entry + w * kChainStride rounded down to 16 bytes: its records start
// in [entry_w, B_w+1) with entry_w >= B_w, so [wb, B_w+1) spans at most kChainWin bytes whatever the
// true entry turns out to be.
__device__ __forceinline__ int64_t ba_wbase(const BaPageCtx& c, int64_t w) {
  const int64_t Bw = c.entry + w * kChainStride;
  return Bw - int64_t((reinterpret_cast<uintptr_t>(c.img) + uintptr_t(Bw)) & 15);
}

// The whole window in one round trip: every thread's vectors loaded together, then stored.
__device__ __forceinline__ void ba_stage(ChainLds& C, const BaPageCtx& c, int64_t wb) {
  constexpr int kNv = (kChainWin + 64) / 16, kPer = (kNv + kBlock - 1) / kBlock;
  const PQH_G uint8_t* src = (const PQH_G uint8_t*)(c.img + wb);
  const int64_t limit = c.e0 - wb;
  uint4 x[kPer];
#pragma unroll
  for (int j = 0; j < kPer; j++) {
    const int k = int(threadIdx.x) + j * kBlock;
    const bool ok = k < kNv && 16 * int64_t(k) < limit;
    x[j] = *reinterpret_cast<const PQH_G uint4*>(src + (ok ? 16 * k : 0));
    if (!ok) x[j] = make_uint4(0, 0, 0, 0);
  }
#pragma unroll
  for (int j = 0; j < kPer; j++) {
    const int k = int(threadIdx.x) + j * kBlock;
    if (k < kNv) reinterpret_cast<uint4*>(C.win)[k] = x[j];
  }
}

// Segment j's records on the true chain after a window's resolution (per thread, in registers):
// their start marks, their count, the index of the first one in the window, and the bytes of the
// window's records before it.
struct SegRecs {
  uint64_t m[kChainWords];
  int32_t cnt, li, lb;
};

// Resolve and summarise one window (whole workgroup; C.win staged from ba_wbase(c, w)): *res (thread
// 0) and every segment's records (sr).
__device__ void ba_window_segs(ChainLds& C, const BaPageCtx& c, int64_t w, int64_t entry64, BaWin* res,
                               SegRecs& sr) {
  const int j = threadIdx.x;
  const int64_t wend64 = c.entry + (w + 1) * kChainStride;
  BaWin r{int32_t(entry64), int32_t(entry64), 0, 0, 0, -1, 0, 0};
#pragma unroll
  for (int k = 0; k < kChainWords; k++) sr.m[k] = 0;
  sr.cnt = sr.li = sr.lb = 0;
  if (entry64 >= c.e0 || entry64 >= wend64) {  // no record starts in the window (or no bytes left)
    if (entry64 >= c.e0 && entry64 < wend64) r.bad = PQH_ERR_EOF;
    if (j == 0) *res = r;
    return;
  }
  const int32_t wb = int32_t(ba_wbase(c, w)), wend = int32_t(wend64), entry = int32_t(entry64);
  chain_resolve(C, wb, wend, int32_t(c.e0), entry);
  const int fb = C.first_bad;
  const int cnt = chain_marks(C, j, wb, entry, fb, sr.m);
  // The segment's records are consecutive on the chain, so their lengths need no LDS reads: record
  // r's length is the next record's start - r's start - 4, and the last one ends at the segment's
  // exit (the start of the next record, or of the invalid record that ended the chain).
  const int32_t s0 = wb + j * kChainSeg, exj = C.exitv[j];
  int32_t first = -1;
#pragma unroll
  for (int k = kChainWords - 1; k >= 0; k--)
    if (sr.m[k]) first = 64 * k + __builtin_ctzll(sr.m[k]);
  const int32_t bytes = cnt > 0 ? exj - (s0 + first) - 4 * cnt : 0;
  // records and bytes of the window both fit 32 bits: one scan of the pair
  uint64_t tot;
  const uint64_t ex = block_exclusive_scan((uint64_t(uint32_t(cnt)) << 32) | uint32_t(bytes), C.wsum, &tot);
  sr.cnt = cnt;
  sr.li = int32_t(ex >> 32);
  sr.lb = int32_t(uint32_t(ex));
  if (j == 0) {
    const int32_t nrec = int32_t(tot >> 32), btot = int32_t(uint32_t(tot));
    r.count = nrec;
    r.bytes = btot;
    if (fb < kBlock) {
      r.bad = C.exitbad[fb];
      r.exit = C.exitv[fb];
    } else {
      // the last segment's exit: the first record start >= wend
      r.exit = C.exitv[(wend - wb + kChainSeg - 1) / kChainSeg - 1];
    }
    *res = r;
  }
}

// The segment's records with window indices in [lo, hi) as their exclusive byte offsets within the
// window: list[i - lo] for record i.
template <class T>
__device__ __forceinline__ void seg_list(const SegRecs& sr, int32_t lo, int32_t hi, T* list) {
  if (sr.li >= hi || sr.li + sr.cnt <= lo) return;
  int32_t li = sr.li, lb = sr.lb, prev = -1;
#pragma unroll
  for (int k = 0; k < kChainWords; k++)
    for (uint64_t x = sr.m[k]; x; x &= x - 1) {
      const int32_t pos = 64 * k + __builtin_ctzll(x);
      if (prev >= 0) lb += pos - prev - 4;
      if (li >= hi) return;
      if (li >= lo) list[li - lo] = uint16_t(lb);
      li++;
      prev = pos;
    }
}

// Resolve and summarise one window into the scratch: the records go to wrec in order as the bytes
// of the records before each one within the window (16 bits: a record starts inside the window, so
// fewer than kChainWin bytes precede it); the window's total is res->bytes: record i's length is
// wrec[i + 1] - wrec[i], the last one's bytes - wrec[count - 1].
__device__ void ba_window(ChainLds& C, const BaPageCtx& c, int64_t w, int64_t entry64, BaWin* res, uint16_t* wrec) {
  SegRecs sr;
  ba_window_segs(C, c, w, entry64, res, sr);
  if (sr.cnt == 0 && threadIdx.x == 0) {
    const int64_t wend64 = c.entry + (w + 1) * kChainStride;
    if (entry64 >= c.e0 || entry64 >= wend64) wrec[0] = 0;
  }
  seg_list(sr, 0, 0x7fffffff, wrec);
}

// Window w > 0 guesses its entry (the first record start >= B_w) from the staged window itself:
// wave 0 tests 64 positions per step for a plausible record (valid, followed by a valid one) and
// takes the shortest of the first one and its next three positions (the last byte of a string
// followed by a small length field reads as a record ~256x longer than the true one a byte later).
// A wrong guess costs k_ba_wstitch a re-resolution, never a wrong result.
__device__ __forceinline__ int32_t ba_guess_entry(const ChainLds& C, int32_t e0, int32_t wb, int32_t Bw) {
  const int lane = threadIdx.x & 63;
  const int32_t staged_end = wb + kChainWin;
  for (int32_t x0 = Bw; x0 < Bw + 1024 && x0 < e0; x0 += 64) {
    const int32_t x = x0 + lane;
    int32_t nx, nx2, l = 0, l2;
    bool ok = x < e0 && chain_ok(C, wb, e0, x, nx, l) && nx + 4 <= staged_end &&
              (nx >= e0 || chain_ok(C, wb, e0, nx, nx2, l2));
    const uint64_t m = __ballot(ok);
    if (m == 0) continue;
    const int f = __builtin_ctzll(m);
    int best = f;
    int32_t bl = __shfl(l, f, 64);
    for (int d = 1; d <= 3 && f + d < 64; d++) {
      const int32_t ld = __shfl(l, f + d, 64);
      if (((m >> (f + d)) & 1) && ld < bl) {
        best = f + d;
        bl = ld;
      }
    }
    return x0 + best;
  }
  return Bw;
}

__global__ __launch_bounds__(256) void k_ba_wspec(DevBatch b, const int2* wins, BaWin* res, uint16_t* wrec) {
  __shared__ ChainLds C;
  const int2 pw = wins[blockIdx.x];
  const BaPageCtx c = ba_page_ctx(b, pw.x);
  BaWin* r = res + blockIdx.x;
  uint16_t* mk = wrec + int64_t(blockIdx.x) * kChainRecs;
  const int64_t Bw = c.entry + int64_t(pw.y) * kChainStride;
  if (!c.ok || Bw >= c.e0) {
    if (threadIdx.x == 0) *r = BaWin{-1, -1, 0, 0, 0, -1, 0, 0};
    return;
  }
  const int64_t wb = ba_wbase(c, pw.y);
  ba_stage(C, c, wb);
  __syncthreads();
  int64_t entry = c.entry;
  if (pw.y > 0) {
    if (threadIdx.x < 64) {
      const int32_t g = ba_guess_entry(C, int32_t(c.e0), int32_t(wb), int32_t(Bw));
      if (threadIdx.x == 0) C.guess = int32_t(g);
    }
    __syncthreads();
    entry = C.guess;
  }
  ba_window(C, c, pw.y, entry, r, mk);
}
// Wave-wide exclusive prefix sum (64-bit).
__device__ __forceinline__ int64_t wave_excl_scan64(int64_t x) {
  const int lane = threadIdx.x & 63;
  int64_t v = x;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int64_t y = __shfl_up(v, off, 64);
    if (lane >= off) v += y;
  }
  return v - x;
}

// One workgroup per PLAIN byte-array page: windows stitched in order (see above).  Wave 0 takes 64
// windows per step: a window whose guessed entry is its predecessor's exit (and before which the
// chain neither ran out of bytes nor reached `count`) gets its bases from two wave scans; the first
// other window (a wrong guess, an invalid record, or the end) is handled one at a time by the
// workgroup exactly as the chain defines it.
__global__ __launch_bounds__(256) void k_ba_wstitch(DevBatch b, const int32_t* ba_pages, const int2* pwin, BaWin* res,
                                                     uint16_t* wrec) {
  __shared__ ChainLds C;
  __shared__ BaWin cur;
  __shared__ int64_t sh[6];  // done, cum, last_base, last_cbase, T, (w | last << 32 | stop << 63)
  const int p = ba_pages[blockIdx.x];
  const int2 wr = pwin[blockIdx.x];
  const BaPageCtx c = ba_page_ctx(b, p);
  if (!c.ok) return;
  int64_t done = 0, cum = 0, T = c.entry;
  int64_t last_base = 0, last_cbase = 0;  // the last window taken: records and bytes before it
  int code = PQH_OK;
  int w = 0, last = -1;
  for (;;) {
    if (threadIdx.x < 64) {  // fast path over the windows whose guesses were right
      const int lane = threadIdx.x;
      bool stop = false;
      for (;;) {
        const int idx = w + lane;
        BaWin x{-1, -1, 0, 0, 0, 0, 0, 0};
        if (idx < wr.y) x = res[wr.x + idx];
        const int64_t ec = done + wave_excl_scan64(x.count), eb = cum + wave_excl_scan64(x.bytes);
        const int32_t pexit = __shfl_up(x.exit, 1, 64);
        const int64_t Tl = lane == 0 ? T : pexit;
        const bool before = idx >= wr.y || ec >= c.count || Tl >= c.e0;  // the loop ends before it
        const uint64_t ev = __ballot(before || x.entry != Tl || x.bad);
        const int f = ev ? __builtin_ctzll(ev) : 64;
        if (lane < f) {
          res[wr.x + idx].base = ec;
          res[wr.x + idx].cbase = eb;
        }
        if (f > 0) {
          last = w + f - 1;
          last_base = __shfl(ec, f - 1, 64);
          last_cbase = __shfl(eb, f - 1, 64);
          done = last_base + __shfl(x.count, f - 1, 64);
          cum = last_cbase + __shfl(x.bytes, f - 1, 64);
          T = __shfl(x.exit, f - 1, 64);
          w += f;
        }
        if (f < 64) {
          stop = __shfl(int(before), f, 64) != 0;
          break;
        }
      }
      if (lane == 0) {
        sh[0] = done;
        sh[1] = cum;
        sh[2] = last_base;
        sh[3] = last_cbase;
        sh[4] = T;
        sh[5] = int64_t(uint32_t(w)) | (int64_t(uint32_t(last + 1)) << 32) | (int64_t(stop) << 62);
      }
    }
    __syncthreads();
    done = sh[0];
    cum = sh[1];
    last_base = sh[2];
    last_cbase = sh[3];
    T = sh[4];
    w = int(uint32_t(sh[5]));
    last = int((sh[5] >> 32) & 0x3fffffff) - 1;
    const bool stop = (sh[5] >> 62) & 1;
    __syncthreads();
    if (stop || w >= wr.y || done >= c.count) {
      if (w < wr.y && done < c.count && T >= c.e0) code = PQH_ERR_EOF;  // no bytes left for the next length
      break;
    }
    // window w: a wrong guess (resolved again from the true entry) or an invalid record
    BaWin* r = res + wr.x + w;
    if (threadIdx.x == 0) cur = *r;
    __syncthreads();
    if (cur.entry != T) {  // the window's guess was not its true entry: resolve it again
      if (T < c.entry + (w + 1) * kChainStride) {  // some record starts in it: stage it
        ba_stage(C, c, ba_wbase(c, w));
        __syncthreads();
      }
      ba_window(C, c, w, T, r, wrec + int64_t(wr.x + w) * kChainRecs);
      __syncthreads();
      if (threadIdx.x == 0) cur = *r;
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      r->base = done;
      r->cbase = cum;
    }
    last = w;
    last_base = done;
    last_cbase = cum;
    done += cur.count;
    cum += cur.bytes;
    if (cur.bad) {
      code = cur.bad;
      w++;
      break;
    }
    T = cur.exit;
    w++;
    __syncthreads();  // cur is read again by the next window
  }
  if (!c.dict) {
    // the page's bytes before its value limit (min(count, records on the chain)) go to tile 0 of its
    // byte sums, the other tiles get 0: k_ba_scan turns them into the page's byte_base, and
    // k_ba_wcopy places every window at byte_base + cbase
    int64_t total = cum;
    if (done > c.count && last >= 0) {  // the last window holds records past `count`
      total = last_cbase + wrec[int64_t(wr.x + last) * kChainRecs + (c.count - last_base)];
    }
    const DevPage P = b.pages[p];
    for (int k = threadIdx.x; k < P.batile_n; k += kBlock) b.basums[P.batile_base + k] = k == 0 ? total : 0;
  }
  if (threadIdx.x == 0) {
    for (; w < wr.y; w++) res[wr.x + w].base = -1;  // windows past the chain's end or `count`
    int32_t* out = c.dict ? b.dcum + b.pages[p].aux_base : nullptr;
    if (done >= c.count) {  // all values read (records past `count` are never looked at)
      if (c.dict) {
        if (c.count == 0) out[0] = 0;
        b.states[p].dict_n = int32_t(c.count);
      } else {
        b.states[p].val_limit = int32_t(c.count);
      }
    } else if (c.dict) {
      atomicMin(&b.states[p].err, (unsigned long long)err_key(0, done, code));
    } else {
      b.states[p].val_limit = int32_t(done);
      atomicMin(&b.states[p].err, (unsigned long long)err_key(3, done, code));
    }
    if (!c.dict) b.states[p].ba_summed = 1;
  }
}

// Dictionary pages, one workgroup per window (list: {window, page}): the window's records as
// cumulative offsets (dcum) at its base.  Data-page windows go to k_ba_wcopy.
__global__ __launch_bounds__(256) void k_ba_wemit(DevBatch b, const int2* list, const BaWin* res,
                                                   const uint16_t* wrec) {
  const int2 wl = list[blockIdx.x];
  const BaWin r = res[wl.x];
  if (r.base < 0 || r.entry < 0) return;
  const int p = wl.y;
  const BaPageCtx c = ba_page_ctx(b, p);
  if (!c.ok || !c.dict) return;
  const uint16_t* src = wrec + int64_t(wl.x) * kChainRecs;
  PQH_G int32_t* out = (PQH_G int32_t*)(b.dcum + b.pages[p].aux_base);
  for (int32_t i = threadIdx.x; i < r.count; i += kBlock) {
    const int64_t idx = r.base + i;
    if (idx >= c.count) break;
    out[idx] = int32_t(r.cbase + src[i]);
    if (idx == c.count - 1) out[c.count] = int32_t(r.cbase + (i + 1 < r.count ? int32_t(src[i + 1]) : r.bytes));
  }
}

// Values of a byte-array data page that decode before the first error known so far.
__device__ __forceinline__ int64_t ba_limit(const DevBatch& b, int page, const DevPage& P, const PageState& S) {
  int64_t lim = S.val_limit;
  if (S.err != kNoError && (S.err >> 56) == 3) {
    const int64_t ei = int64_t((S.err >> 8) & 0xffffffffffffull);
    if (ei < lim) lim = ei;
  }
  if (P.kind == K_DLBA || P.kind == K_DBA) {  // valuesCount of the (suffix) lengths stream
    const int64_t dl = b.dstates[P.kind == K_DBA ? b.num_pages + page : page].limit;
    if (dl < lim) lim = dl;
  }
  return lim;
}

// DELTA_BYTE_ARRAY value i: prefix length (clamped at 0: a negative one adds nothing, and a
// negative total panics, both checked in k_ba_expand) + suffix length.
__device__ __forceinline__ int64_t dba_len(const int32_t* plen, const int32_t* slen, int64_t i) {
  const int32_t p = plen[i];
  return int64_t(p > 0 ? p : 0) + slen[i];
}

// Byte-array dictionary of a page: entry count and cumulative-bytes table (nullptr if failed).
struct BaDict {
  const int32_t* dcum;
  int64_t base;  // payload offset of the dictionary page image
  uint32_t K;
};

__device__ __forceinline__ BaDict ba_dict(const DevBatch& b, const DevPage& P) {
  BaDict d{nullptr, 0, 0};
  if (P.dict_page >= 0) {
    const PageState DS = b.states[P.dict_page];
    if (DS.err == kNoError) {
      const DevPage DP = b.pages[P.dict_page];
      d.dcum = b.dcum + DP.aux_base;
      d.base = DP.image_off;
      d.K = uint32_t(DS.dict_n);
    }
  }
  return d;
}

// Length of value i (aux holds a length, or a dictionary key).
__device__ __forceinline__ int64_t ba_len(const BaDict& d, bool is_dict, int32_t a) {
  if (!is_dict) return a;
  const uint32_t k = uint32_t(a);
  return k < d.K ? int64_t(d.dcum[k + 1]) - d.dcum[k] : 0;
}

// ------------------------------------------------------------------------------------------------
// k_ba_sum: bytes of each kBaTile tile; first negative DELTA_LENGTH length; EOF past valuesCount.
// ------------------------------------------------------------------------------------------------
// Tile k of byte-array page `page`.
__device__ void ba_tile_sum(const DevBatch& b, int page, int32_t k, int64_t* wsum) {
  const DevPage P = b.pages[page];
  const PageState S = b.states[page];
  int64_t s = 0;
  if (!page_failed_before_values(S)) {
    const DevChunk C = b.chunks[P.chunk];
    const int64_t lim = ba_limit(b, page, P, S);
    const int64_t v0 = int64_t(k) * kBaTile;
    const int64_t v1 = v0 + kBaTile < lim ? v0 + kBaTile : lim;
    if (P.value_size > 0) {  // fixed-width page of a FIXED_LEN_BYTE_ARRAY chunk laid out as byte arrays
      if (threadIdx.x == 0) {
        b.basums[P.batile_base + k] = v1 > v0 ? (v1 - v0) * P.value_size : 0;
        b.basums2[P.batile_base + k] = 0;
      }
      return;
    }
    const bool is_dict = P.kind == K_DICT;
    const BaDict d = is_dict ? ba_dict(b, P) : BaDict{nullptr, 0, 0};
    const int32_t* aux = C.aux + S.value_base;
    const bool dba = P.kind == K_DBA;
    const int32_t* aux2 = dba ? C.aux2 + S.value_base : nullptr;
    int64_t first_neg = INT64_MAX, s2 = 0;
    for (int64_t i = v0 + threadIdx.x; i < v1; i += kBlock) {
      const int64_t l = ba_len(d, is_dict, aux[i]);  // DELTA_BYTE_ARRAY: the suffix length
      if (l < 0) {
        if (i < first_neg) first_neg = i;
      } else {
        s += dba ? dba_len(aux2, aux, i) : l;
        s2 += l;
      }
    }
    s2 = block_sum64(dba ? s2 : 0, wsum);
    if (threadIdx.x == 0) b.basums2[P.batile_base + k] = s2;
    if (P.kind == K_DLBA || dba) {
      if (first_neg != INT64_MAX)  // make([]byte, negative) panics (re-panicked, file_reader.go:179-181)
        atomicMin(&b.states[page].err, (unsigned long long)err_key(3, first_neg, PQH_ERR_NEGATIVE_DLBA_LENGTH));
      const int64_t vc = b.dstates[dba ? b.num_pages + page : page].limit;
      if (k == 0 && threadIdx.x == 0 && S.nn > vc)  // lens exhausted: io.EOF (type_bytearray.go:118-121)
        atomicMin(&b.states[page].err, (unsigned long long)err_key(3, vc, PQH_ERR_EOF));
    }
  }
  s = block_sum64(s, wsum);
  if (threadIdx.x == 0) b.basums[P.batile_base + k] = s;
}

// ------------------------------------------------------------------------------------------------
// k_ba_sum: bytes of each kBaTile tile; first negative DELTA_LENGTH length; EOF past valuesCount.
// A PLAIN page, and in page mode (dlba_pages) a DELTA_LENGTH page, is listed once (tile 0): its sums
// (and negative-length checks) were accumulated by k_ba_wemit / k_delta_fused + k_delta_page unless
// the page left that path (ba_summed == 0), in which case this workgroup sums every tile of it.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_ba_sum(DevBatch b, const Tile* tiles, const int32_t* list, int dlba_pages) {
  __shared__ int64_t wsum[4];
  const Tile t = tiles[list[blockIdx.x]];
  const DevPage P = b.pages[t.page];
  if (b.states[t.page].ba_summed) {
    const PageState S = b.states[t.page];
    if (P.kind == K_DLBA) {
      const int64_t vc = b.dstates[t.page].limit;
      if (t.k == 0 && threadIdx.x == 0 && !page_failed_before_values(S) && S.nn > vc)
        atomicMin(&b.states[t.page].err, (unsigned long long)err_key(3, vc, PQH_ERR_EOF));
    }
    return;
  }
  if (P.kind == K_PLAIN_BA || (P.kind == K_DLBA && dlba_pages)) {
    for (int32_t k = 0; k < P.batile_n; k++) ba_tile_sum(b, t.page, k, wsum);
    return;
  }
  ba_tile_sum(b, t.page, t.k, wsum);
}

// ------------------------------------------------------------------------------------------------
// k_ba_scan: one workgroup per byte-array chunk: exclusive scan of its tiles' byte sums (tiles of a
// chunk are contiguous and in page order) -> each tile's first output offset, each page's first
// byte (byte_base), the chunk's byte total.
// ------------------------------------------------------------------------------------------------
// Each thread scans a contiguous run of ceil(n / 256) tiles (independent loads, one block scan), so
// a chunk of thousands of tiles costs one pass instead of one barrier round per 256 tiles.
__device__ int64_t chunk_scan(int64_t* sums, int32_t n, const Tile* tiles, PageState* states, uint64_t* wsum) {
  const int per = (n + kBlock - 1) / kBlock;
  const int i0 = int(threadIdx.x) * per, i1 = i0 + per < n ? i0 + per : n;
  uint64_t local = 0;
  for (int i = i0; i < i1; i += 8) {  // 8 loads in flight
    int64_t x[8];
#pragma unroll
    for (int k = 0; k < 8; k++) x[k] = i + k < i1 ? sums[i + k] : 0;
#pragma unroll
    for (int k = 0; k < 8; k++) local += uint64_t(x[k]);
  }
  uint64_t total;
  int64_t run = int64_t(block_exclusive_scan(local, wsum, &total));
  for (int i = i0; i < i1; i += 8) {
    int64_t x[8];
    Tile tl[8];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      x[k] = i + k < i1 ? sums[i + k] : 0;
      if (states && i + k < i1) tl[k] = tiles[i + k];
    }
#pragma unroll
    for (int k = 0; k < 8; k++) {
      if (i + k >= i1) break;
      sums[i + k] = run;
      if (states && tl[k].k == 0) states[tl[k].page].byte_base = run;
      run += x[k];
    }
  }
  return int64_t(total);
}

__global__ __launch_bounds__(256) void k_ba_scan(DevBatch b, const int32_t* ba_chunks, const Tile* tiles) {
  __shared__ uint64_t wsum[4];
  const int c = ba_chunks[blockIdx.x];
  const DevChunk C = b.chunks[c];
  if (threadIdx.x == 0 && C.offsets) C.offsets[0] = 0;
  const int64_t total = chunk_scan(b.basums + C.batile_base, C.batile_n, tiles + C.batile_base, b.states, wsum);
  if (C.aux2) chunk_scan(b.basums2 + C.batile_base, C.batile_n, tiles + C.batile_base, nullptr, wsum);
  if (threadIdx.x == 0) b.chunk_bytes[c] = total;
}

// Cooperative copy of n bytes by the workgroup: 16-byte aligned stores, each fed by one unaligned
// 16-byte load of the source (the hardware's unaligned dwordx4 load; two aligned loads put
// together with v_alignbyte measured slower: C5 k_ba_expand 0.53 vs 0.57 of peak).  kIn loads in
// flight per thread.  DELTA_LENGTH copies (r06): copy first, 8 in flight.  Nontemporal loads +
// stores (kNt = 2) split the workloads on two boxes: C5z k_ba_expand 0.61-0.65 -> 0.61-0.68 of
// peak, C5 (the BASELINE config) 0.58-0.62 -> 0.55-0.62; kept off (PQH_BA_COPY_NT=2 builds it).
#ifndef PQH_BA_COPY_FIRST
#define PQH_BA_COPY_FIRST 1
#endif
#ifndef PQH_BA_COPY_INFLIGHT
#define PQH_BA_COPY_INFLIGHT 8
#endif
#ifndef PQH_BA_COPY_NT
#define PQH_BA_COPY_NT 0
#endif
typedef unsigned int v4u_a1 __attribute__((ext_vector_type(4), aligned(1)));
template <class T>
__device__ __forceinline__ uint4 nt_load16(const PQH_G T* p) {
  const v4u_a1 v = __builtin_nontemporal_load(reinterpret_cast<const PQH_G v4u_a1*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
template <int kIn = 4, int kNt = 0>  // 16-byte loads in flight per thread; 1: streaming stores, 2: + loads
__device__ __forceinline__ void block_copy(PQH_G uint8_t* dst, const PQH_G uint8_t* src, int64_t n) {
  // destination 16-byte aligned after the head; the source side uses unaligned 16-byte loads
  const int64_t head = int64_t((16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15) < n
                           ? int64_t((16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15) : n;
  if (int64_t(threadIdx.x) < head) dst[threadIdx.x] = src[threadIdx.x];
  const int64_t units = (n - head) >> 4;
  typedef uint4 uint4_u __attribute__((aligned(1)));
  const PQH_G uint4_u* sp = reinterpret_cast<const PQH_G uint4_u*>(src + head);
  PQH_G uint4* d = reinterpret_cast<PQH_G uint4*>(dst + head);
  int64_t u = threadIdx.x;
  if constexpr (kIn == 8) {
    for (; u + 7 * kBlock < units; u += 8 * kBlock) {
      uint4 x0, x1, x2, x3, x4, x5, x6, x7;
      if constexpr (kNt == 2) {
        x0 = nt_load16(sp + u);
        x1 = nt_load16(sp + u + kBlock);
        x2 = nt_load16(sp + u + 2 * kBlock);
        x3 = nt_load16(sp + u + 3 * kBlock);
        x4 = nt_load16(sp + u + 4 * kBlock);
        x5 = nt_load16(sp + u + 5 * kBlock);
        x6 = nt_load16(sp + u + 6 * kBlock);
        x7 = nt_load16(sp + u + 7 * kBlock);
      } else {
        x0 = sp[u], x1 = sp[u + kBlock], x2 = sp[u + 2 * kBlock], x3 = sp[u + 3 * kBlock];
        x4 = sp[u + 4 * kBlock], x5 = sp[u + 5 * kBlock], x6 = sp[u + 6 * kBlock], x7 = sp[u + 7 * kBlock];
      }
      if constexpr (kNt != 0) {
        typedef unsigned int v4u __attribute__((ext_vector_type(4)));
        PQH_G v4u* dv = reinterpret_cast<PQH_G v4u*>(d);
        __builtin_nontemporal_store(v4u{x0.x, x0.y, x0.z, x0.w}, dv + u);
        __builtin_nontemporal_store(v4u{x1.x, x1.y, x1.z, x1.w}, dv + u + kBlock);
        __builtin_nontemporal_store(v4u{x2.x, x2.y, x2.z, x2.w}, dv + u + 2 * kBlock);
        __builtin_nontemporal_store(v4u{x3.x, x3.y, x3.z, x3.w}, dv + u + 3 * kBlock);
        __builtin_nontemporal_store(v4u{x4.x, x4.y, x4.z, x4.w}, dv + u + 4 * kBlock);
        __builtin_nontemporal_store(v4u{x5.x, x5.y, x5.z, x5.w}, dv + u + 5 * kBlock);
        __builtin_nontemporal_store(v4u{x6.x, x6.y, x6.z, x6.w}, dv + u + 6 * kBlock);
        __builtin_nontemporal_store(v4u{x7.x, x7.y, x7.z, x7.w}, dv + u + 7 * kBlock);
        continue;
      }
      d[u] = x0;
      d[u + kBlock] = x1;
      d[u + 2 * kBlock] = x2;
      d[u + 3 * kBlock] = x3;
      d[u + 4 * kBlock] = x4;
      d[u + 5 * kBlock] = x5;
      d[u + 6 * kBlock] = x6;
      d[u + 7 * kBlock] = x7;
    }
  }
  for (; u + 3 * kBlock < units; u += 4 * kBlock) {
    const uint4 x0 = sp[u], x1 = sp[u + kBlock], x2 = sp[u + 2 * kBlock], x3 = sp[u + 3 * kBlock];
    d[u] = x0;
    d[u + kBlock] = x1;
    d[u + 2 * kBlock] = x2;
    d[u + 3 * kBlock] = x3;
  }
  for (; u < units; u += kBlock) d[u] = sp[u];
  const int64_t done = head + units * 16;
  if (int64_t(threadIdx.x) < n - done) dst[done + threadIdx.x] = src[done + threadIdx.x];
}


// Byte copy of one value (unaligned on both sides; values average tens of bytes).
__device__ __forceinline__ void copy_bytes(uint8_t* dst, const uint8_t* src, int64_t len);

// ceil(len / 8) unaligned 8-byte words (len > 0).
__device__ __forceinline__ void copy_words(PQH_G uint8_t* dst, const uint8_t* src_, int64_t len) {
  typedef uint64_t u64u __attribute__((aligned(1)));
  const PQH_G u64u* s = (const PQH_G u64u*)(src_);
  PQH_G u64u* d = (PQH_G u64u*)(dst);
  for (int64_t k = 0; k < len; k += 8) d[k >> 3] = s[k >> 3];
}

// DELTA_BYTE_ARRAY tile (byteArrayDeltaDecoder.decodeValues, type_bytearray.go:213-240): offsets
// from prefix + suffix lengths, the per-value checks in the reference's order (suffix read short,
// negative total, prefix longer than the previous value), and each suffix copied into place after
// its prefix; the prefixes themselves are filled by k_dba_prefix once every suffix is written.
__device__ void dba_expand(const DevBatch& b, const Tile& t, const DevPage& P, const PageState& S, const DevChunk& C,
                           int64_t v0, int64_t v1, uint64_t* wsum) {
  const int32_t* slen = C.aux + S.value_base;
  const int32_t* plen = C.aux2 + S.value_base;
  const int64_t i0 = v0 + 8 * int64_t(threadIdx.x);
  int64_t L[8], sl[8], ssum = 0, lsum = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const bool in = i0 + j < v1;
    sl[j] = in ? slen[i0 + j] : 0;
    L[j] = in ? dba_len(plen, slen, i0 + j) : 0;
    ssum += sl[j];
    lsum += L[j];
  }
  uint64_t tot, stot;
  const int64_t excl = int64_t(block_exclusive_scan(uint64_t(lsum), wsum, &tot));
  const int64_t sexcl = int64_t(block_exclusive_scan(uint64_t(ssum), wsum, &stot));
  const int64_t base = b.basums[P.batile_base + t.k];
  const int64_t sbase = b.basums2[P.batile_base + t.k] - b.basums2[P.batile_base];  // page-relative suffix bytes
  const DeltaState D1 = b.dstates[b.num_pages + t.page];
  const uint8_t* data = b.payload + P.image_off + D1.end_pos;  // suffix bytes follow the two length streams
  const int64_t data_n = S.val_e - D1.end_pos;
  int64_t* offs = C.offsets + S.value_base + 1;
  int64_t o = base + excl, sr = sbase + sexcl;
  int64_t prev_len = i0 > 0 && i0 < v1 ? dba_len(plen, slen, i0 - 1) : 0;  // previousValue starts empty
  int64_t first_bad = INT64_MAX;
  int bad_code = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const int64_t i = i0 + j;
    if (i >= v1) break;
    const int32_t p = plen[i];
    int code = PQH_OK;
    if (sl[j] > 0 && data_n - sr < sl[j]) code = data_n - sr <= 0 ? PQH_ERR_EOF : PQH_ERR_UNEXPECTED_EOF;
    else if (int64_t(p) + sl[j] < 0) code = PQH_ERR_NEGATIVE_DLBA_LENGTH;
    else if (prev_len < p) code = PQH_ERR_DBA_PREFIX;
    if (code != PQH_OK && i < first_bad) {
      first_bad = i;
      bad_code = code;
    }
    const int64_t pp = p > 0 ? p : 0;
    if (code == PQH_OK && sl[j] > 0 && o + L[j] <= C.bytes_cap) copy_bytes(C.bytes + o + pp, data + sr, sl[j]);
    o += L[j];
    offs[i] = o;
    sr += sl[j];
    prev_len = L[j];
  }
  if (first_bad != INT64_MAX) atomicMin(&b.states[t.page].err, (unsigned long long)err_key(3, first_bad, bad_code));
}

__global__ __launch_bounds__(256) void k_dba_expand(DevBatch b, const Tile* tiles) {
  __shared__ uint64_t wsum[4];
  const Tile t = tiles[blockIdx.x];
  const DevPage P = b.pages[t.page];
  if (P.kind != K_DBA) return;
  const PageState S = b.states[t.page];
  if (page_failed_before_values(S)) return;
  const DevChunk C = b.chunks[P.chunk];
  const int64_t lim = ba_limit(b, t.page, P, S);
  const int64_t v0 = int64_t(t.k) * kBaTile;
  const int64_t v1 = v0 + kBaTile < lim ? v0 + kBaTile : lim;
  if (v0 >= v1) return;
  dba_expand(b, t, P, S, C, v0, v1, wsum);
}

// k_dba_prefix: value i's first plen_i bytes equal the previous value's (type_bytearray.go:229-231),
// hence, going back, the suffix bytes of the nearest earlier values whose prefix is shorter:
// byte k of value i is byte k of value m, m = the last j <= i with max(plen_j, 0) <= k, and that
// byte lies in m's suffix, already in place.  Every byte is copied straight from its source.
__global__ __launch_bounds__(256) void k_dba_prefix(DevBatch b, const Tile* tiles) {
  const Tile t = tiles[blockIdx.x];
  const DevPage P = b.pages[t.page];
  if (P.kind != K_DBA) return;
  const PageState S = b.states[t.page];
  if (page_failed_before_values(S)) return;
  const DevChunk C = b.chunks[P.chunk];
  const int64_t lim = ba_limit(b, t.page, P, S);
  const int64_t v0 = int64_t(t.k) * kBaTile;
  const int64_t v1 = v0 + kBaTile < lim ? v0 + kBaTile : lim;
  const int32_t* plen = C.aux2 + S.value_base;
  const int64_t* off = C.offsets + S.value_base;  // off[i] = first byte of value i
  for (int64_t i = v0 + threadIdx.x; i < v1; i += kBlock) {
    int64_t hi = plen[i];
    const int64_t oi = off[i];
    if (hi <= 0 || oi + hi > C.bytes_cap) continue;
    for (int64_t j = i - 1; j >= 0 && hi > 0; j--) {
      const int64_t pj = plen[j] > 0 ? plen[j] : 0;
      if (pj < hi) {  // bytes [pj, hi) of value j are its own suffix bytes
        copy_bytes(C.bytes + oi + pj, C.bytes + off[j] + pj, hi - pj);
        hi = pj;
      }
    }
  }
}
__device__ __forceinline__ void copy_bytes(uint8_t* dst, const uint8_t* src, int64_t len) {
  int64_t k = 0;
  for (; k + 8 <= len; k += 8) {
    uint64_t x;
    __builtin_memcpy(&x, src + k, 8);
    __builtin_memcpy(dst + k, &x, 8);
  }
  for (; k < len; k++) dst[k] = src[k];
}

// ------------------------------------------------------------------------------------------------
// k_ba_expand: per kBaTile tile of a PLAIN / DELTA_LENGTH / dictionary page.
//   * lengths (or dictionary keys) are read with value index = j * 256 + thread (coalesced) into
//     LDS; each thread then scans 8 consecutive lengths (block scan) -> tile-relative offsets;
//   * the offsets go out coalesced; DELTA_LENGTH reads past the page (io.ReadFull short) are found
//     here: the first value whose bytes do not fit is the page's error;
//   * bytes: DELTA_LENGTH strings are contiguous in the page (one cooperative copy); PLAIN and
//     dictionary values are gathered by their threads into an LDS image of kBaOut bytes of the
//     tile's output at a time, then written out in aligned 16-byte stores; tiles of more than
//     kBaOutWindows windows copy each value straight to its place (neighbouring lanes write
//     neighbouring strings).
// ------------------------------------------------------------------------------------------------
constexpr int kBaOut = 16384;       // LDS output window
constexpr int kBaOutWindows = 64;  // tiles with more output bytes copy each value directly

// Bytes [0, len) of a value into LDS at d (any alignment): bytes up to a 4-aligned d, then dwords.
__device__ __forceinline__ void lds_put(uint8_t* d, const PQH_G uint8_t* src, int64_t len) {
  typedef uint32_t u32u __attribute__((aligned(1)));
  int64_t k = 0;
  for (; k < len && ((reinterpret_cast<uintptr_t>(d) + uintptr_t(k)) & 3); k++) d[k] = src[k];
  for (; k + 4 <= len; k += 4) *reinterpret_cast<uint32_t*>(d + k) = *reinterpret_cast<const PQH_G u32u*>(src + k);
  for (; k < len; k++) d[k] = src[k];
}

// kGather = false: DELTA_LENGTH tiles (contiguous strings); true: PLAIN and dictionary tiles.
template <bool kGather>
__device__ __forceinline__ void ba_expand_tile(const DevBatch& b, const Tile& t, uint64_t* wsum, int64_t* s_off,
                                               uint8_t* s_out) {
  const DevPage P = b.pages[t.page];
  const PageState S = b.states[t.page];
  if (page_failed_before_values(S)) return;
  const DevChunk C = b.chunks[P.chunk];
  const int64_t lim = ba_limit(b, t.page, P, S);
  const int64_t v0 = int64_t(t.k) * kBaTile;
  const int64_t v1 = v0 + kBaTile < lim ? v0 + kBaTile : lim;
  if (v0 >= v1) return;
  if (P.value_size > 0) {  // fixed-width page of a FIXED_LEN_BYTE_ARRAY chunk laid out as byte arrays:
    if constexpr (!kGather) {  // its values (already decoded into the values buffer) are contiguous
      const int64_t vs = P.value_size, n = v1 - v0;
      const int64_t base = b.basums[P.batile_base + t.k];
      PQH_G int64_t* offs = C.offsets + S.value_base + 1 + v0;
      for (int64_t i = threadIdx.x; i < n; i += kBlock) offs[i] = base + (i + 1) * vs;
      int64_t len = n * vs;
      if (len > C.bytes_cap - base) len = C.bytes_cap - base;
      if (len > 0) block_copy(C.bytes + base, C.values + (S.value_base + v0) * vs, len);
    }
    return;
  }
  const bool is_dict = P.kind == K_DICT, is_dlba = P.kind == K_DLBA, is_dba = P.kind == K_DBA;
  if (is_dba || is_dlba == kGather) return;  // k_dba_expand; the other kernel
  const BaDict d = is_dict ? ba_dict(b, P) : BaDict{nullptr, 0, 0};
  const int32_t* aux = C.aux + S.value_base + v0;
  const int n = int(v1 - v0), tid = threadIdx.x;
  // DELTA_LENGTH: the tile's strings are contiguous in the page and in the output, and k_ba_scan's
  // bases already fix their extent -- [basums[tile], basums[tile + 1]) (the chunk's byte total after
  // its last tile) -- so the copy is issued first, its loads in flight before the lengths' load and
  // scan instead of after them.  A tile whose lengths sum past that extent (only an erroneous page
  // can) copies the rest after the scan.
  int64_t pre = 0;
  if constexpr (!kGather) {
#if PQH_BA_COPY_FIRST
    const int64_t gi = P.batile_base + t.k, base = b.basums[gi];
    const int64_t nxt = gi + 1 < C.batile_base + C.batile_n ? b.basums[gi + 1] : b.chunk_bytes[P.chunk];
    const int64_t ds = b.dstates[t.page].end_pos, rel0 = base - S.byte_base;
    pre = nxt - base;
    if (pre > S.val_e - ds - rel0) pre = S.val_e - ds - rel0;
    if (pre > C.bytes_cap - base) pre = C.bytes_cap - base;
    if (pre > 0) block_copy<PQH_BA_COPY_INFLIGHT, PQH_BA_COPY_NT>(C.bytes + base, b.payload + P.image_off + ds + rel0, pre);
    else pre = 0;
#endif
  }
  int32_t a[8];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const int idx = j * kBlock + tid;
    a[j] = idx < n ? aux[idx] : 0;
    const int64_t l = idx < n ? ba_len(d, is_dict, a[j]) : 0;
    s_off[idx] = l > 0 ? l : 0;
  }
  __syncthreads();
  int64_t L[8], tsum = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    L[j] = s_off[8 * tid + j];
    tsum += L[j];
  }
  uint64_t tot;
  int64_t o = int64_t(block_exclusive_scan(uint64_t(tsum), wsum, &tot));
#pragma unroll
  for (int j = 0; j < 8; j++) {
    s_off[8 * tid + j] = o;
    o += L[j];
  }
  if (tid == kBlock - 1) s_off[kBaTile] = o;
  __syncthreads();
  const int64_t base = b.basums[P.batile_base + t.k];
  const PQH_G uint8_t* img = b.payload + P.image_off;
  int64_t data_s = 0, data_n = 0;
  if (is_dlba) {
    data_s = b.dstates[t.page].end_pos;
    data_n = S.val_e - data_s;
  }
  int64_t* offs = C.offsets + S.value_base + 1 + v0;
  int64_t first_bad = INT64_MAX;
  int bad_code = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const int idx = j * kBlock + tid;
    if (idx >= n) break;
    const int64_t e = s_off[idx + 1];
    offs[idx] = base + e;
    if (is_dlba) {
      const int64_t l = e - s_off[idx], rem = data_n - (base + s_off[idx] - S.byte_base);
      if (l > 0 && rem < l && v0 + idx < first_bad) {
        first_bad = v0 + idx;
        bad_code = rem <= 0 ? PQH_ERR_EOF : PQH_ERR_UNEXPECTED_EOF;
      }
    }
  }
  if (first_bad != INT64_MAX) atomicMin(&b.states[t.page].err, (unsigned long long)err_key(3, first_bad, bad_code));
  if constexpr (!kGather) {  // the tile's strings are contiguous in the page: one cooperative copy
    const int64_t rel0 = base - S.byte_base;
    int64_t len_all = int64_t(tot);
    if (len_all > data_n - rel0) len_all = data_n - rel0;   // bytes past the page belong to the error
    if (len_all > C.bytes_cap - base) len_all = C.bytes_cap - base;
    if (len_all > pre) block_copy<PQH_BA_COPY_INFLIGHT, PQH_BA_COPY_NT>(C.bytes + base + pre, img + data_s + rel0 + pre, len_all - pre);
    return;
  } else {
  // source of value idx (nullptr: an out-of-range dictionary key, whose page fails)
  auto src_of = [&](int j, int idx) -> const PQH_G uint8_t* {
    if (is_dict) {
      const uint32_t k = uint32_t(a[j]);
      return k < d.K ? b.payload + d.base + 4 * int64_t(k + 1) + d.dcum[k] : nullptr;
    }
    // PLAIN: value i's bytes follow its u32 length
    return img + S.val_s + 4 * (v0 + idx + 1) + (base + s_off[idx] - S.byte_base);
  };
  PQH_G uint8_t* dst = C.bytes + base;
  const int lead = int(reinterpret_cast<uintptr_t>(dst) & 15);
  const int64_t end = lead + int64_t(tot);  // output bytes in coordinates of the aligned start A
  if (end <= kBaOutWindows * int64_t(kBaOut) && base + int64_t(tot) <= C.bytes_cap) {
    PQH_G uint8_t* A = dst - lead;
    for (int64_t w0 = 0; w0 < end; w0 += kBaOut) {  // kBaOut bytes of output per pass
      const int64_t w1 = w0 + kBaOut < end ? w0 + kBaOut : end;
      // the thread's pieces, four at a time: the first 16 bytes of each come from one unaligned
      // 16-byte load, the four loads in flight together (the payload pad covers the over-read);
      // longer pieces continue with lds_put
      typedef uint4 uint4_u __attribute__((aligned(1)));
#pragma unroll
      for (int h = 0; h < 8; h += 4) {
        uint4 v[4];
        const PQH_G uint8_t* sp[4];
        int32_t pl[4], pd[4];
#pragma unroll
        for (int jj = 0; jj < 4; jj++) {
          const int j = h + jj, idx = j * kBlock + tid;
          sp[jj] = nullptr;
          pl[jj] = 0;
          pd[jj] = 0;
          if (idx < n) {
            const int64_t x0 = lead + s_off[idx], x1 = lead + s_off[idx + 1];
            const int64_t c0 = x0 > w0 ? x0 : w0, c1 = x1 < w1 ? x1 : w1;
            if (c0 < c1) {
              const PQH_G uint8_t* src = src_of(j, idx);
              if (src) {
                sp[jj] = src + (c0 - x0);
                pl[jj] = int32_t(c1 - c0);
                pd[jj] = int32_t(c0 - w0);
              }
            }
          }
          v[jj] = make_uint4(0, 0, 0, 0);
          if (sp[jj]) {
            const uint4 x = *reinterpret_cast<const PQH_G uint4_u*>(sp[jj]);
            v[jj] = x;
          }
        }
#pragma unroll
        for (int jj = 0; jj < 4; jj++) {
          if (!sp[jj]) continue;
          uint8_t* d = s_out + pd[jj];
          const uint32_t wv[4] = {v[jj].x, v[jj].y, v[jj].z, v[jj].w};
#pragma unroll
          for (int q = 0; q < 16; q++)
            if (q < pl[jj]) d[q] = uint8_t(wv[q >> 2] >> (8 * (q & 3)));
          if (pl[jj] > 16) lds_put(d + 16, sp[jj] + 16, pl[jj] - 16);
        }
      }
      __syncthreads();
      const int nb = int(w1 - w0);
      for (int c = tid; c < (nb + 15) >> 4; c += kBlock) {
        const int lo = c << 4;
        const int64_t g = w0 + lo;
        if (g >= lead && g + 16 <= end) {
          typedef unsigned int v4u __attribute__((ext_vector_type(4)));
          __builtin_nontemporal_store(*reinterpret_cast<const v4u*>(s_out + lo), reinterpret_cast<PQH_G v4u*>(A + g));
        } else {
          for (int q = 0; q < 16 && lo + q < nb; q++)
            if (g + q >= lead && g + q < end) A[g + q] = s_out[lo + q];
        }
      }
      __syncthreads();
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const int idx = j * kBlock + tid;
    if (idx >= n) break;
    const int64_t o0 = s_off[idx], l = s_off[idx + 1] - o0;
    const PQH_G uint8_t* src = l > 0 ? src_of(j, idx) : nullptr;
    if (src && base + o0 + l <= C.bytes_cap) copy_bytes(dst + o0, src, l);
  }
  }
}

// The tile lists hold indices into the chunk-ordered tile table: DELTA_LENGTH tiles for
// k_ba_expand, PLAIN / dictionary tiles for k_ba_gather (the gather needs more registers, which
// would cost the copy kernel occupancy).
__global__ __launch_bounds__(256) void k_ba_expand(DevBatch b, const Tile* tiles, const int32_t* list) {
  __shared__ uint64_t wsum[4];
  __shared__ int64_t s_off[kBaTile + 1];  // lengths, then tile-relative exclusive offsets
  ba_expand_tile<false>(b, tiles[list[blockIdx.x]], wsum, s_off, nullptr);
}

__global__ __launch_bounds__(256) void k_ba_gather(DevBatch b, const Tile* tiles, const int32_t* list) {
  __shared__ uint64_t wsum[4];
  __shared__ int64_t s_off[kBaTile + 1];
  __shared__ __attribute__((aligned(16))) uint8_t s_out[kBaOut + 16];
  ba_expand_tile<true>(b, tiles[list[blockIdx.x]], wsum, s_off, s_out);
}

// ------------------------------------------------------------------------------------------------
// k_ba_wcopy: PLAIN byte-array data pages, after k_ba_scan, by chain windows (list: {window, page}).
// A window's records are consecutive values of its page; k_ba_wspec left the bytes before each
// record within the window (exclusive offsets) in the window's scratch, and the records' bytes are
// the window's page bytes with the u32 length fields dropped (byteArrayPlainDecoder.next,
// type_bytearray.go:24-45): record i's bytes start at entry + 4 (i + 1) + offset_i.
//   * the window's page bytes (aligned 16-byte loads) and its offsets are staged in LDS, all loads
//     in flight together;
//   * one thread per record writes its chunk offset and copies its bytes from the stage (dwords
//     through alignbit, stored unaligned; neighbouring lanes write neighbouring records);
//   * the grid is persistent: a few workgroups per CU loop over the windows, the next window's
//     metadata chain (window -> page, state -> chunk) loading while this one is copied;
//   * a window whose last record runs past the stage (a string of more than ~1 KiB at its end)
//     copies straight from the page: short records per thread, long ones by the workgroup.
// ------------------------------------------------------------------------------------------------
constexpr int kWStage = kChainWin + 1280;  // staged page bytes: a window plus ~1 KiB of overrun
constexpr int kWV = (kWStage / 16 + kBlock - 1) / kBlock;  // page vectors per thread
constexpr int kWP = (kChainRecs / 2 + kBlock) / kBlock;    // 16 offset pairs per thread
constexpr int kWGrid = (kChainSeg > 64 ? 3 : 6) * 256;       // resident workgroups (LDS-limited per CU)

struct WcopyLds {
  uint32_t stage[kWStage / 4 + 4];
  uint16_t offs[kChainRecs + 8];  // the window's exclusive offsets (staged windows: < 2^16)
};

// One window's geometry and destination (wave-uniform; loaded one window ahead).
struct WGeo {
  int32_t wi, n;     // window, records to emit (0: nothing)
  int32_t in_lead;   // page bytes before the entry in its 16-byte vector
  int32_t nvec;      // staged 16-byte vectors (0: the window is not staged)
  int32_t entry;     // page offset of the first record
  int32_t endo;      // window bytes before record n (the end of the last record emitted)
  int64_t obase;     // chunk-relative first output byte of the window
  int64_t cap;       // output bytes the chunk can take from the window on
  const PQH_G uint8_t* img;
  PQH_G uint8_t* dst;
  PQH_G int64_t* offs_out;
};

__device__ __forceinline__ WGeo wgeo(const DevBatch& b, const int2* list, const BaWin* res, const uint16_t* wrec,
                                     int t) {
  WGeo g{};
  const int2 wl = list[t];
  const BaWin r = res[wl.x];
  const DevPage P = b.pages[wl.y];
  const PageState S = b.states[wl.y];
  g.wi = wl.x;
  g.n = 0;
  if (r.base < 0 || r.entry < 0 || page_failed_before_values(S)) return g;
  int64_t n = ba_limit(b, wl.y, P, S) - r.base;
  if (n > r.count) n = r.count;
  if (n <= 0) return g;
  const DevChunk C = b.chunks[P.chunk];
  g.n = int32_t(n);
  g.endo = n < r.count ? int32_t(wrec[int64_t(wl.x) * kChainRecs + n]) : r.bytes;
  g.img = b.payload + P.image_off;
  g.entry = r.entry;
  g.in_lead = int32_t(reinterpret_cast<uintptr_t>(g.img + r.entry) & 15);
  // exit - entry >= the page bytes of the records (lengths and strings)
  const int64_t span = g.in_lead + (int64_t(r.exit) - r.entry);
  g.nvec = span <= kWStage ? int32_t((span + 15) >> 4) : 0;
  g.obase = S.byte_base + r.cbase;
  g.cap = C.bytes_cap - g.obase;
  g.dst = C.bytes + g.obase;
  g.offs_out = (PQH_G int64_t*)(C.offsets + S.value_base + 1 + r.base);
  return g;
}

// One thread per window: its geometry, so that k_ba_wcopy's workgroups load one record per window
// instead of a chain of dependent loads (window -> page -> state -> chunk).
__global__ __launch_bounds__(256) void k_ba_wgeo(DevBatch b, const int2* list, int32_t nlist, const BaWin* res,
                                                  const uint16_t* wrec, WGeo* geo) {
  const int t = int(blockIdx.x) * kBlock + int(threadIdx.x);
  if (t < nlist) geo[t] = wgeo(b, list, res, wrec, t);
}

// One string of l bytes from staged page bytes (dword array, the string at byte sx) to d.  Short
// strings: five stage dwords, predicated stores, no per-byte loop.  The stage must hold 20 bytes
// from sx's dword on for a short string, l + 4 for a long one.
__device__ __forceinline__ void stage_string_out(const uint32_t* stage, int sx, int l, PQH_G uint8_t* d) {
  typedef uint32_t u32u __attribute__((aligned(1)));
  typedef uint64_t u64u __attribute__((aligned(1)));
  typedef uint16_t u16u __attribute__((aligned(1)));
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  typedef v4u v4uu __attribute__((aligned(1)));
  const int w0 = sx >> 2;
  const uint32_t sh = uint32_t(sx & 3) * 8;
  if (l <= 16) {
    const uint32_t a0 = stage[w0], a1 = stage[w0 + 1], a2 = stage[w0 + 2], a3 = stage[w0 + 3], a4 = stage[w0 + 4];
    const uint32_t v0 = __builtin_amdgcn_alignbit(a1, a0, sh), v1 = __builtin_amdgcn_alignbit(a2, a1, sh),
                   v2 = __builtin_amdgcn_alignbit(a3, a2, sh), v3 = __builtin_amdgcn_alignbit(a4, a3, sh);
    const int nw = l >> 2, tl = l & 3;
    if (nw == 4) {
      const v4u x4 = {v0, v1, v2, v3};
      *reinterpret_cast<PQH_G v4uu*>(d) = x4;
    } else {
      if (nw >= 2) *reinterpret_cast<PQH_G u64u*>(d) = uint64_t(v0) | (uint64_t(v1) << 32);
      if (nw & 1) *reinterpret_cast<PQH_G u32u*>(d + 4 * (nw & 2)) = (nw & 2) ? v2 : v0;
      const uint32_t tv = nw == 0 ? v0 : nw == 1 ? v1 : nw == 2 ? v2 : v3;
      PQH_G uint8_t* dt = d + 4 * nw;
      if (tl & 2) *reinterpret_cast<PQH_G u16u*>(dt) = uint16_t(tv);
      if (tl & 1) dt[tl & 2] = uint8_t(tv >> (8 * (tl & 2)));
    }
  } else {
    int k = 0;
    for (; k + 4 <= l; k += 4) {
      const int q = sx + k;
      *reinterpret_cast<PQH_G u32u*>(d + k) = __builtin_amdgcn_alignbit(stage[(q >> 2) + 1], stage[q >> 2], uint32_t(q & 3) * 8);
    }
    for (; k < l; k++) {
      const int q = sx + k;
      d[k] = uint8_t(stage[q >> 2] >> (8 * (q & 3)));
    }
  }
}

// The window's page vectors and offset pairs into registers (every load unconditional, clamped
// addresses), all in flight together.
__device__ __forceinline__ void wcopy_issue(const WGeo& g, const uint16_t* wrec, uint4 (&x)[kWV], uint32_t (&ov)[kWP]) {
  const int tid = threadIdx.x;
  const PQH_G uint8_t* wb = g.img + g.entry - g.in_lead;
  // (kChainRecs is even: every window's entries start 4-byte aligned)
  const PQH_G uint32_t* wo = (const PQH_G uint32_t*)(wrec + int64_t(g.wi) * kChainRecs);
#pragma unroll
  for (int j = 0; j < kWV; j++) {
    const int k = tid + j * kBlock;
    x[j] = *reinterpret_cast<const PQH_G uint4*>(wb + (k < g.nvec ? 16 * k : 0));
  }
#pragma unroll
  for (int j = 0; j < kWP; j++) {  // offsets 0 .. n - 1, two per dword (offset n is g.endo)
    const int k = tid + j * kBlock;
    ov[j] = wo[2 * k < g.n ? k : 0];
  }
}

__global__ __launch_bounds__(256) void k_ba_wcopy(DevBatch b, const WGeo* geo, int32_t nlist, const uint16_t* wrec) {
  __shared__ WcopyLds L;
  const int tid = threadIdx.x;
  const int grid = int(gridDim.x);
  int t = blockIdx.x;
  if (t >= nlist) return;
  // the next window's geometry (one independent load) in flight during this window
  WGeo g = geo[t];
  uint4 x[kWV];
  uint32_t ov[kWP];
  for (;;) {
    WGeo gn{};
    if (t + grid < nlist) gn = geo[t + grid];
    const int n = g.n;
    const PQH_G uint16_t* wo = (const PQH_G uint16_t*)(wrec + int64_t(g.wi) * kChainRecs);
    if (n > 0 && g.nvec) {
      wcopy_issue(g, wrec, x, ov);
      // every LDS store unconditional too (out-of-range ones to spare slots)
      constexpr int kSpareVec = kWStage / 16;
      constexpr int kSpareRec = kChainRecs + 1;
#pragma unroll
      for (int j = 0; j < kWV; j++) {
        const int k = tid + j * kBlock;
        reinterpret_cast<uint4*>(L.stage)[k < g.nvec ? k : kSpareVec] = x[j];
      }
#pragma unroll
      for (int j = 0; j < kWP; j++) {
        const int k = tid + j * kBlock;
        L.offs[2 * k < n ? 2 * k : kSpareRec] = uint16_t(ov[j]);
        L.offs[2 * k + 1 < n ? 2 * k + 1 : kSpareRec] = uint16_t(ov[j] >> 16);
      }
      if (tid == 0) L.offs[n] = uint16_t(g.endo);  // < 2^16: the staged span holds the records' bytes
      __syncthreads();
      for (int i = tid; i < n; i += kBlock) {
        const int o = L.offs[i], e = L.offs[i + 1];
        g.offs_out[i] = g.obase + e;
        int l = e - o;
        if (o + l > g.cap) l = g.cap > o ? int(g.cap - o) : 0;
        stage_string_out(L.stage, g.in_lead + 4 * (i + 1) + o, l, g.dst + o);
      }
      __syncthreads();  // the stage is read before the next window's stores
    } else if (n > 0) {
      // a record runs past the stage: straight from the page
      const PQH_G uint8_t* src0 = g.img + g.entry;
      constexpr int kLong = 512;
      for (int i = tid; i < n; i += kBlock) {
        const int64_t o = wo[i], l = (i + 1 < n ? int64_t(wo[i + 1]) : g.endo) - o;
        g.offs_out[i] = g.obase + o + l;
        if (l > 0 && l < kLong && o + l <= g.cap) copy_bytes(g.dst + o, src0 + 4 * (i + 1) + o, l);
      }
      for (int i = 0; i < n; i++) {  // uniform: the long records by the whole workgroup
        const int64_t o = wo[i], l = (i + 1 < n ? int64_t(wo[i + 1]) : g.endo) - o;
        if (l < kLong && o + l <= g.cap) continue;
        const int64_t cl = o + l <= g.cap ? l : g.cap - o;
        if (cl > 0) block_copy(g.dst + o, src0 + 4 * (i + 1) + o, cl);
      }
    }
    if (t + grid >= nlist) break;
    g = gn;
    t += grid;
  }
}

// ------------------------------------------------------------------------------------------------
// Fused PLAIN chains (k_ba_chain): chunks whose data pages are all PLAIN byte arrays and which have
// no dictionary page (DevChunk.ba_fused) read their page bytes once.  One workgroup per window,
// taken by ticket in the order (window in page, page) -- every page's window 0, then every window
// 1, ... -- so a window's predecessors in its page hold earlier tickets (resident or done: no
// deadlock) and started a whole round of pages before it (its look-back rarely waits), with a
// decoupled look-back over one 64-bit word per window:
//   * the window is staged and resolved from its guessed entry as in k_ba_wspec, its records into
//     LDS (no scratch), and publishes PARTIAL = (records, guessed entry, exit, invalid record seen);
//     window 0 of a page knows its entry and publishes FINAL = (records of the page up to its end,
//     exit) at once;
//   * wave 0 reads the predecessors' words 64 at a time, newest first (relaxed agent-scope loads:
//     each word is self-contained, so no fence is needed): the nearest FINAL plus the PARTIALs after
//     it give this window's base when every PARTIAL's guessed entry is its predecessor's exit (by
//     induction from the FINAL, each of those windows was resolved from its true entry).  Anything
//     else (a wrong guess, a chain that ended) waits for the predecessor's own FINAL instead;
//   * a wrong guess of its own re-resolves the window from the true entry (LDS still holds the
//     bytes); then it publishes FINAL and writes its offsets and strings straight from LDS.
// Output bases: a page whose chain is exactly notNull records filling its values section has
// val_e - val_s - 4 * notNull string bytes; k_scan sums them into the pages' byte bases (and the
// value bases), and the kernel is launched after it (summing the chunk's earlier pages itself, right
// after the prologue, measured 2% slower on C4: a second round of global loads per window).  The window holding record notNull checks that record's
// end is val_e; a chain that ends early, runs on, fails, or a page that failed earlier sets the
// batch's fallback flag (bafuse[1]), and pqh_batch_sync decodes the batch again with the scratch
// path (k_ba_wspec / wstitch / wcopy), which produces the reference's errors and limits exactly.
// Words: PARTIAL 01 | bad | count:13 | entry - B_w:16 | exit:32;  FINAL 10 | ended | incl:29 | exit:32.
// ------------------------------------------------------------------------------------------------
constexpr uint64_t kPartial = 1ull << 62, kFinal = 2ull << 62, kBadBit = 1ull << 61;
constexpr int64_t kInclMax = (int64_t(1) << 29) - 1;
constexpr int kFuseSpinCap = 1 << 22;  // (never reached: every window a look-back reads is resident)

__device__ __forceinline__ void fuse_fail(const DevBatch& b) {
  __hip_atomic_store(b.bafuse + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ uint64_t fuse_load(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Wave 0: window t (page window w >= 1) -> records before it, the chain's position
// at its start, whether the chain ended before it.  False: no decisive look-back (the caller waits
// for window t - 1's FINAL).
__device__ bool fuse_lookback(const DevBatch& b, int t, int w, int64_t val_s, int64_t* pincl, int64_t* pexit,
                              bool* pended) {
  const int lane = threadIdx.x & 63;
  const int first = t - w;  // the page's window 0 (publishes FINAL only)
  int hi = t - 1;
  int64_t acc = 0, need = -1, exit1 = -1;
  bool ended1 = false;  // window t - 1 ended the chain
  for (bool round0 = true;; round0 = false) {
    const int j = hi - lane;
    const bool in = j >= first;
    uint64_t v = 0;
    for (int spin = 0;; spin++) {
      if (in && v == 0) v = fuse_load(b.bawords + j);
      if (__ballot(in && v == 0) == 0) break;
      if (spin > kFuseSpinCap) {
        if (lane == 0) fuse_fail(b);
        *pended = true;
        return true;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    const bool fin = in && (v >> 62) == 2;
    const uint64_t fm = __ballot(fin);
    const int f = fm ? __builtin_ctzll(fm) : 64;
    const int64_t ex = int64_t(uint32_t(v));
    const int64_t ent = val_s + int64_t(w - (t - j)) * kChainStride + int64_t((v >> 32) & 0xffff);
    const bool bad = (v & kBadBit) != 0;
    int64_t nxt = __shfl_up(ent, 1, 64);  // the entry window j + 1 guessed
    if (lane == 0) nxt = need;
    if (round0) {
      exit1 = __shfl(ex, 0, 64);
      ended1 = __shfl(int(bad), 0, 64) != 0;
    }
    // lanes up to the FINAL: each exit meets its successor's guess; a chain may end only right
    // before window t
    const bool lead = round0 && lane == 0;
    const bool ok = !in || lane > f || ((nxt < 0 || ex == nxt) && (!bad || lead));
    if (__ballot(!ok)) return false;
    int64_t cnt = (in && lane < f) ? int64_t((v >> 48) & 0x1fff) : 0;
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off, 64);
    if (f < 64) {
      const uint64_t vf = __shfl(v, f, 64);
      *pincl = int64_t((vf >> 32) & uint64_t(kInclMax)) + acc + cnt;
      *pexit = exit1;
      *pended = ended1;
      return true;
    }
    acc += cnt;
    need = __shfl(ent, 63, 64);
    hi -= 64;
  }
}

// A wave-uniform value / pointer in scalar registers (the compiler cannot see that a value read from
// LDS is uniform).
__device__ __forceinline__ int64_t uni64(int64_t v) {
  return int64_t((uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(int32_t(uint64_t(v) >> 32)))) << 32) |
                 uint32_t(__builtin_amdgcn_readfirstlane(int32_t(v))));
}
template <class T>
__device__ __forceinline__ T* uni_ptr(T* p) {
  return reinterpret_cast<T*>(uni64(int64_t(reinterpret_cast<uintptr_t>(p))));
}

// The dword at byte q of a staged dword array (any alignment).
__device__ __forceinline__ uint32_t stage_dw(const uint32_t* stage, int q) {
  return __builtin_amdgcn_alignbit(stage[(q >> 2) + 1], stage[q >> 2], uint32_t(q) * 8);  // (shift mod 32)
}

// Records listed per emission pass of k_ba_chain (the window's records are listed and copied in
// passes of this many, so that the list's LDS stays small: 4 workgroups per CU).
constexpr int kChainList = 1024;
constexpr int kChainLongs = 8;  // records past the stage of kLong bytes or more (at most ~2 per window)

__global__ __launch_bounds__(256) void k_ba_chain(DevBatch b, const int2* wins, const int32_t* order, int32_t nwin,
                                                  int32_t use_ticket) {
  __shared__ ChainLds C;
  __shared__ uint16_t list[kChainList + 2];
  __shared__ BaWin R;
  __shared__ int64_t sh[7];
  __shared__ int32_t longs[3 * kChainLongs + 1];  // {index, start, end} of long records past the stage; count
  const int tid = threadIdx.x;
  if (tid == 0) {
    sh[0] = use_ticket ? atomicAdd(b.bafuse, 1u) : blockIdx.x;  // (A/B: the dispatch order itself)
    longs[3 * kChainLongs] = 0;
  }
  __syncthreads();
  if (int(sh[0]) >= nwin) return;
  const int t = order[sh[0]];  // (the window's page-major index: its look-back word)
  const int2 pw = wins[t];
  const int p = pw.x, w = pw.y;
  const PageState S = b.states[p];
  const DevPage P = b.pages[p];
  const int64_t nn = S.nn;
  BaPageCtx c;
  c.ok = S.err == kNoError && nn > 0;
  c.dict = false;
  c.count = nn;
  c.entry = S.val_s;
  c.e0 = S.val_e;
  c.img = b.payload + P.image_off;
  const int64_t Bw = c.entry + int64_t(w) * kChainStride;
  const int64_t wend = Bw + kChainStride;
  // a window starting past the values holds nothing of any chain, and no window of its page that
  // does looks back at it (their bases come first); failed pages were flagged by k_scan
  if (!c.ok || Bw >= c.e0) return;
  const int64_t wb = ba_wbase(c, w);
  ba_stage(C, c, wb);
  __syncthreads();
  const DevChunk D = b.chunks[P.chunk];
  if (tid == 64) {  // k_scan's bases
    sh[4] = S.value_base;
    sh[5] = S.byte_base;
  }
  int64_t entry = c.entry;
  if (w > 0) {
    if (tid < 64) {
      const int32_t g = ba_guess_entry(C, int32_t(c.e0), int32_t(wb), int32_t(Bw));
      if (tid == 0) C.guess = g;
    }
    __syncthreads();
    entry = C.guess;
  }
  SegRecs sr;
  ba_window_segs(C, c, w, entry, &R, sr);
  __syncthreads();
  const int64_t value_base = sh[4], byte_base = sh[5];
  int64_t pincl = 0;
  bool pended = false;
  if (w > 0) {
    if (tid == 0) {  // PARTIAL
      const BaWin r0 = R;
      __hip_atomic_store(b.bawords + t,
                         kPartial | (r0.bad ? kBadBit : 0) | (uint64_t(r0.count) << 48) |
                             (uint64_t(entry - Bw) << 32) | uint64_t(uint32_t(r0.exit)),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (tid < 64) {
      int64_t pi = 0, pe = 0;
      bool en = false;
      if (!fuse_lookback(b, t, w, c.entry, &pi, &pe, &en)) {
        // no decisive look-back: the predecessor's FINAL
        uint64_t v = 0;
        if (tid == 0)
          for (int spin = 0;; spin++) {
            v = fuse_load(b.bawords + t - 1);
            if ((v >> 62) == 2) break;
            if (spin > kFuseSpinCap) {
              fuse_fail(b);
              v = kFinal | kBadBit;
              break;
            }
            __builtin_amdgcn_s_sleep(1);
          }
        v = __shfl(v, 0, 64);
        pi = int64_t((v >> 32) & uint64_t(kInclMax));
        pe = int64_t(uint32_t(v));
        en = (v & kBadBit) != 0;
      }
      if (tid == 0) {
        sh[1] = pi;
        sh[2] = pe;
        sh[3] = en;
      }
    }
    __syncthreads();
    pincl = sh[1];
    const int64_t pexit = sh[2];
    pended = sh[3] != 0;
    if (pended || pexit >= c.e0 || pexit >= wend) {
      // nothing of the chain starts here
      if (tid == 0) {
        const int bad = (!pended && pexit >= c.e0 && pexit < wend) ? PQH_ERR_EOF : 0;
        R = BaWin{int32_t(pexit), int32_t(pexit), 0, bad, 0, 0, 0, 0};
      }
      __syncthreads();
    } else if (pexit != entry) {
      // a wrong guess: resolve again from the true entry
      ba_window_segs(C, c, w, pexit, &R, sr);
      __syncthreads();
    }
  }
  const BaWin r = R;
  if (tid == 0) {
    int64_t incl = pincl + r.count;
    if (incl > kInclMax) incl = kInclMax;
    const bool ended = pended || r.bad != 0;
    __hip_atomic_store(b.bawords + t, kFinal | (ended ? kBadBit : 0) | (uint64_t(incl) << 32) | uint64_t(uint32_t(r.exit)),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (pended || pincl >= nn) return;
  // the window's records before the page's notNull: n of them, their bytes end at endo (the offset
  // of record n, or the window's byte total)
  const int n = int(nn - pincl < r.count ? nn - pincl : r.count);
  if (n < r.count) seg_list(sr, n, n + 1, reinterpret_cast<int64_t*>(sh) + 6);  // (uint16 offset, widened)
  __syncthreads();
  const int64_t endo = n < r.count ? int64_t(uint16_t(sh[6])) : r.bytes;
  if (tid == 0) {
    // the page's check: record nn ends at val_e, or the chain falls short of nn records
    if (pincl + r.count >= nn) {
      if (int64_t(r.entry) + 4 * int64_t(n) + endo != c.e0) fuse_fail(b);
    } else if (r.bad || r.exit >= c.e0) {
      fuse_fail(b);
    }
  }
  if (n == 0) return;
  // emit at the page's guessed byte base
  const int64_t obase = byte_base + (int64_t(r.entry) - c.entry) - 4 * pincl;
  if (obase < 0 || obase + endo > D.bytes_cap || value_base + pincl + n > D.values_cap) {
    if (tid == 0) fuse_fail(b);  // a wrong guess somewhere: never written, the batch goes again
    return;
  }
  // (wave-uniform bases in scalar registers: the stores below address them by 32-bit offsets)
  PQH_G int64_t* offs = uni_ptr(D.offsets + value_base + 1 + pincl);
  PQH_G uint8_t* dst = uni_ptr(D.bytes + obase);
  const int64_t obase_u = uni64(obase);
  const int lead = int(r.entry - wb);  // the entry in the stage
  constexpr int kStaged = kChainWin + 64;
  constexpr int kLong = 512;
  typedef uint32_t u32u __attribute__((aligned(1)));
  for (int base = 0; base < n; base += kChainList) {
    const int hi = n - base < kChainList ? n : base + kChainList;
    seg_list(sr, base, hi < n ? hi + 1 : hi, list);  // records base .. hi (record n's offset is endo)
    __syncthreads();
    for (int i = tid; i < hi - base; i += kBlock) {
      const int gi = base + i;
      const int o = list[i], e = gi + 1 < n ? int(list[i + 1]) : int(endo);  // (endo may pass 2^16)
      offs[uint32_t(gi)] = obase_u + e;
      const int l = e - o;
      const int sx = lead + 4 * (gi + 1) + o;
      if (l >= 4 && l <= 16 && sx + l + 20 <= kStaged) {
        // 4..16 bytes: four dword stores that overlap inside the string (no branch on the length)
        const int h = l >= 8 ? 4 : 0, t = l >= 8 ? l - 8 : l - 4;
        const uint32_t x0 = stage_dw(C.win, sx), x1 = stage_dw(C.win, sx + h), x2 = stage_dw(C.win, sx + t),
                       x3 = stage_dw(C.win, sx + l - 4);
        *reinterpret_cast<PQH_G u32u*>(dst + uint32_t(o)) = x0;
        *reinterpret_cast<PQH_G u32u*>(dst + uint32_t(o + h)) = x1;
        *reinterpret_cast<PQH_G u32u*>(dst + uint32_t(o + t)) = x2;
        *reinterpret_cast<PQH_G u32u*>(dst + uint32_t(o + l - 4)) = x3;
      } else if (sx + l + 20 <= kStaged) {
        stage_string_out(C.win, sx, l, dst + o);
      } else if (l > 0 && l < kLong) {
        copy_bytes(dst + o, c.img + r.entry + 4 * (gi + 1) + o, l);
      } else if (l >= kLong) {  // by the whole workgroup, below
        const int k = atomicAdd(&longs[3 * kChainLongs], 1);
        if (k < kChainLongs) {
          longs[3 * k] = gi;
          longs[3 * k + 1] = o;
          longs[3 * k + 2] = e;
        } else {
          fuse_fail(b);
        }
      }
    }
    __syncthreads();  // the list is read before the next pass writes it
  }
  // the long strings past the stage (at most the last few of the window) by the whole workgroup
  const int nl = longs[3 * kChainLongs] < kChainLongs ? longs[3 * kChainLongs] : kChainLongs;
  for (int k = 0; k < nl; k++) {
    const int gi = longs[3 * k], o = longs[3 * k + 1], e = longs[3 * k + 2];
    block_copy(dst + o, (const PQH_G uint8_t*)(c.img + r.entry + 4 * (gi + 1) + o), e - o);
  }
}
