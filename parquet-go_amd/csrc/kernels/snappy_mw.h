// snappy_mw.h — SNAPPY page decompression over many workgroups per page (SURVEY.md §8(f)3;
// included by decode.hip after snappy_impl.h).
//
// Same contract as k_snappy (golang/snappy v0.0.4 decode_other.go:36-124 + the reference's exact
// size check, compress.go:43-49,131-152), but a page is no longer one workgroup's sequential walk:
//
//   k_snap_spec   one workgroup per 4 KiB window of a page's compressed block.  The element chain
//                 (tags, literal bodies skipped) is resolved thread-parallel: every thread parses
//                 its 16-byte segment speculatively, starting kSnWarm bytes early so that its walk
//                 falls into step with the true chain before its segment begins; rounds then
//                 re-walk, from the exact entry, the first segment whose first element is not where
//                 the segment before it exits (sn_chain).  The window's first thread starts kSnWarm0
//                 bytes before the window (a guess, checked by the stitch).  Out: the window's first
//                 element, its exit, its output bytes, whether its chain meets a malformed element.
//   k_snap_stitch one workgroup per page: wave 0 chains the windows (a window whose guessed entry
//                 is the previous window's exit is taken as is; the rare other one is parsed again
//                 from the true entry by the workgroup), giving every window its true entry and its
//                 output base; the header length, the element structure, the total and the input
//                 end decide the page's status.  DataPageV2 level bytes are copied here.
//   k_snap_emit   one 512-thread workgroup per 64 KiB of a page's output (a "unit", snappy_emit.h):
//                 from the last window whose output base is at or before the unit, window by
//                 window, every thread walks its 16-byte segment from the exact entry the spec /
//                 stitch kept for it (wseg), literal bytes go straight into the unit's LDS image,
//                 copies are listed and resolved in spans of 16 KiB (each copy byte chases its source
//                 through the span's copy map; pointer jumping finishes long chains).  The unit is
//                 written to HBM once, with 16-byte stores.
//                 golang/snappy and C++ snappy encode 64 KiB fragments independently
//                 (snappy encode.go:22-32 maxBlockSize; snappy.cc kBlockSize), so their copies
//                 never reach before a unit; a copy that does (any other encoder) marks the unit.
//   k_snap_fixup  one workgroup per page: the marked units of the page again, in order, with
//                 sources before the unit read from the image in HBM (every earlier unit is final).
#pragma once

#ifndef PQH_SN_WARM  // (experiments: -DPQH_SN_WARM=..., -DPQH_SN_WARM0=...)
#define PQH_SN_WARM 128
#endif
#ifndef PQH_SN_WARM0
#define PQH_SN_WARM0 256
#endif
constexpr int kSnWin = 4096;                 // compressed bytes per spec window
constexpr int kSnWarm0 = PQH_SN_WARM0;       // warm-up of a window's first thread (window > 0)
constexpr int kSnWarm = PQH_SN_WARM;         // warm-up of every other thread (spec windows, 16-byte segments)
constexpr int kSnUnit = 65536;               // output bytes per emit unit
constexpr int kSnSpan = 16384;               // output bytes per copy-resolution span
constexpr int kSnT = 1024;                   // emit / fixup threads (= window walkers)
constexpr int kSnSub = kSnT / kBlock;        // walker segments per spec thread
constexpr int kSnPer = kSnSpan / kSnT;       // span bytes per thread
constexpr int kSnMaxC = kSnWin / 2 + 16;     // copies starting in one window (a copy is >= 2 bytes)
constexpr int kSnLongLit = 1024;             // literals of more unit bytes are copied by the whole workgroup
constexpr int kSnShortLit = 32;              // literals of at most this many unit bytes: a thread each
constexpr int kSnMaxL = kSnWin / kSnLongLit + 4;  // (at most this many start in one window)
constexpr int kSnSpecStage = kSnWin + kSnWarm0 + 64;
constexpr int kSnSpecRounds = 12;            // a speculative window that needs more rounds (inside a long
                                             // literal, usually) is left to the stitch

// One element at stage offset o8 (>= 8 readable stage bytes from o8).
struct SnEl {
  int32_t hdr, off;
  int64_t len;
  bool lit;
};

__device__ __forceinline__ SnEl sn_el(const uint8_t* in, int32_t o8) {
  const uint32_t* in32 = reinterpret_cast<const uint32_t*>(in);
  const uint64_t w = ((uint64_t(in32[(o8 >> 2) + 1]) << 32) | in32[o8 >> 2]) >> (8 * (o8 & 3));
  const uint32_t tag = uint32_t(w & 0xff);
  SnEl e;
  e.off = 0;
  e.lit = (tag & 3) == 0;
  if (e.lit) {
    const uint32_t x = tag >> 2;
    if (x < 60) {
      e.hdr = 1;
      e.len = int64_t(x) + 1;
    } else {
      const int kb = int(x) - 59;
      e.hdr = 1 + kb;
      e.len = int64_t((w >> 8) & (kb == 4 ? 0xffffffffull : ((1ull << (8 * kb)) - 1))) + 1;
    }
  } else if ((tag & 3) == 1) {
    e.hdr = 2;
    e.len = 4 + ((tag >> 2) & 7);
    e.off = int32_t(((tag >> 5) << 8) | ((w >> 8) & 0xff));
  } else if ((tag & 3) == 2) {
    e.hdr = 3;
    e.len = 1 + (tag >> 2);
    e.off = int32_t((w >> 8) & 0xffff);
  } else {
    e.hdr = 5;
    e.len = 1 + (tag >> 2);
    const uint64_t ov = (w >> 8) & 0xffffffffull;
    e.off = ov > 0x7fffffffull ? 0x7fffffff : int32_t(ov);  // beyond any output position: invalid
  }
  return e;
}

// A walk over the elements from `start` while they start before `end` (and before the input end
// n); the ones from count_from on are counted: f = the first of them (or where the walk stopped),
// x = the position after the last (the exit), o = their output bytes, k = their copies.  st 2: an
// element whose header or literal body runs past the input (x = its position).  Before count_from
// (the warm-up) such an element restarts the walk at count_from.
struct SnRun {
  int32_t f, x, o, k, st;
};

__device__ __forceinline__ SnRun sn_run(const uint8_t* in, int32_t a0, int32_t n, int32_t start, int32_t count_from,
                                        int32_t end) {
  SnRun R;
  R.f = -1;
  R.o = 0;
  R.k = 0;
  R.st = 0;
  int32_t pos = start;
  while (pos < end && pos < n) {
    const SnEl e = sn_el(in, pos - a0);
    const int64_t nx = int64_t(pos) + e.hdr + (e.lit ? e.len : 0);
    const bool bad = nx > n;  // golang/snappy: "s > len(src)" / "length > len(src)-s" -> ErrCorrupt
    if (pos < count_from) {
      pos = bad ? count_from : int32_t(nx);
      continue;
    }
    if (R.f < 0) R.f = pos;
    if (bad) {
      R.st = 2;
      R.x = pos;
      return R;
    }
    R.o += int32_t(e.len);
    R.k += !e.lit;
    pos = int32_t(nx);
  }
  if (R.f < 0) R.f = pos;
  R.x = pos;
  return R;
}

template <int NT>
struct SnFix {
  int32_t f[NT], x[NT], o[NT], k[NT];
  uint8_t st[NT];
  int32_t wred[NT / 64];
  int32_t first_bad, u, rounds, unsettled;
};

__device__ __forceinline__ int32_t wave_min32(int32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int32_t y = __shfl_xor(v, o, 64);
    v = y < v ? y : v;
  }
  return v;
}

__device__ __forceinline__ int32_t wave_max32(int32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int32_t y = __shfl_xor(v, o, 64);
    v = y > v ? y : v;
  }
  return v;
}

// Exclusive max over the threads before (-1 for thread 0).
template <int NT>
__device__ __forceinline__ int32_t sn_block_excl_max(SnFix<NT>& F, int32_t v) {
  const int tid = threadIdx.x, lane = tid & 63;
  int32_t incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t y = __shfl_up(incl, o, 64);
    if (lane >= o) incl = y > incl ? y : incl;
  }
  if (lane == 63) F.wred[tid >> 6] = incl;
  __syncthreads();
  int32_t r = __shfl_up(incl, 1, 64);
  if (lane == 0) r = -1;
  for (int w = 0; w < (tid >> 6); w++) r = F.wred[w] > r ? F.wred[w] : r;
  __syncthreads();  // wred is reused
  return r;
}

// Exclusive sum over the threads before; *total = the sum over all.
template <int NT>
__device__ __forceinline__ int32_t sn_block_excl_sum(SnFix<NT>& F, int32_t v, int32_t* total) {
  const int tid = threadIdx.x;
  const uint32_t incl = wave_incl_scan32(uint32_t(v));
  if ((tid & 63) == 63) F.wred[tid >> 6] = int32_t(incl);
  __syncthreads();
  int32_t base = 0, all = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; w++) {
    const int32_t s = F.wred[w];
    if (w < (tid >> 6)) base += s;
    all += s;
  }
  __syncthreads();
  *total = all;
  return base + int32_t(incl) - v;
}

// The element chain over [lo, hi) per thread (segments in order, covering the range the first
// thread counts from): thread 0 walks from start0 counting from count0 (its walk is taken as the
// chain); every other thread warms up from max(lo - warm, floor), so that its walk (almost always)
// falls into step with the true chain before its segment begins.  Rounds then find the first thread
// u whose first element is not its predecessor's exit: threads before u follow the chain exactly, so
// u's true entry e is thread u-1's exit — threads from u whose segment ends at or before e have no
// element (a long literal passes over them), the one holding e walks again from it, the others keep
// their speculation.  A round fixes at least thread u; in practice a few rounds settle a stage.  On
// return (after a barrier) F holds every thread's exact run and F.first_bad the first thread whose
// run meets a malformed element (NT: none).
template <int NT>
__device__ void sn_chain(SnFix<NT>& F, const uint8_t* in, int32_t a0, int32_t n, int32_t lo, int32_t hi,
                         int32_t start0, int32_t count0, int32_t floor, int32_t warm, int max_rounds = NT) {
  const int tid = threadIdx.x;
  {
    const int32_t ws = lo - warm > floor ? lo - warm : floor;
    const SnRun R = tid == 0 ? sn_run(in, a0, n, start0, count0, hi) : sn_run(in, a0, n, ws, lo, hi);
    F.f[tid] = R.f;
    F.x[tid] = R.x;
    F.o[tid] = R.o;
    F.k[tid] = R.k;
    F.st[tid] = uint8_t(R.st);
  }
  if (tid == 0) {
    F.first_bad = NT;
    F.unsettled = 1;
  }
  for (int round = 0; round <= max_rounds; round++) {
    if (tid == 0) F.rounds = round;
    if (tid == 0) F.u = NT;
    __syncthreads();
    if (tid > 0 && (F.st[tid - 1] || F.f[tid] != F.x[tid - 1])) atomicMin(&F.u, tid);
    __syncthreads();
    const int32_t u = F.u;
    if (u == NT || F.st[u - 1]) {  // settled, or the chain meets a malformed element in thread u - 1
      if (tid == 0) {
        if (u < NT) F.first_bad = u - 1;
        F.unsettled = 0;
      }
      break;
    }
    if (round == max_rounds) break;  // (speculative windows: left to the stitch)
    const int32_t e = F.x[u - 1];
    __syncthreads();  // every thread has read this round's state
    if (tid >= u) {
      if (hi <= e) {
        F.f[tid] = e;
        F.x[tid] = e;
        F.o[tid] = 0;
        F.k[tid] = 0;
        F.st[tid] = 0;
      } else if (lo <= e) {
        const SnRun R = sn_run(in, a0, n, e, e, hi);
        F.f[tid] = R.f;
        F.x[tid] = R.x;
        F.o[tid] = R.o;
        F.k[tid] = R.k;
        F.st[tid] = uint8_t(R.st);
      }
    }
  }
  __syncthreads();
}

// uvarint decoded length (binary.Uvarint, at most 10 bytes; > 0xffffffff is ErrCorrupt).  Returns
// the header length, or 0 when malformed.
__device__ __forceinline__ int32_t sn_header(const uint8_t* src, int32_t n, uint64_t* v_out) {
  uint64_t v = 0;
  for (int i = 0; i < 10 && i < n; i++) {
    const uint8_t c = src[i];
    if (i == 9 && c > 1) return 0;
    v |= uint64_t(c & 0x7f) << (7 * i);
    if (c < 0x80) {
      if (v > 0xffffffffull) return 0;
      *v_out = v;
      return i + 1;
    }
  }
  return 0;
}

struct __attribute__((aligned(16))) SnSpecLds {
  uint8_t in[kSnSpecStage];
  SnFix<kBlock> F;
  int16_t sub[kSnSub * kBlock];  // walker segment entries (sn_window)
  int32_t c_mis, c_e, c_O, c_bad;
};

// Window wi of a block src[0, n) with header length hl, its chain from `entry` (exact) or guessed
// (entry < 0): the window's first element, exit, output bytes and status (st 2: malformed).
__device__ int4 sn_window(SnSpecLds& L, const uint8_t* src, int32_t n, int32_t hl, int32_t wi, int32_t entry) {
  const int tid = threadIdx.x;
  const int32_t ws = wi * kSnWin > hl ? wi * kSnWin : hl;
  const int32_t we = (wi + 1) * kSnWin < n ? (wi + 1) * kSnWin : n;
  const bool exact = entry >= 0;
  const int32_t floor = exact ? entry : (wi == 0 ? hl : (ws - kSnWarm0 > hl ? ws - kSnWarm0 : hl));
  const int32_t a0 = floor - int32_t((reinterpret_cast<uintptr_t>(src) + uintptr_t(floor)) & 15);
  __syncthreads();  // earlier readers of the stage are done
  {  // the stage: [a0, we + 16) rounded to 16 bytes (inside the payload pad past n)
    const uint4* sp = reinterpret_cast<const uint4*>(src + a0);
    uint4* lp = reinterpret_cast<uint4*>(L.in);
    const int32_t nu = (we + 16 - a0 + 15) >> 4;
    for (int u = tid; u < nu; u += kBlock) lp[u] = sp[u];
  }
  __syncthreads();
  const int32_t span = we > ws ? we - ws : 0;
  // thread segments of kSnSub walker segments each (the emit units walk the window with one
  // walker per kSnT thread, from the entries this window leaves behind)
  const int32_t S4 = (span + kSnT - 1) / kSnT, S = kSnSub * S4;
  const int32_t lo = ws + (S * tid < span ? S * tid : span);
  const int32_t hi = ws + (S * (tid + 1) < span ? S * (tid + 1) : span);
  const int32_t count0 = exact ? entry : ws;
  sn_chain<kBlock>(L.F, L.in, a0, n, lo, hi, floor, count0, floor, kSnWarm, exact ? kBlock : kSnSpecRounds);
  int32_t osum;
  sn_block_excl_sum<kBlock>(L.F, L.F.o[tid], &osum);
  const int32_t fb = L.F.first_bad;
  int4 r;
  r.x = L.F.f[0];
  r.y = fb < kBlock ? L.F.x[fb] : L.F.x[kBlock - 1];
  r.z = osum;
  r.w = L.F.unsettled ? 3 : (fb < kBlock ? 2 : 0);
  {  // every walker segment's first element (window-relative; we - ws: none in the window)
    int32_t q = L.F.f[tid];
#pragma unroll
    for (int k = 0; k < kSnSub; k++) {
      const int32_t b = lo + k * S4 < hi ? lo + k * S4 : hi;
      while (q < b && q < n && q < hi) {
        const SnEl e = sn_el(L.in, q - a0);
        const int64_t nx = int64_t(q) + e.hdr + (e.lit ? e.len : 0);
        q = nx > n ? n : int32_t(nx);
      }
      L.sub[kSnSub * tid + k] = int16_t((q < we ? q : we) - ws);
    }
  }
  return r;
}

__global__ __launch_bounds__(256) void k_snap_spec(const pqh_codec_page* cps, const int32_t* win_page,
                                                   const int32_t* page_win0, const uint8_t* src_all, int4* wspec,
                                                   int16_t* wseg) {
  __shared__ SnSpecLds L;
  const int32_t w = blockIdx.x;
  const int32_t p = win_page[w];
  const pqh_codec_page cp = cps[p];
  const int32_t raw = cp.raw_len < cp.src_len ? cp.raw_len : cp.src_len;
  const uint8_t* src = src_all + cp.src_offset + raw;
  const int32_t n = cp.src_len - raw;
  uint64_t v;
  const int32_t hl = sn_header(src, n, &v);
  if (hl == 0) {  // the stitch fails the page
    if (threadIdx.x == 0) wspec[w] = make_int4(-1, -1, 0, 2);
    return;
  }
  const int4 r = sn_window(L, src, n, hl, w - page_win0[p], -1);
  if (threadIdx.x == 0) wspec[w] = r;
  // exact when the stitch accepts the guess
  reinterpret_cast<uint2*>(wseg + int64_t(w) * kSnT)[threadIdx.x] = reinterpret_cast<const uint2*>(L.sub)[threadIdx.x];
}

// Per page: status, true window entries / output bases, V2 level bytes.
__global__ __launch_bounds__(256) void k_snap_stitch(const pqh_codec_page* cps, const int32_t* page_win0,
                                                     const int32_t* page_mode, const uint8_t* src_all, uint8_t* dst_all, const int4* wspec,
                                                     int2* wtrue, int16_t* wseg, int32_t* status) {
  __shared__ SnSpecLds L;
  const int tid = threadIdx.x, lane = tid & 63;
  const int32_t p = blockIdx.x;
  const pqh_codec_page cp = cps[p];
  if (cp.codec == PQH_CODEC_GZIP || page_mode[p]) return;  // k_gzip's / k_snappy's
  if (cp.codec != PQH_CODEC_SNAPPY) {       // a plain copy (k_snap_emit's units)
    if (tid == 0) status[p] = cp.src_len == cp.image_len ? PQH_OK : PQH_ERR_DECOMPRESS;
    return;
  }
  uint8_t* dst = dst_all + cp.image_offset;
  const int32_t raw = cp.raw_len < cp.src_len ? cp.raw_len : cp.src_len;
  snap_copy(dst, src_all + cp.src_offset, raw < cp.image_len ? raw : cp.image_len);  // DataPageV2 levels
  const uint8_t* src = src_all + cp.src_offset + raw;
  const int32_t n = cp.src_len - raw;
  uint64_t v = 0;
  const int32_t hl = raw > cp.image_len ? 0 : sn_header(src, n, &v);
  const int32_t total = cp.image_len - raw;
  if (hl == 0 || int64_t(v) != int64_t(total)) {
    if (tid == 0) status[p] = PQH_ERR_DECOMPRESS;
    return;
  }
  const int32_t w0 = page_win0[p], nw = page_win0[p + 1] - w0;
  int32_t e = hl, O = 0, c = 0;
  bool bad = false;
  while (c < nw) {
    if (tid < 64) {  // wave 0 chains up to 64 windows, stopping at the first wrong guess
      const int32_t w = c + lane;
      int4 r = make_int4(0, 0, 0, 0);
      int32_t we = 0;
      if (w < nw) {
        r = wspec[w0 + w];
        we = (w + 1) * kSnWin < n ? (w + 1) * kSnWin : n;
      }
      const int m = nw - c < 64 ? nw - c : 64;
      int32_t my_e = 0, my_O = 0, stop = m, found = 0;
      for (int j = 0; j < m; j++) {
        const int32_t fj = __builtin_amdgcn_readlane(r.x, j), xj = __builtin_amdgcn_readlane(r.y, j);
        const int32_t oj = __builtin_amdgcn_readlane(r.z, j), sj = __builtin_amdgcn_readlane(r.w, j);
        const int32_t wej = __builtin_amdgcn_readlane(we, j);
        if (lane == j) {
          my_e = e;
          my_O = O;
        }
        if (e >= wej) continue;  // no element starts in this window (a long literal spans it)
        if (e != fj || sj) {     // a wrong guess, or the true chain meets a malformed element
          stop = j;
          found = e == fj && sj == 2 ? 2 : 1;  // (3: the window's speculation did not settle)
          break;
        }
        O += oj;
        e = xj;
      }
      if (lane < stop && w < nw) wtrue[w0 + w] = make_int2(my_e, my_O);
      if (lane == 0) {
        L.c_mis = stop;
        L.c_bad = found;
        L.c_e = e;
        L.c_O = O;
      }
    }
    __syncthreads();
    const int32_t stop = L.c_mis, found = L.c_bad;
    e = L.c_e;
    O = L.c_O;
    __syncthreads();
    if (found == 2) {
      bad = true;
      break;
    }
    c += stop;
    if (found == 1) {  // window c guessed its entry wrong: parse it from the true entry
      const int4 r = sn_window(L, src, n, hl, c, e);
      if (tid == 0) wtrue[w0 + c] = make_int2(e, O);
      reinterpret_cast<uint2*>(wseg + int64_t(w0 + c) * kSnT)[tid] = reinterpret_cast<const uint2*>(L.sub)[tid];
      if (r.w) {
        bad = true;
        break;
      }
      O += r.z;
      e = r.y;
      c += 1;
    }
  }
  if (tid == 0) status[p] = (!bad && e == n && O == total) ? PQH_OK : PQH_ERR_DECOMPRESS;
}

// The emit / fixup kernels: snappy_emit.h.
