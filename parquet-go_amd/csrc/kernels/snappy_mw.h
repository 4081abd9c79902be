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
//   k_snap_emit   one 512-thread workgroup per 64 KiB of a page's output (a "unit"): from the last
//                 window starting at or before the unit, its elements are parsed again stage by
//                 stage (same thread-parallel parse from an exact entry), literal bytes go straight
//                 into the unit's LDS image, copies are listed and resolved in spans of 16 KiB by
//                 an output-byte -> copy map and pointer jumping over the span (sources before the
//                 span are already final in LDS).  The unit is written to HBM once, 16-byte stores.
//                 golang/snappy and C++ snappy encode 64 KiB fragments independently
//                 (snappy encode.go:22-32 maxBlockSize; snappy.cc kBlockSize), so their copies
//                 never reach before a unit; a copy that does (any other encoder) marks the unit.
//   k_snap_fixup  one workgroup per page: the marked units of the page again, in order, with
//                 sources before the unit read from the image in HBM (every earlier unit is final).
#pragma once

constexpr int kSnWin = 4096;                 // compressed bytes per spec window
constexpr int kSnWarm0 = 256;                // warm-up of a window's first thread (window > 0)
constexpr int kSnWarm = 128;                 // warm-up of every other thread (spec windows, 16-byte segments)
constexpr int kSnWarmE = 160;                // (emit stages, 8-byte segments)
constexpr int kSnUnit = 65536;               // output bytes per emit unit
constexpr int kSnStage = 4096;               // compressed bytes parsed per emit stage
constexpr int kSnSpan = 16384;               // output bytes per copy-resolution span
constexpr int kSnT = 512;                    // emit / fixup threads
constexpr int kSnPer = kSnSpan / kSnT;       // span bytes per thread
constexpr int kSnMaxC = kSnStage / 2 + 16;   // copies starting in one stage (a copy is >= 2 bytes)
constexpr int kSnMaxL = kSnStage / 64 + 4;   // literals of > 64 unit bytes starting in one stage
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
  const int32_t S = (span + kBlock - 1) / kBlock;
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
  return r;
}

__global__ __launch_bounds__(256) void k_snap_spec(const pqh_codec_page* cps, const int32_t* win_page,
                                                   const int32_t* page_win0, const uint8_t* src_all, int4* wspec,
                                                   int32_t* wseg) {
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
  wseg[int64_t(w) * kBlock + threadIdx.x] = L.F.f[threadIdx.x];  // exact when the stitch accepts the guess
}

// Per page: status, true window entries / output bases, V2 level bytes.
__global__ __launch_bounds__(256) void k_snap_stitch(const pqh_codec_page* cps, const int32_t* page_win0,
                                                     const uint8_t* src_all, uint8_t* dst_all, const int4* wspec,
                                                     int2* wtrue, int32_t* wseg, int32_t* status) {
  __shared__ SnSpecLds L;
  const int tid = threadIdx.x, lane = tid & 63;
  const int32_t p = blockIdx.x;
  const pqh_codec_page cp = cps[p];
  if (cp.codec == PQH_CODEC_GZIP) return;  // k_gzip's
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
      wseg[int64_t(w0 + c) * kBlock + tid] = L.F.f[tid];
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

struct __attribute__((aligned(16))) SnEmitLds {
  uint8_t out[kSnUnit + 64];  // the unit's image
  uint8_t in[kSnStage + 64];  // the stage: block bytes [a0, send + 16)
  uint16_t emap[kSnSpan];     // span byte -> copy (1-based); then (as int16) the byte's pointer
  int32_t cs[kSnMaxC];        // the stage's copies: output start (unit-relative), offset, unit bytes
  int32_t co[kSnMaxC];
  uint8_t cl[kSnMaxC];
  int32_t l_out[kSnMaxL], l_src[kSnMaxL], l_len[kSnMaxL];  // literals of > 64 unit bytes
  SnFix<kSnT> F;
  int32_t nlong, bad, ext, cut, tmax, win;
#ifdef PQH_SNAP_PROF  // timing experiments: clock64() per phase, printed for the first unit
  uint64_t prof[12];
#endif
};

// n bytes from src to dst (global, any alignment) by kSnT threads.
__device__ __forceinline__ void sn_gcopy(uint8_t* dst, const uint8_t* src, int64_t n) {
  const int tid = threadIdx.x;
  const int64_t head0 = int64_t((16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15);
  const int64_t head = head0 < n ? head0 : n;
  if (tid < head) dst[tid] = src[tid];
  typedef uint4 uint4_u __attribute__((aligned(1)));
  const int64_t units = (n - head) >> 4;
  const uint4_u* sp = reinterpret_cast<const uint4_u*>(src + head);
  uint4* dp = reinterpret_cast<uint4*>(dst + head);
  for (int64_t u = tid; u < units; u += kSnT) dp[u] = sp[u];
  const int64_t done = head + units * 16;
  if (tid < n - done) dst[done + tid] = src[done + tid];
}

// The stage's K copies (unit-relative output start cs, offset co, length cl, 0 when the copy has
// no byte in the unit; in output order) resolved into L.out, span by span: each span byte is a literal / gap byte (final in L.out),
// a copy byte whose source precedes the span (final in L.out, or before the unit: read from
// dst_unit in ext mode, else the unit is marked) or a pointer to an earlier span byte; pointer
// jumping then resolves every chain in O(log length) rounds.
__device__ void sn_copies(SnEmitLds& L, int32_t K, int32_t U0, int32_t ulen, bool ext, const uint8_t* dst_unit) {
  const int tid = threadIdx.x;
  int32_t i = 0;
  while (i < K) {
    const int32_t c0 = L.cs[i];
    const int32_t B0 = c0 < 0 ? 0 : (c0 > ulen ? ulen : c0);
    __syncthreads();  // the previous span's readers are done
    if (tid == 0) {
      L.cut = K;
      L.tmax = 0;
    }
    {
      uint4* m4 = reinterpret_cast<uint4*>(L.emap) + tid * (kSnPer / 8);
#pragma unroll
      for (int k = 0; k < kSnPer / 8; k++) m4[k] = make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    {
      int32_t cut = K;
      for (int32_t j = i + tid; j < K; j += kSnT) {
        const int32_t e = L.cs[j] + L.cl[j] < ulen ? L.cs[j] + L.cl[j] : ulen;
        if (e - B0 > kSnSpan) {
          cut = j;
          break;  // (starts rise with j)
        }
      }
      cut = wave_min32(cut);
      if ((tid & 63) == 0 && cut < K) atomicMin(&L.cut, cut);
    }
    __syncthreads();
    const int32_t i1 = L.cut;
    {
      int32_t tm = 0;
      for (int32_t j = i + tid; j < i1; j += kSnT) {
        if (!L.cl[j]) continue;
        const int32_t s = L.cs[j] > 0 ? L.cs[j] : 0;
        const int32_t e = L.cs[j] + L.cl[j] < ulen ? L.cs[j] + L.cl[j] : ulen;
        L.emap[s - B0] = uint16_t(j - i + 1);
        tm = e - B0 > tm ? e - B0 : tm;
      }
      tm = wave_max32(tm);
      if ((tid & 63) == 0 && tm > 0) atomicMax(&L.tmax, tm);
    }
    __syncthreads();
    const int32_t T = L.tmax;
    {  // max-scan: every thread owns kSnPer consecutive entries
      uint4* m4 = reinterpret_cast<uint4*>(L.emap) + tid * (kSnPer / 8);
      uint32_t wv[kSnPer / 2];
#pragma unroll
      for (int k = 0; k < kSnPer / 8; k++) {
        const uint4 x = m4[k];
        wv[4 * k] = x.x;
        wv[4 * k + 1] = x.y;
        wv[4 * k + 2] = x.z;
        wv[4 * k + 3] = x.w;
      }
      uint32_t mx = 0;
#pragma unroll
      for (int k = 0; k < kSnPer / 2; k++) {
        const uint32_t a = wv[k] & 0xffff, c = wv[k] >> 16;
        mx = a > mx ? a : mx;
        mx = c > mx ? c : mx;
      }
      const int32_t run0 = sn_block_excl_max<kSnT>(L.F, int32_t(mx));
      uint32_t run = run0 < 0 ? 0u : uint32_t(run0);
#pragma unroll
      for (int k = 0; k < kSnPer / 2; k++) {
        uint32_t a = wv[k] & 0xffff, c = wv[k] >> 16;
        run = a > run ? a : run;
        a = run;
        run = c > run ? c : run;
        c = run;
        wv[k] = a | (c << 16);
      }
#pragma unroll
      for (int k = 0; k < kSnPer / 8; k++) m4[k] = make_uint4(wv[4 * k], wv[4 * k + 1], wv[4 * k + 2], wv[4 * k + 3]);
    }
    __syncthreads();
    int16_t ptr[kSnPer];
    uint8_t val[kSnPer];
#pragma unroll
    for (int q = 0; q < kSnPer; q++) {
      const int32_t b = q * kSnT + tid;
      ptr[q] = -1;
      val[q] = 0;
      if (b >= T) continue;
      const int32_t pos = B0 + b;
      const int e = L.emap[b];
      const int32_t j = i + e - 1;
      if (e == 0 || pos >= L.cs[j] + L.cl[j]) {
        val[q] = L.out[pos];  // a literal byte (or a byte of an earlier copy of the stage's first span... final)
        continue;
      }
      const int32_t cs = L.cs[j], o = L.co[j];
      const int32_t rel = pos - cs;
      if (o <= 0) continue;  // (a copy of offset 0 fails the unit that owns it)
      const int32_t s = cs - o + (o < L.cl[j] ? rel % o : rel);  // overlapping copies repeat
      if (s >= B0) {
        ptr[q] = int16_t(s - B0);
      } else if (s >= 0) {
        val[q] = L.out[s];
      } else if (ext) {
        if (U0 + s >= 0) val[q] = dst_unit[s];  // (before the output start: its owner failed the page)
      } else {
        L.ext = 1;
      }
    }
    __syncthreads();  // emap no longer read: it becomes the pointer array
    int16_t* P = reinterpret_cast<int16_t*>(L.emap);
#pragma unroll
    for (int q = 0; q < kSnPer; q++) {
      const int32_t b = q * kSnT + tid;
      if (b < T) {
        P[b] = ptr[q];
        L.out[B0 + b] = val[q];
      }
    }
    __syncthreads();
    for (;;) {
      int pending = 0;
#pragma unroll
      for (int q = 0; q < kSnPer; q++) {
        if (ptr[q] < 0) continue;
        const int16_t t = P[ptr[q]];
        if (t < 0) val[q] = L.out[B0 + ptr[q]];
        else pending = 1;
        ptr[q] = t;
      }
      const int more = __syncthreads_or(pending);
#ifdef PQH_SNAP_PROF
      if (tid == 0) L.prof[10] += 1;
#endif
#pragma unroll
      for (int q = 0; q < kSnPer; q++) {
        const int32_t b = q * kSnT + tid;
        if (b < T) {
          P[b] = ptr[q];
          L.out[B0 + b] = val[q];
        }
      }
      __syncthreads();
      if (!more) break;
    }
#ifdef PQH_SNAP_PROF
    if (tid == 0) L.prof[11] += 1;
#endif
    i = i1;
  }
}

// One unit [U0, U1) of a SNAPPY block's output: block src[0, n), output at dst (after the raw
// prefix), true window entries / bases wt[0, nw).  Returns whether a copy reached before the unit
// (not in ext mode, where such sources are read from dst); *bad: a copy of offset 0 or before the
// output start (golang/snappy decode_other.go:104-106).
__device__ bool sn_unit(SnEmitLds& L, const uint8_t* src, int32_t n, uint8_t* dst, int32_t U0, int32_t U1,
                        const int2* wt, int32_t nw, bool ext, bool* bad) {
  const int tid = threadIdx.x;
  const int32_t ulen = U1 - U0;
  __syncthreads();  // an earlier unit's readers of L are done
  if (tid == 0) {  // the last window whose true output base is at or before U0 (wt[0].y == 0)
    int32_t lo = 0, hi = nw - 1;
    while (lo < hi) {
      const int32_t mid = (lo + hi + 1) >> 1;
      if (wt[mid].y <= U0) lo = mid;
      else hi = mid - 1;
    }
    L.win = lo;
    L.bad = 0;
    L.ext = 0;
  }
  __syncthreads();
  const int2 w = wt[L.win];
  int32_t pos = w.x, o = w.y;
#ifdef PQH_SNAP_PROF
  if (tid < 12) L.prof[tid] = 0;
  uint64_t t0 = clock64();
#define SN_T(i) do { __syncthreads(); const uint64_t t1 = clock64(); if (tid == 0) L.prof[i] += t1 - t0; t0 = t1; } while (0)
#else
#define SN_T(i) do {} while (0)
#endif
  while (pos < n && o < U1) {
    const int32_t a0 = pos - int32_t((reinterpret_cast<uintptr_t>(src) + uintptr_t(pos)) & 15);
    const int32_t send = a0 + kSnStage < n ? a0 + kSnStage : n;
    __syncthreads();  // the previous stage's readers are done
    {
      const uint4* sp = reinterpret_cast<const uint4*>(src + a0);
      uint4* lp = reinterpret_cast<uint4*>(L.in);
      const int32_t nu = (send + 16 - a0 + 15) >> 4;
      for (int u = tid; u < nu; u += kSnT) lp[u] = sp[u];
    }
    if (tid == 0) L.nlong = 0;
    __syncthreads();
    const int32_t span = send - pos;
    const int32_t S = (span + kSnT - 1) / kSnT;
    const int32_t lo = pos + (S * tid < span ? S * tid : span);
    const int32_t hi = pos + (S * (tid + 1) < span ? S * (tid + 1) : span);
    SN_T(0);
    sn_chain<kSnT>(L.F, L.in, a0, n, lo, hi, pos, pos, pos, kSnWarmE);
    SN_T(1);
#ifdef PQH_SNAP_PROF
    if (tid == 0) L.prof[9] += L.F.rounds;
#endif
    if (L.F.first_bad < kSnT) {  // (the stitch accepted this chain: cannot happen)
      *bad = true;
      return false;
    }
    int32_t Ot, Kt;
    const int32_t ob = o + sn_block_excl_sum<kSnT>(L.F, L.F.o[tid], &Ot);
    const int32_t kb = sn_block_excl_sum<kSnT>(L.F, L.F.k[tid], &Kt);
    const int32_t stage_hi = send + 16;
    {
      int32_t q = L.F.f[tid], P = ob, k = kb;
      while (q < hi && P < U1) {
        const SnEl e = sn_el(L.in, q - a0);
        const int32_t len = int32_t(e.len);
        if (e.lit) {
          const int32_t body = q + e.hdr;
          const int32_t b0 = P > U0 ? P : U0, b1 = P + len < U1 ? P + len : U1;
          if (b0 < b1) {
            if (b1 - b0 <= 64) {
              for (int32_t b = b0; b < b1; b++) {
                const int32_t s = body + (b - P);
                L.out[b - U0] = s < stage_hi ? L.in[s - a0] : src[s];
              }
            } else {
              const int32_t li = atomicAdd(&L.nlong, 1);
              L.l_out[li] = b0 - U0;
              L.l_src[li] = body + (b0 - P);
              L.l_len[li] = b1 - b0;
            }
          }
          q = body + len;
        } else {
          if (P >= U0 && (e.off == 0 || e.off > P)) L.bad = 1;
          L.cs[k] = P - U0;
          L.co[k] = e.off;
          L.cl[k] = P + len > U0 ? uint8_t(len) : 0;  // (P < U1 here)
          k++;
          q += e.hdr;
        }
        P += len;
      }
      for (; k < kb + L.F.k[tid]; k++) {  // copies past the unit
        L.cs[k] = ulen;
        L.co[k] = 1;
        L.cl[k] = 0;
      }
    }
    __syncthreads();
    if (L.bad) {
      *bad = true;
      return false;
    }
    SN_T(2);
    for (int32_t li = 0; li < L.nlong; li++) {
      const int32_t lo2 = L.l_out[li], ls = L.l_src[li], ln = L.l_len[li];
      for (int32_t j = tid; j < ln; j += kSnT) L.out[lo2 + j] = src[ls + j];
    }
    o += Ot;
    pos = L.F.x[kSnT - 1];
    SN_T(3);
    sn_copies(L, Kt, U0, ulen, ext, dst + U0);
    SN_T(4);
#ifdef PQH_SNAP_PROF
    if (tid == 0) L.prof[8] += 1;
#endif
  }
  __syncthreads();
  {  // the unit to HBM: bytes until the destination is 16-byte aligned, then 16-byte stores
    uint8_t* g = dst + U0;
    const int32_t head0 = int32_t((16 - (reinterpret_cast<uintptr_t>(g) & 15)) & 15);
    const int32_t head = head0 < ulen ? head0 : ulen;
    if (tid < head) g[tid] = L.out[tid];
    const int32_t units = (ulen - head) >> 4;
    const uint32_t* o32 = reinterpret_cast<const uint32_t*>(L.out);
    const int32_t sh = 8 * (head & 3);
    for (int32_t u = tid; u < units; u += kSnT) {
      const int32_t wb = (head + 16 * u) >> 2;
      uint32_t v[4];
      if (sh == 0) {
#pragma unroll
        for (int t = 0; t < 4; t++) v[t] = o32[wb + t];
      } else {
        uint32_t x[5];
#pragma unroll
        for (int t = 0; t < 5; t++) x[t] = o32[wb + t];
#pragma unroll
        for (int t = 0; t < 4; t++) v[t] = __builtin_amdgcn_alignbit(x[t + 1], x[t], uint32_t(sh));
      }
      *reinterpret_cast<uint4*>(g + head + 16 * u) = make_uint4(v[0], v[1], v[2], v[3]);
    }
    const int32_t done = head + units * 16;
    if (tid < ulen - done) g[done + tid] = L.out[done + tid];
  }
  SN_T(5);
#ifdef PQH_SNAP_PROF
  if (tid == 0 && blockIdx.x < 2)
    printf("snapprof unit %d stages %lu | cycles: load %lu chain %lu walk %lu long %lu copies %lu store %lu | rounds %lu jumps %lu spans %lu\n",
           int(blockIdx.x), L.prof[8], L.prof[0], L.prof[1], L.prof[2], L.prof[3], L.prof[4], L.prof[5], L.prof[9], L.prof[10], L.prof[11]);
#endif
  return L.ext != 0;
}

__global__ __launch_bounds__(kSnT) void k_snap_emit(const pqh_codec_page* cps, const int32_t* unit_page,
                                                    const int32_t* page_unit0, const int32_t* page_win0,
                                                    const uint8_t* src_all, uint8_t* dst_all, const int2* wtrue,
                                                    int32_t* status, int32_t* uflag) {
  __shared__ SnEmitLds L;
  const int32_t u = blockIdx.x;
  const int32_t p = unit_page[u];
  const int32_t k = u - page_unit0[p];
  const pqh_codec_page cp = cps[p];
  uint8_t* dst = dst_all + cp.image_offset;
  if (cp.codec != PQH_CODEC_SNAPPY) {  // a plain copy, unit by unit
    const int64_t len = cp.src_len < cp.image_len ? cp.src_len : cp.image_len;
    const int64_t U0 = int64_t(k) * kSnUnit;
    const int64_t m = len - U0 < kSnUnit ? len - U0 : kSnUnit;
    if (m > 0) sn_gcopy(dst + U0, src_all + cp.src_offset + U0, m);
    return;
  }
  if (status[p] != PQH_OK) {
    if (threadIdx.x == 0) uflag[u] = 0;
    return;
  }
  const int32_t raw = cp.raw_len < cp.src_len ? cp.raw_len : cp.src_len;
  const int32_t total = cp.image_len - raw;
  const int32_t U0 = k * kSnUnit, U1 = U0 + kSnUnit < total ? U0 + kSnUnit : total;
  bool bad = false;
  const bool ext = sn_unit(L, src_all + cp.src_offset + raw, cp.src_len - raw, dst + raw, U0, U1,
                           wtrue + page_win0[p], page_win0[p + 1] - page_win0[p], false, &bad);
  if (threadIdx.x == 0) {
    uflag[u] = ext && !bad;
    if (bad) status[p] = PQH_ERR_DECOMPRESS;
  }
}

// The units a copy before the unit marked, again in order, their early sources read from HBM.
__global__ __launch_bounds__(kSnT) void k_snap_fixup(const pqh_codec_page* cps, const int32_t* page_unit0,
                                                     const int32_t* page_win0, const uint8_t* src_all,
                                                     uint8_t* dst_all, const int2* wtrue, int32_t* status,
                                                     const int32_t* uflag) {
  __shared__ SnEmitLds L;
  const int32_t p = blockIdx.x;
  const pqh_codec_page cp = cps[p];
  if (cp.codec != PQH_CODEC_SNAPPY || status[p] != PQH_OK) return;
  const int32_t u0 = page_unit0[p], u1 = page_unit0[p + 1];
  const int32_t raw = cp.raw_len < cp.src_len ? cp.raw_len : cp.src_len;
  const int32_t total = cp.image_len - raw;
  for (int32_t u = u0; u < u1; u++) {
    if (!uflag[u]) continue;
    const int32_t U0 = (u - u0) * kSnUnit, U1 = U0 + kSnUnit < total ? U0 + kSnUnit : total;
    bool bad = false;
    sn_unit(L, src_all + cp.src_offset + raw, cp.src_len - raw, dst_all + cp.image_offset + raw, U0, U1,
            wtrue + page_win0[p], page_win0[p + 1] - page_win0[p], true, &bad);
    __threadfence();
    if (bad) {
      if (threadIdx.x == 0) status[p] = PQH_ERR_DECOMPRESS;
      return;
    }
  }
}
