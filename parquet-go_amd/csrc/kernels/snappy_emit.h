// snappy_emit.h — the output half of the multi-workgroup SNAPPY decoder (k_snap_emit /
// k_snap_fixup; included by decode.hip after snappy_mw.h, whose window tables it reads).
#pragma once

struct __attribute__((aligned(16))) SnEmitLds {
  uint8_t out[kSnUnit + 64];  // the unit's image
  uint8_t in[kSnWin + 64];    // the stage: block bytes [a0, we + 16) of one window
  uint16_t emap[kSnSpan];     // span byte -> copy (1-based)
  int16_t ptr[kSnSpan];       // span byte -> the span byte it copies (-1: final in out)
  uint32_t cbit[kSnSpan / 32];  // the span's copy bytes
  int2 cp[kSnMaxC];           // the window's copies: output start (unit-relative) | offset (clamped to
                              // 2^24 - 1: any larger one reaches before the unit) + length << 24
  int32_t l_out[kSnMaxL], l_src[kSnMaxL], l_len[kSnMaxL];  // literals of > 64 unit bytes
  int32_t wred[kSnT / 64];
  int32_t nlong, nmed, bad, ext, cut, tmax, win;
#ifdef PQH_SNAP_PROF  // timing experiments: clock64() per phase, printed for the first units
  uint64_t prof[12];
#endif
};

__device__ __forceinline__ int32_t sn_excl_sum(SnEmitLds& L, int32_t v, int32_t* total) {
  const int tid = threadIdx.x;
  const uint32_t incl = wave_incl_scan32(uint32_t(v));
  if ((tid & 63) == 63) L.wred[tid >> 6] = int32_t(incl);
  __syncthreads();
  int32_t base = 0, all = 0;
#pragma unroll
  for (int w = 0; w < kSnT / 64; w++) {
    const int32_t x = L.wred[w];
    if (w < (tid >> 6)) base += x;
    all += x;
  }
  __syncthreads();
  *total = all;
  return base + int32_t(incl) - v;
}

__device__ __forceinline__ int32_t sn_excl_max(SnEmitLds& L, int32_t v) {
  const int tid = threadIdx.x, lane = tid & 63;
  int32_t incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t y = __shfl_up(incl, o, 64);
    if (lane >= o) incl = y > incl ? y : incl;
  }
  if (lane == 63) L.wred[tid >> 6] = incl;
  __syncthreads();
  int32_t r = __shfl_up(incl, 1, 64);
  if (lane == 0) r = -1;
  for (int w = 0; w < (tid >> 6); w++) r = L.wred[w] > r ? L.wred[w] : r;
  __syncthreads();
  return r;
}

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

// The window's K copies (unit-relative output start cs, offset co, length cl, 0 when the copy has
// no byte in the unit; in output order) resolved into L.out, span by span: an output-byte -> copy
// map (start markers, max-scan) gives every copy byte its source; sources before the span (final
// in L.out; before the unit: an earlier unit's bytes, read from dst_unit in ext mode, else the unit
// is marked) and literal bytes resolve at once, the rest by pointer jumping over the span.
__device__ void sn_copies(SnEmitLds& L, int32_t K, int32_t U0, int32_t ulen, bool ext, const uint8_t* dst_unit) {
  const int tid = threadIdx.x;
  int32_t i = 0;
#ifdef PQH_SNAP_PROF
  uint64_t c0t = clock64();
#define SC_T(k)                                     \
  do {                                              \
    __syncthreads();                                \
    const uint64_t c1t = clock64();                 \
    if (tid == 0) L.prof[k] += c1t - c0t;           \
    c0t = c1t;                                      \
  } while (0)
#else
#define SC_T(k) \
  do {          \
  } while (0)
#endif
  while (i < K) {
    const int32_t c0 = L.cp[i].x;
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
      for (int k = tid; k < kSnSpan / 32; k += kSnT) L.cbit[k] = 0;
    }
    __syncthreads();
    {
      int32_t cut = K;
      for (int32_t j = i + tid; j < K; j += kSnT) {
        const int2 c = L.cp[j];
        const int32_t ce = c.x + int32_t(uint32_t(c.y) >> 24);
        const int32_t e = ce < ulen ? ce : ulen;
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
        const int2 c = L.cp[j];
        const int32_t len = int32_t(uint32_t(c.y) >> 24);
        if (!len) continue;
        const int32_t st = c.x > 0 ? c.x : 0;
        const int32_t e = c.x + len < ulen ? c.x + len : ulen;
        L.emap[st - B0] = uint16_t(j - i + 1);
        tm = e - B0 > tm ? e - B0 : tm;
        for (int32_t x = st - B0; x < e - B0;) {
          const int32_t wq = x >> 5, b0 = x & 31;
          const int32_t nb = e - B0 - x < 32 - b0 ? e - B0 - x : 32 - b0;
          atomicOr(&L.cbit[wq], (nb == 32 ? ~0u : ((1u << nb) - 1)) << b0);
          x += nb;
        }
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
      const int32_t run0 = sn_excl_max(L, int32_t(mx));
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
    SC_T(5);
    uint32_t pmask = 0;  // this thread's bytes still pointing at a copy byte
    // pass 1: every copy byte's source; a source before the span (final) or on a literal byte of
    // the span (its bit clear) resolves the byte at once; any other byte points at its source's
    // span byte (P >= 0).  Four bytes' lookups in flight before their stores.
#pragma unroll 1
    for (int q0 = 0; q0 < kSnPer; q0 += 4) {
      int32_t pos[4], src[4];
      int kind[4];  // 0 none, 1 value from L.out[src], 2 pointer, 3 before the unit
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int32_t b = (q0 + k) * kSnT + tid;
        pos[k] = B0 + b;
        kind[k] = 0;
        src[k] = 0;
        if (b >= T) continue;
        const int e = L.emap[b];
        if (e == 0) continue;
        const int32_t j = i + e - 1;
        const int2 c = L.cp[j];
        const int32_t cs = c.x, o = c.y & 0xffffff, len = int32_t(uint32_t(c.y) >> 24);
        if (pos[k] >= cs + len || o <= 0) continue;  // a literal byte (or a failed page)
        int32_t rel = pos[k] - cs;
        if (o < len) {  // overlapping copies repeat their first period: rel % o (rel, o < 64: exact in f32)
          const int32_t qq = int32_t(float(rel) * __builtin_amdgcn_rcpf(float(o)) + 1e-3f);
          rel -= qq * o;
        }
        const int32_t s2 = cs - o + rel;
        src[k] = s2;
        if (s2 < 0) kind[k] = 3;
        else if (s2 < B0) kind[k] = 1;
        else kind[k] = ((L.cbit[(s2 - B0) >> 5] >> ((s2 - B0) & 31)) & 1) ? 2 : 1;
      }
      uint8_t v[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        v[k] = 0;
        if (kind[k] == 1) v[k] = L.out[src[k]];
        else if (kind[k] == 3 && ext && U0 + src[k] >= 0) v[k] = dst_unit[src[k]];
      }
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int32_t b = (q0 + k) * kSnT + tid;
        if (b >= T) continue;
        if (kind[k] == 1 || (kind[k] == 3 && ext)) L.out[pos[k]] = v[k];
        if (kind[k] == 3 && !ext) L.ext = 1;
        L.ptr[b] = kind[k] == 2 ? int16_t(src[k] - B0) : int16_t(-1);
        if (kind[k] == 2) pmask |= 1u << (q0 + k);
      }
    }
    __syncthreads();
    // pass 2: pointer jumping without barriers.  A byte whose pointer reaches a resolved byte takes
    // its value (L.out written before P = -1: a wave's LDS writes land in order, so whoever sees
    // P = -1 reads the final byte); otherwise it jumps to its target's pointer.  Any pointer a byte
    // reads (old or already jumped) is a valid earlier byte of its chain, so the chains shorten
    // until every byte is resolved.
    SC_T(6);
    while (pmask) {
#ifdef PQH_SNAP_PROF
      if (tid == 0) L.prof[10] += 1;
#endif
      uint32_t m = pmask;
      while (m) {  // up to four pending bytes' loads in flight together
        int q[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          q[k] = m ? __builtin_ctz(m) : -1;
          m &= m ? m - 1 : 0u;
        }
        int16_t p[4], t[4];
#pragma unroll
        for (int k = 0; k < 4; k++) p[k] = q[k] >= 0 ? __atomic_load_n(&L.ptr[q[k] * kSnT + tid], __ATOMIC_RELAXED) : int16_t(-1);
#pragma unroll
        for (int k = 0; k < 4; k++) t[k] = p[k] >= 0 ? __atomic_load_n(&L.ptr[p[k]], __ATOMIC_RELAXED) : int16_t(0);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");  // a -1 read above: its byte is final
        uint8_t v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) v[k] = (p[k] >= 0 && t[k] < 0) ? L.out[B0 + p[k]] : uint8_t(0);
#pragma unroll
        for (int k = 0; k < 4; k++)
          if (p[k] >= 0 && t[k] < 0) L.out[B0 + q[k] * kSnT + tid] = v[k];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // the bytes before their -1
#pragma unroll
        for (int k = 0; k < 4; k++) {
          if (p[k] < 0) continue;
          __atomic_store_n(&L.ptr[q[k] * kSnT + tid], t[k] < 0 ? int16_t(-1) : t[k], __ATOMIC_RELAXED);
          if (t[k] < 0) pmask &= ~(1u << q[k]);
        }
      }
    }
    __syncthreads();
    SC_T(7);
#ifdef PQH_SNAP_PROF
    if (tid == 0) L.prof[11] += 1;
#endif
    i = i1;
  }
#undef SC_T
}

// One unit [U0, U1) of a SNAPPY block's output: block src[0, n) (header length hl), output at dst
// (after the raw prefix), true window entries / bases wt[0, nw) and per-thread segment entries
// wseg (k_snap_spec / k_snap_stitch).  The unit's windows are walked in order from the last one
// whose output base is at or before U0: every thread walks its 4-byte walker segment from its
// exact entry, once to count (output bytes, copies, literals), once to list literals and copies;
// waves then copy the literals (a lane per byte) and sn_copies resolves the copies.
// Returns whether a copy reached before the unit (not in ext mode, where such sources are read
// from dst); *bad: a copy of offset 0 or reaching before the output start (golang/snappy
// decode_other.go:104-106).
__device__ bool sn_unit(SnEmitLds& L, const uint8_t* src, int32_t n, int32_t hl, uint8_t* dst, int32_t U0, int32_t U1,
                        const int2* wt, const int16_t* wseg, int32_t nw, bool ext, bool* bad) {
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
#ifdef PQH_SNAP_PROF
  if (tid < 12) L.prof[tid] = 0;
  uint64_t t0 = clock64();
#define SN_T(i)                         \
  do {                                  \
    __syncthreads();                    \
    const uint64_t t1 = clock64();      \
    if (tid == 0) L.prof[i] += t1 - t0; \
    t0 = t1;                            \
  } while (0)
#else
#define SN_T(i) \
  do {          \
  } while (0)
#endif
  int32_t w = L.win;
  while (w < nw) {
    const int2 tw = wt[w];
    if (tw.y >= U1) break;
    const int32_t ws = w * kSnWin > hl ? w * kSnWin : hl;
    const int32_t we = (w + 1) * kSnWin < n ? (w + 1) * kSnWin : n;
    if (tw.x >= we) {  // a literal passes over this window: on to the window holding its end
      const int32_t wn = tw.x / kSnWin;
      w = wn > w ? wn : w + 1;
      continue;
    }
    const int32_t a0 = ws - int32_t((reinterpret_cast<uintptr_t>(src) + uintptr_t(ws)) & 15);
    __syncthreads();  // the previous window's readers are done
    {
      const uint4* sp = reinterpret_cast<const uint4*>(src + a0);
      uint4* lp = reinterpret_cast<uint4*>(L.in);
      const int32_t nu = (we + 16 - a0 + 15) >> 4;
      for (int u = tid; u < nu; u += kSnT) lp[u] = sp[u];
    }
    if (tid == 0) L.nlong = 0;
    const int32_t span = we - ws;
    const int32_t S4 = (span + kSnT - 1) / kSnT;
    // one walker segment per thread, from the entry the spec / stitch left for it
    const int32_t hi = ws + (S4 * (tid + 1) < span ? S4 * (tid + 1) : span);
    const int32_t f = ws + wseg[int64_t(w) * kSnT + tid];
    __syncthreads();
    SN_T(0);
    int32_t ot = 0, kt = 0, nlit = 0;
    for (int32_t q = f; q < hi && q < n;) {
      const SnEl e = sn_el(L.in, q - a0);
      ot += int32_t(e.len);
      kt += !e.lit;
      nlit += e.lit;
      q += e.hdr + (e.lit ? int32_t(e.len) : 0);
    }
    int32_t Ot, Kt, Lt;
    const int32_t ob = tw.y + sn_excl_sum(L, ot, &Ot);
    const int32_t kb = sn_excl_sum(L, kt, &Kt);
    const int32_t lb = sn_excl_sum(L, nlit, &Lt);
    SN_T(9);
    int32_t* lit_out = reinterpret_cast<int32_t*>(L.emap);  // the literal list (emap is free until sn_copies)
    int32_t* lit_src = lit_out + kSnMaxC;
    int32_t* lit_len = lit_src + kSnMaxC;
    const int32_t stage_hi = we + 16;
    {
      int32_t q = f, P = ob, k = kb, li = lb;
      while (q < hi && q < n && P < U1) {
        const SnEl e = sn_el(L.in, q - a0);
        const int32_t len = int32_t(e.len);
        if (e.lit) {
          const int32_t body = q + e.hdr;
          const int32_t b0 = P > U0 ? P : U0, b1 = P + len < U1 ? P + len : U1;
          lit_out[li] = b0 - U0;
          lit_src[li] = body + (b0 - P);
          lit_len[li] = 0;
          if (b0 < b1) {
            if (b1 - b0 <= kSnLongLit) {
              lit_len[li] = b1 - b0;
            } else {  // long: copied by the whole workgroup
              const int32_t lg = atomicAdd(&L.nlong, 1);
              L.l_out[lg] = b0 - U0;
              L.l_src[lg] = body + (b0 - P);
              L.l_len[lg] = b1 - b0;
            }
          }
          li++;
          q = body + len;
        } else {
          if (P >= U0 && (e.off == 0 || e.off > P)) L.bad = 1;
          L.cp[k] = make_int2(P - U0, (e.off < 0xffffff ? e.off : 0xffffff) | ((P + len > U0 ? len : 0) << 24));  // (P < U1)
          k++;
          q += e.hdr;
        }
        P += len;
      }
      for (; k < kb + kt; k++) {  // copies past the unit
        L.cp[k] = make_int2(ulen, 1);
      }
      for (; li < lb + nlit; li++) lit_len[li] = 0;  // literals past the unit
    }
    __syncthreads();
    SN_T(1);
    if (L.bad) {
      *bad = true;
      return false;
    }
    {  // literals of up to kSnShortLit bytes: a thread each, byte by byte; longer ones (up to
       // kSnLongLit) listed for the waves: a lane per byte, four literals per step (bytes from the
       // stage, or HBM past it)
      int32_t* med = reinterpret_cast<int32_t*>(L.ptr);  // (ptr is free until sn_copies)
      if (tid == 0) L.nmed = 0;
      __syncthreads();
      for (int32_t li = tid; li < Lt; li += kSnT) {
        const int32_t ln = lit_len[li];
        if (ln == 0) continue;
        if (ln > kSnShortLit) {
          med[atomicAdd(&L.nmed, 1)] = li;
          continue;
        }
        const int32_t lo2 = lit_out[li], ls = lit_src[li];
        for (int32_t x = 0; x < ln; x++) {
          const int32_t sx = ls + x;
          L.out[lo2 + x] = sx < stage_hi ? L.in[sx - a0] : src[sx];
        }
      }
      __syncthreads();
      const int32_t nmed = L.nmed;
      const int lane = tid & 63;
      for (int32_t e0 = 4 * (tid >> 6); e0 < nmed; e0 += 4 * (kSnT / 64)) {  // four literals per step
        int32_t ln[4], lo2[4], ls[4], mx = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const bool on = e0 + k < nmed;
          const int32_t li = on ? med[e0 + k] : 0;
          ln[k] = on ? lit_len[li] : 0;
          lo2[k] = on ? lit_out[li] : 0;
          ls[k] = on ? lit_src[li] : 0;
          mx = ln[k] > mx ? ln[k] : mx;
        }
        for (int32_t x = lane; x < mx; x += 64) {
          uint8_t v[4];
#pragma unroll
          for (int k = 0; k < 4; k++) {
            const int32_t sx = ls[k] + x;
            v[k] = x < ln[k] ? (sx < stage_hi ? L.in[sx - a0] : src[sx]) : uint8_t(0);
          }
#pragma unroll
          for (int k = 0; k < 4; k++)
            if (x < ln[k]) L.out[lo2[k] + x] = v[k];
        }
      }
    }
    for (int32_t li = 0; li < L.nlong; li++) {
      const int32_t lo2 = L.l_out[li], ls = L.l_src[li], ln = L.l_len[li];
      for (int32_t j = tid; j < ln; j += kSnT) L.out[lo2 + j] = src[ls + j];
    }
    SN_T(2);
    sn_copies(L, Kt, U0, ulen, ext, dst + U0);
    SN_T(3);
#ifdef PQH_SNAP_PROF
    if (tid == 0) L.prof[8] += 1;
#endif
    w++;
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
  SN_T(4);
#ifdef PQH_SNAP_PROF
  if (tid == 0 && blockIdx.x < 2)
    printf("snapprof unit %d windows %lu | cycles: load %lu walks %lu lits %lu copies %lu (setup %lu pass1 %lu jump %lu; "
           "spans %lu thread-rounds(t0) %lu) store %lu\n", int(blockIdx.x), L.prof[8], L.prof[0], L.prof[1], L.prof[2],
           L.prof[3], L.prof[5], L.prof[6], L.prof[7], L.prof[11], L.prof[10], L.prof[4]);
  if (tid == 0 && blockIdx.x < 2) printf("snapprof unit %d walk1+scans %lu walk2 %lu\n", int(blockIdx.x), L.prof[9], L.prof[1]);
#endif
#undef SN_T
  return L.ext != 0;
}

__global__ __launch_bounds__(kSnT) void k_snap_emit(const pqh_codec_page* cps, const int32_t* unit_page,
                                                    const int32_t* page_unit0, const int32_t* page_win0,
                                                    const uint8_t* src_all, uint8_t* dst_all, const int2* wtrue,
                                                    const int16_t* wseg, int32_t* status, int32_t* uflag) {
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
  const uint8_t* src = src_all + cp.src_offset + raw;
  const int32_t n = cp.src_len - raw;
  uint64_t v;
  const int32_t hl = sn_header(src, n, &v);  // (valid: the stitch accepted the page)
  const int32_t total = cp.image_len - raw;
  const int32_t U0 = k * kSnUnit, U1 = U0 + kSnUnit < total ? U0 + kSnUnit : total;
  const int32_t w0 = page_win0[p];
  bool bad = false;
  const bool ext = sn_unit(L, src, n, hl, dst + raw, U0, U1, wtrue + w0, wseg + int64_t(w0) * kSnT,
                           page_win0[p + 1] - w0, false, &bad);
  if (threadIdx.x == 0) {
    uflag[u] = ext && !bad;
    if (bad) status[p] = PQH_ERR_DECOMPRESS;
  }
}

// The units a copy before the unit marked, again in order, their early sources read from HBM.
__global__ __launch_bounds__(kSnT) void k_snap_fixup(const pqh_codec_page* cps, const int32_t* page_unit0,
                                                     const int32_t* page_win0, const uint8_t* src_all,
                                                     uint8_t* dst_all, const int2* wtrue, const int16_t* wseg,
                                                     int32_t* status, const int32_t* uflag) {
  __shared__ SnEmitLds L;
  const int32_t p = blockIdx.x;
  const pqh_codec_page cp = cps[p];
  if (cp.codec != PQH_CODEC_SNAPPY || status[p] != PQH_OK) return;
  const int32_t u0 = page_unit0[p], u1 = page_unit0[p + 1];
  const int32_t raw = cp.raw_len < cp.src_len ? cp.raw_len : cp.src_len;
  const uint8_t* src = src_all + cp.src_offset + raw;
  const int32_t n = cp.src_len - raw;
  uint64_t v;
  const int32_t hl = sn_header(src, n, &v);
  const int32_t total = cp.image_len - raw;
  const int32_t w0 = page_win0[p];
  for (int32_t u = u0; u < u1; u++) {
    if (!uflag[u]) continue;
    const int32_t U0 = (u - u0) * kSnUnit, U1 = U0 + kSnUnit < total ? U0 + kSnUnit : total;
    bool bad = false;
    sn_unit(L, src, n, hl, dst_all + cp.image_offset + raw, U0, U1, wtrue + w0, wseg + int64_t(w0) * kSnT,
            page_win0[p + 1] - w0, true, &bad);
    __threadfence();
    if (bad) {
      if (threadIdx.x == 0) status[p] = PQH_ERR_DECOMPRESS;
      return;
    }
  }
}
