// nest_impl.h — levels -> nesting outputs on the device (included by decode.hip).
//
// The reference assembles records from the levels one value at a time (ColumnStore.get
// data_store.go:262-309: d < maxD is a null at depth d; a repeated value collects while the next
// r >= maxR; Column.getNextData/getData schema.go:216-312: a group exists when a child is defined at
// its depth).  Columnar form, per repetition level l with D_l = definition level of its REPEATED node:
//   element of level l starts at slot i   <=>  r_i <= l  and d_i >= D_l           (flag E_l)
//   list of level l starts at slot i      <=>  row start (l == 1) or E_{l-1}(i)     (flag E_{l-1}, E_0 = r_i == 0)
//   list present (possibly empty)         <=>  d_i >= D_l - 1 at its first slot
//   leaf slots = E_L slots; non-null      <=>  d_i == max_def
// so offsets_l[k] = #E_l before the k-th E_{l-1} slot.  With D_0 = 0, E_0 is E_l's formula at l = 0,
// so a window of levels lbase + 1 .. lbase + L (DevNest) computes E_lbase .. E_{lbase+L} the same way
// (flag f of the window = E_{lbase+f}).  Three passes over the level bytes: per-tile
// flag counts (k_nest_count), per-chunk exclusive scans (k_nest_scan), and a write pass with block
// scans (k_nest_write).  Pinned by oracle.nest_levels against the reference's KATs
// (tests/golden/dremel_kat.json).
#pragma once

constexpr int kNestPer = kNestTile / kBlock;  // 32 consecutive slots per thread

// Bytes of x that are >= t (t <= 128, every byte of x < 128): 0x80 in each such byte.  Subtracting
// t from each byte with its top bit forced on never borrows across bytes.
__device__ __forceinline__ uint32_t ge8(uint32_t x, uint32_t t) {
  return ((x | 0x80808080u) - t * 0x01010101u) & 0x80808080u;
}

// Byte flags (0x80 per byte) -> bits 0..3.
__device__ __forceinline__ uint32_t pack4(uint32_t m) {
  uint32_t t = m >> 7;
  t |= t >> 7;
  t |= t >> 14;
  return t & 0xfu;
}

// The flag masks of a thread's 32 slots (bit j = slot j): E_f, V_l, LV (see k_nest_write).  Four
// slots per dword compare at once (ge8); bytes >= 128 (a corrupt stream of 8-bit levels) or levels
// >= 128 take the per-slot path.
__device__ __forceinline__ void nest_masks(const DevNest& N, const DevChunk& C, int64_t s0, int m,
                                           uint32_t E[kNestFlags], uint32_t V[kMaxNest], uint32_t& LV) {
  const int L = N.levels;
#pragma unroll
  for (int f = 0; f < kNestFlags; f++) E[f] = 0;
#pragma unroll
  for (int l = 0; l < kMaxNest; l++) V[l] = 0;
  LV = 0;
  if (m <= 0) return;
  // 32 level bytes of each stream (the level buffers carry 64 bytes of slack past n)
  uint32_t dw[8], rw[8];
  __builtin_memcpy(dw, C.def_levels + s0, 32);
  __builtin_memcpy(rw, C.rep_levels + s0, 32);
  uint32_t hi = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) hi |= dw[k] | rw[k];
  const uint32_t in = m >= kNestPer ? ~0u : (1u << m) - 1;
  if ((hi & 0x80808080u) == 0 && N.max_def < 128 && N.lbase + L < 128) {
    const uint32_t M = uint32_t(N.max_def), lb = uint32_t(N.lbase), d0 = uint32_t(N.d0);
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t d = dw[k], r = rw[k];
      E[0] |= pack4(~ge8(r, lb + 1) & ge8(d, d0)) << (4 * k);  // (lbase 0: r == 0)
#pragma unroll
      for (int l = 1; l <= kMaxNest; l++) {
        if (l <= L) {
          const uint32_t D = uint32_t(N.rep_def[l - 1]);
          E[l] |= pack4(~ge8(r, lb + uint32_t(l) + 1) & ge8(d, D)) << (4 * k);
          V[l - 1] |= pack4(ge8(d, D - 1)) << (4 * k);
        }
      }
      LV |= pack4(ge8(d, M) & ~ge8(d, M + 1)) << (4 * k);
    }
#pragma unroll
    for (int f = 0; f < kNestFlags; f++) E[f] &= in;
#pragma unroll
    for (int l = 0; l < kMaxNest; l++) V[l] &= in;
    LV &= in;
    return;
  }
#pragma unroll
  for (int j = 0; j < kNestPer; j++) {
    const uint32_t d = (dw[j >> 2] >> (8 * (j & 3))) & 0xff, r = (rw[j >> 2] >> (8 * (j & 3))) & 0xff;
    const uint32_t in = j < m ? 1u << j : 0u;
    E[0] |= (r <= uint32_t(N.lbase) && d >= uint32_t(N.d0)) ? in : 0u;
#pragma unroll
    for (int l = 1; l <= kMaxNest; l++) {
      if (l <= L) {
        E[l] |= (r <= uint32_t(N.lbase + l) && d >= uint32_t(N.rep_def[l - 1])) ? in : 0u;
        V[l - 1] |= d + 1 >= uint32_t(N.rep_def[l - 1]) ? in : 0u;
      }
    }
    LV |= d == uint32_t(N.max_def) ? in : 0u;
  }
}

// Flags f and f + 1 of every thread packed in one dword (16 bits each: a tile counts at most
// kNestTile < 2^16 of either), so one 32-bit DPP scan serves two flags.
__device__ __forceinline__ uint32_t nest_pair(const uint32_t E[kNestFlags], int f, int L) {
  uint32_t x = 0;
#pragma unroll
  for (int g = 0; g < kNestFlags; g++) {
    if (g == f) x |= uint32_t(__popc(E[g]));
    if (g == f + 1 && g <= L) x |= uint32_t(__popc(E[g])) << 16;
  }
  return x;
}

__global__ __launch_bounds__(256) void k_nest_count(DevBatch b, const Tile* tiles) {
  __shared__ int32_t cnt[kNestFlags + 1];
  const Tile t = tiles[blockIdx.x];
  const DevNest N = b.nests[t.page];
  const DevChunk C = b.chunks[N.chunk];
  if (threadIdx.x < kNestFlags + 1) cnt[threadIdx.x] = 0;
  __syncthreads();
  const int64_t s0 = int64_t(t.k) * kNestTile + int64_t(threadIdx.x) * kNestPer;
  const int m = s0 < N.n ? (N.n - s0 < kNestPer ? int(N.n - s0) : kNestPer) : 0;
  const int L = N.levels;
  uint32_t E[kNestFlags], V[kMaxNest], LV;
  nest_masks(N, C, s0, m, E, V, LV);
  for (int f = 0; f <= L; f += 2) {  // uniform: flags 0..L only
    const uint32_t x = wave_incl_scan32(nest_pair(E, f, L));
    if ((threadIdx.x & 63) == 63 && x) {
      atomicAdd(&cnt[f], int32_t(x & 0xffffu));
      atomicAdd(&cnt[f + 1], int32_t(x >> 16));
    }
  }
  __syncthreads();
  if (threadIdx.x < kNestFlags) b.nsums[int64_t(N.tile_base + t.k) * kNestFlags + threadIdx.x] = cnt[threadIdx.x];
}

// One workgroup per nested chunk: exclusive scan of every flag over the chunk's tiles (each thread
// a contiguous run of ceil(tile_n / 256) tiles: one block scan per flag).
__global__ __launch_bounds__(256) void k_nest_scan(DevBatch b) {
  __shared__ uint64_t wsum[4];
  const DevNest& N = b.nests[blockIdx.x];  // by reference: the per-level arrays are indexed at run time
  const int per = (N.tile_n + kBlock - 1) / kBlock;
  const int i0 = int(threadIdx.x) * per, i1 = i0 + per < N.tile_n ? i0 + per : N.tile_n;
  for (int f = 0; f <= N.levels; f++) {
    int64_t* slot = b.nsums + int64_t(N.tile_base) * kNestFlags + f;
    uint64_t local = 0;
    for (int i = i0; i < i1; i += 8) {  // 8 loads in flight
      int64_t x[8];
#pragma unroll
      for (int k = 0; k < 8; k++) x[k] = i + k < i1 ? slot[int64_t(i + k) * kNestFlags] : 0;
#pragma unroll
      for (int k = 0; k < 8; k++) local += uint64_t(x[k]);
    }
    uint64_t total;
    int64_t run = int64_t(block_exclusive_scan(local, wsum, &total));
    for (int i = i0; i < i1; i += 8) {
      int64_t x[8];
#pragma unroll
      for (int k = 0; k < 8; k++) x[k] = i + k < i1 ? slot[int64_t(i + k) * kNestFlags] : 0;
#pragma unroll
      for (int k = 0; k < 8; k++) {
        if (i + k >= i1) break;
        slot[int64_t(i + k) * kNestFlags] = run;
        run += x[k];
      }
    }
    if (threadIdx.x == 0) {
      N.totals[f] = int64_t(total);
      // closing offset of level f: its element total after its lists (level f+1's lists = E_f)
      if (f >= 1) N.offsets[f - 1][N.totals[f - 1]] = int32_t(total);
    }
    __syncthreads();
  }
}

// Copy n staged elements (LDS, laid out from a 16-byte aligned origin: element i of the range at
// lds[lead + i]) to dst[0..n) with 16-byte stores; the partial vectors at both ends byte by byte.
template <class T>
__device__ __forceinline__ void nest_flush(PQH_G T* dst, const T* lds, int lead, int n) {
  constexpr int E = 16 / sizeof(T);  // elements per vector
  const int total = lead + n;
  const int nvec = (total + E - 1) / E;
  PQH_G T* origin = dst - lead;
  for (int v = threadIdx.x; v < nvec; v += kBlock) {
    const int i0 = v * E;
    if (i0 >= lead && i0 + E <= total) {
      uint4 x;
      __builtin_memcpy(&x, lds + i0, 16);
      *reinterpret_cast<PQH_G uint4*>(origin + i0) = x;
    } else {
      for (int i = i0; i < i0 + E; i++)
        if (i >= lead && i < total) origin[i] = lds[i];
    }
  }
}

// Write pass: the tile's list offsets / presence per level and its leaf validity are staged in LDS
// (each output range of a tile is contiguous) and flushed with coalesced 16-byte stores.  Per thread
// the 32 slots' flags are bit masks (bit j = slot j): E_f (element / list starts), V_l (list of
// level l present), LV (leaf non-null), so counts are popcounts and positions prefix popcounts.
__global__ __launch_bounds__(256) void k_nest_write(DevBatch b, const Tile* tiles) {
  __shared__ uint64_t wsum[4];
  // list offsets are staged kListPart at a time (a tile rarely starts more lists than that), which
  // halves the LDS of a workgroup (occupancy)
  constexpr int kListPart = kNestTile / 2;
  __shared__ __attribute__((aligned(16))) int32_t st32[kListPart + 4];
  __shared__ __attribute__((aligned(16))) uint8_t st8[kNestTile + 16];
  const Tile t = tiles[blockIdx.x];
  const DevNest N = b.nests[t.page];
  const DevChunk C = b.chunks[N.chunk];
  const int64_t s0 = int64_t(t.k) * kNestTile + int64_t(threadIdx.x) * kNestPer;
  const int m = s0 < N.n ? (N.n - s0 < kNestPer ? int(N.n - s0) : kNestPer) : 0;
  const int L = N.levels;
  uint32_t E[kNestFlags], V[kMaxNest], LV;
  nest_masks(N, C, s0, m, E, V, LV);
  const int64_t* base = b.nsums + int64_t(N.tile_base + t.k) * kNestFlags;
  int32_t lpos[kNestFlags], tot[kNestFlags];
  int64_t gbase[kNestFlags];
#pragma unroll
  for (int f = 0; f < kNestFlags; f++) {
    lpos[f] = 0;
    tot[f] = 0;
    gbase[f] = f <= L ? base[f] : 0;
  }
#pragma unroll
  for (int f = 0; f < kNestFlags; f += 2) {
    if (f > L) break;  // uniform
    // flags f and f + 1 in one block scan of packed 16-bit counts (DPP wave scans)
    const uint32_t x = nest_pair(E, f, L);
    const uint32_t incl = wave_incl_scan32(x);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t* ws = reinterpret_cast<uint32_t*>(wsum);
    if (lane == 63) ws[wv] = incl;
    __syncthreads();
    uint32_t before = 0;
    for (int k = 0; k < wv; k++) before += ws[k];
    const uint32_t tt = ws[0] + ws[1] + ws[2] + ws[3], ex = before + incl - x;
    __syncthreads();
    lpos[f] = int32_t(ex & 0xffffu);
    tot[f] = int32_t(tt & 0xffffu);
    if (f + 1 < kNestFlags) {
      lpos[f + 1] = int32_t(ex >> 16);
      tot[f + 1] = int32_t(tt >> 16);
    }
  }
#pragma unroll
  for (int l = 1; l <= kMaxNest; l++) {  // lists of level l start at the E_{l-1} slots
    if (l > L) break;
    const int lead32 = int(gbase[l - 1] & 3), lead8 = int(gbase[l - 1] & 15);
    for (int p0 = 0; p0 < tot[l - 1]; p0 += kListPart) {  // uniform
      int32_t k = lpos[l - 1];
      for (uint32_t x = E[l - 1]; x; x &= x - 1, k++) {
        const int j = __builtin_ctz(x);
        if (k < p0 || k >= p0 + kListPart) continue;
        st32[lead32 + k - p0] = int32_t(gbase[l] + lpos[l] + __popc(E[l] & ((1u << j) - 1)));
        st8[lead8 + k - p0] = uint8_t((V[l - 1] >> j) & 1);
      }
      __syncthreads();
      const int cnt = tot[l - 1] - p0 < kListPart ? tot[l - 1] - p0 : kListPart;
      nest_flush(N.offsets[l - 1] + gbase[l - 1] + p0, st32, lead32, cnt);
      nest_flush(N.validity[l - 1] + gbase[l - 1] + p0, st8, lead8, cnt);
      __syncthreads();
    }
  }
  if (!N.leaf) return;  // (a window above the innermost level)
  // leaf validity at the E_L slots
  uint32_t EL = 0;
  int32_t lposL = 0, totL = 0;
  int64_t gbaseL = 0;
#pragma unroll
  for (int f = 1; f < kNestFlags; f++)
    if (f == L) {
      EL = E[f];
      lposL = lpos[f];
      totL = tot[f];
      gbaseL = gbase[f];
    }
  const int lead8 = int(gbaseL & 15);
  {
    // the thread's leaf flags compacted to its elements (the non-element slots, few, dropped from
    // the top down), then stored as bytes up to a 4-aligned LDS position and nibble-expanded dwords
    uint32_t c = LV;
    for (uint32_t z = ~EL & (m >= kNestPer ? ~0u : (1u << m) - 1); z;) {
      const int j = 31 - __clz(int(z));
      z &= ~(1u << j);
      c = (c & ((1u << j) - 1)) | (((c >> j) >> 1) << j);
    }
    int pos = lead8 + lposL, left = __popc(EL);
    for (; left > 0 && (pos & 3); left--, c >>= 1) st8[pos++] = uint8_t(c & 1);
    for (; left >= 4; left -= 4, c >>= 4, pos += 4) *reinterpret_cast<uint32_t*>(st8 + pos) = nibble_bytes(c & 15);
    for (; left > 0; left--, c >>= 1) st8[pos++] = uint8_t(c & 1);
  }
  __syncthreads();
  nest_flush(N.leaf_valid + gbaseL, st8, lead8, totL);
}
