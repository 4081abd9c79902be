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
// so offsets_l[k] = #E_l before the k-th E_{l-1} slot.  Three passes over the level bytes: per-tile
// flag counts (k_nest_count), per-chunk exclusive scans (k_nest_scan), and a write pass with block
// scans (k_nest_write).  Pinned by oracle.nest_levels against the reference's KATs
// (tests/golden/dremel_kat.json).
#pragma once

constexpr int kNestPer = kNestTile / kBlock;  // 32 consecutive slots per thread

// Flags of one slot: bit f = E_f (bit 0 = row start).
__device__ __forceinline__ uint32_t nest_flags(const DevNest& N, int32_t d, int32_t r) {
  uint32_t f = r == 0 ? 1u : 0u;
#pragma unroll
  for (int l = 1; l <= kMaxNest; l++)
    if (l <= N.levels && r <= l && d >= N.rep_def[l - 1]) f |= 1u << l;
  return f;
}

__device__ __forceinline__ void nest_load(const DevNest& N, const DevChunk& C, int64_t s0, uint8_t* d, uint8_t* r) {
  // 32 level bytes of each stream; the level buffers carry 64 bytes of slack past n
  __builtin_memcpy(d, C.def_levels + s0, 32);
  __builtin_memcpy(r, C.rep_levels + s0, 32);
}

__global__ __launch_bounds__(256) void k_nest_count(DevBatch b, const Tile* tiles) {
  __shared__ int32_t cnt[kNestFlags];
  const Tile t = tiles[blockIdx.x];
  const DevNest N = b.nests[t.page];
  const DevChunk C = b.chunks[N.chunk];
  if (threadIdx.x < kNestFlags) cnt[threadIdx.x] = 0;
  __syncthreads();
  const int64_t s0 = int64_t(t.k) * kNestTile + int64_t(threadIdx.x) * kNestPer;
  int32_t c[kNestFlags];
#pragma unroll
  for (int f = 0; f < kNestFlags; f++) c[f] = 0;
  if (s0 < N.n) {
    uint8_t d[32], r[32];
    nest_load(N, C, s0, d, r);
    const int m = N.n - s0 < kNestPer ? int(N.n - s0) : kNestPer;
    for (int j = 0; j < m; j++) {
      const uint32_t fl = nest_flags(N, d[j], r[j]);
#pragma unroll
      for (int f = 0; f < kNestFlags; f++) c[f] += (fl >> f) & 1;
    }
  }
#pragma unroll
  for (int f = 0; f < kNestFlags; f++) {
    int32_t x = c[f];
    for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
    if ((threadIdx.x & 63) == 0 && x) atomicAdd(&cnt[f], x);
  }
  __syncthreads();
  if (threadIdx.x < kNestFlags) b.nsums[int64_t(N.tile_base + t.k) * kNestFlags + threadIdx.x] = cnt[threadIdx.x];
}

// One workgroup per nested chunk: exclusive scan of every flag over the chunk's tiles.
__global__ __launch_bounds__(256) void k_nest_scan(DevBatch b) {
  __shared__ int64_t wsum[4];
  __shared__ int64_t carry;
  const DevNest& N = b.nests[blockIdx.x];  // by reference: the per-level arrays are indexed at run time
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  for (int f = 0; f <= N.levels; f++) {
    if (t == 0) carry = 0;
    __syncthreads();
    for (int base = 0; base < N.tile_n; base += kBlock) {
      const int i = base + t;
      int64_t* slot = b.nsums + int64_t(N.tile_base + i) * kNestFlags + f;
      const int64_t x = i < N.tile_n ? *slot : 0;
      int64_t incl = x;
      for (int off = 1; off < 64; off <<= 1) {
        const int64_t y = __shfl_up(incl, off, 64);
        if (lane >= off) incl += y;
      }
      if (lane == 63) wsum[wv] = incl;
      __syncthreads();
      int64_t before = carry;
      for (int k = 0; k < wv; k++) before += wsum[k];
      if (i < N.tile_n) *slot = before + incl - x;
      __syncthreads();
      if (t == 0) carry += wsum[0] + wsum[1] + wsum[2] + wsum[3];
      __syncthreads();
    }
    if (t == 0) {
      N.totals[f] = carry;
      // closing offset of level f: its element total after its lists (level f+1's lists = E_f)
      if (f >= 1) N.offsets[f - 1][N.totals[f - 1]] = int32_t(carry);
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void k_nest_write(DevBatch b, const Tile* tiles) {
  __shared__ uint64_t wsum[4];
  const Tile t = tiles[blockIdx.x];
  const DevNest N = b.nests[t.page];
  const DevChunk C = b.chunks[N.chunk];
  const int64_t s0 = int64_t(t.k) * kNestTile + int64_t(threadIdx.x) * kNestPer;
  const int m = s0 < N.n ? (N.n - s0 < kNestPer ? int(N.n - s0) : kNestPer) : 0;
  const uint8_t* dl = C.def_levels + s0;
  const uint8_t* rl = C.rep_levels + s0;
  const int L = N.levels;
  int32_t c[kNestFlags];
#pragma unroll
  for (int f = 0; f < kNestFlags; f++) c[f] = 0;
  for (int j = 0; j < m; j++) {
    const uint32_t x = nest_flags(N, dl[j], rl[j]);
#pragma unroll
    for (int f = 0; f < kNestFlags; f++) c[f] += (x >> f) & 1;
  }
  const int64_t* base = b.nsums + int64_t(N.tile_base + t.k) * kNestFlags;
  int64_t pos[kNestFlags];  // running index of each flag at this thread's next slot
#pragma unroll
  for (int f = 0; f < kNestFlags; f++) {
    pos[f] = 0;
    if (f <= L) {  // uniform
      uint64_t tot;
      pos[f] = base[f] + int64_t(block_exclusive_scan(uint64_t(c[f]), wsum, &tot));
    }
  }
  for (int j = 0; j < m; j++) {  // the level bytes are L1-resident from the first loop
    const int32_t d = dl[j];
    const uint32_t x = nest_flags(N, d, rl[j]);
#pragma unroll
    for (int l = 1; l <= kMaxNest; l++) {
      if (l <= L && ((x >> (l - 1)) & 1)) {  // a list of level l starts here
        const int64_t k = pos[l - 1];
        N.offsets[l - 1][k] = int32_t(pos[l]);
        N.validity[l - 1][k] = d >= N.rep_def[l - 1] - 1;
      }
      if (l == L && ((x >> l) & 1)) N.leaf_valid[pos[l]] = d == N.max_def;
    }
#pragma unroll
    for (int f = 0; f < kNestFlags; f++) pos[f] += (x >> f) & 1;
  }
}
