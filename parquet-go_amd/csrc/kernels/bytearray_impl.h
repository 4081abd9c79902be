// bytearray_impl.h — BYTE_ARRAY values on the device (included by decode.hip).
//
// Output per chunk: int64 offsets[notNull + 1] + the concatenated bytes (Arrow-style) — what
// decodeValues fills into []interface{} of []byte (type_bytearray.go).  Three producers of
// per-value lengths feed one offsets/copy pipeline:
//   PLAIN       byteArrayPlainDecoder.next (type_bytearray.go:24-45): a [u32 len][bytes] chain,
//               walked by one wave per page (k_ba_walk) -> lengths in aux + the first error;
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
// k_ba_walk: one wave64 per PLAIN byte-array page (data pages and byte-array dictionary pages).
// The chain [u32 len][len bytes] is inherently sequential; the wave reads it through an LDS window
// and records one length (data page) or one cumulative offset (dictionary page) per value,
// flushed 64 at a time with one coalesced store.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_ba_walk(DevBatch b, const int32_t* ba_pages, int32_t n) {
  __shared__ __attribute__((aligned(16))) uint8_t win_all[4][kWin];
  const int lane = threadIdx.x & 63;
  const int wv = int(threadIdx.x >> 6);
  const int idx = __builtin_amdgcn_readfirstlane(int(blockIdx.x) * 4 + wv);
  if (idx >= n) return;
  const int p = ba_pages[idx];
  const DevPage P = b.pages[p];
  const PageState S = b.states[p];
  const bool dict = P.page_type == PQH_DICTIONARY_PAGE;
  if (S.err != kNoError && (dict || page_failed_before_values(S))) return;
  int64_t count, s0, e0;
  int32_t* out;
  if (dict) {  // dictPageReader.read: num_values PLAIN entries over the whole page
    count = P.num_values;
    s0 = 0;
    e0 = P.image_len;
    out = b.dcum + P.aux_base;
  } else {
    count = S.nn;
    s0 = S.val_s;
    e0 = S.val_e;
    out = b.chunks[P.chunk].aux + S.value_base;
  }
  Win w{b.payload + P.image_off, e0, win_all[wv], 0, 0};
  win_load(w, s0, lane);
  int64_t pos = s0, i = 0;
  int32_t cum = 0, mine = 0;
  int code = PQH_OK;
  for (; i < count; i++) {
    const int64_t avail = e0 - pos;
    if (avail < 4) {  // binary.Read of the u32 length
      code = avail <= 0 ? PQH_ERR_EOF : PQH_ERR_UNEXPECTED_EOF;
      break;
    }
    win_ensure(w, pos, 4, lane);
    const uint8_t* q = w.buf + (pos - w.lo);
    const int32_t l = int32_t(uint32_t(q[0]) | (uint32_t(q[1]) << 8) | (uint32_t(q[2]) << 16) | (uint32_t(q[3]) << 24));
    if (l < 0) {
      code = PQH_ERR_NEGATIVE_LENGTH;
      break;
    }
    const int64_t rem = avail - 4;
    if (l > 0 && rem < l) {  // io.ReadFull(len bytes)
      code = rem <= 0 ? PQH_ERR_EOF : PQH_ERR_UNEXPECTED_EOF;
      break;
    }
    pos += 4 + int64_t(l);
    const int32_t rec = dict ? cum : l;
    cum += l;
    if (lane == int(i & 63)) mine = rec;
    if ((i & 63) == 63) out[i - 63 + lane] = mine;
  }
  const int64_t tail = i & 63;
  if (lane < tail) out[i - tail + lane] = mine;
  if (lane == 0) {
    if (dict) {
      out[i] = cum;
      if (code == PQH_OK) b.states[p].dict_n = int32_t(i);
      else atomicMin(&b.states[p].err, (unsigned long long)err_key(0, i, code));
    } else {
      b.states[p].val_limit = int32_t(i);
      if (code != PQH_OK) atomicMin(&b.states[p].err, (unsigned long long)err_key(3, i, code));
    }
  }
}

// Values of a byte-array data page that decode before the first error known so far.
__device__ __forceinline__ int64_t ba_limit(const DevBatch& b, int page, const DevPage& P, const PageState& S) {
  int64_t lim = S.val_limit;
  if (S.err != kNoError && (S.err >> 56) == 3) {
    const int64_t ei = int64_t((S.err >> 8) & 0xffffffffffffull);
    if (ei < lim) lim = ei;
  }
  if (P.kind == K_DLBA) {
    const int64_t dl = b.dstates[page].limit;  // valuesCount of the lengths stream
    if (dl < lim) lim = dl;
  }
  return lim;
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

__device__ __forceinline__ int64_t block_sum64(int64_t x, int64_t* wsum) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
  __syncthreads();
  if (lane == 0) wsum[wv] = x;
  __syncthreads();
  return wsum[0] + wsum[1] + wsum[2] + wsum[3];
}

// ------------------------------------------------------------------------------------------------
// k_ba_sum: bytes of each kBaTile tile; first negative DELTA_LENGTH length; EOF past valuesCount.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_ba_sum(DevBatch b, const Tile* tiles) {
  __shared__ int64_t wsum[4];
  const Tile t = tiles[blockIdx.x];
  const DevPage P = b.pages[t.page];
  const PageState S = b.states[t.page];
  int64_t s = 0;
  if (!page_failed_before_values(S)) {
    const DevChunk C = b.chunks[P.chunk];
    const int64_t lim = ba_limit(b, t.page, P, S);
    const int64_t v0 = int64_t(t.k) * kBaTile;
    const int64_t v1 = v0 + kBaTile < lim ? v0 + kBaTile : lim;
    const bool is_dict = P.kind == K_DICT;
    const BaDict d = is_dict ? ba_dict(b, P) : BaDict{nullptr, 0, 0};
    const int32_t* aux = C.aux + S.value_base;
    int64_t first_neg = INT64_MAX;
    for (int64_t i = v0 + threadIdx.x; i < v1; i += kBlock) {
      const int64_t l = ba_len(d, is_dict, aux[i]);
      if (l < 0) {
        if (i < first_neg) first_neg = i;
      } else {
        s += l;
      }
    }
    if (P.kind == K_DLBA) {
      if (first_neg != INT64_MAX)  // make([]byte, negative) panics (re-panicked, file_reader.go:179-181)
        atomicMin(&b.states[t.page].err, (unsigned long long)err_key(3, first_neg, PQH_ERR_NEGATIVE_DLBA_LENGTH));
      const int64_t vc = b.dstates[t.page].limit;
      if (t.k == 0 && threadIdx.x == 0 && S.nn > vc)  // lens exhausted: io.EOF (type_bytearray.go:118-121)
        atomicMin(&b.states[t.page].err, (unsigned long long)err_key(3, vc, PQH_ERR_EOF));
    }
  }
  s = block_sum64(s, wsum);
  if (threadIdx.x == 0) b.basums[P.batile_base + t.k] = s;
}

// ------------------------------------------------------------------------------------------------
// k_ba_scan: one workgroup per byte-array chunk: exclusive scan of its tiles' byte sums (tiles of a
// chunk are contiguous and in page order) -> each tile's first output offset, each page's first
// byte (byte_base), the chunk's byte total.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_ba_scan(DevBatch b, const int32_t* ba_chunks, const Tile* tiles) {
  __shared__ int64_t wsum[4];
  __shared__ int64_t carry;
  const int c = ba_chunks[blockIdx.x];
  const DevChunk C = b.chunks[c];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (t == 0) {
    carry = 0;
    if (C.offsets) C.offsets[0] = 0;
  }
  __syncthreads();
  for (int base = 0; base < C.batile_n; base += kBlock) {
    const int i = base + t;
    const int64_t x = i < C.batile_n ? b.basums[C.batile_base + i] : 0;
    int64_t incl = x;
    for (int off = 1; off < 64; off <<= 1) {
      const int64_t y = __shfl_up(incl, off, 64);
      if (lane >= off) incl += y;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    int64_t before = carry;
    for (int k = 0; k < wv; k++) before += wsum[k];
    if (i < C.batile_n) {
      const int64_t start = before + incl - x;
      b.basums[C.batile_base + i] = start;
      const Tile tt = tiles[C.batile_base + i];
      if (tt.k == 0) b.states[tt.page].byte_base = start;
    }
    __syncthreads();
    if (t == 0) carry += wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
  }
  if (t == 0) b.chunk_bytes[c] = carry;
}

// Byte copy of one value (unaligned on both sides; values average tens of bytes).
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
// k_ba_expand: per tile, 8 consecutive values per thread: block scan of lengths -> offsets, then
// the bytes of each value copied from its source (page chain / DELTA_LENGTH data / dictionary).
// DELTA_LENGTH reads past the page (io.ReadFull short) are found here: the first value whose bytes
// do not fit is the page's error.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_ba_expand(DevBatch b, const Tile* tiles) {
  __shared__ uint64_t wsum[4];
  const Tile t = tiles[blockIdx.x];
  const DevPage P = b.pages[t.page];
  const PageState S = b.states[t.page];
  if (page_failed_before_values(S)) return;
  const DevChunk C = b.chunks[P.chunk];
  const int64_t lim = ba_limit(b, t.page, P, S);
  const int64_t v0 = int64_t(t.k) * kBaTile;
  const int64_t v1 = v0 + kBaTile < lim ? v0 + kBaTile : lim;
  if (v0 >= v1) return;
  const bool is_dict = P.kind == K_DICT, is_dlba = P.kind == K_DLBA;
  const BaDict d = is_dict ? ba_dict(b, P) : BaDict{nullptr, 0, 0};
  const int32_t* aux = C.aux + S.value_base;
  const int64_t i0 = v0 + 8 * int64_t(threadIdx.x);
  int64_t len[8];
  int32_t a[8];
  int64_t tsum = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    a[j] = i0 + j < v1 ? aux[i0 + j] : 0;
    len[j] = i0 + j < v1 ? ba_len(d, is_dict, a[j]) : 0;
    tsum += len[j] > 0 ? len[j] : 0;
  }
  uint64_t tot;
  const int64_t excl = int64_t(block_exclusive_scan(uint64_t(tsum), wsum, &tot));
  const int64_t base = b.basums[P.batile_base + t.k];
  const uint8_t* img = b.payload + P.image_off;
  int64_t data_s = 0, data_n = 0;
  if (is_dlba) {
    data_s = b.dstates[t.page].end_pos;
    data_n = S.val_e - data_s;
  }
  int64_t* offs = C.offsets + S.value_base + 1;
  int64_t o = base + excl;
  int64_t first_bad = INT64_MAX;
  int bad_code = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const int64_t i = i0 + j;
    if (i >= v1) break;
    const int64_t l = len[j] > 0 ? len[j] : 0;
    const int64_t rel = o - S.byte_base;  // page-relative first byte
    const uint8_t* src = nullptr;
    if (is_dict) {
      const uint32_t k = uint32_t(a[j]);
      if (k < d.K) src = b.payload + d.base + 4 * int64_t(k + 1) + d.dcum[k];
    } else if (is_dlba) {
      const int64_t rem = data_n - rel;
      if (len[j] > 0 && rem < len[j]) {
        if (i < first_bad) {
          first_bad = i;
          bad_code = rem <= 0 ? PQH_ERR_EOF : PQH_ERR_UNEXPECTED_EOF;
        }
      } else {
        src = img + data_s + rel;
      }
    } else {  // PLAIN: value i's bytes follow its u32 length
      src = img + S.val_s + 4 * (i + 1) + rel;
    }
    if (src && l > 0 && o + l <= C.bytes_cap) copy_bytes(C.bytes + o, src, l);
    o += l;
    offs[i] = o;
  }
  if (first_bad != INT64_MAX) atomicMin(&b.states[t.page].err, (unsigned long long)err_key(3, first_bad, bad_code));
}
