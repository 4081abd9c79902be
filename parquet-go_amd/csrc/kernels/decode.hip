// decode.hip — hand-written HIP kernels (gfx950 / CDNA4) for Parquet page decode.
//
// Two-pass design for the sequential chains inside a page (SURVEY.md §7 "Hard parts"):
//   1. k_prologue   one wave64 per page: page framing (page_v1.go:87-122 / page_v2.go:79-131),
//                   the hybrid RLE/bit-packed run-header chain of every stream
//                   (hybrid_decoder.go:81-165) with a run CHECKPOINT at every tile boundary, the
//                   not-null count (helpers.go:133-149, wave-parallel over bit-packed groups), and
//                   the exact first-error position of the reference's streaming decoders;
//   2. k_scan       one workgroup per chunk: dense value offsets = exclusive scan of notNull;
//   3. expand       data-parallel tiles over HBM-resident page images: level bytes, dictionary
//                   gathers (dictionary staged in LDS), PLAIN copies and boolean bit expansion.
// All bandwidth kernels: 16-byte vector loads/stores, no MFMA.
#define PQH_KERNELS_TU 1  // output pointers in the global address space (decode.h)
#include <hip/hip_runtime.h>

#include "launch.h"
#include "pqhip.h"

namespace pqhip {

// ------------------------------------------------------------------------------------------------
// helpers
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t ld64u(const uint8_t* p) {
  uint64_t v;
  __builtin_memcpy(&v, p, 8);
  return v;
}

// 8 bytes at p; bytes at or past `end` read as zero (the reference zero-fills a short bit-packed
// group read: hybrid_decoder.go:132-140).  `end` never exceeds the payload, which carries
// PQH_PAYLOAD_PAD readable bytes, so one 8-byte load at p < end stays inside the allocation.
__device__ __forceinline__ uint64_t ld64_masked(const uint8_t* p, const uint8_t* end) {
  const int64_t n = end - p;
  if (n <= 0) return 0;
  const uint64_t v = ld64u(p);
  return n >= 8 ? v : (v & ((1ull << (8 * n)) - 1));
}

__device__ __forceinline__ int bits_len32(uint32_t v) { return v ? 32 - __clz(int(v)) : 0; }

__device__ __forceinline__ int64_t wave_sum(int64_t x) {
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off, 64);
  return x;
}

// binary.ReadUvarint over img[pos, end) (encoding/binary; readUVariant32 helpers.go:151-167).
__device__ int read_uvarint(const uint8_t* img, int64_t& pos, int64_t end, uint64_t& v) {
  uint64_t x = 0;
  int s = 0;
  for (int i = 0; i < 10; i++) {
    if (pos >= end) return i ? PQH_ERR_UNEXPECTED_EOF : PQH_ERR_EOF;
    uint32_t c = img[pos++];
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

// Workgroup copy of nvec 16-byte vectors from src + 16k into LDS dst[k]; vectors at or past
// `limit` (an offset from src) read as zeros.  Four vectors per thread are in flight at a time
// (loads unconditional from a clamped address, then selected), so a tile costs one round trip per
// 16 KiB instead of one per 4 KiB.
__device__ __forceinline__ void stage_copy(uint4* dst, const uint8_t* src_, int64_t nvec, int64_t limit) {
  // the payload is HBM: global loads (the generic pointer would compile to flat loads)
  const PQH_G uint8_t* src = (const PQH_G uint8_t*)(src_);
  for (int64_t base = 0; base < nvec; base += 4 * kBlock) {
    uint4 x[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int64_t k = base + threadIdx.x + j * kBlock;
      const bool ok = k < nvec && 16 * k < limit;
      x[j] = *reinterpret_cast<const PQH_G uint4*>(src + (ok ? 16 * k : 0));
      if (!ok) x[j] = make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int64_t k = base + threadIdx.x + j * kBlock;
      if (k < nvec) dst[k] = x[j];
    }
  }
}

__device__ __forceinline__ uint32_t mask_w(int w) { return w >= 32 ? 0xffffffffu : ((1u << w) - 1u); }

// Value i of a bit-packed run whose first group starts at byte `data`.
__device__ __forceinline__ uint32_t bp_value(const uint8_t* img, const uint8_t* end, int32_t data, int64_t rel, int w) {
  int64_t bit = rel * w;
  const uint8_t* p = img + data + (bit >> 3);
  return uint32_t(ld64_masked(p, end) >> (bit & 7)) & mask_w(w);
}

// ------------------------------------------------------------------------------------------------
// Hybrid run-header walk (one wave, uniform control flow).  Replays hybridDecoder.next for the
// first N values of a stream: headers, RLE values, the lazy bit-packed group reads and their
// errors; writes a checkpoint for every tile of kHybridTile values; optionally counts values equal
// to `match` (definition levels == maxD -> notNull).
// ------------------------------------------------------------------------------------------------
struct WalkOut {
  uint64_t err;
  int64_t count;
  int64_t fail_index;
};

// Every wave of the page's workgroup walks the same headers (wave-uniform, L2-hot after the first);
// the value counting inside bit-packed runs is split over the nwv waves (wave wv takes every nwv-th
// 64-lane slice) and count is this wave's share; wave 0 alone writes the checkpoints.
// kCount = false compiles the counting out (match must be -1): k_flat's walks, which count nothing.
template <bool kCount = true>
__device__ __forceinline__ WalkOut walk_hybrid(const uint8_t* img, int64_t s, int64_t e, int w, int64_t N, int phase, Ckpt* ck,
                               int match, int lane, int wv = 0, int nwv = 1) {
  WalkOut o{kNoError, 0, N};
  if (N <= 0) return o;
  const int64_t T = kHybridTile;
  if (w == 0) {  // infinite zeros, no reads (hybrid_decoder.go:82-85)
    if (ck && wv == 0)
      for (int64_t k = lane; k * T < N; k += 64) ck[k] = Ckpt{0, 0x7fffffff, 0, 0};
    o.count = match == 0 && wv == 0 ? N : 0;
    return o;
  }
  const uint8_t* end = img + e;
  const int rle_size = (w + 7) >> 3;
  const uint32_t m = mask_w(w);
  int64_t pos = s, produced = 0, next_ck = 0, cnt_lane = 0;
  while (produced < N) {
    uint64_t h;
    int st = read_uvarint(img, pos, e, h);
    if (st) {
      o.err = err_key(phase, produced, st);
      o.fail_index = produced;
      break;
    }
    if (h > 0x7fffffffull) {
      o.err = err_key(phase, produced, PQH_ERR_INT32_RANGE);
      o.fail_index = produced;
      break;
    }
    const bool bp = h & 1;
    int64_t cnt, next, fail = -1;
    int32_t data;
    if (bp) {
      const int64_t groups = int64_t(h >> 1);
      if (groups == 0) {
        o.err = err_key(phase, produced, PQH_ERR_EMPTY_BP_RUN);
        o.fail_index = produced;
        break;
      }
      cnt = groups * 8;
      data = int32_t(pos);
      const int64_t need = cnt < N - produced ? cnt : N - produced;
      const int64_t gneed = (need + 7) >> 3;
      const int64_t gf = pos >= e ? 0 : (e - pos + w - 1) / w;  // first group read that hits EOF
      if (gf < gneed) fail = produced + 8 * gf;
      next = pos + groups * w;
    } else {
      cnt = int64_t(h >> 1);
      if (cnt == 0) {
        o.err = err_key(phase, produced, PQH_ERR_EMPTY_RLE_RUN);
        o.fail_index = produced;
        break;
      }
      if (pos >= e || pos + rle_size > e) {  // readRLERunValue: Read -> EOF or short count
        o.err = err_key(phase, produced, pos >= e ? PQH_ERR_EOF : PQH_ERR_UNEXPECTED_EOF);
        o.fail_index = produced;
        break;
      }
      uint32_t v = 0;
      for (int k = 0; k < rle_size; k++) v |= uint32_t(img[pos + k]) << (8 * k);
      if (w < 32 && (v >> w) != 0) {
        o.err = err_key(phase, produced, PQH_ERR_RLE_VALUE_TOO_LARGE);
        o.fail_index = produced;
        break;
      }
      data = int32_t(v);
      next = pos + rle_size;
    }
    const int64_t valid_end = fail >= 0 ? fail : produced + cnt;
    if (ck) {
      const int32_t nh = int32_t(next < 0x7fffffff ? next : 0x7fffffff) | (bp ? int32_t(0x80000000u) : 0);
      const int32_t rl = int32_t(cnt < 0x7fffffff ? cnt : 0x7fffffff);
      while (next_ck * T < N && next_ck * T < valid_end) {
        if (lane == 0 && wv == 0) ck[next_ck] = Ckpt{int32_t(produced), rl, data, nh};
        next_ck++;
      }
    }
    if (kCount && match >= 0) {
      const int64_t lim = (valid_end < N ? valid_end : N) - produced;
      if (!bp) {
        if (lane == 0 && wv == 0 && data == match) cnt_lane += lim;
      } else if (w == 1) {
        // one bit per value: popcount 128 values per lane-load (16-byte loads, many in flight)
        int64_t ones = 0;
        for (int64_t c0 = int64_t(wv) * 64; c0 * 128 < lim; c0 += int64_t(64) * 8 * nwv) {  // 8 chunks per lane in flight
          uint64_t a[8], bq[8];
#pragma unroll
          for (int k = 0; k < 8; k++) {
            const int64_t c = c0 + int64_t(k) * 64 * nwv + lane;
            const uint8_t* p = img + data + c * 16;
            const bool in = c * 128 < lim;
            a[k] = in ? ld64_masked(p, end) : 0;
            bq[k] = in ? ld64_masked(p + 8, end) : 0;
          }
#pragma unroll
          for (int k = 0; k < 8; k++) {
            const int64_t c = c0 + int64_t(k) * 64 * nwv + lane;
            const int64_t nb = lim - c * 128;  // valid bits in this chunk
            if (nb <= 0) continue;
            const uint64_t ma = nb >= 64 ? ~0ull : ((1ull << nb) - 1);
            const uint64_t mb = nb >= 128 ? ~0ull : nb <= 64 ? 0ull : ((1ull << (nb - 64)) - 1);
            const int64_t valid = nb < 128 ? nb : 128;
            const int64_t pc = __popcll(a[k] & ma) + __popcll(bq[k] & mb);
            ones += pc;
            if (match == 0) cnt_lane += valid - pc;
          }
        }
        if (match == 1) cnt_lane += ones;
      } else if (w == 2 || w == 4 || w == 8) {
        // whole fields per 64-bit word: t = word ^ (match in every field); OR-folding each
        // field's bits into its low bit leaves that bit clear exactly for the matching values
        const uint64_t lowm = w == 2 ? 0x5555555555555555ull : w == 4 ? 0x1111111111111111ull : 0x0101010101010101ull;
        const uint64_t pat = lowm * uint64_t(uint32_t(match));
        const int per = 64 / w;
        const int64_t nw = (lim + per - 1) / per;
        // 16 words per lane in flight (one wave walks a whole page: latency, not bandwidth, bound)
        for (int64_t c0 = int64_t(wv) * 64; c0 < nw; c0 += int64_t(64) * 16 * nwv) {
          uint64_t t[16];
#pragma unroll
          for (int k = 0; k < 16; k++) {
            const int64_t c = c0 + int64_t(k) * 64 * nwv + lane;
            t[k] = c < nw ? ld64_masked(img + data + c * 8, end) : 0;
          }
#pragma unroll
          for (int k = 0; k < 16; k++) {
            const int64_t c = c0 + int64_t(k) * 64 * nwv + lane;
            uint64_t x = t[k] ^ pat;
            x |= x >> 1;
            if (w >= 4) x |= x >> 2;
            if (w == 8) x |= x >> 4;
            const int64_t nv = lim - c * per;  // valid values in this word
            const uint64_t valid = nv >= per ? lowm : nv <= 0 ? 0ull : (lowm & ((1ull << (nv * w)) - 1));
            cnt_lane += __popcll(valid & ~x);
          }
        }
      } else {
#pragma unroll 2
        for (int64_t g = int64_t(wv) * 64 + lane; g * 8 < lim; g += 64 * nwv) {
          const uint64_t q = ld64_masked(img + data + g * w, end);
          const uint64_t q2 = w > 8 ? ld64_masked(img + data + g * w + 8, end) : 0;
          for (int j = 0; j < 8; j++) {
            const int bit = j * w;
            uint32_t v;
            if (bit + w <= 64) v = uint32_t(q >> bit) & m;
            else if (bit >= 64) v = uint32_t(q2 >> (bit - 64)) & m;
            else v = uint32_t((q >> bit) | (q2 << (64 - bit))) & m;
            cnt_lane += (g * 8 + j < lim) && (int(v) == match);
          }
        }
      }
    }
    if (fail >= 0) {
      o.err = err_key(phase, fail, PQH_ERR_EOF);
      o.fail_index = fail;
      break;
    }
    produced += cnt;
    pos = next;
  }
  o.count = wave_sum(cnt_lane);
  return o;
}

// ------------------------------------------------------------------------------------------------
// k_prologue: kNwv waves per page.  kNwv = 1: four pages per workgroup (flat batches: short level
// streams); kNwv = 4: one page per workgroup (batches with repeated columns: long level streams),
// its four waves run the same (wave-uniform) framing and run walks and split the notNull count
// over bit-packed definition levels.
// ------------------------------------------------------------------------------------------------
// k_flat's nullable flat pages (max_def 1, V2): the definition levels [s, e) as ONE bit-packed run of
// width 1 covering the n slots (the reference writer's layout, hybrid_encoder.go:55-70) -> notNull =
// the popcount of its first n bits; -1 for any other stream (the page check then fails and the three
// kernels decode the batch, walking the levels exactly).  Wave-uniform.
__device__ __forceinline__ int64_t flat_def_count(const uint8_t* img, int64_t s, int64_t e, int64_t n, int lane) {
  if (n <= 0) return 0;
  uint64_t h = 0;
  int len = 0;
  for (int k = 0; k < 5 && s + k < e; k++) {
    const uint32_t c = img[s + k];
    h |= uint64_t(c & 0x7f) << (7 * k);
    if (c < 0x80) {
      len = k + 1;
      break;
    }
  }
  if (len == 0 || h > 0x7fffffffull || !(h & 1) || int64_t(h >> 1) * 8 < n) return -1;
  const int64_t data = s + len, nbytes = (n + 7) >> 3;
  if (data + nbytes > e) return -1;
  int64_t cnt = 0;
  for (int64_t i = lane; i < nbytes; i += 64) {
    uint32_t x = img[data + i];
    if (i == nbytes - 1 && (n & 7)) x &= (1u << (n & 7)) - 1;
    cnt += __popc(x);
  }
  for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off, 64);
  return cnt;
}

// kLevels = false (k_flat): the page's column has no level streams, or (nullable flat, V2) one
// single-run definition stream counted by flat_def_count; any other page gets PQH_ERR_INTERNAL,
// which k_flat's check turns into a decode by the three kernels.
template <int kNwv, bool kLevels = true>
__device__ __forceinline__ PageState prologue_page(const DevBatch& b, int p, int lane, int wv, int64_t* s_nn,
                                                   bool store = true) {
  const DevPage P = b.pages[p];
  const DevChunk C = b.chunks[P.chunk];
  const uint8_t* img = b.payload + P.image_off;
  const int64_t L = P.image_len;

  PageState S;
  S.err = P.host_err;
  S.nn = 0;
  S.width = 0;
  S.rep_s = S.rep_e = S.def_s = S.def_e = -1;
  S.val_s = S.val_e = 0;
  S.val_limit = 0;
  S.dict_n = 0;
  S.ba_summed = 0;
  S.value_base = 0;
  S.byte_base = 0;
  uint64_t err = P.host_err;

  if (err == kNoError && P.page_type == PQH_DICTIONARY_PAGE) {
    // dictPageReader.read: PLAIN decode of num_values entries, no error tolerated (page_dict.go:60-70)
    const int64_t n = P.num_values;
    const int vs = P.value_size;
    if (vs > 0) {
      const int64_t cap = L / vs, rem = L - cap * vs;
      if (cap < n) {
        if (P.kind == K_PLAIN_INT96 && rem != 0 && cap == n - 1)
          S.dict_n = int32_t(n);  // the short last entry stays nil: no error (type_int96.go:21-42)
        else if (P.kind == K_PLAIN_INT96 && rem != 0)
          err = err_key(0, cap + 1, PQH_ERR_EOF);
        else
          err = err_key(0, cap, rem == 0 ? PQH_ERR_EOF : PQH_ERR_UNEXPECTED_EOF);
      } else {
        S.dict_n = int32_t(n);
      }
    } else if (P.kind == K_FLBA_NEGATIVE) {  // byteArrayPlainDecoder{length < 0}: first value fails
      if (n > 0) err = err_key(0, 0, PQH_ERR_NEGATIVE_LENGTH);
    }
    // byte-array dictionaries (K_PLAIN_BA): the PLAIN chain is walked by k_ba_walk
  } else if (err == kNoError) {
    const int64_t n = P.num_values;
    const int rw = bits_len32(uint32_t(C.max_rep)), dw = bits_len32(uint32_t(C.max_def));
    int64_t rep_s = -1, rep_e = -1, def_s = -1, def_e = -1, vs, ve = L;
    // --- pageReader.read: level decoders initSize (V1) / init (V2), then valuesDecoder.init ---
    if (P.page_type == PQH_DATA_PAGE) {
      int64_t pos = 0;
      for (int k = 0; k < 2 && err == kNoError; k++) {
        if ((k == 0 ? rw : dw) == 0) continue;
        if (L - pos < 4) {
          err = err_key(0, 1 + k, L - pos == 0 ? PQH_ERR_EOF : PQH_ERR_UNEXPECTED_EOF);
          break;
        }
        const uint32_t size = uint32_t(img[pos]) | (uint32_t(img[pos + 1]) << 8) | (uint32_t(img[pos + 2]) << 16) |
                              (uint32_t(img[pos + 3]) << 24);
        const int64_t s0 = pos + 4;
        const int64_t e0 = s0 + (int64_t(size) < L - s0 ? int64_t(size) : L - s0);
        if (k == 0) {
          rep_s = s0;
          rep_e = e0;
        } else {
          def_s = s0;
          def_e = e0;
        }
        pos = e0;
      }
      vs = pos;
    } else {
      const int64_t rl = P.rep_len, dl = P.def_len;
      if (rl > 0 && rw > 0) {
        rep_s = 0;
        rep_e = rl;
      }
      if (dl > 0 && dw > 0) {
        def_s = rl;
        def_e = rl + dl;
      }
      vs = rl + dl;
    }
    int64_t hs = vs, he = ve;  // value hybrid stream
    if (err == kNoError) {
      if (P.kind == K_DICT) {  // dictDecoder.init (type_dict.go:22-38)
        if (vs >= ve) {
          err = err_key(0, 3, PQH_ERR_EOF);
        } else {
          const int w = img[vs];
          if (w > 32) err = err_key(0, 3, PQH_ERR_DICT_BIT_WIDTH);
          S.width = int16_t(w);
          hs = vs + 1;
        }
      } else if (P.kind == K_RLE_BOOL) {  // booleanRLEDecoder.init -> initSize (type_boolean.go:104-107)
        if (ve - vs < 4) {
          err = err_key(0, 3, ve - vs == 0 ? PQH_ERR_EOF : PQH_ERR_UNEXPECTED_EOF);
        } else {
          const uint32_t size = uint32_t(img[vs]) | (uint32_t(img[vs + 1]) << 8) | (uint32_t(img[vs + 2]) << 16) |
                                (uint32_t(img[vs + 3]) << 24);
          hs = vs + 4;
          he = hs + (int64_t(size) < ve - hs ? int64_t(size) : ve - hs);
          S.width = 1;
        }
      }
    }
    S.rep_s = int32_t(rep_s);
    S.rep_e = int32_t(rep_e);
    S.def_s = int32_t(def_s);
    S.def_e = int32_t(def_e);
    S.val_s = int32_t(hs);
    S.val_e = int32_t(he);
    // --- readValues(numValues) ---
    int64_t flat_nn = -1;  // k_flat: the notNull of a nullable flat page's single-run definition levels
    if constexpr (!kLevels) {
      if (rw > 0 || dw > 1 || (dw == 1 && (P.page_type != PQH_DATA_PAGE_V2 || def_s < 0 ||
                                           (flat_nn = flat_def_count(img, def_s, def_e, n, lane)) < 0)))
        err = err_key(0, 0, PQH_ERR_INTERNAL);
    }
    if (err == kNoError && n > 0) {
      if (kLevels && rw > 0) {  // decodePackedArray(rDecoder, n)
        if (rep_s < 0) {
          err = err_key(1, 0, PQH_ERR_READER_NOT_INITIALIZED);
        } else {
          WalkOut r = walk_hybrid(img, rep_s, rep_e, rw, n, 1, P.ck_rep >= 0 ? b.ckpts + P.ck_rep : nullptr, -1, lane, wv, kNwv);
          err = r.err;
        }
      }
      int64_t nn = !kLevels && dw == 1 ? flat_nn : n;
      if (kLevels && err == kNoError && dw > 0) {  // decodePackedArray(dDecoder, n) + notNull
        if (def_s < 0) {
          err = err_key(2, 0, PQH_ERR_READER_NOT_INITIALIZED);
        } else {
          WalkOut r = walk_hybrid(img, def_s, def_e, dw, n, 2, P.ck_def >= 0 ? b.ckpts + P.ck_def : nullptr, C.max_def, lane, wv, kNwv);
          err = r.err;
          nn = r.count;  // this wave's share: summed below
        }
      }
      if (kNwv > 1 && dw > 0) {  // uniform over the workgroup (same page, same walk)
        if (lane == 0) s_nn[wv] = nn;
        __syncthreads();
        nn = s_nn[0] + s_nn[1] + s_nn[2] + s_nn[3];
      }
      if (err == kNoError) {
        S.nn = int32_t(nn);
        int64_t limit = nn;
        if (nn > 0) {
          const int64_t avail = ve - vs;
          switch (P.kind) {
            case K_DICT:
            case K_RLE_BOOL: {
              WalkOut r = walk_hybrid<kLevels>(img, hs, he, S.width, nn, 3, P.ck_val >= 0 ? b.ckpts + P.ck_val : nullptr, -1,
                                               lane, wv, kNwv);
              err = r.err;
              limit = r.fail_index;
              break;
            }
            case K_PLAIN_FIXED: {  // binary.Read / io.ReadFull per value
              const int64_t cap = avail / P.value_size, rem = avail - cap * P.value_size;
              if (cap < nn) {
                err = err_key(3, cap, rem == 0 ? PQH_ERR_EOF : PQH_ERR_UNEXPECTED_EOF);
                limit = cap;
              }
              break;
            }
            case K_PLAIN_INT96: {  // int96PlainDecoder.decodeValues (type_int96.go:21-42)
              const int64_t cap = avail / 12, rem = avail - cap * 12;
              if (cap < nn) {
                // a short LAST value ends the loop with dst[nn-1] never assigned: success, a nil slot
                // (zeros; k_scan marks it in value_nil); a short value before it: io.EOF next read
                if (rem == 0) err = err_key(3, cap, PQH_ERR_EOF);
                else if (cap != nn - 1) err = err_key(3, cap + 1, PQH_ERR_EOF);
                limit = cap;
              }
              break;
            }
            case K_PLAIN_BOOL: {  // one io.ReadFull(1 byte) per 8 values (type_boolean.go:43-69)
              if (avail * 8 < nn) {
                err = err_key(3, avail * 8, PQH_ERR_EOF);
                limit = avail * 8;
              }
              break;
            }
            case K_DELTA32:
            case K_DELTA64:  // init + block walk in k_delta_walk (atomicMin into the same key)
            case K_DLBA:     // lengths: k_delta_walk; bytes: k_ba_expand
            case K_DBA:      // prefix + suffix lengths: k_delta_walk; bytes: k_dba_expand / k_dba_prefix
            case K_PLAIN_BA: // the [u32 len][bytes] chain: k_ba_walk
              break;
            case K_FLBA_NEGATIVE:
              err = err_key(3, 0, PQH_ERR_NEGATIVE_LENGTH);
              limit = 0;
              break;
            default:
              err = err_key(3, 0, PQH_ERR_UNSUPPORTED);
              limit = 0;
          }
        }
        S.val_limit = int32_t(limit);
      }
    }
  }
  S.err = err;
  if (store && lane == 0 && wv == 0) b.states[p] = S;
  return S;
}

template <int kNwv>
__global__ __launch_bounds__(256) void k_prologue(DevBatch b) {
  __shared__ int64_t s_nn[4];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(int(threadIdx.x >> 6) % kNwv);
  const int p = __builtin_amdgcn_readfirstlane(int(blockIdx.x) * (4 / kNwv) + int(threadIdx.x >> 6) / kNwv);
  if (p >= b.num_pages) return;
  prologue_page<kNwv>(b, p, lane, wv, s_nn);
}

// ------------------------------------------------------------------------------------------------
// k_scan: one workgroup per chunk; dense value offsets.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ bool page_failed_before_values(const PageState& s) {
  return s.err != kNoError && (s.err >> 56) <= 2;
}

__global__ __launch_bounds__(256) void k_scan(DevBatch b) {
  const DevChunk C = b.chunks[blockIdx.x];
  __shared__ int64_t wsum[4];
  __shared__ int64_t carry;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  if (t == 0) carry = 0;
  __syncthreads();
  for (int base = 0; base < C.num_pages; base += 256) {
    const int i = base + t;
    const int p = C.first_page + i;
    int64_t nn = 0;
    if (i < C.num_pages && b.pages[p].page_type != PQH_DICTIONARY_PAGE) {
      const PageState s = b.states[p];
      nn = page_failed_before_values(s) ? 0 : s.nn;
    }
    int64_t x = nn;  // inclusive wave scan
    for (int off = 1; off < 64; off <<= 1) {
      const int64_t y = __shfl_up(x, off, 64);
      if (lane >= off) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    int64_t before = carry;
    for (int k = 0; k < wv; k++) before += wsum[k];
    if (i < C.num_pages) b.states[p].value_base = before + x - nn;
    // a PLAIN INT96 page whose short last value is the reference's nil (prologue: no error, limit =
    // notNull - 1): mark that dense slot (its 12 bytes stay the zeros of the plan-time fill)
    if (C.value_nil && i < C.num_pages && nn > 0 && b.pages[p].kind == K_PLAIN_INT96 &&
        b.pages[p].page_type != PQH_DICTIONARY_PAGE) {
      const PageState s = b.states[p];
      if (s.err == kNoError && s.val_limit == s.nn - 1) C.value_nil[before + x - 1] = 1;
    }
    __syncthreads();
    if (t == 0) carry += wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
  }
  if (!C.ba_fused) return;
  // fused PLAIN chains (k_ba_chain): each page's string bytes taken as val_e - val_s - 4 * notNull,
  // which k_ba_chain verifies; any page error, or a page that cannot be so, sends the batch back to
  // the scratch path (bafuse[1])
  bool fail = false;
  if (t == 0) {
    carry = 0;
    if (C.offsets) C.offsets[0] = 0;
  }
  __syncthreads();
  for (int base = 0; base < C.num_pages; base += 256) {
    const int i = base + t;
    const int p = C.first_page + i;
    int64_t g = 0;
    if (i < C.num_pages) {
      const PageState s = b.states[p];
      if (s.err != kNoError || s.nn > (1 << 29) - 1) fail = true;
      if (s.nn > 0) g = int64_t(s.val_e) - s.val_s - 4 * int64_t(s.nn);
      if (g < 0) fail = true;
    }
    int64_t x = g;
    for (int off = 1; off < 64; off <<= 1) {
      const int64_t y = __shfl_up(x, off, 64);
      if (lane >= off) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();
    int64_t before = carry;
    for (int k = 0; k < wv; k++) before += wsum[k];
    if (i < C.num_pages) b.states[p].byte_base = before + x - g;
    __syncthreads();
    if (t == 0) carry += wsum[0] + wsum[1] + wsum[2] + wsum[3];
    __syncthreads();
  }
  if (t == 0) b.chunk_bytes[blockIdx.x] = carry;
  if (fail) __hip_atomic_store(b.bafuse + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}


// ------------------------------------------------------------------------------------------------
// Tile expansion of a hybrid stream from a checkpoint.  Thread 0 re-walks the (already validated)
// run headers of the tile into an LDS run list.  A tile inside ONE bit-packed run (every
// reference-writer stream: hybrid_encoder.go:55-70) takes the width-templated fast path: each
// thread owns 8 groups of 8 values, strided by the workgroup, with all their loads in flight;
// a tile inside one RLE run is a fill; anything else (pyarrow-style mixed runs) takes the general
// per-group path.
// ------------------------------------------------------------------------------------------------
constexpr int kMaxRuns = 256;

struct RunL {
  int32_t start, end, data, bp;
};

struct TileLds {
  RunL runs[kMaxRuns];
  int32_t nruns;
  int32_t seg_end;
  int32_t next_pos;
  int32_t pad;
};

// Build the run list for values up to t1 starting at run {rs, rl, data, bp} whose successor's
// header is at `pos`.  One thread.
__device__ __noinline__ void build_runs(const uint8_t* img, int w, int64_t t1, int64_t rs, int64_t rl, int32_t data, int32_t bp,
                           int64_t pos, TileLds& L) {
  int n = 0;
  int64_t cur_end = rs + rl;
  L.runs[n++] = RunL{int32_t(rs), int32_t(cur_end < t1 ? cur_end : t1), data, bp};
  const int rle_size = (w + 7) >> 3;
  while (cur_end < t1 && n < kMaxRuns) {
    uint64_t h = 0;
    int64_t pp = pos;
    read_uvarint(img, pp, int64_t(0x7fffffffffffll), h);  // validated by k_prologue
    int64_t cnt;
    int32_t d, isbp;
    if (h & 1) {
      cnt = int64_t(h >> 1) * 8;
      d = int32_t(pp);
      pos = pp + int64_t(h >> 1) * w;
      isbp = 1;
    } else {
      cnt = int64_t(h >> 1);
      uint32_t v = 0;
      for (int k = 0; k < rle_size; k++) v |= uint32_t(img[pp + k]) << (8 * k);
      d = int32_t(v);
      pos = pp + rle_size;
      isbp = 0;
    }
    const int64_t e = cur_end + cnt;
    L.runs[n++] = RunL{int32_t(cur_end), int32_t(e < t1 ? e : t1), d, isbp};
    cur_end = e;
  }
  L.nruns = n;
  L.seg_end = int32_t(cur_end < t1 ? cur_end : t1);
  L.next_pos = int32_t(pos < 0x7fffffff ? pos : 0x7fffffff);
}

__device__ __forceinline__ int find_run(const TileLds& L, int64_t i) {
  int lo = 0, hi = L.nruns - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (L.runs[mid].start <= i) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// General path: up to 8 values [i0, i0+cnt) from the LDS run list.
__device__ __forceinline__ void decode8(const uint8_t* img, const uint8_t* end, int w, const TileLds& L, int64_t i0,
                                        int cnt, uint32_t v[8]) {
  int r = find_run(L, i0);
  RunL R = L.runs[r];
  if (i0 + 8 <= R.end) {
    if (!R.bp) {
      for (int j = 0; j < 8; j++) v[j] = uint32_t(R.data);
      return;
    }
    const int64_t rel = i0 - R.start;
    for (int j = 0; j < 8; j++) v[j] = bp_value(img, end, R.data, rel + j, w);
    return;
  }
  for (int j = 0; j < cnt; j++) {
    const int64_t i = i0 + j;
    while (i >= R.end && r + 1 < L.nruns) R = L.runs[++r];
    v[j] = R.bp ? bp_value(img, end, R.data, i - R.start, w) : uint32_t(R.data);
  }
}

// Fast path for a segment inside ONE bit-packed run: the segment's packed bytes are staged in LDS
// with coalesced, aligned 16-byte loads (all in flight), bytes past the stream end zeroed; each
// value is then two LDS dwords + alignbit, for any width 1..32 at run time.
constexpr int kStageBytes = 16384;

template <class Sink>
__device__ void bp_staged(const uint8_t* img, int64_t e, int w, int64_t data, int64_t rs, int64_t t0, int64_t t1,
                          uint32_t* stage, Sink& sink) {
  const uint32_t m = mask_w(w);
  const uint8_t* end = img + e;
  int64_t chunk = (int64_t(kStageBytes - 32) * 8 / w) & ~int64_t(8 * kBlock - 1);
  if (chunk < 8 * kBlock) chunk = 8 * kBlock;
  for (int64_t c0 = t0; c0 < t1; c0 += chunk) {
    const int64_t c1 = c0 + chunk < t1 ? c0 + chunk : t1;
    const uint8_t* p0 = img + data + ((c0 - rs) >> 3) * w;        // group-aligned start
    const uint8_t* p1 = img + data + ((c1 - rs + 7) >> 3) * w;    // group-rounded end
    const uint8_t* a0 = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(p0) & ~uintptr_t(15));
    const int64_t nvec = (p1 - a0 + 15) >> 4;
    const uint32_t lead_bits = uint32_t(p0 - a0) * 8;
    __syncthreads();  // previous chunk fully consumed
    stage_copy(reinterpret_cast<uint4*>(stage), a0, nvec, end - a0);
    if (end > a0 && end - a0 < nvec * 16 && ((end - a0) & 15)) {
      // the vector holding the stream end: zero the bytes past it (the reference's short group
      // read is zero-filled)
      const int64_t kv = (end - a0) >> 4;
      __syncthreads();  // the copy of vector kv is done
      if (threadIdx.x < 4) {
        const int64_t vb = (end - a0) - 16 * kv - 4 * int64_t(threadIdx.x);
        uint32_t& wq = stage[kv * 4 + threadIdx.x];
        wq = vb >= 4 ? wq : vb <= 0 ? 0u : (wq & ((1u << (8 * vb)) - 1u));
      }
    }
    if (threadIdx.x < 2) stage[nvec * 4 + threadIdx.x] = 0;  // the words after the last one (funnel shifts read k+1, k+2)
    __syncthreads();
    // G values per thread and step (Sink::kGroup): 4 for 4-byte outputs, so that a wave's stores
    // are one contiguous kilobyte
    constexpr int G = Sink::kGroup;
    if (w * G <= 32) {
      // narrow values (levels, booleans, small dictionaries): a thread's G values fit one funnel
      // shift of two LDS dwords
      for (int64_t i0 = c0 + G * int64_t(threadIdx.x); i0 < c1; i0 += G * kBlock) {
        uint32_t v[8];
        const uint32_t bit0 = lead_bits + uint32_t(i0 - c0) * uint32_t(w);
        const uint32_t x = __builtin_amdgcn_alignbit(stage[(bit0 >> 5) + 1], stage[bit0 >> 5], bit0 & 31);
#pragma unroll
        for (int j = 0; j < G; j++) v[j] = (x >> (uint32_t(j) * uint32_t(w))) & m;
        sink(i0, v, int(c1 - i0 < G ? c1 - i0 : G));
      }
      continue;
    }
    if (w * G <= 64) {
      // up to 64 bits per group (dictionary indices up to 16 bits wide, 8-value groups up to 8):
      // two funnel shifts of three LDS dwords (the stage keeps slack words after its last one)
      for (int64_t i0 = c0 + G * int64_t(threadIdx.x); i0 < c1; i0 += G * kBlock) {
        uint32_t v[8];
        const uint32_t bit0 = lead_bits + uint32_t(i0 - c0) * uint32_t(w);
        const uint32_t k0 = bit0 >> 5, sh = bit0 & 31;
        const uint32_t s0 = stage[k0], s1 = stage[k0 + 1], s2 = stage[k0 + 2];
        const uint64_t x = uint64_t(__builtin_amdgcn_alignbit(s1, s0, sh)) |
                           (uint64_t(__builtin_amdgcn_alignbit(s2, s1, sh)) << 32);
#pragma unroll
        for (int j = 0; j < G; j++) v[j] = uint32_t(x >> (uint32_t(j) * uint32_t(w))) & m;
        sink(i0, v, int(c1 - i0 < G ? c1 - i0 : G));
      }
      continue;
    }
    for (int64_t i0 = c0 + G * int64_t(threadIdx.x); i0 < c1; i0 += G * kBlock) {
      uint32_t v[8];
      const uint32_t bit0 = lead_bits + uint32_t(i0 - c0) * uint32_t(w);
#pragma unroll
      for (int j = 0; j < G; j++) {
        const uint32_t bit = bit0 + uint32_t(j) * uint32_t(w);
        const uint32_t lo = stage[bit >> 5], hi = stage[(bit >> 5) + 1];
        v[j] = __builtin_amdgcn_alignbit(hi, lo, bit & 31) & m;
      }
      sink(i0, v, int(c1 - i0 < G ? c1 - i0 : G));
    }
  }
}

// Expand values [t0, t1) of a hybrid stream whose tile checkpoint is `c`; calls sink(i0, v, cnt)
// for every group of up to 8 values.  Must be called by the whole workgroup.
template <class Sink>
__device__ void expand_hybrid(const uint8_t* img, int64_t e, int w, const Ckpt& c, int64_t t0, int64_t t1,
                              TileLds& L, uint32_t* stage, Sink& sink) {
  const uint8_t* end = img + e;
  if (w == 0) {  // all zeros
    __syncthreads();  // LDS the sink reads (a staged dictionary) is ready
    for (int64_t i0 = t0 + 8 * int64_t(threadIdx.x); i0 < t1; i0 += 8 * kBlock) {
      uint32_t v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      sink(i0, v, int(t1 - i0 < 8 ? t1 - i0 : 8));
    }
    return;
  }
  int64_t from = t0;
  int64_t rs = c.run_start, rl = c.run_len, pos = c.next_hdr & 0x7fffffff;
  int32_t data = c.data, bp = (c.next_hdr >> 31) & 1;
  if (bp && rs + rl >= t1 && ((t0 - rs) & 7) == 0 && w <= 32) {
    // the checkpoint's bit-packed run holds the whole tile (every reference-writer stream): no
    // run list, straight to the staged unpack
    bp_staged(img, e, w, data, rs, t0, t1, stage, sink);
    return;
  }
  while (from < t1) {
    if (threadIdx.x == 0) build_runs(img, w, t1, rs, rl, data, bp, pos, L);
    __syncthreads();
    const int64_t seg_end = L.seg_end;
    const RunL r0 = L.runs[0];
    bool done = false;
    if (L.nruns == 1 && r0.end >= seg_end) {  // the whole segment lies in one run
      if (r0.bp) {
        if (((from - r0.start) & 7) == 0 && w <= 32) {
          bp_staged(img, e, w, r0.data, r0.start, from, seg_end, stage, sink);
          done = true;
        }
      } else {
        uint32_t v[8];
        for (int j = 0; j < 8; j++) v[j] = uint32_t(r0.data);
        for (int64_t i0 = from + 8 * int64_t(threadIdx.x); i0 < seg_end; i0 += 8 * kBlock)
          sink(i0, v, int(seg_end - i0 < 8 ? seg_end - i0 : 8));
        done = true;
      }
    }
    if (!done) {
      for (int64_t i0 = from + 8 * int64_t(threadIdx.x); i0 < seg_end; i0 += 8 * kBlock) {
        uint32_t v[8];
        const int cnt = int(seg_end - i0 < 8 ? seg_end - i0 : 8);
        decode8(img, end, w, L, i0, cnt, v);
        sink(i0, v, cnt);
      }
    }
    from = seg_end;
    pos = L.next_pos;
    __syncthreads();
    // the next segment starts exactly at a run header: an empty pseudo-run at `from`
    rs = from;
    rl = 0;
  }
}

// ------------------------------------------------------------------------------------------------
// Sinks: what a decoded group of up to 8 values turns into.
// ------------------------------------------------------------------------------------------------
// decodePackedArray into one byte per level slot.
struct LevelSink {
  static constexpr int kGroup = 8;
  uint8_t* out;
  __device__ __forceinline__ void operator()(int64_t i0, const uint32_t* v, int cnt) const {
    if (cnt == 8) {
      uint64_t x = 0;
      for (int j = 0; j < 8; j++) x |= uint64_t(v[j] & 0xff) << (8 * j);
      __builtin_memcpy(out + i0, &x, 8);
    } else {
      for (int j = 0; j < cnt; j++) out[i0 + j] = uint8_t(v[j]);
    }
  }
};

// booleanRLEDecoder.decodeValues (type_boolean.go:109-120): value == 1.
struct BoolSink {
  static constexpr int kGroup = 8;
  uint8_t* out;
  __device__ __forceinline__ void operator()(int64_t i0, const uint32_t* v, int cnt) const {
    if (cnt == 8) {
      uint64_t x = 0;
      for (int j = 0; j < 8; j++) x |= uint64_t(v[j] == 1) << (8 * j);
      __builtin_memcpy(out + i0, &x, 8);
    } else {
      for (int j = 0; j < cnt; j++) out[i0 + j] = uint8_t(v[j] == 1);
    }
  }
};

// dictDecoder.decodeValues (type_dict.go:40-60): bounds-checked gather of dictionary entries.
// NT: streaming (nontemporal) stores of full 4-byte groups -- k_flat's small batches, whose step
// ends with the kernel (C1 0.0209 -> 0.0185 ms); k_expand keeps cached stores (C2 1.397 vs 1.411 ms).
template <int VS, bool NT = false>
struct DictSink {
  static constexpr int kGroup = VS == 4 ? 4 : 8;
  const uint8_t* dict;  // LDS (fused kernel) or global (large dictionaries)
  uint8_t* out;         // chunk values + value_base * vs
  uint32_t K;
  int vs;               // runtime size when VS == 0
  int64_t* first_bad;   // per-thread min failing index
  uint8_t* nil = nullptr;  // VS == 0 (INT96): value_nil + value_base when the dictionary's last entry
                           // (key K - 1) is the reference's nil: such values are zeros, marked 1
  __device__ __forceinline__ void operator()(int64_t i0, const uint32_t* v, int cnt) const {
    if constexpr (VS == 4) {  // full group of in-range keys: one 16-byte store
      if (cnt == 4 && v[0] < K && v[1] < K && v[2] < K && v[3] < K) {
        const uint32_t* d = reinterpret_cast<const uint32_t*>(dict);
        if constexpr (NT) {
          // out + i0 * 4 is only 4-byte aligned in general (value bases are sums of page value
          // counts), so the vector type says so
          typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
          typedef u32x4 u32x4_a4 __attribute__((aligned(4)));
          const u32x4 a = {d[v[0]], d[v[1]], d[v[2]], d[v[3]]};
          __builtin_nontemporal_store(a, reinterpret_cast<PQH_G u32x4_a4*>((PQH_G uint8_t*)(out) + i0 * 4));
        } else {
          const uint4 a = make_uint4(d[v[0]], d[v[1]], d[v[2]], d[v[3]]);
          __builtin_memcpy(out + i0 * 4, &a, 16);
        }
        return;
      }
    }
    slow(i0, v, cnt);
  }
  __device__ __forceinline__ void slow(int64_t i0, const uint32_t* v, int cnt) const {
    // unrolled over the group (v[] stays in registers); the first out-of-range key of the group
    bool ok = true;
    int jb = 8;
#pragma unroll
    for (int j = 7; j >= 0; j--)
      if (j < cnt && v[j] >= K) jb = j;
    if (jb < 8) {
      ok = false;
      if (i0 + jb < *first_bad) *first_bad = i0 + jb;
    }
    if constexpr (VS == 4) {
      const uint32_t* d = reinterpret_cast<const uint32_t*>(dict);
      if (ok && cnt == 4) {
        uint4 a = make_uint4(d[v[0]], d[v[1]], d[v[2]], d[v[3]]);
        __builtin_memcpy(out + i0 * 4, &a, 16);
      } else if (ok && cnt == 8) {
        uint4 a = make_uint4(d[v[0]], d[v[1]], d[v[2]], d[v[3]]);
        uint4 c = make_uint4(d[v[4]], d[v[5]], d[v[6]], d[v[7]]);
        __builtin_memcpy(out + i0 * 4, &a, 16);
        __builtin_memcpy(out + i0 * 4 + 16, &c, 16);
      } else {
#pragma unroll
        for (int j = 0; j < 8; j++)
          if (j < cnt && v[j] < K) __builtin_memcpy(out + (i0 + j) * 4, &d[v[j]], 4);
      }
    } else if constexpr (VS == 8) {
      const uint64_t* d = reinterpret_cast<const uint64_t*>(dict);
      if (ok && cnt == 8) {
        for (int j = 0; j < 8; j += 2) {
          uint64_t pr[2] = {d[v[j]], d[v[j + 1]]};
          __builtin_memcpy(out + (i0 + j) * 8, pr, 16);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; j++)
          if (j < cnt && v[j] < K) __builtin_memcpy(out + (i0 + j) * 8, &d[v[j]], 8);
      }
    } else {
      for (int j = 0; j < cnt; j++) {
        if (v[j] >= K) continue;
        const uint8_t* src = dict + int64_t(v[j]) * vs;
        uint8_t* dst = out + (i0 + j) * vs;
        if (nil && v[j] == K - 1) {  // dst[i] = uniqueValues[K-1] = nil (type_dict.go:57)
          for (int k = 0; k < vs; k++) dst[k] = 0;
          nil[i0 + j] = 1;
          continue;
        }
        int k = 0;
        for (; k + 4 <= vs; k += 4) {
          uint32_t x;
          __builtin_memcpy(&x, src + k, 4);
          __builtin_memcpy(dst + k, &x, 4);
        }
        for (; k < vs; k++) dst[k] = src[k];
      }
    }
  }
};

// Byte-array dictionary pages: the index stream becomes per-value keys (aux); lengths and bytes are
// resolved against the dictionary's cumulative-bytes table by k_ba_sum / k_ba_expand.
struct KeySink {
  static constexpr int kGroup = 4;
  int32_t* out;  // chunk aux + value_base
  uint32_t K;
  int64_t* first_bad;
  __device__ __forceinline__ void operator()(int64_t i0, const uint32_t* v, int cnt) const {
    if (cnt == 4 && v[0] < K && v[1] < K && v[2] < K && v[3] < K) {
      const uint4 a = make_uint4(v[0], v[1], v[2], v[3]);
      __builtin_memcpy(out + i0, &a, 16);
      return;
    }
    slow(i0, v, cnt);
  }
  __device__ __forceinline__ void slow(int64_t i0, const uint32_t* v, int cnt) const {
    int jb = 8;
#pragma unroll
    for (int j = 7; j >= 0; j--)
      if (j < cnt && v[j] >= K) jb = j;
    if (jb < 8 && i0 + jb < *first_bad) *first_bad = i0 + jb;
    if (cnt == 4) {
      uint4 a = make_uint4(v[0], v[1], v[2], v[3]);
      __builtin_memcpy(out + i0, &a, 16);
    } else if (cnt == 8) {
      uint4 a = make_uint4(v[0], v[1], v[2], v[3]);
      uint4 c = make_uint4(v[4], v[5], v[6], v[7]);
      __builtin_memcpy(out + i0, &a, 16);
      __builtin_memcpy(out + i0 + 4, &c, 16);
    } else {
#pragma unroll
      for (int j = 0; j < 8; j++)
        if (j < cnt) out[i0 + j] = int32_t(v[j]);
    }
  }
};

// ------------------------------------------------------------------------------------------------
// Tile bodies.  Every body reads its page/state/chunk records itself (all depend on t.page only).
// ------------------------------------------------------------------------------------------------
// The tile bodies take the page's state (and checkpoints) from their caller: k_expand reads them
// after k_prologue / k_scan, k_flat from the words its prologue jobs published.
// Ckpt loader for a page's stream table at entry i.
struct CkptPlain {
  const Ckpt* ck;
  __device__ __forceinline__ Ckpt operator()(int32_t i) const { return ck[i]; }
};

template <class CkLoad>
__device__ __forceinline__ void tile_levels_s(const DevBatch& b, const Tile& t, const DevPage& P, const PageState& S,
                                              const CkLoad& ckl, TileLds& L, uint32_t* stage) {
  if (page_failed_before_values(S)) return;
  const DevChunk C = b.chunks[P.chunk];
  const uint8_t* img = b.payload + P.image_off;
  const int64_t n = P.num_values;
  const int64_t t0 = int64_t(t.k) * kHybridTile;
  int64_t t1 = t0 + int64_t(t.span) * kHybridTile;
  if (t1 > n) t1 = n;
  if (t0 >= t1) return;
  for (int s = 0; s < 2; s++) {  // repetition levels first, then definition levels
    const int maxl = s == 0 ? C.max_rep : C.max_def;
    if (maxl <= 0) continue;
    LevelSink sink{(s == 0 ? C.rep_levels : C.def_levels) + P.level_base};
    const Ckpt c = ckl((s == 0 ? P.ck_rep : P.ck_def) + t.k);
    expand_hybrid(img, s == 0 ? S.rep_e : S.def_e, bits_len32(uint32_t(maxl)), c, t0, t1, L, stage, sink);
    __syncthreads();
  }
}

__device__ __forceinline__ void tile_levels(const DevBatch& b, const Tile& t, TileLds& L, uint32_t* stage) {
  const DevPage P = b.pages[t.page];
  const PageState S = b.states[t.page];
  tile_levels_s(b, t, P, S, CkptPlain{b.ckpts}, L, stage);
}

template <class CkLoad, bool NT = false>
__device__ __forceinline__ void tile_dict_s(const DevBatch& b, const Tile& t, const DevPage& P, const DevChunk& C,
                                            const PageState& S, uint32_t K, const uint8_t* dict, const CkLoad& ckl,
                                            TileLds& L, uint32_t* stage, uint32_t* bad_flag = nullptr);

// A dictionary page's `bytes` value bytes (any alignment) into LDS (16-aligned): 16-byte loads, four
// per thread in flight, the tail by dwords.  No barrier: the unpack passes one before any gather.
__device__ __forceinline__ void stage_dict(uint8_t* lds_dst, const uint8_t* src_, int64_t bytes) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef u32x4 u32x4_u __attribute__((aligned(1)));
  const PQH_G uint8_t* src = (const PQH_G uint8_t*)(src_);
  const int64_t nv = bytes >> 4;
  for (int64_t base = 0; base < nv; base += 4 * kBlock) {
    u32x4 x[4];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int64_t k = base + threadIdx.x + j * kBlock;
      x[j] = *reinterpret_cast<const PQH_G u32x4_u*>(src + 16 * (k < nv ? k : 0));
    }
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int64_t k = base + threadIdx.x + j * kBlock;
      if (k < nv) *reinterpret_cast<u32x4*>(lds_dst + 16 * k) = x[j];
    }
  }
  for (int64_t o = 16 * nv + 4 * int64_t(threadIdx.x); o < bytes; o += 4 * kBlock) {
    uint32_t x = 0;
    if (o + 4 <= bytes) __builtin_memcpy(&x, src_ + o, 4);
    else for (int k = 0; o + k < bytes; k++) x |= uint32_t(src_[o + k]) << (8 * k);
    *reinterpret_cast<uint32_t*>(lds_dst + o) = x;
  }
}

template <bool LDS>
__device__ __forceinline__ void tile_dict(const DevBatch& b, const Tile& t, TileLds& L, uint32_t* stage,
                                          uint8_t* dict_lds) {
  const DevPage P = b.pages[t.page];
  const PageState S = b.states[t.page];
  if (page_failed_before_values(S)) return;
  const int64_t t0 = int64_t(t.k) * kHybridTile;
  int64_t t1 = t0 + int64_t(t.span) * kHybridTile;
  if (t1 > S.val_limit) t1 = S.val_limit;
  if (t0 >= t1) return;
  const int vs = P.value_size;
  uint32_t K = 0;
  const uint8_t* dict = nullptr;
  if (P.dict_page >= 0) {
    const PageState DS = b.states[P.dict_page];
    if (DS.err == kNoError) {
      K = uint32_t(DS.dict_n);
      dict = b.payload + b.pages[P.dict_page].image_off;
    }
  }
  if constexpr (LDS) {  // stage the dictionary page's values in LDS (kDictLdsMax bytes at most)
    stage_dict(dict_lds, dict, int64_t(K) * vs);
    dict = dict_lds;
    // no barrier here: expand_hybrid passes one (run list or the unpack's first stage) before any
    // value is gathered
  }
  const DevChunk C = b.chunks[P.chunk];
  tile_dict_s(b, t, P, C, S, K, dict, CkptPlain{b.ckpts}, L, stage);
}

// The gather itself: dictionary `dict` (LDS or global) of K entries.
// bad_flag (k_flat): a key out of range sets it (the batch is decoded again by the three kernels)
// instead of lowering the page's error key.
template <class CkLoad, bool NT>
__device__ __forceinline__ void tile_dict_s(const DevBatch& b, const Tile& t, const DevPage& P, const DevChunk& C,
                                            const PageState& S, uint32_t K, const uint8_t* dict, const CkLoad& ckl,
                                            TileLds& L, uint32_t* stage, uint32_t* bad_flag) {
  if (page_failed_before_values(S)) return;
  const int64_t t0 = int64_t(t.k) * kHybridTile;
  int64_t t1 = t0 + int64_t(t.span) * kHybridTile;
  if (t1 > S.val_limit) t1 = S.val_limit;
  if (t0 >= t1) return;
  const int vs = P.value_size;
  const uint8_t* img = b.payload + P.image_off;
  int64_t first_bad = INT64_MAX;
  uint8_t* out = C.values + S.value_base * vs;
  const Ckpt c = ckl(P.ck_val + t.k);
  if (vs == 0) {
    KeySink sink{C.aux + S.value_base, K, &first_bad};
    expand_hybrid(img, S.val_e, S.width, c, t0, t1, L, stage, sink);
  } else if (vs == 4) {
    DictSink<4, NT> sink{dict, out, K, vs, &first_bad};
    expand_hybrid(img, S.val_e, S.width, c, t0, t1, L, stage, sink);
  } else if (vs == 8) {
    DictSink<8> sink{dict, out, K, vs, &first_bad};
    expand_hybrid(img, S.val_e, S.width, c, t0, t1, L, stage, sink);
  } else {
    DictSink<0> sink{dict, out, K, vs, &first_bad, C.dict_nil && C.value_nil ? C.value_nil + S.value_base : nullptr};
    expand_hybrid(img, S.val_e, S.width, c, t0, t1, L, stage, sink);
  }
  if (first_bad != INT64_MAX) {
    if (bad_flag) __hip_atomic_store(bad_flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else atomicMin(&b.states[t.page].err, (unsigned long long)err_key(3, first_bad, PQH_ERR_DICT_INDEX));
  }
}

template <class CkLoad>
__device__ __forceinline__ void tile_rle_bool_s(const DevBatch& b, const Tile& t, const DevPage& P, const PageState& S,
                                                const CkLoad& ckl, TileLds& L, uint32_t* stage) {
  if (page_failed_before_values(S)) return;
  const int64_t t0 = int64_t(t.k) * kHybridTile;
  int64_t t1 = t0 + int64_t(t.span) * kHybridTile;
  if (t1 > S.val_limit) t1 = S.val_limit;
  if (t0 >= t1) return;
  const DevChunk C = b.chunks[P.chunk];
  BoolSink sink{C.values + S.value_base};
  expand_hybrid(b.payload + P.image_off, S.val_e, 1, ckl(P.ck_val + t.k), t0, t1, L, stage, sink);
}

__device__ __forceinline__ void tile_rle_bool(const DevBatch& b, const Tile& t, TileLds& L, uint32_t* stage) {
  const DevPage P = b.pages[t.page];
  const PageState S = b.states[t.page];
  tile_rle_bool_s(b, t, P, S, CkptPlain{b.ckpts}, L, stage);
}

// PLAIN fixed-width values (int32/int64/float/double/INT96/FLBA): little-endian copy of
// notNull * size bytes (type_int32.go:21-31 ...), 16-byte vector loads and stores, 4 in flight.
__device__ __forceinline__ void tile_copy_s(const DevBatch& b, const Tile& t, const DevPage& P, const DevChunk& C,
                                            const PageState& S) {
  if (page_failed_before_values(S)) return;
  const int64_t total = int64_t(S.val_limit) * P.value_size;
  const int64_t c0 = int64_t(t.k) * kCopyTileBytes;
  int64_t c1 = c0 + kCopyTileBytes;
  if (c1 > total) c1 = total;
  if (c0 >= c1) return;
  const PQH_G uint8_t* src = b.payload + P.image_off + S.val_s;
  PQH_G uint8_t* dst = C.values + S.value_base * P.value_size;
  int64_t o = c0 + 16 * int64_t(threadIdx.x);
  // 8 x 16 B in flight per thread (32 KiB per workgroup); streaming (nontemporal) stores
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  typedef u32x4 u32x4_u __attribute__((aligned(1)));
  for (; o + 16 * 7 * kBlock + 16 <= c1; o += 16 * 8 * kBlock) {
    u32x4 x[8];
#pragma unroll
    for (int k = 0; k < 8; k++) x[k] = *reinterpret_cast<const PQH_G u32x4_u*>(src + o + 16 * k * kBlock);
#pragma unroll
    for (int k = 0; k < 8; k++)
      __builtin_nontemporal_store(x[k], reinterpret_cast<PQH_G u32x4_u*>(dst + o + 16 * k * kBlock));
  }
  for (; o + 16 * 3 * kBlock + 16 <= c1; o += 16 * 4 * kBlock) {
    uint4 a, bb, c, d;
    __builtin_memcpy(&a, src + o, 16);
    __builtin_memcpy(&bb, src + o + 16 * kBlock, 16);
    __builtin_memcpy(&c, src + o + 32 * kBlock, 16);
    __builtin_memcpy(&d, src + o + 48 * kBlock, 16);
    __builtin_memcpy(dst + o, &a, 16);
    __builtin_memcpy(dst + o + 16 * kBlock, &bb, 16);
    __builtin_memcpy(dst + o + 32 * kBlock, &c, 16);
    __builtin_memcpy(dst + o + 48 * kBlock, &d, 16);
  }
  for (; o < c1; o += 16 * kBlock) {
    if (o + 16 <= c1) {
      uint4 a;
      __builtin_memcpy(&a, src + o, 16);
      __builtin_memcpy(dst + o, &a, 16);
    } else {
      for (int64_t k = o; k < c1; k++) dst[k] = src[k];
    }
  }
}

// booleanPlainDecoder (type_boolean.go:43-69): LSB-first bits -> 0/1 bytes.
__device__ __forceinline__ uint32_t nibble_bytes(uint32_t n) { return (n * 0x00204081u) & 0x01010101u; }

__device__ __forceinline__ void tile_bool_plain_s(const DevBatch& b, const Tile& t, const DevPage& P,
                                                  const DevChunk& C, const PageState& S) {
  if (page_failed_before_values(S)) return;
  const int64_t lim = S.val_limit;
  for (int q = 0; q < 2; q++) {
    const int64_t v0 = int64_t(t.k) * kBoolTile + int64_t(q) * (kBoolTile / 2) + int64_t(threadIdx.x) * 64;
    if (v0 >= lim) return;
    const PQH_G uint8_t* src = b.payload + P.image_off + S.val_s + (v0 >> 3);
    PQH_G uint8_t* dst = C.values + S.value_base + v0;
    uint8_t in[8];
    __builtin_memcpy(in, src, 8);
    if (v0 + 64 <= lim) {
      for (int k = 0; k < 4; k++) {
        uint4 o;
        o.x = nibble_bytes(in[2 * k] & 15);
        o.y = nibble_bytes(in[2 * k] >> 4);
        o.z = nibble_bytes(in[2 * k + 1] & 15);
        o.w = nibble_bytes(in[2 * k + 1] >> 4);
        __builtin_memcpy(dst + 16 * k, &o, 16);
      }
    } else {
      for (int64_t j = 0; v0 + j < lim; j++) dst[j] = (in[j >> 3] >> (j & 7)) & 1;
    }
  }
}

__device__ __forceinline__ void tile_copy(const DevBatch& b, const Tile& t) {
  const DevPage P = b.pages[t.page];
  const PageState S = b.states[t.page];
  if (page_failed_before_values(S)) return;
  const DevChunk C = b.chunks[P.chunk];
  tile_copy_s(b, t, P, C, S);
}

__device__ __forceinline__ void tile_bool_plain(const DevBatch& b, const Tile& t) {
  const DevPage P = b.pages[t.page];
  const PageState S = b.states[t.page];
  if (page_failed_before_values(S)) return;
  const DevChunk C = b.chunks[P.chunk];
  tile_bool_plain_s(b, t, P, C, S);
}

// ------------------------------------------------------------------------------------------------
// k_expand: ONE launch for every data-parallel tile of the batch (levels, PLAIN copies, booleans,
// dictionary gathers with the dictionary in LDS, RLE booleans).  Tile kinds are interleaved by the
// planner so every CU sees a mix of byte-copy and bit-unpack work.
// ------------------------------------------------------------------------------------------------
#include "delta_impl.h"
#include "bytearray_impl.h"
#include "nest_impl.h"
#include "snappy_impl.h"
#include "snappy_mw.h"
#include "snappy_emit.h"
#include "gzip_impl.h"

__global__ __launch_bounds__(256) void k_expand(DevBatch b, const Tile* tiles) {
  __shared__ TileLds L;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];  // [stage kStageBytes+16][dictionary]
  uint32_t* stage = reinterpret_cast<uint32_t*>(lds);
  uint8_t* dict_lds = lds + kStageBytes + 16;
  const Tile t = tiles[blockIdx.x];
  switch (t.kind) {
    case TK_LEVELS: tile_levels(b, t, L, stage); break;
    case TK_COPY: tile_copy(b, t); break;
    case TK_BOOL: tile_bool_plain(b, t); break;
    case TK_DICT: tile_dict<true>(b, t, L, stage, dict_lds); break;
    case TK_RLE_BOOL: tile_rle_bool(b, t, L, stage); break;
    default: break;
  }
}

// Dictionaries larger than kDictLdsMax: gathered from global memory (L2 / Infinity Cache).
__global__ __launch_bounds__(256) void k_dict_global(DevBatch b, const Tile* tiles) {
  __shared__ TileLds L;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  tile_dict<false>(b, tiles[blockIdx.x], L, reinterpret_cast<uint32_t*>(lds), nullptr);
}

// ------------------------------------------------------------------------------------------------
// k_flat: a small batch of required flat fixed-width columns (dictionary, PLAIN fixed / INT96,
// PLAIN booleans) in ONE launch, with no workgroup waiting for another.  Every tile assumes its page
// is clean and simple -- the header the planner saw, the notNull count = num_values, a dictionary
// stream that is one bit-packed run over all its values, enough bytes, no earlier page failing --
// and decodes from that speculative state (flat_spec: k_prologue's result for such a page, read
// from the page's first bytes) and the host's page value bases (prefix sums of num_values, k_scan's
// result for such a chunk), all carried by its FlatTile record.  Beside the tiles, one wave per page
// (the launch's first workgroups) runs k_prologue's body on the page, stores the state, and checks
// it against the speculation.  Any difference -- or a dictionary key out of range -- sets
// `flag`: pqh_batch_sync decodes the batch again through k_prologue / k_scan / k_expand (which give
// the reference's errors and limits) and keeps the batch off k_flat from then on.
// ------------------------------------------------------------------------------------------------
// k_prologue's state for a clean, simple page (false: the page is not one; nothing is assumed).
__device__ __forceinline__ bool flat_spec(const DevBatch& b, const DevPage& P, int64_t value_base, PageState& S,
                                          Ckpt& ck, int max_def = 0, Ckpt* ckd = nullptr) {
  S.err = kNoError;
  S.nn = 0;
  S.width = 0;
  S.ba_summed = 0;
  S.rep_s = S.rep_e = S.def_s = S.def_e = -1;
  S.dict_n = 0;
  S.value_base = value_base;
  S.byte_base = 0;
  ck = Ckpt{0, 0x7fffffff, 0, 0};
  if (P.host_err != kNoError) return false;
  const int64_t L = P.image_len, n = P.num_values;
  if (P.page_type == PQH_DICTIONARY_PAGE) {  // dictPageReader: num_values PLAIN entries
    if (P.value_size <= 0 || int64_t(P.value_size) * n > L) return false;
    S.rep_s = S.rep_e = S.def_s = S.def_e = -1;
    S.dict_n = int32_t(n);
    S.val_s = S.val_e = 0;
    S.val_limit = 0;
    return true;
  }
  const int64_t vs = P.page_type == PQH_DATA_PAGE ? 0 : int64_t(P.rep_len) + P.def_len;  // (no level streams)
  S.val_s = int32_t(vs);
  S.val_e = int32_t(L);
  S.val_limit = 0;
  int64_t nn = n;  // notNull
  if (max_def > 0) {
    // nullable flat (V2): the definition levels raw at [rep_len, rep_len + def_len), ONE bit-packed
    // run of width 1 over the n slots; notNull = num_values - num_nulls from the header (the page
    // check counts the levels)
    if (P.page_type != PQH_DATA_PAGE_V2 || max_def != 1 || P.def_len <= 0 || P.num_nulls < 0 || P.num_nulls > n)
      return false;
    S.def_s = P.rep_len;
    S.def_e = P.rep_len + P.def_len;
    nn = n - P.num_nulls;
    if (n > 0) {
      const uint8_t* img = b.payload + P.image_off;
      const uint64_t q = ld64_masked(img + S.def_s, img + S.def_e);
      uint64_t h = 0;
      int len = 0;
      for (int k = 0; k < 5; k++) {
        const uint32_t c = uint32_t(q >> (8 * k)) & 0xff;
        h |= uint64_t(c & 0x7f) << (7 * k);
        if (c < 0x80) {
          len = k + 1;
          break;
        }
      }
      if (len == 0 || S.def_s + len > S.def_e || h > 0x7fffffffull || !(h & 1)) return false;
      const int64_t groups = int64_t(h >> 1), data = S.def_s + len;
      if (groups * 8 < n || data + (n + 7) / 8 > S.def_e) return false;
      const int64_t next = data + groups, cnt = groups * 8;
      if (ckd)
        *ckd = Ckpt{0, int32_t(cnt < 0x7fffffff ? cnt : 0x7fffffff), int32_t(data),
                    int32_t(next < 0x7fffffff ? next : 0x7fffffff) | int32_t(0x80000000u)};
    }
  }
  if (P.kind == K_DICT) {
    if (vs >= L) return false;
    const uint8_t* img = b.payload + P.image_off;
    const uint64_t q0 = ld64_masked(img + vs, img + L);  // the width and up to 5 header bytes
    const int w = int(q0 & 0xff);
    if (w > 32) return false;
    S.width = int16_t(w);
    S.val_s = int32_t(vs + 1);
    if (nn <= 0) return true;
    S.nn = int32_t(nn);
    S.val_limit = int32_t(nn);
    if (w == 0) return true;  // no reads: ck = {0, 2^31-1, 0, 0}, as walk_hybrid's
    // the first run header (at most 5 bytes for a count < 2^31), then one bit-packed run over all n
    uint64_t h = 0;
    int len = 0;
    for (int k = 0; k < 5; k++) {
      const uint32_t c = uint32_t(q0 >> (8 * (k + 1))) & 0xff;
      h |= uint64_t(c & 0x7f) << (7 * k);
      if (c < 0x80) {
        len = k + 1;
        break;
      }
    }
    if (len == 0 || vs + 1 + len > L || h > 0x7fffffffull || !(h & 1)) return false;
    const int64_t groups = int64_t(h >> 1), data = vs + 1 + len;
    if (groups * 8 < nn) return false;
    const int64_t gf = (L - data + w - 1) / w;  // groups readable before EOF
    if (data >= L || gf < (nn + 7) / 8) return false;
    const int64_t next = data + groups * w, cnt = groups * 8;
    ck = Ckpt{0, int32_t(cnt < 0x7fffffff ? cnt : 0x7fffffff), int32_t(data),
              int32_t(next < 0x7fffffff ? next : 0x7fffffff) | int32_t(0x80000000u)};
    return true;
  }
  if (nn <= 0) return P.kind == K_PLAIN_FIXED || P.kind == K_PLAIN_INT96 || P.kind == K_PLAIN_BOOL;
  const int64_t avail = L - vs;
  if (P.kind == K_PLAIN_FIXED || P.kind == K_PLAIN_INT96) {
    if (P.value_size <= 0 || avail / P.value_size < nn) return false;
  } else if (P.kind == K_PLAIN_BOOL) {
    if (avail * 8 < nn) return false;
  } else {
    return false;
  }
  S.nn = int32_t(nn);
  S.val_limit = int32_t(nn);
  return true;
}

struct CkptConst {
  Ckpt c;
  __device__ __forceinline__ Ckpt operator()(int32_t) const { return c; }
};

// One wave: k_prologue's body on page p, its state stored with the page's value base, and the
// speculation checked (flag on any difference).
__device__ __forceinline__ void flat_check(const DevBatch& b, int32_t p, const int64_t* spec_base, uint32_t* flag) {
  const int lane = threadIdx.x & 63;
  const DevPage P = b.pages[p];
  const int64_t vb = spec_base[p];
  PageState spec;
  Ckpt ck;
  const bool ok = flat_spec(b, P, vb, spec, ck, b.chunks[P.chunk].max_def);
  PageState S = prologue_page<1, false>(b, p, lane, 0, nullptr, false);
  S.value_base = vb;
  if (lane == 0) {
    b.states[p] = S;
    const bool same = ok && S.err == spec.err && S.nn == spec.nn && S.width == spec.width && S.rep_s == spec.rep_s &&
                      S.rep_e == spec.rep_e && S.def_s == spec.def_s && S.def_e == spec.def_e &&
                      S.val_s == spec.val_s && S.val_e == spec.val_e && S.val_limit == spec.val_limit &&
                      S.dict_n == spec.dict_n;
    if (!same) __hip_atomic_store(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// blocks [0, njob): the page checks, four pages each (one wave per page); [njob, njob + ntiles):
// k_expand's tiles, from their FlatTile records
__global__ __launch_bounds__(256) void k_flat(DevBatch b, const FlatTile* tiles, int32_t ntiles, int32_t njob,
                                              const int64_t* spec_base, uint32_t* flag) {
  __shared__ TileLds L;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];  // as k_expand
  uint32_t* stage = reinterpret_cast<uint32_t*>(lds);
  uint8_t* dict_lds = lds + kStageBytes + 16;
  if (int32_t(blockIdx.x) < njob) {
    const int p = __builtin_amdgcn_readfirstlane(int(blockIdx.x) * 4 + int(threadIdx.x >> 6));
    if (p < b.num_pages) flat_check(b, p, spec_base, flag);
    return;
  }
  const FlatTile f = tiles[blockIdx.x - njob];
  DevPage P;  // the fields the tile bodies and flat_spec read
  __builtin_memset(&P, 0, sizeof(P));
  P.image_off = f.image_off;
  P.image_len = f.image_len;
  P.page_type = f.page_type;
  P.num_values = f.num_values;
  P.kind = f.kind;
  P.value_size = f.value_size;
  P.rep_len = f.rep_len;
  P.def_len = f.def_len;
  P.host_err = f.host_err;
  P.num_nulls = f.num_nulls;
  DevChunk C;
  __builtin_memset(&C, 0, sizeof(C));
  C.values = f.values;
  const Tile t{0, f.k, f.tkind, f.span};
  uint32_t K = 0;  // the dictionary as its header declares it
  if (f.tkind == TK_DICT && f.dict_off >= 0) {
    const int64_t bytes = int64_t(f.dict_n) * f.value_size;
    if (bytes <= int64_t(f.dict_len)) {
      K = uint32_t(f.dict_n);
      const uint8_t* dict = b.payload + f.dict_off;
      stage_dict(dict_lds, dict, bytes);
    }
  }
  PageState S;
  Ckpt ck, ckd;
  const bool spec_ok = flat_spec(b, P, f.value_base, S, ck, f.max_def, &ckd);
  if (spec_ok) {  // (otherwise the page's check flags it)
    switch (f.tkind) {
      case TK_LEVELS: {  // nullable flat: the definition levels (one bit-packed run of width 1)
        const int64_t t0 = int64_t(t.k) * kHybridTile;
        int64_t t1 = t0 + int64_t(t.span) * kHybridTile;
        if (t1 > P.num_values) t1 = P.num_values;
        LevelSink sink{f.def_out};
        if (f.def_out && t0 < t1) expand_hybrid(b.payload + P.image_off, S.def_e, 1, ckd, t0, t1, L, stage, sink);
        break;
      }
      case TK_COPY: tile_copy_s(b, t, P, C, S); break;
      case TK_BOOL: tile_bool_plain_s(b, t, P, C, S); break;
      case TK_DICT: tile_dict_s<CkptConst, true>(b, t, P, C, S, K, dict_lds, CkptConst{ck}, L, stage, flag); break;
      default: break;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// The hybrid decoder alone (pqh_hybrid_decode, the reference's levelDecoder.next over a whole
// stream, hybrid_decoder.go:81-165): one wave walks the run headers into tile checkpoints (the
// prologue's walk), then one workgroup per kHybridTile tile unpacks its values through the same
// expand_hybrid / bp_staged paths as k_expand, into uint32 values.
// ------------------------------------------------------------------------------------------------
template <int G>
struct RawSink {
  static constexpr int kGroup = G;
  uint32_t* out;
  __device__ __forceinline__ void operator()(int64_t i0, const uint32_t* v, int cnt) const {
#pragma unroll
    for (int j = 0; j < 8; j++)
      if (j < cnt) out[i0 + j] = v[j];
  }
};

__global__ __launch_bounds__(64) void k_hybrid_walk(const uint8_t* s, int64_t len, int w, int64_t n, Ckpt* ck,
                                                    uint64_t* res) {
  const WalkOut o = walk_hybrid(s, 0, len, w, n, 3, ck, -1, int(threadIdx.x));
  if (threadIdx.x == 0) {
    res[0] = o.err;
    res[1] = uint64_t(o.fail_index);
  }
}

template <int G>
__global__ __launch_bounds__(256) void k_hybrid_raw(const uint8_t* s, int64_t len, int w, const Ckpt* ck,
                                                    const uint64_t* res, uint32_t* out) {
  __shared__ TileLds L;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int64_t t0 = int64_t(blockIdx.x) * kHybridTile;
  const int64_t lim = int64_t(res[1]);  // values before the first error
  const int64_t t1 = t0 + kHybridTile < lim ? t0 + kHybridTile : lim;
  if (t0 >= t1) return;
  RawSink<G> sink{out};
  expand_hybrid(s, len, w, ck[blockIdx.x], t0, t1, L, reinterpret_cast<uint32_t*>(lds), sink);
}

// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
hipError_t launch_hybrid_raw(const uint8_t* stream, int64_t len, int32_t width, int64_t n, int group, Ckpt* ck,
                             uint64_t* res, uint32_t* out, hipStream_t s) {
  hipLaunchKernelGGL(k_hybrid_walk, dim3(1), dim3(64), 0, s, stream, len, width, n, ck, res);
  const int64_t tiles = (n + kHybridTile - 1) / kHybridTile;
  if (tiles > 0) {
    if (group == 4)
      hipLaunchKernelGGL(k_hybrid_raw<4>, dim3(unsigned(tiles)), dim3(256), size_t(kStageBytes + 16), s, stream, len,
                         width, ck, res, out);
    else
      hipLaunchKernelGGL(k_hybrid_raw<8>, dim3(unsigned(tiles)), dim3(256), size_t(kStageBytes + 16), s, stream, len,
                         width, ck, res, out);
  }
  return hipGetLastError();
}

hipError_t launch_prologue(const DevBatch& b, bool wide, hipStream_t s) {
  if (b.num_pages <= 0) return hipSuccess;
  if (wide) hipLaunchKernelGGL(k_prologue<4>, dim3(b.num_pages), dim3(256), 0, s, b);
  else hipLaunchKernelGGL(k_prologue<1>, dim3((b.num_pages + 3) / 4), dim3(256), 0, s, b);
  return hipGetLastError();
}

hipError_t launch_scan(const DevBatch& b, hipStream_t s) {
  if (b.num_chunks <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_scan, dim3(b.num_chunks), dim3(256), 0, s, b);
  return hipGetLastError();
}

hipError_t launch_expand(const DevBatch& b, const Tile* tiles, int32_t n, size_t lds_bytes, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_expand, dim3(n), dim3(256), size_t(kStageBytes + 16) + lds_bytes, s, b, tiles);
  return hipGetLastError();
}

hipError_t launch_flat(const DevBatch& b, const FlatTile* tiles, int32_t ntiles, const int64_t* spec_base,
                       uint32_t* flag, size_t lds_bytes, hipStream_t s) {
  const int32_t njob = (b.num_pages + 3) / 4;
  if (ntiles + njob <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_flat, dim3(njob + ntiles), dim3(256), size_t(kStageBytes + 16) + lds_bytes, s, b, tiles, ntiles,
                     njob, spec_base, flag);
  return hipGetLastError();
}

hipError_t launch_snappy(const pqh_codec_page* pages, int32_t n, const uint8_t* src, uint8_t* dst, int32_t* status,
                         hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_snappy, dim3(n), dim3(256), 0, s, pages, src, dst, status, nullptr);
  return hipGetLastError();
}

std::vector<int32_t> snap_plan_tables(const pqh_codec_page* pages, int32_t n, int32_t* n_win, int32_t* n_unit,
                                      int32_t* n_page_mode) {
  std::vector<int32_t> pw(size_t(n) + 1), pu(size_t(n) + 1), pm(size_t(n), 0), wp, up;
  int32_t W = 0, U = 0, M = 0;
  for (int32_t i = 0; i < n; i++) {
    const pqh_codec_page& c = pages[i];
    pw[size_t(i)] = W;
    pu[size_t(i)] = U;
    int64_t nw = 0, nu = 0;
    if (c.codec == PQH_CODEC_SNAPPY) {
      const int64_t raw = c.raw_len < c.src_len ? c.raw_len : c.src_len;
      const int64_t body = int64_t(c.src_len) - raw, out = int64_t(c.image_len) - raw;
      // compresses by 1.25x or less: long literals, k_snappy's bulk copies.  Also every block of
      // more than 2^24 output bytes: k_snap_emit packs a copy's offset in 24 bits (an offset is at
      // most the output position, so only such blocks can hold a copy4 reaching 2^24 or further;
      // golang/snappy accepts offsets up to 2^32, decode_other.go:75-85), k_snappy keeps 31 bits.
      // (Pages that barely compress because they are short literals and copies of random text --
      // C5 -- also stay here: r04 measured the pipeline at 57 vs 32 ms on C5, its speculative
      // window entries almost never resynchronise inside such literals, so k_snap_stitch re-walks
      // the windows one by one.)
      const bool page_mode = 5 * body >= 4 * out || out > (int64_t(1) << 24);
      if (page_mode) {
        pm[size_t(i)] = 1;
        M++;
      } else {
        nw = (body + kSnWin - 1) / kSnWin;
        if (raw <= c.image_len) nu = (out + kSnUnit - 1) / kSnUnit;
      }
    } else if (c.codec != PQH_CODEC_GZIP) {
      nu = ((c.src_len < c.image_len ? c.src_len : c.image_len) + int64_t(kSnUnit) - 1) / kSnUnit;
    }
    for (int64_t j = 0; j < nw; j++) wp.push_back(i);
    for (int64_t j = 0; j < nu; j++) up.push_back(i);
    W += int32_t(nw);
    U += int32_t(nu);
  }
  pw[size_t(n)] = W;
  pu[size_t(n)] = U;
  std::vector<int32_t> t;
  t.reserve(pw.size() + pu.size() + pm.size() + wp.size() + up.size());
  t.insert(t.end(), pw.begin(), pw.end());
  t.insert(t.end(), pu.begin(), pu.end());
  t.insert(t.end(), pm.begin(), pm.end());
  t.insert(t.end(), wp.begin(), wp.end());
  t.insert(t.end(), up.begin(), up.end());
  *n_win = W;
  *n_unit = U;
  *n_page_mode = M;
  return t;
}

void snap_plan_bind(SnapPlan& P, int32_t* tables, int4* wspec, int2* wtrue, int32_t* uflag, int16_t* wseg) {
  P.wseg = wseg;
  P.page_win0 = tables;
  P.page_unit0 = tables + P.n_pages + 1;
  P.page_mode = tables + 2 * (P.n_pages + 1);
  P.win_page = P.page_mode + P.n_pages;
  P.unit_page = P.win_page + P.n_win;
  P.wspec = wspec;
  P.wtrue = wtrue;
  P.uflag = uflag;
}

hipError_t launch_snappy_mw(const pqh_codec_page* pages, const SnapPlan& P, const uint8_t* src, uint8_t* dst,
                            int32_t* status, hipStream_t s, int part) {
  if (P.n_pages <= 0) return hipSuccess;
  const auto on = [&](int k) { return part < 0 || part == k; };
  if (on(0) && P.n_page_mode > 0)  // barely compressible long-literal pages: one workgroup each (bulk copies)
    hipLaunchKernelGGL(k_snappy, dim3(P.n_pages), dim3(256), 0, s, pages, src, dst, status, P.page_mode);
  if (on(1) && P.n_win > 0)
    hipLaunchKernelGGL(k_snap_spec, dim3(P.n_win), dim3(256), 0, s, pages, P.win_page, P.page_win0, src, P.wspec, P.wseg);
  if (on(2))
    hipLaunchKernelGGL(k_snap_stitch, dim3(P.n_pages), dim3(256), 0, s, pages, P.page_win0, P.page_mode, src, dst,
                       P.wspec, P.wtrue, P.wseg, status);
  if (on(3) && P.n_unit > 0)
    hipLaunchKernelGGL(k_snap_emit, dim3(P.n_unit), dim3(kSnT), 0, s, pages, P.unit_page, P.page_unit0, P.page_win0, src,
                       dst, P.wtrue, P.wseg, status, P.uflag);
  if (on(4) && P.n_unit > 0)
    hipLaunchKernelGGL(k_snap_fixup, dim3(P.n_pages), dim3(kSnT), 0, s, pages, P.page_unit0, P.page_win0, src, dst,
                       P.wtrue, P.wseg, status, P.uflag);
  return hipGetLastError();
}

hipError_t launch_gzip(const pqh_codec_page* pages, int32_t n, const uint8_t* src, uint8_t* dst, int32_t* status,
                       hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_gzip, dim3(n), dim3(256), 0, s, pages, src, dst, status);
  return hipGetLastError();
}

hipError_t launch_delta_page(const DevBatch& b, const Tile* streams, int32_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_delta_page, dim3(n), dim3(256), 0, s, b, streams);
  return hipGetLastError();
}

hipError_t launch_delta_init(const DevBatch& b, const int32_t* delta_pages, int32_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_delta_init, dim3((n + 3) / 4), dim3(256), 0, s, b, delta_pages, n);
  return hipGetLastError();
}

// streams [0, n - n_lens): DELTA_BINARY_PACKED / DELTA_BYTE_ARRAY prefixes; [n - n_lens, n):
// DELTA_LENGTH_BYTE_ARRAY lengths (with their tile byte sums)
hipError_t launch_delta_fused(const DevBatch& b, const Tile* streams, int32_t n, int32_t n_lens, hipStream_t s) {
  if (n - n_lens > 0) hipLaunchKernelGGL(k_delta_fused, dim3(n - n_lens), dim3(256), 0, s, b, streams);
  if (n_lens > 0) hipLaunchKernelGGL(k_delta_fused_lens, dim3(n_lens), dim3(256), 0, s, b, streams + (n - n_lens));
#ifdef PQH_FUSED_PROF
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cs) == hipSuccess && cs == hipStreamCaptureStatusNone &&
      hipStreamSynchronize(s) == hipSuccess) {
    unsigned long long h[2][8], z[2][8] = {};
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_fprof), sizeof(h)) == hipSuccess) {
      for (int v = 0; v < 2; v++) {
        if (!h[v][6]) continue;
        const double wg = double(h[v][6]), tl = double(h[v][5] ? h[v][5] : 1);
        fprintf(stderr, "[fused_prof %s] wgs %.0f tiles/wg %.2f | per wg us: body %.2f init %.2f | per tile us: "
                "stage %.2f chase %.2f tables %.2f expand %.2f\n", v ? "lens" : "values", wg, tl / wg,
                h[v][7] / wg / 100.0, h[v][0] / wg / 100.0, h[v][1] / tl / 100.0, h[v][2] / tl / 100.0,
                h[v][3] / tl / 100.0, h[v][4] / tl / 100.0);
      }
      hipMemcpyToSymbol(HIP_SYMBOL(g_fprof), z, sizeof(z));
    }
  }
#endif
  return hipGetLastError();
}

hipError_t launch_delta_split(const DevBatch& b, const int2* wins, const int32_t* order, int32_t n, int32_t n_lens,
                              hipStream_t s) {
  const char* tk = getenv("PQH_SPLIT_TICKET");  // (A/B: "0" = dispatch order instead of tickets)
  const int32_t ticket = !(tk && tk[0] == '0');
  if (n - n_lens > 0)
    hipLaunchKernelGGL(k_delta_split, dim3(n - n_lens), dim3(256), 0, s, b, wins, order, n - n_lens, ticket);
  if (n_lens > 0)
    hipLaunchKernelGGL(k_delta_split_lens, dim3(n_lens), dim3(256), 0, s, b, wins, order + (n - n_lens), n_lens, ticket);
  return hipGetLastError();
}

hipError_t launch_delta_spec(const DevBatch& b, const int32_t* delta_pages, int32_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_delta_spec, dim3((n + 3) / 4), dim3(256), 0, s, b, delta_pages, n);
  return hipGetLastError();
}

hipError_t launch_delta_walk(const DevBatch& b, const int32_t* delta_pages, int32_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_delta_walk, dim3((n + 3) / 4), dim3(256), 0, s, b, delta_pages, n);
  return hipGetLastError();
}

hipError_t launch_delta_sum(const DevBatch& b, const Tile* tiles, int32_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_delta_sum, dim3(n), dim3(256), 0, s, b, tiles);
  return hipGetLastError();
}

hipError_t launch_delta_scan(const DevBatch& b, const int32_t* delta_pages, int32_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_delta_scan, dim3((n + 255) / 256), dim3(256), 0, s, b, delta_pages, n);
  return hipGetLastError();
}

hipError_t launch_delta_expand(const DevBatch& b, const Tile* tiles, int32_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_delta_expand, dim3(n), dim3(256), 0, s, b, tiles);
  return hipGetLastError();
}

hipError_t launch_delta_serial(const DevBatch& b, const int32_t* delta_pages, int32_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_delta_serial, dim3(n), dim3(64), 0, s, b, delta_pages);
  return hipGetLastError();
}

hipError_t launch_ba_wspec(const DevBatch& b, const int2* wins, int32_t n, BaWin* res, uint16_t* wrec,
                           hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_ba_wspec, dim3(n), dim3(256), 0, s, b, wins, res, wrec);
  return hipGetLastError();
}

hipError_t launch_ba_wstitch(const DevBatch& b, const int32_t* ba_pages, const int2* pwin, int32_t n, BaWin* res,
                             uint16_t* wrec, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_ba_wstitch, dim3(n), dim3(256), 0, s, b, ba_pages, pwin, res, wrec);
  return hipGetLastError();
}

hipError_t launch_ba_wemit(const DevBatch& b, const int2* list, int32_t n, const BaWin* res, const uint16_t* wrec,
                           hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_ba_wemit, dim3(n), dim3(256), 0, s, b, list, res, wrec);
  return hipGetLastError();
}

static_assert(sizeof(WGeo) <= kWGeoBytes, "window geometry record");

hipError_t launch_ba_wcopy(const DevBatch& b, const int2* list, int32_t n, const BaWin* res, const uint16_t* wrec,
                           void* geo, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  WGeo* g = static_cast<WGeo*>(geo);
  hipLaunchKernelGGL(k_ba_wgeo, dim3((n + kBlock - 1) / kBlock), dim3(256), 0, s, b, list, n, res, wrec, g);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_ba_wcopy, dim3(n < kWGrid ? n : kWGrid), dim3(256), 0, s, b, g, n, wrec);
  return hipGetLastError();
}

hipError_t launch_ba_chain(const DevBatch& b, const int2* wins, const int32_t* order, int32_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  // windows taken in dispatch order (blockIdx.x) rather than by an atomic ticket: C4 k_ba_chain
  // 0.499 -> 0.481 ms, same box (PQH_CHAIN_TICKET=1 restores the tickets).  Forward progress rests on
  // the dispatcher's increasing workgroup order; should a look-back ever outwait its spin cap, the
  // batch falls back to the scratch path (bafuse[1]), never a wrong result
  const char* tk = getenv("PQH_CHAIN_TICKET");
  hipLaunchKernelGGL(k_ba_chain, dim3(n), dim3(256), 0, s, b, wins, order, n, int32_t(tk && tk[0] == '1'));
  return hipGetLastError();
}

hipError_t launch_ba_sum(const DevBatch& b, const Tile* tiles, const int32_t* list, int32_t n, bool dlba_pages,
                         hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_ba_sum, dim3(n), dim3(256), 0, s, b, tiles, list, int(dlba_pages));
  return hipGetLastError();
}

hipError_t launch_ba_scan(const DevBatch& b, const int32_t* ba_chunks, int32_t n, const Tile* tiles, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_ba_scan, dim3(n), dim3(256), 0, s, b, ba_chunks, tiles);
  return hipGetLastError();
}

hipError_t launch_ba_expand(const DevBatch& b, const Tile* tiles, const int32_t* list, int32_t n_copy, int32_t n_gather,
                            hipStream_t s) {
  if (n_copy > 0) hipLaunchKernelGGL(k_ba_expand, dim3(n_copy), dim3(256), 0, s, b, tiles, list);
  if (n_gather > 0) hipLaunchKernelGGL(k_ba_gather, dim3(n_gather), dim3(256), 0, s, b, tiles, list + n_copy);
  return hipGetLastError();
}

hipError_t launch_nest_count(const DevBatch& b, const Tile* tiles, int32_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_nest_count, dim3(n), dim3(256), 0, s, b, tiles);
  return hipGetLastError();
}

hipError_t launch_nest_scan(const DevBatch& b, int32_t num_nests, hipStream_t s) {
  if (num_nests <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_nest_scan, dim3(num_nests), dim3(256), 0, s, b);
  return hipGetLastError();
}

hipError_t launch_nest_write(const DevBatch& b, const Tile* tiles, int32_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_nest_write, dim3(n), dim3(256), 0, s, b, tiles);
  return hipGetLastError();
}

hipError_t launch_dba_prefix(const DevBatch& b, const Tile* tiles, int32_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_dba_expand, dim3(n), dim3(256), 0, s, b, tiles);
  hipLaunchKernelGGL(k_dba_prefix, dim3(n), dim3(256), 0, s, b, tiles);
  return hipGetLastError();
}

hipError_t launch_dict_global(const DevBatch& b, const Tile* tiles, int32_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_dict_global, dim3(n), dim3(256), size_t(kStageBytes + 16), s, b, tiles);
  return hipGetLastError();
}

}  // namespace pqhip
