// pqgen.cpp — reference-writer-shaped Parquet generator (tooling).  See pqgen.h.
#include "pqgen.h"

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "../host/codec.h"
#include "../host/thrift_compact.h"

using namespace pqhip;

namespace {

enum { BOOLEAN = 0, INT32 = 1, INT64 = 2, INT96 = 3, FLOAT = 4, DOUBLE = 5, BYTE_ARRAY = 6, FLBA = 7 };
enum { E_PLAIN = 0, E_RLE = 3, E_DELTA_BP = 5, E_DLBA = 6, E_DBA = 7, E_RLE_DICT = 8 };

int bits_len(uint64_t v) { return v ? 64 - __builtin_clzll(v) : 0; }

void put_uvarint(std::vector<uint8_t>& o, uint64_t v) {
  while (v >= 0x80) {
    o.push_back(uint8_t(v | 0x80));
    v >>= 7;
  }
  o.push_back(uint8_t(v));
}
void put_varint(std::vector<uint8_t>& o, int64_t v) { put_uvarint(o, (uint64_t(v) << 1) ^ uint64_t(v >> 63)); }
void put_u32(std::vector<uint8_t>& o, uint32_t v) {
  for (int i = 0; i < 4; i++) o.push_back(uint8_t(v >> (8 * i)));
}

// LSB-first packing of 8 values of width w <= 64 (pack8int32_w / pack8int64_w): exactly w bytes.
void pack8(int w, const uint64_t* v, uint8_t* out) {
  memset(out, 0, size_t(w));
  if (w == 0) return;
  const uint64_t mask = w == 64 ? ~0ull : ((1ull << w) - 1);
  unsigned __int128 acc = 0;
  int nb = 0;
  uint8_t* p = out;
  for (int j = 0; j < 8; j++) {
    acc |= static_cast<unsigned __int128>(v[j] & mask) << nb;
    nb += w;
    while (nb >= 8) {
      *p++ = uint8_t(acc);
      acc >>= 8;
      nb -= 8;
    }
  }
}

// Fast packing of n values (n multiple of 8 after padding) of width w <= 32 into out.
void pack_run(int w, const uint32_t* v, int64_t n, uint8_t* out) {
  int64_t groups = (n + 7) / 8;
  memset(out, 0, size_t(groups * w));
  if (w == 0) return;
  uint64_t acc = 0;
  int nb = 0;
  uint8_t* p = out;
  const uint64_t mask = w == 64 ? ~0ull : ((1ull << w) - 1);
  for (int64_t i = 0; i < groups * 8; i++) {
    uint64_t x = i < n ? (v[i] & mask) : 0;
    acc |= x << nb;
    nb += w;
    while (nb >= 8) {
      *p++ = uint8_t(acc);
      acc >>= 8;
      nb -= 8;
    }
  }
}

// hybridEncoder (hybrid_encoder.go): one bit-packed run, padded to a multiple of 8; with n == 0
// the header declares 0 groups but packedArray.flush still appends one zero group.
void hybrid_encode(int w, const uint32_t* v, int64_t n, std::vector<uint8_t>& o) {
  if (w == 0) return;
  int64_t groups = (n + 7) / 8;
  put_uvarint(o, uint64_t(groups << 1) | 1);
  int64_t data_groups = n == 0 ? 1 : groups;
  size_t at = o.size();
  o.resize(at + size_t(data_groups * w));
  pack_run(w, v, n, o.data() + at);
}

// encodeLevelsV1 / booleanRLEEncoder: u32 byte length, then the hybrid stream.
void hybrid_encode_sized(int w, const uint32_t* v, int64_t n, std::vector<uint8_t>& o) {
  if (w == 0) return;
  std::vector<uint8_t> tmp;
  hybrid_encode(w, v, n, tmp);
  put_u32(o, uint32_t(tmp.size()));
  o.insert(o.end(), tmp.begin(), tmp.end());
}

// deltaBitPackEncoder32/64 with blockSize 128, 4 miniblocks (deltabp_encoder.go).
template <typename T, typename U>
void delta_encode(const T* v, int64_t n, std::vector<uint8_t>& o) {
  const int bs = 128, mbc = 4, mbvc = 32;
  std::vector<uint8_t> body;
  auto flush = [&](std::vector<T>& d, T min_delta) {
    for (auto& x : d) x = T(U(x) - U(min_delta));
    put_varint(body, int64_t(min_delta));
    uint8_t widths[4] = {0, 0, 0, 0};
    std::vector<uint8_t> packed;
    int mb = 0;
    for (size_t i = 0; i < d.size(); i += mbvc, mb++) {
      size_t end = std::min(d.size(), i + mbvc);
      U mx = U(d[i]);
      for (size_t j = i; j < end; j++) mx = std::max(mx, U(d[j]));
      int w = bits_len(uint64_t(mx));
      widths[mb] = uint8_t(w);
      uint64_t grp[8];
      uint8_t buf[64];
      for (int g = 0; g < mbvc / 8; g++) {
        for (int k = 0; k < 8; k++) {
          size_t j = i + size_t(g * 8 + k);
          grp[k] = j < end ? uint64_t(U(d[j])) : 0;
        }
        pack8(w, grp, buf);
        packed.insert(packed.end(), buf, buf + w);
      }
    }
    body.insert(body.end(), widths, widths + mbc);
    body.insert(body.end(), packed.begin(), packed.end());
    d.clear();
  };
  std::vector<T> deltas;
  deltas.reserve(bs);
  T min_delta = T(2147483647);  // math.MaxInt32 for both widths (deltabp_encoder.go:209, :271)
  for (int64_t i = 1; i < n; i++) {
    T delta = T(U(v[i]) - U(v[i - 1]));
    deltas.push_back(delta);
    if (delta < min_delta) min_delta = delta;
    if (int(deltas.size()) == bs) {
      flush(deltas, min_delta);
      min_delta = T(2147483647);
    }
  }
  if (n == 1 || !deltas.empty()) flush(deltas, min_delta);
  put_uvarint(o, bs);
  put_uvarint(o, mbc);
  put_uvarint(o, uint64_t(n));
  put_varint(o, n > 0 ? int64_t(v[0]) : 0);
  o.insert(o.end(), body.begin(), body.end());
}

struct Leaf {
  int type = 0, type_length = 0, max_def = 0, max_rep = 0, converted = -1;
  std::vector<std::string> path;
  int value_size() const {
    switch (type) {
      case BOOLEAN: return 1;
      case INT32: case FLOAT: return 4;
      case INT64: case DOUBLE: return 8;
      case INT96: return 12;
      case FLBA: return type_length;
      default: return 0;
    }
  }
};

struct ChunkOut {
  std::vector<uint8_t> bytes;
  bool has_dict = false;
  int64_t data_page_rel = 0;
  int64_t total_uncompressed = 0;
  int64_t num_slots = 0;
  int enc = 0;
  std::string err;
};

struct Ctx {
  const pqg_options* opt;
  int64_t max_page;
};

std::string_view value_at(const Leaf& L, const pqg_column_data& c, int64_t i) {
  if (L.type == BYTE_ARRAY) {
    return std::string_view(reinterpret_cast<const char*>(c.values) + c.offsets[i], size_t(c.offsets[i + 1] - c.offsets[i]));
  }
  int s = L.value_size();
  return std::string_view(reinterpret_cast<const char*>(c.values) + i * s, size_t(s));
}

void plain_value(const Leaf& L, std::string_view v, std::vector<uint8_t>& o) {
  if (L.type == BYTE_ARRAY) put_u32(o, uint32_t(v.size()));
  o.insert(o.end(), v.begin(), v.end());
}

void write_page_header(std::vector<uint8_t>& o, int type, int32_t usize, int32_t csize, bool crc, uint32_t crcv,
                       int32_t num_values, int enc, int32_t nulls, int32_t rows, int32_t dlen, int32_t rlen,
                       bool compressed) {
  TWriter w(o);
  w.i32(1, type);
  w.i32(2, usize);
  w.i32(3, csize);
  if (crc) w.i32(4, int32_t(crcv));
  if (type == 0) {
    w.begin_struct(5);
    w.i32(1, num_values);
    w.i32(2, enc);
    w.i32(3, E_RLE);
    w.i32(4, E_RLE);
    w.end_struct();
  } else if (type == 2) {
    w.begin_struct(7);
    w.i32(1, num_values);
    w.i32(2, E_PLAIN);
    w.end_struct();
  } else {
    w.begin_struct(8);
    w.i32(1, num_values);
    w.i32(2, nulls);
    w.i32(3, rows);
    w.i32(4, enc);
    w.i32(5, dlen);
    w.i32(6, rlen);
    w.boolean(7, compressed);
    w.end_struct();
  }
  w.stop();
}

// One column chunk: writeChunk (chunk_writer.go:154-332) with the page cut of flushPage.
void encode_chunk(const Ctx& ctx, const Leaf& L, const pqg_column_data& c, int64_t s0, int64_t s1, int64_t v0,
                  int64_t v1, ChunkOut& out) {
  const pqg_options& opt = *ctx.opt;
  const int codec = opt.codec;
  const bool v2 = opt.data_page_v2 != 0;
  const int rw = bits_len(uint64_t(L.max_rep)), dw = bits_len(uint64_t(L.max_def));
  const int vsize = L.value_size();
  out.num_slots = s1 - s0;

  // --- dictionary decision: <= MaxInt16 distinct values over the chunk, never for booleans ---
  bool use_dict = c.use_dict && L.type != BOOLEAN;
  std::vector<int32_t> idx;  // per value of the chunk
  std::vector<std::string_view> dict;
  // dict_page_limit > 0 (not the reference writer): the dictionary stops growing at
  // the first value that would push its PLAIN page past the limit (or past 32767 entries); that value
  // and every later one go to pages of the column's own encoding (mid-chunk fallback).
  int64_t fallback_v = v1;
  if (use_dict && (vsize == 4 || vsize == 8) && L.type != BYTE_ARRAY && c.dict_page_limit == 0 &&
      !opt.no_fast_paths) {
    // the same dictionary for 4 / 8-byte values, keyed by their bits in an open-addressing table
    // (at most 32768 entries in 65536 slots) instead of a hash map of string views
    constexpr uint32_t kSlots = 1u << 16;
    std::vector<uint64_t> keys(kSlots);
    std::vector<int32_t> ids(kSlots, -1);
    idx.resize(size_t(v1 - v0));
    for (int64_t i = v0; i < v1 && use_dict; i++) {
      uint64_t x = 0;
      memcpy(&x, c.values + i * vsize, size_t(vsize));
      uint32_t h = uint32_t((x * 0x9e3779b97f4a7c15ull) >> 48);
      while (ids[h] >= 0 && keys[h] != x) h = (h + 1) & (kSlots - 1);
      if (ids[h] < 0) {
        const int32_t k = int32_t(dict.size());
        keys[h] = x;
        ids[h] = k;
        dict.push_back(value_at(L, c, i));
        idx[size_t(i - v0)] = k;
        if (dict.size() > 32767) use_dict = false;
      } else {
        idx[size_t(i - v0)] = ids[h];
      }
    }
    if (!use_dict) {
      idx.clear();
      dict.clear();
    }
  } else if (use_dict) {
    std::unordered_map<std::string_view, int32_t> m;
    m.reserve(1 << 15);
    idx.resize(size_t(v1 - v0));
    int64_t dict_bytes = 0;
    for (int64_t i = v0; i < v1 && use_dict; i++) {
      std::string_view v = value_at(L, c, i);
      auto it = m.find(v);
      if (it == m.end()) {
        const int64_t sz = L.type == BYTE_ARRAY ? 4 + int64_t(v.size()) : int64_t(v.size());
        if (c.dict_page_limit > 0 && (dict_bytes + sz > c.dict_page_limit || dict.size() >= 32767)) {
          fallback_v = i;
          break;
        }
        dict_bytes += sz;
        int32_t k = int32_t(dict.size());
        m.emplace(v, k);
        dict.push_back(v);
        idx[size_t(i - v0)] = k;
        if (dict.size() > 32767) use_dict = false;
      } else {
        idx[size_t(i - v0)] = it->second;
      }
    }
    if (!use_dict) {
      idx.clear();
      dict.clear();
    }
  }
  const int dict_enc = use_dict ? E_RLE_DICT : c.encoding;
  int enc = dict_enc;
  out.enc = c.encoding;
  out.has_dict = use_dict;

  // (the chunk's bytes: values plus a little for levels and headers, reserved once)
  out.bytes.reserve(size_t(std::max<int64_t>(0, (v1 - v0) * std::max(vsize, 1)) + (s1 - s0) / 2 + 4096));
  auto emit_page = [&](int type, std::vector<uint8_t>& lv_rep, std::vector<uint8_t>& lv_def,
                       std::vector<uint8_t>& vals, int32_t nslots, int32_t nulls, int32_t rows) {
    std::vector<uint8_t> block, comp;
    if (type == 3) {
      const size_t vsz = vals.size();
      if (codec == 0) comp.swap(vals);  // UNCOMPRESSED: the values as they are (no copy)
      else if (!compress_block(codec, vals.data(), vals.size(), comp)) out.err = "compress";
      std::vector<uint8_t> crcbuf;
      uint32_t crc = 0;
      if (opt.enable_crc) {
        crcbuf.insert(crcbuf.end(), lv_rep.begin(), lv_rep.end());
        crcbuf.insert(crcbuf.end(), lv_def.begin(), lv_def.end());
        crcbuf.insert(crcbuf.end(), comp.begin(), comp.end());
        crc = crc32_ieee(crcbuf.data(), crcbuf.size());
      }
      int32_t ls = int32_t(lv_rep.size() + lv_def.size());
      write_page_header(out.bytes, 3, int32_t(vsz) + ls, int32_t(comp.size()) + ls, opt.enable_crc, crc,
                        nslots, enc, nulls, rows, int32_t(lv_def.size()), int32_t(lv_rep.size()),
                        codec != 0);
      out.bytes.insert(out.bytes.end(), lv_rep.begin(), lv_rep.end());
      out.bytes.insert(out.bytes.end(), lv_def.begin(), lv_def.end());
      out.bytes.insert(out.bytes.end(), comp.begin(), comp.end());
      out.total_uncompressed += int64_t(vsz) + ls;
      if (codec == 0) comp.swap(vals);
    } else {
      block.insert(block.end(), lv_rep.begin(), lv_rep.end());
      block.insert(block.end(), lv_def.begin(), lv_def.end());
      block.insert(block.end(), vals.begin(), vals.end());
      if (!compress_block(codec, block.data(), block.size(), comp)) out.err = "compress";
      uint32_t crc = opt.enable_crc ? crc32_ieee(comp.data(), comp.size()) : 0;
      write_page_header(out.bytes, type, int32_t(block.size()), int32_t(comp.size()), opt.enable_crc, crc, nslots,
                        type == 2 ? E_PLAIN : enc, nulls, rows, 0, 0, codec != 0);
      out.bytes.insert(out.bytes.end(), comp.begin(), comp.end());
      out.total_uncompressed += int64_t(block.size());
    }
  };

  if (use_dict) {  // dictPageWriter.write (page_dict.go:74-136)
    std::vector<uint8_t> vals, e1, e2;
    for (auto& v : dict) plain_value(L, v, vals);
    emit_page(2, e1, e2, vals, int32_t(dict.size()), 0, 0);
    out.data_page_rel = int64_t(out.bytes.size());
  }

  // Fast path (the same pages as the general loop below, bulk-encoded): a required flat
  // non-dictionary fixed-width column has no levels, so estimateSize() is the value bytes and a page
  // ends after ceil(max_page / size) values (a DELTA page of n values with (n - 1) % 128 == 0 takes
  // one more when values are left).  opt.no_fast_paths = 1 forces the loop (tests compare both).
  if (!opt.no_fast_paths && L.max_rep == 0 && L.max_def == 0 && !use_dict && vsize > 0 && L.type != BOOLEAN &&
      L.type != BYTE_ARRAY &&
      (c.encoding == E_PLAIN || (c.encoding == E_DELTA_BP && (L.type == INT32 || L.type == INT64)))) {
    const int64_t per = (ctx.max_page + vsize - 1) / vsize;
    std::vector<uint8_t> lr, ld, vals;
    for (int64_t pv = v0; pv < v1;) {
      int64_t nv = std::min<int64_t>(per, v1 - pv);
      if (c.encoding == E_DELTA_BP && nv > 0 && (nv - 1) % 128 == 0 && pv + nv < v1) nv++;
      vals.clear();
      if (c.encoding == E_DELTA_BP) {
        if (L.type == INT32)
          delta_encode<int32_t, uint32_t>(reinterpret_cast<const int32_t*>(c.values) + pv, nv, vals);
        else
          delta_encode<int64_t, uint64_t>(reinterpret_cast<const int64_t*>(c.values) + pv, nv, vals);
      } else {
        vals.assign(c.values + pv * vsize, c.values + (pv + nv) * vsize);
      }
      enc = c.encoding;
      emit_page(v2 ? 3 : 0, lr, ld, vals, int32_t(nv), 0, int32_t(nv));
      pv += nv;
    }
    return;
  }

  // --- page cut: estimateSize() >= maxPageSize after a record (data_store.go:138-159) ---
  std::vector<uint32_t> tmp;
  int64_t s = s0, v = v0;
  std::vector<uint8_t> seen(use_dict ? dict.size() : size_t{0});
  std::unordered_set<std::string_view> uniq;
  while (s < s1) {
    int64_t ps = s, pv = v;
    int64_t est_vals = 0, uniq_bytes = 0, uniq_count = 0;
    int32_t rows = 0;
    std::fill(seen.begin(), seen.end(), 0);
    uniq.clear();
    while (s < s1) {
      // one record: first slot + following slots with rep > 0
      int64_t e = s + 1;
      if (L.max_rep > 0)
        while (e < s1 && c.rep_levels[e] > 0) e++;
      for (int64_t k = s; k < e; k++) {
        bool defined = L.max_def == 0 || c.def_levels[k] == L.max_def;
        if (!defined) continue;
        int64_t sz = L.type == BOOLEAN ? 0 : L.type == BYTE_ARRAY ? (c.offsets[v + 1] - c.offsets[v]) : vsize;
        est_vals += sz;
        if (c.use_dict && L.type != BOOLEAN && uniq_count <= 32767) {
          bool fresh;
          if (use_dict && v < fallback_v) {
            int32_t id = idx[size_t(v - v0)];
            fresh = !seen[size_t(id)];
            seen[size_t(id)] = 1;
          } else {
            fresh = uniq.insert(value_at(L, c, v)).second;
          }
          if (fresh) {
            uniq_bytes += sz;
            uniq_count++;
          }
        }
        v++;
      }
      s = e;
      rows++;
      int64_t cnt = s - ps;
      int64_t lvl = ((cnt - 1) / 8) * (rw + dw);
      int64_t est = (c.use_dict && L.type != BOOLEAN) ? uniq_bytes + 4 * (v - pv) + lvl : est_vals + lvl;
      if (pv < fallback_v && v >= fallback_v) break;  // dictionary pages end where the fallback starts
      if (est >= ctx.max_page) {
        // Generator choice (not the reference writer): a DELTA-family page of n values with
        // (n-1) % 128 == 0 cannot be read back by the reference decoder (read-ahead quirk,
        // SURVEY.md A.3), so such a page takes one more record when one is left.
        const bool delta_page = !(use_dict && pv < fallback_v) &&
                                (c.encoding == E_DELTA_BP || c.encoding == E_DLBA || c.encoding == E_DBA);
        const int64_t nv = v - pv;
        if (delta_page && nv > 0 && (nv - 1) % 128 == 0 && s < s1) continue;
        break;
      }
    }
    // encode the page [ps, s) with values [pv, v)
    int32_t nslots = int32_t(s - ps), nvals = int32_t(v - pv);
    std::vector<uint8_t> lr, ld, vals;
    if (L.max_rep > 0) {
      tmp.assign(c.rep_levels + ps, c.rep_levels + s);
      if (v2) hybrid_encode(rw, tmp.data(), nslots, lr);
      else hybrid_encode_sized(rw, tmp.data(), nslots, lr);
    }
    if (L.max_def > 0) {
      tmp.assign(c.def_levels + ps, c.def_levels + s);
      if (v2) hybrid_encode(dw, tmp.data(), nslots, ld);
      else hybrid_encode_sized(dw, tmp.data(), nslots, ld);
    }
    const bool page_dict = use_dict && pv < fallback_v;
    enc = page_dict ? dict_enc : c.encoding;
    if (page_dict) {  // dictEncoder.Close (type_dict.go:113-127)
      int w = bits_len(dict.size());
      vals.push_back(uint8_t(w));
      tmp.assign(idx.begin() + (pv - v0), idx.begin() + (v - v0));
      hybrid_encode(w, tmp.data(), nvals, vals);
    } else if (L.type == BOOLEAN) {
      if (c.encoding == E_RLE) {
        tmp.resize(size_t(nvals));
        for (int32_t k = 0; k < nvals; k++) tmp[size_t(k)] = c.values[pv + k] ? 1 : 0;
        hybrid_encode_sized(1, tmp.data(), nvals, vals);
      } else {  // booleanPlainEncoder: packedArray(1) + flush (always one more group)
        int64_t nb = nvals == 0 ? 1 : (nvals + 7) / 8;
        vals.assign(size_t(nb), 0);
        for (int32_t k = 0; k < nvals; k++)
          if (c.values[pv + k]) vals[size_t(k >> 3)] |= uint8_t(1u << (k & 7));
      }
    } else if (c.encoding == E_DELTA_BP && (L.type == INT32 || L.type == INT64)) {
      if (L.type == INT32)
        delta_encode<int32_t, uint32_t>(reinterpret_cast<const int32_t*>(c.values) + pv, nvals, vals);
      else
        delta_encode<int64_t, uint64_t>(reinterpret_cast<const int64_t*>(c.values) + pv, nvals, vals);
    } else if (c.encoding == E_DLBA || c.encoding == E_DBA) {
      std::vector<int32_t> lens, prefix;
      std::vector<uint8_t> data;
      std::string_view prev;
      for (int64_t k = pv; k < v; k++) {
        std::string_view x = value_at(L, c, k);
        size_t p = 0;
        if (c.encoding == E_DBA) {
          while (p < prev.size() && p < x.size() && prev[p] == x[p]) p++;
          prefix.push_back(int32_t(p));
        }
        lens.push_back(int32_t(x.size() - p));
        data.insert(data.end(), x.begin() + p, x.end());
        prev = x;
      }
      if (c.encoding == E_DBA) delta_encode<int32_t, uint32_t>(prefix.data(), int64_t(prefix.size()), vals);
      delta_encode<int32_t, uint32_t>(lens.data(), int64_t(lens.size()), vals);
      vals.insert(vals.end(), data.begin(), data.end());
    } else {
      for (int64_t k = pv; k < v; k++) plain_value(L, value_at(L, c, k), vals);
    }
    emit_page(v2 ? 3 : 0, lr, ld, vals, nslots, nslots - nvals, rows);
  }
}

void compute_leaves(const pqg_schema_element* sc, int32_t n, std::vector<Leaf>& leaves, std::string& err) {
  struct Fr {
    int remaining;
    int d, r;
    std::vector<std::string> path;
  };
  // readSchema (schema.go:992-1015): root group, then DFS
  std::vector<Fr> st;
  if (n <= 0) {
    err = "empty schema";
    return;
  }
  st.push_back({sc[0].num_children, 0, 0, {}});
  for (int32_t i = 1; i < n; i++) {
    while (!st.empty() && st.back().remaining == 0) st.pop_back();
    if (st.empty()) {
      err = "schema has extra elements";
      return;
    }
    Fr& parent = st.back();
    parent.remaining--;
    const pqg_schema_element& e = sc[i];
    int d = parent.d + (e.repetition == 1 || e.repetition == 2 ? 1 : 0);
    int r = parent.r + (e.repetition == 2 ? 1 : 0);
    std::vector<std::string> path = parent.path;
    path.push_back(e.name);
    if (e.type < 0) {
      st.push_back({e.num_children, d, r, path});
    } else {
      Leaf L;
      L.type = e.type;
      L.type_length = e.type_length;
      L.max_def = d;
      L.max_rep = r;
      L.converted = e.converted_type;
      L.path = path;
      leaves.push_back(L);
    }
  }
}


// Per chunk: what the footer records (ColumnMetaData) and where the chunk starts in the file.
struct ChunkMeta {
  bool has_dict = false;
  int64_t pos = 0, size = 0, data_page_rel = 0, total_uncompressed = 0, num_slots = 0;
  int enc = 0;
};

ChunkMeta meta_of(const ChunkOut& ch, int64_t pos) {
  ChunkMeta m;
  m.has_dict = ch.has_dict;
  m.pos = pos;
  m.size = int64_t(ch.bytes.size());
  m.data_page_rel = ch.data_page_rel;
  m.total_uncompressed = ch.total_uncompressed;
  m.num_slots = ch.num_slots;
  m.enc = ch.enc;
  return m;
}

// The column chunks of row groups [0, num_row_groups) of `columns` (which hold exactly those rows),
// encoded in parallel (row-group-major order).
bool encode_row_groups(const std::vector<Leaf>& leaves, const pqg_column_data* columns, const int64_t* rg_rows,
                       int32_t num_row_groups, const pqg_options* opt, std::vector<ChunkOut>& chunks, std::string& err) {
  const int32_t num_columns = int32_t(leaves.size());
  Ctx ctx{opt, opt->max_page_size > 0 ? opt->max_page_size : (1 << 20)};
  // per column: slot / value start of every row group
  std::vector<std::vector<int64_t>> slot_at(static_cast<size_t>(num_columns)), val_at(static_cast<size_t>(num_columns));
  for (int32_t ci = 0; ci < num_columns; ci++) {
    const Leaf& L = leaves[size_t(ci)];
    const pqg_column_data& c = columns[ci];
    auto& sa = slot_at[size_t(ci)];
    auto& va = val_at[size_t(ci)];
    sa.push_back(0);
    va.push_back(0);
    int64_t s = 0, v = 0;
    for (int32_t r = 0; r < num_row_groups; r++) {
      int64_t recs = 0;
      while (s < c.num_slots && recs < rg_rows[r]) {
        int64_t e2 = s + 1;
        if (L.max_rep > 0)
          while (e2 < c.num_slots && c.rep_levels[e2] > 0) e2++;
        if (L.max_def > 0) {
          for (int64_t k = s; k < e2; k++) v += c.def_levels[k] == L.max_def;
        } else {
          v += e2 - s;
        }
        s = e2;
        recs++;
      }
      if (recs != rg_rows[r]) {
        err = "not enough records for the row groups in column " + std::to_string(ci);
        return false;
      }
      sa.push_back(s);
      va.push_back(v);
    }
    if (v > c.num_values) {
      err = "not enough values in column " + std::to_string(ci);
      return false;
    }
  }
  int64_t nchunks = int64_t(num_row_groups) * num_columns;
  chunks.assign(static_cast<size_t>(nchunks), ChunkOut());
  std::atomic<int64_t> next{0};
  int nt = opt->num_threads > 0 ? opt->num_threads : int(std::thread::hardware_concurrency());
  if (nt < 1) nt = 1;
  if (nt > 16) nt = 16;  // the GPU box's CPU share
  if (nt > nchunks) nt = int(std::max<int64_t>(1, nchunks));
  auto work = [&]() {
    for (;;) {
      int64_t k = next.fetch_add(1);
      if (k >= nchunks) return;
      int32_t r = int32_t(k / num_columns), ci = int32_t(k % num_columns);
      encode_chunk(ctx, leaves[size_t(ci)], columns[ci], slot_at[size_t(ci)][size_t(r)],
                   slot_at[size_t(ci)][size_t(r) + 1], val_at[size_t(ci)][size_t(r)],
                   val_at[size_t(ci)][size_t(r) + 1], chunks[size_t(k)]);
    }
  };
  std::vector<std::thread> th;
  for (int i = 0; i < nt; i++) th.emplace_back(work);
  for (auto& t : th) t.join();
  for (auto& ch : chunks)
    if (!ch.err.empty()) {
      err = ch.err;
      return false;
    }
  return true;
}

// FileMetaData (file_writer.go): schema, rows, one RowGroup per rg_rows entry with its chunks' metas.
std::vector<uint8_t> footer_bytes(const pqg_schema_element* schema, int32_t num_schema, const std::vector<Leaf>& leaves,
                                  const std::vector<ChunkMeta>& metas, const int64_t* rg_rows, int32_t num_row_groups,
                                  const pqg_options* opt) {
  const int32_t num_columns = int32_t(leaves.size());
  std::vector<uint8_t> footer;
  TWriter w(footer);
  w.i32(1, 1);
  w.begin_list(2, T_STRUCT, uint32_t(num_schema));
  for (int32_t i = 0; i < num_schema; i++) {
    const pqg_schema_element& s = schema[i];
    w.begin_elem();
    if (s.type >= 0) w.i32(1, s.type);
    if (s.type == FLBA) w.i32(2, s.type_length);
    if (s.repetition >= 0) w.i32(3, s.repetition);
    w.binary(4, s.name ? s.name : "");
    if (s.type < 0) w.i32(5, s.num_children);
    if (s.converted_type >= 0) w.i32(6, s.converted_type);
    w.end_elem();
  }
  int64_t nrows = 0;
  for (int32_t r = 0; r < num_row_groups; r++) nrows += rg_rows[r];
  w.i64(3, nrows);
  w.begin_list(4, T_STRUCT, uint32_t(num_row_groups));
  for (int32_t r = 0; r < num_row_groups; r++) {
    w.begin_elem();
    w.begin_list(1, T_STRUCT, uint32_t(num_columns));
    int64_t rg_total = 0, rg_comp = 0;
    for (int32_t ci = 0; ci < num_columns; ci++) {
      const ChunkMeta& ch = metas[size_t(r) * size_t(num_columns) + size_t(ci)];
      const Leaf& L = leaves[size_t(ci)];
      w.begin_elem();
      w.i64(2, ch.pos);
      w.begin_struct(3);
      w.i32(1, L.type);
      int nenc = ch.has_dict ? 3 : 2;
      w.begin_list(2, T_I32, uint32_t(nenc));
      w.list_elem_i32(E_RLE);
      w.list_elem_i32(ch.has_dict ? E_PLAIN : ch.enc);
      if (ch.has_dict) w.list_elem_i32(E_RLE_DICT);
      w.begin_list(3, T_BINARY, uint32_t(L.path.size()));
      for (auto& p : L.path) w.list_elem_binary(p);
      w.i32(4, opt->codec);
      w.i64(5, ch.num_slots);
      w.i64(6, ch.total_uncompressed);
      w.i64(7, ch.size);
      w.i64(9, ch.pos + ch.data_page_rel);
      if (ch.has_dict) w.i64(11, ch.pos);
      w.end_struct();
      w.end_elem();
      rg_total += ch.total_uncompressed;
      rg_comp += ch.size;
    }
    w.i64(2, rg_total);
    w.i64(3, rg_rows[r]);
    w.i64(6, rg_comp);
    w.end_elem();
  }
  w.binary(6, "parquet-go_amd pqgen (reference-writer layout)");
  w.stop();
  return footer;
}

}  // namespace

extern "C" {

int64_t pqg_hybrid_encode(int32_t width, const int32_t* values, int64_t n, uint8_t* out, int64_t cap) {
  std::vector<uint8_t> o;
  std::vector<uint32_t> v(values, values + n);
  hybrid_encode(width, v.data(), n, o);
  if (int64_t(o.size()) > cap) return -int64_t(o.size());
  if (!o.empty()) memcpy(out, o.data(), o.size());  // (an empty stream: memcpy needs non-null pointers)
  return int64_t(o.size());
}

int64_t pqg_delta_encode32(const int32_t* values, int64_t n, uint8_t* out, int64_t cap) {
  std::vector<uint8_t> o;
  delta_encode<int32_t, uint32_t>(values, n, o);
  if (int64_t(o.size()) > cap) return -int64_t(o.size());
  if (!o.empty()) memcpy(out, o.data(), o.size());  // (an empty stream: memcpy needs non-null pointers)
  return int64_t(o.size());
}

int64_t pqg_delta_encode64(const int64_t* values, int64_t n, uint8_t* out, int64_t cap) {
  std::vector<uint8_t> o;
  delta_encode<int64_t, uint64_t>(values, n, o);
  if (int64_t(o.size()) > cap) return -int64_t(o.size());
  if (!o.empty()) memcpy(out, o.data(), o.size());  // (an empty stream: memcpy needs non-null pointers)
  return int64_t(o.size());
}

int pqg_write(const pqg_schema_element* schema, int32_t num_schema, const pqg_column_data* columns,
              int32_t num_columns, const int64_t* rg_rows, int32_t num_row_groups, const pqg_options* opt,
              uint8_t** out, int64_t* out_len, char* err, int32_t err_cap) {
  auto fail = [&](const std::string& m) {
    if (err && err_cap > 0) snprintf(err, size_t(err_cap), "%s", m.c_str());
    return 1;
  };
  std::vector<Leaf> leaves;
  std::string e;
  compute_leaves(schema, num_schema, leaves, e);
  if (!e.empty()) return fail(e);
  if (int32_t(leaves.size()) != num_columns) return fail("column count does not match schema leaves");
  std::vector<ChunkOut> chunks;
  if (!encode_row_groups(leaves, columns, rg_rows, num_row_groups, opt, chunks, e)) return fail(e);
  std::vector<ChunkMeta> metas;
  int64_t pos = 4;
  for (auto& ch : chunks) {
    metas.push_back(meta_of(ch, pos));
    pos += int64_t(ch.bytes.size());
  }
  const std::vector<uint8_t> footer = footer_bytes(schema, num_schema, leaves, metas, rg_rows, num_row_groups, opt);
  const int64_t total = pos + int64_t(footer.size()) + 8;
  uint8_t* buf = static_cast<uint8_t*>(malloc(size_t(total)));
  if (!buf) return fail("out of memory");
  uint8_t* p = buf;
  memcpy(p, "PAR1", 4);
  p += 4;
  for (auto& ch : chunks) {
    memcpy(p, ch.bytes.data(), ch.bytes.size());
    p += ch.bytes.size();
  }
  memcpy(p, footer.data(), footer.size());
  p += footer.size();
  uint32_t fl = uint32_t(footer.size());
  memcpy(p, &fl, 4);
  memcpy(p + 4, "PAR1", 4);
  *out = buf;
  *out_len = total;
  return 0;
}

// Streaming: row groups appended to a caller's buffer, the footer at the end.
struct pqg_stream {
  std::vector<pqg_schema_element> schema;
  std::vector<std::string> names;
  std::vector<Leaf> leaves;
  pqg_options opt;
  std::vector<ChunkMeta> metas;
  std::vector<int64_t> rg_rows;
};

pqg_stream* pqg_stream_open(const pqg_schema_element* schema, int32_t num_schema, const pqg_options* opt, char* err,
                            int32_t err_cap) {
  std::vector<Leaf> leaves;
  std::string e;
  compute_leaves(schema, num_schema, leaves, e);
  if (!e.empty()) {
    if (err && err_cap > 0) snprintf(err, size_t(err_cap), "%s", e.c_str());
    return nullptr;
  }
  auto* s = new pqg_stream();
  s->names.reserve(size_t(num_schema));
  for (int32_t i = 0; i < num_schema; i++) s->names.push_back(schema[i].name ? schema[i].name : "");
  for (int32_t i = 0; i < num_schema; i++) {
    pqg_schema_element el = schema[i];
    el.name = s->names[size_t(i)].c_str();
    s->schema.push_back(el);
  }
  s->leaves = std::move(leaves);
  s->opt = *opt;
  return s;
}

int pqg_stream_write(pqg_stream* s, const pqg_column_data* columns, int32_t num_columns, const int64_t* rg_rows,
                     int32_t num_row_groups, uint8_t* dst, int64_t cap, int64_t* pos, char* err, int32_t err_cap) {
  auto fail = [&](const std::string& m) {
    if (err && err_cap > 0) snprintf(err, size_t(err_cap), "%s", m.c_str());
    return 1;
  };
  if (!s || !pos) return fail("null stream");
  if (int32_t(s->leaves.size()) != num_columns) return fail("column count does not match schema leaves");
  std::vector<ChunkOut> chunks;
  std::string e;
  if (!encode_row_groups(s->leaves, columns, rg_rows, num_row_groups, &s->opt, chunks, e)) return fail(e);
  int64_t need = *pos == 0 ? 4 : 0;
  for (auto& ch : chunks) need += int64_t(ch.bytes.size());
  if (*pos + need > cap) return fail("stream buffer too small");
  if (*pos == 0) {
    memcpy(dst, "PAR1", 4);
    *pos = 4;
  }
  for (auto& ch : chunks) {
    s->metas.push_back(meta_of(ch, *pos));
    memcpy(dst + *pos, ch.bytes.data(), ch.bytes.size());
    *pos += int64_t(ch.bytes.size());
  }
  for (int32_t r = 0; r < num_row_groups; r++) s->rg_rows.push_back(rg_rows[r]);
  return 0;
}

int pqg_stream_finish(pqg_stream* s, uint8_t* dst, int64_t cap, int64_t* pos, char* err, int32_t err_cap) {
  auto fail = [&](const std::string& m) {
    if (err && err_cap > 0) snprintf(err, size_t(err_cap), "%s", m.c_str());
    return 1;
  };
  if (!s || !pos) return fail("null stream");
  if (*pos == 0) {
    if (cap < 4) return fail("stream buffer too small");
    memcpy(dst, "PAR1", 4);
    *pos = 4;
  }
  const std::vector<uint8_t> footer = footer_bytes(s->schema.data(), int32_t(s->schema.size()), s->leaves, s->metas,
                                                   s->rg_rows.data(), int32_t(s->rg_rows.size()), &s->opt);
  if (*pos + int64_t(footer.size()) + 8 > cap) return fail("stream buffer too small");
  memcpy(dst + *pos, footer.data(), footer.size());
  *pos += int64_t(footer.size());
  const uint32_t fl = uint32_t(footer.size());
  memcpy(dst + *pos, &fl, 4);
  memcpy(dst + *pos + 4, "PAR1", 4);
  *pos += 8;
  return 0;
}

void pqg_stream_close(pqg_stream* s) { delete s; }

void pqg_free(uint8_t* p) { free(p); }

}  // extern "C"

// ---- the mixed-encoding bench workload's columns (tooling: seeded inputs, not the decode path) ----
namespace {
// splitmix64 of (seed, row group, column, row): a counter-based stream, so any row group (or any
// slice of one) is regenerated exactly, whatever the thread split.
inline uint64_t mix64(uint64_t x) {
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}
inline uint64_t hval(uint64_t seed, int64_t g, int k, int64_t i) {
  return mix64(mix64(seed * 0x100000001b3ull + uint64_t(g) * 977 + uint64_t(k)) ^ uint64_t(i));
}

template <class F>
void par_rows(int64_t rows, int threads, F&& f) {  // f(r0, r1, block)
  int nt = threads > 0 ? threads : int(std::thread::hardware_concurrency());
  nt = std::max(1, std::min(nt, 16));
  if (rows < (int64_t(1) << 16)) nt = 1;
  std::vector<std::thread> th;
  for (int t = 0; t < nt; t++)
    th.emplace_back([&, t]() { f(rows * t / nt, rows * (t + 1) / nt, t); });
  for (auto& x : th) x.join();
}
}  // namespace

extern "C" {

void pqg_mixed_dicts(uint64_t seed, int32_t* d_i32, float* d_f32) {
  for (int k = 0; k < 1000; k++) d_i32[k] = int32_t(uint32_t(hval(seed, -1, 0, k)));
  for (int k = 0; k < 256; k++) d_f32[k] = float(int64_t(hval(seed, -1, 2, k) >> 40) - (int64_t(1) << 23)) / 65536.0f;
}

int64_t pqg_mixed_row_group(uint64_t seed, int32_t g, int64_t rows, int32_t* i32, int64_t* i64, float* f32,
                            double* f64, uint8_t* f64_def, uint8_t* b, uint8_t* uuid, int64_t* ts, int32_t threads) {
  int32_t d_i32[1000];
  float d_f32[256];
  pqg_mixed_dicts(seed, d_i32, d_f32);
  const int nt_max = 16;
  std::vector<int64_t> nn(nt_max + 1, 0), tsum(nt_max + 1, 0);
  // pass 1: everything but the compacted doubles' positions and the timestamps' carries
  par_rows(rows, threads, [&](int64_t r0, int64_t r1, int t) {
    int64_t cnt = 0, s = 0;
    for (int64_t i = r0; i < r1; i++) {
      i32[i] = d_i32[hval(seed, g, 0, i) % 1000];
      i64[i] = int64_t(hval(seed, g, 1, i));
      f32[i] = d_f32[hval(seed, g, 2, i) & 255];
      const uint64_t h3 = hval(seed, g, 3, i);
      f64_def[i] = (h3 % 100) != 0;  // 1% nulls
      cnt += f64_def[i];
      b[i] = uint8_t(hval(seed, g, 4, i) & 1);
      const uint64_t u0 = hval(seed, g, 5, 2 * i), u1 = hval(seed, g, 5, 2 * i + 1);
      memcpy(uuid + 16 * i, &u0, 8);
      memcpy(uuid + 16 * i + 8, &u1, 8);
      s += 1000000 + int64_t(hval(seed, g, 6, i) & 4095);
    }
    nn[size_t(t) + 1] = cnt;
    tsum[size_t(t) + 1] = s;
  });
  for (int t = 0; t < nt_max; t++) {
    nn[size_t(t) + 1] += nn[size_t(t)];
    tsum[size_t(t) + 1] += tsum[size_t(t)];
  }
  // pass 2: the non-null doubles compacted, the timestamps as running sums (a row group's first
  // value starts at its own base: 1.7e18 + g * 2^44, so row groups regenerate independently)
  const int64_t base = 1700000000000000000ll + int64_t(g) * (int64_t(1) << 44);
  par_rows(rows, threads, [&](int64_t r0, int64_t r1, int t) {
    int64_t o = nn[size_t(t)], acc = base + tsum[size_t(t)];
    for (int64_t i = r0; i < r1; i++) {
      if (f64_def[i]) {
        const uint64_t h = hval(seed, g, 3, i) >> 11;
        f64[o++] = double(int64_t(h) - (int64_t(1) << 52)) / double(int64_t(1) << 40);
      }
      acc += 1000000 + int64_t(hval(seed, g, 6, i) & 4095);
      ts[i] = acc;
    }
  });
  return nn[size_t(nt_max)];
}

}  // extern "C"
