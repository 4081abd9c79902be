// thrift_compact.h — Thrift compact-protocol reader/writer for the Parquet footer and page headers
// (the structs of reference parquet/parquet.thrift).  The reference reads them through the
// generated apache/thrift v0.16.0 code (helpers.go:103-109, parquet/parquet.go); the reader below
// restates that library's rules and the generated readers' field / required-field checks (as the
// data tables of thrift_spec.h), so that corrupt footers and headers fail exactly where the
// reference's do.
#pragma once

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "thrift_spec.h"

namespace pqhip {

enum TType : uint8_t {
  T_STOP = 0,
  T_BOOL_TRUE = 1,
  T_BOOL_FALSE = 2,
  T_BYTE = 3,
  T_I16 = 4,
  T_I32 = 5,
  T_I64 = 6,
  T_DOUBLE = 7,
  T_BINARY = 8,
  T_LIST = 9,
  T_SET = 10,
  T_MAP = 11,
  T_STRUCT = 12
};

// ------------------------------------------------------------------------------------------------
// Reader with the semantics of the reference's thrift library (vendored apache/thrift v0.16.0,
// lib/go/thrift/compact_protocol.go + protocol.go Skip): bounded, never reads past `end`; every
// error sets ok=false and later reads return 0.
//   * field header (ReadFieldBegin :429-468): a byte whose low nibble is 0 is STOP whatever its high
//     nibble; id = last + delta, or a zigzag i16 when the delta is 0; nibbles 13-15 are errors;
//     boolean fields carry their value in the header (consumed by the next read_bool);
//   * varints (readVarint64 :747-762) have no length limit (bits past 63 vanish); i32 / i16 truncate;
//   * list / string sizes (ReadListBegin :505-529, ReadString :601-622) must be >= 0 and at most
//     DEFAULT_MAX_MESSAGE_SIZE (configuration.go:30, :305-319); a short string is an error;
//   * skip (protocol.go:92-182) recurses at most DEFAULT_RECURSION_DEPTH (64) levels; a map's
//     unknown key / value nibble reads as STOP and fails when an element is skipped.
// ------------------------------------------------------------------------------------------------
constexpr int64_t kThriftMaxSize = 100 * 1024 * 1024;  // DEFAULT_MAX_MESSAGE_SIZE
constexpr int kThriftMaxDepth = 64;                    // DEFAULT_RECURSION_DEPTH

class TReader {
 public:
  TReader(const uint8_t* p, const uint8_t* end) : p_(p), begin_(p), end_(end) {}
  bool ok() const { return ok_; }
  size_t consumed() const { return size_t(p_ - begin_); }

  uint8_t byte() {
    if (!ok_ || p_ >= end_) return fail();
    return *p_++;
  }
  uint64_t varint64() {
    uint64_t x = 0;
    for (unsigned s = 0;; s += 7) {
      const uint8_t b = byte();
      if (!ok_) return 0;
      if (s < 64) x |= uint64_t(b & 0x7f) << s;
      if (!(b & 0x80)) return x;
    }
  }
  int32_t varint32() { return int32_t(uint32_t(varint64())); }
  int32_t i32() {
    const uint32_t u = uint32_t(varint32());
    return int32_t(u >> 1) ^ -int32_t(u & 1);
  }
  int16_t i16() { return int16_t(i32()); }
  int64_t i64() {
    const uint64_t u = varint64();
    return int64_t(u >> 1) ^ -int64_t(u & 1);
  }
  double dbl() {
    if (!ok_ || end_ - p_ < 8) {
      fail();
      return 0;
    }
    double d;
    memcpy(&d, p_, 8);
    p_ += 8;
    return d;
  }
  bool str(std::string& out) {
    const int32_t n = varint32();
    if (!ok_ || n < 0 || n > kThriftMaxSize || int64_t(n) > end_ - p_) {
      fail();
      return false;
    }
    out.assign(reinterpret_cast<const char*>(p_), size_t(n));
    p_ += n;
    return true;
  }
  // compact type nibble -> wire type (1 = bool), 0 = STOP, 0xff = unknown (getTType :802-830)
  static uint8_t wire_type(uint8_t nib) {
    nib &= 0x0f;
    if (nib == 2) return T_BOOL_TRUE;
    return nib <= T_STRUCT ? nib : 0xff;
  }
  // Field header: false at STOP or on an error.  `last` is the previous field id of this struct.
  bool field(int16_t& last, int16_t& id, uint8_t& type) {
    const uint8_t h = byte();
    if (!ok_ || (h & 0x0f) == T_STOP) return false;
    const int16_t d = int16_t(h >> 4);
    id = d ? int16_t(last + d) : i16();
    type = wire_type(h);
    if (!ok_ || type == 0xff) {
      fail();
      return false;
    }
    if (type == T_BOOL_TRUE) {
      bool_pending_ = true;
      bool_value_ = (h & 0x0f) == T_BOOL_TRUE;
    }
    last = id;
    return true;
  }
  bool read_bool() {  // ReadBool (:546-553): the header's value, else one byte
    if (bool_pending_) {
      bool_pending_ = false;
      return bool_value_;
    }
    return byte() == T_BOOL_TRUE;
  }
  // List / set header: element wire type + size.
  bool list(uint8_t& etype, int32_t& n) {
    const uint8_t h = byte();
    n = h >> 4;
    if (n == 15) n = varint32();
    etype = wire_type(h);
    if (!ok_ || n < 0 || n > kThriftMaxSize || etype == 0xff) {
      fail();
      return false;
    }
    return true;
  }
  void skip(uint8_t type, int depth = kThriftMaxDepth) {
    if (depth <= 0) {
      fail();
      return;
    }
    switch (type) {
      case T_BOOL_TRUE:
      case T_BOOL_FALSE:
        read_bool();
        return;
      case T_BYTE:
        byte();
        return;
      case T_I16:
      case T_I32:
        varint32();
        return;
      case T_I64:
        varint64();
        return;
      case T_DOUBLE:
        dbl();
        return;
      case T_BINARY: {
        std::string s;
        str(s);
        return;
      }
      case T_LIST:
      case T_SET: {
        uint8_t et;
        int32_t n;
        if (!list(et, n)) return;
        for (int32_t i = 0; i < n && ok_; i++) skip(et, depth - 1);
        return;
      }
      case T_MAP: {
        const int32_t n = varint32();
        if (!ok_ || n < 0 || n > kThriftMaxSize) {
          fail();
          return;
        }
        const uint8_t kv = n ? byte() : 0;
        const uint8_t kt = wire_type(kv >> 4), vt = wire_type(kv & 0x0f);
        for (int32_t i = 0; i < n && ok_; i++) {
          skip(kt == 0xff ? 0 : kt, depth - 1);
          skip(vt == 0xff ? 0 : vt, depth - 1);
        }
        return;
      }
      case T_STRUCT: {
        int16_t last = 0, id;
        uint8_t t;
        while (field(last, id, t)) skip(t, depth - 1);
        return;
      }
      default:  // STOP / unknown: "Unknown data type"
        fail();
    }
  }
  uint8_t fail() {
    ok_ = false;
    p_ = end_;
    return 0;
  }

 private:
  const uint8_t* p_;
  const uint8_t* begin_;
  const uint8_t* end_;
  bool ok_ = true;
  bool bool_pending_ = false;
  bool bool_value_ = false;
};

// ------------------------------------------------------------------------------------------------
// Typed struct reader: the generated Go readers of the reference (parquet/parquet.go) as data
// (thrift_spec.h).  A field whose id and wire type match the struct's spec is read (a later
// occurrence replaces an earlier one), any other field is skipped; a required field that was never
// read fails the struct.  List elements are read with the element reader of the spec whatever
// element type the list header names (the generated ReadFieldN loops).
// ------------------------------------------------------------------------------------------------
struct TNode {
  int64_t i = 0;                 // bool / byte / i16 / i32 / i64
  double d = 0;
  std::string s;                 // binary / string
  std::vector<TNode> items;      // list elements
  std::vector<std::pair<int16_t, TNode>> fields;  // struct fields that were read
  const TNode* get(int16_t id) const {
    for (const auto& f : fields)
      if (f.first == id) return &f.second;
    return nullptr;
  }
  int64_t get_i(int16_t id, int64_t dflt = 0) const {
    const TNode* n = get(id);
    return n ? n->i : dflt;
  }
};

bool read_typed(TReader& r, int16_t sid, TNode& out);

inline bool read_elem(TReader& r, uint8_t type, int16_t sub, TNode& v) {
  switch (type) {
    case T_BOOL_TRUE: v.i = r.read_bool(); break;
    case T_BYTE: v.i = int8_t(r.byte()); break;
    case T_I16: v.i = r.i16(); break;
    case T_I32: v.i = r.i32(); break;
    case T_I64: v.i = r.i64(); break;
    case T_DOUBLE: v.d = r.dbl(); break;
    case T_BINARY: r.str(v.s); break;
    case T_STRUCT: return read_typed(r, sub, v);
    default: r.fail();
  }
  return r.ok();
}

inline bool read_typed(TReader& r, int16_t sid, TNode& out) {
  const TStructSpec& S = kTStructs[sid];
  int16_t last = 0, id;
  uint8_t t;
  out.fields.clear();
  while (r.field(last, id, t)) {
    const TFieldSpec* f = nullptr;
    for (int k = 0; k < S.count; k++)
      if (kTFields[S.first + k].id == id) f = &kTFields[S.first + k];
    if (!f || f->type != t) {
      r.skip(t);
      if (!r.ok()) return false;
      continue;
    }
    TNode v;
    if (f->type == T_LIST) {
      uint8_t et;
      int32_t n;
      if (!r.list(et, n)) return false;
      for (int32_t i = 0; i < n; i++) {
        v.items.emplace_back();
        if (!read_elem(r, f->elem, f->sub, v.items.back())) return false;
      }
    } else if (!read_elem(r, f->type, f->sub, v)) {
      return false;
    }
    bool replaced = false;
    for (auto& e : out.fields)
      if (e.first == id) {
        e.second = std::move(v);
        replaced = true;
        break;
      }
    if (!replaced) out.fields.emplace_back(id, std::move(v));
  }
  if (!r.ok()) return false;
  for (int k = 0; k < S.count; k++)  // required fields ("Required field X is not set")
    if (kTFields[S.first + k].required && !out.get(kTFields[S.first + k].id)) {
      r.fail();
      return false;
    }
  return true;
}

// ------------------------------------------------------------------------------------------------
// Writer (used by the file generator that mirrors the reference writer).
// ------------------------------------------------------------------------------------------------
class TWriter {
 public:
  explicit TWriter(std::vector<uint8_t>& out) : out_(out) {}
  void uvarint(uint64_t v) {
    while (v >= 0x80) {
      out_.push_back(uint8_t(v | 0x80));
      v >>= 7;
    }
    out_.push_back(uint8_t(v));
  }
  void zigzag(int64_t v) { uvarint((uint64_t(v) << 1) ^ uint64_t(v >> 63)); }
  void field(int16_t id, uint8_t type) {
    int d = id - last_;
    if (d > 0 && d <= 15) {
      out_.push_back(uint8_t((d << 4) | type));
    } else {
      out_.push_back(type);
      zigzag(id);
    }
    last_ = id;
  }
  void i32(int16_t id, int32_t v) {
    field(id, T_I32);
    zigzag(v);
  }
  void i64(int16_t id, int64_t v) {
    field(id, T_I64);
    zigzag(v);
  }
  void boolean(int16_t id, bool v) { field(id, v ? T_BOOL_TRUE : T_BOOL_FALSE); }
  void binary(int16_t id, const std::string& s) {
    field(id, T_BINARY);
    uvarint(s.size());
    out_.insert(out_.end(), s.begin(), s.end());
  }
  void begin_struct(int16_t id) {
    field(id, T_STRUCT);
    stack_.push_back(last_);
    last_ = 0;
  }
  void end_struct() {
    out_.push_back(T_STOP);
    last_ = stack_.back();
    stack_.pop_back();
  }
  void begin_list(int16_t id, uint8_t etype, uint32_t n) {
    field(id, T_LIST);
    if (n < 15) {
      out_.push_back(uint8_t((n << 4) | etype));
    } else {
      out_.push_back(uint8_t(0xf0 | etype));
      uvarint(n);
    }
  }
  // Struct element inside a list.
  void begin_elem() {
    stack_.push_back(last_);
    last_ = 0;
  }
  void end_elem() { end_struct(); }
  void list_elem_i32(int32_t v) { zigzag(v); }
  void list_elem_binary(const std::string& s) {
    uvarint(s.size());
    out_.insert(out_.end(), s.begin(), s.end());
  }
  void stop() { out_.push_back(T_STOP); }

 private:
  std::vector<uint8_t>& out_;
  int16_t last_ = 0;
  std::vector<int16_t> stack_;
};

}  // namespace pqhip
