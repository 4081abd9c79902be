// thrift_compact.h — minimal Thrift compact-protocol reader/writer for the Parquet footer and page
// headers (the structs of reference parquet/parquet.thrift:516-1056).  The reference reads them
// through the generated apache/thrift v0.16.0 code (helpers.go:103-109, parquet/parquet.go); here
// only the fields the decode path needs are interpreted and everything else is skipped.
#pragma once

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

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
// Reader: bounded, never reads past `end`; every error sets ok=false and further reads return 0.
// ------------------------------------------------------------------------------------------------
class TReader {
 public:
  TReader(const uint8_t* p, const uint8_t* end) : p_(p), begin_(p), end_(end) {}
  bool ok() const { return ok_; }
  size_t consumed() const { return size_t(p_ - begin_); }

  uint8_t byte() {
    if (!ok_ || p_ >= end_) return fail();
    return *p_++;
  }
  uint64_t uvarint() {
    uint64_t x = 0;
    for (int s = 0; s < 70; s += 7) {
      uint8_t b = byte();
      if (!ok_) return 0;
      x |= uint64_t(b & 0x7f) << s;
      if (b < 0x80) return x;
    }
    return fail();
  }
  int64_t zigzag() {
    uint64_t u = uvarint();
    return int64_t(u >> 1) ^ -int64_t(u & 1);
  }
  // Field header: returns false at STOP.  `last` is the previous field id of this struct.
  bool field(int16_t& last, int16_t& id, uint8_t& type) {
    uint8_t h = byte();
    if (!ok_ || h == 0) return false;
    type = h & 0x0f;
    uint8_t d = h >> 4;
    id = d ? int16_t(last + d) : int16_t(zigzag());
    last = id;
    return ok_;
  }
  int64_t integer(uint8_t type) {
    if (type == T_BYTE) return int8_t(byte());
    if (type == T_I16 || type == T_I32 || type == T_I64) return zigzag();
    skip(type);
    ok_ = false;
    return 0;
  }
  bool boolean(uint8_t type) { return type == T_BOOL_TRUE; }
  std::string binary() {
    uint64_t n = uvarint();
    if (!ok_ || n > uint64_t(end_ - p_)) {
      fail();
      return std::string();
    }
    std::string s(reinterpret_cast<const char*>(p_), size_t(n));
    p_ += n;
    return s;
  }
  // List header: element type + size.
  bool list(uint8_t& etype, uint32_t& n) {
    uint8_t h = byte();
    etype = h & 0x0f;
    n = h >> 4;
    if (n == 15) n = uint32_t(uvarint());
    return ok_;
  }
  void skip(uint8_t type, int depth = 0) {
    if (depth > 64) {
      fail();
      return;
    }
    switch (type) {
      case T_BOOL_TRUE:
      case T_BOOL_FALSE:
        return;
      case T_BYTE:
        byte();
        return;
      case T_I16:
      case T_I32:
      case T_I64:
        uvarint();
        return;
      case T_DOUBLE:
        if (end_ - p_ < 8) {
          fail();
          return;
        }
        p_ += 8;
        return;
      case T_BINARY: {
        uint64_t n = uvarint();
        if (n > uint64_t(end_ - p_)) {
          fail();
          return;
        }
        p_ += n;
        return;
      }
      case T_LIST:
      case T_SET: {
        uint8_t et;
        uint32_t n;
        list(et, n);
        for (uint32_t i = 0; i < n && ok_; i++) {
          if (et == T_BOOL_TRUE || et == T_BOOL_FALSE) byte();
          else skip(et, depth + 1);
        }
        return;
      }
      case T_MAP: {
        uint64_t n = uvarint();
        if (n == 0) return;
        uint8_t kv = byte();
        for (uint64_t i = 0; i < n && ok_; i++) {
          skip(kv >> 4, depth + 1);
          skip(kv & 0x0f, depth + 1);
        }
        return;
      }
      case T_STRUCT: {
        int16_t last = 0, id;
        uint8_t t;
        while (field(last, id, t)) skip(t, depth + 1);
        return;
      }
      default:
        fail();
    }
  }

 private:
  uint8_t fail() {
    ok_ = false;
    p_ = end_;
    return 0;
  }
  const uint8_t* p_;
  const uint8_t* begin_;
  const uint8_t* end_;
  bool ok_ = true;
};

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
