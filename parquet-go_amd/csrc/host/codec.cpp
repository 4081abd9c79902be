// codec.cpp — see codec.h.
#include "codec.h"

#include <zlib.h>

#include <algorithm>
#include <cstring>

namespace pqhip {

// encoding/binary.Uvarint as golang/snappy's decodedLen calls it (vendor/github.com/golang/snappy/
// decode.go:32-36): at most 10 bytes, and the 10th byte (bits 63..69) may only be 0 or 1 -- any
// larger value overflows 64 bits and is an error (n < 0), never a silently truncated length.
static bool read_uvarint(const uint8_t*& p, const uint8_t* end, uint64_t& v) {
  v = 0;
  for (int i = 0; i < 10 && p < end; i++) {
    const uint8_t b = *p++;
    if (b < 0x80) {
      if (i == 9 && b > 1) return false;  // overflow
      v |= uint64_t(b) << (7 * i);
      return true;
    }
    v |= uint64_t(b & 0x7f) << (7 * i);
  }
  return false;  // 10 continuation bytes (overflow) or the input ended (n == 0)
}

// Snappy block decoding (format of golang/snappy decode.go): uvarint length, then literal /
// copy elements.  Every copy must reference already produced bytes and stay inside the length.
bool snappy_decompress(const uint8_t* src, size_t n, std::vector<uint8_t>& dst) {
  const uint8_t* p = src;
  const uint8_t* end = src + n;
  uint64_t len;
  if (!read_uvarint(p, end, len)) return false;
  if (len > (uint64_t(1) << 32) - 1) return false;
  dst.resize(size_t(len));
  uint8_t* out = dst.data();
  size_t d = 0;
  while (p < end) {
    uint8_t tag = *p++;
    size_t length, offset;
    switch (tag & 3) {
      case 0: {
        size_t x = tag >> 2;
        if (x >= 60) {
          int k = int(x) - 59;
          if (end - p < k) return false;
          x = 0;
          for (int i = 0; i < k; i++) x |= size_t(p[i]) << (8 * i);
          p += k;
        }
        length = x + 1;
        if (size_t(end - p) < length || len - d < length) return false;
        memcpy(out + d, p, length);
        p += length;
        d += length;
        continue;
      }
      case 1:
        if (end - p < 1) return false;
        length = 4 + ((tag >> 2) & 7);
        offset = (size_t(tag >> 5) << 8) | p[0];
        p += 1;
        break;
      case 2:
        if (end - p < 2) return false;
        length = 1 + (tag >> 2);
        offset = size_t(p[0]) | (size_t(p[1]) << 8);
        p += 2;
        break;
      default:
        if (end - p < 4) return false;
        length = 1 + (tag >> 2);
        offset = size_t(p[0]) | (size_t(p[1]) << 8) | (size_t(p[2]) << 16) | (size_t(p[3]) << 24);
        p += 4;
        break;
    }
    if (offset == 0 || offset > d || len - d < length) return false;
    for (size_t i = 0; i < length; i++) out[d + i] = out[d + i - offset];  // overlap-safe forward copy
    d += length;
  }
  return d == len;
}

static inline uint32_t load32(const uint8_t* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}

static void emit_literal(std::vector<uint8_t>& o, const uint8_t* p, size_t n) {
  if (n == 0) return;
  size_t x = n - 1;
  if (x < 60) {
    o.push_back(uint8_t(x << 2));
  } else {
    int k = x < (1u << 8) ? 1 : x < (1u << 16) ? 2 : x < (1u << 24) ? 3 : 4;
    o.push_back(uint8_t((59 + k) << 2));
    for (int i = 0; i < k; i++) o.push_back(uint8_t(x >> (8 * i)));
  }
  o.insert(o.end(), p, p + n);
}

static void emit_copy(std::vector<uint8_t>& o, size_t offset, size_t len) {
  while (len > 0) {
    size_t l = len;
    if (l > 64) l = (len - 64 < 4) ? 60 : 64;
    o.push_back(uint8_t(((l - 1) << 2) | 2));
    o.push_back(uint8_t(offset));
    o.push_back(uint8_t(offset >> 8));
    len -= l;
  }
}

// Greedy single-probe hash matcher over 64 KiB fragments, emitting snappy block format.
void snappy_compress(const uint8_t* src, size_t n, std::vector<uint8_t>& dst) {
  dst.clear();
  uint64_t v = n;
  while (v >= 0x80) {
    dst.push_back(uint8_t(v | 0x80));
    v >>= 7;
  }
  dst.push_back(uint8_t(v));
  std::vector<int32_t> table(1 << 14);
  for (size_t start = 0; start < n; start += 65536) {
    size_t end = start + 65536 < n ? start + 65536 : n;
    std::fill(table.begin(), table.end(), -1);
    size_t ip = start, lit = start;
    while (ip + 4 <= end) {
      uint32_t cur = load32(src + ip);
      uint32_t h = (cur * 0x1e35a7bdu) >> 18;
      int32_t cand = table[h];
      table[h] = int32_t(ip - start);
      if (cand >= 0 && load32(src + start + cand) == cur) {
        size_t c = start + size_t(cand);
        size_t len = 4;
        while (ip + len < end && src[c + len] == src[ip + len]) len++;
        emit_literal(dst, src + lit, ip - lit);
        emit_copy(dst, ip - c, len);
        ip += len;
        lit = ip;
      } else {
        ip++;
      }
    }
    emit_literal(dst, src + lit, end - lit);
  }
}

// Go's compress/gzip member header (gunzip.go readHeader), from src[pos]: sets *body to the first
// DEFLATE byte.  False on ErrHeader or a short read.  Reserved flag bits are ignored, as in Go.
static bool gzip_header(const uint8_t* src, size_t n, size_t pos, size_t* body) {
  if (n - pos < 10) return false;
  const uint8_t* h = src + pos;
  if (h[0] != 0x1f || h[1] != 0x8b || h[2] != 8) return false;
  const uint8_t flg = h[3];
  size_t q = pos + 10;
  if (flg & 4) {  // FEXTRA
    if (n - q < 2) return false;
    const size_t xlen = size_t(src[q]) | (size_t(src[q + 1]) << 8);
    q += 2;
    if (n - q < xlen) return false;
    q += xlen;
  }
  for (int bit : {8, 16}) {  // FNAME, FCOMMENT: NUL-terminated within 512 bytes
    if (!(flg & bit)) continue;
    size_t i = 0;
    for (;; i++) {
      if (i >= 512 || q + i >= n) return false;
      if (src[q + i] == 0) break;
    }
    q += i + 1;
  }
  if (flg & 2) {  // FHCRC: the low 16 bits of the CRC-32 of the header so far
    if (n - q < 2) return false;
    const uint32_t c = uint32_t(crc32(0L, src + pos, uInt(q - pos)));
    if ((c & 0xffff) != (uint32_t(src[q]) | (uint32_t(src[q + 1]) << 8))) return false;
    q += 2;
  }
  *body = q;
  return true;
}

// Multistream gzip (gzip.NewReader + ReadAll, compress.go:64-77): header, raw DEFLATE (zlib), then
// the CRC-32 / ISIZE trailer, member after member until the input ends.  Output goes to
// out(pos, room) -> pointer with room bytes (nullptr: no more room is a failure).
template <class Out>
static bool gzip_members(const uint8_t* src, size_t n, size_t& pos, Out&& out) {
  size_t in = 0;
  bool first = true;
  while (first || in < n) {
    size_t body;
    if (!gzip_header(src, n, in, &body)) return false;
    z_stream s;
    memset(&s, 0, sizeof(s));
    if (inflateInit2(&s, -MAX_WBITS) != Z_OK) return false;
    s.next_in = const_cast<Bytef*>(src + body);
    s.avail_in = uInt(n - body);
    const size_t ms = pos;
    uLong crc = crc32(0L, Z_NULL, 0);
    int rc;
    do {
      size_t room = 0;
      uint8_t* o = out(pos, room);
      if (!o) {
        inflateEnd(&s);
        return false;
      }
      s.next_out = o;
      s.avail_out = uInt(room);
      rc = inflate(&s, Z_NO_FLUSH);
      const size_t produced = room - s.avail_out;
      crc = crc32(crc, o, uInt(produced));
      pos += produced;
      if (rc != Z_OK && rc != Z_STREAM_END && !(rc == Z_BUF_ERROR && s.avail_out == 0)) {
        inflateEnd(&s);
        return false;
      }
    } while (rc != Z_STREAM_END);
    const size_t t = n - s.avail_in;
    inflateEnd(&s);
    if (n - t < 8) return false;  // trailer: ErrUnexpectedEOF
    const uint8_t* tr = src + t;
    const uint32_t want_crc = uint32_t(tr[0]) | (uint32_t(tr[1]) << 8) | (uint32_t(tr[2]) << 16) | (uint32_t(tr[3]) << 24);
    const uint32_t want_len = uint32_t(tr[4]) | (uint32_t(tr[5]) << 8) | (uint32_t(tr[6]) << 16) | (uint32_t(tr[7]) << 24);
    if (uint32_t(crc) != want_crc || uint32_t(pos - ms) != want_len) return false;  // ErrChecksum
    in = t + 8;
    first = false;
  }
  return true;
}

bool gzip_decompress(const uint8_t* src, size_t n, size_t expected, std::vector<uint8_t>& dst) {
  dst.clear();
  dst.resize(expected > 0 ? expected : 64);
  size_t pos = 0;
  const bool ok = gzip_members(src, n, pos, [&](size_t at, size_t& room) -> uint8_t* {
    if (at == dst.size()) dst.resize(dst.size() * 2);
    room = std::min<size_t>(dst.size() - at, size_t(1) << 30);
    return dst.data() + at;
  });
  if (!ok) return false;
  dst.resize(pos);
  return true;
}

bool gzip_compress(const uint8_t* src, size_t n, std::vector<uint8_t>& dst) {
  z_stream s;
  memset(&s, 0, sizeof(s));
  if (deflateInit2(&s, Z_DEFAULT_COMPRESSION, Z_DEFLATED, 16 + MAX_WBITS, 8, Z_DEFAULT_STRATEGY) != Z_OK)
    return false;
  dst.resize(deflateBound(&s, uLong(n)) + 32);
  s.next_in = const_cast<Bytef*>(src);
  s.avail_in = uInt(n);
  s.next_out = dst.data();
  s.avail_out = uInt(dst.size());
  int rc = deflate(&s, Z_FINISH);
  size_t out = dst.size() - s.avail_out;
  deflateEnd(&s);
  if (rc != Z_STREAM_END) return false;
  dst.resize(out);
  return true;
}

// Snappy block straight into dst[expected]: fails unless it decodes to exactly `expected` bytes.
static bool snappy_into(const uint8_t* src, size_t n, uint8_t* out, size_t expected) {
  const uint8_t* p = src;
  const uint8_t* end = src + n;
  uint64_t len;
  if (!read_uvarint(p, end, len) || len > (uint64_t(1) << 32) - 1 || len != expected) return false;
  size_t d = 0;
  while (p < end) {
    const uint8_t tag = *p++;
    size_t length, offset;
    switch (tag & 3) {
      case 0: {
        size_t x = tag >> 2;
        if (x >= 60) {
          const int k = int(x) - 59;
          if (end - p < k) return false;
          x = 0;
          for (int i = 0; i < k; i++) x |= size_t(p[i]) << (8 * i);
          p += k;
        }
        length = x + 1;
        if (size_t(end - p) < length || len - d < length) return false;
        memcpy(out + d, p, length);
        p += length;
        d += length;
        continue;
      }
      case 1:
        if (end - p < 1) return false;
        length = 4 + ((tag >> 2) & 7);
        offset = (size_t(tag >> 5) << 8) | p[0];
        p += 1;
        break;
      case 2:
        if (end - p < 2) return false;
        length = 1 + (tag >> 2);
        offset = size_t(p[0]) | (size_t(p[1]) << 8);
        p += 2;
        break;
      default:
        if (end - p < 4) return false;
        length = 1 + (tag >> 2);
        offset = size_t(p[0]) | (size_t(p[1]) << 8) | (size_t(p[2]) << 16) | (size_t(p[3]) << 24);
        p += 4;
        break;
    }
    if (offset == 0 || offset > d || len - d < length) return false;
    if (offset >= length) {
      memcpy(out + d, out + d - offset, length);
    } else {
      for (size_t i = 0; i < length; i++) out[d + i] = out[d + i - offset];  // overlapping: forward copy
    }
    d += length;
  }
  return d == len;
}

// Multistream gzip straight into dst[expected]: fails on corrupt input or any other output size
// (more output than `expected` is decoded into a scratch buffer only to fail).
static bool gzip_into(const uint8_t* src, size_t n, uint8_t* dst, size_t expected) {
  size_t pos = 0;
  uint8_t scratch[64];
  const bool ok = gzip_members(src, n, pos, [&](size_t at, size_t& room) -> uint8_t* {
    if (at > expected) return nullptr;
    if (at == expected) {
      room = sizeof(scratch);
      return scratch;
    }
    room = std::min<size_t>(expected - at, size_t(1) << 30);
    return dst + at;
  });
  return ok && pos == expected;
}

bool decompress_into(int codec, const uint8_t* src, size_t n, uint8_t* dst, size_t expected) {
  switch (codec) {
    case 0:
      if (n != expected) return false;
      if (n) memcpy(dst, src, n);
      return true;
    case 1:
      return snappy_into(src, n, dst, expected);
    case 2:
      return gzip_into(src, n, dst, expected);
    default:
      return false;
  }
}

bool decompress_block(int codec, const uint8_t* src, size_t n, size_t expected, std::vector<uint8_t>& dst) {
  switch (codec) {
    case 0:
      dst.assign(src, src + n);
      return true;
    case 1:
      return snappy_decompress(src, n, dst);
    case 2:
      return gzip_decompress(src, n, expected, dst);
    default:
      return false;
  }
}

bool compress_block(int codec, const uint8_t* src, size_t n, std::vector<uint8_t>& dst) {
  switch (codec) {
    case 0:
      dst.assign(src, src + n);
      return true;
    case 1:
      snappy_compress(src, n, dst);
      return true;
    case 2:
      return gzip_compress(src, n, dst);
    default:
      return false;
  }
}

uint32_t crc32_ieee(const uint8_t* p, size_t n) { return uint32_t(crc32(0L, p, uInt(n))); }

}  // namespace pqhip
