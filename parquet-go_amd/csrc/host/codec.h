// codec.h — host block codecs of the page walker (reference compress.go:16-187).
//   UNCOMPRESSED: identity (plainCompressor)
//   SNAPPY:       block format of github.com/golang/snappy v0.0.4 (snappy.Decode / snappy.Encode,
//                 compress.go:43-49) — hand-written, no snappy library in this image
//   GZIP:         RFC 1952 via zlib (Go compress/gzip, compress.go:51-77)
#pragma once

#include <cstddef>
#include <cstdint>
#include <vector>

namespace pqhip {

// Decompress `src` with `codec` into dst (resized).  Returns false on corrupt input or an
// unsupported codec.  `expected` is the header's uncompressed size (a hint; the caller checks it).
bool decompress_block(int codec, const uint8_t* src, size_t n, size_t expected, std::vector<uint8_t>& dst);

// Decompress `src` with `codec` straight into dst[0, expected): true iff the block is valid and
// decodes to exactly `expected` bytes (readPageBlock + newBlockReader's size check).
bool decompress_into(int codec, const uint8_t* src, size_t n, uint8_t* dst, size_t expected);

bool snappy_decompress(const uint8_t* src, size_t n, std::vector<uint8_t>& dst);
void snappy_compress(const uint8_t* src, size_t n, std::vector<uint8_t>& dst);
bool gzip_decompress(const uint8_t* src, size_t n, size_t expected, std::vector<uint8_t>& dst);
bool gzip_compress(const uint8_t* src, size_t n, std::vector<uint8_t>& dst);
bool compress_block(int codec, const uint8_t* src, size_t n, std::vector<uint8_t>& dst);

uint32_t crc32_ieee(const uint8_t* p, size_t n);

}  // namespace pqhip
