// internal.h — host structures shared by the C-ABI implementation files.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "pqhip.h"

struct pqh_host_batch {
  std::vector<pqh_chunk> chunks;
  std::vector<pqh_page> pages;
  std::vector<uint8_t> payload;  // page images, 8-byte aligned, PQH_PAYLOAD_PAD zero bytes at the end
  int64_t payload_bytes = 0;     // without the pad
  double decompress_seconds = 0;
  // device codecs (PQH_LOAD_DEVICE_SNAPPY): payload holds the SOURCE bytes of every page, and
  // codec_pages[i] rebuilds page i's image at pages[i].image_offset of an image buffer of
  // image_bytes (+ PQH_PAYLOAD_PAD)
  std::vector<pqh_codec_page> codec_pages;
  int64_t image_bytes = 0;
};

namespace pqhip {
// getValuesDecoder (chunk_reader.go:106-159) resolved to a kernel kind; value bytes per output value.
int32_t resolve_kind(int32_t physical_type, int32_t type_length, int32_t encoding, int32_t* value_size);
}  // namespace pqhip
