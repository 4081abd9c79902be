// internal.h — host structures shared by the C-ABI implementation files.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "pqhip.h"

struct pqh_host_batch {
  std::vector<pqh_chunk> chunks;
  std::vector<pqh_page> pages;
  // page images (or device-codec source bytes), 64-byte aligned, PQH_PAYLOAD_PAD zero bytes at the
  // end: plain host memory, or (pqh_file_load_pinned) a block of the context's pinned pool, shared
  // with the staged batches created from it and returned to the pool when the last holder lets go
  std::shared_ptr<uint8_t> buf;
  size_t buf_size = 0;           // pad included
  bool pinned = false;
  int64_t payload_bytes = 0;     // without the pad
  const uint8_t* data() const { return buf.get(); }
  size_t size() const { return buf_size; }
  double decompress_seconds = 0;
  // device codecs (PQH_LOAD_DEVICE_SNAPPY): payload holds the SOURCE bytes of every page, and
  // codec_pages[i] rebuilds page i's image at pages[i].image_offset of an image buffer of
  // image_bytes (+ PQH_PAYLOAD_PAD)
  std::vector<pqh_codec_page> codec_pages;
  int64_t image_bytes = 0;
};

namespace pqhip {
// A block of at least `bytes` pinned host memory from the context's pool (nullptr on failure); the
// block goes back to the pool when the returned pointer's last holder releases it.
std::shared_ptr<uint8_t> pinned_acquire(pqh_ctx* ctx, size_t bytes);

// getValuesDecoder (chunk_reader.go:106-159) resolved to a kernel kind; value bytes per output value.
int32_t resolve_kind(int32_t physical_type, int32_t type_length, int32_t encoding, int32_t* value_size);
}  // namespace pqhip
