// launch.h — host-callable launchers of the decode kernels (kernels/decode.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "decode.h"

namespace pqhip {

struct DevBatch {
  const uint8_t* payload;
  const DevPage* pages;
  const DevChunk* chunks;
  PageState* states;
  Ckpt* ckpts;
  int32_t num_pages;
  int32_t num_chunks;
};

hipError_t launch_prologue(const DevBatch& b, hipStream_t s);
hipError_t launch_scan(const DevBatch& b, hipStream_t s);
hipError_t launch_levels(const DevBatch& b, const Tile* tiles, int32_t n, hipStream_t s);
hipError_t launch_copy(const DevBatch& b, const Tile* tiles, int32_t n, hipStream_t s);
hipError_t launch_bool_plain(const DevBatch& b, const Tile* tiles, int32_t n, hipStream_t s);
// Hybrid-driven values: dictionary gathers (value_size 4, 8 or generic) and RLE booleans.
hipError_t launch_dict(const DevBatch& b, const Tile* tiles, int32_t n, int32_t value_size, bool lds,
                       size_t lds_bytes, hipStream_t s);
hipError_t launch_rle_bool(const DevBatch& b, const Tile* tiles, int32_t n, hipStream_t s);

}  // namespace pqhip
