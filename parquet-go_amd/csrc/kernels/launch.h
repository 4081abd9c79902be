// launch.h — host-callable launchers of the decode kernels (kernels/decode.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <vector>

#include "decode.h"
#include "pqhip.h"

namespace pqhip {

struct DevBatch {
  const PQH_G uint8_t* payload;
  const DevPage* pages;
  const DevChunk* chunks;
  PageState* states;
  Ckpt* ckpts;
  int32_t num_pages;
  int32_t num_chunks;
  DeltaState* dstates;   // per page (delta pages only are written)
  DeltaBlock* dblocks;
  uint64_t* dsums;       // per delta tile: sum, then (after k_delta_scan) the tile's base value
  int32_t* dcum;         // byte-array dictionary pages: cumulative entry bytes (num_values + 1 each)
  int64_t* basums;       // per byte-array tile: byte sum, then (after k_ba_scan) the tile's first offset
  int64_t* chunk_bytes;  // per chunk: total string bytes (k_ba_scan)
  const DevNest* nests;  // repeated chunks with nesting outputs
  int64_t* nsums;        // per nest tile: kNestFlags counts, then (after k_nest_scan) bases
  int64_t* basums2;      // DELTA_BYTE_ARRAY: per tile suffix-byte sum, then its first suffix byte
  uint32_t* bafuse;      // fused PLAIN chains: [0] window tickets, [1] fallback flag (zeroed per run)
  uint64_t* bawords;     // fused PLAIN chains: per window FINAL word (zeroed per run)
  DeltaSplit* dsplit;    // page mode: per page, k_delta_split's view of its first delta stream
  uint32_t* dticket;     // k_delta_split: window tickets (zeroed per run)
  uint64_t* dwords;      // k_delta_split: three look-back words per window (zeroed per run)
};

hipError_t launch_prologue(const DevBatch& b, bool wide, hipStream_t s);
// A small batch of required flat fixed-width columns in one launch (k_flat: a check per page,
// speculative tiles from their FlatTile records); flag set = decode again through the three kernels.
hipError_t launch_flat(const DevBatch& b, const FlatTile* tiles, int32_t ntiles, const int64_t* spec_base,
                       uint32_t* flag, size_t lds_bytes, hipStream_t s);
// pqh_hybrid_decode: walk (res[0] = first error key, res[1] = values before it) + unpack (G = group)
hipError_t launch_hybrid_raw(const uint8_t* stream, int64_t len, int32_t width, int64_t n, int group, Ckpt* ck,
                             uint64_t* res, uint32_t* out, hipStream_t s);
// Device codecs: one wave per page rebuilding its image from its (SNAPPY) source bytes.
hipError_t launch_snappy(const pqh_codec_page* pages, int32_t n, const uint8_t* src, uint8_t* dst, int32_t* status,
                         hipStream_t s);
// Device SNAPPY over many workgroups per page (snappy_mw.h): k_snap_spec (per 4 KiB window of a
// block) -> k_snap_stitch (per page) -> k_snap_emit (per 64 KiB of a page's output) -> k_snap_fixup
// (per page).  Plain-copy pages (codec 0) are copied unit by unit; GZIP pages are k_gzip's.
struct SnapPlan {
  int32_t n_pages = 0, n_win = 0, n_unit = 0, n_page_mode = 0;
  int32_t* page_win0 = nullptr;   // [n_pages + 1] first window of each page
  int32_t* page_unit0 = nullptr;  // [n_pages + 1] first unit of each page
  int32_t* page_mode = nullptr;   // [n_pages] 1: a barely compressible SNAPPY page, k_snappy's (one workgroup)
  int32_t* win_page = nullptr;    // [n_win]
  int32_t* unit_page = nullptr;   // [n_unit]
  int4* wspec = nullptr;          // [n_win] speculative window results (first element, exit, output, status)
  int2* wtrue = nullptr;          // [n_win] true entry, output base
  int32_t* uflag = nullptr;       // [n_unit] a copy reached before the unit (k_snap_fixup redoes it)
  int16_t* wseg = nullptr;        // [n_win * 1024] every walker segment's exact first element (window-relative)
};
// Host tables page_win0 | page_unit0 | page_mode | win_page | unit_page of a codec page list
// (device copy: bind).
std::vector<int32_t> snap_plan_tables(const pqh_codec_page* pages, int32_t n, int32_t* n_win, int32_t* n_unit,
                                      int32_t* n_page_mode);
void snap_plan_bind(SnapPlan& P, int32_t* tables, int4* wspec, int2* wtrue, int32_t* uflag, int16_t* wseg);
// part: -1 the whole pipeline, else one kernel of it (0 k_snappy for the page-mode pages, 1 k_snap_spec,
// 2 k_snap_stitch, 3 k_snap_emit, 4 k_snap_fixup), launched in that order (profiled runs time each)
hipError_t launch_snappy_mw(const pqh_codec_page* pages, const SnapPlan& P, const uint8_t* src, uint8_t* dst,
                            int32_t* status, hipStream_t s, int part = -1);
// GZIP pages of the same table (one workgroup per page; the other pages' workgroups exit at once).
hipError_t launch_gzip(const pqh_codec_page* pages, int32_t n, const uint8_t* src, uint8_t* dst, int32_t* status,
                       hipStream_t s);
hipError_t launch_scan(const DevBatch& b, hipStream_t s);
// Fused PLAIN byte-array chains (bytearray_impl.h k_ba_chain): one workgroup per window of wins
// (page-major), dispatched in `order`.
hipError_t launch_ba_chain(const DevBatch& b, const int2* wins, const int32_t* order, int32_t n, hipStream_t s);
// One launch for every data-parallel tile (levels, PLAIN copies, booleans, dictionaries staged in
// LDS, RLE booleans); lds_bytes = the largest LDS-staged dictionary of the batch.
hipError_t launch_expand(const DevBatch& b, const Tile* tiles, int32_t n, size_t lds_bytes, hipStream_t s);
// DELTA_BINARY_PACKED: speculative chain of the whole blocks, then the exact block walk (one wave
// per delta page each).
hipError_t launch_delta_spec(const DevBatch& b, const int32_t* delta_pages, int32_t n, hipStream_t s);
hipError_t launch_delta_walk(const DevBatch& b, const int32_t* delta_pages, int32_t n, hipStream_t s);
// Delta tiles: per-tile sums, per-page scan (seeded with the first value), expand.
hipError_t launch_delta_sum(const DevBatch& b, const Tile* tiles, int32_t n, hipStream_t s);
hipError_t launch_delta_scan(const DevBatch& b, const int32_t* delta_pages, int32_t n, hipStream_t s);
hipError_t launch_delta_expand(const DevBatch& b, const Tile* tiles, int32_t n, hipStream_t s);
// Page mode (many delta streams): init errors of the DELTA_BINARY_PACKED pages before the value
// scan; whole blocks chased and decoded in one workgroup per stream (before the exact walk).
hipError_t launch_delta_init(const DevBatch& b, const int32_t* delta_pages, int32_t n, hipStream_t s);
hipError_t launch_delta_fused(const DevBatch& b, const Tile* streams, int32_t n, int32_t n_lens, hipStream_t s);
// k_delta_split: windows wins[order[i]] = (page, window) by ticket; [0, n - n_lens) of DELTA /
// DELTA_BYTE_ARRAY prefix streams, [n - n_lens, n) of DELTA_LENGTH lengths (two launches)
hipError_t launch_delta_split(const DevBatch& b, const int2* wins, const int32_t* order, int32_t n, int32_t n_lens,
                              hipStream_t s);
// Many delta streams: one workgroup per (page, stream), its tiles in order with a running carry.
hipError_t launch_delta_page(const DevBatch& b, const Tile* streams, int32_t n, hipStream_t s);
// Byte arrays: PLAIN chains (one wave per page, data and dictionary pages), tile byte sums,
// per-chunk offset scan, offsets + byte copy.
// PLAIN chains: every window of every PLAIN page resolved from a guessed entry, windows stitched
// per page (wrong guesses resolved again), records emitted per window.
hipError_t launch_ba_wspec(const DevBatch& b, const int2* wins, int32_t n, BaWin* res, uint16_t* wrec,
                           hipStream_t s);
hipError_t launch_ba_wstitch(const DevBatch& b, const int32_t* ba_pages, const int2* pwin, int32_t n, BaWin* res,
                             uint16_t* wrec, hipStream_t s);
// list: {window, page} of the dictionary pages' windows (k_ba_wemit: cumulative offsets) and of the
// data pages' windows (k_ba_wcopy, after k_ba_scan: offsets + bytes of every record).
hipError_t launch_ba_wemit(const DevBatch& b, const int2* list, int32_t n, const BaWin* res, const uint16_t* wrec,
                           hipStream_t s);
hipError_t launch_ba_wcopy(const DevBatch& b, const int2* list, int32_t n, const BaWin* res, const uint16_t* wrec,
                           void* geo, hipStream_t s);  // geo: kWGeoBytes per window
hipError_t launch_ba_sum(const DevBatch& b, const Tile* tiles, const int32_t* list, int32_t n, bool dlba_pages,
                         hipStream_t s);
hipError_t launch_ba_scan(const DevBatch& b, const int32_t* ba_chunks, int32_t n, const Tile* tiles, hipStream_t s);
hipError_t launch_ba_expand(const DevBatch& b, const Tile* tiles, const int32_t* list, int32_t n_copy, int32_t n_gather,
                            hipStream_t s);
// DELTA_BYTE_ARRAY: every value's shared prefix copied from the suffixes of earlier values.
hipError_t launch_dba_prefix(const DevBatch& b, const Tile* tiles, int32_t n, hipStream_t s);
// Nesting (levels -> list offsets / presence / leaf validity): counts, per-chunk scan, write.
hipError_t launch_nest_count(const DevBatch& b, const Tile* tiles, int32_t n, hipStream_t s);
hipError_t launch_nest_scan(const DevBatch& b, int32_t num_nests, hipStream_t s);
hipError_t launch_nest_write(const DevBatch& b, const Tile* tiles, int32_t n, hipStream_t s);
// Delta pages outside the fast-path geometry (exact sequential decode, one wave per delta page).
hipError_t launch_delta_serial(const DevBatch& b, const int32_t* delta_pages, int32_t n, hipStream_t s);
// Dictionaries too large for LDS.
hipError_t launch_dict_global(const DevBatch& b, const Tile* tiles, int32_t n, hipStream_t s);

}  // namespace pqhip
