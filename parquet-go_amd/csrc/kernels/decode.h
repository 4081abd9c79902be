// decode.h — device-side tables shared by the host batch planner (host/batch.hip) and the HIP
// kernels (kernels/decode.hip).  All page bytes stay in one HBM payload buffer; these tables
// describe where each page image, stream and output lives.
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#define PQH_HD __host__ __device__
#else
#define PQH_HD
#endif

// Output buffers are HBM: in device code their pointers live in the global address space, so every
// access compiles to global_load / global_store (a flat access would also count against LDS waits).
#if defined(__HIP_DEVICE_COMPILE__) && defined(PQH_KERNELS_TU)
#define PQH_G __attribute__((address_space(1)))
#else
#define PQH_G
#endif

namespace pqhip {

// Value decoder kinds: getValuesDecoder (reference chunk_reader.go:106-159) resolved per page.
enum DecoderKind : int32_t {
  K_UNSUPPORTED = 0,
  K_PLAIN_FIXED = 1,  // int32/int64/float/double/FLBA(L>0): binary.Read / ReadFull(L)
  K_PLAIN_INT96 = 2,  // type_int96.go:21-39
  K_PLAIN_BOOL = 3,   // booleanPlainDecoder
  K_RLE_BOOL = 4,     // booleanRLEDecoder: u32 size + hybrid(1)
  K_DICT = 5,         // dictDecoder: width byte + hybrid indices + gather
  K_DELTA32 = 6,      // int32DeltaBPDecoder
  K_DELTA64 = 7,      // int64DeltaBPDecoder
  K_PLAIN_BA = 8,     // byteArrayPlainDecoder, variable length
  K_DLBA = 9,         // byteArrayDeltaLengthDecoder
  K_DBA = 10,         // byteArrayDeltaDecoder
  K_FLBA_NEGATIVE = 11,
  K_DICT_PAGE = 12    // dictionary page (dictPageReader + PLAIN values decoder)
};

// Tile sizes (values or level slots per work item).
constexpr int kBlock = 256;          // threads per workgroup
constexpr int kHybridTile = 8192;    // hybrid-driven tiles (levels, dictionary indices, RLE booleans)
constexpr int kCopyTileBytes = 65536;
constexpr int kBoolTile = 32768;     // PLAIN booleans: 256 threads x 16 bytes x 8 bits
constexpr int kDictLdsMax = 65536;   // dictionaries up to this size are staged in LDS
constexpr uint64_t kNoError = ~0ull;

// Error key: the reference stops at its FIRST error in decode order; the smallest key wins.
PQH_HD inline uint64_t err_key(int phase, int64_t index, int code) {
  uint64_t idx = index < 0 ? 0 : (uint64_t(index) > 0xffffffffffffull ? 0xffffffffffffull : uint64_t(index));
  return (uint64_t(phase) << 56) | (idx << 8) | uint64_t(code & 0xff);
}

struct DevPage {
  int64_t image_off;     // in payload
  int32_t image_len;
  int32_t page_type;     // 0 V1, 3 V2, 2 dictionary
  int32_t num_values;
  int32_t encoding;
  int32_t def_len, rep_len;
  int32_t chunk;
  int32_t kind;          // DecoderKind
  int32_t value_size;    // fixed value bytes (FLBA length etc.)
  int32_t dict_page;     // batch page index of the chunk's dictionary page, -1
  int64_t level_base;    // first level slot of the page in the chunk's level outputs
  int32_t ck_rep, ck_def, ck_val;  // checkpoint table offsets (entries), -1 if none
  int32_t ck_rep_n, ck_def_n, ck_val_n;
  uint64_t host_err;     // error key found by the host planner (header-level), kNoError if none
  int32_t dblk_base;     // DELTA_BINARY_PACKED: first DeltaBlock record, -1 if not a delta page
  int32_t dblk_cap;      // records available (pages of blockSize >= 128)
  int32_t dtile_base;    // first per-tile delta sum
  int32_t dtile_n;       // delta tiles of the page (kDeltaTile values each)
  int32_t aux_base;      // byte-array dictionary page: first entry of its dcum table
  int32_t batile_base;   // byte-array data page: first kBaTile tile sum (chunk-contiguous)
  int32_t batile_n;
  int32_t num_nulls;     // DataPageHeaderV2.num_nulls: k_flat's speculative notNull (checked), else 0
};

struct DevChunk {
  int32_t physical_type, type_length, max_def, max_rep;
  int32_t first_page, num_pages;
  int32_t value_size;    // output bytes per value, 0 = byte array
  int32_t dict_page;     // batch page index or -1
  PQH_G uint8_t* values;
  PQH_G int64_t* offsets;
  PQH_G uint8_t* bytes;
  PQH_G uint8_t* def_levels;
  PQH_G uint8_t* rep_levels;
  int64_t values_cap;    // values capacity (elements)
  int64_t bytes_cap;
  PQH_G int32_t* aux;    // byte arrays: per value slot, length (PLAIN / DELTA_LENGTH / suffix) or dictionary key
  PQH_G int32_t* aux2;   // DELTA_BYTE_ARRAY: per value slot, prefix length
  PQH_G uint8_t* value_nil;  // INT96 chunks that can hold the reference's nil values (a PLAIN page, or a
                             // dictionary whose last entry is short): 1 per nil dense value, else NULL;
                             // zeroed at plan time, only nil slots are ever written (type_int96.go:21-42)
  int32_t batile_base;   // the chunk's byte-array tiles [batile_base, batile_base + batile_n)
  int32_t batile_n;
  int32_t ba_fused;      // PLAIN byte-array data pages only: byte bases guessed by k_scan, k_ba_chain
  int32_t dict_nil;      // the INT96 dictionary's last entry is nil (its page's last value is short)
};

// Written by the prologue (one wave per page) and the scan kernel.  64 bytes.
struct PageState {
  unsigned long long err;  // min err_key, kNoError if none
  int32_t nn;              // not-null count
  int16_t width;           // bit width of the value hybrid stream (dictionary / RLE boolean)
  int16_t ba_summed;       // byte-array data page: its kBaTile byte sums were accumulated by the
                           // length producers (k_ba_wemit / k_delta_page), so k_ba_sum skips it
  int32_t rep_s, rep_e;    // byte ranges in the image; s < 0 = uninitialised decoder
  int32_t def_s, def_e;
  int32_t val_s, val_e;    // values section / value hybrid stream
  int32_t val_limit;       // values before the first phase-3 stream error (== nn if none)
  int32_t dict_n;          // dictionary pages: entries decoded
  int64_t value_base;      // first value of the page in the chunk's dense values
  int64_t byte_base;       // byte arrays: first byte
};

static_assert(sizeof(PageState) == 64, "PageState is one 64-byte record");

// DELTA_BINARY_PACKED (deltabp_decoder.go): per page, written by k_delta_walk.
enum DeltaMode : int32_t { DM_NONE = 0, DM_FAST = 1, DM_SERIAL = 2 };

struct DeltaState {
  int32_t mode;           // DeltaMode
  int32_t block_size;
  int32_t mb_count;
  int32_t mbvc;           // values per miniblock
  int32_t nblocks;        // records written
  int32_t limit;          // values decodable before the first error (<= notNull)
  uint64_t first;         // first value (bits; int32 pages sign-extended)
  int64_t end_pos;        // reader position (image offset) after the walk
  int32_t rec_base;       // first DeltaBlock of this stream within the page's records
  int32_t head_blocks;    // blocks [0, head_blocks) already decoded by k_delta_fused (no records)
  uint64_t head_carry;    // value at position head_blocks * block_size (bits)
  int64_t head_neg;       // DELTA_LENGTH: first negative length among the head blocks (INT64_MAX: none)
};
// k_delta_split: window w of a page's delta stream owns the blocks whose header lies in
// [h0 + w * kSplitStride, h0 + (w + 1) * kSplitStride)
constexpr int kSplitStride = 12288;

// k_delta_split's view of a delta page's first stream (written by k_delta_init, page mode).
struct DeltaSplit {
  int64_t h0;      // image offset of block 0's header
  int64_t e;       // end of the values section (the stream's bytes end at or before it)
  int64_t vcap;    // positions the head emits
  int64_t lim;     // DELTA_LENGTH: positions whose lengths count in the byte-array tile sums
  uint64_t first;  // first value (bits)
  int32_t R;       // blocks of the head: whole blocks [0, R); 0 = not on the split path
  int32_t bs, mbc, mbvc;
};
static_assert(sizeof(DeltaSplit) == 56, "DeltaSplit layout");

// DELTA_BYTE_ARRAY pages carry two length streams: prefix lengths (state at dstates[page]) and the
// DELTA_LENGTH suffix lengths that follow (state at dstates[num_pages + page]).

// One block: data of miniblock m starts at data_off + sum_{j<m} mbvc/8*w_j.  Records of the
// speculative walk (pad == 1) carry only hdr_off: their consumers parse the header.
struct DeltaBlock {
  uint64_t min_delta;
  int32_t data_off;       // image offset of the first miniblock's data
  int32_t hdr_off;        // image offset of the block's header (varint minDelta)
  uint64_t widths;        // miniblock bit widths, 8 bits each (mb_count <= 8 on the fast path)
  uint64_t pad;
};

constexpr int kDeltaTile = 8192;     // values per delta tile (block size must divide 2048)
constexpr int kDeltaBlockMin = 128;  // record capacity assumes blocks of >= 128 values

// Run checkpoint at a tile boundary: the run that contains the tile's first value.
struct Ckpt {
  int32_t run_start;  // value index where the run starts
  int32_t run_len;    // values in the run (clamped to 2^31-1)
  int32_t data;       // bit-packed: byte offset of the run's first group in the image; RLE: value
  int32_t next_hdr;   // byte offset of the next run header (clamped); bit 31 = bit-packed run
};

enum TileKind : int32_t {
  TK_LEVELS = 0,
  TK_COPY = 1,
  TK_BOOL = 2,
  TK_DICT = 3,
  TK_RLE_BOOL = 4,
  TK_DICT_GLOBAL = 5,
  TK_DELTA = 6,         // kDeltaTile values of a DM_FAST delta page
  TK_DELTA_SERIAL = 7,  // a whole DM_SERIAL delta page (exact sequential decoder)
  TK_BA = 8             // kBaTile values of a byte-array data page (k_ba_sum / k_ba_expand)
};

constexpr int kBaTile = 2048;  // byte-array values per tile (one 256 x 8 block scan)

// PLAIN byte-array chains (k_ba_wspec / k_ba_wstitch / k_ba_wemit): windows of 256 segments.
#ifndef PQH_CHAIN_SEG
#define PQH_CHAIN_SEG 124
#endif
constexpr int kChainSeg = PQH_CHAIN_SEG;
constexpr int kChainWin = kChainSeg * kBlock;      // 31744 bytes per window (4 workgroups per CU)
constexpr int kChainWords = (kChainSeg + 63) / 64; // mask words per segment
constexpr int kChainStride = kChainWin - 16;       // window bases: the window staged from a 16-aligned
                                                   // entry >= B_w still covers [entry, B_w+1)
constexpr int kChainRecs = kChainWin / 4 + 2;
constexpr int kWGeoBytes = 64;  // k_ba_wcopy: one window's geometry record      // scratch entries per window (records >= 4 bytes)

// Scratch per window (k_ba_wspec -> k_ba_wstitch -> k_ba_wemit).
struct BaWin {
  int32_t entry;   // the entry the window was resolved from (-1: nothing to do)
  int32_t exit;    // first record start >= B_w+1, or where the chain ended
  int32_t count;   // records on the chain in the window before the first invalid one
  int32_t bad;     // error code of the first invalid record (0: none in the window)
  int64_t bytes;   // byte sum of those records' lengths (dictionary pages)
  int64_t base;    // k_ba_wstitch: records before the window (-1: not emitted)
  int64_t cbase;   // k_ba_wstitch: bytes before the window
  int64_t pad;
};


// Nesting outputs of a repeated chunk (pqh_batch_nesting): list offsets / presence per repetition
// level and leaf validity, from the chunk's decoded level bytes.  A DevNest covers a window of at
// most kMaxNest consecutive levels (lbase + 1 .. lbase + levels); a chunk nested deeper than that has
// one DevNest per window (PQH_MAX_NEST levels in all), each reading the levels once more.
constexpr int kMaxNest = 8;
constexpr int kNestTile = 8192;  // level slots per tile (256 threads x 32)
constexpr int kNestFlags = kMaxNest + 1;  // rows (r == 0) and element starts of levels 1..L

struct DevNest {
  int32_t chunk;
  int32_t levels;        // levels of this window (1..kMaxNest)
  int32_t max_def;
  int32_t tile_base;     // tiles [tile_base, tile_base + tile_n) of the k_nest_* work list
  int32_t tile_n;
  int32_t lbase;         // the window's levels are lbase + 1 .. lbase + levels (0: from the rows)
  int64_t n;             // level slots of the chunk
  int32_t d0;            // definition level of level lbase's REPEATED node (0 when lbase == 0)
  int32_t leaf;          // the window ends at max_rep: it writes the leaf validity
  int32_t rep_def[kMaxNest];  // definition levels of levels lbase + 1 .. lbase + levels
  PQH_G int32_t* offsets[kMaxNest];
  PQH_G uint8_t* validity[kMaxNest];
  PQH_G uint8_t* leaf_valid;
  int64_t* totals;       // kNestFlags per chunk: rows, elements of each level (k_nest_scan)
};

// Work item of k_expand.  Hybrid-driven kinds cover [k, k+span) checkpoint intervals of
// kHybridTile values; TK_COPY covers kCopyTileBytes bytes; TK_BOOL covers kBoolTile values.
struct Tile {
  int32_t page;
  int32_t k;
  int32_t kind;
  int32_t span;
};

// k_flat's tile: the tile and its page's fields, so that loading it is the tile's last dependent
// load before the page bytes.
struct FlatTile {
  int64_t image_off;       // the page image in the payload
  int64_t dict_off;        // its dictionary page's image, -1 if none (or the header failed)
  int64_t value_base;      // speculative: num_values of the chunk's earlier data pages
  PQH_G uint8_t* values;   // the chunk's values
  int32_t image_len, num_values, page_type, kind;
  int32_t value_size, rep_len, def_len, dict_n;  // dict_n: the dictionary page's num_values
  int32_t dict_len, k, span, tkind;
  uint64_t host_err;
  PQH_G uint8_t* def_out;  // nullable flat chunks (max_def 1, V2 pages): the page's definition levels
  int32_t num_nulls, max_def;
};

constexpr int kLevelSpan = 4;  // 32768 level slots per tile
constexpr int kDictSpan = 2;  // 16384 values per tile (8192 / 32768 / 65536 measured slower on C1)

}  // namespace pqhip
