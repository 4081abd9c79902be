// batch.hip — C-ABI implementation of the device side (include/pqhip.h): contexts, memory, and the
// batch planner that replaces pageReader.read + readValues for every page of a set of chunks.
//
// Planning (host, once per batch): resolve each page's decoder (getValuesDecoder,
// chunk_reader.go:106-159), header-level errors, level/value output offsets, checkpoint storage and
// the tile lists of each kernel kind.  Running: one launch per kernel kind for the whole batch on
// the context stream (k_prologue -> k_scan -> k_levels / k_copy / k_bool_plain / k_dict /
// k_rle_bool), optionally bracketed by HIP events.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <memory>
#include <atomic>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../kernels/launch.h"
#include "internal.h"
#include "pqhip.h"

using namespace pqhip;

// Reusable pinned host blocks of a context (pqh_file_load_pinned payloads): a block returns to the
// pool when its last holder (host batch, staged batch) lets go, and is freed with the context (or
// on release, once the context is gone).
struct PinnedPool {
  std::mutex m;
  std::vector<std::pair<uint8_t*, size_t>> free_blocks;
  bool closed = false;
  std::atomic<int64_t> pinned{0};  // bytes pinned by the pool (blocks in use + free)
};

// Device memory of a streaming context (PQH_CTX_STREAMING): one arena, bump-allocated in plan order
// and reset when the context's last live allocation goes (a ring slot holds one batch at a time, so
// every range's batch lays its buffers out again from the bottom: no driver call per range, no
// stream-ordered pool whose cross-stream reuse the copy and side streams would have to be ordered
// against).  Each allocation is followed by a guard gap (PQH_ARENA_GUARD bytes, default 4 KiB);
// with PQH_ARENA_CHECK=1 the gaps hold a canary that pqh_batch_sync verifies, naming the allocation
// a kernel wrote past.
struct DevArena {
  struct Chunk {
    uint8_t* base;
    size_t cap, used;
  };
  struct Guard {
    uint8_t* p;
    size_t bytes, alloc_bytes;
    int32_t index;
  };
  std::mutex m;
  std::vector<Chunk> chunks;
  std::vector<Guard> guards;
  int64_t live = 0;    // allocations not yet freed
  int32_t allocs = 0;  // allocations since the last reset
  size_t want = 0;     // after the arena grew: the size of the one chunk that replaces its chunks
};

struct pqh_ctx {
  std::shared_ptr<PinnedPool> pool = std::make_shared<PinnedPool>();
  DevArena arena;
  int32_t device = 0;
  uint32_t flags = 0;
  hipStream_t stream = nullptr;
  hipStream_t copy_stream = nullptr;  // staged (end-to-end) runs: pinned -> HBM copies
  hipStream_t side = nullptr;         // unprofiled runs: branches beside the main launch sequence
  hipStream_t side2 = nullptr;        //   (the fused PLAIN chains, beside both)
  hipStream_t side3 = nullptr;        //   (the DELTA pages after the value scan, beside k_expand)
  std::string err;
  // Pinned bounce buffer for every copy between HBM and pageable host memory (two halves, so the
  // host-side memcpy of one overlaps the DMA of the other).  Pageable copies never reach the HIP
  // runtime: its on-the-fly pinning of pageable memory faulted ("illegal memory access") on a
  // device-to-host copy into a fresh numpy buffer after earlier large transfers in the process.
  uint8_t* bounce = nullptr;
  hipEvent_t bounce_ev[2] = {nullptr, nullptr};
};

namespace {

thread_local std::string g_err;

int set_err(pqh_ctx* ctx, int code, const std::string& m) {
  if (ctx) ctx->err = m;
  g_err = m;
  return code;
}

#define HIP_TRY(ctx, expr)                                                              \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess)                                                               \
      return set_err(ctx, PQH_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

struct KernelRun {
  int kind;  // index into kKernelNames
  hipEvent_t start, stop;
  int32_t items;
};

const char* kKernelNames[] = {"k_prologue", "k_scan", "k_expand", "k_dict_global",
                              "k_delta_walk", "k_delta_expand", "k_delta_sum_scan",
                              "k_ba_wspec",   "k_ba_sum",    "k_ba_scan",    "k_ba_expand",
                              "k_nest_count", "k_nest_scan", "k_nest_write", "k_delta_serial",
                              "k_dba_prefix", "k_delta_spec", "k_delta_page", "k_delta_init",
                              "k_delta_fused", "k_ba_wstitch", "k_ba_wemit",   "k_snappy",
                              "k_ba_wcopy",   "k_gzip",      "k_snap_spec",  "k_snap_stitch",
                              "k_snap_emit",  "k_snap_fixup", "k_ba_chain",   "k_flat",
                              "k_expand_lev", "k_delta_split"};
constexpr int kNumKernels = 33;
// Batches with at least this many delta streams decode each stream in one workgroup (k_delta_page);
// fewer streams go through per-tile sums, a page scan and per-tile expands (more parallelism).
constexpr size_t kDeltaPageModeMin = 256;

int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// PQH_SYNC_EACH=1 (debugging): direct launches, each followed by a stream synchronisation, so a
// kernel fault is reported against the kernel that caused it.
bool sync_each_enabled() {
  const char* f = getenv("PQH_SYNC_EACH");
  return f && f[0] == '1';
}
thread_local const char* g_fail_kernel = nullptr;
// set by pqh_batch_create_staged in a streaming context around pqh_batch_create: the plan tables are
// uploaded by pqh_batch_run_staged on the copy stream instead of synchronously (a slot's creation then
// never waits behind the other slots' payload copies on the DMA engines)
thread_local bool g_defer_tables = false;

// PQH_SNAPPY_PAGE=1 (A/B experiments): device SNAPPY by k_snappy, one workgroup per page, instead of
// the multi-workgroup pipeline (k_snap_spec / stitch / emit / fixup).
bool snappy_page_mode() {
  const char* f = getenv("PQH_SNAPPY_PAGE");
  return f && f[0] == '1';
}

// PQH_BA_FUSE=0 (A/B experiments, tests): PLAIN-only byte-array chunks take the scratch path
// (k_ba_wspec / wstitch / wcopy) instead of the fused k_ba_chain.
bool fuse_enabled() {
  const char* f = getenv("PQH_BA_FUSE");
  return !(f && f[0] == '0');
}

// PQH_DELTA_SPLIT=1 (opt-in, tests): page-mode delta heads by k_delta_split (12 KiB windows of a
// stream over many workgroups with a decoupled look-back) instead of k_delta_fused (one workgroup per
// stream).  Measured slower at every C3 shard size (59 us per window against 26 us per
// fused tile, 5 vs 8 workgroups per CU), so not the default.
bool split_enabled() {
  const char* f = getenv("PQH_DELTA_SPLIT");
  return f && f[0] == '1';
}

// PQH_NEST_EARLY=0 (A/B experiments, tests): one k_expand launch, the nesting kernels after it.
bool nest_early_enabled() {
  const char* f = getenv("PQH_NEST_EARLY");
  return !(f && f[0] == '0');
}

constexpr size_t kBounceHalf = size_t(16) << 20;

hipError_t bounce_init(pqh_ctx* ctx) {
  if (ctx->bounce) return hipSuccess;
  hipError_t e = hipHostMalloc(reinterpret_cast<void**>(&ctx->bounce), 2 * kBounceHalf, hipHostMallocDefault);
  for (int i = 0; i < 2 && e == hipSuccess; i++) e = hipEventCreateWithFlags(&ctx->bounce_ev[i], hipEventDisableTiming);
  return e;
}

// Pageable host -> device on the context stream; returns when the host buffer may be reused.
hipError_t bounce_h2d(pqh_ctx* ctx, void* dst, const void* src, size_t bytes) {
  hipError_t e = bounce_init(ctx);
  for (size_t off = 0, i = 0; off < bytes && e == hipSuccess; off += kBounceHalf, i++) {
    const size_t n = std::min(kBounceHalf, bytes - off);
    uint8_t* half = ctx->bounce + (i & 1) * kBounceHalf;
    if (i >= 2) e = hipEventSynchronize(ctx->bounce_ev[i & 1]);  // that half's previous copy is done
    if (e != hipSuccess) break;
    memcpy(half, static_cast<const uint8_t*>(src) + off, n);
    e = hipMemcpyAsync(static_cast<uint8_t*>(dst) + off, half, n, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess) e = hipEventRecord(ctx->bounce_ev[i & 1], ctx->stream);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  return e;
}

// Device -> pageable host, ordered after the work already on the context stream; synchronous.
hipError_t bounce_d2h(pqh_ctx* ctx, void* dst, const void* src, size_t bytes) {
  hipError_t e = bounce_init(ctx);
  const size_t nchunks = (bytes + kBounceHalf - 1) / kBounceHalf;
  auto issue = [&](size_t i) {
    const size_t off = i * kBounceHalf, n = std::min(kBounceHalf, bytes - off);
    hipError_t r = hipMemcpyAsync(ctx->bounce + (i & 1) * kBounceHalf, static_cast<const uint8_t*>(src) + off, n,
                                  hipMemcpyDeviceToHost, ctx->stream);
    return r == hipSuccess ? hipEventRecord(ctx->bounce_ev[i & 1], ctx->stream) : r;
  };
  if (e == hipSuccess && nchunks) e = issue(0);
  for (size_t i = 0; i < nchunks && e == hipSuccess; i++) {
    if (i + 1 < nchunks) e = issue(i + 1);  // the other half is free: its memcpy below finished
    if (e == hipSuccess) e = hipEventSynchronize(ctx->bounce_ev[i & 1]);
    if (e != hipSuccess) break;
    const size_t off = i * kBounceHalf;
    memcpy(static_cast<uint8_t*>(dst) + off, ctx->bounce + (i & 1) * kBounceHalf, std::min(kBounceHalf, bytes - off));
  }
  return e;
}

}  // namespace

namespace pqhip {

std::shared_ptr<uint8_t> pinned_acquire(pqh_ctx* ctx, size_t bytes) {
  std::shared_ptr<PinnedPool> pool = ctx->pool;
  uint8_t* p = nullptr;
  size_t cap = 0;
  std::vector<std::pair<uint8_t*, size_t>> drop;
  {
    std::lock_guard<std::mutex> g(pool->m);
    size_t best = SIZE_MAX;
    for (size_t i = 0; i < pool->free_blocks.size(); i++)  // the smallest free block that fits
      if (pool->free_blocks[i].second >= bytes && (best == SIZE_MAX || pool->free_blocks[i].second < pool->free_blocks[best].second))
        best = i;
    if (best != SIZE_MAX) {
      p = pool->free_blocks[best].first;
      cap = pool->free_blocks[best].second;
      pool->free_blocks.erase(pool->free_blocks.begin() + long(best));
    } else {
      // a miss: the free blocks are all too small for this request; release them rather than keep
      // them pinned for the context's life (payloads that keep growing would pile up otherwise)
      drop.swap(pool->free_blocks);
    }
  }
  if (!drop.empty()) hipSetDevice(ctx->device);
  for (auto& fb : drop) {
    hipHostFree(fb.first);
    pool->pinned -= int64_t(fb.second);
  }
  if (!p) {
    // 2 MiB granules; a streaming context's ring reuses one block per slot for ranges of similar
    // but not equal sizes, so its blocks get 1/8 of headroom (and 64 MiB granules past 512 MiB)
    // instead of being re-pinned whenever a range is a little larger than the last
    const bool ring = (ctx->flags & PQH_CTX_STREAMING) != 0;
    const size_t g = ring && bytes > (size_t(512) << 20) ? size_t(64) << 20 : size_t(2) << 20;
    const size_t want = ring ? bytes + bytes / 8 : bytes;
    cap = (std::max<size_t>(want, 1) + g - 1) & ~(g - 1);
    hipSetDevice(ctx->device);
    void* q = nullptr;
    if (hipHostMalloc(&q, cap, hipHostMallocDefault) != hipSuccess) return nullptr;
    p = static_cast<uint8_t*>(q);
    pool->pinned += int64_t(cap);
  }
  return std::shared_ptr<uint8_t>(p, [pool, cap](uint8_t* q) {
    std::lock_guard<std::mutex> g(pool->m);
    if (pool->closed) {
      hipHostFree(q);
      pool->pinned -= int64_t(cap);
    } else {
      pool->free_blocks.emplace_back(q, cap);
    }
  });
}

int32_t resolve_kind(int32_t type, int32_t type_length, int32_t enc, int32_t* vs) {
  if (enc == PQH_ENC_PLAIN_DICTIONARY) enc = PQH_ENC_RLE_DICTIONARY;
  int32_t size = 0;
  switch (type) {
    case PQH_BOOLEAN: size = 1; break;
    case PQH_INT32: case PQH_FLOAT: size = 4; break;
    case PQH_INT64: case PQH_DOUBLE: size = 8; break;
    case PQH_INT96: size = 12; break;
    case PQH_FIXED_LEN_BYTE_ARRAY: size = type_length > 0 ? type_length : 0; break;
    default: size = 0;
  }
  *vs = size;
  switch (type) {
    case PQH_BOOLEAN:
      if (enc == PQH_ENC_PLAIN) return K_PLAIN_BOOL;
      if (enc == PQH_ENC_RLE) return K_RLE_BOOL;
      return K_UNSUPPORTED;
    case PQH_BYTE_ARRAY:
      if (enc == PQH_ENC_PLAIN) return K_PLAIN_BA;
      if (enc == PQH_ENC_DELTA_LENGTH_BYTE_ARRAY) return K_DLBA;
      if (enc == PQH_ENC_DELTA_BYTE_ARRAY) return K_DBA;
      if (enc == PQH_ENC_RLE_DICTIONARY) return K_DICT;
      return K_UNSUPPORTED;
    case PQH_FIXED_LEN_BYTE_ARRAY:
      if (enc == PQH_ENC_PLAIN) return type_length > 0 ? K_PLAIN_FIXED : type_length == 0 ? K_PLAIN_BA : K_FLBA_NEGATIVE;
      if (enc == PQH_ENC_DELTA_BYTE_ARRAY) {
        *vs = 0;
        return K_DBA;
      }
      if (enc == PQH_ENC_RLE_DICTIONARY) return K_DICT;
      return K_UNSUPPORTED;
    case PQH_FLOAT:
    case PQH_DOUBLE:
      if (enc == PQH_ENC_PLAIN) return K_PLAIN_FIXED;
      if (enc == PQH_ENC_RLE_DICTIONARY) return K_DICT;
      return K_UNSUPPORTED;
    case PQH_INT96:
      if (enc == PQH_ENC_PLAIN) return K_PLAIN_INT96;
      if (enc == PQH_ENC_RLE_DICTIONARY) return K_DICT;
      return K_UNSUPPORTED;
    case PQH_INT32:
    case PQH_INT64:
      if (enc == PQH_ENC_PLAIN) return K_PLAIN_FIXED;
      if (enc == PQH_ENC_DELTA_BINARY_PACKED) return type == PQH_INT32 ? K_DELTA32 : K_DELTA64;
      if (enc == PQH_ENC_RLE_DICTIONARY) return K_DICT;
      return K_UNSUPPORTED;
    default:
      return K_UNSUPPORTED;
  }
}

// Chunks output as offsets + bytes: BYTE_ARRAY, and FIXED_LEN_BYTE_ARRAY without a fixed output
// width (type_length <= 0, or DELTA_BYTE_ARRAY pages: the planner then sets value_size 0).
bool is_ba_chunk(const DevChunk& D) {
  return D.physical_type == PQH_BYTE_ARRAY || (D.physical_type == PQH_FIXED_LEN_BYTE_ARRAY && D.value_size == 0);
}

}  // namespace pqhip

struct pqh_batch {
  pqh_ctx* ctx = nullptr;
  std::vector<pqh_chunk> chunks;
  std::vector<pqh_page> pages;
  std::vector<DevPage> hpages;
  std::vector<DevChunk> hchunks;
  std::vector<Tile> expand_tiles;   // k_expand work list (kinds interleaved)
  int32_t expand_lev_n = 0;         // its first expand_lev_n tiles: the level tiles of the chunks with
                                    // nesting outputs, launched first (k_expand_lev) so that the
                                    // nesting kernels run beside the rest of k_expand
  std::vector<Tile> global_tiles;   // k_dict_global work list
  std::vector<Tile> delta_tiles;    // k_delta_sum work list (the TK_DELTA tiles)
  std::vector<Tile> delta_streams;  // k_delta_page work list: (page, 0, stream) with values
  bool delta_page_mode = false;
  int32_t delta_fused_pages = 0;    // page mode: delta pages / streams through k_delta_fused
  int32_t delta_fused_streams = 0;
  int32_t delta_lens_streams = 0;   // the last of delta_streams: DELTA_LENGTH_BYTE_ARRAY pages
  // k_delta_split (page mode): the windows of the streams k_delta_fused would take, page-major
  // (split_wins: (page, window)), and their window-major dispatch order (the DELTA_LENGTH windows'
  // order last, split_nl of them)
  bool split_on = false;
  std::vector<int2> split_wins;
  std::vector<int32_t> split_order;
  int32_t split_nl = 0;
  DeltaSplit* d_dsplit = nullptr;
  uint32_t* d_dticket = nullptr;
  uint64_t* d_dwords = nullptr;
  int2* d_split_wins = nullptr;
  int32_t* d_split_order = nullptr;
  std::vector<int32_t> delta_pages; // k_delta_walk / k_delta_scan work list
  std::vector<Tile> ba_tiles;       // k_ba_sum / k_ba_expand work list (chunk-contiguous)
  std::vector<int32_t> ba_xlist;    // ba_tiles indices: DELTA_LENGTH tiles, then PLAIN / dictionary, then k_ba_sum's
  int32_t ba_sum_off = 0;           // start of k_ba_sum's list in ba_xlist
  int32_t ba_ncopy = 0;             //   (the first ba_ncopy go to k_ba_expand, the rest to k_ba_gather)
  std::vector<int32_t> ba_pages;    // PLAIN byte-array data + dictionary pages (chain walks)
  std::vector<int2> ba_wins, ba_pwin;
  std::vector<int2> ba_wlist;       // {window, page}: dictionary pages' windows (k_ba_wemit), then data pages' (k_ba_wcopy)
  int32_t ba_wdict = 0;             // dictionary windows at the front of ba_wlist
  std::vector<int32_t> ba_chunks;   // k_ba_scan work list
  // Fused PLAIN chains (k_ba_chain): chunks with DevChunk.ba_fused sort last in ba_pages / ba_wins /
  // ba_chunks / the k_ba_sum list, so while ba_fuse_on the scratch path runs over the prefixes below
  // and k_ba_chain over ba_wins[ba_wins_nf:]; a fallback (bafuse[1]) turns it off for good
  bool ba_fuse_on = false;
  int32_t ba_pages_nf = 0, ba_wins_nf = 0, ba_wlist_nf = 0, ba_chunks_nf = 0, ba_sum_nf = 0;
  int32_t ba_fuse_fallbacks = 0;
  uint32_t* d_bafuse = nullptr;
  uint64_t* d_bawords = nullptr;
  std::vector<int32_t> ba_forder;   // k_ba_chain's dispatch order: fused windows by (window in page, page)
  int32_t* d_ba_forder = nullptr;
  std::vector<int64_t> chunk_bytes; // host copy after sync
  std::vector<DevNest> nests;       // repeated chunks with nesting outputs
  std::vector<int32_t> chunk_nest;  // chunk -> nests index, -1
  std::vector<Tile> nest_tiles;     // k_nest_count / k_nest_write work list
  std::vector<int64_t> nest_totals; // host copy after sync (kNestFlags per nest)
  size_t expand_lds = 0;            // dynamic LDS of k_expand: largest staged dictionary
  const uint8_t* d_payload = nullptr;
  void* owned_payload = nullptr;
  // device codecs: source payload (compressed pages) and the page table k_snappy rebuilds the
  // images (owned_payload) from at the start of every run
  void* d_src = nullptr;
  size_t src_bytes = 0;
  pqh_codec_page* d_codec = nullptr;
  int32_t codec_n = 0;
  int32_t codec_gzip = 0;  // GZIP pages among them (k_gzip)
  int32_t* d_codec_status = nullptr;
  std::vector<int32_t> codec_status;  // host copy after sync (per page)
  SnapPlan snap;                      // multi-workgroup SNAPPY tables and scratch (snappy_mw.h)
  int64_t payload_bytes = 0;
  void* h_staged = nullptr;           // staged batches: pinned host page images
  std::shared_ptr<uint8_t> h_pinned_ref;  // ... when they are a pinned host batch's payload (shared)
  size_t staged_bytes = 0;
  hipEvent_t ev_copied = nullptr, ev_done = nullptr;
  bool done_recorded = false;
  hipEvent_t ev_dep[10] = {};      // fork / join points of the side branches
  DevPage* d_pages = nullptr;
  DevChunk* d_chunks = nullptr;
  PageState* d_states = nullptr;
  Ckpt* d_ckpts = nullptr;
  Tile* d_tiles = nullptr;
  Tile* d_dtiles = nullptr;
  int32_t* d_delta_pages = nullptr;
  DeltaState* d_dstates = nullptr;
  DeltaBlock* d_dblocks = nullptr;
  uint64_t* d_dsums = nullptr;
  Tile* d_batiles = nullptr;
  int32_t* d_ba_xlist = nullptr;
  int32_t* d_ba_pages = nullptr;
  int2* d_ba_wins = nullptr;        // (page, window) of every PLAIN chain window
  int2* d_ba_pwin = nullptr;        // per PLAIN page: (first window, windows)
  int2* d_ba_wlist = nullptr;
  BaWin* d_ba_res = nullptr;
  uint16_t* d_ba_wrec = nullptr;     // per window: its records' lengths / cumulative bytes
  void* d_ba_wgeo = nullptr;        // per data-page window: its k_ba_wcopy geometry
  int32_t* d_ba_chunks = nullptr;
  int32_t* d_dcum = nullptr;
  int64_t* d_basums = nullptr;
  int64_t* d_basums2 = nullptr;
  bool has_dba = false;
  int64_t* d_chunk_bytes = nullptr;
  DevNest* d_nests = nullptr;
  Tile* d_nest_tiles = nullptr;
  int64_t* d_nsums = nullptr;
  int64_t* d_ntotals = nullptr;
  std::vector<void*> allocations;
  std::vector<PageState> states;   // host copy after sync
  std::vector<int64_t> chunk_n;    // level slots per chunk
  std::vector<KernelRun> pending;  // events of the last run
  std::vector<pqh_kernel_stat> stats;
  bool synced = false;
  double bytes_read = 0, bytes_written = 0;
  std::vector<double> k_read, k_written;  // per kernel kind algorithmic bytes of one run
  std::vector<hipEvent_t> event_pool;
  size_t event_next = 0;
  hipGraph_t graph = nullptr;        // unprofiled runs: the captured launch sequence
  hipGraphExec_t gexec = nullptr;
  bool graph_failed = false;
  bool flat_on = false;   // the last run went through k_flat
  bool flat_off = false;  // a k_flat speculation failed once: the three kernels from then on
  int32_t flat_fallbacks = 0;
  int32_t regrows = 0;
  std::vector<DeltaState> hdstates;  // (after sync, batches with byte-array length streams) dstates
  std::vector<int32_t> page_nil;   // (after sync) nil INT96 values per page / chunk (value_nil marks)
  std::vector<int64_t> chunk_nil;
  std::vector<int64_t> flat_base;   // k_flat: page value bases if every page is clean (num_values prefixes)
  std::vector<FlatTile> flat_tiles; // k_flat: expand_tiles with their pages' fields
  int64_t* d_flat_base = nullptr;
  FlatTile* d_flat_tiles = nullptr;
  // a ring slot's staged batch (streaming context): the plan tables wait in a pinned block and travel
  // on the copy stream ahead of the range's payload, at its first pqh_batch_run_staged
  struct TableUp {
    void* dst;
    size_t off, bytes;
  };
  std::shared_ptr<uint8_t> h_tables;
  std::vector<TableUp> table_ups;
};

namespace {

size_t arena_guard() {
  static const size_t g = [] {
    const char* f = getenv("PQH_ARENA_GUARD");
    const long long v = f ? atoll(f) : 4096;
    return size_t(v > 0 ? (v + 255) & ~255ll : 0);
  }();
  return g;
}

bool arena_check() {
  static const bool c = [] {
    const char* f = getenv("PQH_ARENA_CHECK");
    return f && f[0] == '1';
  }();
  return c;
}

constexpr uint8_t kCanary = 0xA5;

hipError_t arena_alloc(pqh_ctx* ctx, void** p, size_t bytes) {
  DevArena& A = ctx->arena;
  std::lock_guard<std::mutex> g(A.m);
  const size_t gb = arena_guard();
  const size_t need = ((bytes + 255) & ~size_t(255)) + gb;
  if (A.chunks.empty() || A.chunks.back().cap - A.chunks.back().used < need) {
    size_t cap = std::max({need, A.want, size_t(64) << 20});
    cap = (cap + (size_t(2) << 20) - 1) & ~((size_t(2) << 20) - 1);
    void* q = nullptr;
    const hipError_t e = hipMalloc(&q, cap);
    if (e != hipSuccess) return e;
    A.want = 0;
    A.chunks.push_back({static_cast<uint8_t*>(q), cap, 0});
  }
  DevArena::Chunk& c = A.chunks.back();
  uint8_t* r = c.base + c.used;
  c.used += need;
  if (gb && arena_check()) {
    const hipError_t e = hipMemsetAsync(r + need - gb, kCanary, gb, ctx->stream);
    if (e != hipSuccess) return e;
    A.guards.push_back({r + need - gb, gb, bytes, A.allocs});
  }
  A.allocs++;
  A.live++;
  *p = r;
  return hipSuccess;
}

// Callers free only after the context's streams have drained (pqh_batch_destroy synchronises them).
void arena_free(pqh_ctx* ctx) {
  DevArena& A = ctx->arena;
  std::lock_guard<std::mutex> g(A.m);
  if (--A.live > 0) return;
  A.live = 0;
  A.allocs = 0;
  A.guards.clear();
  if (A.chunks.size() > 1) {  // it grew: one chunk of the peak (+1/8) from the next allocation on
    size_t used = 0;
    for (auto& c : A.chunks) {
      used += c.used;
      hipFree(c.base);
    }
    A.chunks.clear();
    A.want = used + used / 8;
  } else if (!A.chunks.empty()) {
    A.chunks[0].used = 0;
  }
}

void arena_release(pqh_ctx* ctx) {
  DevArena& A = ctx->arena;
  std::lock_guard<std::mutex> g(A.m);
  for (auto& c : A.chunks) hipFree(c.base);
  A.chunks.clear();
}

// (PQH_ARENA_CHECK=1, after a synchronised run) every guard gap still holds the canary; a kernel that
// wrote past an allocation is named by the allocation's index (plan order) and size.
int arena_verify(pqh_ctx* ctx) {
  DevArena& A = ctx->arena;
  std::vector<DevArena::Guard> gs;
  {
    std::lock_guard<std::mutex> g(A.m);
    gs = A.guards;
  }
  std::vector<uint8_t> h;
  std::string bad;
  for (const auto& g : gs) {
    h.resize(g.bytes);
    HIP_TRY(ctx, bounce_d2h(ctx, h.data(), g.p, g.bytes));
    size_t i = 0, n = 0;
    while (i < h.size() && h[i] == kCanary) i++;
    for (size_t k = i; k < h.size(); k++) n += h[k] != kCanary;
    if (i < h.size()) {
      char m[200];
      snprintf(m, sizeof(m), "%sallocation #%d (%zu bytes): guard byte +%zu = 0x%02x, %zu of %zu guard bytes overwritten",
               bad.empty() ? "" : "; ", g.index, g.alloc_bytes, i, h[i], n, h.size());
      bad += m;
    }
  }
  if (!bad.empty()) {
    std::string table;
    for (const auto& g : gs) table += " #" + std::to_string(g.index) + ":" + std::to_string(g.alloc_bytes);
    fprintf(stderr, "pqhip arena: %s\npqhip arena allocations:%s\n", bad.c_str(), table.c_str());
    return set_err(ctx, PQH_ERR_INTERNAL, "arena guard overwritten: " + bad);
  }
  return PQH_OK;
}

// Device buffers of a batch: hipMalloc, or in a streaming context the context's arena.
hipError_t dev_alloc(pqh_ctx* ctx, void** p, size_t bytes) {
  return (ctx->flags & PQH_CTX_STREAMING) ? arena_alloc(ctx, p, bytes) : hipMalloc(p, bytes);
}

void dev_free(pqh_ctx* ctx, void* p) {
  if (!p) return;
  if (ctx->flags & PQH_CTX_STREAMING) arena_free(ctx);
  else hipFree(p);
}

void free_batch(pqh_batch* b) {
  for (hipEvent_t e : b->event_pool) hipEventDestroy(e);
  for (void* p : b->allocations) dev_free(b->ctx, p);
  dev_free(b->ctx, b->owned_payload);
  dev_free(b->ctx, b->d_src);
  if (b->h_staged && !b->h_pinned_ref) hipHostFree(b->h_staged);
  b->h_pinned_ref.reset();
  b->h_tables.reset();
  if (b->ev_copied) hipEventDestroy(b->ev_copied);
  if (b->ev_done) hipEventDestroy(b->ev_done);
  for (hipEvent_t e : b->ev_dep)
    if (e) hipEventDestroy(e);
  if (b->gexec) hipGraphExecDestroy(b->gexec);
  if (b->graph) hipGraphDestroy(b->graph);
}

struct ChunkErr {
  int32_t status = PQH_OK, phase = 0, page = -1;
  int64_t index = 0;
};
ChunkErr chunk_error(const pqh_batch* b, int32_t chunk);

// Every planner buffer starts zeroed (once, at plan time, ordered before the batch's first run on
// the context stream): no kernel can ever read stale memory from an earlier allocation, whichever
// path it takes.
int dalloc(pqh_batch* b, void** p, size_t bytes) {
  if (bytes == 0) bytes = 16;
  hipError_t e = dev_alloc(b->ctx, p, bytes);
  if (e != hipSuccess) return set_err(b->ctx, PQH_ERR_NOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
  b->allocations.push_back(*p);
  e = hipMemsetAsync(*p, 0, bytes, b->ctx->stream);
  if (e != hipSuccess) return set_err(b->ctx, PQH_ERR_HIP, std::string("hipMemsetAsync: ") + hipGetErrorString(e));
  return PQH_OK;
}

hipEvent_t next_event(pqh_batch* b) {
  if (b->event_next == b->event_pool.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    b->event_pool.push_back(e);
  }
  return b->event_pool[b->event_next++];
}

}  // namespace

extern "C" {

int pqh_abi_version(void) { return PQH_ABI_VERSION; }

#ifndef PQH_SOURCE_HASH
#define PQH_SOURCE_HASH "unknown"
#endif
const char* pqh_build_id(void) { return PQH_SOURCE_HASH; }

int pqh_device_count(int32_t* count) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  *count = e == hipSuccess ? n : 0;
  return e == hipSuccess ? PQH_OK : PQH_ERR_NO_DEVICE;
}

int pqh_ctx_create(int32_t device, uint32_t flags, pqh_ctx** out) {
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return set_err(nullptr, PQH_ERR_NO_DEVICE, "no HIP device");
  if (device < 0 || device >= n) return set_err(nullptr, PQH_ERR_ARG, "bad device index");
  pqh_ctx* c = new pqh_ctx();
  c->device = device;
  c->flags = flags;
  // A streaming context (a ring slot) is ONE stream: copy, zero fills and decode in order.  The ring
  // overlaps slots, not a slot's own copy and decode, and every extra stream would share one of the
  // process's few hardware queues with another slot's stream -- a false dependency that holds one
  // slot's work behind another slot's copy.
  const bool one = (flags & PQH_CTX_STREAMING) != 0;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
      (!one && (hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) != hipSuccess ||
                hipStreamCreateWithFlags(&c->side2, hipStreamNonBlocking) != hipSuccess ||
                hipStreamCreateWithFlags(&c->side3, hipStreamNonBlocking) != hipSuccess))) {
    if (c->stream) hipStreamDestroy(c->stream);
    if (c->side) hipStreamDestroy(c->side);
    if (c->side2) hipStreamDestroy(c->side2);
    delete c;
    return set_err(nullptr, PQH_ERR_HIP, "stream creation failed");
  }
  *out = c;
  return PQH_OK;
}

void pqh_ctx_destroy(pqh_ctx* ctx) {
  if (!ctx) return;
  hipSetDevice(ctx->device);
  hipStreamSynchronize(ctx->stream);
  hipStreamDestroy(ctx->stream);
  for (hipStream_t st : {ctx->side, ctx->side2, ctx->side3})
    if (st) {
      hipStreamSynchronize(st);
      hipStreamDestroy(st);
    }
  if (ctx->copy_stream) {
    hipStreamSynchronize(ctx->copy_stream);
    hipStreamDestroy(ctx->copy_stream);
  }
  for (hipEvent_t ev : ctx->bounce_ev)
    if (ev) hipEventDestroy(ev);
  if (ctx->bounce) hipHostFree(ctx->bounce);
  arena_release(ctx);
  {
    std::lock_guard<std::mutex> g(ctx->pool->m);
    ctx->pool->closed = true;
    for (auto& fb : ctx->pool->free_blocks) hipHostFree(fb.first);
    ctx->pool->free_blocks.clear();
  }
  delete ctx;
}

const char* pqh_last_error(const pqh_ctx* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }

void* pqh_ctx_stream(pqh_ctx* ctx) { return ctx ? reinterpret_cast<void*>(ctx->stream) : nullptr; }

int64_t pqh_ctx_pinned_bytes(const pqh_ctx* ctx) { return ctx ? ctx->pool->pinned.load() : 0; }

int pqh_ctx_set_flags(pqh_ctx* ctx, uint32_t flags) {
  if (!ctx) return set_err(nullptr, PQH_ERR_ARG, "null context");
  ctx->flags = (flags & ~PQH_CTX_STREAMING) | (ctx->flags & PQH_CTX_STREAMING);  // (creation only)
  return PQH_OK;
}

int pqh_malloc(pqh_ctx* ctx, void** dptr, size_t bytes) {
  hipSetDevice(ctx->device);
  HIP_TRY(ctx, hipMalloc(dptr, bytes ? bytes : 16));
  return PQH_OK;
}
int pqh_free(pqh_ctx* ctx, void* dptr) {
  HIP_TRY(ctx, hipFree(dptr));
  return PQH_OK;
}
int pqh_host_alloc(pqh_ctx* ctx, void** hptr, size_t bytes) {
  HIP_TRY(ctx, hipHostMalloc(hptr, bytes ? bytes : 16, hipHostMallocDefault));
  return PQH_OK;
}
int pqh_host_free(pqh_ctx* ctx, void* hptr) {
  HIP_TRY(ctx, hipHostFree(hptr));
  return PQH_OK;
}
int pqh_memcpy_h2d(pqh_ctx* ctx, void* dst, const void* src, size_t bytes) {
  HIP_TRY(ctx, bounce_h2d(ctx, dst, src, bytes));
  return PQH_OK;
}
int pqh_memcpy_d2h(pqh_ctx* ctx, void* dst, const void* src, size_t bytes) {
  HIP_TRY(ctx, bounce_d2h(ctx, dst, src, bytes));
  return PQH_OK;
}
int pqh_memcpy_h2d_pinned_async(pqh_ctx* ctx, void* dst, const void* pinned_src, size_t bytes) {
  HIP_TRY(ctx, hipMemcpyAsync(dst, pinned_src, bytes, hipMemcpyHostToDevice, ctx->stream));
  return PQH_OK;
}
int pqh_sync(pqh_ctx* ctx) {
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return PQH_OK;
}

int pqh_batch_create(pqh_ctx* ctx, const pqh_chunk* chunks, int32_t num_chunks, const pqh_page* pages,
                     int32_t num_pages, const void* d_payload, int64_t payload_bytes, pqh_batch** out) {
  *out = nullptr;
  if (!ctx || num_chunks < 0 || num_pages < 0 || (num_pages > 0 && !d_payload))
    return set_err(ctx, PQH_ERR_ARG, "bad batch arguments");
  hipSetDevice(ctx->device);
  pqh_batch* b = new pqh_batch();
  b->ctx = ctx;
  b->chunks.assign(chunks, chunks + num_chunks);
  b->pages.assign(pages, pages + num_pages);
  b->d_payload = static_cast<const uint8_t*>(d_payload);
  b->payload_bytes = payload_bytes;
  b->hpages.resize(size_t(num_pages));
  b->hchunks.resize(size_t(num_chunks));
  b->chunk_n.assign(size_t(num_chunks), 0);
  b->k_read.assign(kNumKernels, 0);
  b->k_written.assign(kNumKernels, 0);

  // ---- per-page planning ----
  int64_t ck_cursor = 0, dblk_cursor = 0, dtile_cursor = 0, dcum_cursor = 0;
  std::vector<int64_t> bytes_est(size_t(num_chunks), 0);
  std::vector<std::vector<Tile>> by_kind(8);
  for (int32_t c = 0; c < num_chunks; c++) {
    const pqh_chunk& C = chunks[c];
    DevChunk& D = b->hchunks[size_t(c)];
    memset(&D, 0, sizeof(D));
    D.physical_type = C.column.physical_type;
    D.type_length = C.column.type_length;
    D.max_def = C.column.max_def;
    D.max_rep = C.column.max_rep;
    D.first_page = C.first_page;
    D.num_pages = C.num_pages;
    D.dict_page = -1;
    int32_t vs = 0;
    resolve_kind(C.column.physical_type, C.column.type_length, PQH_ENC_PLAIN, &vs);
    D.value_size = vs;
    if (C.first_page < 0 || C.num_pages < 0 || int64_t(C.first_page) + C.num_pages > num_pages) {
      delete b;
      return set_err(ctx, PQH_ERR_ARG, "chunk page range out of bounds");
    }
    // FIXED_LEN_BYTE_ARRAY pages with DELTA_BYTE_ARRAY go to byteArrayDeltaDecoder, which yields
    // variable-length []byte with no length check (chunk_reader.go:67-78, type_bytearray.go:189-240):
    // such a chunk is output as offsets + bytes.  Its fixed-width pages (PLAIN, dictionary) decode
    // into the values buffer (scratch) as usual, and k_ba_expand lays them out as byte arrays.
    // (A FIXED_LEN_BYTE_ARRAY chunk whose type_length is <= 0 has no fixed width either.)
    bool flba_var = false;
    if (C.column.physical_type == PQH_FIXED_LEN_BYTE_ARRAY && C.column.type_length > 0)
      for (int32_t i = 0; i < C.num_pages && !flba_var; i++) {
        const int64_t p = int64_t(C.first_page) + i;
        if (p >= 0 && p < num_pages && pages[p].page_type != PQH_DICTIONARY_PAGE &&
            pages[p].encoding == PQH_ENC_DELTA_BYTE_ARRAY)
          flba_var = true;
      }
    if (flba_var) D.value_size = 0;
    const bool ba_chunk = is_ba_chunk(D);
    D.batile_base = int32_t(b->ba_tiles.size());
    if (ba_chunk) b->ba_chunks.push_back(c);
    int64_t level_base = 0;
    for (int32_t i = 0; i < C.num_pages; i++) {
      const int32_t p = C.first_page + i;
      const pqh_page& Q = pages[p];
      DevPage& P = b->hpages[size_t(p)];
      memset(&P, 0, sizeof(P));
      P.image_off = Q.image_offset;
      P.image_len = Q.image_len;
      P.page_type = Q.page_type;
      P.num_values = Q.num_values;
      P.encoding = Q.encoding;
      P.def_len = Q.def_levels_byte_length;
      P.rep_len = Q.rep_levels_byte_length;
      P.num_nulls = Q.page_type == PQH_DATA_PAGE_V2 ? Q.num_nulls : 0;
      P.chunk = c;
      P.dict_page = -1;
      P.ck_rep = P.ck_def = P.ck_val = -1;
      P.dblk_base = -1;
      P.host_err = kNoError;  // (a walker error, host_status, lies after the listed pages: chunk_error)
      if (Q.image_offset < 0 || Q.image_len < 0 || Q.image_offset + Q.image_len > payload_bytes) {
        delete b;
        return set_err(ctx, PQH_ERR_ARG, "page image outside the payload");
      }
      if (Q.page_type == PQH_DICTIONARY_PAGE) {
        // dictPageReader.read (page_dict.go:35-72) + getDictValuesDecoder (chunk_reader.go:17-39)
        int32_t dvs = 0;
        int32_t kind = resolve_kind(C.column.physical_type, C.column.type_length, PQH_ENC_PLAIN, &dvs);
        P.kind = kind;
        P.value_size = dvs;
        // "there should be only one dictionary" (chunk_reader.go:197-199); a dictionary page after data
        // pages is read like any other: the pages before it decode without a dictionary
        if (D.dict_page >= 0) P.host_err = std::min<uint64_t>(P.host_err, err_key(0, 0, PQH_ERR_DICT_PAGE));
        else if (Q.num_values < 0) P.host_err = std::min<uint64_t>(P.host_err, err_key(0, 0, PQH_ERR_PAGE_HEADER));
        else if (Q.encoding != PQH_ENC_PLAIN && Q.encoding != PQH_ENC_PLAIN_DICTIONARY)
          P.host_err = std::min<uint64_t>(P.host_err, err_key(0, 0, PQH_ERR_DICT_PAGE));
        else if (C.column.physical_type == PQH_BOOLEAN)
          P.host_err = std::min<uint64_t>(P.host_err, err_key(0, 0, PQH_ERR_UNSUPPORTED));
        if (kind == K_PLAIN_BA && P.host_err == kNoError) {  // byte-array dictionary: PLAIN chain walk
          P.aux_base = int32_t(dcum_cursor);
          dcum_cursor += int64_t(std::max(0, Q.num_values)) + 1;
          b->ba_pages.push_back(p);
        }
        if (D.dict_page < 0) D.dict_page = p;
        b->bytes_read += Q.image_len;
        continue;
      }
      if (Q.page_type != PQH_DATA_PAGE && Q.page_type != PQH_DATA_PAGE_V2)
        P.host_err = std::min<uint64_t>(P.host_err, err_key(0, 0, PQH_ERR_PAGE_HEADER));
      int32_t pvs = 0;
      int32_t kind = resolve_kind(C.column.physical_type, C.column.type_length, Q.encoding, &pvs);
      P.kind = kind;
      P.value_size = pvs;
      P.dict_page = D.dict_page;
      if (Q.num_values < 0) P.host_err = std::min<uint64_t>(P.host_err, err_key(0, 0, PQH_ERR_PAGE_HEADER));
      if (Q.page_type == PQH_DATA_PAGE_V2 &&
          (Q.rep_levels_byte_length < 0 || Q.def_levels_byte_length < 0 ||
           int64_t(Q.rep_levels_byte_length) + Q.def_levels_byte_length > Q.image_len))
        P.host_err = std::min<uint64_t>(P.host_err, err_key(0, 0, PQH_ERR_PAGE_HEADER));
      if (kind == K_UNSUPPORTED) P.host_err = std::min<uint64_t>(P.host_err, err_key(0, 0, PQH_ERR_UNSUPPORTED));
      const int64_t n = Q.num_values > 0 ? Q.num_values : 0;
      P.level_base = level_base;
      level_base += n;
      b->bytes_read += Q.image_len;
      if ((kind == K_DELTA32 || kind == K_DELTA64 || kind == K_DLBA || kind == K_DBA) && P.host_err == kNoError) {
        // the values decoder is initialised (and may fail) even for pages without values;
        // DELTA_BYTE_ARRAY: two length streams (prefix, suffix), each with its records and tiles
        const int streams = kind == K_DBA ? 2 : 1;
        P.dblk_base = int32_t(dblk_cursor);
        P.dblk_cap = int32_t(streams * (ceil_div(n, kDeltaBlockMin) + 1));
        dblk_cursor += P.dblk_cap;
        P.dtile_base = int32_t(dtile_cursor);
        P.dtile_n = int32_t(ceil_div(n, kDeltaTile));
        dtile_cursor += int64_t(streams) * P.dtile_n;
        b->delta_pages.push_back(p);
        for (int st = 0; st < streams; st++) {  // Tile.kind = stream (k_delta_expand)
          for (int32_t k = 0; k < P.dtile_n; k++) by_kind[TK_DELTA].push_back(Tile{p, k, st, 1});
          if (P.dtile_n > 0) b->delta_streams.push_back(Tile{p, 0, st, 1});
        }
        if (kind == K_DBA) b->has_dba = true;
      }
      const bool ba_page = ba_chunk && (kind == K_PLAIN_BA || kind == K_DLBA || kind == K_DICT || kind == K_DBA ||
                                        (flba_var && kind == K_PLAIN_FIXED));
      if (ba_page && P.host_err == kNoError && n > 0) {
        P.batile_base = int32_t(b->ba_tiles.size());
        P.batile_n = int32_t(ceil_div(n, kBaTile));
        for (int32_t k = 0; k < P.batile_n; k++) b->ba_tiles.push_back(Tile{p, k, TK_BA, 1});
        if (kind == K_PLAIN_BA) b->ba_pages.push_back(p);
        // output bytes: at most the page (PLAIN / DELTA_LENGTH); dictionary gathers are estimated
        // from the dictionary page's mean entry and re-sized after the first run if short
        int64_t est = kind == K_DBA ? 4 * int64_t(Q.image_len) : Q.image_len;  // prefixes repeat bytes
        if (pvs > 0) {  // fixed-width page of a FIXED_LEN_BYTE_ARRAY chunk with DELTA_BYTE_ARRAY pages
          est = n * pvs;
        } else if (kind == K_DICT && D.dict_page >= 0) {
          const pqh_page& DQ = pages[D.dict_page];
          const int64_t nv = std::max(1, DQ.num_values);
          const int64_t mean = std::max<int64_t>(0, DQ.image_len - 4 * nv) / nv;
          est = n * std::min<int64_t>(std::max<int64_t>(DQ.image_len, 0), 2 * mean + 16);
        }
        bytes_est[size_t(c)] += est;
      }
      if (n == 0) continue;
      const int64_t nt = ceil_div(n, kHybridTile);
      if (C.column.max_rep > 0) {
        P.ck_rep = int32_t(ck_cursor);
        P.ck_rep_n = int32_t(nt);
        ck_cursor += nt;
      }
      if (C.column.max_def > 0) {
        P.ck_def = int32_t(ck_cursor);
        P.ck_def_n = int32_t(nt);
        ck_cursor += nt;
      }
      if (kind == K_DICT || kind == K_RLE_BOOL) {
        P.ck_val = int32_t(ck_cursor);
        P.ck_val_n = int32_t(nt);
        ck_cursor += nt;
      }
      if (P.host_err != kNoError) continue;
      if (C.column.max_rep > 0 || C.column.max_def > 0)
        for (int32_t k = 0; k < nt; k += kLevelSpan)
          by_kind[TK_LEVELS].push_back(Tile{p, k, TK_LEVELS, int32_t(std::min<int64_t>(kLevelSpan, nt - k))});
      switch (kind) {
        case K_PLAIN_FIXED:
        case K_PLAIN_INT96: {
          const int64_t ct = ceil_div(n * pvs, kCopyTileBytes);
          for (int32_t k = 0; k < ct; k++) by_kind[TK_COPY].push_back(Tile{p, k, TK_COPY, 1});
          break;
        }
        case K_PLAIN_BOOL: {
          const int64_t bt = ceil_div(n, kBoolTile);
          for (int32_t k = 0; k < bt; k++) by_kind[TK_BOOL].push_back(Tile{p, k, TK_BOOL, 1});
          break;
        }
        case K_RLE_BOOL:
          for (int32_t k = 0; k < nt; k += kDictSpan)
            by_kind[TK_RLE_BOOL].push_back(Tile{p, k, TK_RLE_BOOL, int32_t(std::min<int64_t>(kDictSpan, nt - k))});
          break;
        case K_DICT: {
          int64_t dict_bytes = 0;
          if (D.dict_page >= 0) dict_bytes = int64_t(std::max(0, pages[D.dict_page].num_values)) * pvs;
          const int tk = dict_bytes <= kDictLdsMax ? TK_DICT : TK_DICT_GLOBAL;
          if (tk == TK_DICT) b->expand_lds = std::max<size_t>(b->expand_lds, size_t((dict_bytes + 15) & ~int64_t(15)));
          for (int32_t k = 0; k < nt; k += kDictSpan)
            by_kind[tk].push_back(Tile{p, k, tk, int32_t(std::min<int64_t>(kDictSpan, nt - k))});
          break;
        }
        default:
          break;
      }
    }
    b->chunk_n[size_t(c)] = level_base;
    D.batile_n = int32_t(b->ba_tiles.size()) - D.batile_base;
    // fused PLAIN chain: byte-array chunks of PLAIN data pages only (no dictionary page, nothing the
    // planner already failed)
    D.ba_fused = 0;
    if (ba_chunk && fuse_enabled() && D.value_size == 0 && D.dict_page < 0 && C.num_pages > 0) {
      bool all = true;
      for (int32_t i = 0; i < C.num_pages && all; i++) {
        const DevPage& P = b->hpages[size_t(C.first_page + i)];
        all = P.page_type != PQH_DICTIONARY_PAGE && P.kind == K_PLAIN_BA && P.host_err == kNoError;
      }
      D.ba_fused = all ? 1 : 0;
    }
  }
  {  // fused chunks last in the byte-array lists (their prefixes are the scratch path's while fused)
    auto fused_page = [&](int32_t p) { return b->hchunks[size_t(b->hpages[size_t(p)].chunk)].ba_fused != 0; };
    std::stable_partition(b->ba_pages.begin(), b->ba_pages.end(), [&](int32_t p) { return !fused_page(p); });
    b->ba_pages_nf = int32_t(std::count_if(b->ba_pages.begin(), b->ba_pages.end(), [&](int32_t p) { return !fused_page(p); }));
    std::stable_partition(b->ba_chunks.begin(), b->ba_chunks.end(), [&](int32_t c) { return !b->hchunks[size_t(c)].ba_fused; });
    b->ba_chunks_nf = int32_t(std::count_if(b->ba_chunks.begin(), b->ba_chunks.end(),
                                            [&](int32_t c) { return !b->hchunks[size_t(c)].ba_fused; }));
    b->ba_fuse_on = b->ba_pages_nf < int32_t(b->ba_pages.size());
  }
  // Interleave the kinds proportionally along the dispatch order (k_expand's grid), so that every
  // CU sees a mix of byte-copy and bit-unpack tiles instead of one long phase per kind.
  {
    std::vector<std::pair<double, Tile>> keyed;
    for (int kd : {int(TK_LEVELS), int(TK_COPY), int(TK_BOOL), int(TK_DICT), int(TK_RLE_BOOL)}) {
      const auto& v = by_kind[size_t(kd)];
      for (size_t i = 0; i < v.size(); i++) keyed.push_back({(double(i) + 0.5) / double(v.size()), v[i]});
    }
    std::stable_sort(keyed.begin(), keyed.end(), [](const auto& a, const auto& c) { return a.first < c.first; });
    for (auto& kv : keyed) b->expand_tiles.push_back(kv.second);
    b->global_tiles = by_kind[TK_DICT_GLOBAL];
    b->delta_tiles = by_kind[TK_DELTA];
    for (size_t i = 0; i < b->ba_pages.size(); i++) {  // chain windows: enough to cover the whole page image
      const int32_t p = b->ba_pages[i];
      if (int32_t(i) == b->ba_pages_nf) b->ba_wins_nf = int32_t(b->ba_wins.size());
      const int64_t len = std::max<int64_t>(b->hpages[size_t(p)].image_len, 1);
      const int32_t nw = int32_t((len + kChainStride - 1) / kChainStride);
      b->ba_pwin.push_back(make_int2(int32_t(b->ba_wins.size()), nw));
      for (int32_t w = 0; w < nw; w++) b->ba_wins.push_back(make_int2(p, w));
    }
    if (b->ba_pages_nf == int32_t(b->ba_pages.size())) b->ba_wins_nf = int32_t(b->ba_wins.size());
    for (int dict = 1; dict >= 0; dict--) {
      for (size_t i = 0; i < b->ba_wins.size(); i++) {
        const int32_t p = b->ba_wins[i].x;
        if ((b->hpages[size_t(p)].page_type == PQH_DICTIONARY_PAGE) == bool(dict))
          b->ba_wlist.push_back(make_int2(int32_t(i), p));
      }
      if (dict) b->ba_wdict = int32_t(b->ba_wlist.size());
    }
    b->ba_wlist_nf = int32_t(std::count_if(b->ba_wlist.begin(), b->ba_wlist.end(),
                                           [&](const int2& x) { return x.x < b->ba_wins_nf; }));
    // k_ba_chain takes every page's window 0 first, then every window 1, ...: a window's
    // predecessors started a whole round of pages before it, so its look-back rarely waits
    for (int32_t i = 0; i < int32_t(b->ba_wins.size()) - b->ba_wins_nf; i++) b->ba_forder.push_back(i);
    std::stable_sort(b->ba_forder.begin(), b->ba_forder.end(), [&](int32_t x, int32_t y) {
      return b->ba_wins[size_t(b->ba_wins_nf + x)].y < b->ba_wins[size_t(b->ba_wins_nf + y)].y;
    });
    b->delta_page_mode = b->delta_streams.size() >= kDeltaPageModeMin;
    if (const char* f = getenv("PQH_DELTA_PAGE_MODE"))  // tests: force either path ("0" / "1")
      b->delta_page_mode = f[0] == '1';
    if (b->delta_page_mode) {
      // every delta page is chased + decoded by k_delta_fused after the value scan and then walked
      // exactly.  Byte-array length streams decode all their lengths at load, so an error anywhere
      // in them is a load error; the scan does not need it: it only moves the value offsets of the
      // pages after the failing one, inside a chunk whose result is that error.
      b->delta_fused_pages = int32_t(b->delta_pages.size());
      b->delta_fused_streams = int32_t(b->delta_streams.size());
      // DELTA_LENGTH streams last: k_delta_fused<true> sums their tiles' bytes
      std::stable_partition(b->delta_streams.begin(), b->delta_streams.end(),
                            [&](const Tile& t) { return b->hpages[size_t(t.page)].kind != K_DLBA; });
      b->delta_lens_streams = int32_t(std::count_if(b->delta_streams.begin(), b->delta_streams.end(),
                                                    [&](const Tile& t) { return b->hpages[size_t(t.page)].kind == K_DLBA; }));
      b->split_on = split_enabled();
      if (b->split_on) {
        // windows of kSplitStride bytes over each stream k_delta_fused would take (the first stream
        // of each page), page-major; dispatched window-major (every page's window 0, then every
        // window 1, ...), the DELTA_LENGTH streams' windows in a launch of their own
        std::vector<int32_t> ord[2];
        for (const Tile& t : b->delta_streams) {
          if (t.kind != 0) continue;
          const DevPage& P = b->hpages[size_t(t.page)];
          const int g = P.kind == K_DLBA ? 1 : 0;
          const int32_t nw = int32_t(std::max<int64_t>(1, ceil_div(std::max<int64_t>(P.image_len, 1), kSplitStride)));
          for (int32_t w = 0; w < nw; w++) {
            ord[g].push_back(int32_t(b->split_wins.size()));
            b->split_wins.push_back(make_int2(t.page, w));
          }
        }
        for (int g = 0; g < 2; g++) {
          std::stable_sort(ord[g].begin(), ord[g].end(), [&](int32_t x, int32_t y) {
            return b->split_wins[size_t(x)].y < b->split_wins[size_t(y)].y;
          });
          b->split_order.insert(b->split_order.end(), ord[g].begin(), ord[g].end());
        }
        b->split_nl = int32_t(ord[1].size());
      }
    }
  }

  // k_ba_expand's contiguous copies: DELTA_LENGTH tiles and the fixed-width tiles of FIXED_LEN_BYTE_ARRAY
  // chunks laid out as byte arrays (copied from the values buffer)
  for (size_t i = 0; i < b->ba_tiles.size(); i++) {
    const DevPage& P = b->hpages[size_t(b->ba_tiles[i].page)];
    if (P.kind == K_DLBA || P.value_size > 0) b->ba_xlist.push_back(int32_t(i));
  }
  b->ba_ncopy = int32_t(b->ba_xlist.size());
  for (size_t i = 0; i < b->ba_tiles.size(); i++) {  // dictionary tiles (PLAIN pages: k_ba_wcopy)
    const DevPage& P = b->hpages[size_t(b->ba_tiles[i].page)];
    if (P.kind != K_DLBA && P.kind != K_DBA && P.kind != K_PLAIN_BA && P.value_size == 0) b->ba_xlist.push_back(int32_t(i));
  }
  // k_ba_sum's work list (after the copy + gather lists): every tile, except that PLAIN pages (and in
  // page mode DELTA_LENGTH pages) are represented by their tile 0: their sums come from k_ba_wstitch
  // (the delta kernels); the tile-0 workgroup checks that and otherwise sums the whole page
  b->ba_sum_off = int32_t(b->ba_xlist.size());
  for (int fused = 0; fused < 2; fused++)  // (fused chunks' PLAIN tiles last)
    for (size_t i = 0; i < b->ba_tiles.size(); i++) {
      const Tile& t = b->ba_tiles[i];
      const DevPage& P = b->hpages[size_t(t.page)];
      if (int(b->hchunks[size_t(P.chunk)].ba_fused != 0) != fused) continue;
      if (t.k == 0 || !(P.kind == K_PLAIN_BA || (b->delta_page_mode && P.kind == K_DLBA))) b->ba_xlist.push_back(int32_t(i));
      if (!fused) b->ba_sum_nf = int32_t(b->ba_xlist.size()) - b->ba_sum_off;
    }

  {  // k_flat's speculative value bases (built for every batch, used when k_flat is eligible)
    b->flat_base.assign(size_t(num_pages), 0);
    for (int32_t c = 0; c < num_chunks; c++) {
      const DevChunk& D = b->hchunks[size_t(c)];
      int64_t acc = 0;
      for (int32_t i = 0; i < D.num_pages; i++) {
        const DevPage& P = b->hpages[size_t(D.first_page + i)];
        b->flat_base[size_t(D.first_page + i)] = acc;
        // (nullable chunks: V2 pages' notNull = num_values - num_nulls, checked by k_flat's page checks)
        if (P.page_type != PQH_DICTIONARY_PAGE)
          acc += std::max(0, P.num_values - (D.max_def > 0 ? std::max(0, P.num_nulls) : 0));
      }
    }
  }

  // ---- device allocations ----
  int rc;
  const size_t ntiles = b->expand_tiles.size() + b->global_tiles.size();
  if ((rc = dalloc(b, reinterpret_cast<void**>(&b->d_pages), sizeof(DevPage) * size_t(num_pages))) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&b->d_states), sizeof(PageState) * size_t(num_pages))) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&b->d_ckpts), sizeof(Ckpt) * size_t(ck_cursor))) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&b->d_tiles), sizeof(Tile) * ntiles)) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&b->d_dtiles), sizeof(Tile) * b->delta_tiles.size())) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&b->d_delta_pages), sizeof(int32_t) * b->delta_pages.size())) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&b->d_dstates), sizeof(DeltaState) * 2 * size_t(num_pages))) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&b->d_dblocks), sizeof(DeltaBlock) * size_t(dblk_cursor))) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&b->d_dsums), sizeof(uint64_t) * size_t(dtile_cursor))) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&b->d_batiles), sizeof(Tile) * b->ba_tiles.size())) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&b->d_ba_xlist), sizeof(int32_t) * b->ba_xlist.size())) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&b->d_ba_pages), sizeof(int32_t) * b->ba_pages.size())) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&b->d_ba_wins), sizeof(int2) * b->ba_wins.size())) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&b->d_ba_pwin), sizeof(int2) * b->ba_pwin.size())) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&b->d_ba_wlist), sizeof(int2) * b->ba_wlist.size())) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&b->d_ba_res), sizeof(BaWin) * b->ba_wins.size())) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&b->d_ba_wrec), sizeof(uint16_t) * size_t(kChainRecs) * b->ba_wins.size())) ||
      (rc = dalloc(b, &b->d_ba_wgeo, size_t(kWGeoBytes) * b->ba_wins.size())) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&b->d_ba_chunks), sizeof(int32_t) * b->ba_chunks.size())) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&b->d_dcum), sizeof(int32_t) * size_t(dcum_cursor))) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&b->d_basums), sizeof(int64_t) * b->ba_tiles.size())) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&b->d_basums2), sizeof(int64_t) * b->ba_tiles.size())) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&b->d_bafuse), sizeof(uint32_t) * 8)) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&b->d_flat_base), sizeof(int64_t) * size_t(num_pages))) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&b->d_flat_tiles), sizeof(FlatTile) * b->expand_tiles.size())) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&b->d_bawords), sizeof(uint64_t) * (b->ba_wins.size() - size_t(b->ba_wins_nf)))) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&b->d_ba_forder), sizeof(int32_t) * b->ba_forder.size())) ||
      (b->split_on && (rc = dalloc(b, reinterpret_cast<void**>(&b->d_dsplit), sizeof(DeltaSplit) * size_t(num_pages)))) ||
      (b->split_on && (rc = dalloc(b, reinterpret_cast<void**>(&b->d_dticket), sizeof(uint32_t) * 2))) ||
      (b->split_on && (rc = dalloc(b, reinterpret_cast<void**>(&b->d_dwords), sizeof(uint64_t) * 3 * b->split_wins.size()))) ||
      (b->split_on && (rc = dalloc(b, reinterpret_cast<void**>(&b->d_split_wins), sizeof(int2) * b->split_wins.size()))) ||
      (b->split_on && (rc = dalloc(b, reinterpret_cast<void**>(&b->d_split_order), sizeof(int32_t) * b->split_order.size()))) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&b->d_chunk_bytes), sizeof(int64_t) * size_t(std::max(num_chunks, 1))))) {
    free_batch(b);
    delete b;
    return rc;
  }
  for (int32_t c = 0; c < num_chunks; c++) {
    DevChunk& D = b->hchunks[size_t(c)];
    const int64_t n = b->chunk_n[size_t(c)];
    D.values_cap = n;
    void* p = nullptr;
    const bool ba_chunk = is_ba_chunk(D);
    // values: fixed width, or the fixed-width pages' scratch of a FIXED_LEN_BYTE_ARRAY chunk laid out as byte arrays
    const int32_t vsz = D.value_size > 0 ? D.value_size : (ba_chunk && D.physical_type == PQH_FIXED_LEN_BYTE_ARRAY
                                                                ? std::max(D.type_length, 0) : 0);
    if ((rc = dalloc(b, &p, vsz == 0 && ba_chunk ? 64 : size_t(n) * size_t(std::max(vsz, 1)) + 64))) break;
    D.values = static_cast<uint8_t*>(p);
    if (D.physical_type == PQH_INT96) {
      // the reference's nil values (type_int96.go:21-42): a PLAIN page may end with a short value
      // (known only once notNull is), a dictionary page's last entry may be short (known now)
      bool plain = false, dnil = false;
      for (int32_t i = 0; i < D.num_pages; i++) {
        const DevPage& Q = b->hpages[size_t(D.first_page + i)];
        plain = plain || (Q.page_type != PQH_DICTIONARY_PAGE && Q.kind == K_PLAIN_INT96);
      }
      if (D.dict_page >= 0) {
        const DevPage& Q = b->hpages[size_t(D.dict_page)];
        dnil = Q.host_err == kNoError && Q.kind == K_PLAIN_INT96 && Q.num_values > 0 &&
               int64_t(Q.image_len) / 12 == int64_t(Q.num_values) - 1 && Q.image_len % 12 != 0;
      }
      if (plain || dnil) {
        if ((rc = dalloc(b, &p, size_t(n) + 64))) break;
        D.value_nil = static_cast<uint8_t*>(p);
        D.dict_nil = dnil ? 1 : 0;
      }
    }
    if (ba_chunk) {
      if ((rc = dalloc(b, &p, size_t(n + 1) * sizeof(int64_t)))) break;
      D.offsets = static_cast<int64_t*>(p);
      if ((rc = dalloc(b, &p, size_t(n) * sizeof(int32_t) + 64))) break;
      D.aux = static_cast<int32_t*>(p);
      bool dba = false;
      for (int32_t i = 0; i < D.num_pages; i++) dba = dba || b->hpages[size_t(D.first_page + i)].kind == K_DBA;
      if (dba) {
        if ((rc = dalloc(b, &p, size_t(n) * sizeof(int32_t) + 64))) break;
        D.aux2 = static_cast<int32_t*>(p);
      }
      D.bytes_cap = bytes_est[size_t(c)];
      if ((rc = dalloc(b, &p, size_t(D.bytes_cap) + 64))) break;
      D.bytes = static_cast<uint8_t*>(p);
    }
    if (D.max_def > 0) {
      if ((rc = dalloc(b, &p, size_t(n) + 64))) break;
      D.def_levels = static_cast<uint8_t*>(p);
    }
    if (D.max_rep > 0) {
      if ((rc = dalloc(b, &p, size_t(n) + 64))) break;
      D.rep_levels = static_cast<uint8_t*>(p);
    }
  }
  // nesting outputs of repeated chunks (levels -> list offsets / presence / leaf validity)
  b->chunk_nest.assign(size_t(num_chunks), -1);
  for (int32_t c = 0; c < num_chunks && !rc; c++) {
    const pqh_column& col = chunks[c].column;
    const int64_t n = b->chunk_n[size_t(c)];
    if (col.max_rep <= 0 || col.max_rep > PQH_MAX_NEST || n <= 0) continue;
    bool ok = true;  // repeated-node definition levels must rise strictly within [1, max_def]
    for (int l = 0; l < col.max_rep; l++)
      ok = ok && col.rep_def[l] >= 1 && col.rep_def[l] <= col.max_def && (l == 0 || col.rep_def[l] > col.rep_def[l - 1]);
    if (!ok) continue;
    // windows of kMaxNest levels: one DevNest each (the chunk's are consecutive in b->nests)
    b->chunk_nest[size_t(c)] = int32_t(b->nests.size());
    void* leaf = nullptr;
    if ((rc = dalloc(b, &leaf, size_t(n) + 64))) break;
    for (int32_t l0 = 0; l0 < col.max_rep && !rc; l0 += kMaxNest) {
      DevNest N;
      memset(&N, 0, sizeof(N));
      N.chunk = c;
      N.levels = std::min<int32_t>(kMaxNest, col.max_rep - l0);
      N.lbase = l0;
      N.d0 = l0 > 0 ? col.rep_def[l0 - 1] : 0;
      N.leaf = l0 + N.levels == col.max_rep;
      N.max_def = col.max_def;
      N.n = n;
      N.tile_base = int32_t(b->nest_tiles.size());
      N.tile_n = int32_t(ceil_div(n, kNestTile));
      for (int l = 0; l < N.levels; l++) {
        N.rep_def[l] = col.rep_def[l0 + l];
        void* p = nullptr;
        if ((rc = dalloc(b, &p, size_t(n + 1) * sizeof(int32_t)))) break;
        N.offsets[l] = static_cast<int32_t*>(p);
        if ((rc = dalloc(b, &p, size_t(n) + 64))) break;
        N.validity[l] = static_cast<uint8_t*>(p);
      }
      N.leaf_valid = static_cast<uint8_t*>(leaf);
      for (int32_t k = 0; k < N.tile_n; k++) b->nest_tiles.push_back(Tile{int32_t(b->nests.size()), k, 0, 1});
      b->nests.push_back(N);
    }
    if (rc) break;
  }
  // Tiles in round-robin order over the chunks (tile k of every chunk, then tile k + 1): a chunk's
  // tiles stay in order, as the one-pass write's look-back needs, and the tiles in flight at once
  // spread over the chunks, so a look-back rarely reaches past its first window of 64 tiles.  (Every
  // nesting kernel finds its slots from N.tile_base + t.k, not from the list position.)
  if (!rc && b->nests.size() > 1) {
    std::vector<Tile> rr;
    rr.reserve(b->nest_tiles.size());
    int32_t most = 0;
    for (const DevNest& N : b->nests) most = std::max(most, N.tile_n);
    for (int32_t k = 0; k < most; k++)
      for (size_t i = 0; i < b->nests.size(); i++)
        if (k < b->nests[i].tile_n) rr.push_back(Tile{int32_t(i), k, 0, 1});
    b->nest_tiles.swap(rr);
  }
  if (!rc && !(rc = dalloc(b, reinterpret_cast<void**>(&b->d_nests), sizeof(DevNest) * b->nests.size())) &&
      !(rc = dalloc(b, reinterpret_cast<void**>(&b->d_nest_tiles), sizeof(Tile) * b->nest_tiles.size())) &&
      !(rc = dalloc(b, reinterpret_cast<void**>(&b->d_nsums), sizeof(int64_t) * kNestFlags * b->nest_tiles.size())))
    rc = dalloc(b, reinterpret_cast<void**>(&b->d_ntotals), sizeof(int64_t) * kNestFlags * b->nests.size());
  for (size_t i = 0; i < b->nests.size(); i++) b->nests[i].totals = b->d_ntotals + i * kNestFlags;
  if (rc || (rc = dalloc(b, reinterpret_cast<void**>(&b->d_chunks), sizeof(DevChunk) * size_t(std::max(num_chunks, 1))))) {
    free_batch(b);
    delete b;
    return rc;
  }
  // the level tiles of the nested chunks first, as their own launch: the nesting branch forks after
  // it and overlaps the value tiles (and the byte-array chain) instead of following all of k_expand
  if (!b->nests.empty() && nest_early_enabled()) {
    auto nest_lev = [&](const Tile& t) {
      return t.kind == TK_LEVELS && b->chunk_nest[size_t(b->hpages[size_t(t.page)].chunk)] >= 0;
    };
    std::stable_partition(b->expand_tiles.begin(), b->expand_tiles.end(), nest_lev);
    b->expand_lev_n = int32_t(std::count_if(b->expand_tiles.begin(), b->expand_tiles.end(), nest_lev));
  }
  std::vector<Tile> all(b->expand_tiles);
  all.insert(all.end(), b->global_tiles.begin(), b->global_tiles.end());
  for (const Tile& t : b->expand_tiles) {  // k_flat's records (the chunks' value buffers are known now)
    const DevPage& P = b->hpages[size_t(t.page)];
    FlatTile f;
    memset(&f, 0, sizeof(f));
    f.image_off = P.image_off;
    f.dict_off = -1;
    if (P.dict_page >= 0) {
      const DevPage& D = b->hpages[size_t(P.dict_page)];
      if (D.host_err == kNoError) f.dict_off = D.image_off;
      f.dict_n = D.num_values;
      f.dict_len = D.image_len;
    }
    f.value_base = b->flat_base[size_t(t.page)];
    f.values = b->hchunks[size_t(P.chunk)].values;
    f.image_len = P.image_len;
    f.num_values = P.num_values;
    f.page_type = P.page_type;
    f.kind = P.kind;
    f.value_size = P.value_size;
    f.rep_len = P.rep_len;
    f.def_len = P.def_len;
    f.k = t.k;
    f.span = t.span;
    f.tkind = t.kind;
    f.host_err = P.host_err;
    const DevChunk& C = b->hchunks[size_t(P.chunk)];
    f.max_def = C.max_def;
    f.num_nulls = P.num_nulls;
    f.def_out = C.def_levels ? C.def_levels + P.level_base : nullptr;
    b->flat_tiles.push_back(f);
  }
  // page mode: the (shorter) stream list takes the delta tile list's place
  const std::vector<Tile>& dl = b->delta_page_mode ? b->delta_streams : b->delta_tiles;
  struct Up {
    void* dst;
    const void* src;
    size_t bytes;
  };
  const Up ups[] = {
      {b->d_pages, b->hpages.data(), sizeof(DevPage) * size_t(num_pages)},
      {b->d_chunks, b->hchunks.data(), sizeof(DevChunk) * size_t(num_chunks)},
      {b->d_tiles, all.data(), sizeof(Tile) * ntiles},
      {b->d_dtiles, dl.data(), b->delta_tiles.empty() ? 0 : sizeof(Tile) * dl.size()},
      {b->d_delta_pages, b->delta_pages.data(), sizeof(int32_t) * b->delta_pages.size()},
      {b->d_batiles, b->ba_tiles.data(), sizeof(Tile) * b->ba_tiles.size()},
      {b->d_ba_xlist, b->ba_xlist.data(), sizeof(int32_t) * b->ba_xlist.size()},
      {b->d_ba_pages, b->ba_pages.data(), sizeof(int32_t) * b->ba_pages.size()},
      {b->d_ba_wins, b->ba_wins.data(), sizeof(int2) * b->ba_wins.size()},
      {b->d_ba_pwin, b->ba_pwin.data(), sizeof(int2) * b->ba_pwin.size()},
      {b->d_ba_wlist, b->ba_wlist.data(), sizeof(int2) * b->ba_wlist.size()},
      {b->d_ba_chunks, b->ba_chunks.data(), sizeof(int32_t) * b->ba_chunks.size()},
      {b->d_ba_forder, b->ba_forder.data(), sizeof(int32_t) * b->ba_forder.size()},
      {b->d_split_wins, b->split_wins.data(), sizeof(int2) * b->split_wins.size()},
      {b->d_split_order, b->split_order.data(), sizeof(int32_t) * b->split_order.size()},
      {b->d_nests, b->nests.data(), sizeof(DevNest) * b->nests.size()},
      {b->d_nest_tiles, b->nest_tiles.data(), sizeof(Tile) * b->nest_tiles.size()},
      {b->d_flat_base, b->flat_base.data(), sizeof(int64_t) * size_t(num_pages)},
      {b->d_flat_tiles, b->flat_tiles.data(), sizeof(FlatTile) * b->flat_tiles.size()},
  };
  hipStream_t s = ctx->stream;
  hipError_t e = hipSuccess;
  if (g_defer_tables) {
    size_t total = 0;
    for (const Up& u : ups) total += (u.bytes + 15) & ~size_t(15);
    b->h_tables = pinned_acquire(ctx, total ? total : 16);
    if (!b->h_tables) e = hipErrorOutOfMemory;
    for (size_t i = 0, off = 0; e == hipSuccess && i < sizeof(ups) / sizeof(ups[0]); i++) {
      if (!ups[i].bytes) continue;
      memcpy(b->h_tables.get() + off, ups[i].src, ups[i].bytes);
      b->table_ups.push_back({ups[i].dst, off, ups[i].bytes});
      off += (ups[i].bytes + 15) & ~size_t(15);
    }
  } else {
    for (const Up& u : ups)
      if (e == hipSuccess && u.bytes) e = bounce_h2d(ctx, u.dst, u.src, u.bytes);
  }
  if (e == hipSuccess && num_chunks) e = hipMemsetAsync(b->d_chunk_bytes, 0, sizeof(int64_t) * size_t(num_chunks), s);
  if (e == hipSuccess) e = hipMemsetAsync(b->d_bafuse, 0, sizeof(uint32_t) * 8, s);  // ([4]: k_flat's flag)
  // (deferred tables: nothing to wait for here -- the zero fills stay queued on the context stream and
  // pqh_batch_run_staged orders the copy stream after them; a slot's creation never waits on the GPU)
  if (e == hipSuccess && !g_defer_tables) e = hipStreamSynchronize(s);
  for (hipEvent_t& ev : b->ev_dep)
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  if (e != hipSuccess) {
    free_batch(b);
    delete b;
    return set_err(ctx, PQH_ERR_HIP, std::string("batch upload: ") + hipGetErrorString(e));
  }
  b->stats.resize(kNumKernels);
  for (int k = 0; k < kNumKernels; k++) {
    memset(&b->stats[size_t(k)], 0, sizeof(pqh_kernel_stat));
    snprintf(b->stats[size_t(k)].name, sizeof(b->stats[size_t(k)].name), "%s", kKernelNames[k]);
  }
  *out = b;
  return PQH_OK;
}

namespace {

// Enqueue every kernel of one decode of the batch on stream s (timed with HIP events when prof).
// k_flat (one launch, no workgroup waiting for another; decode.hip): small batches of required
// flat fixed-width columns whose data pages are dictionary, PLAIN fixed / INT96 or PLAIN boolean.
// PQH_FLAT=0 disables it; a failed speculation disables it for the batch.
constexpr size_t kFlatMaxPages = 1024, kFlatMaxTiles = 4096;

bool flat_batch(const pqh_batch* b) {
  const char* f = getenv("PQH_FLAT");
  if ((f && f[0] == '0') || b->flat_off || b->codec_n || b->codec_gzip || b->ba_fuse_on) return false;
  if (!b->delta_pages.empty() || !b->ba_pages.empty() || !b->ba_tiles.empty() || !b->nest_tiles.empty() ||
      !b->global_tiles.empty())
    return false;
  if (b->pages.empty() || b->pages.size() > kFlatMaxPages || b->expand_tiles.size() > kFlatMaxTiles) return false;
  // flat columns, required or nullable (max_def 1: only with V2 pages, whose headers give the
  // speculative notNull and whose levels sit raw at the image's start)
  if (!std::all_of(b->hchunks.begin(), b->hchunks.end(), [](const DevChunk& C) {
        // (INT96 PLAIN chunks too: a page whose short last value is the reference's nil fails the
        // speculation -- flat_spec wants notNull whole values -- and goes through the three
        // kernels, which mark it; a dictionary ending with the nil entry marks from any tile)
        return C.max_rep == 0 && C.max_def <= 1 && C.value_size > 0 && !C.dict_nil;
      }))
    return false;
  return std::all_of(b->hpages.begin(), b->hpages.end(), [&](const DevPage& P) {
    if (P.page_type == PQH_DICTIONARY_PAGE) return true;
    if (b->hchunks[size_t(P.chunk)].max_def > 0 && P.page_type != PQH_DATA_PAGE_V2) return false;
    return P.kind == K_DICT || P.kind == K_PLAIN_FIXED || P.kind == K_PLAIN_INT96 || P.kind == K_PLAIN_BOOL;
  });
}

bool ba_gather_serial();

hipError_t enqueue_run(pqh_batch* b, hipStream_t s, bool prof) {
  DevBatch d{b->d_payload, b->d_pages, b->d_chunks, b->d_states, b->d_ckpts, int32_t(b->pages.size()),
             int32_t(b->chunks.size()), b->d_dstates, b->d_dblocks, b->d_dsums, b->d_dcum, b->d_basums,
             b->d_chunk_bytes, b->d_nests, b->d_nsums, b->d_basums2, b->d_bafuse, b->d_bawords,
             b->split_on ? b->d_dsplit : nullptr, b->d_dticket, b->d_dwords};
  const bool sync_each = sync_each_enabled();
  auto timed = [&](int kind, int32_t items, hipStream_t st, auto&& fn) -> hipError_t {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (prof) {
      e0 = next_event(b);
      e1 = next_event(b);
      hipEventRecord(e0, st);
    }
    hipError_t e = fn(st);
    if (prof) {
      hipEventRecord(e1, st);
      b->pending.push_back(KernelRun{kind, e0, e1, items});
    }
    if (sync_each) {  // debugging: name the kernel whose launch or execution fails
      if (e == hipSuccess) e = hipStreamSynchronize(st);
      if (e == hipSuccess) e = hipGetLastError();
      if (e != hipSuccess) g_fail_kernel = kKernelNames[kind];
    }
    return e;
  };
  hipError_t e = hipSuccess;
  // Unprofiled runs put two independent branches on the context's side stream, beside the main
  // sequence: the PLAIN byte-array chain (k_ba_wspec / wstitch / wemit read only the prologue's
  // page states; latency bound, so it overlaps the bandwidth-bound kernels) and the nesting kernels
  // (read only the levels k_expand wrote; they overlap the byte-array copies).  Both rejoin before
  // anything that reads their results.  Profiled and synchronised runs stay on one stream, so every
  // kernel is timed alone.
  const char* fk = getenv("PQH_FORK");
  hipStream_t side = (!prof && !sync_each && b->ctx->side && !(fk && fk[0] == '0')) ? b->ctx->side : nullptr;
  auto dep = [&](hipStream_t from, hipStream_t to, int k) -> hipError_t {  // `to` waits for `from`'s work so far
    hipError_t r = hipEventRecord(b->ev_dep[k], from);
    return r == hipSuccess ? hipStreamWaitEvent(to, b->ev_dep[k], 0) : r;
  };
  const int32_t ndp = int32_t(b->delta_pages.size()), ndt = int32_t(b->delta_tiles.size());
  b->flat_on = flat_batch(b);
  if (b->flat_on)
    return timed(30, int32_t(b->expand_tiles.size()), s, [&](hipStream_t st) {
      return launch_flat(d, b->d_flat_tiles, int32_t(b->flat_tiles.size()), b->d_flat_base, b->d_bafuse + 4,
                         b->expand_lds, st);
    });
  if (b->codec_n) {  // device codecs: the page images first
    if (snappy_page_mode()) {
      e = timed(22, b->codec_n, s, [&](hipStream_t st) {
        return launch_snappy(b->d_codec, b->codec_n, static_cast<const uint8_t*>(b->d_src),
                             static_cast<uint8_t*>(b->owned_payload), b->d_codec_status, st);
      });
    } else {
      // the multi-workgroup pipeline kernel by kernel (k_snappy = its page-mode pages), each timed
      const int32_t items[5] = {b->snap.n_page_mode, b->snap.n_win, b->codec_n, b->snap.n_unit, b->codec_n};
      for (int part = 0; part < 5 && e == hipSuccess; part++)
        e = timed(part == 0 ? 22 : 24 + part, items[part], s, [&](hipStream_t st) {
          return launch_snappy_mw(b->d_codec, b->snap, static_cast<const uint8_t*>(b->d_src),
                                  static_cast<uint8_t*>(b->owned_payload), b->d_codec_status, st, part);
        });
    }
  }
  if (e == hipSuccess && b->codec_gzip)
    e = timed(24, b->codec_gzip, s, [&](hipStream_t st) {
      return launch_gzip(b->d_codec, b->codec_n, static_cast<const uint8_t*>(b->d_src),
                         static_cast<uint8_t*>(b->owned_payload), b->d_codec_status, st);
    });
  // repeated columns carry long level streams: a workgroup per page splits their notNull count
  const bool wide = std::any_of(b->hchunks.begin(), b->hchunks.end(), [](const DevChunk& c) { return c.max_rep > 0; });
  if (e == hipSuccess && b->ba_fuse_on) {  // fused chains: tickets, fallback flag (k_scan's too), look-back words
    e = hipMemsetAsync(b->d_bafuse, 0, sizeof(uint32_t) * 2, s);
    if (e == hipSuccess)
      e = hipMemsetAsync(b->d_bawords, 0, sizeof(uint64_t) * (b->ba_wins.size() - size_t(b->ba_wins_nf)), s);
  }
  if (e == hipSuccess)
    e = timed(0, int32_t(b->pages.size()), s, [&](hipStream_t st) { return launch_prologue(d, wide, st); });
  // (while the fused chains are on, the scratch path covers the lists' non-fused prefixes)
  const bool fuse = b->ba_fuse_on;
  const int32_t nbp = fuse ? b->ba_pages_nf : int32_t(b->ba_pages.size()), nbt = int32_t(b->ba_tiles.size()),
                nbc = fuse ? b->ba_chunks_nf : int32_t(b->ba_chunks.size());
  // fused PLAIN chains: compute bound (chain resolution), so they run on a stream of their own
  // beside the rest; launched after k_scan, whose page byte bases they use
  const int32_t nfw = fuse ? int32_t(b->ba_wins.size()) - b->ba_wins_nf : 0;
  bool fuse_open = false;
  auto launch_fused = [&]() -> hipError_t {
    hipError_t r = hipSuccess;
    hipStream_t fs = s;
    hipStream_t side2 = side ? b->ctx->side2 : nullptr;
    if (side2) {
      r = dep(s, side2, 4);
      fs = side2;
      fuse_open = true;
    }
    if (r == hipSuccess)
      r = timed(29, nfw, fs, [&](hipStream_t st) {
        return launch_ba_chain(d, b->d_ba_wins + b->ba_wins_nf, b->d_ba_forder, nfw, st);
      });
    return r;
  };
  bool chain_open = false;  // the chain branch has not rejoined the main stream yet
  if (e == hipSuccess && nbp) {
    hipStream_t cs = s;
    if (side) {
      e = dep(s, side, 0);
      cs = side;
      chain_open = true;
    }
    const int32_t nw = fuse ? b->ba_wins_nf : int32_t(b->ba_wins.size());
    if (e == hipSuccess)
      e = timed(7, nw, cs, [&](hipStream_t st) { return launch_ba_wspec(d, b->d_ba_wins, nw, b->d_ba_res, b->d_ba_wrec, st); });
    if (e == hipSuccess)
      e = timed(20, nbp, cs, [&](hipStream_t st) {
        return launch_ba_wstitch(d, b->d_ba_pages, b->d_ba_pwin, nbp, b->d_ba_res, b->d_ba_wrec, st);
      });
    if (e == hipSuccess && b->ba_wdict)
      e = timed(21, b->ba_wdict, cs, [&](hipStream_t st) {
        return launch_ba_wemit(d, b->d_ba_wlist, b->ba_wdict, b->d_ba_res, b->d_ba_wrec, st);
      });
    if (e == hipSuccess && side) e = hipEventRecord(b->ev_dep[1], side);
  }
  auto join_chain = [&]() -> hipError_t {
    if (!chain_open) return hipSuccess;
    chain_open = false;
    return hipStreamWaitEvent(s, b->ev_dep[1], 0);
  };
  // page mode: every delta page gets its init errors now and is chased, decoded and walked after
  // the value scan; tile mode: speculative walk + exact walk now, tiles after the scan
  const int32_t ni = b->delta_page_mode ? b->delta_fused_pages : 0;
  if (e == hipSuccess && ni)
    e = timed(18, ni, s, [&](hipStream_t st) { return launch_delta_init(d, b->d_delta_pages, ni, st); });
  if (e == hipSuccess && ndp > ni)
    e = timed(16, ndp - ni, s, [&](hipStream_t st) { return launch_delta_spec(d, b->d_delta_pages + ni, ndp - ni, st); });
  if (e == hipSuccess && ndp > ni)
    e = timed(4, ndp - ni, s, [&](hipStream_t st) { return launch_delta_walk(d, b->d_delta_pages + ni, ndp - ni, st); });
  if (e == hipSuccess) e = timed(1, int32_t(b->chunks.size()), s, [&](hipStream_t st) { return launch_scan(d, st); });
  if (e == hipSuccess && nfw) e = launch_fused();
  // the DELTA pages' decode (latency / ALU bound) runs beside k_expand's fixed-width and level tiles
  // (bandwidth bound) on a stream of its own when the batch has both; it rejoins before the
  // byte-array kernels, which read DELTA_LENGTH lengths, and at the end
  hipStream_t ds = s;
  bool delta_open = false;
  if (e == hipSuccess && side && ndp && !b->expand_tiles.empty()) {
    e = dep(s, b->ctx->side3, 6);
    ds = b->ctx->side3;
    delta_open = true;
  }
  if (e == hipSuccess && ni && b->split_on) {
    const int32_t nw = int32_t(b->split_order.size());
    e = hipMemsetAsync(b->d_dticket, 0, sizeof(uint32_t) * 2, ds);
    if (e == hipSuccess) e = hipMemsetAsync(b->d_dwords, 0, sizeof(uint64_t) * 3 * b->split_wins.size(), ds);
    if (e == hipSuccess)
      e = timed(32, nw, ds, [&](hipStream_t st) {
        return launch_delta_split(d, b->d_split_wins, b->d_split_order, nw, b->split_nl, st);
      });
    if (e == hipSuccess)
      e = timed(4, ni, ds, [&](hipStream_t st) { return launch_delta_walk(d, b->d_delta_pages, ni, st); });
  } else if (e == hipSuccess && ni) {
    const int32_t nis = b->delta_fused_streams;
    e = timed(19, nis, ds, [&](hipStream_t st) { return launch_delta_fused(d, b->d_dtiles, nis, b->delta_lens_streams, st); });
    if (e == hipSuccess)
      e = timed(4, ni, ds, [&](hipStream_t st) { return launch_delta_walk(d, b->d_delta_pages, ni, st); });
  }
  if (e == hipSuccess && ndt && b->delta_page_mode) {
    const int32_t nds = int32_t(b->delta_streams.size());
    e = timed(17, nds, ds, [&](hipStream_t st) { return launch_delta_page(d, b->d_dtiles, nds, st); });
  } else if (e == hipSuccess && ndt) {
    e = timed(6, ndt, ds, [&](hipStream_t st) { return launch_delta_sum(d, b->d_dtiles, ndt, st); });
    if (e == hipSuccess)
      e = timed(6, ndp, ds, [&](hipStream_t st) { return launch_delta_scan(d, b->d_delta_pages, ndp, st); });
    if (e == hipSuccess) e = timed(5, ndt, ds, [&](hipStream_t st) { return launch_delta_expand(d, b->d_dtiles, ndt, st); });
  }
  if (e == hipSuccess && ndp)  // pages outside the fast-path geometry (most launches exit at once)
    e = timed(14, ndp, ds, [&](hipStream_t st) { return launch_delta_serial(d, b->d_delta_pages, ndp, st); });
  auto join_delta = [&]() -> hipError_t {
    if (!delta_open) return hipSuccess;
    delta_open = false;
    return dep(b->ctx->side3, s, 7);
  };
  // byte-array dictionary keys are checked against the dictionary sizes the chain branch found
  if (e == hipSuccess && b->ba_wdict) e = join_chain();
  const int32_t ne = int32_t(b->expand_tiles.size()), ng = int32_t(b->global_tiles.size());
  const int32_t nl = b->expand_lev_n;  // the nested chunks' level tiles (their own launch, first)
  const int32_t nnt = int32_t(b->nest_tiles.size()), nns = int32_t(b->nests.size());
  bool nest_open = false;
  auto launch_nesting = [&]() -> hipError_t {  // nesting: the levels are complete
    hipError_t r = hipSuccess;
    hipStream_t ns = s;
    if (side) {
      r = dep(s, side, 2);
      ns = side;
      nest_open = true;
    }
    // count / scan / write passes (a one-pass write with look-back bases measured slower: DESIGN §5)
    if (r == hipSuccess)
      r = timed(11, nnt, ns, [&](hipStream_t st) { return launch_nest_count(d, b->d_nest_tiles, nnt, st); });
    if (r == hipSuccess) r = timed(12, nns, ns, [&](hipStream_t st) { return launch_nest_scan(d, nns, st); });
    if (r == hipSuccess)
      r = timed(13, nnt, ns, [&](hipStream_t st) { return launch_nest_write(d, b->d_nest_tiles, nnt, st); });
    return r;
  };
  if (e == hipSuccess && nl)
    e = timed(31, nl, s, [&](hipStream_t st) { return launch_expand(d, b->d_tiles, nl, b->expand_lds, st); });
  if (e == hipSuccess && nnt && nl) e = launch_nesting();
  if (e == hipSuccess && ne > nl)
    e = timed(2, ne - nl, s, [&](hipStream_t st) { return launch_expand(d, b->d_tiles + nl, ne - nl, b->expand_lds, st); });
  if (e == hipSuccess && ng)
    e = timed(3, ng, s, [&](hipStream_t st) { return launch_dict_global(d, b->d_tiles + ne, ng, st); });
  if (e == hipSuccess && nnt && !nl) e = launch_nesting();
  if (e == hipSuccess) e = join_chain();  // byte sums and limits of the PLAIN pages
  if (e == hipSuccess) e = join_delta();  // DELTA_LENGTH lengths
  if (e == hipSuccess && nbt) {
    const int32_t nsum = fuse ? b->ba_sum_nf : int32_t(b->ba_xlist.size()) - b->ba_sum_off;
    e = timed(8, nsum, s, [&](hipStream_t st) {
      return launch_ba_sum(d, b->d_batiles, b->d_ba_xlist + b->ba_sum_off, nsum, b->delta_page_mode, st);
    });
    if (e == hipSuccess)
      e = timed(9, nbc, s, [&](hipStream_t st) { return launch_ba_scan(d, b->d_ba_chunks, nbc, b->d_batiles, st); });
    // k_ba_expand (DELTA_LENGTH / FLBA tiles) and k_ba_gather (dictionary / PLAIN tiles) write
    // disjoint tiles: with both present the gathers run beside the copies on the third side stream
    // (free again: the DELTA branch rejoined above) -- C5's dictionary pages no longer wait for its
    // DELTA_LENGTH copy (0.806 -> 0.792 ms, same box).  Not while the nesting or fused-chain branches
    // are still open: with four streams busy the step varied (C4 1.22-1.38 vs 1.22 ms)
    const int32_t ncp = b->ba_ncopy, ngt = b->ba_sum_off - b->ba_ncopy;
    hipStream_t gs = side && b->ctx->side3 && ncp > 0 && ngt > 0 && !nest_open && !fuse_open && !ba_gather_serial()
                         ? b->ctx->side3 : nullptr;
    if (e == hipSuccess && gs) {
      e = dep(s, gs, 8);
      if (e == hipSuccess)
        e = timed(10, ngt, gs, [&](hipStream_t st) {
          return launch_ba_expand(d, b->d_batiles, b->d_ba_xlist + ncp, 0, ngt, st);
        });
      if (e == hipSuccess)
        e = timed(10, ncp, s, [&](hipStream_t st) { return launch_ba_expand(d, b->d_batiles, b->d_ba_xlist, ncp, 0, st); });
      if (e == hipSuccess) e = dep(gs, s, 9);
    } else if (e == hipSuccess) {
      e = timed(10, nbt, s, [&](hipStream_t st) {  // k_ba_expand + k_ba_gather
        return launch_ba_expand(d, b->d_batiles, b->d_ba_xlist, ncp, ngt, st);
      });
    }
    const int32_t nwd = (fuse ? b->ba_wlist_nf : int32_t(b->ba_wlist.size())) - b->ba_wdict;
    if (e == hipSuccess && nwd)
      e = timed(23, nwd, s, [&](hipStream_t st) {
        return launch_ba_wcopy(d, b->d_ba_wlist + b->ba_wdict, nwd, b->d_ba_res, b->d_ba_wrec, b->d_ba_wgeo, st);
      });
    if (e == hipSuccess && b->has_dba)
      e = timed(15, nbt, s, [&](hipStream_t st) { return launch_dba_prefix(d, b->d_batiles, nbt, st); });
  }
  // rejoin whatever is still open (also after a failed launch, so the main stream's sync covers it)
  if (chain_open) {
    const hipError_t r = join_chain();
    if (e == hipSuccess) e = r;
  }
  if (nest_open) {
    const hipError_t r = dep(side, s, 3);
    if (e == hipSuccess) e = r;
  }
  if (fuse_open) {
    const hipError_t r = dep(b->ctx->side2, s, 5);
    if (e == hipSuccess) e = r;
  }
  if (delta_open) {
    const hipError_t r = join_delta();
    if (e == hipSuccess) e = r;
  }
  return e;
}

// (after sync) the end of page p's length stream(s): DELTA_LENGTH -> its one stream, DELTA_BYTE_ARRAY
// -> the suffix lengths that follow the prefix lengths; val_s when unknown
int64_t dlen_end(const pqh_batch* b, size_t p) {
  const DevPage& P = b->hpages[p];
  const size_t i = P.kind == K_DBA ? b->pages.size() + p : p;
  return i < b->hdstates.size() && b->hdstates[i].end_pos > 0 ? b->hdstates[i].end_pos : b->states[p].val_s;
}

// PQH_BA_GATHER_SERIAL=1: k_ba_gather after k_ba_expand on one stream (the A/B baseline)
bool ba_gather_serial() {
  const char* g = getenv("PQH_BA_GATHER_SERIAL");
  return g && g[0] == '1';
}

bool graphs_enabled() {
  const char* g = getenv("PQH_GRAPH");
  return !(g && g[0] == '0') && !sync_each_enabled();
}

}  // namespace

// A batch's launch sequence is fixed at plan time, so unprofiled runs replay it as one hipGraph
// (captured on the first such run): one submission instead of one per kernel.  Profiled runs
// launch directly, with HIP events around every kernel.
int pqh_batch_run(pqh_batch* b) {
  if (!b) return set_err(nullptr, PQH_ERR_ARG, "null batch");
  pqh_ctx* ctx = b->ctx;
  hipSetDevice(ctx->device);
  const bool prof = (ctx->flags & PQH_CTX_PROFILE) != 0;
  hipStream_t s = ctx->stream;
  b->synced = false;
  hipError_t e = hipSuccess;
  for (const auto& u : b->table_ups)  // a staged batch run without pqh_batch_run_staged: its tables now
    HIP_TRY(ctx, hipMemcpyAsync(u.dst, b->h_tables.get() + u.off, u.bytes, hipMemcpyHostToDevice, s));
  b->table_ups.clear();
  // a k_flat batch is one kernel: launched directly (C1: 0.0126 ms per step against 0.0178 ms as a
  // one-node graph replay, same box -- the replay adds ~6 us per step)
  if (!prof && graphs_enabled() && !b->graph_failed && !flat_batch(b) && !(ctx->flags & PQH_CTX_STREAMING)) {
    if (!b->gexec) {
      e = hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
      if (e == hipSuccess) {
        const hipError_t le = enqueue_run(b, s, false);
        hipGraph_t g = nullptr;
        e = hipStreamEndCapture(s, &g);
        if (e == hipSuccess) e = le;
        if (e == hipSuccess) e = hipGraphInstantiate(&b->gexec, g, nullptr, nullptr, 0);
        b->graph = g;
      }
      if (e != hipSuccess) {  // replay unavailable: launch directly from now on
        (void)hipGetLastError();
        if (b->gexec) hipGraphExecDestroy(b->gexec);
        if (b->graph) hipGraphDestroy(b->graph);
        b->gexec = nullptr;
        b->graph = nullptr;
        b->graph_failed = true;
      }
    }
    e = b->gexec ? hipGraphLaunch(b->gexec, s) : enqueue_run(b, s, false);
  } else {
    g_fail_kernel = nullptr;
    e = enqueue_run(b, s, prof);
  }
  if (e != hipSuccess)
    return set_err(ctx, PQH_ERR_HIP, std::string("launch") + (g_fail_kernel ? std::string(" ") + g_fail_kernel : "") +
                                         ": " + hipGetErrorString(e));
  return PQH_OK;
}

int pqh_batch_sync(pqh_batch* b) {
  if (!b) return set_err(nullptr, PQH_ERR_ARG, "null batch");
  pqh_ctx* ctx = b->ctx;
  hipSetDevice(ctx->device);
  b->states.resize(b->pages.size());
  if (!b->pages.empty()) HIP_TRY(ctx, bounce_d2h(ctx, b->states.data(), b->d_states, sizeof(PageState) * b->pages.size()));
  b->chunk_bytes.assign(b->chunks.size(), 0);
  if (!b->ba_chunks.empty())
    HIP_TRY(ctx, bounce_d2h(ctx, b->chunk_bytes.data(), b->d_chunk_bytes, sizeof(int64_t) * b->chunks.size()));
  b->nest_totals.assign(b->nests.size() * kNestFlags, 0);
  if (!b->nests.empty())
    HIP_TRY(ctx, bounce_d2h(ctx, b->nest_totals.data(), b->d_ntotals, sizeof(int64_t) * b->nest_totals.size()));
  b->codec_status.assign(size_t(b->codec_n), PQH_OK);
  if (b->codec_n)
    HIP_TRY(ctx, bounce_d2h(ctx, b->codec_status.data(), b->d_codec_status, sizeof(int32_t) * size_t(b->codec_n)));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  if ((ctx->flags & PQH_CTX_STREAMING) && arena_check()) {
    const int rc = arena_verify(ctx);
    if (rc) return rc;
  }
  // k_flat's speculation failed (a page not clean and simple, a key out of range): decode the batch
  // again through the three kernels, and keep it there
  if (b->flat_on) {
    uint32_t flag = 0;
    HIP_TRY(ctx, bounce_d2h(ctx, &flag, b->d_bafuse + 4, sizeof(uint32_t)));
    if (flag) {
      b->flat_on = false;
      b->flat_off = true;
      b->flat_fallbacks++;
      HIP_TRY(ctx, hipMemsetAsync(b->d_bafuse + 4, 0, sizeof(uint32_t), ctx->stream));
      if (b->gexec) hipGraphExecDestroy(b->gexec);
      if (b->graph) hipGraphDestroy(b->graph);
      b->gexec = nullptr;
      b->graph = nullptr;
      b->pending.clear();
      b->event_next = 0;
      int rc = pqh_batch_run(b);
      if (rc != PQH_OK) return rc;
      return pqh_batch_sync(b);
    }
  }
  // The per-page results bound every later copy of the outputs (pqh_batch_chunk_out): refuse
  // results that would reach past the planned output buffers instead of handing them out.
  for (size_t p = 0; p < b->pages.size(); p++) {
    const DevPage& P = b->hpages[p];
    const PageState& S = b->states[p];
    if (P.page_type == PQH_DICTIONARY_PAGE) continue;
    const int64_t n = std::max(0, P.num_values);
    if (S.nn < 0 || S.nn > n || S.value_base < 0 || S.value_base + S.nn > b->hchunks[size_t(P.chunk)].values_cap) {
      char msg[160];
      snprintf(msg, sizeof(msg), "device page state out of range: page %zu nn %d of %lld, value_base %lld", p, S.nn,
               (long long)n, (long long)S.value_base);
      return set_err(ctx, PQH_ERR_HIP, msg);
    }
  }
  // Fused PLAIN chains that did not verify (an error, trailing bytes, a chain that ends early):
  // decode the batch again on the scratch path, which gives the reference's errors and limits
  if (b->ba_fuse_on) {
    uint32_t flag = 0;
    HIP_TRY(ctx, bounce_d2h(ctx, &flag, b->d_bafuse + 1, sizeof(uint32_t)));
    if (flag) {
      b->ba_fuse_on = false;
      b->ba_fuse_fallbacks++;
      for (DevChunk& D : b->hchunks) D.ba_fused = 0;
      HIP_TRY(ctx, bounce_h2d(ctx, b->d_chunks, b->hchunks.data(), sizeof(DevChunk) * b->hchunks.size()));
      if (b->gexec) hipGraphExecDestroy(b->gexec);
      if (b->graph) hipGraphDestroy(b->graph);
      b->gexec = nullptr;
      b->graph = nullptr;
      b->pending.clear();
      b->event_next = 0;
      int rc = pqh_batch_run(b);
      if (rc != PQH_OK) return rc;
      return pqh_batch_sync(b);
    }
  }
  // Byte-array outputs sized from an estimate (dictionary gathers): grow the chunks that came out
  // short (and decoded without error), then decode again.  Contents are deterministic, so this
  // happens at most once per batch.
  // A chunk with a failing page needs (and gets) the bytes of the pages before it: what NextRow reads
  // before it meets the error (data_store.go:236-260); the sums at and after a failing page may be
  // garbage, so they never size an allocation.
  bool regrow = false;
  for (int32_t c : b->ba_chunks) {
    DevChunk& D = b->hchunks[size_t(c)];
    if (b->chunk_bytes[size_t(c)] <= D.bytes_cap) continue;
    int64_t cap = b->chunk_bytes[size_t(c)];
    for (int32_t i = 0; i < D.num_pages; i++) {
      const PageState& S = b->states[size_t(D.first_page + i)];
      if (S.err == kNoError) continue;
      cap = 0;  // offsets[value_base of the failing page] = the bytes before it
      if (S.value_base > 0) HIP_TRY(ctx, bounce_d2h(ctx, &cap, D.offsets + S.value_base, sizeof(int64_t)));
      break;
    }
    if (cap <= D.bytes_cap) continue;
    void* np = nullptr;
    HIP_TRY(ctx, dev_alloc(ctx, &np, size_t(cap) + 64));
    for (auto& a : b->allocations)
      if (a == D.bytes) {
        dev_free(ctx, a);
        a = np;
      }
    D.bytes = static_cast<uint8_t*>(np);
    D.bytes_cap = cap;
    regrow = true;
  }
  if (regrow) {
    b->regrows++;
    HIP_TRY(ctx, bounce_h2d(ctx, b->d_chunks, b->hchunks.data(), sizeof(DevChunk) * b->hchunks.size()));
    int rc = pqh_batch_run(b);
    if (rc != PQH_OK) return rc;
    return pqh_batch_sync(b);
  }
  // the reference's nil INT96 values: per page and chunk counts of the value_nil marks, among the
  // values the reference returns (an error page's values before its val_limit; none after a
  // dictionary key error, which returns 0 values, type_dict.go:52-54).  A PLAIN page holds at most
  // one, its short last value, which k_scan marks exactly when the page decoded with val_limit =
  // notNull - 1 -- known from the states; only chunks whose dictionary ends with the nil entry
  // (dict_nil: any value may index it) read their marks back.
  b->page_nil.assign(b->pages.size(), 0);
  b->chunk_nil.assign(b->chunks.size(), 0);
  for (size_t c = 0; c < b->hchunks.size(); c++) {
    const DevChunk& D = b->hchunks[c];
    if (!D.value_nil || D.values_cap <= 0) continue;
    for (int32_t i = 0; i < D.num_pages; i++) {
      const int32_t p = D.first_page + i;
      const PageState& S = b->states[size_t(p)];
      const DevPage& P = b->hpages[size_t(p)];
      if (P.page_type == PQH_DICTIONARY_PAGE || S.nn <= 0 || S.value_base < 0 || S.value_base + S.nn > D.values_cap)
        continue;
      int32_t k = 0;
      if (P.kind == K_PLAIN_INT96) {
        k = S.err == kNoError && S.val_limit == S.nn - 1 ? 1 : 0;
      } else if (P.kind == K_DICT && D.dict_nil && (S.err & 0xff) != PQH_ERR_DICT_INDEX) {
        const int64_t m = S.err == kNoError ? S.nn : std::min<int64_t>(std::max(S.val_limit, 0), S.nn);
        if (m > 0) {
          std::vector<uint8_t> marks(static_cast<size_t>(m));
          HIP_TRY(ctx, bounce_d2h(ctx, marks.data(), D.value_nil + S.value_base, marks.size()));
          for (uint8_t x : marks) k += x != 0;
        }
      }
      b->page_nil[size_t(p)] = k;
      b->chunk_nil[c] += k;
    }
  }
  for (auto& r : b->pending) {
    float ms = 0;
    if (hipEventElapsedTime(&ms, r.start, r.stop) == hipSuccess) {
      pqh_kernel_stat& st = b->stats[size_t(r.kind)];
      st.launches += 1;
      st.work_items = r.items;
      st.total_ms += ms;
    }
  }
  b->pending.clear();
  b->event_next = 0;
  // algorithmic bytes of one run: page bytes read once, dictionaries once per
  // chunk, decoded bytes written; attributed to the kernel that moves them.
  // (where each DELTA_LENGTH / DELTA_BYTE_ARRAY page's length streams end: the byte accounting splits
  // those pages between the delta kernels and k_ba_expand)
  const bool lens = std::any_of(b->hpages.begin(), b->hpages.end(),
                                [](const DevPage& P) { return P.kind == K_DLBA || P.kind == K_DBA; });
  b->hdstates.clear();
  if (lens && !b->pages.empty()) {
    b->hdstates.resize(2 * b->pages.size());
    HIP_TRY(ctx, bounce_d2h(ctx, b->hdstates.data(), b->d_dstates, sizeof(DeltaState) * b->hdstates.size()));
  }
  double wr = 0, plain_written = 0;
  auto fused_chunk = [&](int32_t c) { return b->ba_fuse_on && b->hchunks[size_t(c)].ba_fused != 0; };
  std::fill(b->k_read.begin(), b->k_read.end(), 0.0);
  std::fill(b->k_written.begin(), b->k_written.end(), 0.0);
  for (size_t p = 0; p < b->pages.size(); p++) {
    const DevPage& P = b->hpages[p];
    const PageState& S = b->states[p];
    const DevChunk& C = b->hchunks[size_t(P.chunk)];
    if (P.page_type == PQH_DICTIONARY_PAGE) continue;
    const double n = P.num_values > 0 ? P.num_values : 0;
    const double levels = (C.max_def > 0 ? n : 0) + (C.max_rep > 0 ? n : 0);
    const double vals = double(S.nn) * P.value_size;
    // (fixed-width pages of a chunk laid out as byte arrays: their output is counted with the chunk's bytes)
    wr += levels + (C.value_size > 0 ? vals : 0.0);
    // everything after the prologue is moved by k_expand (or k_dict_global for large dictionaries)
    const int kx = (P.kind == K_DICT && P.dict_page >= 0 &&
                    int64_t(std::max(0, b->pages[size_t(P.dict_page)].num_values)) * P.value_size > kDictLdsMax)
                       ? 3 : 2;
    if (levels > 0) {
      double lb = 0;
      if (S.rep_s >= 0) lb += S.rep_e - S.rep_s;
      if (S.def_s >= 0) lb += S.def_e - S.def_s;
      const int kl = b->expand_lev_n && b->chunk_nest[size_t(P.chunk)] >= 0 ? 31 : 2;  // (k_expand_lev's tiles)
      b->k_read[kl] += lb;
      b->k_written[kl] += levels;
    }
    switch (P.kind) {
      case K_PLAIN_FIXED:
      case K_PLAIN_INT96:
        b->k_read[2] += vals;
        b->k_written[2] += vals;
        break;
      case K_PLAIN_BOOL:
        b->k_read[2] += (S.nn + 7) / 8;
        b->k_written[2] += S.nn;
        break;
      case K_DICT:
        b->k_read[kx] += S.val_e - S.val_s;
        b->k_written[kx] += vals;
        break;
      case K_RLE_BOOL:
        b->k_read[2] += S.val_e - S.val_s;
        b->k_written[2] += S.nn;
        break;
      case K_DELTA32:
      case K_DELTA64: {  // the walks read block headers; k_delta_expand / k_delta_page read the stream once
        const int kd = b->delta_page_mode ? (b->split_on ? 32 : 19) : 5;
        b->k_read[kd] += S.val_e - S.val_s;
        b->k_written[kd] += vals;
        break;
      }
      case K_PLAIN_BA: {  // walked by k_ba_wspec / k_ba_wstitch; values read and offsets + bytes written by
                          // k_ba_wcopy -- or all of it by k_ba_chain
        const int kx = fused_chunk(P.chunk) ? 29 : 23;
        b->k_read[kx] += S.val_e - S.val_s;
        if (S.err == kNoError) {
          const double w = double(S.nn) * 8 + double(S.val_e - S.val_s - 4 * int64_t(S.nn));
          b->k_written[kx] += w;
          if (kx == 23) plain_written += w;
        }
        break;
      }
      case K_DLBA:
      case K_DBA: {  // the length streams read by the delta kernels, the string bytes by k_ba_expand
        const int kd = b->delta_page_mode ? (b->split_on ? 32 : 19) : 5;
        const int64_t le = std::min<int64_t>(std::max<int64_t>(dlen_end(b, p), S.val_s), S.val_e);
        b->k_read[kd] += le - S.val_s;
        b->k_read[10] += S.val_e - le;
        break;
      }
      default:
        break;
    }
  }
  for (size_t c = 0; c < b->hchunks.size(); c++) {  // dictionaries once per chunk
    const DevChunk& C = b->hchunks[c];
    if (C.dict_page < 0) continue;
    const pqh_page& Q = b->pages[size_t(C.dict_page)];
    b->k_read[int64_t(std::max(0, Q.num_values)) * b->hpages[size_t(C.dict_page)].value_size > kDictLdsMax ? 3 : 2] +=
        Q.image_len;
  }
  for (int32_t c : b->ba_chunks) {  // offsets (8 B per value + 1) and string bytes, written by k_ba_expand
    const DevChunk& C = b->hchunks[size_t(c)];
    int64_t nn = 0;
    for (int32_t i = 0; i < C.num_pages; i++)
      if (b->hpages[size_t(C.first_page + i)].page_type != PQH_DICTIONARY_PAGE) nn += b->states[size_t(C.first_page + i)].nn;
    const double w = double(nn + 1) * 8 + double(b->chunk_bytes[size_t(c)]);
    wr += w;
    if (fused_chunk(c)) b->k_written[29] += 8;  // (its pages' offsets and bytes are counted above)
    else b->k_written[10] += w;
  }
  b->k_written[10] -= plain_written;  // the PLAIN pages' share went to k_ba_wcopy
  for (size_t i = 0; i < b->nests.size(); i++) {  // list offsets (4 B) + presence (1 B) per list, leaf validity
    const DevNest& N = b->nests[i];
    double w = 0;
    for (int l = 0; l < N.levels; l++) w += double(b->nest_totals[i * kNestFlags + size_t(l)] + 1) * 4 +
                                          double(b->nest_totals[i * kNestFlags + size_t(l)]);
    if (N.leaf) w += double(b->nest_totals[i * kNestFlags + size_t(N.levels)]);
    wr += w;
    b->k_written[13] += w;
    if (N.lbase == 0) b->k_read[13] += 2.0 * double(N.n);  // (the algorithmic bytes read the levels once)
  }
  b->bytes_written = wr;
  if (b->flat_on) {  // k_flat moved k_expand's bytes
    b->k_read[30] += b->k_read[2];
    b->k_written[30] += b->k_written[2];
    b->k_read[2] = b->k_written[2] = 0;
  }
  for (int k = 0; k < kNumKernels; k++) {
    b->stats[size_t(k)].bytes_read = b->k_read[size_t(k)];
    b->stats[size_t(k)].bytes_written = b->k_written[size_t(k)];
  }
  b->synced = true;
  return PQH_OK;
}

int pqh_batch_page_results(const pqh_batch* b, pqh_page_result* out, int32_t num_pages) {
  if (!b || !b->synced) return set_err(b ? b->ctx : nullptr, PQH_ERR_ARG, "batch not synced");
  for (int32_t p = 0; p < num_pages && size_t(p) < b->pages.size(); p++) {
    const PageState& S = b->states[size_t(p)];
    pqh_page_result& r = out[p];
    memset(&r, 0, sizeof(r));
    if (size_t(p) < b->codec_status.size() && b->codec_status[size_t(p)] != PQH_OK) {
      // the device could not decompress its image (readPageBlock), or a codec guard fired (INTERNAL)
      r.status = b->codec_status[size_t(p)] == PQH_ERR_INTERNAL ? PQH_ERR_INTERNAL : PQH_ERR_DECOMPRESS;
      r.phase = PQH_PHASE_LOAD;
    } else if (S.err != kNoError) {
      r.status = int32_t(S.err & 0xff);
      r.phase = int32_t(S.err >> 56);
      r.index = int64_t((S.err >> 8) & 0xffffffffffffull);
    }
    r.num_non_null = S.nn;
    r.num_nil = size_t(p) < b->page_nil.size() ? b->page_nil[size_t(p)] : 0;
    r.value_offset = S.value_base;
    r.level_offset = b->hpages[size_t(p)].level_base;
  }
  return PQH_OK;
}

// readValues(size) of one page as the reference's pageReader returns it (page_v1.go:33-63,
// page_v2.go:31-60), materialised in host memory from the batch's device outputs: level slots
// [first, first + count) of the page, their definition / repetition levels and the dense values of
// the non-null ones.  Sizes only when the buffers are NULL.
int pqh_batch_page_read(const pqh_batch* b, int32_t page, int64_t first, int64_t count, void* values,
                        int64_t values_cap, int64_t* offsets, int64_t offsets_cap, uint8_t* data, int64_t data_cap,
                        uint8_t* def_levels, uint8_t* rep_levels, uint8_t* value_nil, int64_t value_nil_cap,
                        pqh_page_values* out) {
  if (!b || !out || page < 0 || size_t(page) >= b->pages.size() || first < 0 || count < 0)
    return set_err(b ? b->ctx : nullptr, PQH_ERR_ARG, "bad page read arguments");
  if (!b->synced) return set_err(b->ctx, PQH_ERR_ARG, "batch not synced");
  pqh_ctx* ctx = b->ctx;
  hipSetDevice(ctx->device);
  memset(out, 0, sizeof(*out));
  const DevPage& P = b->hpages[size_t(page)];
  const PageState& S = b->states[size_t(page)];
  const DevChunk& C = b->hchunks[size_t(P.chunk)];
  out->value_size = C.value_size;
  if (P.page_type == PQH_DICTIONARY_PAGE) return set_err(ctx, PQH_ERR_ARG, "dictionary pages have no readValues");
  const int64_t n = std::max(0, P.num_values);
  // dataPageReaderV1/V2.readValues: size is clipped to the values left in the page
  const int64_t s0 = std::min(first, n), s1 = std::min(n, s0 + count);
  out->num_slots = s1 - s0;
  const ChunkErr ce = chunk_error(b, P.chunk);
  if (ce.status != PQH_OK && ce.phase == PQH_PHASE_LOAD) {  // readChunk failed: no page of it is ever read
    out->status = ce.status;
    out->phase = PQH_PHASE_LOAD;
    out->index = ce.index;
    return PQH_OK;
  }
  if (S.err != kNoError) {
    const int phase = int(S.err >> 56);
    const int64_t idx = int64_t((S.err >> 8) & 0xffffffffffffull);
    out->status = int32_t(S.err & 0xff);
    out->phase = phase;
    out->index = idx;
    // The whole-page call (readNextPage, data_store.go:241) fails.  A ranged call of a page whose
    // levels failed fails too, even when its range ends before the failing slot (where the
    // reference would return that range): the device decodes no values of such a page, so there
    // are none to return (documented divergence).  Value errors: below.
    if (phase != PQH_PHASE_VALUES) return PQH_OK;
  }
  if (s1 == s0) {  // nothing left in the page: no values; a byte-array call still gets offsets[0] = 0
    if (offsets && offsets_cap >= 1 && C.value_size == 0 && out->status == PQH_OK) offsets[0] = 0;
    return PQH_OK;
  }
  // levels of the range, and the non-null values before / inside it
  std::vector<uint8_t> defs;
  int64_t nn0 = s0, nn1 = s1 - s0;
  if (C.max_def > 0) {
    defs.resize(size_t(s1));
    HIP_TRY(ctx, bounce_d2h(ctx, defs.data(), C.def_levels + P.level_base, size_t(s1)));
    nn0 = 0;
    nn1 = 0;
    for (int64_t i = 0; i < s1; i++) (i < s0 ? nn0 : nn1) += defs[size_t(i)] == C.max_def;
    if (def_levels) memcpy(def_levels, defs.data() + s0, size_t(s1 - s0));
  }
  if (C.max_rep > 0 && rep_levels)
    HIP_TRY(ctx, bounce_d2h(ctx, rep_levels, C.rep_levels + P.level_base + s0, size_t(s1 - s0)));
  if (out->status != PQH_OK) {  // a value error: decodeValues of this range meets it?
    if (out->index < nn0 + nn1) {
      out->num_non_null = nn1;
      // decodeValues' count: values before the failing one, except the two checks that return 0
      // (type_dict.go:52-54, type_bytearray.go:223-229)
      const bool zero = out->status == PQH_ERR_DICT_INDEX || out->status == PQH_ERR_DBA_PREFIX;
      out->values_read = zero ? 0 : std::max<int64_t>(0, out->index - nn0);
      return PQH_OK;
    }
    out->status = PQH_OK;
    out->phase = 0;
    out->index = 0;
  }
  out->num_non_null = nn1;
  out->values_read = nn1;
  const int64_t v0 = S.value_base + nn0;
  if (value_nil && value_nil_cap < nn1) return set_err(ctx, PQH_ERR_ARG, "value_nil buffer too small");
  if (C.value_nil && nn1 > 0) {  // the reference's nil INT96 values among the returned ones
    std::vector<uint8_t> m(static_cast<size_t>(nn1));
    HIP_TRY(ctx, bounce_d2h(ctx, m.data(), C.value_nil + v0, size_t(nn1)));
    for (uint8_t x : m) out->num_nil += x != 0;
    if (value_nil) memcpy(value_nil, m.data(), size_t(nn1));
  } else if (value_nil && nn1 > 0) {
    memset(value_nil, 0, size_t(nn1));
  }
  if (C.value_size > 0) {
    const int64_t bytes = nn1 * C.value_size;
    if (values) {
      if (values_cap < bytes) return set_err(ctx, PQH_ERR_ARG, "values buffer too small");
      HIP_TRY(ctx, bounce_d2h(ctx, values, C.values + v0 * C.value_size, size_t(bytes)));
    }
    return PQH_OK;
  }
  // byte arrays: offsets relative to the range's first value, then the bytes
  std::vector<int64_t> offs(size_t(nn1 + 1));
  HIP_TRY(ctx, bounce_d2h(ctx, offs.data(), C.offsets + v0, sizeof(int64_t) * size_t(nn1 + 1)));
  out->num_bytes = offs.back() - offs.front();
  if (offsets) {
    if (offsets_cap < nn1 + 1) return set_err(ctx, PQH_ERR_ARG, "offsets buffer too small");
    for (int64_t i = 0; i <= nn1; i++) offsets[i] = offs[size_t(i)] - offs.front();
  }
  if (data && out->num_bytes > 0) {
    if (data_cap < out->num_bytes) return set_err(ctx, PQH_ERR_ARG, "data buffer too small");
    HIP_TRY(ctx, bounce_d2h(ctx, data, C.bytes + offs.front(), size_t(out->num_bytes)));
  }
  return PQH_OK;
}

}  // extern "C"

namespace {
// The first error of a chunk in the reference's order.  readChunk walks the pages and fails at the
// first one it cannot load (chunk_reader.go:182-263): a page whose image the device could not
// decompress (readPageBlock), a page-load error of the planner or the prologue (the decoders'
// selection and init, phase 0), or -- after the listed pages -- the host walker's error
// (host_status); any of these fails the whole row group (chunk_reader.go:394-400).  Otherwise
// readValues errors surface page by page (data_store.go:236-260): the first in page order.
ChunkErr chunk_error(const pqh_batch* b, int32_t chunk) {
  const DevChunk& D = b->hchunks[size_t(chunk)];
  ChunkErr e;
  auto key = [&](int32_t p, uint64_t k) {
    e.status = int32_t(k & 0xff);
    e.phase = int32_t(k >> 56);
    e.index = int64_t((k >> 8) & 0xffffffffffffull);
    e.page = p;
  };
  for (int32_t i = 0; i < D.num_pages; i++) {
    const int32_t p = D.first_page + i;
    if (size_t(p) < b->codec_status.size() && b->codec_status[size_t(p)] != PQH_OK) {
      e.status = b->codec_status[size_t(p)] == PQH_ERR_INTERNAL ? PQH_ERR_INTERNAL : PQH_ERR_DECOMPRESS;
      e.phase = PQH_PHASE_LOAD;
      e.page = p;
      return e;
    }
    const uint64_t k = b->states[size_t(p)].err;
    if (k != kNoError && (k >> 56) == PQH_PHASE_LOAD) {
      key(p, k);
      return e;
    }
  }
  if (b->chunks[size_t(chunk)].host_status != PQH_OK) {
    e.status = b->chunks[size_t(chunk)].host_status;
    e.phase = PQH_PHASE_LOAD;
    return e;  // (page -1: the page the walk stopped at is not in the batch)
  }
  for (int32_t i = 0; i < D.num_pages; i++) {
    const int32_t p = D.first_page + i;
    if (b->states[size_t(p)].err != kNoError) {
      key(p, b->states[size_t(p)].err);
      return e;
    }
  }
  return e;
}
}  // namespace

extern "C" {

int pqh_batch_chunk_out(const pqh_batch* b, int32_t chunk, pqh_chunk_out* out) {
  if (!b || chunk < 0 || size_t(chunk) >= b->chunks.size()) return set_err(b ? b->ctx : nullptr, PQH_ERR_ARG, "bad chunk");
  if (!b->synced) return set_err(b->ctx, PQH_ERR_ARG, "batch not synced");
  const DevChunk& D = b->hchunks[size_t(chunk)];
  memset(out, 0, sizeof(*out));
  out->num_values = b->chunk_n[size_t(chunk)];
  out->value_size = D.value_size;
  out->values = D.value_size > 0 ? D.values : nullptr;
  out->offsets = D.offsets;
  out->bytes = D.bytes;
  // (a failing chunk's byte total past its first failing page may be garbage: never past the buffer)
  out->num_bytes = D.offsets ? std::max<int64_t>(0, std::min(b->chunk_bytes[size_t(chunk)], D.bytes_cap)) : 0;
  out->def_levels = D.def_levels;
  out->rep_levels = D.rep_levels;
  out->value_nil = D.value_nil;
  out->num_nil = size_t(chunk) < b->chunk_nil.size() ? b->chunk_nil[size_t(chunk)] : 0;
  const ChunkErr e = chunk_error(b, chunk);
  out->status = e.status;
  out->error_page = e.page;
  out->error_phase = e.phase;
  out->error_index = e.index;
  int64_t nn = 0;
  for (int32_t i = 0; i < D.num_pages; i++) {
    const int32_t p = D.first_page + i;
    if (b->hpages[size_t(p)].page_type != PQH_DICTIONARY_PAGE) nn += b->states[size_t(p)].nn;
  }
  out->num_non_null = nn;
  return PQH_OK;
}

int pqh_batch_nesting(const pqh_batch* b, int32_t chunk, pqh_nest_out* out) {
  if (!b || !out || chunk < 0 || size_t(chunk) >= b->chunks.size())
    return set_err(b ? b->ctx : nullptr, PQH_ERR_ARG, "bad chunk");
  if (!b->synced) return set_err(b->ctx, PQH_ERR_ARG, "batch not synced");
  memset(out, 0, sizeof(*out));
  const pqh_column& col = b->chunks[size_t(chunk)].column;
  if (col.max_rep == 0) return PQH_OK;
  const int32_t ni = b->chunk_nest[size_t(chunk)];
  if (ni < 0) {
    if (b->chunk_n[size_t(chunk)] == 0) {  // no level slots: empty outputs
      out->num_levels = col.max_rep;
      return PQH_OK;
    }
    return set_err(b->ctx, PQH_ERR_NOT_IMPLEMENTED,
                   "nesting needs max_rep <= PQH_MAX_NEST and the repeated nodes' definition levels");
  }
  const DevChunk& D = b->hchunks[size_t(chunk)];
  for (int32_t i = 0; i < D.num_pages; i++) {
    const PageState& S = b->states[size_t(D.first_page + i)];
    if (S.err != kNoError && out->status == PQH_OK) out->status = int32_t(S.err & 0xff);
  }
  out->num_levels = col.max_rep;
  // the chunk's windows (consecutive DevNests): window flag f counts E_{lbase + f}
  for (int32_t w = ni; w < int32_t(b->nests.size()) && b->nests[size_t(w)].chunk == chunk; w++) {
    const DevNest& N = b->nests[size_t(w)];
    const int64_t* tot = b->nest_totals.data() + size_t(w) * kNestFlags;
    for (int l = 0; l < N.levels; l++) {
      pqh_nest_level& o = out->levels[N.lbase + l];
      o.def_level = N.rep_def[l];
      o.num_lists = tot[l];
      o.offsets = N.offsets[l];
      o.validity = N.validity[l];
    }
    if (N.leaf) {
      out->num_leaf_slots = tot[N.levels];
      out->leaf_validity = N.leaf_valid;
    }
  }
  return PQH_OK;
}

int pqh_batch_kernel_stats(const pqh_batch* b, pqh_kernel_stat* out, int32_t max_stats, int32_t* num_stats) {
  if (!b) return set_err(nullptr, PQH_ERR_ARG, "null batch");
  int32_t n = 0;
  for (int k = 0; k < kNumKernels && n < max_stats; k++) out[n++] = b->stats[size_t(k)];
  *num_stats = n;
  return PQH_OK;
}

int pqh_batch_path_info(const pqh_batch* b, pqh_batch_paths* out) {
  if (!b || !out) return set_err(b ? b->ctx : nullptr, PQH_ERR_ARG, "null batch or output");
  memset(out, 0, sizeof(*out));
  out->flat_active = flat_batch(b) ? 1 : 0;
  out->flat_fallbacks = b->flat_fallbacks;
  out->ba_fuse_active = b->ba_fuse_on ? 1 : 0;
  out->ba_fuse_fallbacks = b->ba_fuse_fallbacks;
  out->regrows = b->regrows;
  out->graph_replay = (graphs_enabled() && !b->graph_failed && !flat_batch(b) &&
                       !(b->ctx->flags & (PQH_CTX_PROFILE | PQH_CTX_STREAMING))) ? 1 : 0;
  return PQH_OK;
}

int pqh_batch_reset_stats(pqh_batch* b) {
  if (!b) return PQH_ERR_ARG;
  for (auto& s : b->stats) {
    s.launches = 0;
    s.total_ms = 0;
  }
  return PQH_OK;
}

int pqh_batch_traffic(const pqh_batch* b, double* bytes_read, double* bytes_written) {
  if (!b || !b->synced) return set_err(b ? b->ctx : nullptr, PQH_ERR_ARG, "batch not synced");
  *bytes_read = b->bytes_read;
  *bytes_written = b->bytes_written;
  return PQH_OK;
}

void pqh_batch_destroy(pqh_batch* b) {
  if (!b) return;
  hipSetDevice(b->ctx->device);
  hipStreamSynchronize(b->ctx->stream);
  if (b->ctx->copy_stream) hipStreamSynchronize(b->ctx->copy_stream);
  free_batch(b);
  delete b;
}

}  // extern "C"

namespace {
// The multi-workgroup SNAPPY plan of a codec page table: its tables in HBM and its scratch.
int snap_plan_alloc(pqh_batch* b, const pqh_codec_page* pages, int32_t n) {
  SnapPlan& P = b->snap;
  P.n_pages = n;
  const std::vector<int32_t> t = snap_plan_tables(pages, n, &P.n_win, &P.n_unit, &P.n_page_mode);
  int32_t* tab = nullptr;
  int4* ws = nullptr;
  int2* wt = nullptr;
  int32_t* uf = nullptr;
  int16_t* seg = nullptr;
  int rc;
  if ((rc = dalloc(b, reinterpret_cast<void**>(&seg), sizeof(int16_t) * 1024 * size_t(P.n_win))) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&tab), sizeof(int32_t) * t.size())) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&ws), sizeof(int4) * size_t(P.n_win))) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&wt), sizeof(int2) * size_t(P.n_win))) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&uf), sizeof(int32_t) * size_t(P.n_unit))))
    return rc;
  const hipError_t e = bounce_h2d(b->ctx, tab, t.data(), sizeof(int32_t) * t.size());
  if (e != hipSuccess) return set_err(b->ctx, PQH_ERR_HIP, std::string("snappy plan: ") + hipGetErrorString(e));
  snap_plan_bind(P, tab, ws, wt, uf, seg);
  return PQH_OK;
}

// Device codecs: the image buffer (zeroed, with its pad) the decode reads, planned over the host
// batch's tables; the source payload at d_src (already in HBM or uploaded by the caller) is
// decompressed into it at the start of every run.
int create_codec_batch(pqh_ctx* ctx, const pqh_host_batch* hb, void* d_src, pqh_batch** out) {
  void* img = nullptr;
  const size_t ibytes = size_t(hb->image_bytes) + PQH_PAYLOAD_PAD;
  HIP_TRY(ctx, dev_alloc(ctx, &img, ibytes));
  hipError_t e = hipMemsetAsync(img, 0, ibytes, ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) {
    dev_free(ctx, img);
    return set_err(ctx, PQH_ERR_HIP, std::string("image buffer: ") + hipGetErrorString(e));
  }
  int rc = pqh_batch_create(ctx, hb->chunks.data(), int32_t(hb->chunks.size()), hb->pages.data(),
                            int32_t(hb->pages.size()), img, hb->image_bytes, out);
  if (rc) {
    dev_free(ctx, img);
    return rc;
  }
  pqh_batch* b = *out;
  b->owned_payload = img;
  b->src_bytes = hb->size();
  b->codec_n = int32_t(hb->codec_pages.size());
  b->codec_gzip = int32_t(std::count_if(hb->codec_pages.begin(), hb->codec_pages.end(),
                                        [](const pqh_codec_page& c) { return c.codec == PQH_CODEC_GZIP; }));
  // d_src passes to the batch only once nothing can fail: on an error the caller still owns (and frees) it
  if ((rc = dalloc(b, reinterpret_cast<void**>(&b->d_codec), sizeof(pqh_codec_page) * size_t(b->codec_n))) ||
      (rc = dalloc(b, reinterpret_cast<void**>(&b->d_codec_status), sizeof(int32_t) * size_t(b->codec_n)))) {
    pqh_batch_destroy(b);
    *out = nullptr;
    return rc;
  }
  e = bounce_h2d(ctx, b->d_codec, hb->codec_pages.data(), sizeof(pqh_codec_page) * size_t(b->codec_n));
  if (e == hipSuccess && (rc = snap_plan_alloc(b, hb->codec_pages.data(), b->codec_n))) {
    pqh_batch_destroy(b);
    *out = nullptr;
    return rc;
  }
  if (e != hipSuccess) {
    pqh_batch_destroy(b);
    *out = nullptr;
    return set_err(ctx, PQH_ERR_HIP, std::string("codec pages: ") + hipGetErrorString(e));
  }
  b->d_src = d_src;
  return PQH_OK;
}
}  // namespace

extern "C" {

int pqh_batch_create_from_host(pqh_ctx* ctx, const pqh_host_batch* hb, pqh_batch** out) {
  *out = nullptr;
  if (!ctx || !hb) return set_err(ctx, PQH_ERR_ARG, "null argument");
  hipSetDevice(ctx->device);
  if (!hb->codec_pages.empty()) {  // source payload to HBM; images rebuilt by every run
    void* src = nullptr;
    HIP_TRY(ctx, dev_alloc(ctx, &src, hb->size()));
    hipError_t e = bounce_h2d(ctx, src, hb->data(), hb->size());
    if (e != hipSuccess) {
      dev_free(ctx, src);
      return set_err(ctx, PQH_ERR_HIP, std::string("source upload: ") + hipGetErrorString(e));
    }
    const int rc = create_codec_batch(ctx, hb, src, out);
    if (rc) dev_free(ctx, src);
    return rc;
  }
  void* d = nullptr;
  const size_t bytes = hb->size();
  HIP_TRY(ctx, dev_alloc(ctx, &d, bytes ? bytes : 16));
  hipError_t e = hb->pinned ? hipMemcpyAsync(d, hb->data(), bytes, hipMemcpyHostToDevice, ctx->stream)
                            : bounce_h2d(ctx, d, hb->data(), bytes);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) {
    dev_free(ctx, d);
    return set_err(ctx, PQH_ERR_HIP, std::string("payload upload: ") + hipGetErrorString(e));
  }
  int rc = pqh_batch_create(ctx, hb->chunks.data(), int32_t(hb->chunks.size()), hb->pages.data(),
                            int32_t(hb->pages.size()), d, hb->payload_bytes, out);
  if (rc) {
    dev_free(ctx, d);
    return rc;
  }
  (*out)->owned_payload = d;
  return PQH_OK;
}

int pqh_batch_create_staged(pqh_ctx* ctx, const pqh_host_batch* hb, pqh_batch** out) {
  *out = nullptr;
  if (!ctx || !hb) return set_err(ctx, PQH_ERR_ARG, "null argument");
  hipSetDevice(ctx->device);
  if (!ctx->copy_stream && !(ctx->flags & PQH_CTX_STREAMING))
    HIP_TRY(ctx, hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking));
  const size_t bytes = hb->size();
  void* h = nullptr;
  std::shared_ptr<uint8_t> pinned = hb->pinned ? hb->buf : nullptr;  // a pinned payload is adopted, not copied
  if (pinned) {
    h = pinned.get();
  } else {
    HIP_TRY(ctx, hipHostMalloc(&h, bytes ? bytes : 16, hipHostMallocDefault));
    if (bytes) memcpy(h, hb->data(), bytes);
  }
  auto free_h = [&]() {
    if (!pinned) hipHostFree(h);
  };
  void* d = nullptr;
  const bool streaming = (ctx->flags & PQH_CTX_STREAMING) != 0;
  hipError_t e = dev_alloc(ctx, &d, bytes ? bytes : 16);
  // the first upload happens here so that planning (which reads nothing from the payload) and the
  // first plain pqh_batch_run see the same bytes as the staged runs; a streaming context leaves it to
  // pqh_batch_run_staged (one H2D per range, on the copy stream)
  if (e == hipSuccess && bytes && !streaming) e = hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess && !streaming) e = hipStreamSynchronize(ctx->stream);
  if (e != hipSuccess) {
    if (d) dev_free(ctx, d);
    free_h();
    return set_err(ctx, PQH_ERR_HIP, std::string("staged payload: ") + hipGetErrorString(e));
  }
  g_defer_tables = streaming && hb->codec_pages.empty();
  int rc = hb->codec_pages.empty() ? pqh_batch_create(ctx, hb->chunks.data(), int32_t(hb->chunks.size()),
                                                       hb->pages.data(), int32_t(hb->pages.size()), d,
                                                       hb->payload_bytes, out)
                                    : create_codec_batch(ctx, hb, d, out);
  g_defer_tables = false;
  if (rc) {
    dev_free(ctx, d);
    free_h();
    return rc;
  }
  pqh_batch* b = *out;
  if (hb->codec_pages.empty()) b->owned_payload = d;  // else: d is the source buffer (b->d_src)
  b->h_staged = h;
  b->h_pinned_ref = pinned;
  b->staged_bytes = bytes;
  if (hipEventCreateWithFlags(&b->ev_copied, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&b->ev_done, hipEventDisableTiming) != hipSuccess) {
    pqh_batch_destroy(b);
    *out = nullptr;
    return set_err(ctx, PQH_ERR_HIP, "staged batch events");
  }
  return PQH_OK;
}

int pqh_decompress_pages(pqh_ctx* ctx, const pqh_codec_page* pages, int32_t num_pages, const void* d_src,
                         void* d_dst, int32_t* status) {
  if (!ctx || num_pages < 0 || (num_pages && (!pages || !status))) return set_err(ctx, PQH_ERR_ARG, "bad arguments");
  if (num_pages == 0) return PQH_OK;
  // the stage loads round addresses down to 16 bytes from d_src (hipMalloc pointers are aligned)
  if ((reinterpret_cast<uintptr_t>(d_src) | reinterpret_cast<uintptr_t>(d_dst)) & 15)
    return set_err(ctx, PQH_ERR_ARG, "pqh_decompress_pages: d_src and d_dst must be 16-byte aligned");
  hipSetDevice(ctx->device);
  pqh_codec_page* dp = nullptr;
  int32_t* ds = nullptr;
  hipError_t e = hipMalloc(&dp, sizeof(pqh_codec_page) * size_t(num_pages));
  if (e == hipSuccess) e = hipMalloc(&ds, sizeof(int32_t) * size_t(num_pages));
  if (e == hipSuccess) e = bounce_h2d(ctx, dp, pages, sizeof(pqh_codec_page) * size_t(num_pages));
  // the multi-workgroup SNAPPY plan (tables + scratch in one allocation)
  SnapPlan P;
  P.n_pages = num_pages;
  const std::vector<int32_t> tab = snap_plan_tables(pages, num_pages, &P.n_win, &P.n_unit, &P.n_page_mode);
  const size_t tb = (sizeof(int32_t) * tab.size() + 15) & ~size_t(15);
  // the walker-segment entries (written as 8-byte stores) start 16-byte aligned after the unit flags
  const size_t ub = (sizeof(int32_t) * size_t(P.n_unit) + 15) & ~size_t(15);
  const size_t sb = tb + sizeof(int4) * size_t(P.n_win) + sizeof(int2) * size_t(P.n_win) + ub +
                    sizeof(int16_t) * 1024 * size_t(P.n_win) + 16;
  void* scratch = nullptr;
  if (e == hipSuccess) e = hipMalloc(&scratch, sb);
  if (e == hipSuccess) e = bounce_h2d(ctx, scratch, tab.data(), sizeof(int32_t) * tab.size());
  if (e == hipSuccess) {
    uint8_t* m = static_cast<uint8_t*>(scratch);
    int4* ws = reinterpret_cast<int4*>(m + tb);
    int2* wt = reinterpret_cast<int2*>(ws + P.n_win);
    int32_t* uf = reinterpret_cast<int32_t*>(wt + P.n_win);
    snap_plan_bind(P, reinterpret_cast<int32_t*>(m), ws, wt, uf, reinterpret_cast<int16_t*>(reinterpret_cast<uint8_t*>(uf) + ub));
    e = snappy_page_mode()
            ? launch_snappy(dp, num_pages, static_cast<const uint8_t*>(d_src), static_cast<uint8_t*>(d_dst), ds, ctx->stream)
            : launch_snappy_mw(dp, P, static_cast<const uint8_t*>(d_src), static_cast<uint8_t*>(d_dst), ds, ctx->stream);
  }
  if (e == hipSuccess && std::any_of(pages, pages + num_pages, [](const pqh_codec_page& c) { return c.codec == PQH_CODEC_GZIP; }))
    e = launch_gzip(dp, num_pages, static_cast<const uint8_t*>(d_src), static_cast<uint8_t*>(d_dst), ds, ctx->stream);
  if (e == hipSuccess) e = bounce_d2h(ctx, status, ds, sizeof(int32_t) * size_t(num_pages));
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (dp) hipFree(dp);
  if (ds) hipFree(ds);
  if (scratch) hipFree(scratch);
  if (e != hipSuccess) return set_err(ctx, PQH_ERR_HIP, std::string("pqh_decompress_pages: ") + hipGetErrorString(e));
  return PQH_OK;
}

int pqh_hybrid_decode(pqh_ctx* ctx, const void* d_stream, int64_t len, int32_t width, int64_t n, int32_t group,
                      uint32_t* d_out, int32_t* status, int64_t* values) {
  if (!ctx || len < 0 || n < 0 || width < 0 || width > 32 || (group != 4 && group != 8) || !status || !values ||
      (n > 0 && !d_out) || (len > 0 && !d_stream) || n > (int64_t(1) << 40))
    return set_err(ctx, PQH_ERR_ARG, "bad hybrid decode arguments");
  hipSetDevice(ctx->device);
  Ckpt* ck = nullptr;
  uint64_t* res = nullptr;
  uint64_t h[2] = {kNoError, 0};
  const size_t nck = size_t((n + kHybridTile - 1) / kHybridTile) + 1;
  hipError_t e = hipMalloc(&ck, sizeof(Ckpt) * nck);
  if (e == hipSuccess) e = hipMalloc(&res, sizeof(h));
  if (e == hipSuccess) e = hipMemsetAsync(ck, 0, sizeof(Ckpt) * nck, ctx->stream);
  if (e == hipSuccess)
    e = launch_hybrid_raw(static_cast<const uint8_t*>(d_stream), len, width, n, group, ck, res, d_out, ctx->stream);
  if (e == hipSuccess) e = bounce_d2h(ctx, h, res, sizeof(h));
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (ck) hipFree(ck);
  if (res) hipFree(res);
  if (e != hipSuccess) return set_err(ctx, PQH_ERR_HIP, std::string("pqh_hybrid_decode: ") + hipGetErrorString(e));
  *status = h[0] == kNoError ? PQH_OK : int32_t(h[0] & 0xff);
  *values = int64_t(h[1]);
  return PQH_OK;
}

int pqh_batch_run_staged(pqh_batch* b) {
  if (!b) return set_err(nullptr, PQH_ERR_ARG, "null batch");
  pqh_ctx* ctx = b->ctx;
  if (!b->h_staged) return set_err(ctx, PQH_ERR_ARG, "batch was not created by pqh_batch_create_staged");
  hipSetDevice(ctx->device);
  // a streaming context copies on its one stream (in order with the plan's zero fills and the
  // decode); otherwise on the copy stream, beside the decode of the previous staged batch
  const bool one = ctx->copy_stream == nullptr;
  hipStream_t cs = one ? ctx->stream : ctx->copy_stream;
  // the copy must not overwrite page images a previous decode of this batch still reads
  if (b->done_recorded && !one) HIP_TRY(ctx, hipStreamWaitEvent(cs, b->ev_done, 0));
  if (!b->table_ups.empty()) {  // deferred plan tables (first run only): after the plan's zero fills
    if (!one) {
      HIP_TRY(ctx, hipEventRecord(b->ev_copied, ctx->stream));
      HIP_TRY(ctx, hipStreamWaitEvent(cs, b->ev_copied, 0));
    }
    for (const auto& u : b->table_ups)
      HIP_TRY(ctx, hipMemcpyAsync(u.dst, b->h_tables.get() + u.off, u.bytes, hipMemcpyHostToDevice, cs));
    b->table_ups.clear();
  }
  if (b->staged_bytes)  // the page images, or with device codecs the source bytes
    HIP_TRY(ctx, hipMemcpyAsync(b->codec_n ? b->d_src : b->owned_payload, b->h_staged, b->staged_bytes,
                                hipMemcpyHostToDevice, cs));
  if (!one) {
    HIP_TRY(ctx, hipEventRecord(b->ev_copied, cs));
    HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, b->ev_copied, 0));
  }
  int rc = pqh_batch_run(b);
  if (rc) return rc;
  HIP_TRY(ctx, hipEventRecord(b->ev_done, ctx->stream));
  b->done_recorded = true;
  return PQH_OK;
}

}  // extern "C"
