/*
 * pqhip.h — C-ABI of libpqhip, the MI355X-native Parquet column-chunk page decoder.
 *
 * This is the drop-in boundary for ONE hot path of github.com/fraugster/parquet-go
 * (mounted at /root/reference): decoding the pages of a column chunk.  The reference
 * decodes a page through the package-internal seam
 *
 *     pageReader{ init(dDecoder, rDecoder, values); read(r, ph, codec, crc); readValues(size); numValues() }
 *                                                     (reference interfaces.go:11-18)
 *     valuesDecoder{ init(io.Reader); decodeValues([]interface{}) (int, error) }   (interfaces.go:29-33)
 *     levelDecoder{ next() (int32, error); init/initSize(io.Reader); maxLevel() }   (hybrid_decoder.go:16-27)
 *
 * and builds those readers in FileReader.readChunk/readPages (chunk_reader.go:182-362).  A cgo
 * shim binds the functions below in place of that seam:
 *
 *   - pqh_file_*        replace readChunk/readPages + readPageBlock/newBlockReader (host side:
 *                       thrift page headers, CRC, GZIP/SNAPPY decompression) and emit a page table;
 *   - pqh_batch_*       replace pageReader.read + readValues(numValues) for every page of a set of
 *                       column chunks: all hybrid RLE/bit-packed streams, DELTA_BINARY_PACKED,
 *                       dictionary gathers, PLAIN values and level decoding run as HIP kernels on
 *                       HBM-resident page images, one launch per kernel kind for the whole batch.
 *
 * Conventions: every function returns a pqh_status (0 = PQH_OK) unless stated otherwise, never
 * aborts, and stores a message retrievable with pqh_last_error / pqh_file_error.  No torch types,
 * plain pointers and sizes only.  Device pointers are HIP device pointers of the context's device.
 */
#ifndef PQHIP_H
#define PQHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PQH_ABI_VERSION 8

/* Bytes of readable slack the device payload buffer must have after its last page image.  The
 * kernels issue (masked) vector loads that may run up to this many bytes past a stream end. */
#define PQH_PAYLOAD_PAD 256

/* parquet.Type (reference parquet/parquet.thrift:32-41) */
enum pqh_physical_type {
  PQH_BOOLEAN = 0,
  PQH_INT32 = 1,
  PQH_INT64 = 2,
  PQH_INT96 = 3,
  PQH_FLOAT = 4,
  PQH_DOUBLE = 5,
  PQH_BYTE_ARRAY = 6,
  PQH_FIXED_LEN_BYTE_ARRAY = 7
};

/* parquet.Encoding (parquet.thrift:414-470) */
enum pqh_encoding {
  PQH_ENC_PLAIN = 0,
  PQH_ENC_PLAIN_DICTIONARY = 2,
  PQH_ENC_RLE = 3,
  PQH_ENC_BIT_PACKED = 4,
  PQH_ENC_DELTA_BINARY_PACKED = 5,
  PQH_ENC_DELTA_LENGTH_BYTE_ARRAY = 6,
  PQH_ENC_DELTA_BYTE_ARRAY = 7,
  PQH_ENC_RLE_DICTIONARY = 8,
  PQH_ENC_BYTE_STREAM_SPLIT = 9
};

/* parquet.PageType (parquet.thrift:498-507) */
enum pqh_page_type {
  PQH_DATA_PAGE = 0,
  PQH_INDEX_PAGE = 1,
  PQH_DICTIONARY_PAGE = 2,
  PQH_DATA_PAGE_V2 = 3
};

/* parquet.CompressionCodec (parquet.thrift:487-496) */
enum pqh_codec {
  PQH_CODEC_UNCOMPRESSED = 0,
  PQH_CODEC_SNAPPY = 1,
  PQH_CODEC_GZIP = 2,
  PQH_CODEC_ZSTD = 6
};

/* Status codes.  Each data-path code names the reference error it stands for. */
typedef enum pqh_status {
  PQH_OK = 0,
  PQH_ERR_EOF = 1,                    /* io.EOF before a needed value (hybrid_decoder.go:142-147, ...) */
  PQH_ERR_UNEXPECTED_EOF = 2,         /* io.ErrUnexpectedEOF: short fixed-size read (binary.Read, ReadFull) */
  PQH_ERR_VARINT_OVERFLOW = 3,        /* encoding/binary: varint overflows a 64-bit integer */
  PQH_ERR_INT32_RANGE = 4,            /* "int32 out of range" (helpers.go:162-164, 181-183) */
  PQH_ERR_EMPTY_BP_RUN = 5,           /* "rle: empty bit-packed run" (hybrid_decoder.go:151-155) */
  PQH_ERR_EMPTY_RLE_RUN = 6,          /* "rle: empty RLE run" (hybrid_decoder.go:158-161) */
  PQH_ERR_RLE_VALUE_TOO_LARGE = 7,    /* "rle: RLE run value is too large" (hybrid_decoder.go:126-128) */
  PQH_ERR_READER_NOT_INITIALIZED = 8, /* "reader is not initialized" (hybrid_decoder.go:86-88) */
  PQH_ERR_DICT_BIT_WIDTH = 9,         /* "invalid bitwidth" (type_dict.go:28-30) */
  PQH_ERR_DICT_INDEX = 10,            /* "dict: invalid index" (type_dict.go:52-54) */
  PQH_ERR_DELTA_BLOCK_SIZE = 11,      /* "invalid block size" (deltabp_decoder.go:56-58) */
  PQH_ERR_DELTA_MINIBLOCKS = 12,      /* "invalid number of mini blocks" / zero miniblock values (:64-71) */
  PQH_ERR_DELTA_VALUE_COUNT = 13,     /* "invalid total value count" (:77-79) */
  PQH_ERR_DELTA_BIT_WIDTH = 14,       /* "invalid miniblock bit width" (:100-104) */
  PQH_ERR_DELTA_STREAM = 15,          /* "invalid stream" / negative remaining (:151-154) */
  PQH_ERR_NEGATIVE_LENGTH = 16,       /* "bytearray/plain: len is negative" (type_bytearray.go:30-34) */
  PQH_ERR_NEGATIVE_DLBA_LENGTH = 17,  /* negative DELTA_LENGTH length: a runtime panic in the reference */
  PQH_ERR_DBA_PREFIX = 18,            /* "invalid prefix len in the stream" (type_bytearray.go:223-226) */
  PQH_ERR_DBA_COUNT = 19,             /* "different number of suffixes and prefixes" (type_bytearray.go:206-208) */
  PQH_ERR_INT96_SHORT = 20,           /* (unused since ABI 7: a short last INT96 value is a nil slot) */
  PQH_ERR_UNSUPPORTED = 21,           /* getValuesDecoder: unsupported (type, encoding) (chunk_reader.go:106-159) */
  PQH_ERR_PAGE_HEADER = 22,           /* negative NumValues / sizes, missing sub-header (page_v1.go:88-94 ...) */
  PQH_ERR_DECOMPRESS = 23,            /* decompression failed or size mismatch (compress.go:131-152) */
  PQH_ERR_CRC = 24,                   /* "CRC32 check failed" (chunk_reader.go:173-177) */
  PQH_ERR_THRIFT = 25,                /* malformed thrift compact structure */
  PQH_ERR_IO = 26,                    /* file I/O */
  PQH_ERR_ARG = 27,                   /* invalid argument to this API */
  PQH_ERR_HIP = 28,                   /* HIP runtime failure */
  PQH_ERR_NOMEM = 29,                 /* allocation failure */
  PQH_ERR_SCHEMA = 30,                /* schema / column metadata inconsistency (chunk_reader.go:303-312) */
  PQH_ERR_DICT_PAGE = 31,             /* second dictionary page / dictionary encoding not PLAIN (chunk_reader.go:197-199, page_dict.go:44-46) */
  PQH_ERR_NO_DEVICE = 32,             /* no HIP device present */
  PQH_ERR_NOT_IMPLEMENTED = 33,       /* decoder kind not (yet) available on the device */
  PQH_ERR_INTERNAL = 34,              /* a device consistency guard fired (an index outside its buffer,
                                         a look-back that never completed): a bug, never a property of
                                         the input -- the chunk's outputs are undefined */
  PQH_ERR_UNSUPPORTED_CODEC = 35      /* the chunk's codec is not decoded by this library (ZSTD, LZ4,
                                         BROTLI, LZO, or any codec a caller registers with
                                         RegisterBlockCompressor, compress.go:119-129,160,182-187): set by
                                         the page walker before any page of the chunk is read, never
                                         a property of the data -- the caller decodes the chunk with the
                                         reference's own readChunk / pageReader path */
} pqh_status;

/* Decode phases, in the order the reference runs them for one page (page_v1.go:33-122). */
enum pqh_phase {
  PQH_PHASE_LOAD = 0,   /* pageReader.read: level initSize, values decoder init      */
  PQH_PHASE_REP = 1,    /* readValues: repetition levels (decodePackedArray)          */
  PQH_PHASE_DEF = 2,    /* readValues: definition levels + not-null count             */
  PQH_PHASE_VALUES = 3  /* readValues: valuesDecoder.decodeValues(notNull)            */
};

/* ---------------------------------------------------------------------------------------------
 * Batch decode (device).  Replaces pageReader.read + readValues(numValues) (page_v1.go:33-122,
 * page_v2.go:31-131, page_dict.go:35-72) for every page of a set of column chunks.
 * ------------------------------------------------------------------------------------------- */

/* Repetition levels the nesting outputs support (the schema walk records the repeated nodes'
 * definition levels up to this depth).  Level bytes are uint8, so no column has more than 255. */
#define PQH_MAX_NEST 32

typedef struct pqh_column {
  int32_t physical_type; /* enum pqh_physical_type */
  int32_t type_length;   /* FIXED_LEN_BYTE_ARRAY length (SchemaElement.type_length) */
  int32_t max_def;       /* Column.MaxDefinitionLevel() (schema.go:904-914) */
  int32_t max_rep;       /* Column.MaxRepetitionLevel() */
  int32_t rep_def[PQH_MAX_NEST]; /* definition level of the k-th REPEATED node on the path
                            (k < max_rep), from readColumnSchema/readGroupSchema (schema.go:893-990);
                            used by the nesting outputs (pqh_batch_nesting), which need
                            max_rep <= PQH_MAX_NEST */
} pqh_column;

/* One page as the reference page walker sees it (parquet.PageHeader fields + the decompressed
 * page image).  For DATA_PAGE and DICTIONARY_PAGE the image is the decompressed block; for
 * DATA_PAGE_V2 it is the raw level bytes followed by the decompressed values section
 * (page_v2.go:113-125: the values section is always passed through the chunk codec). */
typedef struct pqh_page {
  int64_t image_offset;           /* byte offset of the page image in the payload buffer */
  int32_t image_len;              /* bytes in the image */
  int32_t page_type;              /* PQH_DATA_PAGE, PQH_DATA_PAGE_V2 or PQH_DICTIONARY_PAGE */
  int32_t num_values;             /* DataPageHeader(V2).num_values / DictionaryPageHeader.num_values */
  int32_t encoding;               /* values encoding from the header */
  int32_t def_levels_byte_length; /* DataPageHeaderV2 only (else 0) */
  int32_t rep_levels_byte_length; /* DataPageHeaderV2 only (else 0) */
  int32_t chunk;                  /* index of the owning pqh_chunk */
  int32_t num_nulls;              /* DataPageHeaderV2.num_nulls (else 0): a hint only -- the decode counts
                                     the definition levels as the reference does (k_flat speculates
                                     notNull = num_values - num_nulls and checks it) */
} pqh_page;

/* Device-side decompression: where one page's source bytes lie and how its image
 * is rebuilt in HBM (pqh_file_load_ex with PQH_LOAD_DEVICE_SNAPPY).  The image of page i of the host
 * batch is codec page i. */
typedef struct pqh_codec_page {
  int64_t src_offset;   /* page bytes in the source payload: the compressed block (SNAPPY, after the
                           raw prefix), or the finished image (codec 0: copied) */
  int64_t image_offset; /* == pqh_page.image_offset: where the image goes in the image buffer */
  int32_t src_len;      /* source bytes, raw prefix included */
  int32_t image_len;    /* == pqh_page.image_len: the header's uncompressed page size */
  int32_t raw_len;      /* leading bytes stored uncompressed (DataPageV2 levels, page_v2.go:116-125) */
  int32_t codec;        /* PQH_CODEC_SNAPPY, or PQH_CODEC_UNCOMPRESSED for a plain copy */
  int32_t chunk;        /* owning chunk in the host batch */
  int32_t reserved;
} pqh_codec_page;

/* A column chunk: a contiguous range of pages; a dictionary page, if any, comes first
 * (chunk_reader.go:195-227). */
typedef struct pqh_chunk {
  pqh_column column;
  int32_t first_page;  /* index into the page array */
  int32_t num_pages;   /* including the dictionary page */
  int32_t host_status; /* page-walker error for this chunk (readPages failed), else PQH_OK */
  int32_t reserved;
} pqh_chunk;

/* Device-resident result of one chunk, owned by the batch. */
typedef struct pqh_chunk_out {
  int64_t num_values;    /* level slots: Σ num_values of the data pages */
  int64_t num_non_null;  /* Σ notNull (helpers.go:143-145): number of decoded values */
  int32_t value_size;    /* bytes per value (bool: 1, INT96: 12, FLBA: type_length), 0 for BYTE_ARRAY */
  int32_t status;        /* first error of the chunk in page order, or PQH_OK */
  int32_t error_page;    /* page index (batch-global) of that error, or -1 */
  int32_t error_phase;   /* enum pqh_phase of that error */
  int64_t error_index;   /* value / level index of that error inside its page */
  void* values;          /* dense not-null values, natural width, little endian (device) */
  int64_t* offsets;      /* BYTE_ARRAY: num_non_null + 1 byte offsets into bytes (device), else NULL */
  uint8_t* bytes;        /* BYTE_ARRAY data (device), else NULL */
  int64_t num_bytes;     /* BYTE_ARRAY data size */
  uint8_t* def_levels;   /* one byte per level slot, NULL when max_def == 0 (device) */
  uint8_t* rep_levels;   /* one byte per level slot, NULL when max_rep == 0 (device) */
  /* The reference's nil values (INT96 only, type_int96.go:21-42): a PLAIN page whose last value is
   * short returns success with that slot never assigned, and a dictionary page whose last entry is
   * short hands that nil entry to every value that indexes it (type_dict.go:57).  Such values are
   * 12 zero bytes in `values`; value_nil (device, num_non_null bytes) marks them with 1.  NULL for
   * every chunk that cannot hold one (num_nil is then 0). */
  uint8_t* value_nil;
  int64_t num_nil;
} pqh_chunk_out;

/* Nesting of a repeated column, the columnar form of the reference's record
 * assembly (ColumnStore.get data_store.go:262-309, Column.getNextData/getData schema.go:216-312).
 * Level k (1..max_rep) has one list per enclosing instance (rows at level 1, elements of level k-1
 * below); offsets[i]..offsets[i+1] are the list's elements; validity[i] = 1 when the list is present
 * (its parent object exists; it may be empty).  Leaf slots are the elements of the innermost level;
 * leaf_validity = 1 when the value is non-null (d == max_def), i.e. the leaf's dense values are the
 * leaf slots with validity 1, in order. */
typedef struct pqh_nest_level {
  int32_t def_level;     /* definition level of this level's REPEATED node */
  int32_t reserved;
  int64_t num_lists;
  int32_t* offsets;      /* device, num_lists + 1 */
  uint8_t* validity;     /* device, num_lists */
} pqh_nest_level;

typedef struct pqh_nest_out {
  int32_t num_levels;    /* max_rep (0: not a repeated column; outputs empty) */
  int32_t status;        /* PQH_OK, or the chunk's decode error (outputs undefined) */
  int64_t num_leaf_slots;
  uint8_t* leaf_validity;  /* device, num_leaf_slots */
  pqh_nest_level levels[PQH_MAX_NEST];
} pqh_nest_out;

/* Per-page result (host copy). */
typedef struct pqh_page_result {
  int32_t status;       /* pqh_status of the page's first error, PQH_OK if none */
  int32_t phase;        /* enum pqh_phase of that error */
  int64_t index;        /* index at which it happened (level slot, value, or load sub-step) */
  int32_t num_non_null; /* notNull of the page */
  int32_t num_nil;      /* of those values, the reference's nil ones (pqh_chunk_out.value_nil) */
  int64_t value_offset; /* first value of this page in pqh_chunk_out.values */
  int64_t level_offset; /* first level slot of this page in pqh_chunk_out.{def,rep}_levels */
} pqh_page_result;

/* One readValues(size) result materialised on the host (pqh_batch_page_read). */
typedef struct pqh_page_values {
  int32_t status;       /* the reference's readValues error for this call, PQH_OK if none */
  int32_t phase;        /* enum pqh_phase of that error */
  int64_t index;        /* its level-slot / value index inside the page (as pqh_page_result) */
  int64_t num_slots;    /* level slots returned: min(count, num_values - first) */
  int64_t num_non_null; /* notNull of those slots (helpers.go:143-145) */
  int64_t values_read;  /* values decodeValues produced (< num_non_null on a value error) */
  int64_t num_bytes;    /* BYTE_ARRAY: bytes of the returned values */
  int32_t value_size;   /* bytes per fixed-width value, 0 for BYTE_ARRAY */
  int32_t num_nil;      /* returned values that are the reference's nil (INT96; marked in value_nil) */
} pqh_page_values;

typedef struct pqh_kernel_stat {
  char name[32];
  int32_t launches;     /* launches timed */
  int32_t work_items;   /* tiles / pages per launch */
  double total_ms;      /* summed HIP-event time */
  double bytes_read;    /* algorithmic bytes read per launch */
  double bytes_written; /* algorithmic bytes written per launch */
} pqh_kernel_stat;

typedef struct pqh_ctx pqh_ctx;
typedef struct pqh_batch pqh_batch;

#define PQH_CTX_PROFILE 1u /* time every kernel launch with HIP events */
/* A streaming context (creation only; pqh_ctx_set_flags keeps it): one slot of a bounded ring of
 * end-to-end row-group ranges (reader.RowGroupStream: one context per slot, so that a slot's batch
 * creation, sync and destruction wait for that slot's own work only).  It has ONE stream: the H2D of
 * pqh_batch_run_staged, the plan's zero fills and the decode run in order on it (the ring overlaps
 * slots; extra streams per slot would share the process's few hardware queues with other slots'
 * streams).  Its batches bump-allocate from the context's device arena, reset when the context's
 * last batch is destroyed (no driver call per range; PQH_ARENA_GUARD bytes of gap after each buffer,
 * PQH_ARENA_CHECK=1 verifies them at pqh_batch_sync), launch directly (a batch runs once: no graph
 * capture), and pqh_batch_create_staged returns without waiting on the GPU: the page images and the
 * plan tables (from a pinned block of the context's pool) are copied by pqh_batch_run_staged. */
#define PQH_CTX_STREAMING 2u

int pqh_abi_version(void);
/* The build's source hash (sha256 prefix of every source compiled into the library): profiles are
 * stamped with it, so measurements are tied to the code they measured. */
const char* pqh_build_id(void);
int pqh_device_count(int32_t* count);
int pqh_ctx_create(int32_t device, uint32_t flags, pqh_ctx** out);
/* Replace the context's flags (e.g. turn PQH_CTX_PROFILE on for a few runs).  Unprofiled batch runs
 * replay the batch's launch sequence as one captured hipGraph; profiled runs launch each kernel
 * between HIP events. */
int pqh_ctx_set_flags(pqh_ctx* ctx, uint32_t flags);
/* Bytes of pinned host memory the context's pool holds (payload blocks in use by host / staged
 * batches plus the free ones it keeps for reuse): the bound of a streaming ring's pinned staging. */
int64_t pqh_ctx_pinned_bytes(const pqh_ctx* ctx);
void pqh_ctx_destroy(pqh_ctx* ctx);
const char* pqh_last_error(const pqh_ctx* ctx);
/* The HIP stream every decode of this context is ordered on (a hipStream_t): a run is enqueued on
 * it, and branches of the run that the context puts on its own side stream (the byte-array chain,
 * the nesting kernels) fork from and rejoin it inside the run, so work a caller orders on this
 * stream before / after pqh_batch_run sees the whole decode before / after it. */
void* pqh_ctx_stream(pqh_ctx* ctx);

int pqh_malloc(pqh_ctx* ctx, void** dptr, size_t bytes);
int pqh_free(pqh_ctx* ctx, void* dptr);
int pqh_host_alloc(pqh_ctx* ctx, void** hptr, size_t bytes); /* pinned */
int pqh_host_free(pqh_ctx* ctx, void* hptr);
/* Copies between HBM and pageable (or pinned) host memory, ordered after the work already on the
 * context stream; they return when the host buffer is filled / reusable.  They stage through the
 * context's pinned bounce buffer, so the HIP runtime never pins pageable memory on the fly. */
int pqh_memcpy_h2d(pqh_ctx* ctx, void* dst, const void* src, size_t bytes);
int pqh_memcpy_d2h(pqh_ctx* ctx, void* dst, const void* src, size_t bytes);
/* Asynchronous copy on the context stream from PINNED host memory (pqh_host_alloc) to HBM. */
int pqh_memcpy_h2d_pinned_async(pqh_ctx* ctx, void* dst, const void* pinned_src, size_t bytes);
int pqh_sync(pqh_ctx* ctx);

/* Plan a batch: copies the page/chunk tables, sizes and allocates scratch and outputs.
 * d_payload must stay valid and unchanged until the batch is destroyed and must have
 * PQH_PAYLOAD_PAD readable bytes after payload_bytes. */
int pqh_batch_create(pqh_ctx* ctx, const pqh_chunk* chunks, int32_t num_chunks,
                     const pqh_page* pages, int32_t num_pages, const void* d_payload,
                     int64_t payload_bytes, pqh_batch** out);
/* Enqueue the whole decode on the context stream (asynchronous; may be re-run).  Small flat batches
 * (one k_flat launch) and chunks of PLAIN byte-array pages (k_ba_chain) decode speculatively: a
 * speculation that fails is only seen by pqh_batch_sync, so several runs before one sync all replay
 * the speculative path, and their outputs are not the reference's until that sync has re-decoded
 * the batch. */
int pqh_batch_run(pqh_batch* batch);
/* Wait for the last run and copy back per-page results.  When the last run's speculation failed
 * (see pqh_batch_run) or a byte-array output came out short, this re-decodes the batch before
 * returning -- on the three-kernel / scratch path, which the batch then keeps for every later run
 * (pqh_batch_paths counts these fallbacks). */
int pqh_batch_sync(pqh_batch* batch);
/* Which decode paths the batch takes now, and how often pqh_batch_sync fell back (for benchmarks
 * that must report whether a timed run used a fallback path). */
typedef struct pqh_batch_paths {
  int32_t flat_active;       /* runs launch the one k_flat kernel */
  int32_t flat_fallbacks;    /* k_flat speculations that failed (then the three kernels) */
  int32_t ba_fuse_active;    /* runs launch k_ba_chain for PLAIN byte-array chunks */
  int32_t ba_fuse_fallbacks; /* k_ba_chain verifications that failed (then the scratch path) */
  int32_t regrows;           /* re-decodes after growing short byte-array outputs */
  int32_t graph_replay;      /* unprofiled runs replay a captured hipGraph */
  int32_t reserved[2];
} pqh_batch_paths;
int pqh_batch_path_info(const pqh_batch* batch, pqh_batch_paths* out);
int pqh_batch_chunk_out(const pqh_batch* batch, int32_t chunk, pqh_chunk_out* out);
/* Nesting outputs of one chunk (after pqh_batch_sync).  Chunks with max_rep > PQH_MAX_NEST return
 * PQH_ERR_NOT_IMPLEMENTED. */
int pqh_batch_nesting(const pqh_batch* batch, int32_t chunk, pqh_nest_out* out);
int pqh_batch_page_results(const pqh_batch* batch, pqh_page_result* out, int32_t num_pages);
/* Compat path: one page's pageReader.readValues(size) result (reference
 * interfaces.go:11-18, page_v1.go:33-63, page_v2.go:31-60) copied to HOST buffers after
 * pqh_batch_sync, for a cgo shim that boxes it into []interface{} + packedArray levels.
 * Level slots [first, first + count) of the page (count clipped to the page, as readValues clips
 * size); def_levels / rep_levels receive num_slots bytes each (NULL = skip); fixed-width values
 * go to `values` (num_non_null * value_size bytes), byte arrays to offsets (num_non_null + 1,
 * relative to the first returned value) + data (num_bytes); value_nil (NULL = skip) receives
 * num_non_null bytes (value_nil_cap bytes available, PQH_ERR_ARG when fewer), 1 where the value is
 * the reference's nil (INT96, see pqh_chunk_out), which the shim boxes as a nil interface{}.  With NULL value buffers only the sizes are filled in.  On a readValues error (out->status != PQH_OK) nothing is copied, as the
 * reference returns nil slices.  Errors are those of the whole-page call the reference makes
 * (ColumnStore.readNextPage, data_store.go:236-260); a ranged call reports a level error once its
 * range reaches the failing slot and a value error once its values reach the failing value. */
int pqh_batch_page_read(const pqh_batch* batch, int32_t page, int64_t first, int64_t count, void* values,
                        int64_t values_cap, int64_t* offsets, int64_t offsets_cap, uint8_t* data,
                        int64_t data_cap, uint8_t* def_levels, uint8_t* rep_levels, uint8_t* value_nil,
                        int64_t value_nil_cap, pqh_page_values* out);
/* Kernel timing accumulated since the last reset (requires PQH_CTX_PROFILE). */
int pqh_batch_kernel_stats(const pqh_batch* batch, pqh_kernel_stat* out, int32_t max_stats,
                           int32_t* num_stats);
int pqh_batch_reset_stats(pqh_batch* batch);
/* Algorithmic bytes of one run: payload bytes read once, dictionary bytes once per chunk, and
 * decoded bytes written (values, levels, offsets, byte data). */
int pqh_batch_traffic(const pqh_batch* batch, double* bytes_read, double* bytes_written);
void pqh_batch_destroy(pqh_batch* batch);

/* ---------------------------------------------------------------------------------------------
 * Host side: file footer, page walker, decompression.  Replaces NewFileReader's footer read
 * (file_meta.go:18-73), readChunk/readPages (chunk_reader.go:182-362) and readPageBlock /
 * newBlockReader (chunk_reader.go:161-180, compress.go:131-152).  No GPU needed.
 * ------------------------------------------------------------------------------------------- */

typedef struct pqh_file pqh_file;
typedef struct pqh_host_batch pqh_host_batch;

int pqh_file_open(const char* path, pqh_file** out);
/* Reads from memory; the caller keeps data alive until pqh_file_close. */
int pqh_file_open_memory(const void* data, int64_t len, pqh_file** out);
void pqh_file_close(pqh_file* f);
const char* pqh_file_error(const pqh_file* f);
int32_t pqh_file_num_row_groups(const pqh_file* f);
int64_t pqh_file_num_rows(const pqh_file* f);
int64_t pqh_file_row_group_num_rows(const pqh_file* f, int32_t row_group);
int32_t pqh_file_num_columns(const pqh_file* f);
/* Leaf column metadata; path is the dot-joined schema path (Column.FlatName). */
int pqh_file_column(const pqh_file* f, int32_t column, pqh_column* out, char* path,
                    int32_t path_capacity);
/* The full path / schema element name as bytes (names may hold any bytes, NULs included): copies
 * min(length, cap) bytes, returns the length (-1: no such column / element). */
int32_t pqh_file_column_path(const pqh_file* f, int32_t column, char* buf, int32_t cap);
int32_t pqh_file_schema_name(const pqh_file* f, int32_t i, char* buf, int32_t cap);

/* readRowGroupData's checks of column `column` in row group `rg` before any of its pages is read
 * (reference chunk_reader.go:381-393 and readChunk :299-324 when selected, skipChunk :271-297
 * when not): PQH_OK, PQH_ERR_SCHEMA (no such chunk / no metadata / wrong type) or PQH_ERR_IO
 * (file_path set, negative offset).  A row group fails at the first column (in schema order)
 * that fails here or whose chunk fails to load. */
int pqh_file_chunk_check(const pqh_file* f, int32_t rg, int32_t column, int32_t selected);

/* The caller's codec registry (the reference's `compressors` map, compress.go:16-33,160-187; by
 * default UNCOMPRESSED, GZIP, SNAPPY and ZSTD, as its init registers them).  A chunk whose codec is
 * registered but not decoded by this library (any codec but UNCOMPRESSED / SNAPPY / GZIP) fails its
 * load with PQH_ERR_UNSUPPORTED_CODEC before any of its pages is read: the caller decodes that chunk
 * with the reference's own readChunk / pageReader path.  A codec in no registry fails
 * as the reference fails it (decompressBlock: "method not supported"): PQH_ERR_DECOMPRESS at the
 * chunk's first page block, after that page's header and CRC checks.  The cgo shim passes the keys of
 * GetRegisteredBlockCompressors() (compress.go:164-176). */
int pqh_file_set_codecs(pqh_file* f, const int32_t* codecs, int32_t num_codecs);

/* The schema as a flat DFS list (FileMetaData.schema, root first), with the levels the reader
 * derives for every node (readGroupSchema / readColumnSchema, schema.go:893-990): what the record
 * assembly (Column.getData, schema.go:216-312) walks. */
typedef struct pqh_schema_element {
  int32_t physical_type; /* enum pqh_physical_type, -1 for groups */
  int32_t type_length;
  int32_t repetition;    /* 0 REQUIRED, 1 OPTIONAL, 2 REPEATED, -1 unset (root) */
  int32_t num_children;  /* 0 for leaves */
  int32_t column;        /* leaves: index for pqh_file_column / pqh_file_load, else -1 */
  int32_t max_def;       /* the node's maximum definition level */
  int32_t max_rep;       /* the node's maximum repetition level */
  int32_t reserved;
} pqh_schema_element;
int32_t pqh_file_num_schema_elements(const pqh_file* f);
int pqh_file_schema_element(const pqh_file* f, int32_t index, pqh_schema_element* out, char* name,
                            int32_t name_capacity);

/* Walk and decompress the pages of the given leaf columns for row groups [rg_begin, rg_end),
 * producing a page table and one payload of page images (8-byte aligned images). */
int pqh_file_load(pqh_file* f, int32_t rg_begin, int32_t rg_end, const int32_t* columns,
                  int32_t num_columns, int32_t validate_crc, pqh_host_batch** out);
int32_t pqh_host_batch_num_chunks(const pqh_host_batch* hb);
int32_t pqh_host_batch_num_pages(const pqh_host_batch* hb);
const pqh_chunk* pqh_host_batch_chunks(const pqh_host_batch* hb);
const pqh_page* pqh_host_batch_pages(const pqh_host_batch* hb);
const uint8_t* pqh_host_batch_payload(const pqh_host_batch* hb);
int64_t pqh_host_batch_payload_bytes(const pqh_host_batch* hb);
/* Host time spent in decompression / thrift parsing during pqh_file_load (seconds). */
double pqh_host_batch_decompress_seconds(const pqh_host_batch* hb);
void pqh_host_batch_free(pqh_host_batch* hb);

/* Upload a host batch (pinned staging, async H2D on the context stream) and plan it.  The
 * returned batch owns the device copy of the payload. */
int pqh_batch_create_from_host(pqh_ctx* ctx, const pqh_host_batch* hb, pqh_batch** out);

/* End-to-end mode ("pinned H2D on a side stream"; north star: "Decompressed page
 * buffers are staged in HBM with pinned hipMemcpyAsync on a side stream").  Replaces the page-bytes
 * hand-off of readPageBlock -> dataPageReaderV1/V2.read (chunk_reader.go:161-180, page_v2.go:79-131)
 * for a whole batch.  pqh_batch_create_staged keeps a pinned host copy of hb's decompressed page
 * images (the state host decompression leaves them in) plus an HBM payload buffer;
 * pqh_batch_run_staged enqueues the pinned->HBM copy on the context's copy stream and the decode on
 * the compute stream behind it, so successive staged batches (e.g. one per row group) overlap
 * batch i+1's copy with batch i's decode.  A repeat run's copy waits for the previous decode of the
 * same batch.  Asynchronous: pqh_batch_sync / pqh_sync wait. */
int pqh_batch_create_staged(pqh_ctx* ctx, const pqh_host_batch* hb, pqh_batch** out);
/* Device codecs: load with PQH_LOAD_DEVICE_SNAPPY and the pages of SNAPPY chunks stay compressed in
 * the host batch's payload (the SOURCE payload); pqh_host_batch_image_bytes is the size of the page
 * images they rebuild.  Batches made from such a host batch (pqh_batch_create_from_host /
 * pqh_batch_create_staged) upload (or stage) the source payload and begin every run with k_snappy
 * (one wave per page) rebuilding the images in HBM.  A chunk whose page fails to decompress, or
 * whose decoded size differs from the header, reports PQH_ERR_DECOMPRESS like the host walker
 * (readPageBlock / newBlockReader, compress.go:131-152): it fails the whole chunk unless a page
 * before it already failed on the host. */
#define PQH_LOAD_DEVICE_SNAPPY 1u
/* The same for GZIP chunks (gzipCompressor.DecompressBlock, compress.go:64-77): their pages travel
 * compressed and k_gzip (one workgroup per page: Go's multistream gzip.Reader rules for members,
 * headers and CRC-32 / ISIZE trailers; RFC 1951 inflate) rebuilds the images.  The flags combine. */
#define PQH_LOAD_DEVICE_GZIP 2u
int pqh_file_load_ex(pqh_file* f, int32_t rg_begin, int32_t rg_end, const int32_t* columns, int32_t num_columns,
                     int32_t validate_crc, uint32_t flags, pqh_host_batch** out);

/* pqh_file_load_ex whose payload is written straight into pinned host memory from `ctx`'s pool
 * (reused across loads): pqh_batch_create_staged adopts it without a copy, so the page bytes go
 * file -> pinned payload (one decompression or copy, by the walker threads) -> HBM.  The block
 * returns to the pool when the host batch and every staged batch made from it are freed; destroy
 * the context last. */
int pqh_file_load_pinned(pqh_ctx* ctx, pqh_file* f, int32_t rg_begin, int32_t rg_end, const int32_t* columns,
                         int32_t num_columns, int32_t validate_crc, uint32_t flags, pqh_host_batch** out);
int32_t pqh_host_batch_num_codec_pages(const pqh_host_batch* hb);
const pqh_codec_page* pqh_host_batch_codec_pages(const pqh_host_batch* hb);
int64_t pqh_host_batch_image_bytes(const pqh_host_batch* hb);
/* Decompress pages on the device, synchronously (the k_snappy step of a batch run, on its own):
 * d_src / d_dst as described by `pages` (host array), status[i] = PQH_OK or PQH_ERR_DECOMPRESS. */
int pqh_decompress_pages(pqh_ctx* ctx, const pqh_codec_page* pages, int32_t num_pages, const void* d_src,
                         void* d_dst, int32_t* status);

/* The RLE / bit-packing hybrid decoder alone (reference hybridDecoder, hybrid_decoder.go:81-165, the
 * levelDecoder of interfaces.go): n values of width `width` (0..32) from the stream at d_stream
 * (device memory, len bytes, followed by PQH_PAYLOAD_PAD readable bytes) into d_out (device, n
 * uint32), through the device's run walk and unpack (group = 8: the level path, 4: the dictionary
 * path's 4-value groups).  *status = the first error (PQH_OK if none), *values = the values decoded
 * before it (n if none).  Synchronous on the context stream. */
int pqh_hybrid_decode(pqh_ctx* ctx, const void* d_stream, int64_t len, int32_t width, int64_t n, int32_t group,
                      uint32_t* d_out, int32_t* status, int64_t* values);
int pqh_batch_run_staged(pqh_batch* batch);

#ifdef __cplusplus
}
#endif

#endif /* PQHIP_H */
