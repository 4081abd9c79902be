/*
 * pqgen.h — Parquet file generator that mirrors the conventions of the reference WRITER
 * (github.com/fraugster/parquet-go file_writer.go / chunk_writer.go / page_v1.go / page_v2.go /
 * page_dict.go / hybrid_encoder.go / deltabp_encoder.go), SURVEY.md Appendix A.7:
 *
 *   - hybrid streams are ONE bit-packed run padded to 8 (hybrid_encoder.go:55-70);
 *   - dictionary per chunk while <= 32767 distinct values, index width bits.Len(len(dict)),
 *     dictionary page PLAIN (chunk_writer.go:185-209, page_v1.go:185, page_dict.go:97);
 *   - a page is cut after the record that brings the reference's size estimate to >= the max page
 *     size (data_store.go:138-159), 1 MiB by default;
 *   - DELTA_BINARY_PACKED blocks of 128 values in 4 miniblocks (chunk_writer.go:48-78);
 *   - V1 levels RLE with a u32 length prefix; V2 levels raw with lengths in the header.
 *
 * This is tooling (test fixtures, bench inputs), not the decode path and not the oracle.
 */
#ifndef PQGEN_H
#define PQGEN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pqg_schema_element {
  const char* name;
  int32_t type;           /* parquet.Type, or -1 for a group */
  int32_t type_length;
  int32_t repetition;     /* 0 REQUIRED, 1 OPTIONAL, 2 REPEATED, -1 unset (root) */
  int32_t num_children;
  int32_t converted_type; /* -1 none */
} pqg_schema_element;

typedef struct pqg_column_data {
  int32_t encoding;           /* non-dictionary encoding (PLAIN, DELTA_BINARY_PACKED, RLE (bool), DLBA, DBA) */
  int32_t use_dict;           /* reference ColumnStore.useDict: dictionary allowed */
  const uint8_t* values;      /* fixed: num_values * size bytes; byte arrays: data */
  const int64_t* offsets;     /* byte arrays: num_values + 1 */
  int64_t num_values;         /* not-null values in the whole file */
  const uint8_t* def_levels;  /* num_slots bytes, NULL when max_def == 0 */
  const uint8_t* rep_levels;  /* num_slots bytes, NULL when max_rep == 0 */
  int64_t num_slots;          /* level slots in the whole file */
  int64_t dict_page_limit;    /* 0: reference writer; > 0: mid-chunk fallback once the dictionary page
                                 would exceed this many bytes */
} pqg_column_data;

typedef struct pqg_options {
  int32_t data_page_v2;
  int32_t codec;            /* 0 none, 1 snappy, 2 gzip */
  int64_t max_page_size;    /* 0 => 1 MiB */
  int32_t enable_crc;
  int32_t num_threads;      /* 0 => hardware concurrency */
  int32_t no_fast_paths;    /* 1: every chunk through the general page-cut loop (tests: same bytes) */
} pqg_options;

/* Write a whole file to memory.  rg_rows[i] = records in row group i. */
int pqg_write(const pqg_schema_element* schema, int32_t num_schema, const pqg_column_data* columns,
              int32_t num_columns, const int64_t* rg_rows, int32_t num_row_groups,
              const pqg_options* opt, uint8_t** out, int64_t* out_len, char* err, int32_t err_cap);
void pqg_free(uint8_t* p);

/* Streaming writer for files too large to build in one call (the 1B-row bench file): row groups are
 * encoded batch by batch (each call's columns hold exactly its rows) and appended to a caller's
 * buffer at *pos ("PAR1" first); finish appends the footer, its length and "PAR1".  The file is
 * byte-identical to pqg_write of the same rows. */
typedef struct pqg_stream pqg_stream;
pqg_stream* pqg_stream_open(const pqg_schema_element* schema, int32_t num_schema, const pqg_options* opt, char* err,
                            int32_t err_cap);
int pqg_stream_write(pqg_stream* s, const pqg_column_data* columns, int32_t num_columns, const int64_t* rg_rows,
                     int32_t num_row_groups, uint8_t* dst, int64_t cap, int64_t* pos, char* err, int32_t err_cap);
int pqg_stream_finish(pqg_stream* s, uint8_t* dst, int64_t cap, int64_t* pos, char* err, int32_t err_cap);
void pqg_stream_close(pqg_stream* s);

/* The mixed-encoding bench workload (north_star's 1B-row file: BASELINE configs[1]'s six columns plus
 * configs[2]'s DELTA timestamps), generated per row group from a counter-based hash so any row group
 * is regenerated exactly: int32 from a 1000-entry dictionary, int64 uniform, float from a 256-entry
 * dictionary, double (1% null: f64_def per row, f64 the non-null values compacted), boolean,
 * 16-byte uuid, int64 timestamps rising by 1e6 + U[0, 4096) from a per-row-group base.  Returns the
 * non-null double count.  threads <= 0: hardware concurrency (at most 16). */
void pqg_mixed_dicts(uint64_t seed, int32_t* d_i32, float* d_f32);
int64_t pqg_mixed_row_group(uint64_t seed, int32_t g, int64_t rows, int32_t* i32, int64_t* i64, float* f32,
                            double* f64, uint8_t* f64_def, uint8_t* b, uint8_t* uuid, int64_t* ts, int32_t threads);

/* Encoders exposed for unit tests: the reference writer's stream formats. */
int64_t pqg_hybrid_encode(int32_t width, const int32_t* values, int64_t n, uint8_t* out, int64_t cap);
int64_t pqg_delta_encode32(const int32_t* values, int64_t n, uint8_t* out, int64_t cap);
int64_t pqg_delta_encode64(const int64_t* values, int64_t n, uint8_t* out, int64_t cap);

#ifdef __cplusplus
}
#endif
#endif
