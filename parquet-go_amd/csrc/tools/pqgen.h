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
} pqg_options;

/* Write a whole file to memory.  rg_rows[i] = records in row group i. */
int pqg_write(const pqg_schema_element* schema, int32_t num_schema, const pqg_column_data* columns,
              int32_t num_columns, const int64_t* rg_rows, int32_t num_row_groups,
              const pqg_options* opt, uint8_t** out, int64_t* out_len, char* err, int32_t err_cap);
void pqg_free(uint8_t* p);

/* Encoders exposed for unit tests: the reference writer's stream formats. */
int64_t pqg_hybrid_encode(int32_t width, const int32_t* values, int64_t n, uint8_t* out, int64_t cap);
int64_t pqg_delta_encode32(const int32_t* values, int64_t n, uint8_t* out, int64_t cap);
int64_t pqg_delta_encode64(const int64_t* values, int64_t n, uint8_t* out, int64_t cap);

#ifdef __cplusplus
}
#endif
#endif
