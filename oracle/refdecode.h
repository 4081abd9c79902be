/*
 * refdecode.h — CPU ORACLE (test infrastructure only; never part of the product path).
 *
 * A plain-C restatement of the page-decode algorithm of github.com/fraugster/parquet-go
 * (reference mounted at /root/reference).  Every function restates one Go function as a
 * streaming state machine, keeping the reference's quirks; each one cites
 * the file:line it follows.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load this code, and only as the checker / CPU baseline.
 *
 * Parity pinning: the bit-unpack primitive is pinned by the reference's known-answer tables
 * (bitpacking32_test.go:25-654, bitpacking64_test.go:25-1744 -> tests/golden/bitpack*_kat.json)
 * and the decoders are cross-checked against pyarrow 25.0.0 on spec-conforming files.  The Go
 * reference itself cannot be built here (no Go toolchain); see DESIGN.md "Oracle".
 *
 * Status / phase codes are the public ones of include/pqhip.h.
 */
#ifndef PQ_REFDECODE_H
#define PQ_REFDECODE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_column {
  int32_t physical_type;
  int32_t type_length;
  int32_t max_def;
  int32_t max_rep;
} orc_column;

typedef struct orc_page {
  int32_t page_type;     /* 0 DATA_PAGE, 3 DATA_PAGE_V2 */
  int32_t num_values;
  int32_t encoding;
  int32_t def_levels_byte_length;
  int32_t rep_levels_byte_length;
} orc_page;

/* Decoded dictionary page (dictPageReader.values, page_dict.go:35-72). */
typedef struct orc_dict {
  int32_t num_values;
  int32_t value_size;   /* fixed-size element bytes, 0 for byte arrays */
  uint8_t *values;      /* fixed: num_values * value_size bytes; byte arrays: data */
  int64_t *offsets;     /* byte arrays: num_values + 1 */
  int64_t num_bytes;
  int32_t nil_last;     /* the last entry is the reference's nil: an INT96 dictionary page whose
                           last value is short (type_int96.go:21-42); its 12 bytes are zeros */
  int32_t reserved;
} orc_dict;

typedef struct orc_out {
  int32_t status;
  int32_t phase;
  int64_t index;
  int32_t num_values;   /* level slots decoded (n) */
  int32_t nn;           /* not-null count */
  uint8_t *def;         /* n bytes or NULL (max_def == 0) */
  uint8_t *rep;         /* n bytes or NULL (max_rep == 0) */
  int32_t value_size;   /* bytes per value, 0 for byte arrays */
  uint8_t *values;      /* nn * value_size bytes (fixed), or byte array data */
  int64_t values_bytes;
  int64_t *offsets;     /* byte arrays: num_offsets (nn + 1, fewer when the values fail) */
  int64_t num_offsets;
  uint8_t *nil;         /* NULL, or nn bytes: 1 = the value slot is the reference's nil (INT96: a short
                           last PLAIN value, or the nil entry of a short dictionary), zeros in values */
  int64_t num_nil;
} orc_out;

int orc_abi_version(void);

/* unpack8int32_w / unpack8int64_w (bitbacking32.go:10-44, bitpacking64.go:10) */
void orc_unpack8_int32(int32_t width, const uint8_t *data, int32_t out[8]);
void orc_unpack8_int64(int32_t width, const uint8_t *data, int64_t out[8]);
void orc_pack8_int32(int32_t width, const int32_t in[8], uint8_t *data);
void orc_pack8_int64(int32_t width, const int64_t in[8], uint8_t *data);

/* Decode n values of a hybrid RLE/bit-packed stream of the given width (hybridDecoder.next,
 * hybrid_decoder.go:81-165).  Returns the status; *decoded = values produced before an error. */
int orc_hybrid_decode(int32_t width, const uint8_t *buf, int64_t len, int32_t n, int32_t *out,
                      int32_t *decoded);
/* deltaBitPackDecoder32/64 (deltabp_decoder.go): decode up to n values. */
int orc_delta_decode32(const uint8_t *buf, int64_t len, int32_t n, int32_t *out, int32_t *decoded,
                       int32_t *values_count);
int orc_delta_decode64(const uint8_t *buf, int64_t len, int32_t n, int64_t *out, int32_t *decoded,
                       int32_t *values_count);

/* dictPageReader.read (page_dict.go:35-72) on a decompressed dictionary page image. */
int orc_decode_dict_page(const orc_column *col, int32_t num_values, int32_t encoding,
                         const uint8_t *img, int64_t img_len, orc_dict *out);
/* ... with the index of the first value that failed (the values read before it). */
int orc_decode_dict_page_ex(const orc_column *col, int32_t num_values, int32_t encoding,
                            const uint8_t *img, int64_t img_len, orc_dict *out, int64_t *err_index);
void orc_dict_free(orc_dict *d);

/* getValuesDecoder (chunk_reader.go:106-159): PQH_OK or PQH_ERR_UNSUPPORTED. */
int orc_select(const orc_column *col, int32_t encoding);

/* dataPageReaderV1/V2 .read + .readValues(numValues) (page_v1.go:33-122, page_v2.go:31-131) on a
 * page image (V1: decompressed block; V2: raw levels followed by the decompressed values). */
int orc_decode_page(const orc_column *col, const orc_page *pg, const uint8_t *img, int64_t img_len,
                    const orc_dict *dict, orc_out *out);
void orc_out_free(orc_out *o);

#ifdef __cplusplus
}
#endif
#endif
