/*
 * refdecode.c — CPU ORACLE (test infrastructure only).  See refdecode.h.
 *
 * Restates, value by value, the streaming decoders of github.com/fraugster/parquet-go.  The code
 * is deliberately a state machine (the reference's shape), not the two-pass parallel design of
 * the HIP kernels, so that the two implementations are independent.
 */
#include "refdecode.h"

#include <stdlib.h>
#include <string.h>

#include "../include/pqhip.h"

#define ORC_ABI 2

int orc_abi_version(void) { return ORC_ABI; }

/* ---------------------------------------------------------------------------------------------
 * bytes.Reader (Go stdlib) over a sub-slice.  io.LimitReader over a bytes.Reader behaves as a
 * bytes.Reader over the shorter slice, so one type models every reader the decoders see.
 * ------------------------------------------------------------------------------------------- */
typedef struct {
  const uint8_t *b;
  int64_t len;
  int64_t pos;
} rd_t;

static void rd_init(rd_t *r, const uint8_t *b, int64_t len) {
  r->b = b;
  r->len = len < 0 ? 0 : len;
  r->pos = 0;
}

static int64_t rd_avail(const rd_t *r) { return r->len - r->pos; }

/* bytes.Reader.Read: EOF only when nothing is left; otherwise a (possibly short) copy. */
static int rd_read(rd_t *r, uint8_t *dst, int64_t n, int64_t *got) {
  if (r->pos >= r->len) {
    *got = 0;
    return PQH_ERR_EOF;
  }
  int64_t k = rd_avail(r);
  if (k > n) k = n;
  if (dst && k > 0) memcpy(dst, r->b + r->pos, (size_t)k);
  r->pos += k;
  *got = k;
  return PQH_OK;
}

/* io.ReadFull: EOF if nothing read, ErrUnexpectedEOF if short, nothing for n == 0. */
static int rd_read_full(rd_t *r, uint8_t *dst, int64_t n) {
  if (n <= 0) return PQH_OK;
  int64_t k = rd_avail(r);
  if (k <= 0) return PQH_ERR_EOF;
  if (k < n) {
    if (dst) memcpy(dst, r->b + r->pos, (size_t)k);
    r->pos += k;
    return PQH_ERR_UNEXPECTED_EOF;
  }
  if (dst) memcpy(dst, r->b + r->pos, (size_t)n);
  r->pos += n;
  return PQH_OK;
}

static int rd_byte(rd_t *r, uint8_t *b) {
  if (r->pos >= r->len) return PQH_ERR_EOF;
  *b = r->b[r->pos++];
  return PQH_OK;
}

/* binary.ReadUvarint (encoding/binary). */
static int rd_uvarint(rd_t *r, uint64_t *out) {
  uint64_t x = 0;
  unsigned s = 0;
  for (int i = 0; i < 10; i++) {
    uint8_t b;
    if (rd_byte(r, &b) != PQH_OK) return i > 0 ? PQH_ERR_UNEXPECTED_EOF : PQH_ERR_EOF;
    if (b < 0x80) {
      if (i == 9 && b > 1) return PQH_ERR_VARINT_OVERFLOW;
      *out = x | ((uint64_t)b << s);
      return PQH_OK;
    }
    x |= (uint64_t)(b & 0x7f) << s;
    s += 7;
  }
  return PQH_ERR_VARINT_OVERFLOW;
}

/* binary.ReadVarint: zig-zag. */
static int rd_varint(rd_t *r, int64_t *out) {
  uint64_t ux;
  int st = rd_uvarint(r, &ux);
  if (st) return st;
  int64_t x = (int64_t)(ux >> 1);
  if (ux & 1) x = ~x;
  *out = x;
  return PQH_OK;
}

/* readUVariant32 (helpers.go:151-167) */
static int rd_uvar32(rd_t *r, int32_t *out) {
  uint64_t v;
  int st = rd_uvarint(r, &v);
  if (st) return st;
  if (v > 0x7fffffffULL) return PQH_ERR_INT32_RANGE;
  *out = (int32_t)v;
  return PQH_OK;
}

/* readVariant32 (helpers.go:169-185) */
static int rd_var32(rd_t *r, int32_t *out) {
  int64_t v;
  int st = rd_varint(r, &v);
  if (st) return st;
  if (v > 2147483647LL || v < -2147483648LL) return PQH_ERR_INT32_RANGE;
  *out = (int32_t)v;
  return PQH_OK;
}

/* ---------------------------------------------------------------------------------------------
 * Bit packing: value j of a group of 8 occupies bits [j*w, (j+1)*w) of the little-endian byte
 * string, least significant bit first (bitpack_gen.go:19-59; unpack8int32_13 at
 * bitbacking32.go:383-393 is one instance).
 * ------------------------------------------------------------------------------------------- */
static uint64_t get_bits(const uint8_t *data, int64_t bit, int32_t w) {
  uint64_t v = 0;
  for (int32_t k = 0; k < w; k++) {
    int64_t b = bit + k;
    v |= (uint64_t)((data[b >> 3] >> (b & 7)) & 1) << k;
  }
  return v;
}

void orc_unpack8_int32(int32_t w, const uint8_t *data, int32_t out[8]) {
  for (int j = 0; j < 8; j++) out[j] = (int32_t)(uint32_t)get_bits(data, (int64_t)j * w, w);
}

void orc_unpack8_int64(int32_t w, const uint8_t *data, int64_t out[8]) {
  for (int j = 0; j < 8; j++) out[j] = (int64_t)get_bits(data, (int64_t)j * w, w);
}

static void put_bits(uint8_t *data, int64_t bit, int32_t w, uint64_t v) {
  for (int32_t k = 0; k < w; k++) {
    int64_t b = bit + k;
    if ((v >> k) & 1) data[b >> 3] |= (uint8_t)(1u << (b & 7));
  }
}

void orc_pack8_int32(int32_t w, const int32_t in[8], uint8_t *data) {
  memset(data, 0, (size_t)w);
  for (int j = 0; j < 8; j++) put_bits(data, (int64_t)j * w, w, (uint32_t)in[j]);
}

void orc_pack8_int64(int32_t w, const int64_t in[8], uint8_t *data) {
  memset(data, 0, (size_t)w);
  for (int j = 0; j < 8; j++) put_bits(data, (int64_t)j * w, w, (uint64_t)in[j]);
}

/* ---------------------------------------------------------------------------------------------
 * hybridDecoder (hybrid_decoder.go:29-165)
 * ------------------------------------------------------------------------------------------- */
typedef struct {
  rd_t r;
  int has_r;
  int32_t w;
  int32_t rle_size;
  int32_t bp_run[8];
  uint32_t rle_count;
  int32_t rle_value;
  uint32_t bp_count;
  uint8_t bp_pos;
} hybrid_t;

static void hybrid_new(hybrid_t *h, int32_t w) {
  memset(h, 0, sizeof(*h));
  h->w = w;
  h->rle_size = (w + 7) / 8;
}

/* init (hybrid_decoder.go:68-79): buffered or not, the reader is a bytes.Reader over the rest. */
static void hybrid_init(hybrid_t *h, const uint8_t *b, int64_t len) {
  rd_init(&h->r, b, len);
  h->has_r = 1;
}

/* decodeRLEValue (helpers.go:66-81) */
static int32_t decode_rle_value(const uint8_t *b, int32_t n) {
  uint32_t v = 0;
  for (int32_t i = 0; i < n; i++) v |= (uint32_t)b[i] << (8 * i);
  return (int32_t)v;
}

static int clz32(uint32_t v) {
  if (v == 0) return 32;
  return __builtin_clz(v);
}

/* readRLERunValue (hybrid_decoder.go:115-130) */
static int hybrid_read_rle_value(hybrid_t *h) {
  uint8_t v[4] = {0, 0, 0, 0};
  int64_t got;
  int st = rd_read(&h->r, v, h->rle_size, &got);
  if (st) return st;
  if (got != h->rle_size) return PQH_ERR_UNEXPECTED_EOF;
  h->rle_value = decode_rle_value(v, h->rle_size);
  if (clz32((uint32_t)h->rle_value) < 32 - h->w) return PQH_ERR_RLE_VALUE_TOO_LARGE;
  return PQH_OK;
}

/* readBitPackedRun (hybrid_decoder.go:132-140): a single Read whose short count is ignored; the
 * missing bytes stay zero. */
static int hybrid_read_bp_run(hybrid_t *h) {
  uint8_t data[32];
  memset(data, 0, sizeof(data));
  int64_t got;
  int st = rd_read(&h->r, data, h->w, &got);
  if (st) return st;
  orc_unpack8_int32(h->w, data, h->bp_run);
  return PQH_OK;
}

/* readRunHeader (hybrid_decoder.go:142-165) */
static int hybrid_read_run_header(hybrid_t *h) {
  int32_t hd;
  int st = rd_uvar32(&h->r, &hd);
  if (st) return st;
  if (hd & 1) {
    h->bp_count = (uint32_t)(hd >> 1);
    if (h->bp_count == 0) return PQH_ERR_EMPTY_BP_RUN;
    h->bp_pos = 0;
  } else {
    h->rle_count = (uint32_t)(hd >> 1);
    if (h->rle_count == 0) return PQH_ERR_EMPTY_RLE_RUN;
    return hybrid_read_rle_value(h);
  }
  return PQH_OK;
}

/* next (hybrid_decoder.go:81-113) */
static int hybrid_next(hybrid_t *h, int32_t *out) {
  if (h->w == 0) {
    *out = 0;
    return PQH_OK;
  }
  if (!h->has_r) return PQH_ERR_READER_NOT_INITIALIZED;
  int st;
  if (h->rle_count == 0 && h->bp_count == 0 && h->bp_pos == 0) {
    if ((st = hybrid_read_run_header(h))) return st;
  }
  if (h->rle_count > 0) {
    *out = h->rle_value;
    h->rle_count--;
  } else if (h->bp_count > 0 || h->bp_pos > 0) {
    if (h->bp_pos == 0) {
      if ((st = hybrid_read_bp_run(h))) return st;
      h->bp_count--;
    }
    *out = h->bp_run[h->bp_pos];
    h->bp_pos = (uint8_t)((h->bp_pos + 1) % 8);
  } else {
    return PQH_ERR_EOF;
  }
  return PQH_OK;
}

int orc_hybrid_decode(int32_t width, const uint8_t *buf, int64_t len, int32_t n, int32_t *out,
                      int32_t *decoded) {
  hybrid_t h;
  hybrid_new(&h, width);
  hybrid_init(&h, buf, len);
  for (int32_t i = 0; i < n; i++) {
    int st = hybrid_next(&h, &out[i]);
    if (st) {
      *decoded = i;
      return st;
    }
  }
  *decoded = n;
  return PQH_OK;
}

/* ---------------------------------------------------------------------------------------------
 * deltaBitPackDecoder32 / 64 (deltabp_decoder.go:13-333).  One implementation with the value
 * arithmetic done in uint64 and truncated for the 32-bit variant (Go int32 wraps).
 * ------------------------------------------------------------------------------------------- */
typedef struct {
  rd_t *r;
  int is64;
  int32_t block_size, mb_count, values_count, mbvc;
  uint64_t prev, min_delta;
  uint8_t *widths;
  int32_t cur_mb;
  int32_t cur_w;
  int32_t mb_pos;
  int32_t position;
  uint64_t mb_vals[8];
} delta_t;

static void delta_free(delta_t *d) {
  free(d->widths);
  d->widths = NULL;
}

/* readBlockHeader (:51-86 / :210-245) */
static int delta_read_block_header(delta_t *d) {
  int st;
  if ((st = rd_uvar32(d->r, &d->block_size))) return st;
  if (d->block_size <= 0 && d->block_size % 128 != 0) return PQH_ERR_DELTA_BLOCK_SIZE;
  if ((st = rd_uvar32(d->r, &d->mb_count))) return st;
  if (d->mb_count <= 0 || d->block_size % d->mb_count != 0) return PQH_ERR_DELTA_MINIBLOCKS;
  d->mbvc = d->block_size / d->mb_count;
  if (d->mbvc == 0) return PQH_ERR_DELTA_MINIBLOCKS;
  if ((st = rd_uvar32(d->r, &d->values_count))) return st;
  if (d->values_count < 0) return PQH_ERR_DELTA_VALUE_COUNT;
  if (d->is64) {
    int64_t v;
    if ((st = rd_varint(d->r, &v))) return st;
    d->prev = (uint64_t)v;
  } else {
    int32_t v;
    if ((st = rd_var32(d->r, &v))) return st;
    d->prev = (uint64_t)(int64_t)v;
  }
  return PQH_OK;
}

/* readMiniBlockHeader (:88-111 / :247-270) */
static int delta_read_miniblock_header(delta_t *d) {
  int st;
  if (d->is64) {
    int64_t v;
    if ((st = rd_varint(d->r, &v))) return st;
    d->min_delta = (uint64_t)v;
  } else {
    int32_t v;
    if ((st = rd_var32(d->r, &v))) return st;
    d->min_delta = (uint64_t)(int64_t)v;
  }
  /* make([]uint8, miniBlockCount) + io.ReadFull; the bytes are only inspected when the read
   * succeeds, so a count larger than what is left is a short read. */
  free(d->widths);
  d->widths = NULL;
  int64_t avail = rd_avail(d->r);
  if ((int64_t)d->mb_count > avail) {
    rd_read_full(d->r, NULL, avail > 0 ? avail : 0);
    return avail <= 0 ? PQH_ERR_EOF : PQH_ERR_UNEXPECTED_EOF;
  }
  d->widths = (uint8_t *)malloc((size_t)d->mb_count);
  if (!d->widths) return PQH_ERR_NOMEM;
  if ((st = rd_read_full(d->r, d->widths, d->mb_count))) return st;
  int maxw = d->is64 ? 64 : 32;
  for (int32_t i = 0; i < d->mb_count; i++)
    if (d->widths[i] > maxw) return PQH_ERR_DELTA_BIT_WIDTH;
  d->cur_mb = 0;
  return PQH_OK;
}

/* init (:37-49 / :196-208): block header AND the first miniblock header, eagerly. */
static int delta_init(delta_t *d, rd_t *r, int is64) {
  memset(d, 0, sizeof(*d));
  d->r = r;
  d->is64 = is64;
  int st;
  if ((st = delta_read_block_header(d))) return st;
  return delta_read_miniblock_header(d);
}

/* next (:113-174 / :272-333), including the one-delta read-ahead and the padding skip that
 * indexes miniBlockBitWidth with currentMiniBlock for every remaining miniblock (:158, :317). */
static int delta_next(delta_t *d, uint64_t *out) {
  int st;
  if (d->position >= d->values_count) return PQH_ERR_EOF;
  if (d->position % 8 == 0) {
    if (d->position % d->mbvc == 0) {
      if (d->cur_mb >= d->mb_count) {
        if ((st = delta_read_miniblock_header(d))) return st;
      }
      d->cur_w = d->widths[d->cur_mb];
      d->mb_pos = 0;
      d->cur_mb++;
    }
    int32_t w = d->cur_w;
    uint8_t buf[64];
    memset(buf, 0, sizeof(buf));
    if ((st = rd_read_full(d->r, buf, w))) return st;
    if (d->is64) {
      int64_t v[8];
      orc_unpack8_int64(w, buf, v);
      for (int j = 0; j < 8; j++) d->mb_vals[j] = (uint64_t)v[j];
    } else {
      int32_t v[8];
      orc_unpack8_int32(w, buf, v);
      for (int j = 0; j < 8; j++) d->mb_vals[j] = (uint64_t)(int64_t)v[j];
    }
    d->mb_pos += w;
    if (d->position + 8 >= d->values_count) {
      int64_t l = (int64_t)(d->mbvc / 8) * w - d->mb_pos;
      if (l < 0) return PQH_ERR_DELTA_STREAM;
      rd_read_full(d->r, NULL, l); /* errors ignored */
      for (int32_t i = d->cur_mb; i < d->mb_count; i++) {
        int32_t w2 = d->widths[d->cur_mb]; /* sic: currentMiniBlock, not i */
        if (w2 != 0) rd_read_full(d->r, NULL, (int64_t)(d->mbvc / 8) * w2);
      }
    }
  }
  uint64_t ret = d->prev;
  d->prev += d->mb_vals[d->position % 8] + d->min_delta;
  if (!d->is64) d->prev = (uint64_t)(int64_t)(int32_t)(uint32_t)d->prev;
  d->position++;
  *out = ret;
  return PQH_OK;
}

int orc_delta_decode32(const uint8_t *buf, int64_t len, int32_t n, int32_t *out, int32_t *decoded,
                       int32_t *values_count) {
  rd_t r;
  rd_init(&r, buf, len);
  delta_t d;
  int st = delta_init(&d, &r, 0);
  *decoded = 0;
  *values_count = d.values_count;
  if (st) {
    delta_free(&d);
    return st;
  }
  for (int32_t i = 0; i < n; i++) {
    uint64_t v;
    if ((st = delta_next(&d, &v))) {
      *decoded = i;
      delta_free(&d);
      return st;
    }
    out[i] = (int32_t)(uint32_t)v;
  }
  *decoded = n;
  delta_free(&d);
  return PQH_OK;
}

int orc_delta_decode64(const uint8_t *buf, int64_t len, int32_t n, int64_t *out, int32_t *decoded,
                       int32_t *values_count) {
  rd_t r;
  rd_init(&r, buf, len);
  delta_t d;
  int st = delta_init(&d, &r, 1);
  *decoded = 0;
  *values_count = d.values_count;
  if (st) {
    delta_free(&d);
    return st;
  }
  for (int32_t i = 0; i < n; i++) {
    uint64_t v;
    if ((st = delta_next(&d, &v))) {
      *decoded = i;
      delta_free(&d);
      return st;
    }
    out[i] = (int64_t)v;
  }
  *decoded = n;
  delta_free(&d);
  return PQH_OK;
}

/* ---------------------------------------------------------------------------------------------
 * Output buffers
 * ------------------------------------------------------------------------------------------- */
typedef struct {
  uint8_t *p;
  int64_t len, cap;
} buf_t;

static int buf_reserve(buf_t *b, int64_t extra) {
  if (b->len + extra <= b->cap) return PQH_OK;
  int64_t nc = b->cap ? b->cap * 2 : 256;
  while (nc < b->len + extra) nc *= 2;
  uint8_t *np = (uint8_t *)realloc(b->p, (size_t)nc);
  if (!np) return PQH_ERR_NOMEM;
  b->p = np;
  b->cap = nc;
  return PQH_OK;
}

static int buf_append(buf_t *b, const uint8_t *src, int64_t n) {
  int st = buf_reserve(b, n);
  if (st) return st;
  if (n > 0) memcpy(b->p + b->len, src, (size_t)n);
  b->len += n;
  return PQH_OK;
}

/* ---------------------------------------------------------------------------------------------
 * Value decoders.  Each returns the status of decodeValues(dst[:nn]) and the index of the
 * failing value in *err_index.  Fixed-size values are appended to vals; byte arrays to
 * vals (data) + offs (nn + 1 offsets).
 * ------------------------------------------------------------------------------------------- */
typedef struct {
  int kind;          /* decoder kind below */
  int32_t size;      /* fixed value size (plain) / FLBA length */
  rd_t r;            /* page reader for the values section */
  hybrid_t keys;     /* dict / boolean RLE */
  int keys_ok;
  delta_t delta;     /* delta / DLBA lengths */
  int delta_ok;
  int32_t *lens;     /* DLBA lengths (byteArrayDeltaLengthDecoder.lens) */
  int32_t nlens, lens_pos;
  int32_t *prefix;   /* DBA prefix lengths */
  int32_t nprefix;
} vdec_t;

enum {
  VD_PLAIN_FIXED = 1, /* int32/int64/float/double: binary.Read */
  VD_PLAIN_INT96,
  VD_PLAIN_BA,        /* byteArrayPlainDecoder (length 0 = variable) */
  VD_PLAIN_BOOL,
  VD_RLE_BOOL,
  VD_DICT,
  VD_DELTA32,
  VD_DELTA64,
  VD_DLBA,
  VD_DBA
};

static void vdec_free(vdec_t *v) {
  delta_free(&v->delta);
  free(v->lens);
  free(v->prefix);
  memset(v, 0, sizeof(*v));
}

/* getValuesDecoder (chunk_reader.go:106-159) */
static int vdec_select(const orc_column *col, int32_t enc, vdec_t *v) {
  memset(v, 0, sizeof(*v));
  if (enc == PQH_ENC_PLAIN_DICTIONARY) enc = PQH_ENC_RLE_DICTIONARY;
  switch (col->physical_type) {
    case PQH_BOOLEAN:
      if (enc == PQH_ENC_PLAIN) v->kind = VD_PLAIN_BOOL;
      else if (enc == PQH_ENC_RLE) v->kind = VD_RLE_BOOL;
      else return PQH_ERR_UNSUPPORTED;
      v->size = 1;
      return PQH_OK;
    case PQH_BYTE_ARRAY:
      if (enc == PQH_ENC_PLAIN) v->kind = VD_PLAIN_BA;
      else if (enc == PQH_ENC_DELTA_LENGTH_BYTE_ARRAY) v->kind = VD_DLBA;
      else if (enc == PQH_ENC_DELTA_BYTE_ARRAY) v->kind = VD_DBA;
      else if (enc == PQH_ENC_RLE_DICTIONARY) v->kind = VD_DICT;
      else return PQH_ERR_UNSUPPORTED;
      v->size = 0;
      return PQH_OK;
    case PQH_FIXED_LEN_BYTE_ARRAY:
      if (enc == PQH_ENC_PLAIN) v->kind = VD_PLAIN_BA;
      else if (enc == PQH_ENC_DELTA_BYTE_ARRAY) v->kind = VD_DBA;
      else if (enc == PQH_ENC_RLE_DICTIONARY) v->kind = VD_DICT;
      else return PQH_ERR_UNSUPPORTED;
      v->size = col->type_length;
      return PQH_OK;
    case PQH_FLOAT:
    case PQH_DOUBLE:
    case PQH_INT96:
      if (enc == PQH_ENC_PLAIN) v->kind = col->physical_type == PQH_INT96 ? VD_PLAIN_INT96 : VD_PLAIN_FIXED;
      else if (enc == PQH_ENC_RLE_DICTIONARY) v->kind = VD_DICT;
      else return PQH_ERR_UNSUPPORTED;
      v->size = col->physical_type == PQH_FLOAT ? 4 : col->physical_type == PQH_DOUBLE ? 8 : 12;
      return PQH_OK;
    case PQH_INT32:
    case PQH_INT64:
      if (enc == PQH_ENC_PLAIN) v->kind = VD_PLAIN_FIXED;
      else if (enc == PQH_ENC_DELTA_BINARY_PACKED) v->kind = col->physical_type == PQH_INT32 ? VD_DELTA32 : VD_DELTA64;
      else if (enc == PQH_ENC_RLE_DICTIONARY) v->kind = VD_DICT;
      else return PQH_ERR_UNSUPPORTED;
      v->size = col->physical_type == PQH_INT32 ? 4 : 8;
      return PQH_OK;
    default:
      return PQH_ERR_UNSUPPORTED;
  }
}

/* decodeInt32 over a delta32 decoder (helpers.go:119-131) */
static int decode_int32_all(delta_t *d, int32_t **out, int32_t *count) {
  int32_t n = d->values_count;
  *count = 0;
  int32_t *a = (int32_t *)malloc(sizeof(int32_t) * (size_t)(n > 0 ? n : 1));
  if (!a) return PQH_ERR_NOMEM;
  *out = a;
  for (int32_t i = 0; i < n; i++) {
    uint64_t v;
    int st = delta_next(d, &v);
    if (st) return st;
    a[i] = (int32_t)(uint32_t)v;
  }
  *count = n;
  return PQH_OK;
}

/* byteArrayDeltaLengthDecoder.init (type_bytearray.go:104-116) on v->r */
static int dlba_init(vdec_t *v) {
  delta_t d;
  int st = delta_init(&d, &v->r, 0);
  if (st) {
    delta_free(&d);
    return st;
  }
  st = decode_int32_all(&d, &v->lens, &v->nlens);
  v->nlens = d.values_count;
  delta_free(&d);
  v->lens_pos = 0;
  return st;
}

/* valuesDecoder.init for the selected kind (type_*.go) */
static int vdec_init(vdec_t *v, const uint8_t *b, int64_t len) {
  rd_init(&v->r, b, len);
  int st;
  switch (v->kind) {
    case VD_DICT: { /* dictDecoder.init (type_dict.go:22-38) */
      uint8_t w;
      if ((st = rd_read_full(&v->r, &w, 1))) return st;
      if (w > 32) return PQH_ERR_DICT_BIT_WIDTH;
      hybrid_new(&v->keys, w);
      hybrid_init(&v->keys, v->r.b + v->r.pos, v->r.len - v->r.pos);
      v->keys_ok = 1;
      return PQH_OK;
    }
    case VD_RLE_BOOL: { /* booleanRLEDecoder.init -> hybridDecoder(1).initSize (type_boolean.go:104-107) */
      uint8_t sz[4];
      if ((st = rd_read_full(&v->r, sz, 4))) return st;
      uint32_t size = (uint32_t)sz[0] | ((uint32_t)sz[1] << 8) | ((uint32_t)sz[2] << 16) | ((uint32_t)sz[3] << 24);
      int64_t rem = rd_avail(&v->r);
      int64_t l = (int64_t)size < rem ? (int64_t)size : rem;
      hybrid_new(&v->keys, 1);
      hybrid_init(&v->keys, v->r.b + v->r.pos, l);
      v->r.pos += l;
      v->keys_ok = 1;
      return PQH_OK;
    }
    case VD_DELTA32:
    case VD_DELTA64:
      st = delta_init(&v->delta, &v->r, v->kind == VD_DELTA64);
      v->delta_ok = 1;
      return st;
    case VD_DLBA:
      return dlba_init(v);
    case VD_DBA: { /* byteArrayDeltaDecoder.init (type_bytearray.go:195-211) */
      delta_t d;
      st = delta_init(&d, &v->r, 0);
      if (st) {
        delta_free(&d);
        return st;
      }
      st = decode_int32_all(&d, &v->prefix, &v->nprefix);
      v->nprefix = d.values_count;
      delta_free(&d);
      if (st) return st;
      if ((st = dlba_init(v))) return st;
      if (v->nprefix != v->nlens) return PQH_ERR_DBA_COUNT;
      return PQH_OK;
    }
    default:
      return PQH_OK;
  }
}

/* byteArrayPlainDecoder.next (type_bytearray.go:24-45) */
static int ba_plain_next(vdec_t *v, buf_t *vals, int64_t *len_out) {
  int32_t l = v->size;
  int st;
  if (l == 0) {
    uint8_t b4[4];
    if ((st = rd_read_full(&v->r, b4, 4))) return st;
    l = (int32_t)((uint32_t)b4[0] | ((uint32_t)b4[1] << 8) | ((uint32_t)b4[2] << 16) | ((uint32_t)b4[3] << 24));
    if (l < 0) return PQH_ERR_NEGATIVE_LENGTH;
  } else if (l < 0) {
    return PQH_ERR_NEGATIVE_LENGTH;
  }
  if ((st = buf_reserve(vals, l))) return st;
  if ((st = rd_read_full(&v->r, vals->p + vals->len, l))) return st;
  vals->len += l;
  *len_out = l;
  return PQH_OK;
}

/* byteArrayDeltaLengthDecoder.next (type_bytearray.go:118-131) */
static int dlba_next(vdec_t *v, buf_t *vals, int64_t *len_out) {
  if (v->lens_pos >= v->nlens) return PQH_ERR_EOF;
  int32_t size = v->lens[v->lens_pos];
  if (size < 0) return PQH_ERR_NEGATIVE_DLBA_LENGTH; /* make([]byte, size) panics */
  int st;
  if ((st = buf_reserve(vals, size))) return st;
  if ((st = rd_read_full(&v->r, vals->p + vals->len, size))) return st;
  vals->len += size;
  v->lens_pos++;
  *len_out = size;
  return PQH_OK;
}

static int off_push(buf_t *offs, int64_t v) { return buf_append(offs, (const uint8_t *)&v, 8); }

/* Slot i of dst[:nn] stays the reference's nil (an interface{} never assigned): nil->p becomes an
 * nn-byte mask on the first one. */
static int nil_mark(buf_t *nil, int32_t nn, int32_t i) {
  if (!nil) return PQH_OK;
  if (!nil->p) {
    int st = buf_reserve(nil, nn);
    if (st) return st;
    memset(nil->p, 0, (size_t)nn);
    nil->len = nn;
  }
  nil->p[i] = 1;
  return PQH_OK;
}

static const uint8_t kZero12[12] = {0};

/* decodeValues(dst[:nn]); nil (may be NULL) receives the mask of the slots left nil */
static int vdec_decode(vdec_t *v, const orc_dict *dict, int32_t nn, buf_t *vals, buf_t *offs,
                       int64_t *err_index, buf_t *nil) {
  int st = PQH_OK;
  int32_t i;
  int is_ba = (v->size == 0) || v->kind == VD_DBA || v->kind == VD_DLBA;
  *err_index = 0;
  if (v->kind == VD_DICT) is_ba = dict ? dict->value_size == 0 : 0;
  if (is_ba && (st = off_push(offs, 0))) return st;
  switch (v->kind) {
    case VD_PLAIN_FIXED: /* binary.Read per value (type_int32.go:21-31 etc.) */
      for (i = 0; i < nn; i++) {
        if ((st = buf_reserve(vals, v->size))) return st;
        if ((st = rd_read_full(&v->r, vals->p + vals->len, v->size))) break;
        vals->len += v->size;
      }
      break;
    case VD_PLAIN_INT96: /* int96PlainDecoder.decodeValues (type_int96.go:21-42) */
      for (i = 0; i < nn; i++) {
        uint8_t d[12];
        int64_t got;
        st = rd_read(&v->r, d, 12, &got);
        if (got == 12) {
          if ((st = buf_append(vals, d, 12))) return st;
          continue;
        }
        if (st) break; /* n == 0: io.EOF, returned with the values read so far */
        /* a short read (0 < n < 12, err == nil: bytes.Reader hands out what is left) drops the
         * value and leaves the reader at its end.  Before the last slot, the NEXT iteration's Read
         * returns (0, io.EOF).  On the last slot the loop simply ends: decodeValues returns
         * (len(dst), nil) with dst[nn-1] never assigned -- the reference's nil value.  Its 12
         * output bytes are zeros and the nil mask marks it. */
        if (i == nn - 1) {
          if ((st = buf_append(vals, kZero12, 12))) return st;
          if ((st = nil_mark(nil, nn, i))) return st;
          st = PQH_OK;
          i++;
        } else {
          st = PQH_ERR_EOF;
          i++;
        }
        break;
      }
      break;
    case VD_PLAIN_BA:
      for (i = 0; i < nn; i++) {
        int64_t l;
        if ((st = ba_plain_next(v, vals, &l))) break;
        if (v->size == 0 && (st = off_push(offs, vals->len))) return st;
      }
      break;
    case VD_PLAIN_BOOL: /* booleanPlainDecoder.decodeValues (type_boolean.go:43-69) */
      for (i = 0; i < nn; i += 8) {
        uint8_t byte;
        if ((st = rd_read_full(&v->r, &byte, 1))) break;
        for (int j = 0; j < 8 && i + j < nn; j++) {
          uint8_t bit = (byte >> j) & 1;
          if ((st = buf_append(vals, &bit, 1))) return st;
        }
      }
      break;
    case VD_RLE_BOOL: /* booleanRLEDecoder.decodeValues (type_boolean.go:109-120) */
      for (i = 0; i < nn; i++) {
        int32_t x;
        if ((st = hybrid_next(&v->keys, &x))) break;
        uint8_t b = x == 1;
        if ((st = buf_append(vals, &b, 1))) return st;
      }
      break;
    case VD_DICT: { /* dictDecoder.decodeValues (type_dict.go:40-60) */
      int32_t size = dict ? dict->num_values : 0;
      for (i = 0; i < nn; i++) {
        int32_t key;
        if ((st = hybrid_next(&v->keys, &key))) break;
        if (key < 0 || key >= size) {
          st = PQH_ERR_DICT_INDEX;
          break;
        }
        if (dict->value_size > 0) {
          if ((st = buf_append(vals, dict->values + (int64_t)key * dict->value_size, dict->value_size))) return st;
          /* dst[i] = uniqueValues[key]: the nil entry of a short INT96 dictionary page stays nil */
          if (dict->nil_last && key == size - 1 && (st = nil_mark(nil, nn, i))) return st;
        } else {
          int64_t a = dict->offsets[key], b = dict->offsets[key + 1];
          if ((st = buf_append(vals, dict->values + a, b - a))) return st;
          if ((st = off_push(offs, vals->len))) return st;
        }
      }
      break;
    }
    case VD_DELTA32:
    case VD_DELTA64: /* int32DeltaBPDecoder / int64DeltaBPDecoder .decodeValues */
      for (i = 0; i < nn; i++) {
        uint64_t x;
        if ((st = delta_next(&v->delta, &x))) break;
        if (v->kind == VD_DELTA32) {
          int32_t y = (int32_t)(uint32_t)x;
          if ((st = buf_append(vals, (const uint8_t *)&y, 4))) return st;
        } else {
          if ((st = buf_append(vals, (const uint8_t *)&x, 8))) return st;
        }
      }
      break;
    case VD_DLBA:
      for (i = 0; i < nn; i++) {
        int64_t l;
        if ((st = dlba_next(v, vals, &l))) break;
        if ((st = off_push(offs, vals->len))) return st;
      }
      break;
    case VD_DBA: { /* byteArrayDeltaDecoder.decodeValues (type_bytearray.go:213-240) */
      int64_t prev_off = 0, prev_len = 0; /* previousValue = vals[prev_off : prev_off+prev_len] */
      for (i = 0; i < nn; i++) {
        buf_t suffix = {0, 0, 0};
        int64_t sl;
        if ((st = dlba_next(v, &suffix, &sl))) {
          free(suffix.p);
          break;
        }
        int32_t plen = v->prefix[v->lens_pos - 1];
        if ((int64_t)plen + sl < 0) { /* make([]byte, 0, negative) panics */
          free(suffix.p);
          st = PQH_ERR_NEGATIVE_DLBA_LENGTH;
          break;
        }
        if (prev_len < plen) {
          free(suffix.p);
          st = PQH_ERR_DBA_PREFIX;
          break;
        }
        int64_t start = vals->len;
        if (plen > 0) {
          if ((st = buf_reserve(vals, plen))) {
            free(suffix.p);
            return st;
          }
          memmove(vals->p + vals->len, vals->p + prev_off, (size_t)plen);
          vals->len += plen;
        }
        st = buf_append(vals, suffix.p, sl);
        free(suffix.p);
        if (st) return st;
        prev_off = start;
        prev_len = vals->len - start;
        if ((st = off_push(offs, vals->len))) return st;
      }
      break;
    }
    default:
      return PQH_ERR_UNSUPPORTED;
  }
  if (st) *err_index = i;
  return st;
}

/* ---------------------------------------------------------------------------------------------
 * Dictionary page: dictPageReader.read (page_dict.go:35-72) with getDictValuesDecoder
 * (chunk_reader.go:17-39).
 * ------------------------------------------------------------------------------------------- */
/* getValuesDecoder (chunk_reader.go:106-159): PQH_OK or PQH_ERR_UNSUPPORTED for (type, encoding). */
int orc_select(const orc_column *col, int32_t encoding) {
  vdec_t v;
  int st = vdec_select(col, encoding, &v);
  vdec_free(&v);
  return st;
}

int orc_decode_dict_page(const orc_column *col, int32_t num_values, int32_t encoding,
                         const uint8_t *img, int64_t img_len, orc_dict *out) {
  int64_t ei;
  return orc_decode_dict_page_ex(col, num_values, encoding, img, img_len, out, &ei);
}

int orc_decode_dict_page_ex(const orc_column *col, int32_t num_values, int32_t encoding,
                            const uint8_t *img, int64_t img_len, orc_dict *out, int64_t *err_index) {
  memset(out, 0, sizeof(*out));
  *err_index = 0;
  if (num_values < 0) return PQH_ERR_PAGE_HEADER;
  if (encoding != PQH_ENC_PLAIN && encoding != PQH_ENC_PLAIN_DICTIONARY) return PQH_ERR_DICT_PAGE;
  if (col->physical_type == PQH_BOOLEAN) return PQH_ERR_UNSUPPORTED;
  vdec_t v;
  int st = vdec_select(col, PQH_ENC_PLAIN, &v);
  if (st) return st;
  vdec_init(&v, img, img_len);
  buf_t vals = {0, 0, 0}, offs = {0, 0, 0}, nil = {0, 0, 0};
  int64_t ei;
  st = vdec_decode(&v, NULL, num_values, &vals, &offs, &ei, &nil);
  vdec_free(&v);
  *err_index = st ? ei : 0;
  /* (only an INT96 dictionary's last entry can be nil: a short read of it, type_int96.go:21-42) */
  out->nil_last = nil.p != NULL;
  free(nil.p);
  int is_ba = col->physical_type == PQH_BYTE_ARRAY ||
              (col->physical_type == PQH_FIXED_LEN_BYTE_ARRAY && col->type_length == 0);
  if (st) {
    free(vals.p);
    free(offs.p);
    return st;
  }
  out->num_values = num_values;
  out->values = vals.p;
  out->num_bytes = vals.len;
  if (is_ba) {
    out->value_size = 0;
    out->offsets = (int64_t *)offs.p;
  } else {
    free(offs.p);
    out->value_size = col->physical_type == PQH_FIXED_LEN_BYTE_ARRAY ? col->type_length
                      : col->physical_type == PQH_INT32 || col->physical_type == PQH_FLOAT ? 4
                      : col->physical_type == PQH_INT96 ? 12 : 8;
  }
  return PQH_OK;
}

void orc_dict_free(orc_dict *d) {
  free(d->values);
  free(d->offsets);
  memset(d, 0, sizeof(*d));
}

/* bits.Len16 */
static int32_t bits_len16(int32_t v) {
  int32_t n = 0;
  while (v > 0) {
    n++;
    v >>= 1;
  }
  return n;
}

static void set_err(orc_out *o, int st, int phase, int64_t index) {
  o->status = st;
  o->phase = phase;
  o->index = index;
}

/* ---------------------------------------------------------------------------------------------
 * Data pages: dataPageReaderV1/V2 .read then .readValues(numValues).
 * ------------------------------------------------------------------------------------------- */
int orc_decode_page(const orc_column *col, const orc_page *pg, const uint8_t *img, int64_t img_len,
                    const orc_dict *dict, orc_out *out) {
  memset(out, 0, sizeof(*out));
  int32_t n = pg->num_values;
  if (n < 0) {
    set_err(out, PQH_ERR_PAGE_HEADER, PQH_PHASE_LOAD, 0);
    return out->status;
  }
  const int v2 = pg->page_type == PQH_DATA_PAGE_V2;
  const int32_t rw = col->max_rep > 0 ? bits_len16(col->max_rep) : 0;
  const int32_t dw = col->max_def > 0 ? bits_len16(col->max_def) : 0;
  hybrid_t rdec, ddec; /* hybridDecoder(bits.Len16(max)) or constDecoder(0) when max == 0 */
  hybrid_new(&rdec, rw);
  hybrid_new(&ddec, dw);
  /* phase-0 (page load) sub-steps, in the reference's order: 0 decoder selection
   * (getValuesDecoder), 1 rDecoder.initSize, 2 dDecoder.initSize, 3 valuesDecoder.init */
  vdec_t v;
  int st = vdec_select(col, pg->encoding, &v);
  if (st) {
    set_err(out, st, PQH_PHASE_LOAD, 0);
    return out->status;
  }
  rd_t r;
  rd_init(&r, img, img_len);
  const uint8_t *vals_base;
  int64_t vals_len;
  if (!v2) {
    /* page_v1.go:110-120: rDecoder.initSize, dDecoder.initSize, valuesDecoder.init */
    hybrid_t *decs[2] = {&rdec, &ddec};
    for (int k = 0; k < 2; k++) {
      hybrid_t *h = decs[k];
      if (h->w == 0) continue; /* constDecoder / zero width: initSize reads nothing */
      uint8_t sz[4];
      if ((st = rd_read_full(&r, sz, 4))) {
        set_err(out, st, PQH_PHASE_LOAD, 1 + k);
        vdec_free(&v);
        return out->status;
      }
      uint32_t size = (uint32_t)sz[0] | ((uint32_t)sz[1] << 8) | ((uint32_t)sz[2] << 16) | ((uint32_t)sz[3] << 24);
      int64_t l = (int64_t)size < rd_avail(&r) ? (int64_t)size : rd_avail(&r);
      hybrid_init(h, r.b + r.pos, l); /* ReadAll(LimitReader(size)) */
      r.pos += l;
    }
    vals_base = r.b + r.pos;
    vals_len = r.len - r.pos;
  } else {
    /* page_v2.go:91-127 */
    int32_t rl = pg->rep_levels_byte_length, dl = pg->def_levels_byte_length;
    if (rl < 0 || dl < 0 || (int64_t)rl + dl > img_len) {
      set_err(out, PQH_ERR_PAGE_HEADER, PQH_PHASE_LOAD, 0);
      vdec_free(&v);
      return out->status;
    }
    if (rl > 0 && rdec.w > 0) hybrid_init(&rdec, img, rl);
    if (dl > 0 && ddec.w > 0) hybrid_init(&ddec, img + rl, dl);
    vals_base = img + rl + dl;
    vals_len = img_len - rl - dl;
  }
  if ((st = vdec_init(&v, vals_base, vals_len))) {
    set_err(out, st, PQH_PHASE_LOAD, 3);
    vdec_free(&v);
    return out->status;
  }
  /* readValues(numValues) */
  if (n == 0) {
    vdec_free(&v);
    return PQH_OK;
  }
  out->num_values = n;
  if (rw > 0) out->rep = (uint8_t *)malloc((size_t)n);
  if (dw > 0) out->def = (uint8_t *)malloc((size_t)n);
  int32_t x;
  for (int32_t i = 0; i < n; i++) { /* decodePackedArray(rDecoder, size) */
    if ((st = hybrid_next(&rdec, &x))) {
      set_err(out, st, PQH_PHASE_REP, i);
      vdec_free(&v);
      return out->status;
    }
    if (out->rep) out->rep[i] = (uint8_t)x;
  }
  int32_t nn = 0;
  for (int32_t i = 0; i < n; i++) { /* decodePackedArray(dDecoder, size) + notNull */
    if ((st = hybrid_next(&ddec, &x))) {
      set_err(out, st, PQH_PHASE_DEF, i);
      vdec_free(&v);
      return out->status;
    }
    if (out->def) out->def[i] = (uint8_t)x;
    if (x == col->max_def) nn++;
  }
  out->nn = nn;
  buf_t vals = {0, 0, 0}, offs = {0, 0, 0}, nil = {0, 0, 0};
  int64_t ei = 0;
  if (nn != 0) st = vdec_decode(&v, dict, nn, &vals, &offs, &ei, &nil);
  else st = PQH_OK;
  vdec_free(&v);
  if (!st && nil.p) {
    out->nil = nil.p;
    for (int32_t k = 0; k < nn; k++) out->num_nil += nil.p[k];
  } else {
    free(nil.p);
  }
  out->values = vals.p;
  out->values_bytes = vals.len;
  out->offsets = (int64_t *)offs.p;
  out->num_offsets = (int64_t)(offs.len / 8);
  int is_ba = col->physical_type == PQH_BYTE_ARRAY ||
              (col->physical_type == PQH_FIXED_LEN_BYTE_ARRAY && (col->type_length == 0 || pg->encoding == PQH_ENC_DELTA_BYTE_ARRAY));
  out->value_size = is_ba ? 0
                    : col->physical_type == PQH_BOOLEAN ? 1
                    : col->physical_type == PQH_FIXED_LEN_BYTE_ARRAY ? col->type_length
                    : col->physical_type == PQH_INT32 || col->physical_type == PQH_FLOAT ? 4
                    : col->physical_type == PQH_INT96 ? 12 : 8;
  if (nn == 0 && is_ba) {
    int64_t z = 0;
    off_push(&offs, z);
    out->offsets = (int64_t *)offs.p;
    out->num_offsets = 1;
  }
  if (st) set_err(out, st, PQH_PHASE_VALUES, ei);
  return out->status;
}

void orc_out_free(orc_out *o) {
  free(o->nil);
  free(o->def);
  free(o->rep);
  free(o->values);
  free(o->offsets);
  memset(o, 0, sizeof(*o));
}
