// file_reader.cpp — host side of the boundary (include/pqhip.h pqh_file_*):
//   * footer: ReadFileMetaData (reference file_meta.go:18-73) + schema levels
//     (readSchema / readGroupSchema / readColumnSchema, schema.go:893-1015);
//   * page walker: FileReader.readChunk / readPages (chunk_reader.go:182-362) with readPageBlock /
//     newBlockReader (chunk_reader.go:161-180, compress.go:131-152): thrift page headers, optional
//     CRC32, chunk-codec decompression with exact size checks, the V2 rule that the values section
//     is always decompressed (page_v2.go:125), one dictionary page per chunk (:195-227).
// Output: a page table + one payload of decompressed page images for the device batch.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <new>
#include <cstdio>
#include <cstdlib>
#include <atomic>
#include <chrono>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "codec.h"
#include "internal.h"
#include "thrift_compact.h"

using namespace pqhip;

namespace {

struct ColumnMeta {
  pqh_column col;
  std::string path;
};

struct ChunkMeta {
  bool has_meta = false;
  bool has_file_path = false;
  int32_t type = -1;
  int32_t codec = 0;
  int64_t total_compressed = 0;
  int64_t data_page_offset = 0;
  bool has_dict_offset = false;
  int64_t dict_page_offset = 0;
};

struct RowGroupMeta {
  int64_t num_rows = 0;
  std::vector<ChunkMeta> chunks;
};

struct SchemaEl {
  bool has_type = false;
  int32_t type = 0, type_length = 0;
  bool has_type_length = false;
  bool has_rep = false;
  int32_t rep = 0;
  std::string name;
  bool has_children = false;
  int32_t num_children = 0;
};

}  // namespace

// One schema element as the reader's Column tree sees it (schema.go:893-990).
struct SchemaNode {
  SchemaEl el;
  int32_t column = -1;  // leaf: index into pqh_file::columns
  int32_t d = 0, r = 0;
};

struct pqh_file {
  std::vector<SchemaNode> schema;
  int fd = -1;
  void* map = nullptr;
  size_t map_len = 0;
  const uint8_t* data = nullptr;
  int64_t len = 0;
  std::string err;
  int64_t num_rows = 0;
  std::vector<ColumnMeta> columns;
  std::vector<RowGroupMeta> rgs;
  // the caller's codec registry: the reference's compressors map, UNCOMPRESSED / GZIP / SNAPPY / ZSTD
  // by default (compress.go:182-187), plus what RegisterBlockCompressor added (pqh_file_set_codecs)
  std::vector<int32_t> codecs{PQH_CODEC_UNCOMPRESSED, PQH_CODEC_GZIP, PQH_CODEC_SNAPPY, PQH_CODEC_ZSTD};
};

namespace {

// The typed FileMetaData (generated readers of parquet/parquet.go, thrift_compact.h) -> the fields
// the reader uses.
void schema_el(const TNode& n, SchemaEl& e) {
  if (const TNode* t = n.get(1)) e.has_type = true, e.type = int32_t(t->i);
  if (const TNode* t = n.get(2)) e.has_type_length = true, e.type_length = int32_t(t->i);
  if (const TNode* t = n.get(3)) e.has_rep = true, e.rep = int32_t(t->i);
  if (const TNode* t = n.get(4)) e.name = t->s;
  if (const TNode* t = n.get(5)) e.has_children = true, e.num_children = int32_t(t->i);
}

void chunk_meta(const TNode& cc, ChunkMeta& m) {
  m.has_file_path = cc.get(1) != nullptr;
  const TNode* md = cc.get(3);
  if (!md) return;
  m.has_meta = true;  // (its required fields are present: the typed read checked them)
  m.type = int32_t(md->get_i(1));
  m.codec = int32_t(md->get_i(4));
  m.total_compressed = md->get_i(7);
  m.data_page_offset = md->get_i(9);
  if (const TNode* t = md->get(11)) m.has_dict_offset = true, m.dict_page_offset = t->i;
}

// makeSchema + readSchema (schema.go:992-1015, 1048-1079): the elements after the root are read
// as top-level groups / columns until the list ends (the root's num_children is not consulted);
// readGroupSchema / readColumnSchema (:893-990) and getValuesStore (data_store.go:328-362) checks.
struct SchemaBuilder {
  pqh_file* f;
  const std::vector<SchemaEl>& s;  // s[0] = the root
  bool fail(const char* m) {
    f->err = m;
    return false;
  }
  // element i of the list after the root = s[i + 1]
  bool column(int32_t& idx, const std::string& path, int32_t d, int32_t r, const std::vector<int32_t>& rd) {
    const SchemaEl& e = s[size_t(idx) + 1];
    if (e.name.empty()) return fail("name in schema is empty");
    if (!e.has_rep) return fail("field RepetitionType is nil");
    if (e.rep != 0) d++;
    std::vector<int32_t> rd2 = rd;
    if (e.rep == 2) {
      r++;
      rd2.push_back(d);
    }
    if (e.type < 0 || e.type > PQH_FIXED_LEN_BYTE_ARRAY) return fail("unsupported type");
    if (e.type == PQH_FIXED_LEN_BYTE_ARRAY && !e.has_type_length) return fail("type with nil type length");
    ColumnMeta cm;
    cm.col = pqh_column{e.type, e.type_length, d, r, {}};
    for (size_t k = 0; k < rd2.size() && k < PQH_MAX_NEST; k++) cm.col.rep_def[k] = rd2[k];
    cm.path = path.empty() ? e.name : path + "." + e.name;
    f->schema[size_t(idx) + 1] = SchemaNode{e, int32_t(f->columns.size()), d, r};
    f->columns.push_back(cm);
    idx++;
    return true;
  }
  bool group(int32_t& idx, const std::string& path, int32_t d, int32_t r, const std::vector<int32_t>& rd, int depth) {
    const int32_t n = int32_t(s.size()) - 1;
    if (depth > 10000) return fail("schema too deep");
    if (n <= idx) return fail("schema index out of bound");
    const SchemaEl& e = s[size_t(idx) + 1];
    if (e.has_type) return fail("field Type is not nil");
    if (!e.has_children) return fail("the field NumChildren is invalid");
    if (e.num_children <= 0) return fail("the field NumChildren is zero");
    const int32_t l = e.num_children;
    if (int64_t(n) <= int64_t(idx) + l) return fail("not enough element in the schema list");
    std::vector<int32_t> rd2 = rd;
    if (e.has_rep && e.rep != 0) d++;
    if (e.has_rep && e.rep == 2) {
      r++;
      rd2.push_back(d);
    }
    const std::string p = path.empty() ? e.name : path + "." + e.name;
    f->schema[size_t(idx) + 1] = SchemaNode{e, -1, d, r};
    idx++;
    for (int32_t i = 0; i < l; i++) {
      if (n <= idx) return fail("schema index is out of bounds");
      if (!s[size_t(idx) + 1].has_type) {
        if (!group(idx, p, d, r, rd2, depth + 1)) return false;
      } else if (!column(idx, p, d, r, rd2)) {
        return false;
      }
    }
    return true;
  }
  bool build() {
    if (s.empty()) return fail("no schema element found");
    f->schema.assign(s.size(), SchemaNode{});
    f->schema[0].el = s[0];
    const int32_t n = int32_t(s.size()) - 1;
    for (int32_t idx = 0; idx < n;) {
      if (!s[size_t(idx) + 1].has_type) {
        if (!group(idx, "", 0, 0, {}, 0)) return false;
      } else if (!column(idx, "", 0, 0, {})) {
        return false;
      }
    }
    return true;
  }
};

// ReadFileMetaData(r, extraValidation = true) (file_meta.go:23-73, as NewFileReaderWithOptions
// calls it, file_reader.go:38-43): both magics, the footer length, the typed FileMetaData over
// exactly the footer (io.LimitReader), then makeSchema.
bool parse_footer(pqh_file* f) {
  if (f->len < 4 || memcmp(f->data, "PAR1", 4) != 0) {
    f->err = "invalid parquet file header";
    return false;
  }
  if (memcmp(f->data + f->len - 4, "PAR1", 4) != 0) {
    f->err = "invalid parquet file footer";
    return false;
  }
  if (f->len < 8) {
    f->err = "seek for the footer len failed";
    return false;
  }
  int32_t flen;
  memcpy(&flen, f->data + f->len - 8, 4);
  if (flen <= 0) {
    f->err = "invalid footer len";
    return false;
  }
  if (int64_t(flen) > f->len - 8) {
    f->err = "seek file meta data failed";
    return false;
  }
  TReader r(f->data + f->len - 8 - flen, f->data + f->len - 8);
  TNode meta;
  if (!read_typed(r, TS_FILE_META_DATA, meta)) {
    f->err = "read file meta failed (thrift)";
    return false;
  }
  std::vector<SchemaEl> schema;
  for (const TNode& n : meta.get(2)->items) {
    SchemaEl e;
    schema_el(n, e);
    schema.push_back(e);
  }
  f->num_rows = meta.get_i(3);
  for (const TNode& g : meta.get(4)->items) {
    RowGroupMeta rg;
    rg.num_rows = g.get_i(3);
    for (const TNode& cc : g.get(1)->items) {
      ChunkMeta m;
      chunk_meta(cc, m);
      rg.chunks.push_back(m);
    }
    f->rgs.push_back(std::move(rg));
  }
  return SchemaBuilder{f, schema}.build();
}

struct PageHdr {
  int32_t type = -1, usize = 0, csize = 0;
  bool has_crc = false;
  int32_t crc = 0;
  bool has_dp = false, has_dict = false, has_v2 = false;
  int32_t num_values = 0, encoding = 0;
  int32_t def_enc = 0, rep_enc = 0;  // DataPageHeader level encodings
  int32_t def_len = 0, rep_len = 0;
  int32_t num_nulls = 0;             // DataPageHeaderV2 (a hint for k_flat's speculation)
};

bool parse_page_header(TReader& r, PageHdr& h) {
  TNode n;
  if (!read_typed(r, TS_PAGE_HEADER, n)) return false;
  h.type = int32_t(n.get_i(1));
  h.usize = int32_t(n.get_i(2));
  h.csize = int32_t(n.get_i(3));
  if (const TNode* c = n.get(4)) h.has_crc = true, h.crc = int32_t(c->i);
  if (const TNode* d = n.get(5)) {
    h.has_dp = true;
    if (h.type == PQH_DATA_PAGE) {
      h.num_values = int32_t(d->get_i(1));
      h.encoding = int32_t(d->get_i(2));
      h.def_enc = int32_t(d->get_i(3));
      h.rep_enc = int32_t(d->get_i(4));
    }
  }
  if (const TNode* d = n.get(7)) {
    h.has_dict = true;
    if (h.type == PQH_DICTIONARY_PAGE) {
      h.num_values = int32_t(d->get_i(1));
      h.encoding = int32_t(d->get_i(2));
    }
  }
  if (const TNode* d = n.get(8)) {
    h.has_v2 = true;
    if (h.type == PQH_DATA_PAGE_V2) {
      h.num_values = int32_t(d->get_i(1));
      h.num_nulls = int32_t(d->get_i(2));
      h.encoding = int32_t(d->get_i(4));
      h.def_len = int32_t(d->get_i(5));
      h.rep_len = int32_t(d->get_i(6));
    }
  }
  return true;
}

// ------------------------------------------------------------------------------------------------
// The page walk in two passes, so that every page image is written once, straight to its place in
// the batch payload (pinned host memory with pqh_file_load_pinned):
//   plan (per chunk, parallel): readPages' header walk with every check that does not need the
//     decompressed bytes, each page's image size (the header's uncompressed size) and place;
//   materialise (per page, parallel): decompress (or copy) the page into its place; a page that
//     fails ends its chunk there (pages after it are dropped, as readPages stops).
// ------------------------------------------------------------------------------------------------
struct PageOp {
  pqh_page pg;            // image_offset: relative to the chunk's image area
  const uint8_t* block;   // the page's bytes in the file (readPageBlock)
  int64_t got = 0;        // bytes read
  int64_t levels = 0;     // V2: raw level bytes in front of the (compressed) values
  bool raw = false;       // device codecs: the page travels compressed (SNAPPY) and k_snappy rebuilds it
  int64_t src_off = 0;    // device codecs: its source bytes in the chunk's source area
  int64_t src_len = 0;
  bool failed = false;    // materialise: decompression failed or the size differs
};

struct ChunkPlan {
  pqh_chunk chunk;
  std::vector<PageOp> ops;
  int32_t codec = 0;
  int64_t image = 0;      // image area bytes (64-aligned pages)
  int64_t src = 0;        // device codecs: source area bytes
  int64_t image_base = 0, src_base = 0;  // global offsets (assigned after planning)
  double seconds = 0;
};

// The decoded length a snappy block announces (its uvarint header), -1 if malformed.
int64_t snappy_announced(const uint8_t* p, size_t n) {
  uint64_t v = 0;
  for (size_t i = 0; i < n && i < 10; i++) {
    if (i == 9 && p[i] > 1) return -1;
    v |= uint64_t(p[i] & 0x7f) << (7 * i);
    if (p[i] < 0x80) return v > 0xffffffffull ? -1 : int64_t(v);
  }
  return -1;
}

// Device codecs: can a SNAPPY block of n bytes decode to exactly `expected` bytes?  (A wrong or
// malformed announced length, or more output than the format can encode in n bytes, fails exactly
// as the host decode would: readPageBlock's ErrCorrupt / size check, compress.go:131-152.)
bool snappy_plausible(const uint8_t* p, size_t n, int64_t expected) {
  if (expected < 0) return false;
  const int64_t v = snappy_announced(p, n);
  return v == expected && v <= 22 * int64_t(n) + 64;  // a 3-byte copy element yields <= 64 bytes
}

int64_t align64(int64_t x) { return (x + 63) & ~int64_t(63); }

// Device codecs: pages whose compressed values are at least this fraction of their decompressed
// size stay on the host-decompressed route (PQH_DEVICE_CODEC_MAX_RATIO overrides it; 0 sends every
// page of a device-codec chunk to the device, as before ABI 8)
double device_codec_max_ratio() {
  const char* v = getenv("PQH_DEVICE_CODEC_MAX_RATIO");
  return v ? atof(v) : 0.95;
}

// Plan: readChunk + readPages for one chunk (chunk_reader.go:182-362), page by page in the
// reference's order of checks.  The walk stops at the first page it cannot read (host_status, with
// the pages before it listed); the checks of each listed page that belong to the decoders (the
// values decoder's selection and init, the level decoders' initSize) run on the device, and the
// batch orders every error of the chunk as the reference's walk would meet them (chunk_error).
void plan_chunk(const pqh_file* f, const ColumnMeta& col, const ChunkMeta& m, int validate_crc, bool dev_codecs,
                uint32_t flags, ChunkPlan& w) {
  auto t0 = std::chrono::steady_clock::now();
  w.chunk.column = col.col;
  w.chunk.first_page = 0;
  w.chunk.num_pages = 0;
  w.chunk.host_status = PQH_OK;
  w.codec = m.codec;
  auto fail = [&](int code) { w.chunk.host_status = code; };
  if (m.has_file_path) return fail(PQH_ERR_IO);  // "nyi: data is in another file"
  if (!m.has_meta) return fail(PQH_ERR_SCHEMA);  // "missing meta data for Column"
  if (m.type != col.col.physical_type) return fail(PQH_ERR_SCHEMA);  // "wrong type in Column chunk metadata"
  // A codec the caller's registry holds but this library does not decode (the reference's ZSTD, or
  // one registered through RegisterBlockCompressor: compress.go:119-129,160,182-187) is not a
  // property of the data: the chunk is handed back before any page is read, never reported as a
  // corrupt page.  (A codec in no registry fails as the reference fails it: decompressBlock's
  // "method not supported", at the first page's block -- materialise / decompress_into.)
  if (m.codec != PQH_CODEC_UNCOMPRESSED && m.codec != PQH_CODEC_SNAPPY && m.codec != PQH_CODEC_GZIP &&
      std::find(f->codecs.begin(), f->codecs.end(), m.codec) != f->codecs.end())
    return fail(PQH_ERR_UNSUPPORTED_CODEC);
  int64_t pos = m.has_dict_offset ? m.dict_page_offset : m.data_page_offset;
  if (pos < 0) return fail(PQH_ERR_IO);  // Seek: negative position
  int64_t count = 0;
  bool have_dict = false;
  const int32_t max_def = col.col.max_def, max_rep = col.col.max_rep;
  // this chunk's pages stay compressed for the device (the layout is the device-codec one whenever
  // some selected chunk's codec is decoded on the device)
  const bool dev = dev_codecs && ((m.codec == PQH_CODEC_SNAPPY && (flags & PQH_LOAD_DEVICE_SNAPPY)) ||
                                  (m.codec == PQH_CODEC_GZIP && (flags & PQH_LOAD_DEVICE_GZIP)));
  const double max_ratio = device_codec_max_ratio();
  while (m.total_compressed - count > 0) {
    // readThrift(PageHeader): reads past the end of the file fail like any short read
    TReader r(f->data + std::min(pos, f->len), f->data + f->len);
    PageHdr h;
    if (!parse_page_header(r, h)) return fail(PQH_ERR_THRIFT);
    pos += int64_t(r.consumed());
    count += int64_t(r.consumed());
    PageOp op;
    memset(&op.pg, 0, sizeof(op.pg));
    op.pg.page_type = h.type;
    op.pg.num_values = h.num_values;
    op.pg.encoding = h.encoding;
    // readPageBlock (:161-180): sizes, io.ReadAll(io.LimitReader), CRC
    auto read_block = [&]() -> int {
      if (h.csize < 0 || h.usize < 0) return PQH_ERR_PAGE_HEADER;  // "invalid page data size"
      const int64_t avail = std::max<int64_t>(0, f->len - pos);
      op.got = h.csize < avail ? h.csize : avail;
      op.block = f->data + std::min(pos, f->len);
      pos += op.got;
      count += op.got;
      if (validate_crc && h.has_crc && crc32_ieee(op.block, size_t(op.got)) != uint32_t(h.crc)) return PQH_ERR_CRC;
      return PQH_OK;
    };
    // newBlockReader (compress.go:131-152) of the (values) section [levels, got): what can be decided
    // without decompressing; the rest is decided when the page is materialised
    auto block_reader = [&](int64_t levels) -> int {
      if (int64_t(h.csize) - levels < 0 || int64_t(h.usize) - levels < 0) return PQH_ERR_PAGE_HEADER;
      if (op.got != h.csize) return PQH_ERR_DECOMPRESS;  // "compressed data must be %d byte"
      if (m.codec == PQH_CODEC_UNCOMPRESSED && h.csize != h.usize) return PQH_ERR_DECOMPRESS;
      // a page whose values barely compress (>= 0.95 of their size) saves no PCIe bytes by
      // travelling compressed: the host decompresses it, the device only copies the image (C5's
      // random strings: k_snappy's page mode took 32 ms for pages that shrink by 0.2%)
      const bool raw = dev && (max_ratio <= 0 || double(h.csize - levels) < max_ratio * double(h.usize - levels));
      if (raw && m.codec == PQH_CODEC_SNAPPY && !snappy_plausible(op.block + levels, size_t(op.got - levels), int64_t(h.usize) - levels))
        return PQH_ERR_DECOMPRESS;
      op.levels = levels;
      op.raw = raw;
      op.src_len = raw ? op.got : h.usize;
      op.pg.image_len = h.usize;
      return PQH_OK;
    };
    auto place = [&]() {
      op.pg.image_offset = align64(w.image);
      w.image = op.pg.image_offset + op.pg.image_len;
      if (dev_codecs) {
        op.src_off = align64(w.src);
        w.src = op.src_off + op.src_len;
      }
      w.ops.push_back(op);
    };
    int rc;
    if (h.type == PQH_DICTIONARY_PAGE) {
      if (have_dict) return fail(PQH_ERR_DICT_PAGE);  // "there should be only one dictionary"
      // getDictValuesDecoder (:17-39): no BOOLEAN dictionaries
      if (col.col.physical_type == PQH_BOOLEAN) return fail(PQH_ERR_UNSUPPORTED);
      // dictPageReader.read (page_dict.go:35-72)
      if (!h.has_dict) return fail(PQH_ERR_PAGE_HEADER);
      if (h.num_values < 0) return fail(PQH_ERR_PAGE_HEADER);
      if (h.encoding != PQH_ENC_PLAIN && h.encoding != PQH_ENC_PLAIN_DICTIONARY) return fail(PQH_ERR_DICT_PAGE);
      if ((rc = read_block()) || (rc = block_reader(0))) return fail(rc);
      place();  // its PLAIN values are decoded (and may fail) on the device
      have_dict = true;
      if (m.has_dict_offset && m.dict_page_offset != pos) {  // seek to DataPageOffset
        if (m.data_page_offset < 0) return fail(PQH_ERR_IO);
        count += m.data_page_offset - pos;
        pos = m.data_page_offset;
      }
      continue;
    }
    if (h.type == PQH_DATA_PAGE) {
      // dataPageReaderV1.init (page_v1.go:65-85): the level decoders need RLE when their level is used
      if (!h.has_dp) return fail(PQH_ERR_PAGE_HEADER);
      if (max_rep > 0 && h.rep_enc != PQH_ENC_RLE) return fail(PQH_ERR_UNSUPPORTED);
      if (max_def > 0 && h.def_enc != PQH_ENC_RLE) return fail(PQH_ERR_UNSUPPORTED);
      // .read (:87-122): NumValues, block, decompression (the values decoder: on the device)
      if (h.num_values < 0) return fail(PQH_ERR_PAGE_HEADER);
      if ((rc = read_block()) || (rc = block_reader(0))) return fail(rc);
    } else if (h.type == PQH_DATA_PAGE_V2) {
      // dataPageReaderV2.read (page_v2.go:79-131)
      if (!h.has_v2) return fail(PQH_ERR_PAGE_HEADER);
      if (h.num_values < 0 || h.rep_len < 0 || h.def_len < 0) return fail(PQH_ERR_PAGE_HEADER);
      int32_t vs;  // getValuesDecoder runs before the block is read here (:107-112)
      if (resolve_kind(col.col.physical_type, col.col.type_length, h.encoding, &vs) == 0) return fail(PQH_ERR_UNSUPPORTED);
      if ((rc = read_block())) return fail(rc);
      const int64_t levels = int64_t(h.rep_len) + h.def_len;
      // the level slices of the block: out of range is a runtime panic in the reference (:117-123)
      if (levels > op.got) return fail(PQH_ERR_PAGE_HEADER);
      // the values section is decompressed regardless of is_compressed (page_v2.go:125)
      if ((rc = block_reader(levels))) return fail(rc);
      op.pg.def_levels_byte_length = h.def_len;
      op.pg.rep_levels_byte_length = h.rep_len;
      op.pg.num_nulls = h.num_nulls;
    } else {
      return fail(PQH_ERR_PAGE_HEADER);  // "DATA_PAGE or DATA_PAGE_V2 type supported"
    }
    place();
  }
  w.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// Materialise one planned page: host codecs -> its image at `img`; device codecs -> its source
// bytes at `src` (compressed SNAPPY, or the decompressed image of another codec) + its codec page.
void materialise(const ChunkPlan& w, PageOp& op, uint8_t* img, uint8_t* src) {
  if (op.raw) {  // SNAPPY / GZIP for the device: raw levels + compressed values, as stored
    memcpy(src + op.src_off, op.block, size_t(op.got));
    return;
  }
  uint8_t* dst = src ? src + op.src_off : img + op.pg.image_offset;
  if (op.levels) memcpy(dst, op.block, size_t(op.levels));
  op.failed = !decompress_into(w.codec, op.block + op.levels, size_t(op.got - op.levels), dst + op.levels,
                               size_t(op.pg.image_len - op.levels));
}

int file_error(pqh_file* f, int code, const std::string& m) {
  if (f) f->err = m;
  return code;
}

}  // namespace

extern "C" {

int pqh_file_open_memory(const void* data, int64_t len, pqh_file** out) {
  *out = nullptr;
  pqh_file* f = new pqh_file();
  f->data = static_cast<const uint8_t*>(data);
  f->len = len;
  if (!parse_footer(f)) {
    *out = f;
    return PQH_ERR_SCHEMA;
  }
  *out = f;
  return PQH_OK;
}

int pqh_file_open(const char* path, pqh_file** out) {
  *out = nullptr;
  int fd = open(path, O_RDONLY);
  pqh_file* f = new pqh_file();
  *out = f;
  if (fd < 0) return file_error(f, PQH_ERR_IO, std::string("cannot open ") + path);
  struct stat sb;
  if (fstat(fd, &sb) != 0 || sb.st_size <= 0) {
    close(fd);
    return file_error(f, PQH_ERR_IO, "cannot stat file");
  }
  void* m = mmap(nullptr, size_t(sb.st_size), PROT_READ, MAP_PRIVATE, fd, 0);
  if (m == MAP_FAILED) {
    close(fd);
    return file_error(f, PQH_ERR_IO, "mmap failed");
  }
  f->fd = fd;
  f->map = m;
  f->map_len = size_t(sb.st_size);
  f->data = static_cast<const uint8_t*>(m);
  f->len = int64_t(sb.st_size);
  if (!parse_footer(f)) return PQH_ERR_SCHEMA;
  return PQH_OK;
}

void pqh_file_close(pqh_file* f) {
  if (!f) return;
  if (f->map) munmap(f->map, f->map_len);
  if (f->fd >= 0) close(f->fd);
  delete f;
}

const char* pqh_file_error(const pqh_file* f) { return f ? f->err.c_str() : "null file"; }
int32_t pqh_file_num_row_groups(const pqh_file* f) { return int32_t(f->rgs.size()); }
int64_t pqh_file_num_rows(const pqh_file* f) { return f->num_rows; }
int64_t pqh_file_row_group_num_rows(const pqh_file* f, int32_t rg) {
  return rg >= 0 && size_t(rg) < f->rgs.size() ? f->rgs[size_t(rg)].num_rows : -1;
}
int32_t pqh_file_num_columns(const pqh_file* f) { return int32_t(f->columns.size()); }

int32_t pqh_file_num_schema_elements(const pqh_file* f) { return f ? int32_t(f->schema.size()) : 0; }

int pqh_file_schema_element(const pqh_file* f, int32_t i, pqh_schema_element* out, char* name, int32_t cap) {
  if (!f || !out || i < 0 || size_t(i) >= f->schema.size()) return PQH_ERR_ARG;
  const SchemaNode& n = f->schema[size_t(i)];
  out->physical_type = n.el.has_type ? n.el.type : -1;
  out->type_length = n.el.type_length;
  out->repetition = n.el.has_rep ? n.el.rep : -1;
  out->num_children = n.el.has_children ? n.el.num_children : 0;
  out->column = n.column;
  out->max_def = n.d;
  out->max_rep = n.r;
  out->reserved = 0;
  if (name && cap > 0) {
    const size_t k = std::min(n.el.name.size(), size_t(cap - 1));
    memcpy(name, n.el.name.data(), k);
    name[k] = 0;
  }
  return PQH_OK;
}

int pqh_file_column(const pqh_file* f, int32_t column, pqh_column* out, char* path, int32_t cap) {
  if (!f || column < 0 || size_t(column) >= f->columns.size()) return PQH_ERR_ARG;
  *out = f->columns[size_t(column)].col;
  if (path && cap > 0) {
    const std::string& p = f->columns[size_t(column)].path;
    size_t n = std::min(p.size(), size_t(cap - 1));
    memcpy(path, p.data(), n);
    path[n] = 0;
  }
  return PQH_OK;
}

int pqh_file_load(pqh_file* f, int32_t rg_begin, int32_t rg_end, const int32_t* columns, int32_t num_columns,
                  int32_t validate_crc, pqh_host_batch** out) {
  return pqh_file_load_ex(f, rg_begin, rg_end, columns, num_columns, validate_crc, 0, out);
}

}  // extern "C"

namespace {

int file_load(pqh_ctx* ctx, pqh_file* f, int32_t rg_begin, int32_t rg_end, const int32_t* columns,
              int32_t num_columns, int32_t validate_crc, uint32_t flags, pqh_host_batch** out) {
  *out = nullptr;
  if (!f) return PQH_ERR_ARG;
  if (rg_begin < 0 || rg_end > int32_t(f->rgs.size()) || rg_begin > rg_end)
    return file_error(f, PQH_ERR_ARG, "row group range out of bounds");
  for (int32_t i = 0; i < num_columns; i++)
    if (columns[i] < 0 || size_t(columns[i]) >= f->columns.size()) return file_error(f, PQH_ERR_ARG, "bad column");
  const int64_t nchunks = int64_t(rg_end - rg_begin) * num_columns;
  std::vector<ChunkPlan> work(static_cast<size_t>(nchunks));
  const bool timing = getenv("PQH_WALK_TIMING") != nullptr;
  auto tw = std::chrono::steady_clock::now();
  auto lap = [&](const char* what) {
    if (!timing) return;
    auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "[walk] %s %.4f s\n", what, std::chrono::duration<double>(t - tw).count());
    tw = t;
  };
  // device codecs only when some selected chunk has a codec the flags put on the device
  // (otherwise the plain layout)
  bool dev = false;
  if (flags & (PQH_LOAD_DEVICE_SNAPPY | PQH_LOAD_DEVICE_GZIP))
    for (int32_t rg = rg_begin; rg < rg_end && !dev; rg++)
      for (int32_t i = 0; i < num_columns && !dev; i++) {
        const RowGroupMeta& g = f->rgs[size_t(rg)];
        if (size_t(columns[i]) >= g.chunks.size() || !g.chunks[size_t(columns[i])].has_meta) continue;
        const int32_t c = g.chunks[size_t(columns[i])].codec;
        dev = (c == PQH_CODEC_SNAPPY && (flags & PQH_LOAD_DEVICE_SNAPPY)) ||
              (c == PQH_CODEC_GZIP && (flags & PQH_LOAD_DEVICE_GZIP));
      }
  // walker threads: one per hardware thread up to 16 (the host share a GPU box grants), or
  // PQH_WALK_THREADS (a streaming ring leaves cores to the batch creation beside its walks)
  int nt = int(std::thread::hardware_concurrency());
  if (nt > 16) nt = 16;
  if (const char* w = getenv("PQH_WALK_THREADS")) nt = atoi(w);
  if (nt < 1) nt = 1;
  auto parallel = [&](int64_t items, auto&& fn) {
    std::atomic<int64_t> next{0};
    const int k = int(std::min<int64_t>(nt, std::max<int64_t>(items, 1)));
    std::vector<std::thread> th;
    for (int i = 0; i < k; i++)
      th.emplace_back([&]() {
        for (int64_t j; (j = next.fetch_add(1)) < items;) fn(j);
      });
    for (auto& t : th) t.join();
  };
  // pass 1: plan every chunk
  parallel(nchunks, [&](int64_t k) {
    const int32_t rg = rg_begin + int32_t(k / num_columns);
    const int32_t ci = columns[k % num_columns];
    const RowGroupMeta& g = f->rgs[size_t(rg)];
    ChunkPlan& w = work[size_t(k)];
    if (size_t(ci) >= g.chunks.size()) {  // "column index %d is out of bounds"
      w.chunk.column = f->columns[size_t(ci)].col;
      w.chunk.host_status = PQH_ERR_SCHEMA;
      return;
    }
    plan_chunk(f, f->columns[size_t(ci)], g.chunks[size_t(ci)], validate_crc, dev, flags, w);
  });
  lap("plan");
  // layout: chunk areas back to back (64-aligned); the payload is the images (host codecs) or the
  // source bytes (device codecs)
  int64_t images = 0, sources = 0;
  std::vector<std::pair<size_t, size_t>> page_list;  // (chunk, op)
  for (size_t k = 0; k < work.size(); k++) {
    work[k].image_base = align64(images);
    images = work[k].image_base + work[k].image;
    work[k].src_base = align64(sources);
    sources = work[k].src_base + work[k].src;
    for (size_t i = 0; i < work[k].ops.size(); i++) page_list.emplace_back(k, i);
  }
  const int64_t payload_bytes = dev ? sources : images;
  pqh_host_batch* hb = new pqh_host_batch();
  const size_t total = size_t(payload_bytes) + PQH_PAYLOAD_PAD;
  uint8_t* base = nullptr;
  if (ctx) {
    hb->buf = pinned_acquire(ctx, total);
    hb->pinned = true;
  } else {  // uninitialised (the walker threads write every byte: images, gaps, pad)
    hb->buf = std::shared_ptr<uint8_t>(new (std::nothrow) uint8_t[total], std::default_delete<uint8_t[]>());
  }
  if (!hb->buf) {
    delete hb;
    return file_error(f, PQH_ERR_NOMEM, "payload allocation failed");
  }
  hb->buf_size = total;
  base = hb->buf.get();
  lap("alloc");
  // pass 2: every page to its place (pages of all chunks spread over the threads); alignment gaps
  // and the pad are zeroed
  parallel(int64_t(page_list.size()), [&](int64_t j) {
    ChunkPlan& w = work[page_list[size_t(j)].first];
    PageOp& op = w.ops[page_list[size_t(j)].second];
    materialise(w, op, dev ? nullptr : base + w.image_base, dev ? base + w.src_base : nullptr);
  });
  lap("materialise");
  {
    int64_t end = 0;  // zero every gap between areas / pages
    auto zero_to = [&](int64_t off) {
      if (off > end) memset(base + end, 0, size_t(off - end));
    };
    for (auto& w : work) {
      for (auto& op : w.ops) {
        const int64_t o = dev ? w.src_base + op.src_off : w.image_base + op.pg.image_offset;
        zero_to(o);
        end = std::max(end, o + (dev ? op.src_len : int64_t(op.pg.image_len)));
      }
    }
    zero_to(int64_t(total));
  }
  lap("gaps");
  int64_t image = 0;
  for (auto& w : work) {
    // a page that failed to decompress ends its chunk there (readPages returns the error)
    size_t keep = w.ops.size();
    for (size_t i = 0; i < w.ops.size(); i++)
      if (w.ops[i].failed) {
        keep = i;
        w.chunk.host_status = PQH_ERR_DECOMPRESS;
        break;
      }
    pqh_chunk c = w.chunk;
    c.first_page = int32_t(hb->pages.size());
    c.num_pages = int32_t(keep);
    const int32_t ci = int32_t(hb->chunks.size());
    for (size_t i = 0; i < keep; i++) {
      const PageOp& op = w.ops[i];
      pqh_page pg = op.pg;
      pg.image_offset += w.image_base;
      pg.chunk = ci;
      hb->pages.push_back(pg);
      if (dev) {
        pqh_codec_page cp;
        memset(&cp, 0, sizeof(cp));
        cp.src_offset = w.src_base + op.src_off;
        cp.image_offset = pg.image_offset;
        cp.src_len = int32_t(op.src_len);
        cp.image_len = pg.image_len;
        cp.raw_len = op.raw ? int32_t(op.levels) : 0;
        cp.codec = op.raw ? w.codec : PQH_CODEC_UNCOMPRESSED;
        cp.chunk = ci;
        hb->codec_pages.push_back(cp);
      }
    }
    hb->chunks.push_back(c);
    hb->decompress_seconds += w.seconds;
    image = std::max(image, w.image_base + w.image);
  }
  hb->image_bytes = dev ? images : 0;
  hb->payload_bytes = payload_bytes;
  lap("tables");
  *out = hb;
  return PQH_OK;
}

}  // namespace

extern "C" {

int pqh_file_load_ex(pqh_file* f, int32_t rg_begin, int32_t rg_end, const int32_t* columns, int32_t num_columns,
                     int32_t validate_crc, uint32_t flags, pqh_host_batch** out) {
  return file_load(nullptr, f, rg_begin, rg_end, columns, num_columns, validate_crc, flags, out);
}

int pqh_file_load_pinned(pqh_ctx* ctx, pqh_file* f, int32_t rg_begin, int32_t rg_end, const int32_t* columns,
                         int32_t num_columns, int32_t validate_crc, uint32_t flags, pqh_host_batch** out) {
  *out = nullptr;
  if (!ctx) return file_error(f, PQH_ERR_ARG, "null context");
  return file_load(ctx, f, rg_begin, rg_end, columns, num_columns, validate_crc, flags, out);
}

int32_t pqh_file_column_path(const pqh_file* f, int32_t column, char* buf, int32_t cap) {
  if (!f || column < 0 || size_t(column) >= f->columns.size()) return -1;
  const std::string& p = f->columns[size_t(column)].path;
  if (buf && cap > 0) memcpy(buf, p.data(), std::min(p.size(), size_t(cap)));
  return int32_t(p.size());
}

int32_t pqh_file_schema_name(const pqh_file* f, int32_t i, char* buf, int32_t cap) {
  if (!f || i < 0 || size_t(i) >= f->schema.size()) return -1;
  const std::string& n = f->schema[size_t(i)].el.name;
  if (buf && cap > 0) memcpy(buf, n.data(), std::min(n.size(), size_t(cap)));
  return int32_t(n.size());
}

int pqh_file_set_codecs(pqh_file* f, const int32_t* codecs, int32_t n) {
  if (!f || n < 0 || (n > 0 && !codecs)) return PQH_ERR_ARG;
  f->codecs.assign(codecs, codecs + n);
  return PQH_OK;
}

int pqh_file_chunk_check(const pqh_file* f, int32_t rg, int32_t column, int32_t selected) {
  // readRowGroupData's per-column checks before any page is read (chunk_reader.go:381-393), and
  // skipChunk's (:271-297) for a column that is not selected
  if (!f || rg < 0 || size_t(rg) >= f->rgs.size() || column < 0 || size_t(column) >= f->columns.size())
    return PQH_ERR_ARG;
  const RowGroupMeta& g = f->rgs[size_t(rg)];
  if (size_t(column) >= g.chunks.size()) return PQH_ERR_SCHEMA;  // "column index %d is out of bounds"
  const ChunkMeta& m = g.chunks[size_t(column)];
  if (m.has_file_path) return PQH_ERR_IO;
  if (!m.has_meta) return PQH_ERR_SCHEMA;
  if (m.type != f->columns[size_t(column)].col.physical_type) return PQH_ERR_SCHEMA;
  const int64_t off = m.has_dict_offset ? m.dict_page_offset : m.data_page_offset;
  if ((selected ? off : off + m.total_compressed) < 0) return PQH_ERR_IO;  // Seek: negative position
  return PQH_OK;
}

int32_t pqh_host_batch_num_codec_pages(const pqh_host_batch* hb) { return int32_t(hb->codec_pages.size()); }
const pqh_codec_page* pqh_host_batch_codec_pages(const pqh_host_batch* hb) { return hb->codec_pages.data(); }
int64_t pqh_host_batch_image_bytes(const pqh_host_batch* hb) { return hb->image_bytes; }
int32_t pqh_host_batch_num_chunks(const pqh_host_batch* hb) { return int32_t(hb->chunks.size()); }
int32_t pqh_host_batch_num_pages(const pqh_host_batch* hb) { return int32_t(hb->pages.size()); }
const pqh_chunk* pqh_host_batch_chunks(const pqh_host_batch* hb) { return hb->chunks.data(); }
const pqh_page* pqh_host_batch_pages(const pqh_host_batch* hb) { return hb->pages.data(); }
const uint8_t* pqh_host_batch_payload(const pqh_host_batch* hb) { return hb->data(); }
int64_t pqh_host_batch_payload_bytes(const pqh_host_batch* hb) { return hb->payload_bytes; }
double pqh_host_batch_decompress_seconds(const pqh_host_batch* hb) { return hb->decompress_seconds; }
void pqh_host_batch_free(pqh_host_batch* hb) { delete hb; }

}  // extern "C"
