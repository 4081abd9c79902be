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
};

namespace {

bool parse_schema_el(TReader& r, SchemaEl& e) {
  int16_t last = 0, id;
  uint8_t t;
  while (r.field(last, id, t)) {
    switch (id) {
      case 1: e.has_type = true; e.type = int32_t(r.integer(t)); break;
      case 2: e.type_length = int32_t(r.integer(t)); break;
      case 3: e.has_rep = true; e.rep = int32_t(r.integer(t)); break;
      case 4: e.name = r.binary(); break;
      case 5: e.has_children = true; e.num_children = int32_t(r.integer(t)); break;
      default: r.skip(t);
    }
  }
  return r.ok();
}

bool parse_column_meta(TReader& r, ChunkMeta& m) {
  int16_t last = 0, id;
  uint8_t t;
  m.has_meta = true;
  while (r.field(last, id, t)) {
    switch (id) {
      case 1: m.type = int32_t(r.integer(t)); break;
      case 4: m.codec = int32_t(r.integer(t)); break;
      case 7: m.total_compressed = r.integer(t); break;
      case 9: m.data_page_offset = r.integer(t); break;
      case 11: m.has_dict_offset = true; m.dict_page_offset = r.integer(t); break;
      default: r.skip(t);
    }
  }
  return r.ok();
}

bool parse_row_group(TReader& r, RowGroupMeta& g) {
  int16_t last = 0, id;
  uint8_t t;
  while (r.field(last, id, t)) {
    if (id == 1 && t == T_LIST) {
      uint8_t et;
      uint32_t n;
      r.list(et, n);
      for (uint32_t i = 0; i < n && r.ok(); i++) {
        ChunkMeta cm;
        int16_t l2 = 0, id2;
        uint8_t t2;
        while (r.field(l2, id2, t2)) {
          if (id2 == 1) {
            cm.has_file_path = true;
            r.skip(t2);
          } else if (id2 == 3 && t2 == T_STRUCT) {
            parse_column_meta(r, cm);
          } else {
            r.skip(t2);
          }
        }
        g.chunks.push_back(cm);
      }
    } else if (id == 3) {
      g.num_rows = r.integer(t);
    } else {
      r.skip(t);
    }
  }
  return r.ok();
}

// readSchema (schema.go:992-1015) and its group/column readers: levels and error rules.
bool build_columns(pqh_file* f, const std::vector<SchemaEl>& s) {
  if (s.empty()) {
    f->err = "empty schema";
    return false;
  }
  struct Frame {
    int32_t remaining;
    int32_t d, r;
    std::string path;
    std::vector<int32_t> rep_def;  // definition level of each REPEATED node above
  };
  std::vector<Frame> st;
  const SchemaEl& root = s[0];
  if (root.has_type || !root.has_children || root.num_children <= 0) {
    f->err = "invalid schema root";
    return false;
  }
  st.push_back({root.num_children, 0, 0, "", {}});
  f->schema.assign(s.size(), SchemaNode{});
  f->schema[0].el = root;
  for (size_t i = 1; i < s.size(); i++) {
    while (!st.empty() && st.back().remaining == 0) st.pop_back();
    if (st.empty()) {
      f->err = "schema has trailing elements";
      return false;
    }
    Frame& parent = st.back();
    parent.remaining--;
    const SchemaEl& e = s[i];
    if (e.name.empty()) {
      f->err = "name in schema is empty";
      return false;
    }
    const std::string path = parent.path.empty() ? e.name : parent.path + "." + e.name;
    int32_t d = parent.d, r = parent.r;
    std::vector<int32_t> rd = parent.rep_def;
    if (e.has_type) {
      if (!e.has_rep) {
        f->err = "field RepetitionType is nil";
        return false;
      }
      if (e.rep != 0) d++;
      if (e.rep == 2) {
        r++;
        rd.push_back(d);
      }
      ColumnMeta cm;
      cm.col = pqh_column{e.type, e.type_length, d, r, {0, 0, 0, 0, 0, 0, 0, 0}};
      for (size_t k = 0; k < rd.size() && k < PQH_MAX_NEST; k++) cm.col.rep_def[k] = rd[k];
      cm.path = path;
      f->schema[i] = SchemaNode{e, int32_t(f->columns.size()), d, r};
      f->columns.push_back(cm);
    } else {
      if (!e.has_children || e.num_children <= 0) {
        f->err = "group without children";
        return false;
      }
      if (e.has_rep && e.rep != 0) d++;
      if (e.has_rep && e.rep == 2) {
        r++;
        rd.push_back(d);
      }
      f->schema[i] = SchemaNode{e, -1, d, r};
      st.push_back({e.num_children, d, r, path, rd});
    }
  }
  for (auto& fr : st)
    if (fr.remaining > 0) {
      f->err = "not enough element in the schema list";
      return false;
    }
  return true;
}

bool parse_footer(pqh_file* f) {
  if (f->len < 12 || memcmp(f->data, "PAR1", 4) != 0 || memcmp(f->data + f->len - 4, "PAR1", 4) != 0) {
    f->err = "invalid parquet file magic";
    return false;
  }
  uint32_t flen;
  memcpy(&flen, f->data + f->len - 8, 4);
  if (int64_t(flen) > f->len - 12) {
    f->err = "invalid footer length";
    return false;
  }
  const uint8_t* p = f->data + f->len - 8 - flen;
  TReader r(p, f->data + f->len - 8);
  std::vector<SchemaEl> schema;
  int16_t last = 0, id;
  uint8_t t;
  while (r.field(last, id, t)) {
    if (id == 2 && t == T_LIST) {
      uint8_t et;
      uint32_t n;
      r.list(et, n);
      for (uint32_t i = 0; i < n && r.ok(); i++) {
        SchemaEl e;
        parse_schema_el(r, e);
        schema.push_back(e);
      }
    } else if (id == 3) {
      f->num_rows = r.integer(t);
    } else if (id == 4 && t == T_LIST) {
      uint8_t et;
      uint32_t n;
      r.list(et, n);
      for (uint32_t i = 0; i < n && r.ok(); i++) {
        RowGroupMeta g;
        parse_row_group(r, g);
        f->rgs.push_back(std::move(g));
      }
    } else {
      r.skip(t);
    }
  }
  if (!r.ok()) {
    f->err = "corrupt footer (thrift)";
    return false;
  }
  return build_columns(f, schema);
}

struct PageHdr {
  int32_t type = -1, usize = 0, csize = 0;
  bool has_crc = false;
  int32_t crc = 0;
  bool has_dp = false, has_dict = false, has_v2 = false;
  int32_t num_values = 0, encoding = 0;
  int32_t def_len = 0, rep_len = 0;
};

bool parse_page_header(TReader& r, PageHdr& h) {
  int16_t last = 0, id;
  uint8_t t;
  while (r.field(last, id, t)) {
    switch (id) {
      case 1: h.type = int32_t(r.integer(t)); break;
      case 2: h.usize = int32_t(r.integer(t)); break;
      case 3: h.csize = int32_t(r.integer(t)); break;
      case 4: h.has_crc = true; h.crc = int32_t(r.integer(t)); break;
      case 5:
      case 7:
      case 8: {
        if (t != T_STRUCT) {
          r.skip(t);
          break;
        }
        if (id == 5) h.has_dp = true;
        if (id == 7) h.has_dict = true;
        if (id == 8) h.has_v2 = true;
        int16_t l2 = 0, i2;
        uint8_t t2;
        while (r.field(l2, i2, t2)) {
          if (i2 == 1) h.num_values = int32_t(r.integer(t2));
          else if (i2 == 2 && id != 8) h.encoding = int32_t(r.integer(t2));
          else if (i2 == 4 && id == 8) h.encoding = int32_t(r.integer(t2));
          else if (i2 == 5 && id == 8) h.def_len = int32_t(r.integer(t2));
          else if (i2 == 6 && id == 8) h.rep_len = int32_t(r.integer(t2));
          else r.skip(t2);
        }
        break;
      }
      default:
        r.skip(t);
    }
  }
  return r.ok();
}

struct ChunkWork {
  pqh_chunk chunk;
  std::vector<pqh_page> pages;  // image_offset relative to `bytes` (device codecs: to the image space)
  std::vector<uint8_t> bytes;
  double seconds = 0;
  bool device_codecs = false;   // bytes = source bytes; images rebuilt on the device
  std::vector<pqh_codec_page> cps;
  int64_t image = 0;            // device codecs: image space used so far
};

// Device codecs: the page's source bytes (raw prefix a, then b) go to `bytes`; its image (of
// image_len bytes) gets a place in the image space.
void append_source(ChunkWork& w, pqh_page& pg, const uint8_t* a, size_t na, const uint8_t* b, size_t nb,
                   int64_t image_len, int32_t codec) {
  const size_t off = (w.bytes.size() + 63) & ~size_t(63);
  w.bytes.resize(off + na + nb);
  if (na) memcpy(w.bytes.data() + off, a, na);
  if (nb) memcpy(w.bytes.data() + off + na, b, nb);
  const int64_t img = (w.image + 63) & ~int64_t(63);
  w.image = img + image_len;
  pg.image_offset = img;
  pg.image_len = int32_t(image_len);
  pqh_codec_page cp;
  memset(&cp, 0, sizeof(cp));
  cp.src_offset = int64_t(off);
  cp.image_offset = img;
  cp.src_len = int32_t(na + nb);
  cp.image_len = int32_t(image_len);
  cp.raw_len = codec == PQH_CODEC_SNAPPY ? int32_t(na) : 0;
  cp.codec = codec;
  w.cps.push_back(cp);
}

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

void append_image(ChunkWork& w, pqh_page& pg, const uint8_t* a, size_t na, const uint8_t* b, size_t nb) {
  size_t off = (w.bytes.size() + 63) & ~size_t(63);
  w.bytes.resize(off + na + nb);
  if (na) memcpy(w.bytes.data() + off, a, na);
  if (nb) memcpy(w.bytes.data() + off + na, b, nb);
  pg.image_offset = int64_t(off);
  pg.image_len = int32_t(na + nb);
}

// readChunk + readPages for one chunk.
void walk_chunk(const pqh_file* f, const ColumnMeta& col, const ChunkMeta& m, int validate_crc, ChunkWork& w) {
  auto t0 = std::chrono::steady_clock::now();
  w.chunk.column = col.col;
  w.chunk.first_page = 0;
  w.chunk.num_pages = 0;
  w.chunk.host_status = PQH_OK;
  auto fail = [&](int code) { w.chunk.host_status = code; };
  if (m.has_file_path) return fail(PQH_ERR_IO);  // "nyi: data is in another file"
  if (!m.has_meta) return fail(PQH_ERR_SCHEMA);
  if (m.type != col.col.physical_type) return fail(PQH_ERR_SCHEMA);
  int64_t pos = m.has_dict_offset ? m.dict_page_offset : m.data_page_offset;
  int64_t count = 0;
  bool have_dict = false;
  std::vector<uint8_t> out;
  while (m.total_compressed - count > 0) {
    if (pos < 0 || pos > f->len) return fail(PQH_ERR_IO);
    TReader r(f->data + pos, f->data + f->len);
    PageHdr h;
    if (!parse_page_header(r, h)) return fail(PQH_ERR_THRIFT);
    pos += int64_t(r.consumed());
    count += int64_t(r.consumed());
    if (h.csize < 0 || h.usize < 0) return fail(PQH_ERR_PAGE_HEADER);  // readPageBlock
    const int64_t avail = f->len - pos;
    const int64_t got = h.csize < avail ? h.csize : avail;  // io.ReadAll(io.LimitReader)
    const uint8_t* block = f->data + pos;
    pos += got;
    count += got;
    if (validate_crc && h.has_crc && crc32_ieee(block, size_t(got)) != uint32_t(h.crc)) return fail(PQH_ERR_CRC);
    pqh_page pg;
    memset(&pg, 0, sizeof(pg));
    pg.page_type = h.type;
    pg.num_values = h.num_values;
    pg.encoding = h.encoding;
    pg.chunk = 0;
    const bool dev = w.device_codecs && m.codec == PQH_CODEC_SNAPPY;
    // whole-block pages (V1 data / dictionary): decompressed here, or left for the device
    auto whole_block = [&]() -> bool {
      if (dev) {
        if (!snappy_plausible(block, size_t(got), h.usize)) return false;
        append_source(w, pg, block, 0, block, size_t(got), h.usize, PQH_CODEC_SNAPPY);
        w.cps.back().raw_len = 0;
        return true;
      }
      if (!decompress_block(m.codec, block, size_t(got), size_t(h.usize), out) || int64_t(out.size()) != h.usize)
        return false;
      if (w.device_codecs) append_source(w, pg, out.data(), out.size(), nullptr, 0, int64_t(out.size()), PQH_CODEC_UNCOMPRESSED);
      else append_image(w, pg, out.data(), out.size(), nullptr, 0);
      return true;
    };
    if (h.type == PQH_DICTIONARY_PAGE) {
      if (have_dict) return fail(PQH_ERR_DICT_PAGE);
      if (!h.has_dict) return fail(PQH_ERR_PAGE_HEADER);
      if (got != h.csize) return fail(PQH_ERR_DECOMPRESS);
      if (!whole_block()) return fail(PQH_ERR_DECOMPRESS);
      w.pages.push_back(pg);
      have_dict = true;
      if (m.has_dict_offset && m.dict_page_offset != pos) {  // seek to DataPageOffset
        count += m.data_page_offset - pos;
        pos = m.data_page_offset;
      }
      continue;
    }
    if (h.type == PQH_DATA_PAGE) {
      if (!h.has_dp) return fail(PQH_ERR_PAGE_HEADER);
      if (got != h.csize) return fail(PQH_ERR_DECOMPRESS);
      if (!whole_block()) return fail(PQH_ERR_DECOMPRESS);
    } else if (h.type == PQH_DATA_PAGE_V2) {
      if (!h.has_v2) return fail(PQH_ERR_PAGE_HEADER);
      if (h.num_values < 0 || h.rep_len < 0 || h.def_len < 0) return fail(PQH_ERR_PAGE_HEADER);
      const int64_t levels = int64_t(h.rep_len) + h.def_len;
      if (levels > got) return fail(PQH_ERR_PAGE_HEADER);  // slice out of range in the reference
      if (got != h.csize) return fail(PQH_ERR_DECOMPRESS);
      // the values section is decompressed regardless of is_compressed (page_v2.go:125)
      if (dev) {
        if (!snappy_plausible(block + levels, size_t(got - levels), int64_t(h.usize) - levels))
          return fail(PQH_ERR_DECOMPRESS);
        append_source(w, pg, block, size_t(levels), block + levels, size_t(got - levels), h.usize, PQH_CODEC_SNAPPY);
      } else {
        if (!decompress_block(m.codec, block + levels, size_t(got - levels), size_t(h.usize - levels), out) ||
            int64_t(out.size()) != int64_t(h.usize) - levels)
          return fail(PQH_ERR_DECOMPRESS);
        if (w.device_codecs)
          append_source(w, pg, block, size_t(levels), out.data(), out.size(), int64_t(levels) + int64_t(out.size()),
                        PQH_CODEC_UNCOMPRESSED);
        else
          append_image(w, pg, block, size_t(levels), out.data(), out.size());
      }
      pg.def_levels_byte_length = h.def_len;
      pg.rep_levels_byte_length = h.rep_len;
    } else {
      return fail(PQH_ERR_PAGE_HEADER);  // "DATA_PAGE or DATA_PAGE_V2 type supported"
    }
    w.pages.push_back(pg);
  }
  w.seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
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

int pqh_file_load_ex(pqh_file* f, int32_t rg_begin, int32_t rg_end, const int32_t* columns, int32_t num_columns,
                     int32_t validate_crc, uint32_t flags, pqh_host_batch** out) {
  *out = nullptr;
  if (!f) return PQH_ERR_ARG;
  if (rg_begin < 0 || rg_end > int32_t(f->rgs.size()) || rg_begin > rg_end)
    return file_error(f, PQH_ERR_ARG, "row group range out of bounds");
  for (int32_t i = 0; i < num_columns; i++)
    if (columns[i] < 0 || size_t(columns[i]) >= f->columns.size()) return file_error(f, PQH_ERR_ARG, "bad column");
  const int64_t nchunks = int64_t(rg_end - rg_begin) * num_columns;
  std::vector<ChunkWork> work(static_cast<size_t>(nchunks));
  // device codecs only when some selected chunk is SNAPPY (otherwise the plain layout)
  bool dev = false;
  if (flags & PQH_LOAD_DEVICE_SNAPPY)
    for (int32_t rg = rg_begin; rg < rg_end && !dev; rg++)
      for (int32_t i = 0; i < num_columns && !dev; i++) {
        const RowGroupMeta& g = f->rgs[size_t(rg)];
        dev = size_t(columns[i]) < g.chunks.size() && g.chunks[size_t(columns[i])].has_meta &&
              g.chunks[size_t(columns[i])].codec == PQH_CODEC_SNAPPY;
      }
  for (auto& w : work) w.device_codecs = dev;
  std::atomic<int64_t> next{0};
  auto worker = [&]() {
    for (;;) {
      int64_t k = next.fetch_add(1);
      if (k >= nchunks) return;
      const int32_t rg = rg_begin + int32_t(k / num_columns);
      const int32_t ci = columns[k % num_columns];
      const RowGroupMeta& g = f->rgs[size_t(rg)];
      ChunkWork& w = work[size_t(k)];
      if (size_t(ci) >= g.chunks.size()) {  // "column index %d is out of bounds"
        w.chunk.column = f->columns[size_t(ci)].col;
        w.chunk.host_status = PQH_ERR_SCHEMA;
        continue;
      }
      walk_chunk(f, f->columns[size_t(ci)], g.chunks[size_t(ci)], validate_crc, w);
    }
  };
  int nt = int(std::thread::hardware_concurrency());
  if (nt > 16) nt = 16;
  if (nt < 1) nt = 1;
  if (nt > nchunks) nt = int(nchunks > 0 ? nchunks : 1);
  std::vector<std::thread> th;
  for (int i = 0; i < nt; i++) th.emplace_back(worker);
  for (auto& t : th) t.join();

  pqh_host_batch* hb = new pqh_host_batch();
  size_t total = 0;
  for (auto& w : work) total = ((total + 63) & ~size_t(63)) + w.bytes.size();
  hb->payload.reserve(total + PQH_PAYLOAD_PAD);
  int64_t image = 0;
  for (auto& w : work) {
    size_t base = (hb->payload.size() + 63) & ~size_t(63);
    hb->payload.resize(base);
    hb->payload.insert(hb->payload.end(), w.bytes.begin(), w.bytes.end());
    const int64_t ibase = dev ? (image + 63) & ~int64_t(63) : int64_t(base);
    pqh_chunk c = w.chunk;
    c.first_page = int32_t(hb->pages.size());
    c.num_pages = int32_t(w.pages.size());
    const int32_t ci = int32_t(hb->chunks.size());
    for (size_t i = 0; i < w.pages.size(); i++) {
      pqh_page pg = w.pages[i];
      pg.image_offset += ibase;
      pg.chunk = ci;
      hb->pages.push_back(pg);
      if (dev) {
        pqh_codec_page cp = w.cps[i];
        cp.src_offset += int64_t(base);
        cp.image_offset += ibase;
        cp.chunk = ci;
        hb->codec_pages.push_back(cp);
      }
    }
    if (dev) image = ibase + w.image;
    hb->chunks.push_back(c);
    hb->decompress_seconds += w.seconds;
  }
  hb->image_bytes = dev ? image : 0;
  hb->payload_bytes = int64_t(hb->payload.size());
  hb->payload.resize(hb->payload.size() + PQH_PAYLOAD_PAD, 0);
  *out = hb;
  return PQH_OK;
}

int32_t pqh_host_batch_num_codec_pages(const pqh_host_batch* hb) { return int32_t(hb->codec_pages.size()); }
const pqh_codec_page* pqh_host_batch_codec_pages(const pqh_host_batch* hb) { return hb->codec_pages.data(); }
int64_t pqh_host_batch_image_bytes(const pqh_host_batch* hb) { return hb->image_bytes; }
int32_t pqh_host_batch_num_chunks(const pqh_host_batch* hb) { return int32_t(hb->chunks.size()); }
int32_t pqh_host_batch_num_pages(const pqh_host_batch* hb) { return int32_t(hb->pages.size()); }
const pqh_chunk* pqh_host_batch_chunks(const pqh_host_batch* hb) { return hb->chunks.data(); }
const pqh_page* pqh_host_batch_pages(const pqh_host_batch* hb) { return hb->pages.data(); }
const uint8_t* pqh_host_batch_payload(const pqh_host_batch* hb) { return hb->payload.data(); }
int64_t pqh_host_batch_payload_bytes(const pqh_host_batch* hb) { return hb->payload_bytes; }
double pqh_host_batch_decompress_seconds(const pqh_host_batch* hb) { return hb->decompress_seconds; }
void pqh_host_batch_free(pqh_host_batch* hb) { delete hb; }

}  // extern "C"
