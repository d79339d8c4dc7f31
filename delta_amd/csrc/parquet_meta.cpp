#include "parquet_meta.h"

#include <algorithm>
#include <cstring>
#include <functional>

#include "common.h"
#include "snappy_host.h"

namespace dr {
namespace pq {
namespace {

// ---- Thrift compact protocol reader ----------------------------------------------------------
enum CType { CT_STOP = 0, CT_TRUE = 1, CT_FALSE = 2, CT_BYTE = 3, CT_I16 = 4, CT_I32 = 5, CT_I64 = 6,
             CT_DOUBLE = 7, CT_BINARY = 8, CT_LIST = 9, CT_SET = 10, CT_MAP = 11, CT_STRUCT = 12 };

struct TReader {
  const uint8_t* p;
  const uint8_t* end;
  void need(size_t n) const {
    if (size_t(end - p) < n) fail(DR_E_PARQUET, "truncated thrift structure");
  }
  uint8_t byte() { need(1); return *p++; }
  uint64_t varint() {
    uint64_t v = 0;
    for (int s = 0; s < 70; s += 7) {
      uint8_t b = byte();
      v |= uint64_t(b & 0x7f) << s;
      if (!(b & 0x80)) return v;
    }
    fail(DR_E_PARQUET, "bad varint");
  }
  int64_t zigzag() { uint64_t v = varint(); return int64_t(v >> 1) ^ -int64_t(v & 1); }
  std::string binary() {
    uint64_t n = varint();
    need(n);
    std::string s(reinterpret_cast<const char*>(p), n);
    p += n;
    return s;
  }
  void skip(int t) {
    switch (t) {
      case CT_TRUE: case CT_FALSE: return;
      case CT_BYTE: byte(); return;
      case CT_I16: case CT_I32: case CT_I64: varint(); return;
      case CT_DOUBLE: need(8); p += 8; return;
      case CT_BINARY: { uint64_t n = varint(); need(n); p += n; return; }
      case CT_LIST: case CT_SET: {
        uint8_t h = byte();
        uint64_t n = h >> 4;
        if (n == 15) n = varint();
        int et = h & 15;
        for (uint64_t i = 0; i < n; ++i) {
          if (et == CT_TRUE || et == CT_FALSE) byte(); else skip(et);
        }
        return;
      }
      case CT_MAP: {
        uint64_t n = varint();
        if (!n) return;
        uint8_t kv = byte();
        for (uint64_t i = 0; i < n; ++i) { skip(kv >> 4); skip(kv & 15); }
        return;
      }
      case CT_STRUCT: {
        int16_t last = 0;
        for (;;) {
          int id, ft;
          if (!field(&last, &id, &ft)) return;
          skip(ft);
        }
      }
      default: fail(DR_E_PARQUET, fmt("bad thrift type %d", t));
    }
  }
  // Reads a field header; returns false on STOP.
  bool field(int16_t* last, int* id, int* type) {
    uint8_t h = byte();
    if (h == 0) return false;
    *type = h & 15;
    int d = h >> 4;
    if (d) *id = *last + d; else *id = int(zigzag());
    *last = int16_t(*id);
    return true;
  }
  // list header -> (size, elem type)
  uint64_t list(int* et) {
    uint8_t h = byte();
    uint64_t n = h >> 4;
    if (n == 15) n = varint();
    *et = h & 15;
    return n;
  }
  // Iterates a struct: fn(id, type) must consume the value or return false to skip it.
  void each(const std::function<bool(int, int)>& fn) {
    int16_t last = 0;
    for (;;) {
      int id, t;
      if (!field(&last, &id, &t)) return;
      if (!fn(id, t)) skip(t);
    }
  }
};

SchemaElement read_schema_element(TReader& r) {
  SchemaElement e;
  r.each([&](int id, int t) {
    switch (id) {
      case 1: e.type = int(r.zigzag()); return true;
      case 2: e.type_length = int(r.zigzag()); return true;
      case 3: e.repetition = int(r.zigzag()); return true;
      case 4: e.name = r.binary(); return true;
      case 5: e.num_children = int(r.zigzag()); return true;
      case 6: e.converted_type = int(r.zigzag()); return true;
      default: return false;
    }
  });
  return e;
}

ColumnChunk read_column_chunk(TReader& r) {
  ColumnChunk c;
  r.each([&](int id, int t) {
    if (id != 3 || t != CT_STRUCT) return false;  // meta_data
    r.each([&](int mid, int mt) {
      switch (mid) {
        case 1: c.type = int(r.zigzag()); return true;
        case 3: {
          int et;
          uint64_t n = r.list(&et);
          std::string path;
          for (uint64_t i = 0; i < n; ++i) { if (i) path += "."; path += r.binary(); }
          c.path = path;
          return true;
        }
        case 4: c.codec = int(r.zigzag()); return true;
        case 5: c.num_values = r.zigzag(); return true;
        case 6: c.total_uncompressed = r.zigzag(); return true;
        case 7: c.total_compressed = r.zigzag(); return true;
        case 9: c.data_page_offset = r.zigzag(); return true;
        case 11: c.dictionary_page_offset = r.zigzag(); return true;
        default: return false;
      }
    });
    return true;
  });
  return c;
}

RowGroup read_row_group(TReader& r) {
  RowGroup g;
  r.each([&](int id, int t) {
    switch (id) {
      case 1: {
        int et;
        uint64_t n = r.list(&et);
        for (uint64_t i = 0; i < n; ++i) g.cols.push_back(read_column_chunk(r));
        return true;
      }
      case 3: g.num_rows = r.zigzag(); return true;
      default: return false;
    }
  });
  return g;
}

// Builds the leaf list (dotted paths, max def/rep levels) from the flattened schema.
void build_leaves(FileMeta& m) {
  size_t idx = 1;  // element 0 is the root
  struct Frame { std::string path; std::vector<std::string> parts; int def, rep; std::vector<int> def_of; };
  std::function<void(const Frame&, int)> rec = [&](const Frame& parent, int nchildren) {
    for (int c = 0; c < nchildren; ++c) {
      if (idx >= m.schema.size()) fail(DR_E_PARQUET, "schema truncated");
      const SchemaElement& e = m.schema[idx++];
      Frame f = parent;
      f.path = parent.path.empty() ? e.name : parent.path + "." + e.name;
      f.parts.push_back(e.name);
      if (e.repetition == OPTIONAL) f.def += 1;
      if (e.repetition == REPEATED) { f.def += 1; f.rep += 1; }
      f.def_of.push_back(f.def);
      if (e.num_children > 0) {
        rec(f, e.num_children);
      } else {
        Leaf l;
        l.path = f.path; l.parts = f.parts; l.type = e.type;
        l.max_def = f.def; l.max_rep = f.rep; l.def_of = f.def_of;
        m.leaves.push_back(l);
      }
    }
  };
  if (m.schema.empty()) fail(DR_E_PARQUET, "empty schema");
  rec(Frame{"", {}, 0, 0, {}}, m.schema[0].num_children);
}

}  // namespace

const Leaf* FileMeta::leaf(const std::string& path) const {
  for (const Leaf& l : leaves) if (l.path == path) return &l;
  return nullptr;
}
int FileMeta::leaf_index(const std::string& path) const {
  for (size_t i = 0; i < leaves.size(); ++i) if (leaves[i].path == path) return int(i);
  return -1;
}

FileMeta parse_footer(const uint8_t* file, uint64_t len) {
  if (len < 12 || memcmp(file, "PAR1", 4) || memcmp(file + len - 4, "PAR1", 4))
    fail(DR_E_PARQUET, "not a parquet file (missing PAR1 magic)");
  uint32_t flen;
  memcpy(&flen, file + len - 8, 4);
  if (uint64_t(flen) + 12 > len) fail(DR_E_PARQUET, "bad footer length");
  TReader r{file + len - 8 - flen, file + len - 8};
  FileMeta m;
  r.each([&](int id, int t) {
    switch (id) {
      case 2: {
        int et;
        uint64_t n = r.list(&et);
        for (uint64_t i = 0; i < n; ++i) m.schema.push_back(read_schema_element(r));
        return true;
      }
      case 3: m.num_rows = r.zigzag(); return true;
      case 4: {
        int et;
        uint64_t n = r.list(&et);
        for (uint64_t i = 0; i < n; ++i) m.row_groups.push_back(read_row_group(r));
        return true;
      }
      case 6: m.created_by = r.binary(); return true;
      default: return false;
    }
  });
  build_leaves(m);
  return m;
}

std::vector<Page> walk_pages(const uint8_t* file, uint64_t len, const ColumnChunk& cc) {
  int64_t start = cc.data_page_offset;
  if (cc.dictionary_page_offset > 0 && cc.dictionary_page_offset < start) start = cc.dictionary_page_offset;
  if (start < 4 || uint64_t(start + cc.total_compressed) > len)
    fail(DR_E_PARQUET, fmt("column chunk %s out of file bounds", cc.path.c_str()));
  std::vector<Page> pages;
  int64_t values_seen = 0;
  const uint8_t* p = file + start;
  const uint8_t* end = file + start + cc.total_compressed;
  while (p < end && values_seen < cc.num_values) {
    TReader r{p, end};
    Page pg;
    r.each([&](int id, int t) {
      switch (id) {
        case 1: pg.page_type = int(r.zigzag()); return true;
        case 2: pg.uncompressed_size = r.zigzag(); return true;
        case 3: pg.compressed_size = r.zigzag(); return true;
        case 5:  // DataPageHeader
          r.each([&](int did, int dt) {
            switch (did) {
              case 1: pg.num_values = int32_t(r.zigzag()); return true;
              case 2: pg.encoding = int32_t(r.zigzag()); return true;
              case 3: pg.def_enc = int32_t(r.zigzag()); return true;
              case 4: pg.rep_enc = int32_t(r.zigzag()); return true;
              default: return false;
            }
          });
          return true;
        case 7:  // DictionaryPageHeader
          r.each([&](int did, int dt) {
            switch (did) {
              case 1: pg.num_values = int32_t(r.zigzag()); return true;
              case 2: pg.encoding = int32_t(r.zigzag()); return true;
              default: return false;
            }
          });
          return true;
        case 8:  // DataPageHeaderV2
          r.each([&](int did, int dt) {
            switch (did) {
              case 1: pg.num_values = int32_t(r.zigzag()); return true;
              case 4: pg.encoding = int32_t(r.zigzag()); return true;
              case 5: pg.v2_def_len = int32_t(r.zigzag()); return true;
              case 6: pg.v2_rep_len = int32_t(r.zigzag()); return true;
              case 7: pg.v2_compressed = dt == CT_TRUE ? 1 : 0; return true;
              default: return false;
            }
          });
          return true;
        default: return false;
      }
    });
    pg.data_off = int64_t(r.p - file);
    if (pg.compressed_size < 0 || r.p + pg.compressed_size > end)
      fail(DR_E_PARQUET, fmt("page of %s overruns its column chunk", cc.path.c_str()));
    p = r.p + pg.compressed_size;
    if (pg.page_type == DATA_PAGE || pg.page_type == DATA_PAGE_V2) values_seen += pg.num_values;
    if (pg.page_type == DATA_PAGE || pg.page_type == DATA_PAGE_V2 || pg.page_type == DICTIONARY_PAGE)
      pages.push_back(pg);
  }
  return pages;
}

// ---- host decode ----------------------------------------------------------------------------
namespace {

int bit_width(int max_level) {
  int w = 0;
  while ((1 << w) <= max_level) ++w;
  return max_level == 0 ? 0 : w;
}

// RLE / bit-packed hybrid decoder (Parquet Encodings: RLE).
void rle_decode(const uint8_t* p, const uint8_t* end, int width, int64_t count, std::vector<uint32_t>& out) {
  int64_t got = 0;
  const int bytes = (width + 7) / 8;
  while (got < count) {
    if (p >= end) fail(DR_E_PARQUET, "RLE run truncated");
    uint64_t h = 0;
    int s = 0;
    for (;;) {
      if (p >= end) fail(DR_E_PARQUET, "RLE header truncated");
      uint8_t b = *p++;
      h |= uint64_t(b & 0x7f) << s;
      s += 7;
      if (!(b & 0x80)) break;
    }
    if (h & 1) {  // bit-packed: (h>>1) groups of 8
      int64_t n = int64_t(h >> 1) * 8;
      uint64_t acc = 0;
      int have = 0;
      for (int64_t i = 0; i < n; ++i) {
        while (have < width) {
          if (p >= end) { if (got >= count) return; fail(DR_E_PARQUET, "bit-packed run truncated"); }
          acc |= uint64_t(*p++) << have;
          have += 8;
        }
        uint32_t v = width ? uint32_t(acc & ((1ull << width) - 1)) : 0;
        acc >>= width;
        have -= width;
        if (got < count) { out.push_back(v); ++got; }
      }
    } else {
      int64_t n = int64_t(h >> 1);
      uint32_t v = 0;
      for (int b = 0; b < bytes; ++b) { if (p >= end) fail(DR_E_PARQUET, "RLE value truncated"); v |= uint32_t(*p++) << (8 * b); }
      for (int64_t i = 0; i < n && got < count; ++i, ++got) out.push_back(v);
    }
  }
}

void plain_values(const uint8_t* p, const uint8_t* end, int type, int64_t n, HostColumn& col) {
  if (type == BYTE_ARRAY) {
    for (int64_t i = 0; i < n; ++i) {
      if (end - p < 4) fail(DR_E_PARQUET, "byte array length truncated");
      uint32_t l;
      memcpy(&l, p, 4);
      p += 4;
      if (uint64_t(end - p) < l) fail(DR_E_PARQUET, "byte array truncated");
      col.svals.emplace_back(reinterpret_cast<const char*>(p), l);
      p += l;
    }
  } else if (type == INT64) {
    if (end - p < n * 8) fail(DR_E_PARQUET, "int64 values truncated");
    for (int64_t i = 0; i < n; ++i) { int64_t v; memcpy(&v, p + 8 * i, 8); col.ivals.push_back(v); }
  } else if (type == INT32) {
    if (end - p < n * 4) fail(DR_E_PARQUET, "int32 values truncated");
    for (int64_t i = 0; i < n; ++i) { int32_t v; memcpy(&v, p + 4 * i, 4); col.ivals.push_back(v); }
  } else if (type == BOOLEAN) {
    for (int64_t i = 0; i < n; ++i) {
      if (p + i / 8 >= end) fail(DR_E_PARQUET, "boolean values truncated");
      col.ivals.push_back((p[i / 8] >> (i % 8)) & 1);
    }
  } else {
    fail(DR_E_UNSUPPORTED, fmt("host decode: unsupported physical type %d", type));
  }
}

}  // namespace

HostColumn decode_column_host(const uint8_t* file, uint64_t len, const ColumnChunk& cc, const Leaf& leaf) {
  if (cc.codec != UNCOMPRESSED && cc.codec != SNAPPY)
    fail(DR_E_UNSUPPORTED, fmt("codec %d not supported (column %s)", cc.codec, cc.path.c_str()));
  HostColumn col;
  HostColumn dict;
  bool have_dict = false;
  std::vector<uint8_t> buf;
  for (const Page& pg : walk_pages(file, len, cc)) {
    const uint8_t* body = file + pg.data_off;
    // DATA_PAGE_V2 keeps the level sections uncompressed in front of the (maybe compressed) values.
    int64_t lv = pg.page_type == DATA_PAGE_V2 ? pg.v2_def_len + pg.v2_rep_len : 0;
    bool compressed = cc.codec == SNAPPY && !(pg.page_type == DATA_PAGE_V2 && !pg.v2_compressed);
    buf.resize(size_t(pg.uncompressed_size));
    if (lv) memcpy(buf.data(), body, size_t(lv));
    if (compressed) {
      if (!snappy_decompress(body + lv, size_t(pg.compressed_size - lv), buf.data() + lv,
                             size_t(pg.uncompressed_size - lv)))
        fail(DR_E_PARQUET, fmt("corrupt snappy page in %s", cc.path.c_str()));
    } else {
      memcpy(buf.data() + lv, body + lv, size_t(pg.uncompressed_size - lv));
    }
    const uint8_t* p = buf.data();
    const uint8_t* end = p + buf.size();
    if (pg.page_type == DICTIONARY_PAGE) {
      dict = HostColumn();
      plain_values(p, end, leaf.type, pg.num_values, dict);
      have_dict = true;
      continue;
    }
    std::vector<uint32_t> rep, def;
    if (pg.page_type == DATA_PAGE_V2) {
      if (leaf.max_rep) rle_decode(p, p + pg.v2_rep_len, bit_width(leaf.max_rep), pg.num_values, rep);
      if (leaf.max_def) rle_decode(p + pg.v2_rep_len, p + lv, bit_width(leaf.max_def), pg.num_values, def);
      p += lv;
    } else {
      for (int which = 0; which < 2; ++which) {
        int maxl = which == 0 ? leaf.max_rep : leaf.max_def;
        if (!maxl) continue;
        if (end - p < 4) fail(DR_E_PARQUET, "level length truncated");
        uint32_t l;
        memcpy(&l, p, 4);
        p += 4;
        if (uint64_t(end - p) < l) fail(DR_E_PARQUET, "levels truncated");
        rle_decode(p, p + l, bit_width(maxl), pg.num_values, which == 0 ? rep : def);
        p += l;
      }
    }
    int64_t nonnull = 0;
    for (int64_t i = 0; i < pg.num_values; ++i) {
      uint32_t d = leaf.max_def ? def[i] : 0;
      uint32_t rr = leaf.max_rep ? rep[i] : 0;
      col.def.push_back(uint8_t(d));
      col.rep.push_back(uint8_t(rr));
      if (int(d) == leaf.max_def) ++nonnull;
    }
    if (pg.encoding == PLAIN) {
      plain_values(p, end, leaf.type, nonnull, col);
    } else if (pg.encoding == PLAIN_DICTIONARY || pg.encoding == RLE_DICTIONARY) {
      if (!have_dict) fail(DR_E_PARQUET, "dictionary-encoded page without a dictionary");
      if (nonnull == 0) continue;
      if (p >= end) fail(DR_E_PARQUET, "dictionary indices truncated");
      int w = *p++;
      std::vector<uint32_t> idx;
      rle_decode(p, end, w, nonnull, idx);
      for (uint32_t k : idx) {
        if (leaf.type == BYTE_ARRAY) {
          if (k >= dict.svals.size()) fail(DR_E_PARQUET, "dictionary index out of range");
          col.svals.push_back(dict.svals[k]);
        } else {
          if (k >= dict.ivals.size()) fail(DR_E_PARQUET, "dictionary index out of range");
          col.ivals.push_back(dict.ivals[k]);
        }
      }
    } else if (pg.encoding == RLE && leaf.type == BOOLEAN) {
      if (end - p < 4) fail(DR_E_PARQUET, "boolean RLE truncated");
      p += 4;
      std::vector<uint32_t> v;
      rle_decode(p, end, 1, nonnull, v);
      for (uint32_t b : v) col.ivals.push_back(b);
    } else {
      fail(DR_E_UNSUPPORTED, fmt("encoding %d not supported (column %s)", pg.encoding, cc.path.c_str()));
    }
  }
  return col;
}

}  // namespace pq
}  // namespace dr

namespace dr {
namespace pq {
namespace {

struct Run { uint32_t v; int64_t n; };

// RLE/bit-packed hybrid -> runs (bit-packed groups become length-1 runs, merged when equal).
void rle_runs(const uint8_t* p, const uint8_t* end, int width, int64_t count, std::vector<Run>& out) {
  int64_t got = 0;
  const int bytes = (width + 7) / 8;
  auto push = [&](uint32_t v, int64_t n) {
    if (n <= 0) return;
    if (!out.empty() && out.back().v == v) out.back().n += n; else out.push_back({v, n});
  };
  while (got < count) {
    if (p >= end) fail(DR_E_PARQUET, "RLE run truncated");
    uint64_t h = 0;
    int s = 0;
    for (;;) {
      if (p >= end) fail(DR_E_PARQUET, "RLE header truncated");
      uint8_t b = *p++;
      h |= uint64_t(b & 0x7f) << s;
      s += 7;
      if (!(b & 0x80)) break;
    }
    if (h & 1) {
      int64_t n = int64_t(h >> 1) * 8;
      uint64_t acc = 0;
      int have = 0;
      for (int64_t i = 0; i < n && got < count; ++i) {
        while (have < width) { acc |= uint64_t(p < end ? *p : 0) << have; ++p; have += 8; }
        uint32_t v = width ? uint32_t(acc & ((1ull << width) - 1)) : 0;
        acc >>= width;
        have -= width;
        push(v, 1);
        ++got;
      }
    } else {
      int64_t n = int64_t(h >> 1);
      uint32_t v = 0;
      for (int b = 0; b < bytes; ++b) { if (p >= end) fail(DR_E_PARQUET, "RLE value truncated"); v |= uint32_t(*p++) << (8 * b); }
      n = std::min(n, count - got);
      push(v, n);
      got += n;
    }
  }
}

int bw(int max_level) {
  int w = 0;
  while ((1 << w) <= max_level) ++w;
  return max_level == 0 ? 0 : w;
}

struct ValueStream {
  const uint8_t* p = nullptr;
  const uint8_t* end = nullptr;
  int type = 0;
  int64_t bool_bit = 0;
  bool dict = false;
  std::vector<uint32_t> idx;
  size_t idx_pos = 0;
  const HostColumn* dictv = nullptr;
  void next(Entry& e) {
    if (dict) {
      if (idx_pos >= idx.size()) fail(DR_E_PARQUET, "dictionary indices exhausted");
      uint32_t k = idx[idx_pos++];
      if (type == BYTE_ARRAY) {
        if (k >= dictv->svals.size()) fail(DR_E_PARQUET, "dictionary index out of range");
        e.sval = dictv->svals[k];
      } else {
        if (k >= dictv->ivals.size()) fail(DR_E_PARQUET, "dictionary index out of range");
        e.ival = dictv->ivals[k];
      }
      return;
    }
    if (type == BYTE_ARRAY) {
      if (end - p < 4) fail(DR_E_PARQUET, "byte array length truncated");
      uint32_t l;
      memcpy(&l, p, 4);
      p += 4;
      if (uint64_t(end - p) < l) fail(DR_E_PARQUET, "byte array truncated");
      e.sval.assign(reinterpret_cast<const char*>(p), l);
      p += l;
    } else if (type == INT64) {
      if (end - p < 8) fail(DR_E_PARQUET, "int64 truncated");
      memcpy(&e.ival, p, 8);
      p += 8;
    } else if (type == INT32) {
      if (end - p < 4) fail(DR_E_PARQUET, "int32 truncated");
      int32_t v;
      memcpy(&v, p, 4);
      e.ival = v;
      p += 4;
    } else if (type == BOOLEAN) {
      if (p + bool_bit / 8 >= end) fail(DR_E_PARQUET, "boolean truncated");
      e.ival = (p[bool_bit / 8] >> (bool_bit % 8)) & 1;
      ++bool_bit;
    } else if (type == INT96) {
      if (end - p < 12) fail(DR_E_PARQUET, "int96 truncated");
      memcpy(&e.ival, p, 8);  // nanos-of-day (not used by replay)
      p += 12;
    } else {
      fail(DR_E_UNSUPPORTED, fmt("unsupported physical type %d", type));
    }
  }
};

}  // namespace

std::vector<Entry> sparse_entries(const uint8_t* file, uint64_t len, const ColumnChunk& cc, const Leaf& leaf,
                                  int thr, int64_t row_base) {
  if (cc.codec != UNCOMPRESSED && cc.codec != SNAPPY)
    fail(DR_E_UNSUPPORTED, fmt("codec %d not supported (column %s)", cc.codec, cc.path.c_str()));
  std::vector<Entry> out;
  HostColumn dict;
  bool have_dict = false;
  std::vector<uint8_t> buf;
  int64_t row = row_base - 1;
  for (const Page& pg : walk_pages(file, len, cc)) {
    const uint8_t* body = file + pg.data_off;
    int64_t lv = pg.page_type == DATA_PAGE_V2 ? pg.v2_def_len + pg.v2_rep_len : 0;
    bool compressed = cc.codec == SNAPPY && !(pg.page_type == DATA_PAGE_V2 && !pg.v2_compressed);
    buf.resize(size_t(pg.uncompressed_size) + 16);
    if (lv) memcpy(buf.data(), body, size_t(lv));
    if (compressed) {
      if (!snappy_decompress(body + lv, size_t(pg.compressed_size - lv), buf.data() + lv,
                             size_t(pg.uncompressed_size - lv)))
        fail(DR_E_PARQUET, fmt("corrupt snappy page in %s", cc.path.c_str()));
    } else {
      memcpy(buf.data() + lv, body + lv, size_t(pg.uncompressed_size - lv));
    }
    const uint8_t* p = buf.data();
    const uint8_t* end = p + pg.uncompressed_size;
    if (pg.page_type == DICTIONARY_PAGE) {
      dict = HostColumn();
      plain_values(p, end, leaf.type, pg.num_values, dict);
      have_dict = true;
      continue;
    }
    std::vector<Run> rep, def;
    if (pg.page_type == DATA_PAGE_V2) {
      if (leaf.max_rep) rle_runs(p, p + pg.v2_rep_len, bw(leaf.max_rep), pg.num_values, rep);
      if (leaf.max_def) rle_runs(p + pg.v2_rep_len, p + lv, bw(leaf.max_def), pg.num_values, def);
      p += lv;
    } else {
      for (int which = 0; which < 2; ++which) {
        int maxl = which == 0 ? leaf.max_rep : leaf.max_def;
        if (!maxl) continue;
        if (end - p < 4) fail(DR_E_PARQUET, "level length truncated");
        uint32_t l;
        memcpy(&l, p, 4);
        p += 4;
        if (uint64_t(end - p) < l) fail(DR_E_PARQUET, "levels truncated");
        rle_runs(p, p + l, bw(maxl), pg.num_values, which == 0 ? rep : def);
        p += l;
      }
    }
    if (rep.empty()) rep.push_back({0, pg.num_values});
    if (def.empty()) def.push_back({uint32_t(leaf.max_def), pg.num_values});
    ValueStream vs;
    vs.p = p; vs.end = end; vs.type = leaf.type;
    if (pg.encoding == PLAIN_DICTIONARY || pg.encoding == RLE_DICTIONARY) {
      if (!have_dict) fail(DR_E_PARQUET, "dictionary-encoded page without a dictionary");
      int64_t nonnull = 0;
      for (auto& r : def) if (int(r.v) == leaf.max_def) nonnull += r.n;
      vs.dict = true;
      vs.dictv = &dict;
      if (nonnull) {
        if (p >= end) fail(DR_E_PARQUET, "dictionary indices truncated");
        int w = *p;
        rle_decode(p + 1, end, w, nonnull, vs.idx);
      }
    } else if (pg.encoding == RLE && leaf.type == BOOLEAN) {
      int64_t nonnull = 0;
      for (auto& r : def) if (int(r.v) == leaf.max_def) nonnull += r.n;
      std::vector<uint32_t> bits;
      if (nonnull) rle_decode(p + 4, end, 1, nonnull, bits);
      dict.ivals.assign(bits.begin(), bits.end());  // reuse as an index-free stream
      vs.dict = true;
      vs.dictv = &dict;
      vs.type = INT64;
      vs.idx.resize(bits.size());
      for (size_t i = 0; i < bits.size(); ++i) vs.idx[i] = uint32_t(i);
    } else if (pg.encoding != PLAIN) {
      fail(DR_E_UNSUPPORTED, fmt("encoding %d not supported (column %s)", pg.encoding, cc.path.c_str()));
    }
    // walk rep/def runs in lockstep
    size_t ri = 0, di = 0;
    int64_t rleft = rep[0].n, dleft = def[0].n;
    int64_t done = 0;
    while (done < pg.num_values) {
      int64_t n = std::min(rleft, dleft);
      const uint32_t rv = rep[ri].v, dv = def[di].v;
      if (int(dv) < thr) {
        if (rv == 0) row += n;
      } else {
        for (int64_t k = 0; k < n; ++k) {
          if (rv == 0) ++row;
          Entry e;
          e.row = row;
          e.def = uint8_t(dv);
          e.rep = uint8_t(rv);
          e.has_value = int(dv) == leaf.max_def;
          e.ival = 0;
          if (e.has_value) vs.next(e);
          out.push_back(std::move(e));
        }
      }
      done += n;
      rleft -= n;
      dleft -= n;
      if (!rleft && ++ri < rep.size()) rleft = rep[ri].n;
      if (!dleft && ++di < def.size()) dleft = def[di].n;
      if ((ri >= rep.size() || di >= def.size()) && done < pg.num_values)
        fail(DR_E_PARQUET, "level runs shorter than num_values");
    }
  }
  return out;
}

}  // namespace pq
}  // namespace dr
