// CPU restatement of Delta Lake snapshot state reconstruction -- TEST INFRASTRUCTURE ONLY.
//
// The in-run CPU baseline of bench.py (`cpu_baseline.kind = "port"`) and the full-size parity
// checker of the GPU path. Independent of the product (its own listing, JSON scanner, Parquet +
// SNAPPY reader); never linked into libdeltareplay.
//
// Follows the reference step by step (D/ = core/src/main/scala/org/apache/spark/sql/delta/):
//  * LogSegment: newest complete checkpoint + contiguous deltas after it
//    (D/SnapshotManagement.scala:82-179, D/Checkpoints.scala:210-218);
//  * loadActions: checkpoint rows then JSON lines, in file order (D/Snapshot.scala:231-263);
//  * canonicalizePath (D/Snapshot.scala:301-328) and the URI-equality replay key
//    (D/actions/actions.scala:208-213);
//  * repartition(P, coalesce(add.path, remove.path)) + sortWithinPartitions("file")
//    (D/Snapshot.scala:103-104): P hash partitions, each keeping replay order;
//  * InMemoryLogReplay.append/checkpoint per partition: HashMap last-writer-wins, tombstones kept
//    iff delTimestamp > minFileRetentionTimestamp, output sorted by path
//    (D/actions/InMemoryLogReplay.scala:43-77);
//  * computedState counters (D/Snapshot.scala:140-151).
// Parity pinned by tests/test_oracle_cpp.py against the Python oracle (which is pinned to the
// reference's golden logs) and, at full size, by bench.py against the GPU's key sums.
//
// usage: replay_oracle <_delta_log dir> <minFileRetentionTimestamp> [--threads T] [--partitions P]
// prints one JSON line with counts, order-free key checksums (sum of the top 32 bits of xxh64 of
// each survivor's key, as dr_counts.live_key_sum / tomb_key_sum) and timings: read_s (file bytes into
// memory, untimed by the baseline), parse_s (checkpoint decode + JSON lines) and replay_s
// (canonicalize, partition, last-writer-wins, retention, per-partition sort by path).
// Allocation-free per action: paths are views into the file / page buffers or per-thread arenas.
#include <dirent.h>
#include <sys/stat.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <map>
#include <stdexcept>
#include <string>
#include <thread>
#include <iterator>
#include <array>
#include <memory>
#include <unordered_map>
#include <vector>

namespace {

// ---- xxHash64 (same key function as the device path, for order-free checksums) -----------------
const uint64_t P1 = 0x9E3779B185EBCA87ull, P2 = 0xC2B2AE3D27D4EB4Full, P3 = 0x165667B19E3779F9ull,
               P4 = 0x85EBCA77C2B2AE63ull, P5 = 0x27D4EB2F165667C5ull;
inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
inline uint64_t rd64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }
inline uint32_t rd32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
inline uint64_t xround(uint64_t a, uint64_t i) { return rotl(a + i * P2, 31) * P1; }
uint64_t xxh64(const uint8_t* p, size_t len) {
  const uint8_t* end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = P1 + P2, v2 = P2, v3 = 0, v4 = 0 - P1;
    do {
      v1 = xround(v1, rd64(p)); v2 = xround(v2, rd64(p + 8)); v3 = xround(v3, rd64(p + 16)); v4 = xround(v4, rd64(p + 24));
      p += 32;
    } while (p <= end - 32);
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    for (uint64_t v : {v1, v2, v3, v4}) { h ^= xround(0, v); h = h * P1 + P4; }
  } else {
    h = P5;
  }
  h += len;
  while (p + 8 <= end) { h ^= xround(0, rd64(p)); h = rotl(h, 27) * P1 + P4; p += 8; }
  if (p + 4 <= end) { h ^= uint64_t(rd32(p)) * P1; h = rotl(h, 23) * P2 + P3; p += 4; }
  while (p < end) { h ^= uint64_t(*p) * P5; h = rotl(h, 11) * P1; ++p; }
  h ^= h >> 33; h *= P2; h ^= h >> 29; h *= P3; h ^= h >> 32;
  return h ? h : 1;
}

[[noreturn]] void die(const std::string& m) { throw std::runtime_error(m); }

std::vector<uint8_t> read_all(const std::string& p) {
  std::ifstream f(p, std::ios::binary | std::ios::ate);
  if (!f) die("cannot open " + p);
  const std::streamsize n = f.tellg();
  std::vector<uint8_t> b;
  b.reserve(size_t(n) + 16);  // readable slack past the end for 8-byte loads
  b.resize(size_t(n));
  f.seekg(0);
  if (n && !f.read(reinterpret_cast<char*>(b.data()), n)) die("cannot read " + p);
  return b;
}

// ---- string views and per-thread arenas (no allocation per action) ---------------------------------
struct SV {
  const char* p = nullptr;
  uint32_t n = 0;
  bool eq(const char* s, size_t k) const { return n == k && !memcmp(p, s, k); }
};
inline bool operator<(const SV& a, const SV& b) {
  const int c = memcmp(a.p, b.p, std::min(a.n, b.n));
  return c ? c < 0 : a.n < b.n;
}

// Bump allocator in 4 MiB blocks: stable addresses, one per thread.
struct Arena {
  std::vector<std::unique_ptr<char[]>> blocks;
  size_t used = 0, cap = 0;
  char* take(size_t n) {
    if (used + n > cap) {
      cap = std::max<size_t>(n, size_t(4) << 20);
      blocks.emplace_back(new char[cap]);
      used = 0;
    }
    char* r = blocks.back().get() + used;
    used += n;
    return r;
  }
};

// ---- actions -------------------------------------------------------------------------------------
enum Kind : uint8_t { NONE = 0, ADD = 1, REMOVE = 2, META = 3, TXN = 4, PROT = 5, OTHER = 6 };
struct Action {
  Kind kind = NONE;
  bool has_delts = false;
  SV path;               // raw path (unescaped), a view into a file buffer, a page buffer or an arena
  int64_t size = 0;
  int64_t delts = 0;
};

// ---- JSON line scanner (SingleAction envelope) ----------------------------------------------------
struct J {
  const char* p; const char* e; Arena* arena; bool bad = false;
  void ws() { while (p < e && (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\n')) ++p; }
  bool lit(const char* s) { size_t n = strlen(s); if (size_t(e - p) >= n && !memcmp(p, s, n)) { p += n; return true; } bad = true; return false; }
  // A string token: a view of its raw body, unescaped into the arena only when it holds escapes
  // (and `out` wants the value).
  bool str(SV* out, bool want = true) {
    ws();
    if (p >= e || *p != '"') { bad = true; return false; }
    const char* b = ++p;
    bool esc = false;
    for (;;) {  // the closing quote: the next '"' preceded by an even run of backslashes
      const char* q = static_cast<const char*>(memchr(p, '"', size_t(e - p)));
      if (!q) { p = e; bad = true; return false; }
      const char* r = q;
      while (r > b && r[-1] == '\\') --r;
      if (r != q) esc = true;
      p = q + 1;
      if (((q - r) & 1) == 0) break;
    }
    const char* end = p - 1;
    if (!esc && memchr(b, '\\', size_t(end - b))) esc = true;
    if (!out || !want) return true;
    if (!esc) { *out = SV{b, uint32_t(end - b)}; return true; }
    char* o = arena->take(size_t(end - b));
    size_t k = 0;
    for (const char* q = b; q < end;) {
      char c = *q++;
      if (c != '\\') { o[k++] = c; continue; }
      char x = *q++;
      if (x == 'u') {
        if (end - q < 4) { bad = true; return false; }
        unsigned cp = 0;
        for (int i = 0; i < 4; ++i) { char h = *q++; cp = cp * 16 + (h >= '0' && h <= '9' ? h - '0' : (h | 32) - 'a' + 10); }
        if (cp >= 0xD800 && cp < 0xDC00 && end - q >= 6 && q[0] == '\\' && q[1] == 'u') {
          unsigned lo = 0;
          for (int i = 0; i < 4; ++i) { char h = q[2 + i]; lo = lo * 16 + (h >= '0' && h <= '9' ? h - '0' : (h | 32) - 'a' + 10); }
          if (lo >= 0xDC00 && lo < 0xE000) { cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00); q += 6; }
        }
        if (cp < 0x80) o[k++] = char(cp);
        else if (cp < 0x800) { o[k++] = char(0xC0 | (cp >> 6)); o[k++] = char(0x80 | (cp & 63)); }
        else if (cp < 0x10000) { o[k++] = char(0xE0 | (cp >> 12)); o[k++] = char(0x80 | ((cp >> 6) & 63)); o[k++] = char(0x80 | (cp & 63)); }
        else { o[k++] = char(0xF0 | (cp >> 18)); o[k++] = char(0x80 | ((cp >> 12) & 63)); o[k++] = char(0x80 | ((cp >> 6) & 63)); o[k++] = char(0x80 | (cp & 63)); }
        continue;
      }
      o[k++] = x == 'n' ? '\n' : x == 't' ? '\t' : x == 'r' ? '\r' : x == 'b' ? '\b' : x == 'f' ? '\f' : x;
    }
    *out = SV{o, uint32_t(k)};
    return true;
  }
  void skip() {
    ws();
    if (p >= e) { bad = true; return; }
    if (*p == '"') { str(nullptr); return; }
    if (*p == '{' || *p == '[') {
      int d = 0;
      while (p < e) {
        if (*p == '"') { str(nullptr); if (bad) return; continue; }
        if (*p == '{' || *p == '[') ++d;
        else if ((*p == '}' || *p == ']') && --d == 0) { ++p; return; }
        ++p;
      }
      bad = true;
      return;
    }
    const char* b = p;
    while (p < e && (isalnum((unsigned char)*p) || *p == '-' || *p == '+' || *p == '.')) ++p;
    if (p == b) bad = true;
  }
  bool null() { ws(); if (e - p >= 4 && !memcmp(p, "null", 4)) { p += 4; return true; } return false; }
  bool i64(int64_t* v) {
    ws();
    bool neg = p < e && *p == '-';
    if (neg) ++p;
    const char* b = p;
    uint64_t x = 0;
    while (p < e && *p >= '0' && *p <= '9') x = x * 10 + uint64_t(*p++ - '0');
    if (p == b || (p < e && (*p == '.' || *p == 'e' || *p == 'E'))) { bad = true; return false; }
    *v = neg ? -int64_t(x) : int64_t(x);
    return true;
  }
};

bool parse_file_obj(J& j, Action& a) {
  j.ws();
  if (!j.lit("{")) return false;
  j.ws();
  if (j.p < j.e && *j.p == '}') { ++j.p; return true; }
  for (;;) {
    SV k;
    if (!j.str(&k)) return false;
    j.ws();
    if (!j.lit(":")) return false;
    if (k.eq("path", 4)) { a.path = SV{}; if (!j.null() && !j.str(&a.path)) return false; }
    else if (k.eq("size", 4)) { if (!j.null() && !j.i64(&a.size)) return false; }
    else if (k.eq("deletionTimestamp", 17)) { if (j.null()) a.has_delts = false; else { if (!j.i64(&a.delts)) return false; a.has_delts = true; } }
    else { j.skip(); if (j.bad) return false; }
    j.ws();
    if (j.p < j.e && *j.p == ',') { ++j.p; continue; }
    if (j.p < j.e && *j.p == '}') { ++j.p; return true; }
    return false;
  }
}

// Returns the unwrapped action (priority add > remove > metaData > txn > protocol > cdc > commitInfo).
Action parse_line(const char* b, const char* e, Arena* arena) {
  J j{b, e, arena};
  Action add, rm, out;
  bool ha = false, hr = false, hm = false, ht = false, hp = false, ho = false;
  j.ws();
  if (j.p >= j.e) return out;
  if (!j.lit("{")) return out;
  j.ws();
  if (j.p < j.e && *j.p == '}') return out;
  for (;;) {
    SV k;
    if (!j.str(&k)) return Action();
    j.ws();
    if (!j.lit(":")) return Action();
    if (j.null()) {
    } else if (k.eq("add", 3)) { add.kind = ADD; if (!parse_file_obj(j, add)) return Action(); ha = true; }
    else if (k.eq("remove", 6)) { rm.kind = REMOVE; if (!parse_file_obj(j, rm)) return Action(); hr = true; }
    else {
      if (k.eq("metaData", 8)) hm = true;
      else if (k.eq("txn", 3)) ht = true;
      else if (k.eq("protocol", 8)) hp = true;
      else if (k.eq("cdc", 3) || k.eq("commitInfo", 10)) ho = true;
      j.skip();
    }
    if (j.bad) return Action();
    j.ws();
    if (j.p < j.e && *j.p == ',') { ++j.p; continue; }
    if (j.p < j.e && *j.p == '}') break;
    return Action();
  }
  if (ha) return add;
  if (hr) return rm;
  if (hm) { out.kind = META; return out; }
  if (ht) { out.kind = TXN; return out; }
  if (hp) { out.kind = PROT; return out; }
  if (ho) { out.kind = OTHER; return out; }
  return out;
}

// ---- minimal Parquet reader (Thrift compact footer, v1/v2 pages, SNAPPY, RLE/bit-packed,
//      PLAIN + dictionary) for add.path, add.size, remove.path, remove.deletionTimestamp ---------
struct TR {
  const uint8_t* p; const uint8_t* e;
  uint8_t b() { if (p >= e) die("thrift eof"); return *p++; }
  uint64_t vi() { uint64_t v = 0; for (int s = 0;; s += 7) { uint8_t x = b(); v |= uint64_t(x & 127) << s; if (!(x & 128)) return v; } }
  int64_t zz() { uint64_t v = vi(); return int64_t(v >> 1) ^ -int64_t(v & 1); }
  std::string bin() { uint64_t n = vi(); if (uint64_t(e - p) < n) die("thrift bin"); std::string s((const char*)p, n); p += n; return s; }
  void skip(int t) {
    switch (t) {
      case 1: case 2: return;
      case 3: b(); return;
      case 4: case 5: case 6: vi(); return;
      case 7: p += 8; return;
      case 8: { uint64_t n = vi(); p += n; return; }
      case 9: case 10: { uint8_t h = b(); uint64_t n = h >> 4; if (n == 15) n = vi(); for (uint64_t i = 0; i < n; ++i) { if ((h & 15) <= 2) b(); else skip(h & 15); } return; }
      case 11: { uint64_t n = vi(); if (!n) return; uint8_t kv = b(); for (uint64_t i = 0; i < n; ++i) { skip(kv >> 4); skip(kv & 15); } return; }
      case 12: { int16_t last = 0; int id, ty; while (field(&last, &id, &ty)) skip(ty); return; }
      default: die("thrift type");
    }
  }
  bool field(int16_t* last, int* id, int* ty) {
    uint8_t h = b();
    if (!h) return false;
    *ty = h & 15;
    int d = h >> 4;
    *id = d ? *last + d : int(zz());
    *last = int16_t(*id);
    return true;
  }
  uint64_t list(int* et) { uint8_t h = b(); uint64_t n = h >> 4; if (n == 15) n = vi(); *et = h & 15; return n; }
};

struct SchemaEl { int type = -1, rep = -1, nch = 0; std::string name; };
struct Chunk { std::string path; int type = -1, codec = 0; int64_t nval = 0, tcomp = 0, dpo = -1, dicto = -1; };
struct RG { int64_t rows = 0; std::vector<Chunk> cols; };
struct Leaf { std::string path; int type; int maxdef; int maxrep; std::vector<int> def_of; };

bool snappy(const uint8_t* in, size_t n, uint8_t* out, size_t olen) {
  size_t ip = 0, op = 0;
  uint64_t tot = 0;
  for (int s = 0; ip < n; s += 7) { uint8_t x = in[ip++]; tot |= uint64_t(x & 127) << s; if (!(x & 128)) break; }
  if (tot != olen) return false;
  while (ip < n) {
    uint8_t t = in[ip++];
    if ((t & 3) == 0) {
      size_t l = t >> 2;
      if (l >= 60) { size_t nb = l - 59; l = 0; for (size_t i = 0; i < nb; ++i) l |= size_t(in[ip + i]) << (8 * i); ip += nb; }
      l += 1;
      if (ip + l > n || op + l > olen) return false;
      memcpy(out + op, in + ip, l); ip += l; op += l;
    } else {
      size_t l, off;
      if ((t & 3) == 1) { l = ((t >> 2) & 7) + 4; off = (size_t(t >> 5) << 8) | in[ip]; ip += 1; }
      else if ((t & 3) == 2) { l = (t >> 2) + 1; off = in[ip] | (size_t(in[ip + 1]) << 8); ip += 2; }
      else { l = (t >> 2) + 1; off = rd32(in + ip); ip += 4; }
      if (!off || off > op || op + l > olen) return false;
      for (size_t i = 0; i < l; ++i) out[op + i] = out[op - off + i];
      op += l;
    }
  }
  return op == olen;
}

void rle(const uint8_t* p, const uint8_t* e, int w, int64_t cnt, std::vector<uint32_t>& out) {
  int64_t got = 0;
  while (got < cnt) {
    if (p >= e) die("rle eof");
    uint64_t h = 0;
    for (int s = 0;; s += 7) { uint8_t x = *p++; h |= uint64_t(x & 127) << s; if (!(x & 128)) break; }
    if (h & 1) {
      int64_t n = int64_t(h >> 1) * 8;
      uint64_t acc = 0; int have = 0;
      for (int64_t i = 0; i < n; ++i) {
        while (have < w) { acc |= uint64_t(p < e ? *p : 0) << have; ++p; have += 8; }
        uint32_t v = w ? uint32_t(acc & ((1ull << w) - 1)) : 0;
        acc >>= w; have -= w;
        if (got < cnt) { out.push_back(v); ++got; }
      }
    } else {
      uint32_t v = 0;
      for (int i = 0; i < (w + 7) / 8; ++i) v |= uint32_t(*p++) << (8 * i);
      for (int64_t i = 0; i < int64_t(h >> 1) && got < cnt; ++i, ++got) out.push_back(v);
    }
  }
}
int bwidth(int m) { int w = 0; while ((1 << w) <= m) ++w; return m ? w : 0; }

// Decoded flat column: def per row, values per row (string views into the page buffers it owns, or
// ints).
struct Col {
  std::vector<uint8_t> def;
  std::vector<SV> s;
  std::vector<int64_t> i;
  std::vector<std::vector<uint8_t>> bufs;  // decompressed pages the views point into
};

// One page of a column chunk: header fields and where its body lies.
struct Page { int pt = -1, enc = 0, nv = 0, v2d = 0, v2r = 0, v2c = 1; int64_t us = 0, cs = 0; const uint8_t* body = nullptr; };

// Page headers of a chunk, in order (Thrift PageHeader, parquet-format PageHeader fields 1-8).
std::vector<Page> chunk_pages(const uint8_t* f, const Chunk& c) {
  int64_t st = c.dpo;
  if (c.dicto > 0 && c.dicto < st) st = c.dicto;
  const uint8_t* p = f + st;
  const uint8_t* ce = p + c.tcomp;
  std::vector<Page> pages;
  int64_t seen = 0;
  while (p < ce && seen < c.nval) {
    TR r{p, ce};
    Page pg;
    int16_t last = 0; int id, ty;
    while (r.field(&last, &id, &ty)) {
      if (id == 1) pg.pt = int(r.zz());
      else if (id == 2) pg.us = r.zz();
      else if (id == 3) pg.cs = r.zz();
      else if (id == 5 || id == 7 || id == 8) {
        int16_t l2 = 0; int i2, t2;
        while (r.field(&l2, &i2, &t2)) {
          if (i2 == 1) pg.nv = int(r.zz());
          else if ((id != 8 && i2 == 2) || (id == 8 && i2 == 4)) pg.enc = int(r.zz());
          else if (id == 8 && i2 == 5) pg.v2d = int(r.zz());
          else if (id == 8 && i2 == 6) pg.v2r = int(r.zz());
          else if (id == 8 && i2 == 7) pg.v2c = t2 == 1;
          else r.skip(t2);
        }
      } else r.skip(ty);
    }
    pg.body = r.p;
    p = pg.body + pg.cs;
    if (pg.pt != 0 && pg.pt != 2 && pg.pt != 3) continue;
    if (pg.pt != 2) seen += pg.nv;
    pages.push_back(pg);
  }
  return pages;
}

// Decompressed body of a page (v2 levels are stored uncompressed ahead of the values).
std::vector<uint8_t> page_bytes(const Chunk& c, const Page& pg) {
  const int64_t lv = pg.pt == 3 ? pg.v2d + pg.v2r : 0;
  std::vector<uint8_t> buf(size_t(pg.us) + 16, 0);
  memcpy(buf.data(), pg.body, size_t(lv));
  const bool comp = c.codec == 1 && !(pg.pt == 3 && !pg.v2c);
  if (comp) { if (!snappy(pg.body + lv, size_t(pg.cs - lv), buf.data() + lv, size_t(pg.us - lv))) die("snappy"); }
  else if (c.codec == 0) memcpy(buf.data() + lv, pg.body + lv, size_t(pg.us - lv));
  else die("codec");
  return buf;
}

// PLAIN values of a leaf (BYTE_ARRAY, INT64, INT32).
void plain_values(const Leaf& l, const uint8_t*& q, int64_t n, std::vector<SV>* S, std::vector<int64_t>* I) {
  for (int64_t k = 0; k < n; ++k) {
    if (l.type == 6) { uint32_t len = rd32(q); q += 4; S->push_back(SV{(const char*)q, len}); q += len; }
    else if (l.type == 2) { I->push_back(int64_t(rd64(q))); q += 8; }
    else if (l.type == 1) { I->push_back(int32_t(rd32(q))); q += 4; }
    else die("type");
  }
}

// One data page -> def level and value per row.
void decode_data_page(const Chunk& c, const Leaf& l, const Page& pg, const std::vector<SV>& ds,
                      const std::vector<int64_t>& di, Col& out) {
  out.bufs.push_back(page_bytes(c, pg));
  const std::vector<uint8_t>& buf = out.bufs.back();
  const uint8_t* q = buf.data();
  const uint8_t* qe = q + pg.us;
  const int64_t lv = pg.pt == 3 ? pg.v2d + pg.v2r : 0;
  std::vector<uint32_t> defs;
  if (pg.pt == 3) { if (l.maxdef) rle(q + pg.v2r, q + lv, bwidth(l.maxdef), pg.nv, defs); q += lv; }
  else if (l.maxdef) { uint32_t n = rd32(q); q += 4; rle(q, q + n, bwidth(l.maxdef), pg.nv, defs); q += n; }
  int64_t nn = 0;
  for (int k = 0; k < pg.nv; ++k) nn += (l.maxdef ? int(defs[k]) : 0) == l.maxdef;
  std::vector<SV> S; std::vector<int64_t> I;
  if (pg.enc == 0) plain_values(l, q, nn, &S, &I);
  else if (pg.enc == 2 || pg.enc == 8) {
    std::vector<uint32_t> ix;
    if (nn) { int w = *q++; rle(q, qe, w, nn, ix); }
    for (uint32_t x : ix) { if (l.type == 6) S.push_back(ds.at(x)); else I.push_back(di.at(x)); }
  } else die("encoding");
  size_t vi = 0;
  for (int k = 0; k < pg.nv; ++k) {
    uint8_t d = uint8_t(l.maxdef ? defs[k] : 0);
    out.def.push_back(d);
    if (d == l.maxdef) { if (l.type == 6) out.s.push_back(S[vi++]); else out.i.push_back(I[vi++]); }
    else { if (l.type == 6) out.s.push_back(SV{}); else out.i.push_back(0); }
  }
}

// A column chunk's pages decoded by `threads` workers (pages are independent once the dictionary
// page is read), concatenated in page order.
void decode_chunk(const uint8_t* f, const Chunk& c, const Leaf& l, int threads, Col& out) {
  const std::vector<Page> pages = chunk_pages(f, c);
  std::vector<SV> ds;
  std::vector<int64_t> di;
  std::vector<const Page*> data;
  for (const Page& pg : pages) {
    if (pg.pt == 2) {
      if (!data.empty()) die("dictionary page after data pages");
      ds.clear(); di.clear();
      out.bufs.push_back(page_bytes(c, pg));
      const uint8_t* q = out.bufs.back().data();
      plain_values(l, q, pg.nv, &ds, &di);
    } else {
      data.push_back(&pg);
    }
  }
  std::vector<Col> parts(data.size());
  std::atomic<size_t> next{0};
  auto work = [&] {
    for (size_t k; (k = next++) < data.size();) decode_data_page(c, l, *data[k], ds, di, parts[k]);
  };
  std::vector<std::thread> ts;
  for (int t = 1; t < threads && size_t(t) < data.size(); ++t) ts.emplace_back(work);
  work();
  for (auto& t : ts) t.join();
  for (Col& pc : parts) {
    out.def.insert(out.def.end(), pc.def.begin(), pc.def.end());
    out.s.insert(out.s.end(), pc.s.begin(), pc.s.end());
    out.i.insert(out.i.end(), pc.i.begin(), pc.i.end());
    for (auto& b : pc.bufs) out.bufs.push_back(std::move(b));
  }
}

// Decoded hot columns of every checkpoint row group, kept alive while actions point into them.
std::vector<std::array<Col, 4>> g_ck_cols;

void read_checkpoint(const std::vector<uint8_t>& f, std::vector<Action>& acts, int threads) {
  const size_t n = f.size();
  uint32_t fl = rd32(f.data() + n - 8);
  TR r{f.data() + n - 8 - fl, f.data() + n - 8};
  std::vector<SchemaEl> sch;
  std::vector<RG> rgs;
  int16_t last = 0; int id, ty;
  while (r.field(&last, &id, &ty)) {
    if (id == 2) {
      int et; uint64_t c = r.list(&et);
      for (uint64_t i = 0; i < c; ++i) {
        SchemaEl e; int16_t l2 = 0; int i2, t2;
        while (r.field(&l2, &i2, &t2)) {
          if (i2 == 1) e.type = int(r.zz()); else if (i2 == 3) e.rep = int(r.zz());
          else if (i2 == 4) e.name = r.bin(); else if (i2 == 5) e.nch = int(r.zz()); else r.skip(t2);
        }
        sch.push_back(e);
      }
    } else if (id == 4) {
      int et; uint64_t c = r.list(&et);
      for (uint64_t i = 0; i < c; ++i) {
        RG g; int16_t l2 = 0; int i2, t2;
        while (r.field(&l2, &i2, &t2)) {
          if (i2 == 1) {
            int e3; uint64_t nc = r.list(&e3);
            for (uint64_t k = 0; k < nc; ++k) {
              Chunk ck; int16_t l3 = 0; int i3, t3;
              while (r.field(&l3, &i3, &t3)) {
                if (i3 == 3) {
                  int16_t l4 = 0; int i4, t4;
                  while (r.field(&l4, &i4, &t4)) {
                    if (i4 == 1) ck.type = int(r.zz());
                    else if (i4 == 3) { int e5; uint64_t np = r.list(&e5); for (uint64_t q = 0; q < np; ++q) { if (q) ck.path += "."; ck.path += r.bin(); } }
                    else if (i4 == 4) ck.codec = int(r.zz()); else if (i4 == 5) ck.nval = r.zz();
                    else if (i4 == 7) ck.tcomp = r.zz(); else if (i4 == 9) ck.dpo = r.zz();
                    else if (i4 == 11) ck.dicto = r.zz(); else r.skip(t4);
                  }
                } else r.skip(t3);
              }
              g.cols.push_back(ck);
            }
          } else if (i2 == 3) g.rows = r.zz(); else r.skip(t2);
        }
        rgs.push_back(g);
      }
    } else r.skip(ty);
  }
  // leaves
  std::map<std::string, Leaf> leaves;
  size_t idx = 1;
  std::function<void(std::string, int, int, std::vector<int>, int)> rec = [&](std::string pre, int d, int rp, std::vector<int> dof, int nch) {
    for (int c = 0; c < nch; ++c) {
      const SchemaEl& e = sch[idx++];
      std::string path = pre.empty() ? e.name : pre + "." + e.name;
      int d2 = d + (e.rep >= 1), r2 = rp + (e.rep == 2);
      auto dof2 = dof; dof2.push_back(d2);
      if (e.nch) rec(path, d2, r2, dof2, e.nch); else leaves[path] = Leaf{path, e.type, d2, r2, dof2};
    }
  };
  rec("", 0, 0, {}, sch[0].nch);
  const char* names[4] = {"add.path", "add.size", "remove.path", "remove.deletionTimestamp"};
  int64_t rbase = 0;
  std::vector<std::pair<const RG*, int64_t>> groups;
  for (auto& g : rgs) { groups.push_back({&g, rbase}); rbase += g.rows; }
  size_t base_act = acts.size();
  acts.resize(base_act + size_t(rbase));
  // decode: one task per (row group, hot column), so a table with few row groups still uses every
  // thread; then one task per row group assembles its rows (unwrap: add > remove > the rest)
  const size_t col0 = g_ck_cols.size();
  g_ck_cols.resize(col0 + groups.size());
  std::array<Col, 4>* cols = g_ck_cols.data() + col0;
  std::vector<std::array<bool, 4>> has(groups.size(), std::array<bool, 4>{false, false, false, false});
  std::atomic<size_t> next{0};
  auto decode = [&] {
    for (;;) {
      const size_t task = next++;
      if (task >= groups.size() * 4) return;
      const size_t gi = task / 4;
      const int k = int(task % 4);
      const RG& g = *groups[gi].first;
      auto it = leaves.find(names[k]);
      if (it == leaves.end()) continue;
      for (auto& c : g.cols)
        if (c.path == names[k]) { decode_chunk(f.data(), c, it->second, threads, cols[gi][size_t(k)]); has[gi][size_t(k)] = true; }
    }
  };
  const Leaf* la = leaves.count("add.path") ? &leaves["add.path"] : nullptr;
  const Leaf* lr = leaves.count("remove.path") ? &leaves["remove.path"] : nullptr;
  const int add_size_def = leaves.count("add.size") ? leaves["add.size"].maxdef : 0;
  const int rm_ts_def = leaves.count("remove.deletionTimestamp") ? leaves["remove.deletionTimestamp"].maxdef : 0;
  std::atomic<size_t> next_g{0};
  auto assemble = [&] {
    for (;;) {
      const size_t gi = next_g++;
      if (gi >= groups.size()) return;
      const RG& g = *groups[gi].first;
      auto& cs = cols[gi];
      const auto& h = has[gi];
      for (int64_t i = 0; i < g.rows; ++i) {
        Action& a = acts[base_act + size_t(groups[gi].second + i)];
        if (h[0] && cs[0].def[i] >= la->def_of[0]) {
          a.kind = ADD; a.path = cs[0].s[i];
          if (h[1] && cs[1].def[i] == add_size_def) a.size = cs[1].i[i];
        } else if (h[2] && cs[2].def[i] >= lr->def_of[0]) {
          a.kind = REMOVE; a.path = cs[2].s[i];
          if (h[3] && cs[3].def[i] == rm_ts_def) { a.has_delts = true; a.delts = cs[3].i[i]; }
        } else {
          a.kind = OTHER;  // protocol/metaData/txn rows: counted, not keyed
        }
      }
    }
  };
  auto tq0 = std::chrono::steady_clock::now();
  {
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t) ts.emplace_back(decode);
    for (auto& t : ts) t.join();
  }
  if (getenv("ORACLE_TIMING")) fprintf(stderr, "  decode %.3fs\n", std::chrono::duration<double>(std::chrono::steady_clock::now() - tq0).count());
  {
    std::vector<std::thread> ts;
    for (int t = 0; t < threads; ++t) ts.emplace_back(assemble);
    for (auto& t : ts) t.join();
  }
}

// ---- listing (D/SnapshotManagement.scala:82-179) -----------------------------------------------
bool digits(const std::string& s) { return !s.empty() && std::all_of(s.begin(), s.end(), ::isdigit); }

struct Seg { int64_t ckv = -1; std::vector<std::string> ckpt, deltas; };
Seg segment(const std::string& log) {
  DIR* d = opendir(log.c_str());
  if (!d) die("no log dir");
  std::vector<std::string> names;
  while (dirent* e = readdir(d)) names.push_back(e->d_name);
  closedir(d);
  std::sort(names.begin(), names.end());
  std::map<std::pair<int64_t, int>, std::vector<std::string>> cks;
  std::map<int64_t, std::string> js;
  for (auto& n : names) {
    auto dot = n.find('.');
    if (dot == std::string::npos || !digits(n.substr(0, dot))) continue;
    int64_t v = std::stoll(n.substr(0, dot));
    std::string rest = n.substr(dot);
    if (rest == ".json") js[v] = n;
    else if (rest == ".checkpoint.parquet") cks[{v, 0}].push_back(n);
    else if (rest.rfind(".checkpoint.", 0) == 0 && rest.size() > 8 && rest.substr(rest.size() - 8) == ".parquet") {
      std::string mid = rest.substr(12, rest.size() - 20);
      auto d2 = mid.find('.');
      if (d2 != std::string::npos) cks[{v, std::stoi(mid.substr(d2 + 1))}].push_back(n);
    }
  }
  Seg s;
  for (auto it = cks.rbegin(); it != cks.rend(); ++it) {
    int parts = it->first.second;
    if ((parts == 0 && it->second.size() == 1) || (parts > 0 && int(it->second.size()) == parts)) {
      s.ckv = it->first.first; s.ckpt = it->second; break;
    }
  }
  for (auto& kv : js) if (kv.first > s.ckv) s.deltas.push_back(kv.second);
  return s;
}

// canonicalizePath (D/Snapshot.scala:317-328) restated for the local filesystem, and the URI-equality
// replay key (D/actions/actions.scala:208-213): an unqualified absolute path becomes file:// +
// its Hadoop-normalised form; "file:///x" and "file:/x" are one key.
void canonical_key(SV raw, Arena& ar, SV* canon, SV* key) {
  SV c = raw;
  if (raw.n && raw.p[0] == '/') {
    char* o = ar.take(size_t(raw.n) + 7);
    memcpy(o, "file://", 7);
    uint32_t w = 7;
    for (uint32_t k = 0; k < raw.n; ++k) {
      if (raw.p[k] == '/' && w > 7 && o[w - 1] == '/') continue;
      o[w++] = raw.p[k];
    }
    if (w > 8 && o[w - 1] == '/') --w;
    c = SV{o, w};
  }
  *canon = c;
  if (c.n >= 8 && !memcmp(c.p, "file:///", 8)) {
    char* o = ar.take(c.n - 2);
    memcpy(o, "file:/", 6);
    memcpy(o + 6, c.p + 8, c.n - 8);
    *key = SV{o, c.n - 2};
  } else {
    *key = c;
  }
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) { fprintf(stderr, "usage: replay_oracle <_delta_log> <cutoff> [--threads T] [--partitions P]\n"); return 2; }
  std::string log = argv[1];
  int64_t cutoff = std::stoll(argv[2]);
  int threads = int(std::thread::hardware_concurrency());
  int parts = 50;
  for (int i = 3; i + 1 < argc; i += 2) {
    if (!strcmp(argv[i], "--threads")) threads = std::max(1, atoi(argv[i + 1]));
    else if (!strcmp(argv[i], "--partitions")) parts = std::max(1, atoi(argv[i + 1]));
  }
  try {
    // the segment's bytes are read before the clock starts (the GPU's timed region, too, starts
    // with its inputs resident)
    auto tr = std::chrono::steady_clock::now();
    Seg seg = segment(log);
    std::sort(seg.ckpt.begin(), seg.ckpt.end());
    std::vector<std::vector<uint8_t>> ckfiles, jfiles;
    for (auto& c : seg.ckpt) ckfiles.push_back(read_all(log + "/" + c));
    for (auto& d : seg.deltas) jfiles.push_back(read_all(log + "/" + d));
    const double read_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - tr).count();
    auto t0 = std::chrono::steady_clock::now();
    std::vector<Action> acts;
    int64_t ck_rows = 0;
    for (auto& f : ckfiles) {
      const size_t before = acts.size();
      read_checkpoint(f, acts, threads);
      ck_rows += int64_t(acts.size() - before);
    }
    // JSON: all lines of all deltas, parsed by `threads` workers over line ranges
    std::vector<std::pair<const char*, const char*>> lines;
    for (auto& f : jfiles) {
      const char* p = (const char*)f.data();
      const char* e = p + f.size();
      while (p < e) {
        const char* nl = (const char*)memchr(p, '\n', size_t(e - p));
        if (!nl) nl = e;
        lines.push_back({p, nl});
        p = nl + 1;
      }
    }
    std::vector<Arena> arenas(static_cast<size_t>(threads));
    const size_t base = acts.size();
    acts.resize(base + lines.size());
    {
      std::vector<std::thread> ts;
      const size_t per = (lines.size() + size_t(threads) - 1) / size_t(threads);
      for (int t = 0; t < threads; ++t)
        ts.emplace_back([&, t] {
          const size_t b = size_t(t) * per, e = std::min(lines.size(), b + per);
          for (size_t i = b; i < e; ++i) acts[base + i] = parse_line(lines[i].first, lines[i].second, &arenas[size_t(t)]);
        });
      for (auto& t : ts) t.join();
    }
    auto t1 = std::chrono::steady_clock::now();
    // canonical path, URI key and its xxh64 per file action
    const size_t N = acts.size();
    std::vector<SV> canon(N), key(N);
    std::vector<uint64_t> hash(N, 0);
    {
      std::vector<std::thread> ts;
      const size_t per = (N + size_t(threads) - 1) / size_t(threads);
      for (int t = 0; t < threads; ++t)
        ts.emplace_back([&, t] {
          const size_t b = size_t(t) * per, e = std::min(N, b + per);
          for (size_t i = b; i < e; ++i)
            if ((acts[i].kind == ADD || acts[i].kind == REMOVE) && acts[i].path.p) {
              canonical_key(acts[i].path, arenas[size_t(t)], &canon[i], &key[i]);
              hash[i] = xxh64((const uint8_t*)key[i].p, key[i].n);
            }
        });
      for (auto& t : ts) t.join();
    }
    // repartition(P, coalesce(add.path, remove.path)) + sortWithinPartitions("file"): a stable
    // counting sort by partition (each thread's contiguous range, ranges concatenated in order)
    const size_t P = size_t(parts), T = size_t(threads);
    std::vector<uint64_t> cnt(T * P, 0);
    const size_t per = (N + T - 1) / T;
    auto part_of = [&](size_t i) { return size_t((hash[i] >> 32) % P); };
    {
      std::vector<std::thread> ts;
      for (size_t t = 0; t < T; ++t)
        ts.emplace_back([&, t] {
          const size_t b = t * per, e = std::min(N, b + per);
          for (size_t i = b; i < e; ++i) if (hash[i]) ++cnt[t * P + part_of(i)];
        });
      for (auto& t : ts) t.join();
    }
    std::vector<uint64_t> off(T * P + 1, 0), pstart(P + 1, 0);
    {
      uint64_t acc = 0;
      for (size_t q = 0; q < P; ++q) {
        pstart[q] = acc;
        for (size_t t = 0; t < T; ++t) { off[t * P + q] = acc; acc += cnt[t * P + q]; }
      }
      pstart[P] = acc;
    }
    std::vector<uint32_t> order(pstart[P]);
    {
      std::vector<std::thread> ts;
      for (size_t t = 0; t < T; ++t)
        ts.emplace_back([&, t] {
          const size_t b = t * per, e = std::min(N, b + per);
          std::vector<uint64_t> cur(off.begin() + long(t * P), off.begin() + long(t * P + P));
          for (size_t i = b; i < e; ++i) if (hash[i]) order[cur[part_of(i)]++] = uint32_t(i);
        });
      for (auto& t : ts) t.join();
    }
    // InMemoryLogReplay per partition: one open-addressing table keyed by the URI key (hash, then
    // bytes) holding the last action; an add makes the path live, a remove a tombstone
    // (activeFiles / tombstones with the opposite entry dropped, D/actions/InMemoryLogReplay.scala:54-63)
    struct PartOut { int64_t files = 0, size = 0, tombs = 0; uint64_t lks = 0, tks = 0; };
    std::vector<PartOut> po(P);
    std::atomic<size_t> nextp{0};
    {
      std::vector<std::thread> ts;
      for (size_t t = 0; t < T; ++t)
        ts.emplace_back([&] {
          std::vector<uint32_t> slot;
          std::vector<std::pair<SV, uint32_t>> out;
          for (;;) {
            const size_t q = nextp++;
            if (q >= P) return;
            const uint64_t n = pstart[q + 1] - pstart[q];
            size_t cap = 16;
            while (cap < 2 * n) cap <<= 1;
            slot.assign(cap, 0xFFFFFFFFu);
            for (uint64_t k = pstart[q]; k < pstart[q + 1]; ++k) {
              const uint32_t i = order[k];
              size_t h = size_t(hash[i]) & (cap - 1);
              for (;;) {
                const uint32_t j = slot[h];
                if (j == 0xFFFFFFFFu) { slot[h] = i; break; }
                if (hash[j] == hash[i] && key[j].n == key[i].n && !memcmp(key[j].p, key[i].p, key[i].n)) {
                  slot[h] = i;  // last writer wins
                  break;
                }
                h = (h + 1) & (cap - 1);
              }
            }
            out.clear();
            PartOut& o = po[q];
            for (uint32_t i : slot) {
              if (i == 0xFFFFFFFFu) continue;
              const Action& a = acts[i];
              if (a.kind == ADD) {
                out.push_back({canon[i], i});
                o.files++; o.size += a.size; o.lks += hash[i] >> 32;
              } else if ((a.has_delts ? a.delts : 0) > cutoff) {  // getTombstones: delTimestamp > cutoff
                out.push_back({canon[i], i});
                o.tombs++; o.tks += hash[i] >> 32;
              }
            }
            std::sort(out.begin(), out.end(), [](const std::pair<SV, uint32_t>& x, const std::pair<SV, uint32_t>& y) {
              return x.first < y.first;
            });  // checkpoint(): sortBy(_.path)
          }
        });
      for (auto& t : ts) t.join();
    }
    auto t2 = std::chrono::steady_clock::now();
    PartOut tot;
    for (auto& o : po) { tot.files += o.files; tot.size += o.size; tot.tombs += o.tombs; tot.lks += o.lks; tot.tks += o.tks; }
    const int64_t nfa = int64_t(pstart[P]);
    double ps = std::chrono::duration<double>(t1 - t0).count(), rs = std::chrono::duration<double>(t2 - t1).count();
    printf("{\"num_files\":%lld,\"size_in_bytes\":%lld,\"num_removes\":%lld,\"num_actions\":%lld,"
           "\"num_file_actions\":%lld,\"checkpoint_rows\":%lld,\"live_key_sum\":%llu,\"tomb_key_sum\":%llu,"
           "\"threads\":%d,\"partitions\":%d,\"read_s\":%.6f,\"parse_s\":%.6f,\"replay_s\":%.6f,\"total_s\":%.6f}\n",
           (long long)tot.files, (long long)tot.size, (long long)tot.tombs, (long long)acts.size(), (long long)nfa,
           (long long)ck_rows, (unsigned long long)tot.lks, (unsigned long long)tot.tks, threads, parts, read_s, ps, rs,
           ps + rs);
  } catch (const std::exception& e) {
    fprintf(stderr, "replay_oracle: %s\n", e.what());
    return 1;
  }
  return 0;
}
