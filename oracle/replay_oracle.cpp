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

// Each checkpoint file's footer (row groups, leaves) and its first action index, for the
// full-record pass (--record-sums).
struct CkFile { const std::vector<uint8_t>* f; std::vector<RG> rgs; std::map<std::string, Leaf> leaves; size_t base_act; };
std::vector<CkFile> g_ck_files;

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
  g_ck_files.push_back(CkFile{&f, rgs, leaves, base_act});
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

// ---- full-record checksums (--record-sums; definition in oracle/delta_oracle.py:record_hash) -----
uint64_t xxh64s(const uint8_t* p, size_t len, uint64_t seed) {
  const uint8_t* end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
    do {
      v1 = xround(v1, rd64(p)); v2 = xround(v2, rd64(p + 8)); v3 = xround(v3, rd64(p + 16)); v4 = xround(v4, rd64(p + 24));
      p += 32;
    } while (p <= end - 32);
    h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    for (uint64_t v : {v1, v2, v3, v4}) { h ^= xround(0, v); h = h * P1 + P4; }
  } else {
    h = seed + P5;
  }
  h += len;
  while (p + 8 <= end) { h ^= xround(0, rd64(p)); h = rotl(h, 27) * P1 + P4; p += 8; }
  if (p + 4 <= end) { h ^= uint64_t(rd32(p)) * P1; h = rotl(h, 23) * P2 + P3; p += 4; }
  while (p < end) { h ^= uint64_t(*p) * P5; h = rotl(h, 11) * P1; ++p; }
  h ^= h >> 33; h *= P2; h ^= h >> 29; h *= P3; h ^= h >> 32;
  return h;
}
uint64_t xxh64sv(SV s, uint64_t seed) { return xxh64s((const uint8_t*)s.p, s.n, seed); }

const uint64_t kRecSeed = 0x5EED, kGold = 0x9E3779B97F4A7C15ull, kNullV = 0x5BD1E9955BD1E995ull;

// A map value: entries in first-position order, a repeated key keeps its last value (Jackson into a
// Map, as the Python dict).
struct MapV {
  bool null = true;
  std::vector<std::pair<SV, std::pair<bool, SV>>> e;  // key -> (value null, value)
  void put(SV k, bool vnull, SV v) {
    for (auto& x : e) if (x.first.n == k.n && !memcmp(x.first.p, k.p, k.n)) { x.second = {vnull, v}; return; }
    e.push_back({k, {vnull, v}});
  }
  uint64_t hash(uint64_t ks, uint64_t vs) const {
    if (null) return 0;
    uint64_t h = 1 + e.size();
    for (auto& x : e) h += xxh64sv(x.first, ks) * kGold + (x.second.first ? kNullV : xxh64sv(x.second.second, vs));
    return h;
  }
};

struct Rec {
  SV path;
  int64_t size = 0, mtime = 0, delts = 0;
  bool has_delts = false, efm = false, stats_null = true;
  SV stats;
  MapV pv, tags;
};

uint64_t rec_hash(const Rec& r, int side) {
  uint64_t w[8];
  w[0] = uint64_t(side);
  w[1] = xxh64sv(r.path, 0);
  w[2] = uint64_t(r.size);
  if (side == 0) { w[3] = uint64_t(r.mtime); w[4] = 0; w[5] = r.stats_null ? 0 : xxh64sv(r.stats, 1); }
  else { w[3] = r.has_delts ? uint64_t(r.delts) : 0; w[4] = (r.has_delts ? 1u : 0u) | (r.efm ? 2u : 0u); w[5] = 0; }
  w[6] = r.pv.hash(2, 3);
  w[7] = r.tags.hash(4, 5);
  static const uint32_t field_mask = [] {  // diagnostics: DR_RECORD_FIELDS keeps these words (as the device)
    const char* m = getenv("DR_RECORD_FIELDS");
    return m ? uint32_t(strtoul(m, nullptr, 0)) : 0xffu;
  }();
  for (int k = 0; k < 8; ++k) if (!((field_mask >> k) & 1u)) w[k] = 0;
  uint8_t b[64];
  memcpy(b, w, 64);  // little-endian host
  return xxh64s(b, 64, kRecSeed);
}

// {"k": "v" | null, ...} -> map (null literal -> null map)
bool parse_map(J& j, MapV& m) {
  if (j.null()) { m = MapV(); return true; }
  m = MapV();
  m.null = false;
  j.ws();
  if (!j.lit("{")) return false;
  j.ws();
  if (j.p < j.e && *j.p == '}') { ++j.p; return true; }
  for (;;) {
    SV k, v;
    if (!j.str(&k)) return false;
    j.ws();
    if (!j.lit(":")) return false;
    if (j.null()) m.put(k, true, SV{});
    else { if (!j.str(&v)) return false; m.put(k, false, v); }
    j.ws();
    if (j.p < j.e && *j.p == ',') { ++j.p; continue; }
    if (j.p < j.e && *j.p == '}') { ++j.p; return true; }
    return false;
  }
}

bool parse_bool(J& j, bool* b) {
  j.ws();
  if (j.e - j.p >= 4 && !memcmp(j.p, "true", 4)) { j.p += 4; *b = true; return true; }
  if (j.e - j.p >= 5 && !memcmp(j.p, "false", 5)) { j.p += 5; *b = false; return true; }
  return false;
}

// The whole add / remove object of a survivor line (Jackson defaults: absent primitives 0/false,
// absent Options / maps null; a repeated member keeps its last value).
bool parse_record_obj(J& j, Rec& r) {
  j.ws();
  if (!j.lit("{")) return false;
  j.ws();
  if (j.p < j.e && *j.p == '}') { ++j.p; return true; }
  for (;;) {
    SV k;
    if (!j.str(&k)) return false;
    j.ws();
    if (!j.lit(":")) return false;
    if (k.eq("path", 4)) { if (!j.null() && !j.str(&r.path)) return false; }
    else if (k.eq("size", 4)) { if (j.null()) r.size = 0; else if (!j.i64(&r.size)) return false; }
    else if (k.eq("modificationTime", 16)) { if (j.null()) r.mtime = 0; else if (!j.i64(&r.mtime)) return false; }
    else if (k.eq("deletionTimestamp", 17)) { if (j.null()) r.has_delts = false; else { if (!j.i64(&r.delts)) return false; r.has_delts = true; } }
    else if (k.eq("extendedFileMetadata", 20)) { if (j.null()) r.efm = false; else if (!parse_bool(j, &r.efm)) return false; }
    else if (k.eq("stats", 5)) { if (j.null()) r.stats_null = true; else { if (!j.str(&r.stats)) return false; r.stats_null = false; } }
    else if (k.eq("partitionValues", 15)) { if (!parse_map(j, r.pv)) return false; }
    else if (k.eq("tags", 4)) { if (!parse_map(j, r.tags)) return false; }
    else { j.skip(); if (j.bad) return false; }
    j.ws();
    if (j.p < j.e && *j.p == ',') { ++j.p; continue; }
    if (j.p < j.e && *j.p == '}') { ++j.p; return true; }
    return false;
  }
}

// The survivor record of a JSON line: the object of its side ("add" / "remove"; the last such member).
bool json_record(const char* b, const char* e, int side, Arena* ar, Rec& r) {
  J j{b, e, ar};
  const char* want = side == 0 ? "add" : "remove";
  const size_t wn = side == 0 ? 3 : 6;
  j.ws();
  if (!j.lit("{")) return false;
  bool found = false;
  for (;;) {
    SV k;
    if (!j.str(&k)) return false;
    j.ws();
    if (!j.lit(":")) return false;
    if (k.eq(want, wn) && !j.null()) { r = Rec(); if (!parse_record_obj(j, r)) return false; found = true; }
    else { j.skip(); if (j.bad) return false; }
    j.ws();
    if (j.p < j.e && *j.p == ',') { ++j.p; continue; }
    if (j.p < j.e && *j.p == '}') break;
    return false;
  }
  return found;
}

// A column chunk decoded with its repetition and definition levels (one entry per level; values at
// entries with def == maxdef). PLAIN / dictionary BYTE_ARRAY, INT64, INT32 and PLAIN BOOLEAN.
struct LevCol {
  std::vector<uint8_t> def, rep;
  std::vector<SV> s;
  std::vector<int64_t> i;
  std::vector<std::vector<uint8_t>> bufs;
};

void level_chunk(const uint8_t* f, const Chunk& c, const Leaf& l, LevCol& out) {
  std::vector<SV> ds;
  std::vector<int64_t> di;
  for (const Page& pg : chunk_pages(f, c)) {
    out.bufs.push_back(page_bytes(c, pg));
    const uint8_t* q = out.bufs.back().data();
    if (pg.pt == 2) {
      ds.clear(); di.clear();
      plain_values(l, q, pg.nv, &ds, &di);
      continue;
    }
    const uint8_t* qe = q + pg.us;
    std::vector<uint32_t> reps, defs;
    if (pg.pt == 3) {
      if (l.maxrep) rle(q, q + pg.v2r, bwidth(l.maxrep), pg.nv, reps);
      if (l.maxdef) rle(q + pg.v2r, q + pg.v2r + pg.v2d, bwidth(l.maxdef), pg.nv, defs);
      q += pg.v2r + pg.v2d;
    } else {
      if (l.maxrep) { uint32_t n = rd32(q); q += 4; rle(q, q + n, bwidth(l.maxrep), pg.nv, reps); q += n; }
      if (l.maxdef) { uint32_t n = rd32(q); q += 4; rle(q, q + n, bwidth(l.maxdef), pg.nv, defs); q += n; }
    }
    int64_t nn = 0;
    for (int k = 0; k < pg.nv; ++k) nn += (l.maxdef ? int(defs[size_t(k)]) : 0) == l.maxdef;
    std::vector<SV> S; std::vector<int64_t> I;
    if (pg.enc == 0 && l.type == 0) {
      for (int64_t k = 0; k < nn; ++k) I.push_back((q[k >> 3] >> (k & 7)) & 1);
    } else if (pg.enc == 0) {
      plain_values(l, q, nn, &S, &I);
    } else if (pg.enc == 2 || pg.enc == 8) {
      std::vector<uint32_t> ix;
      if (nn) { int w = *q++; rle(q, qe, w, nn, ix); }
      for (uint32_t x : ix) { if (l.type == 6) S.push_back(ds.at(x)); else I.push_back(di.at(x)); }
    } else die("encoding");
    size_t vi = 0;
    for (int k = 0; k < pg.nv; ++k) {
      const uint8_t d = uint8_t(l.maxdef ? defs[size_t(k)] : 0);
      out.def.push_back(d);
      out.rep.push_back(uint8_t(l.maxrep ? reps[size_t(k)] : 0));
      if (d == l.maxdef) { if (l.type == 6) out.s.push_back(S[vi++]); else out.i.push_back(I[vi++]); }
      else { if (l.type == 6) out.s.push_back(SV{}); else out.i.push_back(0); }
    }
  }
}

// Level entry ranges of the rows of a leaf (rows start where rep == 0).
std::vector<size_t> row_starts(const LevCol& c) {
  std::vector<size_t> st;
  for (size_t k = 0; k < c.def.size(); ++k) if (c.rep[k] == 0) st.push_back(k);
  st.push_back(c.def.size());
  return st;
}

// Full-record sums of the checkpoint survivors of one row group: `surv[row]` 1 = live add,
// 2 = kept tombstone.
void ck_rowgroup_sums(const CkFile& cf, const RG& g, const SV* canon, const uint8_t* surv, uint64_t* sums,
                      uint64_t* hashes) {
  bool want[2] = {false, false};
  for (int64_t r = 0; r < g.rows; ++r) if (surv[r]) want[surv[r] - 1] = true;
  for (int side = 0; side < 2; ++side) {
    if (!want[side]) continue;
    const std::string pre = side == 0 ? "add." : "remove.";
    struct L { const Leaf* leaf = nullptr; LevCol col; std::vector<size_t> st; };
    auto load = [&](const std::string& name) {
      auto out = std::make_unique<L>();
      auto it = cf.leaves.find(pre + name);
      if (it == cf.leaves.end()) return out;
      for (const Chunk& c : g.cols)
        if (c.path == pre + name) { out->leaf = &it->second; level_chunk(cf.f->data(), c, it->second, out->col); }
      if (out->leaf) out->st = row_starts(out->col);
      return out;
    };
    auto size = load("size"), mt = load("modificationTime"), dts = load("deletionTimestamp"),
         efm = load("extendedFileMetadata"), stats = load("stats"), pvk = load("partitionValues.key_value.key"),
         pvv = load("partitionValues.key_value.value"), tk = load("tags.key_value.key"), tv = load("tags.key_value.value");
    auto flat_i = [&](const L& l, int64_t r, int64_t* v) {
      if (!l.leaf) return false;
      const size_t k = l.st[size_t(r)];
      if (l.col.def[k] != l.leaf->maxdef) return false;
      *v = l.col.i[k];
      return true;
    };
    auto map_of = [&](const L& k, const L& v, int64_t r, MapV& m) {
      m = MapV();
      if (!k.leaf) return;
      const size_t a = k.st[size_t(r)], b = k.st[size_t(r) + 1];
      if (k.col.def[a] < k.leaf->def_of[size_t(k.leaf->def_of.size()) - 3]) return;  // the map itself is null
      m.null = false;
      if (k.col.def[a] < k.leaf->maxdef) return;  // empty map
      for (size_t e = a; e < b; ++e) {
        const bool vnull = !v.leaf || v.col.def[e] != v.leaf->maxdef;
        m.put(k.col.s[e], vnull, vnull ? SV{} : v.col.s[e]);
      }
    };
    for (int64_t r = 0; r < g.rows; ++r) {
      if (surv[r] != side + 1) continue;
      Rec rec;
      rec.path = canon[r];  // canonical form of the path leaf's value
      int64_t x;
      if (flat_i(*size, r, &x)) rec.size = x;
      if (side == 0) {
        if (flat_i(*mt, r, &x)) rec.mtime = x;
        if (stats->leaf && stats->col.def[stats->st[size_t(r)]] == stats->leaf->maxdef) {
          rec.stats_null = false;
          rec.stats = stats->col.s[stats->st[size_t(r)]];
        }
      } else {
        if (flat_i(*dts, r, &x)) { rec.has_delts = true; rec.delts = x; }
        if (flat_i(*efm, r, &x)) rec.efm = x != 0;
      }
      map_of(*pvk, *pvv, r, rec.pv);
      map_of(*tk, *tv, r, rec.tags);
      const uint64_t h = rec_hash(rec, side);
      sums[side] += h;
      if (hashes) hashes[r] = h;
    }
  }
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) { fprintf(stderr, "usage: replay_oracle <_delta_log> <cutoff> [--threads T] [--partitions P]\n"); return 2; }
  std::string log = argv[1];
  int64_t cutoff = std::stoll(argv[2]);
  int threads = int(std::thread::hardware_concurrency());
  int parts = 50;
  bool want_records = false;
  std::string hash_prefix;  // --record-hashes <prefix>: every survivor's record hash, <prefix>.live / .tomb
  for (int i = 3; i < argc; ++i) {
    if (!strcmp(argv[i], "--record-sums")) { want_records = true; continue; }
    if (i + 1 >= argc) break;
    if (!strcmp(argv[i], "--record-hashes")) { want_records = true; hash_prefix = argv[++i]; continue; }
    if (!strcmp(argv[i], "--threads")) threads = std::max(1, atoi(argv[++i]));
    else if (!strcmp(argv[i], "--partitions")) parts = std::max(1, atoi(argv[++i]));
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
    std::vector<uint8_t> surv(want_records ? N : 0, 0);  // 1 live add, 2 kept tombstone (--record-sums)
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
                if (want_records) surv[i] = 1;
              } else if ((a.has_delts ? a.delts : 0) > cutoff) {  // getTombstones: delTimestamp > cutoff
                out.push_back({canon[i], i});
                o.tombs++; o.tks += hash[i] >> 32;
                if (want_records) surv[i] = 2;
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
    // full-record checksums (untimed): JSON survivors re-read from their lines, checkpoint survivors
    // from every leaf of their side, one task per row group
    char recs[160] = "";
    if (want_records) {
      auto tr0 = std::chrono::steady_clock::now();
      std::vector<std::array<uint64_t, 2>> ts_sum(T, std::array<uint64_t, 2>{0, 0});
      std::vector<uint64_t> rh(hash_prefix.empty() ? 0 : N, 0);  // per action (survivors only)
      std::vector<uint8_t> bad(T, 0);
      {
        std::vector<std::thread> ts;
        const size_t nl = lines.size(), per_l = (nl + T - 1) / T;
        for (size_t t = 0; t < T; ++t)
          ts.emplace_back([&, t] {
            const size_t b = t * per_l, e = std::min(nl, b + per_l);
            for (size_t k = b; k < e; ++k) {
              const uint8_t sv = surv[base + k];
              if (!sv) continue;
              Rec r;
              if (!json_record(lines[k].first, lines[k].second, sv - 1, &arenas[t], r)) { bad[t] = 1; continue; }
              r.path = canon[base + k];  // the record's path is the canonical one (D/Snapshot.scala:98-101)
              const uint64_t h = rec_hash(r, sv - 1);
              ts_sum[t][sv - 1] += h;
              if (!rh.empty()) rh[base + k] = h;
            }
          });
        for (auto& t : ts) t.join();
      }
      {
        struct Task { const CkFile* cf; const RG* g; size_t row0; };
        std::vector<Task> tasks;
        for (const CkFile& cf : g_ck_files) {
          size_t r0 = cf.base_act;
          for (const RG& g : cf.rgs) { tasks.push_back({&cf, &g, r0}); r0 += size_t(g.rows); }
        }
        std::atomic<size_t> nt{0};
        std::vector<std::thread> ts;
        for (size_t t = 0; t < T; ++t)
          ts.emplace_back([&, t] {
            for (size_t k; (k = nt++) < tasks.size();) {
              uint64_t sm[2] = {0, 0};
              ck_rowgroup_sums(*tasks[k].cf, *tasks[k].g, canon.data() + tasks[k].row0, surv.data() + tasks[k].row0, sm,
                               rh.empty() ? nullptr : rh.data() + tasks[k].row0);
              ts_sum[t][0] += sm[0];
              ts_sum[t][1] += sm[1];
            }
          });
        for (auto& t : ts) t.join();
      }
      uint64_t ls = 0, tsm = 0;
      for (auto& x : ts_sum) { ls += x[0]; tsm += x[1]; }
      for (uint8_t b : bad) if (b) die("unreadable survivor line in the record pass");
      if (!rh.empty()) {  // the multisets of record hashes, for an exact comparison of sorted lists
        for (int side = 0; side < 2; ++side) {
          std::vector<uint64_t> v;
          for (size_t i = 0; i < N; ++i) if (surv[i] == side + 1) v.push_back(rh[i]);
          const std::string fn = hash_prefix + (side == 0 ? ".live" : ".tomb");
          FILE* f = fopen(fn.c_str(), "wb");
          if (!f || fwrite(v.data(), 8, v.size(), f) != v.size()) die("cannot write " + fn);
          fclose(f);
        }
      }
      snprintf(recs, sizeof recs, ",\"live_record_sum\":%llu,\"tomb_record_sum\":%llu,\"record_s\":%.3f",
               (unsigned long long)ls, (unsigned long long)tsm,
               std::chrono::duration<double>(std::chrono::steady_clock::now() - tr0).count());
    }
    printf("{\"num_files\":%lld,\"size_in_bytes\":%lld,\"num_removes\":%lld,\"num_actions\":%lld,"
           "\"num_file_actions\":%lld,\"checkpoint_rows\":%lld,\"live_key_sum\":%llu,\"tomb_key_sum\":%llu,"
           "\"threads\":%d,\"partitions\":%d,\"read_s\":%.6f,\"parse_s\":%.6f,\"replay_s\":%.6f,\"total_s\":%.6f%s}\n",
           (long long)tot.files, (long long)tot.size, (long long)tot.tombs, (long long)acts.size(), (long long)nfa,
           (long long)ck_rows, (unsigned long long)tot.lks, (unsigned long long)tot.tks, threads, parts, read_s, ps, rs,
           ps + rs, recs);
  } catch (const std::exception& e) {
    fprintf(stderr, "replay_oracle: %s\n", e.what());
    return 1;
  }
  return 0;
}
