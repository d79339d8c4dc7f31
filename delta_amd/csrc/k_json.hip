// K1: newline-delimited JSON commit files -> action records (replaces Spark's JsonFileFormat +
// Jackson over Action.logSchema, D/DeltaLogFileIndex.scala:67, D/Snapshot.scala:244-263).
//
// Stage 1 (k_json_count / k_json_newlines): a structural index of the newline bytes, built from
// 16-byte vector loads; a raw '\n' can never sit inside a JSON string, so every newline is a line
// boundary. Stage 2 (k_json_parse): one lane per line walks the line once through a 16-byte
// register window, classifies the SingleAction envelope with unwrap priority
// (D/actions/actions.scala:523-541), pulls add/remove path/size/deletionTimestamp and hashes the
// path (K3's xxh64) while its bytes are still in cache.
#include "dev_common.h"
#include "kernels.h"

namespace dr {
namespace dev {

constexpr int JSON_THREADS = 256;
constexpr int JSON_BYTES_PER_THREAD = 64;
constexpr int JSON_BYTES_PER_BLOCK = JSON_THREADS * JSON_BYTES_PER_THREAD;

__device__ __forceinline__ uint32_t count_nl_word(uint32_t w) {
  // bytes equal to 0x0a -> 0x80 in that byte lane
  const uint32_t x = w ^ 0x0a0a0a0au;
  const uint32_t t = (x - 0x01010101u) & ~x & 0x80808080u;
  return __builtin_popcount(t);
}

__global__ void __launch_bounds__(JSON_THREADS) k_json_count(const uint8_t* __restrict__ buf, uint64_t len,
                                                            uint32_t* __restrict__ block_counts) {
  __shared__ uint32_t red[JSON_THREADS / 64];
  const uint64_t base = uint64_t(blockIdx.x) * JSON_BYTES_PER_BLOCK + uint64_t(threadIdx.x) * JSON_BYTES_PER_THREAD;
  uint32_t c = 0;
  if (base + JSON_BYTES_PER_THREAD <= len) {
    const uint4* p = reinterpret_cast<const uint4*>(buf + base);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint4 v = p[i];
      c += count_nl_word(v.x) + count_nl_word(v.y) + count_nl_word(v.z) + count_nl_word(v.w);
    }
  } else {
    for (uint64_t i = base; i < len; ++i) c += buf[i] == '\n';
  }
  for (int o = 32; o > 0; o >>= 1) c += __shfl_down(c, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t s = 0;
    for (int i = 0; i < JSON_THREADS / 64; ++i) s += red[i];
    block_counts[blockIdx.x] = s;
  }
}

// Writes the byte position of every newline, in order: nl[block_off[b] + rank] = pos.
__global__ void __launch_bounds__(JSON_THREADS) k_json_newlines(const uint8_t* __restrict__ buf, uint64_t len,
                                                               const uint64_t* __restrict__ block_off,
                                                               uint64_t* __restrict__ nl) {
  __shared__ uint32_t wsum[JSON_THREADS / 64];
  const uint64_t base = uint64_t(blockIdx.x) * JSON_BYTES_PER_BLOCK + uint64_t(threadIdx.x) * JSON_BYTES_PER_THREAD;
  uint32_t words[16];
  uint32_t c = 0;
  const bool full = base + JSON_BYTES_PER_THREAD <= len;
  if (full) {
    const uint4* p = reinterpret_cast<const uint4*>(buf + base);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint4 v = p[i];
      words[4 * i] = v.x; words[4 * i + 1] = v.y; words[4 * i + 2] = v.z; words[4 * i + 3] = v.w;
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) c += count_nl_word(words[i]);
  } else {
    for (uint64_t i = base; i < len; ++i) c += buf[i] == '\n';
  }
  // block-wide exclusive scan of c
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t incl = c;
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) wsum[wv] = incl;
  __syncthreads();
  uint32_t woff = 0;
  for (int i = 0; i < wv; ++i) woff += wsum[i];
  uint64_t out = block_off[blockIdx.x] + woff + incl - c;
  if (full) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      uint32_t x = words[i] ^ 0x0a0a0a0au;
      uint32_t t = (x - 0x01010101u) & ~x & 0x80808080u;
      while (t) {
        int b = __builtin_ctz(t) >> 3;
        nl[out++] = base + 4 * i + b;
        t &= t - 1;
      }
    }
  } else {
    for (uint64_t i = base; i < len; ++i)
      if (buf[i] == '\n') nl[out++] = i;
  }
}

// ---- per-line JSON scanner ----------------------------------------------------------------------
struct Scan {
  const uint8_t* p;
  const uint8_t* end;
  const uint8_t* wbase;
  uint4 w;
  bool bad;

  __device__ __forceinline__ uint8_t at(const uint8_t* q) {
    const uint8_t* a = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(q) & ~uintptr_t(15));
    if (a != wbase) {
      wbase = a;
      w = *reinterpret_cast<const uint4*>(a);
    }
    const uint32_t off = uint32_t(q - a);
    const uint32_t word = off < 8 ? (off < 4 ? w.x : w.y) : (off < 12 ? w.z : w.w);
    return uint8_t(word >> ((off & 3) * 8));
  }
  __device__ __forceinline__ uint8_t peek() { return p < end ? at(p) : 0; }
  __device__ __forceinline__ void ws() {
    while (p < end) {
      uint8_t c = at(p);
      if (c != ' ' && c != '\t' && c != '\r' && c != '\n') break;
      ++p;
    }
  }
  __device__ __forceinline__ bool expect(uint8_t c) {
    ws();
    if (p < end && at(p) == c) { ++p; return true; }
    bad = true;
    return false;
  }
  // At an opening quote: returns the content span, sets *esc if it holds a backslash escape.
  __device__ bool string(const uint8_t** s, uint32_t* n, bool* esc) {
    ws();
    if (p >= end || at(p) != '"') { bad = true; return false; }
    ++p;
    const uint8_t* b = p;
    bool e = false;
    while (p < end) {
      uint8_t c = at(p);
      if (c == '"') {
        *s = b; *n = uint32_t(p - b); *esc = e; ++p;
        return true;
      }
      if (c == '\\') { e = true; p += 2; continue; }
      ++p;
    }
    bad = true;
    return false;
  }
  __device__ bool literal(const char* lit, int n) {
    for (int i = 0; i < n; ++i) {
      if (p + i >= end || at(p + i) != uint8_t(lit[i])) { bad = true; return false; }
    }
    p += n;
    return true;
  }
  // Skips any JSON value (object/array via a bracket depth counter that honours strings).
  __device__ void skip_value() {
    ws();
    if (p >= end) { bad = true; return; }
    uint8_t c = at(p);
    if (c == '"') { const uint8_t* s; uint32_t n; bool e; string(&s, &n, &e); return; }
    if (c == '{' || c == '[') {
      int depth = 0;
      while (p < end) {
        c = at(p);
        if (c == '"') { const uint8_t* s; uint32_t n; bool e; string(&s, &n, &e); if (bad) return; continue; }
        if (c == '{' || c == '[') ++depth;
        else if (c == '}' || c == ']') { if (--depth == 0) { ++p; return; } }
        ++p;
      }
      bad = true;
      return;
    }
    if (c == 't') { literal("true", 4); return; }
    if (c == 'f') { literal("false", 5); return; }
    if (c == 'n') { literal("null", 4); return; }
    // number
    const uint8_t* b = p;
    while (p < end) {
      c = at(p);
      if ((c >= '0' && c <= '9') || c == '-' || c == '+' || c == '.' || c == 'e' || c == 'E') ++p;
      else break;
    }
    if (p == b) bad = true;
  }
  __device__ __forceinline__ bool is_null() {
    ws();
    if (p + 4 <= end && at(p) == 'n') return literal("null", 4);
    return false;
  }
  // Integral JSON number -> int64 (Spark's LongType accepts VALUE_NUMBER_INT only).
  __device__ bool int64v(int64_t* out) {
    ws();
    bool neg = false;
    if (p < end && at(p) == '-') { neg = true; ++p; }
    uint64_t v = 0;
    const uint8_t* b = p;
    while (p < end) {
      uint8_t c = at(p);
      if (c < '0' || c > '9') break;
      v = v * 10 + (c - '0');
      ++p;
    }
    if (p == b || p - b > 19) { bad = true; return false; }
    uint8_t c = peek();
    if (c == '.' || c == 'e' || c == 'E') { bad = true; return false; }
    *out = neg ? -int64_t(v) : int64_t(v);
    return true;
  }
  __device__ bool key_is(const uint8_t* s, uint32_t n, const char* k, uint32_t kn) {
    if (n != kn) return false;
    for (uint32_t i = 0; i < n; ++i)
      if (at(s + i) != uint8_t(k[i])) return false;
    return true;
  }
};

struct FileFields {
  const uint8_t* path;
  uint32_t path_len;
  bool path_esc, path_null, has_delts;
  int64_t size, delts;
};

// Parses the inner object of an add/remove (AddFile / RemoveFile field names,
// D/actions/actions.scala:220-320); unknown fields are skipped (FAIL_ON_UNKNOWN_PROPERTIES=false).
__device__ bool parse_file_object(Scan& s, FileFields& f) {
  f.path = nullptr; f.path_len = 0; f.path_esc = false; f.path_null = true; f.has_delts = false;
  f.size = 0; f.delts = 0;
  if (!s.expect('{')) return false;
  s.ws();
  if (s.peek() == '}') { ++s.p; return true; }
  for (;;) {
    const uint8_t* k; uint32_t kn; bool ke;
    if (!s.string(&k, &kn, &ke)) return false;
    if (!s.expect(':')) return false;
    if (s.key_is(k, kn, "path", 4)) {
      if (!s.is_null()) {
        if (s.bad) return false;
        bool e;
        if (!s.string(&f.path, &f.path_len, &e)) return false;
        f.path_esc = e;
        f.path_null = false;
      } else {
        f.path_null = true;
      }
    } else if (s.key_is(k, kn, "size", 4)) {
      if (!s.is_null()) { if (s.bad || !s.int64v(&f.size)) return false; } else { f.size = 0; }
    } else if (s.key_is(k, kn, "deletionTimestamp", 17)) {
      if (!s.is_null()) {
        if (s.bad || !s.int64v(&f.delts)) return false;
        f.has_delts = true;
      } else {
        f.has_delts = false;
      }
    } else {
      s.skip_value();
      if (s.bad) return false;
    }
    s.ws();
    uint8_t c = s.peek();
    if (c == ',') { ++s.p; continue; }
    if (c == '}') { ++s.p; return true; }
    s.bad = true;
    return false;
  }
}

__global__ void __launch_bounds__(256) k_json_parse(JsonParseArgs a) {
  const uint64_t line = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (line >= a.nlines) return;
  const uint64_t b = line == 0 ? 0 : a.nl[line - 1] + 1;
  const uint64_t e = a.nl[line];
  const uint64_t idx = a.base + line;
  Scan s{a.buf + b, a.buf + e, nullptr, make_uint4(0, 0, 0, 0), false};
  uint8_t kind = K_NONE, flags = 0;
  FileFields add, rm;
  bool has_add = false, has_rm = false, has_meta = false, has_txn = false, has_prot = false, has_cdc = false,
       has_ci = false;
  s.ws();
  if (s.p < s.end) {
    if (s.expect('{')) {
      s.ws();
      if (s.peek() == '}') {
        ++s.p;
      } else {
        for (;;) {
          const uint8_t* k; uint32_t kn; bool ke;
          if (!s.string(&k, &kn, &ke) || !s.expect(':')) break;
          if (s.is_null()) {
            // a null member is an absent member
          } else if (s.bad) {
            break;
          } else if (s.key_is(k, kn, "add", 3)) {
            if (!parse_file_object(s, add)) break;
            has_add = true;
          } else if (s.key_is(k, kn, "remove", 6)) {
            if (!parse_file_object(s, rm)) break;
            has_rm = true;
          } else {
            if (s.key_is(k, kn, "metaData", 8)) has_meta = true;
            else if (s.key_is(k, kn, "txn", 3)) has_txn = true;
            else if (s.key_is(k, kn, "protocol", 8)) has_prot = true;
            else if (s.key_is(k, kn, "cdc", 3)) has_cdc = true;
            else if (s.key_is(k, kn, "commitInfo", 10)) has_ci = true;
            s.skip_value();
            if (s.bad) break;
          }
          s.ws();
          uint8_t c = s.peek();
          if (c == ',') { ++s.p; continue; }
          if (c == '}') { ++s.p; break; }
          s.bad = true;
          break;
        }
      }
      s.ws();
      if (s.p != s.end) s.bad = true;
    }
    if (s.bad) {
      kind = K_ERROR;  // Spark PERMISSIVE: a malformed record becomes an all-null row (ignored)
    } else if (has_add) {
      kind = K_ADD;
    } else if (has_rm) {
      kind = K_REMOVE;
    } else if (has_meta) {
      kind = K_METADATA;
    } else if (has_txn) {
      kind = K_TXN;
    } else if (has_prot) {
      kind = K_PROTOCOL;
    } else if (has_cdc) {
      kind = K_CDC;
    } else if (has_ci) {
      kind = K_COMMITINFO;
    }
  }
  uint64_t key = 0;
  const uint8_t* path = nullptr;
  uint32_t plen = 0;
  int64_t size = 0, delts = 0;
  if (kind == K_ADD || kind == K_REMOVE) {
    const FileFields& f = kind == K_ADD ? add : rm;
    path = f.path;
    plen = f.path_len;
    size = f.size;
    delts = f.delts;
    if (f.has_delts) flags |= F_HAS_DELTS;
    if (f.path_null) flags |= F_PATH_NULL;
    if (f.path_esc) flags |= F_PATH_ESCAPED;
    if (f.path_esc || path_is_special(path, plen)) {
      flags |= F_SPECIAL_PATH;
      atomicAdd(reinterpret_cast<unsigned long long*>(a.special_count), 1ull);
      atomicAdd(reinterpret_cast<unsigned long long*>(a.special_bytes), (unsigned long long)(plen + 8));
    } else if (!f.path_null) {
      key = path_key(path, plen);
    }
  } else if (kind != K_NONE && kind != K_ERROR && kind != K_COMMITINFO && kind != K_CDC) {
    // protocol / metaData / txn: reduced on the host (the reference's single `null` partition)
    const unsigned long long slot = atomicAdd(reinterpret_cast<unsigned long long*>(a.nonfile_count), 1ull);
    if (slot < a.nonfile_cap) a.nonfile_idx[slot] = line;
  }
  if (kind == K_ERROR) atomicAdd(reinterpret_cast<unsigned long long*>(a.error_count), 1ull);
  a.kind[idx] = kind;
  a.flags[idx] = flags;
  a.key[idx] = key;
  a.path_ptr[idx] = reinterpret_cast<uint64_t>(path);
  a.path_len[idx] = plen;
  a.size[idx] = size;
  a.delts[idx] = delts;
  a.src_off[idx] = b;
  a.src_len[idx] = uint32_t(e - b);
}

}  // namespace dev

// ---- launchers -----------------------------------------------------------------------------------
uint64_t json_num_blocks(uint64_t len) { return (len + dev::JSON_BYTES_PER_BLOCK - 1) / dev::JSON_BYTES_PER_BLOCK; }

void launch_json_count(const uint8_t* buf, uint64_t len, uint32_t* block_counts, hipStream_t st) {
  uint64_t nb = json_num_blocks(len);
  if (nb) hipLaunchKernelGGL(dev::k_json_count, dim3(unsigned(nb)), dim3(dev::JSON_THREADS), 0, st, buf, len, block_counts);
}

void launch_json_newlines(const uint8_t* buf, uint64_t len, const uint64_t* block_off, uint64_t* nl, hipStream_t st) {
  uint64_t nb = json_num_blocks(len);
  if (nb) hipLaunchKernelGGL(dev::k_json_newlines, dim3(unsigned(nb)), dim3(dev::JSON_THREADS), 0, st, buf, len, block_off, nl);
}

void launch_json_parse(const JsonParseArgs& a, hipStream_t st) {
  if (!a.nlines) return;
  hipLaunchKernelGGL(dev::k_json_parse, dim3(unsigned((a.nlines + 255) / 256)), dim3(256), 0, st, a);
}

}  // namespace dr
