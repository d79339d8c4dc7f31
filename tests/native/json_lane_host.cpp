// Host build of the K1 line walker (delta_amd/csrc/json_lane.h) for CPU fuzzing against Python's
// json module (tests/test_json_lane.py). Test infrastructure only.
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../delta_amd/csrc/json_lane.h"

extern "C" int jl_parse(const unsigned char* line, unsigned n, unsigned align, int general, unsigned char* kind,
                        unsigned char* flags, unsigned* path_off, unsigned* path_len, long long* size,
                        long long* delts) {
  // place the line at the requested alignment inside a 16-byte aligned, padded buffer filled with
  // bytes that must never influence the result
  std::vector<unsigned char> buf(n + 64 + 32);
  unsigned char* base = buf.data();
  while (reinterpret_cast<uintptr_t>(base) & 15) ++base;
  std::memset(buf.data(), '"', buf.size());
  std::memcpy(base + (align & 15), line, n);
  dr::jl::LineOut o;
  if (general) dr::jl::parse_line_general(base + (align & 15), n, o);
  else dr::jl::parse_line(base + (align & 15), n, o);
  *kind = o.kind;
  *flags = o.flags;
  *path_off = o.path_off;
  *path_len = o.path_len;
  *size = o.size;
  *delts = o.delts;
  return o.hard;
}

// classify() against a per-byte restatement of the five tokenizer classes on `n` pseudo-random
// windows (JSON punctuation, whitespace, control and high bytes mixed in); returns the first
// mismatching window + 1, or 0.
extern "C" long long jl_classify_check(unsigned long long seed, long long n) {
  const char pick[] = "\"\\{}[]:, \t\r\nab\x01\x80\xff";
  unsigned long long x = seed | 1;
  for (long long it = 0; it < n; ++it) {
    unsigned char b[16];
    for (int k = 0; k < 16; ++k) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      b[k] = (x & 3) == 0 ? static_cast<unsigned char>(pick[(x >> 2) % 18]) : static_cast<unsigned char>(x >> 8);
    }
    uint32_t w[4];
    std::memcpy(w, b, 16);
    dr::jl::Win m;
    dr::jl::classify(w, m);
    uint32_t q = 0, bs = 0, st = 0, sp = 0, ct = 0;
    for (int k = 0; k < 16; ++k) {
      const unsigned char c = b[k];
      if (c == '"') q |= 1u << k;
      if (c == '\\') bs |= 1u << k;
      if (c == '{' || c == '}' || c == '[' || c == ']' || c == ':' || c == ',') st |= 1u << k;
      if (c == ' ') sp |= 1u << k;
      if (c < 0x20) ct |= 1u << k;
    }
    if (q != m.q || bs != m.bs || st != m.st || sp != m.sp || ct != m.ctrl) return it + 1;
  }
  return 0;
}
