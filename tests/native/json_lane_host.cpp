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
