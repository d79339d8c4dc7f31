#include "snappy_host.h"

#include <cstring>

namespace dr {

bool snappy_uncompressed_length(const uint8_t* in, size_t n, uint64_t* out) {
  uint64_t v = 0;
  for (size_t i = 0; i < n && i < 10; ++i) {
    v |= uint64_t(in[i] & 0x7f) << (7 * i);
    if (!(in[i] & 0x80)) { *out = v; return true; }
  }
  return false;
}

bool snappy_decompress(const uint8_t* in, size_t n, uint8_t* out, size_t out_len) {
  size_t ip = 0;
  uint64_t total = 0;
  while (ip < n && (in[ip] & 0x80)) ++ip;
  if (ip >= n || !snappy_uncompressed_length(in, n, &total) || total != out_len) return false;
  ++ip;
  size_t op = 0;
  while (ip < n) {
    const uint8_t tag = in[ip++];
    const uint32_t t = tag & 3;
    if (t == 0) {  // literal
      uint64_t len = tag >> 2;
      if (len >= 60) {
        const uint32_t nb = uint32_t(len - 59);
        if (ip + nb > n) return false;
        len = 0;
        for (uint32_t b = 0; b < nb; ++b) len |= uint64_t(in[ip + b]) << (8 * b);
        ip += nb;
      }
      len += 1;
      if (ip + len > n || op + len > out_len) return false;
      memcpy(out + op, in + ip, len);
      ip += len;
      op += len;
    } else {
      uint64_t len, off;
      if (t == 1) {
        if (ip + 1 > n) return false;
        len = ((tag >> 2) & 7) + 4;
        off = (uint64_t(tag >> 5) << 8) | in[ip];
        ip += 1;
      } else if (t == 2) {
        if (ip + 2 > n) return false;
        len = (tag >> 2) + 1;
        off = uint64_t(in[ip]) | (uint64_t(in[ip + 1]) << 8);
        ip += 2;
      } else {
        if (ip + 4 > n) return false;
        len = (tag >> 2) + 1;
        off = uint64_t(in[ip]) | (uint64_t(in[ip + 1]) << 8) | (uint64_t(in[ip + 2]) << 16) |
              (uint64_t(in[ip + 3]) << 24);
        ip += 4;
      }
      if (off == 0 || off > op || op + len > out_len) return false;
      for (uint64_t k = 0; k < len; ++k) out[op + k] = out[op - off + k];  // overlap-safe
      op += len;
    }
  }
  return op == out_len;
}

}  // namespace dr
