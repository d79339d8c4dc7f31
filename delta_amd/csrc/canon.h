// Canonicalisation of one special path (D/Snapshot.scala:317-328), shared by k_canon and the
// small-segment tail kernel (k_json.hip:k_tail_post).
#pragma once
#include "dev_common.h"
#include "kernels.h"

namespace dr {
namespace dev {

__device__ __forceinline__ void canon_one(const CanonArgs& a, uint64_t i) {

  const uint8_t f = a.act.flags[i];
  if (!(f & F_SPECIAL_PATH)) return;
  const uint8_t* src = reinterpret_cast<const uint8_t*>(a.act.path_ptr[i]);
  const uint32_t n = a.act.path_len[i];
  const uint64_t need = 2ull * (n + 8) + 16;
  const unsigned long long at = atomicAdd(reinterpret_cast<unsigned long long*>(a.arena_fill), (unsigned long long)need);
  if (at + need > a.arena_cap) return;  // host sized the arena from the same counters
  uint8_t* out = a.arena + at;
  uint32_t m;
  uint8_t* body = out + 7;  // room for a "file://" prefix
  if (f & F_PATH_ESCAPED) m = json_unescape(src, n, body);
  else { for (uint32_t k = 0; k < n; ++k) body[k] = src[k]; m = n; }
  uint8_t* res = body;
  if (m > 0 && body[0] == '/') {
    // Hadoop Path normalisation ('//' collapse, no trailing '/'), then makeQualified on the local
    // filesystem: scheme "file", empty authority -> "file://" + path.
    uint32_t w = 0;
    for (uint32_t k = 0; k < m; ++k) {
      if (body[k] == '/' && w > 0 && body[w - 1] == '/') continue;
      body[w++] = body[k];
    }
    if (w > 1 && body[w - 1] == '/') --w;
    res = out;
    const char pre[7] = {'f', 'i', 'l', 'e', ':', '/', '/'};
    for (int k = 0; k < 7; ++k) out[k] = uint8_t(pre[k]);
    m = w + 7;
  }
  // key bytes (URI-equality form) for hashing, written after the output string
  uint8_t* kb = res + m + 8;
  const uint32_t sk = key_skip(res, m);
  uint32_t kn = 0;
  for (uint32_t k = 0; k < m; ++k) {
    if (sk && (k == 5 || k == 6)) continue;
    kb[kn++] = res[k];
  }
  a.act.path_ptr[i] = reinterpret_cast<uint64_t>(res);
  a.act.path_len[i] = m;
  if (a.act.path_ref) a.act.path_ref[i] = pack_ref(reinterpret_cast<uint64_t>(res), m);
  a.act.key[i] = path_key(kb, kn);
}

}  // namespace dev
}  // namespace dr
