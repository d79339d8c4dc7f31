// Device-side helpers shared by the replay kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace dr {
namespace dev {

// ---- action kinds (SingleAction envelope, D/actions/actions.scala:514-541) ------------------
enum Kind : uint8_t { K_NONE = 0, K_ADD = 1, K_REMOVE = 2, K_METADATA = 3, K_TXN = 4, K_PROTOCOL = 5,
                      K_CDC = 6, K_COMMITINFO = 7, K_ERROR = 15 };
// action flags
enum Flag : uint8_t { F_HAS_DELTS = 1, F_SPECIAL_PATH = 2, F_PATH_ESCAPED = 4, F_PATH_NULL = 8,
                      F_FROM_CKPT = 16 };
// replay classes carried in the partition records (low 2 bits of the meta word)
enum Class : uint32_t { C_ADD = 0, C_REMOVE_KEEP = 1, C_REMOVE_DROP = 2 };

// A 16-byte load through the global address space (a flat load also counts against the LDS
// counter, so every LDS access after it waits for it too).
typedef unsigned int gu32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 gload16(const uint4* p) {
#if defined(__HIP_DEVICE_COMPILE__)
  const gu32x4 v = *(const __attribute__((address_space(1))) gu32x4*)(p);
  return make_uint4(v.x, v.y, v.z, v.w);
#else
  return *p;
#endif
}

// A dword store through the global address space (through a pointer loaded from a descriptor the
// compiler emits a flat store, which also counts against the LDS counter).
__device__ __forceinline__ void gstore32(uint32_t* p, uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  *(__attribute__((address_space(1))) uint32_t*)(p) = v;
#else
  *p = v;
#endif
}

// ---- unaligned little-endian loads from byte buffers (buffers are padded by >= 16 bytes) -----
__device__ __forceinline__ uint32_t ld_u32a(const uint8_t* p) {  // aligned dword
  return *reinterpret_cast<const uint32_t*>(p);
}
__device__ __forceinline__ uint64_t load_u64(const uint8_t* p) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint8_t* b = p - (a & 3u);  // pointer arithmetic, not an integer round trip: an LDS pointer stays one
  const uint32_t sh = uint32_t(a & 3);
  const uint32_t w0 = ld_u32a(b), w1 = ld_u32a(b + 4), w2 = ld_u32a(b + 8);
  const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sh);
  const uint32_t hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
  return uint64_t(lo) | (uint64_t(hi) << 32);
}
__device__ __forceinline__ uint32_t load_u32(const uint8_t* p) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint8_t* b = p - (a & 3u);
  return __builtin_amdgcn_alignbyte(ld_u32a(b + 4), ld_u32a(b), uint32_t(a & 3));
}

// ---- xxHash64 (seed 0) ------------------------------------------------------------------------
constexpr uint64_t P1 = 0x9E3779B185EBCA87ull, P2 = 0xC2B2AE3D27D4EB4Full, P3 = 0x165667B19E3779F9ull,
                   P4 = 0x85EBCA77C2B2AE63ull, P5 = 0x27D4EB2F165667C5ull;
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t xx_round(uint64_t acc, uint64_t in) {
  acc += in * P2;
  acc = rotl64(acc, 31);
  return acc * P1;
}
__device__ __forceinline__ uint64_t xx_merge(uint64_t h, uint64_t v) {
  h ^= xx_round(0, v);
  return h * P1 + P4;
}
// xxh64 of p[0..len). Keys are hash | (hash == 0) so that 0 can mark an empty table slot.
__device__ inline uint64_t xxh64(const uint8_t* p, uint32_t len, uint64_t seed = 0) {
  const uint8_t* end = p + len;
  uint64_t h;
  if (len >= 32) {
    uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
    const uint8_t* lim = end - 32;
    do {
      v1 = xx_round(v1, load_u64(p));
      v2 = xx_round(v2, load_u64(p + 8));
      v3 = xx_round(v3, load_u64(p + 16));
      v4 = xx_round(v4, load_u64(p + 24));
      p += 32;
    } while (p <= lim);
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    h = xx_merge(h, v1);
    h = xx_merge(h, v2);
    h = xx_merge(h, v3);
    h = xx_merge(h, v4);
  } else {
    h = seed + P5;
  }
  h += len;
  while (p + 8 <= end) {
    h ^= xx_round(0, load_u64(p));
    h = rotl64(h, 27) * P1 + P4;
    p += 8;
  }
  if (p + 4 <= end) {
    h ^= uint64_t(load_u32(p)) * P1;
    h = rotl64(h, 23) * P2 + P3;
    p += 4;
  }
  while (p < end) {
    h ^= uint64_t(*p) * P5;
    h = rotl64(h, 11) * P1;
    ++p;
  }
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return h;
}
// Packed path reference (k_bucket_verify's gathers): address | length << 48 (0: a length that does not
// fit 16 bits; such a path sends its bucket to the exact reducer).
__device__ __forceinline__ uint64_t pack_ref(uint64_t ptr, uint32_t len) {
  return len < 0xffffu ? (ptr | (uint64_t(len) << 48)) : 0ull;
}

__device__ __forceinline__ uint64_t path_key(const uint8_t* p, uint32_t len) {
  const uint64_t h = xxh64(p, len);
  return h ? h : 1;
}

// Byte-equality of two device strings.
__device__ inline bool bytes_equal(const uint8_t* a, const uint8_t* b, uint32_t n) {
  uint32_t i = 0;
  for (; i + 8 <= n; i += 8)
    if (load_u64(a + i) != load_u64(b + i)) return false;
  for (; i < n; ++i)
    if (a[i] != b[i]) return false;
  return true;
}

// A path needs host-independent canonicalization (D/Snapshot.scala:317-328) when it is absolute
// without a scheme ("/x" -> "file:///x"), carries a `file:` scheme (URI-equality key), or was
// JSON-escaped. Everything else (relative, URI-safe) is its own canonical form and key.
__device__ __forceinline__ bool path_is_special(const uint8_t* p, uint32_t len) {
  if (len == 0) return false;
  if (p[0] == '/') return true;
  if (len >= 5 && p[0] == 'f' && p[1] == 'i' && p[2] == 'l' && p[3] == 'e' && p[4] == ':') return true;
  return false;
}

// ---- JSON string escapes ------------------------------------------------------------------------
__device__ inline int hexval(uint8_t c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

// JSON string unescape into out; returns the output length (UTF-8).
__device__ inline uint32_t json_unescape(const uint8_t* s, uint32_t n, uint8_t* out) {
  uint32_t o = 0;
  for (uint32_t i = 0; i < n; ++i) {
    uint8_t c = s[i];
    if (c != '\\' || i + 1 >= n) { out[o++] = c; continue; }
    uint8_t e = s[++i];
    switch (e) {
      case 'b': out[o++] = '\b'; break;
      case 'f': out[o++] = '\f'; break;
      case 'n': out[o++] = '\n'; break;
      case 'r': out[o++] = '\r'; break;
      case 't': out[o++] = '\t'; break;
      case 'u': {
        uint32_t cp = 0;
        for (int k = 0; k < 4 && i + 1 < n; ++k) cp = cp * 16 + uint32_t(hexval(s[++i]) & 15);
        if (cp >= 0xD800 && cp < 0xDC00 && i + 6 < n && s[i + 1] == '\\' && s[i + 2] == 'u') {
          uint32_t lo = 0;
          for (int k = 0; k < 4; ++k) lo = lo * 16 + uint32_t(hexval(s[i + 3 + k]) & 15);
          if (lo >= 0xDC00 && lo < 0xE000) { cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00); i += 6; }
        }
        if (cp < 0x80) out[o++] = uint8_t(cp);
        else if (cp < 0x800) { out[o++] = uint8_t(0xC0 | (cp >> 6)); out[o++] = uint8_t(0x80 | (cp & 63)); }
        else if (cp < 0x10000) {
          out[o++] = uint8_t(0xE0 | (cp >> 12)); out[o++] = uint8_t(0x80 | ((cp >> 6) & 63));
          out[o++] = uint8_t(0x80 | (cp & 63));
        } else {
          out[o++] = uint8_t(0xF0 | (cp >> 18)); out[o++] = uint8_t(0x80 | ((cp >> 12) & 63));
          out[o++] = uint8_t(0x80 | ((cp >> 6) & 63)); out[o++] = uint8_t(0x80 | (cp & 63));
        }
        break;
      }
      default: out[o++] = e; break;  // \" \\ \/
    }
  }
  return o;
}

// Replay key of a canonical path: java.net.URI equality treats "file:///x" and "file:/x" alike.
__device__ __forceinline__ uint32_t key_skip(const uint8_t* p, uint32_t n) {
  return (n >= 8 && p[0] == 'f' && p[1] == 'i' && p[2] == 'l' && p[3] == 'e' && p[4] == ':' && p[5] == '/' &&
          p[6] == '/' && p[7] == '/') ? 2u : 0u;
}
__device__ inline bool key_equal(const uint8_t* a, uint32_t an, const uint8_t* b, uint32_t bn) {
  const uint32_t sa = key_skip(a, an), sb = key_skip(b, bn);
  if (an - sa != bn - sb) return false;
  // compare "file:" (5 bytes) then the remainder after the skipped "//"
  if (sa | sb) {
    for (uint32_t i = 0; i < 5; ++i) if (a[i] != b[i]) return false;
    return bytes_equal(a + 5 + sa, b + 5 + sb, an - sa - 5);
  }
  return bytes_equal(a, b, an);
}


// The readback's completion word (ReadbackArgs::flag): every thread's span stores are fenced to the
// system scope before one thread publishes the sequence number the host spins on.
template <class Readback>  // ReadbackArgs (kernels.h)
__device__ __forceinline__ void readback_flag(const Readback& a) {
  if (!a.flag) return;
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(a.flag, a.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace dev
}  // namespace dr
