// Checkpoint page encoding on the device (D/Checkpoints.scala:229-365 writes the
// state with Spark's Parquet writer). For one leaf column and one row group: per row its level
// count and value bytes (k_enc_count), scanned, then its definition / repetition levels and its
// PLAIN values (k_enc_fill: INT64 / INT32 little-endian, BYTE_ARRAY 4-byte length + bytes, BOOLEAN
// one byte per value until k_enc_pack bit-packs it), then the levels bit-packed for the
// RLE/bit-packing hybrid (k_enc_pack). The host writes the page headers and the footer (Thrift).
#include "dev_common.h"
#include "kernels.h"

namespace dr {
namespace dev {

constexpr int ENC_T = 256;

__device__ __forceinline__ bool enc_null(const EncLeaf& L, uint64_t i) {
  return (L.null && L.null[i]) || (L.vflags && !(L.vflags[i] & L.vbit));
}

__device__ __forceinline__ uint32_t str_len(const EncLeaf& L, uint64_t i) {
  return L.kind == ENC_STR_PTR ? L.slen[i] : uint32_t(L.off[i + 1] - L.off[i]);
}

__global__ void __launch_bounds__(ENC_T) k_enc_count(EncArgs a) {
  const uint64_t g = a.r0 + uint64_t(blockIdx.x) * ENC_T + threadIdx.x;
  if (g >= a.r1) return;
  const uint64_t row = g - a.r0;
  uint32_t lev = 1, vb = 0;
  if (g >= a.side_lo && g < a.side_lo + a.n) {
    const uint64_t i = g - a.side_lo;
    const EncLeaf& L = a.L;
    if (L.kind == ENC_MAP_KEY || L.kind == ENC_MAP_VAL) {
      const uint64_t e0 = L.entry_off[i], e1 = L.entry_off[i + 1];
      if (!enc_null(L, i) && e1 > e0) {
        lev = uint32_t(e1 - e0);
        for (uint64_t e = e0; e < e1; ++e)
          if (L.kind == ENC_MAP_KEY || !L.enull[e]) vb += 4 + uint32_t(L.eoff[e + 1] - L.eoff[e]);
      }
    } else if (!enc_null(L, i)) {
      switch (L.kind) {
        case ENC_STR_PTR:
        case ENC_STR_OFF: vb = 4 + str_len(L, i); break;
        case ENC_I64: vb = 8; break;
        case ENC_I32: vb = 4; break;
        default: vb = 1; break;  // BOOLEAN: one byte until packed
      }
    }
  }
  a.nlev[row] = lev;
  a.vbytes[row] = vb;
}

__device__ __forceinline__ void put_u32(uint8_t* p, uint32_t v) {
  p[0] = uint8_t(v); p[1] = uint8_t(v >> 8); p[2] = uint8_t(v >> 16); p[3] = uint8_t(v >> 24);
}

__global__ void __launch_bounds__(ENC_T) k_enc_fill(EncArgs a) {
  const uint64_t g = a.r0 + uint64_t(blockIdx.x) * ENC_T + threadIdx.x;
  if (g >= a.r1) return;
  const uint64_t row = g - a.r0;
  uint64_t lo = a.lev_off[row];
  uint8_t* v = a.vals + a.val_off[row];
  const EncLeaf& L = a.L;
  const bool map = L.kind == ENC_MAP_KEY || L.kind == ENC_MAP_VAL;
  if (!(g >= a.side_lo && g < a.side_lo + a.n)) {
    a.def[lo] = 0;
    if (map) a.rep[lo] = 0;
    return;
  }
  const uint64_t i = g - a.side_lo;
  if (map) {
    const uint64_t e0 = L.entry_off[i], e1 = L.entry_off[i + 1];
    if (enc_null(L, i)) {
      a.def[lo] = uint8_t(L.def_null);
      a.rep[lo] = 0;
      return;
    }
    if (e1 == e0) {  // empty map: the map is defined, no key_value
      a.def[lo] = uint8_t(L.def_null + 1);
      a.rep[lo] = 0;
      return;
    }
    for (uint64_t e = e0; e < e1; ++e, ++lo) {
      a.rep[lo] = e == e0 ? 0 : 1;
      const bool vnull = L.kind == ENC_MAP_VAL && L.enull[e];
      a.def[lo] = uint8_t(vnull ? L.def_null + 2 : L.def_present);
      if (!vnull) {
        const uint32_t n = uint32_t(L.eoff[e + 1] - L.eoff[e]);
        put_u32(v, n);
        const uint8_t* src = L.ebytes + L.eoff[e];
        for (uint32_t k = 0; k < n; ++k) v[4 + k] = src[k];
        v += 4 + n;
      }
    }
    return;
  }
  if (enc_null(L, i)) {
    a.def[lo] = uint8_t(L.def_null);
    return;
  }
  a.def[lo] = uint8_t(L.def_present);
  switch (L.kind) {
    case ENC_STR_PTR:
    case ENC_STR_OFF: {
      const uint32_t n = str_len(L, i);
      const uint8_t* src = L.kind == ENC_STR_PTR ? reinterpret_cast<const uint8_t*>(L.sptr[i]) : L.bytes + L.off[i];
      put_u32(v, n);
      for (uint32_t k = 0; k < n; ++k) v[4 + k] = src[k];
      break;
    }
    case ENC_I64: {
      const uint64_t x = uint64_t(L.i64[i]);
      put_u32(v, uint32_t(x));
      put_u32(v + 4, uint32_t(x >> 32));
      break;
    }
    case ENC_I32: put_u32(v, L.i32[i]); break;
    default: v[0] = L.b8 ? (L.b8[i] ? 1 : 0) : L.i32 ? (L.i32[i] ? 1 : 0) : 0; break;
  }
}

__global__ void __launch_bounds__(ENC_T) k_enc_pack(const uint8_t* in, uint64_t n, int width, uint8_t* out) {
  const uint64_t grp = uint64_t(blockIdx.x) * ENC_T + threadIdx.x;
  if (grp * 8 >= n) return;
  uint64_t bits = 0;
  for (int k = 0; k < 8; ++k) {
    const uint64_t j = grp * 8 + k;
    const uint64_t x = j < n ? in[j] : 0;
    bits |= x << (width * k);
  }
  for (int b = 0; b < width; ++b) out[grp * width + b] = uint8_t(bits >> (8 * b));
}

}  // namespace dev

void launch_enc_count(const EncArgs& a, hipStream_t st) {
  if (a.r1 > a.r0) DR_LAUNCH(dev::k_enc_count, dim3(unsigned((a.r1 - a.r0 + dev::ENC_T - 1) / dev::ENC_T)), dim3(dev::ENC_T), 0, st, a);
}
void launch_enc_fill(const EncArgs& a, hipStream_t st) {
  if (a.r1 > a.r0) DR_LAUNCH(dev::k_enc_fill, dim3(unsigned((a.r1 - a.r0 + dev::ENC_T - 1) / dev::ENC_T)), dim3(dev::ENC_T), 0, st, a);
}
void launch_enc_pack(const uint8_t* in, uint64_t n, int width, uint8_t* out, hipStream_t st) {
  const uint64_t groups = (n + 7) / 8;
  if (groups) DR_LAUNCH(dev::k_enc_pack, dim3(unsigned((groups + dev::ENC_T - 1) / dev::ENC_T)), dim3(dev::ENC_T), 0, st, in, n, width, out);
}

// ---- SNAPPY compression (pages of the checkpoint writer) ------------------------------------------
namespace dev {
// 8 KiB fragments (inside the reader's 64 KiB blocks, so its fragment rule holds): a 1M-row part's
// pages give ~37K lanes instead of ~4.6K, and the lane-serial parse is 8x shorter.
constexpr uint32_t SC_FRAG = 8192;
constexpr uint32_t SC_SLOT = SC_FRAG + SC_FRAG / 6 + 64;  // worst case: all literals
constexpr int SC_BITS = 9;                                 // hash table entries per lane: 2^9 (1 KiB)

__device__ __forceinline__ uint32_t ld32(const uint8_t* p) {
  return uint32_t(p[0]) | (uint32_t(p[1]) << 8) | (uint32_t(p[2]) << 16) | (uint32_t(p[3]) << 24);
}

__device__ uint32_t emit_literal(uint8_t* d, uint32_t o, const uint8_t* s, uint32_t n) {
  const uint32_t m = n - 1;
  if (m < 60) {
    d[o++] = uint8_t(m << 2);
  } else if (m < 256) {
    d[o++] = uint8_t(60 << 2);
    d[o++] = uint8_t(m);
  } else {
    d[o++] = uint8_t(61 << 2);
    d[o++] = uint8_t(m);
    d[o++] = uint8_t(m >> 8);
  }
  for (uint32_t k = 0; k < n; ++k) d[o + k] = s[k];
  return o + n;
}

__device__ uint32_t emit_copy(uint8_t* d, uint32_t o, uint32_t off, uint32_t len) {
  while (len > 0) {
    // pieces of at most 64 bytes, never leaving fewer than 4 for a COPY_1 tail
    uint32_t l = len > 64 ? (len - 64 < 4 ? 60 : 64) : len;
    if (l >= 4 && l <= 11 && off < 2048) {
      d[o++] = uint8_t(1 | ((l - 4) << 2) | ((off >> 8) << 5));
      d[o++] = uint8_t(off);
    } else {
      d[o++] = uint8_t(2 | ((l - 1) << 2));
      d[o++] = uint8_t(off);
      d[o++] = uint8_t(off >> 8);
    }
    len -= l;
  }
  return o;
}

__global__ void __launch_bounds__(64) k_snap_compress(const uint8_t* in, uint64_t n, uint8_t* out, uint32_t* out_len,
                                                      uint32_t nfrag) {
  __shared__ uint16_t table[64][1 << SC_BITS];
  const uint32_t lane = threadIdx.x;
  const uint32_t f = blockIdx.x * 64 + lane;
  uint16_t* tab = table[lane];
  for (uint32_t k = 0; k < (1u << SC_BITS); ++k) tab[k] = 0xffff;
  if (f >= nfrag) return;
  const uint8_t* s = in + uint64_t(f) * SC_FRAG;
  const uint32_t len = uint32_t(min(uint64_t(SC_FRAG), n - uint64_t(f) * SC_FRAG));
  uint8_t* d = out + uint64_t(f) * SC_SLOT;
  uint32_t o = 0, ip = 0, lit = 0;
  if (len >= 16) {
    const uint32_t limit = len - 4;
    while (ip <= limit) {
      const uint32_t cur = ld32(s + ip);
      const uint32_t h = (cur * 0x1e35a7bdu) >> (32 - SC_BITS);
      const uint32_t cand = tab[h];
      tab[h] = uint16_t(ip);
      if (cand != 0xffffu && cand < ip && ld32(s + cand) == cur) {
        uint32_t m = 4;
        while (ip + m < len && s[cand + m] == s[ip + m]) ++m;
        if (ip > lit) o = emit_literal(d, o, s + lit, ip - lit);
        o = emit_copy(d, o, ip - cand, m);
        ip += m;
        lit = ip;
      } else {
        ++ip;
      }
    }
  }
  if (len > lit) o = emit_literal(d, o, s + lit, len - lit);
  out_len[f] = o;
}
}  // namespace dev

uint64_t snap_compress_slot() { return dev::SC_SLOT; }

void launch_snap_compress(const uint8_t* in, uint64_t n, uint8_t* out, uint32_t* out_len, hipStream_t st) {
  const uint32_t nfrag = uint32_t((n + dev::SC_FRAG - 1) / dev::SC_FRAG);
  if (nfrag) DR_LAUNCH(dev::k_snap_compress, dim3((nfrag + 63) / 64), dim3(64), 0, st, in, n, out, out_len, nfrag);
}

}  // namespace dr
