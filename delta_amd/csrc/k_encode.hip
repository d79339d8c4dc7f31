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

}  // namespace dr
