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
        case ENC_INT96: vb = 12; break;
        case ENC_FLBA_BE: vb = L.width; break;
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
    case ENC_INT96: {
      // Spark's INT96 timestamp (ParquetWriteSupport, DateTimeUtils.toJulianDay): nanoseconds of the
      // day (int64) then the Julian day number (int32), little-endian; days by floor division
      const int64_t us = L.i64[i];
      const int64_t day = us >= 0 ? us / 86400000000ll : -((-us + 86399999999ll) / 86400000000ll);
      const uint64_t nanos = uint64_t(us - day * 86400000000ll) * 1000ull;
      put_u32(v, uint32_t(nanos));
      put_u32(v + 4, uint32_t(nanos >> 32));
      put_u32(v + 8, uint32_t(int32_t(day + 2440588)));
      break;
    }
    case ENC_FLBA_BE: {
      // unscaled decimal, two's complement, big-endian in `width` bytes (Spark's binary decimals)
      const uint64_t lo = uint64_t(L.i64[i]), hi = uint64_t(L.i64hi ? L.i64hi[i] : (L.i64[i] < 0 ? -1 : 0));
      for (uint32_t k = 0; k < L.width; ++k) {
        const uint32_t bit = 8 * (L.width - 1 - k);
        v[k] = uint8_t(bit < 64 ? lo >> bit : bit < 128 ? hi >> (bit - 64) : (hi >> 63 ? 0xff : 0));
      }
      break;
    }
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
// One workgroup per 8 KiB fragment of the page body (fragments sit inside the reader's 64 KiB
// blocks, so its fragment rule holds: no element straddles one, no copy reaches before it):
//  1. the fragment is staged in LDS with 16-byte loads;
//  2. a 4096-entry table keeps, per hash of 4 bytes, the EARLIEST position in the fragment
//     (atomicMin, every position in parallel) -- a valid match candidate for every later position;
//  3. thread t compresses its 64-byte slice greedily against the whole fragment (matches verified
//     on the LDS bytes, cut at the slice end), into its LDS output slot;
//  4. a block scan of the slot sizes packs the slots contiguously (LDS) and the fragment's elements
//     leave with 16-byte stores to out + f * SC_SLOT; out_len[f] is their length.
// k_snap_gather then compacts the fragments into one stream.
constexpr uint32_t SC_FRAG = 8192;
constexpr int SC_T = 128;
constexpr uint32_t SC_SLICE = SC_FRAG / SC_T;              // 64 input bytes per thread
constexpr uint32_t SC_OMAX = SC_SLICE + 8;                 // a slice's worst case: one literal, 2-byte tag
constexpr uint32_t SC_SLOT = 9632;                         // >= SC_T * (SC_SLICE + 2), 16-byte multiple
constexpr int SC_TBITS = 12;

__device__ __forceinline__ uint32_t lds32u(const uint8_t* p) {  // 4 bytes at any LDS address
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(p - (a & 3u));
  return __builtin_amdgcn_alignbyte(w[1], w[0], uint32_t(a & 3u));
}
__device__ __forceinline__ uint32_t sc_hash(uint32_t x) { return (x * 0x1e35a7bdu) >> (32 - SC_TBITS); }

__device__ uint32_t emit_literal(uint8_t* d, uint32_t o, const uint8_t* s, uint32_t n) {
  const uint32_t m = n - 1;
  if (m < 60) {
    d[o++] = uint8_t(m << 2);
  } else {
    d[o++] = uint8_t(60 << 2);
    d[o++] = uint8_t(m);
  }
  for (uint32_t k = 0; k < n; ++k) d[o + k] = s[k];
  return o + n;
}

__device__ uint32_t emit_copy(uint8_t* d, uint32_t o, uint32_t off, uint32_t len) {
  // len <= 64 (a slice), off < 8192
  if (len >= 4 && len <= 11 && off < 2048) {
    d[o++] = uint8_t(1 | ((len - 4) << 2) | ((off >> 8) << 5));
    d[o++] = uint8_t(off);
  } else {
    d[o++] = uint8_t(2 | ((len - 1) << 2));
    d[o++] = uint8_t(off);
    d[o++] = uint8_t(off >> 8);
  }
  return o;
}

__global__ void __launch_bounds__(SC_T) k_snap_compress(const uint8_t* __restrict__ in, uint64_t n,
                                                        uint8_t* __restrict__ out, uint32_t* __restrict__ out_len) {
  __shared__ __attribute__((aligned(16))) uint8_t frag[SC_FRAG + 16];
  __shared__ uint32_t table[1u << SC_TBITS];
  __shared__ __attribute__((aligned(16))) uint8_t obuf[SC_T * SC_OMAX];
  __shared__ __attribute__((aligned(16))) uint8_t cbuf[SC_SLOT];
  __shared__ uint32_t wsum[SC_T / 64];
  const uint32_t f = blockIdx.x, t = threadIdx.x;
  const uint64_t base = uint64_t(f) * SC_FRAG;
  const uint32_t len = uint32_t(min(uint64_t(SC_FRAG), n - base));
  const uint32_t nv = (len + 15) / 16;  // the input buffer is readable up to 16 bytes past n
  for (uint32_t v = t; v < nv; v += SC_T)
    *reinterpret_cast<uint4*>(frag + 16 * v) = *reinterpret_cast<const uint4*>(in + base + 16 * v);
  for (uint32_t k = t; k < (1u << SC_TBITS); k += SC_T) table[k] = 0xffffffffu;
  __syncthreads();
  for (uint32_t i = t; i + 4 <= len; i += SC_T) atomicMin(&table[sc_hash(lds32u(frag + i))], i);
  __syncthreads();
  const uint32_t s0 = t * SC_SLICE, s1 = min(len, s0 + SC_SLICE);
  uint8_t* d = obuf + t * SC_OMAX;
  uint32_t o = 0;
  if (s0 < s1) {
    uint32_t ip = s0, lit = s0;
    while (ip + 4 <= s1) {
      const uint32_t cur = lds32u(frag + ip);
      const uint32_t cand = table[sc_hash(cur)];
      if (cand < ip && lds32u(frag + cand) == cur) {
        const uint32_t maxm = s1 - ip;
        uint32_t m = 4;
        while (m + 4 <= maxm && lds32u(frag + cand + m) == lds32u(frag + ip + m)) m += 4;
        while (m < maxm && frag[cand + m] == frag[ip + m]) ++m;
        if (ip > lit) o = emit_literal(d, o, frag + lit, ip - lit);
        o = emit_copy(d, o, ip - cand, m);
        ip += m;
        lit = ip;
      } else {
        ++ip;
      }
    }
    if (s1 > lit) o = emit_literal(d, o, frag + lit, s1 - lit);
  }
  // block exclusive scan of the slot sizes
  const uint32_t lane = t & 63, wv = t >> 6;
  uint32_t incl = o;
  for (int k = 1; k < 64; k <<= 1) {
    const uint32_t y = __shfl_up(incl, k, 64);
    if (lane >= uint32_t(k)) incl += y;
  }
  if (lane == 63) wsum[wv] = incl;
  __syncthreads();
  uint32_t woff = 0, total = 0;
  for (uint32_t w = 0; w < SC_T / 64; ++w) {
    woff += w < wv ? wsum[w] : 0u;
    total += wsum[w];
  }
  const uint32_t at = woff + incl - o;
  for (uint32_t k = 0; k < o; ++k) cbuf[at + k] = d[k];
  __syncthreads();
  uint8_t* dst = out + uint64_t(f) * SC_SLOT;
  for (uint32_t v = t; v < (total + 15) / 16; v += SC_T)
    *reinterpret_cast<uint4*>(dst + 16 * v) = *reinterpret_cast<const uint4*>(cbuf + 16 * v);
  if (t == 0) out_len[f] = total;
}

// Fragment f's elements to dst + off[f] (off: exclusive scan of out_len).
__global__ void __launch_bounds__(256) k_snap_gather(const uint8_t* __restrict__ slots, const uint32_t* __restrict__ len,
                                                     const uint64_t* __restrict__ off, uint8_t* __restrict__ dst) {
  const uint32_t f = blockIdx.x;
  const uint8_t* s = slots + uint64_t(f) * SC_SLOT;
  uint8_t* d = dst + off[f];
  for (uint32_t k = threadIdx.x; k < len[f]; k += 256) d[k] = s[k];
}
}  // namespace dev

uint64_t snap_compress_slot() { return dev::SC_SLOT; }
uint64_t snap_compress_frag() { return dev::SC_FRAG; }

void launch_snap_compress(const uint8_t* in, uint64_t n, uint8_t* out, uint32_t* out_len, hipStream_t st) {
  const uint32_t nfrag = uint32_t((n + dev::SC_FRAG - 1) / dev::SC_FRAG);
  if (nfrag) DR_LAUNCH(dev::k_snap_compress, dim3(nfrag), dim3(dev::SC_T), 0, st, in, n, out, out_len);
}

void launch_snap_gather(const uint8_t* slots, const uint32_t* len, const uint64_t* off, uint32_t nfrag, uint8_t* dst,
                        hipStream_t st) {
  if (nfrag) DR_LAUNCH(dev::k_snap_gather, dim3(nfrag), dim3(256), 0, st, slots, len, off, dst);
}

}  // namespace dr
