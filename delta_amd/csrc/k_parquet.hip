// K2b: Parquet page decode on the GPU (replaces Spark's ParquetFileFormat / parquet-mr record
// assembly over the checkpoint, D/DeltaLogFileIndex.scala:68, D/Snapshot.scala:244-263).
//
// Pages are planned on the host (footer + page headers) and inflated by k_snappy.hip. Then one
// wave per page decodes:
//  * dictionary pages -> a pool of (address, length) or int64 values;
//  * v1/v2 data pages of the flat file-action columns (add.path, add.size, remove.path,
//    remove.deletionTimestamp): RLE/bit-packed definition levels expanded run-by-run by the whole
//    wave into LDS, value ranks by ballot prefix counts, values from PLAIN (fixed width, or
//    length-prefixed byte arrays walked through a 1 KiB register window with readlane) or
//    PLAIN_DICTIONARY/RLE_DICTIONARY indices.
#include "dev_common.h"
#include "kernels.h"

namespace dr {
namespace dev {

enum PqErr : uint32_t { PQE_SNAPPY = 1, PQE_LEVELS = 2, PQE_VALUES = 3, PQE_DICT = 4, PQE_ENCODING = 5 };

__device__ __forceinline__ void set_err(uint32_t* e, uint32_t code) { atomicCAS(e, 0u, code); }

__device__ __forceinline__ int level_width(int max_level) {
  int w = 0;
  while ((1 << w) <= max_level) ++w;
  return max_level == 0 ? 0 : w;
}

// ---- wave-wide RLE / bit-packed hybrid expansion ---------------------------------------------------
// All lanes hold the same (uniform) state; each call expands the next n values into dst[0..n).
struct Rle {
  const uint8_t* p;
  const uint8_t* end;
  int width;
  uint32_t left;
  bool packed;
  uint32_t value;
  const uint8_t* pk;   // packed-run data
  uint64_t bit;        // bit offset into pk
  bool bad;

  __device__ void init(const uint8_t* b, const uint8_t* e, int w) {
    p = b; end = e; width = w; left = 0; packed = false; value = 0; pk = nullptr; bit = 0; bad = false;
  }
  __device__ bool next_run() {
    uint64_t h = 0;
    int s = 0;
    for (;;) {
      if (p >= end || s > 35) { bad = true; return false; }
      const uint8_t b = *p++;
      h |= uint64_t(b & 0x7f) << s;
      s += 7;
      if (!(b & 0x80)) break;
    }
    if (h & 1) {
      packed = true;
      left = uint32_t(h >> 1) * 8;
      pk = p;
      bit = 0;
      const uint64_t bytes = (uint64_t(left) * uint64_t(width) + 7) / 8;
      p += bytes;  // may run past `end` for a final short group: values beyond are never read
    } else {
      packed = false;
      left = uint32_t(h >> 1);
      value = 0;
      for (int b = 0; b < (width + 7) / 8; ++b) {
        if (p >= end) { bad = true; return false; }
        value |= uint32_t(*p++) << (8 * b);
      }
    }
    if (left == 0 && !packed) return next_run();
    return true;
  }
  // Threads tid (of nt, all holding the same state) expand the next n values into dst[0..n).
  template <typename T>
  __device__ void expand(T* dst, uint32_t n, int tid, int nt = 64) {
    uint32_t done = 0;
    while (done < n) {
      if (left == 0 && !next_run()) return;
      const uint32_t take = min(left, n - done);
      if (!packed) {
        for (uint32_t i = tid; i < take; i += nt) dst[done + i] = T(value);
      } else {
        const uint64_t mask = width >= 32 ? 0xffffffffull : ((1ull << width) - 1);
        for (uint32_t i = tid; i < take; i += nt) {
          const uint64_t b = bit + uint64_t(i) * width;
          dst[done + i] = T((load_u64(pk + (b >> 3)) >> (b & 7)) & mask);
        }
        bit += uint64_t(take) * width;
      }
      left -= take;
      done += take;
    }
  }
};

// ---- length-prefixed BYTE_ARRAY walker over a 1 KiB register window ---------------------------------
// Lane l holds bytes [wb + 16 l, wb + 16 l + 16). The walk position is wave-uniform; dwords are read
// with readlane, so one step costs a handful of scalar-latency instructions, not an LDS/L2 round trip.
struct ByteArrayWalker {
  const uint8_t* base;   // page values start (any alignment)
  const uint8_t* end;
  const uint8_t* wb;     // window base (16-byte aligned)
  uint4 w;
  uint64_t pos;          // offset of the next value's length prefix from `base`
  bool bad;

  __device__ void load_window(const uint8_t* at, int lane) {
    wb = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(at) & ~uintptr_t(15));
    w = *reinterpret_cast<const uint4*>(wb + 16 * lane);
  }
  __device__ __forceinline__ uint32_t dword(uint32_t di) {
    const uint32_t which = di & 3;
    const uint32_t v = which == 0 ? w.x : which == 1 ? w.y : which == 2 ? w.z : w.w;
    return uint32_t(__builtin_amdgcn_readlane(int(v), int(di >> 2)));
  }
  __device__ void init(const uint8_t* b, const uint8_t* e, int lane) {
    base = b; end = e; pos = 0; bad = false;
    load_window(b, lane);
  }
  // Next value: returns its address and length; wave-uniform.
  __device__ __forceinline__ const uint8_t* next(uint32_t* len, int lane) {
    const uint8_t* at = base + pos;
    if (at + 4 > end) { bad = true; *len = 0; return at; }
    uint32_t r = uint32_t(at - wb);
    if (r + 8 > 1024) {
      load_window(at, lane);
      r = uint32_t(at - wb);
    }
    const uint32_t di = r >> 2;
    const uint32_t l = __builtin_amdgcn_alignbyte(dword(di + 1), dword(di), r & 3);
    if (uint64_t(end - at - 4) < l) { bad = true; *len = 0; return at; }
    *len = l;
    pos += 4 + uint64_t(l);
    return at + 4;
  }
};

// ---- parallel boundaries of length-prefixed BYTE_ARRAY values -----------------------------------------
// PLAIN BYTE_ARRAY values are [u32 len][bytes]...: a serial chain. For strings without NUL bytes and
// lengths < 64 KiB every true boundary p has b[p+2] == b[p+3] == 0 while no position inside a string
// does (paths are URI strings). A candidate is a position with two zero bytes at +2/+3 whose value
// fits the page and whose successor is a candidate or the region end. Pages are cut into 4 KiB tiles
// (all pages' tiles in one grid): tiles count their candidates, a global scan orders them, tiles
// write them, and the chain is then VALIDATED -- B[0] = start, B[k+1] = B[k] + 4 + len(B[k]), the
// last value ends at the region end -- which proves B equals the true chain. Any failure (NUL
// bytes, huge values, corrupt data) leaves ba_ok = 0 and the serial walker decodes the page.
constexpr int BA_T = 256;
constexpr uint32_t BA_POS = 64;               // positions per thread
constexpr uint32_t BA_TILE = BA_T * BA_POS;   // region bytes per tile (workgroup)

__device__ __forceinline__ bool ba_region(const PageDesc& pg, const uint8_t** b, const uint8_t** e) {
  const uint8_t* p = reinterpret_cast<const uint8_t*>(pg.dst);
  const uint8_t* end = p + pg.usize;
  if (pg.kind == PG_DATA_V2) {
    p += pg.v2_rep_len + pg.v2_def_len;
  } else if (pg.kind != PG_DICT) {
    for (int sec = 0; sec < 2; ++sec) {  // repetition levels, then definition levels
      if ((sec == 0 ? pg.max_rep : pg.max_def) <= 0) continue;
      if (end - p < 4) return false;
      const uint32_t l = load_u32(p);
      if (uint64_t(end - p - 4) < l) return false;
      p += 4 + l;
    }
  }
  *b = p;
  *e = end;
  return true;
}

__device__ __forceinline__ bool ba_cand(const uint8_t* b, uint64_t S, uint64_t p, uint64_t* next) {
  if (p + 4 > S) return false;
  const uint32_t w = load_u32(b + p);
  if (w >> 16) return false;  // bytes +2/+3 must be zero
  const uint64_t nx = p + 4 + w;
  if (nx > S || (w && !b[p + 4])) return false;
  *next = nx;
  return true;
}

__device__ __forceinline__ uint32_t zero_nibble(uint32_t v) {  // bit k: byte k of v is zero
  const uint32_t zb = ~(((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v | 0x7F7F7F7Fu);  // 0x80 per zero byte
  uint32_t g = zb >> 7;
  g |= g >> 7;
  g |= g >> 14;
  return g & 0xFu;
}

// r06: the chain through the kept candidates (each one's successor is the next) is checked in
// k_ba_count, where the successors are at hand, and the tiles' ends in k_ba_write (ba_link); a third
// pass over the ranks (k_ba_check) did it before.
constexpr uint32_t BA_NONE = 0xFFFFFFFFu;

// Bit j of the result: region offset q0 + j is a kept candidate. The thread's 64 positions start
// 16-byte aligned in absolute address; their +1..+4 bytes come from five 16-byte loads.
__device__ __forceinline__ uint64_t ba_kept(const uint8_t* b, uint64_t S, int64_t q0) {
  if (q0 + int64_t(BA_POS) <= 0 || q0 >= int64_t(S)) return 0ull;
  const uint4* a4 = reinterpret_cast<const uint4*>(b + q0);  // 16-byte aligned by construction
  uint64_t z0 = 0;
  uint32_t z1 = 0;
#pragma unroll
  for (int v = 0; v < 5; ++v) {
    const uint4 x = a4[v];
    const uint32_t m = zero_nibble(x.x) | (zero_nibble(x.y) << 4) | (zero_nibble(x.z) << 8) | (zero_nibble(x.w) << 12);
    if (v < 4) z0 |= uint64_t(m) << (16 * v);
    else z1 = m;
  }
  auto zs = [&](int k) { return (z0 >> k) | (uint64_t(z1) << (64 - k)); };
  // A true boundary's zero run (the length's high bytes) ends at +3: the string's first byte is
  // non-zero unless the string is empty (all four length bytes zero). This drops the shifted
  // candidates inside the run (p-1 when len < 256), which would otherwise survive the successor
  // check by chance.
  const uint64_t cm = zs(2) & zs(3) & (~zs(4) | (z0 & zs(1)));
  uint64_t kept = 0;
  for (uint64_t m = cm; m;) {
    const int j = __builtin_ctzll(m);
    m &= m - 1;
    const int64_t p = q0 + j;
    if (p < 0) continue;
    uint64_t nx, nn;
    if (ba_cand(b, S, uint64_t(p), &nx) && (nx == S || ba_cand(b, S, nx, &nn))) kept |= 1ull << j;
  }
  return kept;
}

struct BaTile {
  const PageDesc* pg;
  const uint8_t* b;
  uint64_t S;
  int64_t q0;      // region offset of this thread's first position
  bool ok;
};
__device__ __forceinline__ BaTile ba_tile(const ParquetArgs& a, uint32_t tile) {
  const uint2 tp = a.ba_tiles[tile];
  BaTile r;
  r.pg = &a.pages[tp.x];
  const uint8_t *b, *e;
  r.ok = ba_region(*r.pg, &b, &e);
  r.b = b;
  r.S = r.ok ? uint64_t(e - b) : 0;
  const int64_t lead = int64_t(reinterpret_cast<uintptr_t>(b) & 15);  // tiles are absolute-aligned
  r.q0 = -lead + int64_t(tp.y) * BA_TILE + int64_t(BA_POS) * int64_t(threadIdx.x);
  return r;
}

__device__ __forceinline__ uint32_t block_sum(uint32_t v, uint32_t* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t s = 0;
  for (int k = 0; k < BA_T / 64; ++k) s += red[k];
  return s;
}

// The tile's bytes (+ a margin for the successors of its last candidates) staged in LDS with
// coalesced 16-byte loads: every candidate check reads the length at the candidate and at its
// successor, two dependent reads that went to L1/L2 (the kernel waited on memory 73 % of its wave
// cycles, PMC r02).
constexpr uint32_t BA_MARGIN = 4096;
struct BaStage {
  const uint32_t* w;  // staged words; byte k = region offset t0 + k
  int64_t t0;
  uint64_t n;         // staged bytes
};
__device__ __forceinline__ uint32_t stage_u32(const BaStage& st, uint64_t k) {  // bytes k .. k+3
  const uint32_t i = uint32_t(k >> 2), sh = uint32_t(k & 3);
  return __builtin_amdgcn_alignbyte(st.w[i + 1], st.w[i], sh);
}
__device__ __forceinline__ uint8_t stage_u8(const BaStage& st, uint64_t k) {
  return uint8_t(st.w[k >> 2] >> (8 * (k & 3)));
}
__device__ __forceinline__ bool ba_cand_st(const uint8_t* b, uint64_t S, uint64_t p, uint64_t* next, const BaStage& st) {
  if (p + 4 > S) return false;
  const uint64_t k = uint64_t(int64_t(p) - st.t0);
  const bool in = k + 8 <= st.n;
  const uint32_t w = in ? stage_u32(st, k) : load_u32(b + p);
  if (w >> 16) return false;  // bytes +2/+3 must be zero
  const uint64_t nx = p + 4 + w;
  if (nx > S || (w && !(in ? stage_u8(st, k + 4) : b[p + 4]))) return false;
  *next = nx;
  return true;
}
__device__ __forceinline__ uint64_t ba_kept_st(const uint8_t* b, uint64_t S, int64_t q0, const BaStage& st) {
  if (q0 + int64_t(BA_POS) <= 0 || q0 >= int64_t(S)) return 0ull;
  const uint4* a4 = reinterpret_cast<const uint4*>(st.w) + (q0 - st.t0) / 16;
  uint64_t z0 = 0;
  uint32_t z1 = 0;
#pragma unroll
  for (int v = 0; v < 5; ++v) {
    const uint4 x = a4[v];
    const uint32_t m = zero_nibble(x.x) | (zero_nibble(x.y) << 4) | (zero_nibble(x.z) << 8) | (zero_nibble(x.w) << 12);
    if (v < 4) z0 |= uint64_t(m) << (16 * v);
    else z1 = m;
  }
  auto zs = [&](int k) { return (z0 >> k) | (uint64_t(z1) << (64 - k)); };
  const uint64_t cm = zs(2) & zs(3) & (~zs(4) | (z0 & zs(1)));
  uint64_t kept = 0;
  for (uint64_t m = cm; m;) {
    const int j = __builtin_ctzll(m);
    m &= m - 1;
    const int64_t p = q0 + j;
    if (p < 0) continue;
    uint64_t nx, nn;
    if (ba_cand_st(b, S, uint64_t(p), &nx, st) && (nx == S || ba_cand_st(b, S, nx, &nn, st))) kept |= 1ull << j;
  }
  return kept;
}

// T1: kept candidates per tile; each thread's 64-bit kept mask is stored for T2. The chain is checked
// here, where the successors are at hand: inside each thread (BaChain), from each thread's last kept
// value to the next thread's first, and the tile's ends are left for T2 (ba_link).
__global__ void __launch_bounds__(BA_T) k_ba_count(ParquetArgs a) {
  __shared__ uint32_t red[BA_T / 64];
  __shared__ uint32_t tfirst[BA_T], tsucc[BA_T];
  __shared__ unsigned long long wbal[BA_T / 64];
  __shared__ uint32_t tile_bad;
  __shared__ __attribute__((aligned(16))) uint32_t stw[(BA_TILE + BA_MARGIN) / 4 + 8];
  const BaTile tl = ba_tile(a, blockIdx.x);
  // stage [t0, t0 + staged) of the region: t0 = thread 0's first position (16-byte aligned in
  // absolute address), up to the region end + 16 (the arena pads every page body by 16 bytes)
  BaStage st{stw, tl.q0 - int64_t(BA_POS) * int64_t(threadIdx.x), 0};
  if (tl.ok) {
    const int64_t hi = min(st.t0 + int64_t(BA_TILE + BA_MARGIN), int64_t(tl.S) + 16);
    const uint64_t nb = hi > st.t0 ? uint64_t(hi - st.t0) & ~uint64_t(15) : 0;
    const uint4* g4 = reinterpret_cast<const uint4*>(tl.b + st.t0);
    uint4* s4 = reinterpret_cast<uint4*>(stw);
    // every load of the thread in flight before any is written (global loads: through the page
    // pointer the compiler had emitted flat loads, each waited on before the next was issued)
    constexpr uint32_t PER = ((BA_TILE + BA_MARGIN) / 16 + BA_T - 1) / BA_T;
    const uint32_t nv = uint32_t(nb / 16);
    if (nv) {
      uint4 v[PER];
#pragma unroll
      for (uint32_t k = 0; k < PER; ++k) v[k] = gload16(g4 + min(threadIdx.x + k * BA_T, nv - 1));
#pragma unroll
      for (uint32_t k = 0; k < PER; ++k)
        if (threadIdx.x + k * BA_T < nv) s4[threadIdx.x + k * BA_T] = v[k];
    }
    st.n = nb;
  }
  if (threadIdx.x == 0) tile_bad = 0;
  __syncthreads();
  const uint64_t km = tl.ok ? (st.n >= uint64_t(tl.q0 - st.t0) + 80 ? ba_kept_st(tl.b, tl.S, tl.q0, st)
                                                                    : ba_kept(tl.b, tl.S, tl.q0))
                            : 0ull;
  a.ba_kept[uint64_t(blockIdx.x) * BA_T + threadIdx.x] = km;
  // the chain through this thread's kept values: each one's successor (its length read again, from
  // the stage when it lies there) must be the next kept one
  auto succ = [&](uint64_t p) -> uint64_t {
    const uint64_t k = p - uint64_t(st.t0);
    return p + 4 + (k + 8 <= st.n ? stage_u32(st, k) : load_u32(tl.b + p));
  };
  const uint32_t t = threadIdx.x, wv = t >> 6, ln = t & 63u;
  uint32_t cfirst = BA_NONE, clsucc = BA_NONE;
  bool cbad = false;
  if (km) {
    uint64_t m = km;
    const uint64_t p0 = uint64_t(tl.q0 + __builtin_ctzll(m));
    m &= m - 1;
    uint64_t nx = succ(p0);
    while (m) {
      const uint64_t p = uint64_t(tl.q0 + __builtin_ctzll(m));
      m &= m - 1;
      cbad |= nx != p;
      nx = succ(p);
    }
    cfirst = uint32_t(p0);
    clsucc = uint32_t(nx);
  }
  tfirst[t] = cfirst;
  tsucc[t] = clsucc;
  const unsigned long long bal = __ballot(km != 0ull);
  if (ln == 0) wbal[wv] = bal;
  __syncthreads();
  if (km) {
    // the next thread holding a kept value (a value longer than a thread's 64 bytes skips threads)
    uint32_t u = BA_NONE;
    const unsigned long long above = ln == 63 ? 0ull : (wbal[wv] >> (ln + 1)) << (ln + 1);
    if (above) {
      u = wv * 64 + uint32_t(__builtin_ctzll(above));
    } else {
      for (uint32_t x = wv + 1; x < BA_T / 64; ++x)
        if (wbal[x]) { u = x * 64 + uint32_t(__builtin_ctzll(wbal[x])); break; }
    }
    if (cbad || (u != BA_NONE && tfirst[u] != clsucc)) tile_bad = 1;
  }
  // the tile's ends: its first kept value, and the successor of its last
  uint32_t* link = a.ba_link + 3ull * blockIdx.x;
  if (t == 0) {
    int lo = -1, hi = -1;
    for (uint32_t x = 0; x < BA_T / 64; ++x)
      if (wbal[x]) {
        if (lo < 0) lo = int(x * 64 + __builtin_ctzll(wbal[x]));
        hi = int(x * 64 + 63 - __builtin_clzll(wbal[x]));
      }
    link[0] = lo < 0 ? BA_NONE : tfirst[lo];
    link[1] = hi < 0 ? BA_NONE : tsucc[hi];
  }
  const uint32_t s = block_sum(uint32_t(__builtin_popcountll(km)), red);
  if (threadIdx.x == 0) {
    a.ba_tile_cnt[blockIdx.x] = s;
    if (a.ba_tiles[blockIdx.x].y == 0) a.ba_ok[tl.pg->ba_slot] = tl.ok ? 1u : 0u;
    link[2] = tile_bad;
  }
}

// T2: kept candidates written in order (page-relative rank = scanned tile offset + block prefix).
__global__ void __launch_bounds__(BA_T) k_ba_write(ParquetArgs a) {
  __shared__ uint32_t wsum[BA_T / 64];
  const BaTile tl = ba_tile(a, blockIdx.x);
  if (!tl.ok) return;
  const PageDesc pg = *tl.pg;
  uint64_t km = a.ba_kept[uint64_t(blockIdx.x) * BA_T + threadIdx.x];
  const uint32_t c = uint32_t(__builtin_popcountll(km));
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t incl = c;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  if (lane == 63) wsum[wv] = incl;
  __syncthreads();
  uint32_t woff = 0;
  for (int k = 0; k < wv; ++k) woff += wsum[k];
  const uint32_t first = uint32_t(pg.hit_base);  // the page's first tile
  const uint64_t rank0 = a.ba_tile_off[blockIdx.x] - a.ba_tile_off[first] + woff + incl - c;
  const uint64_t cap = pg.usize / 4 + 2;
  const uint64_t boff = uint64_t(tl.b - reinterpret_cast<const uint8_t*>(pg.dst));
  uint32_t* vals = a.ba_vals + pg.ba_base;
  uint64_t o = rank0;
  while (km) {
    const int j = __builtin_ctzll(km);
    km &= km - 1;
    if (o < cap) vals[o] = uint32_t(uint64_t(tl.q0 + j) + boff);
    ++o;
  }
  // the page's last tile publishes the count
  const bool last = blockIdx.x + 1 == a.nba_tiles || a.ba_tiles[blockIdx.x + 1].x != a.ba_tiles[blockIdx.x].x;
  if (threadIdx.x == 0 && last)
    a.ba_count[pg.ba_slot] = uint32_t(a.ba_tile_off[blockIdx.x + 1] - a.ba_tile_off[first]);
  // the chain's ends (k_ba_count checked it inside the tile): the page's first value starts at
  // region offset 0, the successor of the tile's last value is the first value of the page's next
  // tile holding one, or the region end; a page whose values exceed the rank list's room fails too
  if (threadIdx.x == 0) {
    const uint32_t* L = a.ba_link + 3ull * blockIdx.x;
    bool bad = L[2] != 0;
    if (blockIdx.x == first) bad |= tl.S > 0 && L[0] != 0;
    if (L[1] != BA_NONE) {
      uint64_t want = tl.S;
      for (uint32_t u = blockIdx.x + 1; u < a.nba_tiles && a.ba_tiles[u].x == a.ba_tiles[blockIdx.x].x; ++u)
        if (a.ba_link[3ull * u] != BA_NONE) { want = a.ba_link[3ull * u]; break; }
      bad |= uint64_t(L[1]) != want;
    }
    if (last) bad |= a.ba_tile_off[blockIdx.x + 1] - a.ba_tile_off[first] > cap;
    if (bad) a.ba_ok[pg.ba_slot] = 0;
  }
}

// ---- dictionary pages --------------------------------------------------------------------------------
// Pages whose values are all independent of each other (byte arrays with validated parallel
// boundaries, fixed-width values) are spread over DICT_SLICES workgroups of 256 lanes each; the
// rest (the serial byte-array walk) take one wave per page in k_pq_dict.
constexpr uint32_t DICT_SLICES = 16;
__device__ __forceinline__ bool dict_fast(const ParquetArgs& a, const PageDesc& pg) {
  if (pg.phys == 6) return pg.ba && a.ba_ok[pg.ba_slot] && a.ba_count[pg.ba_slot] == pg.num_values;
  return (pg.phys == 2 || pg.phys == 1) && uint64_t(pg.num_values) * (pg.phys == 2 ? 8 : 4) <= pg.usize;
}

__global__ void __launch_bounds__(256) k_pq_dict_fast(ParquetArgs a) {
  const PageDesc pg = a.pages[blockIdx.x];
  if (pg.kind != PG_DICT || !dict_fast(a, pg)) return;
  const uint8_t* p = reinterpret_cast<const uint8_t*>(pg.dst);
  const uint32_t stride = 256 * DICT_SLICES;
  if (pg.phys == 6) {
    const uint32_t* vals = a.ba_vals + pg.ba_base;  // boundaries found in parallel (k_ba_*)
    for (uint32_t k = blockIdx.y * 256 + threadIdx.x; k < pg.num_values; k += stride) {
      const uint32_t off = vals[k];
      a.dict_ptr[pg.dict_base + k] = reinterpret_cast<uint64_t>(p + off + 4);
      a.dict_len[pg.dict_base + k] = load_u32(p + off);
    }
    return;
  }
  const bool w8 = pg.phys == 2;
  for (uint32_t k = blockIdx.y * 256 + threadIdx.x; k < pg.num_values; k += stride)
    a.dict_ptr[pg.dict_base + k] = w8 ? load_u64(p + 8ull * k) : uint64_t(int64_t(int32_t(load_u32(p + 4ull * k))));
}

__global__ void __launch_bounds__(64) k_pq_dict(ParquetArgs a) {
  const uint32_t i = blockIdx.x;
  if (i >= a.npages) return;
  const PageDesc pg = a.pages[i];
  if (pg.kind != PG_DICT) return;
  const int lane = threadIdx.x;
  const uint8_t* p = reinterpret_cast<const uint8_t*>(pg.dst);
  const uint8_t* end = p + pg.usize;
  if (dict_fast(a, pg)) return;  // k_pq_dict_fast
  if (pg.phys == 6) {  // BYTE_ARRAY: chain walk
    __shared__ uint64_t sp[64];
    __shared__ uint32_t sl[64];
    ByteArrayWalker wk;
    wk.init(p, end, lane);
    for (uint32_t k0 = 0; k0 < pg.num_values; k0 += 64) {
      const uint32_t cnt = min(64u, pg.num_values - k0);
      for (uint32_t k = 0; k < cnt; ++k) {
        uint32_t l;
        const uint8_t* v = wk.next(&l, lane);
        if (lane == 0) { sp[k] = reinterpret_cast<uint64_t>(v); sl[k] = l; }
      }
      if (wk.bad) { if (lane == 0) set_err(a.error, PQE_DICT); return; }
      __syncthreads();
      if (uint32_t(lane) < cnt) {
        a.dict_ptr[pg.dict_base + k0 + lane] = sp[lane];
        a.dict_len[pg.dict_base + k0 + lane] = sl[lane];
      }
      __syncthreads();
    }
    return;
  }
  const uint32_t width = pg.phys == 2 ? 8 : pg.phys == 1 ? 4 : 0;
  if (!width) { if (lane == 0) set_err(a.error, PQE_ENCODING); return; }
  if (uint64_t(pg.num_values) * width > pg.usize) { if (lane == 0) set_err(a.error, PQE_DICT); return; }
  for (uint32_t k = lane; k < pg.num_values; k += 64) {
    a.dict_ptr[pg.dict_base + k] = width == 8 ? load_u64(p + 8ull * k)
                                              : uint64_t(int64_t(int32_t(load_u32(p + 4ull * k))));
  }
}

// ---- data pages ----------------------------------------------------------------------------------------
// One 256-lane workgroup per page, 1024 levels per segment: levels expanded run by run by the whole
// workgroup into LDS, value ranks by wave ballots + a workgroup prefix, then every lane writes rows.
// The serial byte-array walk (pages whose boundaries were not validated) runs on wave 0.
constexpr uint32_t SEG = 1024;   // levels per segment
constexpr int PQD_T = 256;

__global__ void __launch_bounds__(PQD_T) k_pq_data(ParquetArgs a) {
  const uint32_t pi = blockIdx.x;
  if (pi >= a.npages) return;
  // the descriptor copied once (read through a reference, each field was re-loaded after every
  // store the compiler could not prove it does not alias: serial loads inside the loops)
  const PageDesc pg = a.pages[pi];
  if (pg.kind == PG_DICT) return;
  __shared__ uint8_t defs[SEG];
  __shared__ uint8_t reps[SEG];
  __shared__ uint32_t idxs[SEG];
  __shared__ uint64_t vptr[SEG];
  __shared__ uint32_t vlen[SEG];
  __shared__ uint32_t wcnt[PQD_T / 64];
  __shared__ uint32_t s_bad;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const FlatColumn col = a.cols[pg.col];
  const uint8_t* p = reinterpret_cast<const uint8_t*>(pg.dst);
  const uint8_t* end = p + pg.usize;
  Rle defr, repr;
  defr.init(p, p, 0);
  repr.init(p, p, 0);
  if (pg.kind == PG_DATA_V2) {
    if (pg.max_rep > 0) repr.init(p, p + pg.v2_rep_len, level_width(pg.max_rep));
    defr.init(p + pg.v2_rep_len, p + pg.v2_rep_len + pg.v2_def_len, level_width(pg.max_def));
    p += pg.v2_rep_len + pg.v2_def_len;
  } else if (pg.max_rep > 0 || pg.max_def > 0) {
    if (pg.max_rep > 0) {
      if (end - p < 4) { if (tid == 0) set_err(a.error, PQE_LEVELS); return; }
      const uint32_t l = load_u32(p);
      p += 4;
      if (uint64_t(end - p) < l) { if (tid == 0) set_err(a.error, PQE_LEVELS); return; }
      repr.init(p, p + l, level_width(pg.max_rep));
      p += l;
    }
  }
  if (pg.kind != PG_DATA_V2 && pg.max_def > 0) {
    if (end - p < 4) { if (tid == 0) set_err(a.error, PQE_LEVELS); return; }
    const uint32_t l = load_u32(p);
    p += 4;
    if (uint64_t(end - p) < l) { if (tid == 0) set_err(a.error, PQE_LEVELS); return; }
    defr.init(p, p + l, level_width(pg.max_def));
    p += l;
  }
  const bool dict = pg.encoding == 2 || pg.encoding == 8;
  const bool rle_bool = pg.encoding == 3 && pg.phys == 0;
  Rle ir;
  ir.init(p, p, 0);
  if (dict) {
    if (pg.dict < 0) { if (tid == 0) set_err(a.error, PQE_DICT); return; }
    const int w = p < end ? *p : 0;
    ir.init(p + 1, end, w);
  } else if (rle_bool) {
    ir.init(p + 4, end, 1);
  } else if (pg.encoding != 0) {
    if (tid == 0) set_err(a.error, PQE_ENCODING);
    return;
  }
  const uint32_t dict_base = dict ? a.pages[pg.dict].dict_base : 0;
  const uint32_t dict_n = dict ? a.pages[pg.dict].num_values : 0;
  const uint32_t width = pg.phys == 2 ? 8 : pg.phys == 1 ? 4 : 0;
  ByteArrayWalker wk;
  const bool ba_fast = pg.phys == 6 && !dict && pg.ba && a.ba_ok[pg.ba_slot];
  const uint32_t* ba_vals = a.ba_vals + pg.ba_base;
  const uint32_t ba_n = ba_fast ? a.ba_count[pg.ba_slot] : 0;
  const uint8_t* body = reinterpret_cast<const uint8_t*>(pg.dst);
  const bool walk = pg.phys == 6 && !dict && !ba_fast;
  if (walk && wv == 0) wk.init(p, end, lane);
  if (tid == 0) s_bad = 0;
  uint64_t vbase = 0;  // values consumed before this segment (PLAIN fixed / boolean)
  for (uint32_t s0 = 0; s0 < pg.num_values; s0 += SEG) {
    const uint32_t n = min(SEG, pg.num_values - s0);
    if (pg.max_rep > 0) {
      repr.expand(reps, n, tid, PQD_T);
      if (repr.bad) { if (tid == 0) set_err(a.error, PQE_LEVELS); return; }
    }
    if (pg.max_def > 0) {
      defr.expand(defs, n, tid, PQD_T);
      if (defr.bad) { if (tid == 0) set_err(a.error, PQE_LEVELS); return; }
    } else {
      for (uint32_t i = tid; i < n; i += PQD_T) defs[i] = 0;
    }
    __syncthreads();
    // value rank of each level within the segment
    uint32_t nv = 0;
    for (uint32_t b = 0; b < n; b += PQD_T) {
      const uint32_t i = b + tid;
      const bool isv = i < n && int(defs[i]) == pg.max_def;
      const unsigned long long m = __ballot(isv);
      if (lane == 0) wcnt[wv] = uint32_t(__popcll(m));
      __syncthreads();
      uint32_t before = nv, tot = 0;
      for (int k = 0; k < PQD_T / 64; ++k) {
        before += k < wv ? wcnt[k] : 0u;
        tot += wcnt[k];
      }
      if (isv) idxs[i] = before + uint32_t(__popcll(m & ((1ull << lane) - 1ull)));
      nv += tot;
      __syncthreads();
    }
    // values of this segment
    if (dict || rle_bool) {
      ir.expand(vlen, nv, tid, PQD_T);  // dictionary indices / booleans (reuse vlen as scratch)
      if (ir.bad) { if (tid == 0) set_err(a.error, dict ? PQE_DICT : PQE_VALUES); return; }
    } else if (ba_fast) {
      if (vbase + nv > ba_n) { if (tid == 0) set_err(a.error, PQE_VALUES); return; }
    } else if (walk) {
      if (wv == 0) {
        for (uint32_t k = 0; k < nv; ++k) {
          uint32_t l;
          const uint8_t* v = wk.next(&l, lane);
          if (lane == 0) { vptr[k] = reinterpret_cast<uint64_t>(v); vlen[k] = l; }
        }
        if (wk.bad && lane == 0) s_bad = 1;
      }
      __syncthreads();
      if (s_bad) { if (tid == 0) set_err(a.error, PQE_VALUES); return; }
    } else if (width) {
      if ((vbase + nv) * width > uint64_t(end - p)) { if (tid == 0) set_err(a.error, PQE_VALUES); return; }
    } else if (pg.phys == 0) {
      if ((vbase + nv + 7) / 8 > uint64_t(end - p)) { if (tid == 0) set_err(a.error, PQE_VALUES); return; }
    } else {
      if (tid == 0) set_err(a.error, PQE_ENCODING);
      return;
    }
    __syncthreads();
    for (uint32_t i = tid; i < n; i += PQD_T) {
      const uint64_t row = pg.row_base + s0 + i;
      const uint8_t d = defs[i];
      col.def[row] = d;
      if (pg.max_rep > 0) col.rep[row] = reps[i];
      if (int(d) != pg.max_def) continue;
      const uint32_t k = idxs[i];
      if (dict) {
        const uint32_t j = vlen[k];
        if (j >= dict_n) { set_err(a.error, PQE_DICT); continue; }
        if (pg.phys == 6) {
          col.sptr[row] = a.dict_ptr[dict_base + j];
          col.slen[row] = a.dict_len[dict_base + j];
        } else {
          col.ival[row] = int64_t(a.dict_ptr[dict_base + j]);
        }
      } else if (rle_bool) {
        col.ival[row] = vlen[k] & 1;
      } else if (ba_fast) {
        const uint32_t off = ba_vals[vbase + k];
        col.sptr[row] = reinterpret_cast<uint64_t>(body + off + 4);
        col.slen[row] = load_u32(body + off);
      } else if (pg.phys == 6) {
        col.sptr[row] = vptr[k];
        col.slen[row] = vlen[k];
      } else if (width == 8) {
        col.ival[row] = int64_t(load_u64(p + 8 * (vbase + k)));
      } else if (width == 4) {
        col.ival[row] = int64_t(int32_t(load_u32(p + 4 * (vbase + k))));
      } else {
        const uint64_t b = vbase + k;
        col.ival[row] = (p[b >> 3] >> (b & 7)) & 1;
      }
    }
    vbase += nv;
    __syncthreads();
  }
}

// Checkpoint row -> action. unwrap priority add > remove (D/actions/actions.scala:523-541);
// rows holding neither are protocol/metaData/txn rows decoded on the host.
// r06: a wave's 64 paths lie together in a PLAIN page's body (~6 KiB): the wave copies that span into
// LDS with coalesced 16-byte loads and every lane hashes its path from there -- one lane per path
// reading its own bytes from global memory was 64 scattered requests per load (0.48 ms on config 3).
// Paths elsewhere (dictionary entries, a span crossing pages that lie apart) are read in place.
constexpr uint32_t ASM_T = 256, ASM_STAGE = 8192;
__device__ __forceinline__ void asm_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__global__ void __launch_bounds__(ASM_T) k_ckpt_assemble(CkptAssembleArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t stage[ASM_T / 64][ASM_STAGE + 32];
  const uint64_t r = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const bool live = r < a.nrows;  // (no early exit: the wave stages its paths together)
  const uint64_t idx = a.row_base + r;
  uint8_t kind = K_NONE, flags = F_FROM_CKPT;
  const uint8_t* path = nullptr;
  uint32_t plen = 0;
  int64_t size = 0, delts = 0;
  const int ad = live ? int(a.add_path.def[r]) : 0;
  const int rd = live && a.has_rm ? int(a.rm_path.def[r]) : 0;
  if (live && ad >= a.add_def) {
    kind = K_ADD;
    if (ad == a.add_path_max) {
      path = reinterpret_cast<const uint8_t*>(a.add_path.sptr[r]);
      plen = a.add_path.slen[r];
    } else {
      flags |= F_PATH_NULL;
    }
    if (a.add_size.def[r] == a.add_size_max) size = a.add_size.ival[r];
  } else if (live && a.has_rm && rd >= a.rm_def) {
    kind = K_REMOVE;
    if (rd == a.rm_path_max) {
      path = reinterpret_cast<const uint8_t*>(a.rm_path.sptr[r]);
      plen = a.rm_path.slen[r];
    } else {
      flags |= F_PATH_NULL;
    }
    if (a.rm_delts.def && a.rm_delts.def[r] == a.rm_delts_max) {
      delts = a.rm_delts.ival[r];
      flags |= F_HAS_DELTS;
    }
  }
  const bool hashed = (kind == K_ADD || kind == K_REMOVE) && !(flags & F_PATH_NULL);
  // the wave's span of path bytes
  uint64_t lo = hashed ? reinterpret_cast<uint64_t>(path) : ~0ull;
  uint64_t hi = hashed ? reinterpret_cast<uint64_t>(path) + plen : 0ull;
  for (int o = 32; o > 0; o >>= 1) {
    lo = min(lo, (uint64_t)__shfl_xor((unsigned long long)lo, o, 64));
    hi = max(hi, (uint64_t)__shfl_xor((unsigned long long)hi, o, 64));
  }
  const uint64_t a0 = lo & ~uint64_t(15);
  const bool staged = hi > lo && hi - a0 <= ASM_STAGE;  // wave-uniform
  uint8_t* stw = stage[threadIdx.x >> 6];
  if (staged) {
    const uint32_t nq = uint32_t((hi - a0 + 15) >> 4);
    const uint4* src = reinterpret_cast<const uint4*>(a0);  // (page bodies are padded by 16 bytes)
    for (uint32_t k = threadIdx.x & 63u; k < nq; k += 64) reinterpret_cast<uint4*>(stw)[k] = src[k];
    asm_wave_sync();
  }
  uint64_t key = 0;
  if (hashed) {
    const uint8_t* hp = staged ? stw + (reinterpret_cast<uint64_t>(path) - a0) : path;
    if (path_is_special(hp, plen)) {
      flags |= F_SPECIAL_PATH;
      atomicAdd(reinterpret_cast<unsigned long long*>(a.special_count), 1ull);
      atomicAdd(reinterpret_cast<unsigned long long*>(a.special_bytes), (unsigned long long)(plen + 8));
    } else {
      key = path_key(hp, plen);
    }
  }
  if (!live) return;
  a.act.kind[idx] = kind;
  a.act.flags[idx] = flags;
  a.act.key[idx] = key;
  a.act.path_ptr[idx] = reinterpret_cast<uint64_t>(path);
  a.act.path_len[idx] = plen;
  if (a.act.path_ref) a.act.path_ref[idx] = pack_ref(reinterpret_cast<uint64_t>(path), plen);
  a.act.size[idx] = size;
  a.act.delts[idx] = delts;
  a.act.src_off[idx] = r;
  a.act.src_len[idx] = 0;
}

}  // namespace dev

uint32_t ba_tile_bytes() { return dev::BA_TILE; }
void launch_ba_bounds(const ParquetArgs& a, hipStream_t st, ScanScratch scan_scratch) {
  if (!a.nba_tiles) return;
  DR_LAUNCH(dev::k_ba_count, dim3(a.nba_tiles), dim3(dev::BA_T), 0, st, a);
  launch_scan_u32(a.ba_tile_cnt, a.ba_tile_off, a.nba_tiles, scan_scratch, st);
  DR_LAUNCH(dev::k_ba_write, dim3(a.nba_tiles), dim3(dev::BA_T), 0, st, a);
}
void launch_pq_dict(const ParquetArgs& a, hipStream_t st) {
  if (!a.npages) return;
  DR_LAUNCH(dev::k_pq_dict_fast, dim3(a.npages, dev::DICT_SLICES), dim3(256), 0, st, a);
  DR_LAUNCH(dev::k_pq_dict, dim3(a.npages), dim3(64), 0, st, a);
}
void launch_pq_data(const ParquetArgs& a, hipStream_t st) {
  if (a.npages) DR_LAUNCH(dev::k_pq_data, dim3(a.npages), dim3(dev::PQD_T), 0, st, a);
}
void launch_ckpt_assemble(const CkptAssembleArgs& a, hipStream_t st) {
  if (a.nrows)
    DR_LAUNCH(dev::k_ckpt_assemble, dim3(unsigned((a.nrows + dev::ASM_T - 1) / dev::ASM_T)), dim3(dev::ASM_T), 0, st, a);
}

}  // namespace dr
