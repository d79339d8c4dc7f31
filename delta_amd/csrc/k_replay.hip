// K3/K4: path-hash partition + per-bucket last-writer-wins (replaces the shuffle
// `repartition(50, coalesce(add.path, remove.path))` + `sortWithinPartitions("file")` +
// InMemoryLogReplay.append/checkpoint, D/Snapshot.scala:103-110,
// D/actions/InMemoryLogReplay.scala:43-77).
//
// 16-byte records {xxh64(path) lo, hi, meta = action_index << 2 | class, add.size (32-bit field)}
// are partitioned on the top `bucket_bits` of the key: tiles count buckets in LDS into a bucket-major
// matrix whose exclusive scan gives each (bucket, tile) its output range, so the scatter needs no
// global atomics. Each bucket is then reduced by one workgroup: an LDS open-addressing table keyed by
// the full 64-bit key keeps atomicMax(meta), i.e. the action with the largest (version, line) ordinal
// wins -- exactly the reference's "last action per path" (action index order == input_file_name
// order, stable within a file). Every loser is byte-verified against its winner (k_bucket_verify), so
// a 64-bit collision is detected and that bucket is redone by the exact kernel (k_bucket_exact); an
// LDS-table overflow goes to the finer-grained reducer (k_bucket_reduce64). (r04: full 64-bit keys in
// the records -- the 45 key bits of r01-r03 collided about once per 16M-action replay and sent a bucket
// through k_bucket_reduce64 on every step.)
#include "dev_common.h"
#include "kernels.h"
#include "canon.h"

namespace dr {
namespace dev {

// ---- scans ----------------------------------------------------------------------------------------
constexpr int SCAN_T = 1024;

__global__ void __launch_bounds__(SCAN_T) k_scan_reduce(const uint32_t* in, uint64_t n, uint64_t* sums) {
  __shared__ uint64_t red[SCAN_T / 64];
  const uint64_t i = uint64_t(blockIdx.x) * SCAN_T + threadIdx.x;
  uint64_t v = i < n ? in[i] : 0;
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t s = 0;
    for (int k = 0; k < SCAN_T / 64; ++k) s += red[k];
    sums[blockIdx.x] = s;
  }
}

// Single-block exclusive scan of u64 values in place; data[n] receives the total.
__global__ void __launch_bounds__(SCAN_T) k_scan_single(uint64_t* data, uint64_t n) {
  __shared__ uint64_t wsum[SCAN_T / 64];
  __shared__ uint64_t carry;
  if (threadIdx.x == 0) carry = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (uint64_t base = 0; base < n; base += SCAN_T) {
    const uint64_t i = base + threadIdx.x;
    uint64_t v = i < n ? data[i] : 0, incl = v;
    for (int o = 1; o < 64; o <<= 1) {
      uint64_t t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    uint64_t woff = 0;
    for (int k = 0; k < wv; ++k) woff += wsum[k];
    const uint64_t c = carry;
    if (i < n) data[i] = c + woff + incl - v;
    __syncthreads();
    if (threadIdx.x == SCAN_T - 1) carry = c + woff + incl;
    __syncthreads();
  }
  if (threadIdx.x == 0) data[n] = carry;
}

__global__ void __launch_bounds__(SCAN_T) k_scan_apply(const uint32_t* in, uint64_t n, const uint64_t* sums,
                                                      uint64_t* out) {
  __shared__ uint64_t wsum[SCAN_T / 64];
  const uint64_t i = uint64_t(blockIdx.x) * SCAN_T + threadIdx.x;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t v = i < n ? in[i] : 0, incl = v;
  for (int o = 1; o < 64; o <<= 1) {
    uint64_t t = __shfl_up(incl, o, 64);
    if (lane >= o) incl += t;
  }
  if (lane == 63) wsum[wv] = incl;
  __syncthreads();
  uint64_t woff = 0;
  for (int k = 0; k < wv; ++k) woff += wsum[k];
  if (i < n) out[i] = sums[blockIdx.x] + woff + incl - v;
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) out[n] = sums[gridDim.x];
}

// ---- canonicalization of special paths (D/Snapshot.scala:317-328) -------------------------------
__global__ void k_canon(CanonArgs a) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < a.n) canon_one(a, i);
}

// ---- partition ----------------------------------------------------------------------------------
__device__ __forceinline__ bool is_file_action(uint8_t kind, uint8_t flags) {
  return (kind == K_ADD || kind == K_REMOVE) && !(flags & F_PATH_NULL);
}
__device__ __forceinline__ uint32_t bucket_of(uint64_t key, int bits) {
  return bits ? uint32_t(key >> (64 - bits)) : 0u;
}
// the 32 key bits directly below the bucket bits: the LDS table's probe start and sub-pass selector
__device__ __forceinline__ uint32_t rkey_of(uint64_t key, int bits) { return uint32_t(key >> (32 - bits)); }

// add.size in the record's 32-bit field; ~0u sends the reducer to size[] (negative or >= 2^32 - 1)
__device__ __forceinline__ uint32_t size_field(int64_t s) {
  return (s >= 0 && s < int64_t(0xffffffffll)) ? uint32_t(s) : 0xffffffffu;
}

#ifndef DR_PART_T
#define DR_PART_T 1024
#endif
#ifndef DR_RED_T
#define DR_RED_T 512
#endif
constexpr int PART_T = DR_PART_T;
constexpr int PART_STEPS = 16 * 1024 / PART_T;          // 4 actions per thread per step
constexpr int PART_TILE = PART_T * 4 * PART_STEPS;      // 65536 actions per tile: ~8 records per (bucket, tile) run
constexpr int PART_MAX_BITS = 13;                       // LDS: 2 x 8192 x 4 B in the scatter (2 workgroups/CU)

// Every thread owns 4 consecutive actions per step: one dword of kind bytes, one of flag bytes and
// two 16-byte key loads (10 B per action). For a state whose producers did not write the packed path
// references (address + length, in action order: one 8-byte load per path in k_bucket_verify's
// gathers) it packs them here from path_ptr / path_len.
__global__ void __launch_bounds__(PART_T) k_bucket_hist(PartitionArgs a) {
  __shared__ uint32_t hist[1 << PART_MAX_BITS];
  const uint32_t nb = 1u << a.bucket_bits;
  for (uint32_t b = threadIdx.x; b < nb; b += PART_T) hist[b] = 0;
  __syncthreads();
  const uint32_t tile = blockIdx.x;
  const uint64_t base = uint64_t(tile) * PART_TILE;
  // (block-uniform) the producers already wrote the packed path references (parse_launch's states)
  const bool pack = a.path_ptr != nullptr;
  for (int k = 0; k < PART_STEPS; ++k) {
    const uint64_t i0 = base + (uint64_t(k) * PART_T + threadIdx.x) * 4;
    if (i0 >= a.n) break;
    if (i0 + 4 <= a.n) {
      const uint32_t kd = *reinterpret_cast<const uint32_t*>(a.kind + i0);
      const uint32_t fl = *reinterpret_cast<const uint32_t*>(a.flags + i0);
      const uint4 k01 = *reinterpret_cast<const uint4*>(a.key + i0);
      const uint4 k23 = *reinterpret_cast<const uint4*>(a.key + i0 + 2);
      const uint64_t ks[4] = {uint64_t(k01.x) | uint64_t(k01.y) << 32, uint64_t(k01.z) | uint64_t(k01.w) << 32,
                              uint64_t(k23.x) | uint64_t(k23.y) << 32, uint64_t(k23.z) | uint64_t(k23.w) << 32};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (is_file_action(uint8_t(kd >> (8 * j)), uint8_t(fl >> (8 * j))))
          atomicAdd(&hist[bucket_of(ks[j], a.bucket_bits)], 1u);
      if (!pack) continue;
      const uint4 p01 = *reinterpret_cast<const uint4*>(a.path_ptr + i0);
      const uint4 p23 = *reinterpret_cast<const uint4*>(a.path_ptr + i0 + 2);
      const uint4 ln = *reinterpret_cast<const uint4*>(a.path_len + i0);
      *reinterpret_cast<ulonglong2*>(a.path_ref + i0) =
          make_ulonglong2(pack_ref(uint64_t(p01.x) | uint64_t(p01.y) << 32, ln.x),
                          pack_ref(uint64_t(p01.z) | uint64_t(p01.w) << 32, ln.y));
      *reinterpret_cast<ulonglong2*>(a.path_ref + i0 + 2) =
          make_ulonglong2(pack_ref(uint64_t(p23.x) | uint64_t(p23.y) << 32, ln.z),
                          pack_ref(uint64_t(p23.z) | uint64_t(p23.w) << 32, ln.w));
    } else {
      for (uint64_t i = i0; i < a.n; ++i) {
        if (is_file_action(a.kind[i], a.flags[i])) atomicAdd(&hist[bucket_of(a.key[i], a.bucket_bits)], 1u);
        if (pack) a.path_ref[i] = pack_ref(a.path_ptr[i], a.path_len[i]);
      }
    }
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < nb; b += PART_T) a.tile_count[uint64_t(b) * a.ntiles + tile] = hist[b];
}

// One file action into its bucket: the 16-byte record {key lo, key hi, index << 2 | class, size
// field}. `val` is add.size for an add and remove.deletionTimestamp for a remove.
__device__ __forceinline__ void scatter_one(const PartitionArgs& a, uint64_t i, uint8_t kind, uint8_t flags,
                                            uint64_t key, int64_t val, const uint32_t* base, uint32_t* cnt) {
  const uint32_t b = bucket_of(key, a.bucket_bits);
  const uint32_t pos = base[b] + atomicAdd(&cnt[b], 1u);
  uint32_t cls = C_ADD, sz = 0;
  if (kind == K_REMOVE) {
    // RemoveFile.delTimestamp = deletionTimestamp.getOrElse(0) (D/actions/actions.scala:318-319);
    // kept iff delTimestamp > minFileRetentionTimestamp (D/actions/InMemoryLogReplay.scala:67-69)
    const int64_t dt = (flags & F_HAS_DELTS) ? val : 0;
    cls = dt > a.cutoff ? C_REMOVE_KEEP : C_REMOVE_DROP;
  } else {
    sz = size_field(val);
  }
  *reinterpret_cast<uint4*>(a.rec + pos) = make_uint4(uint32_t(key), uint32_t(key >> 32), uint32_t(i << 2) | cls, sz);
}

// size[] is read only by waves that hold an add and delts[] only by waves that hold a remove with a
// deletionTimestamp (runs of one kind are long: whole checkpoints, whole commits), so each action
// costs kind + flags + key + one 8-byte value = 18 B in, 16 B out.
__global__ void __launch_bounds__(PART_T) k_bucket_scatter(PartitionArgs a) {
  __shared__ uint32_t base[1 << PART_MAX_BITS];
  __shared__ uint32_t cnt[1 << PART_MAX_BITS];
  const uint32_t nb = 1u << a.bucket_bits;
  // XCD-aware tiles (r06): workgroup i runs on XCD i % 8, so it takes the (i / 8)-th tile of XCD
  // (i % 8)'s contiguous share -- adjacent tiles' runs of a bucket share their boundary lines, which
  // then fill in one L2 (0.285 -> 0.276 ms on config 3)
  const uint32_t per = (a.ntiles + 7) / 8, xcd = blockIdx.x % 8, slot = blockIdx.x / 8;
  const uint32_t tile = xcd * per + slot;
  if (tile >= a.ntiles) return;  // (the grid is rounded up to a multiple of 8)
  for (uint32_t b = threadIdx.x; b < nb; b += PART_T) {
    base[b] = uint32_t(a.tile_off[uint64_t(b) * a.ntiles + tile]);
    cnt[b] = 0;
  }
  __syncthreads();
  const uint64_t tb = uint64_t(tile) * PART_TILE;
  for (int k = 0; k < PART_STEPS; ++k) {
    const uint64_t i0 = tb + (uint64_t(k) * PART_T + threadIdx.x) * 4;
    if (i0 >= a.n) break;
    if (i0 + 4 <= a.n) {
      const uint32_t kd = *reinterpret_cast<const uint32_t*>(a.kind + i0);
      const uint32_t fl = *reinterpret_cast<const uint32_t*>(a.flags + i0);
      const uint4 k01 = *reinterpret_cast<const uint4*>(a.key + i0);
      const uint4 k23 = *reinterpret_cast<const uint4*>(a.key + i0 + 2);
      const uint64_t ks[4] = {uint64_t(k01.x) | uint64_t(k01.y) << 32, uint64_t(k01.z) | uint64_t(k01.w) << 32,
                              uint64_t(k23.x) | uint64_t(k23.y) << 32, uint64_t(k23.z) | uint64_t(k23.w) << 32};
      bool any_file = false, any_add = false, any_del = false;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint8_t kj = uint8_t(kd >> (8 * j)), fj = uint8_t(fl >> (8 * j));
        const bool f = is_file_action(kj, fj);
        any_file |= f;
        any_add |= f && kj == K_ADD;
        any_del |= f && kj == K_REMOVE && (fj & F_HAS_DELTS);
      }
      if (!__ballot(any_file)) continue;  // wave-uniform
      int64_t val[4] = {0, 0, 0, 0};
      if (__ballot(any_add)) {
        const uint4 s01 = *reinterpret_cast<const uint4*>(a.size + i0);
        const uint4 s23 = *reinterpret_cast<const uint4*>(a.size + i0 + 2);
        const int64_t sv[4] = {int64_t(uint64_t(s01.x) | uint64_t(s01.y) << 32),
                               int64_t(uint64_t(s01.z) | uint64_t(s01.w) << 32),
                               int64_t(uint64_t(s23.x) | uint64_t(s23.y) << 32),
                               int64_t(uint64_t(s23.z) | uint64_t(s23.w) << 32)};
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (uint8_t(kd >> (8 * j)) == K_ADD) val[j] = sv[j];
      }
      if (__ballot(any_del)) {
        const uint4 d01 = *reinterpret_cast<const uint4*>(a.delts + i0);
        const uint4 d23 = *reinterpret_cast<const uint4*>(a.delts + i0 + 2);
        const int64_t dv[4] = {int64_t(uint64_t(d01.x) | uint64_t(d01.y) << 32),
                               int64_t(uint64_t(d01.z) | uint64_t(d01.w) << 32),
                               int64_t(uint64_t(d23.x) | uint64_t(d23.y) << 32),
                               int64_t(uint64_t(d23.z) | uint64_t(d23.w) << 32)};
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (uint8_t(kd >> (8 * j)) == K_REMOVE) val[j] = dv[j];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint8_t kj = uint8_t(kd >> (8 * j)), fj = uint8_t(fl >> (8 * j));
        if (is_file_action(kj, fj)) scatter_one(a, i0 + j, kj, fj, ks[j], val[j], base, cnt);
      }
    } else {
      for (uint64_t i = i0; i < a.n; ++i) {
        const uint8_t kj = a.kind[i], fj = a.flags[i];
        if (!is_file_action(kj, fj)) continue;
        const int64_t v = kj == K_ADD ? a.size[i] : ((fj & F_HAS_DELTS) ? a.delts[i] : 0);
        scatter_one(a, i, kj, fj, a.key[i], v, base, cnt);
      }
    }
  }
}

__global__ void k_bucket_offsets(const uint64_t* tile_off, uint32_t nb, uint32_t nt, uint64_t* bucket_off) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b <= nb) bucket_off[b] = tile_off[uint64_t(b) * nt];
}

// ---- per-bucket reduce ------------------------------------------------------------------------------
constexpr int RED_T = DR_RED_T;
// LDS table slots: 8 B key + 4 B winner meta + 2 B loser count = 49 KiB, 3 workgroups per CU
constexpr int TS_MAX = 3584;
constexpr int HELD_MAX = TS_MAX / 4 * 3;  // a bucket of at most this many records is held in registers
constexpr int RED_RPT = (HELD_MAX + RED_T - 1) / RED_T;

struct BucketTotals {
  uint64_t live, tomb, size, lks, tks;
};

// Block-wide sums of the survivor statistics, stored per bucket (summed by k_sum_stats: no
// contended global atomics).
__device__ void store_totals(ReduceArgs& a, uint32_t b, BucketTotals t) {
  __shared__ unsigned long long red[5][RED_T / 64];
  for (int o = 32; o > 0; o >>= 1) {
    t.live += __shfl_down(t.live, o, 64);
    t.tomb += __shfl_down(t.tomb, o, 64);
    t.size += __shfl_down(t.size, o, 64);
    t.lks += __shfl_down(t.lks, o, 64);
    t.tks += __shfl_down(t.tks, o, 64);
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][wv] = t.live; red[1][wv] = t.tomb; red[2][wv] = t.size; red[3][wv] = t.lks; red[4][wv] = t.tks;
  }
  __syncthreads();
  if (threadIdx.x < 5) {
    unsigned long long s = 0;
    for (int k = 0; k < RED_T / 64; ++k) s += red[threadIdx.x][k];
    a.bstats[uint64_t(b) * 5 + threadIdx.x] = s;
  }
}

// totals[0] live, [2] tombstones, [1] size sum, [5] live checksum, [6] tombstone checksum
__global__ void __launch_bounds__(1024) k_sum_stats(const unsigned long long* bstats, uint32_t nb,
                                                    unsigned long long* totals) {
  __shared__ unsigned long long red[5][16];
  unsigned long long s[5] = {0, 0, 0, 0, 0};
  for (uint32_t b = threadIdx.x; b < nb; b += 1024)
    for (int k = 0; k < 5; ++k) s[k] += bstats[uint64_t(b) * 5 + k];
  for (int k = 0; k < 5; ++k)
    for (int o = 32; o > 0; o >>= 1) s[k] += __shfl_down(s[k], o, 64);
  if ((threadIdx.x & 63) == 0)
    for (int k = 0; k < 5; ++k) red[k][threadIdx.x >> 6] = s[k];
  __syncthreads();
  if (threadIdx.x < 5) {
    unsigned long long t = 0;
    for (int w = 0; w < 16; ++w) t += red[threadIdx.x][w];
    const int slot[5] = {0, 2, 1, 5, 6};
    totals[slot[threadIdx.x]] = t;
  }
}

__device__ __forceinline__ uint4 load_rec(const PartRec* r, uint64_t e) {
  return *reinterpret_cast<const uint4*>(r + e);
}
__device__ __forceinline__ uint64_t rec_key(uint4 r) { return uint64_t(r.x) | (uint64_t(r.y) << 32); }
// add.size of a record (the 32-bit field, or size[] by action index when it did not fit)
__device__ __forceinline__ uint64_t rec_size(const ReduceArgs& a, uint4 r) {
  return r.w != 0xffffffffu ? uint64_t(r.w) : uint64_t(a.size[r.z >> 2]);
}

// Appends one wave's flagged values to an LDS-counted list region (order across waves is free).
__device__ __forceinline__ void wave_append(bool f, uint32_t v, uint32_t* cnt, uint32_t* out) {
  const unsigned long long bl = __ballot(f);
  if (!bl) return;
  const int lane = threadIdx.x & 63;
  uint32_t o = 0;
  if (lane == __ffsll(bl) - 1) o = atomicAdd(cnt, uint32_t(__popcll(bl)));
  o = __shfl(o, __ffsll(bl) - 1, 64);
  if (f) out[o + uint32_t(__popcll(bl & ((1ull << lane) - 1ull)))] = v;
}
__device__ __forceinline__ void wave_append2(bool f, uint2 v, uint32_t* cnt, uint2* out) {
  const unsigned long long bl = __ballot(f);
  if (!bl) return;
  const int lane = threadIdx.x & 63;
  uint32_t o = 0;
  if (lane == __ffsll(bl) - 1) o = atomicAdd(cnt, uint32_t(__popcll(bl)));
  o = __shfl(o, __ffsll(bl) - 1, 64);
  if (f) out[o + uint32_t(__popcll(bl & ((1ull << lane) - 1ull)))] = v;
}

// 16 bytes at byte offset `off` (0..15) of the 32 bytes lo:hi (little-endian).
__device__ __forceinline__ uint4 window16(uint4 lo, uint4 hi, uint32_t off) {
  const uint32_t dw = off >> 2, sb = off & 3;
  auto pick = [&](uint32_t k) -> uint32_t {  // dword k + dw of lo:hi, k in 0..4
    const uint32_t j = k + dw;
    return j == 0 ? lo.x : j == 1 ? lo.y : j == 2 ? lo.z : j == 3 ? lo.w
         : j == 4 ? hi.x : j == 5 ? hi.y : j == 6 ? hi.z : hi.w;
  };
  const uint32_t a0 = pick(0), a1 = pick(1), a2 = pick(2), a3 = pick(3), a4 = pick(4);
  return make_uint4(__builtin_amdgcn_alignbyte(a1, a0, sb), __builtin_amdgcn_alignbyte(a2, a1, sb),
                    __builtin_amdgcn_alignbyte(a3, a2, sb), __builtin_amdgcn_alignbyte(a4, a3, sb));
}

constexpr uint64_t PREF_PTR = (1ull << 48) - 1;
// Differences (masked to the string) in path bytes [i, i + 16) of p and q, rem = n - i; plo/phi and
// qlo/qhi are the aligned 16-byte blocks holding them (po, qo: the strings' offsets in their blocks).
__device__ __forceinline__ uint32_t block_diff(uint4 plo, uint4 phi, uint32_t po, uint4 qlo, uint4 qhi, uint32_t qo,
                                               uint32_t rem) {
  const uint4 x = window16(plo, phi, po), y = window16(qlo, qhi, qo);
  uint4 d = make_uint4(x.x ^ y.x, x.y ^ y.y, x.z ^ y.z, x.w ^ y.w);
  if (rem < 16) {  // bytes past the string end do not count
    const uint32_t m0 = rem >= 4 ? 0xffffffffu : (1u << (8 * rem)) - 1u;
    const uint32_t m1 = rem >= 8 ? 0xffffffffu : rem <= 4 ? 0u : (1u << (8 * (rem - 4))) - 1u;
    const uint32_t m2 = rem >= 12 ? 0xffffffffu : rem <= 8 ? 0u : (1u << (8 * (rem - 8))) - 1u;
    const uint32_t m3 = rem <= 12 ? 0u : (1u << (8 * (rem - 12))) - 1u;
    d.x &= m0; d.y &= m1; d.z &= m2; d.w &= m3;
  }
  return d.x | d.y | d.z | d.w;
}

// Byte equality of p[0..n) and q[0..n) by one lane: aligned 16-byte loads (each block once; past
// the string its last block again), no early exit, so the loads of successive blocks are independent.
__device__ bool bytes_equal16(const uint8_t* p, const uint8_t* q, uint32_t n) {
  const uint4* pa = reinterpret_cast<const uint4*>(reinterpret_cast<uintptr_t>(p) & ~uintptr_t(15));
  const uint4* qa = reinterpret_cast<const uint4*>(reinterpret_cast<uintptr_t>(q) & ~uintptr_t(15));
  const uint32_t po = uint32_t(reinterpret_cast<uintptr_t>(p) & 15), qo = uint32_t(reinterpret_cast<uintptr_t>(q) & 15);
  const uint32_t pblocks = (po + n + 15) >> 4, qblocks = (qo + n + 15) >> 4;
  // the first 128 bytes: every 16-byte block of both paths requested before any is compared (a
  // lane compares one pair alone, so one round trip instead of one per block). Blocks past a string
  // re-read its last one (their bytes are masked by block_diff): as conditional loads the compiler
  // split each into four dword loads under branches
  constexpr uint32_t PRE = 9;
  uint4 pb[PRE], qb[PRE];
  if (n == 0) return true;
#pragma unroll
  for (uint32_t k = 0; k < PRE; ++k) {
    pb[k] = gload16(pa + min(k, pblocks - 1));
    qb[k] = gload16(qa + min(k, qblocks - 1));
  }
  uint32_t diff = 0;
#pragma unroll
  for (uint32_t k = 1; k < PRE; ++k) {
    const uint32_t i = 16 * (k - 1);
    if (i < n) diff |= block_diff(pb[k - 1], pb[k], po, qb[k - 1], qb[k], qo, n - i);
  }
  if (n <= 16 * (PRE - 1)) return diff == 0;
  uint4 plo = pb[PRE - 1], qlo = qb[PRE - 1];
  for (uint32_t i = 16 * (PRE - 1), k = PRE; i < n; i += 16, ++k) {
    const uint4 phi = gload16(pa + min(k, pblocks - 1)), qhi = gload16(qa + min(k, qblocks - 1));
    diff |= block_diff(plo, phi, po, qlo, qhi, qo, n - i);
    plo = phi;
    qlo = qhi;
  }
  return diff == 0;
}

constexpr int VER_G = 8;  // lanes per verified pair

__device__ __forceinline__ uint4 shfl_down4(uint4 v, int width) {
  return make_uint4(__shfl_down(v.x, 1, width), __shfl_down(v.y, 1, width), __shfl_down(v.z, 1, width),
                    __shfl_down(v.w, 1, width));
}

// Every (loser, winner) pair of a bucket must name the same path (URI-equality key): a mismatch is
// a 64-bit path-hash collision and sends the bucket to the exact reducer (as does a path too long
// for a packed reference). Eight lanes compare one pair: lane j loads aligned 16-byte block j of
// both strings (a wave instruction requests eight whole paths of each side at once, every block
// once) and takes block j + 1 from its neighbour by a shuffle; lanes 0..6 each compare 16 path
// bytes, and the group ORs its differences. Unequal bytes get the URI-key comparison (file:/// vs
// file:/ spellings) on the group's first lane. The pairs of a winner sit together (k_bucket_reduce
// groups them), so the groups that share a winner fetch its reference and bytes once from HBM.
constexpr int VER_T = 256;
__global__ void __launch_bounds__(VER_T) k_bucket_verify(ReduceArgs a) {
  const uint32_t b = blockIdx.x;
  const uint32_t n = a.pair_count[b];
  if (!n) return;
  const uint2* pr = a.out_pair + a.bucket_off[b];
  const uint32_t j = threadIdx.x & (VER_G - 1);
  bool bad = false;
  uint32_t vbytes = 0;  // (vstats) path bytes this lane group compared
  for (uint32_t k0 = 0; k0 < n; k0 += VER_T / VER_G) {
    const uint32_t k = k0 + threadIdx.x / VER_G;
    uint32_t diff = 0;
    bool nul = false;
    const uint8_t *p = nullptr, *q = nullptr;
    uint32_t pn = 0, qn = 0;
    if (k < n) {
      const uint2 ix = pr[k];
#ifdef DR_VERIFY_EXP_NOREFS  // timing experiment only: the loser's reference stands for both (no winner gather)
      const uint64_t vx = a.path_ref[ix.x], vy = vx + (ix.y & 0u);
#else
      const uint64_t vx = a.path_ref[ix.x], vy = a.path_ref[ix.y];
#endif
      nul = !vx || !vy;
      p = reinterpret_cast<const uint8_t*>(vx & PREF_PTR);
      q = reinterpret_cast<const uint8_t*>(vy & PREF_PTR);
      pn = uint32_t(vx >> 48);
      qn = uint32_t(vy >> 48);
#ifdef DR_VERIFY_EXP_NOBYTES  // timing experiment only (scripts/build_variant.sh): pairs + references, no path bytes
      if (true) {
        diff = (nul || pn != qn) ? 1u : 0u;
      } else
#endif
      if (nul || pn != qn) {
        diff = 1;
      } else {
        if (j == 0) vbytes += 2 * pn;
        const uint4* pa = reinterpret_cast<const uint4*>(reinterpret_cast<uintptr_t>(p) & ~uintptr_t(15));
        const uint4* qa = reinterpret_cast<const uint4*>(reinterpret_cast<uintptr_t>(q) & ~uintptr_t(15));
        const uint32_t po = uint32_t(reinterpret_cast<uintptr_t>(p) & 15);
        const uint32_t qo = uint32_t(reinterpret_cast<uintptr_t>(q) & 15);
        const uint32_t pblocks = (po + pn + 15) >> 4, qblocks = (qo + pn + 15) >> 4;
        // step: lane j loads aligned block B + j of each string (a block past the string re-reads
        // its last one) and takes block B + j + 1 from lane j + 1; lanes 0..6 compare path bytes
        // [16 (B + j), +16)
        for (uint32_t B = 0; 16 * B < pn; B += VER_G - 1) {
          // (unconditional loads, clamped to the string's last block: see bytes_equal16)
          const uint4 plo = gload16(pa + min(B + j, pblocks - 1)), qlo = gload16(qa + min(B + j, qblocks - 1));
          const uint4 phi = shfl_down4(plo, VER_G), qhi = shfl_down4(qlo, VER_G);
          const uint32_t i = 16 * (B + j);
          if (j < VER_G - 1 && i < pn) diff |= block_diff(plo, phi, po, qlo, qhi, qo, pn - i);
        }
      }
    }
    // OR over the pair's eight lanes
    for (int o = 1; o < VER_G; o <<= 1) diff |= __shfl_xor(diff, o, 64);
    if (k < n && j == 0 && diff) {
      // equal bytes => equal URI keys; otherwise only file:/// vs file:/ spellings can still match
      if (nul || !key_equal(p, pn, q, qn)) bad = true;
    }
  }
  if (__syncthreads_or(bad) && threadIdx.x == 0) a.exact_list[atomicAdd(&a.totals[4], 1ull)] = b;
  if (a.vstats) {  // block-uniform: the bucket's {pairs, bytes} in its own slots (no contended atomics)
    __shared__ unsigned long long vsum;
    if (threadIdx.x == 0) vsum = 0;
    __syncthreads();
    unsigned long long v = vbytes;
    for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(&vsum, v);
    __syncthreads();
    if (threadIdx.x == 0) {
      a.vstats[2 * uint64_t(b)] = n;
      a.vstats[2 * uint64_t(b) + 1] = vsum;
    }
  }
}

// Per-slot loser counts packed two to a word (slot s: word s >> 1, bits 16 (s & 1)): members - 1 of
// each slot, replaced in place by each slot's first pair position (an exclusive scan over the n
// slots, n <= TS_MAX and even, by one RED_T workgroup); returns the total. Counts and positions stay
// below 2^16 (a pass holds at most a few thousand records), so the halves never carry into each other.
__device__ uint32_t scan_loser_slots(uint32_t* w, uint32_t n) {
  __shared__ uint32_t wsum[RED_T / 64];
  constexpr uint32_t PER = (TS_MAX / 2 + RED_T - 1) / RED_T;  // words per thread
  const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const uint32_t nw = n >> 1;
  uint32_t v[2 * PER], s = 0;
#pragma unroll
  for (uint32_t k = 0; k < PER; ++k) {
    const uint32_t i = t * PER + k;
    const uint32_t x = i < nw ? w[i] : 0u;
    const uint32_t lo = x & 0xffffu, hi = x >> 16;
    v[2 * k] = lo ? lo - 1u : 0u;
    v[2 * k + 1] = hi ? hi - 1u : 0u;
    s += v[2 * k] + v[2 * k + 1];
  }
  uint32_t incl = s;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(incl, o, 64);
    if (lane >= uint32_t(o)) incl += y;
  }
  if (lane == 63) wsum[wv] = incl;
  __syncthreads();
  uint32_t base = 0, total = 0;
  for (uint32_t q = 0; q < RED_T / 64; ++q) {
    base += q < wv ? wsum[q] : 0u;
    total += wsum[q];
  }
  uint32_t run = base + incl - s;
#pragma unroll
  for (uint32_t k = 0; k < PER; ++k) {
    const uint32_t i = t * PER + k;
    const uint32_t lo = run;
    run += v[2 * k];
    if (i < nw) w[i] = lo | (run << 16);
    run += v[2 * k + 1];
  }
  __syncthreads();
  return total;
}

// Table of ts slots (a multiple of 64, at most TS_MAX): a key's probe starts at its low 32 bits scaled
// to ts (independent of the bucket and sub-pass bits, which sit above them), linear probing wraps.
__device__ __forceinline__ uint32_t slot_start(uint64_t key, uint32_t ts) {
  return uint32_t((uint64_t(uint32_t(key)) * ts) >> 32);
}
__device__ __forceinline__ uint32_t table_slots(uint64_t m) {
  return uint32_t(min<uint64_t>(TS_MAX, max<uint64_t>(64, (2 * m + 63) & ~uint64_t(63))));
}

// Inserts key k with action meta z: table[k] = max(meta + 1) -- the largest action index wins.
// Returns the slot, or ts when the table is full.
__device__ __forceinline__ uint32_t table_insert(unsigned long long* tkey, uint32_t* tval, uint32_t* tcnt, uint32_t ts,
                                                 unsigned long long k, uint32_t z) {
  uint32_t s = slot_start(k, ts);
  for (uint32_t probe = 0; probe < ts; ++probe) {
    const unsigned long long old = atomicCAS(&tkey[s], 0ull, k);
    if (old == 0ull || old == k) {
      atomicMax(&tval[s], z + 1u);
      atomicAdd(&tcnt[s >> 1], 1u << (16 * (s & 1)));
      return s;
    }
    s = s + 1 == ts ? 0u : s + 1;
  }
  return ts;
}

// One record after the inserts: its slot's winner decides. Winners are classified (live add, kept
// tombstone, or dropped); a loser is paired with its winner for k_bucket_verify.
struct RedOut {
  bool isl, ist, isp;
  uint32_t idx, win;
};
__device__ __forceinline__ RedOut classify(const ReduceArgs& a, uint4 r, uint32_t w, uint64_t& size,
                                           uint64_t& lks, uint64_t& tks) {
  RedOut o{false, false, false, r.z >> 2, w >> 2};
  const unsigned long long k = rec_key(r);
  if (w == r.z) {
    const uint32_t cls = r.z & 3;
    if (cls == C_ADD) {
      o.isl = true;
      size += rec_size(a, r);
      lks += k >> 32;
    } else if (cls == C_REMOVE_KEEP) {
      o.ist = true;
      tks += k >> 32;
    }
  } else {
    o.isp = true;
  }
  return o;
}

// The bucket's {live, tomb, size, live sum, tomb sum}: the counts from the append counters, the sums
// reduced over the workgroup (no contended global atomics: k_sum_stats adds the buckets).
__device__ void store_sums(ReduceArgs& a, uint32_t b, uint32_t nl, uint32_t nt, uint64_t size, uint64_t lks,
                           uint64_t tks) {
  __shared__ unsigned long long red[3][RED_T / 64];
  for (int o = 32; o > 0; o >>= 1) {
    size += __shfl_down(size, o, 64);
    lks += __shfl_down(lks, o, 64);
    tks += __shfl_down(tks, o, 64);
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[0][wv] = size; red[1][wv] = lks; red[2][wv] = tks; }
  __syncthreads();
  if (threadIdx.x < 5) {
    unsigned long long v = threadIdx.x == 0 ? nl : nt;
    if (threadIdx.x >= 2) {
      v = 0;
      for (int k = 0; k < RED_T / 64; ++k) v += red[threadIdx.x - 2][k];
    }
    a.bstats[uint64_t(b) * 5 + threadIdx.x] = v;
  }
}

// K4: one workgroup per bucket. An LDS open-addressing table keyed by the full 64-bit path key keeps
// atomicMax(meta + 1): the action with the largest (version, line) ordinal wins -- exactly the
// reference's "last action per path" (D/actions/InMemoryLogReplay.scala:43-77). Survivors go to the
// bucket's region of the live / tombstone lists; every loser is paired (by action index) with its
// winner for k_bucket_verify, the pairs grouped by winner (a counting sort on the table slot: the
// verifier's lane groups that share a winner then request its lines in one instruction; without the
// grouping k_bucket_verify took 0.46 instead of 0.40 ms on config 3). A bucket of up to HELD_MAX
// records is held in registers (loaded once, all loads in flight before the first use) and each
// record keeps its table slot between the insert and the classification; a larger one is reduced in
// sub-passes by the next key bits, re-read from HBM. The table is sized to the bucket (2 slots per
// record), so its clearing costs what it holds. An LDS-table overflow sends the bucket to the
// finer-grained fallback reducer.
__global__ void __launch_bounds__(RED_T) k_bucket_reduce(ReduceArgs a) {
  __shared__ unsigned long long tkey[TS_MAX];
  __shared__ uint32_t tval[TS_MAX];
  __shared__ uint32_t tcnt[TS_MAX / 2];  // u16 per slot: members, then its next pair position
  __shared__ uint32_t nl, nt, overflow;
  const uint32_t b = blockIdx.x;
  const int bits = a.bucket_bits;
  const uint64_t beg = a.bucket_off[b], end = a.bucket_off[b + 1];
  const uint64_t m = end - beg;
  if (threadIdx.x == 0) { nl = 0; nt = 0; overflow = 0; }
  uint64_t size = 0, lks = 0, tks = 0;
  uint32_t pbase = 0;  // pairs of the earlier sub-passes
  // a loser's pair at its slot's next position: the pairs of one winner end up next to each other
  auto put_pair = [&](const RedOut& o, uint32_t s) {
    if (!o.isp) return;
    const uint32_t sh = 16 * (s & 1);
    const uint32_t at = pbase + ((atomicAdd(&tcnt[s >> 1], 1u << sh) >> sh) & 0xffffu);
    a.out_pair[beg + at] = make_uint2(o.idx, o.win);
  };
  if (m <= uint64_t(HELD_MAX)) {
    const uint32_t ts = table_slots(m);
    uint4 r[RED_RPT];
#pragma unroll
    for (int q = 0; q < RED_RPT; ++q) {
      const uint64_t e = beg + threadIdx.x + uint64_t(q) * RED_T;
      r[q] = e < end ? load_rec(a.rec, e) : make_uint4(0, 0, 0, 0);
    }
    for (uint32_t s = threadIdx.x; s < ts; s += RED_T) { tkey[s] = 0; tval[s] = 0; }
    for (uint32_t s = threadIdx.x; s < ts / 2; s += RED_T) tcnt[s] = 0;
    __syncthreads();
    uint32_t sl[RED_RPT];
#pragma unroll
    for (int q = 0; q < RED_RPT; ++q) {
      sl[q] = 0;
      if (beg + threadIdx.x + uint64_t(q) * RED_T >= end) continue;
      sl[q] = table_insert(tkey, tval, tcnt, ts, rec_key(r[q]), r[q].z);
      if (sl[q] == ts) overflow = 1;
    }
    __syncthreads();
    if (!overflow) {
      const uint32_t npass = scan_loser_slots(tcnt, ts);
#pragma unroll
      for (int q = 0; q < RED_RPT; ++q) {
        const bool in = beg + threadIdx.x + uint64_t(q) * RED_T < end;
        if (!__ballot(in)) break;  // wave-uniform: later rows are past the bucket for every lane
        RedOut o{false, false, false, 0, 0};
        if (in) o = classify(a, r[q], tval[sl[q]] - 1u, size, lks, tks);
        put_pair(o, sl[q]);
        wave_append(o.isl, o.idx, &nl, a.out_live + beg);
        wave_append(o.ist, o.idx, &nt, a.out_tomb + beg);
      }
      pbase = npass;
    }
  } else {
    // sub-passes by the top sbits of the 32 key bits below the bucket bits, each at most 3/4 TS_MAX
    // records on average
    int sbits = 0;
    while ((m >> sbits) > uint64_t(HELD_MAX)) ++sbits;
    const uint32_t ts = TS_MAX;
    for (uint32_t sp = 0; sp < (1u << sbits); ++sp) {
      __syncthreads();
      for (uint32_t s = threadIdx.x; s < ts; s += RED_T) { tkey[s] = 0; tval[s] = 0; }
      for (uint32_t s = threadIdx.x; s < ts / 2; s += RED_T) tcnt[s] = 0;
      __syncthreads();
      for (uint64_t e = beg + threadIdx.x; e < end; e += RED_T) {
        const uint4 r = load_rec(a.rec, e);
        if ((rkey_of(rec_key(r), bits) >> (32 - sbits)) != sp) continue;
        if (table_insert(tkey, tval, tcnt, ts, rec_key(r), r.z) == ts) overflow = 1;
      }
      __syncthreads();
      if (overflow) break;
      const uint32_t npass = scan_loser_slots(tcnt, ts);
      for (uint64_t e0 = beg; e0 < end; e0 += RED_T) {
        const uint64_t e = e0 + threadIdx.x;
        RedOut o{false, false, false, 0, 0};
        uint32_t s = 0;
        if (e < end) {
          const uint4 r = load_rec(a.rec, e);
          const unsigned long long k = rec_key(r);
          if ((rkey_of(k, bits) >> (32 - sbits)) == sp) {
            s = slot_start(k, ts);
            while (tkey[s] != k) s = s + 1 == ts ? 0u : s + 1;
            o = classify(a, r, tval[s] - 1u, size, lks, tks);
          }
        }
        put_pair(o, s);
        wave_append(o.isl, o.idx, &nl, a.out_live + beg);
        wave_append(o.ist, o.idx, &nt, a.out_tomb + beg);
      }
      pbase += npass;
    }
  }
  __syncthreads();
  const uint32_t vl = nl, vt = nt;
  if (threadIdx.x == 0) {
    a.live_count[b] = vl;
    a.tomb_count[b] = vt;
    a.pair_count[b] = overflow ? 0 : pbase;
    if (overflow) a.redo_list[atomicAdd(&a.totals[3], 1ull)] = b;
  }
  store_sums(a, b, vl, vt, size, lks, tks);
}

// Fallback for buckets whose LDS table overflowed (or every bucket, under the DR_FLAG_REDUCE64 test
// hook): the same last-writer-wins keyed by the full 64-bit path hash in finer sub-passes, byte-verified
// inline. A 64-bit collision (or overflow) hands the bucket on to the exact O(m^2) kernel.
constexpr int TS64 = 4096;
__device__ void reduce64_bucket(ReduceArgs& a, uint32_t b) {
  __shared__ unsigned long long tkey[TS64];
  __shared__ uint32_t tval[TS64];
  __shared__ uint32_t nl, nt, collide, overflow;
  __syncthreads();  // the previous bucket of this workgroup is done with the shared state
  const uint64_t beg = a.bucket_off[b], end = a.bucket_off[b + 1];
  const uint64_t m = end - beg;
  int sbits = 0;
  while ((m >> sbits) > uint64_t(TS64 / 2)) ++sbits;
  if (threadIdx.x == 0) { nl = 0; nt = 0; collide = 0; overflow = 0; }
  BucketTotals tot{0, 0, 0, 0, 0};
  for (uint32_t sp = 0; sp < (1u << sbits); ++sp) {
    __syncthreads();
    for (int s = threadIdx.x; s < TS64; s += RED_T) { tkey[s] = 0; tval[s] = 0; }
    __syncthreads();
    for (uint64_t e = beg + threadIdx.x; e < end; e += RED_T) {
      const uint4 r = load_rec(a.rec, e);
      const uint64_t k = rec_key(r);
      if (sbits && uint32_t(k & ((1u << sbits) - 1)) != sp) continue;
      uint32_t s = uint32_t(k >> 20) & (TS64 - 1);
      for (int probe = 0;; ++probe) {
        if (probe >= TS64) { overflow = 1; break; }
        const unsigned long long old = atomicCAS(&tkey[s], 0ull, (unsigned long long)k);
        if (old == 0ull || old == k) { atomicMax(&tval[s], r.z + 1u); break; }
        s = (s + 1) & (TS64 - 1);
      }
    }
    __syncthreads();
    if (overflow) break;
    for (uint64_t e0 = beg; e0 < end; e0 += RED_T) {
      const uint64_t e = e0 + threadIdx.x;
      bool isl = false, ist = false;
      uint32_t idx = 0;
      if (e < end) {
        const uint4 r = load_rec(a.rec, e);
        idx = r.z >> 2;
        const uint64_t k = rec_key(r);
        if (!sbits || uint32_t(k & ((1u << sbits) - 1)) == sp) {
          uint32_t s = uint32_t(k >> 20) & (TS64 - 1);
          while (tkey[s] != k) s = (s + 1) & (TS64 - 1);
          const uint32_t w = tval[s] - 1u;
          if (w == r.z) {
            if ((r.z & 3) == C_ADD) {
              isl = true;
              ++tot.live;
              tot.size += rec_size(a, r);
              tot.lks += k >> 32;
            } else if ((r.z & 3) == C_REMOVE_KEEP) {
              ist = true;
              ++tot.tomb;
              tot.tks += k >> 32;
            }
          } else {
            const uint32_t wi = w >> 2;
            const uint8_t* p = reinterpret_cast<const uint8_t*>(a.path_ptr[idx]);
            const uint8_t* q = reinterpret_cast<const uint8_t*>(a.path_ptr[wi]);
            const uint32_t pn = a.path_len[idx], qn = a.path_len[wi];
            if (!(pn == qn && bytes_equal16(p, q, pn)) && !key_equal(p, pn, q, qn)) collide = 1;
          }
        }
      }
      wave_append(isl, idx, &nl, a.out_live + beg);
      wave_append(ist, idx, &nt, a.out_tomb + beg);
    }
  }
  __syncthreads();
  const bool redo = collide || overflow;
  if (threadIdx.x == 0) {
    a.live_count[b] = redo ? 0 : nl;
    a.tomb_count[b] = redo ? 0 : nt;
    if (redo) a.exact_list[atomicAdd(&a.totals[4], 1ull)] = b;
  }
  store_totals(a, b, redo ? BucketTotals{0, 0, 0, 0, 0} : tot);
}

// Exact fallback: each record is a winner iff no other record with an equal path has a larger
// action index. O(m^2) per bucket; only reached on a 64-bit path-hash collision.
__device__ void exact_bucket(ReduceArgs& a, uint32_t b) {
  __shared__ uint32_t nl, nt;
  __syncthreads();  // the previous bucket of this workgroup is done with the shared state
  const uint64_t beg = a.bucket_off[b], end = a.bucket_off[b + 1];
  if (threadIdx.x == 0) { nl = 0; nt = 0; }
  __syncthreads();
  BucketTotals tot{0, 0, 0, 0, 0};
  for (uint64_t e = beg + threadIdx.x; e < end; e += RED_T) {
    const uint4 r = load_rec(a.rec, e);
    const uint32_t idx = r.z >> 2;
    const uint64_t k = rec_key(r);
    const uint8_t* p = reinterpret_cast<const uint8_t*>(a.path_ptr[idx]);
    const uint32_t pn = a.path_len[idx];
    bool win = true;
    for (uint64_t f = beg; f < end && win; ++f) {
      if (f == e) continue;
      const uint4 q = load_rec(a.rec, f);
      const uint32_t j = q.z >> 2;
      if (rec_key(q) != k || j <= idx) continue;
      if (key_equal(p, pn, reinterpret_cast<const uint8_t*>(a.path_ptr[j]), a.path_len[j])) win = false;
    }
    if (!win) continue;
    if ((r.z & 3) == C_ADD) {
      ++tot.live;
      tot.size += rec_size(a, r);
      tot.lks += k >> 32;
      a.out_live[beg + atomicAdd(&nl, 1u)] = idx;
    } else if ((r.z & 3) == C_REMOVE_KEEP) {
      ++tot.tomb;
      tot.tks += k >> 32;
      a.out_tomb[beg + atomicAdd(&nt, 1u)] = idx;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    a.live_count[b] = nl;
    a.tomb_count[b] = nt;
  }
  store_totals(a, b, tot);
}

// The fallbacks walk their bucket list grid-stride; the list length is read on the device when only
// its bound n is known on the host (a few buckets out of thousands: no grid of idle workgroups).
__global__ void __launch_bounds__(RED_T) k_bucket_reduce64(ReduceArgs a, const uint32_t* buckets, uint32_t n,
                                                       const unsigned long long* count) {
  const uint32_t lim = count ? uint32_t(min(*count, (unsigned long long)n)) : n;
  for (uint32_t i = blockIdx.x; i < lim; i += gridDim.x) reduce64_bucket(a, buckets[i]);
}
__global__ void __launch_bounds__(RED_T) k_bucket_exact(ReduceArgs a, const uint32_t* buckets, uint32_t n,
                                                    const unsigned long long* count) {
  const uint32_t lim = count ? uint32_t(min(*count, (unsigned long long)n)) : n;
  for (uint32_t i = blockIdx.x; i < lim; i += gridDim.x) exact_bucket(a, buckets[i]);
}

__device__ __forceinline__ void k_compact_one(const CompactArgs& a) {
  const uint32_t b = blockIdx.x;
  if (b >= a.nbuckets) return;
  const uint32_t c = a.counts[b];
  const uint64_t src = a.bucket_off[b], dst = a.dst_off[b];
  for (uint32_t k = threadIdx.x; k < c; k += blockDim.x) a.dst[dst + k] = a.src[src + k];
}
__global__ void k_compact(CompactArgs a) { k_compact_one(a); }

// Both survivor lists at once (blockIdx.y: 0 live, 1 tombstones).
__global__ void k_compact2(CompactArgs l, CompactArgs t) {
  k_compact_one(blockIdx.y ? t : l);
}

// Large replays (more than 2^13 * 2048 file actions, config 4): K3's scatter keeps per-tile LDS cursors
// for at most 2^13 buckets, so buckets average over 2048 records and K4 would take several sub-passes,
// each reading the whole bucket twice. k_bucket_split refines every bucket b into 2^sbits sub-buckets
// by the next key bits -- exactly bucket_of(key, bits + sbits) -- writing the records once more
// (order within a bucket is free: K4's last-writer-wins is an atomicMax on the action index) and
// the refined offsets, so K4 runs one pass per refined bucket. Records stay in registers between the
// count and the write (up to SPLIT_T * SPLIT_RPT per bucket; larger buckets read twice).
constexpr int SPLIT_T = 1024, SPLIT_RPT = 16;
__global__ void __launch_bounds__(SPLIT_T) k_bucket_split(SplitArgs a) {
  __shared__ uint32_t cnt[64], cur[64];
  const uint32_t b = blockIdx.x, S = 1u << a.sbits;
  const uint64_t beg = a.bucket_off[b], end = a.bucket_off[b + 1];
  const uint64_t m = end - beg;
  if (threadIdx.x < S) cnt[threadIdx.x] = 0;
  __syncthreads();
  auto sub_of = [&](uint4 r) { return rkey_of(rec_key(r), a.bits) >> (32 - a.sbits); };
  const bool held = m <= uint64_t(SPLIT_T) * SPLIT_RPT;  // block-uniform
  uint4 r[SPLIT_RPT];
  if (held) {
#pragma unroll
    for (int q = 0; q < SPLIT_RPT; ++q) {
      const uint64_t e = beg + threadIdx.x + uint64_t(q) * SPLIT_T;
      if (e < end) r[q] = load_rec(a.rec, e);
    }
#pragma unroll
    for (int q = 0; q < SPLIT_RPT; ++q)
      if (beg + threadIdx.x + uint64_t(q) * SPLIT_T < end) atomicAdd(&cnt[sub_of(r[q])], 1u);
  } else {
    for (uint64_t e = beg + threadIdx.x; e < end; e += SPLIT_T) atomicAdd(&cnt[sub_of(load_rec(a.rec, e))], 1u);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t run = 0;
    for (uint32_t j = 0; j < S; ++j) {
      cur[j] = run;
      a.out_off[uint64_t(b) * S + j] = beg + run;
      run += cnt[j];
    }
  }
  __syncthreads();
  if (held) {
#pragma unroll
    for (int q = 0; q < SPLIT_RPT; ++q)
      if (beg + threadIdx.x + uint64_t(q) * SPLIT_T < end) {
        const uint32_t at = atomicAdd(&cur[sub_of(r[q])], 1u);
        *reinterpret_cast<uint4*>(a.out + beg + at) = r[q];
      }
  } else {
    for (uint64_t e = beg + threadIdx.x; e < end; e += SPLIT_T) {
      const uint4 x = load_rec(a.rec, e);
      const uint32_t at = atomicAdd(&cur[sub_of(x)], 1u);
      *reinterpret_cast<uint4*>(a.out + beg + at) = x;
    }
  }
  if (b + 1 == gridDim.x && threadIdx.x == 0) a.out_off[uint64_t(gridDim.x) * S] = end;
}

// Exclusive scans of the per-bucket live and tombstone counts in one workgroup (each thread owns a
// run of ceil(nb / 1024) buckets: 8 for K3's 2^13, 64 for a split replay's 2^16); off[nb] is the total.
// With `bstats` it also sums the buckets' {live, tomb, size, live sum, tomb sum} into totals[0, 2, 1,
// 5, 6] (r06: k_sum_stats' launch folded in).
constexpr int SSCAN_T = 1024;
__global__ void __launch_bounds__(SSCAN_T) k_survivor_scan(const uint32_t* lc, const uint32_t* tc, uint32_t nb,
                                                           uint64_t* loff, uint64_t* toff,
                                                           const unsigned long long* bstats,
                                                           unsigned long long* totals) {
  __shared__ unsigned long long ws[2][SSCAN_T / 64];
  __shared__ unsigned long long red[5][SSCAN_T / 64];
  const uint32_t per = (nb + SSCAN_T - 1) / SSCAN_T;
  const uint32_t b0 = min(nb, threadIdx.x * per), b1 = min(nb, b0 + per);
  unsigned long long sl = 0, st = 0;
  for (uint32_t b = b0; b < b1; ++b) { sl += lc[b]; st += tc[b]; }
  if (bstats) {  // block-uniform; bucket b by thread b mod 1024 (consecutive threads, consecutive rows)
    unsigned long long s[5] = {0, 0, 0, 0, 0};
    for (uint32_t b = threadIdx.x; b < nb; b += SSCAN_T)
      for (int k = 0; k < 5; ++k) s[k] += bstats[uint64_t(b) * 5 + k];
    for (int k = 0; k < 5; ++k)
      for (int o = 32; o > 0; o >>= 1) s[k] += __shfl_down(s[k], o, 64);
    if ((threadIdx.x & 63) == 0)
      for (int k = 0; k < 5; ++k) red[k][threadIdx.x >> 6] = s[k];
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  unsigned long long il = sl, it = st;
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long xl = __shfl_up(il, o, 64), xt = __shfl_up(it, o, 64);
    if (lane >= o) { il += xl; it += xt; }
  }
  if (lane == 63) { ws[0][wv] = il; ws[1][wv] = it; }
  __syncthreads();
  unsigned long long ol = il - sl, ot = it - st;
  for (int w = 0; w < wv; ++w) { ol += ws[0][w]; ot += ws[1][w]; }
  for (uint32_t b = b0; b < b1; ++b) {
    loff[b] = ol; toff[b] = ot;
    ol += lc[b]; ot += tc[b];
  }
  if (threadIdx.x == SSCAN_T - 1) { loff[nb] = ol; toff[nb] = ot; }
  if (bstats && threadIdx.x < 5) {  // (red was written before the scan's barrier)
    unsigned long long v = 0;
    for (int w = 0; w < SSCAN_T / 64; ++w) v += red[threadIdx.x][w];
    const int slot[5] = {0, 2, 1, 5, 6};
    totals[slot[threadIdx.x]] = v;
  }
}

}  // namespace dev

uint64_t scan_scratch_bytes(uint64_t n) {
  return (n / dev::SCAN_T + 2) * sizeof(uint64_t);
}

void launch_scan_u32(const uint32_t* in, uint64_t* out, uint64_t n, ScanScratch scratch, hipStream_t st) {
  uint64_t nb = (n + dev::SCAN_T - 1) / dev::SCAN_T;
  if (nb == 0) {
    (void)hipMemsetAsync(out, 0, sizeof(uint64_t), st);
    return;
  }
  if (!scratch.p || scratch.bytes < scan_scratch_bytes(n))
    throw std::runtime_error("scan of " + std::to_string(n) + " counts needs " + std::to_string(scan_scratch_bytes(n)) +
                             " scratch bytes, the caller's scratch holds " + std::to_string(scratch.bytes));
  uint64_t* sums = static_cast<uint64_t*>(scratch.p);
  DR_LAUNCH(dev::k_scan_reduce, dim3(unsigned(nb)), dim3(dev::SCAN_T), 0, st, in, n, sums);
  DR_LAUNCH(dev::k_scan_single, dim3(1), dim3(dev::SCAN_T), 0, st, sums, nb);
  DR_LAUNCH(dev::k_scan_apply, dim3(unsigned(nb)), dim3(dev::SCAN_T), 0, st, in, n, sums, out);
}

void launch_canon(const CanonArgs& a, hipStream_t st) {
  if (a.n) DR_LAUNCH(dev::k_canon, dim3(unsigned((a.n + 255) / 256)), dim3(256), 0, st, a);
}

uint32_t part_tiles(uint64_t n) { return uint32_t((n + dev::PART_TILE - 1) / dev::PART_TILE); }
uint32_t part_max_bucket_bits() { return dev::PART_MAX_BITS; }

void launch_bucket_hist(const PartitionArgs& a, hipStream_t st) {
  if (a.ntiles) DR_LAUNCH(dev::k_bucket_hist, dim3(a.ntiles), dim3(dev::PART_T), 0, st, a);
}

void launch_bucket_scatter(const PartitionArgs& a, hipStream_t st) {
  if (a.ntiles) DR_LAUNCH(dev::k_bucket_scatter, dim3(8 * ((a.ntiles + 7) / 8)), dim3(dev::PART_T), 0, st, a);
}

void launch_bucket_offsets(const uint64_t* tile_off, uint32_t nb, uint32_t nt, uint64_t* bucket_off, hipStream_t st) {
  DR_LAUNCH(dev::k_bucket_offsets, dim3((nb + 1 + 255) / 256), dim3(256), 0, st, tile_off, nb, nt, bucket_off);
}

void launch_bucket_reduce(const ReduceArgs& a, hipStream_t st) {
  if (a.nbuckets) DR_LAUNCH(dev::k_bucket_reduce, dim3(a.nbuckets), dim3(dev::RED_T), 0, st, a);
}

void launch_bucket_verify(const ReduceArgs& a, hipStream_t st) {
  if (a.nbuckets) DR_LAUNCH(dev::k_bucket_verify, dim3(a.nbuckets), dim3(dev::VER_T), 0, st, a);
}

void launch_bucket_reduce64(const ReduceArgs& a, const uint32_t* buckets, uint32_t nb, hipStream_t st,
                            const unsigned long long* count) {
  const uint32_t g = count ? std::min(nb, 256u) : nb;
  if (nb) DR_LAUNCH(dev::k_bucket_reduce64, dim3(g), dim3(dev::RED_T), 0, st, a, buckets, nb, count);
}

void launch_bucket_exact(const ReduceArgs& a, const uint32_t* buckets, uint32_t nb, hipStream_t st,
                         const unsigned long long* count) {
  const uint32_t g = count ? std::min(nb, 256u) : nb;
  if (nb) DR_LAUNCH(dev::k_bucket_exact, dim3(g), dim3(dev::RED_T), 0, st, a, buckets, nb, count);
}

void launch_sum_stats(const ReduceArgs& a, hipStream_t st) {
  DR_LAUNCH(dev::k_sum_stats, dim3(1), dim3(1024), 0, st, a.bstats, a.nbuckets, a.totals);
}

void launch_compact(const CompactArgs& a, hipStream_t st) {
  if (a.nbuckets) DR_LAUNCH(dev::k_compact, dim3(a.nbuckets), dim3(64), 0, st, a);
}

void launch_compact2(const CompactArgs& live, const CompactArgs& tomb, hipStream_t st) {
  if (live.nbuckets) DR_LAUNCH(dev::k_compact2, dim3(live.nbuckets, 2), dim3(64), 0, st, live, tomb);
}

void launch_bucket_split(const SplitArgs& a, uint32_t nbuckets, hipStream_t st) {
  if (a.sbits < 1 || a.sbits > 6) throw std::runtime_error("bucket split: 1..6 refinement bits");
  if (nbuckets) DR_LAUNCH(dev::k_bucket_split, dim3(nbuckets), dim3(dev::SPLIT_T), 0, st, a);
}

void launch_survivor_scan(const uint32_t* lc, const uint32_t* tc, uint32_t nb, uint64_t* loff, uint64_t* toff,
                          hipStream_t st, const unsigned long long* bstats, unsigned long long* totals) {
  // each thread scans a run of ceil(nb / 1024) buckets, so any count works (a 2^13-bucket
  // K3 refined by 6 bits gives K4 2^19 buckets past ~2^29 actions); the bound only catches garbage
  if (nb > (1u << 26)) throw std::runtime_error("survivor scan: too many buckets");
  DR_LAUNCH(dev::k_survivor_scan, dim3(1), dim3(dev::SSCAN_T), 0, st, lc, tc, nb, loff, toff, bstats, totals);
}

}  // namespace dr
