// Multi-GPU path-hash sharding: every path-keyed action depends only on actions with
// the same path, so after the local parse each rank sends its file actions to owner(path) and every
// owner runs K3/K4 on its shard alone. Records leave a rank grouped by owner and, inside a group, in
// the rank's replay order; ranks hold contiguous slices of the segment (checkpoint row groups, then
// commits), so an owner that concatenates what it receives in rank order sees its actions in the
// global replay order -- last-writer-wins needs nothing else. The owner's verdicts (live / kept
// tombstone / dropped) travel back to the sender, which owns the full record bytes for export.
#include "dev_common.h"
#include "kernels.h"

namespace dr {
namespace dev {

constexpr int SH_T = 256;
constexpr int SH_ITEMS = 16;
constexpr int SH_TILE = SH_T * SH_ITEMS;
constexpr int SH_MAXW = 64;

__device__ __forceinline__ bool shard_sends(uint8_t kind, uint8_t flags) {
  return (kind == K_ADD || kind == K_REMOVE) && !(flags & F_PATH_NULL);
}
// owner(key): the low 32 key bits scaled to [0, world). The partition inside an owner uses the top
// key bits (bucket_of), so the two are independent.
__device__ __forceinline__ uint32_t owner_of(uint64_t key, uint32_t world) {
  return uint32_t((uint64_t(uint32_t(key)) * world) >> 32);
}

// per-tile counts and canonical path bytes per owner, stored owner-major: blk_count[d * ntiles + tile]
// (a tile's bytes are stored saturated at 2^32 - 1, which k_shard_sizes reports as an error)
constexpr uint32_t SH_BYTES_SAT = 0xffffffffu;
__global__ void __launch_bounds__(SH_T) k_shard_count(ShardArgs a) {
  __shared__ uint32_t h[SH_MAXW];
  __shared__ unsigned long long hb[SH_MAXW];
  for (int d = threadIdx.x; d < SH_MAXW; d += SH_T) { h[d] = 0; hb[d] = 0; }
  __syncthreads();
  const uint64_t base = uint64_t(blockIdx.x) * SH_TILE;
  for (int k = 0; k < SH_ITEMS; ++k) {
    const uint64_t i = base + uint64_t(k) * SH_T + threadIdx.x;
    if (i < a.n && shard_sends(a.kind[i], a.flags[i])) {
      const uint32_t d = owner_of(a.key[i], a.world);
      atomicAdd(&h[d], 1u);
      atomicAdd(&hb[d], (unsigned long long)a.path_len[i]);
    }
  }
  __syncthreads();
  for (uint32_t d = threadIdx.x; d < a.world; d += SH_T) {
    a.blk_count[uint64_t(d) * a.ntiles + blockIdx.x] = h[d];
    if (a.blk_bytes) a.blk_bytes[uint64_t(d) * a.ntiles + blockIdx.x] = uint32_t(min(hb[d], (unsigned long long)SH_BYTES_SAT));
  }
}

// per-owner send counts and path bytes from the scanned matrices: out[d] records, out[W + d] bytes,
// out[2W] non-zero when a tile's byte count saturated
__global__ void __launch_bounds__(256) k_shard_sizes(const uint32_t* blk_bytes, const uint64_t* blk_off,
                                                     const uint64_t* byte_off, uint32_t world, uint64_t ntiles,
                                                     uint64_t* out) {
  const uint32_t d = threadIdx.x;
  if (d < world) {
    out[d] = blk_off[uint64_t(d + 1) * ntiles] - blk_off[uint64_t(d) * ntiles];
    out[world + d] = byte_off[uint64_t(d + 1) * ntiles] - byte_off[uint64_t(d) * ntiles];
  }
  bool sat = false;
  for (uint64_t c = threadIdx.x; c < uint64_t(world) * ntiles; c += blockDim.x) sat |= blk_bytes[c] == SH_BYTES_SAT;
  sat = __syncthreads_or(sat);
  if (threadIdx.x == 0) out[2 * world] = sat ? 1 : 0;
}

// the partial computedState sums one rank contributes to the table-wide all-reduce: from the owner
// side's reducer totals ([0] live, [1] size, [2] tombstones, [5] / [6] key sums, [7] file actions)
// and the sender side's parse counters ([3] malformed lines)
__global__ void k_shard_partials(const unsigned long long* totals, const uint64_t* parse_ctr, int64_t n_actions,
                                 int64_t* out) {
  if (threadIdx.x != 0) return;
  out[0] = int64_t(totals[0]);
  out[1] = int64_t(totals[1]);
  out[2] = int64_t(totals[2]);
  out[3] = n_actions;
  out[4] = int64_t(totals[7]);
  out[5] = int64_t(parse_ctr[3]);
  out[6] = int64_t(totals[5]);
  out[7] = int64_t(totals[6]);
}

// stable scatter: slot = blk_off[d * ntiles + tile] + rank of the action among the tile's earlier
// actions with the same owner (ballot ranks inside a wave, LDS prefix over the waves, running cursor)
__global__ void __launch_bounds__(SH_T) k_shard_scatter(ShardArgs a) {
  __shared__ uint32_t wc[SH_T / 64][SH_MAXW];
  __shared__ uint32_t cur[SH_MAXW];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int d = threadIdx.x; d < SH_MAXW; d += SH_T) cur[d] = 0;
  const uint64_t base = uint64_t(blockIdx.x) * SH_TILE;
  const uint64_t lt = (1ull << lane) - 1ull;
  for (int k = 0; k < SH_ITEMS; ++k) {
    const uint64_t i = base + uint64_t(k) * SH_T + threadIdx.x;
    const bool s = i < a.n && shard_sends(a.kind[i], a.flags[i]);
    const uint32_t d = s ? owner_of(a.key[i], a.world) : 0xffffffffu;
    uint32_t r = 0;
    for (uint32_t q = 0; q < a.world; ++q) {
      const unsigned long long m = __ballot(d == q);
      if (d == q) r = uint32_t(__popcll(m & lt));
      if (lane == 0) wc[wv][q] = uint32_t(__popcll(m));
    }
    __syncthreads();
    if (s) {
      uint32_t before = cur[d];
      for (int w = 0; w < wv; ++w) before += wc[w][d];
      a.send_idx[a.blk_off[uint64_t(d) * a.ntiles + blockIdx.x] + before + r] = uint32_t(i);
    }
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < a.world; q += SH_T) {
      uint32_t t = 0;
      for (int w = 0; w < SH_T / 64; ++w) t += wc[w][q];
      cur[q] += t;
    }
    __syncthreads();
  }
}

// fixed-size record per sent action + its canonical path length (for the byte offsets)
__global__ void k_shard_pack(ShardArgs a, ShardRec* rec, uint32_t* plen_out) {
  const uint64_t j = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (j >= a.nsend) return;
  const uint32_t i = a.send_idx[j];
  ShardRec r;
  r.key = a.key[i];
  r.size = a.size[i];
  r.delts = a.delts[i];
  r.plen = a.path_len[i];
  r.kind = a.kind[i];
  r.flags = a.flags[i];
  r.pad = 0;
  rec[j] = r;
  plen_out[j] = r.plen;
}

// receiver: records -> action arrays (path_ptr from the scanned path offsets)
__global__ void k_shard_unpack(const ShardRec* rec, uint64_t n, const uint8_t* path_base, const uint64_t* poff,
                               ActionArrays act) {
  const uint64_t j = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const ShardRec r = rec[j];
  act.kind[j] = r.kind;
  act.flags[j] = r.flags;
  act.key[j] = r.key;
  act.size[j] = r.size;
  act.delts[j] = r.delts;
  act.path_len[j] = r.plen;
  act.path_ptr[j] = reinterpret_cast<uint64_t>(path_base + poff[j]);
  act.src_off[j] = j;
  act.src_len[j] = 0;
}

__global__ void k_shard_plen(const ShardRec* rec, uint64_t n, uint32_t* plen) {
  const uint64_t j = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (j < n) plen[j] = rec[j].plen;
}

// verdict[idx[j]] = v for the first *n_dev (<= n) entries of a survivor list (its length read on the
// device: no round trip between the reducer and the verdict return)
__global__ void k_verdict_set(const uint32_t* idx, uint64_t n, const unsigned long long* n_dev, uint8_t v,
                              uint8_t* verdict) {
  const uint64_t j = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t lim = n_dev ? min(uint64_t(*n_dev), n) : n;
  if (j < lim) verdict[idx[j]] = v;
}

__global__ void k_verdict_flags(const uint8_t* verdict, uint64_t n, uint32_t* f_live, uint32_t* f_tomb) {
  const uint64_t j = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint8_t v = verdict[j];
  f_live[j] = v == 1;
  f_tomb[j] = v == 2;
}

__global__ void k_verdict_collect(const uint8_t* verdict, const uint32_t* send_idx, uint64_t n, uint8_t want,
                                  const uint64_t* pos, uint32_t* out) {
  const uint64_t j = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (j < n && verdict[j] == want) out[pos[j]] = send_idx[j];
}

}  // namespace dev

static inline unsigned grid_for(uint64_t n, unsigned t) { return unsigned((n + t - 1) / t); }

uint64_t shard_tiles(uint64_t n) { return (n + dev::SH_TILE - 1) / dev::SH_TILE; }
uint32_t shard_max_world() { return dev::SH_MAXW; }

void launch_shard_count(const ShardArgs& a, hipStream_t st) {
  if (a.ntiles) DR_LAUNCH(dev::k_shard_count, dim3(unsigned(a.ntiles)), dim3(dev::SH_T), 0, st, a);
}
void launch_shard_scatter(const ShardArgs& a, hipStream_t st) {
  if (a.ntiles) DR_LAUNCH(dev::k_shard_scatter, dim3(unsigned(a.ntiles)), dim3(dev::SH_T), 0, st, a);
}
void launch_shard_pack(const ShardArgs& a, ShardRec* rec, uint32_t* plen, hipStream_t st) {
  if (a.nsend) DR_LAUNCH(dev::k_shard_pack, dim3(grid_for(a.nsend, 256)), dim3(256), 0, st, a, rec, plen);
}
void launch_shard_plen(const ShardRec* rec, uint64_t n, uint32_t* plen, hipStream_t st) {
  if (n) DR_LAUNCH(dev::k_shard_plen, dim3(grid_for(n, 256)), dim3(256), 0, st, rec, n, plen);
}
void launch_shard_unpack(const ShardRec* rec, uint64_t n, const uint8_t* path_base, const uint64_t* poff,
                         const ActionArrays& act, hipStream_t st) {
  if (n) DR_LAUNCH(dev::k_shard_unpack, dim3(grid_for(n, 256)), dim3(256), 0, st, rec, n, path_base, poff, act);
}
void launch_verdict_set(const uint32_t* idx, uint64_t n, const unsigned long long* n_dev, uint8_t v, uint8_t* verdict,
                        hipStream_t st) {
  if (n) DR_LAUNCH(dev::k_verdict_set, dim3(grid_for(n, 256)), dim3(256), 0, st, idx, n, n_dev, v, verdict);
}
void launch_shard_sizes(const uint32_t* blk_bytes, const uint64_t* blk_off, const uint64_t* byte_off, uint32_t world,
                        uint64_t ntiles, uint64_t* out, hipStream_t st) {
  DR_LAUNCH(dev::k_shard_sizes, dim3(1), dim3(256), 0, st, blk_bytes, blk_off, byte_off, world, ntiles, out);
}
void launch_shard_partials(const unsigned long long* totals, const uint64_t* parse_ctr, int64_t n_actions,
                           int64_t* out, hipStream_t st) {
  DR_LAUNCH(dev::k_shard_partials, dim3(1), dim3(64), 0, st, totals, parse_ctr, n_actions, out);
}
void launch_verdict_flags(const uint8_t* verdict, uint64_t n, uint32_t* f_live, uint32_t* f_tomb, hipStream_t st) {
  if (n) DR_LAUNCH(dev::k_verdict_flags, dim3(grid_for(n, 256)), dim3(256), 0, st, verdict, n, f_live, f_tomb);
}
void launch_verdict_collect(const uint8_t* verdict, const uint32_t* send_idx, uint64_t n, uint8_t want,
                            const uint64_t* pos, uint32_t* out, hipStream_t st) {
  if (n)
    DR_LAUNCH(dev::k_verdict_collect, dim3(grid_for(n, 256)), dim3(256), 0, st, verdict, send_idx, n, want,
                       pos, out);
}

}  // namespace dr
