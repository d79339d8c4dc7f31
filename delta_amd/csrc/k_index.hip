// Incremental tail apply: a device-resident open-addressing index of the
// state's winners, {xxh64 path key -> winning action + 1}. The reference rebuilds the state from the
// last checkpoint on every update (D/SnapshotManagement.scala:286-330); here a commit's file actions
// probe and update only their own keys -- last writer wins because store positions grow with
// (version, line) order, so atomicMax of (action + 1) is InMemoryLogReplay.append's "later action
// replaces" (D/actions/InMemoryLogReplay.scala:43-60) -- and the counters move by the difference
// between the old and the new winner of each touched path (retention: tombstones are kept iff
// delTimestamp > minFileRetentionTimestamp, :67-69). Every winner is byte-compared with each action
// that hit its slot, so a 64-bit key collision of two distinct paths is detected and the host falls
// back to the full K3/K4 reduction.
#include "dev_common.h"
#include "kernels.h"
#include "ix_dev.h"

namespace dr {
namespace dev {
// Index of a chain's first image: survivors [lo, hi) of a full replay (distinct paths).
__global__ void __launch_bounds__(IX_T) k_ix_build(IndexArgs a) {
  const uint64_t i = a.lo + uint64_t(blockIdx.x) * IX_T + threadIdx.x;
  if (i >= a.hi) return;
  bool fresh;
  const uint32_t s = ix_insert(a.keys, a.mask, a.key[i], &fresh);
  if (!fresh) {  // two survivors share a 64-bit key: distinct paths by construction
    atomicOr(a.ctr + IX_C_COLLIDE, 1ull);
    return;
  }
  atomicAdd(a.ctr + IX_C_NEW_SLOTS, 1ull);
  a.vals[s] = uint32_t(i + 1);
  if (a.kind[i] == K_REMOVE) tomb_append(a, i, ix_delts(a, i));
}

__global__ void __launch_bounds__(IX_T) k_ix_touch(IndexArgs a) {
  const uint64_t i = a.lo + uint64_t(blockIdx.x) * IX_T + threadIdx.x;
  if (i < a.hi) ix_touch_one(a, i);
}

__global__ void __launch_bounds__(IX_T) k_ix_delta(IndexArgs a) {
  const uint64_t i = a.lo + uint64_t(blockIdx.x) * IX_T + threadIdx.x;
  Contrib c{0, 0, 0, 0, 0};
  unsigned long long files = 0;
  if (i < a.hi) ix_delta_one(a, i, c, files);
  flush_contrib(a, c, files);
}

// Both passes for a tail of at most IX_T actions (a streamed commit): one workgroup, the passes
// separated by a barrier (the slots' atomicMax results are device-scope atomics, complete and
// visible to the workgroup after the fence and the barrier).
__global__ void __launch_bounds__(IX_T) k_ix_touch_delta(IndexArgs a) {
  const uint64_t i = a.lo + threadIdx.x;
  if (i < a.hi) ix_touch_one(a, i);
  __threadfence();
  __syncthreads();
  Contrib c{0, 0, 0, 0, 0};
  unsigned long long files = 0;
  if (i < a.hi) ix_delta_one(a, i, c, files);
  flush_contrib(a, c, files);
}

// A later cutoff expires the base's tombstones with old_cut < delTimestamp <= new_cut.
__global__ void __launch_bounds__(IX_T) k_ix_expire(IndexArgs a, uint64_t n, ReadbackArgs rb) {
  const uint64_t j = uint64_t(blockIdx.x) * IX_T + threadIdx.x;
  Contrib c{0, 0, 0, 0, 0};
  if (j < n) expire_one(a, j, c);
  flush_contrib(a, c, 0);
  if (!rb.n[0]) return;
  // the readback by the last workgroup to finish: its counters are final once every other
  // workgroup has counted itself done (each after its atomics, fenced)
  __shared__ bool last;
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(a.ctr + IX_C_DONE, 1ull) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;
  __threadfence();
#pragma unroll
  for (int s = 0; s < READBACK_SPANS; ++s)
    for (uint32_t k = threadIdx.x; k < rb.n[s]; k += IX_T)
      rb.dst[s][k] = __hip_atomic_load(rb.src[s] + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  readback_flag(rb);
}

// Keep the candidates that are still tombstones of the head at its cutoff (a.new_cut).
__global__ void __launch_bounds__(IX_T) k_ix_tomb_compact(IndexArgs a, const ulonglong2* in, uint64_t n,
                                                          ulonglong2* out) {
  const uint64_t j = uint64_t(blockIdx.x) * IX_T + threadIdx.x;
  if (j >= n) return;
  const ulonglong2 e = in[j];
  const uint64_t x = e.x;
  if (int64_t(e.y) <= a.new_cut) return;
  const uint32_t s = ix_find(a.keys, a.mask, a.key[x]);
  if (s == IX_NONE || a.vals[s] != uint32_t(x + 1)) return;
  const unsigned long long at = atomicAdd(a.ctr + IX_C_TOMB_FILL, 1ull);
  out[at] = e;
}

// Revert one apply on a copy of the values: its first touches restore the slots' previous values.
__global__ void __launch_bounds__(IX_T) k_ix_undo(IndexArgs a, uint32_t* vals, const uint2* undo, uint64_t n) {
  const uint64_t j = uint64_t(blockIdx.x) * IX_T + threadIdx.x;
  if (j >= n) return;
  const uint2 u = undo[j];
  const uint32_t s = ix_find(a.keys, a.mask, a.key[u.x]);
  if (s != IX_NONE) vals[s] = u.y;
}

__global__ void __launch_bounds__(IX_T) k_ix_classify(IndexArgs a, const uint32_t* vals, uint64_t cap, int64_t cut,
                                                      uint32_t* lf, uint32_t* tf) {
  const uint64_t s = uint64_t(blockIdx.x) * IX_T + threadIdx.x;
  if (s >= cap) return;
  const uint32_t v = vals[s];
  uint32_t l = 0, t = 0;
  if (v) {
    const uint64_t x = uint64_t(v) - 1;
    if (a.kind[x] == K_ADD) l = 1;
    else if (ix_delts(a, x) > cut) t = 1;
  }
  lf[s] = l;
  tf[s] = t;
}

__global__ void __launch_bounds__(IX_T) k_ix_emit(const uint32_t* vals, uint64_t cap, const uint32_t* lf,
                                                  const uint64_t* lp, const uint32_t* tf, const uint64_t* tp,
                                                  uint32_t* live, uint32_t* tomb) {
  const uint64_t s = uint64_t(blockIdx.x) * IX_T + threadIdx.x;
  if (s >= cap) return;
  if (lf[s]) live[lp[s]] = vals[s] - 1;
  else if (tf[s]) tomb[tp[s]] = vals[s] - 1;
}

__global__ void __launch_bounds__(IX_T) k_ix_rehash(const unsigned long long* ok, const uint32_t* ov, uint64_t ocap,
                                                    unsigned long long* nk, uint32_t* nv, uint64_t nmask) {
  const uint64_t s = uint64_t(blockIdx.x) * IX_T + threadIdx.x;
  if (s >= ocap) return;
  const unsigned long long k = ok[s];
  if (!k) return;
  bool fresh;
  const uint32_t t = ix_insert(nk, nmask, k, &fresh);
  nv[t] = ov[s];
}

}  // namespace dev

static unsigned ix_grid(uint64_t n) { return unsigned((n + dev::IX_T - 1) / dev::IX_T); }

void launch_ix_build(const IndexArgs& a, hipStream_t st) {
  if (a.hi > a.lo) DR_LAUNCH(dev::k_ix_build, dim3(ix_grid(a.hi - a.lo)), dim3(dev::IX_T), 0, st, a);
}
void launch_ix_touch(const IndexArgs& a, hipStream_t st) {
  if (a.hi - a.lo <= uint64_t(dev::IX_T)) return;  // launch_ix_delta runs both passes in one workgroup
  if (a.hi > a.lo) DR_LAUNCH(dev::k_ix_touch, dim3(ix_grid(a.hi - a.lo)), dim3(dev::IX_T), 0, st, a);
}
void launch_ix_delta(const IndexArgs& a, hipStream_t st) {
  if (a.hi <= a.lo) return;
  if (a.hi - a.lo <= uint64_t(dev::IX_T)) DR_LAUNCH(dev::k_ix_touch_delta, dim3(1), dim3(dev::IX_T), 0, st, a);
  else DR_LAUNCH(dev::k_ix_delta, dim3(ix_grid(a.hi - a.lo)), dim3(dev::IX_T), 0, st, a);
}
void launch_ix_expire(const IndexArgs& a, uint64_t n, hipStream_t st, const ReadbackArgs* rb) {
  ReadbackArgs none{};
  if (n) DR_LAUNCH(dev::k_ix_expire, dim3(ix_grid(n)), dim3(dev::IX_T), 0, st, a, n, rb ? *rb : none);
}
void launch_ix_tomb_compact(const IndexArgs& a, const ulonglong2* in, uint64_t n, ulonglong2* out, hipStream_t st) {
  if (n) DR_LAUNCH(dev::k_ix_tomb_compact, dim3(ix_grid(n)), dim3(dev::IX_T), 0, st, a, in, n, out);
}
void launch_ix_undo(const IndexArgs& a, uint32_t* vals, const uint2* undo, uint64_t n, hipStream_t st) {
  if (n) DR_LAUNCH(dev::k_ix_undo, dim3(ix_grid(n)), dim3(dev::IX_T), 0, st, a, vals, undo, n);
}
void launch_ix_classify(const IndexArgs& a, const uint32_t* vals, uint64_t cap, int64_t cut, uint32_t* lf,
                        uint32_t* tf, hipStream_t st) {
  if (cap) DR_LAUNCH(dev::k_ix_classify, dim3(ix_grid(cap)), dim3(dev::IX_T), 0, st, a, vals, cap, cut, lf, tf);
}
void launch_ix_emit(const uint32_t* vals, uint64_t cap, const uint32_t* lf, const uint64_t* lp, const uint32_t* tf,
                    const uint64_t* tp, uint32_t* live, uint32_t* tomb, hipStream_t st) {
  if (cap) DR_LAUNCH(dev::k_ix_emit, dim3(ix_grid(cap)), dim3(dev::IX_T), 0, st, vals, cap, lf, lp, tf, tp, live, tomb);
}
void launch_ix_rehash(const unsigned long long* ok, const uint32_t* ov, uint64_t ocap, unsigned long long* nk,
                      uint32_t* nv, uint64_t nmask, hipStream_t st) {
  if (ocap) DR_LAUNCH(dev::k_ix_rehash, dim3(ix_grid(ocap)), dim3(dev::IX_T), 0, st, ok, ov, ocap, nk, nv, nmask);
}

}  // namespace dr
