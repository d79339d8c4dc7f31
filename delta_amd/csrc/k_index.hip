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

namespace dr {
namespace dev {

constexpr uint32_t IX_NONE = 0xffffffffu;
constexpr int IX_T = 256;

__device__ __forceinline__ bool ix_file_action(const IndexArgs& a, uint64_t i) {
  const uint8_t k = a.kind[i];
  return (k == K_ADD || k == K_REMOVE) && !(a.flags[i] & F_PATH_NULL);
}
__device__ __forceinline__ int64_t ix_delts(const IndexArgs& a, uint64_t i) {
  return (a.flags[i] & F_HAS_DELTS) ? a.delts[i] : 0;
}
__device__ __forceinline__ bool ix_same_path(const IndexArgs& a, uint64_t i, uint64_t j) {
  return key_equal(reinterpret_cast<const uint8_t*>(a.path_ptr[i]), a.path_len[i],
                   reinterpret_cast<const uint8_t*>(a.path_ptr[j]), a.path_len[j]);
}

// slot of key k, inserted if absent; *fresh tells whether this call inserted it
__device__ uint32_t ix_insert(unsigned long long* keys, uint64_t mask, uint64_t k, bool* fresh) {
  uint64_t s = k & mask;
  *fresh = false;
  for (;;) {
    unsigned long long x = keys[s];
    if (x == 0) {
      x = atomicCAS(keys + s, 0ull, (unsigned long long)k);
      if (x == 0) {
        *fresh = true;
        return uint32_t(s);
      }
    }
    if (x == k) return uint32_t(s);
    s = (s + 1) & mask;
  }
}

__device__ uint32_t ix_find(const unsigned long long* keys, uint64_t mask, uint64_t k) {
  uint64_t s = k & mask;
  for (;;) {
    const unsigned long long x = keys[s];
    if (x == k) return uint32_t(s);
    if (x == 0) return IX_NONE;
    s = (s + 1) & mask;
  }
}

// Contribution of winner x to (files, size, removes, live checksum, tombstone checksum) at cutoff.
struct Contrib {
  unsigned long long f, sz, r, lks, tks;
};
__device__ __forceinline__ void contrib_add(Contrib& c, const IndexArgs& a, uint64_t x, int64_t cut, bool neg) {
  unsigned long long f = 0, sz = 0, r = 0, lk = 0, tk = 0;
  const unsigned long long top = a.key[x] >> 32;
  if (a.kind[x] == K_ADD) {
    f = 1;
    sz = (unsigned long long)a.size[x];
    lk = top;
  } else if (ix_delts(a, x) > cut) {
    r = 1;
    tk = top;
  }
  if (neg) { f = 0ull - f; sz = 0ull - sz; r = 0ull - r; lk = 0ull - lk; tk = 0ull - tk; }
  c.f += f; c.sz += sz; c.r += r; c.lks += lk; c.tks += tk;
}

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  return v;
}
__device__ void flush_contrib(const IndexArgs& a, Contrib c, unsigned long long files) {
  c.f = wave_sum(c.f); c.sz = wave_sum(c.sz); c.r = wave_sum(c.r);
  c.lks = wave_sum(c.lks); c.tks = wave_sum(c.tks); files = wave_sum(files);
  if ((threadIdx.x & 63) == 0) {
    if (c.f) atomicAdd(a.ctr + IX_C_FILES, c.f);
    if (c.sz) atomicAdd(a.ctr + IX_C_SIZE, c.sz);
    if (c.r) atomicAdd(a.ctr + IX_C_REMOVES, c.r);
    if (c.lks) atomicAdd(a.ctr + IX_C_LKS, c.lks);
    if (c.tks) atomicAdd(a.ctr + IX_C_TKS, c.tks);
    if (files) atomicAdd(a.ctr + IX_C_FILE_ACTIONS, files);
  }
}

__device__ __forceinline__ void tomb_append(const IndexArgs& a, uint64_t x) {
  const unsigned long long at = atomicAdd(a.ctr + IX_C_TOMB_FILL, 1ull);
  if (at < a.tomb_cap) a.tomb_list[at] = uint32_t(x);
  else atomicOr(a.ctr + IX_C_COLLIDE, 2ull);  // host sized the list: never expected
}

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
  if (a.kind[i] == K_REMOVE) tomb_append(a, i);
}

// Pass 1 of an apply: every file action of the tail claims its slot and raises it to itself.
__device__ __forceinline__ void ix_touch_one(const IndexArgs& a, uint64_t i) {
  const uint64_t t = i - a.lo;
  if (!ix_file_action(a, i)) {
    a.t_slot[t] = IX_NONE;
    return;
  }
  bool fresh;
  const uint32_t s = ix_insert(a.keys, a.mask, a.key[i], &fresh);
  if (fresh) atomicAdd(a.ctr + IX_C_NEW_SLOTS, 1ull);
  a.t_slot[t] = s;
  a.t_prev[t] = atomicMax(a.vals + s, uint32_t(i + 1));
}
__global__ void __launch_bounds__(IX_T) k_ix_touch(IndexArgs a) {
  const uint64_t i = a.lo + uint64_t(blockIdx.x) * IX_T + threadIdx.x;
  if (i < a.hi) ix_touch_one(a, i);
}

// Pass 2: the first toucher of each slot (the one whose atomicMax saw a pre-tail value) moves the
// counters from the old winner to the final one and logs the old value for older states; every
// action checks its bytes against the final winner (and the first toucher against the old one).
__device__ __forceinline__ void ix_delta_one(const IndexArgs& a, uint64_t i, Contrib& c, unsigned long long& files) {
  const uint64_t t = i - a.lo;
  const uint32_t s = a.t_slot[t];
  if (s == IX_NONE) return;
  files = 1;
  // an atomic load: in k_ix_touch_delta the slot was raised by this workgroup's atomics (at L2)
  const uint64_t w = uint64_t(__hip_atomic_load(a.vals + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) - 1;
  if (w != i && !ix_same_path(a, i, w)) atomicOr(a.ctr + IX_C_COLLIDE, 1ull);
  const uint32_t prev = a.t_prev[t];
  if (uint64_t(prev) <= a.lo) {
    if (prev) {
      const uint64_t o = uint64_t(prev) - 1;
      if (!ix_same_path(a, i, o)) atomicOr(a.ctr + IX_C_COLLIDE, 1ull);
      contrib_add(c, a, o, a.old_cut, true);
    }
    contrib_add(c, a, w, a.new_cut, false);
    if (a.kind[w] == K_REMOVE && ix_delts(a, w) > a.new_cut) tomb_append(a, w);
    const unsigned long long u = atomicAdd(a.ctr + IX_C_UNDO_FILL, 1ull);
    a.undo[u] = make_uint2(uint32_t(i), prev);
  }
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
__global__ void __launch_bounds__(IX_T) k_ix_expire(IndexArgs a, uint64_t n) {
  const uint64_t j = uint64_t(blockIdx.x) * IX_T + threadIdx.x;
  Contrib c{0, 0, 0, 0, 0};
  if (j < n) {
    const uint64_t x = a.tomb_list[j];
    if (x < a.lo) {  // this apply's own tombstones were counted at the new cutoff
      const int64_t dt = ix_delts(a, x);
      if (dt > a.old_cut && dt <= a.new_cut) {
        const uint32_t s = ix_find(a.keys, a.mask, a.key[x]);
        if (s != IX_NONE && a.vals[s] == uint32_t(x + 1)) {
          c.r = 0ull - 1ull;
          c.tks = 0ull - (unsigned long long)(a.key[x] >> 32);
        }
      }
    }
  }
  flush_contrib(a, c, 0);
}

// Keep the candidates that are still tombstones of the head at its cutoff (a.new_cut).
__global__ void __launch_bounds__(IX_T) k_ix_tomb_compact(IndexArgs a, const uint32_t* in, uint64_t n, uint32_t* out) {
  const uint64_t j = uint64_t(blockIdx.x) * IX_T + threadIdx.x;
  if (j >= n) return;
  const uint64_t x = in[j];
  if (ix_delts(a, x) <= a.new_cut) return;
  const uint32_t s = ix_find(a.keys, a.mask, a.key[x]);
  if (s == IX_NONE || a.vals[s] != uint32_t(x + 1)) return;
  const unsigned long long at = atomicAdd(a.ctr + IX_C_TOMB_FILL, 1ull);
  out[at] = uint32_t(x);
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
void launch_ix_expire(const IndexArgs& a, uint64_t n, hipStream_t st) {
  if (n) DR_LAUNCH(dev::k_ix_expire, dim3(ix_grid(n)), dim3(dev::IX_T), 0, st, a, n);
}
void launch_ix_tomb_compact(const IndexArgs& a, const uint32_t* in, uint64_t n, uint32_t* out, hipStream_t st) {
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
