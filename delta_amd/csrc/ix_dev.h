// Device side of the incremental apply's index (k_index.hip): probing, the counters' deltas and
// the two passes over a tail's file actions, shared with the small-tail apply kernel (k_json.hip
// k_apply_small).
#pragma once
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
__device__ inline uint32_t ix_insert(unsigned long long* keys, uint64_t mask, uint64_t k, bool* fresh) {
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

// ix_insert for a few keys (a streamed commit's): every probe is the compare-and-swap itself, one
// round trip to L2 per probe instead of a load and then the swap
__device__ inline uint32_t ix_insert_cas(unsigned long long* keys, uint64_t mask, uint64_t k, bool* fresh) {
  uint64_t s = k & mask;
  *fresh = false;
  for (;;) {
    const unsigned long long x = atomicCAS(keys + s, 0ull, (unsigned long long)k);
    if (x == 0) {
      *fresh = true;
      return uint32_t(s);
    }
    if (x == k) return uint32_t(s);
    s = (s + 1) & mask;
  }
}

__device__ inline uint32_t ix_find(const unsigned long long* keys, uint64_t mask, uint64_t k) {
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
__device__ inline void flush_contrib(const IndexArgs& a, Contrib c, unsigned long long files) {
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

// Expiry of tombstone candidate j (k_ix_expire, and the one-launch apply's fused expiry): a
// candidate from an earlier apply whose delTimestamp now falls at or under the cutoff leaves the
// tombstone count while it is still its path's winner. The slot value is read at L2 (the fused apply
// raised it with atomics in the same workgroup).
__device__ __forceinline__ void expire_entry(const IndexArgs& a, const ulonglong2 e, Contrib& c) {
  const uint64_t x = e.x;
  const int64_t dt = int64_t(e.y);
  if (x < a.lo && dt > a.old_cut && dt <= a.new_cut) {  // this apply's own tombstones: counted at the new cutoff
    const uint32_t s = ix_find(a.keys, a.mask, a.key[x]);
    if (s != IX_NONE && __hip_atomic_load(a.vals + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == uint32_t(x + 1)) {
      c.r += 0ull - 1ull;
      c.tks += 0ull - (unsigned long long)(a.key[x] >> 32);
    }
  }
}

__device__ __forceinline__ void expire_one(const IndexArgs& a, uint64_t j, Contrib& c) {
  expire_entry(a, a.tomb_list[j], c);
}

__device__ __forceinline__ void tomb_append(const IndexArgs& a, uint64_t x, int64_t dt) {
  const unsigned long long at = atomicAdd(a.ctr + IX_C_TOMB_FILL, 1ull);
  if (at < a.tomb_cap) a.tomb_list[at] = make_ulonglong2(x, (unsigned long long)dt);
  else atomicOr(a.ctr + IX_C_COLLIDE, 2ull);  // host sized the list: never expected
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
    if (a.kind[w] == K_REMOVE) {
      const int64_t dt = ix_delts(a, w);
      if (dt > a.new_cut) tomb_append(a, w, dt);
    }
    const unsigned long long u = atomicAdd(a.ctr + IX_C_UNDO_FILL, 1ull);
    a.undo[u] = make_uint2(uint32_t(i), prev);
  }
}

// The two passes for a tail of one workgroup (k_apply_small / k_apply_commit), one action per thread
// with its slot and previous value in registers: pass 1 also settles the base's old winner -- its
// counters and its bytes -- before the barrier, so that pass 2 waits only on the final winner.
struct IxTouch {
  uint32_t s = IX_NONE, prev = 0;
  bool old_bad = false;
  Contrib old{0, 0, 0, 0, 0};
  Contrib own{0, 0, 0, 0, 0};  // this action's own contribution as a winner (ix_touch_pre_v)
  bool own_remove = false, own_set = false;
  int64_t own_dt = 0;
};
__device__ __forceinline__ void ix_touch_pre(const IndexArgs& a, uint64_t i, IxTouch& T) {
  if (!ix_file_action(a, i)) return;
  bool fresh;
  T.s = ix_insert_cas(a.keys, a.mask, a.key[i], &fresh);
  if (fresh) atomicAdd(a.ctr + IX_C_NEW_SLOTS, 1ull);
  T.prev = atomicMax(a.vals + T.s, uint32_t(i + 1));
  if (T.prev && uint64_t(T.prev) <= a.lo) {
    const uint64_t o = uint64_t(T.prev) - 1;
    T.old_bad = !ix_same_path(a, i, o);
    contrib_add(T.old, a, o, a.old_cut, true);
  }
}
// ix_touch_pre with the action's fields in registers (the appending thread's own action), and the
// slot's value read speculatively beside the first probe: when the key sits in its home slot (the
// usual case at load <= 1/2) the old winner's fields are fetched beside the atomicMax instead of
// after it -- three dependent round trips instead of five.
struct IxOld {
  uint64_t pp, key;
  uint32_t pl;
  uint8_t kind, flags;
  int64_t size, delts;
};
__device__ __forceinline__ void ix_old_load(const IndexArgs& a, uint64_t o, IxOld& r) {
  r.pp = a.path_ptr[o];
  r.pl = a.path_len[o];
  r.kind = a.kind[o];
  r.flags = a.flags[o];
  r.key = a.key[o];
  r.size = a.size[o];
  r.delts = a.delts[o];
}
__device__ __forceinline__ void ix_touch_pre_v(const IndexArgs& a, uint64_t i, uint8_t kind, uint8_t flags, uint64_t key,
                                               uint64_t pp, uint32_t pl, int64_t size, int64_t delts, IxTouch& T) {
  if (!((kind == K_ADD || kind == K_REMOVE) && !(flags & F_PATH_NULL))) return;
  {  // as the final winner (the usual case): contrib_add's terms from registers
    const unsigned long long top = key >> 32;
    const int64_t dt = (flags & F_HAS_DELTS) ? delts : 0;
    const bool add = kind == K_ADD, tomb = !add && dt > a.new_cut;
    T.own = Contrib{add ? 1ull : 0ull, add ? (unsigned long long)size : 0ull, tomb ? 1ull : 0ull, add ? top : 0ull,
                    tomb ? top : 0ull};
    T.own_remove = tomb;
    T.own_dt = dt;
    T.own_set = true;
  }
  const uint64_t s0 = key & a.mask;
  const uint32_t spec = __hip_atomic_load(a.vals + s0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  bool fresh;
  T.s = ix_insert_cas(a.keys, a.mask, key, &fresh);
  if (fresh) atomicAdd(a.ctr + IX_C_NEW_SLOTS, 1ull);
  const uint32_t guess = (uint64_t(T.s) == s0 && !fresh) ? spec : 0u;
  IxOld r{};
  if (guess && uint64_t(guess) <= a.lo) ix_old_load(a, uint64_t(guess) - 1, r);
  T.prev = atomicMax(a.vals + T.s, uint32_t(i + 1));
  if (T.prev && uint64_t(T.prev) <= a.lo) {
    const uint64_t o = uint64_t(T.prev) - 1;
    if (T.prev != guess) ix_old_load(a, o, r);  // another tail action raised the slot first (rare)
    T.old_bad = !key_equal(reinterpret_cast<const uint8_t*>(pp), pl, reinterpret_cast<const uint8_t*>(r.pp), r.pl);
    unsigned long long f = 0, sz = 0, rr = 0, lk = 0, tk = 0;
    const unsigned long long top = r.key >> 32;
    if (r.kind == K_ADD) {
      f = 1;
      sz = (unsigned long long)r.size;
      lk = top;
    } else if (((r.flags & F_HAS_DELTS) ? r.delts : 0) > a.old_cut) {
      rr = 1;
      tk = top;
    }
    T.old = Contrib{0ull - f, 0ull - sz, 0ull - rr, 0ull - lk, 0ull - tk};
  }
}

// flush_contrib for one workgroup: per-counter sums in LDS (zeroed by the caller before a barrier),
// then one global atomic per counter
__device__ __forceinline__ void flush_contrib_block(const IndexArgs& a, const Contrib& c, unsigned long long files,
                                                    unsigned long long* sums /* 6, LDS */) {
  if (c.f) atomicAdd(sums + 0, c.f);
  if (c.sz) atomicAdd(sums + 1, c.sz);
  if (c.r) atomicAdd(sums + 2, c.r);
  if (c.lks) atomicAdd(sums + 3, c.lks);
  if (c.tks) atomicAdd(sums + 4, c.tks);
  if (files) atomicAdd(sums + 5, files);
  __syncthreads();
  const uint32_t t = threadIdx.x;
  if (t < 6 && sums[t]) atomicAdd(a.ctr + (t < 5 ? t : uint32_t(IX_C_FILE_ACTIONS)), sums[t]);
}

__device__ __forceinline__ void ix_delta_post(const IndexArgs& a, uint64_t i, const IxTouch& T, Contrib& c,
                                              unsigned long long& files) {
  if (T.s == IX_NONE) return;
  files = 1;
  const uint64_t w = uint64_t(__hip_atomic_load(a.vals + T.s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) - 1;
  if (w != i && !ix_same_path(a, i, w)) atomicOr(a.ctr + IX_C_COLLIDE, 1ull);
  if (uint64_t(T.prev) <= a.lo) {
    if (T.old_bad) atomicOr(a.ctr + IX_C_COLLIDE, 1ull);
    c.f += T.old.f; c.sz += T.old.sz; c.r += T.old.r; c.lks += T.old.lks; c.tks += T.old.tks;
    bool tomb;
    int64_t dt;
    if (w == i && T.own_set) {
      c.f += T.own.f; c.sz += T.own.sz; c.r += T.own.r; c.lks += T.own.lks; c.tks += T.own.tks;
      tomb = T.own_remove;
      dt = T.own_dt;
    } else {
      contrib_add(c, a, w, a.new_cut, false);
      dt = ix_delts(a, w);
      tomb = a.kind[w] == K_REMOVE && dt > a.new_cut;
    }
    // both slots claimed before either is written (one round trip)
    const unsigned long long u = atomicAdd(a.ctr + IX_C_UNDO_FILL, 1ull);
    const unsigned long long at = tomb ? atomicAdd(a.ctr + IX_C_TOMB_FILL, 1ull) : 0ull;
    a.undo[u] = make_uint2(uint32_t(i), T.prev);
    if (tomb) {
      if (at < a.tomb_cap) a.tomb_list[at] = make_ulonglong2(w, (unsigned long long)dt);
      else atomicOr(a.ctr + IX_C_COLLIDE, 2ull);  // host sized the list: never expected
    }
  }
}
}  // namespace dev
}  // namespace dr
