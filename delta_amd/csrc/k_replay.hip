// K3/K4: path-hash partition + per-bucket last-writer-wins (replaces the shuffle
// `repartition(50, coalesce(add.path, remove.path))` + `sortWithinPartitions("file")` +
// InMemoryLogReplay.append/checkpoint, D/Snapshot.scala:103-110,
// D/actions/InMemoryLogReplay.scala:43-77).
//
// Records {key = xxh64(path), meta = action_index << 2 | class} are radix-partitioned on the top
// `bucket_bits` of the key (one LDS-aggregated pass). Each bucket is then reduced by one
// workgroup: an LDS open-addressing table keyed by the 64-bit path key keeps atomicMax(meta),
// i.e. the action with the largest (version, line) ordinal wins -- exactly the reference's
// "last action per path" (action index order == input_file_name order, stable within a file).
// Losers are byte-verified against their winner (hash collisions are resolved exactly by
// k_bucket_exact). Winners are compacted and bitonic-sorted by key in LDS, so the state is stored
// hash-ordered per bucket (deterministic, and ready for incremental merges).
#include "dev_common.h"
#include "kernels.h"

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
// Replay key of a canonical path: java.net.URI equality treats "file:///x" and "file:/x" alike.
__device__ __forceinline__ uint32_t key_skip(const uint8_t* p, uint32_t n) {
  return (n >= 8 && p[0] == 'f' && p[1] == 'i' && p[2] == 'l' && p[3] == 'e' && p[4] == ':' && p[5] == '/' &&
          p[6] == '/' && p[7] == '/') ? 2u : 0u;
}
__device__ bool key_equal(const uint8_t* a, uint32_t an, const uint8_t* b, uint32_t bn) {
  const uint32_t sa = key_skip(a, an), sb = key_skip(b, bn);
  if (an - sa != bn - sb) return false;
  // compare "file:" (5 bytes) then the remainder after the skipped "//"
  if (sa | sb) {
    for (uint32_t i = 0; i < 5; ++i) if (a[i] != b[i]) return false;
    return bytes_equal(a + 5 + sa, b + 5 + sb, an - sa - 5);
  }
  return bytes_equal(a, b, an);
}

__global__ void k_canon(CanonArgs a) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  const uint8_t f = a.act.flags[i];
  if (!(f & F_SPECIAL_PATH)) return;
  const uint8_t* src = reinterpret_cast<const uint8_t*>(a.act.path_ptr[i]);
  const uint32_t n = a.act.path_len[i];
  const uint64_t need = 2ull * (n + 8) + 16;
  const unsigned long long at = atomicAdd(reinterpret_cast<unsigned long long*>(a.arena_fill), (unsigned long long)need);
  if (at + need > a.arena_cap) return;  // host sized the arena from the same counters
  uint8_t* out = a.arena + at;
  uint32_t m;
  uint8_t* body = out + 7;  // room for a "file://" prefix
  if (f & F_PATH_ESCAPED) m = json_unescape(src, n, body);
  else { for (uint32_t k = 0; k < n; ++k) body[k] = src[k]; m = n; }
  uint8_t* res = body;
  if (m > 0 && body[0] == '/') {
    // Hadoop Path normalisation ('//' collapse, no trailing '/'), then makeQualified on the local
    // filesystem: scheme "file", empty authority -> "file://" + path.
    uint32_t w = 0;
    for (uint32_t k = 0; k < m; ++k) {
      if (body[k] == '/' && w > 0 && body[w - 1] == '/') continue;
      body[w++] = body[k];
    }
    if (w > 1 && body[w - 1] == '/') --w;
    res = out;
    const char pre[7] = {'f', 'i', 'l', 'e', ':', '/', '/'};
    for (int k = 0; k < 7; ++k) out[k] = uint8_t(pre[k]);
    m = w + 7;
  }
  // key bytes (URI-equality form) for hashing, written after the output string
  uint8_t* kb = res + m + 8;
  const uint32_t sk = key_skip(res, m);
  uint32_t kn = 0;
  for (uint32_t k = 0; k < m; ++k) {
    if (sk && (k == 5 || k == 6)) continue;
    kb[kn++] = res[k];
  }
  a.act.path_ptr[i] = reinterpret_cast<uint64_t>(res);
  a.act.path_len[i] = m;
  a.act.key[i] = path_key(kb, kn);
}

// ---- partition --------------------------------------------------------------------------------------
__device__ __forceinline__ bool is_file_action(uint8_t kind, uint8_t flags) {
  return (kind == K_ADD || kind == K_REMOVE) && !(flags & F_PATH_NULL);
}
__device__ __forceinline__ uint32_t bucket_of(uint64_t key, int bits) {
  return bits ? uint32_t(key >> (64 - bits)) : 0u;
}

constexpr int PART_T = 256;
constexpr int PART_ITEMS = 16;               // actions per thread
constexpr int PART_TILE = PART_T * PART_ITEMS;
constexpr int LDS_HIST_MAX = 8192;           // buckets aggregated in LDS

__global__ void __launch_bounds__(PART_T) k_bucket_hist(PartitionArgs a) {
  __shared__ uint32_t hist[LDS_HIST_MAX];
  const uint32_t nb = 1u << a.bucket_bits;
  const bool lds = nb <= LDS_HIST_MAX;
  if (lds) for (uint32_t b = threadIdx.x; b < nb; b += PART_T) hist[b] = 0;
  __syncthreads();
  const uint64_t base = uint64_t(blockIdx.x) * PART_TILE;
  for (int k = 0; k < PART_ITEMS; ++k) {
    const uint64_t i = base + uint64_t(k) * PART_T + threadIdx.x;
    if (i >= a.n || !is_file_action(a.kind[i], a.flags[i])) continue;
    const uint32_t b = bucket_of(a.key[i], a.bucket_bits);
    if (lds) atomicAdd(&hist[b], 1u); else atomicAdd(&a.bucket_count[b], 1u);
  }
  __syncthreads();
  if (lds)
    for (uint32_t b = threadIdx.x; b < nb; b += PART_T)
      if (hist[b]) atomicAdd(&a.bucket_count[b], hist[b]);
}

__global__ void __launch_bounds__(PART_T) k_bucket_scatter(PartitionArgs a) {
  __shared__ uint32_t hist[LDS_HIST_MAX];
  __shared__ uint32_t gbase[LDS_HIST_MAX];
  const uint32_t nb = 1u << a.bucket_bits;
  const bool lds = nb <= LDS_HIST_MAX;
  if (lds) for (uint32_t b = threadIdx.x; b < nb; b += PART_T) hist[b] = 0;
  __syncthreads();
  const uint64_t base = uint64_t(blockIdx.x) * PART_TILE;
  uint32_t rank[PART_ITEMS];
  uint32_t bk[PART_ITEMS];
  for (int k = 0; k < PART_ITEMS; ++k) {
    const uint64_t i = base + uint64_t(k) * PART_T + threadIdx.x;
    bk[k] = 0xffffffffu;
    if (i >= a.n || !is_file_action(a.kind[i], a.flags[i])) continue;
    const uint32_t b = bucket_of(a.key[i], a.bucket_bits);
    bk[k] = b;
    if (lds) rank[k] = atomicAdd(&hist[b], 1u);
    else rank[k] = atomicAdd(&a.bucket_count[b], 1u);
  }
  __syncthreads();
  if (lds)
    for (uint32_t b = threadIdx.x; b < nb; b += PART_T)
      if (hist[b]) gbase[b] = atomicAdd(&a.bucket_count[b], hist[b]);
  __syncthreads();
  for (int k = 0; k < PART_ITEMS; ++k) {
    if (bk[k] == 0xffffffffu) continue;
    const uint64_t i = base + uint64_t(k) * PART_T + threadIdx.x;
    const uint32_t b = bk[k];
    const uint64_t pos = a.bucket_off[b] + (lds ? gbase[b] + rank[k] : rank[k]);
    uint32_t cls = C_ADD;
    if (a.kind[i] == K_REMOVE) {
      // RemoveFile.delTimestamp = deletionTimestamp.getOrElse(0) (D/actions/actions.scala:318-319);
      // kept iff delTimestamp > minFileRetentionTimestamp (D/actions/InMemoryLogReplay.scala:67-69)
      const int64_t dt = (a.flags[i] & F_HAS_DELTS) ? a.delts[i] : 0;
      cls = dt > a.cutoff ? C_REMOVE_KEEP : C_REMOVE_DROP;
    }
    a.rec_key[pos] = a.key[i];
    a.rec_meta[pos] = uint32_t(i << 2) | cls;
  }
}

// ---- per-bucket reduce ------------------------------------------------------------------------------
constexpr int RED_T = 256;
constexpr int TS = 4096;  // LDS table slots (keys 32 KiB + metas 16 KiB)

__device__ __forceinline__ uint32_t sub_of(uint64_t key, int bits, int sbits) {
  return sbits ? uint32_t((key << bits) >> (64 - sbits)) : 0u;
}

__global__ void __launch_bounds__(RED_T) k_bucket_reduce(ReduceArgs a) {
  __shared__ unsigned long long tkey[TS];
  __shared__ uint32_t tval[TS];
  __shared__ uint32_t spos[TS];   // compacted survivors (slot indices), later sorted
  __shared__ uint32_t nsurv, collide, overflow;
  __shared__ uint32_t wl[RED_T / 64], wt[RED_T / 64];
  const uint32_t b = blockIdx.x;
  const uint64_t beg = a.bucket_off[b], end = a.bucket_off[b + 1];
  const uint64_t m = end - beg;
  // sub-passes keep the distinct keys per pass well under the table size
  int sbits = 0;
  while ((m >> sbits) > uint64_t(TS / 2)) ++sbits;
  if (threadIdx.x == 0) { collide = 0; overflow = 0; }
  uint64_t live = 0, tomb = 0, size_sum = 0, lks = 0, tks = 0;
  uint32_t live_w = 0, tomb_w = 0;  // survivors written so far (block-uniform)
  for (uint32_t sp = 0; sp < (1u << sbits); ++sp) {
    __syncthreads();
    for (int s = threadIdx.x; s < TS; s += RED_T) { tkey[s] = 0; tval[s] = 0; }
    if (threadIdx.x == 0) nsurv = 0;
    __syncthreads();
    // insert: table[key] = max(meta)  (largest action index wins)
    for (uint64_t e = beg + threadIdx.x; e < end; e += RED_T) {
      const uint64_t k = a.rec_key[e];
      if (sub_of(k, a.bucket_bits, sbits) != sp) continue;
      const uint32_t mt = a.rec_meta[e];
      uint32_t s = uint32_t(k) & (TS - 1);
      for (int probe = 0;; ++probe) {
        if (probe >= TS) { overflow = 1; break; }
        const unsigned long long old = atomicCAS(&tkey[s], 0ull, (unsigned long long)k);
        if (old == 0ull || old == k) { atomicMax(&tval[s], mt + 1u); break; }
        s = (s + 1) & (TS - 1);
      }
    }
    __syncthreads();
    if (overflow) break;
    // winners: aggregates; losers: verify their path equals the winner's
    for (uint64_t e = beg + threadIdx.x; e < end; e += RED_T) {
      const uint64_t k = a.rec_key[e];
      if (sub_of(k, a.bucket_bits, sbits) != sp) continue;
      const uint32_t mt = a.rec_meta[e];
      uint32_t s = uint32_t(k) & (TS - 1);
      while (tkey[s] != k) s = (s + 1) & (TS - 1);
      const uint32_t w = tval[s] - 1u;
      const uint32_t idx = mt >> 2;
      if (w == mt) {
        if ((mt & 3) == C_ADD) { ++live; size_sum += uint64_t(a.size[idx]); lks += k; }
        else if ((mt & 3) == C_REMOVE_KEEP) { ++tomb; tks += k; }
      } else if (a.verify_bytes) {
        const uint32_t wi = w >> 2;
        const uint8_t* p = reinterpret_cast<const uint8_t*>(a.path_ptr[idx]);
        const uint8_t* q = reinterpret_cast<const uint8_t*>(a.path_ptr[wi]);
        if (!key_equal(p, a.path_len[idx], q, a.path_len[wi])) collide = 1;
      }
    }
    // compact surviving slots
    for (int s = threadIdx.x; s < TS; s += RED_T) {
      const uint32_t v = tval[s];
      if (v && ((v - 1u) & 3) != C_REMOVE_DROP) spos[atomicAdd(&nsurv, 1u)] = uint32_t(s);
    }
    __syncthreads();
    // bitonic sort of the survivors by key (pad to a power of two with sentinel slots)
    const uint32_t ns = nsurv;
    uint32_t np = 1;
    while (np < ns) np <<= 1;
    for (uint32_t t = ns + threadIdx.x; t < np; t += RED_T) spos[t] = 0xffffffffu;
    __syncthreads();
    for (uint32_t ksz = 2; ksz <= np; ksz <<= 1) {
      for (uint32_t j = ksz >> 1; j > 0; j >>= 1) {
        for (uint32_t t = threadIdx.x; t < np; t += RED_T) {
          const uint32_t u = t ^ j;
          if (u > t) {
            const uint32_t x = spos[t], y = spos[u];
            // sentinels (0xffffffff) order after every real key
            const bool gt = x == 0xffffffffu ? (y != 0xffffffffu)
                                             : (y == 0xffffffffu ? false : tkey[x] > tkey[y]);
            const bool up = (t & ksz) == 0;
            if (gt == up) { spos[t] = y; spos[u] = x; }
          }
        }
        __syncthreads();
      }
    }
    // write survivors in key order: live and tombstone lists, via per-wave ballots
    for (uint32_t base = 0; base < ns; base += RED_T) {
      const uint32_t t = base + threadIdx.x;
      uint32_t v = 0;
      if (t < ns) v = tval[spos[t]] - 1u;
      const bool isl = t < ns && (v & 3) == C_ADD;
      const bool ist = t < ns && (v & 3) == C_REMOVE_KEEP;
      const unsigned long long bl = __ballot(isl), bt = __ballot(ist);
      const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
      const unsigned long long lt = (1ull << lane) - 1ull;
      if (lane == 0) { wl[wv] = uint32_t(__popcll(bl)); wt[wv] = uint32_t(__popcll(bt)); }
      __syncthreads();
      uint32_t ol = 0, ot = 0, sl = 0, st = 0;
      for (int k = 0; k < RED_T / 64; ++k) {
        if (k < wv) { ol += wl[k]; ot += wt[k]; }
        sl += wl[k]; st += wt[k];
      }
      if (isl) a.out_live[beg + live_w + ol + uint32_t(__popcll(bl & lt))] = v >> 2;
      if (ist) a.out_tomb[beg + tomb_w + ot + uint32_t(__popcll(bt & lt))] = v >> 2;
      live_w += sl;
      tomb_w += st;
      __syncthreads();
    }
  }
  // block totals
  __shared__ unsigned long long red[5][RED_T / 64];
  for (int o = 32; o > 0; o >>= 1) {
    live += __shfl_down(live, o, 64);
    tomb += __shfl_down(tomb, o, 64);
    size_sum += __shfl_down(size_sum, o, 64);
    lks += __shfl_down(lks, o, 64);
    tks += __shfl_down(tks, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = live; red[1][threadIdx.x >> 6] = tomb; red[2][threadIdx.x >> 6] = size_sum;
    red[3][threadIdx.x >> 6] = lks; red[4][threadIdx.x >> 6] = tks;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long L = 0, T = 0, S = 0, LK = 0, TK = 0;
    for (int k = 0; k < RED_T / 64; ++k) {
      L += red[0][k]; T += red[1][k]; S += red[2][k]; LK += red[3][k]; TK += red[4][k];
    }
    if (collide || overflow) {
      a.live_count[b] = 0;
      a.tomb_count[b] = 0;
      if (collide) {
        const unsigned long long c = atomicAdd(&a.totals[3], 1ull);
        a.collide_list[c] = b;
      } else {
        const unsigned long long c = atomicAdd(&a.totals[4], 1ull);
        a.overflow_list[c] = b;
      }
    } else {
      a.live_count[b] = live_w;
      a.tomb_count[b] = tomb_w;
      atomicAdd(&a.totals[0], L);
      atomicAdd(&a.totals[1], S);
      atomicAdd(&a.totals[2], T);
      atomicAdd(&a.totals[5], LK);
      atomicAdd(&a.totals[6], TK);
    }
  }
}

// Exact fallback for buckets with a 64-bit key collision (or an LDS table overflow): each record
// is a winner iff no other record with an equal path has a larger action index. O(m^2) per bucket;
// only reached on collisions, which a 64-bit hash makes vanishingly rare.
__global__ void __launch_bounds__(RED_T) k_bucket_exact(ReduceArgs a, const uint32_t* buckets) {
  __shared__ uint32_t nl, nt;
  __shared__ unsigned long long red[5][RED_T / 64];
  const uint32_t b = buckets[blockIdx.x];
  const uint64_t beg = a.bucket_off[b], end = a.bucket_off[b + 1];
  if (threadIdx.x == 0) { nl = 0; nt = 0; }
  __syncthreads();
  uint64_t live = 0, tomb = 0, size_sum = 0, lks = 0, tks = 0;
  for (uint64_t e = beg + threadIdx.x; e < end; e += RED_T) {
    const uint64_t k = a.rec_key[e];
    const uint32_t mt = a.rec_meta[e];
    const uint32_t idx = mt >> 2;
    const uint8_t* p = reinterpret_cast<const uint8_t*>(a.path_ptr[idx]);
    const uint32_t pn = a.path_len[idx];
    bool win = true;
    for (uint64_t f = beg; f < end && win; ++f) {
      if (f == e || a.rec_key[f] != k) continue;
      const uint32_t mf = a.rec_meta[f];
      if ((mf >> 2) <= idx) continue;
      const uint32_t j = mf >> 2;
      if (key_equal(p, pn, reinterpret_cast<const uint8_t*>(a.path_ptr[j]), a.path_len[j])) win = false;
    }
    if (!win) continue;
    if ((mt & 3) == C_ADD) {
      ++live;
      size_sum += uint64_t(a.size[idx]);
      lks += k;
      a.out_live[beg + atomicAdd(&nl, 1u)] = idx;
    } else if ((mt & 3) == C_REMOVE_KEEP) {
      ++tomb;
      tks += k;
      a.out_tomb[beg + atomicAdd(&nt, 1u)] = idx;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    live += __shfl_down(live, o, 64);
    tomb += __shfl_down(tomb, o, 64);
    size_sum += __shfl_down(size_sum, o, 64);
    lks += __shfl_down(lks, o, 64);
    tks += __shfl_down(tks, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = live; red[1][threadIdx.x >> 6] = tomb; red[2][threadIdx.x >> 6] = size_sum;
    red[3][threadIdx.x >> 6] = lks; red[4][threadIdx.x >> 6] = tks;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long L = 0, T = 0, S = 0, LK = 0, TK = 0;
    for (int k = 0; k < RED_T / 64; ++k) {
      L += red[0][k]; T += red[1][k]; S += red[2][k]; LK += red[3][k]; TK += red[4][k];
    }
    a.live_count[b] = nl;
    a.tomb_count[b] = nt;
    atomicAdd(&a.totals[0], L);
    atomicAdd(&a.totals[1], S);
    atomicAdd(&a.totals[2], T);
    atomicAdd(&a.totals[5], LK);
    atomicAdd(&a.totals[6], TK);
  }
}

__global__ void k_compact(CompactArgs a) {
  const uint32_t b = blockIdx.x;
  if (b >= a.nbuckets) return;
  const uint32_t c = a.counts[b];
  const uint64_t src = a.bucket_off[b], dst = a.dst_off[b];
  for (uint32_t k = threadIdx.x; k < c; k += blockDim.x) a.dst[dst + k] = a.src[src + k];
}

}  // namespace dev

uint64_t scan_scratch_bytes(uint64_t n) {
  return (n / dev::SCAN_T + 2) * sizeof(uint64_t);
}

void launch_scan_u32(const uint32_t* in, uint64_t* out, uint64_t n, void* scratch, hipStream_t st) {
  uint64_t nb = (n + dev::SCAN_T - 1) / dev::SCAN_T;
  if (nb == 0) {
    (void)hipMemsetAsync(out, 0, sizeof(uint64_t), st);
    return;
  }
  uint64_t* sums = static_cast<uint64_t*>(scratch);
  hipLaunchKernelGGL(dev::k_scan_reduce, dim3(unsigned(nb)), dim3(dev::SCAN_T), 0, st, in, n, sums);
  hipLaunchKernelGGL(dev::k_scan_single, dim3(1), dim3(dev::SCAN_T), 0, st, sums, nb);
  hipLaunchKernelGGL(dev::k_scan_apply, dim3(unsigned(nb)), dim3(dev::SCAN_T), 0, st, in, n, sums, out);
}

void launch_canon(const CanonArgs& a, hipStream_t st) {
  if (a.n) hipLaunchKernelGGL(dev::k_canon, dim3(unsigned((a.n + 255) / 256)), dim3(256), 0, st, a);
}

void launch_bucket_hist(const PartitionArgs& a, hipStream_t st) {
  uint64_t nb = (a.n + dev::PART_TILE - 1) / dev::PART_TILE;
  if (nb) hipLaunchKernelGGL(dev::k_bucket_hist, dim3(unsigned(nb)), dim3(dev::PART_T), 0, st, a);
}

void launch_bucket_scatter(const PartitionArgs& a, hipStream_t st) {
  uint64_t nb = (a.n + dev::PART_TILE - 1) / dev::PART_TILE;
  if (nb) hipLaunchKernelGGL(dev::k_bucket_scatter, dim3(unsigned(nb)), dim3(dev::PART_T), 0, st, a);
}

void launch_bucket_reduce(const ReduceArgs& a, hipStream_t st) {
  if (a.nbuckets) hipLaunchKernelGGL(dev::k_bucket_reduce, dim3(a.nbuckets), dim3(dev::RED_T), 0, st, a);
}

void launch_bucket_exact(const ReduceArgs& a, const uint32_t* buckets, uint32_t nb, hipStream_t st) {
  if (nb) hipLaunchKernelGGL(dev::k_bucket_exact, dim3(nb), dim3(dev::RED_T), 0, st, a, buckets);
}

void launch_compact(const CompactArgs& a, hipStream_t st) {
  if (a.nbuckets) hipLaunchKernelGGL(dev::k_compact, dim3(a.nbuckets), dim3(64), 0, st, a);
}

}  // namespace dr
