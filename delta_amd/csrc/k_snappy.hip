// K2a: parallel SNAPPY page decompression for checkpoint column chunks.
//
// A raw snappy stream is a varint length followed by literal/copy elements. The element chain is
// serial and a 1 MiB page of paths holds ~144K elements, so a per-page decoder is latency bound
// (measured 1.28 s for config 3 with one lane per page). This decoder is fully parallel:
//
//  A k_snap_spec    one lane per 256-byte chunk of compressed input parses elements
//                   *speculatively* (starting 64 bytes early as a warm-up) and records the
//                   positions it visited in the chunk (256-bit bitmap) and where it left it.
//  B k_snap_resolve one wave per page checks 64 chunks at a time with a ballot: a chunk whose
//                   true entry (the previous chunk's exit) is on its speculative chain is correct
//                   (chains that meet coincide from then on). Only breaks -- a mis-speculated
//                   chunk or one spanned by a long literal -- are walked serially.
//  C k_snap_count   per chunk: output bytes and copy elements of its true elements.
//  D k_snap_scan    per page: exclusive scan of chunk outputs (copy counts: a global scan).
//  E k_snap_emit    per chunk: literal bytes go straight to the output, copies become 8-byte
//                   records {out, len, offset}. The compressor compresses 64 KiB fragments
//                   independently, so no element straddles a fragment and no copy reaches before
//                   its fragment; violations flag the page for k_snap_serial.
//  F k_snap_exec    one 1024-thread workgroup per 64 KiB output block resolves every copied
//                   byte to its literal origin by pointer jumping on a u16 map in LDS
//                   (src[p] = p - offset; literal bytes are their own roots) and gathers it.
//
// Chunk walkers (A, C, E) stage their page bytes into LDS with coalesced loads and parse from LDS.
#include "dev_common.h"
#include "kernels.h"

namespace dr {
namespace dev {

constexpr uint32_t SNAP_CH = 256;            // compressed bytes per speculation chunk
constexpr uint32_t SNAP_BLOCK = 65536;       // snappy compressor fragment size
constexpr uint32_t SNAP_WU = 256;            // speculation warm-up bytes (0.6% mis-speculation on path pages)
constexpr uint32_t WG_CHUNKS = 256;          // chunks (threads) per chunk-walker workgroup
constexpr uint32_t STAGE_BYTES = WG_CHUNKS * SNAP_CH + SNAP_WU + 64;

struct Elem {
  uint32_t hdr;   // header bytes (tag + length/offset bytes)
  uint32_t len;   // output bytes
  uint32_t off;   // copy offset (0 for a literal)
};

__device__ __forceinline__ Elem snap_decode(uint64_t w) {
  const uint32_t tag = uint32_t(w & 0xff);
  Elem e;
  switch (tag & 3) {
    case 0: {
      const uint32_t l = tag >> 2;
      if (l < 60) { e.hdr = 1; e.len = l + 1; }
      else {
        const uint32_t nb = l - 59;
        const uint64_t v = (w >> 8) & ((nb >= 4) ? 0xffffffffull : ((1ull << (8 * nb)) - 1));
        e.hdr = 1 + nb; e.len = uint32_t(v) + 1;
      }
      e.off = 0;
      break;
    }
    case 1: e.hdr = 2; e.len = ((tag >> 2) & 7) + 4; e.off = ((tag >> 5) << 8) | uint32_t((w >> 8) & 0xff); break;
    case 2: e.hdr = 3; e.len = (tag >> 2) + 1; e.off = uint32_t((w >> 8) & 0xffff); break;
    default: e.hdr = 5; e.len = (tag >> 2) + 1; e.off = uint32_t((w >> 8) & 0xffffffffull); break;
  }
  return e;
}
__device__ __forceinline__ Elem snap_elem(const uint8_t* p) { return snap_decode(load_u64(p)); }
__device__ __forceinline__ uint64_t snap_adv(const Elem& e) { return uint64_t(e.hdr) + (e.off ? 0u : e.len); }

__device__ __forceinline__ uint32_t chunk_page(const uint32_t* chunk_base, uint32_t npages, uint32_t c) {
  uint32_t lo = 0, hi = npages;  // last page with chunk_base[p] <= c
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (chunk_base[mid] <= c) lo = mid; else hi = mid;
  }
  return lo;
}

// ---- LDS staging of a workgroup's input range -------------------------------------------------------
// Bytes of the page input from (chunk j0 start - warm-up) to (chunk j0+cnt end + 16) are copied
// into `buf` with coalesced dword loads; `lo` is the page offset of buf[0] (dword aligned in
// absolute address, so it may sit up to 3 bytes before the page input).
struct Staged {
  int64_t lo;
  uint64_t hi;
};

__device__ Staged stage_input(uint8_t* buf, const uint8_t* in, uint64_t n_in, uint32_t j0, uint32_t cnt) {
  uint64_t lo = uint64_t(j0) * SNAP_CH;
  lo = lo >= SNAP_WU ? lo - SNAP_WU : 0;
  const uint64_t hi = min(uint64_t(j0 + cnt) * SNAP_CH + 16, uint64_t(n_in) + 8);
  const uintptr_t a0 = (reinterpret_cast<uintptr_t>(in) + lo) & ~uintptr_t(3);
  const int64_t lo_al = int64_t(a0) - int64_t(reinterpret_cast<uintptr_t>(in));
  const uint32_t nd = uint32_t((int64_t(hi) - lo_al + 3) / 4) + 2;
  uint32_t* b32 = reinterpret_cast<uint32_t*>(buf);
  const uint32_t* g32 = reinterpret_cast<const uint32_t*>(a0);
  for (uint32_t i = threadIdx.x; i < nd; i += blockDim.x) b32[i] = g32[i];
  __syncthreads();
  return Staged{lo_al, hi};
}

// 8 bytes at page offset pos from the staged copy.
__device__ __forceinline__ uint64_t staged_u64(const uint8_t* buf, const Staged& s, uint64_t pos) {
  const uint32_t r = uint32_t(int64_t(pos) - s.lo);
  const uint32_t* b32 = reinterpret_cast<const uint32_t*>(buf);
  const uint32_t di = r >> 2, sh = r & 3;
  const uint32_t w0 = b32[di], w1 = b32[di + 1], w2 = b32[di + 2];
  return uint64_t(__builtin_amdgcn_alignbyte(w1, w0, sh)) | (uint64_t(__builtin_amdgcn_alignbyte(w2, w1, sh)) << 32);
}

// Workgroup g covers chunks [wg_chunk0[g], ...) of one page.
struct WgInfo {
  uint32_t p, j0, cnt;   // page, first chunk (page-relative), chunks in this workgroup
};
__device__ __forceinline__ WgInfo wg_info(const SnappyArgs& a) {
  const uint32_t c = a.wg_chunk0[blockIdx.x];
  const uint32_t p = chunk_page(a.chunk_base, a.npages, c);
  const uint32_t j0 = c - a.chunk_base[p];
  const uint32_t nc = a.chunk_base[p + 1] - a.chunk_base[p];
  return WgInfo{p, j0, min(WG_CHUNKS, nc - j0)};
}

// A: speculative parse.
__global__ void __launch_bounds__(WG_CHUNKS) k_snap_spec(SnappyArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[STAGE_BYTES + 32];
  const WgInfo g = wg_info(a);
  const SnapPage& pg = a.pages[g.p];
  const Staged s = stage_input(buf, reinterpret_cast<const uint8_t*>(pg.in), pg.n_in, g.j0, g.cnt);
  if (threadIdx.x >= g.cnt) return;
  const uint32_t j = g.j0 + threadIdx.x;
  const uint32_t c = a.chunk_base[g.p] + j;
  const uint64_t cs = uint64_t(j) * SNAP_CH;
  const uint64_t ce = min(cs + SNAP_CH, uint64_t(pg.n_in));
  uint32_t vis[SNAP_CH / 32];
#pragma unroll
  for (int k = 0; k < int(SNAP_CH / 32); ++k) vis[k] = 0;
  uint64_t pos = cs >= SNAP_WU ? cs - SNAP_WU : 0;
  while (pos < ce) {
    if (pos >= cs) {
      const uint32_t r = uint32_t(pos - cs);
#pragma unroll
      for (int k = 0; k < int(SNAP_CH / 32); ++k)
        if (int(r >> 5) == k) vis[k] |= 1u << (r & 31);
    }
    pos += snap_adv(snap_decode(staged_u64(buf, s, pos)));
  }
  a.spec_exit[c] = pos > 0xffffffffull ? 0xffffffffu : uint32_t(pos);
#pragma unroll
  for (int k = 0; k < int(SNAP_CH / 32); ++k) a.vis[uint64_t(c) * (SNAP_CH / 32) + k] = vis[k];
}

// B: true chunk entries, 64 chunks per ballot.
__global__ void __launch_bounds__(64) k_snap_resolve(SnappyArgs a) {
  const uint32_t p = blockIdx.x;
  if (p >= a.npages) return;
  const SnapPage& pg = a.pages[p];
  const uint8_t* in = reinterpret_cast<const uint8_t*>(pg.in);
  const uint32_t c0 = a.chunk_base[p], nc = a.chunk_base[p + 1] - c0;
  const int lane = threadIdx.x;
  uint64_t e = 0;  // true entry of chunk `base`
  uint32_t base = 0;
  while (base < nc) {
    const uint32_t j = base + lane;
    const bool valid = j < nc;
    uint32_t x = 0, word = 0;
    const uint64_t cs = uint64_t(j) * SNAP_CH;
    const uint64_t ce = min(cs + SNAP_CH, uint64_t(pg.n_in));
    if (valid) x = a.spec_exit[c0 + j];
    uint64_t cand = __shfl_up(uint64_t(x), 1, 64);
    if (lane == 0) cand = e;
    const bool skip = cand >= ce;
    if (valid && !skip) word = a.vis[uint64_t(c0 + j) * (SNAP_CH / 32) + uint32_t((cand - cs) >> 5)];
    const bool ok = valid && !skip && ((word >> ((cand - cs) & 31)) & 1u);
    const unsigned long long brk = __ballot(valid && !ok);
    const uint32_t f = brk ? uint32_t(__builtin_ctzll(brk)) : 64u;  // first chunk needing care
    if (valid && uint32_t(lane) <= f) a.entry[c0 + j] = uint32_t(min(cand, uint64_t(0xffffffffu)));
    const uint32_t cnt = min(64u, nc - base);
    if (f >= cnt) {
      e = uint32_t(__builtin_amdgcn_readlane(int(x), int(cnt - 1)));
      base += cnt;
      continue;
    }
    // chunk base+f: its true entry is cand_f (all earlier lanes were consistent). Walk it from a
    // 512-byte register window (lane l holds 8 bytes) instead of dependent global loads.
    uint64_t ef = __shfl(cand, int(f), 64);
    const uint64_t fcs = uint64_t(base + f) * SNAP_CH;
    const uint64_t fce = min(fcs + SNAP_CH, uint64_t(pg.n_in));
    if (ef < fce) {
      const uintptr_t wa = (reinterpret_cast<uintptr_t>(in) + fcs) & ~uintptr_t(7);
      const int64_t wb = int64_t(wa) - int64_t(reinterpret_cast<uintptr_t>(in));
      const uint2 w = reinterpret_cast<const uint2*>(wa)[lane];
      while (ef < fce) {
        const uint32_t r = uint32_t(int64_t(ef) - wb);
        uint64_t hdr;
        if (r + 12 <= 512) {
          const uint32_t di = r >> 2, sh = r & 3;
          auto dw = [&](uint32_t d) -> uint32_t {
            return uint32_t(__builtin_amdgcn_readlane(int((d & 1) ? w.y : w.x), int(d >> 1)));
          };
          const uint32_t d0 = dw(di), d1 = dw(di + 1), d2 = dw(di + 2);
          hdr = uint64_t(__builtin_amdgcn_alignbyte(d1, d0, sh)) | (uint64_t(__builtin_amdgcn_alignbyte(d2, d1, sh)) << 32);
        } else {
          hdr = load_u64(in + ef);
        }
        ef += snap_adv(snap_decode(hdr));
      }
    }
    e = ef;
    base += f + 1;
  }
}

// C: output bytes / copy elements produced by the true elements of each chunk.
__global__ void __launch_bounds__(WG_CHUNKS) k_snap_count(SnappyArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[STAGE_BYTES + 32];
  const WgInfo g = wg_info(a);
  const SnapPage& pg = a.pages[g.p];
  const Staged s = stage_input(buf, reinterpret_cast<const uint8_t*>(pg.in), pg.n_in, g.j0, g.cnt);
  if (threadIdx.x >= g.cnt) return;
  const uint32_t j = g.j0 + threadIdx.x;
  const uint32_t c = a.chunk_base[g.p] + j;
  const uint64_t cs = uint64_t(j) * SNAP_CH;
  const uint64_t ce = min(cs + SNAP_CH, uint64_t(pg.n_in));
  uint64_t pos = a.entry[c], out = 0;
  uint32_t copies = 0;
  while (pos < ce) {
    const Elem el = snap_decode(staged_u64(buf, s, pos));
    out += el.len;
    copies += el.off != 0;
    pos += snap_adv(el);
  }
  a.chunk_out[c] = out > 0xffffffffull ? 0xffffffffu : uint32_t(out);
  a.chunk_copies[c] = copies;
}

// D: per-page exclusive scan of chunk outputs (one wave per page).
__global__ void __launch_bounds__(64) k_snap_scan(SnappyArgs a) {
  const uint32_t p = blockIdx.x;
  if (p >= a.npages) return;
  const uint32_t c0 = a.chunk_base[p], nc = a.chunk_base[p + 1] - c0;
  const int lane = threadIdx.x;
  uint64_t carry = 0;
  for (uint32_t base = 0; base < nc; base += 64) {
    const uint32_t j = base + lane;
    const uint64_t v = j < nc ? a.chunk_out[c0 + j] : 0;
    uint64_t incl = v;
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    if (j < nc) a.chunk_out_start[c0 + j] = uint32_t(carry + incl - v);
    carry += __shfl(incl, 63, 64);
  }
  if (lane == 0 && carry != a.pages[p].n_out) atomicOr(&a.pages_bad[p], 1u);  // size mismatch
}

// E: literal bytes to the output, copies to records.
__global__ void __launch_bounds__(WG_CHUNKS) k_snap_emit(SnappyArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[STAGE_BYTES + 32];
  const WgInfo g = wg_info(a);
  const SnapPage& pg = a.pages[g.p];
  const Staged s = stage_input(buf, reinterpret_cast<const uint8_t*>(pg.in), pg.n_in, g.j0, g.cnt);
  if (threadIdx.x >= g.cnt) return;
  const uint32_t j = g.j0 + threadIdx.x;
  const uint32_t c = a.chunk_base[g.p] + j;
  const uint64_t cs = uint64_t(j) * SNAP_CH;
  const uint64_t ce = min(cs + SNAP_CH, uint64_t(pg.n_in));
  uint8_t* out = reinterpret_cast<uint8_t*>(pg.out);
  uint64_t pos = a.entry[c], o = a.chunk_out_start[c];
  uint64_t rec = a.chunk_rec_start[c];
  bool bad = false;
  while (pos < ce) {
    const Elem el = snap_decode(staged_u64(buf, s, pos));
    if (o + el.len > pg.n_out || (el.len && (o >> 16) != ((o + el.len - 1) >> 16))) { bad = true; break; }
    if (el.off == 0) {
      if (pos + el.hdr + el.len > pg.n_in) { bad = true; break; }
      const uint64_t lp = pos + el.hdr;
      if (lp + el.len + 4 <= s.hi) {
        for (uint32_t i = 0; i < el.len; ++i) out[o + i] = buf[uint32_t(int64_t(lp + i) - s.lo)];
      } else {  // a long literal running past the staged range
        const uint8_t* sp = reinterpret_cast<const uint8_t*>(pg.in) + lp;
        for (uint32_t i = 0; i < el.len; ++i) out[o + i] = sp[i];
      }
    } else {
      if (el.off > (o & (SNAP_BLOCK - 1)) || el.len > 0xffff) { bad = true; break; }  // copy crosses its fragment
      a.recs[rec++] = uint64_t(o) | (uint64_t(el.len) << 32) | (uint64_t(el.off) << 48);
    }
    o += el.len;
    pos += snap_adv(el);
  }
  if (bad) atomicOr(&a.pages_bad[g.p], 8u);
}

// F: one 1024-thread workgroup per 64 KiB output block.
constexpr int EXEC_T = 1024;

__global__ void __launch_bounds__(EXEC_T) k_snap_exec(SnappyArgs a) {
  __shared__ uint16_t src[SNAP_BLOCK];
  __shared__ uint32_t s_j0, s_j1, s_changed;
  const uint32_t b = blockIdx.x;
  const uint32_t p = a.block_page[b];
  if (a.pages_bad[p]) return;
  const SnapPage& pg = a.pages[p];
  uint8_t* out = reinterpret_cast<uint8_t*>(pg.out);
  const uint32_t k = b - pg.block_base;
  const uint64_t bs = uint64_t(k) * SNAP_BLOCK;
  const uint64_t be = min(bs + SNAP_BLOCK, uint64_t(pg.n_out));
  const uint32_t nbytes = uint32_t(be - bs);
  const uint32_t c0 = a.chunk_base[p], c1 = a.chunk_base[p + 1];
  const int t = threadIdx.x;
  if (t == 0) {
    uint32_t lo = c0, hi = c1;  // first chunk whose output reaches past bs
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (uint64_t(a.chunk_out_start[mid]) + a.chunk_out[mid] <= bs) lo = mid + 1; else hi = mid;
    }
    s_j0 = lo;
    hi = c1;  // first chunk starting at or after be
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (a.chunk_out_start[mid] < be) lo = mid + 1; else hi = mid;
    }
    s_j1 = lo;
  }
  for (uint32_t i = t; i < nbytes; i += EXEC_T) src[i] = uint16_t(i);
  __syncthreads();
  const uint64_t r0 = a.chunk_rec_start[s_j0];
  const uint64_t r1 = a.chunk_rec_start[s_j1];
  for (uint64_t r = r0 + t; r < r1; r += EXEC_T) {
    const uint64_t w = a.recs[r];
    const uint64_t o = uint32_t(w);
    if (o < bs || o >= be) continue;
    const uint32_t len = uint32_t((w >> 32) & 0xffff), off = uint32_t(w >> 48);
    const uint32_t rel = uint32_t(o - bs);
    for (uint32_t i = 0; i < len; ++i) src[rel + i] = uint16_t(rel + i - off);
  }
  __syncthreads();
  for (int round = 0; round < 17; ++round) {
    if (t == 0) s_changed = 0;
    __syncthreads();
    uint32_t ch = 0;
    for (uint32_t i = t; i < nbytes; i += EXEC_T) {
      const uint32_t x = src[i];
      const uint32_t y = src[x];
      if (y != x) { src[i] = uint16_t(y); ch = 1; }
    }
    if (__any(ch) && (t & 63) == 0) s_changed = 1;
    __syncthreads();
    if (!s_changed) break;
  }
  __threadfence_block();
  for (uint32_t i = t; i < nbytes; i += EXEC_T) {
    const uint32_t r = src[i];
    if (r != i) out[bs + i] = out[bs + r];
  }
}

// Serial fallback for pages whose structure the parallel path could not use.
__global__ void k_snap_serial(SnappyArgs a) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= a.npages || !a.pages_bad[p]) return;
  const SnapPage& pg = a.pages[p];
  const uint8_t* in = reinterpret_cast<const uint8_t*>(pg.in);
  uint8_t* out = reinterpret_cast<uint8_t*>(pg.out);
  uint64_t ip = 0, op = 0;
  while (ip < pg.n_in) {
    const Elem el = snap_elem(in + ip);
    if (op + el.len > pg.n_out) { atomicCAS(a.error, 0u, 1u); return; }
    if (el.off == 0) {
      if (ip + el.hdr + el.len > pg.n_in) { atomicCAS(a.error, 0u, 1u); return; }
      for (uint32_t i = 0; i < el.len; ++i) out[op + i] = in[ip + el.hdr + i];
    } else {
      if (el.off > op) { atomicCAS(a.error, 0u, 1u); return; }
      for (uint32_t i = 0; i < el.len; ++i) out[op + i] = out[op - el.off + i];
    }
    op += el.len;
    ip += snap_adv(el);
  }
  if (op != pg.n_out) atomicCAS(a.error, 0u, 1u);
}

// Uncompressed pages and the raw level prefix of DATA_PAGE_V2 pages: one workgroup per job.
__global__ void __launch_bounds__(256) k_page_copy(const CopyJob* jobs, uint32_t njobs) {
  const uint32_t j = blockIdx.x;
  if (j >= njobs) return;
  const uint8_t* s = reinterpret_cast<const uint8_t*>(jobs[j].src);
  uint8_t* d = reinterpret_cast<uint8_t*>(jobs[j].dst);
  const uint64_t n = jobs[j].n;
  for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) d[i] = s[i];
}

}  // namespace dev

uint32_t snappy_wg_chunks() { return dev::WG_CHUNKS; }

void launch_snappy(const SnappyArgs& a, hipStream_t st, void* scan_scratch) {
  if (!a.npages) return;
  hipLaunchKernelGGL(dev::k_snap_spec, dim3(a.nwg), dim3(dev::WG_CHUNKS), 0, st, a);
  hipLaunchKernelGGL(dev::k_snap_resolve, dim3(a.npages), dim3(64), 0, st, a);
  hipLaunchKernelGGL(dev::k_snap_count, dim3(a.nwg), dim3(dev::WG_CHUNKS), 0, st, a);
  hipLaunchKernelGGL(dev::k_snap_scan, dim3(a.npages), dim3(64), 0, st, a);
  launch_scan_u32(a.chunk_copies, a.chunk_rec_start, a.nchunks, scan_scratch, st);
  hipLaunchKernelGGL(dev::k_snap_emit, dim3(a.nwg), dim3(dev::WG_CHUNKS), 0, st, a);
  hipLaunchKernelGGL(dev::k_snap_exec, dim3(a.nblocks), dim3(dev::EXEC_T), 0, st, a);
  hipLaunchKernelGGL(dev::k_snap_serial, dim3((a.npages + 63) / 64), dim3(64), 0, st, a);
}

void launch_page_copy(const CopyJob* jobs, uint32_t njobs, hipStream_t st) {
  if (njobs) hipLaunchKernelGGL(dev::k_page_copy, dim3(njobs), dim3(256), 0, st, jobs, njobs);
}

}  // namespace dr
