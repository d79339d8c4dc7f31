// K2a: parallel SNAPPY page decompression for checkpoint column chunks.
//
// A raw snappy stream is a varint length followed by literal/copy elements. The element chain is
// serial and a 1 MiB page of paths holds ~144K elements, so a per-page decoder is latency bound
// (measured 1.28 s for config 3 with one lane per page). This decoder is fully parallel:
//
//  A k_snap_spec    one lane per SNAP_CH = 128-byte chunk of compressed input parses elements
//                   *speculatively* (starting SNAP_WU = 256 bytes early as a warm-up) and records the
//                   positions it visited in the chunk (a bitmap in registers) and where it left it.
//  B k_snap_assume / k_snap_entries: every chunk's true entry, in parallel: a chunk whose true
//                   entry (the previous chunk's exit) is on its speculative chain is correct
//                   (chains that meet coincide from then on); an isolated mis-speculated chunk is
//                   walked from its true entry. Runs of mis-speculation and chunks spanned by long
//                   literals send the page to k_snap_resolve from its first such chunk (one wave
//                   per page, 64 chunks per ballot, spanned chunks skipped in one step).
//  C k_snap_count   per chunk: output bytes and elements of its true elements (counted by the
//                   speculative walk from the chunk's first visited position; re-walked only when
//                   the true entry differs, and then the chunk's visited bitmap is rewritten with
//                   the true chain: every chunk's bits at or after its entry are its element starts).
//  D k_snap_scan    per page: exclusive scan of chunk outputs, and the chunk holding each 64 KiB
//                   output block's first element. The compressor compresses 64 KiB fragments
//                   independently, so no element straddles a fragment and no copy reaches before it.
//  E k_snap_exec    one 1024-thread workgroup per 64 KiB output block decodes its chunks' element
//                   headers from the start bitmaps (a workgroup scan of the lengths gives each its
//                   output offset), resolves every copied byte to its literal origin by pointer
//                   jumping on a u16 map in LDS (src[p] = p - offset; literal bytes are their own
//                   roots), then rebuilds the block's bytes in the same LDS and stores them with
//                   dword stores. Violations of the fragment rules flag the page for k_snap_serial.
//
// Chunk walkers (A) stage their page bytes into LDS with coalesced loads and parse from LDS.
#include "dev_common.h"
#include "kernels.h"
#include "wave.h"

namespace dr {
namespace dev {

#ifndef DR_SNAP_CH
// r05: 128 B chunks with a 256 B warm-up, SNAPPY-minus-exec 1.356 -> 1.264 ms on config 3 (r02 tried
// 128 B chunks, but two full-size config-3 pages then failed the size check: the resolver's
// concurrent region walks of a page, fixed in r05 by walking a page's regions in order)
#define DR_SNAP_CH 128
#endif
constexpr uint32_t SNAP_CH = DR_SNAP_CH;     // compressed bytes per speculation chunk (a multiple of 128)
constexpr uint32_t SNAP_BLOCK = 65536;       // snappy compressor fragment size
#ifndef DR_SNAP_WU
#define DR_SNAP_WU 256
#endif
// speculation warm-up bytes (r01 at 256 B chunks: 64/128 B sent too many pages to k_snap_resolve, 3x/20x
// slower; 160-256 B within 1 %, 192 B best. r05 at 128 B chunks, SNAPPY-minus-exec at scale 0.25:
// 160 B 0.582 ms (the resolver doubles), 192 B 0.493, 224 B 0.460-0.469, 256 B 0.483, 288 B 0.473;
// at full config 3: 224 B 1.289 ms, 256 B 1.264, r04's 256 B chunks + 192 B 1.356)
constexpr uint32_t SNAP_WU = DR_SNAP_WU;
#ifndef DR_SNAP_WG_CHUNKS
#define DR_SNAP_WG_CHUNKS 256
#endif
constexpr uint32_t WG_CHUNKS = DR_SNAP_WG_CHUNKS;  // chunks (threads) per chunk-walker workgroup
constexpr uint32_t STAGE_BYTES = (WG_CHUNKS * SNAP_CH + SNAP_WU + 96) * 65 / 64 + 16;  // + skew

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

// Input bytes an element occupies and the output bytes it produces, without branches (the
// speculative walkers only need these; lanes then never split on the element type).
// Selects written as mask blends: as conditional expressions the compiler made the walkers' steps
// divergent branches again (six per element in k_snap_spec's loop).
__device__ __forceinline__ uint32_t sel32(bool c, uint32_t x, uint32_t y) { return y ^ ((x ^ y) & (0u - uint32_t(c))); }
__device__ __forceinline__ void snap_step(uint64_t w, uint32_t* adv, uint32_t* out) {
  const uint32_t tag = uint32_t(w & 0xff), t = tag & 3, l6 = tag >> 2;
  const bool lit = t == 0;
  const uint32_t nb = l6 > 59u ? l6 - 59u : 0u;                      // long literal: length bytes
  const uint32_t lmask = sel32(nb >= 4u, 0xffffffffu, (1u << (8u * (nb & 3u))) - 1u);
  const uint32_t lit_len = sel32(nb != 0u, uint32_t(w >> 8) & lmask, l6);  // minus one
  const uint32_t hdr = ((0x5320u >> (4 * t)) & 0xfu) + sel32(lit, 1u + nb, 0u);
  const uint32_t len = sel32(lit, lit_len + 1u, sel32(t == 1, (l6 & 7) + 4, l6 + 1));
  *out = len;
  *adv = hdr + sel32(lit, len, 0u);
}
// The same with conditional expressions (compiled to branches): the window walkers of k_snap_assume
// and k_snap_count measured faster with it (0.033 / 0.049 ms against 0.038 / 0.062 at scale 0.25).
__device__ __forceinline__ void snap_step_br(uint64_t w, uint32_t* adv, uint32_t* out) {
  const uint32_t tag = uint32_t(w & 0xff), t = tag & 3, l6 = tag >> 2;
  const uint32_t nb = l6 >= 60 ? l6 - 59 : 0;
  const uint32_t lmask = nb >= 4 ? 0xffffffffu : ((1u << (8 * nb)) - 1u);
  const uint32_t lit_len = nb ? uint32_t(w >> 8) & lmask : l6;
  const uint32_t hdr = t == 0 ? 1 + nb : ((0x5320u >> (4 * t)) & 0xfu);
  const uint32_t len = t == 0 ? lit_len + 1 : t == 1 ? ((l6 & 7) + 4) : l6 + 1;
  *out = len;
  *adv = hdr + (t == 0 ? len : 0u);
}

// Page of chunk c: the plan's per-chunk table (one load), built once when the segment is staged.
__device__ __forceinline__ uint32_t chunk_page(const SnappyArgs& a, uint32_t c) { return a.chunk_page[c]; }

// ---- LDS staging of a workgroup's input range -------------------------------------------------------
// Bytes of the page input from (chunk j0 start - warm-up) to (chunk j0+cnt end + 16) are copied
// into `buf` with coalesced dword loads; `lo` is the page offset of buf[0] (dword aligned in
// absolute address, so it may sit up to 3 bytes before the page input).
// The staged copy is skewed by one dword per 256 bytes: lane l walks chunk l, SNAP_CH bytes after
// lane l-1, so unskewed the lanes at the same relative offset would hit one LDS bank or two (with
// 128-byte chunks the skew still gives the 64 lanes 64 distinct banks).
struct Staged {
  int64_t lo;
  uint64_t hi;
};
__device__ __forceinline__ uint32_t skew(uint32_t dw) { return dw + (dw >> 6); }
#ifndef DR_STAGE_BATCH
#define DR_STAGE_BATCH 8
#endif
constexpr uint32_t STAGE_BATCH = DR_STAGE_BATCH;

__device__ Staged stage_input(uint8_t* buf, const uint8_t* in, uint64_t n_in, uint32_t j0, uint32_t cnt) {
  uint64_t lo = uint64_t(j0) * SNAP_CH;
  lo = lo >= SNAP_WU ? lo - SNAP_WU : 0;
  const uint64_t hi = min(uint64_t(j0 + cnt) * SNAP_CH + 16, uint64_t(n_in) + 8);
  const uintptr_t a0 = (reinterpret_cast<uintptr_t>(in) + lo) & ~uintptr_t(15);
  const int64_t lo_al = int64_t(a0) - int64_t(reinterpret_cast<uintptr_t>(in));
  const uint32_t nv = uint32_t((int64_t(hi) - lo_al + 15) / 16) + 1;  // 16-byte vectors (+ 8-byte reads past hi)
  uint32_t* b32 = reinterpret_cast<uint32_t*>(buf);
  const uint4* g4 = reinterpret_cast<const uint4*>(a0);
  // 16-byte global loads, STAGE_BATCH in flight per lane before any is written to LDS (indices past
  // the range re-read its last vector instead of branching, so the loads issue back to back; a
  // guarded loop waited for each load before issuing the next: 16 round trips per lane in k_snap_spec);
  // a vector's 4 dwords never straddle a skew step
  for (uint32_t i0 = threadIdx.x; i0 < nv; i0 += STAGE_BATCH * blockDim.x) {
    uint4 v[STAGE_BATCH];
#pragma unroll
    for (uint32_t k = 0; k < STAGE_BATCH; ++k) v[k] = gload16(g4 + min(i0 + k * blockDim.x, nv - 1));
#pragma unroll
    for (uint32_t k = 0; k < STAGE_BATCH; ++k) {
      const uint32_t i = i0 + k * blockDim.x;
      if (i < nv) {
        uint32_t* d = b32 + skew(4 * i);
        d[0] = v[k].x; d[1] = v[k].y; d[2] = v[k].z; d[3] = v[k].w;
      }
    }
  }
  __syncthreads();
  return Staged{lo_al, hi};
}

// The element header at page offset pos from the staged copy: bytes pos .. pos+4 (a tag and at most
// four length / offset bytes) in the low 40 bits, from two dword reads (higher bits unspecified).
__device__ __forceinline__ uint64_t staged_u64(const uint8_t* buf, const Staged& s, uint64_t pos) {
  const uint32_t r = uint32_t(int64_t(pos) - s.lo);
  const uint32_t* b32 = reinterpret_cast<const uint32_t*>(buf);
  const uint32_t di = r >> 2, sh = r & 3;
  const uint32_t w0 = b32[skew(di)], w1 = b32[skew(di + 1)];
  return ((uint64_t(w1) << 32) | w0) >> (8 * sh);
}

// Workgroup g covers chunks [wg_chunk0[g], ...) of one page.
struct WgInfo {
  uint32_t p, j0, cnt;   // page, first chunk (page-relative), chunks in this workgroup
};
__device__ __forceinline__ WgInfo wg_info(const SnappyArgs& a) {
  const uint32_t c = a.wg_chunk0[blockIdx.x];
  const uint32_t p = chunk_page(a, c);
  const uint32_t j0 = c - a.chunk_base[p];
  const uint32_t nc = a.chunk_base[p + 1] - a.chunk_base[p];
  return WgInfo{p, j0, min(WG_CHUNKS, nc - j0)};
}

// A: speculative parse, one lane per chunk. (Two chunks interleaved per lane, to overlap two chains
// of dependent LDS reads, measured 6x slower at half the lanes per workgroup: r02.)
struct SpecChain {
  // visited bitmap in registers (statically indexed: each step ORs its bit into the selected word
  // with selects, so the walk issues no LDS read-modify-write of its own)
  uint32_t lv[SNAP_CH / 32];
  uint64_t pos, cs, ce, first, out;
  uint32_t elems;
};
// A chunk past the workgroup's (not live) gets an empty walk parked at `park`, a staged position,
// so the unconditional header read of the step loop stays inside the stage.
__device__ __forceinline__ void spec_init(SpecChain& w, uint32_t j, uint64_t n_in, bool live, uint64_t park) {
#pragma unroll
  for (int k = 0; k < int(SNAP_CH / 32); ++k) w.lv[k] = 0;
  w.cs = uint64_t(j) * SNAP_CH;
  w.ce = live ? min(w.cs + SNAP_CH, n_in) : park;
  w.pos = !live ? park : w.cs >= SNAP_WU ? w.cs - SNAP_WU : 0;
  w.first = ~0ull;
  w.out = 0;
  w.elems = 0;
}
// One element of the walk from its header word `hw` (only when w.pos < w.ce).
__device__ __forceinline__ void spec_step(SpecChain& w, uint64_t hw) {
  uint32_t adv, len;
  snap_step(hw, &adv, &len);
  if (w.pos >= w.cs) {
    const uint32_t r = uint32_t(w.pos - w.cs);
    const uint32_t wi = r >> 5, bit = 1u << (r & 31);
#pragma unroll
    for (int k = 0; k < int(SNAP_CH / 32); ++k) w.lv[k] |= wi == uint32_t(k) ? bit : 0u;
    if (w.first == ~0ull) w.first = w.pos;
    w.out += len;
    ++w.elems;
  }
  w.pos += adv;
}
__device__ __forceinline__ void spec_store(const SnappyArgs& a, const SpecChain& w, uint32_t c) {
  a.spec_exit[c] = w.pos > 0xffffffffull ? 0xffffffffu : uint32_t(w.pos);
#pragma unroll
  for (int k = 0; k < int(SNAP_CH / 32); k += 4)
    *reinterpret_cast<uint4*>(&a.vis[uint64_t(c) * (SNAP_CH / 32) + k]) = make_uint4(w.lv[k], w.lv[k + 1], w.lv[k + 2], w.lv[k + 3]);
  // the chunk's output bytes / elements if its true entry is its first visited position (nearly
  // always): k_snap_count then only re-walks the exceptions
  a.spec_first[c] = w.first > 0xffffffffull ? 0xffffffffu : uint32_t(w.first);
  a.chunk_out[c] = w.out > 0xffffffffull ? 0xffffffffu : uint32_t(w.out);
  a.chunk_elems[c] = w.elems;
}

__global__ void __launch_bounds__(WG_CHUNKS) k_snap_spec(SnappyArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t buf[STAGE_BYTES + 32];
  const WgInfo g = wg_info(a);
  const SnapPage pg = a.pages[g.p];
  const Staged s = stage_input(buf, reinterpret_cast<const uint8_t*>(pg.in), pg.n_in, g.j0, g.cnt);
  const bool live = threadIdx.x < g.cnt;
  SpecChain w;
  spec_init(w, g.j0 + threadIdx.x, pg.n_in, live, uint64_t(g.j0) * SNAP_CH);
  // the warm-up before the chunk (two thirds of the steps) advances the position only
  while (w.pos < w.cs && w.pos < w.ce) {
    uint32_t adv, len;
    snap_step(staged_u64(buf, s, w.pos), &adv, &len);
    w.pos += adv;
  }
  while (w.pos < w.ce) spec_step(w, staged_u64(buf, s, w.pos));
  if (live) spec_store(a, w, a.chunk_base[g.p] + g.j0 + threadIdx.x);
}

// A lane's serial element walk from e (a true element start) to the end ce of its chunk through
// its own 64-byte LDS window (`win`: the lane's 17-dword slot, padded against bank conflicts),
// refilled with four 16-byte loads when the next header leaves it: one round trip per dozen or so
// elements instead of one per element. Returns the exit; out / elems: the walked elements' output
// bytes and count; `lv` (when given): the bitmap of the visited positions relative to `cs`.
constexpr uint32_t WIN_DW = 17;
__device__ uint64_t walk_window(const uint8_t* in, uint64_t e, uint64_t ce, uint32_t* win, uint64_t* out,
                                uint32_t* elems, uint64_t cs = 0, uint32_t* lv = nullptr) {
  const uintptr_t ib = reinterpret_cast<uintptr_t>(in);
  uintptr_t wa = 0;
  bool have = false;
  uint64_t o = 0;
  uint32_t k = 0;
  if (lv) {
#pragma unroll
    for (int q = 0; q < int(SNAP_CH / 32); ++q) lv[q] = 0;
  }
  while (e < ce) {
    if (lv) {  // statically indexed: each step ORs its bit into the selected word
      const uint32_t r = uint32_t(e - cs), wi = r >> 5, bit = 1u << (r & 31);
#pragma unroll
      for (int q = 0; q < int(SNAP_CH / 32); ++q) lv[q] |= wi == uint32_t(q) ? bit : 0u;
    }
    const uintptr_t ea = ib + e;
    if (!have || ea < wa || ea + 8 > wa + 64) {  // reads reach at most 63 bytes past the page input (padded)
      wa = ea & ~uintptr_t(15);
      const uint4* g = reinterpret_cast<const uint4*>(wa);
      const uint4 v0 = gload16(g), v1 = gload16(g + 1), v2 = gload16(g + 2), v3 = gload16(g + 3);
      win[0] = v0.x; win[1] = v0.y; win[2] = v0.z; win[3] = v0.w;
      win[4] = v1.x; win[5] = v1.y; win[6] = v1.z; win[7] = v1.w;
      win[8] = v2.x; win[9] = v2.y; win[10] = v2.z; win[11] = v2.w;
      win[12] = v3.x; win[13] = v3.y; win[14] = v3.z; win[15] = v3.w;
      have = true;
    }
    const uint32_t r = uint32_t(ea - wa), di = r >> 2, sh = r & 3;
    const uint64_t hdr = ((uint64_t(win[di + 1]) << 32) | win[di]) >> (8 * sh);  // 5 header bytes at least
    uint32_t adv, len;
    snap_step_br(hdr, &adv, &len);
    o += len;
    ++k;
    e += adv;
  }
  *out = o;
  *elems = k;
  return e;
}

// B1: every chunk's exit x[c] assuming its entry is the previous chunk's speculative exit
// a = spec_exit[c-1] (chunk 0: entry 0, exact): a at or past the chunk end -> a; a on the chunk's
// speculative chain (visited bitmap) -> spec_exit[c] (chains that meet coincide); otherwise a
// serial walk of the chunk from a.
__global__ void __launch_bounds__(256) k_snap_assume(SnappyArgs a) {
  __shared__ uint32_t wins[256 * WIN_DW];
  const uint32_t c = blockIdx.x * 256 + threadIdx.x;
  if (c >= a.nchunks) return;
  const uint32_t p = chunk_page(a, c);
  const SnapPage& pg = a.pages[p];
  const uint32_t j = c - a.chunk_base[p];
  const uint64_t cs = uint64_t(j) * SNAP_CH;
  const uint64_t ce = min(cs + SNAP_CH, uint64_t(pg.n_in));
  const uint64_t e = j == 0 ? 0 : a.spec_exit[c - 1];
  uint64_t x;
  if (e >= ce) x = e;
  else if (j == 0 || ((a.vis[uint64_t(c) * (SNAP_CH / 32) + uint32_t((e - cs) >> 5)] >> ((e - cs) & 31)) & 1u))
    x = a.spec_exit[c];
  else {
    uint64_t o;
    uint32_t k;
    x = walk_window(reinterpret_cast<const uint8_t*>(pg.in), e, ce, wins + threadIdx.x * WIN_DW, &o, &k);
  }
  a.assumed_exit[c] = uint32_t(min(x, uint64_t(0xffffffffu)));
}

// B2: true entries E[c] = T[c-1] (the true exit of chunk c-1). Chunk k "breaks" when its exit
// under the assumed entry differs from its speculative exit. A genuine break (the assumed entry was
// true) is always followed by an artefact break of the next chunk (its assumed entry, the broken
// chunk's speculative exit, is wrong) unless that chunk happens to agree; so along a run of
// consecutive breaks, breaks at even distance from the run's start are genuine, provided each chunk
// after a genuine break re-synchronises with its speculative chain (checked here). Then:
//   c-2 not genuine -> E[c] = assumed_exit[c-1];
//   c-2 genuine     -> chunk c-1 starts at assumed_exit[c-2] and must re-synchronise:
//                      E[c] = spec_exit[c-1].
// A failed re-synchronisation (or a chunk spanned right after a break) records the page's first
// such chunk; the serial resolver recomputes the page's entries from there. Such a chunk's entry is
// set to ~0 here: k_snap_resolve stops where its walk agrees with the entries written here, so an
// entry left over from an earlier replay of the same pages must never be mistaken for one (that
// sent a page to the serial decoder on every replay after the first: 138 ms at config 4 scale 0.1).
__device__ __forceinline__ bool broke(const SnappyArgs& a, uint32_t c) { return a.assumed_exit[c] != a.spec_exit[c]; }

constexpr uint32_t MAX_RUN = 32;
__global__ void __launch_bounds__(256) k_snap_entries(SnappyArgs a) {
  const uint32_t c = blockIdx.x * 256 + threadIdx.x;
  if (c >= a.nchunks) return;
  const uint32_t p = chunk_page(a, c);
  const uint32_t j = c - a.chunk_base[p];
  if (j == 0) { a.entry[c] = 0; return; }
  const uint32_t b = c - 1;  // page-relative j-1
  bool genuine = false;
  if (j >= 2 && broke(a, b - 1)) {
    // length of the run of breaks ending at c-2 (page-relative chunk 0 never breaks)
    uint32_t r = 0;
    while (r < MAX_RUN && j - 2 > r && broke(a, b - 2 - r)) ++r;
    if (r == MAX_RUN) {
      a.chunk_flag[a.chunk_base[p] + (j - 2 > MAX_RUN ? j - 2 - MAX_RUN : 0u)] = 1;
      a.entry[c] = 0xffffffffu;  // unknown: k_snap_resolve rewrites it (never a stale value of an earlier replay)
      return;
    }
    genuine = (r & 1u) == 0;
  }
  if (!genuine) {
    a.entry[c] = a.assumed_exit[b];
    return;
  }
  const SnapPage& pg = a.pages[p];
  const uint64_t cs = uint64_t(j - 1) * SNAP_CH;
  const uint64_t ce = min(cs + SNAP_CH, uint64_t(pg.n_in));
  const uint64_t e = a.assumed_exit[b - 1];  // chunk c-1's true entry
  const bool resync = e < ce && ((a.vis[uint64_t(b) * (SNAP_CH / 32) + uint32_t((e - cs) >> 5)] >> ((e - cs) & 31)) & 1u);
  if (!resync) {
    a.chunk_flag[c - 2] = 1;
    a.entry[c] = 0xffffffffu;
    return;
  }
  a.entry[c] = a.spec_exit[b];
}

// B3a: the regions to resolve serially: a flagged chunk with no other flag in the REGION_GAP
// chunks before it (on the same page) starts a region (chunk_flag bit 1); later flags nearby are
// covered by it. Each page holding a region is listed once (region[], region_count).
constexpr uint32_t RESOLVE_MARGIN = 8;
constexpr uint32_t REGION_GAP = 80;
__global__ void __launch_bounds__(256) k_snap_regions(SnappyArgs a) {
  const uint32_t c = blockIdx.x * 256 + threadIdx.x;
  if (c >= a.nchunks || !a.chunk_flag[c]) return;
  const uint32_t p = chunk_page(a, c);
  const uint32_t c0 = a.chunk_base[p];
  const uint32_t lo = c >= c0 + REGION_GAP ? c - REGION_GAP : c0;
  for (uint32_t k = lo; k < c; ++k)
    if (a.chunk_flag[k]) return;
  a.chunk_flag[c] = 3;  // still nonzero for the other chunks' gap checks
  if (atomicExch(&a.page_mark[p], 1u) == 0u) {
    const unsigned long long slot = atomicAdd(a.region_count, 1ull);
    a.region[slot] = p;
  }
}

// B3b: one wave per page holding regions, its regions in ascending order (r05: one wave per region
// let a later region start from an entry an earlier, still running walk of the same page had yet to
// correct -- unflagged wrong entries after chunks spanned by long literals; the page then failed the
// size check and went to the serial decoder; scripts/snappy_entries_sim.py order="interleave"). From
// RESOLVE_MARGIN chunks before the flag (entries there are exact) the true chain is followed 64
// chunks per ballot, rewriting entries, until a whole 64-chunk step beyond the flag has no break,
// agrees with the entries k_snap_entries wrote (from there on they are exact again) and has no flag
// in it or within REGION_GAP after it; a region starting inside an earlier walk's range is covered
// by it. A chunk whose entry lies past its end (a long literal spans it) jumps to the chunk holding
// that entry.
__global__ void __launch_bounds__(64) k_snap_resolve(SnappyArgs a) {
  constexpr uint32_t VW = SNAP_CH / 32;  // visited-bitmap words per chunk
  constexpr uint32_t CB_WORDS = (SNAP_CH + 16) / 4;
  __shared__ uint32_t cb32[CB_WORDS + 4];
  __shared__ uint32_t nx[2][SNAP_CH];
  const uint64_t nreg = *a.region_count;
  for (uint64_t rg = blockIdx.x; rg < nreg; rg += gridDim.x) {
    const uint32_t p = a.region[rg];
    const SnapPage& pg = a.pages[p];
    const uint8_t* in = reinterpret_cast<const uint8_t*>(pg.in);
    const uint32_t c0 = a.chunk_base[p], nc = a.chunk_base[p + 1] - c0;
    const int lane = threadIdx.x;
    const uint64_t t0 = a.rstats ? __builtin_amdgcn_s_memtime() : 0;
    uint32_t n_win = 0, n_walk = 0, n_span = 0;
    uint32_t done = 0;  // chunks [0, done) of the page: resolved by an earlier walk
    for (uint32_t q0 = 0; q0 < nc; q0 += 64) {
    unsigned long long starts = __ballot(q0 + uint32_t(lane) < nc && (a.chunk_flag[c0 + q0 + lane] & 2u));
    while (starts) {
    const uint32_t jf = q0 + uint32_t(__builtin_ctzll(starts));
    starts &= starts - 1;
    if (jf < done) continue;
    uint32_t base = jf > RESOLVE_MARGIN ? jf - RESOLVE_MARGIN : 0u;
    uint64_t e = base == 0 ? 0 : a.entry[c0 + base];  // true entry of chunk `base`
    while (base < nc) {
      ++n_win;
      const uint32_t j = base + lane;
      const bool valid = j < nc;
      uint32_t x = 0, old = 0;
      uint32_t vw[VW];
#pragma unroll
      for (uint32_t k = 0; k < VW; ++k) vw[k] = 0;
      const uint64_t cs = uint64_t(j) * SNAP_CH;
      const uint64_t ce = min(cs + SNAP_CH, uint64_t(pg.n_in));
      if (valid) {
        x = a.spec_exit[c0 + j];
        old = a.entry[c0 + j];
        // the lane's whole visited bitmap: a break further on is re-checked without another load
        const uint4* vp = reinterpret_cast<const uint4*>(&a.vis[uint64_t(c0 + j) * VW]);
#pragma unroll
        for (uint32_t k = 0; k < VW; k += 4) {
          const uint4 q = vp[k / 4];
          vw[k] = q.x; vw[k + 1] = q.y; vw[k + 2] = q.z; vw[k + 3] = q.w;
        }
      }
      auto on_chain = [&](uint64_t c) -> bool {  // c (< ce) on this lane's speculative chain
        const uint32_t r = uint32_t(c - cs), wi = r >> 5;
        uint32_t word = vw[0];
#pragma unroll
        for (uint32_t k = 1; k < VW; ++k) word = wi == k ? vw[k] : word;
        return (word >> (r & 31)) & 1u;
      };
      uint64_t cand = __shfl_up(uint64_t(x), 1, 64);
      if (lane == 0) cand = e;
      bool ok = valid && cand < ce && on_chain(cand);
      unsigned long long brk = __ballot(valid && !ok);
      uint32_t f = brk ? uint32_t(__builtin_ctzll(brk)) : 64u;  // first chunk needing care
      uint32_t cv = uint32_t(min(cand, uint64_t(0xffffffffu)));
      const bool agree = __ballot(valid && (cv != old)) == 0ull;
      if (valid && uint32_t(lane) <= f) a.entry[c0 + j] = cv;
      const uint32_t cnt = min(64u, nc - base);
      if (f >= cnt) {
        if (agree && base > jf) {
          // back in step with k_snap_entries -- unless a flagged chunk lies in this window or within
          // REGION_GAP after it: such a flag starts no region of its own (k_snap_regions), so this
          // walk must carry on through it (r02: a page whose flags 70 chunks apart were left with an
          // unknown entry went to the serial decoder)
          bool fl = false;
          for (uint32_t q = base + uint32_t(lane); q < min(nc, base + cnt + REGION_GAP); q += 64) fl |= a.chunk_flag[c0 + q] != 0;
          if (__ballot(fl) == 0ull) break;
        }
        e = uint32_t(__builtin_amdgcn_readlane(int(x), int(cnt - 1)));
        base += cnt;
        continue;
      }
      // breaks inside this window, one after another: walk the broken chunk from its true entry;
      // its exit is the next chunk's true entry, checked against that lane's bitmap in registers
      // (r03: every break reloaded the window's exits and bitmaps -- three dependent round trips per
      // chunk, 12 ms on a page whose chunks all broke)
      bool next_window = true;
      while (true) {
        const uint64_t ef0 = __shfl(cand, int(f), 64);
        const uint64_t fcs = uint64_t(base + f) * SNAP_CH;
        const uint64_t fce = min(fcs + SNAP_CH, uint64_t(pg.n_in));
        if (ef0 >= fce) {
          // chunks base+f .. (the chunk holding ef0) - 1 hold no element start: entry = ef0
          ++n_span;
          const uint32_t jt = uint32_t(min(ef0 / SNAP_CH, uint64_t(nc)));
          for (uint32_t q = base + f + 1 + lane; q < jt; q += 64) a.entry[c0 + q] = uint32_t(min(ef0, uint64_t(0xffffffffu)));
          e = ef0;
          base = jt > base + f ? jt : base + f + 1;
          next_window = false;
          break;
        }
        // chunk base+f's exit from its true entry ef0, by the whole wave: every position of the chunk
        // gets the start of the element after the one starting there (nx), then pointer doubling --
        // eight rounds, as elements are at least two bytes long and a chunk holds at most 128 --
        // leaves the exit of the chain from ef0. r03 walked the chain element by element on one
        // lane: ~500 clocks per element, 13 ms for a page of consecutive int64 dictionary values
        // whose speculation broke on a quarter of its chunks.
        ++n_walk;
        const uint32_t lim = uint32_t(fce - fcs);
        for (uint32_t q = lane; q < CB_WORDS; q += 64) {  // the chunk's bytes, +16 for its last headers
          uint32_t v = 0;
#pragma unroll
          for (uint32_t k = 0; k < 4; ++k) {
            const uint64_t pos = fcs + 4 * q + k;
            v |= pos < pg.n_in ? uint32_t(in[pos]) << (8 * k) : 0u;
          }
          cb32[q] = v;
        }
        __syncthreads();
        for (uint32_t q = lane; q < SNAP_CH; q += 64) {
          uint32_t nv = q;
          if (q < lim) {
            const uint32_t di = q >> 2, sh = q & 3;
            const uint32_t w0 = cb32[di], w1 = cb32[di + 1], w2 = cb32[di + 2];
            const uint64_t hdr = uint64_t(__builtin_amdgcn_alignbyte(w1, w0, sh)) |
                                 (uint64_t(__builtin_amdgcn_alignbyte(w2, w1, sh)) << 32);
            uint32_t adv, len;
            snap_step(hdr, &adv, &len);
            nv = q + adv;
          }
          nx[0][q] = nv;
        }
        __syncthreads();
        uint32_t cur = 0;
        for (int rd = 0; rd < 8; ++rd) {
          for (uint32_t q = lane; q < SNAP_CH; q += 64) {
            const uint32_t v = nx[cur][q];
            nx[cur ^ 1u][q] = v < lim ? nx[cur][v] : v;
          }
          __syncthreads();
          cur ^= 1u;
        }
        const uint64_t ef = fcs + nx[cur][uint32_t(min(ef0 - fcs, uint64_t(SNAP_CH - 1)))];
        if (f + 1 >= cnt) {  // the window's last chunk: its exit enters the next window
          e = ef;
          base += f + 1;
          next_window = false;
          break;
        }
        // chunk base+f+1's true entry is ef; later lanes keep their candidates
        if (uint32_t(lane) == f + 1) {
          cand = ef;
          ok = valid && cand < ce && on_chain(cand);
          cv = uint32_t(min(cand, uint64_t(0xffffffffu)));
        }
        brk = __ballot(valid && !ok && uint32_t(lane) > f);
        const uint32_t f2 = brk ? uint32_t(__builtin_ctzll(brk)) : 64u;
        if (valid && uint32_t(lane) > f && uint32_t(lane) <= f2) a.entry[c0 + j] = cv;
        f = f2;
        if (f >= cnt) break;  // the rest of the window is on its chains: the next window decides
      }
      if (next_window) {
        e = uint32_t(__builtin_amdgcn_readlane(int(x), int(cnt - 1)));
        base += cnt;
      }
    }
    done = base < nc ? min(nc, base + 64u) : nc;  // the walk stopped in window [base, base + 64)
    }
    }
    if (a.rstats && lane == 0) {
      uint64_t* r = a.rstats + rg * 4;
      r[0] = __builtin_amdgcn_s_memtime() - t0;
      r[1] = n_win;
      r[2] = n_walk;
      r[3] = n_span;
    }
  }
}

// C: output bytes / elements produced by the true elements of each chunk: the speculative counts
// unless the true entry differs from the chunk's first speculatively visited position. Such a chunk
// is walked from its true entry and its visited bitmap rewritten with the true chain, so that for
// every chunk the bits at or after its entry are exactly its element starts (k_snap_exec reads them).
__global__ void __launch_bounds__(256) k_snap_count(SnappyArgs a) {
  __shared__ uint32_t wins[256 * WIN_DW];
  const uint32_t c = blockIdx.x * 256 + threadIdx.x;
  if (c >= a.nchunks) return;
  const uint32_t pos0 = a.entry[c];
  if (pos0 == a.spec_first[c]) return;
  const uint32_t p = chunk_page(a, c);
  const SnapPage& pg = a.pages[p];
  const uint64_t cs = uint64_t(c - a.chunk_base[p]) * SNAP_CH;
  const uint64_t ce = min(cs + SNAP_CH, uint64_t(pg.n_in));
  uint64_t out = 0;
  uint32_t elems = 0;
  uint32_t lv[SNAP_CH / 32];
  walk_window(reinterpret_cast<const uint8_t*>(pg.in), pos0, ce, wins + threadIdx.x * WIN_DW, &out, &elems, cs, lv);
#pragma unroll
  for (int k = 0; k < int(SNAP_CH / 32); k += 4)
    *reinterpret_cast<uint4*>(&a.vis[uint64_t(c) * (SNAP_CH / 32) + k]) = make_uint4(lv[k], lv[k + 1], lv[k + 2], lv[k + 3]);
  a.chunk_out[c] = out > 0xffffffffull ? 0xffffffffu : uint32_t(out);
  a.chunk_elems[c] = elems;
}

// D: per-page exclusive scan of chunk outputs: one 256-thread workgroup per page, each thread
// summing a contiguous run of chunks, a block scan of the run sums, then the run's prefixes.
constexpr int SCAN_T = 256;
__global__ void __launch_bounds__(SCAN_T) k_snap_scan(SnappyArgs a) {
  __shared__ uint32_t wsum[SCAN_T / 64];
  const uint32_t p = blockIdx.x;
  if (p >= a.npages) return;
  const uint32_t c0 = a.chunk_base[p], nc = a.chunk_base[p + 1] - c0;
  const uint32_t t = threadIdx.x, wv = t >> 6;
  // the chunk holding each output block's first element (no element straddles a block, so that
  // element starts the block): block k of the page is first produced by the chunk whose output range
  // [at, at + out) holds k * SNAP_BLOCK; blocks no chunk claims keep ~0 (k_snap_exec: bad page)
  const uint32_t bb = a.pages[p].block_base, nb = (a.pages[p].n_out + SNAP_BLOCK - 1) / SNAP_BLOCK;
  for (uint32_t k = t; k < nb; k += SCAN_T) a.block_chunk[bb + k] = 0xffffffffu;
  __syncthreads();
  // tiles of SCAN_T consecutive chunks (coalesced loads and stores), a block scan per tile and the
  // running offset across tiles (page outputs fit 32 bits: chunk_out_start is u32)
  uint32_t carry = 0;
  uint64_t mine = 0;  // this thread's outputs, summed in 64 bits for the size check (a saturated
                      // chunk output must not wrap into a matching size)
  for (uint32_t base = 0; base < nc; base += SCAN_T) {
    const uint32_t j = base + t;
    const uint32_t n = j < nc ? a.chunk_out[c0 + j] : 0u;
    mine += n;
    const uint32_t incl = wv::scan_incl(n, 0u, [](uint32_t x, uint32_t y) { return x + y; });
    if ((t & 63) == 63) wsum[wv] = incl;
    __syncthreads();
    uint32_t before = 0, tile = 0;
#pragma unroll
    for (uint32_t q = 0; q < SCAN_T / 64; ++q) {
      before += q < wv ? wsum[q] : 0u;
      tile += wsum[q];
    }
    const uint32_t at = carry + before + incl - n;
    if (j < nc) {
      a.chunk_out_start[c0 + j] = at;
      if (n) {
        const uint64_t k0 = (uint64_t(at) + SNAP_BLOCK - 1) / SNAP_BLOCK, k1 = min((uint64_t(at) + n - 1) / SNAP_BLOCK + 1, uint64_t(nb));
        for (uint64_t k = k0; k < k1; ++k) a.block_chunk[bb + k] = c0 + j;
      }
    }
    carry += tile;
    __syncthreads();  // the wave sums are rewritten by the next tile
  }
  __shared__ unsigned long long tsum;
  if (t == 0) tsum = 0;
  __syncthreads();
  for (int o = 32; o > 0; o >>= 1) mine += __shfl_down(mine, o, 64);
  if ((t & 63) == 0) atomicAdd(&tsum, (unsigned long long)mine);
  __syncthreads();
  if (t == 0 && tsum != a.pages[p].n_out) atomicOr(&a.pages_bad[p], 1u);  // size mismatch
}

// E: k_snap_exec -- one 1024-thread workgroup per 64 KiB output block, fed by the compressed page
// itself (r05: the 8-byte element records k_snap_emit wrote to HBM at 2.4x amplification and this
// kernel read back are gone, and so is the emit launch).
//  0. the block's chunks are [block_chunk[b], the chunk holding the next block's first element]; the
//     bits of a chunk's visited bitmap at or after its true entry are exactly its element starts
//     (chains that meet coincide; k_snap_count rewrote the chunks whose true chain is another one).
//     The chunks' compressed bytes are staged in the LDS (in the map's space, not yet in use);
//  1. each thread counts the start bits of four bitmap words; a workgroup scan ranks them, and the
//     elements are cut into runs of EXEC_RUN: in round q thread t walks run q * 1024 + t from its
//     first start, element after element through the staged headers, keeping them in registers;
//     a scan of the runs' lengths gives each run its output offset (from the first chunk's
//     k_snap_scan offset); once the stage is released the elements of this block set their start
//     bit and the map entry of their first byte (src[rel] = rel - offset; a literal points at
//     itself). Runs of a wave are consecutive, so the lanes work in step and their map and literal
//     writes sit a run apart in the LDS banks (r05's first cuts: 16 compressed positions per thread
//     in 16 KiB passes -- three decodes per element, lanes waiting on the densest one, 51.6 K clocks
//     per block for this phase against 12.4 K for reading emit's records; then one long run per
//     thread -- 41 K, its lanes' writes 64 output bytes apart, in two LDS banks);
//  2. every byte's map entry from the last start at or before it, then pointer jumping until every
//     byte points at its literal origin (u16 map of the block in LDS, roots in registers);
//  3. the LDS becomes the block's bytes (lower half) and its compressed input (upper half); each
//     thread walks its elements again from its first start and copies its literals LDS -> LDS,
//     reads batched ahead of writes; long literals go to whole waves;
//  4. each thread gathers its groups' bytes from their roots and stores them (coalesced dwords).
// Every element of the chunk range is checked (a copy reaching before its fragment, an element
// straddling a block, literal bytes past the page) and the block's elements must cover it exactly;
// anything else -- or a block of more than EXEC_EMAX * 1024 elements or 128 KiB of compressed
// input, which the SNAPPY compressor's output never has -- flags the page for k_snap_serial.
constexpr int EXEC_T = 1024;
#ifndef DR_EXEC_EMAX
#define DR_EXEC_EMAX 32
#endif
#ifndef DR_EXEC_EHELD
#define DR_EXEC_EHELD 16
#endif
constexpr uint32_t EXEC_EMAX = DR_EXEC_EMAX;        // elements per thread: 32 K per block (alternating 1-byte literals and 4-byte copies: 26 K)
constexpr uint32_t EXEC_EHELD = DR_EXEC_EHELD;      // elements per thread kept in registers through the jumping
constexpr uint32_t EXEC_LONG = 256;                 // literal records queued for the cooperative copy (at most)
#ifndef DR_EXEC_LONG_LEN
#define DR_EXEC_LONG_LEN 64
#endif
constexpr uint32_t EXEC_LONG_LEN = DR_EXEC_LONG_LEN;  // literals longer than this are copied by a whole wave
#ifndef DR_EXEC_SPLIT
#define DR_EXEC_SPLIT 4
#endif
constexpr uint32_t EXEC_SPLIT = DR_EXEC_SPLIT;  // map groups whose reads are issued before their writes (divides 16; 1: 2.725 ms, 4: 2.693, 16: spills, 2.83)

// An element's fields from its header word.
struct SnapEl {
  uint32_t len, hdr, off;  // output bytes, header bytes, copy offset
  bool lit;
};
__device__ __forceinline__ SnapEl snap_fields(uint64_t w) {
  uint32_t adv, len;
  snap_step(w, &adv, &len);
  const uint32_t tag = uint32_t(w & 0xff), t = tag & 3u, w8 = uint32_t(w >> 8);
  SnapEl e;
  e.len = len;
  e.lit = t == 0;
  e.hdr = e.lit ? adv - len : adv;
  e.off = t == 1 ? (((tag >> 5) << 8) | (w8 & 0xffu)) : t == 2 ? (w8 & 0xffffu) : w8;
  return e;
}
// Header bytes at byte offset o of a dword-addressed LDS buffer (the low five are exact).
__device__ __forceinline__ uint64_t lds_hdr(const uint32_t* b32, uint32_t o) {
  const uint32_t di = o >> 2, sh = o & 3;
  return ((uint64_t(b32[di + 1]) << 32) | b32[di]) >> (8 * sh);
}
// Exclusive workgroup scan (EXEC_T threads) of x; `total` gets the sum. Contains one barrier; the
// caller separates two calls by another (the wave sums are reused).
__device__ __forceinline__ uint32_t block_excl(uint32_t x, uint32_t* wsum, uint32_t& total) {
  const uint32_t incl = wv::scan_incl(x, 0u, [](uint32_t p, uint32_t q) { return p + q; });
  const uint32_t wi = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 63) wsum[wi] = incl;
  __syncthreads();
  uint32_t before = 0, tot = 0;
#pragma unroll
  for (uint32_t q = 0; q < EXEC_T / 64; ++q) {
    const uint32_t v = wsum[q];
    before += q < wi ? v : 0u;
    tot += v;
  }
  total = tot;
  return before + incl - x;
}
// An element in a register: a literal EL_LIT | hdr << 24 | (len - 1); a copy hdr << 24 |
// (len - 1) << 16 | offset (hdr: header bytes, 1..5; a copy's len - 1 < 64 once validated).
constexpr uint32_t EL_LIT = 0x80000000u;

__global__ void __launch_bounds__(EXEC_T) k_snap_exec(SnappyArgs a) {
  __shared__ __attribute__((aligned(16))) uint16_t src[SNAP_BLOCK];  // stage, then map, then bytes + input
  __shared__ uint32_t s_bad, s_nlong, s_cov;
  __shared__ uint32_t s_wsum[EXEC_T / 64];
  __shared__ uint32_t s_first[EXEC_T];  // each thread's first element (page-relative position)
  __shared__ uint64_t s_long[EXEC_LONG];  // queued long literal records
  __shared__ uint32_t starts_mem[SNAP_BLOCK / 32 + 2];  // element start bits, after two zero words
  uint32_t* const starts = starts_mem + 2;
  const uint32_t b = blockIdx.x;
  const uint32_t p = a.block_page[b];
  if (a.pages_bad[p]) return;
  const SnapPage pg = a.pages[p];
  const uint8_t* in = reinterpret_cast<const uint8_t*>(pg.in);
  uint8_t* out = reinterpret_cast<uint8_t*>(pg.out);
  const uint64_t bs = uint64_t(b - pg.block_base) * SNAP_BLOCK;
  const uint64_t be = min(bs + SNAP_BLOCK, uint64_t(pg.n_out));
  const uint32_t nbytes = uint32_t(be - bs);
  const int t = threadIdx.x;
  // diagnostic phase stamps (DR_SNAP_DEBUG allocates the buffer; null otherwise)
  auto stamp = [&](int k) {
    if (a.stamps && t == 0) a.stamps[uint64_t(b) * 16 + k] = __builtin_amdgcn_s_memtime();
  };
  stamp(0);
  // 0. the block's chunk range and compressed range [P_lo, P_hi) (block-uniform)
  const uint32_t c0 = a.chunk_base[p], ncp = a.chunk_base[p + 1] - c0;
  const uint32_t cl = a.block_chunk[b];
  const bool last_blk = b + 1 >= a.nblocks || a.block_page[b + 1] != p;
  const uint32_t cn = last_blk ? c0 + ncp : a.block_chunk[b + 1] + 1u;  // ~0 (unclaimed) wraps to 0
  const bool range_ok = cl >= c0 && cl < c0 + ncp && cn > cl && cn <= c0 + ncp;
  const uint64_t P_lo = range_ok ? uint64_t(cl - c0) * SNAP_CH : 0;
  const uint64_t P_hi = range_ok ? min(uint64_t(cn - c0) * SNAP_CH, uint64_t(pg.n_in)) : 0;
  const uintptr_t ib = reinterpret_cast<uintptr_t>(in);
  const uint32_t sh0 = uint32_t((ib + P_lo) & 15);  // the stage's first byte sits sh0 bytes into a vector
  const uint32_t nv_all = uint32_t((sh0 + (P_hi - P_lo) + 8 + 15) / 16);  // headers read 8 bytes past the range
  if (!range_ok || P_hi <= P_lo || nv_all * 16 > 2 * SNAP_BLOCK) {
    if (t == 0) atomicOr(&a.pages_bad[p], 16u);
    return;
  }
  if (t == 0) {
    s_bad = 0;
    s_nlong = 0;
    s_cov = 0;
  }
  for (uint32_t w = t; w < SNAP_BLOCK / 32 + 2; w += EXEC_T) starts_mem[w] = 0;
  // the block's loads, all issued before any is used (one HBM round trip): its chunks' start bitmaps
  // (four words per thread, half a chunk: one 16-byte load) and entries, the first chunk's output
  // offset, and its chunks' compressed bytes, which go into the map's space
  const uint32_t W = (cn - cl) * (SNAP_CH / 32);
  const bool has_words = 4 * uint32_t(t) < W;
  uint4 vw = make_uint4(0, 0, 0, 0);
  uint64_t ent = 0;
  if (has_words) {
    vw = *reinterpret_cast<const uint4*>(&a.vis[uint64_t(cl) * (SNAP_CH / 32) + 4 * uint32_t(t)]);
    ent = a.entry[cl + (4 * uint32_t(t)) / (SNAP_CH / 32)];
  }
  const uint32_t out0 = a.chunk_out_start[cl];
  const uint4* g4 = reinterpret_cast<const uint4*>(ib + P_lo - sh0);
  uint4* s4 = reinterpret_cast<uint4*>(src);
  {
    constexpr uint32_t PER = 2 * SNAP_BLOCK / 16 / EXEC_T;  // 8 vectors per thread at most
    uint4 v[PER];
#pragma unroll
    for (uint32_t k = 0; k < PER; ++k)
      if (uint32_t(t) + k * EXEC_T < nv_all) v[k] = gload16(g4 + uint32_t(t) + k * EXEC_T);
#pragma unroll
    for (uint32_t k = 0; k < PER; ++k)
      if (uint32_t(t) + k * EXEC_T < nv_all) s4[uint32_t(t) + k * EXEC_T] = v[k];
  }
  // 1a. the start bits masked to each chunk's true chain and to the range (positions are
  //     page-relative and fit 32 bits: a page is at most 4 GiB)
  const uint32_t plo = uint32_t(P_lo), phi = uint32_t(P_hi);
  const uint32_t q0 = plo + uint32_t(t) * 128;  // the thread's first position
  uint32_t wd[4] = {vw.x, vw.y, vw.z, vw.w};
  if (has_words) {
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
      const uint32_t ws = q0 + 32 * q;  // the word's first position
      const uint32_t lo_cut = ent > ws ? min(uint32_t(ent - ws), 32u) : 0u;
      const uint32_t hi_cut = ws >= phi ? 0u : min(phi - ws, 32u);  // positions below the range end
      const uint32_t keep = (lo_cut >= 32 ? 0u : ~0u << lo_cut) & (hi_cut >= 32 ? ~0u : (1u << hi_cut) - 1u);
      wd[q] &= keep;
    }
  }
  stamp(1);
  const uint32_t cnt = __popc(wd[0]) + __popc(wd[1]) + __popc(wd[2]) + __popc(wd[3]);
  uint32_t n_el;
  const uint32_t ex = block_excl(cnt, s_wsum, n_el);
  const uint32_t E = (n_el + EXEC_T - 1) / EXEC_T;  // elements per thread (block-uniform)
  if (E > EXEC_EMAX) {
    if (t == 0) atomicOr(&a.pages_bad[p], 16u);
    return;
  }
  // 1b. the first element of every thread whose share [kE, kE + E) starts among this thread's start
  //     bits: the r-th set bit of a word by a branch-free binary search on popcounts
  if (E) {
    for (uint32_t k = (ex + E - 1) / E; k * E < ex + cnt; ++k) {
      uint32_t r = k * E - ex, w = 0, base = q0;
#pragma unroll
      for (uint32_t q = 0; q < 4; ++q) {  // the word holding rank r
        const uint32_t pc = __popc(wd[q]);
        const bool here = r < pc && w == 0 && base == q0 + 32 * q;
        w = here ? wd[q] : w;
        const bool past = base == q0 + 32 * q && !here;
        r -= past ? pc : 0u;
        base += past ? 32u : 0u;
      }
      uint32_t pos = 0;
#pragma unroll
      for (uint32_t width = 16; width; width >>= 1) {
        const uint32_t c = __popc(w & ((1u << width) - 1u));
        const bool up = r >= c;
        r -= up ? c : 0u;
        w = up ? w >> width : w;
        pos += up ? width : 0u;
      }
      s_first[k] = base + pos;
    }
  }
  stamp(2);
  __syncthreads();
  stamp(3);
  // 1c. thread t walks its share of elements through the staged headers, keeping each in a register
  const uint32_t mine = n_el > uint32_t(t) * E ? min(E, n_el - uint32_t(t) * E) : 0u;
  const uint32_t first = mine ? s_first[t] : 0u;
  const uint32_t* stage32 = reinterpret_cast<const uint32_t*>(src);
  const uint32_t so_lim = nv_all * 16 - 8;  // the last staged header start
  uint32_t el[EXEC_EMAX];
  uint32_t sum = 0;
  bool bad = false;
  {
    // Branch-free decode (mask blends, not ?:): written with conditional expressions and
    // short-circuit tests, and the page size read inside the loop, the compiler turned each element
    // into a dozen divergent branches and a global load
    const uint64_t n_in = pg.n_in;
    const auto sel = sel32;
    uint32_t pos = first;
#pragma unroll
    for (uint32_t k = 0; k < EXEC_EMAX; ++k) {
      el[k] = 0;
      if (k < mine) {
        const uint32_t so = pos - plo + sh0;
        const uint64_t w = lds_hdr(stage32, min(so, so_lim));
        const uint32_t tag = uint32_t(w) & 0xffu, ty = tag & 3u, l6 = tag >> 2, w8 = uint32_t(w >> 8);
        const bool lit = ty == 0u, c1 = ty == 1u;
        const uint32_t nb = l6 > 59u ? l6 - 59u : 0u;  // a literal's extra length bytes
        const uint32_t lmask = sel(nb >= 4u, ~0u, (1u << (8u * (nb & 3u))) - 1u);
        const uint32_t lit_len = sel(nb != 0u, w8 & lmask, l6) + 1u;
        const uint32_t len = sel(lit, lit_len, sel(c1, (l6 & 7u) + 4u, l6 + 1u));
        const uint32_t hdr = ((0x5320u >> (4u * ty)) & 15u) + sel(lit, 1u + nb, 0u);  // 1 + nb, 2, 3, 5
        const uint32_t off = sel(c1, ((tag >> 5) << 8) | (w8 & 0xffu), w8 & 0xffffu);
        const uint32_t adv = hdr + sel(lit, len, 0u);
        // a literal past the page or longer than a fragment, a copy offset no fragment has (copy-4's
        // upper offset bytes): the page is not one the parallel path can take
        const bool bad_lit = (len > SNAP_BLOCK) | (uint64_t(pos) + adv > n_in);
        const bool bad_cp = (ty == 3u) & ((w8 >> 16) != 0u);
        bad |= (so > so_lim) | (lit & bad_lit) | (!lit & bad_cp);
        el[k] = (hdr << 24) | sel(lit, EL_LIT | ((len - 1u) & 0xffffu), ((len - 1u) << 16) | off);
        sum += sel(lit, min(len, SNAP_BLOCK), len);
        pos += adv;
      }
    }
  }
  uint32_t tot_out;
  const uint32_t o_first = out0 + block_excl(sum, s_wsum, tot_out);  // page-relative output offset of the thread's first element
  stamp(4);
  __syncthreads();  // every thread is done with the stage (and the scan words)
  // 1d. start bits and first-byte map entries of this block's elements
  const uint32_t bs32 = uint32_t(bs), be32 = uint32_t(be);
  uint32_t cov = 0;
  {
    uint32_t o = o_first;
#pragma unroll
    for (uint32_t k = 0; k < EXEC_EMAX; ++k) {
      if (k < mine) {
        const uint32_t x = el[k];
        const bool lit = x & EL_LIT;
        const uint32_t len = lit ? (x & 0xffffu) + 1u : ((x >> 16) & 0x7fu) + 1u;
        const uint32_t off = x & 0xffffu;
        const uint32_t rel = o - bs32;
        // tests combined without short circuits: one divergent branch per element, not four
        const bool hit = (o < be32) & (o + len > bs32);
        const bool cut = (o < bs32) | (o + len > be32) | (!lit & ((off == 0u) | (off > rel)));
        bad |= hit & cut;  // straddles the block, or a copy reaching before its fragment
        if (hit & !cut) {
          atomicOr(&starts[rel >> 5], 1u << (rel & 31));
          src[rel] = uint16_t(lit ? rel : rel - off);
          cov += len;
        }
        o += len;
      }
    }
  }
  if (bad) s_bad = 1;
  {
    const uint32_t cw = wv::scan_incl(cov, 0u, [](uint32_t x, uint32_t y) { return x + y; });
    if ((t & 63) == 63) atomicAdd(&s_cov, cw);
  }
  __syncthreads();
  stamp(5);
  if (s_bad || s_cov != nbytes) {  // block-uniform: the block's elements must cover it exactly
    if (t == 0) atomicOr(&a.pages_bad[p], 32u);
    return;
  }
  // Byte ownership: thread t owns the 4-byte groups i0 = 4 (t + 1024 j), j < 16; k = 4 j + e.
  // 1b. every byte's element starts at the last start bit <= it. A copy is at most 64 bytes long,
  //     so a byte with no start in the 64 bytes up to it lies in a long literal. Copy bytes point
  //     at i - offset, literal bytes at themselves (i - start + src[start] covers both). Each group
  //     is read and written as one 8-byte word; element starts keep their value, so reading
  //     src[start] never races.
  // 2. pointer jumping over the same bytes, current pointers in registers. No barriers: every value
  //    read is an ancestor of the byte (older or newer, both valid) and ancestors have smaller
  //    indices, so each step strictly moves towards the root (literal bytes are their own roots).
  //    Pointers are read 8 at a time so the LDS reads are in flight together.
  uint32_t xp[32];    // current pointers of the 4-byte groups, two u16 per register; roots at the end
  {
    uint32_t act = 0;   // groups with a byte not yet at its root
    // groups in batches of EXEC_SPLIT: a batch's reads, then its writes (element starts keep their
    // value, so no read depends on a write; the compiler cannot see that and otherwise orders each
    // group's reads after the previous group's write)
    const bool part = nbytes != SNAP_BLOCK;  // block-uniform: a page's last block
#pragma unroll
    for (uint32_t jb = 0; jb < 16; jb += EXEC_SPLIT) {
      // staged so a batch's LDS reads are in flight together: start words and group entries, then
      // the starts the groups continue (pinned by an empty asm: the compiler would otherwise sink
      // each read into the branch of groups whose first byte is no start, one round trip per group;
      // a volatile read did pin them, but as flat loads each waited on alone)
      uint32_t w0[EXEC_SPLIT], prev[EXEC_SPLIT], pv[EXEC_SPLIT];
      bool pvalid[EXEC_SPLIT];
      uint2 g[EXEC_SPLIT];
#pragma unroll
      for (uint32_t q = 0; q < EXEC_SPLIT; ++q) {
        const uint32_t i0 = 4 * (uint32_t(t) + EXEC_T * (jb + q));
        const uint32_t wi = i0 >> 5, sh = i0 & 31;
        w0[q] = starts[wi];
        const uint32_t w1 = starts[int32_t(wi) - 1], w2 = starts[int32_t(wi) - 2];  // zero words before the block
        g[q] = *reinterpret_cast<const uint2*>(&src[i0]);
        // the last start before the group among the 64..95 bytes before it, branch-free: the highest
        // set bit of (m0, w1) as one 64-bit word, else of w2 (__clz(0) = 32, __clzll(0) = 64)
        const uint32_t m0 = w0[q] & ((1u << sh) - 1u);
        const uint64_t x64 = (uint64_t(m0) << 32) | w1;
        const uint32_t pa = wi * 32 + 31 - uint32_t(__clzll(int64_t(x64)));
        pvalid[q] = (x64 | w2) != 0;
        prev[q] = x64 ? pa : pa - uint32_t(__clz(int32_t(w2)));
      }
#pragma unroll
      for (uint32_t q = 0; q < EXEC_SPLIT; ++q) pv[q] = src[pvalid[q] ? prev[q] : 0u];
#pragma unroll
      for (uint32_t q = 0; q < EXEC_SPLIT; ++q) asm volatile("" : "+v"(pv[q]));
#pragma unroll
      for (uint32_t q = 0; q < EXEC_SPLIT; ++q) {
        const uint32_t j = jb + q;
        const uint32_t i0 = 4 * (uint32_t(t) + EXEC_T * j);
        // byte i of an element starting at st maps to i + (src[st] - st): minus the offset for a
        // copy, 0 for a literal (and for a byte with no start in the 64..95 bytes before it, which
        // lies in a long literal: copies are at most 64 bytes, checked above)
        const int32_t dp = pvalid[q] ? int32_t(pv[q]) - int32_t(prev[q]) : 0;
        const uint32_t sb = w0[q] >> (i0 & 31);  // start bits of the group's bytes (bits 0..3)
        const int32_t d0 = (sb & 1u) ? int32_t(g[q].x & 0xffffu) - int32_t(i0) : dp;
        const int32_t d1 = (sb & 2u) ? int32_t(g[q].x >> 16) - int32_t(i0 + 1) : d0;
        const int32_t d2 = (sb & 4u) ? int32_t(g[q].y & 0xffffu) - int32_t(i0 + 2) : d1;
        const int32_t d3 = (sb & 8u) ? int32_t(g[q].y >> 16) - int32_t(i0 + 3) : d2;
        xp[2 * j] = uint32_t(int32_t(i0) + d0) | (uint32_t(int32_t(i0 + 1) + d1) << 16);
        xp[2 * j + 1] = uint32_t(int32_t(i0 + 2) + d2) | (uint32_t(int32_t(i0 + 3) + d3) << 16);
        // a group is active while a byte points away from itself
        if ((d0 | d1 | d2 | d3) != 0) act |= 1u << j;
        if (part && i0 + 4 > nbytes) {  // past the block end: the identity
          const uint32_t x0 = i0 < nbytes ? (xp[2 * j] & 0xffffu) : i0, x1 = i0 + 1 < nbytes ? (xp[2 * j] >> 16) : i0 + 1;
          const uint32_t x2 = i0 + 2 < nbytes ? (xp[2 * j + 1] & 0xffffu) : i0 + 2, x3 = i0 + 3 < nbytes ? (xp[2 * j + 1] >> 16) : i0 + 3;
          xp[2 * j] = x0 | (x1 << 16);
          xp[2 * j + 1] = x2 | (x3 << 16);
          if (xp[2 * j] == (i0 | ((i0 + 1) << 16)) && xp[2 * j + 1] == ((i0 + 2) | ((i0 + 3) << 16))) act &= ~(1u << j);
        }
      }
#pragma unroll
      for (uint32_t j = jb; j < jb + EXEC_SPLIT; ++j) {
        const uint32_t i0 = 4 * (uint32_t(t) + EXEC_T * j);
        if (i0 < nbytes) *reinterpret_cast<uint2*>(&src[i0]) = make_uint2(xp[2 * j], xp[2 * j + 1]);
      }
    }
    __syncthreads();
    stamp(6);
    uint32_t rounds = 0;
    while (act) {
      ++rounds;
      if (a.stamps && rounds <= 3) {  // (DR_SNAP_DEBUG) active groups at the start of rounds 1..3, one atomic per wave
        uint32_t v = __popc(act);
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if ((t & 63) == 0) atomicAdd(reinterpret_cast<unsigned long long*>(&a.stamps[uint64_t(b) * 16 + 10 + rounds]),
                                     (unsigned long long)v);
      }
#pragma unroll
      for (uint32_t j = 0; j < 16; ++j) {
        if (act & (1u << j)) {
          const uint32_t a0 = xp[2 * j], a1 = xp[2 * j + 1];
          const uint32_t y0 = src[a0 & 0xffffu], y1 = src[a0 >> 16], y2 = src[a1 & 0xffffu], y3 = src[a1 >> 16];
          const uint32_t b0 = y0 | (y1 << 16), b1 = y2 | (y3 << 16);
          if (b0 == a0 && b1 == a1) {
            act &= ~(1u << j);
          } else {
            xp[2 * j] = b0;
            xp[2 * j + 1] = b1;
            *reinterpret_cast<uint2*>(&src[4 * (uint32_t(t) + EXEC_T * j)]) = make_uint2(b0, b1);
          }
        }
      }
    }
    if (a.stamps) atomicMax(reinterpret_cast<unsigned long long*>(&a.stamps[uint64_t(b) * 16 + 14]), (unsigned long long)rounds);
  }
  __syncthreads();
  stamp(7);
  // 3. the LDS becomes the block's bytes (lower half) and its compressed input (upper half: the
  //    block's whole range, headers included, so each thread walks its elements again from it)
  uint8_t* bytes = reinterpret_cast<uint8_t*>(src);
  uint8_t* stage = bytes + SNAP_BLOCK;
  const bool staged = nv_all * 16 <= SNAP_BLOCK;  // block-uniform
  if (staged) {  // all of a thread's loads in flight at once (nv_all <= SNAP_BLOCK / 16: four per thread)
    uint4* u4 = reinterpret_cast<uint4*>(stage);
    constexpr uint32_t PER = SNAP_BLOCK / 16 / EXEC_T;
    uint4 v[PER];
#pragma unroll
    for (uint32_t k = 0; k < PER; ++k) v[k] = gload16(g4 + min(uint32_t(t) + k * EXEC_T, nv_all - 1));
#pragma unroll
    for (uint32_t k = 0; k < PER; ++k)
      if (uint32_t(t) + k * EXEC_T < nv_all) u4[uint32_t(t) + k * EXEC_T] = v[k];
  }
  __syncthreads();
  stamp(8);
  // a literal of this block (rel, len, page-relative input position ip): LDS -> LDS copy, or queued
  // for a whole wave when long
  auto copy_lit = [&](uint32_t rel, uint32_t len, uint64_t ip) {
    if (len > EXEC_LONG_LEN) {  // queued while there is room, else copied by this lane below
      const uint32_t slot = atomicAdd(&s_nlong, 1u);
      if (slot < EXEC_LONG) {
        s_long[slot] = uint64_t(rel) | (uint64_t(len - 1) << 16) | (uint64_t(uint32_t(ip)) << 32);
        return;
      }
    }
    if (!staged) {  // a poorly compressible block: its input does not fit the stage; read it in place
      const uint8_t* sp = in + ip;
      for (uint32_t i = 0; i < len; ++i) bytes[rel + i] = sp[i];
      return;
    }
    // byte head up to a 4-byte aligned destination, then aligned dword stores of realigned source
    // dwords (five reads in flight before four writes: one LDS round trip per 16 bytes), a byte tail
    uint32_t q = uint32_t(ip - P_lo) + sh0 + SNAP_BLOCK;
    uint32_t d = rel, n = len;
    // the byte head and tail each from one realigned 4-byte read (reads past the range stay in
    // the stage: it holds 8 bytes past it), their byte stores issued together
    const auto read4 = [&](uint32_t at) {
      const uint32_t* pa = reinterpret_cast<const uint32_t*>(bytes + (at & ~3u));
      return __builtin_amdgcn_alignbyte(pa[1], pa[0], at & 3u);
    };
    if (const uint32_t h = min((4u - (d & 3u)) & 3u, n)) {
      const uint32_t v = read4(q);
      bytes[d] = uint8_t(v);
      if (h > 1) bytes[d + 1] = uint8_t(v >> 8);
      if (h > 2) bytes[d + 2] = uint8_t(v >> 16);
      d += h;
      q += h;
      n -= h;
    }
    const uint32_t sh = q & 3;
    const uint32_t* qa = reinterpret_cast<const uint32_t*>(bytes + (q & ~3u));
    uint32_t* da = reinterpret_cast<uint32_t*>(bytes + d);
    for (; n >= 16; n -= 16) {
      const uint32_t s0 = qa[0], s1 = qa[1], s2 = qa[2], s3 = qa[3], s4 = qa[4];
      da[0] = __builtin_amdgcn_alignbyte(s1, s0, sh);
      da[1] = __builtin_amdgcn_alignbyte(s2, s1, sh);
      da[2] = __builtin_amdgcn_alignbyte(s3, s2, sh);
      da[3] = __builtin_amdgcn_alignbyte(s4, s3, sh);
      qa += 4;
      da += 4;
    }
    for (; n >= 4; n -= 4) {
      *da++ = __builtin_amdgcn_alignbyte(qa[1], qa[0], sh);
      ++qa;
    }
    if (n) {  // fewer than 4 bytes left
      d = uint32_t(reinterpret_cast<uint8_t*>(da) - bytes);
      q = uint32_t(reinterpret_cast<const uint8_t*>(qa) - bytes) + sh;
      const uint32_t v = read4(q);
      bytes[d] = uint8_t(v);
      if (n > 1) bytes[d + 1] = uint8_t(v >> 8);
      if (n > 2) bytes[d + 2] = uint8_t(v >> 16);
    }
  };
  // the thread's elements again from its first start: from the registers when the thread has at
  // most EXEC_EHELD (its elements stayed live through the jumping), else re-read from the stage
  if (E <= EXEC_EHELD) {  // block-uniform
    uint32_t pos = first, o = o_first;
#pragma unroll
    for (uint32_t k = 0; k < EXEC_EHELD; ++k) {
      if (k < mine) {
        const uint32_t x = el[k];
        const bool lit = x & EL_LIT;
        const uint32_t len = lit ? (x & 0xffffu) + 1u : ((x >> 16) & 0x7fu) + 1u;
        const uint32_t hdr = (x >> 24) & 7u;
        if (lit && o >= bs32 && o < be32) copy_lit(o - bs32, len, pos + hdr);
        o += len;
        pos += hdr + (lit ? len : 0u);
      }
    }
  } else {
    const uint32_t* st32 = reinterpret_cast<const uint32_t*>(stage);
    uint32_t pos = first, o = o_first;
    for (uint32_t k = 0; k < mine; ++k) {
      const uint64_t w = staged ? lds_hdr(st32, pos - plo + sh0) : load_u64(in + pos);
      const SnapEl e = snap_fields(w);
      if (e.lit && o >= bs32 && o < be32) copy_lit(o - bs32, e.len, pos + e.hdr);
      o += e.len;
      pos += e.hdr + (e.lit ? e.len : 0u);
    }
  }
  __syncthreads();
  stamp(9);
  const uint32_t nlong = min(s_nlong, EXEC_LONG);
  for (uint32_t L = uint32_t(t) >> 6; L < nlong; L += EXEC_T / 64) {  // long literals: one wave each
    const uint64_t wl = s_long[L];
    const uint32_t rel = uint32_t(wl & 0xffff);
    const uint32_t len = uint32_t((wl >> 16) & 0xffff) + 1;
    const uint32_t ipo = uint32_t(wl >> 32);
    if (staged) {
      const uint32_t q = ipo - uint32_t(P_lo) + sh0 + SNAP_BLOCK;
      for (uint32_t i = uint32_t(t) & 63; i < len; i += 64) bytes[rel + i] = bytes[q + i];
    } else {
      const uint8_t* ip = in + ipo;
      for (uint32_t i = uint32_t(t) & 63; i < len; i += 64) bytes[rel + i] = ip[i];
    }
  }
  __syncthreads();
  stamp(10);
  // 4. gather and store: the thread's 4-byte groups are the ones it resolved (roots still in
  //    registers); a wave's 64 groups are 256 contiguous bytes, so literal bytes (their own roots)
  //    and runs of one copy read consecutive LDS banks, and the dword stores coalesce
  uint8_t* dst = out + bs;
  uint32_t word[16];
#pragma unroll
  for (uint32_t j = 0; j < 16; ++j) {  // groups past the block end hold the identity (in the LDS)
    const uint32_t r01 = xp[2 * j], r23 = xp[2 * j + 1];
    word[j] = uint32_t(bytes[r01 & 0xffffu]) | (uint32_t(bytes[r01 >> 16]) << 8) |
              (uint32_t(bytes[r23 & 0xffffu]) << 16) | (uint32_t(bytes[r23 >> 16]) << 24);
  }
  if ((reinterpret_cast<uintptr_t>(dst) & 3) == 0 && nbytes == SNAP_BLOCK) {  // block-uniform
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) gstore32(reinterpret_cast<uint32_t*>(dst + 4 * (uint32_t(t) + EXEC_T * j)), word[j]);
  } else {  // a page's last block: bytes back to the LDS, then byte stores
    __syncthreads();
    uint32_t* b32 = reinterpret_cast<uint32_t*>(src);
#pragma unroll
    for (uint32_t j = 0; j < 16; ++j) b32[uint32_t(t) + EXEC_T * j] = word[j];
    __syncthreads();
    for (uint32_t i = t; i < nbytes; i += EXEC_T) dst[i] = bytes[i];
  }
  stamp(15);
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
    if ((in[ip] & 3u) == 0) {  // literal (a copy with offset 0 is corrupt, below)
      if (ip + el.hdr + el.len > pg.n_in) { atomicCAS(a.error, 0u, 1u); return; }
      for (uint32_t i = 0; i < el.len; ++i) out[op + i] = in[ip + el.hdr + i];
    } else {
      if (el.off == 0 || el.off > op) { atomicCAS(a.error, 0u, 1u); return; }
      for (uint32_t i = 0; i < el.len; ++i) out[op + i] = out[op - el.off + i];
    }
    op += el.len;
    ip += snap_adv(el);
  }
  if (op != pg.n_out) atomicCAS(a.error, 0u, 1u);
}

// Uncompressed pages, the raw level prefix of DATA_PAGE_V2 pages and the literal runs of pages the
// compressor could not shrink: PAGE_COPY_SLICES workgroups per job (r06: one, byte by byte, copied
// config 3's 7 MB at 77 GB/s -- ~100 jobs of up to 64 KiB). The destination is written in 16-byte
// stores; the source, at any byte offset from it, is read as aligned dwords and realigned.
constexpr uint32_t PAGE_COPY_SLICES = 16;
__global__ void __launch_bounds__(256) k_page_copy(const CopyJob* jobs, uint32_t njobs) {
  const uint32_t j = blockIdx.x, t = threadIdx.x, y = blockIdx.y;
  if (j >= njobs) return;
  const uint8_t* s = reinterpret_cast<const uint8_t*>(jobs[j].src);
  uint8_t* d = reinterpret_cast<uint8_t*>(jobs[j].dst);
  const uint64_t n = jobs[j].n;
  const uint64_t head = min(n, uint64_t((16u - (reinterpret_cast<uintptr_t>(d) & 15u)) & 15u));
  const uint64_t nv = (n - head) / 16;
  if (y == 0) {
    for (uint64_t i = t; i < head; i += 256) d[i] = s[i];
    for (uint64_t i = head + nv * 16 + t; i < n; i += 256) d[i] = s[i];
  }
  const uint8_t* s1 = s + head;
  uint4* d1 = reinterpret_cast<uint4*>(d + head);
  const uint32_t r = uint32_t(reinterpret_cast<uintptr_t>(s1) & 3u);
  const uint32_t* sw = reinterpret_cast<const uint32_t*>(s1 - r);
  for (uint64_t k = uint64_t(y) * 256 + t; k < nv; k += 256ull * PAGE_COPY_SLICES) {
    const uint32_t* w = sw + 4 * k;
    const uint32_t a0 = w[0], a1 = w[1], a2 = w[2], a3 = w[3];
    if (r == 0) {  // (uniform per job)
      d1[k] = make_uint4(a0, a1, a2, a3);
    } else {  // the fifth dword holds the chunk's last byte (r >= 1): inside the source
      const uint32_t a4 = w[4];
      d1[k] = make_uint4(__builtin_amdgcn_alignbyte(a1, a0, r), __builtin_amdgcn_alignbyte(a2, a1, r),
                         __builtin_amdgcn_alignbyte(a3, a2, r), __builtin_amdgcn_alignbyte(a4, a3, r));
    }
  }
}

}  // namespace dev

uint32_t snappy_wg_chunks() { return dev::WG_CHUNKS; }
uint32_t snappy_chunk_bytes() { return dev::SNAP_CH; }

void launch_snappy(const SnappyArgs& a, hipStream_t st, ScanScratch scan_scratch) {
  (void)scan_scratch;
  if (!a.npages) return;
  DR_LAUNCH(dev::k_snap_spec, dim3(a.nwg), dim3(dev::WG_CHUNKS), 0, st, a);
  const unsigned g = (a.nchunks + 255) / 256;
  DR_LAUNCH(dev::k_snap_assume, dim3(g), dim3(256), 0, st, a);
  DR_LAUNCH(dev::k_snap_entries, dim3(g), dim3(256), 0, st, a);
  DR_LAUNCH(dev::k_snap_regions, dim3(g), dim3(256), 0, st, a);
  DR_LAUNCH(dev::k_snap_resolve, dim3(512), dim3(64), 0, st, a);
  DR_LAUNCH(dev::k_snap_count, dim3(g), dim3(256), 0, st, a);
  DR_LAUNCH(dev::k_snap_scan, dim3(a.npages), dim3(dev::SCAN_T), 0, st, a);
  DR_LAUNCH(dev::k_snap_exec, dim3(a.nblocks), dim3(dev::EXEC_T), 0, st, a);
  DR_LAUNCH(dev::k_snap_serial, dim3((a.npages + 63) / 64), dim3(64), 0, st, a);
}

void launch_page_copy(const CopyJob* jobs, uint32_t njobs, hipStream_t st) {
  if (njobs) DR_LAUNCH(dev::k_page_copy, dim3(njobs, dev::PAGE_COPY_SLICES), dim3(256), 0, st, jobs, njobs);
}

}  // namespace dr
