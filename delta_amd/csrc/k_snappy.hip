// K2a: parallel SNAPPY page decompression for checkpoint column chunks.
//
// A raw snappy stream is a varint length followed by literal/copy elements; the element chain is
// serial, which with ~144K elements per 1 MiB page of paths makes a per-page decoder latency
// bound (measured: 1.28 s for config 3 with one lane per page). This decoder splits the work:
//
//  A  k_snap_spec     one lane per 256-byte chunk of compressed input parses elements
//                     *speculatively* from the chunk start and records the positions it visited
//                     (256-bit bitmap) and where it left the chunk.
//  B  k_snap_resolve  one wave per page walks the chunks in order carrying the true element
//                     boundary; where the true entry is on the speculative chain the chunk is
//                     already correct (chains that meet coincide from then on), otherwise the
//                     wave re-parses until it meets the chain. Mis-speculation is rare because
//                     a wrong start re-synchronises within a few elements.
//  C  k_snap_count    one lane per chunk re-walks its true elements: output bytes per chunk.
//  D  k_snap_blocks   per page: exclusive scan of chunk outputs; one lane per chunk records the
//                     input position of every element that starts a 64 KiB output block.
//  E  k_snap_exec     one lane per 64 KiB output block executes its elements. The snappy
//                     compressor compresses 64 KiB fragments independently, so copies never reach
//                     before their block; any page that violates this (or whose blocks do not
//                     start on an element) is flagged and decoded by k_snap_serial instead.
#include "dev_common.h"
#include "kernels.h"

namespace dr {
namespace dev {

constexpr uint32_t SNAP_CH = 256;            // compressed bytes per speculation chunk
constexpr uint32_t SNAP_BLOCK = 65536;       // snappy compressor fragment size

struct Elem {
  uint32_t hdr;   // header bytes (tag + length/offset bytes)
  uint32_t len;   // output bytes
  uint32_t off;   // copy offset (0 for a literal)
};

// Decodes the element header at p (reads up to 5 bytes; buffers are padded).
__device__ __forceinline__ Elem snap_elem(const uint8_t* p) {
  const uint64_t w = load_u64(p);
  const uint32_t tag = uint32_t(w & 0xff);
  Elem e;
  switch (tag & 3) {
    case 0: {
      uint32_t l = tag >> 2;
      if (l < 60) { e.hdr = 1; e.len = l + 1; }
      else {
        const uint32_t nb = l - 59;
        const uint64_t v = (w >> 8) & ((nb >= 4) ? 0xffffffffull : ((1ull << (8 * nb)) - 1));
        e.hdr = 1 + nb;
        e.len = uint32_t(v) + 1;
      }
      e.off = 0;
      break;
    }
    case 1:
      e.hdr = 2;
      e.len = ((tag >> 2) & 7) + 4;
      e.off = ((tag >> 5) << 8) | uint32_t((w >> 8) & 0xff);
      break;
    case 2:
      e.hdr = 3;
      e.len = (tag >> 2) + 1;
      e.off = uint32_t((w >> 8) & 0xffff);
      break;
    default:
      e.hdr = 5;
      e.len = (tag >> 2) + 1;
      e.off = uint32_t((w >> 8) & 0xffffffffull);
      break;
  }
  return e;
}
// input bytes consumed by an element (header + literal payload)
__device__ __forceinline__ uint64_t snap_adv(const Elem& e) { return uint64_t(e.hdr) + (e.off ? 0u : e.len); }

__device__ __forceinline__ uint32_t chunk_page(const uint32_t* chunk_base, uint32_t npages, uint32_t c) {
  uint32_t lo = 0, hi = npages;  // last page with chunk_base[p] <= c
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (chunk_base[mid] <= c) lo = mid; else hi = mid;
  }
  return lo;
}

// A: speculative parse of every chunk.
__global__ void __launch_bounds__(256) k_snap_spec(SnappyArgs a) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= a.nchunks) return;
  const uint32_t p = chunk_page(a.chunk_base, a.npages, c);
  const SnapPage& pg = a.pages[p];
  const uint8_t* in = reinterpret_cast<const uint8_t*>(pg.in);
  const uint64_t cs = uint64_t(c - a.chunk_base[p]) * SNAP_CH;
  const uint64_t ce = min(cs + SNAP_CH, uint64_t(pg.n_in));
  uint32_t vis[SNAP_CH / 32];
#pragma unroll
  for (int k = 0; k < int(SNAP_CH / 32); ++k) vis[k] = 0;
  uint64_t pos = cs;
  while (pos < ce) {
    const uint32_t r = uint32_t(pos - cs);
#pragma unroll
    for (int k = 0; k < int(SNAP_CH / 32); ++k)
      if (int(r >> 5) == k) vis[k] |= 1u << (r & 31);
    pos += snap_adv(snap_elem(in + pos));
  }
  a.spec_exit[c] = pos > 0xffffffffull ? 0xffffffffu : uint32_t(pos);
#pragma unroll
  for (int k = 0; k < int(SNAP_CH / 32); ++k) a.vis[uint64_t(c) * (SNAP_CH / 32) + k] = vis[k];
}

// B: true chunk entries. One wave per page; lane 0 carries the entry, the wave prefetches the
// speculative exits and bitmaps 64 chunks at a time.
__global__ void __launch_bounds__(64) k_snap_resolve(SnappyArgs a) {
  const uint32_t p = blockIdx.x;
  if (p >= a.npages) return;
  const SnapPage& pg = a.pages[p];
  const uint8_t* in = reinterpret_cast<const uint8_t*>(pg.in);
  const uint32_t c0 = a.chunk_base[p], nc = a.chunk_base[p + 1] - c0;
  const int lane = threadIdx.x;
  uint64_t e = 0;  // true entry of the current chunk (relative to pg.in)
  for (uint32_t base = 0; base < nc; base += 64) {
    const uint32_t j = base + lane;
    uint32_t x = 0, v[SNAP_CH / 32];
    if (j < nc) {
      x = a.spec_exit[c0 + j];
#pragma unroll
      for (int k = 0; k < int(SNAP_CH / 32); ++k) v[k] = a.vis[uint64_t(c0 + j) * (SNAP_CH / 32) + k];
    }
    const uint32_t cnt = min(64u, nc - base);
    for (uint32_t l = 0; l < cnt; ++l) {
      const uint64_t cs = uint64_t(base + l) * SNAP_CH;
      const uint64_t ce = min(cs + SNAP_CH, uint64_t(pg.n_in));
      if (lane == 0) a.entry[c0 + base + l] = uint32_t(min(e, uint64_t(0xffffffffu)));
      if (e >= ce) continue;  // an element spans this whole chunk
      const uint32_t r = uint32_t(e - cs);
      uint32_t word = 0;
#pragma unroll
      for (int k = 0; k < int(SNAP_CH / 32); ++k) {
        const uint32_t vk = __shfl(v[k], int(l), 64);
        if (int(r >> 5) == k) word = vk;
      }
      if ((word >> (r & 31)) & 1u) {
        e = __shfl(x, int(l), 64);
        continue;
      }
      // mis-speculated: walk from the true entry until meeting the speculative chain
      uint64_t pos = e;
      bool met = false;
      while (pos < ce) {
        pos += snap_adv(snap_elem(in + pos));
        if (pos < ce) {
          const uint32_t rr = uint32_t(pos - cs);
          uint32_t w2 = 0;
#pragma unroll
          for (int k = 0; k < int(SNAP_CH / 32); ++k) {
            const uint32_t vk = __shfl(v[k], int(l), 64);
            if (int(rr >> 5) == k) w2 = vk;
          }
          if ((w2 >> (rr & 31)) & 1u) { met = true; break; }
        }
      }
      e = met ? uint64_t(__shfl(x, int(l), 64)) : pos;
    }
  }
}

// C: output bytes produced by the true elements starting in each chunk.
__global__ void __launch_bounds__(256) k_snap_count(SnappyArgs a) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= a.nchunks) return;
  const uint32_t p = chunk_page(a.chunk_base, a.npages, c);
  const SnapPage& pg = a.pages[p];
  const uint8_t* in = reinterpret_cast<const uint8_t*>(pg.in);
  const uint64_t cs = uint64_t(c - a.chunk_base[p]) * SNAP_CH;
  const uint64_t ce = min(cs + SNAP_CH, uint64_t(pg.n_in));
  uint64_t pos = a.entry[c];
  uint64_t out = 0;
  while (pos < ce) {
    const Elem el = snap_elem(in + pos);
    out += el.len;
    pos += snap_adv(el);
  }
  a.chunk_out[c] = out > 0xffffffffull ? 0xffffffffu : uint32_t(out);
}

// D: per-page exclusive scan of chunk outputs (one wave per page), then block starts.
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
  if (lane == 0 && carry != a.pages[p].n_out) atomicOr(&a.pages_bad[p], 1u);  // output size mismatch
}

__global__ void __launch_bounds__(256) k_snap_blocks(SnappyArgs a) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= a.nchunks) return;
  const uint32_t p = chunk_page(a.chunk_base, a.npages, c);
  const SnapPage& pg = a.pages[p];
  const uint8_t* in = reinterpret_cast<const uint8_t*>(pg.in);
  const uint64_t cs = uint64_t(c - a.chunk_base[p]) * SNAP_CH;
  const uint64_t ce = min(cs + SNAP_CH, uint64_t(pg.n_in));
  uint64_t pos = a.entry[c];
  uint64_t out = a.chunk_out_start[c];
  const uint32_t nb = (pg.n_out + SNAP_BLOCK - 1) / SNAP_BLOCK;
  while (pos < ce) {
    const Elem el = snap_elem(in + pos);
    if ((out & (SNAP_BLOCK - 1)) == 0 && (out >> 16) < nb) a.block_in[pg.block_base + uint32_t(out >> 16)] = uint32_t(pos);
    if (el.len && (out >> 16) != ((out + el.len - 1) >> 16))
      atomicOr(&a.pages_bad[p], 2u);  // an element straddles a 64 KiB output boundary
    out += el.len;
    pos += snap_adv(el);
  }
}

// E: one lane per 64 KiB output block.
__global__ void __launch_bounds__(64) k_snap_exec(SnappyArgs a) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= a.nblocks) return;
  const uint32_t p = a.block_page[b];
  if (a.pages_bad[p]) return;
  const SnapPage& pg = a.pages[p];
  const uint8_t* in = reinterpret_cast<const uint8_t*>(pg.in);
  uint8_t* out = reinterpret_cast<uint8_t*>(pg.out);
  const uint32_t k = b - pg.block_base;
  uint64_t op = uint64_t(k) * SNAP_BLOCK;
  const uint64_t oend = min(op + SNAP_BLOCK, uint64_t(pg.n_out));
  const uint64_t bstart = op;
  uint64_t ip = a.block_in[b];
  while (op < oend) {
    if (ip >= pg.n_in) { atomicOr(&a.pages_bad[p], 4u); return; }
    const Elem el = snap_elem(in + ip);
    if (op + el.len > oend) { atomicOr(&a.pages_bad[p], 4u); return; }
    if (el.off == 0) {
      const uint8_t* s = in + ip + el.hdr;
      if (ip + el.hdr + el.len > pg.n_in) { atomicOr(&a.pages_bad[p], 4u); return; }
      uint32_t i = 0;
      for (; i + 8 <= el.len; i += 8) {
        const uint64_t w = load_u64(s + i);
#pragma unroll
        for (int q = 0; q < 8; ++q) out[op + i + q] = uint8_t(w >> (8 * q));
      }
      for (; i < el.len; ++i) out[op + i] = s[i];
    } else {
      if (el.off > op - bstart) { atomicOr(&a.pages_bad[p], 8u); return; }  // copy crosses its fragment
      const uint8_t* s = out + op - el.off;
      if (el.off >= 8) {
        uint32_t i = 0;
        for (; i + 8 <= el.len; i += 8) {
          const uint64_t w = load_u64(s + i);
#pragma unroll
          for (int q = 0; q < 8; ++q) out[op + i + q] = uint8_t(w >> (8 * q));
        }
        for (; i < el.len; ++i) out[op + i] = s[i];
      } else {
        for (uint32_t i = 0; i < el.len; ++i) out[op + i] = s[i];
      }
    }
    op += el.len;
    ip += snap_adv(el);
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
      if (el.off == 0 || el.off > op) { atomicCAS(a.error, 0u, 1u); return; }
      for (uint32_t i = 0; i < el.len; ++i) out[op + i] = out[op - el.off + i];
    }
    op += el.len;
    ip += snap_adv(el);
  }
  if (op != pg.n_out) atomicCAS(a.error, 0u, 1u);
}

// Uncompressed pages and the raw level prefix of DATA_PAGE_V2 pages: one wave per copy job.
__global__ void __launch_bounds__(256) k_page_copy(const CopyJob* jobs, uint32_t njobs) {
  const uint32_t j = blockIdx.x;
  if (j >= njobs) return;
  const uint8_t* s = reinterpret_cast<const uint8_t*>(jobs[j].src);
  uint8_t* d = reinterpret_cast<uint8_t*>(jobs[j].dst);
  const uint64_t n = jobs[j].n;
  for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) d[i] = s[i];
}

}  // namespace dev

void launch_snappy(const SnappyArgs& a, hipStream_t st) {
  if (!a.npages) return;
  const unsigned gc = (a.nchunks + 255) / 256;
  hipLaunchKernelGGL(dev::k_snap_spec, dim3(gc), dim3(256), 0, st, a);
  hipLaunchKernelGGL(dev::k_snap_resolve, dim3(a.npages), dim3(64), 0, st, a);
  hipLaunchKernelGGL(dev::k_snap_count, dim3(gc), dim3(256), 0, st, a);
  hipLaunchKernelGGL(dev::k_snap_scan, dim3(a.npages), dim3(64), 0, st, a);
  hipLaunchKernelGGL(dev::k_snap_blocks, dim3(gc), dim3(256), 0, st, a);
  hipLaunchKernelGGL(dev::k_snap_exec, dim3((a.nblocks + 63) / 64), dim3(64), 0, st, a);
  hipLaunchKernelGGL(dev::k_snap_serial, dim3((a.npages + 63) / 64), dim3(64), 0, st, a);
}

void launch_page_copy(const CopyJob* jobs, uint32_t njobs, hipStream_t st) {
  if (njobs) hipLaunchKernelGGL(dev::k_page_copy, dim3(njobs), dim3(256), 0, st, jobs, njobs);
}

}  // namespace dr
