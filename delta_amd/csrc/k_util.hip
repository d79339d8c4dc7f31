// Small gather kernels used to move result subsets to the host in one transfer each.
#include "dev_common.h"
#include "kernels.h"
#include <algorithm>
#include <stdexcept>
#include <string>

namespace dr {
namespace dev {

__global__ void k_iota_u32(uint32_t* out, uint64_t n) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) out[i] = uint32_t(i);
}

template <typename T, typename I>
__global__ void k_gather(const T* __restrict__ src, const I* __restrict__ idx, uint64_t n, T* __restrict__ dst) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[idx[i]];
}

// out[off[i] .. off[i] + len[i]) = bytes at ptr[i]. GATHER_G lanes per string, grid-stride: the
// lanes store the string's 16-byte-aligned destination chunks whole (a source dword-aligned 16-byte
// load plus one dword, funnel-shifted into place) and its unaligned head and tail bytewise. r04: one
// wave per string with byte copies left 46 of 64 lanes idle on a 110-byte path and waited for a round
// trip per string (2.95 ms for config 3's 10M live paths).
constexpr uint32_t GATHER_G = 4;
__global__ void __launch_bounds__(256) k_gather_bytes(const uint64_t* __restrict__ ptr, const uint32_t* __restrict__ len,
                                                      const uint64_t* __restrict__ off, uint64_t n,
                                                      uint8_t* __restrict__ out) {
  const uint32_t gl = threadIdx.x % GATHER_G;
  const uint64_t step = uint64_t(gridDim.x) * (blockDim.x / GATHER_G);
  for (uint64_t s = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) / GATHER_G; s < n; s += step) {
    const uint8_t* p = reinterpret_cast<const uint8_t*>(ptr[s]);
    const uint32_t L = len[s];
    uint8_t* o = out + off[s];
    const uint32_t head = min(L, (16u - uint32_t(reinterpret_cast<uintptr_t>(o) & 15u)) & 15u);
    const uint32_t nch = (L - head) / 16;
    for (uint32_t k = gl; k < head; k += GATHER_G) o[k] = p[k];
    for (uint32_t k = head + 16 * nch + gl; k < L; k += GATHER_G) o[k] = p[k];
    const uint8_t* end = p + L;
    for (uint32_t c = gl; c < nch; c += GATHER_G) {
      const uint8_t* sp = p + head + 16 * c;
      const uint32_t sh = uint32_t(reinterpret_cast<uintptr_t>(sp) & 3u);
      const uint8_t* sa = sp - sh;
      uint4 r;
      if (sa + 20 <= end) {  // every source byte read lies inside the string
        const uint4 v = *reinterpret_cast<const uint4*>(sa);
        const uint32_t w4 = *reinterpret_cast<const uint32_t*>(sa + 16);
        r.x = __builtin_amdgcn_alignbyte(v.y, v.x, sh);
        r.y = __builtin_amdgcn_alignbyte(v.z, v.y, sh);
        r.z = __builtin_amdgcn_alignbyte(v.w, v.z, sh);
        r.w = __builtin_amdgcn_alignbyte(w4, v.w, sh);
      } else {
        uint32_t w[4];
#pragma unroll
        for (int d = 0; d < 4; ++d)
          w[d] = uint32_t(sp[4 * d]) | uint32_t(sp[4 * d + 1]) << 8 | uint32_t(sp[4 * d + 2]) << 16 |
                 uint32_t(sp[4 * d + 3]) << 24;
        r = make_uint4(w[0], w[1], w[2], w[3]);
      }
      *reinterpret_cast<uint4*>(o + head + 16 * c) = r;
    }
  }
}

// One action per thread from src[i] to dst[i] across the nine action arrays, src_id[i] = sid: an
// applied tail's actions appended to the chain store in one launch (instead of nine copies and a
// fill, each a dispatch of its own on the per-commit path).
__global__ void __launch_bounds__(256) k_append_actions(AppendArgs a) {
  const uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  if (a.ctr && i < a.nctr) a.ctr[i] = i == a.ctr_at ? a.ctr_val : 0ull;
  if (i >= a.n) return;
  a.dst.kind[i] = a.src.kind[i];
  a.dst.flags[i] = a.src.flags[i];
  a.dst.key[i] = a.src.key[i];
  a.dst.path_ptr[i] = a.src.path_ptr[i];
  a.dst.path_len[i] = a.src.path_len[i];
  a.dst.size[i] = a.src.size[i];
  a.dst.delts[i] = a.src.delts[i];
  a.dst.src_off[i] = a.src.src_off[i];
  a.dst.src_len[i] = a.src.src_len[i];
  a.src_id[i] = a.sid;
}

__global__ void __launch_bounds__(256) k_readback(ReadbackArgs a) {
#pragma unroll
  for (int s = 0; s < READBACK_SPANS; ++s)
    for (uint32_t k = threadIdx.x; k < a.n[s]; k += 256) a.dst[s][k] = a.src[s][k];
  readback_flag(a);
}

// Host-resolved floating-point partition values into their K5 cache rows: row[k] gets bits[k] (the
// low 32 bits when w32 is given, else all 64) and its null byte (fix_fp_values: one upload, one launch).
__global__ void k_scatter_fp(const uint64_t* __restrict__ rows, const uint64_t* __restrict__ bits,
                             const uint8_t* __restrict__ nulls, uint64_t n, uint32_t* w32, int64_t* w64,
                             uint8_t* isnull) {
  const uint64_t k = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const uint64_t r = rows[k];
  if (w32) w32[r] = uint32_t(bits[k]);
  else w64[r] = int64_t(bits[k]);
  isnull[r] = nulls[k];
}

// dst[i] = src[i] - base: a row range's offset column rebased on the device (dr_state_export_range)
__global__ void k_rebase_i64(const int64_t* __restrict__ src, uint64_t n, int64_t base, int64_t* __restrict__ dst) {
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x)
    dst[i] = src[i] - base;
}

// Survivor lists in action order (engine.hip:order_lists): a list of distinct indices below nbits
// becomes a bitmap (one atomicOr per entry), the words' popcounts are scanned, and every word writes
// its set bits' indices at its offset -- a sort of a set in O(n + nbits / 32), no comparisons.
__global__ void k_bits_mark(const uint32_t* __restrict__ list, uint64_t n, uint64_t nbits, uint32_t* __restrict__ bm) {
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint32_t v = list[i];
    if (v < nbits) atomicOr(bm + (v >> 5), 1u << (v & 31u));  // (an entry out of range is lost: the count check sees it)
  }
}
__global__ void k_bits_popc(const uint32_t* __restrict__ bm, uint64_t w, uint32_t* __restrict__ cnt) {
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < w; i += uint64_t(gridDim.x) * blockDim.x)
    cnt[i] = uint32_t(__builtin_popcount(bm[i]));
}
__global__ void k_bits_emit(const uint32_t* __restrict__ bm, uint64_t w, const uint64_t* __restrict__ off,
                            uint32_t* __restrict__ out) {
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < w; i += uint64_t(gridDim.x) * blockDim.x) {
    uint32_t b = bm[i];
    uint64_t o = off[i];
    while (b) {
      out[o++] = uint32_t(i << 5) + uint32_t(__builtin_ctz(b));
      b &= b - 1u;
    }
  }
}

// Export of deletionTimestamp: valid = F_HAS_DELTS of the action's flags, and an absent one reads 0.
__global__ void k_delts_fix(const uint8_t* __restrict__ flags, const int64_t* __restrict__ delts, uint64_t n,
                            uint8_t* __restrict__ valid, int64_t* __restrict__ out) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t v = flags[i] & 1u;
  valid[i] = v;
  out[i] = v ? delts[i] : 0;
}

}  // namespace dev

namespace {
thread_local LaunchHook t_hook = nullptr;
thread_local void* t_hook_user = nullptr;
}  // namespace
void set_launch_hook(LaunchHook hook, void* user) {
  t_hook = hook;
  t_hook_user = user;
}
void launch_grid_check(const char* kernel, dim3 grid, dim3 block) {
  if (uint64_t(grid.x) * block.x >= (uint64_t(1) << 32) || uint64_t(grid.y) * block.y >= (uint64_t(1) << 32) ||
      uint64_t(grid.z) * block.z >= (uint64_t(1) << 32))
    throw std::runtime_error(std::string("launch of ") + kernel + ": grid of 2^32 or more work items in one dimension");
}

bool launch_events(const char* kernel, hipEvent_t* start, hipEvent_t* stop) {
  return t_hook && t_hook(t_hook_user, kernel, start, stop);
}

void launch_gather_u64(const uint64_t* src, const uint32_t* idx, uint64_t n, uint64_t* dst, hipStream_t st) {
  if (n) DR_LAUNCH((dev::k_gather<uint64_t, uint32_t>), dim3(unsigned((n + 255) / 256)), dim3(256), 0, st, src, idx, n, dst);
}
void launch_gather_u32(const uint32_t* src, const uint32_t* idx, uint64_t n, uint32_t* dst, hipStream_t st) {
  if (n) DR_LAUNCH((dev::k_gather<uint32_t, uint32_t>), dim3(unsigned((n + 255) / 256)), dim3(256), 0, st, src, idx, n, dst);
}
void launch_gather_u8(const uint8_t* src, const uint32_t* idx, uint64_t n, uint8_t* dst, hipStream_t st) {
  if (n) DR_LAUNCH((dev::k_gather<uint8_t, uint32_t>), dim3(unsigned((n + 255) / 256)), dim3(256), 0, st, src, idx, n, dst);
}
void launch_iota_u32(uint32_t* out, uint64_t n, hipStream_t st) {
  if (n) DR_LAUNCH(dev::k_iota_u32, dim3(unsigned((n + 255) / 256)), dim3(256), 0, st, out, n);
}
void launch_gather_u16(const uint16_t* src, const uint32_t* idx, uint64_t n, uint16_t* dst, hipStream_t st) {
  if (n) DR_LAUNCH((dev::k_gather<uint16_t, uint32_t>), dim3(unsigned((n + 255) / 256)), dim3(256), 0, st, src, idx, n, dst);
}
void launch_gather_u64_by64(const uint64_t* src, const uint64_t* idx, uint64_t n, uint64_t* dst, hipStream_t st) {
  if (n) DR_LAUNCH((dev::k_gather<uint64_t, uint64_t>), dim3(unsigned((n + 255) / 256)), dim3(256), 0, st, src, idx, n, dst);
}
void launch_gather_bytes(const uint64_t* ptr, const uint32_t* len, const uint64_t* off, uint64_t n, uint8_t* out,
                         hipStream_t st) {
  if (n) DR_LAUNCH(dev::k_gather_bytes, dim3(unsigned(std::min<uint64_t>((n + 256 / dev::GATHER_G - 1) / (256 / dev::GATHER_G), 1u << 16))), dim3(256), 0, st, ptr, len, off, n, out);
}

void launch_rebase_i64(const int64_t* src, uint64_t n, int64_t base, int64_t* dst, hipStream_t st) {
  if (n)
    DR_LAUNCH(dev::k_rebase_i64, dim3(unsigned(std::min<uint64_t>((n + 255) / 256, 1u << 16))), dim3(256), 0, st, src, n,
              base, dst);
}

static dim3 grid_stride(uint64_t n) { return dim3(unsigned(std::min<uint64_t>((n + 255) / 256, 1u << 16))); }
void launch_bits_mark(const uint32_t* list, uint64_t n, uint64_t nbits, uint32_t* bm, hipStream_t st) {
  if (n) DR_LAUNCH(dev::k_bits_mark, grid_stride(n), dim3(256), 0, st, list, n, nbits, bm);
}
void launch_bits_popc(const uint32_t* bm, uint64_t w, uint32_t* cnt, hipStream_t st) {
  if (w) DR_LAUNCH(dev::k_bits_popc, grid_stride(w), dim3(256), 0, st, bm, w, cnt);
}
void launch_bits_emit(const uint32_t* bm, uint64_t w, const uint64_t* off, uint32_t* out, hipStream_t st) {
  if (w) DR_LAUNCH(dev::k_bits_emit, grid_stride(w), dim3(256), 0, st, bm, w, off, out);
}

void launch_delts_fix(const uint8_t* flags, const int64_t* delts, uint64_t n, uint8_t* valid, int64_t* out,
                      hipStream_t st) {
  if (n) DR_LAUNCH(dev::k_delts_fix, dim3(unsigned((n + 255) / 256)), dim3(256), 0, st, flags, delts, n, valid, out);
}

void launch_scatter_fp(const uint64_t* rows, const uint64_t* bits, const uint8_t* nulls, uint64_t n, uint32_t* w32,
                       int64_t* w64, uint8_t* isnull, hipStream_t st) {
  if (n) DR_LAUNCH(dev::k_scatter_fp, dim3(unsigned((n + 255) / 256)), dim3(256), 0, st, rows, bits, nulls, n, w32, w64,
                   isnull);
}

void launch_readback(const ReadbackArgs& a, hipStream_t st) {
  DR_LAUNCH(dev::k_readback, dim3(1), dim3(256), 0, st, a);
}

void launch_append_actions(const AppendArgs& a, hipStream_t st) {
  const uint64_t n = std::max<uint64_t>(a.n, a.ctr ? a.nctr : 0);
  if (n) DR_LAUNCH(dev::k_append_actions, dim3(unsigned((n + 255) / 256)), dim3(256), 0, st, a);
}

}  // namespace dr
