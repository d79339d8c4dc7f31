// Wave64 cross-lane primitives on DPP (gfx9 data-parallel primitives): a lane shift and inclusive
// scans built from row shifts within each 16-lane row plus three readlanes joining the rows. A
// __shfl_up is a ds_bpermute -- an LDS round trip per step -- so a six-step shuffle scan costs six
// LDS latencies; these cost four DPP ALU ops and three readlanes. Used by the small-segment JSON
// walker (k_json.hip: build_tape, tape_lines), where one wave works alone and every latency shows.
#pragma once
#include <cstdint>
#include <hip/hip_runtime.h>

namespace dr {
namespace wv {

// x of the lane `Ctrl` names; lanes whose source lies outside the row (or the wave) keep `old`
template <int Ctrl>
__device__ __forceinline__ uint32_t dpp(uint32_t old, uint32_t x) {
  return uint32_t(__builtin_amdgcn_update_dpp(int(old), int(x), Ctrl, 0xF, 0xF, false));
}

constexpr int DPP_ROW_SHR = 0x110;   // + n: row_shr:n
constexpr int DPP_WAVE_SHR1 = 0x138;
constexpr int DPP_WAVE_SHL1 = 0x130;

// x of lane - 1; lane 0 gets `in`
__device__ __forceinline__ uint32_t shr1(uint32_t x, uint32_t in) { return dpp<DPP_WAVE_SHR1>(in, x); }
// x of lane + 1; lane 63 gets `in`
__device__ __forceinline__ uint32_t shl1(uint32_t x, uint32_t in) { return dpp<DPP_WAVE_SHL1>(in, x); }

__device__ __forceinline__ uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// Inclusive scan over the wave's lanes in lane order: op(earlier, later) must be associative with
// identity `id`.
template <class Op>
__device__ __forceinline__ uint32_t scan_incl(uint32_t x, uint32_t id, Op op) {
  x = op(dpp<DPP_ROW_SHR + 1>(id, x), x);
  x = op(dpp<DPP_ROW_SHR + 2>(id, x), x);
  x = op(dpp<DPP_ROW_SHR + 4>(id, x), x);
  x = op(dpp<DPP_ROW_SHR + 8>(id, x), x);
  const uint32_t r0 = uint32_t(__builtin_amdgcn_readlane(int(x), 15));
  const uint32_t r1 = uint32_t(__builtin_amdgcn_readlane(int(x), 31));
  const uint32_t r2 = uint32_t(__builtin_amdgcn_readlane(int(x), 47));
  const uint32_t p2 = op(r0, r1), p3 = op(p2, r2);
  const uint32_t row = lane_id() >> 4;
  const uint32_t pre = (row & 2u) ? ((row & 1u) ? p3 : p2) : ((row & 1u) ? r0 : id);
  return op(pre, x);
}

__device__ __forceinline__ uint32_t last_uniform(uint32_t x) { return uint32_t(__builtin_amdgcn_readlane(int(x), 63)); }

}  // namespace wv
}  // namespace dr
