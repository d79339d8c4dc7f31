// Small gather kernels used to move result subsets to the host in one transfer each.
#include "dev_common.h"
#include "kernels.h"

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

// out[off[i] .. off[i] + len[i]) = bytes at ptr[i]; one wave per string.
__global__ void k_gather_bytes(const uint64_t* __restrict__ ptr, const uint32_t* __restrict__ len,
                               const uint64_t* __restrict__ off, uint64_t n, uint8_t* __restrict__ out) {
  const uint64_t s = uint64_t(blockIdx.x) * (blockDim.x / 64) + (threadIdx.x >> 6);
  if (s >= n) return;
  const uint8_t* p = reinterpret_cast<const uint8_t*>(ptr[s]);
  uint8_t* o = out + off[s];
  for (uint32_t k = threadIdx.x & 63; k < len[s]; k += 64) o[k] = p[k];
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
  if (n) DR_LAUNCH(dev::k_gather_bytes, dim3(unsigned((n + 3) / 4)), dim3(256), 0, st, ptr, len, off, n, out);
}

}  // namespace dr
