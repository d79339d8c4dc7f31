// Calibration of rocprofv3's FETCH_SIZE for this repo's access patterns (MI355X_MICROARCH.md: the x2
// correction is established only for 16 B/lane coalesced streaming reads; other widths are
// uncalibrated). Each kernel reads a known number of distinct HBM bytes exactly once, from a buffer
// far larger than the 256 MiB Infinity Cache, with at most one wave per CU so that a line fetched
// once stays in L1/L2 until every lane that needs it has read it:
//   stream16  16 B per lane, coalesced (the guide's reference pattern)
//   lines     K1's pattern (k_json_lines): lane l walks its own ~300-byte line in 32-byte window pairs
//   gather    k_bucket_verify's pattern: whole records in random order, eight lanes per record (one
//             16-byte block each); records are single 128-byte lines so each line is fetched once
// Known bytes / FETCH_SIZE per dispatch = the correction factor for that pattern (bench.py applies it).
// Build: hipcc --offload-arch=gfx950 -O3 -o build/fetch_calib scripts/fetch_calib.hip
// Run:   rocprofv3 --pmc FETCH_SIZE --kernel-trace -d <dir> -o calib --output-format csv -- build/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                   \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

__global__ void __launch_bounds__(256) stream16(const uint4* __restrict__ in, uint64_t n16, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint4 v = in[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// 64 lines of LINE bytes per wave-step, lane l walks line l in 32-byte pairs of 16-byte loads.
constexpr uint32_t LINE = 320;
__global__ void __launch_bounds__(64) lines(const uint8_t* __restrict__ in, uint64_t nlines, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t l0 = uint64_t(blockIdx.x) * 64; l0 < nlines; l0 += uint64_t(gridDim.x) * 64) {
    const uint64_t l = l0 + threadIdx.x;
    if (l >= nlines) break;
    const uint4* q = reinterpret_cast<const uint4*>(in + l * LINE);
    for (uint32_t j = 0; j < LINE / 16; j += 2) {
      const uint4 a = q[j], b = q[j + 1];
      acc ^= a.x ^ a.y ^ b.z ^ b.w;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// records of 128 bytes (8 blocks) read in the order perm[], 8 lanes per record
constexpr uint32_t REC = 128;
__global__ void __launch_bounds__(256) gather(const uint8_t* __restrict__ in, const uint32_t* __restrict__ perm,
                                              uint64_t nrec, uint32_t* out) {
  uint32_t acc = 0;
  const uint32_t j = threadIdx.x & 7;
  for (uint64_t k = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) / 8; k < nrec;
       k += uint64_t(gridDim.x) * blockDim.x / 8) {
    const uint4 v = reinterpret_cast<const uint4*>(in + uint64_t(perm[k]) * REC)[j];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const uint64_t bytes = uint64_t(2) << 30;  // 2 GiB: 8x the Infinity Cache
  uint8_t* buf;
  uint32_t *out, *perm;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&out, 4));
  CK(hipMemset(buf, 1, bytes));
  const uint64_t nrec = bytes / REC;
  std::vector<uint32_t> h(nrec);
  for (uint64_t i = 0; i < nrec; ++i) h[i] = uint32_t(i);
  srand(7);
  for (uint64_t i = nrec - 1; i > 0; --i) std::swap(h[i], h[uint64_t(rand()) % (i + 1)]);
  CK(hipMalloc(&perm, nrec * 4));
  CK(hipMemcpy(perm, h.data(), nrec * 4, hipMemcpyHostToDevice));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(stream16, dim3(cus * 8), dim3(256), 0, 0, reinterpret_cast<const uint4*>(buf), bytes / 16, out);
    hipLaunchKernelGGL(lines, dim3(cus), dim3(64), 0, 0, buf, bytes / LINE, out);
    hipLaunchKernelGGL(gather, dim3(cus), dim3(256), 0, 0, buf, perm, nrec, out);
    CK(hipDeviceSynchronize());
  }
  std::printf("{\"bytes_stream16\": %llu, \"bytes_lines\": %llu, \"bytes_gather\": %llu, \"perm_bytes\": %llu}\n",
              (unsigned long long)(bytes / 16 * 16), (unsigned long long)(bytes / LINE * LINE),
              (unsigned long long)(nrec * REC), (unsigned long long)(nrec * 4));
  return 0;
}
