// Calibration: scattered writes on gfx950 -- the radix sort's digit-run
// scatter and the list kernels' record stores.  Every lane writes one piece of
// P bytes (P/4 consecutive words, P-aligned) at a random P-aligned offset of a
// 16 GiB buffer; reported: GB/s of pieces written, for P = 4 .. 128, and the
// coalesced stream for comparison.  A piece smaller than the DRAM burst costs
// a read-modify-write if the memory side does not merge neighbours.
//
//   hipcc -O3 --offload-arch=gfx950 scripts/calib_scatter.hip -o scripts/calib_scatter
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// W words a piece; pieces = number of pieces; buffer of m words
template <int W>
__global__ void k_scatter(uint32_t *__restrict__ buf, uint64_t m, uint64_t pieces, uint64_t seed) {
  const uint64_t slots = m / W;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < pieces;
       i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t *p = buf + (mix(i ^ seed) % slots) * W;
    if (W == 1) {
      p[0] = (uint32_t)i;
    } else if (W == 2) {
      *reinterpret_cast<uint2 *>(p) = make_uint2((uint32_t)i, 1u);
    } else {
#pragma unroll
      for (int k = 0; k < W; k += 4)
        *reinterpret_cast<uint4 *>(p + k) = make_uint4((uint32_t)i, 1u, 2u, 3u);
    }
  }
}

__global__ void k_stream(uint32_t *__restrict__ buf, uint64_t words) {
  for (uint64_t i = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) * 4; i < words;
       i += (uint64_t)gridDim.x * blockDim.x * 4)
    *reinterpret_cast<uint4 *>(buf + i) = make_uint4(1u, 2u, 3u, 4u);
}

template <int W>
static double run(uint32_t *buf, uint64_t m) {
  const uint64_t bytes = 4ull << 30, pieces = bytes / (4 * W);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(k_scatter<W>, dim3(8192), dim3(256), 0, 0, buf, m, pieces, 1ull);
  CK(hipEventRecord(a));
  hipLaunchKernelGGL(k_scatter<W>, dim3(8192), dim3(256), 0, 0, buf, m, pieces, 2ull);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return bytes / (ms / 1e3) / 1e9;
}

int main() {
  const uint64_t m = 4ull << 30;  // 16 GiB of words
  uint32_t *buf;
  CK(hipMalloc(&buf, m * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  hipLaunchKernelGGL(k_stream, dim3(8192), dim3(256), 0, 0, buf, m);
  CK(hipEventRecord(a));
  hipLaunchKernelGGL(k_stream, dim3(8192), dim3(256), 0, 0, buf, m);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  printf("{\"stream_gbs\": %.0f}\n", m * 4.0 / (ms / 1e3) / 1e9);
  printf("{\"piece_bytes\": 4, \"gbs\": %.0f}\n", run<1>(buf, m));
  printf("{\"piece_bytes\": 8, \"gbs\": %.0f}\n", run<2>(buf, m));
  printf("{\"piece_bytes\": 16, \"gbs\": %.0f}\n", run<4>(buf, m));
  printf("{\"piece_bytes\": 32, \"gbs\": %.0f}\n", run<8>(buf, m));
  printf("{\"piece_bytes\": 64, \"gbs\": %.0f}\n", run<16>(buf, m));
  printf("{\"piece_bytes\": 128, \"gbs\": %.0f}\n", run<32>(buf, m));
  CK(hipFree(buf));
  return 0;
}
