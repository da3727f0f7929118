// Calibration of FETCH_SIZE for sparse and random 4-byte reads on gfx950
// (is k_tree's read traffic FETCH_SIZE or twice it?).
//
// Over an 8 GiB buffer (far past L2 and the Infinity Cache):
//   stride128  one 4-byte load per 128-byte line      (64 Mi loads)
//   stride64   one 4-byte load per 64-byte half line  (128 Mi loads)
//   stream     every 4-byte word once, 16 B per lane   (the guide's case)
//   random     64 Mi 4-byte loads at random words
// If DRAM moves 128-byte lines for sparse loads, stride128 and stride64 take
// the same time (both touch every line); if it moves 64-byte halves,
// stride128 takes half as long.  Run under rocprofv3 --pmc to see the
// TCC_EA0_RDREQ / FETCH_SIZE each kernel is charged.
//
//   hipcc -O3 --offload-arch=gfx950 scripts/calib_fetch.hip -o scripts/calib_fetch
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

__global__ void k_stride(const uint32_t *__restrict__ a, uint64_t n, uint32_t words,
                         uint32_t *__restrict__ out) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    acc += a[i * words];
  if (acc == 0x9E3779B9u) out[0] = acc;  // keeps the loads
}

__global__ void k_stream(const uint4 *__restrict__ a, uint64_t n, uint32_t *__restrict__ out) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9E3779B9u) out[0] = acc;
}

__global__ void k_random(const uint32_t *__restrict__ a, uint64_t words, uint64_t n,
                         uint32_t *__restrict__ out) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t h = (i + 1) * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 32;
    acc += a[h % words];
  }
  if (acc == 0x9E3779B9u) out[0] = acc;
}

int main() {
  const uint64_t bytes = 8ull << 30, words = bytes / 4;
  uint32_t *a, *out;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(a, 1, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const dim3 G(256 * 64), B(256);
  auto timed = [&](const char *name, double touched_gb, auto launch) {
    launch();  // warm-up
    CK(hipDeviceSynchronize());
    float best = 1e9f;
    for (int r = 0; r < 3; r++) {
      CK(hipEventRecord(e0));
      launch();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    printf("%-10s %8.3f ms  %6.2f GB of lines touched  %6.2f TB/s if every touched line moved\n",
           name, best, touched_gb, touched_gb / best);
  };
  const uint64_t n128 = bytes / 128, n64 = bytes / 64, nr = 64ull << 20;
  timed("stride128", bytes / 1e9, [&] { hipLaunchKernelGGL(k_stride, G, B, 0, 0, a, n128, 32u, out); });
  timed("stride64", bytes / 1e9, [&] { hipLaunchKernelGGL(k_stride, G, B, 0, 0, a, n64, 16u, out); });
  timed("stream", bytes / 1e9,
        [&] { hipLaunchKernelGGL(k_stream, G, B, 0, 0, (const uint4 *)a, bytes / 16, out); });
  timed("random", nr * 128 / 1e9, [&] { hipLaunchKernelGGL(k_random, G, B, 0, 0, a, words, nr, out); });
  CK(hipFree(a));
  CK(hipFree(out));
  return 0;
}
