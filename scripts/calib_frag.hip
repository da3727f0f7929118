// Calibration: does the physical layout of a table change the random-read
// rate?  The giant path's walk (k_walk) slows ~1.8x per node between 5.4e8 and
// 2e9 nodes while its L2 misses and HBM bytes stay linear and its UTCL1
// translation misses go from 36% to 61% of requests (profiles/r05_config5_*).
// calib_chase.hip saw no cliff up to 64 GiB -- on one fresh allocation.
//
//   mode 0 ("fresh"): the table is allocated on an empty device;
//   mode 1 ("frag"): the device is first filled with 2 MiB allocations, every
//   other one freed, so the table is made of 2 MiB pieces scattered over VRAM.
//
// Reported: dependent 8-byte loads per second (one chain a lane, 2 Mi lanes)
// over tables of 2 to 32 GiB.
//
//   hipcc -O3 --offload-arch=gfx950 scripts/calib_frag.hip -o scripts/calib_frag
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

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

__global__ void k_init(uint64_t *tab, uint64_t m) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < m;
       i += (uint64_t)gridDim.x * blockDim.x)
    tab[i] = mix(i) % m;
}

__global__ __launch_bounds__(1024) void k_chase(const uint64_t *__restrict__ tab, uint64_t m,
                                                uint32_t steps, uint64_t *__restrict__ out) {
  const uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint64_t x = mix(g + 12345) % m;
  for (uint32_t s = 0; s < steps; s++) x = tab[x];
  if (x == 0xFFFFFFFFFFFFFFFFull) out[0] = x;  // keeps the loads alive
}

static double run(const uint64_t *tab, uint64_t m, uint32_t lanes, uint32_t steps, uint64_t *out) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const uint32_t blocks = lanes / 1024;
  hipLaunchKernelGGL(k_chase, dim3(blocks), dim3(1024), 0, 0, tab, m, steps, out);  // warm
  CK(hipEventRecord(a));
  hipLaunchKernelGGL(k_chase, dim3(blocks), dim3(1024), 0, 0, tab, m, steps, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return (double)lanes * steps / (ms / 1e3);
}

int main(int argc, char **argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 0;
  const double fill_gib = argc > 2 ? atof(argv[2]) : 200.0;
  uint64_t *out;
  CK(hipMalloc(&out, 64));
  std::vector<void *> pieces;
  if (mode == 1) {
    const size_t piece = 2u << 20;
    const size_t n = (size_t)(fill_gib * (1u << 30) / piece);
    for (size_t i = 0; i < n; i++) {
      void *p = nullptr;
      if (hipMalloc(&p, piece) != hipSuccess) {
        (void)hipGetLastError();
        break;
      }
      pieces.push_back(p);
    }
    size_t freed = 0;
    for (size_t i = 0; i < pieces.size(); i += 2) {
      CK(hipFree(pieces[i]));
      pieces[i] = nullptr;
      freed++;
    }
    fprintf(stderr, "frag: %zu pieces of 2 MiB, %zu freed\n", pieces.size(), freed);
  }
  const uint32_t lanes = 1u << 21, steps = (uint32_t)((1ull << 30) / lanes);
  for (uint64_t gib : {2, 4, 8, 16, 32}) {
    if (mode == 1 && (double)gib > fill_gib / 2 - 1) break;
    const uint64_t m = (gib << 30) / 8;
    uint64_t *tab = nullptr;
    CK(hipMalloc(&tab, m * 8));
    hipLaunchKernelGGL(k_init, dim3(16384), dim3(256), 0, 0, tab, m);
    CK(hipDeviceSynchronize());
    printf("{\"mode\": \"%s\", \"gib\": %llu, \"lanes\": %u, \"loads_per_s\": %.3g}\n",
           mode ? "frag" : "fresh", (unsigned long long)gib, lanes, run(tab, m, lanes, steps, out));
    fflush(stdout);
    CK(hipFree(tab));
  }
  for (void *p : pieces)
    if (p) CK(hipFree(p));
  CK(hipFree(out));
  return 0;
}
