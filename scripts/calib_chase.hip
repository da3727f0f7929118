// Calibration: dependent random reads (pointer chasing) on gfx950, the access
// pattern of the giant path's walk (k_walk) and ranking (k_lvl_walk).
//
// A table of M u64 words, word i = a hashed random index in [0, M).  Each lane
// runs C independent chains of S dependent steps (x = tab[x]); the chains of a
// lane interleave, so C loads are in flight a lane.  Reported: steps per
// second over all lanes, for table footprints from 1 to 16 GiB (TLB reach and
// the caches) and C = 1, 2, 4.
//
//   hipcc -O3 --offload-arch=gfx950 scripts/calib_chase.hip -o scripts/calib_chase
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

__global__ void k_init(uint64_t *tab, uint64_t m) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < m;
       i += (uint64_t)gridDim.x * blockDim.x)
    tab[i] = mix(i) % m;
}

template <int C>
__global__ __launch_bounds__(1024) void k_chase(const uint64_t *__restrict__ tab, uint64_t m,
                                                uint32_t steps, uint64_t *__restrict__ out) {
  const uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint64_t x[C];
#pragma unroll
  for (int c = 0; c < C; c++) x[c] = mix(g * C + c + 12345) % m;
  for (uint32_t s = 0; s < steps; s++) {
#pragma unroll
    for (int c = 0; c < C; c++) x[c] = tab[x[c]];
  }
  uint64_t acc = 0;
#pragma unroll
  for (int c = 0; c < C; c++) acc ^= x[c];
  if (acc == 0xFFFFFFFFFFFFFFFFull) out[0] = acc;  // keeps the loads alive
}

// one chain a lane plus a 4-byte record a step into the lane's own slot
// (consecutive words), stored WB words at a time: the walk's slot writes
template <int WB>
__global__ __launch_bounds__(1024) void k_chase_w(const uint64_t *__restrict__ tab, uint64_t m,
                                                  uint32_t steps, uint32_t *__restrict__ slots) {
  const uint64_t g = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint64_t x = mix(g + 12345) % m;
  uint32_t q[WB];
  uint32_t *sl = slots + g * steps;
  for (uint32_t s = 0; s < steps; s += WB) {
#pragma unroll
    for (int k = 0; k < WB; k++) {
      x = tab[x];
      q[k] = (uint32_t)x;
    }
#pragma unroll
    for (int k = 0; k < WB; k += 4)
      *reinterpret_cast<uint4 *>(sl + s + k) = make_uint4(q[k], q[k + 1], q[k + 2], q[k + 3]);
  }
}

template <int WB>
static double run_w(const uint64_t *tab, uint64_t m, uint32_t lanes, uint32_t steps, uint32_t *slots) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const uint32_t blocks = lanes / 1024;
  hipLaunchKernelGGL(k_chase_w<WB>, dim3(blocks), dim3(1024), 0, 0, tab, m, steps, slots);
  CK(hipEventRecord(a));
  hipLaunchKernelGGL(k_chase_w<WB>, dim3(blocks), dim3(1024), 0, 0, tab, m, steps, slots);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return (double)lanes * steps / (ms / 1e3);
}

template <int C>
static double run(const uint64_t *tab, uint64_t m, uint32_t lanes, uint32_t steps, uint64_t *out) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const uint32_t blocks = lanes / 1024;
  hipLaunchKernelGGL(k_chase<C>, dim3(blocks), dim3(1024), 0, 0, tab, m, steps, out);  // warm
  CK(hipEventRecord(a));
  hipLaunchKernelGGL(k_chase<C>, dim3(blocks), dim3(1024), 0, 0, tab, m, steps, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return (double)lanes * C * steps / (ms / 1e3);
}

int main() {
  const uint64_t mmax = 1ull << 33;  // 64 GiB of u64
  uint64_t *tab, *out;
  CK(hipMalloc(&tab, mmax * 8));
  CK(hipMalloc(&out, 64));
  uint32_t *slots;
  CK(hipMalloc(&slots, (1ull << 30) * 4));
  for (uint64_t m = 1ull << 27; m <= mmax; m <<= 1) {
    hipLaunchKernelGGL(k_init, dim3(16384), dim3(256), 0, 0, tab, m);
    CK(hipDeviceSynchronize());
    for (uint32_t lanes : {1u << 19, 1u << 21}) {
      const uint32_t steps = (uint32_t)((1ull << 30) / lanes);  // 1 Gi loads a run
      printf("{\"gib\": %.0f, \"lanes\": %u, \"c1\": %.3g, \"c2\": %.3g, \"c4\": %.3g}\n",
             m * 8.0 / (1 << 30), lanes, run<1>(tab, m, lanes, steps, out),
             run<2>(tab, m, lanes, steps / 2, out), run<4>(tab, m, lanes, steps / 4, out));
      printf("{\"gib\": %.0f, \"lanes\": %u, \"store16\": %.3g, \"store32\": %.3g, \"store64\": %.3g}\n",
             m * 8.0 / (1 << 30), lanes, run_w<4>(tab, m, lanes, steps, slots),
             run_w<8>(tab, m, lanes, steps, slots), run_w<16>(tab, m, lanes, steps, slots));
      fflush(stdout);
    }
  }
  CK(hipFree(tab));
  CK(hipFree(out));
  CK(hipFree(slots));
  return 0;
}
