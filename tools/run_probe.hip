// Run-length probe (not part of libsort): how the write side of a digit pass
// depends on the length of its digit runs.  Compute-free skeleton of the tile
// pass: tile t (T keys, wave-striped loads like k_tile_pass) is staged through
// LDS and written as R runs of T/R keys, run r to region r of the output
// (regions of n/R keys, so tile t's run r follows tile t-1's run r exactly as
// in a pass over uniform digits).  Tiles are XCD-contiguous (xcd_tile_of_block).
// Also a pair form: u64 keys + u32 values, both through LDS.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/run_probe tools/run_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__device__ __forceinline__ uint32_t xcd_tile() {
  const uint32_t g = gridDim.x, q = g >> 3, r = g & 7u, x = blockIdx.x & 7u, i = blockIdx.x >> 3;
  return x * q + min(x, r) + i;
}

// B threads, T = B * I keys per tile, R runs
template <int B, int I, int R, typename K>
__global__ __launch_bounds__(B) void runs_keys(const K* __restrict__ in, K* __restrict__ out, size_t n) {
  constexpr int T = B * I, RUN = T / R;
  __shared__ K s[T];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const uint32_t t = xcd_tile();
  const size_t base = (size_t)t * T;
  K v[I];
#pragma unroll
  for (int i = 0; i < I; ++i) v[i] = __builtin_nontemporal_load(&in[base + w * (64 * I) + i * 64 + l]);
#pragma unroll
  for (int i = 0; i < I; ++i) s[T - 1 - (w * (64 * I) + i * 64 + l)] = v[i];
  __syncthreads();
  const size_t region = n / R;
#pragma unroll
  for (int i = 0; i < I; ++i) {
    const int p = i * B + threadIdx.x;
    const int r = p / RUN, q = p % RUN;
    out[r * region + (size_t)t * RUN + q] = s[p];
  }
}

template <int B, int I, int R>
__global__ __launch_bounds__(B) void runs_pairs(const uint64_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                uint64_t* __restrict__ kout, uint32_t* __restrict__ vout, size_t n) {
  constexpr int T = B * I, RUN = T / R;
  __shared__ uint64_t sk[T];
  __shared__ uint32_t sv[T];
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const uint32_t t = xcd_tile();
  const size_t base = (size_t)t * T;
  uint64_t k[I];
  uint32_t v[I];
#pragma unroll
  for (int i = 0; i < I; ++i) {
    k[i] = __builtin_nontemporal_load(&kin[base + w * (64 * I) + i * 64 + l]);
    v[i] = __builtin_nontemporal_load(&vin[base + w * (64 * I) + i * 64 + l]);
  }
#pragma unroll
  for (int i = 0; i < I; ++i) {
    sk[T - 1 - (w * (64 * I) + i * 64 + l)] = k[i];
    sv[T - 1 - (w * (64 * I) + i * 64 + l)] = v[i];
  }
  __syncthreads();
  const size_t region = n / R;
#pragma unroll
  for (int i = 0; i < I; ++i) {
    const int p = i * B + threadIdx.x;
    const int r = p / RUN, q = p % RUN;
    kout[r * region + (size_t)t * RUN + q] = sk[p];
    vout[r * region + (size_t)t * RUN + q] = sv[p];
  }
}

template <typename F>
double time_it(F f) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<float> t;
  for (int it = 0; it < 23; ++it) {
    CK(hipEventRecord(e0));
    f();
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    if (it >= 3) t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2] * 1e3;
}

int main(int argc, char** argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 28;
  const size_t n = (size_t)1 << lg;
  uint64_t *a, *b;
  CK(hipMalloc(&a, n * 8)); CK(hipMalloc(&b, n * 8));
  uint32_t *va, *vb;
  CK(hipMalloc(&va, n * 4)); CK(hipMalloc(&vb, n * 4));
  CK(hipMemset(a, 1, n * 8)); CK(hipMemset(va, 2, n * 4));
  uint32_t* a32 = (uint32_t*)a;
  uint32_t* b32 = (uint32_t*)b;
#define K32(B, I, R)                                                                                            \
  {                                                                                                             \
    double us = time_it([&] { hipLaunchKernelGGL((runs_keys<B, I, R, uint32_t>), dim3(n / (B * I)), dim3(B), 0, 0, \
                                                 a32, b32, n); });                                              \
    printf("u32 keys  tile %5d (%4d x %2d) runs %3d (%3d keys = %4d B): %7.1f us  %5.0f GB/s\n", B * I, B, I, R, \
           B * I / R, B * I / R * 4, us, 8.0 * n / us / 1e3);                                                   \
  }
#define K64(B, I, R)                                                                                            \
  {                                                                                                             \
    double us = time_it([&] { hipLaunchKernelGGL((runs_keys<B, I, R, uint64_t>), dim3(n / (B * I)), dim3(B), 0, 0, \
                                                 a, b, n); });                                                  \
    printf("u64 keys  tile %5d (%4d x %2d) runs %3d (%3d keys = %4d B): %7.1f us  %5.0f GB/s\n", B * I, B, I, R, \
           B * I / R, B * I / R * 8, us, 16.0 * n / us / 1e3);                                                  \
  }
#define PR(B, I, R)                                                                                             \
  {                                                                                                             \
    double us = time_it([&] { hipLaunchKernelGGL((runs_pairs<B, I, R>), dim3(n / (B * I)), dim3(B), 0, 0, a, va, b, \
                                                 vb, n); });                                                    \
    printf("u64+u32   tile %5d (%4d x %2d) runs %3d (%3d pairs):           %7.1f us  %5.0f GB/s\n", B * I, B, I, \
           R, B * I / R, us, 24.0 * n / us / 1e3);                                                              \
  }
  // u32 keys (n keys): copy-like (1 run), 16 runs, 256 runs at growing tiles
  K32(256, 16, 1) K32(256, 16, 16) K32(256, 16, 256) K32(512, 16, 256) K32(1024, 16, 256) K32(512, 32, 256)
  K32(1024, 8, 256) K32(256, 32, 256)
  // u64 keys
  K64(512, 8, 1) K64(512, 8, 256) K64(1024, 8, 256) K64(512, 16, 256)
  // (u64, u32) pairs
  PR(512, 8, 1) PR(512, 8, 16) PR(512, 8, 256) PR(1024, 8, 256) PR(512, 16, 256) PR(256, 16, 256)
  return 0;
}
