// Calibration / ceiling tool (not part of libsort):
//  * copy kernels with 4-byte and 16-byte accesses over a buffer of known size:
//    the HBM copy bandwidth on this box, and the FETCH_SIZE / WRITE_SIZE
//    calibration for the access widths the sort kernels use;
//  * rocPRIM's radix_sort_keys on the same 2^k uint32 PCG-like keys, as a
//    known-good reference sort on the same hardware (timing only).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/calib_copy tools/calib_copy.hip
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/device/device_radix_sort.hpp>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void copy_kernel_b4(const uint32_t* __restrict__ in, uint32_t* __restrict__ out, size_t n) {
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = in[i];
}
__global__ void copy_kernel_b16(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n4) {
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) out[i] = in[i];
}
__global__ void fill_keys(uint32_t* k, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { uint64_t x = (i + 1) * 0x9E3779B97F4A7C15ull; x ^= x >> 29; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 32; k[i] = (uint32_t)x; }
}

int main(int argc, char** argv) {
  int lg = argc > 1 ? atoi(argv[1]) : 28;
  size_t n = (size_t)1 << lg;
  uint32_t *a, *b, *c;
  CK(hipMalloc(&a, n * 4)); CK(hipMalloc(&b, n * 4)); CK(hipMalloc(&c, n * 4));
  hipLaunchKernelGGL(fill_keys, dim3((n + 255) / 256), dim3(256), 0, 0, a, n);
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int grid = 256 * 8;
  float ms;
  for (int w = 0; w < 2; ++w) {
    for (int it = 0; it < 3; ++it) {
      CK(hipEventRecord(e0));
      if (w == 0) hipLaunchKernelGGL(copy_kernel_b4, dim3(grid), dim3(256), 0, 0, a, b, n);
      else hipLaunchKernelGGL(copy_kernel_b16, dim3(grid), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, n / 4);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
      if (it == 2) printf("copy_%s: %zu bytes moved in %.3f ms = %.1f GB/s\n", w ? "b16" : "b4", 2 * n * 4, ms,
                          2.0 * n * 4 / (ms * 1e-3) / 1e9);
    }
  }
  // rocPRIM reference sort (keys only, all 32 bits)
  size_t tmp_bytes = 0;
  CK(rocprim::radix_sort_keys(nullptr, tmp_bytes, a, c, n));
  void* tmp; CK(hipMalloc(&tmp, tmp_bytes));
  for (int it = 0; it < 6; ++it) {
    CK(hipEventRecord(e0));
    CK(rocprim::radix_sort_keys(tmp, tmp_bytes, a, c, n));
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1)); CK(hipEventElapsedTime(&ms, e0, e1));
    if (it >= 3) printf("rocprim::radix_sort_keys 2^%d u32: %.3f ms = %.2f Gkeys/s\n", lg, ms, n / (ms * 1e-3) / 1e9);
  }
  std::vector<uint32_t> h(n);
  CK(hipMemcpy(h.data(), c, n * 4, hipMemcpyDeviceToHost));
  for (size_t i = 1; i < n; ++i) if (h[i] < h[i - 1]) { printf("rocprim result unsorted at %zu\n", i); return 1; }
  printf("ok\n");
  return 0;
}
