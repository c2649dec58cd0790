// HBM ceiling probe (not part of libsort): which access shape a sort pass can
// hope to reach on this box.  All kernels move the same 2^lg uint32 buffer.
//  copy16_gs     grid-stride 16-B copy, 8 blocks/CU (the original calibration)
//  copy16_u4     one-shot, 4 x 16 B per thread in flight, 16 KiB per block
//  copy16_u4_nt  same, nontemporal stores
//  copy4_tile    the tile pass's load shape: 16 x 4 B per lane, wave-striped
//  tile_lds      copy4_tile staged through LDS with a barrier (pass skeleton)
//  read16_u4     read-only stream (sum), one store per block
//  write16_u4    write-only stream
//  scatter*      pass write skeleton: 16 or 256 runs per tile, aligned or
//                misaligned run starts, round-robin or XCD-contiguous tiles
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bw_probe tools/bw_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__global__ void copy16_gs(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n4) {
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) out[i] = in[i];
}

template <bool NT>
__global__ __launch_bounds__(256) void copy16_u4(const uint4* __restrict__ in, uint4* __restrict__ out) {
  size_t base = (size_t)blockIdx.x * 1024 + threadIdx.x;
  uint4 v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = in[base + k * 256];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    if (NT) {
      __builtin_nontemporal_store(v[k].x, &out[base + k * 256].x);
      __builtin_nontemporal_store(v[k].y, &out[base + k * 256].y);
      __builtin_nontemporal_store(v[k].z, &out[base + k * 256].z);
      __builtin_nontemporal_store(v[k].w, &out[base + k * 256].w);
    } else {
      out[base + k * 256] = v[k];
    }
  }
}

// 4096-key tile: wave w owns keys [w*1024, (w+1)*1024), lane l item i at w*1024 + i*64 + l
__global__ __launch_bounds__(256) void copy4_tile(const uint32_t* __restrict__ in, uint32_t* __restrict__ out) {
  int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  size_t base = (size_t)blockIdx.x * 4096 + w * 1024 + l;
  uint32_t v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = in[base + i * 64];
#pragma unroll
  for (int i = 0; i < 16; ++i) out[base + i * 64] = v[i];
}

__global__ __launch_bounds__(256) void tile_lds(const uint32_t* __restrict__ in, uint32_t* __restrict__ out) {
  __shared__ uint32_t s[4096];
  int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  size_t base = (size_t)blockIdx.x * 4096;
  uint32_t v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = in[base + w * 1024 + i * 64 + l];
  // reversed placement so the compiler cannot fold the round trip
#pragma unroll
  for (int i = 0; i < 16; ++i) s[4095 - (w * 1024 + i * 64 + l)] = v[i];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 16; ++i) out[base + i * 256 + threadIdx.x] = s[i * 256 + threadIdx.x];
}

__global__ __launch_bounds__(256) void read16_u4(const uint4* __restrict__ in, uint32_t* __restrict__ sink) {
  size_t base = (size_t)blockIdx.x * 1024 + threadIdx.x;
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint4 v = in[base + k * 256];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9e3779b9u) sink[blockIdx.x] = acc;  // practically never: keeps the loads alive
}

__global__ __launch_bounds__(256) void write16_u4(uint4* __restrict__ out, uint32_t seed) {
  size_t base = (size_t)blockIdx.x * 1024 + threadIdx.x;
#pragma unroll
  for (int k = 0; k < 4; ++k) out[base + k * 256] = make_uint4(seed, (uint32_t)base, k, seed ^ k);
}


// Scatter skeleton of a digit pass without the ranking: tile t (4096 keys,
// read like copy4_tile) writes R runs of 4096/R keys, run r to region r of
// the output (region stride n/R + MIS words, so runs start misaligned when
// MIS != 0).  The LDS stage of tile_lds is kept.
// XCD=true: block b handles tile (b % 8) * (T / 8) + b / 8, so each XCD
// (blocks are dealt round-robin over the 8 XCDs) walks one contiguous range
// and the lines shared by neighbouring tiles' runs meet in one L2.
template <int R, int MIS, bool XCD = false>
__global__ __launch_bounds__(256) void scatter_runs(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                    size_t n) {
  __shared__ uint32_t s[4096];
  constexpr int RUN = 4096 / R;
  int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const uint32_t t = XCD ? (blockIdx.x % 8) * (gridDim.x / 8) + blockIdx.x / 8 : blockIdx.x;
  size_t base = (size_t)t * 4096;
  uint32_t v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = in[base + w * 1024 + i * 64 + l];
#pragma unroll
  for (int i = 0; i < 16; ++i) s[4095 - (w * 1024 + i * 64 + l)] = v[i];
  __syncthreads();
  const size_t region = n / R + MIS;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int p = i * 256 + threadIdx.x;
    const int r = p / RUN, q = p % RUN;
    out[r * region + (size_t)t * RUN + q] = s[p];
  }
}

// scatter_runs<16, MIS> with line-aligned stores: each run (RUN keys, global
// start misaligned by MIS words) is padded in front to a 32-key line
// boundary in a virtual index space; each wave store covers whole lines.
template <int MIS, bool XCD>
__global__ __launch_bounds__(256) void scatter16_alst(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                      size_t n) {
  __shared__ uint32_t s[4096];
  constexpr int R = 16, RUN = 256;
  constexpr int PAD = (MIS % 32);
  constexpr int VRUN = (PAD + RUN + 31) / 32 * 32;
  constexpr int VTOT = VRUN * R;
  int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const uint32_t t = XCD ? (blockIdx.x % 8) * (gridDim.x / 8) + blockIdx.x / 8 : blockIdx.x;
  size_t base = (size_t)t * 4096;
  uint32_t v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = in[base + w * 1024 + i * 64 + l];
#pragma unroll
  for (int i = 0; i < 16; ++i) s[4095 - (w * 1024 + i * 64 + l)] = v[i];
  __syncthreads();
  const size_t region = n / R + MIS;
#pragma unroll
  for (int i = 0; i < (VTOT + 255) / 256; ++i) {
    const int vi = i * 256 + threadIdx.x;
    const int r = vi / VRUN, q = vi % VRUN - PAD;
    if (vi < VTOT && q >= 0 && q < RUN) out[r * region + (size_t)t * RUN + q] = s[r * RUN + q];
  }
}

__global__ __launch_bounds__(256) void copy4_tile_mis(const uint32_t* __restrict__ in, uint32_t* __restrict__ out) {
  int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  size_t base = (size_t)blockIdx.x * 4096 + w * 1024 + l;
  uint32_t v[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) v[i] = in[base + i * 64];
#pragma unroll
  for (int i = 0; i < 16; ++i) out[base + i * 64 + 7] = v[i];
}

__global__ void fill_keys(uint32_t* k, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) { uint64_t x = (i + 1) * 0x9E3779B97F4A7C15ull; x ^= x >> 29; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 32; k[i] = (uint32_t)x; }
}

int main(int argc, char** argv) {
  int lg = argc > 1 ? atoi(argv[1]) : 28;
  size_t n = (size_t)1 << lg;  // must be a multiple of 4096
  uint32_t *a, *b, *sink;
  CK(hipMalloc(&a, n * 4)); CK(hipMalloc(&b, n * 4 + 4096 * 64)); CK(hipMalloc(&sink, n / 1024 * 4));
  hipLaunchKernelGGL(fill_keys, dim3((n + 255) / 256), dim3(256), 0, 0, a, n);
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const int kIters = 20;
  const char* names[] = {"copy16_gs", "copy16_u4", "copy16_u4_nt", "copy4_tile", "tile_lds", "read16_u4", "write16_u4",
                         "scatter16_al", "scatter16_mis", "scatter256_al", "scatter256_mis", "scat16_mis_xcd",
                         "scat256_mis_xcd", "scat16_al_xcd", "scat256_al_xcd", "copy4_tile_mis", "scat16_mis_alst",
                         "scat16_mis_alst_xcd"};
  const double bytes[] = {8.0 * n, 8.0 * n, 8.0 * n, 8.0 * n, 8.0 * n, 4.0 * n, 4.0 * n, 8.0 * n,
                          8.0 * n, 8.0 * n, 8.0 * n, 8.0 * n, 8.0 * n, 8.0 * n, 8.0 * n, 8.0 * n, 8.0 * n, 8.0 * n};
  const int first = argc > 2 ? atoi(argv[2]) : 0;
  for (int v = first; v < 18; ++v) {
    std::vector<float> t;
    for (int it = 0; it < kIters + 3; ++it) {
      CK(hipEventRecord(e0));
      switch (v) {
        case 0: hipLaunchKernelGGL(copy16_gs, dim3(256 * 8), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, n / 4); break;
        case 1: hipLaunchKernelGGL(copy16_u4<false>, dim3(n / 4096), dim3(256), 0, 0, (const uint4*)a, (uint4*)b); break;
        case 2: hipLaunchKernelGGL(copy16_u4<true>, dim3(n / 4096), dim3(256), 0, 0, (const uint4*)a, (uint4*)b); break;
        case 3: hipLaunchKernelGGL(copy4_tile, dim3(n / 4096), dim3(256), 0, 0, a, b); break;
        case 4: hipLaunchKernelGGL(tile_lds, dim3(n / 4096), dim3(256), 0, 0, a, b); break;
        case 5: hipLaunchKernelGGL(read16_u4, dim3(n / 4096), dim3(256), 0, 0, (const uint4*)a, sink); break;
        case 6: hipLaunchKernelGGL(write16_u4, dim3(n / 4096), dim3(256), 0, 0, (uint4*)b, (uint32_t)it); break;
        case 7: hipLaunchKernelGGL((scatter_runs<16, 0>), dim3(n / 4096), dim3(256), 0, 0, a, b, n); break;
        case 8: hipLaunchKernelGGL((scatter_runs<16, 7>), dim3(n / 4096), dim3(256), 0, 0, a, b, n); break;
        case 9: hipLaunchKernelGGL((scatter_runs<256, 0>), dim3(n / 4096), dim3(256), 0, 0, a, b, n); break;
        case 10: hipLaunchKernelGGL((scatter_runs<256, 7>), dim3(n / 4096), dim3(256), 0, 0, a, b, n); break;
        case 11: hipLaunchKernelGGL((scatter_runs<16, 7, true>), dim3(n / 4096), dim3(256), 0, 0, a, b, n); break;
        case 12: hipLaunchKernelGGL((scatter_runs<256, 7, true>), dim3(n / 4096), dim3(256), 0, 0, a, b, n); break;
        case 13: hipLaunchKernelGGL((scatter_runs<16, 0, true>), dim3(n / 4096), dim3(256), 0, 0, a, b, n); break;
        case 14: hipLaunchKernelGGL((scatter_runs<256, 0, true>), dim3(n / 4096), dim3(256), 0, 0, a, b, n); break;
        case 15: hipLaunchKernelGGL(copy4_tile_mis, dim3(n / 4096), dim3(256), 0, 0, a, b); break;
        case 16: hipLaunchKernelGGL((scatter16_alst<7, false>), dim3(n / 4096), dim3(256), 0, 0, a, b, n); break;
        case 17: hipLaunchKernelGGL((scatter16_alst<7, true>), dim3(n / 4096), dim3(256), 0, 0, a, b, n); break;
      }
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (it >= 3) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    float med = t[t.size() / 2];
    printf("%-13s 2^%d u32: median %.1f us = %.0f GB/s (best %.1f us = %.0f GB/s)\n", names[v], lg, med * 1e3,
           bytes[v] / (med * 1e-3) / 1e9, t[0] * 1e3, bytes[v] / (t[0] * 1e-3) / 1e9);
  }
  return 0;
}
