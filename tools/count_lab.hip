// Count-kernel lab (not part of libsort): per-tile digit histograms of 2^lg
// PCG keys (the tile path's count read), library kernel vs LDS layouts.
// Every variant is checked against the library kernel's counts.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/count_lab tools/count_lab.hip
#include "../gpu-radix-sort_amd/csrc/radix_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

namespace lsort {
int timing_start(const char*, hipStream_t, uint64_t) { return -1; }
void timing_stop(int, hipStream_t) {}
int get_algorithm() { return 3; }
int get_hybrid_mode() { return 0; }
int get_bucket_mode() { return 1; }
}  // namespace lsort

using namespace lsort;

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// COPIES copies of the histogram, interleaved (entry d of copy c at d*COPIES + c)
// so copies of one digit sit in neighbouring banks; lane l uses copy l % COPIES.
// PERWAVE: one histogram per wave (padded row), copy = wave.
template <int BITS, int BLOCK, int COPIES, bool PERWAVE>
__global__ __launch_bounds__(BLOCK) void k_counts_x(const uint32_t* __restrict__ keys, RadixDigit op,
                                                    uint32_t* __restrict__ counts) {
  constexpr int RADIX = 1 << BITS;
  constexpr int TILE = BLOCK * 16;
  constexpr int WAVES = BLOCK / 64;
  constexpr int ROW = RADIX + 1;
  constexpr int WORDS = PERWAVE ? WAVES * ROW : RADIX * COPIES;
  __shared__ uint32_t s_h[WORDS];
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < WORDS; i += BLOCK) s_h[i] = 0u;
  __syncthreads();
  const uint4* vp = reinterpret_cast<const uint4*>(keys + (uint64_t)blockIdx.x * TILE);
  uint4 v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = vp[j * BLOCK + tid];
  const uint32_t c = PERWAVE ? (tid / 64) * ROW : tid % COPIES;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t d = op(vec_elem(v[j], q));
      atomicAdd(&s_h[PERWAVE ? c + d : d * COPIES + c], 1u);
    }
  __syncthreads();
  for (uint32_t d = tid; d < RADIX; d += BLOCK) {
    uint32_t s = 0;
    if constexpr (PERWAVE) {
#pragma unroll
      for (int w = 0; w < WAVES; ++w) s += s_h[w * ROW + d];
    } else {
#pragma unroll
      for (int k = 0; k < COPIES; ++k) s += s_h[d * COPIES + k];
    }
    counts[(size_t)blockIdx.x * RADIX + d] = s;
  }
}

// Wave-aggregated: the lanes of one item with equal digits (ballot match)
// add their count once, from the group's first lane (no same-address lanes
// inside an LDS atomic).
template <int BITS, int BLOCK>
__global__ __launch_bounds__(BLOCK) void k_counts_match(const uint32_t* __restrict__ keys, RadixDigit op,
                                                        uint32_t* __restrict__ counts) {
  constexpr int RADIX = 1 << BITS;
  constexpr int TILE = BLOCK * 16;
  __shared__ uint32_t s_h[RADIX];
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < RADIX; i += BLOCK) s_h[i] = 0u;
  __syncthreads();
  const uint32_t* kp = keys + (uint64_t)blockIdx.x * TILE + (tid / 64) * 1024 + (tid & 63);
  uint32_t k[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) k[j] = kp[j * 64];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t d = op(k[j]);
    uint32_t lo = 0u, hi = 0u;
#pragma unroll
    for (int bit = 0; bit < BITS - 1; ++bit) {
      const uint32_t X = (uint32_t)__builtin_amdgcn_sbfe(d, bit, 1);
      const uint64_t m = ballot_nz(X);
      lo = __builtin_amdgcn_bitop3_b32(X, lo, (uint32_t)m, 0xDE);
      hi = __builtin_amdgcn_bitop3_b32(X, hi, (uint32_t)(m >> 32), 0xDE);
    }
    const uint32_t X = (uint32_t)__builtin_amdgcn_sbfe(d, BITS - 1, 1);
    const uint64_t m = ballot_nz(X);
    const uint32_t plo = __builtin_amdgcn_bitop3_b32(X, lo, (uint32_t)m, 0x21);
    const uint32_t phi = __builtin_amdgcn_bitop3_b32(X, hi, (uint32_t)(m >> 32), 0x21);
    const uint32_t below = __builtin_amdgcn_mbcnt_hi(phi, __builtin_amdgcn_mbcnt_lo(plo, 0u));
    if (below == 0) atomicAdd(&s_h[d], (uint32_t)(__builtin_popcount(plo) + __builtin_popcount(phi)));
  }
  __syncthreads();
  for (uint32_t d = tid; d < RADIX; d += BLOCK) counts[(size_t)blockIdx.x * RADIX + d] = s_h[d];
}

// TPB tiles per block: every thread issues the loads of all TPB tiles first
// (more bytes in flight per CU), then counts tile by tile into its own LDS
// histogram; nontemporal 16-byte loads like the library kernel.
template <int BITS, int BLOCK, int TPB>
__global__ __launch_bounds__(BLOCK) void k_counts_multi(const uint32_t* __restrict__ keys, RadixDigit op,
                                                        uint32_t* __restrict__ counts) {
  constexpr int RADIX = 1 << BITS;
  constexpr int TILE = BLOCK * 16;
  __shared__ uint32_t s_h[TPB][RADIX];
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < TPB * RADIX; i += BLOCK) (&s_h[0][0])[i] = 0u;
  __syncthreads();
  typedef unsigned int nv4 __attribute__((ext_vector_type(4)));
  const nv4* vp = reinterpret_cast<const nv4*>(keys + (uint64_t)blockIdx.x * TPB * TILE);
  nv4 v[TPB][4];
#pragma unroll
  for (int t = 0; t < TPB; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j) v[t][j] = __builtin_nontemporal_load(&vp[t * (TILE / 4) + j * BLOCK + tid]);
#pragma unroll
  for (int t = 0; t < TPB; ++t)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) atomicAdd(&s_h[t][op(v[t][j][q])], 1u);
  __syncthreads();
  for (uint32_t i = tid; i < TPB * RADIX; i += BLOCK)
    counts[(size_t)blockIdx.x * TPB * RADIX + i] = (&s_h[0][0])[i];
}

struct Variant {
  std::string name;
  std::function<void()> launch;
  std::vector<float> us;
  bool ok = false;
};

int main(int argc, char** argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 28;
  const size_t n = (size_t)1 << lg;
  CK(hipSetDevice(0));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  uint32_t *keys, *c_ref, *c_out;
  CK(hipMalloc(&keys, n * 4));
  CK(populate_device(keys, n, 0, st));
  const size_t cw = (n / 4096) * 256;  // enough for both geometries
  CK(hipMalloc(&c_ref, cw * 4));
  CK(hipMalloc(&c_out, cw * 4));
  std::vector<Variant> V;
  const RadixDigit op8{8, 255}, op4{4, 15};
  const uint32_t t8 = (uint32_t)(n / 8192), t4 = (uint32_t)(n / 4096);
  auto add = [&](const char* name, std::function<void()> f) { V.push_back({name, f}); };
  // 8-bit, 512-thread tiles (the per-pass counts of 8-bit sorts)
  add("8b lib (1 copy)", [&] {
    hipLaunchKernelGGL((k_tile_counts<8, 512, 16, uint32_t>), dim3(t8), dim3(512), 0, st, keys, (uint32_t)n, op8,
                       c_out, nullptr, 0u);
  });
  add("8b 2 copies", [&] { hipLaunchKernelGGL((k_counts_x<8, 512, 2, false>), dim3(t8), dim3(512), 0, st, keys, op8, c_out); });
  add("8b 4 copies", [&] { hipLaunchKernelGGL((k_counts_x<8, 512, 4, false>), dim3(t8), dim3(512), 0, st, keys, op8, c_out); });
  add("8b per-wave", [&] { hipLaunchKernelGGL((k_counts_x<8, 512, 1, true>), dim3(t8), dim3(512), 0, st, keys, op8, c_out); });
  add("8b match", [&] { hipLaunchKernelGGL((k_counts_match<8, 512>), dim3(t8), dim3(512), 0, st, keys, op8, c_out); });
  add("8b 2 tiles/block", [&] { hipLaunchKernelGGL((k_counts_multi<8, 512, 2>), dim3(t8 / 2), dim3(512), 0, st, keys, op8, c_out); });
  add("8b 4 tiles/block", [&] { hipLaunchKernelGGL((k_counts_multi<8, 512, 4>), dim3(t8 / 4), dim3(512), 0, st, keys, op8, c_out); });
  add("8b 1 tile nt", [&] { hipLaunchKernelGGL((k_counts_multi<8, 512, 1>), dim3(t8), dim3(512), 0, st, keys, op8, c_out); });
  // 4-bit, 256-thread tiles (pass-0 counts of 4-bit sorts)
  add("4b lib (16 copies)", [&] {
    hipLaunchKernelGGL((k_tile_counts<4, 256, 16, uint32_t>), dim3(t4), dim3(256), 0, st, keys, (uint32_t)n, op4,
                       c_out, nullptr, 0u);
  });
  add("4b 16 interleaved", [&] { hipLaunchKernelGGL((k_counts_x<4, 256, 16, false>), dim3(t4), dim3(256), 0, st, keys, op4, c_out); });
  add("4b 4 interleaved", [&] { hipLaunchKernelGGL((k_counts_x<4, 256, 4, false>), dim3(t4), dim3(256), 0, st, keys, op4, c_out); });
  add("4b per-wave", [&] { hipLaunchKernelGGL((k_counts_x<4, 256, 1, true>), dim3(t4), dim3(256), 0, st, keys, op4, c_out); });
  add("4b match", [&] { hipLaunchKernelGGL((k_counts_match<4, 256>), dim3(t4), dim3(256), 0, st, keys, op4, c_out); });
  add("4b 2 tiles/block", [&] { hipLaunchKernelGGL((k_counts_multi<4, 256, 2>), dim3(t4 / 2), dim3(256), 0, st, keys, op4, c_out); });
  add("4b 4 tiles/block", [&] { hipLaunchKernelGGL((k_counts_multi<4, 256, 4>), dim3(t4 / 4), dim3(256), 0, st, keys, op4, c_out); });

  // correctness: each family against its library kernel
  std::vector<uint32_t> ref, got;
  for (size_t i = 0; i < V.size(); ++i) {
    V[i].launch();
    CK(hipStreamSynchronize(st));
    const bool b8 = V[i].name[0] == '8';
    const size_t words = b8 ? (size_t)t8 * 256 : (size_t)t4 * 16;
    got.resize(words);
    CK(hipMemcpy(got.data(), c_out, words * 4, hipMemcpyDeviceToHost));
    if (V[i].name.find("lib") != std::string::npos) ref = got;
    V[i].ok = got == ref;
  }
  for (int r = 0; r < 15; ++r)
    for (auto& v : V) {
      CK(hipEventRecord(e0, st));
      v.launch();
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 2) v.us.push_back(ms * 1e3f);
    }
  for (auto& v : V) {
    std::sort(v.us.begin(), v.us.end());
    const float med = v.us[v.us.size() / 2];
    printf("%-22s median %7.1f us  best %7.1f us  %6.0f GB/s read  %s\n", v.name.c_str(), med, v.us[0],
           4.0 * n / (med * 1e-6) / 1e9, v.ok ? "exact" : "MISMATCH");
  }
  return 0;
}
