// Bucket-sort lab 4 (not part of libsort): a counting placement with a
// smaller LDS footprint for the 4K-key buckets of the headline (256-thread
// blocks), so that more blocks fit on a CU:
//   cnt2  4096 cells of u32 (16 2-bit residual counts; the cell's key count
//         is their sum: two popcounts) + u16 cell starts: 24 KB instead of
//         33 KB.  A 2-bit count overflows at 4 equal keys (~4% of uniform
//         4096-key buckets over 2^16 values): the block then sorts by four
//         stable 4-bit LSD steps (correct, ~2x the cost).
//   WPE   amdgpu_waves_per_eu lower bound (VGPR budget: 5 -> 96, 6 -> 80)
// and, for the 16K-key buckets of configs[2] (1024-thread blocks), the
// product's counting placement with the LDS trimmed to the key overlay (68 KB,
// so two blocks fit) under a 64-VGPR budget (waves_per_eu 8).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/bucket_lab4 tools/bucket_lab4.hip
//   tools/bucket_lab4 [filter,...]
#include "../gpu-radix-sort_amd/csrc/radix_kernels.hip"

#include <algorithm>
#include <cstdio>
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

__device__ __forceinline__ uint32_t f2sum(uint32_t w) {
  return (uint32_t)__builtin_popcount(w & 0x55555555u) + 2u * (uint32_t)__builtin_popcount(w & 0xAAAAAAAAu);
}

// stable 4-bit LSD steps over the low 16 bits (the overflow fallback); keys
// in k (pads 0xffffffff), s_keys holds >= BLOCK * ITEMS keys
template <int BLOCK, int ITEMS>
__device__ void lsd16(uint32_t (&k)[ITEMS], uint32_t* s_keys, WaveCount (*s_whist)[16], uint32_t* s_wsum) {
  constexpr int WAVES = BLOCK / kWave;
  const int tid = threadIdx.x, lane = tid & 63, w = tid / 64;
  const uint32_t wbase = w * ITEMS * kWave;
  uint32_t rk[ITEMS];
  for (uint32_t shift = 0; shift < 16; shift += 4) {
    const RadixDigit op{shift, 15u};
    for (int d = lane; d < 16; d += kWave) s_whist[w][d] = 0;
    rank_items_t<4, true, ITEMS>(k, rk, s_whist[w], 0u, wbase, lane, op);
    __syncthreads();
    uint32_t cnt_d = 0;
    if (tid < 16) {
#pragma unroll
      for (int i = 0; i < WAVES; ++i) cnt_d += s_whist[i][tid];
    }
    uint32_t total;
    const uint32_t excl = block_exclusive_scan<BLOCK>(cnt_d, s_wsum, total);
    if (tid < 16) {
      uint32_t run = excl;
#pragma unroll
      for (int i = 0; i < WAVES; ++i) {
        const uint32_t c = s_whist[i][tid];
        s_whist[i][tid] = (WaveCount)run;
        run += c;
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) s_keys[s_whist[w][op(k[j])] + rk[j]] = k[j];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) k[j] = s_keys[wbase + j * kWave + lane];
    __syncthreads();
  }
}

template <int BLOCK, int ITEMS>
constexpr int cnt2_words() {  // u32 words: 4096 cells + 2048 (4096 u16 starts), or the key overlay
  return 6144 > BLOCK * ITEMS ? 6144 : BLOCK * ITEMS;
}

template <int BLOCK, int ITEMS, int WPE, bool INL = false>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void k_cnt2(
    const uint32_t* in, uint32_t* out, const uint32_t* bstart, const uint32_t* blen, const uint32_t* nb,
    uint32_t* ovf_n, uint32_t* ovf_list) {
  constexpr int PER = kCntCells / BLOCK;
  __shared__ uint32_t s_w[cnt2_words<BLOCK, ITEMS>()];
  __shared__ uint32_t s_wsum[BLOCK / kWave];
  __shared__ WaveCount s_whist[BLOCK / kWave][16];
  __shared__ uint32_t s_flag;
  if (blockIdx.x >= *nb) return;
  const uint32_t b = blockIdx.x, start = bstart[b], len = blen[b];
  const int tid = threadIdx.x, lane = tid & 63, w = tid / 64;
  const uint32_t wbase = w * ITEMS * kWave;
  uint16_t* s_st = reinterpret_cast<uint16_t*>(s_w + kCntCells);
  auto ci = [&](uint32_t c) -> uint32_t { return (c % PER) * BLOCK + c / PER; };
  uint32_t k[ITEMS], rk[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = wbase + j * kWave + lane;
    k[j] = i < len ? load_stream(&in[(size_t)start + i]) : 0xffffffffu;
  }
#pragma unroll
  for (int q = 0; q < PER; ++q) s_w[q * BLOCK + tid] = 0u;
  if (tid == 0) s_flag = 0u;
  __syncthreads();
  bool ovf = false;
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (wbase + j * kWave + lane < len) {
      const uint32_t v = k[j] & 0xffffu, sh = 2u * (v & 15u);
      const uint32_t old = atomicAdd(&s_w[ci(v >> 4)], 1u << sh);
      rk[j] = (old >> sh) & 3u;
      ovf |= rk[j] == 3u;
    }
  if (__any(ovf) && lane == 0) s_flag = 1u;
  __syncthreads();
  if (s_flag) {
    if constexpr (INL) {
      lsd16<BLOCK, ITEMS>(k, s_w, s_whist, s_wsum);
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) {
        const uint32_t i = wbase + j * kWave + lane;
        if (i < len) out[(size_t)start + i] = k[j];
      }
    } else if (tid == 0) {
      // a 2-bit count overflowed: listed for the LSD-step launch (nothing written)
      ovf_list[atomicAdd(ovf_n, 1u)] = b;
    }
    return;
  }
  uint32_t cnt[PER], sum = 0;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    cnt[q] = f2sum(s_w[q * BLOCK + tid]);
    sum += cnt[q];
  }
  uint32_t total;
  uint32_t run = block_exclusive_scan<BLOCK>(sum, s_wsum, total);
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    s_st[q * BLOCK + tid] = (uint16_t)run;
    run += cnt[q];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (wbase + j * kWave + lane < len) {
      const uint32_t v = k[j] & 0xffffu, c = ci(v >> 4);
      const uint32_t wd = s_w[c];
      rk[j] += (uint32_t)s_st[c] + f2sum(wd & ((1u << (2u * (v & 15u))) - 1u));
    }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (wbase + j * kWave + lane < len) s_w[rk[j]] = k[j];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t p = wbase + j * kWave + lane;
    if (p < len) out[(size_t)start + p] = s_w[p];
  }
}

// the product's placement (3-bit fields, u64 cells) with LDS = max(cells, keys)
template <int BLOCK, int ITEMS, int WPE>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void k_cnt3(
    const uint32_t* in, uint32_t* out, const uint32_t* bstart, const uint32_t* blen, const uint32_t* nb) {
  constexpr int PER = kCntCells / BLOCK, CAP = BLOCK * ITEMS;
  constexpr int WORDS = (8 * kCntCells > 4 * CAP ? 8 * kCntCells : 4 * CAP) / 8;
  __shared__ uint64_t s_cw[WORDS];
  __shared__ uint32_t s_wsum[BLOCK / kWave];
  if (blockIdx.x >= *nb) return;
  const uint32_t b = blockIdx.x, start = bstart[b], len = blen[b];
  const int tid = threadIdx.x, lane = tid & 63, w = tid / 64;
  const uint32_t wbase = w * ITEMS * kWave;
  auto ci = [&](uint32_t c) -> uint32_t { return (c % PER) * BLOCK + c / PER; };
  uint32_t k[ITEMS], rk[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = wbase + j * kWave + lane;
    k[j] = i < len ? load_stream(&in[(size_t)start + i]) : 0xffffffffu;
  }
#pragma unroll
  for (int q = 0; q < PER; ++q) s_cw[q * BLOCK + tid] = 0ull;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (wbase + j * kWave + lane < len) {
      const uint32_t v = k[j] & 0xffffu, sh = 3u * (v & 15u);
      const uint64_t old = atomicAdd((unsigned long long*)&s_cw[ci(v >> 4)], (1ull << sh) + (1ull << 48));
      rk[j] = (uint32_t)(old >> sh) & 7u;
    }
  __syncthreads();
  uint64_t cw[PER];
  uint32_t sum = 0;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    cw[q] = s_cw[q * BLOCK + tid];
    sum += (uint32_t)(cw[q] >> 48);
  }
  uint32_t total;
  uint32_t run = block_exclusive_scan<BLOCK>(sum, s_wsum, total);
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const uint32_t c = (uint32_t)(cw[q] >> 48);
    s_cw[q * BLOCK + tid] = (cw[q] & 0xFFFFFFFFFFFFull) | ((uint64_t)run << 48);
    run += c;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (wbase + j * kWave + lane < len) {
      const uint32_t v = k[j] & 0xffffu;
      const uint64_t c = s_cw[ci(v >> 4)];
      rk[j] += (uint32_t)(c >> 48) + field3_sum(c & ((1ull << (3u * (v & 15u))) - 1ull));
    }
  __syncthreads();
  uint32_t* s_keys = reinterpret_cast<uint32_t*>(s_cw);
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (wbase + j * kWave + lane < len) s_keys[rk[j]] = k[j];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t p = wbase + j * kWave + lane;
    if (p < len) out[(size_t)start + p] = s_keys[p];
  }
}

__global__ void fill(uint32_t* k, size_t n, uint32_t S, uint32_t lbits) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t x = (i + 1) * 0x9E3779B97F4A7C15ull;
  x ^= x >> 29; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 32;
  k[i] = ((uint32_t)(i / S) << lbits) | (uint32_t)(x & ((1ull << lbits) - 1));
}

int main(int argc, char** argv) {
  const size_t NMAX = (size_t)1 << 30;
  uint32_t *in, *out, *bs, *bl, *nb, *ov, *ovn, *ovl;
  CK(hipMalloc(&in, NMAX * 4)); CK(hipMalloc(&out, NMAX * 4));
  CK(hipMalloc(&bs, (NMAX / 1024 + 1) * 4)); CK(hipMalloc(&bl, (NMAX / 1024 + 1) * 4)); CK(hipMalloc(&nb, 4)); CK(hipMalloc(&ov, 4));
  CK(hipMalloc(&ovn, 4)); CK(hipMalloc(&ovl, (NMAX / 1024 + 1) * 4));
  hipStream_t st; CK(hipStreamCreate(&st));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  struct V { std::string name; int lg; uint32_t S; std::function<void(uint32_t)> launch; };
  std::vector<V> vs;
  vs.push_back({"c2 prod3F 256x17", 28, 4096, [&](uint32_t m) {
    CK(hipMemsetAsync(ovn, 0, 4, st));
    hipLaunchKernelGGL((k_bucket_count<256, 17, RadixDigit, kCnt3F>), dim3(m), dim3(256), 0, st, in, out, bs, bl, nb, 1u << 30, nullptr, 16u, 0u, ov, nullptr, 0u, ovn, ovl, nullptr, nullptr);
    hipLaunchKernelGGL((k_bucket_sort<4, 256, 17, RadixDigit, uint32_t, NoValue, 0, true>), dim3(512), dim3(256), 0, st, in, out, (const NoValue*)nullptr, (NoValue*)nullptr, bs, bl, ovn, m, ovl, 16u, 0u, ov, nullptr, 0u); }});
  vs.push_back({"c2 prod 256x17", 28, 4096, [&](uint32_t m) {
    CK(hipMemsetAsync(ovn, 0, 4, st));
    hipLaunchKernelGGL((k_bucket_count<256, 17, RadixDigit, kCnt2F>), dim3(m), dim3(256), 0, st, in, out, bs, bl, nb, 1u << 30, nullptr, 16u, 0u, ov, nullptr, 0u, ovn, ovl, nullptr, nullptr);
    hipLaunchKernelGGL((k_bucket_sort<4, 256, 17, RadixDigit, uint32_t, NoValue, 0, true>), dim3(512), dim3(256), 0, st, in, out, (const NoValue*)nullptr, (NoValue*)nullptr, bs, bl, ovn, m, ovl, 16u, 0u, ov, nullptr, 0u); }});
  // (the overflowed buckets: the product's LSD-step kernel over the list,
  // grid 1024 over min(*ovn, 1024); the lab's uniform keys overflow ~4% of
  // 65536 buckets, so the list launch takes a grid of the list's bound)
#define CNT2(W) vs.push_back({"c2 cnt2 256x17 wpe=" #W, 28, 4096, [&](uint32_t m) { \
    CK(hipMemsetAsync(ovn, 0, 4, st)); \
    hipLaunchKernelGGL((k_cnt2<256, 17, W>), dim3(m), dim3(256), 0, st, in, out, bs, bl, nb, ovn, ovl); \
    hipLaunchKernelGGL((k_bucket_sort<4, 256, 17, RadixDigit, uint32_t, NoValue, 0, false>), dim3(m / 8), dim3(256), 0, st, \
                       out, out, (const NoValue*)nullptr, (NoValue*)nullptr, bs, bl, ovn, m / 8, ovl, 16u, 0u, ov, nullptr, 0u); }});
  CNT2(1) CNT2(6) CNT2(8)
  vs.push_back({"c2 cnt2 inline-fallback 256x17", 28, 4096, [&](uint32_t m) {
    hipLaunchKernelGGL((k_cnt2<256, 17, 1, true>), dim3(m), dim3(256), 0, st, in, out, bs, bl, nb, ovn, ovl); }});
#define CNT3(B, I, S, LG, W) vs.push_back({"c" #LG " cnt3 " #B "x" #I " wpe=" #W, LG == 30 ? 30 : 28, S, [&](uint32_t m) { \
    hipLaunchKernelGGL((k_cnt3<B, I, W>), dim3(m), dim3(B), 0, st, in, out, bs, bl, nb); }});
  CNT3(256, 17, 4096, 2, 1) CNT3(256, 17, 4096, 2, 5)
  vs.push_back({"c3 prod 1024x17", 30, 16384, [&](uint32_t m) {
    CK(hipMemsetAsync(ovn, 0, 4, st));
    hipLaunchKernelGGL((k_bucket_count<1024, 17, RadixDigit, kCnt3F>), dim3(m), dim3(1024), 0, st, in, out, bs, bl, nb, 1u << 30, nullptr, 16u, 0u, ov, nullptr, 0u, ovn, ovl, nullptr, nullptr);
    hipLaunchKernelGGL((k_bucket_sort<8, 1024, 17, RadixDigit, uint32_t, NoValue, 0, true>), dim3(512), dim3(1024), 0, st, in, out, (const NoValue*)nullptr, (NoValue*)nullptr, bs, bl, ovn, m, ovl, 16u, 0u, ov, nullptr, 0u); }});
  CNT3(1024, 17, 16384, 30, 1) CNT3(1024, 17, 16384, 30, 8) CNT3(512, 34, 16384, 30, 4)
  const char* filt = argc > 1 ? argv[1] : nullptr;
  std::vector<uint32_t> h;
  for (auto& v : vs) {
    if (filt) {
      bool hit = false;
      std::string f(filt);
      for (size_t a = 0; a <= f.size();) {
        size_t e = f.find(',', a);
        if (e == std::string::npos) e = f.size();
        if (e > a && v.name.find(f.substr(a, e - a)) != std::string::npos) hit = true;
        a = e + 1;
      }
      if (!hit) continue;
    }
    const size_t n = (size_t)1 << v.lg;
    const uint32_t m = (uint32_t)(n / v.S);
    hipLaunchKernelGGL(fill, dim3((n + 255) / 256), dim3(256), 0, st, in, n, v.S, 16u);
    std::vector<uint32_t> hs(m), hl(m, v.S);
    for (uint32_t b = 0; b < m; ++b) hs[b] = b * v.S;
    CK(hipMemcpyAsync(bs, hs.data(), m * 4, hipMemcpyHostToDevice, st));
    CK(hipMemcpyAsync(bl, hl.data(), m * 4, hipMemcpyHostToDevice, st));
    CK(hipMemcpyAsync(nb, &m, 4, hipMemcpyHostToDevice, st));
    CK(hipStreamSynchronize(st));
    h.resize(n);
    CK(hipMemcpy(h.data(), in, n * 4, hipMemcpyDeviceToHost));
    uint64_t sum0 = 0; uint32_t x0 = 0;
    for (size_t i = 0; i < n; ++i) { sum0 += h[i]; x0 ^= h[i]; }
    std::vector<float> us;
    for (int r = 0; r < 10; ++r) {
      CK(hipEventRecord(e0, st));
      v.launch(m);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 2) us.push_back(ms * 1e3f);
    }
    CK(hipMemcpy(h.data(), out, n * 4, hipMemcpyDeviceToHost));
    uint64_t sum1 = 0; uint32_t x1 = 0; bool sorted = true;
    for (size_t i = 0; i < n; ++i) { sum1 += h[i]; x1 ^= h[i]; if (i && h[i - 1] > h[i]) sorted = false; }
    std::sort(us.begin(), us.end());
    const float med = us[us.size() / 2];
    printf("%-28s 2^%d keys: median %7.1f us  best %7.1f  %5.0f GB/s  %s\n", v.name.c_str(), v.lg, med, us[0],
           8.0 * n / (med * 1e-6) / 1e9, (sorted && sum0 == sum1 && x0 == x1) ? "sorted" : (sum0 == sum1 && x0 == x1 ? "permutation" : "WRONG"));
    fflush(stdout);
  }
  return 0;
}
