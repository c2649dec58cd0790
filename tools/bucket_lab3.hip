// Bucket-sort lab 3 (not part of libsort): the counting placement of the
// keys-only bucket sort (bucket_count_place) in persistent blocks that load
// the NEXT bucket's keys into registers while the current one is counted,
// scanned and placed -- for the 16K-key buckets of configs[2] (1024-thread
// blocks, one per CU: without it the load and the LDS phases of a CU never
// overlap) and the 4K buckets of the headline.  RAW: the phase barriers are
// raw s_barrier + lgkmcnt(0) (a __syncthreads() may drain the prefetch).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/bucket_lab3 tools/bucket_lab3.hip
//   tools/bucket_lab3 [filter,...]
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

template <bool RAW>
__device__ __forceinline__ void bar() {
  if constexpr (RAW) {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  } else {
    __syncthreads();
  }
}

template <int BLOCK, bool RAW>
__device__ __forceinline__ uint32_t bscan(uint32_t v, uint32_t* s_wsum) {
  constexpr int WAVES = BLOCK / kWave;
  const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, kWave);
    if (lane >= o) x += y;
  }
  if (lane == kWave - 1) s_wsum[w] = x;
  bar<RAW>();
  uint32_t pre = 0;
#pragma unroll
  for (int i = 0; i < WAVES; ++i) pre += (i < w) ? s_wsum[i] : 0u;
  return pre + x - v;
}

// the product's counting placement for lbits = 16 (no overflow fallback: the
// lab's keys have no duplicates that overflow), barriers per RAW
template <int BLOCK, int ITEMS, bool RAW>
__device__ __forceinline__ void place16(const uint32_t (&k)[ITEMS], uint64_t* s_cw, uint32_t* s_wsum,
                                        uint32_t* out, uint32_t start, uint32_t len) {
  constexpr int PER = kCntCells / BLOCK;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
  const uint32_t wbase = w * ITEMS * kWave;
  auto ci = [&](uint32_t c) -> uint32_t { return (c % PER) * BLOCK + c / PER; };
  uint32_t rk[ITEMS];
#pragma unroll
  for (int q = 0; q < PER; ++q) s_cw[q * BLOCK + tid] = 0ull;
  bar<RAW>();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (wbase + j * kWave + lane < len) {
      const uint32_t v = k[j] & 0xffffu, sh = 3u * (v & 15u);
      const uint64_t old = atomicAdd((unsigned long long*)&s_cw[ci(v >> 4)], (1ull << sh) + (1ull << 48));
      rk[j] = (uint32_t)(old >> sh) & 7u;
    }
  bar<RAW>();
  uint64_t cw[PER];
  uint32_t sum = 0;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    cw[q] = s_cw[q * BLOCK + tid];
    sum += (uint32_t)(cw[q] >> 48);
  }
  uint32_t run = bscan<BLOCK, RAW>(sum, s_wsum);
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const uint32_t c = (uint32_t)(cw[q] >> 48);
    s_cw[q * BLOCK + tid] = (cw[q] & 0xFFFFFFFFFFFFull) | ((uint64_t)run << 48);
    run += c;
  }
  bar<RAW>();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (wbase + j * kWave + lane < len) {
      const uint32_t v = k[j] & 0xffffu;
      const uint64_t c = s_cw[ci(v >> 4)];
      rk[j] += (uint32_t)(c >> 48) + field3_sum(c & ((1ull << (3u * (v & 15u))) - 1ull));
    }
  bar<RAW>();
  uint32_t* s_keys = reinterpret_cast<uint32_t*>(s_cw);
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (wbase + j * kWave + lane < len) s_keys[rk[j]] = k[j];
  bar<RAW>();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t p = wbase + j * kWave + lane;
    if (p < len) out[(size_t)start + p] = s_keys[p];
  }
}

template <int BLOCK, int ITEMS>
constexpr int lds_words() {
  return (8 * kCntCells > 4 * BLOCK * ITEMS ? 8 * kCntCells : 4 * BLOCK * ITEMS) / 8;
}

// one bucket per block (the product's shape, with the trimmed LDS footprint)
template <int BLOCK, int ITEMS>
__global__ __launch_bounds__(BLOCK) void k_one(const uint32_t* in, uint32_t* out, const uint32_t* bstart,
                                               const uint32_t* blen, const uint32_t* nb) {
  __shared__ uint64_t s_cw[lds_words<BLOCK, ITEMS>()];
  __shared__ uint32_t s_wsum[BLOCK / kWave];
  if (blockIdx.x >= *nb) return;
  const uint32_t b = blockIdx.x, start = bstart[b], len = blen[b];
  const uint32_t wbase = (threadIdx.x / kWave) * ITEMS * kWave, lane = threadIdx.x & 63;
  uint32_t k[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = wbase + j * kWave + lane;
    k[j] = i < len ? load_stream(&in[(size_t)start + i]) : 0xffffffffu;
  }
  place16<BLOCK, ITEMS, false>(k, s_cw, s_wsum, out, start, len);
}

// persistent: bucket b, b + grid, ...; the next bucket's keys load into kn
// while the current one is placed
template <int BLOCK, int ITEMS, bool RAW>
__global__ __launch_bounds__(BLOCK) void k_pf(const uint32_t* in, uint32_t* out, const uint32_t* bstart,
                                              const uint32_t* blen, const uint32_t* nb) {
  __shared__ uint64_t s_cw[lds_words<BLOCK, ITEMS>()];
  __shared__ uint32_t s_wsum[BLOCK / kWave];
  const uint32_t m = *nb;
  uint32_t b = blockIdx.x;
  if (b >= m) return;
  const uint32_t wbase = (threadIdx.x / kWave) * ITEMS * kWave, lane = threadIdx.x & 63;
  uint32_t start = bstart[b], len = blen[b];
  uint32_t k[ITEMS], kn[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = wbase + j * kWave + lane;
    k[j] = i < len ? load_stream(&in[(size_t)start + i]) : 0xffffffffu;
  }
  for (;;) {
    const uint32_t nx = b + gridDim.x;
    uint32_t ns = 0, nl = 0;
    if (nx < m) {
      ns = bstart[nx];
      nl = blen[nx];
    }
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t i = wbase + j * kWave + lane;
      kn[j] = i < nl ? load_stream(&in[(size_t)ns + i]) : 0xffffffffu;
    }
    place16<BLOCK, ITEMS, RAW>(k, s_cw, s_wsum, out, start, len);
    bar<RAW>();  // the last LDS reads before the next bucket's zeroing
    if (nx >= m) break;
    b = nx;
    start = ns;
    len = nl;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) k[j] = kn[j];
  }
}

// the floor: load, through LDS (same footprint), store
template <int BLOCK, int ITEMS>
__global__ __launch_bounds__(BLOCK) void k_copy(const uint32_t* in, uint32_t* out, const uint32_t* bstart,
                                                const uint32_t* blen, const uint32_t* nb) {
  __shared__ uint32_t s_keys[2 * lds_words<BLOCK, ITEMS>()];
  if (blockIdx.x >= *nb) return;
  const uint32_t b = blockIdx.x, start = bstart[b], len = blen[b];
  const uint32_t wbase = (threadIdx.x / kWave) * ITEMS * kWave, lane = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = wbase + j * kWave + lane;
    if (i < len) s_keys[len - 1 - i] = load_stream(&in[(size_t)start + i]);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = wbase + j * kWave + lane;
    if (i < len) out[(size_t)start + i] = s_keys[len - 1 - i];
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
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t NMAX = (size_t)1 << 30;
  uint32_t *in, *out, *bs, *bl, *nb, *ov, *ovn, *ovl;
  CK(hipMalloc(&in, NMAX * 4)); CK(hipMalloc(&out, NMAX * 4));
  CK(hipMalloc(&bs, (NMAX / 1024 + 1) * 4)); CK(hipMalloc(&bl, (NMAX / 1024 + 1) * 4)); CK(hipMalloc(&nb, 4)); CK(hipMalloc(&ov, 4));
  CK(hipMalloc(&ovn, 4)); CK(hipMalloc(&ovl, (NMAX / 1024 + 1) * 4));
  hipStream_t st; CK(hipStreamCreate(&st));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  struct V { std::string name; int lg; uint32_t S; std::function<void(uint32_t)> launch; };
  std::vector<V> vs;
  // configs[2] class: 2^30 keys in 16K buckets, 1024 x 17
  vs.push_back({"c3 copy 1024x17", 30, 16384, [&](uint32_t m) {
    hipLaunchKernelGGL((k_copy<1024, 17>), dim3(m), dim3(1024), 0, st, in, out, bs, bl, nb); }});
  vs.push_back({"c3 prod 1024x17", 30, 16384, [&](uint32_t m) {
    CK(hipMemsetAsync(ovn, 0, 4, st));
    hipLaunchKernelGGL((k_bucket_count<1024, 17, RadixDigit, kCnt3F>), dim3(m), dim3(1024), 0, st, in, out, bs, bl, nb, 1u << 30, nullptr, 16u, 0u, ov, nullptr, 0u, ovn, ovl);
    hipLaunchKernelGGL((k_bucket_sort<8, 1024, 17, RadixDigit, uint32_t, NoValue, 0, true>), dim3(512), dim3(1024), 0, st, in, out, (const NoValue*)nullptr, (NoValue*)nullptr, bs, bl, ovn, m, ovl, 16u, 0u, ov, nullptr, 0u); }});
  vs.push_back({"c3 one 1024x17", 30, 16384, [&](uint32_t m) {
    hipLaunchKernelGGL((k_one<1024, 17>), dim3(m), dim3(1024), 0, st, in, out, bs, bl, nb); }});
  vs.push_back({"c3 one 512x34", 30, 16384, [&](uint32_t m) {
    hipLaunchKernelGGL((k_one<512, 34>), dim3(m), dim3(512), 0, st, in, out, bs, bl, nb); }});
  for (int g : {1, 2}) {
    vs.push_back({"c3 pf 1024x17 sync g=" + std::to_string(g), 30, 16384, [&, g](uint32_t m) {
      hipLaunchKernelGGL((k_pf<1024, 17, false>), dim3(std::min<uint32_t>(m, g * cus)), dim3(1024), 0, st, in, out, bs, bl, nb); }});
    vs.push_back({"c3 pf 1024x17 raw g=" + std::to_string(g), 30, 16384, [&, g](uint32_t m) {
      hipLaunchKernelGGL((k_pf<1024, 17, true>), dim3(std::min<uint32_t>(m, g * cus)), dim3(1024), 0, st, in, out, bs, bl, nb); }});
  }
  // headline class: 2^28 keys in 4K buckets, 256 x 17
  vs.push_back({"c2 copy 256x17", 28, 4096, [&](uint32_t m) {
    hipLaunchKernelGGL((k_copy<256, 17>), dim3(m), dim3(256), 0, st, in, out, bs, bl, nb); }});
  vs.push_back({"c2 prod 256x17", 28, 4096, [&](uint32_t m) {
    CK(hipMemsetAsync(ovn, 0, 4, st));
    hipLaunchKernelGGL((k_bucket_count<256, 17, RadixDigit, kCnt2F>), dim3(m), dim3(256), 0, st, in, out, bs, bl, nb, 1u << 30, nullptr, 16u, 0u, ov, nullptr, 0u, ovn, ovl);
    hipLaunchKernelGGL((k_bucket_sort<4, 256, 17, RadixDigit, uint32_t, NoValue, 0, true>), dim3(512), dim3(256), 0, st, in, out, (const NoValue*)nullptr, (NoValue*)nullptr, bs, bl, ovn, m, ovl, 16u, 0u, ov, nullptr, 0u); }});
  vs.push_back({"c2 one 256x17", 28, 4096, [&](uint32_t m) {
    hipLaunchKernelGGL((k_one<256, 17>), dim3(m), dim3(256), 0, st, in, out, bs, bl, nb); }});
  for (int g : {2, 3, 4}) {
    vs.push_back({"c2 pf 256x17 raw g=" + std::to_string(g), 28, 4096, [&, g](uint32_t m) {
      hipLaunchKernelGGL((k_pf<256, 17, true>), dim3(std::min<uint32_t>(m, g * cus)), dim3(256), 0, st, in, out, bs, bl, nb); }});
  }
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
    const uint32_t m = (uint32_t)(n / v.S), lbits = 16;
    hipLaunchKernelGGL(fill, dim3((n + 255) / 256), dim3(256), 0, st, in, n, v.S, lbits);
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
