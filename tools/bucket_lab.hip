// Bucket-sort lab (not part of libsort): k_bucket_sort on 2^lg keys cut into
// buckets of S keys whose top 16 bits are the bucket index (the state after
// 16 bits of MSD passes over uniform keys), sorted on their low 16 bits.
// Every variant is checked: output globally sorted and a permutation of the
// input (sum and xor).  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/bucket_lab tools/bucket_lab.hip
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

__global__ void fill(uint32_t* k, size_t n, uint32_t S, uint32_t jitter) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t x = (i + 1) * 0x9E3779B97F4A7C15ull;
  x ^= x >> 29; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 32;
  k[i] = ((uint32_t)(i / S) << 16) | (uint32_t)(x & 0xffffu);
}

int main(int argc, char** argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 28;
  const size_t n = (size_t)1 << lg;
  uint32_t *in, *out, *bs, *bl, *nb, *ov;
  CK(hipMalloc(&in, n * 4)); CK(hipMalloc(&out, n * 4));
  CK(hipMalloc(&bs, (n / 1024 + 1) * 4)); CK(hipMalloc(&bl, (n / 1024 + 1) * 4)); CK(hipMalloc(&nb, 4)); CK(hipMalloc(&ov, 4));
  hipStream_t st; CK(hipStreamCreate(&st));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<uint32_t> h(n);
  struct V { std::string name; uint32_t S; std::function<void(uint32_t)> launch; };
  std::vector<V> vs;
#define BVG(BITS, B, I, S_, LB, G)                                                                                \
  vs.push_back({#BITS "-bit " #B "x" #I " S=" #S_ " lbits=" #LB " grid=" #G, S_, [&](uint32_t m) {               \
                  hipLaunchKernelGGL((k_bucket_sort<BITS, B, I>), dim3(G ? std::min<uint32_t>(m, G) : m), dim3(B), 0, \
                                     st, in, out, (const NoValue*)nullptr, (NoValue*)nullptr, bs, bl, nb, 1u << 30,  \
                                     nullptr, LB##u, 0u, ov, nullptr, 0u);                                           \
                }});
#define BVL(BITS, B, I, S_, LB) BVG(BITS, B, I, S_, LB, 0)
#define BV(BITS, B, I, S_) BVL(BITS, B, I, S_, 16)
  BV(4, 256, 17, 4096)
  for (auto& v : vs) {
    const uint32_t m = (uint32_t)(n / v.S);
    hipLaunchKernelGGL(fill, dim3((n + 255) / 256), dim3(256), 0, st, in, n, v.S, 0u);
    std::vector<uint32_t> hs(m), hl(m, v.S);
    for (uint32_t b = 0; b < m; ++b) hs[b] = b * v.S;
    CK(hipMemcpyAsync(bs, hs.data(), m * 4, hipMemcpyHostToDevice, st));
    CK(hipMemcpyAsync(bl, hl.data(), m * 4, hipMemcpyHostToDevice, st));
    CK(hipMemcpyAsync(nb, &m, 4, hipMemcpyHostToDevice, st));
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(h.data(), in, n * 4, hipMemcpyDeviceToHost));
    uint64_t sum0 = 0; uint32_t x0 = 0;
    for (auto x : h) { sum0 += x; x0 ^= x; }
    std::vector<float> us;
    for (int r = 0; r < 12; ++r) {
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
    printf("%-26s 2^%d keys: median %7.1f us  best %7.1f  %5.0f GB/s (8 B/key)  %s\n", v.name.c_str(), lg, med, us[0],
           8.0 * n / (med * 1e-6) / 1e9, (sorted && sum0 == sum1 && x0 == x1) ? "sorted" : (sum0 == sum1 && x0 == x1 ? "permutation" : "WRONG"));
  }
  // (u64 key, u32 value) buckets: key = bucket << 48 | 48 random bits
  {
    const size_t np = n / 2;
    uint64_t *k64, *o64;
    uint32_t *vv, *ov32;
    CK(hipMalloc(&k64, np * 8)); CK(hipMalloc(&o64, np * 8)); CK(hipMalloc(&vv, np * 4)); CK(hipMalloc(&ov32, np * 4));
    std::vector<uint64_t> hk(np);
    const uint32_t S = 4096, m = (uint32_t)(np / S);
    for (size_t i = 0; i < np; ++i) {
      uint64_t x = (i + 1) * 0x9E3779B97F4A7C15ull;
      x ^= x >> 29; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 32;
      hk[i] = ((uint64_t)(i / S) << 48) | (x & 0xFFFFFFFFFFFFull);
    }
    CK(hipMemcpy(k64, hk.data(), np * 8, hipMemcpyHostToDevice));
    std::vector<uint32_t> hs(m), hl(m, S), hv(np);
    for (uint32_t b = 0; b < m; ++b) hs[b] = b * S;
    for (size_t i = 0; i < np; ++i) hv[i] = (uint32_t)i;
    CK(hipMemcpy(vv, hv.data(), np * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(bs, hs.data(), m * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(bl, hl.data(), m * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(nb, &m, 4, hipMemcpyHostToDevice));
    auto run = [&](const char* name, std::function<void()> f) {
      std::vector<float> us;
      for (int r = 0; r < 12; ++r) {
        CK(hipEventRecord(e0, st)); f(); CK(hipEventRecord(e1, st)); CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1)); if (r >= 2) us.push_back(ms * 1e3f);
      }
      std::sort(us.begin(), us.end());
      std::vector<uint64_t> ok(np);
      CK(hipMemcpy(ok.data(), o64, np * 8, hipMemcpyDeviceToHost));
      bool sorted = true;
      for (size_t i = 1; i < np; ++i) if (ok[i - 1] > ok[i]) { sorted = false; break; }
      printf("pairs %-34s 2^%d pairs: median %7.1f us  %s\n", name, lg - 1, us[us.size() / 2], sorted ? "sorted" : "not sorted");
    };
#define PV(B, I, LB, FX)                                                                                         \
    run(#B "x" #I " lbits=" #LB " fix=" #FX, [&] {                                                             \
      hipLaunchKernelGGL((k_bucket_sort<8, B, I, RadixDigit, uint64_t, uint32_t, FX>), dim3(m), dim3(B), 0, st, k64, o64, \
                         vv, ov32, bs, bl, nb, 1u << 30, nullptr, LB##u, 0u, ov, nullptr, 0u);                        \
    });
    PV(512, 9, 0, 0) PV(512, 9, 8, 0) PV(512, 9, 16, 0) PV(512, 9, 48, 0) PV(512, 9, 48, 16) PV(256, 17, 48, 16)
  }
  return 0;
}
