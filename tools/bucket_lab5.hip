// Bucket-sort lab 5 (not part of libsort): VERDICT r04 item 4's two ideas for
// the headline's keys-only bucket phase (k_bucket_count kCnt2F: 52% of its
// LDS-active cycles are bank-conflict stalls), on exact 4096-key buckets of
// 2^28 keys sharing their top 16 bits (uniform low 16 bits):
//   prod     the product kernel (2-bit cells; an overflowing bucket, ~4%,
//            is listed and not written -- timed alone, as its first launch)
//   regen    regenerate from the counts: the keys are counted with
//            non-returning atomics (no rank kept), the cells scanned, and each
//            thread writes its 16 cells' values (value repeated by its count)
//            into LDS at the cell starts, then the bucket is stored
//            coalesced -- no per-key position reads, no rank registers
//   lab 2F   prod restated (no list arguments), and "swz" the same with the
//            cell index XOR-swizzled (c ^ ((c >> 6) & 63)) before the column
//            map for the atomics and the position reads
// Verification: each bucket sorted, same sum / xor as the input.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/bucket_lab5 tools/bucket_lab5.hip
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

template <int BLOCK, int ITEMS, bool SWZ>
__global__ __launch_bounds__(BLOCK) void k_regen(const uint32_t* in, uint32_t* out, const uint32_t* bstart,
                                                 const uint32_t* blen, const uint32_t* nb, uint32_t* ovf_n) {
  constexpr int PER = kCntCells / BLOCK, CAP = BLOCK * ITEMS;
  // the cells (16 KB), then the bucket's keys as written back over them (the
  // cells are in registers once the scan's barrier has passed): 17 KB
  __shared__ uint32_t s_w[CAP > kCntCells ? CAP : kCntCells];
  uint32_t* const s_out = s_w;
  __shared__ uint32_t s_ws[BLOCK / kWave];
  if (blockIdx.x >= *nb) return;
  const uint32_t b = blockIdx.x, start = bstart[b], len = blen[b];
  const int tid = threadIdx.x, lane = tid & 63, w = tid / 64;
  const uint32_t wbase = w * ITEMS * kWave;
  auto ci = [&](uint32_t c) -> uint32_t { return (c % PER) * BLOCK + c / PER; };
  uint32_t hi = 0;
  {
    uint32_t k[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t i = wbase + j * kWave + lane;
      k[j] = i < len ? load_stream(&in[(size_t)start + i]) : 0u;
    }
    hi = in[start] & 0xFFFF0000u;
#pragma unroll
    for (int q = 0; q < PER; ++q) s_w[q * BLOCK + tid] = 0u;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j)
      if (wbase + j * kWave + lane < len) {
        const uint32_t v = k[j] & 0xFFFFu;
        atomicAdd(&s_w[ci(v >> 4)], 1u << (2u * (v & 15u)));  // (no return: no rank)
      }
  }
  __syncthreads();
  uint32_t cw[PER], sum = 0;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    cw[q] = s_w[q * BLOCK + tid];
    sum += field2_sum(cw[q]);
  }
  uint32_t total;
  uint32_t run = block_exclusive_scan<BLOCK>(sum, s_ws, total);
  // a wrapped count loses keys: the sum of the fields falls short of len
  if (total != len) {
    if (tid == 0) atomicAdd(ovf_n, 1u);
    return;
  }
  // emit: cell c = tid * PER + q holds the values (c << 4 | f), count field f
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    uint32_t x = cw[q];
    const uint32_t cbase = hi | ((uint32_t)(tid * PER + q) << 4);
    while (x) {
      const uint32_t f = (uint32_t)__builtin_ctz(x) >> 1;
      const uint32_t c = (x >> (2u * f)) & 3u;
      x &= ~(3u << (2u * f));
      const uint32_t val = cbase | f;
      s_out[run] = val;
      if (c > 1) s_out[run + 1] = val;
      if (c > 2) s_out[run + 2] = val;
      run += c;
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t p = wbase + j * kWave + lane;
    if (p < len) out[(size_t)start + p] = s_out[p];
  }
}

// the product's 2-bit placement restated (kCnt2F, 256 x 17), with the cell
// index optionally XOR-swizzled before the column map (SWZ): for uniform keys
// the cells are random, so any bijection leaves the bank statistics alone --
// this measures it
template <int BLOCK, int ITEMS, bool SWZ>
__global__ __launch_bounds__(BLOCK) void k_cnt2_lab(const uint32_t* in, uint32_t* out, const uint32_t* bstart,
                                                    const uint32_t* blen, const uint32_t* nb, uint32_t* ovf_n) {
  constexpr int PER = kCntCells / BLOCK;
  __shared__ uint32_t s_w[kCntCells + kCntCells / 2];  // cells | u16 starts (the keys over both)
  __shared__ uint32_t s_ws[BLOCK / kWave + 1];
  if (blockIdx.x >= *nb) return;
  const uint32_t b = blockIdx.x, start = bstart[b], len = blen[b];
  const int tid = threadIdx.x, lane = tid & 63, w = tid / 64;
  const uint32_t wbase = w * ITEMS * kWave;
  uint16_t* const s_st = reinterpret_cast<uint16_t*>(s_w + kCntCells);
  auto ci = [&](uint32_t c) -> uint32_t {
    if (SWZ) c ^= (c >> 6) & 63u;
    return (c % PER) * BLOCK + c / PER;
  };
  uint32_t k[ITEMS], rk[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = wbase + j * kWave + lane;
    k[j] = i < len ? load_stream(&in[(size_t)start + i]) : 0u;
  }
#pragma unroll
  for (int q = 0; q < PER; ++q) s_w[q * BLOCK + tid] = 0u;
  if (tid == 0) s_ws[BLOCK / kWave] = 0u;
  __syncthreads();
  bool ovf = false;
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (wbase + j * kWave + lane < len) {
      const uint32_t v = k[j] & 0xFFFFu, sh = 2u * (v & 15u);
      rk[j] = (atomicAdd(&s_w[ci(v >> 4)], 1u << sh) >> sh) & 3u;
      ovf |= rk[j] == 3u;
    }
  if (__any(ovf) && lane == 0) atomicAdd(&s_ws[BLOCK / kWave], 1u);
  __syncthreads();
  if (s_ws[BLOCK / kWave]) {
    if (tid == 0) atomicAdd(ovf_n, 1u);
    return;
  }
  uint32_t cnt[PER], sum = 0;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    cnt[q] = field2_sum(s_w[q * BLOCK + tid]);
    sum += cnt[q];
  }
  uint32_t total;
  uint32_t run = block_exclusive_scan<BLOCK>(sum, s_ws, total);
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    s_st[q * BLOCK + tid] = (uint16_t)run;
    run += cnt[q];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (wbase + j * kWave + lane < len) {
      const uint32_t v = k[j] & 0xFFFFu, c = ci(v >> 4);
      rk[j] += (uint32_t)s_st[c] + field2_sum(s_w[c] & ((1u << (2u * (v & 15u))) - 1u));
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

__global__ void fill(uint32_t* k, size_t n, uint32_t S) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t x = (i + 1) * 0x9E3779B97F4A7C15ull;
  x ^= x >> 29; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 32;
  k[i] = ((uint32_t)(i / S) << 16) | (uint32_t)(x & 0xFFFFu);
}

int main(int argc, char** argv) {
  const size_t n = (size_t)1 << 28;
  const uint32_t S = 4096, m = (uint32_t)(n / S);
  uint32_t *in, *out, *bs, *bl, *nb, *ov, *ovn, *ovl, *rn, *rl;
  CK(hipMalloc(&in, n * 4)); CK(hipMalloc(&out, n * 4));
  CK(hipMalloc(&bs, m * 4)); CK(hipMalloc(&bl, m * 4)); CK(hipMalloc(&nb, 4)); CK(hipMalloc(&ov, 4));
  CK(hipMalloc(&ovn, 4)); CK(hipMalloc(&ovl, m * 4)); CK(hipMalloc(&rn, 4)); CK(hipMalloc(&rl, m * 4));
  hipStream_t st; CK(hipStreamCreate(&st));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<uint32_t> hs(m), hl(m, S);
  for (uint32_t b = 0; b < m; ++b) hs[b] = b * S;
  CK(hipMemcpy(bs, hs.data(), m * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(bl, hl.data(), m * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(nb, &m, 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(fill, dim3((n + 255) / 256), dim3(256), 0, st, in, n, S);
  CK(hipStreamSynchronize(st));
  std::vector<uint32_t> h(n);
  CK(hipMemcpy(h.data(), in, n * 4, hipMemcpyDeviceToHost));
  std::vector<uint64_t> bsum(m, 0);
  std::vector<uint32_t> bx(m, 0);
  for (size_t i = 0; i < n; ++i) { bsum[i / S] += h[i]; bx[i / S] ^= h[i]; }
  struct V { std::string name; std::function<void()> launch; };
  std::vector<V> vs;
  vs.push_back({"prod 2F 256x17", [&] {
    hipLaunchKernelGGL((k_bucket_count<256, 17, RadixDigit, kCnt2F>), dim3(m), dim3(256), 0, st, in, out, bs, bl, nb,
                       m, nullptr, 16u, 0u, ov, nullptr, 0u, ovn, ovl, rn, rl); }});
  vs.push_back({"lab 2F 256x17", [&] {
    hipLaunchKernelGGL((k_cnt2_lab<256, 17, false>), dim3(m), dim3(256), 0, st, in, out, bs, bl, nb, ovn); }});
  vs.push_back({"lab 2F swz 256x17", [&] {
    hipLaunchKernelGGL((k_cnt2_lab<256, 17, true>), dim3(m), dim3(256), 0, st, in, out, bs, bl, nb, ovn); }});
  vs.push_back({"regen 256x17", [&] {
    hipLaunchKernelGGL((k_regen<256, 17, false>), dim3(m), dim3(256), 0, st, in, out, bs, bl, nb, ovn); }});
  vs.push_back({"regen 512x9", [&] {
    hipLaunchKernelGGL((k_regen<512, 9, false>), dim3(m), dim3(512), 0, st, in, out, bs, bl, nb, ovn); }});
  for (auto& v : vs) {
    std::vector<float> us;
    for (int r = 0; r < 10; ++r) {
      CK(hipMemsetAsync(ovn, 0, 4, st));
      CK(hipMemsetAsync(rn, 0, 4, st));
      CK(hipMemsetAsync(out, 0, n * 4, st));
      CK(hipEventRecord(e0, st));
      v.launch();
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 2) us.push_back(ms * 1e3f);
    }
    uint32_t novf = 0, nrty = 0;
    CK(hipMemcpy(&novf, ovn, 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(&nrty, rn, 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(h.data(), out, n * 4, hipMemcpyDeviceToHost));
    uint32_t good = 0, skipped = 0, bad = 0;
    for (uint32_t b = 0; b < m; ++b) {
      const uint32_t* p = &h[(size_t)b * S];
      uint64_t s = 0; uint32_t x = 0; bool sorted = true, zero = true;
      for (uint32_t i = 0; i < S; ++i) { s += p[i]; x ^= p[i]; if (i && p[i - 1] > p[i]) sorted = false; if (p[i]) zero = false; }
      if (zero) ++skipped; else if (sorted && s == bsum[b] && x == bx[b]) ++good; else ++bad;
    }
    std::sort(us.begin(), us.end());
    printf("%-18s median %7.1f us  best %7.1f  buckets sorted %u, left (overflow) %u, WRONG %u  (listed %u + %u)\n",
           v.name.c_str(), us[us.size() / 2], us[0], good, skipped, bad, novf, nrty);
    fflush(stdout);
  }
  return 0;
}
