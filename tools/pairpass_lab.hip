// Pair-pass lab (not part of libsort): the stable 8-bit pass of (u64 key, u32
// payload) pairs -- configs[4]'s two digit passes -- in isolation, 2^28 pairs,
// run offsets precomputed on the host (as the count kernel + column scan give
// them).  Variants, each checked bit-exact against the product kernel
// (k_tile_pass<8, 512, 16, u64, u32>, 8192-pair tiles, payloads staged
// through the key buffer):
//   prod         the product kernel (one block per tile)
//   pf           persistent blocks (2 per CU), each walking its XCD's tiles;
//                the next tile's keys are loaded as soon as this tile's keys
//                sit in LDS and its payloads once this tile's payloads do, so
//                the loads are in flight through the store phases
//   copy         the same tiles loaded and stored in place (floor)
// Each with and without the next-digit byte stream (dout) the product's
// depth 0 writes.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -o tools/pairpass_lab tools/pairpass_lab.hip
//   tools/pairpass_lab [filter]
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

// gofs[t * 256 + d]: where tile t's run of digit d starts in the output
template <int BLOCK, int ITEMS, bool DOUT, int KPF>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_pair_pass_pf(const uint64_t* __restrict__ kin, uint64_t* __restrict__ kout,
                                                        const uint32_t* __restrict__ vin, uint32_t* __restrict__ vout,
                                                        uint8_t* __restrict__ dout, const uint32_t* __restrict__ gofs,
                                                        uint32_t T, RadixDigit op, RadixDigit op_next) {
  constexpr int RADIX = 256, WAVES = BLOCK / kWave, TILE = BLOCK * ITEMS, WSPAN = ITEMS * kWave;
  __shared__ uint64_t s_keys[TILE];
  __shared__ WaveCount s_whist[WAVES][RADIX];
  __shared__ uint32_t s_ob[RADIX];
  __shared__ uint32_t s_wsum[WAVES];
  const int tid = threadIdx.x, lane = tid & 63, w = tid / 64;
  const uint32_t wbase = w * WSPAN;
  // this block's tiles: XCD x = blockIdx % 8 owns a contiguous range, its
  // blocks take every (G / 8)-th tile of it
  const uint32_t G = gridDim.x, x = blockIdx.x & 7u, gx = G >> 3, i0 = blockIdx.x >> 3;
  const uint32_t q = T >> 3, r = T & 7u;
  const uint32_t lo = x * q + min(x, r), hi = lo + q + (x < r ? 1u : 0u);
  uint32_t t = lo + i0;
  if (t >= hi) return;
  uint64_t k[ITEMS];
  uint32_t v[ITEMS];
  {
    const uint64_t* kp = kin + (size_t)t * TILE + wbase + lane;
    const uint32_t* vp = vin + (size_t)t * TILE + wbase + lane;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) k[j] = load_stream(&kp[j * kWave]);
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) v[j] = load_stream(&vp[j * kWave]);
  }
  uint32_t go = tid < RADIX ? gofs[(size_t)t * RADIX + tid] : 0u;
  for (;;) {
    const uint32_t tn = t + gx;
    const bool more = tn < hi;
    for (int d = lane; d < RADIX; d += kWave) s_whist[w][d] = 0u;
    uint32_t rk[ITEMS];
    rank_items_t<8, true, ITEMS>(k, rk, s_whist[w], 0u, wbase, lane, op);
    __syncthreads();
    uint32_t cnt_d = 0;
    if (tid < RADIX) {
#pragma unroll
      for (int i = 0; i < WAVES; ++i) cnt_d += s_whist[i][tid];
    }
    uint32_t total;
    const uint32_t excl = block_exclusive_scan<BLOCK>(cnt_d, s_wsum, total);
    if (tid < RADIX) {
      uint32_t run = excl;
#pragma unroll
      for (int i = 0; i < WAVES; ++i) {
        const uint32_t c = s_whist[i][tid];
        s_whist[i][tid] = (WaveCount)run;
        run += c;
      }
      s_ob[tid] = go - excl;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t pos = s_whist[w][op(k[j])] + rk[j];
      s_keys[pos] = k[j];
      rk[j] = pos;
    }
    // the next tile's keys (and run offsets) while this tile is written
    if (KPF && more) {
      const uint64_t* kp = kin + (size_t)tn * TILE + wbase + lane;
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) k[j] = load_stream(&kp[j * kWave]);
      go = tid < RADIX ? gofs[(size_t)tn * RADIX + tid] : 0u;
    }
    __syncthreads();
    uint32_t obk[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t i = tid + j * BLOCK;
      const uint64_t kk = s_keys[i];
      obk[j] = s_ob[op(kk)];
      kout[obk[j] + i] = kk;
      if constexpr (DOUT) dout[obk[j] + i] = (uint8_t)op_next(kk);
    }
    __syncthreads();
    uint32_t* const s_v = reinterpret_cast<uint32_t*>(s_keys);
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) s_v[rk[j]] = v[j];
    if (KPF && more) {
      const uint32_t* vp = vin + (size_t)tn * TILE + wbase + lane;
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) v[j] = load_stream(&vp[j * kWave]);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t i = tid + j * BLOCK;
      vout[obk[j] + i] = s_v[i];
    }
    if (!more) break;
    if (!KPF) {
      const uint64_t* kp = kin + (size_t)tn * TILE + wbase + lane;
      const uint32_t* vp = vin + (size_t)tn * TILE + wbase + lane;
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) k[j] = load_stream(&kp[j * kWave]);
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) v[j] = load_stream(&vp[j * kWave]);
      go = tid < RADIX ? gofs[(size_t)tn * RADIX + tid] : 0u;
    }
    __syncthreads();  // (s_v read before the next tile's scatter; s_ob before its rewrite)
    t = tn;
  }
}

// TPB consecutive tiles per block, the tile loop fully unrolled (straight-line
// code: the register allocation of the one-tile kernel plus the prefetched
// next keys / payloads), prefetch as in k_pair_pass_pf
// ABL (ablations, wrong results): 1 = order-free LDS-atomic rank instead of
// the stable ballot rank, 2 = no key stores, 3 = no payload staging / stores
template <int BLOCK, int ITEMS, bool DOUT, int TPB, int ABL = 0>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_pair_pass_tpb(const uint64_t* __restrict__ kin, uint64_t* __restrict__ kout,
                                                         const uint32_t* __restrict__ vin, uint32_t* __restrict__ vout,
                                                         uint8_t* __restrict__ dout, const uint32_t* __restrict__ gofs,
                                                         RadixDigit op, RadixDigit op_next) {
  constexpr int RADIX = 256, WAVES = BLOCK / kWave, TILE = BLOCK * ITEMS, WSPAN = ITEMS * kWave;
  __shared__ uint64_t s_keys[TILE];
  __shared__ WaveCount s_whist[WAVES][RADIX];
  __shared__ uint32_t s_ob[RADIX];
  __shared__ uint32_t s_wsum[WAVES];
  const int tid = threadIdx.x, lane = tid & 63, w = tid / 64;
  const uint32_t wbase = w * WSPAN;
  const uint32_t t0 = xcd_tile_of_block() * TPB;
  uint64_t k[ITEMS];
  uint32_t v[ITEMS];
  {
    const uint64_t* kp = kin + (size_t)t0 * TILE + wbase + lane;
    const uint32_t* vp = vin + (size_t)t0 * TILE + wbase + lane;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) k[j] = load_stream(&kp[j * kWave]);
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) v[j] = load_stream(&vp[j * kWave]);
  }
  uint32_t go = tid < RADIX ? gofs[(size_t)t0 * RADIX + tid] : 0u;
#pragma unroll
  for (int s = 0; s < TPB; ++s) {
    const uint32_t tn = t0 + s + 1;
    const bool more = s + 1 < TPB;
    if (s) __syncthreads();
    for (int d = lane; d < RADIX; d += kWave) s_whist[w][d] = 0u;
    uint32_t rk[ITEMS];
    if constexpr (ABL == 1) {
      uint32_t* const cw = reinterpret_cast<uint32_t*>(s_keys) + w * RADIX;  // (free until the scatter)
      for (int d = lane; d < RADIX; d += kWave) cw[d] = 0u;
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) rk[j] = atomicAdd(&cw[op(k[j])], 1u);
      for (int d = lane; d < RADIX; d += kWave) s_whist[w][d] = (WaveCount)cw[d];
    } else {
      rank_items_t<8, true, ITEMS>(k, rk, s_whist[w], 0u, wbase, lane, op);
    }
    __syncthreads();
    uint32_t cnt_d = 0;
    if (tid < RADIX) {
#pragma unroll
      for (int i = 0; i < WAVES; ++i) cnt_d += s_whist[i][tid];
    }
    uint32_t total;
    const uint32_t excl = block_exclusive_scan<BLOCK>(cnt_d, s_wsum, total);
    if (tid < RADIX) {
      uint32_t run = excl;
#pragma unroll
      for (int i = 0; i < WAVES; ++i) {
        const uint32_t c = s_whist[i][tid];
        s_whist[i][tid] = (WaveCount)run;
        run += c;
      }
      s_ob[tid] = go - excl;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t pos = s_whist[w][op(k[j])] + rk[j];
      s_keys[pos] = k[j];
      rk[j] = pos;
    }
    if (more) {
      const uint64_t* kp = kin + (size_t)tn * TILE + wbase + lane;
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) k[j] = load_stream(&kp[j * kWave]);
      go = tid < RADIX ? gofs[(size_t)tn * RADIX + tid] : 0u;
    }
    __syncthreads();
    uint32_t obk[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t i = tid + j * BLOCK;
      const uint64_t kk = s_keys[i];
      obk[j] = s_ob[op(kk)];
      if constexpr (ABL == 2) asm volatile("" ::"v"(kk), "v"(obk[j]));
      else kout[obk[j] + i] = kk;
      if constexpr (DOUT) dout[obk[j] + i] = (uint8_t)op_next(kk);
    }
    if constexpr (ABL == 3) {
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) asm volatile("" ::"v"(v[j]), "v"(rk[j]), "v"(obk[j]));
      continue;
    }
    __syncthreads();
    uint32_t* const s_v = reinterpret_cast<uint32_t*>(s_keys);
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) s_v[rk[j]] = v[j];
    if (more) {
      const uint32_t* vp = vin + (size_t)tn * TILE + wbase + lane;
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) v[j] = load_stream(&vp[j * kWave]);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t i = tid + j * BLOCK;
      vout[obk[j] + i] = s_v[i];
    }
  }
}

// floor: the same tile loads and coalesced stores of both arrays, no sort
template <int BLOCK, int ITEMS>
__global__ __launch_bounds__(BLOCK) void k_pair_copy(const uint64_t* __restrict__ kin, uint64_t* __restrict__ kout,
                                                     const uint32_t* __restrict__ vin, uint32_t* __restrict__ vout) {
  constexpr int TILE = BLOCK * ITEMS;
  const uint32_t t = xcd_tile_of_block();
  const size_t b = (size_t)t * TILE + threadIdx.x;
  uint64_t k[ITEMS];
  uint32_t v[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) k[j] = load_stream(&kin[b + j * BLOCK]);
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) v[j] = load_stream(&vin[b + j * BLOCK]);
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) kout[b + j * BLOCK] = k[j];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) vout[b + j * BLOCK] = v[j];
}

__global__ void fill(uint64_t* k, uint32_t* v, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t x = (i + 1) * 0x9E3779B97F4A7C15ull;
  x ^= x >> 29; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 32; x *= 0x94D049BB133111EBull; x ^= x >> 31;
  k[i] = x;
  v[i] = (uint32_t)i;
}

int main(int argc, char** argv) {
  const size_t n = (size_t)1 << 28;
  constexpr int TILE = 8192;
  const uint32_t T = (uint32_t)(n / TILE);
  const char* filt = argc > 1 ? argv[1] : nullptr;
  const RadixDigit op{56, 255}, opn{48, 255};
  uint64_t *kin, *kout;
  uint32_t *vin, *vout, *gofs, *gofs16, *C, *Bz, *Dz;
  uint8_t* dout;
  CK(hipMalloc(&kin, n * 8)); CK(hipMalloc(&kout, n * 8));
  CK(hipMalloc(&vin, n * 4)); CK(hipMalloc(&vout, n * 4));
  CK(hipMalloc(&dout, n));
  CK(hipMalloc(&gofs, (size_t)T * 256 * 4));
  CK(hipMalloc(&gofs16, (size_t)(T / 2) * 256 * 4));
  CK(hipMalloc(&C, (size_t)T * 256 * 4));
  CK(hipMalloc(&Bz, (size_t)T * 256 * 4));
  CK(hipMalloc(&Dz, 256 * 4));
  CK(hipMemset(Bz, 0, (size_t)T * 256 * 4));
  CK(hipMemset(Dz, 0, 256 * 4));
  hipStream_t st; CK(hipStreamCreate(&st));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, 0));
  const uint32_t cus = prop.multiProcessorCount;
  hipLaunchKernelGGL(fill, dim3((n + 255) / 256), dim3(256), 0, st, kin, vin, n);
  CK(hipStreamSynchronize(st));
  // run offsets on the host: gofs[t][d] = digit start + keys of digit d in tiles < t
  // (gofs16: the same over 16384-pair tiles)
  for (int tl : {TILE, 2 * TILE}) {
    const uint32_t T = (uint32_t)(n / tl);
    std::vector<uint64_t> hk(n);
    CK(hipMemcpy(hk.data(), kin, n * 8, hipMemcpyDeviceToHost));
    std::vector<uint32_t> cnt((size_t)T * 256, 0), g((size_t)T * 256);
    for (size_t i = 0; i < n; ++i) cnt[(i / tl) * 256 + (hk[i] >> 56)]++;
    std::vector<uint64_t> tot(256, 0);
    for (uint32_t t = 0; t < T; ++t)
      for (int d = 0; d < 256; ++d) tot[d] += cnt[(size_t)t * 256 + d];
    uint64_t run = 0;
    std::vector<uint64_t> cur(256);
    for (int d = 0; d < 256; ++d) cur[d] = run, run += tot[d];
    for (uint32_t t = 0; t < T; ++t)
      for (int d = 0; d < 256; ++d) {
        g[(size_t)t * 256 + d] = (uint32_t)cur[d];
        cur[d] += cnt[(size_t)t * 256 + d];
      }
    if (tl == TILE) {
      CK(hipMemcpy(gofs, g.data(), g.size() * 4, hipMemcpyHostToDevice));
      CK(hipMemcpy(C, g.data(), g.size() * 4, hipMemcpyHostToDevice));
    } else {
      CK(hipMemcpy(gofs16, g.data(), g.size() * 4, hipMemcpyHostToDevice));
    }
  }
  struct V { std::string name; int check; std::function<void()> launch; };
  std::vector<V> vs;
  for (int dd = 0; dd < 2; ++dd) {
    const bool D = dd == 1;
    HybridGeo geo{};
    geo.dout = D ? dout : nullptr;
    vs.push_back({std::string("prod") + (D ? " dout" : ""), 0, [=] {
      hipLaunchKernelGGL((k_tile_pass<8, 512, 16, uint64_t, uint32_t, false, RadixDigit, RadixDigit, 0>), dim3(T), dim3(512),
                         0, st, kin, kout, vin, vout, (uint32_t)n, op, opn, C, Bz, Dz, (uint32_t*)nullptr, geo); }});
#define PF(B, I, KPF, BPC)                                                                                         \
    vs.push_back({std::string("pf" #B "x" #I " kpf" #KPF " bpc" #BPC) + (D ? " dout" : ""), D ? 2 : 1, [=] {       \
      const uint32_t G = std::min<uint32_t>(T, (BPC) * cus) & ~7u;                                                 \
      if (D) hipLaunchKernelGGL((k_pair_pass_pf<B, I, true, KPF>), dim3(G), dim3(B), 0, st, kin, kout, vin, vout,  \
                                dout, gofs, T, op, opn);                                                           \
      else hipLaunchKernelGGL((k_pair_pass_pf<B, I, false, KPF>), dim3(G), dim3(B), 0, st, kin, kout, vin, vout,   \
                              dout, gofs, T, op, opn); }});
#define TPBV(N)                                                                                                    \
    vs.push_back({std::string("tpb" #N) + (D ? " dout" : ""), D ? 2 : 1, [=] {                                      \
      if (D) hipLaunchKernelGGL((k_pair_pass_tpb<512, 16, true, N>), dim3(T / N), dim3(512), 0, st, kin, kout, vin,  \
                                vout, dout, gofs, op, opn);                                                        \
      else hipLaunchKernelGGL((k_pair_pass_tpb<512, 16, false, N>), dim3(T / N), dim3(512), 0, st, kin, kout, vin,   \
                              vout, dout, gofs, op, opn); }});
    TPBV(1)
#define ABLV(A)                                                                                                    \
    vs.push_back({std::string("tpb1 ABL" #A) + (D ? " dout" : ""), -1, [=] {                                       \
      if (D) hipLaunchKernelGGL((k_pair_pass_tpb<512, 16, true, 1, A>), dim3(T), dim3(512), 0, st, kin, kout, vin,   \
                                vout, dout, gofs, op, opn);                                                        \
      else hipLaunchKernelGGL((k_pair_pass_tpb<512, 16, false, 1, A>), dim3(T), dim3(512), 0, st, kin, kout, vin,    \
                              vout, dout, gofs, op, opn); }});
    ABLV(1) ABLV(2) ABLV(3)
    // 16384-pair tiles (64-pair runs), one 1024-thread block per CU (LDS 137 KB)
    vs.push_back({std::string("t16k 1024x16") + (D ? " dout" : ""), D ? 2 : 1, [=] {
      if (D) hipLaunchKernelGGL((k_pair_pass_tpb<1024, 16, true, 1>), dim3(T / 2), dim3(1024), 0, st, kin, kout, vin,
                                vout, dout, gofs16, op, opn);
      else hipLaunchKernelGGL((k_pair_pass_tpb<1024, 16, false, 1>), dim3(T / 2), dim3(1024), 0, st, kin, kout, vin,
                              vout, dout, gofs16, op, opn); }});
  }
  vs.push_back({"copy", -1, [=] {
    hipLaunchKernelGGL((k_pair_copy<512, 16>), dim3(T), dim3(512), 0, st, kin, kout, vin, vout); }});
  // reference outputs: the product kernel with dout
  std::vector<uint64_t> rk(n), hk(n);
  std::vector<uint32_t> rv(n), hv(n);
  std::vector<uint8_t> rd(n), hd(n);
  {
    HybridGeo geo{};
    geo.dout = dout;
    hipLaunchKernelGGL((k_tile_pass<8, 512, 16, uint64_t, uint32_t, false, RadixDigit, RadixDigit, 0>), dim3(T), dim3(512),
                       0, st, kin, kout, vin, vout, (uint32_t)n, op, opn, C, Bz, Dz, (uint32_t*)nullptr, geo);
    CK(hipStreamSynchronize(st));
    CK(hipMemcpy(rk.data(), kout, n * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(rv.data(), vout, n * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(rd.data(), dout, n, hipMemcpyDeviceToHost));
    bool ok = true;
    for (size_t i = 1; i < n && ok; ++i)
      if ((rk[i - 1] >> 56) > (rk[i] >> 56) || ((rk[i - 1] >> 56) == (rk[i] >> 56) && rv[i - 1] >= rv[i])) ok = false;
    printf("product output %s\n", ok ? "stable-partitioned" : "WRONG");
  }
  for (auto& v : vs) {
    if (filt && v.name.find(filt) == std::string::npos) continue;
    std::vector<float> us;
    for (int r = 0; r < 12; ++r) {
      CK(hipMemsetAsync(kout, 0, 4096, st));
      CK(hipEventRecord(e0, st));
      v.launch();
      CK(hipGetLastError());
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1));
      if (r >= 2) us.push_back(ms * 1e3f);
    }
    const char* verdict = "-";
    if (v.check >= 0) {
      CK(hipMemcpy(hk.data(), kout, n * 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(hv.data(), vout, n * 4, hipMemcpyDeviceToHost));
      bool ok = hk == rk && hv == rv;
      if (v.check == 2) {
        CK(hipMemcpy(hd.data(), dout, n, hipMemcpyDeviceToHost));
        ok = ok && hd == rd;
      }
      verdict = ok ? "exact" : "WRONG";
    }
    std::sort(us.begin(), us.end());
    const float med = us[us.size() / 2];
    printf("%-28s median %7.1f us  best %7.1f  %5.0f GB/s  %s\n", v.name.c_str(), med, us[0], 24.0 * n / (med * 1e-6) / 1e9,
           verdict);
    fflush(stdout);
  }
  return 0;
}
