// Pair bucket-sort lab (not part of libsort): the on-chip sort of the MSD
// hybrid's (u64 key, u32 payload) buckets -- configs[4]'s ~4096-pair buckets
// that share their top 16 key bits -- in isolation, exact 4096-pair buckets.
//   prod    the product kernel (k_bucket_sort FIX=16: two stable 8-bit ballot
//           steps over key bits 32..47, then runs of equal bits 32..63
//           insertion-sorted by the whole key)
//   cnt     a counting placement over bits 32..47 (4096 u64 cells of 16 3-bit
//           counts + the cell start, one LDS atomic per pair as the keys-only
//           k_bucket_count), each pair scattered to its position with its
//           bucket slot (u16); runs of equal bits 32..47 (a field count >= 2,
//           read from the cell words the thread scanned) insertion-sorted by
//           (key, slot): stable without ranks in input order
//   copy    the same LDS footprint, load + LDS write + read back + store
// Verification: sorted by key, payload (= input index) increasing inside
// equal keys, same multiset (sums).  Keys: 48 random bits, or (ties) the low
// 32 bits from 3 values, so most runs hold equal whole keys.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/pair_lab tools/pair_lab.hip
//   tools/pair_lab [filter] [inplace|ragged|inplace,ragged]
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

// counting placement of (u64 key, u32 payload) pairs on the 16 bits below
// the bucket's 16 (bits lbits-16 .. lbits-1 of the key), runs fixed by (key,
// slot).  LDS: keys | payloads | slots; the cells overlay the keys.
template <int BLOCK, int ITEMS, int WPE>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void k_pair_cnt(
    const uint64_t* kin, const uint32_t* vin, uint64_t* kout, uint32_t* vout, const uint32_t* bstart,
    const uint32_t* blen, const uint32_t* nb, uint32_t lbits, uint32_t* ovf_n, uint32_t* ovf_list) {
  constexpr int CAP = BLOCK * ITEMS, PER = kCntCells / BLOCK;
  static_assert(CAP * 8 >= kCntCells * 8, "cells overlay the keys");
  __shared__ uint64_t s_k[CAP];
  __shared__ uint32_t s_v[CAP];
  __shared__ uint16_t s_i[CAP];
  __shared__ uint32_t s_ws[BLOCK / kWave];
  if (blockIdx.x >= *nb) return;
  const uint32_t b = blockIdx.x, start = bstart[b], len = blen[b];
  const int tid = threadIdx.x, lane = tid & 63, w = tid / 64;
  const uint32_t wbase = w * ITEMS * kWave;
  uint64_t* const cw = s_k;  // 4096 cells: 16 3-bit counts | key count (then start) << 48
  auto ci = [&](uint32_t c) -> uint32_t { return (c % PER) * BLOCK + c / PER; };
  const uint32_t fs = lbits - 16;
  uint64_t k[ITEMS];
  uint32_t v[ITEMS], rk[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = wbase + j * kWave + lane;
    k[j] = i < len ? load_stream(&kin[(size_t)start + i]) : 0ull;
    v[j] = i < len ? load_stream(&vin[(size_t)start + i]) : 0u;
  }
#pragma unroll
  for (int q = 0; q < PER; ++q) cw[q * BLOCK + tid] = 0ull;
  __syncthreads();
  bool ovf = false;
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (wbase + j * kWave + lane < len) {
      const uint32_t x = (uint32_t)(k[j] >> fs) & 0xFFFFu, sh = 3u * (x & 15u);
      const uint64_t old = atomicAdd((unsigned long long*)&cw[ci(x >> 4)], (1ull << sh) + (1ull << 48));
      rk[j] = (uint32_t)(old >> sh) & 7u;
      ovf |= rk[j] == 7u;
    }
  if (__any(ovf) && lane == 0) atomicOr((unsigned long long*)&cw[0], 1ull << 63);
  __syncthreads();
  if (cw[0] >> 63) {
    if (tid == 0) ovf_list[atomicAdd(ovf_n, 1u)] = b;
    return;
  }
  uint64_t c[PER];
  uint32_t sum = 0;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    c[q] = cw[q * BLOCK + tid];
    sum += (uint32_t)(c[q] >> 48);
  }
  uint32_t total;
  uint32_t run = block_exclusive_scan<BLOCK>(sum, s_ws, total);
  uint32_t cst[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    cst[q] = run;
    cw[q * BLOCK + tid] = (c[q] & 0xFFFFFFFFFFFFull) | ((uint64_t)run << 48);
    run += (uint32_t)(c[q] >> 48);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (wbase + j * kWave + lane < len) {
      const uint32_t x = (uint32_t)(k[j] >> fs) & 0xFFFFu;
      const uint64_t cc = cw[ci(x >> 4)];
      rk[j] += (uint32_t)(cc >> 48) + field3_sum(cc & ((1ull << (3u * (x & 15u))) - 1ull));
    }
  __syncthreads();  // the pairs take the cells' place
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (wbase + j * kWave + lane < len) {
      s_k[rk[j]] = k[j];
      s_v[rk[j]] = v[j];
      s_i[rk[j]] = (uint16_t)(wbase + j * kWave + lane);
    }
  __syncthreads();
  // runs: the thread's cells are c = tid * PER + q, at positions cst[q]..;
  // a field with count >= 2 is a run of equal bits fs..fs+15
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    constexpr uint64_t B0 = 0x249249249249ull;
    const uint64_t f = c[q] & 0xFFFFFFFFFFFFull;
    // fields whose count >= 2: bit 1 or bit 2 of the field set
    uint64_t m = ((f >> 1) | (f >> 2)) & B0;
    while (m) {
      const uint32_t r = (uint32_t)__builtin_ctzll(m) / 3u;
      m &= m - 1;
      const uint32_t L = (uint32_t)(f >> (3u * r)) & 7u;
      const uint32_t p = cst[q] + field3_sum(f & ((1ull << (3u * r)) - 1ull));
      for (uint32_t a = 1; a < L; ++a) {
        const uint64_t xk = s_k[p + a];
        const uint32_t xv = s_v[p + a];
        const uint16_t xi = s_i[p + a];
        uint32_t z = a;
        while (z > 0) {
          const uint64_t yk = s_k[p + z - 1];
          if (yk < xk || (yk == xk && s_i[p + z - 1] < xi)) break;
          s_k[p + z] = yk;
          s_v[p + z] = s_v[p + z - 1];
          s_i[p + z] = s_i[p + z - 1];
          --z;
        }
        s_k[p + z] = xk;
        s_v[p + z] = xv;
        s_i[p + z] = xi;
      }
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t p = wbase + j * kWave + lane;
    if (p < len) {
      kout[(size_t)start + p] = s_k[p];
      vout[(size_t)start + p] = s_v[p];
    }
  }
}

// cnt2: the same placement with 10 B of LDS per pair instead of 14: keys and
// slots are placed (cells over the keys); after the runs are fixed the keys
// are written out, then the payloads are put at their INPUT slots over the
// key array and gathered through the slots (vout[p] = s_v[s_i[p]]).
template <int BLOCK, int ITEMS, int WPE>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void k_pair_cnt2(
    const uint64_t* kin, const uint32_t* vin, uint64_t* kout, uint32_t* vout, const uint32_t* bstart,
    const uint32_t* blen, const uint32_t* nb, uint32_t lbits, uint32_t* ovf_n, uint32_t* ovf_list) {
  constexpr int CAP = BLOCK * ITEMS, PER = kCntCells / BLOCK;
  static_assert(CAP >= kCntCells, "cells overlay the keys");
  __shared__ uint64_t s_k[CAP];
  __shared__ uint16_t s_i[CAP];
  __shared__ uint32_t s_ws[BLOCK / kWave];
  if (blockIdx.x >= *nb) return;
  const uint32_t b = blockIdx.x, start = bstart[b], len = blen[b];
  const int tid = threadIdx.x, lane = tid & 63, w = tid / 64;
  const uint32_t wbase = w * ITEMS * kWave;
  uint64_t* const cw = s_k;
  auto ci = [&](uint32_t c) -> uint32_t { return (c % PER) * BLOCK + c / PER; };
  const uint32_t fs = lbits - 16;
  uint64_t k[ITEMS];
  uint32_t v[ITEMS], rk[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = wbase + j * kWave + lane;
    k[j] = i < len ? load_stream(&kin[(size_t)start + i]) : 0ull;
    v[j] = i < len ? load_stream(&vin[(size_t)start + i]) : 0u;
  }
#pragma unroll
  for (int q = 0; q < PER; ++q) cw[q * BLOCK + tid] = 0ull;
  __syncthreads();
  bool ovf = false;
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (wbase + j * kWave + lane < len) {
      const uint32_t x = (uint32_t)(k[j] >> fs) & 0xFFFFu, sh = 3u * (x & 15u);
      const uint64_t old = atomicAdd((unsigned long long*)&cw[ci(x >> 4)], (1ull << sh) + (1ull << 48));
      rk[j] = (uint32_t)(old >> sh) & 7u;
      ovf |= rk[j] == 7u;
    }
  if (__any(ovf) && lane == 0) atomicOr((unsigned long long*)&cw[0], 1ull << 63);
  __syncthreads();
  if (cw[0] >> 63) {
    if (tid == 0) ovf_list[atomicAdd(ovf_n, 1u)] = b;
    return;
  }
  uint64_t c[PER];
  uint32_t sum = 0;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    c[q] = cw[q * BLOCK + tid];
    sum += (uint32_t)(c[q] >> 48);
  }
  uint32_t total;
  uint32_t run = block_exclusive_scan<BLOCK>(sum, s_ws, total);
  uint32_t cst[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    cst[q] = run;
    cw[q * BLOCK + tid] = (c[q] & 0xFFFFFFFFFFFFull) | ((uint64_t)run << 48);
    run += (uint32_t)(c[q] >> 48);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (wbase + j * kWave + lane < len) {
      const uint32_t x = (uint32_t)(k[j] >> fs) & 0xFFFFu;
      const uint64_t cc = cw[ci(x >> 4)];
      rk[j] += (uint32_t)(cc >> 48) + field3_sum(cc & ((1ull << (3u * (x & 15u))) - 1ull));
    }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (wbase + j * kWave + lane < len) {
      s_k[rk[j]] = k[j];
      s_i[rk[j]] = (uint16_t)(wbase + j * kWave + lane);
    }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    constexpr uint64_t B0 = 0x249249249249ull;
    const uint64_t f = c[q] & 0xFFFFFFFFFFFFull;
    uint64_t m = ((f >> 1) | (f >> 2)) & B0;
    while (m) {
      const uint32_t r = (uint32_t)__builtin_ctzll(m) / 3u;
      m &= m - 1;
      const uint32_t L = (uint32_t)(f >> (3u * r)) & 7u;
      const uint32_t p = cst[q] + field3_sum(f & ((1ull << (3u * r)) - 1ull));
      for (uint32_t a = 1; a < L; ++a) {
        const uint64_t xk = s_k[p + a];
        const uint16_t xi = s_i[p + a];
        uint32_t z = a;
        while (z > 0) {
          const uint64_t yk = s_k[p + z - 1];
          if (yk < xk || (yk == xk && s_i[p + z - 1] < xi)) break;
          s_k[p + z] = yk;
          s_i[p + z] = s_i[p + z - 1];
          --z;
        }
        s_k[p + z] = xk;
        s_i[p + z] = xi;
      }
    }
  }
  __syncthreads();
  uint32_t sl[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t p = wbase + j * kWave + lane;
    if (p < len) {
      kout[(size_t)start + p] = s_k[p];
      sl[j] = s_i[p];
    }
  }
  __syncthreads();
  uint32_t* const s_v = reinterpret_cast<uint32_t*>(s_k);
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) s_v[wbase + j * kWave + lane] = v[j];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t p = wbase + j * kWave + lane;
    if (p < len) vout[(size_t)start + p] = s_v[sl[j]];
  }
}

// cnt3: cnt2 with the key and its slot packed into ONE u64 in LDS: the
// bucket's pairs share the key bits above lbits (48), so p = (key's low 48
// bits << 16) | slot orders exactly as (key, slot) -- one random 8-byte store
// per pair instead of 8 + 2, the run fix-up compares and moves one word, and
// LDS is 8 B per slot.
template <int BLOCK, int ITEMS, int WPE>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void k_pair_cnt3(
    const uint64_t* kin, const uint32_t* vin, uint64_t* kout, uint32_t* vout, const uint32_t* bstart,
    const uint32_t* blen, const uint32_t* nb, uint32_t lbits, uint32_t* ovf_n, uint32_t* ovf_list) {
  constexpr int CAP = BLOCK * ITEMS, PER = kCntCells / BLOCK;
  static_assert(CAP >= kCntCells, "cells overlay the keys");
  __shared__ uint64_t s_p[CAP];
  __shared__ uint32_t s_ws[BLOCK / kWave];
  if (blockIdx.x >= *nb) return;
  const uint32_t b = blockIdx.x, start = bstart[b], len = blen[b];
  const int tid = threadIdx.x, lane = tid & 63, w = tid / 64;
  const uint32_t wbase = w * ITEMS * kWave;
  uint64_t* const cw = s_p;
  auto ci = [&](uint32_t c) -> uint32_t { return (c % PER) * BLOCK + c / PER; };
  const uint32_t fs = lbits - 16;
  const uint64_t lmask = (1ull << lbits) - 1ull;
  uint64_t k[ITEMS];
  uint32_t v[ITEMS], rk[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = wbase + j * kWave + lane;
    k[j] = i < len ? load_stream(&kin[(size_t)start + i]) : 0ull;
    v[j] = i < len ? load_stream(&vin[(size_t)start + i]) : 0u;
  }
  const uint64_t khi = kin[start] & ~lmask;  // the bits every pair of the bucket shares
#pragma unroll
  for (int q = 0; q < PER; ++q) cw[q * BLOCK + tid] = 0ull;
  __syncthreads();
  bool ovf = false;
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (wbase + j * kWave + lane < len) {
      const uint32_t x = (uint32_t)(k[j] >> fs) & 0xFFFFu, sh = 3u * (x & 15u);
      const uint64_t old = atomicAdd((unsigned long long*)&cw[ci(x >> 4)], (1ull << sh) + (1ull << 48));
      rk[j] = (uint32_t)(old >> sh) & 7u;
      ovf |= rk[j] == 7u;
    }
  if (__any(ovf) && lane == 0) atomicOr((unsigned long long*)&cw[0], 1ull << 63);
  __syncthreads();
  if (cw[0] >> 63) {
    if (tid == 0) ovf_list[atomicAdd(ovf_n, 1u)] = b;
    return;
  }
  uint64_t c[PER];
  uint32_t sum = 0;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    c[q] = cw[q * BLOCK + tid];
    sum += (uint32_t)(c[q] >> 48);
  }
  uint32_t total;
  uint32_t run = block_exclusive_scan<BLOCK>(sum, s_ws, total);
  uint32_t cst[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    cst[q] = run;
    cw[q * BLOCK + tid] = (c[q] & 0xFFFFFFFFFFFFull) | ((uint64_t)run << 48);
    run += (uint32_t)(c[q] >> 48);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (wbase + j * kWave + lane < len) {
      const uint32_t x = (uint32_t)(k[j] >> fs) & 0xFFFFu;
      const uint64_t cc = cw[ci(x >> 4)];
      rk[j] += (uint32_t)(cc >> 48) + field3_sum(cc & ((1ull << (3u * (x & 15u))) - 1ull));
    }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (wbase + j * kWave + lane < len) s_p[rk[j]] = ((k[j] & lmask) << 16) | (uint64_t)(wbase + j * kWave + lane);
  __syncthreads();
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    constexpr uint64_t B0 = 0x249249249249ull;
    const uint64_t f = c[q] & 0xFFFFFFFFFFFFull;
    uint64_t m = ((f >> 1) | (f >> 2)) & B0;
    while (m) {
      const uint32_t r = (uint32_t)__builtin_ctzll(m) / 3u;
      m &= m - 1;
      const uint32_t L = (uint32_t)(f >> (3u * r)) & 7u;
      const uint32_t p = cst[q] + field3_sum(f & ((1ull << (3u * r)) - 1ull));
      for (uint32_t a = 1; a < L; ++a) {
        const uint64_t x = s_p[p + a];
        uint32_t z = a;
        while (z > 0 && s_p[p + z - 1] > x) {
          s_p[p + z] = s_p[p + z - 1];
          --z;
        }
        s_p[p + z] = x;
      }
    }
  }
  __syncthreads();
  uint32_t sl[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t pos = wbase + j * kWave + lane;
    sl[j] = 0u;
    if (pos < len) {
      const uint64_t x = s_p[pos];
      kout[(size_t)start + pos] = khi | (x >> 16);
      sl[j] = (uint32_t)x & 0xFFFFu;
    }
  }
  __syncthreads();
  uint32_t* const s_v = reinterpret_cast<uint32_t*>(s_p);
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) s_v[wbase + j * kWave + lane] = v[j];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t pos = wbase + j * kWave + lane;
    if (pos < len) vout[(size_t)start + pos] = s_v[sl[j]];
  }
}

// copy floor of cnt2's footprint (10 B per pair)
template <int BLOCK, int ITEMS>
__global__ __launch_bounds__(BLOCK) void k_pair_copy2(const uint64_t* kin, const uint32_t* vin, uint64_t* kout,
                                                      uint32_t* vout, const uint32_t* bstart, const uint32_t* blen,
                                                      const uint32_t* nb) {
  constexpr int CAP = BLOCK * ITEMS;
  __shared__ uint64_t s_k[CAP];
  __shared__ uint16_t s_i[CAP];
  if (blockIdx.x >= *nb) return;
  const uint32_t b = blockIdx.x, start = bstart[b], len = blen[b];
  const int tid = threadIdx.x, lane = tid & 63, w = tid / 64;
  const uint32_t wbase = w * ITEMS * kWave;
  uint64_t k[ITEMS];
  uint32_t v[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = wbase + j * kWave + lane;
    k[j] = i < len ? load_stream(&kin[(size_t)start + i]) : 0ull;
    v[j] = i < len ? load_stream(&vin[(size_t)start + i]) : 0u;
  }
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = wbase + j * kWave + lane;
    s_k[(i * 33) % CAP] = k[j];
    s_i[(i * 33) % CAP] = (uint16_t)i;
  }
  __syncthreads();
  uint32_t sl[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t p = wbase + j * kWave + lane;
    if (p < len) kout[(size_t)start + p] = s_k[p];
    sl[j] = s_i[p];
  }
  __syncthreads();
  uint32_t* const s_v = reinterpret_cast<uint32_t*>(s_k);
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) s_v[wbase + j * kWave + lane] = v[j];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t p = wbase + j * kWave + lane;
    if (p < len) vout[(size_t)start + p] = s_v[sl[j] % CAP];
  }
}

template <int BLOCK, int ITEMS>
__global__ __launch_bounds__(BLOCK) void k_pair_copy(const uint64_t* kin, const uint32_t* vin, uint64_t* kout,
                                                     uint32_t* vout, const uint32_t* bstart, const uint32_t* blen,
                                                     const uint32_t* nb) {
  constexpr int CAP = BLOCK * ITEMS;
  __shared__ uint64_t s_k[CAP];
  __shared__ uint32_t s_v[CAP];
  __shared__ uint16_t s_i[CAP];
  if (blockIdx.x >= *nb) return;
  const uint32_t b = blockIdx.x, start = bstart[b], len = blen[b];
  const int tid = threadIdx.x, lane = tid & 63, w = tid / 64;
  const uint32_t wbase = w * ITEMS * kWave;
  uint64_t k[ITEMS];
  uint32_t v[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = wbase + j * kWave + lane;
    k[j] = i < len ? load_stream(&kin[(size_t)start + i]) : 0ull;
    v[j] = i < len ? load_stream(&vin[(size_t)start + i]) : 0u;
  }
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = wbase + j * kWave + lane;
    s_k[(i * 33) % CAP] = k[j];
    s_v[(i * 33) % CAP] = v[j];
    s_i[(i * 33) % CAP] = (uint16_t)i;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t p = wbase + j * kWave + lane;
    if (p < len) {
      kout[(size_t)start + p] = s_k[p] + s_i[p];
      vout[(size_t)start + p] = s_v[p];
    }
  }
}

// one block per bucket: keys (bucket << 48) | 48 random bits, payload = index
__global__ void fill(uint64_t* k, uint32_t* v, const uint32_t* bs, const uint32_t* bl, int ties) {
  const uint32_t b = blockIdx.x;
  for (uint32_t i = bs[b] + threadIdx.x; i < bs[b] + bl[b]; i += blockDim.x) {
    uint64_t x = (i + 1ull) * 0x9E3779B97F4A7C15ull;
    x ^= x >> 29; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 32; x *= 0x94D049BB133111EBull; x ^= x >> 31;
    uint64_t lo = x & 0xFFFFFFFFFFFFull;
    if (ties) lo = (lo & 0xFFFF00000000ull) | (lo % 3u);
    k[i] = ((uint64_t)b << 48) | lo;
    v[i] = i;
  }
}

int main(int argc, char** argv) {
  const size_t n = (size_t)1 << 28;
  const uint32_t S = 4096, m = (uint32_t)(n / S);
  uint64_t *kin, *kout;
  uint32_t *vin, *vout, *bs, *bl, *nb, *ov, *ovn, *ovl;
  CK(hipMalloc(&kin, n * 8)); CK(hipMalloc(&kout, n * 8));
  CK(hipMalloc(&vin, n * 4)); CK(hipMalloc(&vout, n * 4));
  CK(hipMalloc(&bs, m * 4)); CK(hipMalloc(&bl, m * 4)); CK(hipMalloc(&nb, 4)); CK(hipMalloc(&ov, 4));
  CK(hipMalloc(&ovn, 4)); CK(hipMalloc(&ovl, m * 4));
  hipStream_t st; CK(hipStreamCreate(&st));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  // modes (argv[2]): "inplace" sorts kin/vin in place (refilled before each
  // run, as the product's bucket phase does), "ragged" gives the buckets
  // lengths 4096 +- up to 192 (pairwise, so the total stays 2^28) and
  // starts off 4096-alignment, as a sort's 16-bit buckets are
  const std::string mode = argc > 2 ? argv[2] : "";
  const bool inplace = mode.find("inplace") != std::string::npos, ragged = mode.find("ragged") != std::string::npos;
  std::vector<uint32_t> hs(m), hl(m, S);
  if (ragged)
    for (uint32_t b = 0; b + 1 < m; b += 2) {
      const uint32_t d = (b * 2654435761u >> 7) % 385u;
      hl[b] = S - 192 + d;
      hl[b + 1] = S + 192 - d;
    }
  for (uint32_t b = 0, at = 0; b < m; ++b) hs[b] = at, at += hl[b];
  CK(hipMemcpy(bs, hs.data(), m * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(bl, hl.data(), m * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(nb, &m, 4, hipMemcpyHostToDevice));
  uint64_t* ko = inplace ? kin : kout;
  uint32_t* vo = inplace ? vin : vout;
  struct V { std::string name; bool check; std::function<void()> launch; };
  std::vector<V> vs;
  vs.push_back({"prod 512x9", true, [&] {
    hipLaunchKernelGGL((k_bucket_sort<8, 512, 9, RadixDigit, uint64_t, uint32_t, 16>), dim3(m), dim3(512), 0, st,
                       kin, ko, vin, vo, bs, bl, nb, m, nullptr, 48u, 0u, ov, nullptr, 0u); }});
  vs.push_back({"pairs-prod 1024x5", true, [&] {
    CK(hipMemsetAsync(ovn, 0, 4, st));
    hipLaunchKernelGGL((k_bucket_pairs<1024, 5, RadixDigit>), dim3(m), dim3(1024), 0, st, kin, ko, vin, vo, bs, bl, nb,
                       m, nullptr, 48u, 0ull, ov, nullptr, 0u, ovn, ovl); }});
#define CNT(B, I, W) vs.push_back({"cnt " #B "x" #I " wpe" #W, true, [&] {                                   \
    CK(hipMemsetAsync(ovn, 0, 4, st));                                                                          \
    hipLaunchKernelGGL((k_pair_cnt<B, I, W>), dim3(m), dim3(B), 0, st, kin, vin, ko, vo, bs, bl, nb, 48u, ovn, ovl); }});
  CNT(1024, 5, 1)
#define CNT2(B, I, W) vs.push_back({"cnt2 " #B "x" #I " wpe" #W, true, [&] {                                 \
    CK(hipMemsetAsync(ovn, 0, 4, st));                                                                          \
    hipLaunchKernelGGL((k_pair_cnt2<B, I, W>), dim3(m), dim3(B), 0, st, kin, vin, ko, vo, bs, bl, nb, 48u, ovn, ovl); }});
  CNT2(1024, 5, 1)
#define CNT3(B, I, W) vs.push_back({"cnt3 " #B "x" #I " wpe" #W, true, [&] {                                 \
    CK(hipMemsetAsync(ovn, 0, 4, st));                                                                          \
    hipLaunchKernelGGL((k_pair_cnt3<B, I, W>), dim3(m), dim3(B), 0, st, kin, vin, ko, vo, bs, bl, nb, 48u, ovn, ovl); }});
  CNT3(1024, 5, 1) CNT3(1024, 5, 8) CNT3(512, 9, 1) CNT3(512, 9, 8) CNT3(256, 17, 1)
  vs.push_back({"copy2 512x9", false, [&] {
    hipLaunchKernelGGL((k_pair_copy2<512, 9>), dim3(m), dim3(512), 0, st, kin, vin, ko, vo, bs, bl, nb); }});
  vs.push_back({"copy2 1024x5", false, [&] {
    hipLaunchKernelGGL((k_pair_copy2<1024, 5>), dim3(m), dim3(1024), 0, st, kin, vin, ko, vo, bs, bl, nb); }});
  vs.push_back({"copy 512x9", false, [&] {
    hipLaunchKernelGGL((k_pair_copy<512, 9>), dim3(m), dim3(512), 0, st, kin, vin, ko, vo, bs, bl, nb); }});
  const char* filt = argc > 1 ? argv[1] : nullptr;
  std::vector<uint64_t> hk(n);
  std::vector<uint32_t> hv(n);
  for (int ties = 0; ties < 2; ++ties) {
    auto refill = [&] {
      hipLaunchKernelGGL(fill, dim3(m), dim3(256), 0, st, kin, vin, bs, bl, ties);
      CK(hipStreamSynchronize(st));
    };
    refill();
    for (auto& v : vs) {
      if (filt && v.name.find(filt) == std::string::npos) continue;
      std::vector<float> us;
      CK(hipMemsetAsync(ovn, 0, 4, st));
      for (int r = 0; r < 10; ++r) {
        if (inplace) refill();
        CK(hipEventRecord(e0, st));
        v.launch();
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 2) us.push_back(ms * 1e3f);
      }
      uint32_t novf = 0;
      CK(hipMemcpy(&novf, ovn, 4, hipMemcpyDeviceToHost));
      const char* verdict = "-";
      if (v.check) {
        CK(hipMemcpy(hk.data(), ko, n * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hv.data(), vo, n * 4, hipMemcpyDeviceToHost));
        bool ok = true;
        uint64_t sk = 0, sv = 0;
        for (size_t i = 0; i < n; ++i) {
          sk += hk[i]; sv += hv[i];
          if (i && (hk[i - 1] > hk[i] || (hk[i - 1] == hk[i] && hv[i - 1] >= hv[i]))) ok = false;
        }
        if (inplace) refill();
        // the input's sums (keys and indices)
        uint64_t ek = 0, ev = 0;
        std::vector<uint64_t> ik(n);
        CK(hipMemcpy(ik.data(), kin, n * 8, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < n; ++i) { ek += ik[i]; ev += (uint32_t)i; }
        verdict = (ok && sk == ek && sv == ev) ? "sorted+stable" : (novf ? "ovf-listed" : "WRONG");
      }
      std::sort(us.begin(), us.end());
      const float med = us[us.size() / 2];
      printf("%-22s ties=%d: median %7.1f us  best %7.1f  %5.0f GB/s  ovf %u  %s\n", v.name.c_str(), ties, med, us[0],
             24.0 * n / (med * 1e-6) / 1e9, novf, verdict);
      fflush(stdout);
    }
  }
  return 0;
}
