// Bucket-sort lab 2 (not part of libsort): variants of the MSD hybrid's
// keys-only bucket sort on 2^lg keys in buckets of S keys whose top 16 bits
// are the bucket index, sorted on their low `lbits` bits:
//   prod    k_bucket_sort (4-bit LSD steps, ballot ranks, atomic first step)
//   chain2  the same steps, each wave's items ranked as two independent
//           counter chains (items [0, 9) and [9, 17)), the second chain's
//           ranks offset by the first chain's per-digit totals afterwards
//   cnt12   a counting sort of the bucket by the top 12 of its lbits bits
//           (4096 LDS counters, atomic ranks), then each key placed inside
//           its cell by the cell's remaining low bits (cells hold ~1 key)
// Every variant is checked: output sorted and a permutation of the input.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/bucket_lab2 tools/bucket_lab2.hip
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

// ---- chain2: two independent counter chains per wave ------------------------
template <int BITS, int ITEMS>
__device__ __forceinline__ void rank2(const uint32_t (&k)[ITEMS], uint32_t (&rk)[ITEMS], WaveCount* rowA,
                                      WaveCount* rowB, uint32_t lane, RadixDigit op) {
  constexpr int HA = (ITEMS + 1) / 2;
  constexpr int RADIX = 1 << BITS;
  uint32_t dg[ITEMS];
  auto one = [&](int j, WaveCount* row) {
    const uint32_t d = op(k[j]);
    dg[j] = d;
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
    const uint32_t cnt = (uint32_t)(__builtin_popcount(plo) + __builtin_popcount(phi));
    const uint32_t base = row[d];
    rk[j] = base + below;
    row[d] = (WaveCount)(base + cnt);
  };
#pragma unroll
  for (int t = 0; t < HA; ++t) {
    one(t, rowA);
    if (HA + t < ITEMS) one(HA + t, rowB);
  }
#pragma unroll
  for (int j = HA; j < ITEMS; ++j) rk[j] += rowA[dg[j]];
  if (lane < (uint32_t)RADIX) rowA[lane] = (WaveCount)(rowA[lane] + rowB[lane]);
}

template <int BLOCK, int ITEMS>
__global__ __launch_bounds__(BLOCK) void k_chain2(const uint32_t* in, uint32_t* out, const uint32_t* bstart,
                                                  const uint32_t* blen, const uint32_t* nb, uint32_t lbits) {
  constexpr int BITS = 4, RADIX = 16, WAVES = BLOCK / kWave, WSPAN = ITEMS * kWave;
  __shared__ uint32_t s_keys[BLOCK * ITEMS];
  __shared__ WaveCount s_whist[WAVES][RADIX];
  __shared__ WaveCount s_rowb[WAVES][RADIX];
  __shared__ WaveCount s_off[WAVES][RADIX];
  __shared__ uint32_t s_acnt[WAVES][RADIX];
  if (blockIdx.x >= *nb) return;
  const uint32_t b = blockIdx.x, start = bstart[b], len = blen[b];
  const int tid = threadIdx.x, lane = tid & 63, w = tid / 64;
  const uint32_t wbase = w * WSPAN;
  uint32_t k[ITEMS], rk[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = wbase + j * kWave + lane;
    k[j] = i < len ? load_stream(&in[(size_t)start + i]) : 0xffffffffu;
  }
  for (uint32_t shift = 0; shift < lbits; shift += BITS) {
    const RadixDigit op{shift, 15u};
    if (shift == 0) {
      for (int d = lane; d < RADIX; d += kWave) s_acnt[w][d] = 0u;
#pragma unroll
      for (int j = 0; j < ITEMS; ++j)
        if (wbase + j * kWave + lane < len) rk[j] = atomicAdd(&s_acnt[w][op(k[j])], 1u);
      if (wbase + WSPAN > len) {
#pragma unroll
        for (int j = 0; j < ITEMS; ++j)
          if (wbase + j * kWave + lane >= len) rk[j] = atomicAdd(&s_acnt[w][op(k[j])], 1u);
      }
      for (int d = lane; d < RADIX; d += kWave) s_whist[w][d] = (WaveCount)s_acnt[w][d];
    } else {
      for (int d = lane; d < RADIX; d += kWave) {
        s_whist[w][d] = 0;
        s_rowb[w][d] = 0;
      }
      rank2<BITS, ITEMS>(k, rk, s_whist[w], s_rowb[w], lane, op);
    }
    __syncthreads();
    uint32_t col = 0, mine = 0;
    if (lane < RADIX) {
#pragma unroll
      for (int i = 0; i < WAVES; ++i) {
        const uint32_t c = s_whist[i][lane];
        col += c;
        mine += i < w ? c : 0u;
      }
    }
    uint32_t x = col;
#pragma unroll
    for (int o = 1; o < RADIX; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, RADIX);
      if ((lane & (RADIX - 1)) >= o) x += y;
    }
    if (lane < RADIX) s_off[w][lane] = (WaveCount)(x - col + mine);
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) s_keys[s_off[w][op(k[j])] + rk[j]] = k[j];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) k[j] = s_keys[wbase + j * kWave + lane];
  }
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = wbase + j * kWave + lane;
    if (i < len) out[(size_t)start + i] = k[j];
  }
}

// ---- cnt12: counting sort by the top 12 of lbits bits + in-cell placement ----
template <int BLOCK, int ITEMS, int WIN = 0, bool PF = false>
__global__ __launch_bounds__(BLOCK) void k_cnt12(const uint32_t* in, uint32_t* out, const uint32_t* bstart,
                                                 const uint32_t* blen, const uint32_t* nb, uint32_t lbits) {
  constexpr int CELLS = 4096, PER = CELLS / BLOCK, WAVES = BLOCK / kWave, WSPAN = ITEMS * kWave;
  __shared__ uint32_t s_keys[BLOCK * ITEMS];
  __shared__ uint32_t s_cnt[CELLS + 1];
  __shared__ uint32_t s_wsum[WAVES];
  const uint32_t nbk = *nb;
  uint32_t b = blockIdx.x;
  if (b >= nbk) return;
  uint32_t start = bstart[b], len = blen[b];
  const int tid = threadIdx.x, lane = tid & 63, w = tid / 64;
  const uint32_t wbase = w * WSPAN;
  const uint32_t cs = lbits > 12 ? lbits - 12 : 0;  // cell = (key & lmask) >> cs
  const uint32_t lmask = lbits >= 32 ? 0xffffffffu : (1u << lbits) - 1u;
  uint32_t k[ITEMS], rk[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = wbase + j * kWave + lane;
    k[j] = i < len ? load_stream(&in[(size_t)start + i]) : 0u;
  }
  for (;;) {
  const uint32_t b2 = PF ? b + gridDim.x : nbk;
  uint32_t kn[ITEMS], nstart = 0, nlen = 0;
  if (b2 < nbk) {
    nstart = bstart[b2];
    nlen = blen[b2];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t i = wbase + j * kWave + lane;
      kn[j] = i < nlen ? load_stream(&in[(size_t)nstart + i]) : 0u;
    }
  }
  // cell c's counter at (c % PER) * BLOCK + c / PER: a thread's PER cells
  // are one column, read and written conflict-free
  auto ci = [&](uint32_t c) -> uint32_t { return c >= (uint32_t)CELLS ? (uint32_t)CELLS : (c % PER) * BLOCK + c / PER; };
#pragma unroll
  for (int q = 0; q < PER; ++q) s_cnt[q * BLOCK + tid] = 0u;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (wbase + j * kWave + lane < len) rk[j] = atomicAdd(&s_cnt[ci((k[j] & lmask) >> cs)], 1u);
  __syncthreads();
  uint32_t c[PER], sum = 0;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    c[q] = s_cnt[q * BLOCK + tid];
    sum += c[q];
  }
  uint32_t tot;
  uint32_t run = block_exclusive_scan<BLOCK>(sum, s_wsum, tot);
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    s_cnt[q * BLOCK + tid] = run;
    run += c[q];
  }
  if (tid == 0) s_cnt[CELLS] = len;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (wbase + j * kWave + lane < len) s_keys[s_cnt[ci((k[j] & lmask) >> cs)] + rk[j]] = k[j];
  __syncthreads();
  // position p holds a key of its cell; its final place: the cell's start +
  // the cell's keys smaller than it (ties by position)
  if (WIN && cs) {
    // the cell mates within WIN positions either side, found by cell id;
    // a cell reaching the window's edge takes the full loop
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t p = wbase + j * kWave + lane;
      if (p < len) {
        const uint32_t x = s_keys[p], cx = (x & lmask) >> cs;
        uint32_t before = 0, less = 0;
        bool edge = false;
#pragma unroll
        for (int o = -WIN; o <= WIN; ++o) {
          if (o == 0) continue;
          const int q = (int)p + o;
          const uint32_t y = (q >= 0 && q < (int)len) ? s_keys[q] : ~x;
          const bool same = ((y & lmask) >> cs) == cx && q >= 0 && q < (int)len;
          before += (same && o < 0) ? 1u : 0u;
          less += same && (y < x || (y == x && o < 0)) ? 1u : 0u;
          if ((o == -WIN || o == WIN) && same) edge = true;
        }
        uint32_t fin = p - before + less;
        if (edge) {
          const uint32_t a = s_cnt[ci(cx)], e = s_cnt[ci(cx + 1)];
          uint32_t l2 = 0;
          for (uint32_t q = a; q < e; ++q) {
            const uint32_t y = s_keys[q];
            l2 += (y < x) || (y == x && q < p) ? 1u : 0u;
          }
          fin = a + l2;
        }
        out[(size_t)start + fin] = x;
      }
    }
  } else {
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t p = wbase + j * kWave + lane;
    if (p < len) {
      const uint32_t x = s_keys[p];
      uint32_t fin = p;
      if (cs) {
        const uint32_t cell = (x & lmask) >> cs;
        const uint32_t a = s_cnt[ci(cell)], e = s_cnt[ci(cell + 1)];
        uint32_t less = 0;
        for (uint32_t q = a; q < e; ++q) {
          const uint32_t y = s_keys[q];
          less += (y < x) || (y == x && q < p) ? 1u : 0u;
        }
        fin = a + less;
      }
      out[(size_t)start + fin] = x;
    }
  }
  }
  if (!(b2 < nbk)) break;
  __syncthreads();
  b = b2;
  start = nstart;
  len = nlen;
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) k[j] = kn[j];
  }
}

// ---- cntP: CBITS-bit cells, two 16-bit counters per LDS word, every item's
// in-cell placement issued together (one pass over the largest cell) --------
template <int BLOCK, int ITEMS, int CBITS>
__global__ __launch_bounds__(BLOCK) void k_cntP(const uint32_t* in, uint32_t* out, const uint32_t* bstart,
                                                const uint32_t* blen, const uint32_t* nb, uint32_t lbits) {
  constexpr int CELLS = 1 << CBITS, WORDS = CELLS / 2, PW = WORDS / BLOCK, WAVES = BLOCK / kWave;
  constexpr int WSPAN = ITEMS * kWave;
  static_assert(PW >= 1, "cells per thread");
  __shared__ uint32_t s_keys[BLOCK * ITEMS];
  __shared__ uint32_t s_c[WORDS];
  __shared__ uint32_t s_wsum[WAVES];
  if (blockIdx.x >= *nb) return;
  const uint32_t b = blockIdx.x, start = bstart[b], len = blen[b];
  const int tid = threadIdx.x, lane = tid & 63, w = tid / 64;
  const uint32_t wbase = w * WSPAN;
  const uint32_t cs = lbits > CBITS ? lbits - CBITS : 0;
  const uint32_t lmask = lbits >= 32 ? 0xffffffffu : (1u << lbits) - 1u;
  uint32_t k[ITEMS], rk[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = wbase + j * kWave + lane;
    k[j] = i < len ? load_stream(&in[(size_t)start + i]) : 0u;
  }
  auto wi = [&](uint32_t pc) -> uint32_t { return (pc % PW) * BLOCK + pc / PW; };
#pragma unroll
  for (int q = 0; q < PW; ++q) s_c[q * BLOCK + tid] = 0u;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (wbase + j * kWave + lane < len) {
      const uint32_t c = (k[j] & lmask) >> cs, sh = (c & 1u) << 4;
      rk[j] = (atomicAdd(&s_c[wi(c >> 1)], 1u << sh) >> sh) & 0xffffu;
    }
  __syncthreads();
  uint32_t wv[PW], sum = 0;
#pragma unroll
  for (int q = 0; q < PW; ++q) {
    wv[q] = s_c[q * BLOCK + tid];
    sum += (wv[q] & 0xffffu) + (wv[q] >> 16);
  }
  uint32_t tot;
  uint32_t run = block_exclusive_scan<BLOCK>(sum, s_wsum, tot);
#pragma unroll
  for (int q = 0; q < PW; ++q) {
    const uint32_t lo = wv[q] & 0xffffu;
    s_c[q * BLOCK + tid] = run | ((run + lo) << 16);
    run += lo + (wv[q] >> 16);
  }
  __syncthreads();
  auto cstart = [&](uint32_t c) -> uint32_t {
    return c >= (uint32_t)CELLS ? len : (s_c[wi(c >> 1)] >> ((c & 1u) << 4)) & 0xffffu;
  };
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (wbase + j * kWave + lane < len) s_keys[cstart((k[j] & lmask) >> cs) + rk[j]] = k[j];
  __syncthreads();
  if (!cs) {
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t p = wbase + j * kWave + lane;
      if (p < len) out[(size_t)start + p] = s_keys[p];
    }
    return;
  }
  uint32_t a[ITEMS], e[ITEMS], less[ITEMS], span = 0;
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t p = wbase + j * kWave + lane;
    k[j] = p < len ? s_keys[p] : 0u;
    const uint32_t c = (k[j] & lmask) >> cs;
    a[j] = cstart(c);
    e[j] = p < len ? cstart(c + 1) : a[j];
    less[j] = 0;
    span = e[j] - a[j] > span ? e[j] - a[j] : span;
  }
  for (uint32_t r = 0; r < span; ++r) {
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t q = a[j] + r;
      if (q < e[j]) {
        const uint32_t p = wbase + j * kWave + lane;
        const uint32_t y = s_keys[q];
        less[j] += (y < k[j]) || (y == k[j] && q < p) ? 1u : 0u;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (wbase + j * kWave + lane < len) out[(size_t)start + a[j] + less[j]] = k[j];
}

// ---- cntF: 4096 cells by the top 12 of lbits bits (12 < lbits <= 16); each
// cell one u64 holding a 3-bit count per residual value (low lbits-12 bits),
// so one atomic gives a key's rank among its equals and the scan leaves the
// cell start in the word's top 16 bits: position = start + counts of the
// smaller residuals + rank. A count reaching 7 (8+ equal keys) sends the
// bucket to the loop placement (cnt12's) ------------------------------------

template <int BLOCK, int ITEMS>
__global__ __launch_bounds__(BLOCK) void k_cntF(const uint32_t* in, uint32_t* out, const uint32_t* bstart,
                                                const uint32_t* blen, const uint32_t* nb, uint32_t lbits) {
  constexpr int CELLS = 4096, PER = CELLS / BLOCK, WAVES = BLOCK / kWave, WSPAN = ITEMS * kWave;
  __shared__ uint32_t s_keys[BLOCK * ITEMS];
  __shared__ uint64_t s_w[CELLS];
  __shared__ uint32_t s_wsum[WAVES];
  __shared__ uint32_t s_ovf;
  if (blockIdx.x >= *nb) return;
  const uint32_t b = blockIdx.x, start = bstart[b], len = blen[b];
  const int tid = threadIdx.x, lane = tid & 63, w = tid / 64;
  const uint32_t wbase = w * WSPAN;
  const uint32_t rb = lbits - 12, lmask = (1u << lbits) - 1u, rmask = (1u << rb) - 1u;
  auto ci = [&](uint32_t c) -> uint32_t { return (c % PER) * BLOCK + c / PER; };
  uint32_t k[ITEMS], rk[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = wbase + j * kWave + lane;
    k[j] = i < len ? load_stream(&in[(size_t)start + i]) : 0u;
  }
#pragma unroll
  for (int q = 0; q < PER; ++q) s_w[q * BLOCK + tid] = 0ull;
  if (tid == 0) s_ovf = 0u;
  __syncthreads();
  bool ovf = false;
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (wbase + j * kWave + lane < len) {
      const uint32_t v = k[j] & lmask, sh = 3u * (v & rmask);
      const uint64_t old = atomicAdd((unsigned long long*)&s_w[ci(v >> rb)], 1ull << sh);
      rk[j] = (uint32_t)(old >> sh) & 7u;
      ovf |= rk[j] == 7u;
    }
  if (__any(ovf) && lane == 0) s_ovf = 1u;
  __syncthreads();
  if (s_ovf) {
    // loop placement over u32 cell counters
    uint32_t* s_cnt = reinterpret_cast<uint32_t*>(s_w);
    const uint32_t cs = rb;
    auto cj = [&](uint32_t c) -> uint32_t { return c >= (uint32_t)CELLS ? (uint32_t)CELLS : (c % PER) * BLOCK + c / PER; };
    __syncthreads();
#pragma unroll
    for (int q = 0; q < PER; ++q) s_cnt[q * BLOCK + tid] = 0u;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j)
      if (wbase + j * kWave + lane < len) rk[j] = atomicAdd(&s_cnt[cj((k[j] & lmask) >> cs)], 1u);
    __syncthreads();
    uint32_t c[PER], sum = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      c[q] = s_cnt[q * BLOCK + tid];
      sum += c[q];
    }
    uint32_t tot;
    uint32_t run = block_exclusive_scan<BLOCK>(sum, s_wsum, tot);
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      s_cnt[q * BLOCK + tid] = run;
      run += c[q];
    }
    if (tid == 0) s_cnt[CELLS] = len;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j)
      if (wbase + j * kWave + lane < len) s_keys[s_cnt[cj((k[j] & lmask) >> cs)] + rk[j]] = k[j];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t p = wbase + j * kWave + lane;
      if (p < len) {
        const uint32_t x = s_keys[p], cell = (x & lmask) >> cs;
        const uint32_t a = s_cnt[cj(cell)], e = s_cnt[cj(cell + 1)];
        uint32_t less = 0;
        for (uint32_t q = a; q < e; ++q) {
          const uint32_t y = s_keys[q];
          less += (y < x) || (y == x && q < p) ? 1u : 0u;
        }
        out[(size_t)start + a + less] = x;
      }
    }
    return;
  }
  uint64_t wv[PER];
  uint32_t sum = 0;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    wv[q] = s_w[q * BLOCK + tid];
    sum += field3_sum(wv[q]);
  }
  uint32_t tot;
  uint32_t run = block_exclusive_scan<BLOCK>(sum, s_wsum, tot);
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    s_w[q * BLOCK + tid] = wv[q] | ((uint64_t)run << 48);
    run += field3_sum(wv[q]);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (wbase + j * kWave + lane < len) {
      const uint32_t v = k[j] & lmask;
      const uint64_t cw = s_w[ci(v >> rb)];
      const uint32_t below = field3_sum(cw & ((1ull << (3u * (v & rmask))) - 1ull));
      s_keys[(uint32_t)(cw >> 48) + below + rk[j]] = k[j];
    }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t p = wbase + j * kWave + lane;
    if (p < len) out[(size_t)start + p] = s_keys[p];
  }
}

// ---- cntFP: cntF over a grid-stride list of buckets, the next bucket's keys
// loaded into registers while the current one is placed ----------------------
template <int BLOCK, int ITEMS>
__global__ __launch_bounds__(BLOCK) void k_cntFP(const uint32_t* in, uint32_t* out, const uint32_t* bstart,
                                                 const uint32_t* blen, const uint32_t* nb, uint32_t lbits) {
  constexpr int CELLS = 4096, PER = CELLS / BLOCK, WSPAN = ITEMS * kWave;
  __shared__ uint32_t s_keys[BLOCK * ITEMS];
  __shared__ uint64_t s_w[CELLS];
  __shared__ uint32_t s_wsum[BLOCK / kWave];
  const uint32_t nbk = *nb;
  const int tid = threadIdx.x, lane = tid & 63, w = tid / 64;
  const uint32_t wbase = w * WSPAN;
  const uint32_t rb = lbits - 12, lmask = (1u << lbits) - 1u, rmask = (1u << rb) - 1u;
  auto ci = [&](uint32_t c) -> uint32_t { return (c % PER) * BLOCK + c / PER; };
  uint32_t b = blockIdx.x;
  if (b >= nbk) return;
  uint32_t start = bstart[b], len = blen[b];
  uint32_t k[ITEMS], kn[ITEMS], rk[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = wbase + j * kWave + lane;
    k[j] = i < len ? load_stream(&in[(size_t)start + i]) : 0u;
  }
  while (true) {
    const uint32_t b2 = b + gridDim.x;
    uint32_t nstart = 0, nlen = 0;
    if (b2 < nbk) {
      nstart = bstart[b2];
      nlen = blen[b2];
    }
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t i = wbase + j * kWave + lane;
      kn[j] = i < nlen ? load_stream(&in[(size_t)nstart + i]) : 0u;
    }
#pragma unroll
    for (int q = 0; q < PER; ++q) s_w[q * BLOCK + tid] = 0ull;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j)
      if (wbase + j * kWave + lane < len) {
        const uint32_t v = k[j] & lmask, sh = 3u * (v & rmask);
        const uint64_t old = atomicAdd((unsigned long long*)&s_w[ci(v >> rb)], 1ull << sh);
        rk[j] = (uint32_t)(old >> sh) & 7u;
      }
    __syncthreads();
    uint64_t wv[PER];
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      wv[q] = s_w[q * BLOCK + tid];
      sum += field3_sum(wv[q]);
    }
    uint32_t tot;
    uint32_t run = block_exclusive_scan<BLOCK>(sum, s_wsum, tot);
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      s_w[q * BLOCK + tid] = wv[q] | ((uint64_t)run << 48);
      run += field3_sum(wv[q]);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j)
      if (wbase + j * kWave + lane < len) {
        const uint32_t v = k[j] & lmask;
        const uint64_t cw = s_w[ci(v >> rb)];
        const uint32_t below = field3_sum(cw & ((1ull << (3u * (v & rmask))) - 1ull));
        s_keys[(uint32_t)(cw >> 48) + below + rk[j]] = k[j];
      }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t p = wbase + j * kWave + lane;
      if (p < len) out[(size_t)start + p] = s_keys[p];
    }
    if (b2 >= nbk) break;
    __syncthreads();
    b = b2;
    start = nstart;
    len = nlen;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) k[j] = kn[j];
  }
}

// ---- cntG: cntF without per-slot guards: buffer loads/stores bounded by the
// bucket (out-of-range lanes read 0 / are dropped), slots past len count into
// a dummy cell word and place into dummy LDS slots ----------------------------
template <int BLOCK, int ITEMS, int NT = 0>
__global__ __launch_bounds__(BLOCK) void k_cntG(const uint32_t* in, uint32_t* out, const uint32_t* bstart,
                                                const uint32_t* blen, const uint32_t* nb, uint32_t lbits) {
  constexpr int CELLS = 4096, PER = CELLS / BLOCK, WSPAN = ITEMS * kWave, CAP = BLOCK * ITEMS;
  constexpr int WORDS = (CELLS + 1) > (CAP + kWave + 1) / 2 ? (CELLS + 1) : (CAP + kWave + 1) / 2;
  __shared__ uint64_t s_w[WORDS];
  __shared__ uint32_t s_wsum[BLOCK / kWave];
  __shared__ uint32_t s_ovf;
  if (blockIdx.x >= *nb) return;
  const uint32_t b = blockIdx.x, start = bstart[b], len = blen[b];
  const int tid = threadIdx.x, lane = tid & 63, w = tid / 64;
  const uint32_t wbase = w * WSPAN;
  const uint32_t rb = lbits - 12, lmask = (1u << lbits) - 1u, rmask = (1u << rb) - 1u;
  auto ci = [&](uint32_t c) -> uint32_t { return (c % PER) * BLOCK + c / PER; };
  const auto rin = __builtin_amdgcn_make_buffer_rsrc((void*)(in + start), 0, len * 4u, 0x00020000);
  const auto rout = __builtin_amdgcn_make_buffer_rsrc((void*)(out + start), 0, len * 4u, 0x00020000);
  uint32_t k[ITEMS], rk[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    k[j] = __builtin_amdgcn_raw_buffer_load_b32(rin, (wbase + j * kWave + lane) * 4u, 0, NT);
#pragma unroll
  for (int q = 0; q < PER; ++q) s_w[q * BLOCK + tid] = 0ull;
  if (tid == 0) {
    s_ovf = 0u;
    s_w[CELLS] = 0ull;
  }
  __syncthreads();
  bool ovf = false;
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const bool ok = wbase + j * kWave + lane < len;
    const uint32_t v = k[j] & lmask, sh = 3u * (v & rmask);
    const uint64_t old = atomicAdd((unsigned long long*)&s_w[ok ? ci(v >> rb) : (uint32_t)CELLS], 1ull << sh);
    rk[j] = (uint32_t)(old >> sh) & 7u;
    ovf |= ok && rk[j] == 7u;
  }
  if (__any(ovf) && lane == 0) s_ovf = 1u;
  __syncthreads();
  if (s_ovf) return;  // (lab: the dup case is not timed with this kernel)
  uint64_t wv[PER];
  uint32_t sum = 0;
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    wv[q] = s_w[q * BLOCK + tid];
    sum += field3_sum(wv[q]);
  }
  uint32_t tot;
  uint32_t run = block_exclusive_scan<BLOCK>(sum, s_wsum, tot);
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    s_w[q * BLOCK + tid] = wv[q] | ((uint64_t)run << 48);
    run += field3_sum(wv[q]);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const bool ok = wbase + j * kWave + lane < len;
    const uint32_t v = k[j] & lmask;
    const uint64_t cw = s_w[ok ? ci(v >> rb) : (uint32_t)CELLS];
    const uint32_t pos = (uint32_t)(cw >> 48) + field3_sum(cw & ((1ull << (3u * (v & rmask))) - 1ull)) + rk[j];
    rk[j] = ok ? pos : (uint32_t)CAP + lane;
  }
  __syncthreads();
  uint32_t* s_keys = reinterpret_cast<uint32_t*>(s_w);
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) s_keys[rk[j]] = k[j];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t p = wbase + j * kWave + lane;
    __builtin_amdgcn_raw_buffer_store_b32(s_keys[p], rout, p * 4u, 0, NT);
  }
}

// ---- cntW: the product's bucket_count_place under a waves-per-EU bound ------
template <int BLOCK, int ITEMS, int WPE>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void k_cntW(
    const uint32_t* in, uint32_t* out, const uint32_t* bstart, const uint32_t* blen, const uint32_t* nb,
    uint32_t lbits) {
  __shared__ uint64_t s_cw[cnt_lds_words<BLOCK * ITEMS>()];
  __shared__ uint32_t s_wsum[BLOCK / kWave];
  __shared__ uint32_t s_flag;
  if (blockIdx.x >= *nb) return;
  const uint32_t b = blockIdx.x, start = bstart[b], len = blen[b];
  const int lane = threadIdx.x & 63, w = threadIdx.x / 64;
  const uint32_t wbase = w * ITEMS * kWave;
  uint32_t k[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = wbase + j * kWave + lane;
    k[j] = i < len ? load_stream(&in[(size_t)start + i]) : 0xffffffffu;
  }
  bucket_count_place<BLOCK, ITEMS>(k, s_cw, out, start, len, lbits, 0u);
}

// ---- abl: cntF's phases cut at STAGE (0 copy with the same LDS, 1 + atomics,
// 2 + scan, 3 + placement = cntF without the fallback) ------------------------
template <int BLOCK, int ITEMS, int STAGE>
__global__ __launch_bounds__(BLOCK) void k_abl(const uint32_t* in, uint32_t* out, const uint32_t* bstart,
                                               const uint32_t* blen, const uint32_t* nb, uint32_t lbits) {
  constexpr int CELLS = 4096, PER = CELLS / BLOCK, WSPAN = ITEMS * kWave;
  __shared__ uint64_t s_w[cnt_lds_words<BLOCK * ITEMS>()];
  __shared__ uint32_t s_wsum[BLOCK / kWave];
  if (blockIdx.x >= *nb) return;
  const uint32_t b = blockIdx.x, start = bstart[b], len = blen[b];
  const int tid = threadIdx.x, lane = tid & 63, w = tid / 64;
  const uint32_t wbase = w * WSPAN;
  const uint32_t rb = lbits - 12, lmask = (1u << lbits) - 1u, rmask = (1u << rb) - 1u;
  auto ci = [&](uint32_t c) -> uint32_t { return (c % PER) * BLOCK + c / PER; };
  uint32_t k[ITEMS], rk[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = wbase + j * kWave + lane;
    k[j] = i < len ? load_stream(&in[(size_t)start + i]) : 0u;
    rk[j] = i;
  }
  if (STAGE >= 1) {
#pragma unroll
    for (int q = 0; q < PER; ++q) s_w[q * BLOCK + tid] = 0ull;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j)
      if (wbase + j * kWave + lane < len) {
        const uint32_t v = k[j] & lmask, sh = 3u * (v & rmask);
        const uint64_t old = atomicAdd((unsigned long long*)&s_w[ci(v >> rb)], 1ull << sh);
        rk[j] = STAGE >= 3 ? (uint32_t)(old >> sh) & 7u : rk[j] + ((uint32_t)(old >> sh) & 7u) * 0u + (uint32_t)(old == 0xffffffffffffull);
      }
    __syncthreads();
  }
  if (STAGE >= 2) {
    uint64_t wv[PER];
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      wv[q] = s_w[q * BLOCK + tid];
      sum += field3_sum(wv[q]);
    }
    uint32_t tot;
    uint32_t run = block_exclusive_scan<BLOCK>(sum, s_wsum, tot);
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      s_w[q * BLOCK + tid] = wv[q] | ((uint64_t)run << 48);
      run += field3_sum(wv[q]);
    }
    __syncthreads();
  }
  if (STAGE >= 3) {
#pragma unroll
    for (int j = 0; j < ITEMS; ++j)
      if (wbase + j * kWave + lane < len) {
        const uint32_t v = k[j] & lmask;
        const uint64_t cw = s_w[ci(v >> rb)];
        rk[j] += (uint32_t)(cw >> 48) + field3_sum(cw & ((1ull << (3u * (v & rmask))) - 1ull));
      }
    __syncthreads();
  }
  uint32_t* s_keys = reinterpret_cast<uint32_t*>(s_w);
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (wbase + j * kWave + lane < len) s_keys[rk[j] < len ? rk[j] : 0] = k[j];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t p = wbase + j * kWave + lane;
    if (p < len) out[(size_t)start + p] = s_keys[p];
  }
}

// ---- copy: the floor (load, through LDS, store) -----------------------------
template <int BLOCK, int ITEMS>
__global__ __launch_bounds__(BLOCK) void k_copy(const uint32_t* in, uint32_t* out, const uint32_t* bstart,
                                                const uint32_t* blen, const uint32_t* nb, uint32_t) {
  constexpr int WSPAN = ITEMS * kWave;
  __shared__ uint32_t s_keys[BLOCK * ITEMS];
  if (blockIdx.x >= *nb) return;
  const uint32_t b = blockIdx.x, start = bstart[b], len = blen[b];
  const int tid = threadIdx.x, lane = tid & 63, w = tid / 64;
  const uint32_t wbase = w * WSPAN;
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

__global__ void fill(uint32_t* k, size_t n, uint32_t S, uint32_t lbits, uint32_t dupmask) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t x = (i + 1) * 0x9E3779B97F4A7C15ull;
  x ^= x >> 29; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 32;
  const uint32_t low = (uint32_t)(x & ((1ull << lbits) - 1)) & dupmask;
  k[i] = ((uint32_t)(i / S) << lbits) | low;
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
  struct V { std::string name; uint32_t S, lbits; std::function<void(uint32_t)> launch; uint32_t dup = 0xffffffffu; };
  std::vector<V> vs;
  vs.push_back({"copy 256x17 (floor)", 4096, 16, [&](uint32_t m) {
    hipLaunchKernelGGL((k_copy<256, 17>), dim3(m), dim3(256), 0, st, in, out, bs, bl, nb, 16u);
  }});
  for (uint32_t lb : {16u, 14u, 13u}) {
    vs.push_back({"cntF 256x17 lbits=" + std::to_string(lb), 4096, lb, [&, lb](uint32_t m) {
      hipLaunchKernelGGL((k_cntF<256, 17>), dim3(m), dim3(256), 0, st, in, out, bs, bl, nb, lb);
    }});
  }
  vs.push_back({"cntF 256x17 lbits=16 dup(ovf)", 4096, 16, [&](uint32_t m) {
    hipLaunchKernelGGL((k_cntF<256, 17>), dim3(m), dim3(256), 0, st, in, out, bs, bl, nb, 16u);
  }, 0xf0f0u});
  vs.push_back({"cntF 512x9 lbits=16", 4096, 16, [&](uint32_t m) {
    hipLaunchKernelGGL((k_cntF<512, 9>), dim3(m), dim3(512), 0, st, in, out, bs, bl, nb, 16u);
  }});
#define PRODC(B, I, S) \
  vs.push_back({"prodCNT " #B "x" #I " S=" #S, S, 16, [&](uint32_t m) { \
    hipLaunchKernelGGL((k_bucket_sort<4, B, I, RadixDigit, uint32_t, NoValue, 0, true>), dim3(m), dim3(B), 0, st, in, out, \
                       (const NoValue*)nullptr, (NoValue*)nullptr, bs, bl, nb, 1u << 30, nullptr, 16u, 0u, ov, nullptr, 0u); \
  }});
  vs.push_back({"cntG 256x17", 4096, 16, [&](uint32_t m) {
    hipLaunchKernelGGL((k_cntG<256, 17>), dim3(m), dim3(256), 0, st, in, out, bs, bl, nb, 16u);
  }});
  vs.push_back({"cntG 512x9", 4096, 16, [&](uint32_t m) {
    hipLaunchKernelGGL((k_cntG<512, 9>), dim3(m), dim3(512), 0, st, in, out, bs, bl, nb, 16u);
  }});
  vs.push_back({"cntG 512x8", 4096, 16, [&](uint32_t m) {
    hipLaunchKernelGGL((k_cntG<512, 8>), dim3(m), dim3(512), 0, st, in, out, bs, bl, nb, 16u);
  }});
  vs.push_back({"cntG 512x9 nt", 4096, 16, [&](uint32_t m) {
    hipLaunchKernelGGL((k_cntG<512, 9, 2>), dim3(m), dim3(512), 0, st, in, out, bs, bl, nb, 16u);
  }});
  vs.push_back({"cntG 512x17 S=8192", 8192, 16, [&](uint32_t m) {
    hipLaunchKernelGGL((k_cntG<512, 17>), dim3(m), dim3(512), 0, st, in, out, bs, bl, nb, 16u);
  }});
#define CNTW(B, I, WPE) \
  vs.push_back({"cntW " #B "x" #I " wpe=" #WPE, 4096, 16, [&](uint32_t m) { \
    hipLaunchKernelGGL((k_cntW<B, I, WPE>), dim3(m), dim3(B), 0, st, in, out, bs, bl, nb, 16u); \
  }});
  CNTW(512, 8, 1)
  CNTW(512, 8, 6)
  CNTW(512, 8, 8)
  CNTW(256, 17, 1)
  CNTW(256, 17, 5)
  CNTW(256, 17, 6)
  CNTW(256, 16, 6)
#define ABL(B, I, ST) \
  vs.push_back({"abl " #B "x" #I " stage=" #ST, 4096, 16, [&](uint32_t m) { \
    hipLaunchKernelGGL((k_abl<B, I, ST>), dim3(m), dim3(B), 0, st, in, out, bs, bl, nb, 16u); \
  }});
  ABL(256, 17, 0) ABL(256, 17, 1) ABL(256, 17, 2) ABL(256, 17, 3)
  ABL(512, 8, 0) ABL(512, 8, 1) ABL(512, 8, 2) ABL(512, 8, 3)
  PRODC(256, 17, 4096)
  PRODC(512, 9, 4096)
  PRODC(512, 8, 4096)
  PRODC(1024, 5, 4096)
  PRODC(512, 17, 8192)
  PRODC(1024, 9, 8192)
  PRODC(1024, 17, 16384)
  PRODC(512, 34, 16384)
  PRODC(512, 32, 16384)
  vs.push_back({"prodCNT 512x9 dup(ovf)", 4096, 16, [&](uint32_t m) {
    hipLaunchKernelGGL((k_bucket_sort<4, 512, 9, RadixDigit, uint32_t, NoValue, 0, true>), dim3(m), dim3(512), 0, st, in, out,
                       (const NoValue*)nullptr, (NoValue*)nullptr, bs, bl, nb, 1u << 30, nullptr, 16u, 0u, ov, nullptr, 0u);
  }, 0xf0f0u});
  for (uint32_t g : {512u, 768u, 1024u, 1536u}) {
    vs.push_back({"cntFP 512x9 g=" + std::to_string(g), 4096, 16, [&, g](uint32_t m) {
      hipLaunchKernelGGL((k_cntFP<512, 9>), dim3(std::min(m, g)), dim3(512), 0, st, in, out, bs, bl, nb, 16u);
    }});
    vs.push_back({"cntFP 256x17 g=" + std::to_string(g), 4096, 16, [&, g](uint32_t m) {
      hipLaunchKernelGGL((k_cntFP<256, 17>), dim3(std::min(m, g)), dim3(256), 0, st, in, out, bs, bl, nb, 16u);
    }});
  }
  vs.push_back({"cntF 1024x5 lbits=16", 4096, 16, [&](uint32_t m) {
    hipLaunchKernelGGL((k_cntF<1024, 5>), dim3(m), dim3(1024), 0, st, in, out, bs, bl, nb, 16u);
  }});
  vs.push_back({"cntF 1024x9 S=8192 lbits=16", 8192, 16, [&](uint32_t m) {
    hipLaunchKernelGGL((k_cntF<1024, 9>), dim3(m), dim3(1024), 0, st, in, out, bs, bl, nb, 16u);
  }});
  vs.push_back({"cntF 512x17 S=8192 lbits=16", 8192, 16, [&](uint32_t m) {
    hipLaunchKernelGGL((k_cntF<512, 17>), dim3(m), dim3(512), 0, st, in, out, bs, bl, nb, 16u);
  }});
  for (uint32_t lb : {16u, 12u}) {
    vs.push_back({"prod 256x17 lbits=" + std::to_string(lb), 4096, lb, [&, lb](uint32_t m) {
      hipLaunchKernelGGL((k_bucket_sort<4, 256, 17>), dim3(m), dim3(256), 0, st, in, out, (const NoValue*)nullptr,
                         (NoValue*)nullptr, bs, bl, nb, 1u << 30, nullptr, lb, 0u, ov, nullptr, 0u);
    }});
    vs.push_back({"chain2 256x17 lbits=" + std::to_string(lb), 4096, lb, [&, lb](uint32_t m) {
      hipLaunchKernelGGL((k_chain2<256, 17>), dim3(m), dim3(256), 0, st, in, out, bs, bl, nb, lb);
    }});
    vs.push_back({"cnt12 256x17 lbits=" + std::to_string(lb), 4096, lb, [&, lb](uint32_t m) {
      hipLaunchKernelGGL((k_cnt12<256, 17>), dim3(m), dim3(256), 0, st, in, out, bs, bl, nb, lb);
    }});
    vs.push_back({"cnt12pf 256x17 lbits=" + std::to_string(lb), 4096, lb, [&, lb](uint32_t m) {
      hipLaunchKernelGGL((k_cnt12<256, 17, 0, true>), dim3(std::min(m, 1024u)), dim3(256), 0, st, in, out, bs, bl, nb, lb);
    }});
    vs.push_back({"cnt12pf2k 256x17 lbits=" + std::to_string(lb), 4096, lb, [&, lb](uint32_t m) {
      hipLaunchKernelGGL((k_cnt12<256, 17, 0, true>), dim3(std::min(m, 2048u)), dim3(256), 0, st, in, out, bs, bl, nb, lb);
    }});
    vs.push_back({"cntW3 256x17 lbits=" + std::to_string(lb), 4096, lb, [&, lb](uint32_t m) {
      hipLaunchKernelGGL((k_cnt12<256, 17, 3>), dim3(m), dim3(256), 0, st, in, out, bs, bl, nb, lb);
    }});
    vs.push_back({"cntW4 256x17 lbits=" + std::to_string(lb), 4096, lb, [&, lb](uint32_t m) {
      hipLaunchKernelGGL((k_cnt12<256, 17, 4>), dim3(m), dim3(256), 0, st, in, out, bs, bl, nb, lb);
    }});
    vs.push_back({"cntP12 256x17 lbits=" + std::to_string(lb), 4096, lb, [&, lb](uint32_t m) {
      hipLaunchKernelGGL((k_cntP<256, 17, 12>), dim3(m), dim3(256), 0, st, in, out, bs, bl, nb, lb);
    }});
    vs.push_back({"cntP13 256x17 lbits=" + std::to_string(lb), 4096, lb, [&, lb](uint32_t m) {
      hipLaunchKernelGGL((k_cntP<256, 17, 13>), dim3(m), dim3(256), 0, st, in, out, bs, bl, nb, lb);
    }});
    vs.push_back({"cntP14 256x17 lbits=" + std::to_string(lb), 4096, lb, [&, lb](uint32_t m) {
      hipLaunchKernelGGL((k_cntP<256, 17, 14>), dim3(m), dim3(256), 0, st, in, out, bs, bl, nb, lb);
    }});
  }
  vs.push_back({"cntP13 512x17 S=8192 lbits=16", 8192, 16, [&](uint32_t m) {
    hipLaunchKernelGGL((k_cntP<512, 17, 13>), dim3(m), dim3(512), 0, st, in, out, bs, bl, nb, 16u);
  }});
  vs.push_back({"cntP14 512x17 S=8192 lbits=16", 8192, 16, [&](uint32_t m) {
    hipLaunchKernelGGL((k_cntP<512, 17, 14>), dim3(m), dim3(512), 0, st, in, out, bs, bl, nb, 16u);
  }});
  vs.push_back({"prod 512x17 S=8192 lbits=16", 8192, 16, [&](uint32_t m) {
    hipLaunchKernelGGL((k_bucket_sort<4, 512, 17>), dim3(m), dim3(512), 0, st, in, out, (const NoValue*)nullptr,
                       (NoValue*)nullptr, bs, bl, nb, 1u << 30, nullptr, 16u, 0u, ov, nullptr, 0u);
  }});
  vs.push_back({"cnt12 512x17 S=8192 lbits=16", 8192, 16, [&](uint32_t m) {
    hipLaunchKernelGGL((k_cnt12<512, 17>), dim3(m), dim3(512), 0, st, in, out, bs, bl, nb, 16u);
  }});
  const char* filt = argc > 2 ? argv[2] : nullptr;
  for (auto& v : vs) {
    if (filt) {  // comma-separated name substrings
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
    const uint32_t m = (uint32_t)(n / v.S);
    hipLaunchKernelGGL(fill, dim3((n + 255) / 256), dim3(256), 0, st, in, n, v.S, v.lbits, v.dup);
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
    printf("%-30s 2^%d keys: median %7.1f us  best %7.1f  %5.0f GB/s (8 B/key)  %s\n", v.name.c_str(), lg, med, us[0],
           8.0 * n / (med * 1e-6) / 1e9, (sorted && sum0 == sum1 && x0 == x1) ? "sorted" : (sum0 == sum1 && x0 == x1 ? "permutation" : "WRONG"));
    fflush(stdout);
  }
  return 0;
}
