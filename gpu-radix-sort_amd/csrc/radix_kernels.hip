// radix_kernels.hip -- gfx950 kernels and the LSD pass driver of libsort.
//
// One digit pass (reference: SortState::Step, sort.cu:322-346, which runs
// gpu_radix_sort_local + sum_scan_blelloch + gpu_glbl_shuffle per 2-bit
// digit) is re-designed here as a reduce-then-scan over even-share tile
// ranges with 4- or 8-bit digits:
//
//   k_upsweep    each block reads its contiguous range of tiles once (16-byte
//                loads) and builds the digit histogram in LDS (wave-private
//                rows, ds_add), written digit-major: counts[d * grid + b].
//   k_scan_tiles Blelloch-style exclusive scan of counts: per-thread serial
//                up-sweep, wave64 __shfl_up scan, LDS combine of wave totals,
//                per-thread down-sweep; one total per 4096-counter tile.
//   k_scan_single second-level scan of the tile totals (one block).
//   k_downsweep  each block re-reads its tiles in order; per tile it ranks the
//                keys stably with wave64 ballot match (no atomics), forms the
//                locally sorted tile in LDS and writes every digit run to
//                global memory as one contiguous, coalesced stretch at
//                scan[d][b] + running offset.
//
// The global base of block b's run of digit d is l1[i] + l2[i / 4096] with
// i = d * grid + b (the add of the second-level scan is folded into the
// consumers instead of a separate pass; scan.cu:16-58 does it as a kernel).
#include "radix.h"

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <type_traits>

namespace lsort {

constexpr int kWave = 64;

// ----------------------------------------------------------------------------
// digit extractors
// ----------------------------------------------------------------------------
struct RadixDigit {
  uint32_t shift;
  uint32_t mask;
  __device__ __forceinline__ uint32_t operator()(uint32_t k) const { return (k >> shift) & mask; }
  __device__ __forceinline__ uint32_t operator()(uint64_t k) const {
    return (uint32_t)(k >> shift) & mask;
  }
};

// Range partition: bucket = number of splitters <= key (splitters ascending).
struct SplitDigit {
  uint32_t nsplit;
  uint32_t s[kMaxSplit];
  __device__ __forceinline__ uint32_t operator()(uint32_t k) const {
    uint32_t lo = 0, hi = nsplit;
    while (lo < hi) {
      uint32_t mid = (lo + hi) >> 1;
      if (s[mid] <= k) lo = mid + 1; else hi = mid;
    }
    return lo;
  }
};

template <typename K> struct VecOf;
template <> struct VecOf<uint32_t> { using type = uint4; static constexpr int n = 4; };
template <> struct VecOf<uint64_t> { using type = ulonglong2; static constexpr int n = 2; };

__device__ __forceinline__ uint32_t vec_elem(const uint4& v, int c) {
  return c == 0 ? v.x : c == 1 ? v.y : c == 2 ? v.z : v.w;
}
__device__ __forceinline__ uint64_t vec_elem(const ulonglong2& v, int c) { return c == 0 ? v.x : v.y; }

__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }

__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Exclusive scan of one value per thread over the block.  Inclusive wave64
// scan by __shfl_up (6 steps), wave totals through LDS.  The caller must put
// a barrier between two uses of s_wsum.
template <int BLOCK>
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* s_wsum, uint32_t& total) {
  constexpr int WAVES = BLOCK / kWave;
  const int lane = threadIdx.x & (kWave - 1);
  const int w = threadIdx.x / kWave;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    uint32_t y = __shfl_up(x, o, kWave);
    if (lane >= o) x += y;
  }
  if (lane == kWave - 1) s_wsum[w] = x;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < WAVES; ++i) {
    uint32_t s = s_wsum[i];
    pre += (i < w) ? s : 0u;
    tot += s;
  }
  total = tot;
  return pre + x - v;
}

// Even-share tile range of block b (reference has one 128-key block per tile;
// here a block walks a contiguous range so its digit runs stay in order).
__device__ __forceinline__ void tile_range(uint32_t b, uint32_t grid, uint32_t num_tiles,
                                           uint32_t& t0, uint32_t& t1) {
  t0 = (uint32_t)(((uint64_t)b * num_tiles) / grid);
  t1 = (uint32_t)(((uint64_t)(b + 1) * num_tiles) / grid);
}

// ----------------------------------------------------------------------------
// upsweep: per-block digit histogram
// ----------------------------------------------------------------------------
template <int BITS, int BLOCK, int ITEMS, bool VEC, typename K, typename Op>
__global__ __launch_bounds__(BLOCK) void k_upsweep(const K* __restrict__ keys, uint32_t n,
                                                   uint32_t num_tiles, uint32_t grid, Op op,
                                                   uint32_t* __restrict__ counts) {
  constexpr int RADIX = 1 << BITS;
  constexpr int WAVES = BLOCK / kWave;
  constexpr int TILE = BLOCK * ITEMS;
  __shared__ uint32_t s_hist[WAVES][RADIX];
  const int tid = threadIdx.x;
  const int w = tid / kWave;
  for (int i = tid; i < WAVES * RADIX; i += BLOCK) (&s_hist[0][0])[i] = 0u;
  __syncthreads();

  uint32_t t0, t1;
  tile_range(blockIdx.x, grid, num_tiles, t0, t1);
  const uint64_t beg = (uint64_t)t0 * TILE;
  const uint64_t end = umin64((uint64_t)t1 * TILE, (uint64_t)n);
  uint64_t full_end = beg;
  if (VEC) {
    using V = typename VecOf<K>::type;
    constexpr int PER = VecOf<K>::n;
    constexpr int NV = ITEMS / PER;
    full_end = end >= beg ? beg + ((end - beg) / TILE) * TILE : beg;
    for (uint64_t base = beg; base < full_end; base += TILE) {
      const V* vp = reinterpret_cast<const V*>(keys + base);
      V v[NV];
#pragma unroll
      for (int j = 0; j < NV; ++j) v[j] = vp[j * BLOCK + tid];
#pragma unroll
      for (int j = 0; j < NV; ++j) {
#pragma unroll
        for (int c = 0; c < PER; ++c) atomicAdd(&s_hist[w][op(vec_elem(v[j], c))], 1u);
      }
    }
  }
  for (uint64_t i = full_end + tid; i < end; i += BLOCK) atomicAdd(&s_hist[w][op(keys[i])], 1u);
  __syncthreads();
  for (int d = tid; d < RADIX; d += BLOCK) {
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < WAVES; ++i) s += s_hist[i][d];
    counts[(size_t)d * grid + blockIdx.x] = s;
  }
}

// ----------------------------------------------------------------------------
// two-level exclusive scan of the digit-major counters
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(kScanBlock) void k_scan_tiles(const uint32_t* __restrict__ in,
                                                            uint32_t* __restrict__ out, uint32_t m,
                                                            uint32_t* __restrict__ tile_sums) {
  __shared__ uint32_t s_wsum[kScanBlock / kWave];
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanItems;
  uint32_t x[kScanItems];
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {  // up-sweep: serial per thread
    x[j] = (base + j < m) ? in[base + j] : 0u;
    s += x[j];
  }
  uint32_t total;
  uint32_t run = block_exclusive_scan<kScanBlock>(s, s_wsum, total);
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {  // down-sweep
    if (base + j < m) out[base + j] = run;
    run += x[j];
  }
  if (threadIdx.x == 0) tile_sums[blockIdx.x] = total;
}

// Single-block exclusive scan in place of m values (any m), chunked with carry.
__global__ __launch_bounds__(kScanBlock) void k_scan_single(uint32_t* __restrict__ data, uint32_t m) {
  __shared__ uint32_t s_wsum[kScanBlock / kWave];
  uint32_t carry = 0;
  for (uint64_t chunk = 0; chunk < m; chunk += kScanTile) {
    const uint64_t base = chunk + (uint64_t)threadIdx.x * kScanItems;
    uint32_t x[kScanItems];
    uint32_t s = 0;
#pragma unroll
    for (int j = 0; j < kScanItems; ++j) {
      x[j] = (base + j < m) ? data[base + j] : 0u;
      s += x[j];
    }
    uint32_t total;
    uint32_t run = carry + block_exclusive_scan<kScanBlock>(s, s_wsum, total);
#pragma unroll
    for (int j = 0; j < kScanItems; ++j) {
      if (base + j < m) data[base + j] = run;
      run += x[j];
    }
    carry += total;
    __syncthreads();
  }
}

// ----------------------------------------------------------------------------
// downsweep: stable local rank + coalesced scatter
// ----------------------------------------------------------------------------
template <int BITS, int BLOCK, int ITEMS, typename K, typename V, typename Op>
__global__ __launch_bounds__(BLOCK) void k_downsweep(const K* __restrict__ kin, K* __restrict__ kout,
                                                     const V* __restrict__ vin, V* __restrict__ vout,
                                                     uint32_t n, uint32_t num_tiles, uint32_t grid,
                                                     Op op, const uint32_t* __restrict__ l1,
                                                     const uint32_t* __restrict__ l2) {
  constexpr bool HAS_V = !std::is_same<V, NoValue>::value;
  using VS = typename std::conditional<HAS_V, V, uint8_t>::type;  // LDS value type
  constexpr int RADIX = 1 << BITS;
  constexpr int WAVES = BLOCK / kWave;
  constexpr int TILE = BLOCK * ITEMS;
  constexpr int WSPAN = ITEMS * kWave;  // keys per wave per tile
  static_assert(RADIX <= BLOCK, "one digit per thread in the block phase");

  __shared__ K s_keys[TILE];
  __shared__ VS s_vals[HAS_V ? TILE : 1];
  __shared__ uint32_t s_whist[WAVES][RADIX];
  __shared__ uint32_t s_gbase[RADIX];
  __shared__ uint32_t s_outbase[RADIX];
  __shared__ uint32_t s_wsum[WAVES];

  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int w = tid / kWave;

  uint32_t t0, t1;
  tile_range(blockIdx.x, grid, num_tiles, t0, t1);
  if (tid < RADIX) {
    const size_t i = (size_t)tid * grid + blockIdx.x;
    s_gbase[tid] = l1[i] + l2[i / kScanTile];
  }

  for (uint32_t t = t0; t < t1; ++t) {
    const uint64_t tile_base = (uint64_t)t * TILE;
    const uint32_t valid = (uint32_t)umin64((uint64_t)TILE, (uint64_t)n - tile_base);
    const bool full = valid == TILE;
    const uint32_t wbase = w * WSPAN;

    for (int d = lane; d < RADIX; d += kWave) s_whist[w][d] = 0u;

    K k[ITEMS];
    VS v[ITEMS];
    uint32_t rk[ITEMS];
    if (full) {
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) {
        const uint64_t e = tile_base + wbase + j * kWave + lane;
        k[j] = kin[e];
        if constexpr (HAS_V) v[j] = vin[e];
      }
    } else {
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) {
        const uint32_t e = wbase + j * kWave + lane;
        const bool ok = e < valid;
        k[j] = ok ? kin[tile_base + e] : (K)0;
        if constexpr (HAS_V) v[j] = ok ? vin[tile_base + e] : (VS)0;
      }
    }

    // Wave-level multi-split: items in order, lanes in order => stable.
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t d = op(k[j]);
      const bool ok = full || (wbase + j * kWave + lane < valid);
      uint64_t peers = __ballot(ok);
#pragma unroll
      for (int bit = 0; bit < BITS; ++bit) {
        const bool x = (d >> bit) & 1u;
        const uint64_t m = __ballot(x);
        peers &= x ? m : ~m;
      }
      const uint32_t below = mbcnt64(peers);
      const uint32_t cnt = (uint32_t)__popcll(peers);
      const uint32_t base = s_whist[w][d];
      rk[j] = base + below;
      if (ok && below + 1u == cnt) s_whist[w][d] = base + cnt;
    }
    __syncthreads();

    // Per digit: tile count, block exclusive scan, wave prefixes.
    uint32_t cnt_d = 0;
    if (tid < RADIX) {
#pragma unroll
      for (int i = 0; i < WAVES; ++i) cnt_d += s_whist[i][tid];
    }
    uint32_t tile_total;
    const uint32_t excl = block_exclusive_scan<BLOCK>(cnt_d, s_wsum, tile_total);
    if (tid < RADIX) {
      uint32_t run = excl;
#pragma unroll
      for (int i = 0; i < WAVES; ++i) {
        const uint32_t c = s_whist[i][tid];
        s_whist[i][tid] = run;
        run += c;
      }
      const uint32_t g = s_gbase[tid];
      s_outbase[tid] = g - excl;
      s_gbase[tid] = g + cnt_d;
    }
    __syncthreads();

    // Locally sorted tile in LDS.
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const bool ok = full || (wbase + j * kWave + lane < valid);
      if (ok) {
        const uint32_t pos = s_whist[w][op(k[j])] + rk[j];
        s_keys[pos] = k[j];
        if constexpr (HAS_V) s_vals[pos] = v[j];
      }
    }
    __syncthreads();

    // Coalesced write of the digit runs.
    for (uint32_t i = tid; i < valid; i += BLOCK) {
      const K kk = s_keys[i];
      const uint32_t o = s_outbase[op(kk)] + i;
      kout[o] = kk;
      if constexpr (HAS_V) vout[o] = s_vals[i];
    }
    __syncthreads();
  }
}

// ----------------------------------------------------------------------------
// group boundaries
// ----------------------------------------------------------------------------
// From the scan of a single-pass sort: bounds[g] = global start of digit g.
__global__ void k_bounds_from_scan(const uint32_t* __restrict__ l1, const uint32_t* __restrict__ l2,
                                   uint32_t grid, uint32_t ngroups, uint32_t* __restrict__ bounds) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g < ngroups) {
    const size_t i = (size_t)g * grid;
    bounds[g] = l1[i] + l2[i / kScanTile];
  }
}

// From sorted data (reference gpu_groups, sort.cu:14-27, plus the host fill
// loop sort.cu:384-391, but writing the exclusive prefix for empty groups in
// the same launch): position i writes bounds[g] = i for every group g in
// (group(i-1), group(i)]; position n closes the remaining groups.
template <typename K>
__global__ void k_group_bounds(const K* __restrict__ sorted, uint32_t n, uint32_t shift,
                               uint32_t gmask, uint32_t ngroups, uint32_t* __restrict__ bounds) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= n; i += stride) {
    const int64_t cur = i < n ? (int64_t)((uint32_t)(sorted[i] >> shift) & gmask) : (int64_t)ngroups;
    const int64_t prev = i > 0 ? (int64_t)((uint32_t)(sorted[i - 1] >> shift) & gmask) : -1;
    if (cur != prev) {
      const int64_t last = cur < (int64_t)ngroups ? cur : (int64_t)ngroups - 1;
      for (int64_t g = prev + 1; g <= last; ++g) bounds[g] = (uint32_t)i;
    }
  }
}

// ----------------------------------------------------------------------------
// histogram (bits <= 12 in LDS; wider bins with global atomics)
// ----------------------------------------------------------------------------
template <int BITS>
__global__ __launch_bounds__(256) void k_hist_lds(const uint32_t* __restrict__ keys, uint32_t n,
                                                  uint32_t shift, uint32_t* __restrict__ hist) {
  constexpr int BINS = 1 << BITS;
  __shared__ uint32_t s_h[BINS];
  for (int i = threadIdx.x; i < BINS; i += 256) s_h[i] = 0u;
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride)
    atomicAdd(&s_h[(keys[i] >> shift) & (BINS - 1)], 1u);
  __syncthreads();
  for (int i = threadIdx.x; i < BINS; i += 256) {
    const uint32_t c = s_h[i];
    if (c) atomicAdd(&hist[i], c);
  }
}

__global__ void k_hist_global(const uint32_t* __restrict__ keys, uint32_t n, uint32_t shift,
                              uint32_t mask, uint32_t* __restrict__ hist) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    atomicAdd(&hist[(keys[i] >> shift) & mask], 1u);
}

// Sizes of the buckets of a partition = per-digit column sums of counts.
__global__ void k_bucket_sizes(const uint32_t* __restrict__ counts, uint32_t grid, uint32_t nb,
                               uint32_t* __restrict__ out) {
  const uint32_t d = blockIdx.x;
  uint32_t s = 0;
  for (uint32_t b = threadIdx.x; b < grid; b += blockDim.x) s += counts[(size_t)d * grid + b];
  for (int o = kWave / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, kWave);
  __shared__ uint32_t s_p[16];
  if ((threadIdx.x & 63) == 0) s_p[threadIdx.x / 64] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (uint32_t i = 0; i < blockDim.x / 64; ++i) t += s_p[i];
    if (d < nb) out[d] = t;
  }
}

// ----------------------------------------------------------------------------
// segment gather copy
// ----------------------------------------------------------------------------
__global__ void k_segment_copy(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                               const uint64_t* __restrict__ tab, uint64_t nseg) {
  for (uint64_t s = blockIdx.x; s < nseg; s += gridDim.x) {
    const uint64_t so = tab[s], dof = tab[nseg + s], len = tab[2 * nseg + s];
    for (uint64_t j = threadIdx.x; j < len; j += blockDim.x) dst[dof + j] = src[so + j];
  }
}

// ----------------------------------------------------------------------------
// PCG32 stream on the device (utils.cu:65-80 + LCG skip-ahead)
// ----------------------------------------------------------------------------
__host__ __device__ inline uint64_t pcg_advance(uint64_t state, uint64_t delta) {
  uint64_t acc_mult = 1u, acc_plus = 0u, cur_mult = kPcgMult, cur_plus = kPcgInc;
  while (delta > 0) {
    if (delta & 1u) {
      acc_mult *= cur_mult;
      acc_plus = acc_plus * cur_mult + cur_plus;
    }
    cur_plus = (cur_mult + 1u) * cur_plus;
    cur_mult *= cur_mult;
    delta >>= 1;
  }
  return acc_mult * state + acc_plus;
}

__host__ __device__ inline uint32_t pcg_output(uint64_t x) {
  const uint32_t count = (uint32_t)(x >> 59);
  x ^= x >> 18;
  const uint32_t v = (uint32_t)(x >> 27);
  return (v >> count) | (v << ((0u - count) & 31u));
}

constexpr int kPopItems = 16;
__global__ __launch_bounds__(256) void k_populate(uint32_t* __restrict__ out, uint64_t n, uint64_t first) {
  __shared__ uint32_t s_v[256 * kPopItems];
  const uint64_t block_start = (uint64_t)blockIdx.x * 256 * kPopItems;
  const uint64_t my = block_start + (uint64_t)threadIdx.x * kPopItems;
  uint64_t st = pcg_advance(kPcgInit, first + my);
#pragma unroll
  for (int j = 0; j < kPopItems; ++j) {
    s_v[threadIdx.x * kPopItems + j] = pcg_output(st);
    st = st * kPcgMult + kPcgInc;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kPopItems; ++j) {
    const uint64_t e = block_start + (uint64_t)j * 256 + threadIdx.x;
    if (e < n) out[e] = s_v[j * 256 + threadIdx.x];
  }
}

// ============================================================================
// host side: workspace and pass driver
// ============================================================================
#define LS_TRY(...)                        \
  do {                                     \
    hipError_t e__ = (__VA_ARGS__);        \
    if (e__ != hipSuccess) return e__;     \
  } while (0)

hipError_t Workspace::ensure_counts(size_t m) {
  const size_t l2 = (m + kScanTile - 1) / kScanTile + 1;
  if (m > counts_cap) {
    if (counts) { (void)hipFree(counts); counts = nullptr; }
    if (scan_l1) { (void)hipFree(scan_l1); scan_l1 = nullptr; }
    counts_cap = 0;
    LS_TRY(hipMalloc(&counts, m * sizeof(uint32_t)));
    LS_TRY(hipMalloc(&scan_l1, m * sizeof(uint32_t)));
    counts_cap = m;
  }
  if (l2 > l2_cap) {
    if (scan_l2) { (void)hipFree(scan_l2); scan_l2 = nullptr; }
    l2_cap = 0;
    LS_TRY(hipMalloc(&scan_l2, l2 * sizeof(uint32_t)));
    l2_cap = l2;
  }
  return hipSuccess;
}

hipError_t Workspace::ensure_hbuf(size_t bytes) {
  if (bytes <= hbuf_cap) return hipSuccess;
  for (auto& p : hbuf) {
    if (p) { (void)hipFree(p); p = nullptr; }
  }
  hbuf_cap = 0;
  LS_TRY(hipMalloc(&hbuf[0], bytes));
  LS_TRY(hipMalloc(&hbuf[1], bytes));
  hbuf_cap = bytes;
  return hipSuccess;
}

hipError_t Workspace::ensure_bounds(size_t m) {
  if (m <= dbounds_cap) return hipSuccess;
  if (dbounds) { (void)hipFree(dbounds); dbounds = nullptr; }
  dbounds_cap = 0;
  LS_TRY(hipMalloc(&dbounds, m * sizeof(uint32_t)));
  dbounds_cap = m;
  return hipSuccess;
}

hipError_t Workspace::ensure_seg(size_t m) {
  if (!seg_evt) LS_TRY(hipEventCreateWithFlags(&seg_evt, hipEventDisableTiming));
  if (m <= seg_cap) return hipSuccess;
  if (seg_dev) { (void)hipFree(seg_dev); seg_dev = nullptr; }
  if (seg_host) { (void)hipHostFree(seg_host); seg_host = nullptr; }
  seg_cap = 0;
  LS_TRY(hipMalloc(&seg_dev, m * sizeof(uint64_t)));
  LS_TRY(hipHostMalloc(&seg_host, m * sizeof(uint64_t), hipHostMallocDefault));
  seg_cap = m;
  return hipSuccess;
}

void Workspace::release() {
  int prev = -1;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(device);
  if (stream) (void)hipStreamSynchronize(stream);
  for (auto p : {(void*)counts, (void*)scan_l1, (void*)scan_l2, hbuf[0], hbuf[1], (void*)dbounds,
                 (void*)seg_dev, (void*)hist_tmp})
    if (p) (void)hipFree(p);
  if (seg_host) (void)hipHostFree(seg_host);
  counts = scan_l1 = scan_l2 = dbounds = hist_tmp = nullptr;
  hbuf[0] = hbuf[1] = nullptr;
  seg_dev = seg_host = nullptr;
  counts_cap = l2_cap = hbuf_cap = dbounds_cap = seg_cap = hist_tmp_cap = 0;
  if (prev >= 0) (void)hipSetDevice(prev);
}

namespace {

// Blocks per launch for the even-share passes.  The counters array holds
// RADIX * grid entries, so the grid is kept moderate (4 blocks per CU).
uint32_t pass_grid(const Workspace& ws, uint32_t num_tiles) {
  const uint32_t per_cu = 4;
  const uint32_t g = (uint32_t)std::max(1, ws.num_cus) * per_cu;
  return std::max(1u, std::min(num_tiles, g));
}

hipError_t run_scan(Workspace& ws, uint32_t m, hipStream_t st) {
  const uint32_t tiles = (m + kScanTile - 1) / kScanTile;
  ScopedTimer tm("scan", st, m);
  hipLaunchKernelGGL(k_scan_tiles, dim3(tiles), dim3(kScanBlock), 0, st, ws.counts, ws.scan_l1, m,
                     ws.scan_l2);
  LS_TRY(hipGetLastError());
  hipLaunchKernelGGL(k_scan_single, dim3(1), dim3(kScanBlock), 0, st, ws.scan_l2, tiles);
  return hipGetLastError();
}

template <int BITS, typename K, typename V, typename Op>
hipError_t run_pass(Workspace& ws, const K* kin, K* kout, const V* vin, V* vout, size_t n, Op op,
                    hipStream_t st) {
  constexpr int ITEMS = sizeof(K) == 8 ? kItemsU64 : kItemsU32;
  constexpr int TILE = kBlock * ITEMS;
  constexpr int RADIX = 1 << BITS;
  const uint32_t num_tiles = (uint32_t)((n + TILE - 1) / TILE);
  const uint32_t grid = pass_grid(ws, num_tiles);
  const uint32_t m = RADIX * grid;
  LS_TRY(ws.ensure_counts(m));
  {
    ScopedTimer tm("upsweep", st, n);
    const bool vec = (reinterpret_cast<uintptr_t>(kin) % 16) == 0;
    if (vec)
      hipLaunchKernelGGL((k_upsweep<BITS, kBlock, ITEMS, true, K, Op>), dim3(grid), dim3(kBlock), 0,
                         st, kin, (uint32_t)n, num_tiles, grid, op, ws.counts);
    else
      hipLaunchKernelGGL((k_upsweep<BITS, kBlock, ITEMS, false, K, Op>), dim3(grid), dim3(kBlock), 0,
                         st, kin, (uint32_t)n, num_tiles, grid, op, ws.counts);
    LS_TRY(hipGetLastError());
  }
  LS_TRY(run_scan(ws, m, st));
  {
    ScopedTimer tm("downsweep", st, n);
    hipLaunchKernelGGL((k_downsweep<BITS, kBlock, ITEMS, K, V, Op>), dim3(grid), dim3(kBlock), 0, st,
                       kin, kout, vin, vout, (uint32_t)n, num_tiles, grid, op, ws.scan_l1,
                       ws.scan_l2);
    LS_TRY(hipGetLastError());
  }
  return hipSuccess;
}

template <typename K, typename V>
hipError_t run_digit_pass(Workspace& ws, int bits, const K* kin, K* kout, const V* vin, V* vout,
                          size_t n, uint32_t shift, uint32_t nbits, hipStream_t st) {
  RadixDigit op{shift, (nbits >= 32) ? 0xffffffffu : ((1u << nbits) - 1u)};
  if (bits == 8) return run_pass<8>(ws, kin, kout, vin, vout, n, op, st);
  if (bits == 4) return run_pass<4>(ws, kin, kout, vin, vout, n, op, st);
  return hipErrorInvalidValue;
}

template <typename K, typename V>
hipError_t copy_buf(K* dst, const K* src, V* vdst, const V* vsrc, size_t n, hipStream_t st) {
  if (dst != src) LS_TRY(hipMemcpyAsync(dst, src, n * sizeof(K), hipMemcpyDeviceToDevice, st));
  if constexpr (!std::is_same<V, NoValue>::value) {
    if (vdst != vsrc) LS_TRY(hipMemcpyAsync(vdst, vsrc, n * sizeof(V), hipMemcpyDeviceToDevice, st));
  }
  return hipSuccess;
}

// LSD over bits [lo, hi) with ping-pong between out and tmp.
template <typename K, typename V>
hipError_t sort_impl(Workspace& ws, const K* in, K* out, K* tmp, const V* vin, V* vout, V* vtmp,
                     size_t n, int lo, int hi, int bits, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (n > 0xffffffffull) return hipErrorInvalidValue;
  const int width = hi - lo;
  const int P = num_passes(width, bits);
  if (P == 0) return copy_buf(out, in, vout, vin, n, st);
  const bool inplace = (const void*)in == (const void*)out;
  // dst of pass p: when in != out, out for (P-1-p) even; when in == out, tmp
  // for even p (the final pass lands in tmp when P is odd -> one copy).
  auto dst_is_out = [&](int p) { return inplace ? (p & 1) != 0 : ((P - 1 - p) & 1) == 0; };
  const K* ksrc = in;
  const V* vsrc = vin;
  for (int p = 0; p < P; ++p) {
    const int shift = lo + p * bits;
    const int nb = std::min(bits, hi - shift);
    K* kdst = dst_is_out(p) ? out : tmp;
    V* vdst = dst_is_out(p) ? vout : vtmp;
    LS_TRY(run_digit_pass<K, V>(ws, bits, ksrc, kdst, vsrc, vdst, n, (uint32_t)shift, (uint32_t)nb, st));
    ksrc = kdst;
    vsrc = vdst;
  }
  if (ksrc != out) LS_TRY(copy_buf(out, ksrc, vout, vsrc, n, st));
  return hipSuccess;
}

}  // namespace

hipError_t sort_u32(Workspace& ws, const uint32_t* in, uint32_t* out, uint32_t* tmp, size_t n, int lo,
                    int hi, int digit_bits, uint32_t* d_bounds, hipStream_t st) {
  LS_TRY((sort_impl<uint32_t, NoValue>(ws, in, out, tmp, nullptr, nullptr, nullptr, n, lo, hi,
                                      digit_bits, st)));
  if (d_bounds) {
    const int width = hi - lo;
    const uint32_t ngroups = 1u << width;
    ScopedTimer tm("bounds", st, n);
    if (n == 0) {
      LS_TRY(hipMemsetAsync(d_bounds, 0, (size_t)ngroups * sizeof(uint32_t), st));
    } else if (num_passes(width, digit_bits) == 1) {
      // single pass: the counters of that pass are still in the workspace
      constexpr int TILE = kBlock * kItemsU32;
      const uint32_t grid = pass_grid(ws, (uint32_t)((n + TILE - 1) / TILE));
      hipLaunchKernelGGL(k_bounds_from_scan, dim3((ngroups + 255) / 256), dim3(256), 0, st, ws.scan_l1,
                         ws.scan_l2, grid, ngroups, d_bounds);
      LS_TRY(hipGetLastError());
    } else {
      const uint32_t blocks = (uint32_t)std::min<uint64_t>((n + 256) / 256, 4096);
      hipLaunchKernelGGL(k_group_bounds<uint32_t>, dim3(blocks), dim3(256), 0, st, out, (uint32_t)n,
                         (uint32_t)lo, ngroups - 1u, ngroups, d_bounds);
      LS_TRY(hipGetLastError());
    }
  }
  return hipSuccess;
}

hipError_t sort_pairs_u32_u32(Workspace& ws, const uint32_t* kin, const uint32_t* vin, uint32_t* kout,
                              uint32_t* vout, uint32_t* ktmp, uint32_t* vtmp, size_t n, int lo, int hi,
                              int digit_bits, hipStream_t st) {
  return sort_impl<uint32_t, uint32_t>(ws, kin, kout, ktmp, vin, vout, vtmp, n, lo, hi, digit_bits, st);
}

hipError_t sort_pairs_u64_u32(Workspace& ws, const uint64_t* kin, const uint32_t* vin, uint64_t* kout,
                              uint32_t* vout, uint64_t* ktmp, uint32_t* vtmp, size_t n, int lo, int hi,
                              int digit_bits, hipStream_t st) {
  return sort_impl<uint64_t, uint32_t>(ws, kin, kout, ktmp, vin, vout, vtmp, n, lo, hi, digit_bits, st);
}

hipError_t histogram_u32(Workspace& ws, const uint32_t* keys, size_t n, int shift, int bits,
                         uint32_t* d_hist, hipStream_t st) {
  if (bits < 1 || bits > 16 || shift < 0 || shift + bits > 32 || n > 0xffffffffull)
    return hipErrorInvalidValue;
  const uint32_t bins = 1u << bits;
  LS_TRY(hipMemsetAsync(d_hist, 0, bins * sizeof(uint32_t), st));
  if (n == 0) return hipSuccess;
  ScopedTimer tm("histogram", st, n);
  const uint32_t blocks =
      (uint32_t)std::min<uint64_t>((n + 255) / 256, (uint64_t)std::max(1, ws.num_cus) * 4);
  switch (bits) {
#define LS_H(B)                                                                                    \
  case B:                                                                                          \
    hipLaunchKernelGGL(k_hist_lds<B>, dim3(blocks), dim3(256), 0, st, keys, (uint32_t)n,           \
                       (uint32_t)shift, d_hist);                                                   \
    break;
    LS_H(1) LS_H(2) LS_H(3) LS_H(4) LS_H(5) LS_H(6) LS_H(7) LS_H(8) LS_H(9) LS_H(10) LS_H(11) LS_H(12)
#undef LS_H
    default:
      hipLaunchKernelGGL(k_hist_global, dim3(blocks * 4), dim3(256), 0, st, keys, (uint32_t)n,
                         (uint32_t)shift, bins - 1u, d_hist);
  }
  return hipGetLastError();
}

hipError_t partition_u32(Workspace& ws, const uint32_t* in, uint32_t* out, size_t n,
                         const uint32_t* splitters, int nsplit, uint32_t* d_counts, hipStream_t st) {
  if (nsplit < 0 || nsplit > kMaxSplit || n > 0xffffffffull) return hipErrorInvalidValue;
  for (int i = 1; i < nsplit; ++i)
    if (splitters[i] < splitters[i - 1]) return hipErrorInvalidValue;
  SplitDigit op{};
  op.nsplit = (uint32_t)nsplit;
  for (int i = 0; i < nsplit; ++i) op.s[i] = splitters[i];
  const uint32_t nb = (uint32_t)nsplit + 1u;
  if (n == 0) {
    if (d_counts) LS_TRY(hipMemsetAsync(d_counts, 0, nb * sizeof(uint32_t), st));
    return hipSuccess;
  }
  const int bits = nb <= 16 ? 4 : 8;
  if (bits == 4)
    LS_TRY((run_pass<4, uint32_t, NoValue>(ws, in, out, nullptr, nullptr, n, op, st)));
  else
    LS_TRY((run_pass<8, uint32_t, NoValue>(ws, in, out, nullptr, nullptr, n, op, st)));
  if (d_counts) {
    constexpr int TILE = kBlock * kItemsU32;
    const uint32_t grid = pass_grid(ws, (uint32_t)((n + TILE - 1) / TILE));
    hipLaunchKernelGGL(k_bucket_sizes, dim3(nb), dim3(256), 0, st, ws.counts, grid, nb, d_counts);
    LS_TRY(hipGetLastError());
  }
  return hipSuccess;
}

hipError_t segment_copy_u32(Workspace& ws, const uint32_t* src, uint32_t* dst, size_t nseg,
                            const uint64_t* src_off, const uint64_t* dst_off, const uint64_t* len,
                            hipStream_t st) {
  if (nseg == 0) return hipSuccess;
  LS_TRY(ws.ensure_seg(3 * nseg));
  // the pinned staging may still feed the previous call's upload
  LS_TRY(hipEventSynchronize(ws.seg_evt));
  uint64_t total = 0;
  for (size_t i = 0; i < nseg; ++i) {
    ws.seg_host[i] = src_off[i];
    ws.seg_host[nseg + i] = dst_off[i];
    ws.seg_host[2 * nseg + i] = len[i];
    total += len[i];
  }
  LS_TRY(hipMemcpyAsync(ws.seg_dev, ws.seg_host, 3 * nseg * sizeof(uint64_t), hipMemcpyHostToDevice, st));
  LS_TRY(hipEventRecord(ws.seg_evt, st));
  ScopedTimer tm("segcopy", st, total);
  const uint32_t blocks = (uint32_t)std::min<size_t>(nseg, 8192);
  hipLaunchKernelGGL(k_segment_copy, dim3(blocks), dim3(256), 0, st, src, dst, ws.seg_dev, (uint64_t)nseg);
  return hipGetLastError();
}

hipError_t populate_device(uint32_t* out, size_t n, uint64_t first, hipStream_t st) {
  if (n == 0) return hipSuccess;
  ScopedTimer tm("populate", st, n);
  const uint64_t per_block = 256ull * kPopItems;
  const uint64_t blocks = (n + per_block - 1) / per_block;
  if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_populate, dim3((uint32_t)blocks), dim3(256), 0, st, out, (uint64_t)n, first);
  return hipGetLastError();
}

}  // namespace lsort
