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
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstring>
#include <thread>
#include <type_traits>

namespace lsort {

constexpr int kWave = 64;

// ----------------------------------------------------------------------------
// digit extractors
// ----------------------------------------------------------------------------
// Digit = bits [shift, shift + popcount(mask)) of the key; mask = 2^w - 1 with
// w <= 8 (one digit of a pass).
struct RadixDigit {
  uint32_t shift;
  uint32_t mask;
  // one v_bfe_u32 (the width is wave-uniform: s_bcnt1 of the mask, hoisted)
  __device__ __forceinline__ uint32_t operator()(uint32_t k) const {
    return __builtin_amdgcn_ubfe(k, shift, (uint32_t)__builtin_popcount(mask));
  }
  __device__ __forceinline__ uint32_t operator()(uint64_t k) const {
    return (uint32_t)(k >> shift) & mask;
  }
};

// Digit of (key - bias): the keys of a range-restricted sort lie in
// [bias, bias + 2^w) and are ordered by the low w bits of key - bias (w is
// often a digit short of 32: the multi-GPU schedule's rounds).  A type of its
// own so the plain sorts keep their one-instruction digit.
struct BiasedDigit {
  uint32_t shift;
  uint32_t mask;
  uint32_t bias;
  __device__ __forceinline__ uint32_t operator()(uint32_t k) const {
    return __builtin_amdgcn_ubfe(k - bias, shift, (uint32_t)__builtin_popcount(mask));
  }
  __device__ __forceinline__ uint32_t operator()(uint64_t k) const { return (uint32_t)((k - bias) >> shift) & mask; }
};

// Digit of (key - bias) for 64-bit keys with a 64-bit bias: the multi-GPU
// pair partition over the populated key range (keys in [bias, bias +
// 2^(shift + 8)), distrib.cpp range_partition).
struct BiasedDigit64 {
  uint64_t bias;
  uint32_t shift;
  uint32_t mask;
  __device__ __forceinline__ uint32_t operator()(uint64_t k) const { return (uint32_t)((k - bias) >> shift) & mask; }
  __device__ __forceinline__ uint32_t operator()(uint32_t k) const {
    return (uint32_t)(((uint64_t)k - bias) >> shift) & mask;
  }
};

template <typename Op> __host__ __device__ Op make_digit(uint32_t shift, uint32_t mask, uint32_t bias);
template <> __host__ __device__ inline RadixDigit make_digit<RadixDigit>(uint32_t shift, uint32_t mask, uint32_t) {
  return RadixDigit{shift, mask};
}
template <> __host__ __device__ inline BiasedDigit make_digit<BiasedDigit>(uint32_t shift, uint32_t mask,
                                                                            uint32_t bias) {
  return BiasedDigit{shift, mask, bias};
}

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

// Bucket = lut[key >> shift] & mask: a table over the top 32 - shift bits
// (shift >= 20: at most 4096 one-byte entries), staged into LDS by the
// kernels that use it (bind_op).  The mask (radix - 1) keeps a bad table
// entry from indexing outside the kernel's counters.  Used by the range
// partition of the multi-GPU schedule (buckets = (round, destination rank)).
struct LutDigit {
  const uint8_t* g;  // device table, 1 << (32 - shift) entries
  uint32_t shift;
  uint32_t mask;
  const uint8_t* s;  // LDS copy, set by bind_op
  __device__ __forceinline__ uint32_t operator()(uint32_t k) const { return s[k >> shift] & mask; }
  __device__ __forceinline__ uint32_t operator()(uint64_t k) const { return s[(uint32_t)(k >> 32) >> shift] & mask; }
};
constexpr int kLutMaxBytes = 4096;

template <typename Op> struct OpLds { static constexpr int bytes = 1; };
template <> struct OpLds<LutDigit> { static constexpr int bytes = kLutMaxBytes; };

// Stages the op's table (if any) into `smem`; the caller puts a barrier
// between this and the op's first use.
template <typename Op>
__device__ __forceinline__ Op bind_op(Op op, uint8_t* smem, uint32_t tid, uint32_t nthreads) {
  if constexpr (std::is_same<Op, LutDigit>::value) {
    const uint32_t words = (1u << (32 - op.shift)) / 4u;
    for (uint32_t i = tid; i < words; i += nthreads)
      reinterpret_cast<uint32_t*>(smem)[i] = reinterpret_cast<const uint32_t*>(op.g)[i];
    op.s = smem;
  }
  (void)smem; (void)tid; (void)nthreads;
  return op;
}

template <typename K> struct VecOf;
template <> struct VecOf<uint32_t> { using type = uint4; static constexpr int n = 4; };
template <> struct VecOf<uint64_t> { using type = ulonglong2; static constexpr int n = 2; };

__device__ __forceinline__ uint32_t vec_elem(const uint4& v, int c) {
  return c == 0 ? v.x : c == 1 ? v.y : c == 2 ? v.z : v.w;
}
__device__ __forceinline__ uint64_t vec_elem(const ulonglong2& v, int c) { return c == 0 ? v.x : v.y; }

__device__ __forceinline__ uint64_t umin64(uint64_t a, uint64_t b) { return a < b ? a : b; }

// Streaming loads of a pass's input tile: every key is read exactly once per
// pass, so the loads are marked nontemporal (global_load ... nt) and do not
// take L2 lines from the scattered output, whose partial lines at digit-run
// ends merge there.  Measured on MI355X (tools/pass_lab, 2^28 keys, 4-bit
// pass): 408 -> 371 us; in the bench's sort 422 -> 401 us per pass.
// Nontemporal STORES were slower (457 us): the run ends need the L2
// write-combining.  LIBSORT_NT_LOADS=0 at build time turns this off (A/B).
#ifndef LIBSORT_NT_LOADS
#define LIBSORT_NT_LOADS 1
#endif
template <typename T>
__device__ __forceinline__ T load_stream(const T* p) {
#if LIBSORT_NT_LOADS
  return __builtin_nontemporal_load(p);
#else
  return *p;
#endif
}
// 16-byte form for the count kernels' vector loads.  Nontemporal there too:
// with plain loads the count read allocated L2 lines and paid the write-back
// of the previous pass's dirty output lines (measured in the sort, 2^28 keys:
// 4-bit pass-0 counts 236 -> 178 us, 8-bit sort 2.83 -> 2.65 ms).
#ifndef LIBSORT_NT_COUNTS
#define LIBSORT_NT_COUNTS LIBSORT_NT_LOADS
#endif
template <typename VT>
__device__ __forceinline__ VT load_count_vec(const VT* p) {
#if LIBSORT_NT_COUNTS
  typedef unsigned int nv4 __attribute__((ext_vector_type(4)));
  const nv4 x = __builtin_nontemporal_load(reinterpret_cast<const nv4*>(p));
  VT r;
  static_assert(sizeof(VT) == sizeof(nv4), "16-byte vectors");
  __builtin_memcpy(&r, &x, sizeof(r));
  return r;
#else
  return *p;
#endif
}


// Ballot of x != 0 as one v_cmp (left to itself the compiler re-derives the
// predicate from the digit with a shift and a signed compare).
__device__ __forceinline__ uint64_t ballot_nz(uint32_t x) {
  uint64_t m;
  asm("v_cmp_ne_u32_e64 %0, 0, %1" : "=s"(m) : "v"(x));
  return m;
}

// Stable rank of each item among this wave's items of the same digit, items
// in order j = 0..ITEMS-1 and lanes in order within an item.  The peers of a
// lane (the lanes with the same digit) come from BITS ballots: per bit a
// sign-extended extract X (0 or ~0), one v_cmp for the ballot m, and one
// v_bitop3 per 32-bit half accumulating the mismatches (m ^ X) | mis; the last
// bit's bitop3 yields ~mismatch = peers directly.  `row` is the wave's zeroed
// per-digit counter row in LDS; every peer writes the same new count (no
// branch).  FULL: every lane holds a valid key (no predicate).  (A leader-only
// ds_add_rtn + ds_bpermute variant, which lets the items' LDS round trips
// overlap, cost 20-30 VGPRs and one wave/SIMD of occupancy and was slower.)
template <int BITS, bool FULL, int ITEMS, typename K, typename Op, typename R>
__device__ __forceinline__ void rank_items_t(const K (&k)[ITEMS], uint32_t (&rk)[ITEMS], R* row,
                                             uint32_t valid, uint32_t wbase, uint32_t lane, Op op) {
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t d = op(k[j]);
    uint32_t lo = 0u, hi = 0u;
#pragma unroll
    for (int bit = 0; bit < BITS - 1; ++bit) {
      const uint32_t X = (uint32_t)__builtin_amdgcn_sbfe(d, bit, 1);
      const uint64_t m = ballot_nz(X);
      lo = __builtin_amdgcn_bitop3_b32(X, lo, (uint32_t)m, 0xDE);          // (X ^ m) | lo
      hi = __builtin_amdgcn_bitop3_b32(X, hi, (uint32_t)(m >> 32), 0xDE);
    }
    const uint32_t X = (uint32_t)__builtin_amdgcn_sbfe(d, BITS - 1, 1);
    const uint64_t m = ballot_nz(X);
    uint32_t plo = __builtin_amdgcn_bitop3_b32(X, lo, (uint32_t)m, 0x21);  // ~((X ^ m) | lo)
    uint32_t phi = __builtin_amdgcn_bitop3_b32(X, hi, (uint32_t)(m >> 32), 0x21);
    bool ok = true;
    if constexpr (!FULL) {
      ok = wbase + j * kWave + lane < valid;
      const uint64_t vm = __ballot(ok);
      plo &= (uint32_t)vm;
      phi &= (uint32_t)(vm >> 32);
    }
    const uint32_t below = __builtin_amdgcn_mbcnt_hi(phi, __builtin_amdgcn_mbcnt_lo(plo, 0u));
    const uint32_t cnt = (uint32_t)(__builtin_popcount(plo) + __builtin_popcount(phi));
    const uint32_t base = row[d];
    rk[j] = base + below;
    if (FULL || ok) row[d] = (R)(base + cnt);  // all peers write the same value
  }
}

template <int BITS, int ITEMS, typename K, typename Op, typename R>
__device__ __forceinline__ void rank_items(const K (&k)[ITEMS], uint32_t (&rk)[ITEMS], R* row,
                                           bool full, uint32_t valid, uint32_t wbase, uint32_t lane,
                                           Op op) {
  if (full)
    rank_items_t<BITS, true, ITEMS>(k, rk, row, valid, wbase, lane, op);
  else
    rank_items_t<BITS, false, ITEMS>(k, rk, row, valid, wbase, lane, op);
}

// Per-wave digit counter of the tile pass: 16-bit (a wave ranks at most 1024
// keys and the running offsets stay below the 8192-key tile), which keeps the
// 8-bit pass's 8 x 256 counters at 4 KB (measured no slower than 32-bit ones
// for 4- and 8-bit digits, tools/ab_c5.sh + tools/ab_libs.sh).
using WaveCount = uint16_t;
__device__ __forceinline__ uint32_t ob_base(uint32_t o) { return o; }
__device__ __forceinline__ uint32_t ob_base(const uint2& o) { return o.x; }

// Writes the locally sorted tile s_keys[0..valid) (and values) to global
// memory: position i goes to outbase[digit] + i.  Full tiles are unrolled so
// each thread's ITEMS LDS reads and stores issue back to back.
template <int BLOCK, int ITEMS, bool HAS_V, typename K, typename VS, typename V, typename Op>
__device__ __forceinline__ void write_tile(const K* s_keys, const VS* s_vals, const uint32_t* s_outbase,
                                           K* __restrict__ kout, V* __restrict__ vout, uint32_t valid,
                                           Op op) {
  const uint32_t tid = threadIdx.x;
  if (valid == (uint32_t)(BLOCK * ITEMS)) {
    K kk[ITEMS];
    uint32_t o[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) kk[j] = s_keys[tid + j * BLOCK];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) o[j] = s_outbase[op(kk[j])] + tid + j * BLOCK;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      kout[o[j]] = kk[j];
      if constexpr (HAS_V) vout[o[j]] = s_vals[tid + j * BLOCK];
    }
  } else {
    for (uint32_t i = tid; i < valid; i += BLOCK) {
      const K kk = s_keys[i];
      const uint32_t o = s_outbase[op(kk)] + i;
      kout[o] = kk;
      if constexpr (HAS_V) vout[o] = s_vals[i];
    }
  }
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

  const uint32_t wbase = w * WSPAN;
  // Register double buffer: the loads of tile t+1 are issued before tile t is
  // ranked, so their HBM latency overlaps the rank / scan / scatter of tile t.
  K k[ITEMS], kn[ITEMS];
  VS v[ITEMS], vn[ITEMS];
#define LS_LOAD_TILE(KK, VV, T)                                                        \
  do {                                                                                 \
    const uint64_t tb_ = (uint64_t)(T) * TILE;                                         \
    const uint32_t va_ = (uint32_t)umin64((uint64_t)TILE, (uint64_t)n - tb_);          \
    const K* kp_ = kin + tb_ + wbase + lane;                                           \
    const V* vp_ = HAS_V ? vin + tb_ + wbase + lane : nullptr;                         \
    if (va_ == TILE) {                                                                 \
      _Pragma("unroll") for (int j = 0; j < ITEMS; ++j) {                              \
        KK[j] = kp_[j * kWave];                                                        \
        if constexpr (HAS_V) VV[j] = vp_[j * kWave];                                   \
      }                                                                                \
    } else {                                                                           \
      _Pragma("unroll") for (int j = 0; j < ITEMS; ++j) {                              \
        const bool ok_ = wbase + j * kWave + lane < va_;                               \
        KK[j] = ok_ ? kp_[j * kWave] : (K)0;                                           \
        if constexpr (HAS_V) VV[j] = ok_ ? vp_[j * kWave] : (VS)0;                     \
      }                                                                                \
    }                                                                                  \
  } while (0)
  if (t0 < t1) LS_LOAD_TILE(k, v, t0);

  for (uint32_t t = t0; t < t1; ++t) {
    const uint64_t tile_base = (uint64_t)t * TILE;
    const uint32_t valid = (uint32_t)umin64((uint64_t)TILE, (uint64_t)n - tile_base);
    const bool full = valid == TILE;

    if (t + 1 < t1) LS_LOAD_TILE(kn, vn, t + 1);
    for (int d = lane; d < RADIX; d += kWave) s_whist[w][d] = 0u;
    uint32_t rk[ITEMS];

    // Wave-level multi-split: items in order, lanes in order => stable.
    rank_items<BITS, ITEMS>(k, rk, s_whist[w], full, valid, wbase, lane, op);
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
    write_tile<BLOCK, ITEMS, HAS_V>(s_keys, s_vals, s_outbase, kout, vout, valid, op);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      k[j] = kn[j];
      if constexpr (HAS_V) v[j] = vn[j];
    }
  }
#undef LS_LOAD_TILE
}

// ============================================================================
// onesweep path: one histogram read for all digits, then ONE kernel per digit
// pass with decoupled look-back over dynamically numbered tiles.
// ============================================================================
constexpr uint32_t kFlagAgg = 1u << 30;  // status word: tile aggregate published
constexpr uint32_t kFlagInc = 2u << 30;  // status word: inclusive prefix published
constexpr uint32_t kValMask = (1u << 30) - 1u;
constexpr uint32_t kSpinLimit = 1u << 24;

__device__ __forceinline__ void st_agent(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Histograms of the 8-bit windows at shifts lo, lo+8, ... (window q keeps
// min(8, hi - (lo+8q)) bits).  4-bit digit histograms are nibble sums of these.
// Also zeroes the first look-back status buffer (rows of this sort's tiles).
template <typename K, int NW>
__global__ __launch_bounds__(256) void k_window_hist(const K* __restrict__ keys, uint32_t n, uint32_t lo,
                                                     uint32_t hi, uint32_t* __restrict__ whist,
                                                     uint32_t* __restrict__ zero_buf, uint32_t zero_words) {
  constexpr int NWAVE = 4;  // wave-private copies: fewer same-address LDS atomics
  constexpr int UNROLL = 4;  // 16-byte loads in flight per lane
  __shared__ uint32_t s_h[NWAVE][NW][256];
  const int wv = threadIdx.x / kWave;
  for (int i = threadIdx.x; i < NWAVE * NW * 256; i += 256) (&s_h[0][0][0])[i] = 0u;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  const uint64_t gid = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  for (uint64_t i = gid; i < zero_words; i += stride) zero_buf[i] = 0u;
  uint32_t msk[NW];
#pragma unroll
  for (int q = 0; q < NW; ++q) {
    const int s = (int)lo + 8 * q;
    const int nb = min(8, (int)hi - s);
    msk[q] = nb <= 0 ? 0u : ((1u << nb) - 1u);
  }
  __syncthreads();
  auto count = [&](K k) {
#pragma unroll
    for (int q = 0; q < NW; ++q)
      if (msk[q]) atomicAdd(&s_h[wv][q][(uint32_t)(k >> (lo + 8 * q)) & msk[q]], 1u);
  };
  using V = typename VecOf<K>::type;
  constexpr int PER = VecOf<K>::n;
  const uint64_t nvec = ((reinterpret_cast<uintptr_t>(keys) % 16) == 0) ? n / PER : 0;
  const V* vp = reinterpret_cast<const V*>(keys);
  uint64_t i = gid;
  for (; i + (UNROLL - 1) * stride < nvec; i += UNROLL * stride) {
    V v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) v[u] = vp[i + u * stride];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u)
#pragma unroll
      for (int c = 0; c < PER; ++c) count(vec_elem(v[u], c));
  }
  for (; i < nvec; i += stride) {
    const V v = vp[i];
#pragma unroll
    for (int c = 0; c < PER; ++c) count(vec_elem(v, c));
  }
  for (uint64_t e = nvec * PER + gid; e < n; e += stride) count(keys[e]);
  __syncthreads();
  for (int e = threadIdx.x; e < NW * 256; e += 256) {
    uint32_t c = 0;
#pragma unroll
    for (int x = 0; x < NWAVE; ++x) c += (&s_h[x][0][0])[e];
    if (c) atomicAdd(&whist[e], c);
  }
}

// gbase[p][d] = exclusive scan over digits of pass p's histogram.
template <int BITS>
__global__ __launch_bounds__(256) void k_pass_offsets(const uint32_t* __restrict__ whist,
                                                      uint32_t* __restrict__ gbase) {
  constexpr int RADIX = 1 << BITS;
  __shared__ uint32_t s_wsum[4];
  const int p = blockIdx.x;
  const int d = threadIdx.x;
  uint32_t c = 0;
  if (d < RADIX) {
    if (BITS == 8) {
      c = whist[p * 256 + d];
    } else {  // BITS == 4: nibble of window p/2
      const uint32_t* w = whist + (p >> 1) * 256;
      if ((p & 1) == 0) {
        for (int h = 0; h < 16; ++h) c += w[h * 16 + d];
      } else {
        for (int l = 0; l < 16; ++l) c += w[d * 16 + l];
      }
    }
  }
  uint32_t total;
  const uint32_t ex = block_exclusive_scan<256>(c, s_wsum, total);
  if (d < RADIX) gbase[p * RADIX + d] = ex;
}

template <int BITS, int BLOCK, int ITEMS, typename K, typename V, int ABL = 0>
__global__ __launch_bounds__(BLOCK) void k_onesweep(const K* __restrict__ kin, K* __restrict__ kout,
                                                    const V* __restrict__ vin, V* __restrict__ vout,
                                                    uint32_t n, RadixDigit op, uint32_t* status,
                                                    uint32_t* __restrict__ status_next,
                                                    const uint32_t* __restrict__ gbase,
                                                    uint32_t* tile_counter, uint32_t* err) {
  constexpr bool HAS_V = !std::is_same<V, NoValue>::value;
  using VS = typename std::conditional<HAS_V, V, uint8_t>::type;
  constexpr int RADIX = 1 << BITS;
  constexpr int WAVES = BLOCK / kWave;
  constexpr int TILE = BLOCK * ITEMS;
  constexpr int WSPAN = ITEMS * kWave;
  static_assert(RADIX <= BLOCK, "one digit per thread in the block phase");

  __shared__ K s_keys[TILE];
  __shared__ VS s_vals[HAS_V ? TILE : 1];
  __shared__ uint32_t s_whist[WAVES][RADIX];
  __shared__ uint32_t s_outbase[RADIX];
  __shared__ uint32_t s_wsum[WAVES];

  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int w = tid / kWave;

  // Tile id = dispatch order.  A single ticket counter saturates at ~88
  // atomics/us (MI355X_MICROARCH "dequeue"), i.e. ~750 us for 64K tiles, so
  // the look-back relies on the in-order workgroup dispatch observed on
  // gfx950 instead; every wait is bounded (kSpinLimit) and reported in *err.
  const uint32_t t = blockIdx.x;
  for (int d = lane; d < RADIX; d += kWave) s_whist[w][d] = 0u;
  if (status_next != nullptr && tid < RADIX) status_next[(size_t)t * RADIX + tid] = 0u;

  const uint64_t tile_base = (uint64_t)t * TILE;
  const uint32_t valid = (uint32_t)umin64((uint64_t)TILE, (uint64_t)n - tile_base);
  const bool full = valid == TILE;
  const uint32_t wbase = w * WSPAN;

  K k[ITEMS];
  VS v[ITEMS];
  uint32_t rk[ITEMS];
  {
    // one 64-bit base per lane, immediate offsets per item
    const K* kp = kin + tile_base + wbase + lane;
    const V* vp = HAS_V ? vin + tile_base + wbase + lane : nullptr;
    if (full) {
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) {
        k[j] = load_stream(&kp[j * kWave]);
        if constexpr (HAS_V) v[j] = load_stream(&vp[j * kWave]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) {
        const bool ok = wbase + j * kWave + lane < valid;
        k[j] = ok ? kp[j * kWave] : (K)0;
        if constexpr (HAS_V) v[j] = ok ? vp[j * kWave] : (VS)0;
      }
    }
  }

  rank_items<BITS, ITEMS>(k, rk, s_whist[w], full, valid, wbase, lane, op);
  __syncthreads();

  uint32_t cnt_d = 0;
  if (tid < RADIX) {
#pragma unroll
    for (int i = 0; i < WAVES; ++i) cnt_d += s_whist[i][tid];
    // publish this tile's aggregate as early as possible
    st_agent(status + (size_t)t * RADIX + tid, (t == 0 ? kFlagInc : kFlagAgg) | cnt_d);
  }
  uint32_t tile_total;
  const uint32_t excl = block_exclusive_scan<BLOCK>(cnt_d, s_wsum, tile_total);
  if (tid < RADIX) {
    uint32_t prefix = 0;
    if (t > 0 && ABL != 3) {
      // Windowed look-back: LB predecessor words per round trip (independent
      // loads in flight), consumed nearest-first until an inclusive prefix.
      // 64-B rows (4-bit) are cheap to over-read; 1-KB rows (8-bit) are not
      constexpr int LB = RADIX <= 16 ? 8 : 2;
      int64_t j = (int64_t)t - 1;
      uint32_t spins = 0;
      bool done = false;
      while (!done) {
        uint32_t sv[LB];
#pragma unroll
        for (int i = 0; i < LB; ++i)
          sv[i] = (j - i >= 0) ? ld_agent(status + (size_t)(j - i) * RADIX + tid) : kFlagInc;
        int used = 0;
#pragma unroll
        for (int i = 0; i < LB; ++i) {
          if (done || used < i) continue;  // stop at the first unpublished word
          if ((sv[i] & ~kValMask) == 0u) continue;
          prefix += sv[i] & kValMask;
          used = i + 1;
          done = (sv[i] & kFlagInc) != 0u;
        }
        j -= used;
        if (!done && used < LB) {
          if (++spins > kSpinLimit) {
            atomicOr(err, 1u);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      st_agent(status + (size_t)t * RADIX + tid, kFlagInc | (prefix + cnt_d));
    }
    uint32_t run = excl;
#pragma unroll
    for (int i = 0; i < WAVES; ++i) {
      const uint32_t c = s_whist[i][tid];
      s_whist[i][tid] = run;
      run += c;
    }
    s_outbase[tid] = gbase[tid] + prefix - excl;
  }
  __syncthreads();

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

  if constexpr (ABL == 0) {
    write_tile<BLOCK, ITEMS, HAS_V>(s_keys, s_vals, s_outbase, kout, vout, valid, op);
    return;
  }
  for (uint32_t i = tid; i < valid; i += BLOCK) {
    const K kk = s_keys[i];
    const uint32_t o = s_outbase[op(kk)] + i;
    if constexpr (ABL == 0) {
    } else if constexpr (ABL == 1) {  // diagnostic: coalesced writes (wrong result)
      kout[tile_base + i] = kk + o;
    } else {  // diagnostic: no global writes (wrong result)
      asm volatile("" ::"v"(kk), "v"(o));
    }
  }
}

// ============================================================================
// tile-offset path ("tiles"): per-tile digit counts -> two-level column scan
// -> one pass kernel per digit whose tiles know their global run offsets up
// front (no look-back).  With 4-bit digits the pass kernel also counts the
// NEXT digit of every key per destination tile (LDS-aggregated atomics), so
// the keys are read once per pass plus once per sort.
// Layout: C[tile][RADIX] uint32; chunk totals B[chunk][RADIX] with
// kColRows tiles per chunk.  After the scan, tile t's run of digit d starts
// at C[t][d] + B[t / kColRows][d].
// ============================================================================
constexpr int kColRowsPerLane = 16;
// Rows of C per column-scan chunk.  RADIX 256 has one row-lane per column, so
// a lane walks its chunk's rows in one sequential pass and a chunk can be long
// (fewer chunk totals for k_colscan_wide, whose column reads are strided).
#ifndef LIBSORT_COL_ROWS256
#define LIBSORT_COL_ROWS256 64
#endif
constexpr int col_chunk_rows(int radix) { return radix >= 256 ? LIBSORT_COL_ROWS256 : kColRowsPerLane * (256 / radix); }

// Per-tile digit counts of the first pass; also zeroes `zero_buf` (the
// next-pass count buffer).  One block per tile.
// TAB: the tiles of an MSD hybrid depth (tiles[t] = first key, keys; rows of
// blocks past *ntiles are written as zeros: the column scan covers the grid).
template <int BITS, int BLOCK, int ITEMS, typename K, typename Op = RadixDigit, bool TAB = false>
__global__ __launch_bounds__(BLOCK) void k_tile_counts(const K* __restrict__ keys, uint32_t n, Op op_in,
                                                       uint32_t* __restrict__ counts,
                                                       uint32_t* __restrict__ zero_buf, uint32_t zero_words,
                                                       const uint4* __restrict__ tiles,
                                                       const uint32_t* __restrict__ ntiles) {
  constexpr int RADIX = 1 << BITS;
  constexpr int TILE = BLOCK * ITEMS;
  constexpr int COPIES = RADIX <= 16 ? 16 : 1;  // spread same-digit LDS atomics
  __shared__ uint32_t s_h[COPIES][RADIX];
  __shared__ __attribute__((aligned(16))) uint8_t s_lut[OpLds<Op>::bytes];
  const uint32_t tid = threadIdx.x;
  uint64_t tile_base = (uint64_t)blockIdx.x * TILE;
  uint32_t valid;
  if constexpr (TAB) {
    if (blockIdx.x < *ntiles) {
      const uint4 te = tiles[blockIdx.x];
      tile_base = te.x;
      valid = te.y;
    } else {
      valid = 0;
    }
  } else {
    valid = (uint32_t)umin64((uint64_t)TILE, (uint64_t)n - tile_base);
  }
  using VT = typename VecOf<K>::type;
  constexpr int PER = VecOf<K>::n;
  const bool vec = valid == TILE && (reinterpret_cast<uintptr_t>(keys + tile_base) % 16) == 0;
  // TAB tiles start anywhere (a piece of a multi-GPU round's receive buffer,
  // a hybrid child): their keys are read as the 16-byte-ALIGNED words
  // covering them (aligned in absolute address, not relative to `keys`,
  // which may itself sit off a 16-byte boundary), masked to the tile.  Those
  // words never leave the allocation: device allocations start and end on
  // 16-byte (in fact page) boundaries.
  const bool cover = TAB && !vec && valid > 0;
  VT v[ITEMS / PER];
  if (vec) {
    // the tile's loads go out before the table staging and the barrier
    // (LutDigit: the multi-GPU partition's counts 485 -> 369 us at 2^29 keys)
    const VT* vp = reinterpret_cast<const VT*>(keys + tile_base);
#pragma unroll
    for (int j = 0; j < ITEMS / PER; ++j) v[j] = load_count_vec(&vp[j * BLOCK + tid]);
  }
  const Op op = bind_op(op_in, s_lut, tid, BLOCK);
  for (uint32_t i = tid; i < COPIES * RADIX; i += BLOCK) (&s_h[0][0])[i] = 0u;
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + tid; i < zero_words; i += (uint64_t)gridDim.x * BLOCK)
    zero_buf[i] = 0u;
  __syncthreads();
  const uint32_t cp = tid % COPIES;
  if (vec) {
#pragma unroll
    for (int j = 0; j < ITEMS / PER; ++j)
#pragma unroll
      for (int c = 0; c < PER; ++c) atomicAdd(&s_h[cp][op(vec_elem(v[j], c))], 1u);
  } else if (cover) {
    // mis: keys of the first aligned word before the tile
    const uint32_t mis = (uint32_t)((reinterpret_cast<uintptr_t>(keys + tile_base) & 15u) / sizeof(K));
    const VT* vp = reinterpret_cast<const VT*>(keys + tile_base - mis);
    const uint32_t span = valid + mis;
    const uint32_t nv = (span + PER - 1) / PER;
    for (uint32_t q = tid; q < nv; q += BLOCK) {
      const VT x = load_count_vec(&vp[q]);
#pragma unroll
      for (int c = 0; c < PER; ++c) {
        const uint32_t i = q * PER + c;
        if (i >= mis && i < span) atomicAdd(&s_h[cp][op(vec_elem(x, c))], 1u);
      }
    }
  } else {
    for (uint32_t i = tid; i < valid; i += BLOCK) atomicAdd(&s_h[cp][op(keys[tile_base + i])], 1u);
  }
  __syncthreads();
  for (uint32_t d = tid; d < RADIX; d += BLOCK) {
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < COPIES; ++c) s += s_h[c][d];
    counts[(size_t)blockIdx.x * RADIX + d] = s;
  }
}

// Per-tile 8-bit digit counts from the digit stream the previous pass wrote
// (k_tile_pass geo.dout): one byte per key instead of the key (u32: 4 B, u64:
// 8 B).  The tile's bytes are read as the 16-byte words that cover them (any
// alignment: the hybrid's tiles start anywhere); bytes outside the tile are
// masked.  TAB / rows past *ntiles as k_tile_counts.
template <int BLOCK, int TILE, bool TAB = false>
__global__ __launch_bounds__(BLOCK) void k_tile_counts_u8(const uint8_t* __restrict__ dig, uint32_t n,
                                                          uint32_t* __restrict__ counts,
                                                          const uint4* __restrict__ tiles,
                                                          const uint32_t* __restrict__ ntiles) {
  constexpr int RADIX = 256;
  constexpr int COPIES = 2;  // halves the same-bin LDS atomics of a wave's neighbours
  __shared__ uint32_t s_h[COPIES][RADIX];
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < COPIES * RADIX; i += BLOCK) (&s_h[0][0])[i] = 0u;
  __syncthreads();
  uint64_t tile_base = (uint64_t)blockIdx.x * TILE;
  uint32_t valid;
  if constexpr (TAB) {
    if (blockIdx.x < *ntiles) {
      const uint4 te = tiles[blockIdx.x];
      tile_base = te.x;
      valid = te.y;
    } else {
      valid = 0;
    }
  } else {
    valid = (uint32_t)umin64((uint64_t)TILE, (uint64_t)n - tile_base);
  }
  uint32_t* h = s_h[(tid / kWave) % COPIES];
  const uint64_t end = tile_base + valid;
  if (valid == TILE && (tile_base & 15u) == 0) {
    for (uint32_t q = tid; q < TILE / 16; q += BLOCK) {
      const uint4 x = load_count_vec(reinterpret_cast<const uint4*>(dig + tile_base) + q);
      const uint32_t wd[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
      for (int c = 0; c < 16; ++c) atomicAdd(&h[(wd[c >> 2] >> (8 * (c & 3))) & 0xffu], 1u);
    }
  } else if (valid) {
    const uint64_t a0 = tile_base & ~(uint64_t)15;
    for (uint64_t a = a0 + 16ull * tid; a < end; a += 16ull * BLOCK) {
      const uint4 x = load_count_vec(reinterpret_cast<const uint4*>(dig + a));
      const uint32_t wd[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
      for (int c = 0; c < 16; ++c)
        if (a + c >= tile_base && a + c < end) atomicAdd(&h[(wd[c >> 2] >> (8 * (c & 3))) & 0xffu], 1u);
    }
  }
  __syncthreads();
  for (uint32_t d = tid; d < RADIX; d += BLOCK) {
    uint32_t s = 0;
#pragma unroll
    for (int c = 0; c < COPIES; ++c) s += s_h[c][d];
    counts[(size_t)blockIdx.x * RADIX + d] = s;
  }
}

// The column scan turns the per-tile counts C[tile][RADIX] into each tile's
// run offsets: offset(t, d) = C'[t][d] + B[t / CH][d] + D[d] with C' the
// chunk-local exclusive scan (chunks of CH = col_chunk_rows(RADIX)
// rows), B the exclusive scan over chunks and D the digit starts.  The level
// above each kernel runs in that kernel's last-arriving block (last_arriver),
// so a 4-bit pass needs one scan kernel and an 8-bit pass two.

// Last-arriver hand-off (MI355X_MICROARCH.md "Workgroup dispatch, XCD
// placement & inter-workgroup visibility", the counter row of its table):
// every block has published its values with sc1 (write-through) stores; each
// wave waits for them (vmcnt(0)), the block joins a barrier, and one lane adds
// to an agent-scope ticket.  The block whose add returned count - 1 is the
// last: it reads everyone's values with sc1 loads (ld_agent) after a barrier.
// Returns true in that block; it resets the ticket for the next launch.
__device__ __forceinline__ bool last_arriver(uint32_t* ticket, uint32_t count, uint32_t* s_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *s_flag = (t == count - 1u) ? 1u : 0u;
  }
  __syncthreads();
  return *s_flag != 0u;
}

// Level 1: block c owns rows [c*CH, (c+1)*CH).  Thread (row-lane s, column d)
// sums its kColRowsPerLane contiguous rows, the row-lanes are scanned through
// LDS, and the rows are rewritten with the chunk-local exclusive prefix.
// Returns the chunk total of column d (valid for s == 0).
template <int RADIX>
__device__ __forceinline__ uint32_t colscan_chunk(uint32_t* __restrict__ C, uint32_t rows, uint32_t* s_sum) {
  constexpr int L = 256 / RADIX;
  constexpr int CH = col_chunk_rows(RADIX);
  const uint32_t d = threadIdx.x % RADIX, s = threadIdx.x / RADIX;
  if constexpr (L == 1) {
    // one row-lane: exclusive scan down the column in one pass, 16 rows per batch
    const uint64_t r0 = (uint64_t)blockIdx.x * CH;
    uint32_t run = 0;
#pragma unroll
    for (int h = 0; h < CH; h += kColRowsPerLane) {
      uint32_t x[kColRowsPerLane];
#pragma unroll
      for (int i = 0; i < kColRowsPerLane; ++i) x[i] = (r0 + h + i < rows) ? C[(r0 + h + i) * RADIX + d] : 0u;
#pragma unroll
      for (int i = 0; i < kColRowsPerLane; ++i) {
        if (r0 + h + i < rows) C[(r0 + h + i) * RADIX + d] = run;
        run += x[i];
      }
    }
    (void)s_sum;
    (void)s;
    return run;
  } else {
    const uint64_t r0 = (uint64_t)blockIdx.x * CH + (uint64_t)s * kColRowsPerLane;
    uint32_t x[kColRowsPerLane];
    uint32_t sum = 0;
#pragma unroll
    for (int i = 0; i < kColRowsPerLane; ++i) {
      x[i] = (r0 + i < rows) ? C[(r0 + i) * RADIX + d] : 0u;
      sum += x[i];
    }
    s_sum[threadIdx.x] = sum;
    __syncthreads();
    uint32_t run = 0, tot = 0;
    for (uint32_t q = 0; q < (uint32_t)L; ++q) {
      const uint32_t v = s_sum[q * RADIX + d];
      run += q < s ? v : 0u;
      tot += v;
    }
#pragma unroll
    for (int i = 0; i < kColRowsPerLane; ++i) {
      if (r0 + i < rows) C[(r0 + i) * RADIX + d] = run;
      run += x[i];
    }
    return tot;
  }
}

// RADIX <= 32: level 1 per block; the last block scans the chunk totals
// B[nchunks][RADIX] in place (exclusive over chunks) and writes the digit
// starts D[RADIX].
template <int RADIX>
__global__ __launch_bounds__(256) void k_colscan_small(uint32_t* __restrict__ C, uint32_t rows, uint32_t* B,
                                                       uint32_t nchunks, uint32_t* __restrict__ D, uint32_t* ticket) {
  constexpr int L = 256 / RADIX;
  __shared__ uint32_t s_sum[256];
  __shared__ uint32_t s_wsum[4];
  __shared__ uint32_t s_flag;
  const uint32_t d = threadIdx.x % RADIX, s = threadIdx.x / RADIX;
  const uint32_t tot = colscan_chunk<RADIX>(C, rows, s_sum);
  if (s == 0) st_agent(&B[(size_t)blockIdx.x * RADIX + d], tot);
  if (!last_arriver(ticket, gridDim.x, &s_flag)) return;
  const uint32_t per = (nchunks + L - 1) / L;  // chunk rows per row-lane
  const uint32_t a = s * per, b = min(nchunks, a + per);
  // sc1 loads in unrolled batches of 8 (one L2 round trip per batch, not per row)
  constexpr int BATCH = 8;
  uint32_t sum = 0;
  for (uint32_t r0 = a; r0 < b; r0 += BATCH) {
    uint32_t v[BATCH];
#pragma unroll
    for (int i = 0; i < BATCH; ++i) v[i] = (r0 + i < b) ? ld_agent(&B[(size_t)(r0 + i) * RADIX + d]) : 0u;
#pragma unroll
    for (int i = 0; i < BATCH; ++i) sum += v[i];
  }
  s_sum[threadIdx.x] = sum;
  __syncthreads();
  uint32_t run = 0, col = 0;
  for (uint32_t q = 0; q < (uint32_t)L; ++q) {
    const uint32_t v = s_sum[q * RADIX + d];
    run += q < s ? v : 0u;
    col += v;
  }
  uint32_t total_unused;
  const uint32_t ds = block_exclusive_scan<256>(s == 0 ? col : 0u, s_wsum, total_unused);
  if (s == 0) D[d] = ds;
  for (uint32_t r0 = a; r0 < b; r0 += BATCH) {
    uint32_t v[BATCH];
#pragma unroll
    for (int i = 0; i < BATCH; ++i) v[i] = (r0 + i < b) ? ld_agent(&B[(size_t)(r0 + i) * RADIX + d]) : 0u;
#pragma unroll
    for (int i = 0; i < BATCH; ++i) {
      if (r0 + i < b) B[(size_t)(r0 + i) * RADIX + d] = run;
      run += v[i];
    }
  }
  if (threadIdx.x == 0) *ticket = 0u;
}

// RADIX = 256, level 1: chunk totals to B with plain stores (the next kernel
// reads them).
template <int RADIX>
__global__ __launch_bounds__(256) void k_colscan_l1(uint32_t* __restrict__ C, uint32_t rows,
                                                    uint32_t* __restrict__ B) {
  __shared__ uint32_t s_sum[256];
  const uint32_t tot = colscan_chunk<RADIX>(C, rows, s_sum);
  if (threadIdx.x < (uint32_t)RADIX) B[(size_t)blockIdx.x * RADIX + threadIdx.x] = tot;
}

// RADIX = 256, level 2: block d scans column d of B[nchunks][RADIX] in place
// (exclusive) and publishes the column total; the last block turns the totals
// into the digit starts D.
template <int RADIX>
__global__ __launch_bounds__(256) void k_colscan_wide(uint32_t* __restrict__ B, uint32_t nchunks, uint32_t* D,
                                                      uint32_t* ticket) {
  static_assert(RADIX == 256, "one thread per digit in the last block");
  __shared__ uint32_t s_wsum[4];
  __shared__ uint32_t s_flag;
  const uint32_t d = blockIdx.x;
  const uint32_t per = (nchunks + 255) / 256;
  const uint32_t a = threadIdx.x * per, b = min(nchunks, a + per);
  uint32_t sum = 0;
  for (uint32_t r = a; r < b; ++r) sum += B[(size_t)r * RADIX + d];
  uint32_t total;
  uint32_t run = block_exclusive_scan<256>(sum, s_wsum, total);
  for (uint32_t r = a; r < b; ++r) {
    const uint32_t v = B[(size_t)r * RADIX + d];
    B[(size_t)r * RADIX + d] = run;
    run += v;
  }
  if (threadIdx.x == 0) st_agent(&D[d], total);
  if (!last_arriver(ticket, gridDim.x, &s_flag)) return;
  uint32_t total_unused;
  const uint32_t ds = block_exclusive_scan<256>(ld_agent(&D[threadIdx.x]), s_wsum, total_unused);
  D[threadIdx.x] = ds;
  if (threadIdx.x == 0) *ticket = 0u;
}

// Tile handled by block b of a launch whose tiles are independent.  Blocks
// are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md "Workgroup
// dispatch"; speed only, never correctness), so XCD x = b % 8 is given the
// contiguous tile range [x*q + min(x, r), ...) of a q*8 + r grid: the lines
// where neighbouring tiles' digit runs meet are then written through one L2
// and merge there instead of leaving two L2s as partial lines (measured on
// MI355X: 4-bit pass 467 -> 428 us at 2^28 keys; a 256-run scatter probe
// 1305 -> 603 us).  A bijection for every grid size.
__device__ __forceinline__ uint32_t xcd_tile_of(uint32_t b, uint32_t g) {
  const uint32_t q = g >> 3, r = g & 7u, x = b & 7u, i = b >> 3;
  return x * q + min(x, r) + i;
}
__device__ __forceinline__ uint32_t xcd_tile_of_block() { return xcd_tile_of(blockIdx.x, gridDim.x); }

// Tile geometry of the MSD hybrid (sort_hybrid_u32): at depth k >= 1 the
// tiles are cut per segment (the keys sharing their top 4k or 8k bits), so
// tile t = tiles[t] = (first key, keys, segment); the run offsets of segment s
// are D[s * RADIX + d] + the column prefix; and the fused next-digit counts
// go to the next depth's tiles, cut the same way per child (segment * RADIX +
// digit): child c starts at ncstart[c] and its first tile is nctile0[c].
// The slice cursors, kRsvCurStride words apart: every depth-0 tile adds to up
// to 16 of them, ~1M agent-scope adds per 2^28 keys, and same-line atomics
// serialise (all 128 cursors in 4 lines: the depth-0 pass took 2.7 ms instead
// of 0.4).  33 lines apart (an odd line count) puts them on different channels.
constexpr uint32_t kRsvCurStride = 33 * 32;
// Word of slice e = digit * 8 + range's cursor.  8-bit digits: digits 2i and
// 2i + 1 of a range share one 64-bit word (low / high half), so a tile makes
// 128 adds instead of 256 (the halves never carry: a slice holds < 2^32 keys).
__host__ __device__ inline size_t rsv_cur_index(uint32_t e, int radix) {
  if (radix < 256) return (size_t)e * kRsvCurStride;
  const uint32_t d = e / 8u, x = e % 8u;
  return ((size_t)(d >> 1) * 8u + x) * kRsvCurStride + (d & 1u);
}
struct HybridGeo {
  const uint4* tiles;        // GEO & 1: this depth's tile table
  const uint32_t* ntiles;    // GEO & 1: this depth's tile count (blocks past it exit)
  const uint32_t* ncstart;   // GEO & 2: next depth's child starts
  const uint32_t* nctile0;   // GEO & 2: next depth's first tile per child
  uint8_t* dout;             // 8-bit passes (any GEO): op_next of every written key at its output position, or null
  // GEO & 4 (reserved placement, keys-only depth 0 without a count pass;
  // sort_hybrid "Reserved depth 0"): slice e = digit * 8 + range, range
  // = blockIdx.x & 7 (the tile range xcd_tile_of_block gives those blocks)
  // (GEO & 5, a piece sort's depth 0 over its table: slice e = (segment *
  // RADIX + digit) * 8 + range)
  uint32_t* rcur;            // [NS] keys reserved in each slice so far
  const uint32_t* rslice;    // [3][NS] slice start | capacity | first next-depth tile
  uint32_t* rflag;           // set to 1 when a tile's reservation passed its slice's capacity
  uint32_t rns;              // NS: the slices (RADIX * 8 per segment)
  // 24-bit keys of the multi-GPU exchange (round 5; distrib.cpp "wire24"):
  // the partition scatter writes each key's low 16 bits to o16 and bits
  // 16..23 to o8 instead of kout (its top byte is the partition digit, known
  // to the receiver from the piece); a piece sort's depth 0 (GEO 5) reads them
  // back from i16 / i8, the top byte from seghi[segment]
  uint16_t* o16 = nullptr;
  uint8_t* o8 = nullptr;
  const uint16_t* i16 = nullptr;
  const uint8_t* i8 = nullptr;
  const uint32_t* seghi = nullptr;  // [segment] its keys' top byte << 24
};

// The pass kernel of the tile-offset path: the onesweep tile body with the
// run offsets read from the scanned counts.  FUSE: also count the next digit
// (op_next) of every written key per destination tile into C_next (4-bit
// digits: a run of one digit covers at most two destination tiles, so the
// per-tile aggregate has 2 x RADIX x RADIX entries, laid out [slot][d][dn]:
// a wave's sorted keys mostly share d and slot, so its LDS atomics spread
// over consecutive dn banks).  FUSE: the tile's row of C is zeroed after use
// (it becomes the C_next of the pass after the next); otherwise the count
// kernel rewrites every row.
#ifdef LIBSORT_TP_WAVES_PER_EU  // A/B knob: occupancy target of the pass kernel
#define LS_TP_ATTR __attribute__((amdgpu_waves_per_eu(LIBSORT_TP_WAVES_PER_EU)))
#else
#define LS_TP_ATTR
#endif
// ANY_ORDER (the keys-only MSD hybrid's digit passes): the bucket sort orders
// every bucket completely afterwards, so a pass need not keep the input order
// within a digit run; the rank is then one LDS atomic per key instead of the
// ballot rank.  LIBSORT_HYB_ATOMIC_RANK=0 at build time keeps the ballot rank.
#ifndef LIBSORT_HYB_ATOMIC_RANK
#define LIBSORT_HYB_ATOMIC_RANK 1
#endif
template <int BITS, int BLOCK, int ITEMS, typename K, typename V, bool FUSE, typename Op = RadixDigit,
          typename OpN = RadixDigit, int GEO = 0, bool ANY_ORDER = false>
__global__ __launch_bounds__(BLOCK) LS_TP_ATTR void k_tile_pass(const K* __restrict__ kin, K* __restrict__ kout,
                                                     const V* __restrict__ vin, V* __restrict__ vout,
                                                     uint32_t n, Op op_in, OpN op_next,
                                                     uint32_t* __restrict__ C, const uint32_t* __restrict__ B,
                                                     const uint32_t* __restrict__ D, uint32_t* __restrict__ C_next,
                                                     HybridGeo geo) {
  constexpr bool HAS_V = !std::is_same<V, NoValue>::value;
  using VS = typename std::conditional<HAS_V, V, uint8_t>::type;
  constexpr int RADIX = 1 << BITS;
  constexpr int WAVES = BLOCK / kWave;
  constexpr int TILE = BLOCK * ITEMS;
  constexpr int WSPAN = ITEMS * kWave;
  constexpr int CH = col_chunk_rows(RADIX);
  constexpr int NEXT = 2 * RADIX * RADIX;
  constexpr int SPLIT = 2;  // store phase in two unrolled halves (register pressure)
  constexpr int SP = ITEMS / SPLIT;
  static_assert(RADIX <= BLOCK, "one digit per thread in the block phase");
  static_assert(!FUSE || (BITS == 4 && NEXT % BLOCK == 0), "fused next-pass counts: 4-bit digits");

  // STAGE_V (pair tiles of 8192 or 16384 64-bit keys): the values are not
  // given LDS of their own; after the keys have been written to HBM they are
  // scattered into the key buffer and written from there (8192-pair tiles:
  // LDS 69 KB per block instead of 101 KB, two blocks per CU; 16384: 137 KB,
  // one block of 1024 threads).
  constexpr bool STAGE_V = HAS_V && sizeof(K) == 8 && (TILE == 8192 || TILE == 16384);
  static_assert(!STAGE_V || (!FUSE && sizeof(VS) <= sizeof(K)), "staged values: 8-bit pair tiles");
  // LDS per block (occupancy: 160 KiB per CU): the per-wave digit counters
  // are 16-bit, and the destination-tile entries exist only for FUSE.
  using OB = typename std::conditional<FUSE, uint2, uint32_t>::type;
  __shared__ K s_keys[TILE];
  __shared__ VS s_vals[HAS_V && !STAGE_V ? TILE : 1];
  __shared__ WaveCount s_whist[WAVES][RADIX];
  __shared__ OB s_ob[RADIX];  // run base - local start (FUSE: and the local position where the run enters the next tile)
  __shared__ uint32_t s_tfirst[FUSE ? RADIX : 1];
  __shared__ uint32_t s_next[FUSE ? NEXT : 1];
  __shared__ uint32_t s_wsum[WAVES];
  __shared__ __attribute__((aligned(16))) uint8_t s_lut[OpLds<Op>::bytes];
  constexpr bool ATOMIC_RANK = ANY_ORDER && LIBSORT_HYB_ATOMIC_RANK && !HAS_V;
  // (the partition scatter of the 24-bit exchange: geo.o16 / geo.o8)
  constexpr bool PLANAR_OUT = GEO == 0 && !FUSE && sizeof(K) == 4 && !HAS_V;
  __shared__ uint32_t s_acnt[ATOMIC_RANK ? WAVES : 1][ATOMIC_RANK ? RADIX : 1];
  // GEO & 4: the tile's runs go where it reserves them (an agent-scope add
  // per digit on its range's slice cursor) instead of where a count pass and
  // a column scan put them; keys only (any order within a run).
  constexpr bool RSV = (GEO & 4) != 0;
  static_assert(!RSV || (ANY_ORDER && !HAS_V && (GEO & 2) == 0), "reserved placement: keys-only depth 0");
  __shared__ uint32_t s_over;

  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int w = tid / kWave;
  const uint32_t rx = blockIdx.x & 7u;  // RSV: the tile's range (t lies in range rx's tiles)
  uint64_t tile_base;
  uint32_t valid, seg = 0, t, row;  // row: the tile's count row (its table entry's w)
  if constexpr ((GEO & 1) != 0) {
    // the grid is a bound: blocks past this depth's tile count exit, and the
    // XCD-contiguous map is over the count, so every XCD gets its share (a
    // map over the bound, loading the count and the table entry together:
    // 424 vs 415 us per pass, 3 interleaved runs, profiles/r06n_tile_map_ab.txt)
    const uint32_t g = *geo.ntiles;
    if (blockIdx.x >= g) return;
    t = xcd_tile_of(blockIdx.x, g);
    const uint4 te = geo.tiles[t];
    tile_base = te.x;
    valid = te.y;
    seg = te.z;
    row = te.w;
  } else {
    t = xcd_tile_of_block();
    row = t;
    tile_base = (uint64_t)t * TILE;
    valid = (uint32_t)umin64((uint64_t)TILE, (uint64_t)n - tile_base);
  }
  const Op op = bind_op(op_in, s_lut, tid, BLOCK);
  if constexpr (OpLds<Op>::bytes > 1) __syncthreads();
  for (int d = lane; d < RADIX; d += kWave) s_whist[w][d] = 0u;
  if constexpr (FUSE) {
#pragma unroll
    for (int q = 0; q < NEXT / BLOCK; ++q) s_next[tid + q * BLOCK] = 0u;
  }
  // this tile's run offsets (independent of every other tile)
  uint32_t gofs = 0, ncs = 0, nct = 0, rcap = 0, rsv = 0;
  unsigned long long rsv64 = 0;  // RSV, 8-bit: the old value of an even digit's pair word
  if constexpr (RSV) {
    if (tid == 0) s_over = 0u;
    if (tid < RADIX) {
      const uint32_t e = (seg * RADIX + (uint32_t)tid) * 8u + rx;
      ncs = geo.rslice[e];
      rcap = geo.rslice[geo.rns + e];
      nct = geo.rslice[2 * geo.rns + e];
    }
  } else if (tid < RADIX) {
    gofs = C[(size_t)row * RADIX + tid] + B[(size_t)(row / CH) * RADIX + tid] + D[(size_t)seg * RADIX + tid];
    if constexpr (FUSE) C[(size_t)row * RADIX + tid] = 0u;  // the C_next of the pass after the next
    if constexpr (FUSE && (GEO & 2) != 0) {
      // the next depth's child of digit tid (loaded with the offsets, not
      // after the rank where the block would wait for it)
      ncs = geo.ncstart[seg * RADIX + tid];
      nct = geo.nctile0[seg * RADIX + tid];
    }
  }
  const bool full = valid == TILE;
  const uint32_t wbase = w * WSPAN;
  // the next 8-bit pass's digit stream (geo.dout)
  constexpr bool DOUT = !FUSE && BITS == 8 &&
                        (std::is_same<OpN, RadixDigit>::value || std::is_same<OpN, BiasedDigit>::value);
  uint8_t* const dout = geo.dout;

  K k[ITEMS];
  VS v[ITEMS];
  uint32_t rk[ITEMS];
  // keys only: waves issuing their tile's loads go first (8-bit sort of 2^28
  // keys 2.66 -> 2.62 ms, c3 10.69 -> 10.54 ms, interleaved A/B runs; 4-bit
  // unchanged; pairs 0.6% slower, so not for them)
  if constexpr (!HAS_V) __builtin_amdgcn_s_setprio(2);
  // (GEO 5 over 24-bit pieces: geo.i16 / geo.i8 instead of kin)
  constexpr bool PLANAR_IN = (GEO & 5) == 5 && sizeof(K) == 4 && !HAS_V;
  if (PLANAR_IN && geo.i8 != nullptr) {
    // the tile's two planes staged through s_keys (free until the scatter):
    // dword loads from the dword-aligned floor of each plane's byte range (a
    // piece, hence a tile, starts at any key), then 2- and 1-byte LDS reads.
    // (Per-key ushort / ubyte global loads -- 2 x 16 small loads per thread
    // -- ran the depth-0 pass at 361 us against 251 us for u32 keys,
    // profiles/r05f_shape8_*.)  A read past the 16-bit plane's end lands in
    // the 8-bit plane, one past that in the receive buffer's unused quarter.
    static_assert(sizeof(K) * TILE >= 3 * TILE + 8, "staging fits s_keys");
    const uint32_t hi = geo.seghi[seg];
    uint8_t* const st = reinterpret_cast<uint8_t*>(s_keys);
    // (aligned on the ABSOLUTE address: a plane starts at any byte of the
    // receive buffer -- round offset a, 2 * n_recv + a)
    const uint8_t* const p16 = reinterpret_cast<const uint8_t*>(geo.i16) + 2 * tile_base;
    const uint8_t* const p8 = geo.i8 + tile_base;
    const uint32_t a16 = (uint32_t)(reinterpret_cast<uintptr_t>(p16) & 3u);
    const uint32_t a8 = (uint32_t)(reinterpret_cast<uintptr_t>(p8) & 3u);
    const uint32_t* g16 = reinterpret_cast<const uint32_t*>(p16 - a16);
    const uint32_t* g8 = reinterpret_cast<const uint32_t*>(p8 - a8);
    const uint32_t n16 = (a16 + 2 * valid + 3) / 4, n8 = (a8 + valid + 3) / 4;
    uint32_t* const st16 = reinterpret_cast<uint32_t*>(st);
    uint32_t* const st8 = reinterpret_cast<uint32_t*>(st + 2 * TILE + 4);
    constexpr int Q16 = (2 * TILE + 4 + 4 * BLOCK - 1) / (4 * BLOCK), Q8 = (TILE + 4 + 4 * BLOCK - 1) / (4 * BLOCK);
    uint32_t w16[Q16], w8[Q8];
#pragma unroll
    for (int q = 0; q < Q16; ++q) {
      const uint32_t i = tid + q * BLOCK;
      w16[q] = i < n16 ? load_stream(&g16[i]) : 0u;
    }
#pragma unroll
    for (int q = 0; q < Q8; ++q) {
      const uint32_t i = tid + q * BLOCK;
      w8[q] = i < n8 ? load_stream(&g8[i]) : 0u;
    }
#pragma unroll
    for (int q = 0; q < Q16; ++q)
      if ((uint32_t)(tid + q * BLOCK) < n16) st16[tid + q * BLOCK] = w16[q];
#pragma unroll
    for (int q = 0; q < Q8; ++q)
      if ((uint32_t)(tid + q * BLOCK) < n8) st8[tid + q * BLOCK] = w8[q];
    __syncthreads();
    const uint16_t* const l16 = reinterpret_cast<const uint16_t*>(st + a16);
    const uint8_t* const l8 = reinterpret_cast<const uint8_t*>(st8) + a8;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t i = wbase + j * kWave + lane;
      k[j] = (full || i < valid) ? (K)(hi | ((uint32_t)l8[i] << 16) | (uint32_t)l16[i]) : (K)0;
    }
    __syncthreads();  // (s_keys is the scatter's next)
  } else {
    const K* kp = kin + tile_base + wbase + lane;
    const V* vp = HAS_V ? vin + tile_base + wbase + lane : nullptr;
    if (full) {
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) {
        k[j] = load_stream(&kp[j * kWave]);
        if constexpr (HAS_V) v[j] = load_stream(&vp[j * kWave]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) {
        const bool ok = wbase + j * kWave + lane < valid;
        k[j] = ok ? kp[j * kWave] : (K)0;
        if constexpr (HAS_V) v[j] = ok ? vp[j * kWave] : (VS)0;
      }
    }
  }
  if constexpr (!HAS_V) __builtin_amdgcn_s_setprio(0);
  if constexpr (ATOMIC_RANK) {
    // (one wave's LDS operations complete in order: zeroing, atomics, copy)
    for (int d = lane; d < RADIX; d += kWave) s_acnt[w][d] = 0u;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j)
      if (full || wbase + j * kWave + lane < valid) rk[j] = atomicAdd(&s_acnt[w][op(k[j])], 1u);
    for (int d = lane; d < RADIX; d += kWave) s_whist[w][d] = (WaveCount)s_acnt[w][d];
  } else {
    rank_items<BITS, ITEMS>(k, rk, s_whist[w], full, valid, wbase, lane, op);
  }
  __syncthreads();

  uint32_t cnt_d = 0;
  if (tid < RADIX) {
#pragma unroll
    for (int i = 0; i < WAVES; ++i) cnt_d += s_whist[i][tid];
    // RSV: the reservation is issued here and its value first used after the
    // LDS scatter below (the add's round trip overlaps the scan and scatter)
    if constexpr (RSV) {
      if constexpr (RADIX >= 256) {
        // (waves 0 .. RADIX / 64 - 1 whole: every lane takes part)
        const uint32_t odd = __shfl_down(cnt_d, 1);
        if ((tid & 1) == 0 && (cnt_d | odd))
          rsv64 = __hip_atomic_fetch_add(
              reinterpret_cast<unsigned long long*>(
                  &geo.rcur[rsv_cur_index((seg * RADIX + (uint32_t)tid) * 8u + rx, RADIX)]),
              (unsigned long long)cnt_d | ((unsigned long long)odd << 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else if (cnt_d) {
        rsv = __hip_atomic_fetch_add(&geo.rcur[rsv_cur_index((seg * RADIX + (uint32_t)tid) * 8u + rx, RADIX)], cnt_d,
                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  uint32_t tile_total;
  const uint32_t excl = block_exclusive_scan<BLOCK>(cnt_d, s_wsum, tile_total);
  if (tid < RADIX) {
    uint32_t run = excl;
#pragma unroll
    for (int i = 0; i < WAVES; ++i) {
      const uint32_t c = s_whist[i][tid];
      s_whist[i][tid] = (WaveCount)run;
      run += c;
    }
    const uint32_t ob = gofs - excl;
    if constexpr (RSV) {
      // (after the scatter)
    } else if constexpr (FUSE && (GEO & 2) != 0) {
      // next depth's tiles are cut per child: position p of child c is in
      // tile nctile0[c] + (p - ncstart[c]) / TILE
      const uint32_t tl = (gofs - ncs) / TILE;
      s_ob[tid] = make_uint2(ob, ncs + (tl + 1) * TILE - ob);
      s_tfirst[tid] = nct + tl;
    } else if constexpr (FUSE) {
      const uint32_t tf = gofs / TILE;
      s_ob[tid] = make_uint2(ob, (tf + 1) * TILE - ob);
      s_tfirst[tid] = tf;
    } else {
      s_ob[tid] = ob;
    }
  }
  __syncthreads();

#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const bool ok = full || (wbase + j * kWave + lane < valid);
    if (ok) {
      const uint32_t pos = s_whist[w][op(k[j])] + rk[j];
      s_keys[pos] = k[j];
      if constexpr (STAGE_V) rk[j] = pos;
      else if constexpr (HAS_V) s_vals[pos] = v[j];
    }
  }
  if constexpr (RSV) {
    if constexpr (RADIX >= 256)
      if (tid < RADIX) {
        const uint32_t hi = __shfl_up((uint32_t)(rsv64 >> 32), 1);
        rsv = (tid & 1) ? hi : (uint32_t)rsv64;
      }
    if (tid < RADIX) {
      // the run of digit tid lands at [slice start + rsv, + cnt_d) of its
      // slice; the next depth's tiles are numbered per slice (capacity)
      if (cnt_d && rsv + cnt_d > rcap) s_over = 1u;
      gofs = ncs + rsv;
      const uint32_t ob = gofs - excl;
      if constexpr (FUSE) {
        const uint32_t tl = rsv / TILE;
        s_ob[tid] = make_uint2(ob, ncs + (tl + 1) * TILE - ob);
        s_tfirst[tid] = nct + tl;
      } else {
        s_ob[tid] = ob;
      }
    }
  }
  __syncthreads();
  if constexpr (RSV) {
    // a slice overflowed (its sampled capacity was short): this tile writes
    // nothing, the flag sends the whole sort to the fallback (sort_hybrid)
    if (s_over) {
      if (tid == 0) __hip_atomic_fetch_or(geo.rflag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
  }

  if constexpr (STAGE_V) {
    // keys (remembering each written position's run base), then the values
    // through the same buffer
    uint32_t obk[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t i = tid + j * BLOCK;
      if (full || i < valid) {
        const K kk = s_keys[i];
        obk[j] = ob_base(s_ob[op(kk)]);
        kout[obk[j] + i] = kk;
        if constexpr (DOUT)
          if (dout) dout[obk[j] + i] = (uint8_t)op_next(kk);
      }
    }
    __syncthreads();
    VS* s_v = reinterpret_cast<VS*>(s_keys);
#pragma unroll
    for (int j = 0; j < ITEMS; ++j)
      if (full || wbase + j * kWave + lane < valid) s_v[rk[j]] = v[j];
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t i = tid + j * BLOCK;
      if (full || i < valid) vout[obk[j] + i] = s_v[i];
    }
    return;
  }

  if (full) {
    // unrolled halves: the LDS reads of a half issue back to back, then its
    // global stores, then (FUSE) its next-digit LDS atomics
#pragma unroll
    for (int h = 0; h < SPLIT; ++h) {
      K kk[SP];
      OB ob[SP];
#pragma unroll
      for (int j = 0; j < SP; ++j) kk[j] = s_keys[tid + (h * SP + j) * BLOCK];
#pragma unroll
      for (int j = 0; j < SP; ++j) ob[j] = s_ob[op(kk[j])];
#pragma unroll
      for (int j = 0; j < SP; ++j) {
        const uint32_t i = tid + (h * SP + j) * BLOCK;
        if (PLANAR_OUT && geo.o16 != nullptr) {
          geo.o16[ob_base(ob[j]) + i] = (uint16_t)kk[j];
          geo.o8[ob_base(ob[j]) + i] = (uint8_t)((uint32_t)kk[j] >> 16);
        } else {
          kout[ob_base(ob[j]) + i] = kk[j];
        }
        if constexpr (HAS_V) vout[ob_base(ob[j]) + i] = s_vals[i];
        if constexpr (DOUT)
          if (dout) dout[ob_base(ob[j]) + i] = (uint8_t)op_next(kk[j]);
      }
      if constexpr (FUSE) {
#pragma unroll
        for (int j = 0; j < SP; ++j) {
          const uint32_t i = tid + (h * SP + j) * BLOCK;
          const uint32_t slot = i >= ob[j].y ? (uint32_t)(RADIX * RADIX) : 0u;
          const uint32_t e = slot + op(kk[j]) * RADIX + op_next(kk[j]);
          // a wave whose 64 keys share (digit, slot, next digit) -- constant
          // high bits -- adds 64 once instead of 64 same-address LDS atomics
          const uint32_t e0 = __builtin_amdgcn_readfirstlane(e);
          if (__ballot(e != e0) == 0) {
            if (lane == 0) atomicAdd(&s_next[e0], (uint32_t)kWave);
          } else {
            atomicAdd(&s_next[e], 1u);
          }
        }
      }
    }
  } else {
    for (uint32_t i = tid; i < valid; i += BLOCK) {
      const K kk = s_keys[i];
      const uint32_t d = op(kk);
      const OB ob = s_ob[d];
      if (PLANAR_OUT && geo.o16 != nullptr) {
        geo.o16[ob_base(ob) + i] = (uint16_t)kk;
        geo.o8[ob_base(ob) + i] = (uint8_t)((uint32_t)kk >> 16);
      } else {
        kout[ob_base(ob) + i] = kk;
      }
      if constexpr (HAS_V) vout[ob_base(ob) + i] = s_vals[i];
      if constexpr (DOUT)
        if (dout) dout[ob_base(ob) + i] = (uint8_t)op_next(kk);
      if constexpr (FUSE) {
        const uint32_t slot = i >= ob.y ? (uint32_t)(RADIX * RADIX) : 0u;
        atomicAdd(&s_next[slot + d * RADIX + op_next(kk)], 1u);
      }
    }
  }
  if constexpr (FUSE) {
    __syncthreads();
#pragma unroll
    for (int q = 0; q < NEXT / BLOCK; ++q) {
      const uint32_t e = tid + q * BLOCK;
      const uint32_t c = s_next[e];
      if (c) {
        const uint32_t slot = e / (RADIX * RADIX), d = (e / RADIX) % RADIX, dn = e % RADIX;
        atomicAdd(&C_next[(size_t)(s_tfirst[d] + slot) * RADIX + dn], c);
      }
    }
  }
}

// ============================================================================
// Bucket sort: the last level of the MSD hybrid (DESIGN.md §3 "MSD passes +
// bucket sort").  Block b sorts bucket b (bstart[b], blen[b] <= BLOCK*ITEMS
// keys that share every bit above `lbits`) entirely on chip: the keys are
// loaded once into registers, then each BITS-bit LSD step over bits
// [0, lbits) is a stable wave64 ballot rank (rank_items_t), a block scan of
// the digit counts and an LDS scatter, read back in item order; the sorted
// bucket is written out coalesced.  One HBM read and one write per key for
// the low lbits bits instead of lbits/BITS digit passes.  Slots past the end
// of the bucket hold 0xffffffff: they are last in item order and carry the
// largest digit, so every step keeps them behind the real keys and the steps
// run without predicates (range sorts, Op = BiasedDigit: digits of key -
// bias, pads bias - 1).  Grid: an upper bound of buckets; min(*nb, nb_cap)
// is the bucket count; bucket = ilist[block] when a list is given.  A bucket
// larger than the block is left alone, counted in *oversized and (when olist
// is given, up to olist_cap) listed for a block of the next size.  in may equal
// out (a block holds its whole bucket before it writes).
// FIX > 0 (64-bit keys, whose buckets keep 48 bits to sort): the on-chip LSD
// steps cover only the top FIX of the lbits bits; keys then equal in all
// their higher bits form runs (4096 uniform keys over 2^16 values of the top
// FIX = 16 bits: ~128 runs of 2, a few of 3), which are insertion-sorted on
// the whole key in LDS by the thread holding the run's first key -- stable,
// since only larger keys move.  A bucket with a run longer than 64 reloads
// its keys and runs every step instead.
// Keys only (FIX == 0): the first step ranks by LDS atomics instead of the
// ballot rank.  A bucket's input order is arbitrary and equal keys are
// indistinguishable, so the first LSD step need not be stable; only the pads
// must stay behind the real keys of their digit (each wave's pads take their
// ranks after its keys; later waves hold pads only).  LIBSORT_BUCKET_ATOMIC0=0
// at build time keeps the ballot rank (A/B).
#ifndef LIBSORT_BUCKET_ATOMIC0
#define LIBSORT_BUCKET_ATOMIC0 1
#endif
// CNT (32-bit keys only, lbits <= 16; the host picks it): a counting sort on
// chip instead of the LSD steps, bucket_count_place below.
//
// bucket_count_place: the bucket's keys (k, slots past len unused) by their
// low lbits bits v = (key - bias) mod 2^lbits, in 4096 cells c = the top 12
// bits of v and, when lbits > 12, rb = lbits - 12 residual bits r.  Each cell
// is one u64 of 3-bit counts, one per residual value, and the cell's key count
// in the top 16 bits: one LDS atomic per key adds 1 << 3r + 1 << 48 and
// returns the key's rank among its equals (equal keys are indistinguishable,
// so atomic order is as good as any); the block scan of the cell counts
// replaces them with the cell start, and a key's
// position is start + the counts of the smaller residuals (three masked
// popcounts) + its rank.  A 3-bit count that reaches 7 (8+ equal keys) would
// carry: the function then returns false without writing, and the caller
// sorts the bucket by the LSD steps instead (k_bucket_sort; duplicate-heavy
// inputs put whole buckets in one cell, so any per-cell search would grow
// with the square of the cell).  lbits <= 12 places by u32 cell counters (a
// cell is one value).  Every key is placed in LDS (over the cell words, once
// the positions are in registers: 32 KB of LDS per block, not 32 KB + the
// bucket), then the bucket is written out coalesced.  Measured, uniform 2^28 keys in 2^16 buckets (lbits 16):
// the 4-step LSD kernel ~1.0 ms, this path ~0.5 ms.
constexpr int kCntCells = 4096;
__device__ __forceinline__ uint32_t field3_sum(uint64_t w) {
  constexpr uint64_t B0 = 0x249249249249ull;  // bit 0 of each 3-bit count (16 of them)
  return (uint32_t)__popcll(w & B0) + 2u * (uint32_t)__popcll(w & (B0 << 1)) +
         4u * (uint32_t)__popcll(w & (B0 << 2));
}
// Counting modes (the host picks one per launch from lbits and the block):
//   kCntSmall  lbits <= 12: one value per cell, u32 counters;
//   kCnt3      13..16 bits: u64 cells of 16 3-bit residual counts + the key
//              count (overflow at 8 equal keys);
//   kCnt3F     the same, lbits == 16 known at compile time;
//   kCnt2F     lbits == 16, buckets of <= ~5K keys (256-thread blocks): u32
//              cells of 16 2-bit counts, the cell's key count their sum (two
//              popcounts), the cell starts as u16 (24 KB instead of 32 KB of
//              LDS, ~60 instead of ~93 VGPRs: six blocks per CU instead of
//              five).  A 2-bit count overflows at 4 equal keys -- ~4% of the
//              uniform 4096-key buckets of a 2^28 sort (~1/16 key per value)
//              -- and such a bucket goes to the LSD steps (the list launch).
constexpr int kCntSmall = 0, kCnt3 = 1, kCnt3F = 2, kCnt2F = 3;
template <int CAP, int MODE>
constexpr int cnt_lds_words() {  // u64 words: the cell words (and starts), or the keys placed over them
  // (bytes: 2-bit cells + u16 starts 24 KB; u32 counters (kCntSmall) 16 KB,
  // so the bucket's keys set the size there: ~17 KB, 8+ blocks per CU; 3-bit
  // cells 32 KB)
  constexpr int cells = MODE == kCnt2F ? 4 * kCntCells + 2 * kCntCells : MODE == kCntSmall ? 4 * kCntCells
                                                                                        : 8 * kCntCells;
  return (cells > 4 * CAP ? cells : 4 * CAP + 7) / 8;
}
// Exclusive block scan whose wave sums live in `s` (any LDS words the
// block's other waves are done with: the caller's barrier before, and the
// barrier after, keep them from being overwritten while read).
template <int BLOCK>
__device__ __forceinline__ uint32_t block_exclusive_scan_in(uint32_t v, uint32_t* s) {
  uint32_t total;
  const uint32_t ex = block_exclusive_scan<BLOCK>(v, s, total);
  __syncthreads();
  return ex;
}
__device__ __forceinline__ uint32_t field2_sum(uint32_t w) {
  return (uint32_t)__builtin_popcount(w & 0x55555555u) + 2u * (uint32_t)__builtin_popcount(w & 0xAAAAAAAAu);
}
// The weight up to which an overflowed 2-bit bucket is retried with 3-bit
// cells (kCnt2F: the threads that saw a count wrap; a uniform bucket's
// overflow is one value with 4 keys: 1-2).
constexpr uint32_t kRetryMax = 16;
// kCnt2F's inline retry (INL) of a lightly overflowed bucket (a value with 4+
// keys wrapped its 2-bit count: ~4% of the uniform 4096-key buckets of a 2^28
// sort), in the same 24 KB: 3-bit u64 cells over HALF the cell space at a
// time (2048 cells = 16 KB), each key counted and placed in the half its cell
// falls in, the second half's starts after the first half's keys.  Sets rk[j]
// to every key's position; false when a 3-bit count would wrap too (8+ equal
// keys: the caller lists the bucket for the LSD steps).  Replaces round 4's
// separate 3-bit LIST launch over those buckets (~45 us per 2^28 sort: two
// latency-bound rounds of ~20 us buckets).
template <int BLOCK, int ITEMS, typename ValFn>
__device__ __forceinline__ bool retry3_halves(const uint32_t (&k)[ITEMS], uint32_t (&rk)[ITEMS], uint32_t* s_mem,
                                              uint32_t* s_wsum, uint32_t len, uint32_t wbase, uint32_t lane,
                                              ValFn val) {
  constexpr uint32_t HC = kCntCells / 2, PER2 = HC / BLOCK;
  static_assert(PER2 >= 1 && HC % BLOCK == 0, "half-cells per thread");
  uint64_t* const s_c = reinterpret_cast<uint64_t*>(s_mem);
  const uint32_t tid = threadIdx.x;
  auto ci2 = [&](uint32_t c) -> uint32_t { return (c % PER2) * BLOCK + c / PER2; };
  uint32_t base = 0;
#pragma unroll 1
  for (uint32_t h = 0; h < 2; ++h) {
    __syncthreads();  // the region's previous use (the 2-bit cells; half 0) is over
#pragma unroll
    for (uint32_t q = 0; q < PER2; ++q) s_c[q * BLOCK + tid] = 0ull;
    __syncthreads();
    bool ovf = false;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j)
      if (wbase + j * kWave + lane < len) {
        const uint32_t v = val(k[j]), c = v >> 4;
        if ((c / HC) == h) {
          const uint32_t sh = 3u * (v & 15u);
          const uint64_t old = atomicAdd((unsigned long long*)&s_c[ci2(c % HC)], (1ull << sh) + (1ull << 48));
          rk[j] = (uint32_t)(old >> sh) & 7u;
          ovf |= rk[j] == 7u;
        }
      }
    if (__any(ovf) && lane == 0) atomicOr((unsigned long long*)&s_c[0], 1ull << 63);
    __syncthreads();
    if (s_c[0] >> 63) return false;
    uint64_t cw[PER2];
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t q = 0; q < PER2; ++q) {
      cw[q] = s_c[q * BLOCK + tid];
      sum += (uint32_t)(cw[q] >> 48);
    }
    uint32_t total;
    uint32_t run = block_exclusive_scan<BLOCK>(sum, s_wsum, total) + base;
#pragma unroll
    for (uint32_t q = 0; q < PER2; ++q) {
      s_c[q * BLOCK + tid] = (cw[q] & 0xFFFFFFFFFFFFull) | ((uint64_t)run << 48);
      run += (uint32_t)(cw[q] >> 48);
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j)
      if (wbase + j * kWave + lane < len) {
        const uint32_t v = val(k[j]), c = v >> 4;
        if ((c / HC) == h) {
          const uint64_t cc = s_c[ci2(c % HC)];
          rk[j] += (uint32_t)(cc >> 48) + field3_sum(cc & ((1ull << (3u * (v & 15u))) - 1ull));
        }
      }
    base += total;
  }
  return true;
}

// The counting placement works in exactly the cell words (32 KB: five blocks
// of 256 threads per CU): the overflow flag is a spare bit of a cell word,
// the block scan's wave sums borrow cell words once every wave holds its
// cells in registers, and the keys are placed over the words.  Returns false
// (nothing written) on a count overflow.  Returns 0 when placed, else the
// overflow's weight: kCnt2F the threads that saw a count wrap (a uniform
// bucket's overflow is one value with 4 keys: 1-2; a duplicate-heavy bucket
// wraps in most threads), the other modes 1.
template <int BLOCK, int ITEMS, int MODE, typename Op, bool INL = false>
__device__ __forceinline__ uint32_t bucket_count_place(const uint32_t (&k)[ITEMS], uint64_t* s_cw, uint32_t* out,
                                                   uint32_t start, uint32_t len, uint32_t lbits_in, uint32_t bias) {
  constexpr int PER = kCntCells / BLOCK;
  static_assert(PER >= 1 && kCntCells % BLOCK == 0, "cells per thread");
  constexpr bool FIXED = MODE == kCnt3F || MODE == kCnt2F;
  constexpr bool BIAS = !std::is_same<Op, RadixDigit>::value;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
  const uint32_t wbase = w * ITEMS * kWave;
  const uint32_t lbits = FIXED ? 16u : lbits_in;
  const uint32_t rb = FIXED ? 4u : lbits > 12 ? lbits - 12 : 0u;
  const uint32_t lmask = (1u << lbits) - 1u, rmask = (1u << rb) - 1u;
  // cell c's counter at (c % PER) * BLOCK + c / PER: the PER cells a thread
  // scans are one LDS column, read and written without bank conflicts
  auto ci = [&](uint32_t c) -> uint32_t { return (c % PER) * BLOCK + c / PER; };
  auto val = [&](uint32_t x) -> uint32_t { return (BIAS ? x - bias : x) & lmask; };
  uint32_t* const s_keys = reinterpret_cast<uint32_t*>(s_cw);
  auto valid = [&](int j) { return wbase + j * kWave + lane < len; };

  uint32_t rk[ITEMS];
  uint32_t rkp[(ITEMS + 1) / 2];  // kCntSmall: packed 16-bit ranks / positions
  if constexpr (MODE == kCnt2F) {
    // (24 KB of cells and starts: six blocks per CU with room for the flag
    // and the wave sums of their own)
    uint32_t* const s_w = s_keys;                                              // 4096 u32 cells
    uint16_t* const s_st = reinterpret_cast<uint16_t*>(s_keys + kCntCells);  // 4096 u16 starts
    __shared__ uint32_t s_ws2[BLOCK / kWave + 1];                            // wave sums | overflow flag
#pragma unroll
    for (int q = 0; q < PER; ++q) s_w[q * BLOCK + tid] = 0u;
    if (tid == 0) s_ws2[BLOCK / kWave] = 0u;
    __syncthreads();
    bool ovf = false;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j)
      if (valid(j)) {
        const uint32_t v = val(k[j]), sh = 2u * (v & 15u);
        rk[j] = (atomicAdd(&s_w[ci(v >> 4)], 1u << sh) >> sh) & 3u;
        ovf |= rk[j] == 3u;
      }
    const uint64_t bal = __ballot(ovf);
    if (bal && lane == 0) atomicAdd(&s_ws2[BLOCK / kWave], (uint32_t)__popcll(bal));
    __syncthreads();
    if (const uint32_t sev = s_ws2[BLOCK / kWave]) {
      // light (a few values with 4+ keys): the 3-bit retry inline (INL);
      // heavy, or a 3-bit wrap: the caller lists the bucket
      if (!INL || sev > kRetryMax) return sev;
      if (!retry3_halves<BLOCK, ITEMS>(k, rk, s_keys, s_ws2, len, wbase, lane, val)) return kRetryMax + 1;
    } else {
      uint32_t cnt[PER], sum = 0;
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        cnt[q] = field2_sum(s_w[q * BLOCK + tid]);
        sum += cnt[q];
      }
      uint32_t total;
      uint32_t run = block_exclusive_scan<BLOCK>(sum, s_ws2, total);
#pragma unroll
      for (int q = 0; q < PER; ++q) {
        s_st[q * BLOCK + tid] = (uint16_t)run;
        run += cnt[q];
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < ITEMS; ++j)
        if (valid(j)) {
          const uint32_t v = val(k[j]), c = ci(v >> 4);
          rk[j] += (uint32_t)s_st[c] + field2_sum(s_w[c] & ((1u << (2u * (v & 15u))) - 1u));
        }
    }
  } else if constexpr (MODE != kCntSmall) {
#pragma unroll
    for (int q = 0; q < PER; ++q) s_cw[q * BLOCK + tid] = 0ull;
    __syncthreads();
    bool ovf = false;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j)
      if (valid(j)) {
        const uint32_t v = val(k[j]), sh = 3u * (v & rmask);
        const uint64_t old = atomicAdd((unsigned long long*)&s_cw[ci(v >> rb)], (1ull << sh) + (1ull << 48));
        rk[j] = (uint32_t)(old >> sh) & 7u;
        ovf |= rk[j] == 7u;
      }
    // the overflow flag is bit 63 of cell 0 (a count uses 13 of its 16 bits):
    // no LDS beyond the cells (__syncthreads_or would take 256 bytes)
    if (__any(ovf) && lane == 0) atomicOr((unsigned long long*)&s_cw[0], 1ull << 63);
    __syncthreads();
    if (s_cw[0] >> 63) return 1u;
    uint64_t cw[PER];
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      cw[q] = s_cw[q * BLOCK + tid];
      sum += (uint32_t)(cw[q] >> 48);
    }
    // (256-thread blocks: the wave sums borrow cell words, so the block needs
    // exactly 32 KB -- five per CU; larger blocks keep 64 B of their own: the
    // aliasing made the 64-VGPR 1024-thread class spill to scratch)
    uint32_t run;
    if constexpr (BLOCK == 256) {
      __syncthreads();
      run = block_exclusive_scan_in<BLOCK>(sum, s_keys);
    } else {
      __shared__ uint32_t s_ws[BLOCK / kWave];
      uint32_t total;
      run = block_exclusive_scan<BLOCK>(sum, s_ws, total);
    }
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const uint32_t n = (uint32_t)(cw[q] >> 48);
      s_cw[q * BLOCK + tid] = (cw[q] & 0xFFFFFFFFFFFFull) | ((uint64_t)run << 48);
      run += n;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j)
      if (valid(j)) {
        const uint32_t v = val(k[j]);
        const uint64_t c = s_cw[ci(v >> rb)];
        rk[j] += (uint32_t)(c >> 48) + field3_sum(c & ((1ull << (3u * (v & rmask))) - 1ull));
      }
  } else {
    // lbits <= 12: one value per cell, u32 counters (an atomic's return is
    // the key's rank among its equals: no overflow)
    // (ranks and positions < CAP < 2^16: two per register, so the kernel
    // fits 72 VGPRs and seven blocks per CU)
    uint32_t* const s_cnt = s_keys;
#pragma unroll
    for (int q = 0; q < PER; ++q) s_cnt[q * BLOCK + tid] = 0u;
#pragma unroll
    for (int q = 0; q < (ITEMS + 1) / 2; ++q) rkp[q] = 0u;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j)
      if (valid(j)) rkp[j >> 1] |= atomicAdd(&s_cnt[ci(val(k[j]))], 1u) << (16 * (j & 1));
    __syncthreads();
    uint32_t sum = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) sum += s_cnt[q * BLOCK + tid];
    // (the wave sums in 64 B of their own, so the counters stay in LDS and
    // are read again below instead of held in registers: fewer VGPRs, more
    // blocks per CU -- the multi-GPU round sorts' buckets take this path)
    __shared__ uint32_t s_wsS[BLOCK / kWave];
    uint32_t total;
    uint32_t run = block_exclusive_scan<BLOCK>(sum, s_wsS, total);
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const uint32_t c = s_cnt[q * BLOCK + tid];
      s_cnt[q * BLOCK + tid] = run;
      run += c;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j)
      if (valid(j)) rkp[j >> 1] += s_cnt[ci(val(k[j]))] << (16 * (j & 1));
  }
  __syncthreads();  // the keys take the words' place
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (valid(j)) s_keys[MODE == kCntSmall ? (rkp[j >> 1] >> (16 * (j & 1))) & 0xFFFFu : rk[j]] = k[j];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t p = wbase + j * kWave + lane;
    if (p < len) out[(size_t)start + p] = s_keys[p];
  }
  return 0u;
}

// The counting placement's own kernel (32-bit keys without values, lbits <=
// 16; the host picks it): block b places bucket b with bucket_count_place in
// exactly the cell words' LDS (32 KB: five 256-thread blocks per CU; the
// 16K-key buckets of configs[2]: 68 KB and a 64-VGPR budget, two 1024-thread
// blocks per CU).  A bucket larger than the block is listed for the next
// size (as k_bucket_sort); one whose 3-bit counts overflowed (8+ equal keys)
// is written nothing and listed in ovf_list (*ovf_n entries) for the LSD
// steps of k_bucket_sort LIST, so this kernel holds no LSD-step code.
// LIST: a persistent grid over ilist[0, min(*nb, nb_cap)) -- the 3-bit retry
// of the buckets whose 2-bit counts overflowed.  An overflowed bucket is
// written nothing and listed: in retry_list when given and its overflow
// weighs <= kRetryMax (a few values with 4+ keys), else in ovf_list (the LSD
// steps of k_bucket_sort LIST), so this kernel holds no LSD-step code.
template <int BLOCK, int ITEMS, typename Op, int MODE, bool LIST = false, bool INL = false>
__global__ __launch_bounds__(BLOCK)
__attribute__((amdgpu_waves_per_eu(
    BLOCK >= 1024 && ITEMS <= 17 && MODE != kCntSmall ? 8 : (BLOCK == 256 && ITEMS <= 17 && MODE == kCntSmall) ? 7 : 1,
    8)))
void k_bucket_count(const uint32_t* in, uint32_t* out, const uint32_t* __restrict__ bstart,
                    const uint32_t* __restrict__ blen, const uint32_t* __restrict__ nb, uint32_t nb_cap,
                    const uint32_t* __restrict__ ilist, uint32_t lbits, uint32_t bias,
                    uint32_t* __restrict__ oversized, uint32_t* __restrict__ olist, uint32_t olist_cap,
                    uint32_t* __restrict__ ovf_n, uint32_t* __restrict__ ovf_list, uint32_t* __restrict__ retry_n,
                    uint32_t* __restrict__ retry_list) {
  constexpr int CAP = BLOCK * ITEMS;
  static_assert(CAP < 65536, "16-bit cell starts");
  __shared__ uint64_t s_cw[cnt_lds_words<CAP, MODE>()];
  const uint32_t wbase = (threadIdx.x / kWave) * ITEMS * kWave, lane = threadIdx.x & (kWave - 1);
  auto one = [&](const uint32_t b) {
    const uint32_t start = bstart[b], len = blen[b];
    if (len > (uint32_t)CAP) {
      if (threadIdx.x == 0) {
        const uint32_t slot = atomicAdd(oversized, 1u);
        if (olist && slot < olist_cap) olist[slot] = b;
      }
      return;
    }
    if (len == 0) return;
    uint32_t k[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t i = wbase + j * kWave + lane;
      k[j] = i < len ? load_stream(&in[(size_t)start + i]) : 0u;
    }
    const uint32_t sev = bucket_count_place<BLOCK, ITEMS, MODE, Op, INL>(k, s_cw, out, start, len, lbits, bias);
    if (sev && threadIdx.x == 0) {  // (in == out keeps the bucket for the next try)
      if (!INL && retry_list && sev <= kRetryMax)
        retry_list[atomicAdd(retry_n, 1u)] = b;
      else
        ovf_list[atomicAdd(ovf_n, 1u)] = b;
    }
  };
  if constexpr (LIST) {
    const uint32_t cnt = min(*nb, nb_cap);
    for (uint32_t bi = blockIdx.x; bi < cnt; bi += gridDim.x) {
      one(ilist[bi]);
      __syncthreads();  // (the LDS of one bucket before the next one's)
    }
  } else {
    if (blockIdx.x >= min(*nb, nb_cap)) return;
    one(ilist ? ilist[blockIdx.x] : blockIdx.x);
  }
}

// The counting placement for (u64 key, u32 payload) buckets (configs[4]'s
// stable pair sort; round 5).  The bucket's pairs share
// every bit of key - bias above lbits (<= 48); x = bits [lbits - 16, lbits)
// are counted in 4096 u64 cells of 16 3-bit counts (+ the cell's pair count,
// then its start, in the top 16 bits), one LDS atomic per pair, and each pair
// is placed at cell start + the counts of the smaller x in its cell + its
// rank among equal x (atomic order: arbitrary).  What goes there is ONE u64,
// p = (the low lbits of key - bias) << 16 | the pair's input slot, which
// orders exactly as (key, slot): a run of equal x -- a field count >= 2,
// found in the cell words the thread scanned (4096 uniform pairs over 2^16
// values: ~128 runs of 2) -- is insertion-sorted on p, so equal keys end in
// input order and the sort is stable without a stable rank.  The keys are
// written out (the shared high bits put back), then the payloads are put at
// their input slots over the same LDS and gathered through the slots.  LDS: 8
// B per slot (the 32 KB of cells over them); 1024-thread blocks of 5 slots
// (2^28 pairs) at 63 VGPRs, two blocks per CU.  tools/pair_lab, 4096-pair
// buckets of 2^28 pairs (profiles/r05g_pair_lab.txt): the two 8-bit ballot
// steps + fix-up of k_bucket_sort FIX 1682-1791 us; this layout 1385-1400 us
// (key and slot in separate LDS arrays 1474-1506 us, payloads placed too
// 1475-1490 us); a copy through the same LDS footprint 1157 us.  A 3-bit count
// that would wrap (8+ pairs with equal x) writes nothing and lists the bucket
// (ovf_list) for k_bucket_sort's LSD steps; a bucket over the block is listed
// (olist).
template <int BLOCK, int ITEMS, typename Op>
__global__ __launch_bounds__(BLOCK) void k_bucket_pairs(const uint64_t* kin, uint64_t* kout, const uint32_t* vin,
                                                        uint32_t* vout, const uint32_t* __restrict__ bstart,
                                                        const uint32_t* __restrict__ blen,
                                                        const uint32_t* __restrict__ nb, uint32_t nb_cap,
                                                        const uint32_t* __restrict__ ilist, uint32_t lbits,
                                                        uint64_t bias, uint32_t* __restrict__ oversized,
                                                        uint32_t* __restrict__ olist, uint32_t olist_cap,
                                                        uint32_t* __restrict__ ovf_n, uint32_t* __restrict__ ovf_list) {
  constexpr int CAP = BLOCK * ITEMS, PER = kCntCells / BLOCK;
  static_assert(CAP >= kCntCells && CAP < 65536 && kCntCells % BLOCK == 0, "cells over the slots; u16 slots");
  __shared__ uint64_t s_p[CAP];
  __shared__ uint32_t s_ws[BLOCK / kWave];
  if (blockIdx.x >= min(*nb, nb_cap)) return;
  const uint32_t b = ilist ? ilist[blockIdx.x] : blockIdx.x;
  const uint32_t start = bstart[b], len = blen[b];
  if (len > (uint32_t)CAP) {
    if (threadIdx.x == 0) {
      const uint32_t slot = atomicAdd(oversized, 1u);
      if (olist && slot < olist_cap) olist[slot] = b;
    }
    return;
  }
  if (len == 0) return;
  const uint32_t tid = threadIdx.x, lane = tid & (kWave - 1), wbase = (tid / kWave) * ITEMS * kWave;
  uint64_t* const cw = s_p;
  auto ci = [&](uint32_t c) -> uint32_t { return (c % PER) * BLOCK + c / PER; };
  const uint32_t fs = lbits - 16;
  const uint64_t lmask = (1ull << lbits) - 1ull;
  auto valid = [&](int j) { return wbase + j * kWave + lane < len; };
  uint64_t k[ITEMS];
  uint32_t v[ITEMS], rk[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = wbase + j * kWave + lane;
    k[j] = i < len ? load_stream(&kin[(size_t)start + i]) : 0ull;
    v[j] = i < len ? load_stream(&vin[(size_t)start + i]) : 0u;
  }
  // (key - bias from here on; subtracted after every load is in flight -- in
  // the load's select it waited for each load in turn: 1640 vs 1510 us)
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) k[j] -= bias;
  const uint64_t khi = (kin[start] - bias) & ~lmask;  // the bits every pair of the bucket shares
#pragma unroll
  for (int q = 0; q < PER; ++q) cw[q * BLOCK + tid] = 0ull;
  __syncthreads();
  bool ovf = false;
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (valid(j)) {
      const uint32_t x = (uint32_t)(k[j] >> fs) & 0xFFFFu, sh = 3u * (x & 15u);
      const uint64_t old = atomicAdd((unsigned long long*)&cw[ci(x >> 4)], (1ull << sh) + (1ull << 48));
      rk[j] = (uint32_t)(old >> sh) & 7u;
      ovf |= rk[j] == 7u;
    }
  // (the overflow flag: bit 63 of cell 0; a pair count uses 13 of 16 bits)
  if (__any(ovf) && lane == 0) atomicOr((unsigned long long*)&cw[0], 1ull << 63);
  __syncthreads();
  if (cw[0] >> 63) {
    if (tid == 0) ovf_list[atomicAdd(ovf_n, 1u)] = b;  // nothing written: in == out keeps the bucket
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
    if (valid(j)) {
      const uint32_t x = (uint32_t)(k[j] >> fs) & 0xFFFFu;
      const uint64_t cc = cw[ci(x >> 4)];
      rk[j] += (uint32_t)(cc >> 48) + field3_sum(cc & ((1ull << (3u * (x & 15u))) - 1ull));
    }
  __syncthreads();  // the packed pairs take the cells' place
#pragma unroll
  for (int j = 0; j < ITEMS; ++j)
    if (valid(j)) s_p[rk[j]] = ((k[j] & lmask) << 16) | (uint64_t)(wbase + j * kWave + lane);
  __syncthreads();
  // runs of equal x: this thread's cells c = tid * PER + q start at cst[q]
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    constexpr uint64_t B0 = 0x249249249249ull;  // bit 0 of each 3-bit field
    const uint64_t f = c[q] & 0xFFFFFFFFFFFFull;
    uint64_t m = ((f >> 1) | (f >> 2)) & B0;  // fields whose count is >= 2
    while (m) {
      const uint32_t r = (uint32_t)__builtin_ctzll(m) / 3u;
      m &= m - 1;
      const uint32_t L = (uint32_t)(f >> (3u * r)) & 7u;
      const uint32_t p = cst[q] + field3_sum(f & ((1ull << (3u * r)) - 1ull));
      for (uint32_t a = 1; a < L; ++a) {  // stable: p orders as (key, input slot)
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
      kout[(size_t)start + pos] = (khi | (x >> 16)) + bias;
      sl[j] = (uint32_t)x & 0xFFFFu;
    }
  }
  __syncthreads();  // the payloads take the keys' place, at their input slots
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

// LIST: a persistent grid walks a list of buckets (ilist[0, min(*nb,
// nb_cap))) -- the launch after the counting placement, over its overflow
// list.
template <int BITS, int BLOCK, int ITEMS, typename Op = RadixDigit, typename K = uint32_t, typename V = NoValue,
          int FIX = 0, bool LIST = false>
__global__ __launch_bounds__(BLOCK) void k_bucket_sort(const K* in, K* out, const V* vin, V* vout,
                                                       const uint32_t* __restrict__ bstart,
                                                       const uint32_t* __restrict__ blen,
                                                       const uint32_t* __restrict__ nb, uint32_t nb_cap,
                                                       const uint32_t* __restrict__ ilist, uint32_t lbits,
                                                       uint32_t bias, uint32_t* __restrict__ oversized,
                                                       uint32_t* __restrict__ olist, uint32_t olist_cap) {
  constexpr bool HAS_V = !std::is_same<V, NoValue>::value;
  using VS = typename std::conditional<HAS_V, V, uint8_t>::type;
  constexpr int RADIX = 1 << BITS;
  constexpr int WAVES = BLOCK / kWave;
  constexpr int CAP = BLOCK * ITEMS;
  constexpr int WSPAN = ITEMS * kWave;
  constexpr uint32_t kMaxRun = 64;
  constexpr uint32_t kRunList = FIX > 0 ? 2 * kWave : 1;  // run starts listed per wave (FIX)
  static_assert(RADIX <= BLOCK && CAP < 65536, "one digit per thread; 16-bit wave counters");
  static_assert(FIX == 0 || (sizeof(K) == 8 && FIX % BITS == 0 && FIX <= 32), "tie fix-up: 64-bit keys");
  __shared__ K s_keys[CAP];
  __shared__ VS s_vals[HAS_V ? CAP : 1];
  __shared__ WaveCount s_whist[WAVES][RADIX];
  __shared__ WaveCount s_off[RADIX <= kWave ? WAVES : 1][RADIX];
  __shared__ uint32_t s_wsum[WAVES];
  __shared__ uint16_t s_runs[FIX > 0 ? WAVES : 1][kRunList];
  constexpr bool ATOMIC0 = LIBSORT_BUCKET_ATOMIC0 && !HAS_V && FIX == 0;
  __shared__ uint32_t s_acnt[ATOMIC0 ? WAVES : 1][ATOMIC0 ? RADIX : 1];
  K* const sk = s_keys;
  auto one = [&](const uint32_t b) {
  const uint32_t start = bstart[b], len = blen[b];
  if (len > (uint32_t)CAP) {
    if (threadIdx.x == 0) {
      const uint32_t slot = atomicAdd(oversized, 1u);
      if (olist && slot < olist_cap) olist[slot] = b;
    }
    return;
  }
  if (len == 0) return;
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int w = tid / kWave;
  const uint32_t wbase = w * WSPAN;
  const K pad = (K)bias - (K)1;  // every digit of key - bias maximal
  K k[ITEMS];
  VS v[ITEMS];
  uint32_t rk[ITEMS];
  auto load = [&]() {
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) {
      const uint32_t i = wbase + j * kWave + lane;
      k[j] = i < len ? load_stream(&in[(size_t)start + i]) : pad;
      if constexpr (HAS_V) v[j] = i < len ? load_stream(&vin[(size_t)start + i]) : (VS)0;
    }
  };
  // LSD steps over bits [lo_bit, hi_bit) of (key - bias); on return k, v hold
  // the bucket in that order (slot j of wave w = position wbase + j*64 + lane)
  // and s_keys / s_vals the same
  auto steps = [&](uint32_t lo_bit, uint32_t hi_bit) {
    for (uint32_t shift = lo_bit; shift < hi_bit; shift += BITS) {
      const uint32_t nbits = min((uint32_t)BITS, hi_bit - shift);
      const Op op = make_digit<Op>(shift, (1u << nbits) - 1u, bias);
      if (ATOMIC0 && shift == 0) {
        // (one wave's LDS operations complete in order: the zeroing, the
        // keys' atomics, the pads' atomics, the copy to the 16-bit row)
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
        for (int d = lane; d < RADIX; d += kWave) s_whist[w][d] = 0;
        rank_items_t<BITS, true, ITEMS>(k, rk, s_whist[w], 0u, wbase, lane, op);
      }
      __syncthreads();
      if constexpr (RADIX <= kWave) {
        // every wave derives its own run offsets (lane d: the digit-d keys of
        // all waves for smaller digits, plus those of earlier waves): no
        // block scan, two barriers per step
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
        for (int j = 0; j < ITEMS; ++j) {
          const uint32_t pos = s_off[w][op(k[j])] + rk[j];
          sk[pos] = k[j];
          if constexpr (HAS_V) s_vals[pos] = v[j];
        }
      } else {
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
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
          const uint32_t pos = s_whist[w][op(k[j])] + rk[j];
          sk[pos] = k[j];
          if constexpr (HAS_V) s_vals[pos] = v[j];
        }
      }
      __syncthreads();
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) {
        k[j] = sk[wbase + j * kWave + lane];
        if constexpr (HAS_V) v[j] = s_vals[wbase + j * kWave + lane];
      }
    }
  };
  load();
  if constexpr (FIX > 0) {
    const uint32_t fs = lbits > (uint32_t)FIX ? lbits - FIX : 0u;  // keys equal above fs form the runs
    steps(fs, lbits);
    if (fs > 0) {
      // run starts (a key whose bits above fs equal the next position's but
      // not the previous one's) from registers: position p = wbase + j*64 +
      // lane holds k[j]; its neighbours are the adjacent lanes (DPP wave
      // shifts), the adjacent items across lanes 63 / 0 (readlane) and LDS
      // across waves.  The starts are listed per wave, then one lane per run
      // sorts it (the divergent work once per wave, not once per item).
      // (the bits above lbits are the bucket's, so 32 bits from fs decide a
      // tie: FIX <= 32)
      auto hi = [&](K x) -> uint32_t { return (uint32_t)((K)(x - bias) >> fs); };
      auto dpp = [](uint32_t x, uint32_t old, auto ctrl) -> uint32_t {
        return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)x, decltype(ctrl)::value, 0xf, 0xf, false);
      };
      auto readlane = [](uint32_t x, int l) -> uint32_t { return (uint32_t)__builtin_amdgcn_readlane((int)x, l); };
      using WaveShr1 = std::integral_constant<int, 0x138>;  // lane i <- lane i - 1
      using WaveShl1 = std::integral_constant<int, 0x130>;  // lane i <- lane i + 1
      uint32_t h[ITEMS];
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) h[j] = hi(k[j]);
      uint32_t nruns = 0;
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) {
        const uint32_t p = wbase + j * kWave + lane;
        const uint32_t before = j > 0 ? readlane(h[j - 1], kWave - 1) : (wbase > 0 ? hi(sk[wbase - 1]) : 0u);
        const uint32_t after = j + 1 < ITEMS ? readlane(h[j + 1], 0)
                                             : (wbase + WSPAN < len ? hi(sk[wbase + WSPAN]) : 0u);
        // (the shifts run with every lane active: a DPP source lane that is
        // off in EXEC reads as invalid)
        const uint32_t hp = dpp(h[j], before, WaveShr1{});
        const uint32_t hn = dpp(h[j], after, WaveShl1{});
        const bool tie_prev = (p > 0) & (p < len) & (hp == h[j]);
        const bool tie_next = (p + 1 < len) & (hn == h[j]);
        const bool st = tie_next && !tie_prev;
        const uint64_t m = __ballot(st);
        if (st) {
          const uint32_t idx = nruns + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
          if (idx < kRunList) s_runs[w][idx] = (uint16_t)p;
        }
        nruns += (uint32_t)__popcll(m);
      }
      uint32_t long_run = nruns > kRunList ? 1u : 0u;
      if (!long_run) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t r0 = 0; r0 < nruns; r0 += kWave) {
          if (r0 + lane < nruns) {
            // a stable insertion sort of sk[p, p + L) on key - bias
            const uint32_t p = s_runs[w][r0 + lane];
            const uint32_t h0 = hi(sk[p]);
            uint32_t L = 2;
            while (L <= kMaxRun && p + L < len && hi(sk[p + L]) == h0) ++L;
            if (L > kMaxRun) {
              long_run = 1;
            } else {
              for (uint32_t a = 1; a < L; ++a) {
                const K x = sk[p + a];
                VS xv;
                if constexpr (HAS_V) xv = s_vals[p + a];
                uint32_t c = a;
                while (c > 0 && (K)(sk[p + c - 1] - bias) > (K)(x - bias)) {
                  sk[p + c] = sk[p + c - 1];
                  if constexpr (HAS_V) s_vals[p + c] = s_vals[p + c - 1];
                  --c;
                }
                sk[p + c] = x;
                if constexpr (HAS_V) s_vals[p + c] = xv;
              }
            }
          }
        }
      }
      if (__syncthreads_or((int)long_run)) {
        // a long run of equal high bits: every step from the input order
        load();
        steps(0, lbits);
      } else {
#pragma unroll
        for (int j = 0; j < ITEMS; ++j) {
          k[j] = sk[wbase + j * kWave + lane];
          if constexpr (HAS_V) v[j] = s_vals[wbase + j * kWave + lane];
        }
      }
    }
  } else {
    steps(0, lbits);
  }
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t i = wbase + j * kWave + lane;
    if (i < len) {
      out[(size_t)start + i] = k[j];
      if constexpr (HAS_V) vout[(size_t)start + i] = v[j];
    }
  }
  };  // one(b)
  if constexpr (LIST) {
    const uint32_t cnt = min(*nb, nb_cap);
    for (uint32_t bi = blockIdx.x; bi < cnt; bi += gridDim.x) {
      one(ilist[bi]);
      __syncthreads();  // the LDS of one bucket before the next one's
    }
  } else {
    if (blockIdx.x >= min(*nb, nb_cap)) return;
    one(ilist ? ilist[blockIdx.x] : blockIdx.x);
  }
}

// MSD hybrid planning (sort_hybrid_u32).  After the column scan of depth k
// (per-tile counts C' chunk-local, chunk prefixes B, digit starts D over all
// `rows` scanned rows), one thread per child (segment s, digit d):
//   P(t, d) = C'[t][d] + B[t / CH][d]  (the digit-d keys in tiles < t; the
//             column total past the last row),
//   size    = P(t1, d) - P(t0, d) over the segment's tiles [t0, t1),
//   start   = cstart[s] + the sizes of digits < d in s,
//   segbase[s][d] = start - P(t0, d)  (the pass adds P(t, d): the run of
//             tile t lands at start + the digit-d keys of the earlier tiles
//             of its segment),
// and the child's start, size and tile count for the next depth.  Depth 0
// (fixed tiles) has one segment, tiles [0, fixed_tiles), starting at 0.
// The last block to finish (ticket) then, when asked, scans the children's
// tile counts into ctile0_next[0..m] (*ntiles = the next depth's tile count)
// and copies the counter words ctr[11..14] (stats = ctr + 11) to the host's
// pinned mirror: no separate prefix launch, no copy.
template <int RADIX, int TILE>
__global__ __launch_bounds__(256) void k_hyb_children(const uint32_t* __restrict__ C, const uint32_t* __restrict__ B,
                                                      const uint32_t* __restrict__ D, uint32_t rows, uint32_t nkeys,
                                                      uint32_t nseg, const uint32_t* __restrict__ ctile0,
                                                      const uint32_t* __restrict__ cstart, uint32_t fixed_tiles,
                                                      uint32_t* __restrict__ segbase, uint32_t* __restrict__ ncstart,
                                                      uint32_t* __restrict__ nsize, uint32_t* __restrict__ ntl,
                                                      uint32_t* __restrict__ stats, uint32_t cap1, uint32_t* ticket,
                                                      uint32_t* __restrict__ ctile0_next, uint32_t* __restrict__ ntiles,
                                                      const uint32_t* ctr_words, uint32_t* __restrict__ host_words,
                                                      uint32_t* host_seq, uint32_t seq) {
  static_assert(RADIX == 16 || RADIX == 256, "4- or 8-bit digits");
  constexpr int CH = col_chunk_rows(RADIX);
  __shared__ uint32_t s_wsum[4];
  __shared__ uint32_t s_flag;
  const uint32_t g = blockIdx.x * 256 + threadIdx.x;
  const uint32_t seg = g / RADIX, d = g % RADIX;
  const bool live = seg < nseg;
  uint32_t t0 = 0, t1 = fixed_tiles, cs = 0;
  if (ctile0 && live) {
    t0 = ctile0[seg];
    t1 = ctile0[seg + 1];
    cs = cstart[seg];
  }
  const uint32_t total = (d + 1 < (uint32_t)RADIX ? D[d + 1] : nkeys) - D[d];
  auto P = [&](uint32_t t) -> uint32_t {
    return t < rows ? C[(size_t)t * RADIX + d] + B[(size_t)(t / CH) * RADIX + d] : total;
  };
  const uint32_t p0 = live ? P(t0) : 0u;
  const uint32_t size = (live && t1 > t0) ? P(t1) - p0 : 0u;
  uint32_t excl;
  if constexpr (RADIX == 16) {
    const uint32_t l = threadIdx.x & 15u;
    uint32_t x = size;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 16);
      if (l >= (uint32_t)o) x += y;
    }
    excl = x - size;
  } else {
    uint32_t tot;
    excl = block_exclusive_scan<256>(size, s_wsum, tot);
  }
  if (stats) {
    // the last depth: the largest bucket (stats[0]) and the buckets over the
    // first bucket-sort block (stats[1])
    uint32_t mx = size;
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor(mx, o));
    if ((threadIdx.x & (kWave - 1)) == 0 && mx) atomicMax(&stats[0], mx);
    if (size > cap1) atomicAdd(&stats[1], 1u);
  }
  if (live) {
    const uint32_t start = cs + excl;
    segbase[g] = start - p0;
    ncstart[g] = start;
    nsize[g] = size;
    if (ntl) st_agent(&ntl[g], (size + TILE - 1) / TILE);
  }
  if (!ctile0_next && !host_words) return;
  if (!last_arriver(ticket, gridDim.x, &s_flag)) return;
  if (ctile0_next) {
    const uint32_t m = nseg * RADIX, per = (m + 255) / 256;
    const uint32_t a = min(m, threadIdx.x * per), b = min(m, a + per);
    // (batches of 16 loads in flight: a loop of single loads waits on each)
    uint32_t sum = 0;
    for (uint32_t i = a; i < b; i += 16) {
      uint32_t v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = i + q < b ? ld_agent(&ntl[i + q]) : 0u;
#pragma unroll
      for (int q = 0; q < 16; ++q) sum += v[q];
    }
    uint32_t tot;
    uint32_t run = block_exclusive_scan<256>(sum, s_wsum, tot);
    for (uint32_t i = a; i < b; i += 16) {
      uint32_t v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) v[q] = i + q < b ? ld_agent(&ntl[i + q]) : 0u;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        if (i + q < b) ctile0_next[i + q] = run;
        run += v[q];
      }
    }
    if (threadIdx.x == 0) {
      ctile0_next[m] = tot;
      *ntiles = tot;
    }
  }
  if (host_words) {
    if (threadIdx.x < 4) {
      __hip_atomic_store(&host_words[threadIdx.x], ld_agent(&ctr_words[threadIdx.x]), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
      __threadfence_system();
    }
    __syncthreads();
    // then the sequence word the host polls (wait_host_word)
    if (threadIdx.x == 0) __hip_atomic_store(host_seq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (threadIdx.x == 0) *ticket = 0u;
}

// The hybrid's counter words: zero, and [9] = the bucket count.
__global__ void k_hyb_init(uint32_t* __restrict__ ctr, uint32_t nb) {
  if (threadIdx.x < 16) ctr[threadIdx.x] = threadIdx.x == 9 ? nb : 0u;
}

// The next depth's tile table: tile t belongs to the child c with
// ctile0[c] <= t < ctile0[c + 1] (binary search; empty children have no
// tiles); rows [0, bound) of Czero (its fused counts) are zeroed.
template <int RADIX, int TILE>
__global__ __launch_bounds__(256) void k_hyb_expand(const uint32_t* __restrict__ ctile0, uint32_t m,
                                                    const uint32_t* __restrict__ ncstart,
                                                    const uint32_t* __restrict__ nsize,
                                                    const uint32_t* __restrict__ ntiles, uint32_t bound,
                                                    uint4* __restrict__ tiles, uint32_t* __restrict__ Czero) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  if (t >= bound) return;
  if (Czero) {
#pragma unroll
    for (int q = 0; q < RADIX; q += 4)
      *reinterpret_cast<uint4*>(&Czero[(size_t)t * RADIX + q]) = make_uint4(0u, 0u, 0u, 0u);
  }
  if (t >= *ntiles) return;
  uint32_t lo = 0, hi = m;  // largest c with ctile0[c] <= t
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (ctile0[mid] <= t) lo = mid; else hi = mid;
  }
  const uint32_t k = t - ctile0[lo];
  tiles[t] = make_uint4(ncstart[lo] + k * TILE, min((uint32_t)TILE, nsize[lo] - k * TILE), lo, t);
}

// ---- Reserved depth 0 (sort_hybrid, keys-only 32-bit sorts: 4- and 8-bit digits) ----
// The depth-0 pass places a tile's digit runs by reserving space in slices
// (k_tile_pass GEO & 4) instead of reading offsets from a count pass + column
// scan: one HBM read of the keys less.  Slice e = digit d * 8 + range x, range
// x = the tiles blocks b with b % 8 == x take (xcd_tile_of_block: contiguous).
// Its capacity comes from a stratified sample of the range; a tile that finds
// its slice full writes nothing and raises a flag, and the host then runs the
// LSD sort from the untouched input (sort_hybrid).
constexpr int kRsvRanges = 8;
// hyb_host word the samplers raise to the sort's sequence number after their
// size estimates (the host polls it instead of recording an event)
constexpr uint32_t kHybSeqWord = 511;
constexpr uint32_t kHybSeqWord2 = 510;  // k_hyb_children's, after the bucket stats

// Waits until the pinned word *w == v (a kernel's system-scope store): a
// pause spin for the first ~100 us (the usual wait: the word arrives while the
// last queued kernel runs, and the host must see it at once to keep the GPU
// fed), then yields the core between polls, then (after 20 ms: a stream with
// much queued ahead, e.g. a round sort behind an exchange) sleeps 50 us per
// poll.  After LIBSORT_HOST_WAIT_MS (default 1000 ms) it synchronises the
// stream instead, after which the word must hold v (ADVICE r04;
// test_gpu_parity.py::test_host_word_wait_fallback forces this branch).
inline int host_wait_limit_ms() {
  static const int ms = [] {
    const char* e = getenv("LIBSORT_HOST_WAIT_MS");
    return e && *e ? std::max(0, atoi(e)) : 1000;
  }();
  return ms;
}
inline hipError_t wait_host_word(const uint32_t* w, uint32_t v, hipStream_t st) {
  const volatile uint32_t* p = w;
  const auto t0 = std::chrono::steady_clock::now();
  const auto limit = std::chrono::milliseconds(host_wait_limit_ms());
  for (uint32_t i = 1; *p != v; ++i) {
    if ((i & 255u) == 0) {
      const auto dt = std::chrono::steady_clock::now() - t0;
      if (dt >= limit) {
        const hipError_t e = hipStreamSynchronize(st);
        if (e != hipSuccess) return e;
        return *p == v ? hipSuccess : hipErrorUnknown;
      }
      if (dt > std::chrono::milliseconds(20))
        std::this_thread::sleep_for(std::chrono::microseconds(50));
      else if (dt > std::chrono::microseconds(100))
        std::this_thread::yield();
    }
    __builtin_ia32_pause();
  }
  std::atomic_thread_fence(std::memory_order_acquire);
  return hipSuccess;
}
constexpr int kRsvBlocks = 32;  // sampling blocks per range
// samples per thread: 4 for 4-bit digits (32768 per range, ~2048 per slice),
// 16 for 8-bit (131072 per range, ~512 per slice)
template <int RADIX> constexpr int rsv_per_thread() { return RADIX >= 256 ? 16 : 4; }
template <int RADIX> constexpr uint32_t rsv_samples() { return kRsvBlocks * 256 * rsv_per_thread<RADIX>(); }
// capacity of a slice with s of S samples over a range of N > S keys:
// (s + 5 sqrt(s) + 24) * N / S, at most N (a range of <= S keys is counted
// exactly), rounded up to whole tiles (the next depth's tiles start aligned).
// Over the RADIX slices of a range that is at most N (1 + 5 sqrt(RADIX / S) +
// 25 RADIX / S) + RADIX TILE: 4-bit (S = 32768, TILE = 4096) 1.123 N +
// 16 TILE, 8-bit (S = 131072, TILE = 8192) 1.270 N + 256 TILE, so the slices
// of n keys fit in rsv_capacity_bound(n) words.  A slice overflows when its
// digit's keys exceed the estimate by 5 sigma (~3e-7 per slice on any input:
// the strata make the sample at least as good as a random one).
inline size_t rsv_capacity_bound(size_t n, int bits) {
  return bits == 4 ? n + n / 8 + n / 64 + (size_t)8 * 16 * 4096 + 1024
                   : n + n / 4 + n / 32 + (size_t)8 * 256 * 8192 + 1024;
}

__host__ __device__ inline void rsv_range(uint32_t x, uint32_t tiles, uint32_t tile, uint64_t n, uint64_t* k0,
                                          uint64_t* k1) {
  const uint32_t q = tiles >> 3, r = tiles & 7u;
  const uint64_t t0 = (uint64_t)x * q + (x < r ? x : r), t1 = t0 + q + (x < r ? 1u : 0u);
  *k0 = t0 * tile < n ? t0 * tile : n;
  *k1 = t1 * tile < n ? t1 * tile : n;
}

// Grid kRsvRanges * kRsvBlocks: block (x, j) samples range x, writes its
// digit counts to part[block][RADIX] (sc1) and zeroes part of the next
// depth's count rows Czero[0, zero_words) (4-bit: the fused counts land
// there); the last block sums the samples, sets each slice's start /
// capacity / first next-depth row (rslice), the estimated digit sizes (est,
// the host's pinned mirror), the hybrid's counter words, and zeroes the
// slice cursors.  Thread d < RADIX of the last block owns slices d * 8 + x.
template <int RADIX, int TILE, typename Op>
__global__ __launch_bounds__(256) void k_rsv_sample(const uint32_t* __restrict__ keys, uint32_t n, uint32_t tiles,
                                                    Op op, uint32_t* part, uint32_t* __restrict__ rslice,
                                                    uint32_t* __restrict__ rcur, uint32_t* __restrict__ est,
                                                    uint32_t* __restrict__ Czero, uint32_t zero_words,
                                                    uint32_t* ticket, uint32_t* __restrict__ ctr, uint32_t nb,
                                                    bool short_caps, uint32_t seq) {
  static_assert(RADIX <= 256, "one digit per thread");
  constexpr int NS = RADIX * kRsvRanges;
  constexpr int PT = rsv_per_thread<RADIX>();
  constexpr uint32_t S = rsv_samples<RADIX>();
  __shared__ uint32_t s_h[RADIX];
  __shared__ uint32_t s_wsum[2][4];
  __shared__ uint32_t s_flag;
  const uint32_t tid = threadIdx.x;
  const uint32_t x = blockIdx.x / kRsvBlocks, j = blockIdx.x % kRsvBlocks;
  for (uint32_t i = (blockIdx.x * 256 + tid) * 4; i < zero_words; i += gridDim.x * 256 * 4)
    *reinterpret_cast<uint4*>(&Czero[i]) = make_uint4(0u, 0u, 0u, 0u);
  if (tid < RADIX) s_h[tid] = 0u;
  __syncthreads();
  uint64_t k0, k1;
  rsv_range(x, tiles, TILE, n, &k0, &k1);
  const uint64_t N = k1 - k0;
  uint32_t kv[PT];
  bool ok[PT];
#pragma unroll
  for (int q = 0; q < PT; ++q) {
    const uint32_t i = (j * 256 + tid) * PT + q;  // sample i of S
    uint64_t pos;
    if (N <= S) {
      pos = k0 + i;  // every key once
      ok[q] = i < N;
    } else {
      // stratum i of the range, a hashed point inside it
      uint32_t h = (i + 1u) * 0x9E3779B1u ^ (x + 1u) * 0x85EBCA77u;
      h ^= h >> 15;
      h *= 0x2C1B3C6Du;
      h ^= h >> 12;
      pos = k0 + ((uint64_t)i * N + (((uint64_t)h * N) >> 32)) / S;
      ok[q] = true;
    }
    kv[q] = ok[q] ? keys[pos] : 0u;  // (all loads issued before the first atomic)
  }
#pragma unroll
  for (int q = 0; q < PT; ++q)
    if (ok[q]) atomicAdd(&s_h[op(kv[q])], 1u);
  __syncthreads();
  if (tid < RADIX) st_agent(&part[(size_t)blockIdx.x * RADIX + tid], s_h[tid]);
  if (!last_arriver(ticket, gridDim.x, &s_flag)) return;
  uint32_t cap[kRsvRanges], ntl[kRsvRanges], scap = 0, stl = 0;
  double est_d = 0.0;
#pragma unroll
  for (int xr = 0; xr < kRsvRanges; ++xr) {
    cap[xr] = ntl[xr] = 0u;
    if (tid < (uint32_t)RADIX) {
      uint32_t sc = 0;
      for (int b = 0; b < kRsvBlocks; ++b) sc += ld_agent(&part[(size_t)(xr * kRsvBlocks + b) * RADIX + tid]);
      uint64_t a0, a1;
      rsv_range(xr, tiles, TILE, n, &a0, &a1);
      const uint64_t Nx = a1 - a0;
      uint32_t c;
      if (Nx <= S) {
        c = sc;
        est_d += sc;
      } else {
        const double w = (double)Nx / S;
        est_d += sc * w;
        c = (uint32_t)min((double)Nx, ceil(((double)sc + 5.0 * sqrt((double)sc) + 24.0) * w));
      }
      if (short_caps) c /= 2;  // (test knob: half the estimate)
      ntl[xr] = (c + TILE - 1) / TILE;
      cap[xr] = ntl[xr] * TILE;
      scap += cap[xr];
      stl += ntl[xr];
    }
  }
  uint32_t tot_c, tot_t;
  uint32_t start = block_exclusive_scan<256>(scap, s_wsum[0], tot_c);
  uint32_t row0 = block_exclusive_scan<256>(stl, s_wsum[1], tot_t);
  if (tid < (uint32_t)RADIX) {
#pragma unroll
    for (int xr = 0; xr < kRsvRanges; ++xr) {
      const uint32_t e = tid * kRsvRanges + xr;
      rslice[e] = start;
      rslice[NS + e] = cap[xr];
      rslice[2 * NS + e] = row0;
      rcur[rsv_cur_index(e, RADIX)] = 0u;
      start += cap[xr];
      row0 += ntl[xr];
    }
    // est: the host's pinned mirror (read after the stream event that
    // follows this kernel; no copy kernel in between)
    __hip_atomic_store(&est[tid], (uint32_t)min(4294967295.0, est_d + 0.5), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    __threadfence_system();
  }
  __syncthreads();
  if (tid == 0) __hip_atomic_store(&est[kHybSeqWord], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (tid == 0) rslice[3 * NS] = tot_t;
  if (tid < 16) ctr[tid] = tid == 9 ? nb : 0u;  // (k_hyb_init's words)
  if (tid == 0) *ticket = 0u;
}

// Reserved depth 0 of a piece sort (sort_pieces_u32: a multi-GPU round's
// receive buffer, pieces of nseg segments): slice e = (segment * RADIX +
// digit) * 8 + range, NS = nseg * RADIX * 8 <= kRsvMaxSlices.  Range x = the
// tiles [t0, t1) that blocks b % 8 == x take (xcd_tile_of over the depth-0
// table), i.e. the keys of global rank [kb(t0), kb(t1)) in piece order; a
// sample's rank is mapped to its piece by binary search over the pieces'
// cumulative key counts pcum[np + 1], and it counts for (its piece's
// segment, its digit).  PER samples per thread (rsv_pc_per: several
// children per range); otherwise as k_rsv_sample.  est[0] = the largest child's estimated
// size (the host's skew check).
constexpr uint32_t kRsvMaxSlices = 4096;
// samples per thread: 4, 8 or 16 (32768, 65536 or 131072 per range), the
// fewest giving >= 256 per slice.  The samples are random gathers (~70 us per
// 2^20 of them on MI355X), so they are sized to the slices, not fixed: the
// capacity slack at 256 per slice is ~41% of the keys (memory, not passes).
inline int rsv_pc_per(uint32_t nc) { return nc <= 128 ? 4 : nc <= 256 ? 8 : 16; }
constexpr uint32_t kRsvLdsCum = 2048;
template <int RADIX, int TILE, int PER, typename Op>
__global__ __launch_bounds__(256) void k_rsv_sample_pc(const uint32_t* __restrict__ keys,
                                                       const uint8_t* __restrict__ keys8,
                                                       const uint4* __restrict__ pieces,
                                                       const uint32_t* __restrict__ pcum, uint32_t np, uint32_t nseg,
                                                       uint32_t T0, uint32_t n, Op op, uint32_t* part,
                                                       uint32_t* __restrict__ rslice, uint32_t* __restrict__ rcur,
                                                       uint32_t* __restrict__ est, uint32_t* __restrict__ Czero,
                                                       uint32_t zero_words, uint32_t* ticket,
                                                       uint32_t* __restrict__ ctr, uint32_t nb, bool short_caps,
                                                       uint32_t seq) {
  constexpr uint32_t S = kRsvBlocks * 256 * PER;
  constexpr uint32_t kMaxChildren = kRsvMaxSlices / kRsvRanges;
  __shared__ uint32_t s_h[kMaxChildren];
  __shared__ uint32_t s_wsum[2][4];
  __shared__ uint32_t s_flag, s_max;
  __shared__ uint64_t s_kb[kRsvRanges + 1];
  __shared__ uint32_t s_cum[kRsvLdsCum], s_off[kRsvLdsCum], s_w[kRsvLdsCum];
  __shared__ uint16_t s_seg[kRsvLdsCum];
  const uint32_t tid = threadIdx.x, NC = nseg * RADIX, NS = NC * kRsvRanges;
  const uint32_t x = blockIdx.x / kRsvBlocks, j = blockIdx.x % kRsvBlocks;
  for (uint32_t i = (blockIdx.x * 256 + tid) * 4; i < zero_words; i += gridDim.x * 256 * 4)
    *reinterpret_cast<uint4*>(&Czero[i]) = make_uint4(0u, 0u, 0u, 0u);
  for (uint32_t c = tid; c < NC; c += 256) s_h[c] = 0u;
  // the cumulative counts, and the pieces' first tiles, key offsets and
  // segments, are read from LDS when they fit (a round's np = sources *
  // segments, 512 at 8 GPUs): the searches below are chains of dependent
  // loads, ~1 us each from HBM
  const bool lds = np < kRsvLdsCum;
  if (lds)
    for (uint32_t i = tid; i <= np; i += 256) {
      const uint32_t c = pcum[i];
      s_cum[i] = c;
      if (i < np) {
        const uint4 pc = pieces[i];
        s_w[i] = pc.w;
        s_off[i] = pc.x - c;  // (mod 2^32: key index = rank + s_off)
        s_seg[i] = pc.z;
      }
    }
  const uint32_t* cum = lds ? s_cum : pcum;
  __syncthreads();
  // keys before depth-0 tile t (the tiles of piece p are full but its last)
  auto kb = [&](uint32_t t) -> uint64_t {
    if (t >= T0) return n;
    auto w = [&](uint32_t p) { return lds ? s_w[p] : pieces[p].w; };
    uint32_t lo = 0, hi = np;
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (w(mid) <= t) lo = mid; else hi = mid;
    }
    return (uint64_t)cum[lo] + (uint64_t)(t - w(lo)) * TILE;
  };
  // range xr = the keys [s_kb[xr], s_kb[xr + 1]): the 9 bounds are searched
  // once, by 9 threads, not per use
  const uint32_t q8 = T0 >> 3, r8 = T0 & 7u;
  if (tid <= (uint32_t)kRsvRanges) s_kb[tid] = kb(tid * q8 + min(tid, r8));
  __syncthreads();
  const uint64_t k0 = s_kb[x], N = s_kb[x + 1] - k0;
  // three phases over the thread's samples so that each phase's loads are
  // all in flight together: ranks + piece searches (LDS, lock-step levels),
  // the pieces (LDS, or global past kRsvLdsCum), then the keys
  uint64_t rank[PER];
  uint32_t lo[PER], kv[PER], sg[PER];
  bool ok[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const uint32_t i = (j * 256 + tid) * PER + q;
    if (N <= S) {
      rank[q] = k0 + i;
      ok[q] = i < N;
    } else {
      uint32_t h = (i + 1u) * 0x9E3779B1u ^ (x + 1u) * 0x85EBCA77u;
      h ^= h >> 15;
      h *= 0x2C1B3C6Du;
      h ^= h >> 12;
      rank[q] = k0 + ((uint64_t)i * N + (((uint64_t)h * N) >> 32)) / S;
      ok[q] = true;
    }
    lo[q] = 0u;
  }
  // lo = the last piece with cum[lo] <= rank (the piece holding that rank)
  for (uint32_t step = np > 1 ? 1u << (31 - __builtin_clz(np - 1)) : 0u; step; step >>= 1) {
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const uint32_t m = lo[q] + step;
      if (m < np && cum[m] <= rank[q]) lo[q] = m;
    }
  }
  uint32_t off[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    if (lds) {
      off[q] = s_off[lo[q]];
      sg[q] = s_seg[lo[q]];
    } else {
      const uint4 pc = pieces[lo[q]];
      off[q] = pc.x - cum[lo[q]];
      sg[q] = pc.z;
    }
  }
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    // (24-bit pieces: depth 0's digit lies in bits 16..23, the i8 plane)
    const uint32_t at = (uint32_t)rank[q] + off[q];
    kv[q] = !ok[q] ? 0u : keys8 ? (uint32_t)keys8[at] << 16 : keys[at];
  }
#pragma unroll
  for (int q = 0; q < PER; ++q)
    if (ok[q]) atomicAdd(&s_h[sg[q] * RADIX + op(kv[q])], 1u);
  __syncthreads();
  for (uint32_t c = tid; c < NC; c += 256) st_agent(&part[(size_t)blockIdx.x * NC + c], s_h[c]);
  // two levels: range x's last block sums its range's kRsvBlocks rows into
  // the range's first row (ticket[1 + x]), the last of those finishes
  // (ticket[0]); a thread per child, all its loads in flight together
  if (!last_arriver(ticket + 1 + x, kRsvBlocks, &s_flag)) return;
  for (uint32_t c = tid; c < NC; c += 256) {
    uint32_t v[kRsvBlocks], sc = 0;
#pragma unroll
    for (int b = 0; b < kRsvBlocks; ++b) v[b] = ld_agent(&part[(size_t)(x * kRsvBlocks + b) * NC + c]);
#pragma unroll
    for (int b = 0; b < kRsvBlocks; ++b) sc += v[b];
    st_agent(&part[(size_t)x * kRsvBlocks * NC + c], sc);
  }
  if (tid == 0) ticket[1 + x] = 0u;
  if (!last_arriver(ticket, kRsvRanges, &s_flag)) return;
  // thread tid: children [tid * CPT, ...), their 8 range slices each
  // (contiguous slices e = c * 8 + range)
  const uint32_t CPT = (NC + 255) / 256;
  uint32_t scap = 0, stl = 0, mx = 0;
  if (tid == 0) s_max = 0u;
  for (uint32_t cc = 0; cc < CPT; ++cc) {
    const uint32_t c = tid * CPT + cc;
    if (c >= NC) break;
    double est_c = 0.0;
    uint32_t scx[kRsvRanges];
#pragma unroll
    for (int xr = 0; xr < kRsvRanges; ++xr) scx[xr] = ld_agent(&part[(size_t)xr * kRsvBlocks * NC + c]);
#pragma unroll
    for (uint32_t xr = 0; xr < (uint32_t)kRsvRanges; ++xr) {
      const uint32_t sc = scx[xr];
      const uint64_t Nx = s_kb[xr + 1] - s_kb[xr];
      uint32_t cap;
      if (Nx <= S) {
        cap = sc;
        est_c += sc;
      } else {
        const double w = (double)Nx / S;
        est_c += sc * w;
        cap = (uint32_t)min((double)Nx, ceil(((double)sc + 5.0 * sqrt((double)sc) + 24.0) * w));
      }
      if (short_caps) cap /= 2;
      const uint32_t nt = (cap + TILE - 1) / TILE;
      // (capacity and tile count kept in rslice for the second sweep below)
      rslice[NS + c * kRsvRanges + xr] = nt * TILE;
      scap += nt * TILE;
      stl += nt;
    }
    mx = max(mx, (uint32_t)min(4294967295.0, est_c + 0.5));
  }
  atomicMax(&s_max, mx);
  uint32_t tot_c, tot_t;
  uint32_t start = block_exclusive_scan<256>(scap, s_wsum[0], tot_c);
  uint32_t row0 = block_exclusive_scan<256>(stl, s_wsum[1], tot_t);
  __threadfence_block();
  for (uint32_t cc = 0; cc < CPT; ++cc) {
    const uint32_t c = tid * CPT + cc;
    if (c >= NC) break;
    for (uint32_t xr = 0; xr < (uint32_t)kRsvRanges; ++xr) {
      const uint32_t e = c * kRsvRanges + xr;
      const uint32_t cap = rslice[NS + e];
      rslice[e] = start;
      rslice[2 * NS + e] = row0;
      rcur[rsv_cur_index(e, RADIX)] = 0u;
      start += cap;
      row0 += cap / TILE;
    }
  }
  __syncthreads();
  if (tid == 0) {
    rslice[3 * NS] = tot_t;
    __hip_atomic_store(&est[0], s_max, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __threadfence_system();
    __hip_atomic_store(&est[kHybSeqWord], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (tid < 16) ctr[tid] = tid == 9 ? nb : 0u;  // (k_hyb_init's words; k_hyb_pieces sets ctr[0] after)
  if (tid == 0) *ticket = 0u;
}

// After the reserved depth-0 pass: the next depth's tile table, the
// children's starts in the next depth's (compact) output, their tile (row)
// ranges and the tile count.  FUSED (4-bit): the count rows are numbered by
// slice capacity (slice e's rows [row0[e], row0[e] + ceil(cap / TILE)); the
// fused counts of depth 0 went there), each listed tile carries its row
// (entry w); otherwise (8-bit: the next depth's counts are read from the
// table) row = the tile's index.  Only the tiles that hold keys are listed,
// so no block is spent on the capacity slack.  On overflow (*flag) there are
// no tiles and (FUSED) the next depth's count rows are zeroed, so the later
// depths do nothing (the host then sorts from the input).  Grid: ceil(bound
// / 256), bound = the rows the next depth scans.
template <int RADIX, int TILE, bool FUSED>
__global__ __launch_bounds__(256) void k_rsv_tiles(const uint32_t* __restrict__ rslice,
                                                   const uint32_t* __restrict__ rcur, const uint32_t* __restrict__ flag,
                                                   uint32_t bound, uint4* __restrict__ tiles,
                                                   uint32_t* __restrict__ cstart, uint32_t* __restrict__ ctile0,
                                                   uint32_t* __restrict__ ntiles, uint32_t* __restrict__ Czero,
                                                   uint32_t nc) {
  // nc children (segments x RADIX digits), NS = nc * 8 slices; thread tid
  // holds slices [tid * SPT, (tid + 1) * SPT)
  constexpr uint32_t kMaxSpt = kRsvMaxSlices / 256;
  // ~65.6 KB of static LDS (4 x 4097 words + s_wsum): gfx950 gives a
  // workgroup 160 KB; gfx942 and older (64 KB) could not launch this kernel,
  // and this library is built for gfx950 only (Makefile ARCH)
  static_assert((4 * kRsvMaxSlices + 2) * 4 + 32 <= 160 * 1024, "k_rsv_tiles: LDS beyond gfx950's 160 KB");
  __shared__ uint32_t s_row0[kRsvMaxSlices + 1];  // first count row per slice (capacity), [NS] = rows
  __shared__ uint32_t s_a0[kRsvMaxSlices + 1];    // first listed tile per slice, [NS] = tiles
  __shared__ uint32_t s_keys[kRsvMaxSlices];
  __shared__ uint32_t s_kb[kRsvMaxSlices];        // keys of the slices before
  __shared__ uint32_t s_wsum[2][4];
  const uint32_t tid = threadIdx.x, NS = nc * kRsvRanges, SPT = (NS + 255) / 256;
  const bool over = *flag != 0u;
  uint32_t keys[kMaxSpt], nl = 0, dk = 0;
#pragma unroll
  for (uint32_t q = 0; q < kMaxSpt; ++q) {
    const uint32_t e = tid * SPT + q;
    keys[q] = (q < SPT && e < NS && !over) ? rcur[rsv_cur_index(e, RADIX)] : 0u;
    nl += (keys[q] + TILE - 1) / TILE;
    dk += keys[q];
  }
  uint32_t listed, total_keys;
  uint32_t a0 = block_exclusive_scan<256>(nl, s_wsum[0], listed);
  uint32_t before = block_exclusive_scan<256>(dk, s_wsum[1], total_keys);
  for (uint32_t e = tid; e <= NS; e += 256) s_row0[e] = rslice[2 * NS + e];
#pragma unroll
  for (uint32_t q = 0; q < kMaxSpt; ++q) {
    const uint32_t e = tid * SPT + q;
    if (q < SPT && e < NS) {
      s_a0[e] = a0;
      s_keys[e] = keys[q];
      s_kb[e] = before;
      a0 += (keys[q] + TILE - 1) / TILE;
      before += keys[q];
    }
  }
  if (tid == 0) s_a0[NS] = listed;
  __syncthreads();
  if (blockIdx.x == 0) {
    for (uint32_t c = tid; c < nc; c += 256) {
      cstart[c] = s_kb[c * kRsvRanges];
      ctile0[c] = FUSED ? s_row0[c * kRsvRanges] : s_a0[c * kRsvRanges];
    }
    if (tid == 0) {
      ctile0[nc] = FUSED ? s_row0[NS] : listed;
      *ntiles = listed;
    }
  }
  const uint32_t t = blockIdx.x * 256 + tid;
  if (t >= bound) return;
  if (FUSED && over) {
#pragma unroll
    for (int q = 0; q < RADIX; q += 4)
      *reinterpret_cast<uint4*>(&Czero[(size_t)t * RADIX + q]) = make_uint4(0u, 0u, 0u, 0u);
  }
  if (t >= listed) return;
  uint32_t lo = 0, hi = NS;  // the slice e with a0[e] <= t < a0[e + 1]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (s_a0[mid] <= t) lo = mid; else hi = mid;
  }
  const uint32_t k = t - s_a0[lo];
  tiles[t] = make_uint4(rslice[lo] + k * TILE, min((uint32_t)TILE, s_keys[lo] - k * TILE), lo / kRsvRanges,
                        FUSED ? s_row0[lo] + k : t);
}

// bounds[g] = exclusive scan of window 0 (the whole group when width <= 8).
__global__ __launch_bounds__(256) void k_bounds_from_window(const uint32_t* __restrict__ whist,
                                                            uint32_t ngroups, uint32_t* __restrict__ bounds) {
  __shared__ uint32_t s_wsum[4];
  const uint32_t g = threadIdx.x;
  const uint32_t c = g < ngroups ? whist[g] : 0u;
  uint32_t total;
  const uint32_t ex = block_exclusive_scan<256>(c, s_wsum, total);
  if (g < ngroups) bounds[g] = ex;
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
// loop sort.cu:384-391, but writing the exclusive prefix for every empty
// group in parallel): bounds[] is first filled with the sentinel ~0u; each
// position where the group changes marks bounds[group] = i (k_bounds_mark);
// an empty group then takes the start of the next non-empty group, i.e. a
// suffix minimum over bounds (k_bounds_min_blocks -> k_bounds_min_top ->
// k_bounds_min_apply), and trailing empty groups become n.  Every thread
// does O(16) work whatever the width (up to 2^31 groups).
constexpr int kBmItems = 16, kBmBlock = 256, kBmTile = kBmItems * kBmBlock;
template <typename K>
__global__ void k_bounds_mark(const K* __restrict__ sorted, uint32_t n, uint32_t shift, uint32_t gmask,
                              uint32_t* __restrict__ bounds) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t cur = (uint32_t)(sorted[i] >> shift) & gmask;
    if (i == 0 || cur != ((uint32_t)(sorted[i - 1] >> shift) & gmask)) bounds[cur] = (uint32_t)i;
  }
}

// The same for uint32 keys, 16 consecutive keys per thread (four 16-byte
// loads when the array is 16-byte aligned) and the previous key once: the
// grid-stride form above ran the 2^28-key, width-16 gpuPartial's boundaries
// at ~550 us against ~200 us for one read of the keys.
constexpr int kBmkItems = 16;
__global__ __launch_bounds__(256) void k_bounds_mark_u32(const uint32_t* __restrict__ sorted, uint32_t n,
                                                         uint32_t shift, uint32_t gmask, uint32_t vec,
                                                         uint32_t* __restrict__ bounds) {
  const uint64_t i0 = ((uint64_t)blockIdx.x * 256 + threadIdx.x) * kBmkItems;
  if (i0 >= n) return;
  uint32_t k[kBmkItems];
  if (vec && i0 + kBmkItems <= n) {
    const uint4* p = reinterpret_cast<const uint4*>(sorted + i0);
#pragma unroll
    for (int q = 0; q < kBmkItems / 4; ++q) {
      const uint4 v = load_count_vec(&p[q]);
      k[4 * q] = v.x;
      k[4 * q + 1] = v.y;
      k[4 * q + 2] = v.z;
      k[4 * q + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < kBmkItems; ++j) k[j] = i0 + j < n ? sorted[i0 + j] : 0u;
  }
  // (the sentinel ~0u is no group: width <= 31)
  uint32_t prev = i0 ? (sorted[i0 - 1] >> shift) & gmask : ~0u;
#pragma unroll
  for (int j = 0; j < kBmkItems; ++j) {
    if (i0 + j >= n) break;
    const uint32_t g = (k[j] >> shift) & gmask;
    if (g != prev) bounds[g] = (uint32_t)(i0 + j);
    prev = g;
  }
}

// Boundaries of a two-pass LSD partial sort (tile path) without reading the
// sorted keys: pass 0 sorted by the low digit l (BITS bits), pass 1 by the
// high digit d (the remaining width - BITS bits) of its input `mid` (= pass
// 0's output, ordered by l).  The number of keys of group (d, l) or below in
// (d, l) order is D[d] + the keys of digit d in mid[0, pos_l), pos_l = the
// first position of mid whose low digit is >= l -- which is the run start of
// digit d in pos_l's tile (C + B + D of pass 1's column scan: the offset
// k_tile_pass gives that tile's run) plus the keys of digit d in the tile
// before pos_l.  Block l: pos_l by a 256-ary search over mid, the partial
// tile's digit counts in LDS, then bounds[(d << BITS) | l] for every d.
// ~4 KB x 2^BITS of reads instead of a pass over the keys (the 2^28-key,
// width-16 gpuPartial: ~200 us of k_bounds_mark_u32 otherwise).
template <int BITS, int TILE>
__global__ __launch_bounds__(256) void k_bounds_lsd2(const uint32_t* __restrict__ mid, uint32_t n, uint32_t lo,
                                                     uint32_t dmask, const uint32_t* __restrict__ C,
                                                     const uint32_t* __restrict__ B, const uint32_t* __restrict__ D,
                                                     uint32_t* __restrict__ bounds) {
  constexpr uint32_t RADIX = 1u << BITS;
  constexpr int CH = col_chunk_rows(RADIX);
  __shared__ uint32_t s_h[RADIX];
  __shared__ uint32_t s_first;
  __shared__ uint64_t s_lo, s_hi;
  const uint32_t l = blockIdx.x, tid = threadIdx.x;
  auto low = [&](uint64_t i) { return (mid[i] >> lo) & (RADIX - 1u); };
  for (uint32_t d = tid; d < RADIX; d += 256) s_h[d] = 0u;
  if (tid == 0) {
    s_lo = 0;
    s_hi = n;
  }
  __syncthreads();
  // pos_l = the first i in [0, n) with low(i) >= l (n when none): the answer
  // lies in [s_lo, s_hi]; 256 evenly spaced probes per round narrow it to
  // one step, then the last <= 256 candidates are checked one per thread
  for (;;) {
    const uint64_t a = s_lo, z = s_hi;
    __syncthreads();
    if (z - a <= 256) {
      if (tid == 0) s_first = (uint32_t)z;
      __syncthreads();
      if (a + tid < z && low(a + tid) >= l) atomicMin(&s_first, (uint32_t)(a + tid));
      __syncthreads();
      break;
    }
    const uint64_t step = (z - a + 255) / 256;
    const uint32_t nv = (uint32_t)((z - a + step - 1) / step);  // probes inside [a, z)
    if (tid == 0) s_first = nv;
    __syncthreads();
    if (tid < nv && low(a + (uint64_t)tid * step) >= l) atomicMin(&s_first, tid);
    __syncthreads();
    const uint32_t f = s_first;  // first probe at or past pos_l (nv: none)
    if (tid == 0) {
      if (f > 0) s_lo = a + (uint64_t)(f - 1) * step + 1;
      s_hi = f < nv ? a + (uint64_t)f * step : z;
    }
    __syncthreads();
  }
  const uint32_t pos = s_first;
  const uint32_t t = pos / TILE, t0 = t * TILE;
  for (uint32_t i = t0 + tid; i < pos; i += 256) atomicAdd(&s_h[(mid[i] >> (lo + BITS)) & dmask], 1u);
  __syncthreads();
  const uint32_t tiles = (n + TILE - 1) / TILE;
  for (uint32_t d = tid; d <= dmask; d += 256) {
    uint32_t base;
    if (t < tiles)
      base = C[(size_t)t * RADIX + d] + B[(size_t)(t / CH) * RADIX + d] + D[d];
    else  // pos == n at a tile edge: every key of digit d lies before
      base = d < dmask ? D[d + 1] : n;
    bounds[((size_t)d << BITS) | l] = base + s_h[d];
  }
}

// min over each kBmTile-entry block of bounds -> mins[block]
__global__ __launch_bounds__(kBmBlock) void k_bounds_min_blocks(const uint32_t* __restrict__ bounds, uint64_t ng,
                                                              uint32_t* __restrict__ mins) {
  __shared__ uint32_t s_m[kBmBlock / kWave];
  const uint64_t base = (uint64_t)blockIdx.x * kBmTile + (uint64_t)threadIdx.x * kBmItems;
  uint32_t m = ~0u;
#pragma unroll
  for (int j = 0; j < kBmItems; ++j)
    if (base + j < ng) m = min(m, bounds[base + j]);
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) m = min(m, (uint32_t)__shfl_xor(m, o, kWave));
  if ((threadIdx.x & (kWave - 1)) == 0) s_m[threadIdx.x / kWave] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t r = ~0u;
    for (int w = 0; w < kBmBlock / kWave; ++w) r = min(r, s_m[w]);
    mins[blockIdx.x] = r;
  }
}

// In-place exclusive suffix minimum of mins[0..nb) (one block): mins[b] =
// min over mins[b+1 ..].  Thread t owns a contiguous chunk.
__global__ __launch_bounds__(1024) void k_bounds_min_top(uint32_t* __restrict__ mins, uint32_t nb) {
  __shared__ uint32_t s_c[1024];
  const uint32_t t = threadIdx.x, per = (nb + 1023) / 1024;
  const uint32_t a = min(nb, t * per), z = min(nb, a + per);
  uint32_t m = ~0u;
  for (uint32_t i = a; i < z; ++i) m = min(m, mins[i]);
  s_c[t] = m;
  __syncthreads();
  // inclusive suffix min over the chunk minima (Hillis-Steele, 10 steps)
  for (uint32_t o = 1; o < 1024; o <<= 1) {
    const uint32_t v = t + o < 1024 ? s_c[t + o] : ~0u;
    __syncthreads();
    s_c[t] = min(s_c[t], v);
    __syncthreads();
  }
  uint32_t run = t + 1 < 1024 ? s_c[t + 1] : ~0u;  // suffix of the chunks after t
  for (uint32_t i = z; i > a; --i) {
    const uint32_t v = mins[i - 1];
    mins[i - 1] = run;
    run = min(run, v);
  }
}

// bounds[g] = min(bounds[g..]) with the sentinel mapped to n
__global__ __launch_bounds__(kBmBlock) void k_bounds_min_apply(uint32_t* __restrict__ bounds, uint64_t ng,
                                                             const uint32_t* __restrict__ carry, uint32_t n) {
  __shared__ uint32_t s_c[kBmBlock];
  const uint32_t t = threadIdx.x;
  const uint64_t base = (uint64_t)blockIdx.x * kBmTile + (uint64_t)t * kBmItems;
  uint32_t v[kBmItems], m = ~0u;
#pragma unroll
  for (int j = 0; j < kBmItems; ++j) {
    v[j] = base + j < ng ? bounds[base + j] : ~0u;
    m = min(m, v[j]);
  }
  s_c[t] = m;
  __syncthreads();
  for (uint32_t o = 1; o < kBmBlock; o <<= 1) {
    const uint32_t w = t + o < kBmBlock ? s_c[t + o] : ~0u;
    __syncthreads();
    s_c[t] = min(s_c[t], w);
    __syncthreads();
  }
  uint32_t run = min(carry[blockIdx.x], t + 1 < kBmBlock ? s_c[t + 1] : ~0u);
#pragma unroll
  for (int j = kBmItems - 1; j >= 0; --j) {
    run = min(run, v[j]);
    if (base + j < ng) bounds[base + j] = run == ~0u ? n : run;
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

// Few large segments: block (x, y) copies elements [x*4096, (x+1)*4096) of
// segment y (blocks past the segment's end exit).
constexpr int kSegPiece = 4096;
__global__ __launch_bounds__(256) void k_segment_copy2d(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst,
                                                        const uint64_t* __restrict__ tab, uint32_t nseg) {
  const uint32_t s = blockIdx.y;
  const uint64_t len = tab[2 * nseg + s];
  const uint64_t a = (uint64_t)blockIdx.x * kSegPiece;
  if (a >= len) return;
  const uint32_t* sp = src + tab[s] + a;
  uint32_t* dp = dst + tab[nseg + s] + a;
  // (written as a branch on the remainder: a umin64 here compiled to an
  // s_cselect on a stale SCC, i.e. m = 4096 in the partial branch)
  const uint64_t rem = len - a;
  if (rem >= (uint64_t)kSegPiece) {
    uint32_t v[kSegPiece / 256];
#pragma unroll
    for (int j = 0; j < kSegPiece / 256; ++j) v[j] = sp[threadIdx.x + j * 256];
#pragma unroll
    for (int j = 0; j < kSegPiece / 256; ++j) dp[threadIdx.x + j * 256] = v[j];
  } else {
    const uint32_t m = (uint32_t)rem;
    for (uint32_t j = threadIdx.x; j < m; j += 256) dp[j] = sp[j];
  }
}

// The same gather from 24-bit pieces (distrib.cpp "wire24"): key = hi |
// lo8 << 16 | lo16; table src_off | dst_off | len | hi (top byte << 24) per
// segment (the piece sort's fallback, and every round sort the reserved depth
// 0 cannot take).
__global__ __launch_bounds__(256) void k_segment_copy2d_planar(const uint16_t* __restrict__ s16,
                                                               const uint8_t* __restrict__ s8,
                                                               uint32_t* __restrict__ dst,
                                                               const uint64_t* __restrict__ tab, uint32_t nseg) {
  const uint32_t s = blockIdx.y;
  const uint64_t len = tab[2 * nseg + s];
  const uint64_t a = (uint64_t)blockIdx.x * kSegPiece;
  if (a >= len) return;
  const uint64_t so = tab[s] + a;
  const uint32_t hi = (uint32_t)tab[3 * nseg + s];
  uint32_t* dp = dst + tab[nseg + s] + a;
  const uint64_t rem = len - a;
  if (rem >= (uint64_t)kSegPiece) {
    uint32_t v[kSegPiece / 256];
#pragma unroll
    for (int j = 0; j < kSegPiece / 256; ++j) {
      const uint64_t i = so + threadIdx.x + j * 256;
      v[j] = hi | ((uint32_t)s8[i] << 16) | (uint32_t)s16[i];
    }
#pragma unroll
    for (int j = 0; j < kSegPiece / 256; ++j) dp[threadIdx.x + j * 256] = v[j];
  } else {
    const uint32_t m = (uint32_t)rem;
    for (uint32_t j = threadIdx.x; j < m; j += 256) dp[j] = hi | ((uint32_t)s8[so + j] << 16) | (uint32_t)s16[so + j];
  }
}

// ----------------------------------------------------------------------------
// delta-coded exchange of sorted runs (pylibsort.distrib "msdz" schedule for
// link-bound world sizes): groups of 64 consecutive keys of a sorted run keep
// their first key as a 32-bit base and the 63 gaps to the previous key in w
// bits, w = bits of the largest in-group gap of the whole run.  Layout:
// bases[ng] then ng groups of 2w dwords (64 gaps x w bits; lane 0's gap is 0).
// ----------------------------------------------------------------------------
constexpr int kDeltaGroup = 64;

__device__ __forceinline__ uint32_t delta_bits(uint32_t maxgap) { return maxgap ? 32u - __clz(maxgap) : 0u; }

// The kernels below step over chunks of kDeltaChunk groups (4096 keys) per
// 256-thread block: wave v of the block takes the chunk's groups v, v + 4,
// ... (16 groups, one coalesced load each, all issued before any use); the
// pack assembles the chunk's payload in LDS and writes it (and the bases)
// with block-wide coalesced stores, the unpack stages it the same way.  (The
// per-wave form before, 4 groups per wave and 2w-dword stores per group:
// 116 / 96 us per 2^26-key piece, 2.5 / 3.0 TB/s; profiles/r06d.)
constexpr int kDeltaChunk = 64;
constexpr int kDeltaWaveGroups = kDeltaChunk / 4;

// Largest in-group gap of the sorted run keys[0..n) -> atomicMax into *maxgap
// (zeroed by the caller).
__global__ __launch_bounds__(256) void k_delta_maxgap(const uint32_t* __restrict__ keys, uint64_t n,
                                                      uint32_t* __restrict__ maxgap) {
  constexpr int U = kDeltaWaveGroups;
  const uint32_t lane = threadIdx.x & (kWave - 1);
  const uint64_t ng = (n + kDeltaGroup - 1) / kDeltaGroup;
  const uint64_t wpb = blockDim.x / kWave;
  uint32_t m = 0;
  for (uint64_t g0 = ((uint64_t)blockIdx.x * wpb + threadIdx.x / kWave) * U; g0 < ng;
       g0 += (uint64_t)gridDim.x * wpb * U) {
    uint32_t k[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = (g0 + u) * kDeltaGroup + lane;
      k[u] = i < n ? keys[i] : 0u;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t prev = __shfl_up(k[u], 1, kWave);
      const uint64_t i = (g0 + u) * kDeltaGroup + lane;
      if (lane > 0 && i < n) m = max(m, k[u] - prev);
    }
  }
  // one atomic per block: same-address atomics from every wave serialise
  // (16K of them took ~0.8 ms at 2^27 keys)
  __shared__ uint32_t s_m[256 / kWave];
  for (int o = kWave / 2; o > 0; o >>= 1) m = max(m, (uint32_t)__shfl_xor(m, o, kWave));
  if (lane == 0) s_m[threadIdx.x / kWave] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (uint32_t i = 1; i < blockDim.x / kWave; ++i) m = max(m, s_m[i]);
    // (only a block above the word's current value adds its atomic: the
    // word only grows, and most blocks' maxima are below it by then)
    if (m && m > __hip_atomic_load(maxgap, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(maxgap, m);
  }
}

// Pack: w read from *maxgap on the device (so the pack can be queued before
// the host knows it).  Gap j of a group goes to bits [j w, j w + w) of its 2w
// dwords (LDS atomicOr; zero gaps skip it).
__global__ __launch_bounds__(256) void k_delta_pack(const uint32_t* __restrict__ keys, uint64_t n,
                                                    const uint32_t* __restrict__ maxgap, uint32_t* __restrict__ out) {
  constexpr int U = kDeltaWaveGroups;
  __shared__ uint32_t s_p[kDeltaChunk * 2 * 32];  // 2w <= 64 dwords per group
  __shared__ uint32_t s_b[kDeltaChunk];
  const uint32_t lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
  const uint32_t w = delta_bits(*maxgap);
  const uint64_t ng = (n + kDeltaGroup - 1) / kDeltaGroup;
  const uint64_t nch = (ng + kDeltaChunk - 1) / kDeltaChunk;
  uint32_t* const payload = out + ng;
  for (uint64_t c = blockIdx.x; c < nch; c += gridDim.x) {
    const uint64_t gb = c * kDeltaChunk;
    const uint32_t gn = (uint32_t)min((uint64_t)kDeltaChunk, ng - gb);
    const uint32_t pw = gn * 2u * w;
    uint32_t k[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = (gb + (uint64_t)u * 4 + wv) * kDeltaGroup + lane;
      k[u] = i < n ? keys[i] : 0u;
    }
    for (uint32_t i = threadIdx.x; i < pw; i += 256) s_p[i] = 0u;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t gl = (uint32_t)u * 4u + wv;  // (wave-uniform)
      if (gl < gn) {
        const uint64_t i = (gb + gl) * kDeltaGroup + lane;
        const uint32_t prev = __shfl_up(k[u], 1, kWave);
        if (lane == 0) s_b[gl] = k[u];
        const uint32_t gap = (lane > 0 && i < n) ? k[u] - prev : 0u;
        if (gap) {
          const uint32_t bit = lane * w, q = gl * 2u * w + (bit >> 5), r = bit & 31u;
          atomicOr(&s_p[q], gap << r);
          if (r + w > 32u) atomicOr(&s_p[q + 1], gap >> (32u - r));
        }
      }
    }
    __syncthreads();
    if (threadIdx.x < gn) out[gb + threadIdx.x] = s_b[threadIdx.x];
    uint32_t* const dst = payload + gb * 2u * w;
    for (uint32_t i = threadIdx.x; i < pw; i += 256) dst[i] = s_p[i];
    __syncthreads();  // (the next chunk zeroes s_p)
  }
}

// Unpack: the chunk's bases and payload staged in LDS (coalesced loads); a
// group's 64 keys are taken by 16 lanes x 4 consecutive keys (a wave: 4
// groups per step), each lane's 4 gaps summed in registers and the lanes'
// sums scanned over 16 lanes (a third of the per-key VALU work of a 64-lane
// scan per group); the keys go out through LDS in 64-key coalesced stores.
__global__ __launch_bounds__(256) void k_delta_unpack(const uint32_t* __restrict__ in, uint64_t n, uint32_t w,
                                                      uint32_t* __restrict__ keys) {
  __shared__ uint32_t s_p[kDeltaChunk * 2 * 32];
  __shared__ uint32_t s_b[kDeltaChunk];
  const uint32_t lane = threadIdx.x & (kWave - 1), wv = threadIdx.x / kWave;
  const uint32_t sub = lane >> 4, l16 = lane & 15u, j0 = l16 * 4u;
  const uint64_t ng = (n + kDeltaGroup - 1) / kDeltaGroup;
  const uint64_t nch = (ng + kDeltaChunk - 1) / kDeltaChunk;
  const uint32_t* const payload = in + ng;
  const uint32_t mask = w >= 32u ? 0xffffffffu : ((1u << w) - 1u);
  for (uint64_t c = blockIdx.x; c < nch; c += gridDim.x) {
    const uint64_t gb = c * kDeltaChunk;
    const uint32_t gn = (uint32_t)min((uint64_t)kDeltaChunk, ng - gb);
    const uint32_t pw = gn * 2u * w;
    const uint32_t* const src = payload + gb * 2u * w;
    for (uint32_t i = threadIdx.x; i < pw; i += 256) s_p[i] = src[i];
    if (threadIdx.x < gn) s_b[threadIdx.x] = in[gb + threadIdx.x];
    __syncthreads();
    constexpr int ST = kDeltaWaveGroups / 4;
    uint32_t v[ST][4];
#pragma unroll
    for (int st = 0; st < ST; ++st) {
      const uint32_t gl = wv * kDeltaWaveGroups + (uint32_t)st * 4u + sub;
      const bool live = gl < gn;
      uint32_t x[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        uint32_t gap = 0u;
        if (w && live) {
          const uint32_t* const g = s_p + gl * 2u * w;
          const uint32_t bit = (j0 + (uint32_t)e) * w, q = bit >> 5, r = bit & 31u;
          const uint32_t lo = g[q], hi = r + w > 32u ? g[q + 1] : 0u;
          gap = (uint32_t)((((uint64_t)hi << 32) | lo) >> r) & mask;
        }
        x[e] = e ? x[e - 1] + gap : gap;
      }
      uint32_t t = x[3];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        const uint32_t y = __shfl_up(t, o, 16);
        if ((int)l16 >= o) t += y;
      }
      const uint32_t base = (live ? s_b[gl] : 0u) + (t - x[3]);
#pragma unroll
      for (int e = 0; e < 4; ++e) v[st][e] = base + x[e];
    }
    // the chunk's keys through LDS (over the payload words, read by now), so
    // every store instruction writes 64 consecutive keys whatever the
    // destination's alignment (the rounds decode at arbitrary key offsets)
    __syncthreads();
#pragma unroll
    for (int st = 0; st < ST; ++st) {
      const uint32_t gl = wv * kDeltaWaveGroups + (uint32_t)st * 4u + sub;
      *reinterpret_cast<uint4*>(&s_p[gl * kDeltaGroup + j0]) = make_uint4(v[st][0], v[st][1], v[st][2], v[st][3]);
    }
    __syncthreads();
    const uint64_t k0 = gb * kDeltaGroup;
    const uint32_t nk = (uint32_t)min((uint64_t)kDeltaChunk * kDeltaGroup, n - k0);
    for (uint32_t i = threadIdx.x; i < nk; i += 256) keys[k0 + i] = s_p[i];
    __syncthreads();  // (the next chunk restages s_p)
  }
}

// Merge of two sorted runs (merge path).  Block b writes outputs
// [b*T, (b+1)*T): both split points by binary search on the diagonals, the
// two input ranges staged in LDS, then each thread merges ITEMS outputs from
// its own diagonal.  Ties take a first (keys only: order among equal keys is
// invisible).
// The split of diagonal d: the first i in [lo, hi) with a[i] > b[d - 1 - i]
// (f(i) = a[i] - b[d - 1 - i] is non-decreasing; hi when there is none).  The
// probes alternate a secant step on f between the bracket's known values and
// a bisection: exact for any input (only the bracket decides), ~8 dependent
// probes instead of ~27 for the uniform runs of the coded rounds (each probe
// is a global load pair; the split kernel is one such chain long).
__device__ __forceinline__ uint64_t merge_path_split(const uint32_t* a, uint64_t na, const uint32_t* b, uint64_t nb,
                                                     uint64_t d) {
  uint64_t lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
  // f at the bracket's outer neighbours, when probed (fl <= 0 at lo - 1, fr > 0 at hi)
  double fl = 0.0, fr = 0.0;
  bool have_l = false, have_r = false;
  for (int step = 0; lo < hi; ++step) {
    uint64_t mid = (lo + hi) >> 1;
    if ((step & 1) == 0 && have_l && have_r && hi - lo > 8) {
      // secant between (lo - 1, fl) and (hi, fr) for the zero of f
      const double x = (double)(lo - 1) + (0.0 - fl) * (double)(hi - lo + 1) / (fr - fl);
      const double xc = x < (double)lo ? (double)lo : x > (double)(hi - 1) ? (double)(hi - 1) : x;
      mid = (uint64_t)xc;
    }
    const double f = (double)a[mid] - (double)b[d - mid - 1];
    if (f <= 0.0) {
      lo = mid + 1;
      fl = f;
      have_l = true;
    } else {
      hi = mid;
      fr = f;
      have_r = true;
    }
  }
  return lo;
}

// Split points of every merge tile: splits[t] = elements of a among the
// first t * tile outputs (t = 0..tiles), one thread each.
__global__ __launch_bounds__(256) void k_merge_splits(const uint32_t* __restrict__ a, uint64_t na,
                                                      const uint32_t* __restrict__ b, uint64_t nb, uint32_t tile,
                                                      uint64_t tiles, uint64_t* __restrict__ splits) {
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (t > tiles) return;
  const uint64_t d = t * tile < na + nb ? t * tile : na + nb;
  splits[t] = merge_path_split(a, na, b, nb, d);
}

__global__ __launch_bounds__(256) void k_merge_u32(const uint32_t* __restrict__ a, uint64_t na,
                                                   const uint32_t* __restrict__ b, uint64_t nb,
                                                   const uint64_t* __restrict__ splits, uint32_t* __restrict__ out) {
  constexpr int T = 256, ITEMS = 8, TILE = T * ITEMS;
  __shared__ uint32_t s[TILE];
  const uint64_t total = na + nb;
  const uint64_t d0 = (uint64_t)blockIdx.x * TILE;
  const uint64_t d1 = d0 + TILE < total ? d0 + TILE : total;
  const uint64_t a0 = splits[blockIdx.x], a1 = splits[blockIdx.x + 1];
  const uint32_t la = (uint32_t)(a1 - a0), lb = (uint32_t)((d1 - d0) - la);
  const uint64_t b0 = d0 - a0;
  for (uint32_t i = threadIdx.x; i < la + lb; i += T) s[i] = i < la ? a[a0 + i] : b[b0 + (i - la)];
  __syncthreads();
  const uint32_t* sa = s;
  const uint32_t* sb = s + la;
  const uint32_t len = la + lb;
  const uint32_t dd = threadIdx.x * ITEMS;
  uint32_t v[ITEMS];
  uint32_t m = 0;
  if (dd < len) {
    uint32_t lo = dd > lb ? dd - lb : 0u, hi = dd < la ? dd : la;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      if (sa[mid] <= sb[dd - mid - 1]) lo = mid + 1;
      else hi = mid;
    }
    uint32_t ia = lo, ib = dd - lo;
    m = min((uint32_t)ITEMS, len - dd);
#pragma unroll
    for (uint32_t j = 0; j < (uint32_t)ITEMS; ++j) {
      if (j < m) {
        const bool take_a = ib >= lb || (ia < la && sa[ia] <= sb[ib]);
        v[j] = take_a ? sa[ia++] : sb[ib++];
      }
    }
  }
  // through LDS again, so the global stores are lane-contiguous
  __syncthreads();
#pragma unroll
  for (uint32_t j = 0; j < (uint32_t)ITEMS; ++j)
    if (j < m) s[dd + j] = v[j];
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < len; i += T) out[d0 + i] = s[i];
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

hipError_t Workspace::ensure_pipeline(size_t bytes) {
  if (!copy_stream) LS_TRY(hipStreamCreateWithFlags(&copy_stream, hipStreamNonBlocking));
  for (auto& e : pipe_evt)
    if (!e) LS_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  if (!plan_dev) LS_TRY(hipMalloc(&plan_dev, kPlanWords * sizeof(uint32_t)));
  if (!plan_host) LS_TRY(hipHostMalloc(&plan_host, kPlanWords * sizeof(uint32_t), hipHostMallocDefault));
  if (bytes <= pbuf_cap) return hipSuccess;
  if (pbuf) { (void)hipFree(pbuf); pbuf = nullptr; }
  pbuf_cap = 0;
  LS_TRY(hipMalloc(&pbuf, bytes));
  pbuf_cap = bytes;
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

hipError_t Workspace::ensure_tiles(size_t count_words, size_t chunk_words) {
  part_pending.valid = false;  // every tile-path user starts here: a pending partition scatter is void
  if (count_words > tc_cap) {
    for (auto& p : tc) {
      if (p) { (void)hipFree(p); p = nullptr; }
    }
    tc_cap = 0;
    LS_TRY(hipMalloc(&tc[0], count_words * sizeof(uint32_t)));
    LS_TRY(hipMalloc(&tc[1], count_words * sizeof(uint32_t)));
    tc_cap = count_words;
  }
  if (chunk_words > tb_cap) {
    if (tb) { (void)hipFree(tb); tb = nullptr; }
    tb_cap = 0;
    LS_TRY(hipMalloc(&tb, chunk_words * sizeof(uint32_t)));
    tb_cap = chunk_words;
  }
  if (!tticket) {
    LS_TRY(hipMalloc(&tticket, 64 * sizeof(uint32_t)));
    LS_TRY(hipMemset(tticket, 0, 64 * sizeof(uint32_t)));  // last-arriver tickets start (and end) at zero
    LS_TRY(hipDeviceSynchronize());  // once: the sort streams are non-blocking w.r.t. the null stream
  }
  return hipSuccess;
}

hipError_t Workspace::ensure_hybrid(size_t words) {
  if (!hyb_evt) LS_TRY(hipEventCreateWithFlags(&hyb_evt, hipEventDisableTiming));
  if (!hyb_host) {
    LS_TRY(hipHostMalloc(&hyb_host, 512 * sizeof(uint32_t), hipHostMallocDefault));
    std::memset(hyb_host, 0, 512 * sizeof(uint32_t));  // (the sequence word starts below every sort's)
  }
  if (words <= hyb_cap) return hipSuccess;
  if (hyb) { (void)hipFree(hyb); hyb = nullptr; }
  hyb_cap = 0;
  LS_TRY(hipMalloc(&hyb, words * sizeof(uint32_t)));
  hyb_cap = words;
  return hipSuccess;
}

hipError_t Workspace::ensure_rsv(size_t words) {
  if (words <= rsv_cap) return hipSuccess;
  if (rsv) { (void)hipFree(rsv); rsv = nullptr; }
  rsv_cap = 0;
  LS_TRY(hipMalloc(&rsv, words * sizeof(uint32_t)));
  rsv_cap = words;
  return hipSuccess;
}

hipError_t Workspace::ensure_dstream(size_t bytes) {
  bytes = (bytes + 64) & ~(size_t)15;  // the count kernel reads whole 16-byte words
  if (bytes <= dstream_cap) return hipSuccess;
  if (dstream) { (void)hipFree(dstream); dstream = nullptr; }
  dstream_cap = 0;
  LS_TRY(hipMalloc(&dstream, bytes));
  dstream_cap = bytes;
  return hipSuccess;
}

hipError_t Workspace::ensure_onesweep(size_t status_words) {
  if (!os_small) {
    LS_TRY(hipMalloc(&os_small, kOsSmallWords * sizeof(uint32_t)));
    LS_TRY(hipMemset(os_small, 0, kOsSmallWords * sizeof(uint32_t)));
  }
  if (status_words <= os_status_cap) return hipSuccess;
  for (auto& p : os_status) {
    if (p) { (void)hipFree(p); p = nullptr; }
  }
  os_status_cap = 0;
  LS_TRY(hipMalloc(&os_status[0], status_words * sizeof(uint32_t)));
  LS_TRY(hipMalloc(&os_status[1], status_words * sizeof(uint32_t)));
  LS_TRY(hipMemset(os_status[1], 0, status_words * sizeof(uint32_t)));
  os_status_cap = status_words;
  return hipSuccess;
}

void Workspace::release() {
  int prev = -1;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(device);
  if (stream) (void)hipStreamSynchronize(stream);
  for (auto p : {(void*)counts, (void*)scan_l1, (void*)scan_l2, hbuf[0], hbuf[1], (void*)dbounds,
                 (void*)seg_dev, (void*)hist_tmp, (void*)os_status[0], (void*)os_status[1],
                 (void*)os_small})
    if (p) (void)hipFree(p);
  os_status[0] = os_status[1] = os_small = nullptr;
  for (auto p : {(void*)tc[0], (void*)tc[1], (void*)tb, (void*)tticket})
    if (p) (void)hipFree(p);
  tc[0] = tc[1] = tb = tticket = nullptr;
  tc_cap = tb_cap = 0;
  if (hyb) (void)hipFree(hyb);
  if (dstream) (void)hipFree(dstream);
  dstream = nullptr;
  if (rsv) (void)hipFree(rsv);
  rsv = nullptr;
  rsv_cap = 0;
  dstream_cap = 0;
  if (hyb_host) (void)hipHostFree(hyb_host);
  hyb = hyb_host = nullptr;
  hyb_cap = 0;
  os_status_cap = 0;
  if (seg_host) (void)hipHostFree(seg_host);
  if (copy_stream) (void)hipStreamSynchronize(copy_stream);
  if (pbuf) (void)hipFree(pbuf);
  if (plan_dev) (void)hipFree(plan_dev);
  if (plan_host) (void)hipHostFree(plan_host);
  pbuf = nullptr;
  plan_dev = plan_host = nullptr;
  pbuf_cap = 0;
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
  RadixDigit op{shift, (1u << nbits) - 1u};  // nbits <= 8
  if (bits == 8) return run_pass<8>(ws, kin, kout, vin, vout, n, op, st);
  if (bits == 4) return run_pass<4>(ws, kin, kout, vin, vout, n, op, st);
  return hipErrorInvalidValue;
}

// Which pass algorithm a sort with `bits`-bit digits over n keys runs.
int choose_algorithm(size_t n, int bits) {
  const int a = get_algorithm();
  if (a == 2) return 2;
  if (a == 1 && n < (1ull << 30)) return 1;  // onesweep status words carry 30-bit counts
  // auto / tiles (and onesweep beyond its range): the tile-offset path, whose
  // 32-bit offsets cover every n < 2^32.  Measured on MI355X at 2^28 keys:
  // 4-bit digits 3.81 ms (fused counts, 432 us/pass) vs onesweep 5.41 ms;
  // 8-bit digits 2.94 ms (count 234 + scan 33 + pass 464 us) vs onesweep 3.60 ms.
  (void)bits;
  return 3;
}

// Tile-offset path geometry.  4-bit digits: 256-thread tiles of 4096 keys and
// the next pass's counts fused into the pass kernel.  8-bit digits: 512-thread
// tiles of 8192 keys (longer digit runs, fewer count rows) and a separate
// per-tile count kernel per pass.
// Pairs with 64-bit keys at 8-bit digits: 16 pairs per thread, their values
// staged through the key buffer after the keys are written (k_tile_pass
// STAGE_V).  A compute-free skeleton of the pair scatter (tools/run_probe,
// 2^28 pairs) runs 1219 us with 16-pair runs and 1096 us with 32-pair runs.
// (u64, u32) pairs: 1024-thread tiles of 16384 pairs (64-pair runs; LDS 137
// KB, one block per CU): the pass is its two run-scatter store phases
// (tools/pairpass_lab ablations), and longer runs cost less: 1406 vs 1505 us
// per 2^28-pair pass in the lab, profiles/r05o_pairpass_t16k.txt.
// LIBSORT_TP8_PAIR_BLOCK=512 keeps the 8192-pair tiles, LIBSORT_TP8_PAIR_ITEMS=8
// halves either.
#ifndef LIBSORT_TP8_PAIR_ITEMS
#define LIBSORT_TP8_PAIR_ITEMS 16
#endif
template <typename K, typename V = NoValue>
constexpr int tp_items(int bits) {
  return sizeof(K) != 8 ? 16 : (bits == 8 && !std::is_same<V, NoValue>::value) ? LIBSORT_TP8_PAIR_ITEMS : 8;
}
#ifndef LIBSORT_TP8_BLOCK
#define LIBSORT_TP8_BLOCK 512  // threads of an 8-bit tile (16 keys each)
#endif
#ifndef LIBSORT_TP8_BLOCK64
#define LIBSORT_TP8_BLOCK64 512  // threads of an 8-bit tile of 64-bit keys (8 keys each)
#endif
#ifndef LIBSORT_TP4_BLOCK
#define LIBSORT_TP4_BLOCK 256  // threads of a 4-bit tile (A/B knob)
#endif
#ifndef LIBSORT_TP8_PAIR_BLOCK
#define LIBSORT_TP8_PAIR_BLOCK 1024  // threads of an 8-bit tile of (u64, u32) pairs
#endif
template <typename K, typename V = NoValue>
constexpr int tp_block(int bits) {
  return bits == 4 ? LIBSORT_TP4_BLOCK
         : sizeof(K) == 8 ? ((bits == 8 && std::is_same<V, uint32_t>::value) ? LIBSORT_TP8_PAIR_BLOCK
                                                                             : LIBSORT_TP8_BLOCK64)
                          : LIBSORT_TP8_BLOCK;
}
// The MSD hybrid's depths >= 1 of (u64, u32) pairs keep 512-thread tiles of
// 8192 pairs: their tiles come from a table, and the table load that gives
// a tile its first key precedes every key load, a latency that one block per
// CU cannot hide (the 16384-pair pass there: 1440 -> 1530 us; at depth 0 and
// in the LSD passes, which compute their tiles, 1622 -> 1530 us with the
// digit stream).
template <typename K, typename V = NoValue>
constexpr int tp_block_tab(int bits) {
  return (bits == 8 && sizeof(K) == 8 && std::is_same<V, uint32_t>::value) ? LIBSORT_TP8_BLOCK64
                                                                           : tp_block<K, V>(bits);
}
template <typename K, typename V = NoValue>
uint32_t tp_tiles(size_t n, int bits) {
  const uint64_t t = (uint64_t)tp_block<K, V>(bits) * tp_items<K, V>(bits);
  return (uint32_t)((n + t - 1) / t);
}
// The LSD passes' tiles (sort_impl's tile path: gpuPartial, range and
// fallback sorts): 8-bit u32 keys may take their own block size
// (LIBSORT_TP8_LSD_BLOCK, an A/B build knob: 1024 = 16384-key tiles, 64-key
// runs) without changing the MSD hybrid's tiles.
#ifndef LIBSORT_TP8_LSD_BLOCK
#define LIBSORT_TP8_LSD_BLOCK 512
#endif
template <typename K, typename V = NoValue>
constexpr int tp_block_lsd(int bits) {
  return (bits == 8 && sizeof(K) == 4 && std::is_same<V, NoValue>::value) ? LIBSORT_TP8_LSD_BLOCK
                                                                         : tp_block<K, V>(bits);
}
template <typename K, typename V = NoValue>
uint32_t tp_tiles_lsd(size_t n, int bits) {
  const uint64_t t = (uint64_t)tp_block_lsd<K, V>(bits) * tp_items<K, V>(bits);
  return (uint32_t)((n + t - 1) / t);
}
inline uint32_t tp_chunks(uint32_t tiles, int bits) {
  const uint32_t ch = (uint32_t)col_chunk_rows(1 << bits);
  return (tiles + ch - 1) / ch;
}

template <int BITS, typename K, typename Op = RadixDigit, typename V = NoValue, int B = tp_block<K, V>(BITS)>
hipError_t tiles_counts(Workspace& ws, const K* in, size_t n, Op op, uint32_t tiles, uint32_t* C,
                        uint32_t* zero, uint32_t zero_words, hipStream_t st) {
  // the same tiles as the pass kernel (B threads of tp_items keys), a
  // different block shape: 4-bit u32 tiles are counted by 512 threads x 8
  // keys (179 -> 170 us at 2^28 keys, interleaved A/B; the pass itself is
  // faster as 256 x 16)
  constexpr int CB = (BITS == 4 && sizeof(K) == 4) ? 512 : B;
  constexpr int CI = B * tp_items<K, V>(BITS) / CB;
  static_assert(CB * CI == B * tp_items<K, V>(BITS), "count tiles = pass tiles");
  ScopedTimer tm("tilecounts", st, n);
  hipLaunchKernelGGL((k_tile_counts<BITS, CB, CI, K, Op>), dim3(tiles), dim3(CB), 0, st, in, (uint32_t)n, op, C, zero,
                     zero_words, nullptr, nullptr);
  return hipGetLastError();
}

// Digit starts of the last column scan (the tile path's bucket boundaries).
inline uint32_t* tiles_digit_starts(Workspace& ws, uint32_t tiles, int bits) {
  return ws.tb + (size_t)tp_chunks(tiles, bits) * (1u << bits);
}

template <int BITS>
hipError_t tiles_colscan(Workspace& ws, uint32_t* C, uint32_t tiles, hipStream_t st) {
  constexpr int RADIX = 1 << BITS;
  const uint32_t chunks = tp_chunks(tiles, BITS);
  uint32_t* D = tiles_digit_starts(ws, tiles, BITS);
  ScopedTimer tm("colscan", st, tiles);
  if constexpr (RADIX <= 32) {
    hipLaunchKernelGGL(k_colscan_small<RADIX>, dim3(chunks), dim3(256), 0, st, C, tiles, ws.tb, chunks, D, ws.tticket);
  } else {
    hipLaunchKernelGGL(k_colscan_l1<RADIX>, dim3(chunks), dim3(256), 0, st, C, tiles, ws.tb);
    LS_TRY(hipGetLastError());
    hipLaunchKernelGGL(k_colscan_wide<RADIX>, dim3(RADIX), dim3(256), 0, st, ws.tb, chunks, D, ws.tticket);
  }
  return hipGetLastError();
}

// 8-bit passes over 64-bit keys hand the next pass its digits as a byte
// stream (k_tile_pass geo.dout -> k_tile_counts_u8): the next count reads 1 B
// per key instead of 8 (c5: 5.21 -> 5.02 ms).  Not for 32-bit keys: the byte
// stores beside 4-byte keys made the u32 pass 1716 -> 2557 us at 2^30 (c3
// 10.03 -> 12.29 ms).  LIBSORT_DSTREAM=0 turns it off (A/B).
// Reserved depth 0 (k_rsv_sample + k_tile_pass GEO & 4): the default for
// keys-only 32-bit hybrid sorts; LIBSORT_HYB_RESERVE=0 keeps the count pass,
// =nomem acts as if the slices could not be allocated (the same count pass),
// =short halves every sampled capacity (tests: the overflow fallback).  Read
// per call (the tests switch it in process).
inline int rsv_mode() {
  const char* s = getenv("LIBSORT_HYB_RESERVE");
  if (!s) return 1;
  return s[0] == '0' ? 0 : s[0] == 's' ? 2 : s[0] == 'n' ? 3 : 1;
}

// The 2-bit counting cells for 256-thread bucket blocks (kCnt2F);
// LIBSORT_BUCKET2=0 keeps the 3-bit cells (A/B).
inline bool bucket2_on() {
  static const bool on = [] {
    const char* s = getenv("LIBSORT_BUCKET2");
    return !(s && s[0] == '0');
  }();
  return on;
}

// kCnt2F's lightly overflowed buckets retried inline with 3-bit half cells
// (retry3_halves) instead of by a LIST launch: an A/B build only
// (-DLIBSORT_BUCKET2_INLINE_AB=1, then LIBSORT_BUCKET2_INLINE=1): measured
// 449 -> 956 us for the bucket phase of a 2^28 sort, 3 interleaved runs each,
// profiles/r05d_bucket2_inline_ab.txt -- the rarely taken branch costs every
// block its registers and occupancy.  The product build does not instantiate it.
#ifndef LIBSORT_BUCKET2_INLINE_AB
#define LIBSORT_BUCKET2_INLINE_AB 0
#endif
inline bool bucket2_inline_on() {
  static const bool on = [] {
    const char* s = getenv("LIBSORT_BUCKET2_INLINE");
    return LIBSORT_BUCKET2_INLINE_AB && s && s[0] == '1';
  }();
  return on;
}

// Threads of the 3-bit retry blocks over the 2-bit kernel's overflowed
// buckets (a persistent LIST launch).  512 (half the keys per thread, twice
// the threads per CU at the same register budget): headline bucket phase
// 440-445 -> 434-437 us, 3 interleaved runs each (profiles/r05y_*).
#ifndef LIBSORT_RETRY_BLOCK
#define LIBSORT_RETRY_BLOCK 512
#endif
constexpr int kRetryBlock = LIBSORT_RETRY_BLOCK;

// (u64 key, u32 payload) buckets by the counting placement (k_bucket_pairs);
// LIBSORT_PAIR_COUNT=0 keeps the LSD steps + fix-up (A/B).
inline bool pair_count_on() {
  static const bool on = [] {
    const char* s = getenv("LIBSORT_PAIR_COUNT");
    return !(s && s[0] == '0');
  }();
  return on;
}

inline bool dstream_on() {
  static const bool on = [] {
    const char* s = getenv("LIBSORT_DSTREAM");
    return !(s && s[0] == '0');
  }();
  return on;
}

// The same digit stream for the 32-bit keys-only hybrid at 8-bit digits
// (configs[2]): the reserved depth 0 writes each key's next digit at its
// slice position, and depth 1 counts those bytes instead of re-reading the
// keys (804 us per 2^30-key sort).  LIBSORT_DSTREAM_U32=1: A/B only (VERDICT
// r05 item 4b; round 3 measured the byte stores costing the pass more than
// the count saves).
inline bool dstream_u32_on() {
  static const bool on = [] {
    const char* s = getenv("LIBSORT_DSTREAM_U32");
    return s && s[0] == '1';
  }();
  return on;
}

// Sort prologue of the tile path: buffers, and (4-bit) the pass-0 counts.
template <typename K, typename V, typename Op = RadixDigit>
hipError_t tiles_prologue(Workspace& ws, const K* in, size_t n, int lo, int hi, int bits, hipStream_t st,
                          uint32_t bias = 0) {
  const uint32_t tiles = tp_tiles_lsd<K, V>(n, bits);
  const uint32_t radix = 1u << bits;
  LS_TRY(ws.ensure_tiles((size_t)tiles * radix, ((size_t)tp_chunks(tiles, bits) + 1) * radix));
  if (bits == 8 && sizeof(K) == 8 && dstream_on() && num_passes(hi - lo, 8) > 1) LS_TRY(ws.ensure_dstream(n));
  if (bits != 4) return hipSuccess;
  const int nb = std::min(4, hi - lo);
  return tiles_counts<4, K, Op, V>(ws, in, n, make_digit<Op>((uint32_t)lo, (1u << nb) - 1u, bias), tiles, ws.tc[0],
                                ws.tc[1], tiles * 16u, st);
}

// Counts of an 8-bit pass from the digit stream (tiles: the pass's tiles, or
// a hybrid depth's table when tab != null).
template <typename K, typename V, bool TAB = false, int B = tp_block<K, V>(8)>
hipError_t tiles_counts_u8(Workspace& ws, size_t n, uint32_t rows, uint32_t* C, const uint4* tab,
                           const uint32_t* ntab, hipStream_t st) {
  constexpr int TILE = B * tp_items<K, V>(8);
  ScopedTimer tm("tilecounts", st, n);
  hipLaunchKernelGGL((k_tile_counts_u8<B, TILE, TAB>), dim3(rows), dim3(B), 0, st, ws.dstream, (uint32_t)n, C, tab,
                     ntab);
  return hipGetLastError();
}

// A/B build only (-DLIBSORT_AB_LSD_ANY_ORDER=1): the LSD passes rank by LDS
// atomics like the hybrid's (NOT stable: wrong partial sorts) -- the price of
// the stable ballot rank, for timing.
#ifndef LIBSORT_AB_LSD_ANY_ORDER
#define LIBSORT_AB_LSD_ANY_ORDER 0
#endif
template <int BITS, typename K, typename V, typename Op = RadixDigit>
hipError_t tiles_pass(Workspace& ws, const K* kin, K* kout, const V* vin, V* vout, size_t n, int p, int P,
                      int lo, int hi, hipStream_t st, uint32_t bias = 0) {
  constexpr int B = tp_block_lsd<K, V>(BITS);
  const uint32_t tiles = tp_tiles_lsd<K, V>(n, BITS);
  const int shift = lo + BITS * p;
  const int nb = std::min(BITS, hi - shift);
  const Op op = make_digit<Op>((uint32_t)shift, (1u << nb) - 1u, bias);
  // 4-bit (fused): counts of this pass were produced by the previous pass (or
  // the prologue) in tc[p & 1]; otherwise count this pass's input now.
  // LIBSORT_TP_FUSE=0 turns the fusion off (A/B measurement).
  static const bool fuse_on = [] {
    const char* s = getenv("LIBSORT_TP_FUSE");
    return !(s && s[0] == '0');
  }();
  const bool fused_counts = BITS == 4 && fuse_on;
  uint32_t* cur = fused_counts ? ws.tc[p & 1] : ws.tc[0];
  uint32_t* nxt = ws.tc[(p + 1) & 1];
  // 8-bit: pass p >= 1 counts the digit stream pass p - 1 wrote; pass p
  // writes one for pass p + 1
  const bool dstream = BITS == 8 && sizeof(K) == 8 && dstream_on() && ws.dstream_cap >= n;
  if (dstream && p >= 1)
    LS_TRY((tiles_counts_u8<K, V>(ws, n, tiles, cur, nullptr, nullptr, st)));
  else if (!fused_counts && !(BITS == 4 && p == 0))
    LS_TRY((tiles_counts<BITS, K, Op, V, B>(ws, kin, n, op, tiles, cur, nullptr, 0, st)));
  LS_TRY(tiles_colscan<BITS>(ws, cur, tiles, st));
  ws.last_pass_counts = cur;
  const bool fuse = fused_counts && p + 1 < P;
  const bool dnext = dstream && p + 1 < P;
  const int nb2 = (fuse || dnext) ? std::min(BITS, hi - shift - BITS) : 1;
  const Op op_next = make_digit<Op>((uint32_t)((fuse || dnext) ? shift + BITS : 0), (1u << nb2) - 1u, bias);
  HybridGeo geo{};
  geo.dout = dnext ? ws.dstream : nullptr;
  ScopedTimer tm("tilepass", st, n);
  if (fuse)
    hipLaunchKernelGGL((k_tile_pass<BITS, B, tp_items<K, V>(BITS), K, V, BITS == 4, Op, Op>), dim3(tiles), dim3(B), 0, st,
                       kin, kout, vin, vout, (uint32_t)n, op, op_next, cur, ws.tb, tiles_digit_starts(ws, tiles, BITS),
                       nxt, HybridGeo{});
  else
    hipLaunchKernelGGL((k_tile_pass<BITS, B, tp_items<K, V>(BITS), K, V, false, Op, Op, 0,
                                    LIBSORT_AB_LSD_ANY_ORDER && std::is_same<V, NoValue>::value>),
                       dim3(tiles), dim3(B), 0, st, kin,
                       kout, vin, vout, (uint32_t)n, op, op_next, cur, ws.tb, tiles_digit_starts(ws, tiles, BITS),
                       nxt, geo);
  return hipGetLastError();
}

template <typename K>
constexpr int os_items() { return sizeof(K) == 8 ? kOsItemsU64 : kOsItemsU32; }

// Threads per onesweep tile (256 / 512 / 1024); LIBSORT_OS_BLOCK overrides.
int os_block() {
  const char* s = getenv("LIBSORT_OS_BLOCK");
  const int b = s ? atoi(s) : kOsBlock;
  return (b == 512 || b == 1024) ? b : 256;
}

// memset of the small block, window histograms (+ zero of status buffer 0),
// per-pass digit bases.
template <typename K>
hipError_t onesweep_prologue(Workspace& ws, const K* in, size_t n, int lo, int hi, int bits, int P,
                             uint32_t tiles, hipStream_t st) {
  const int radix = 1 << bits;
  LS_TRY(ws.ensure_onesweep((size_t)tiles * radix));
  LS_TRY(hipMemsetAsync(ws.os_small, 0, kOsZeroWords * sizeof(uint32_t), st));
  const int nw = (hi - lo + 7) / 8;
  const uint32_t blocks = (uint32_t)std::min<uint64_t>((n + 1023) / 1024, (uint64_t)std::max(1, ws.num_cus) * 4);
  const uint32_t zero_words = tiles * (uint32_t)radix;
  {
    ScopedTimer tm("whist", st, n);
#define LS_W(NW)                                                                                     \
  case NW:                                                                                         \
    hipLaunchKernelGGL((k_window_hist<K, NW>), dim3(blocks), dim3(256), 0, st, in, (uint32_t)n,    \
                       (uint32_t)lo, (uint32_t)hi, ws.os_small + kOsWhist, ws.os_status[0],        \
                       zero_words);                                                                \
    break;
    switch (nw) {
      LS_W(1) LS_W(2) LS_W(3) LS_W(4) LS_W(5) LS_W(6) LS_W(7) LS_W(8)
      default: return hipErrorInvalidValue;
    }
#undef LS_W
    LS_TRY(hipGetLastError());
  }
  if (bits == 8)
    hipLaunchKernelGGL(k_pass_offsets<8>, dim3(P), dim3(256), 0, st, ws.os_small + kOsWhist,
                       ws.os_small + kOsGbase);
  else
    hipLaunchKernelGGL(k_pass_offsets<4>, dim3(P), dim3(256), 0, st, ws.os_small + kOsWhist,
                       ws.os_small + kOsGbase);
  return hipGetLastError();
}

template <int BITS, typename K, typename V>
hipError_t onesweep_pass(Workspace& ws, const K* kin, K* kout, const V* vin, V* vout, size_t n, int p,
                         int P, uint32_t shift, uint32_t nbits, uint32_t tiles, hipStream_t st) {
  constexpr int RADIX = 1 << BITS;
  RadixDigit op{shift, (1u << nbits) - 1u};  // nbits <= 8
  uint32_t* status = ws.os_status[p & 1];
  uint32_t* next = (p + 1 < P) ? ws.os_status[(p + 1) & 1] : nullptr;
  ScopedTimer tm("onesweep", st, n);
#define LS_OS(B, A)                                                                                      \
  hipLaunchKernelGGL((k_onesweep<BITS, B, os_items<K>(), K, V, A>), dim3(tiles), dim3(B), 0, st, kin, kout, \
                     vin, vout, (uint32_t)n, op, status, next, ws.os_small + kOsGbase + p * RADIX,        \
                     ws.os_small + kOsCounters + p, ws.os_small + kOsErr)
  const char* abl = getenv("LIBSORT_DIAG_ABLATION");  // diagnostics only: 1 = coalesced, 2 = no writes
  const int a = (abl && std::is_same<V, NoValue>::value) ? atoi(abl) : 0;
  switch (os_block() * 4 + (a >= 1 && a <= 3 ? a : 0)) {
    case 512 * 4 + 3: LS_OS(512, 3); break;
    case 256 * 4 + 3: LS_OS(256, 3); break;
    case 1024 * 4: LS_OS(1024, 0); break;
    case 512 * 4: LS_OS(512, 0); break;
    case 512 * 4 + 1: LS_OS(512, 1); break;
    case 512 * 4 + 2: LS_OS(512, 2); break;
    case 256 * 4 + 1: LS_OS(256, 1); break;
    case 256 * 4 + 2: LS_OS(256, 2); break;
    default: LS_OS(256, 0); break;
  }
#undef LS_OS
  return hipGetLastError();
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
                     size_t n, int lo, int hi, int bits, hipStream_t st, uint32_t bias = 0) {
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
  // a biased (range-restricted) sort always takes the tile path (onesweep's
  // window histogram and reduce-then-scan read raw key bits)
  constexpr bool kCanBias = std::is_same<K, uint32_t>::value && std::is_same<V, NoValue>::value;
  if (bias && (!kCanBias || (bits != 4 && bits != 8))) return hipErrorInvalidValue;
  const int algo = bias ? 3 : (bits == 4 || bits == 8) ? choose_algorithm(n, bits) : 2;
  const bool os = algo == 1;
  const bool tp = algo == 3;
  ws.last_algo = algo;
  const int OS_TILE = os_block() * os_items<K>();
  const uint32_t tiles = (uint32_t)((n + OS_TILE - 1) / OS_TILE);
  if (os) LS_TRY(onesweep_prologue<K>(ws, in, n, lo, hi, bits, P, tiles, st));
  if (tp && bias) {
    if constexpr (kCanBias) LS_TRY((tiles_prologue<K, V, BiasedDigit>(ws, in, n, lo, hi, bits, st, bias)));
  } else if (tp) {
    LS_TRY((tiles_prologue<K, V>(ws, in, n, lo, hi, bits, st)));
  }
  for (int p = 0; p < P; ++p) {
    const int shift = lo + p * bits;
    const int nb = std::min(bits, hi - shift);
    K* kdst = dst_is_out(p) ? out : tmp;
    V* vdst = dst_is_out(p) ? vout : vtmp;
    if (tp && bias) {
      if constexpr (kCanBias) {
        if (bits == 4)
          LS_TRY((tiles_pass<4, K, V, BiasedDigit>(ws, ksrc, kdst, vsrc, vdst, n, p, P, lo, hi, st, bias)));
        else
          LS_TRY((tiles_pass<8, K, V, BiasedDigit>(ws, ksrc, kdst, vsrc, vdst, n, p, P, lo, hi, st, bias)));
      }
    } else if (tp) {
      if (bits == 4)
        LS_TRY((tiles_pass<4, K, V>(ws, ksrc, kdst, vsrc, vdst, n, p, P, lo, hi, st)));
      else
        LS_TRY((tiles_pass<8, K, V>(ws, ksrc, kdst, vsrc, vdst, n, p, P, lo, hi, st)));
    } else if (os) {
      if (bits == 8)
        LS_TRY((onesweep_pass<8, K, V>(ws, ksrc, kdst, vsrc, vdst, n, p, P, (uint32_t)shift, (uint32_t)nb, tiles, st)));
      else
        LS_TRY((onesweep_pass<4, K, V>(ws, ksrc, kdst, vsrc, vdst, n, p, P, (uint32_t)shift, (uint32_t)nb, tiles, st)));
    } else {
      LS_TRY(run_digit_pass<K, V>(ws, bits, ksrc, kdst, vsrc, vdst, n, (uint32_t)shift, (uint32_t)nb, st));
    }
    ksrc = kdst;
    vsrc = vdst;
  }
  if (ksrc != out) LS_TRY(copy_buf(out, ksrc, vout, vsrc, n, st));
  return hipSuccess;
}

// gpuPartial boundaries from the sorted keys (n > 0): sentinel fill, marks,
// suffix-minimum scan (k_bounds_*).  Scratch: ws.hist_tmp.
hipError_t group_bounds(Workspace& ws, const uint32_t* sorted, size_t n, int lo, uint32_t ngroups, uint32_t* d_bounds,
                        hipStream_t st) {
  const uint64_t nb = ((uint64_t)ngroups + kBmTile - 1) / kBmTile;
  if (ws.hist_tmp_cap < nb) {
    if (ws.hist_tmp) { (void)hipFree(ws.hist_tmp); ws.hist_tmp = nullptr; }
    ws.hist_tmp_cap = 0;
    LS_TRY(hipMalloc(&ws.hist_tmp, nb * sizeof(uint32_t)));
    ws.hist_tmp_cap = nb;
  }
  LS_TRY(hipMemsetAsync(d_bounds, 0xff, (size_t)ngroups * sizeof(uint32_t), st));
  const uint32_t blocks = (uint32_t)((n + 256 * kBmkItems - 1) / (256 * kBmkItems));
  const uint32_t vec = (reinterpret_cast<uintptr_t>(sorted) & 15u) == 0 ? 1u : 0u;
  hipLaunchKernelGGL(k_bounds_mark_u32, dim3(blocks), dim3(256), 0, st, sorted, (uint32_t)n, (uint32_t)lo,
                     ngroups - 1u, vec, d_bounds);
  LS_TRY(hipGetLastError());
  hipLaunchKernelGGL(k_bounds_min_blocks, dim3((uint32_t)nb), dim3(kBmBlock), 0, st, d_bounds, (uint64_t)ngroups,
                     ws.hist_tmp);
  LS_TRY(hipGetLastError());
  hipLaunchKernelGGL(k_bounds_min_top, dim3(1), dim3(1024), 0, st, ws.hist_tmp, (uint32_t)nb);
  LS_TRY(hipGetLastError());
  hipLaunchKernelGGL(k_bounds_min_apply, dim3((uint32_t)nb), dim3(kBmBlock), 0, st, d_bounds, (uint64_t)ngroups,
                     ws.hist_tmp, (uint32_t)n);
  return hipGetLastError();
}

// ----------------------------------------------------------------------------
// MSD hybrid for full sorts of uint32 keys (DESIGN.md §3 "MSD passes +
// bucket sort"): all 32 bits, or a range sort's W bits of key - bias (keys in
// [bias, bias + 2^W)).  DEPTHS = 16 / BITS digit passes from the TOP digit down,
// each a stable partition of every segment (keys sharing the digits above) by
// its next digit, cut into segment-aligned tiles; then every one of the 2^16
// buckets (keys sharing their top 16 of W bits, ~n / 65536 keys) is sorted
// on its low W - 16 bits on chip by k_bucket_sort.  HBM passes: DEPTHS + 1 instead of
// 32 / BITS.  Keys only: order among equal keys is not observable.
// Buffers: depth k reads buf[k] and writes buf[k + 1] with buf[0] = in,
// buf[odd] = tmp, buf[even > 0] = out; DEPTHS is even, so the buckets are
// sorted in place in out.
// Host checks (the stream is synchronised twice, without idling the GPU):
// after the first column scan, a top digit holding more than 1.5 n / RADIX
// keys (a skewed input, buckets would overflow) abandons the hybrid
// (*handled = false: the caller runs the LSD sort; in is untouched); after
// the bucket sort, buckets too large for a block (counted on the device) are
// sorted by an LSD sort of out in place.
#ifndef LIBSORT_BUCKET64_FIX
#define LIBSORT_BUCKET64_FIX 16
#endif
#ifndef LIBSORT_BUCKET64_BLOCK
#define LIBSORT_BUCKET64_BLOCK 512
#endif
constexpr size_t kHybMinKeys = 1ull << 27;
// 64-bit keys: the LSD sort needs 8 (16) passes, so the hybrid pays from 2^25
// keys (tools/hyb_sizes.py: (u64, u32) pairs 2^24 0.91x, 2^25 1.41x, 2^26 2.14x)
constexpr size_t kHybMinKeys64 = 1ull << 25;
// (u32 buckets of the top 16 bits: up to ~8.3K keys on average in the
// 512-thread class; 64-bit keys keep the 2^28 + 2^24 bound of round 2)
constexpr size_t kHybMaxKeys = (1ull << 30) + (1ull << 24);  // keys only (class 5 above 2^29 + 2^23)
constexpr size_t kHybMaxKeysPairs = (1ull << 29) + (1ull << 23);
constexpr size_t kHybMaxKeys64 = (1ull << 28) + (1ull << 24);
// Range sorts (W bits of key - lo, W < 32: 7 LSD passes at the 8-GPU rounds'
// W = 27, buckets of W - 16 = 11 bits) gain from fewer keys: the round sorts of
// configs[3]'s schedule (tools/round_sorts.py, 2^29 keys per rank in 4 rounds)
// 100M keys 1.44 -> 1.23 ms, 120M 1.49 -> 1.34 ms.
constexpr size_t kHybMinKeysRange = (1ull << 26) + (1ull << 24);
// u32 sorts' lower bound (A/B knob LIBSORT_HYB_MIN_LOG2, read once, for both)
inline size_t hyb_min_keys_u32(bool range) {
  static const int lg = [] {
    const char* s = getenv("LIBSORT_HYB_MIN_LOG2");
    const int v = s && *s ? atoi(s) : 0;
    return v >= 10 && v <= 28 ? v : 0;
  }();
  return lg ? (size_t)1 << lg : range ? kHybMinKeysRange : kHybMinKeys;
}


// The hybrid waits on the host twice per call (its skew and bucket-size
// read-backs), which a stream under graph capture cannot do: captured sorts
// take the LSD passes (hipStreamIsCapturing).
inline int hybrid_mode_for(hipStream_t st) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone) return 0;
  return get_hybrid_mode();
}

// Pre-partitioned input of the hybrid (sort_pieces_u32): depth 0's tiles are
// cut per PIECE instead of over the whole input.  Piece p = keys in[off_p,
// off_p + len_p) of segment seg_p; the keys of segment s share every bit above
// the W sorted bits, segments increase with s, and the output holds them in
// segment order (segment s from cstart[s]).  The table on the device (built by
// the host, uploaded once): pieces[np] as uint4 (off, len, seg, first tile),
// then ctile0[nseg + 1] (each segment's first tile; ctile0[nseg] = T0) and
// cstart[nseg] (each segment's output start).
struct HybPieces {
  const uint32_t* dev;  // the table above
  uint32_t np, nseg;
  uint32_t tiles;       // T0 = sum over pieces of ceil(len / TILE)
  int depths;           // digit passes (the bucket sort covers W - BITS * depths bits)
  double fill;          // populated segments / nseg (sizes the bucket blocks)
  const uint32_t* cum;  // [np + 1] keys before each piece (the reserved depth 0's sampler)
  // 24-bit pieces (sort_pieces_planar_u32): the low 16 bits, bits 16..23, and
  // per segment its keys' top byte << 24; null: u32 keys in `in`
  const uint16_t* i16 = nullptr;
  const uint8_t* i8 = nullptr;
  const uint32_t* seghi = nullptr;
};

// Words of the reserved depth 0's slices: n keys plus each slice's sampled
// slack (k_rsv_sample: (s + 5 sqrt(s) + 24) N / S per slice, rounded up to
// whole tiles), over NS = nc * 8 slices, S samples per range: at most
// n (1 + 5 sqrt(nc / S) + 25 nc / S) + NS * TILE.
inline size_t rsv_capacity_bound_nc(size_t n, uint32_t nc, uint32_t S, uint32_t tile) {
  const double f = 5.0 * std::sqrt((double)nc / S) + 25.0 * nc / S;
  return n + (size_t)std::ceil((double)n * f) + (size_t)nc * kRsvRanges * tile + 1024;
}

// Depth 0 of a pre-partitioned input: tile t of piece p (first tile w <= t <
// next piece's first tile) = (off + k * TILE, min(TILE, len - k * TILE), seg),
// k = t - w (binary search over the pieces); the segments' first tiles and
// output starts are copied to the depth-0 parent arrays, ctr[0] = T0.
template <int TILE>
__global__ __launch_bounds__(256) void k_hyb_pieces(const uint4* __restrict__ pieces, uint32_t np,
                                                    const uint32_t* __restrict__ segtab, uint32_t nseg, uint32_t T0,
                                                    uint4* __restrict__ tiles, uint32_t* __restrict__ ctile0,
                                                    uint32_t* __restrict__ cstart, uint32_t* __restrict__ ctr) {
  const uint32_t t = blockIdx.x * 256 + threadIdx.x;
  if (t <= nseg) ctile0[t] = segtab[t];
  if (t < nseg) cstart[t] = segtab[nseg + 1 + t];
  if (t == 0) ctr[0] = T0;
  if (t >= T0) return;
  uint32_t lo = 0, hi = np;  // largest p with first tile <= t
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (pieces[mid].w <= t) lo = mid; else hi = mid;
  }
  const uint4 pc = pieces[lo];
  const uint32_t k = t - pc.w;
  tiles[t] = make_uint4(pc.x + k * TILE, min((uint32_t)TILE, pc.y - k * TILE), pc.z, t);
}

template <int BITS, typename Op, typename K = uint32_t, typename V = NoValue>
hipError_t sort_hybrid(Workspace& ws, const K* in, K* out, K* tmp, const V* vin, V* vout, V* vtmp, size_t n, int W,
                       uint32_t bias, hipStream_t st, bool* handled, uint64_t span = 0,
                       const HybPieces* pc = nullptr) {
  constexpr int RADIX = 1 << BITS;
  // depths >= 1 (tiles from a table) and depth 0 of a whole array (tiles
  // computed: B0 threads, TILE0 keys; the same but for (u64, u32) pairs)
  constexpr int B = tp_block_tab<K, V>(BITS);
  constexpr int ITEMS = tp_items<K, V>(BITS);
  constexpr int TILE = B * ITEMS;
  constexpr int B0 = tp_block<K, V>(BITS);
  constexpr int TILE0 = B0 * ITEMS;
  static_assert(TILE0 == TILE || !std::is_same<V, NoValue>::value, "keys-only: one tile size");
  // digit passes: 16 / BITS over the top 16 of the W bits, or (pieces) the
  // caller's count; the last one writes out: depth k writes out when
  // depths - 1 - k is even, tmp otherwise (depth 0 reads in)
  const int DEPTHS = pc ? pc->depths : 16 / BITS;
  const uint32_t nseg0 = pc ? pc->nseg : 1u;  // segments entering depth 0
  const uint64_t NB64 = (uint64_t)nseg0 << (BITS * DEPTHS);  // buckets
  if (DEPTHS < 1 || NB64 > (1ull << 22) || (pc && (const void*)in == (const void*)out)) return hipErrorInvalidValue;
  const uint32_t NB = (uint32_t)NB64;
  const uint32_t lbits = (uint32_t)(W - BITS * DEPTHS);  // bits the bucket sort orders
  *handled = false;
  // bucket-sort blocks (256 x items keys), in two sizes: the first holds the
  // mean bucket of uniform keys + 3.5 sigma (all but a few of the 65536
  // buckets), those few are listed for the second, 6 x 256 keys larger.
  // Classes: first size 9 / 13 / 17 / 19 keys per thread.
  constexpr uint32_t kListCap = 1024;
  // a range sort's keys lie in [bias, bias + span), span in (2^(W-1), 2^W]:
  // only the first span / 2^(W-16) of the 16-bit prefixes (and span / 2^(W-BITS)
  // of the top digits) are populated, each by n * 2^(W-16) / span keys on
  // average (range rounds of the multi-GPU sort: a W = 27 round spans ~0.8 of
  // 2^27, which the full-width shares would take for skew)
  const double fill = pc ? pc->fill : span ? (double)span / std::ldexp(1.0, W) : 1.0;
  const double mean = (double)n / (NB * fill);
  const double need = mean + 3.5 * std::sqrt(mean);
  // class 4 (32-bit keys): 512-thread blocks of 17 keys per thread for
  // buckets of ~8K keys (full sorts up to 2^29 + 2^23 keys); class 5 (32-bit
  // keys without values, the counting placement only): 1024 x 17 for ~16K
  // keys (2^30-key sorts: configs[2]); without it such a sort takes the LSD
  // passes.  libsortSetBucketMode(0) / LIBSORT_BUCKET_COUNT=0 keeps the LSD
  // steps.
  constexpr bool kCntOk = sizeof(K) == 4 && std::is_same<V, NoValue>::value;
  const bool cnt = kCntOk && get_bucket_mode() == 1 && W - BITS * DEPTHS <= 16;
  const int cls = need <= 256.0 * 9 ? 0 : need <= 256.0 * 13 ? 1 : need <= 256.0 * 17 ? 2 :
                  (need <= 256.0 * 19 || sizeof(K) == 8) ? 3 : need <= 256.0 * 34 ? 4 : 5;
  if (cls == 5 && !cnt) return hipSuccess;  // (not handled: the LSD sort)
  static constexpr int kItems1[6] = {9, 13, 17, 19, 34, 68};  // per 256 threads
  // the two blocks' slots (64-bit keys: 512-thread blocks, keys per thread
  // rounded up)
  constexpr int BB = sizeof(K) == 8 ? LIBSORT_BUCKET64_BLOCK : 256;
  const int BBc = cls == 5 ? 1024 : cls == 4 ? 512 : BB;
  const int extra = cls == 5 ? 24 : cls == 4 ? 12 : 6;  // second block: 6 (12, 24) x 256 more slots
  const uint32_t cap1 = (uint32_t)BBc * (((uint32_t)kItems1[cls] * 256u + BBc - 1) / BBc);
  const uint32_t cap = (uint32_t)BBc * (((uint32_t)(kItems1[cls] + extra) * 256u + BBc - 1) / BBc);
  const uint32_t T0 = pc ? pc->tiles : (uint32_t)((n + TILE0 - 1) / TILE0);  // depth 0's tiles
  const uint32_t Tt = pc ? pc->tiles : (uint32_t)((n + TILE - 1) / TILE);    // n in table-depth tiles
  // reserved depth 0 (32-bit keys only, in != out: the fallback re-reads in):
  // no count pass; depth 0 writes slices of ws.rsv (tile rows of depth 1
  // numbered by slice capacity, at most tb1)
  // (pieces: slices per (segment, digit, range), at most kRsvMaxSlices)
  constexpr bool kRsvOk = sizeof(K) == 4 && std::is_same<V, NoValue>::value;
  const uint32_t rnc = (pc ? nseg0 : 1u) * (uint32_t)RADIX;  // children of depth 0
  const uint32_t rns = rnc * kRsvRanges;                      // slices
  int rmode = kRsvOk && DEPTHS > 1 && (const void*)in != (const void*)out && (!pc || (pc->cum && rns <= kRsvMaxSlices))
                  ? rsv_mode()
                  : 0;
  const int rper = rsv_pc_per(rnc);
  const size_t rbound = pc ? rsv_capacity_bound_nc(n, rnc, kRsvBlocks * 256 * rper, TILE)
                           : rsv_capacity_bound(n, BITS);
  const uint32_t tb1 = (uint32_t)((rbound + TILE - 1) / TILE) + rns;
  // the cursors after the slices, 256-byte aligned (8-bit: 64-bit adds)
  const size_t rcur_off = (rbound + 63) & ~(size_t)63;
  // The slices (~1.14 n words at 4-bit digits, ~1.28 n at 8-bit) stay cached
  // in the workspace like its other buffers (grow-only, freed by
  // libsortRelease).  If they cannot be allocated, depth 0 takes the count
  // pass instead: the sort needs no more memory than before.
  // (LIBSORT_HYB_RESERVE=nomem: as if the allocation failed -- tests)
  if (rmode == 3 || (rmode && ws.ensure_rsv(rcur_off + (size_t)rns * kRsvCurStride) != hipSuccess)) {
    (void)hipGetLastError();
    rmode = 0;
  }
  const bool rsv = rmode != 0;
  // 24-bit pieces are read by the reserved depth 0 only: otherwise the
  // caller's gather (which unpacks them) and LSD sort
  if (pc && pc->i8 && !rsv) return hipSuccess;
  uint32_t rseq = 0;  // the sampler's sequence word (wait_host_word)
  uint32_t sseq = 0;  // the last depth's children (bucket stats)
  // segments of depth k (each child has at most one partial tile)
  auto nseg_at = [&](int k) { return nseg0 << (BITS * k); };
  auto tbound = [&](int k) { return k == 0 ? T0 : (k == 1 && rsv) ? tb1 : Tt + nseg_at(k); };
  uint32_t TB = 0;
  for (int k = 0; k < DEPTHS; ++k) TB = std::max(TB, tbound(k));
  LS_TRY(ws.ensure_tiles((size_t)TB * RADIX, ((size_t)tp_chunks(TB, BITS) + 1) * RADIX));
  // hybrid block: tiles[2] | segbase | cstart[2] | nsize | ctile0[2] | ntl | counters
  const size_t w_tiles = (size_t)TB * 4;
  const size_t rsv_words = (size_t)kRsvRanges * kRsvBlocks * rnc + 3 * (size_t)rns + 16;
  const size_t words =
      2 * w_tiles + NB + 2 * (size_t)NB + NB + 2 * ((size_t)NB + 1) + NB + 16 + kListCap + NB + NB + rsv_words;
  LS_TRY(ws.ensure_hybrid(words));
  uint32_t* h = ws.hyb;
  uint4* tiles[2] = {reinterpret_cast<uint4*>(h), reinterpret_cast<uint4*>(h + w_tiles)};
  h += 2 * w_tiles;
  uint32_t* segbase = h; h += NB;
  uint32_t* cstart[2] = {h, h + NB}; h += 2 * (size_t)NB;
  uint32_t* nsize = h; h += NB;
  uint32_t* ctile0[2] = {h, h + NB + 1}; h += 2 * ((size_t)NB + 1);
  uint32_t* ntl = h; h += NB;
  uint32_t* ctr = h;  // [k] tiles of depth k (k <= 4), [7] the LSD-step list after 2-bit cells (flist2),
                      // [8] buckets over the first block, [9] bucket count, [10] over the
                      // second, [11] largest bucket, [12] buckets over the first block (planning),
                      // [13] largest child of depth 0 (pieces), [14] reserved depth 0 overflow,
                      // [15] buckets whose counting placement overflowed
  h += 16;
  uint32_t* olist = h;  // the buckets over the first block (kListCap)
  h += kListCap;
  uint32_t* flist = h;  // the buckets whose counting placement overflowed (ctr[15] of NB)
  h += NB;
  uint32_t* flist2 = h;  // kCnt2F: the buckets for the LSD steps (ctr[7] of NB)
  h += NB;
  // reserved depth 0: sample partials | slices (start | capacity | first tile,
  // + the tile count) | cursors | estimated digit sizes; ctr[14] = overflow
  uint32_t* rpart = h; h += (size_t)kRsvRanges * kRsvBlocks * rnc;
  uint32_t* rslice = h; h += 3 * (size_t)rns + 16;
  uint32_t* rcur = rsv ? ws.rsv + rcur_off : nullptr;  // kRsvCurStride apart
  uint32_t* Cn0 = ws.tc[1];  // depth 1's count rows (the fused counts of depth 0)
  if (!rsv) {  // (reserved depth 0: k_rsv_sample sets them)
    hipLaunchKernelGGL(k_hyb_init, dim3(1), dim3(64), 0, st, ctr, NB);  // one launch, not two memsets (4 fills)
    LS_TRY(hipGetLastError());
  } else {
    // Reserved depth 0: sample -> slices (the depth-0 pass reserves its runs
    // in them; the next depth's tiles and child starts from the cursors)
    const Op op0 = make_digit<Op>((uint32_t)(W - BITS), (uint32_t)RADIX - 1u, bias);
    ScopedTimer tm("rsvsample", st, n);
    rseq = ++ws.hyb_seq;
    if (pc) {
      auto smp = rper == 4 ? k_rsv_sample_pc<RADIX, TILE, 4, Op>
                 : rper == 8 ? k_rsv_sample_pc<RADIX, TILE, 8, Op> : k_rsv_sample_pc<RADIX, TILE, 16, Op>;
      hipLaunchKernelGGL(smp, dim3(kRsvRanges * kRsvBlocks), dim3(256), 0, st,
                         reinterpret_cast<const uint32_t*>(in), pc->i8, reinterpret_cast<const uint4*>(pc->dev), pc->cum,
                         pc->np, nseg0, T0, (uint32_t)n, op0, rpart, rslice, rcur, ws.hyb_host, Cn0,
                         BITS == 4 ? tb1 * (uint32_t)RADIX : 0u, ws.tticket + 32, ctr, NB, rmode == 2, rseq);
    } else {
      hipLaunchKernelGGL((k_rsv_sample<RADIX, TILE, Op>), dim3(kRsvRanges * kRsvBlocks), dim3(256), 0, st,
                         reinterpret_cast<const uint32_t*>(in), (uint32_t)n, T0, op0, rpart, rslice, rcur,
                         ws.hyb_host, Cn0, BITS == 4 ? tb1 * (uint32_t)RADIX : 0u, ws.tticket + 32, ctr, NB,
                         rmode == 2, rseq);
    }
    LS_TRY(hipGetLastError());
  }
  if (pc) {
    // depth 0's tile table and parent arrays from the piece table
    const uint32_t g = std::max(T0, pc->nseg + 1);
    hipLaunchKernelGGL((k_hyb_pieces<TILE>), dim3((g + 255) / 256), dim3(256), 0, st,
                       reinterpret_cast<const uint4*>(pc->dev), pc->np, pc->dev + 4 * (size_t)pc->np, pc->nseg, T0,
                       tiles[0], ctile0[0], cstart[0], ctr);
    LS_TRY(hipGetLastError());
  }
  const bool dstream = BITS == 8 && dstream_on() && (sizeof(K) == 8 || (kRsvOk && !pc && dstream_u32_on()));
  // (reserved depth 0: the stream in the slices' coordinates)
  if (dstream) LS_TRY(ws.ensure_dstream(rsv ? std::max(n, rcur_off) : n));
  ws.part_pending.valid = false;

  // keys only: the passes may reorder within a run (k_tile_pass ANY_ORDER)
  constexpr bool kAnyOrder = std::is_same<V, NoValue>::value;
  auto buf = [&](int k) -> K* {
    return k == 0 ? const_cast<K*>(in) : (k == 1 && rsv) ? reinterpret_cast<K*>(ws.rsv) : ((DEPTHS - k) & 1) ? tmp : out;
  };
  auto vbuf = [&](int k) -> V* { return k == 0 ? const_cast<V*>(vin) : ((DEPTHS - k) & 1) ? vtmp : vout; };
  for (int k = 0; k < DEPTHS; ++k) {
    const bool last = k == DEPTHS - 1;
    const bool tab = k > 0 || pc;  // this depth's tiles come from a table
    const uint32_t rows = tbound(k);
    const uint32_t nseg = nseg_at(k);
    const uint32_t m = nseg * RADIX;  // children
    const Op op = make_digit<Op>((uint32_t)(W - BITS * (k + 1)), (uint32_t)RADIX - 1u, bias);
    const Op op_next = make_digit<Op>((uint32_t)(last ? 0 : W - BITS * (k + 2)), (uint32_t)RADIX - 1u, bias);
    uint32_t* C = (BITS == 4) ? ws.tc[k & 1] : ws.tc[0];
    uint32_t* Cn = ws.tc[(k + 1) & 1];
    const K* src = buf(k);
    K* dst = buf(k + 1);
    const V* vsrc = vbuf(k);
    V* vdst = vbuf(k + 1);
    if constexpr (kRsvOk) {
      if (k == 0 && rsv) {
        // Reserved depth 0 (sampled above): the pass reserves its runs in the
        // slices; the next depth's tiles and child starts from the cursors
        HybridGeo g0{tiles[0], ctr, nullptr, nullptr, nullptr, rcur, rslice, ctr + 14, rns};
        if (dstream && !last) g0.dout = ws.dstream;  // (the next depth's digits, slice positions)
        if (pc) {
          g0.i16 = pc->i16;
          g0.i8 = pc->i8;
          g0.seghi = pc->seghi;
        }
        {
          ScopedTimer tm("tilepass", st, n);
          if (pc)
            hipLaunchKernelGGL((k_tile_pass<BITS, B, ITEMS, K, V, BITS == 4, Op, Op, 5, true>), dim3(T0), dim3(B), 0,
                               st, src, dst, vsrc, vdst, (uint32_t)n, op, op_next, C, ws.tb, segbase, Cn, g0);
          else
            hipLaunchKernelGGL((k_tile_pass<BITS, B, ITEMS, K, V, BITS == 4, Op, Op, 4, true>), dim3(T0), dim3(B), 0,
                               st, src, dst, vsrc, vdst, (uint32_t)n, op, op_next, C, ws.tb, segbase, Cn, g0);
          LS_TRY(hipGetLastError());
        }
        {
          ScopedTimer tm("hybplan", st, m);
          hipLaunchKernelGGL((k_rsv_tiles<RADIX, TILE, BITS == 4>), dim3((tb1 + 255) / 256), dim3(256), 0, st, rslice,
                             rcur, ctr + 14, tb1, tiles[1], cstart[1], ctile0[1], ctr + 1, Cn, rnc);
          LS_TRY(hipGetLastError());
        }
        // skew check on the sampled digit (pieces: child) sizes (the pass
        // keeps the GPU busy; it wrote only ws.rsv, so abandoning leaves in
        // intact).  The sampler raised its sequence word in the pinned
        // mirror after the sizes: polled, not an event (an event record
        // stalls the stream ~6 us).
        LS_TRY(wait_host_word(ws.hyb_host + kHybSeqWord, rseq, st));
        if (pc) {
          if ((double)ws.hyb_host[0] / (double)(1ull << (BITS * (DEPTHS - 1))) > 0.9 * cap) return hipSuccess;
        } else {
          uint32_t mx = 0;
          for (int d = 0; d < RADIX; ++d) mx = std::max(mx, ws.hyb_host[d]);
          const double share = (double)n / (RADIX * fill);
          if ((double)mx > 1.25 * share + 4.0 * std::sqrt(share) + 32.0 ||
              (double)mx / (double)(NB / RADIX) > 0.9 * cap)
            return hipSuccess;
        }
        continue;
      }
    }
    // counts of this depth: depth 0 reads the keys (pieces: tile by tile from
    // the table); 4-bit deeper depths were counted by the previous pass
    // (fused); 8-bit deeper depths read the keys tile by tile from the table
    if (k == 0 && !pc) {
      LS_TRY((tiles_counts<BITS, K, Op, V>(ws, src, n, op, T0, C, BITS == 4 ? Cn : nullptr,
                                           BITS == 4 ? T0 * (uint32_t)RADIX : 0u, st)));
    } else if (BITS == 8 && dstream && k > 0) {
      // the digits depth k - 1 wrote (1 B per key)
      LS_TRY((tiles_counts_u8<K, V, true, B>(ws, n, rows, C, tiles[k & 1], ctr + k, st)));
    } else if (BITS == 8 || k == 0) {
      ScopedTimer tm("tilecounts", st, n);
      hipLaunchKernelGGL((k_tile_counts<BITS, B, ITEMS, K, Op, true>), dim3(rows), dim3(B), 0, st, src,
                         (uint32_t)n, op, C, nullptr, 0u, tiles[k & 1], ctr + k);
      LS_TRY(hipGetLastError());
    }
    LS_TRY(tiles_colscan<BITS>(ws, C, rows, st));
    const uint32_t* D = tiles_digit_starts(ws, rows, BITS);
    if (k == 0 && !pc) {
      // the top digit's sizes, for the skew check below
      LS_TRY(hipMemcpyAsync(ws.hyb_host, D, RADIX * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
      LS_TRY(hipEventRecord(ws.hyb_evt, st));
    }
    {
      ScopedTimer tm("hybplan", st, m);
      // stats: the last depth's bucket sizes (ctr[11], [12]); pieces, depth 0
      // of several: its largest child (ctr[13]) for the skew check
      // (the last depth: ctr[11..14] -> hyb_host[256..259], written by the
      // kernel's last block and read back while the last pass runs; other
      // depths: the next depth's tile prefix in the last block)
      uint32_t* stats = last ? ctr + 11 : (pc && k == 0) ? ctr + 13 : nullptr;
      hipLaunchKernelGGL((k_hyb_children<RADIX, TILE>), dim3((m + 255) / 256), dim3(256), 0, st, C, ws.tb, D, rows,
                         (uint32_t)n, nseg, tab ? ctile0[k & 1] : nullptr, cstart[k & 1], T0, segbase,
                         cstart[(k + 1) & 1], nsize, last ? nullptr : ntl, stats, cap1, ws.tticket + 48,
                         last ? nullptr : ctile0[(k + 1) & 1], ctr + k + 1, ctr + 11,
                         last ? ws.hyb_host + 256 : nullptr, ws.hyb_host + kHybSeqWord2, last ? ++ws.hyb_seq : 0u);
      LS_TRY(hipGetLastError());
      if (last) {
        sseq = ws.hyb_seq;
      } else if (pc && k == 0) {
        LS_TRY(hipMemcpyAsync(ws.hyb_host + 260, ctr + 13, sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        LS_TRY(hipEventRecord(ws.hyb_evt, st));
      }
      if (!last) {
        const uint32_t nb_ = tbound(k + 1);
        hipLaunchKernelGGL((k_hyb_expand<RADIX, TILE>), dim3((nb_ + 255) / 256), dim3(256), 0, st,
                           ctile0[(k + 1) & 1], m, cstart[(k + 1) & 1], nsize, ctr + k + 1, nb_,
                           tiles[(k + 1) & 1], BITS == 4 ? Cn : nullptr);
        LS_TRY(hipGetLastError());
      }
    }
    HybridGeo geo{tiles[k & 1], ctr + k, cstart[(k + 1) & 1], ctile0[(k + 1) & 1], nullptr, nullptr, nullptr, nullptr, 0u};
    if (BITS == 8 && dstream && !last) geo.dout = ws.dstream;  // the next depth's digits
    {
      ScopedTimer tm("tilepass", st, n);
      if (BITS == 4 && !last) {
        if (!tab)
          hipLaunchKernelGGL((k_tile_pass<BITS, B0, ITEMS, K, V, BITS == 4, Op, Op, 2, kAnyOrder>),
                             dim3(rows), dim3(B0), 0, st, src, dst, vsrc, vdst, (uint32_t)n, op, op_next, C,
                             ws.tb, segbase, Cn, geo);
        else
          hipLaunchKernelGGL((k_tile_pass<BITS, B, ITEMS, K, V, BITS == 4, Op, Op, 3, kAnyOrder>),
                             dim3(rows), dim3(B), 0, st, src, dst, vsrc, vdst, (uint32_t)n, op, op_next, C,
                             ws.tb, segbase, Cn, geo);
      } else if (!tab) {
        hipLaunchKernelGGL((k_tile_pass<BITS, B0, ITEMS, K, V, false, Op, Op, 0, kAnyOrder>), dim3(rows),
                           dim3(B0), 0, st, src, dst, vsrc, vdst, (uint32_t)n, op, op_next, C, ws.tb, segbase,
                           Cn, geo);
      } else {
        hipLaunchKernelGGL((k_tile_pass<BITS, B, ITEMS, K, V, false, Op, Op, 1, kAnyOrder>), dim3(rows),
                           dim3(B), 0, st, src, dst, vsrc, vdst, (uint32_t)n, op, op_next, C, ws.tb, segbase,
                           Cn, geo);
      }
      LS_TRY(hipGetLastError());
    }
    if (k == 0 && !pc) {
      // skew check (the pass above keeps the GPU busy meanwhile; it wrote
      // only tmp, so abandoning here leaves in intact)
      LS_TRY(hipEventSynchronize(ws.hyb_evt));
      uint32_t mx = 0;
      for (int d = 0; d < RADIX; ++d) {
        const uint32_t e = d + 1 < RADIX ? ws.hyb_host[d + 1] : (uint32_t)n;
        mx = std::max(mx, e - ws.hyb_host[d]);
      }
      // a top digit well above its share (beyond sampling noise), or one
      // whose buckets would average > 0.9 of a block: the LSD sort instead
      const double share = (double)n / (RADIX * fill);
      if ((double)mx > 1.25 * share + 4.0 * std::sqrt(share) + 32.0 ||
          (double)mx / (double)(NB / RADIX) > 0.9 * cap)
        return hipSuccess;
    } else if (k == 0 && !last) {
      // pieces: a depth-0 child whose buckets would average > 0.9 of a block
      // (a skewed input): the caller's LSD sort instead (in is untouched)
      LS_TRY(hipEventSynchronize(ws.hyb_evt));
      if ((double)ws.hyb_host[260] / (double)(1ull << (BITS * (DEPTHS - 1))) > 0.9 * cap) return hipSuccess;
    }
  }
  // the bucket sizes (read back while the last pass runs): a bucket larger
  // than the second block, or more buckets over the first than its list
  // holds -> the LSD sort of out (any order sorts) instead of the bucket sort
  // (polled: the children kernel raised the sequence word after them)
  LS_TRY(wait_host_word(ws.hyb_host + kHybSeqWord2, sseq, st));
  // reserved depth 0 overflowed (a slice's sample undercounted it): the
  // later depths did nothing; the caller's LSD sort from the input instead
  if (rsv && ws.hyb_host[259]) return hipSuccess;
  *handled = true;
  if (ws.hyb_host[257] > kListCap || ws.hyb_host[256] > cap) {
    // pieces: every bit (the segments' own bits vary across out)
    if (pc) return sort_impl<K, V>(ws, out, out, tmp, vout, vout, vtmp, n, 0, 8 * (int)sizeof(K), BITS, st);
    return sort_impl<K, V>(ws, out, out, tmp, vout, vout, vtmp, n, 0, W, BITS, st, bias);
  }
  // bucket sort of the NB buckets in place in out (cstart/nsize of the last
  // depth's children)
  {
    ScopedTimer tm("bucketsort", st, n);
    const uint32_t* bstart = cstart[DEPTHS & 1];
    // 64-bit keys: 512-thread blocks (BB; the same slots in half the keys per
    // thread: 152 -> ~90 VGPRs for (u64, u32) pairs at 17 slots per 256)
    // 64-bit keys: on-chip steps over the top 16 of the 48 bucket bits, then
    // the tie fix-up (k_bucket_sort FIX)
    constexpr int FIXB = sizeof(K) == 8 ? LIBSORT_BUCKET64_FIX : 0;
    constexpr bool kPairCnt = sizeof(K) == 8 && std::is_same<V, uint32_t>::value && FIXB > 0;
    // the second size's grid: the buckets over the first block, as planned
    // (k_hyb_children's count, the same cap as the first launch lists by);
    // none: no launch
    const uint32_t n2 = std::min<uint32_t>(ws.hyb_host[257], kListCap);
    // 32-bit keys without values, lbits <= 16: the counting placement
    // (k_bucket_sort CNT, `cnt` above)
    auto launch = [&](auto cnt_c) -> hipError_t {
      constexpr bool C = decltype(cnt_c)::value;
      // 2-bit cells (256-thread blocks, lbits 16): their lightly overflowed
      // buckets (a value with 4+ keys; ~4% of uniform 4096-key buckets) and
      // the buckets over the first block get a 3-bit retry in blocks of the
      // second size (a persistent LIST launch over flist, count ctr[15]: no
      // separate second-size launch); heavy overflows, and the retry's, go
      // to the LSD steps (flist2, count ctr[7]); other modes list straight
      // for the LSD steps (flist)
      const bool two = C && lbits == 16 && BB == 256 && cls <= 3 && bucket2_on();
      // (u64 key, u32 payload) pairs: k_bucket_pairs (LIBSORT_PAIR_COUNT=0:
      // the LSD steps + fix-up of k_bucket_sort FIX)
      const bool pcnt = kPairCnt && lbits >= 16 && lbits <= 48 && pair_count_on();
      // (inline: the retry list holds only the buckets over the first block,
      // so the 3-bit LIST launch runs only when the planning counted any)
      const bool inl = two && bucket2_inline_on();
      uint32_t* const lsd_n = two ? ctr + 7 : ctr + 15;  // the LSD steps' list
      uint32_t* const lsd_l = two ? flist2 : flist;
      uint32_t* const rty_n = two ? ctr + 15 : nullptr;
      uint32_t* const rty_l = two ? flist : nullptr;
#if LIBSORT_BUCKET2_INLINE_AB
#define LS_BS_INL(B, I, G, NBP, CAPN, IL, OV, OL)                                                            \
  hipLaunchKernelGGL((k_bucket_count<B, (I), Op, kCnt2F, false, true>), dim3(G), dim3(B), 0, st, ci_, co_, \
                     bstart, nsize, NBP, CAPN, IL, lbits, bias, OV, OL, ocap_, lsd_n, lsd_l, rty_n, rty_l)
#else
#define LS_BS_INL(B, I, G, NBP, CAPN, IL, OV, OL) (void)0
#endif
#define LS_BSX(B, I, G, NBP, CAPN, IL, OV, OL)                                                                   \
  if constexpr (C) {                                                                                             \
    const uint32_t* ci_ = reinterpret_cast<const uint32_t*>(out);                                                \
    uint32_t* co_ = reinterpret_cast<uint32_t*>(out);                                                            \
    const uint32_t ocap_ = (OL) == flist ? NB : kListCap;                                                        \
    if (lbits <= 12)                                                                                             \
      hipLaunchKernelGGL((k_bucket_count<B, (I), Op, kCntSmall>), dim3(G), dim3(B), 0, st, ci_, co_, bstart,     \
                         nsize, NBP, CAPN, IL, lbits, bias, OV, OL, ocap_, lsd_n, lsd_l, rty_n, rty_l);             \
    else if (lbits != 16)                                                                                        \
      hipLaunchKernelGGL((k_bucket_count<B, (I), Op, kCnt3>), dim3(G), dim3(B), 0, st, ci_, co_, bstart, nsize,  \
                         NBP, CAPN, IL, lbits, bias, OV, OL, ocap_, lsd_n, lsd_l, rty_n, rty_l);                    \
    else if (B == 256 && two && inl)                                                                             \
      LS_BS_INL(B, I, G, NBP, CAPN, IL, OV, OL);                                                                 \
    else if (B == 256 && two)                                                                                    \
      hipLaunchKernelGGL((k_bucket_count<B, (I), Op, kCnt2F>), dim3(G), dim3(B), 0, st, ci_, co_, bstart, nsize, \
                         NBP, CAPN, IL, lbits, bias, OV, OL, ocap_, lsd_n, lsd_l, rty_n, rty_l);                    \
    else                                                                                                         \
      hipLaunchKernelGGL((k_bucket_count<B, (I), Op, kCnt3F>), dim3(G), dim3(B), 0, st, ci_, co_, bstart, nsize, \
                         NBP, CAPN, IL, lbits, bias, OV, OL, ocap_, lsd_n, lsd_l, rty_n, rty_l);                    \
  } else if (pcnt) {                                                                                             \
    if constexpr (kPairCnt) {                                                                                    \
      /* (u64, u32) pairs: the counting placement, 1024-thread blocks of at least the slots asked for */         \
      constexpr int PI_ = std::max(4, ((B) * (I) + 1023) / 1024);                                                \
      hipLaunchKernelGGL((k_bucket_pairs<1024, PI_, Op>), dim3(G), dim3(1024), 0, st,                            \
                         reinterpret_cast<const uint64_t*>(out), reinterpret_cast<uint64_t*>(out),               \
                         reinterpret_cast<const uint32_t*>(vout), reinterpret_cast<uint32_t*>(vout), bstart,     \
                         nsize, NBP, CAPN, IL, lbits, (uint64_t)bias, OV, OL, kListCap, ctr + 15, flist);        \
    }                                                                                                            \
  } else {                                                                                                       \
    hipLaunchKernelGGL((k_bucket_sort<BITS, B, (I), Op, K, V, FIXB>), dim3(G), dim3(B), 0, st, out, out, vout, vout, \
                       bstart, nsize, NBP, CAPN, IL, lbits, bias, OV, OL, kListCap);                             \
  }
#define LS_BS(I, G, NBP, CAPN, IL, OV, OL) LS_BSX(BB, ((I) * 256 + BB - 1) / BB, G, NBP, CAPN, IL, OV, OL)
#define LS_BS2(I)                                                   \
  if (two) {                                                        \
    /* the buckets over the first block join the retry list */      \
    LS_BS(I, NB, ctr + 9, NB, nullptr, ctr + 15, flist);            \
  } else {                                                          \
    LS_BS(I, NB, ctr + 9, NB, nullptr, ctr + 8, olist);             \
    LS_TRY(hipGetLastError());                                      \
    if (n2) {                                                       \
      LS_BS(I + 6, n2, ctr + 8, kListCap, olist, ctr + 10, nullptr); \
    }                                                               \
  }
#define LS_BS512(I, G, NBP, CAPN, IL, OV, OL) LS_BSX(512, I, G, NBP, CAPN, IL, OV, OL)
#define LS_BS1024(I, G, NBP, CAPN, IL, OV, OL) LS_BSX(1024, I, G, NBP, CAPN, IL, OV, OL)
      // the buckets the counting placement listed (3-bit overflow: 8+ equal
      // keys), by the LSD steps in blocks of the second size: a persistent
      // grid over the list (none listed: the blocks read the count and exit)
#define LS_BSL(B, I)                                                                                               \
  if constexpr (C) {                                                                                               \
    if (two && (!inl || n2 > 0)) {                                                                                 \
      hipLaunchKernelGGL((k_bucket_count<kRetryBlock, ((I) * 256 + kRetryBlock - 1) / kRetryBlock, Op, kCnt3F, true>), \
                         dim3(std::min<uint32_t>(NB, (uint32_t)std::max(1, ws.num_cus) * 5)), dim3(kRetryBlock), 0, st, \
                         reinterpret_cast<const uint32_t*>(out), reinterpret_cast<uint32_t*>(out), bstart, nsize,  \
                         ctr + 15, NB, flist, lbits, bias, ctr + 10, nullptr, 0u, ctr + 7, flist2, nullptr,        \
                         nullptr);                                                                                 \
      LS_TRY(hipGetLastError());                                                                                   \
    }                                                                                                              \
    hipLaunchKernelGGL((k_bucket_sort<BITS, B, (I), Op, K, V, 0, true>),                                           \
                       dim3(std::min<uint32_t>(NB, (uint32_t)std::max(1, ws.num_cus) * 2)), dim3(B), 0, st, out,   \
                       out, vout, vout, bstart, nsize, lsd_n, NB, lsd_l, lbits, bias, ctr + 14, nullptr, 0u);       \
    LS_TRY(hipGetLastError());                                                                                     \
  } else if constexpr (kPairCnt) {                                                                                 \
    if (pcnt) {                                                                                                    \
      /* the pairs whose 3-bit counts would wrap (8+ equal x; their length <= cap, the planning's bound):        \
         the LSD steps + fix-up, persistent over flist */                                                          \
      hipLaunchKernelGGL((k_bucket_sort<BITS, B, (I), Op, K, V, FIXB, true>),                                      \
                         dim3(std::min<uint32_t>(NB, (uint32_t)std::max(1, ws.num_cus) * 2)), dim3(B), 0, st, out, \
                         out, vout, vout, bstart, nsize, ctr + 15, NB, flist, lbits, bias, ctr + 14, nullptr, 0u);  \
      LS_TRY(hipGetLastError());                                                                                   \
    }                                                                                                              \
  }
      switch (cls) {
        case 0: LS_BS2(9); LS_TRY(hipGetLastError()); LS_BSL(BB, (15 * 256 + BB - 1) / BB); break;
        case 1: LS_BS2(13); LS_TRY(hipGetLastError()); LS_BSL(BB, (19 * 256 + BB - 1) / BB); break;
        case 2: LS_BS2(17); LS_TRY(hipGetLastError()); LS_BSL(BB, (23 * 256 + BB - 1) / BB); break;
        case 3: LS_BS2(19); LS_TRY(hipGetLastError()); LS_BSL(BB, (25 * 256 + BB - 1) / BB); break;
        case 4:
          if constexpr (sizeof(K) == 4) {
            LS_BS512(17, NB, ctr + 9, NB, nullptr, ctr + 8, olist);
            LS_TRY(hipGetLastError());
            if (n2) {
              LS_BS512(23, n2, ctr + 8, kListCap, olist, ctr + 10, nullptr);
            }
            LS_TRY(hipGetLastError());
            LS_BSL(512, 23);
          }
          break;
        default:
          if constexpr (C) {
            LS_BS1024(17, NB, ctr + 9, NB, nullptr, ctr + 8, olist);
            LS_TRY(hipGetLastError());
            if (n2) {
              LS_BS1024(23, n2, ctr + 8, kListCap, olist, ctr + 10, nullptr);
            }
            LS_TRY(hipGetLastError());
            LS_BSL(1024, 23);
          }
          break;
      }
      return hipGetLastError();
    };
    if constexpr (kCntOk) {
      if (cnt)
        LS_TRY(launch(std::true_type{}));
      else
        LS_TRY(launch(std::false_type{}));
    } else {
      LS_TRY(launch(std::false_type{}));
    }
#undef LS_BSL
#undef LS_BSX
#undef LS_BS1024
#undef LS_BS512
#undef LS_BS2
#undef LS_BS
  }
  return hipSuccess;
}

}  // namespace

hipError_t sort_u32(Workspace& ws, const uint32_t* in, uint32_t* out, uint32_t* tmp, size_t n, int lo,
                    int hi, int digit_bits, uint32_t* d_bounds, hipStream_t st, uint32_t bias, bool range,
                    uint64_t span) {
  if (bias && d_bounds) return hipErrorInvalidValue;
  const int hyb = hybrid_mode_for(st);
  // the hybrid needs the sorted bits to determine the key: a full 32-bit
  // sort, or a range sort (keys in [bias, bias + 2^hi)) of >= 20 bits
  const bool whole = !d_bounds && lo == 0 && ((hi == 32 && !bias) || (range && hi >= 20));
  if (whole && (digit_bits == 4 || digit_bits == 8) &&
      ((hyb == 1 && n >= hyb_min_keys_u32(range && hi < 32) && n <= kHybMaxKeys) || (hyb == 2 && n >= 1024 && n <= kHybMaxKeys)) &&
      (get_algorithm() == 0 || get_algorithm() == 3) && in != tmp) {
    bool handled = false;
    NoValue* nv = nullptr;
    if (bias && digit_bits == 4)
      LS_TRY((sort_hybrid<4, BiasedDigit>(ws, in, out, tmp, nv, nv, nv, n, hi, bias, st, &handled, span)));
    else if (bias)
      LS_TRY((sort_hybrid<8, BiasedDigit>(ws, in, out, tmp, nv, nv, nv, n, hi, bias, st, &handled, span)));
    else if (digit_bits == 4)
      LS_TRY((sort_hybrid<4, RadixDigit>(ws, in, out, tmp, nv, nv, nv, n, hi, 0u, st, &handled, span)));
    else
      LS_TRY((sort_hybrid<8, RadixDigit>(ws, in, out, tmp, nv, nv, nv, n, hi, 0u, st, &handled, span)));
    if (handled) {
      ws.last_algo = 4;
      return hipSuccess;
    }
  }
  LS_TRY((sort_impl<uint32_t, NoValue>(ws, in, out, tmp, nullptr, nullptr, nullptr, n, lo, hi,
                                      digit_bits, st, bias)));
  if (d_bounds) {
    const int width = hi - lo;
    const uint32_t ngroups = 1u << width;
    ScopedTimer tm("bounds", st, n);
    if (n == 0) {
      LS_TRY(hipMemsetAsync(d_bounds, 0, (size_t)ngroups * sizeof(uint32_t), st));
    } else if (ws.last_algo == 3 && num_passes(width, digit_bits) == 1) {
      // tile path, single pass: the column scan's digit starts
      LS_TRY(hipMemcpyAsync(d_bounds, tiles_digit_starts(ws, tp_tiles_lsd<uint32_t>(n, digit_bits), digit_bits),
                            (size_t)ngroups * sizeof(uint32_t), hipMemcpyDeviceToDevice, st));
    } else if (ws.last_algo == 3 && num_passes(width, digit_bits) == 2 && ws.last_pass_counts) {
      // two passes: from the last pass's counts and the middle buffer (tmp)
      const uint32_t tiles = tp_tiles_lsd<uint32_t>(n, digit_bits);
      const uint32_t dmask = (1u << (width - digit_bits)) - 1u;
      if (digit_bits == 8) {
        constexpr int T8 = tp_block_lsd<uint32_t>(8) * tp_items<uint32_t>(8);
        hipLaunchKernelGGL((k_bounds_lsd2<8, T8>), dim3(256), dim3(256), 0, st, tmp, (uint32_t)n, (uint32_t)lo, dmask,
                           ws.last_pass_counts, ws.tb, tiles_digit_starts(ws, tiles, 8), d_bounds);
      } else {
        constexpr int T4 = tp_block_lsd<uint32_t>(4) * tp_items<uint32_t>(4);
        hipLaunchKernelGGL((k_bounds_lsd2<4, T4>), dim3(16), dim3(256), 0, st, tmp, (uint32_t)n, (uint32_t)lo, dmask,
                           ws.last_pass_counts, ws.tb, tiles_digit_starts(ws, tiles, 4), d_bounds);
      }
      LS_TRY(hipGetLastError());
    } else if (ws.last_algo == 3) {
      LS_TRY(group_bounds(ws, out, n, lo, ngroups, d_bounds, st));
    } else if (ws.last_algo == 1 && width <= 8) {
      // onesweep: window 0 holds exactly the group histogram
      hipLaunchKernelGGL(k_bounds_from_window, dim3(1), dim3(256), 0, st, ws.os_small + kOsWhist, ngroups,
                         d_bounds);
      LS_TRY(hipGetLastError());
    } else if (num_passes(width, digit_bits) == 1) {
      // single pass: the counters of that pass are still in the workspace
      constexpr int TILE = kBlock * kItemsU32;
      const uint32_t grid = pass_grid(ws, (uint32_t)((n + TILE - 1) / TILE));
      hipLaunchKernelGGL(k_bounds_from_scan, dim3((ngroups + 255) / 256), dim3(256), 0, st, ws.scan_l1,
                         ws.scan_l2, grid, ngroups, d_bounds);
      LS_TRY(hipGetLastError());
    } else {
      LS_TRY(group_bounds(ws, out, n, lo, ngroups, d_bounds, st));
    }
  }
  return hipSuccess;
}

// Keys per piece-sort below which auto mode gathers and runs the LSD sort
// (the hybrid's ~10 launches per depth outweigh its saved passes).
constexpr size_t kPiecesMinKeys = 1ull << 20;

namespace {
// 24-bit pieces (sort_pieces_planar_u32): planes of the low 16 bits and bits
// 16..23; the keys of segment s have top byte hi0 + s
struct PlanarPieces {
  const uint16_t* i16 = nullptr;
  const uint8_t* i8 = nullptr;
  uint32_t hi0 = 0;
};

hipError_t sort_pieces_impl(Workspace& ws, const uint32_t* in, const PlanarPieces& pl, uint32_t* out, uint32_t* tmp,
                            size_t n, const uint64_t* off, const uint64_t* len, const uint32_t* seg, size_t np,
                            uint32_t nseg, int bits, int digit_bits, hipStream_t st, uint32_t bias) {
  const bool planar = pl.i8 != nullptr;
  if (n == 0) return hipSuccess;
  if (n > 0xffffffffull || in == out || tmp == out || tmp == in || nseg == 0 || nseg > (1u << 20) || bits < 0 ||
      bits > 32 || (digit_bits != 4 && digit_bits != 8) ||
      (planar && (bits != 24 || bias != 0 || !pl.i16 || pl.hi0 + nseg > 256u)))
    return hipErrorInvalidValue;
  // the non-empty pieces, checked: segments non-decreasing and < nseg, offsets
  // below 2^32, lengths summing to n
  std::vector<size_t> keep;
  keep.reserve(np);
  uint64_t total = 0, maxlen = 0;
  uint32_t prev = 0;
  for (size_t p = 0; p < np; ++p) {
    if (seg[p] < prev || seg[p] >= nseg) return hipErrorInvalidValue;
    prev = seg[p];
    if (!len[p]) continue;
    if (off[p] + len[p] > 0xffffffffull) return hipErrorInvalidValue;
    total += len[p];
    maxlen = std::max(maxlen, len[p]);
    keep.push_back(p);
  }
  if (total != n || keep.size() > 65535) return hipErrorInvalidValue;
  const uint32_t K = (uint32_t)keep.size();
  // segment sizes: the largest sets the digit passes, the populated ones the
  // bucket blocks' size class (a round's last group may span many empty
  // digits)
  std::vector<uint64_t> segsize(nseg, 0);
  for (size_t p : keep) segsize[seg[p]] += len[p];
  uint64_t maxseg = 0;
  uint32_t npop = 0;
  // the populated segments only, renumbered in order (empty segments hold no
  // keys, so the output order is unchanged; a round over many empty digits
  // would otherwise launch a bucket block per empty bucket: 2^29 keys in the
  // 8-GPU shape, a round of 233 digits with 9 populated, ~0.7 ms of empty
  // blocks)
  std::vector<uint32_t> cseg(nseg, 0);
  for (uint32_t s = 0; s < nseg; ++s) {
    maxseg = std::max(maxseg, segsize[s]);
    cseg[s] = npop;
    if (segsize[s]) segsize[npop++] = segsize[s];
  }
  segsize.resize(npop);
  nseg = npop;
  // digit passes: the fewest that bring the largest segment's mean bucket
  // (its keys / RADIX^d, values uniform within a segment) to <= 8320 keys
  // (the 512 x 17-key block holds that + 3.5 sigma), within `bits`
  const int hyb = hybrid_mode_for(st);
  int depths = 0;
  if (bits > 0 && (hyb == 2 ? n >= 1024 : (hyb == 1 && n >= kPiecesMinKeys))) {
    for (int d = 1; d * digit_bits <= bits; ++d) {
      depths = d;
      if ((double)maxseg / std::ldexp(1.0, d * digit_bits) <= 8320.0) break;
    }
    if (((uint64_t)nseg << (digit_bits * depths)) > (1ull << 22)) depths = 0;
  }
  // host table (pinned staging, one upload): pieces uint4 (off, len, seg,
  // first tile) | ctile0[nseg + 1] | cstart[nseg] | cum[K + 1] (keys before
  // each piece) | (8-byte aligned) the gather table of the fallback:
  // src_off[K] | dst_off[K] | len[K] (uint64)
  // (24-bit pieces: a 4th gather column, each piece's top byte << 24, and
  // after it seghi[nseg] (u32) for the reserved depth 0's loader)
  const uint32_t TILE = (uint32_t)(tp_block<uint32_t>(digit_bits) * tp_items<uint32_t>(digit_bits));
  const size_t w32 = 4 * (size_t)K + 2 * (size_t)nseg + 1 + (size_t)K + 1;
  const size_t g64 = (w32 + 1) / 2;  // first uint64 word of the gather table
  const size_t gcols = planar ? 4 : 3;
  const size_t words = g64 + gcols * (size_t)K + (planar ? ((size_t)nseg + 1) / 2 : 0);
  LS_TRY(ws.ensure_seg(words));
  LS_TRY(hipEventSynchronize(ws.seg_evt));  // the staging may still feed the previous upload
  uint32_t* h32 = reinterpret_cast<uint32_t*>(ws.seg_host);
  uint64_t* hg = ws.seg_host + g64;
  uint32_t* ct0 = h32 + 4 * (size_t)K;
  uint32_t* cst = ct0 + nseg + 1;
  uint32_t* pcum = cst + nseg;
  {
    uint64_t run = 0;
    for (uint32_t s = 0; s < nseg; ++s) {
      cst[s] = (uint32_t)run;
      run += segsize[s];
    }
  }
  uint32_t tile = 0, i = 0, run = 0;
  std::vector<uint64_t> dpos(cst, cst + nseg);
  for (uint32_t s = 0; s <= nseg; ++s) {
    ct0[s] = tile;  // segment s's pieces start at this tile
    for (; i < K && (s == nseg || cseg[seg[keep[i]]] == s); ++i) {
      const size_t p = keep[i];
      const uint32_t cs = cseg[seg[p]];
      pcum[i] = run;
      run += (uint32_t)len[p];
      h32[4 * (size_t)i + 0] = (uint32_t)off[p];
      h32[4 * (size_t)i + 1] = (uint32_t)len[p];
      h32[4 * (size_t)i + 2] = cs;
      h32[4 * (size_t)i + 3] = tile;
      tile += (uint32_t)((len[p] + TILE - 1) / TILE);
      hg[i] = off[p];
      hg[K + i] = dpos[cs];
      hg[2 * (size_t)K + i] = len[p];
      if (planar) hg[3 * (size_t)K + i] = (uint64_t)(pl.hi0 + seg[p]) << 24;
      dpos[cs] += len[p];
    }
  }
  pcum[K] = run;
  uint32_t* shi = reinterpret_cast<uint32_t*>(hg + gcols * (size_t)K);
  if (planar)
    for (uint32_t i2 = 0; i2 < K; ++i2) shi[cseg[seg[keep[i2]]]] = (pl.hi0 + seg[keep[i2]]) << 24;
  LS_TRY(hipMemcpyAsync(ws.seg_dev, ws.seg_host, words * sizeof(uint64_t), hipMemcpyHostToDevice, st));
  // seg_evt guards the staging against the next call; a sort the hybrid
  // handled has already waited for a kernel behind this copy (the bucket
  // stats' sequence word), so only the other paths record it (an event
  // costs the stream ~6 us)
  if (depths > 0) {
    const uint32_t* dev32 = reinterpret_cast<const uint32_t*>(ws.seg_dev);
    HybPieces pc{dev32, K, nseg, tile, depths, (double)npop / nseg, dev32 + (pcum - h32)};
    if (planar) {
      pc.i16 = pl.i16;
      pc.i8 = pl.i8;
      pc.seghi = reinterpret_cast<const uint32_t*>(ws.seg_dev + g64 + gcols * (size_t)K);
    }
    bool handled = false;
    NoValue* nv = nullptr;
    hipError_t e;
    if (bias && digit_bits == 4)
      e = sort_hybrid<4, BiasedDigit>(ws, in, out, tmp, nv, nv, nv, n, bits, bias, st, &handled, 0, &pc);
    else if (bias)
      e = sort_hybrid<8, BiasedDigit>(ws, in, out, tmp, nv, nv, nv, n, bits, bias, st, &handled, 0, &pc);
    else if (digit_bits == 4)
      e = sort_hybrid<4, RadixDigit>(ws, in, out, tmp, nv, nv, nv, n, bits, 0u, st, &handled, 0, &pc);
    else
      e = sort_hybrid<8, RadixDigit>(ws, in, out, tmp, nv, nv, nv, n, bits, 0u, st, &handled, 0, &pc);
    if (e != hipSuccess) {
      // a failure may come before the sequence-word wait: guard the staging
      // with the event after all, so the next call's
      // hipEventSynchronize(seg_evt) covers this call's upload
      (void)hipEventRecord(ws.seg_evt, st);
      return e;
    }
    if (handled) {
      ws.last_algo = 4;
      return hipSuccess;
    }
  }
  LS_TRY(hipEventRecord(ws.seg_evt, st));
  // small or skewed: gather the pieces into segment order, LSD sort in place
  // (bits == 0: the segments are single values, already in order); 24-bit
  // pieces are unpacked by the gather
  if (planar) {
    if (K > 65535) return hipErrorInvalidValue;
    {
      ScopedTimer tm("segcopy", st, n);
      hipLaunchKernelGGL(k_segment_copy2d_planar, dim3((uint32_t)((maxlen + kSegPiece - 1) / kSegPiece), K),
                         dim3(256), 0, st, pl.i16, pl.i8, out, ws.seg_dev + g64, K);
      LS_TRY(hipGetLastError());
    }
    // the unpacked keys lie in [top byte of the first populated segment,
    // that of the last + 1) << 24: a range sort of that span (the range
    // hybrid for large rounds) instead of a 32-bit LSD sort -- the rounds of
    // more than 32 segments or without the reserved depth 0
    const uint32_t s0 = seg[keep[0]], s1 = seg[keep[K - 1]];
    const uint32_t lo_key = (pl.hi0 + s0) << 24;
    const uint64_t span = (uint64_t)(s1 - s0 + 1) << 24;
    int W = 24;
    while (((uint64_t)1 << W) < span) ++W;
    return sort_u32(ws, out, out, tmp, n, 0, W, digit_bits, nullptr, st, lo_key, true, span);
  } else {
    LS_TRY(segment_copy_dev_u32(in, out, ws.seg_dev + g64, K, maxlen, n, st));
  }
  if (bits == 0) return hipSuccess;
  return sort_impl<uint32_t, NoValue>(ws, out, out, tmp, nullptr, nullptr, nullptr, n, 0, 32, digit_bits, st);
}
}  // namespace

hipError_t sort_pieces_u32(Workspace& ws, const uint32_t* in, uint32_t* out, uint32_t* tmp, size_t n,
                           const uint64_t* off, const uint64_t* len, const uint32_t* seg, size_t np, uint32_t nseg,
                           int bits, int digit_bits, hipStream_t st, uint32_t bias) {
  return sort_pieces_impl(ws, in, PlanarPieces{}, out, tmp, n, off, len, seg, np, nseg, bits, digit_bits, st, bias);
}

hipError_t sort_pieces_planar_u32(Workspace& ws, const uint16_t* in16, const uint8_t* in8, uint32_t hi0,
                                  uint32_t* out, uint32_t* tmp, size_t n, const uint64_t* off, const uint64_t* len,
                                  const uint32_t* seg, size_t np, uint32_t nseg, int digit_bits, hipStream_t st) {
  // (in: any pointer distinct from out and tmp; the planes are read instead)
  return sort_pieces_impl(ws, reinterpret_cast<const uint32_t*>(in16), PlanarPieces{in16, in8, hi0}, out, tmp, n, off,
                          len, seg, np, nseg, 24, digit_bits, st, 0u);
}

hipError_t sort_pairs_u32_u32(Workspace& ws, const uint32_t* kin, const uint32_t* vin, uint32_t* kout,
                              uint32_t* vout, uint32_t* ktmp, uint32_t* vtmp, size_t n, int lo, int hi,
                              int digit_bits, hipStream_t st) {
  // full-width sorts: the MSD hybrid (stable; the payloads travel with the keys)
  const int hyb = hybrid_mode_for(st);
  if (lo == 0 && hi == 32 && (digit_bits == 8 || digit_bits == 4) &&
      ((hyb == 1 && n >= kHybMinKeys && n <= kHybMaxKeysPairs) || (hyb == 2 && n >= 1024 && n <= kHybMaxKeysPairs)) &&
      (get_algorithm() == 0 || get_algorithm() == 3) && kin != ktmp) {
    bool handled = false;
    if (digit_bits == 8)
      LS_TRY((sort_hybrid<8, RadixDigit, uint32_t, uint32_t>(ws, kin, kout, ktmp, vin, vout, vtmp, n, 32, 0u, st,
                                                              &handled)));
    else
      LS_TRY((sort_hybrid<4, RadixDigit, uint32_t, uint32_t>(ws, kin, kout, ktmp, vin, vout, vtmp, n, 32, 0u, st,
                                                              &handled)));
    if (handled) {
      ws.last_algo = 4;
      return hipSuccess;
    }
  }
  return sort_impl<uint32_t, uint32_t>(ws, kin, kout, ktmp, vin, vout, vtmp, n, lo, hi, digit_bits, st);
}

// 64-bit keys (alone or with u32 / u64 payloads), full-width sorts with 8-bit
// digits: the MSD hybrid (two digit passes over the top 16 bits, buckets
// sorted on chip on the low 48 bits, stable: the passes and the on-chip steps
// keep the order of equal keys, so a payload keeps its input order).
template <typename V>
hipError_t sort_64_hybrid_or_lsd(Workspace& ws, const uint64_t* kin, uint64_t* kout, uint64_t* ktmp, const V* vin,
                                 V* vout, V* vtmp, size_t n, int lo, int hi, int digit_bits, hipStream_t st) {
  const int hyb = hybrid_mode_for(st);
  if (lo == 0 && hi == 64 && (digit_bits == 8 || digit_bits == 4) &&
      ((hyb == 1 && n >= kHybMinKeys64 && n <= kHybMaxKeys64) || (hyb == 2 && n >= 1024 && n <= kHybMaxKeys64)) &&
      (get_algorithm() == 0 || get_algorithm() == 3) && (const void*)kin != (const void*)ktmp) {
    bool handled = false;
    if (digit_bits == 8)
      LS_TRY((sort_hybrid<8, RadixDigit, uint64_t, V>(ws, kin, kout, ktmp, vin, vout, vtmp, n, 64, 0u, st, &handled)));
    else
      LS_TRY((sort_hybrid<4, RadixDigit, uint64_t, V>(ws, kin, kout, ktmp, vin, vout, vtmp, n, 64, 0u, st, &handled)));
    if (handled) {
      ws.last_algo = 4;
      return hipSuccess;
    }
  }
  return sort_impl<uint64_t, V>(ws, kin, kout, ktmp, vin, vout, vtmp, n, lo, hi, digit_bits, st);
}

hipError_t sort_pairs_u64_u32(Workspace& ws, const uint64_t* kin, const uint32_t* vin, uint64_t* kout,
                              uint32_t* vout, uint64_t* ktmp, uint32_t* vtmp, size_t n, int lo, int hi,
                              int digit_bits, hipStream_t st) {
  return sort_64_hybrid_or_lsd<uint32_t>(ws, kin, kout, ktmp, vin, vout, vtmp, n, lo, hi, digit_bits, st);
}

hipError_t sort_u64(Workspace& ws, const uint64_t* in, uint64_t* out, uint64_t* tmp, size_t n, int lo, int hi,
                    int digit_bits, hipStream_t st) {
  NoValue* nv = nullptr;
  return sort_64_hybrid_or_lsd<NoValue>(ws, in, out, tmp, nv, nv, nv, n, lo, hi, digit_bits, st);
}

hipError_t sort_pairs_u64_u64(Workspace& ws, const uint64_t* kin, const uint64_t* vin, uint64_t* kout,
                              uint64_t* vout, uint64_t* ktmp, uint64_t* vtmp, size_t n, int lo, int hi,
                              int digit_bits, hipStream_t st) {
  return sort_64_hybrid_or_lsd<uint64_t>(ws, kin, kout, ktmp, vin, vout, vtmp, n, lo, hi, digit_bits, st);
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

namespace {
// One tile-offset pass whose digit is `op` (a table lookup, or the 8-bit
// digit of key - bias): per-tile counts, column scan, pass kernel; bucket
// starts = row 0 of the scanned chunk totals.  u64 keys: the table indexes
// the top bits of the key's high word.
template <int BITS, typename K, typename V, typename Op>
hipError_t partition_op_impl(Workspace& ws, const K* in, K* out, const V* vin, V* vout, size_t n, Op op,
                             const Workspace::PartToken& tok, int nbuckets, uint32_t* d_bounds, hipStream_t st,
                             int phase, uint16_t* o16 = nullptr, uint8_t* o8 = nullptr) {
  constexpr int RADIX = 1 << BITS;
  // ((u64, u32) pairs at 8 bits: 8192-pair tiles whose payloads are staged
  // through the key buffer; per 2^28 pairs, count + scatter 1.73 ms against
  // 1.82 with the sort's 16384-pair tiles and 1.90 with 4096-pair tiles and
  // LDS of their own, tools/partition_time.py, profiles/r05t_*)
  constexpr int B = tp_block_tab<K, V>(BITS);
  constexpr int TILE = B * tp_items<K, V>(BITS);
  const uint32_t tiles = (uint32_t)((n + TILE - 1) / TILE);
  if (phase != kPartScatter) {
    LS_TRY(ws.ensure_tiles((size_t)tiles * RADIX, ((size_t)tp_chunks(tiles, BITS) + 1) * RADIX));
    LS_TRY((tiles_counts<BITS, K, Op, V, B>(ws, in, n, op, tiles, ws.tc[0], nullptr, 0, st)));
    LS_TRY(tiles_colscan<BITS>(ws, ws.tc[0], tiles, st));
    if (d_bounds)
      LS_TRY(hipMemcpyAsync(d_bounds, tiles_digit_starts(ws, tiles, BITS), (size_t)nbuckets * sizeof(uint32_t),
                            hipMemcpyDeviceToDevice, st));
    if (phase == kPartCount) {
      ws.part_pending = tok;  // the scanned counts stay in the workspace for the scatter call
      return hipSuccess;
    }
  } else if (!(ws.part_pending == tok)) {
    return hipErrorInvalidValue;  // no matching count call, or the workspace was used in between
  }
  ws.part_pending.valid = false;
  {
    ScopedTimer tm("partition", st, n);
    HybridGeo g{};
    g.o16 = o16;  // (24-bit planes instead of out: the multi-GPU exchange)
    g.o8 = o8;
    hipLaunchKernelGGL((k_tile_pass<BITS, B, tp_items<K, V>(BITS), K, V, false, Op>), dim3(tiles), dim3(B), 0, st, in,
                       out, vin, vout, (uint32_t)n, op, RadixDigit{0u, 1u}, ws.tc[0], (const uint32_t*)ws.tb,
                       (const uint32_t*)tiles_digit_starts(ws, tiles, BITS), ws.tc[1], g);
    LS_TRY(hipGetLastError());
  }
  return hipSuccess;
}

template <typename K, typename V>
bool partition_args_ok(const K* in, K* out, const V* vin, V* vout, size_t n, int phase) {
  const bool need_out = phase != kPartCount;
  if (!in || (need_out && (!out || (const void*)in == (const void*)out))) return false;
  if constexpr (!std::is_same<V, NoValue>::value) {
    if (!vin || (need_out && (!vout || (const void*)vin == (const void*)vout))) return false;
  }
  return n <= 0xffffffffull;
}

template <typename K, typename V>
hipError_t partition_lut_any(Workspace& ws, const K* in, K* out, const V* vin, V* vout, size_t n,
                             const uint8_t* d_lut, int lut_shift, int nbuckets, uint32_t* d_bounds, hipStream_t st,
                             int phase = kPartBoth) {
  if (n > 0xffffffffull || lut_shift < 20 || lut_shift > 30 || nbuckets < 1 || nbuckets > 256)
    return hipErrorInvalidValue;
  if (n == 0) {
    if (d_bounds && phase != kPartScatter)
      LS_TRY(hipMemsetAsync(d_bounds, 0, (size_t)nbuckets * sizeof(uint32_t), st));
    return hipSuccess;
  }
  if (!partition_args_ok(in, out, vin, vout, n, phase) || !d_lut || (reinterpret_cast<uintptr_t>(d_lut) & 3u))
    return hipErrorInvalidValue;
  const Workspace::PartToken tok{in, vin, n, d_lut, lut_shift, nbuckets, 0, st, true};
  // digit width by bucket count: 16 -> 4-bit tiles, 32 -> 5-bit (the 8-rank x 4-round exchange), else 8-bit
  if (nbuckets <= 16)
    return partition_op_impl<4, K, V>(ws, in, out, vin, vout, n, LutDigit{d_lut, (uint32_t)lut_shift, 15u, nullptr},
                                      tok, nbuckets, d_bounds, st, phase);
  if (nbuckets <= 32)
    return partition_op_impl<5, K, V>(ws, in, out, vin, vout, n, LutDigit{d_lut, (uint32_t)lut_shift, 31u, nullptr},
                                      tok, nbuckets, d_bounds, st, phase);
  return partition_op_impl<8, K, V>(ws, in, out, vin, vout, n, LutDigit{d_lut, (uint32_t)lut_shift, 255u, nullptr},
                                    tok, nbuckets, d_bounds, st, phase);
}

// 256 buckets by the 8-bit digit (key - bias) >> shift (keys in [bias, bias +
// 2^(shift + 8)): the digit is masked, so a key outside only lands in a wrong
// bucket, never outside the counters).
template <typename K, typename V>
hipError_t partition_range_any(Workspace& ws, const K* in, K* out, const V* vin, V* vout, size_t n, uint64_t bias,
                               int shift, uint32_t* d_bounds, hipStream_t st, int phase) {
  if (n > 0xffffffffull || shift < 0 || shift + 8 > 8 * (int)sizeof(K)) return hipErrorInvalidValue;
  if (n == 0) {
    if (d_bounds && phase != kPartScatter) LS_TRY(hipMemsetAsync(d_bounds, 0, 256 * sizeof(uint32_t), st));
    return hipSuccess;
  }
  if (!partition_args_ok(in, out, vin, vout, n, phase)) return hipErrorInvalidValue;
  const Workspace::PartToken tok{in, vin, n, nullptr, shift, 256, bias, st, true};
  if constexpr (sizeof(K) == 4)
    return partition_op_impl<8, K, V>(ws, in, out, vin, vout, n, BiasedDigit{(uint32_t)shift, 255u, (uint32_t)bias},
                                      tok, 256, d_bounds, st, phase);
  else
    return partition_op_impl<8, K, V>(ws, in, out, vin, vout, n, BiasedDigit64{bias, (uint32_t)shift, 255u}, tok,
                                      256, d_bounds, st, phase);
}

// min and max of the keys into d_mm[0], d_mm[1] (d_mm[0] starts at ~0, d_mm[1]
// at 0: k_minmax_init)
template <typename K>
__global__ void k_minmax_init(K* mm) {
  mm[0] = ~(K)0;
  mm[1] = 0;
}
template <typename K>
__global__ __launch_bounds__(256) void k_minmax(const K* __restrict__ keys, uint64_t n, K* __restrict__ mm) {
  K lo = ~(K)0, hi = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const K x = load_stream(&keys[i]);
    lo = x < lo ? x : lo;
    hi = x > hi ? x : hi;
  }
  for (int o = 32; o > 0; o >>= 1) {
    const K a = __shfl_xor(lo, o), b = __shfl_xor(hi, o);
    lo = a < lo ? a : lo;
    hi = b > hi ? b : hi;
  }
  if ((threadIdx.x & (kWave - 1)) == 0) {
    atomicMin(&mm[0], lo);
    atomicMax(&mm[1], hi);
  }
}
template <typename K>
hipError_t minmax_any(Workspace& ws, const K* keys, size_t n, K* d_mm, hipStream_t st) {
  hipLaunchKernelGGL(k_minmax_init<K>, dim3(1), dim3(1), 0, st, d_mm);
  LS_TRY(hipGetLastError());
  if (n == 0) return hipSuccess;
  ScopedTimer tm("minmax", st, n);
  const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, (uint64_t)std::max(1, ws.num_cus) * 8);
  hipLaunchKernelGGL(k_minmax<K>, dim3((uint32_t)blocks), dim3(256), 0, st, keys, (uint64_t)n, d_mm);
  return hipGetLastError();
}
}  // namespace

hipError_t partition_lut_u32(Workspace& ws, const uint32_t* in, uint32_t* out, size_t n, const uint8_t* d_lut,
                             int lut_shift, int nbuckets, uint32_t* d_bounds, hipStream_t st, int phase) {
  return partition_lut_any<uint32_t, NoValue>(ws, in, out, nullptr, nullptr, n, d_lut, lut_shift, nbuckets, d_bounds,
                                              st, phase);
}

hipError_t partition_lut_planar_u32(Workspace& ws, const uint32_t* in, uint16_t* o16, uint8_t* o8, size_t n,
                                   const uint8_t* d_lut, int lut_shift, int nbuckets, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (n > 0xffffffffull || !in || !o16 || !o8 || lut_shift != 24 || nbuckets != 256 || !d_lut) return hipErrorInvalidValue;
  const Workspace::PartToken tok{in, nullptr, n, d_lut, lut_shift, nbuckets, 0, st, true};
  // (out: unused -- the planes are written; the scatter follows partition_lut_u32's count call)
  return partition_op_impl<8, uint32_t, NoValue>(ws, in, reinterpret_cast<uint32_t*>(o16), nullptr, nullptr, n,
                                                 LutDigit{d_lut, (uint32_t)lut_shift, 255u, nullptr}, tok, nbuckets,
                                                 nullptr, st, kPartScatter, o16, o8);
}

hipError_t partition_lut_pairs_u64_u32(Workspace& ws, const uint64_t* kin, const uint32_t* vin, uint64_t* kout,
                                       uint32_t* vout, size_t n, const uint8_t* d_lut, int lut_shift, int nbuckets,
                                       uint32_t* d_bounds, hipStream_t st, int phase) {
  return partition_lut_any<uint64_t, uint32_t>(ws, kin, kout, vin, vout, n, d_lut, lut_shift, nbuckets, d_bounds, st,
                                               phase);
}

hipError_t partition_range_u32(Workspace& ws, const uint32_t* in, uint32_t* out, size_t n, uint32_t bias, int shift,
                               uint32_t* d_bounds, hipStream_t st, int phase) {
  return partition_range_any<uint32_t, NoValue>(ws, in, out, nullptr, nullptr, n, bias, shift, d_bounds, st, phase);
}

hipError_t partition_range_pairs_u64_u32(Workspace& ws, const uint64_t* kin, const uint32_t* vin, uint64_t* kout,
                                         uint32_t* vout, size_t n, uint64_t bias, int shift, uint32_t* d_bounds,
                                         hipStream_t st, int phase) {
  return partition_range_any<uint64_t, uint32_t>(ws, kin, kout, vin, vout, n, bias, shift, d_bounds, st, phase);
}

hipError_t minmax_u32(Workspace& ws, const uint32_t* keys, size_t n, uint32_t* d_mm, hipStream_t st) {
  return minmax_any<uint32_t>(ws, keys, n, d_mm, st);
}

hipError_t minmax_u64(Workspace& ws, const uint64_t* keys, size_t n, uint64_t* d_mm, hipStream_t st) {
  return minmax_any<uint64_t>(ws, keys, n, d_mm, st);
}

hipError_t segment_copy_dev_u32(const uint32_t* src, uint32_t* dst, const uint64_t* d_tab, size_t nseg,
                                uint64_t maxlen, uint64_t total, hipStream_t st) {
  if (nseg == 0 || maxlen == 0) return hipSuccess;
  if (nseg > 65535) return hipErrorInvalidValue;
  ScopedTimer tm("segcopy", st, total);
  const uint64_t px = (maxlen + kSegPiece - 1) / kSegPiece;
  if (px > 0x7fffffffull) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_segment_copy2d, dim3((uint32_t)px, (uint32_t)nseg), dim3(256), 0, st, src, dst, d_tab,
                     (uint32_t)nseg);
  return hipGetLastError();
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

hipError_t delta_maxgap_u32(const uint32_t* keys, size_t n, uint32_t* d_maxgap, hipStream_t st) {
  LS_TRY(hipMemsetAsync(d_maxgap, 0, sizeof(uint32_t), st));
  if (n < 2) return hipSuccess;
  const uint64_t ng = (n + kDeltaGroup - 1) / kDeltaGroup;
  const uint32_t blocks = (uint32_t)std::min<uint64_t>((ng + kDeltaChunk - 1) / kDeltaChunk, 1024);
  hipLaunchKernelGGL(k_delta_maxgap, dim3(blocks), dim3(256), 0, st, keys, (uint64_t)n, d_maxgap);
  return hipGetLastError();
}

hipError_t delta_pack_u32(const uint32_t* keys, size_t n, const uint32_t* d_maxgap, uint32_t* out, hipStream_t st) {
  if (n == 0) return hipSuccess;
  const uint64_t ng = (n + kDeltaGroup - 1) / kDeltaGroup;
  const uint32_t blocks = (uint32_t)std::min<uint64_t>((ng + kDeltaChunk - 1) / kDeltaChunk, 8192);
  hipLaunchKernelGGL(k_delta_pack, dim3(blocks), dim3(256), 0, st, keys, (uint64_t)n, d_maxgap, out);
  return hipGetLastError();
}

hipError_t delta_unpack_u32(const uint32_t* in, size_t n, uint32_t w, uint32_t* keys, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (w > 32) return hipErrorInvalidValue;
  const uint64_t ng = (n + kDeltaGroup - 1) / kDeltaGroup;
  const uint32_t blocks = (uint32_t)std::min<uint64_t>((ng + kDeltaChunk - 1) / kDeltaChunk, 8192);
  hipLaunchKernelGGL(k_delta_unpack, dim3(blocks), dim3(256), 0, st, in, (uint64_t)n, w, keys);
  return hipGetLastError();
}

hipError_t merge_u32(const uint32_t* a, size_t na, const uint32_t* b, size_t nb, uint32_t* out, hipStream_t st) {
  const uint64_t total = (uint64_t)na + nb;
  if (total == 0) return hipSuccess;
  const uint64_t tiles = (total + 2047) / 2048;
  if (tiles > 0x7fffffffull) return hipErrorInvalidValue;
  // split points in stream-ordered memory: no workspace, so merges on one
  // stream never wait for sorts on another
  uint64_t* splits = nullptr;
  LS_TRY(hipMallocAsync(reinterpret_cast<void**>(&splits), (tiles + 1) * sizeof(uint64_t), st));
  ScopedTimer tm("merge", st, total);
  hipLaunchKernelGGL(k_merge_splits, dim3((uint32_t)((tiles + 1 + 255) / 256)), dim3(256), 0, st, a, (uint64_t)na, b,
                     (uint64_t)nb, 2048u, tiles, splits);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_merge_u32, dim3((uint32_t)tiles), dim3(256), 0, st, a, (uint64_t)na, b, (uint64_t)nb,
                       (const uint64_t*)splits, out);
    e = hipGetLastError();
  }
  const hipError_t f = hipFreeAsync(splits, st);
  return e != hipSuccess ? e : f;
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
