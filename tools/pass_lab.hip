// Pass-kernel lab (not part of libsort): times variants of the 4-bit tile pass
// on identical inputs (pass 0 of a 2^lg PCG key array, counts and column scan
// from the library's own host helpers), checks each variant bit-exact against
// the library kernel (keys out and the fused next-pass counts), and breaks a
// block's lifetime into phases with s_memtime stamps.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/pass_lab tools/pass_lab.hip
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

// digit starts of the column scan (the lab's kernels add them like k_tile_pass)
__device__ const uint32_t* g_lab_D;

__device__ __forceinline__ uint32_t mbcnt64(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// ---------------------------------------------------------------------------
// Instrumented copy of k_tile_pass<4, 256, 16, u32, NoValue, FUSE=true>:
// stamps[t][8] = s_memtime at the phase boundaries of wave 0.
constexpr int kStamps = 8;
__device__ __forceinline__ uint64_t stamp() { return __builtin_amdgcn_s_memtime(); }

template <int BITS, int BLOCK, int ITEMS>
__global__ __launch_bounds__(BLOCK) void k_pass_prof(const uint32_t* __restrict__ kin, uint32_t* __restrict__ kout,
                                                     uint32_t n, RadixDigit op, RadixDigit op_next,
                                                     uint32_t* __restrict__ C, const uint32_t* __restrict__ B,
                                                     uint32_t* __restrict__ C_next, uint64_t* __restrict__ stamps) {
  using K = uint32_t;
  constexpr int RADIX = 1 << BITS;
  constexpr int WAVES = BLOCK / kWave;
  constexpr int TILE = BLOCK * ITEMS;
  constexpr int WSPAN = ITEMS * kWave;
  constexpr int CH = kColRowsPerLane * (256 / RADIX);
  __shared__ K s_keys[TILE];
  __shared__ uint32_t s_whist[WAVES][RADIX];
  __shared__ uint32_t s_outbase[RADIX];
  __shared__ uint32_t s_tfirst[RADIX];
  __shared__ uint32_t s_next[RADIX * 2 * RADIX];
  __shared__ uint32_t s_wsum[WAVES];
  uint64_t ts[kStamps];
  ts[0] = stamp();
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int w = tid / kWave;
  const uint32_t t = blockIdx.x;
  for (int d = lane; d < RADIX; d += kWave) s_whist[w][d] = 0u;
  for (int i = tid; i < RADIX * 2 * RADIX; i += BLOCK) s_next[i] = 0u;
  uint32_t gofs = 0;
  if (tid < RADIX) {
    gofs = C[(size_t)t * RADIX + tid] + B[(size_t)(t / CH) * RADIX + tid] + g_lab_D[tid];
    C[(size_t)t * RADIX + tid] = 0u;
  }
  const uint64_t tile_base = (uint64_t)t * TILE;
  const uint32_t valid = TILE;
  const bool full = true;
  const uint32_t wbase = w * WSPAN;
  K k[ITEMS];
  uint32_t rk[ITEMS];
  const K* kp = kin + tile_base + wbase + lane;
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) k[j] = kp[j * kWave];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  ts[1] = stamp();
  rank_items<BITS, ITEMS>(k, rk, s_whist[w], full, valid, wbase, lane, op);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  ts[2] = stamp();
  __syncthreads();
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
    s_outbase[tid] = gofs - excl;
    s_tfirst[tid] = gofs / TILE;
  }
  __syncthreads();
  ts[3] = stamp();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t pos = s_whist[w][op(k[j])] + rk[j];
    s_keys[pos] = k[j];
  }
  __syncthreads();
  ts[4] = stamp();
  for (uint32_t i = tid; i < valid; i += BLOCK) {
    const K kk = s_keys[i];
    const uint32_t d = op(kk);
    const uint32_t o = s_outbase[d] + i;
    kout[o] = kk;
    const uint32_t slot = o / TILE - s_tfirst[d];
    atomicAdd(&s_next[(d * 2 + slot) * RADIX + op_next(kk)], 1u);
  }
  ts[5] = stamp();
  __syncthreads();
  for (int e = tid; e < RADIX * 2 * RADIX; e += BLOCK) {
    const uint32_t c = s_next[e];
    if (c) {
      const uint32_t d = e / (2 * RADIX), slot = (e / RADIX) & 1u, dn = e % RADIX;
      atomicAdd(&C_next[(size_t)(s_tfirst[d] + slot) * RADIX + dn], c);
    }
  }
  ts[6] = stamp();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  ts[7] = stamp();
  if (tid == 0) {
#pragma unroll
    for (int i = 0; i < kStamps; ++i) stamps[(size_t)t * kStamps + i] = ts[i];
  }
}

// ---------------------------------------------------------------------------
// Candidate pass kernel (4-bit, fused next-pass counts, full tiles only here):
//  * rank without the valid-lane predicate, sign-extended bit extract feeding
//    both the ballot and the mismatch OR, and every peer writing base+cnt;
//  * CHAINS independent per-wave counter rows ("virtual waves": items split in
//    CHAINS contiguous groups, ranked in (wave, chain) order) so the LDS
//    read->write chains overlap;
//  * unrolled store phase: one ds_read_b64 per key gives (run base, local
//    position where the run crosses into the next destination tile).
template <int CHAINS>
__device__ __forceinline__ void rank_full4(const uint32_t (&k)[16], uint32_t (&rk)[16], uint32_t (*rows)[16],
                                           RadixDigit op) {
  constexpr int PER = 16 / CHAINS;
#pragma unroll
  for (int jj = 0; jj < PER; ++jj) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      const int j = c * PER + jj;
      const uint32_t d = op(k[j]);
      uint32_t mis_lo = 0u, mis_hi = 0u;
#pragma unroll
      for (int bit = 0; bit < 4; ++bit) {
        const uint32_t X = (uint32_t)__builtin_amdgcn_sbfe((int)d, bit, 1);
        const uint64_t m = __ballot(X != 0u);
        mis_lo |= (uint32_t)m ^ X;
        mis_hi |= (uint32_t)(m >> 32) ^ X;
      }
      const uint64_t peers = ~(((uint64_t)mis_hi << 32) | mis_lo);
      const uint32_t below = mbcnt64(peers);
      const uint32_t cnt = (uint32_t)__popcll(peers);
      const uint32_t base = rows[c][d];
      rk[j] = base + below;
      rows[c][d] = base + cnt;  // every peer writes the same value
    }
  }
}

template <int CHAINS, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_pass_x(
    const uint32_t* __restrict__ kin, uint32_t* __restrict__ kout, RadixDigit op, RadixDigit op_next,
    uint32_t* __restrict__ C, const uint32_t* __restrict__ B, uint32_t* __restrict__ C_next) {
  constexpr int BITS = 4, BLOCK = 256, ITEMS = 16;
  constexpr int RADIX = 1 << BITS;
  constexpr int WAVES = BLOCK / kWave;
  constexpr int VW = WAVES * CHAINS;
  constexpr int TILE = BLOCK * ITEMS;
  constexpr int WSPAN = ITEMS * kWave;
  constexpr int CH = kColRowsPerLane * (256 / RADIX);
  __shared__ uint32_t s_keys[TILE];
  __shared__ uint32_t s_whist[VW][RADIX];
  __shared__ uint2 s_ob[RADIX];  // (run base, split position)
  __shared__ uint32_t s_tfirst[RADIX];
  __shared__ uint32_t s_next[RADIX * 2 * RADIX];
  __shared__ uint32_t s_wsum[WAVES];
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int w = tid / kWave;
  const uint32_t t = blockIdx.x;
  for (int i = lane; i < CHAINS * RADIX; i += kWave) (&s_whist[w * CHAINS][0])[i] = 0u;
  for (int i = tid; i < RADIX * 2 * RADIX; i += BLOCK) s_next[i] = 0u;
  uint32_t gofs = 0;
  if (tid < RADIX) {
    gofs = C[(size_t)t * RADIX + tid] + B[(size_t)(t / CH) * RADIX + tid] + g_lab_D[tid];
    C[(size_t)t * RADIX + tid] = 0u;
  }
  const uint64_t tile_base = (uint64_t)t * TILE;
  uint32_t k[ITEMS], rk[ITEMS];
  const uint32_t* kp = kin + tile_base + w * WSPAN + lane;
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) k[j] = kp[j * kWave];
  rank_full4<CHAINS>(k, rk, &s_whist[w * CHAINS], op);
  __syncthreads();
  uint32_t cnt_d = 0;
  if (tid < RADIX) {
#pragma unroll
    for (int i = 0; i < VW; ++i) cnt_d += s_whist[i][tid];
  }
  uint32_t tile_total;
  const uint32_t excl = block_exclusive_scan<BLOCK>(cnt_d, s_wsum, tile_total);
  if (tid < RADIX) {
    uint32_t run = excl;
#pragma unroll
    for (int i = 0; i < VW; ++i) {
      const uint32_t c = s_whist[i][tid];
      s_whist[i][tid] = run;
      run += c;
    }
    const uint32_t ob = gofs - excl, tf = gofs / TILE;
    s_ob[tid] = make_uint2(ob, (tf + 1) * TILE - ob);
    s_tfirst[tid] = tf;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) s_keys[s_whist[w * CHAINS + j / (ITEMS / CHAINS)][op(k[j])] + rk[j]] = k[j];
  __syncthreads();
  uint32_t kk[ITEMS];
  uint2 ob[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) kk[j] = s_keys[tid + j * BLOCK];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) ob[j] = s_ob[op(kk[j])];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) kout[ob[j].x + tid + j * BLOCK] = kk[j];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t slot = (uint32_t)(tid + j * BLOCK) >= ob[j].y ? 1u : 0u;
    atomicAdd(&s_next[(op(kk[j]) * 2 + slot) * RADIX + op_next(kk[j])], 1u);
  }
  __syncthreads();
  for (int e = tid; e < RADIX * 2 * RADIX; e += BLOCK) {
    const uint32_t c = s_next[e];
    if (c) {
      const uint32_t d = e / (2 * RADIX), slot = (e / RADIX) & 1u, dn = e % RADIX;
      atomicAdd(&C_next[(size_t)(s_tfirst[d] + slot) * RADIX + dn], c);
    }
  }
}

// Persistent variant: grid = CUs x blocks-per-CU, block b walks tiles
// b, b+G, b+2G...; the keys (and run offsets) of the next tile are loaded into
// registers while the current tile is ranked, scattered and stored.
template <int CHAINS, int SPLIT>
__global__ __launch_bounds__(256) void k_pass_y(const uint32_t* __restrict__ kin, uint32_t* __restrict__ kout,
                                                RadixDigit op, RadixDigit op_next, uint32_t* __restrict__ C,
                                                const uint32_t* __restrict__ B, uint32_t* __restrict__ C_next,
                                                uint32_t tiles) {
  constexpr int BITS = 4, BLOCK = 256, ITEMS = 16;
  constexpr int RADIX = 1 << BITS;
  constexpr int WAVES = BLOCK / kWave;
  constexpr int VW = WAVES * CHAINS;
  constexpr int TILE = BLOCK * ITEMS;
  constexpr int WSPAN = ITEMS * kWave;
  constexpr int CH = kColRowsPerLane * (256 / RADIX);
  constexpr int SPER = ITEMS / SPLIT;  // store-phase items per sub-loop
  __shared__ uint32_t s_keys[TILE];
  __shared__ uint32_t s_whist[VW][RADIX];
  __shared__ uint2 s_ob[RADIX];
  __shared__ uint32_t s_tfirst[RADIX];
  __shared__ uint32_t s_next[RADIX * 2 * RADIX];
  __shared__ uint32_t s_wsum[WAVES];
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int w = tid / kWave;
  uint32_t t = blockIdx.x;
  uint32_t kn[ITEMS];
  uint32_t gn = 0;
  if (t < tiles) {
    const uint32_t* kp = kin + (uint64_t)t * TILE + w * WSPAN + lane;
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) kn[j] = kp[j * kWave];
    if (tid < RADIX) gn = C[(size_t)t * RADIX + tid] + B[(size_t)(t / CH) * RADIX + tid];
  }
  while (t < tiles) {
    uint32_t k[ITEMS], rk[ITEMS];
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) k[j] = kn[j];
    const uint32_t gofs = gn;
    if (tid < RADIX) C[(size_t)t * RADIX + tid] = 0u;
    const uint32_t tn = t + gridDim.x;
    if (tn < tiles) {
      const uint32_t* kp = kin + (uint64_t)tn * TILE + w * WSPAN + lane;
#pragma unroll
      for (int j = 0; j < ITEMS; ++j) kn[j] = kp[j * kWave];
      if (tid < RADIX) gn = C[(size_t)tn * RADIX + tid] + B[(size_t)(tn / CH) * RADIX + tid];
    }
    for (int i = lane; i < CHAINS * RADIX; i += kWave) (&s_whist[w * CHAINS][0])[i] = 0u;
    for (int i = tid; i < RADIX * 2 * RADIX; i += BLOCK) s_next[i] = 0u;
    rank_full4<CHAINS>(k, rk, &s_whist[w * CHAINS], op);
    __syncthreads();
    uint32_t cnt_d = 0;
    if (tid < RADIX) {
#pragma unroll
      for (int i = 0; i < VW; ++i) cnt_d += s_whist[i][tid];
    }
    uint32_t tile_total;
    const uint32_t excl = block_exclusive_scan<BLOCK>(cnt_d, s_wsum, tile_total);
    if (tid < RADIX) {
      uint32_t run = excl;
#pragma unroll
      for (int i = 0; i < VW; ++i) {
        const uint32_t c = s_whist[i][tid];
        s_whist[i][tid] = run;
        run += c;
      }
      const uint32_t ob = gofs - excl, tf = gofs / TILE;
      s_ob[tid] = make_uint2(ob, (tf + 1) * TILE - ob);
      s_tfirst[tid] = tf;
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) s_keys[s_whist[w * CHAINS + j / (ITEMS / CHAINS)][op(k[j])] + rk[j]] = k[j];
    __syncthreads();
#pragma unroll
    for (int h = 0; h < SPLIT; ++h) {
      uint32_t kk[SPER];
      uint2 ob[SPER];
#pragma unroll
      for (int j = 0; j < SPER; ++j) kk[j] = s_keys[tid + (h * SPER + j) * BLOCK];
#pragma unroll
      for (int j = 0; j < SPER; ++j) ob[j] = s_ob[op(kk[j])];
#pragma unroll
      for (int j = 0; j < SPER; ++j) kout[ob[j].x + tid + (h * SPER + j) * BLOCK] = kk[j];
#pragma unroll
      for (int j = 0; j < SPER; ++j) {
        const uint32_t slot = (uint32_t)(tid + (h * SPER + j) * BLOCK) >= ob[j].y ? 1u : 0u;
        atomicAdd(&s_next[(op(kk[j]) * 2 + slot) * RADIX + op_next(kk[j])], 1u);
      }
    }
    __syncthreads();
    for (int e = tid; e < RADIX * 2 * RADIX; e += BLOCK) {
      const uint32_t c = s_next[e];
      if (c) {
        const uint32_t d = e / (2 * RADIX), slot = (e / RADIX) & 1u, dn = e % RADIX;
        atomicAdd(&C_next[(size_t)(s_tfirst[d] + slot) * RADIX + dn], c);
      }
    }
    __syncthreads();
    t = tn;
  }
}

// Lean variant (full tiles): one v_bfe per digit, ballots straight from the
// sign-extended bit (inline v_cmp so the compiler cannot re-derive it),
// v_bitop3 mismatch accumulation, block phase in wave 0 (16-lane scan),
// next-pass count table laid out [slot][dn][d] so its index is one 8-bit
// field of the key.
template <bool ASM>
__device__ __forceinline__ uint64_t ballot_nz_lab(uint32_t x) {
  if constexpr (ASM) {
    uint64_t m;
    asm("v_cmp_ne_u32_e64 %0, 0, %1" : "=s"(m) : "v"(x));
    return m;
  } else {
    return __ballot(x != 0u);
  }
}

template <int CHAINS, bool LASTW, bool ASM>
__device__ __forceinline__ void rank_lean4(const uint32_t (&k)[16], uint32_t (&rk)[16], uint32_t* rows,
                                           uint32_t shift, uint32_t nb, uint32_t* dummy) {
  constexpr int PER = 16 / CHAINS;
#pragma unroll
  for (int jj = 0; jj < PER; ++jj) {
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) {
      const int j = c * PER + jj;
      const uint32_t d = __builtin_amdgcn_ubfe(k[j], shift, nb);
      uint32_t lo = 0u, hi = 0u;
#pragma unroll
      for (int bit = 0; bit < 3; ++bit) {
        const uint32_t X = (uint32_t)__builtin_amdgcn_sbfe(d, bit, 1);
        const uint64_t m = ballot_nz_lab<ASM>(X);
        lo = __builtin_amdgcn_bitop3_b32(X, lo, (uint32_t)m, 0xDE);
        hi = __builtin_amdgcn_bitop3_b32(X, hi, (uint32_t)(m >> 32), 0xDE);
      }
      const uint32_t X = (uint32_t)__builtin_amdgcn_sbfe(d, 3, 1);
      const uint64_t m = ballot_nz_lab<ASM>(X);
      const uint32_t plo = __builtin_amdgcn_bitop3_b32(X, lo, (uint32_t)m, 0x21);  // ~((X^m)|lo)
      const uint32_t phi = __builtin_amdgcn_bitop3_b32(X, hi, (uint32_t)(m >> 32), 0x21);
      const uint32_t below = __builtin_amdgcn_mbcnt_hi(phi, __builtin_amdgcn_mbcnt_lo(plo, 0u));
      const uint32_t cnt = __builtin_popcount(plo) + __builtin_popcount(phi);
      uint32_t* row = rows + c * 16;
      const uint32_t base = row[d];
      rk[j] = base + below;
      if constexpr (LASTW) {
        uint32_t* dst = (below + 1u == cnt) ? &row[d] : dummy;
        *dst = base + cnt;
      } else {
        row[d] = base + cnt;
      }
    }
  }
}

// Tile handled by block b.  XCD: blocks are dealt round-robin over the 8
// XCDs, so give XCD x = b % 8 the contiguous tile range [start_x, start_x +
// count_x) -- neighbouring tiles, whose digit runs share the boundary lines,
// then write through the same L2.  A bijection for any grid size.
template <bool XCD>
__device__ __forceinline__ uint32_t tile_of_block() {
  if constexpr (!XCD) {
    return blockIdx.x;
  } else {
    const uint32_t g = gridDim.x, q = g >> 3, r = g & 7u, x = blockIdx.x & 7u, i = blockIdx.x >> 3;
    return x * q + min(x, r) + i;
  }
}

// ABL (timing ablations, output wrong): 1 = write the sorted tile back to its
// own tile (contiguous, copy-like addresses), 2 = no global key stores,
// 3 = 2 + no next-pass count atomics/flush, 4 = 3 + no ballot rank
// (identity positions), 5 = 4 + no LDS scatter/read-back (keys go straight
// from the load registers to a dummy-conditioned store), 6 = full kernel but
// no global flush of the next-pass counts, 7 = full kernel without counting.
template <int CHAINS, bool LASTW, int SPLIT, bool ASM = true, int BLOCK = 256, bool XCD = false, int ABL = 0,
          int MINB = 1, bool PACK = false>
__global__ __launch_bounds__(BLOCK, MINB) void k_pass_z(const uint32_t* __restrict__ kin, uint32_t* __restrict__ kout,
                                                uint32_t shift, uint32_t nb, uint32_t* __restrict__ C,
                                                const uint32_t* __restrict__ B, uint32_t* __restrict__ C_next) {
  constexpr int ITEMS = 16, RADIX = 16;
  constexpr int WAVES = BLOCK / kWave;
  constexpr int VW = WAVES * CHAINS;
  constexpr int TILE = BLOCK * ITEMS;
  constexpr int WSPAN = ITEMS * kWave;
  constexpr int CH = kColRowsPerLane * (256 / RADIX);
  constexpr int SPER = ITEMS / SPLIT;
  __shared__ uint32_t s_keys[TILE];
  __shared__ uint32_t s_whist[VW * RADIX];
  __shared__ uint32_t s_dummy[BLOCK];
  __shared__ uint2 s_ob[RADIX];
  __shared__ uint32_t s_tfirst[RADIX];
  __shared__ uint32_t s_next[2 * RADIX * RADIX];  // [slot][d][dn]
  const int tid = threadIdx.x;
  const int lane = tid & (kWave - 1);
  const int w = tid / kWave;
  const uint32_t t = tile_of_block<XCD>();
  if (lane < CHAINS * RADIX) s_whist[w * CHAINS * RADIX + lane] = 0u;
#pragma unroll
  for (int q = 0; q < 2 * RADIX * RADIX / BLOCK; ++q) s_next[tid + q * BLOCK] = 0u;
  uint32_t gofs = 0;
  if (tid < RADIX) {
    gofs = C[(size_t)t * RADIX + tid] + B[(size_t)(t / CH) * RADIX + tid] + g_lab_D[tid];
    C[(size_t)t * RADIX + tid] = 0u;
  }
  uint32_t k[ITEMS], rk[ITEMS];
  uint32_t rkp[ITEMS / 2];  // PACK: two 16-bit ranks per register across the block phase
  const uint32_t* kp = kin + (uint64_t)t * TILE + w * WSPAN + lane;
  // ABL 8: nontemporal key stores, 9: nontemporal key loads, 10: both (exact kernels)
  constexpr bool NTS = ABL == 8 || ABL == 10, NTL = ABL == 9 || ABL == 10;
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) k[j] = NTL ? __builtin_nontemporal_load(&kp[j * kWave]) : kp[j * kWave];
  if constexpr (ABL >= 4 && ABL < 6) {
#pragma unroll
    for (int j = 0; j < ITEMS; ++j) rk[j] = w * WSPAN + j * kWave + lane;
  } else {
    rank_lean4<CHAINS, LASTW, ASM>(k, rk, &s_whist[w * CHAINS * RADIX], shift, nb, &s_dummy[tid]);
  }
  if constexpr (PACK) {
#pragma unroll
    for (int j = 0; j < ITEMS / 2; ++j) rkp[j] = rk[2 * j] | (rk[2 * j + 1] << 16);
  }
  __syncthreads();
  if (w == 0) {
    const uint32_t d = lane & (RADIX - 1);
    uint32_t v[VW], tot = 0;
#pragma unroll
    for (int r = 0; r < VW; ++r) { v[r] = s_whist[r * RADIX + d]; tot += v[r]; }
    uint32_t x = tot;
#pragma unroll
    for (int o = 1; o < RADIX; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, RADIX);
      if ((int)d >= o) x += y;
    }
    const uint32_t excl = x - tot;
    if (lane < RADIX) {
      uint32_t run = excl;
#pragma unroll
      for (int r = 0; r < VW; ++r) { s_whist[r * RADIX + d] = run; run += v[r]; }
      const uint32_t ob = gofs - excl, tf = gofs / TILE;
      s_ob[d] = make_uint2(ob, (tf + 1) * TILE - ob);
      s_tfirst[d] = tf;
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const uint32_t d = __builtin_amdgcn_ubfe(k[j], shift, nb);
    if constexpr (ABL == 5) {
      if (k[j] == 0x9e3779b9u) kout[t] = rk[j];
    } else if constexpr (ABL == 4) {
      s_keys[rk[j]] = k[j] + d;
    } else {
      const uint32_t r = PACK ? ((j & 1) ? (rkp[j / 2] >> 16) : (rkp[j / 2] & 0xFFFFu)) : rk[j];
      s_keys[s_whist[(w * CHAINS + j / (ITEMS / CHAINS)) * RADIX + d] + r] = k[j];
    }
  }
  __syncthreads();
  if constexpr (ABL != 5)
#pragma unroll
  for (int h = 0; h < SPLIT; ++h) {
    uint32_t kk[SPER];
    uint2 ob[SPER];
#pragma unroll
    for (int j = 0; j < SPER; ++j) kk[j] = s_keys[tid + (h * SPER + j) * BLOCK];
#pragma unroll
    for (int j = 0; j < SPER; ++j) ob[j] = s_ob[__builtin_amdgcn_ubfe(kk[j], shift, 4)];
#pragma unroll
    for (int j = 0; j < SPER; ++j) {
      if constexpr (NTS) __builtin_nontemporal_store(kk[j], &kout[ob[j].x + tid + (h * SPER + j) * BLOCK]);
      else if constexpr (ABL == 0 || ABL >= 6) kout[ob[j].x + tid + (h * SPER + j) * BLOCK] = kk[j];
      if constexpr (ABL == 1) kout[(size_t)t * TILE + tid + (h * SPER + j) * BLOCK] = kk[j] + ob[j].x;
      if constexpr (ABL >= 2 && ABL < 6) if (kk[j] == 0x9e3779b9u && ob[j].x == 7u) kout[t] = 1u;
    }
#pragma unroll
    for (int j = 0; j < SPER; ++j) {
      if constexpr (ABL < 3 || ABL == 6 || ABL >= 8) {
        const uint32_t slot = (uint32_t)(tid + (h * SPER + j) * BLOCK) >= ob[j].y ? 256u : 0u;
        const uint32_t dd = __builtin_amdgcn_ubfe(kk[j], shift, 4), dn = __builtin_amdgcn_ubfe(kk[j], shift + 4, 4);
        atomicAdd(&s_next[slot + dd * 16 + dn], 1u);
      }
    }
  }
  __syncthreads();
  if constexpr (ABL < 3 || ABL >= 8)
#pragma unroll
  for (int q = 0; q < 2 * RADIX * RADIX / BLOCK; ++q) {
    const int e = tid + q * BLOCK;
    const uint32_t c = s_next[e];
    if (c) atomicAdd(&C_next[(size_t)(s_tfirst[(e >> 4) & 15] + (uint32_t)(e >> 8)) * RADIX + (e & 15)], c);
  }
}

// ---------------------------------------------------------------------------
struct Lab {
  size_t n;
  uint32_t tiles;
  Workspace ws;
  uint32_t *in, *out, *C0;
  hipStream_t st;
  hipEvent_t e0, e1;
  RadixDigit op{0, 15}, op_next{4, 15};
  size_t cwords;
  std::vector<uint32_t> exp_out, exp_cn;  // host expectations
};

struct Variant {
  const char* name;
  std::function<void()> launch;
  std::vector<float> us;
  bool checked = false, ok = false;
};

void run_once(Lab& L, Variant& v) {
  CK(hipMemcpyAsync(L.ws.tc[0], L.C0, L.cwords * 4, hipMemcpyDeviceToDevice, L.st));
  CK(hipMemsetAsync(L.ws.tc[1], 0, L.cwords * 4, L.st));
  CK(hipMemsetAsync(L.out, 0xff, 4096, L.st));
  CK(hipEventRecord(L.e0, L.st));
  v.launch();
  CK(hipGetLastError());
  CK(hipEventRecord(L.e1, L.st));
  CK(hipEventSynchronize(L.e1));
  float ms;
  CK(hipEventElapsedTime(&ms, L.e0, L.e1));
  v.us.push_back(ms * 1e3f);
}

void check(Lab& L, Variant& v) {
  std::vector<uint32_t> a(L.n), c(L.cwords);
  CK(hipMemcpy(a.data(), L.out, L.n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(c.data(), L.ws.tc[1], L.cwords * 4, hipMemcpyDeviceToHost));
  size_t bad = 0, first = ~(size_t)0, badc = 0;
  for (size_t i = 0; i < L.n; ++i)
    if (a[i] != L.exp_out[i]) { if (!bad) first = i; ++bad; }
  for (size_t i = 0; i < L.cwords; ++i) badc += c[i] != L.exp_cn[i];
  v.checked = true;
  v.ok = bad == 0 && badc == 0;
  if (!v.ok) printf("  %s: %zu key mismatches (first %zu), %zu count mismatches\n", v.name, bad, first, badc);
}

int main(int argc, char** argv) {
  Lab L;
  const int lg = argc > 1 ? atoi(argv[1]) : 28;
  const int rounds = argc > 2 ? atoi(argv[2]) : 15;
  const int block = argc > 3 ? atoi(argv[3]) : 256;
  const uint32_t tile = block * 16;
  L.n = (size_t)1 << lg;
  L.tiles = (uint32_t)((L.n + tile - 1) / tile);
  L.cwords = (size_t)L.tiles * 16;
  CK(hipSetDevice(0));
  L.ws.device = 0;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  L.ws.num_cus = prop.multiProcessorCount;
  CK(hipStreamCreateWithFlags(&L.st, hipStreamNonBlocking));
  CK(hipEventCreate(&L.e0));
  CK(hipEventCreate(&L.e1));
  CK(hipMalloc(&L.in, L.n * 4));
  CK(hipMalloc(&L.out, L.n * 4));
  CK(populate_device(L.in, L.n, 0, L.st));
  CK(tiles_prologue<uint32_t>(L.ws, L.in, L.n, 0, 32, 4, L.st));  // buffers (sized for 4096-key tiles)
  if (block == 512) {
    hipLaunchKernelGGL((k_tile_counts<4, 512, 16, uint32_t>), dim3(L.tiles), dim3(512), 0, L.st, L.in, (uint32_t)L.n,
                       RadixDigit{0, 15}, L.ws.tc[0], L.ws.tc[1], L.tiles * 16u);
    CK(hipGetLastError());
  }
  CK(tiles_colscan<4>(L.ws, L.ws.tc[0], L.tiles, L.st));
  {
    const uint32_t* dptr = tiles_digit_starts(L.ws, L.tiles, 4);
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_lab_D), &dptr, sizeof(dptr)));
  }
  CK(hipMalloc(&L.C0, L.cwords * 4));
  CK(hipMemcpyAsync(L.C0, L.ws.tc[0], L.cwords * 4, hipMemcpyDeviceToDevice, L.st));
  CK(hipStreamSynchronize(L.st));

  // host expectation: stable partition by bits [0,4), counts of bits [4,8) per output tile
  {
    std::vector<uint32_t> h(L.n);
    CK(hipMemcpy(h.data(), L.in, L.n * 4, hipMemcpyDeviceToHost));
    size_t cnt[16] = {0}, pos[16];
    for (size_t i = 0; i < L.n; ++i) cnt[h[i] & 15]++;
    size_t run = 0;
    for (int d = 0; d < 16; ++d) { pos[d] = run; run += cnt[d]; }
    L.exp_out.resize(L.n);
    for (size_t i = 0; i < L.n; ++i) L.exp_out[pos[h[i] & 15]++] = h[i];
    L.exp_cn.assign(L.cwords, 0);
    for (size_t i = 0; i < L.n; ++i) L.exp_cn[(i / tile) * 16 + ((L.exp_out[i] >> 4) & 15)]++;
  }

  const uint32_t* B = L.ws.tb;
  const dim3 grid(L.tiles), blk(256), blk512(512);
  uint64_t* d_st;
  CK(hipMalloc(&d_st, (size_t)L.tiles * kStamps * 8));
  std::vector<Variant> V;
  if (block == 256) {
    V.push_back({"lib fused", [&] {
      hipLaunchKernelGGL((k_tile_pass<4, 256, 16, uint32_t, NoValue, true>), grid, blk, 0, L.st, L.in, L.out,
                         (const NoValue*)nullptr, (NoValue*)nullptr, (uint32_t)L.n, L.op, L.op_next, L.ws.tc[0], B,
                         tiles_digit_starts(L.ws, L.tiles, 4), L.ws.tc[1]);
    }});
    V.push_back({"z c1 s2 xcd", [&] {
      hipLaunchKernelGGL((k_pass_z<1, false, 2, true, 256, true>), grid, blk, 0, L.st, L.in, L.out, 0u, 4u, L.ws.tc[0], B,
                         L.ws.tc[1]);
    }});
    V.push_back({"z c1 s2 xcd pack", [&] {
      hipLaunchKernelGGL((k_pass_z<1, false, 2, true, 256, true, 0, 1, true>), grid, blk, 0, L.st, L.in, L.out, 0u, 4u,
                         L.ws.tc[0], B, L.ws.tc[1]);
    }});
    V.push_back({"z c1 s2 xcd pack minb8", [&] {
      hipLaunchKernelGGL((k_pass_z<1, false, 2, true, 256, true, 0, 8, true>), grid, blk, 0, L.st, L.in, L.out, 0u, 4u,
                         L.ws.tc[0], B, L.ws.tc[1]);
    }});
    V.push_back({"z c1 s2 xcd minb8", [&] {
      hipLaunchKernelGGL((k_pass_z<1, false, 2, true, 256, true, 0, 8, false>), grid, blk, 0, L.st, L.in, L.out, 0u, 4u,
                         L.ws.tc[0], B, L.ws.tc[1]);
    }});
    V.push_back({"z xcd NT stores", [&] {
      hipLaunchKernelGGL((k_pass_z<1, false, 2, true, 256, true, 8>), grid, blk, 0, L.st, L.in, L.out, 0u, 4u, L.ws.tc[0],
                         B, L.ws.tc[1]);
    }});
    V.push_back({"z xcd NT loads", [&] {
      hipLaunchKernelGGL((k_pass_z<1, false, 2, true, 256, true, 9>), grid, blk, 0, L.st, L.in, L.out, 0u, 4u, L.ws.tc[0],
                         B, L.ws.tc[1]);
    }});
    V.push_back({"z xcd NT both", [&] {
      hipLaunchKernelGGL((k_pass_z<1, false, 2, true, 256, true, 10>), grid, blk, 0, L.st, L.in, L.out, 0u, 4u, L.ws.tc[0],
                         B, L.ws.tc[1]);
    }});
    V.push_back({"ABL contiguous stores", [&] {
      hipLaunchKernelGGL((k_pass_z<1, false, 2, true, 256, true, 1>), grid, blk, 0, L.st, L.in, L.out, 0u, 4u, L.ws.tc[0],
                         B, L.ws.tc[1]);
    }});
    V.push_back({"ABL no key stores", [&] {
      hipLaunchKernelGGL((k_pass_z<1, false, 2, true, 256, true, 2>), grid, blk, 0, L.st, L.in, L.out, 0u, 4u, L.ws.tc[0],
                         B, L.ws.tc[1]);
    }});
    V.push_back({"ABL +no counts", [&] {
      hipLaunchKernelGGL((k_pass_z<1, false, 2, true, 256, true, 3>), grid, blk, 0, L.st, L.in, L.out, 0u, 4u, L.ws.tc[0],
                         B, L.ws.tc[1]);
    }});
    V.push_back({"ABL +no rank", [&] {
      hipLaunchKernelGGL((k_pass_z<1, false, 2, true, 256, true, 4>), grid, blk, 0, L.st, L.in, L.out, 0u, 4u, L.ws.tc[0],
                         B, L.ws.tc[1]);
    }});
    V.push_back({"ABL stores, no flush", [&] {
      hipLaunchKernelGGL((k_pass_z<1, false, 2, true, 256, true, 6>), grid, blk, 0, L.st, L.in, L.out, 0u, 4u, L.ws.tc[0],
                         B, L.ws.tc[1]);
    }});
    V.push_back({"ABL stores, no counting", [&] {
      hipLaunchKernelGGL((k_pass_z<1, false, 2, true, 256, true, 7>), grid, blk, 0, L.st, L.in, L.out, 0u, 4u, L.ws.tc[0],
                         B, L.ws.tc[1]);
    }});
    V.push_back({"ABL +no lds tile", [&] {
      hipLaunchKernelGGL((k_pass_z<1, false, 2, true, 256, true, 5>), grid, blk, 0, L.st, L.in, L.out, 0u, 4u, L.ws.tc[0],
                         B, L.ws.tc[1]);
    }});
  } else {
    V.push_back({"z512 c1 s2", [&] {
      hipLaunchKernelGGL((k_pass_z<1, false, 2, true, 512, false>), grid, blk512, 0, L.st, L.in, L.out, 0u, 4u, L.ws.tc[0],
                         B, L.ws.tc[1]);
    }});
    V.push_back({"z512 c1 s2 xcd", [&] {
      hipLaunchKernelGGL((k_pass_z<1, false, 2, true, 512, true>), grid, blk512, 0, L.st, L.in, L.out, 0u, 4u, L.ws.tc[0],
                         B, L.ws.tc[1]);
    }});
    V.push_back({"z512 c2 s2 xcd", [&] {
      hipLaunchKernelGGL((k_pass_z<2, false, 2, true, 512, true>), grid, blk512, 0, L.st, L.in, L.out, 0u, 4u, L.ws.tc[0],
                         B, L.ws.tc[1]);
    }});
    V.push_back({"z512 c1 s4 xcd", [&] {
      hipLaunchKernelGGL((k_pass_z<1, false, 4, true, 512, true>), grid, blk512, 0, L.st, L.in, L.out, 0u, 4u, L.ws.tc[0],
                         B, L.ws.tc[1]);
    }});
  }
  for (int bpc : std::vector<int>{}) {
    static char names[16][48];
    static int ni = 0;
    snprintf(names[ni], 48, "y chains2 split1 bpc%d", bpc);
    V.push_back({names[ni++], [&, bpc] {
      hipLaunchKernelGGL((k_pass_y<2, 1>), dim3(L.ws.num_cus * bpc), blk, 0, L.st, L.in, L.out, L.op, L.op_next,
                         L.ws.tc[0], B, L.ws.tc[1], L.tiles);
    }});
    snprintf(names[ni], 48, "y chains2 split2 bpc%d", bpc);
    V.push_back({names[ni++], [&, bpc] {
      hipLaunchKernelGGL((k_pass_y<2, 2>), dim3(L.ws.num_cus * bpc), blk, 0, L.st, L.in, L.out, L.op, L.op_next,
                         L.ws.tc[0], B, L.ws.tc[1], L.tiles);
    }});
  }
  Variant prof{"instrumented lib fused", [&] {
    hipLaunchKernelGGL((k_pass_prof<4, 256, 16>), grid, blk, 0, L.st, L.in, L.out, (uint32_t)L.n, L.op, L.op_next,
                       L.ws.tc[0], B, L.ws.tc[1], d_st);
  }};

  // warm-up (clocks), correctness, then interleaved timing rounds
  for (int r = 0; r < 20; ++r) run_once(L, V[0]);
  printf("2^%d keys, %u-key tiles, %u tiles\n", lg, tile, L.tiles);
  for (auto& v : V) {
    v.us.clear();
    run_once(L, v);
    if (std::string(v.name).find("unfused") == std::string::npos && std::string(v.name).find("ABL") != 0)
      check(L, v);
    v.us.clear();
  }
  for (int r = 0; r < rounds; ++r)
    for (auto& v : V) run_once(L, v);
  for (auto& v : V) {
    std::sort(v.us.begin(), v.us.end());
    const float med = v.us[v.us.size() / 2];
    printf("%-26s median %7.1f us  best %7.1f us  %6.0f GB/s  %s\n", v.name, med, v.us[0],
           8.0 * L.n / (med * 1e-6) / 1e9, v.checked ? (v.ok ? "exact" : "MISMATCH") : "(unchecked)");
  }

  if (block != 256) return 0;
  // phase profile of the library kernel
  run_once(L, prof);
  check(L, prof);
  std::vector<uint64_t> h((size_t)L.tiles * kStamps);
  CK(hipMemcpy(h.data(), d_st, h.size() * 8, hipMemcpyDeviceToHost));
  const char* ph[] = {"load wait", "rank", "scan+2 barriers", "lds scatter+barrier", "store loop", "flush atomics",
                      "store drain"};
  double sum[kStamps] = {0}, life = 0;
  for (uint32_t t = 0; t < L.tiles; ++t) {
    const uint64_t* s = &h[(size_t)t * kStamps];
    for (int i = 1; i < kStamps; ++i) sum[i] += (double)(s[i] - s[i - 1]);
    life += (double)(s[kStamps - 1] - s[0]);
  }
  printf("instrumented: %.1f us, %s; phase means (wave 0, s_memtime cycles):\n", prof.us[0], prof.ok ? "exact" : "MISMATCH");
  for (int i = 1; i < kStamps; ++i) printf("  %-22s %8.0f  (%4.1f%%)\n", ph[i - 1], sum[i] / L.tiles, 100.0 * sum[i] / life);
  printf("  lifetime %.0f cycles\n", life / L.tiles);
  return 0;
}
