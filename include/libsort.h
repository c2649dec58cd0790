/*
 * libsort.h -- C ABI of the MI355X-native libsort (gfx950, HIP).
 *
 * Part 1 is the drop-in boundary: the seven entry points of the reference
 * jssmith/gpu-radix-sort `libsort/libsort.h:12-44`, with the SAME names and the
 * SAME C types, so that the unchanged callers link and run against this
 * library:
 *   - Go (cgo, --std=gnu99)     benchmark/pkg/sort/libsort.go:11-77
 *   - Python (ctypes)           faasTest/pylibsort/__init__.py:13-20, sort.py:94-126, data.py:313-317
 *   - C++ harness               localTest/tests.cpp:56,107,117  benchmarks.cpp:44,57,105-109
 * Under C++ every declaration is extern "C"; under plain C (cgo) they are
 * ordinary prototypes, as in the reference header.
 *
 * Part 2 is additive (new names only; Part 1 is unchanged by it): device-
 * resident entry points used by the multi-GPU driver and the benchmark, the
 * north-star aliases gpuFullSort / gpuPartialSort, and timing hooks.
 *
 * Error convention (reference invokers.cu:18-20,30-33,49-57): every `bool`
 * entry point returns false on failure and prints one line to stderr.  Unlike
 * the reference (utils.h:71-78) a HIP error never calls exit(); the message is
 * also available from libsortLastError().
 */
#ifndef LIBSORT_MI355X_LIBSORT_H
#define LIBSORT_MI355X_LIBSORT_H

#include <stdint.h>
#include <stdbool.h>
#include <stddef.h>

#ifdef __cplusplus
#define LIBSORT_API extern "C"
#else
#define LIBSORT_API
#endif

/* ======================= Part 1: reference ABI ============================ */

/* Replaces utils.cu:10-32.  Must be called exactly once per process before the
 * host-pointer entry points; a second call prints a message and returns false.
 * Returns false (loudly) when no HIP device is present. */
LIBSORT_API bool initLibSort(void);

/* Replaces invokers.cu:15-41 (gpuPartial).  Stable partition of h_in[0..len)
 * by the group value (x >> offset) & (2^width - 1), in place; prior order is
 * preserved inside each group.  boundaries (caller-allocated, 2^width uint32)
 * receives, for every group g, the index of its first element, i.e. the
 * number of elements whose group is < g (the exclusive prefix of group counts,
 * the contract checked by localTest/tests.cpp:41-83).  Requires
 * len <= UINT32_MAX, 1 <= width <= 31 and offset + width <= 32.  Odd widths
 * are supported exactly (the reference silently sorts one extra bit, sort.cu:323). */
LIBSORT_API bool gpuPartial(uint32_t* h_in, uint32_t* boundaries, size_t h_in_len,
                            uint32_t offset, uint32_t width);

/* Replaces invokers.cu:45-64 (providedGpu).  Ascending in-place sort of
 * len uint32 keys on a GPU taken from the device pool.  len <= UINT32_MAX. */
LIBSORT_API bool providedGpu(unsigned int* h_in, size_t len);

/* Replaces invokers.cu:68-71 (providedCpu): std::sort on the host. */
LIBSORT_API bool providedCpu(unsigned int* in, size_t len);

/* Replaces utils.cu:65-80: PCG32 (XSH-RR) stream with process-wide state that
 * persists across calls; bit-identical to the reference generator. */
LIBSORT_API void populateInput(uint32_t* arr, size_t nelem);

/* Replaces invokers.cu:73-85: the same calls bracketed by roctx ranges
 * ("gpuPartialProfile" / "providedGpuProfile") for rocprofv3 --marker-trace. */
LIBSORT_API bool gpuPartialProfile(uint32_t* h_in, uint32_t* boundaries, size_t h_in_len,
                                   uint32_t offset, uint32_t width);
LIBSORT_API bool providedGpuProfile(unsigned int* h_in, size_t h_in_len);

/* ======================= Part 2: additive API ============================= */

/* North-star names (BASELINE.json): aliases of providedGpu / gpuPartial. */
LIBSORT_API bool gpuFullSort(unsigned int* h_in, size_t len);
LIBSORT_API bool gpuPartialSort(uint32_t* h_in, uint32_t* boundaries, size_t h_in_len,
                                uint32_t offset, uint32_t width);

/* Device-resident sort of uint32 keys on the caller's current HIP device,
 * enqueued on `stream` (a hipStream_t; NULL = the null stream).  Sorts bits
 * [offset, offset+width) stably (width = 32 - offset for a full sort).
 * d_in is read-only; the result is written to d_out; d_tmp is scratch of n
 * keys.  d_in may equal d_out (in place); d_tmp must alias neither.
 * d_boundaries (nullable, device, 2^width uint32) receives the same
 * boundaries as gpuPartial.  The work is enqueued on `stream`; the call
 * returns before it completes, except that a full-width sort served by the
 * MSD hybrid (libsortSetHybrid) waits on the host for two small read-backs
 * while its first and last digit passes run.  Under stream capture (HIP
 * graphs) the hybrid is never taken, so a captured call never waits.  With
 * d_in != d_out the hybrid's first pass places its runs in sampled slices of
 * a cached per-device buffer of ~1.14 n (4-bit digits) / ~1.28 n (8-bit) keys
 * instead of reading the keys twice (LIBSORT_HYB_RESERVE=0: the count pass
 * instead). */
LIBSORT_API bool libsortSortKeysU32(const uint32_t* d_in, uint32_t* d_out, uint32_t* d_tmp,
                                    size_t n, uint32_t offset, uint32_t width,
                                    uint32_t* d_boundaries, void* stream);

/* Full sort of keys known to lie in [lo, hi) (lo < hi <= 2^32): the digits
 * are taken from key - lo, so ceil(log2(hi - lo) / digit bits) passes instead
 * of 32 / digit bits (a round of the multi-GPU schedule spans about 2^27
 * key values: 7 four-bit passes instead of 8).  Keys outside [lo, hi) give an
 * unspecified order (no fault).  Same buffers as libsortSortKeysU32. */
LIBSORT_API bool libsortSortKeysRangeU32(const uint32_t* d_in, uint32_t* d_out, uint32_t* d_tmp,
                                         size_t n, uint32_t lo, uint64_t hi, void* stream);

/* Sort of pre-partitioned keys: the receive buffer of a multi-GPU round,
 * whose pieces arrive already partitioned by the senders' top-digit pass
 * (the gather fused into the next pass's tile loader
 * as a segment table).  Piece p = d_in[off[p], off[p] + len[p]) belongs to
 * segment seg[p]; off/len/seg are host arrays of npieces entries listed in
 * non-decreasing segment order, seg[p] < nseg.  Every key of segment s has
 * the same bits [bits, 32), and those increase with s.  d_out receives the
 * n = sum(len) keys in ascending order; d_tmp is scratch of n keys; d_in,
 * d_out and d_tmp are distinct.  The digit passes start from the pieces'
 * own tiles (no gather copy and no pass over the bits the segments already
 * fix); small or skewed inputs are gathered and LSD-sorted instead.  Waits on
 * the host like the hybrid sorts (libsortSetHybrid). */
LIBSORT_API bool libsortSortPiecesU32(const uint32_t* d_in, uint32_t* d_out, uint32_t* d_tmp, size_t n,
                                      const uint64_t* off, const uint64_t* len, const uint32_t* seg,
                                      size_t npieces, uint32_t nseg, uint32_t bits, void* stream);

/* Stable key-value sort: 64-bit keys, 32-bit payloads (BASELINE config C5). */
LIBSORT_API bool libsortSortPairsU64U32(const uint64_t* d_kin, const uint32_t* d_vin,
                                        uint64_t* d_kout, uint32_t* d_vout,
                                        uint64_t* d_ktmp, uint32_t* d_vtmp, size_t n,
                                        uint32_t offset, uint32_t width, void* stream);

/* Sort of 64-bit keys by bits [offset, offset+width) (width = 64 - offset for
 * a full sort; stable).  Same buffer rules as libsortSortKeysU32 (d_in may
 * equal d_out, d_tmp distinct).  SURVEY.md §8(f) row 4: 64-bit keys beyond C5. */
LIBSORT_API bool libsortSortKeysU64(const uint64_t* d_in, uint64_t* d_out, uint64_t* d_tmp,
                                    size_t n, uint32_t offset, uint32_t width, void* stream);

/* Stable key-value sort: 64-bit keys, 64-bit payloads (e.g. row ids past
 * 2^32 or packed records). */
LIBSORT_API bool libsortSortPairsU64U64(const uint64_t* d_kin, const uint64_t* d_vin,
                                        uint64_t* d_kout, uint64_t* d_vout,
                                        uint64_t* d_ktmp, uint64_t* d_vtmp, size_t n,
                                        uint32_t offset, uint32_t width, void* stream);

/* Stable key-value sort: 32-bit keys, 32-bit payloads. */
LIBSORT_API bool libsortSortPairsU32U32(const uint32_t* d_kin, const uint32_t* d_vin,
                                        uint32_t* d_kout, uint32_t* d_vout,
                                        uint32_t* d_ktmp, uint32_t* d_vtmp, size_t n,
                                        uint32_t offset, uint32_t width, void* stream);

/* Histogram of (key >> shift) & (2^bits - 1), bits <= 16, into d_hist
 * (2^bits uint32, overwritten). */
LIBSORT_API bool libsortHistogramU32(const uint32_t* d_keys, size_t n, uint32_t shift,
                                     uint32_t bits, uint32_t* d_hist, void* stream);

/* Stable partition by range: element x goes to bucket b = #{i : x >= splitters[i]}
 * (host array, ascending, nsplit <= 255).  d_out receives the buckets in order;
 * d_counts (nullable, device, nsplit+1 uint32) receives the bucket sizes. */
LIBSORT_API bool libsortPartitionU32(const uint32_t* d_in, uint32_t* d_out, size_t n,
                                     const uint32_t* splitters, uint32_t nsplit,
                                     uint32_t* d_counts, void* stream);

/* Stable partition by table: element x goes to bucket lut[x >> lut_shift]
 * (d_lut: device, 1 << (32 - lut_shift) one-byte entries, 4-byte aligned,
 * 20 <= lut_shift <= 30, every entry < nbuckets <= 256).  d_out (!= d_in)
 * receives the buckets in order; d_bounds (nullable, device, nbuckets uint32)
 * the bucket starts.  One tile-offset pass (per-tile counts, column scan,
 * scatter); the multi-GPU schedule partitions by (round, destination rank)
 * with it. */
LIBSORT_API bool libsortPartitionLutU32(const uint32_t* d_in, uint32_t* d_out, size_t n,
                                        const uint8_t* d_lut, uint32_t lut_shift,
                                        uint32_t nbuckets, uint32_t* d_bounds, void* stream);

/* The same for (uint64 key, uint32 payload) pairs, bucket = lut[(key >> 32) >>
 * lut_shift]; keys and payloads move together (out of place, stable). */
LIBSORT_API bool libsortPartitionLutU64U32(const uint64_t* d_kin, const uint32_t* d_vin,
                                           uint64_t* d_kout, uint32_t* d_vout, size_t n,
                                           const uint8_t* d_lut, uint32_t lut_shift,
                                           uint32_t nbuckets, uint32_t* d_bounds, void* stream);

/* The same partitions in two calls, so a caller can read the bucket sizes
 * while the data moves: ...Count runs the per-tile counts and the column scan
 * and writes the bucket starts to d_bounds (device, nbuckets uint32);
 * ...Scatter then moves the data.  The scatter call must follow its count call
 * with the same input, table, shift, bucket count and stream, with no other
 * libsort sort/partition on that device's workspace in between (otherwise it
 * returns false).  The multi-GPU schedule reads the sizes, gathers them and
 * issues its exchange while the scatter runs. */
LIBSORT_API bool libsortPartitionLutCountU32(const uint32_t* d_in, size_t n, const uint8_t* d_lut,
                                             uint32_t lut_shift, uint32_t nbuckets, uint32_t* d_bounds,
                                             void* stream);
LIBSORT_API bool libsortPartitionLutScatterU32(const uint32_t* d_in, uint32_t* d_out, size_t n,
                                               const uint8_t* d_lut, uint32_t lut_shift, uint32_t nbuckets,
                                               void* stream);
LIBSORT_API bool libsortPartitionLutCountU64U32(const uint64_t* d_kin, const uint32_t* d_vin, size_t n,
                                                const uint8_t* d_lut, uint32_t lut_shift, uint32_t nbuckets,
                                                uint32_t* d_bounds, void* stream);
LIBSORT_API bool libsortPartitionLutScatterU64U32(const uint64_t* d_kin, const uint32_t* d_vin,
                                                  uint64_t* d_kout, uint32_t* d_vout, size_t n,
                                                  const uint8_t* d_lut, uint32_t lut_shift,
                                                  uint32_t nbuckets, void* stream);

/* The same two-call partitions by the 8-bit RANGE digit (key - bias) >> shift
 * (256 buckets; every key in [bias, bias + 2^(shift + 8)); 0 <= shift <= 24
 * for u32 keys, <= 56 for u64 keys): the multi-GPU rounds over a key range
 * narrower than the top digit (IDs, timestamps, keys below 2^26 at 8 GPUs;
 * bias and shift from libsortDistribRangeDigit over the ranks' smallest and
 * largest keys).  Same call-order rule as the table partitions above. */
LIBSORT_API bool libsortPartitionRangeCountU32(const uint32_t* d_in, size_t n, uint32_t bias, uint32_t shift,
                                               uint32_t* d_bounds, void* stream);
LIBSORT_API bool libsortPartitionRangeScatterU32(const uint32_t* d_in, uint32_t* d_out, size_t n, uint32_t bias,
                                                 uint32_t shift, void* stream);
LIBSORT_API bool libsortPartitionRangeCountU64U32(const uint64_t* d_kin, const uint32_t* d_vin, size_t n,
                                                  uint64_t bias, uint32_t shift, uint32_t* d_bounds, void* stream);
LIBSORT_API bool libsortPartitionRangeScatterU64U32(const uint64_t* d_kin, const uint32_t* d_vin, uint64_t* d_kout,
                                                    uint32_t* d_vout, size_t n, uint64_t bias, uint32_t shift,
                                                    void* stream);

/* Smallest and largest key: d_minmax[0], d_minmax[1] (device; n == 0 gives
 * the largest value of the type, then 0). */
LIBSORT_API bool libsortMinMaxU32(const uint32_t* d_keys, size_t n, uint32_t* d_minmax, void* stream);
LIBSORT_API bool libsortMinMaxU64(const uint64_t* d_keys, size_t n, uint64_t* d_minmax, void* stream);

/* libsortSortPiecesU32 for pieces partitioned by the range digit: every key of
 * segment s has the same bits [bits, 32) of key - bias (bits = the range
 * digit's shift), increasing with s. */
LIBSORT_API bool libsortSortPiecesRangeU32(const uint32_t* d_in, uint32_t* d_out, uint32_t* d_tmp, size_t n,
                                           const uint64_t* off, const uint64_t* len, const uint32_t* seg,
                                           size_t npieces, uint32_t nseg, uint32_t bits, uint32_t bias, void* stream);

/* Gather-copy of nseg segments: dst[dst_off[i] + j] = src[src_off[i] + j] for
 * j < len[i].  The three tables are host arrays.  Used to put exchanged
 * buckets into bucket-major / rank-minor order between distributed rounds. */
LIBSORT_API bool libsortSegmentCopyU32(const uint32_t* d_src, uint32_t* d_dst, size_t nseg,
                                       const uint64_t* src_off, const uint64_t* dst_off,
                                       const uint64_t* len, void* stream);

/* Delta-coded sorted runs (the "msdz" exchange of pylibsort.distrib for
 * link-bound world sizes).  A sorted uint32 run of n keys is coded in groups
 * of 64: the group's first key (uint32) and its 64 gaps to the previous key in
 * w bits, w = bit width of the largest in-group gap of the run (0 when every
 * group holds one value).  Coded size: ceil(n/64) * (1 + 2w) uint32 words,
 * bases first.
 * libsortDeltaMaxGapU32 writes the largest in-group gap to *d_maxgap (device);
 * libsortDeltaPackU32 codes the run with w taken from *d_maxgap on the device
 * (so it can be queued before the host knows w); libsortDeltaUnpackU32
 * decodes n keys given w (`bits`); libsortMergeU32 merges two sorted runs
 * into d_out (distinct from both). */
LIBSORT_API bool libsortDeltaMaxGapU32(const uint32_t* d_keys, size_t n, uint32_t* d_maxgap, void* stream);
LIBSORT_API bool libsortDeltaPackU32(const uint32_t* d_keys, size_t n, const uint32_t* d_maxgap, uint32_t* d_out,
                                     void* stream);
LIBSORT_API bool libsortDeltaUnpackU32(const uint32_t* d_in, size_t n, uint32_t bits, uint32_t* d_keys, void* stream);
LIBSORT_API bool libsortMergeU32(const uint32_t* d_a, size_t na, const uint32_t* d_b, size_t nb, uint32_t* d_out,
                                 void* stream);

/* Multi-GPU sort in one process (replaces the
 * reference's distributed drivers localTest/benchmarks.cpp:70-160 and
 * benchmark/pkg/sort/distrib.go:90-179, whose exchange goes through host
 * memory or files).  The ranks' shards are exchanged over a single-process
 * RCCL communicator (ncclCommInitAll over the ranks' devices, xGMI
 * point-to-point); the result is the reference's equal re-cut: rank r holds
 * keys [r*S, (r+1)*S) of the sorted whole, S = ceil(N / nranks)
 * (distrib.go:113).
 *
 * gpuDistribSort: h_in[0..len) (host) is cut into ngpu shards of
 * ceil(len/ngpu) keys, sorted across ngpu devices taken from the device pool
 * (ngpu <= 0: all of them) and copied back in place; ascending, the same
 * result as providedGpu / std::sort, for len up to ngpu * (2^32 - 1).
 * Blocks while the devices are busy, like the other pool entry points. */
LIBSORT_API bool gpuDistribSort(uint32_t* h_in, size_t len, int ngpu);

/* Device-resident form: rank r's shard d_in[r] (n_in[r] <= 2^32-1 keys in
 * memory of device devices[r], read-only) -> d_out[r] (device devices[r],
 * capacity ceil(N/nranks) keys), n_out[r] (host) = keys written.  Devices may
 * repeat (ranks sharing a GPU run one after another and exchange by device
 * copies; RCCL refuses two ranks on one GPU).  Synchronous: returns when every
 * device is done.  flags: LIBSORT_DISTRIB_LSD runs the reference's BSP LSD
 * rounds (8-bit digits, bucket-major / rank-minor re-cut after every round)
 * instead of the default top-digit rounds; LIBSORT_DISTRIB_COPY exchanges with
 * peer copies (hipMemcpyPeerAsync) instead of RCCL; LIBSORT_DISTRIB_SELF_RCCL
 * sends a rank's own pieces through RCCL too (tests). */
#define LIBSORT_DISTRIB_LSD 1u
#define LIBSORT_DISTRIB_COPY 2u
#define LIBSORT_DISTRIB_SELF_RCCL 4u
/* LIBSORT_DISTRIB_WIRE32: keys cross the links as 32-bit words.  By default
 * the top-digit rounds at 4-bit digits send 24 bits per key (two planes: the
 * low 16 bits and bits 16..23; the top byte is the partition digit the piece
 * already names), 3 bytes instead of 4; LIBSORT_DISTRIB_WIRE24=0 in the
 * environment does the same as this flag. */
#define LIBSORT_DISTRIB_WIRE32 8u
/* LIBSORT_DISTRIB_CODED: gap-coded rounds -- each sender sorts its outgoing
 * pieces of a round and sends them as gaps (64-key groups: a base word and
 * 2w words, w = the bits of the piece's largest gap; ~0.3 of the 32-bit
 * bytes for uniform keys), the receiver decodes them and merges its sorted
 * runs.  Fewer bytes on the links for more GPU work (a merge level per
 * doubling of nranks): the default at two ranks on two GPUs over RCCL, where
 * one xGMI link carries half of every shard.  LIBSORT_DISTRIB_CODED=1 / 0 in
 * the environment forces it on / off.  Same result (a full sort is unique);
 * the skew fallback to the LSD rounds is unchanged. */
#define LIBSORT_DISTRIB_CODED 16u
LIBSORT_API bool libsortDistribSortU32(int nranks, const int* devices, const uint32_t* const* d_in,
                                       const size_t* n_in, uint32_t* const* d_out, size_t* n_out,
                                       uint32_t flags);

/* The same engine for (uint64 key, uint32 payload) pairs, stable (BASELINE
 * configs[4]: 2^31 pairs over 8 GPUs): rank r's shard (d_kin[r], d_vin[r],
 * n_in[r] pairs on devices[r]) -> (d_kout[r], d_vout[r]) = pairs [r*S,
 * (r+1)*S) of the stably sorted whole (payloads of equal keys keep the input
 * order: shard 0 first).  The top-digit rounds on the key's top 8 bits with a
 * stable pair sort per round.  flags: LIBSORT_DISTRIB_COPY /
 * LIBSORT_DISTRIB_SELF_RCCL (not _LSD).  Synchronous. */
LIBSORT_API bool libsortDistribSortPairsU64U32(int nranks, const int* devices, const uint64_t* const* d_kin,
                                               const uint32_t* const* d_vin, const size_t* n_in,
                                               uint64_t* const* d_kout, uint32_t* const* d_vout, size_t* n_out,
                                               uint32_t flags);

/* Both engines above, nranks > 1 on distinct GPUs over RCCL: each rank
 * partitions its keys in two parts (the first half, then the rest) so that
 * the exchange of the first part's pieces starts while the second part is
 * partitioned; ranks sharing a GPU (device-copy exchanges) keep one part.
 * Results are the same.  LIBSORT_DISTRIB_PARTS=1 / 2 in the environment
 * forces one / two parts. */

/* Stage trace of the multi-GPU engines on stderr (what a hang would stop at):
 * one line per stage -- partition counts / scatter issued, counts read, plan,
 * round k issued, round k arrived and sorted on each rank, re-cut -- with the
 * milliseconds since the call started.  Tracing waits for each round's
 * arrival on the host, so it serialises the overlap: a diagnostic, not a
 * timing mode.  on: 1 / 0; returns the previous setting (initially
 * LIBSORT_DISTRIB_TRACE=1 in the environment). */
LIBSORT_API int libsortSetDistribTrace(int on);

/* Whether the multi-GPU engine's compute and communication streams of
 * devices[0] (its context over these nranks devices) run concurrently in the
 * calling process: one spinning single-wave kernel of spin_us microseconds on
 * each; ms[0..3] receives the start and end of the first and the start and
 * end of the second, in milliseconds after a common event.  Windows that do
 * not overlap mean the two streams share one hardware queue (more streams on
 * the device than GPU_MAX_HW_QUEUES).  A diagnostic; synchronous. */
LIBSORT_API bool libsortDistribOverlapProbe(int nranks, const int* devices, uint32_t spin_us, double* ms);

/* Bytes each rank sent to the other ranks in the exchange rounds (its own
 * pieces and the final re-cut's surplus keys excluded) in the last
 * libsortDistribSort* / gpuDistribSort call over nranks ranks:
 * per_rank[0..nranks).  false if none ran. */
LIBSORT_API bool libsortDistribLastBytes(int nranks, uint64_t* per_rank);

/* Host plan of the multi-GPU top-digit rounds (pylibsort.distrib and the
 * single-process engine above both run it; csrc/distrib_plan.h).
 * counts[r * 256 + g] = keys of rank r whose top 8 bits are g (exact, from
 * each rank's partition pass).  Writes lut[g] = round * nranks + rank of
 * digit g -- contiguous digit ranges in key order, about 1/nranks of the keys
 * per rank, `rounds` rounds per rank growing by `growth` -- and est[r] = keys
 * rank r receives.  nranks * rounds <= 256.  Host only (no device needed). */
LIBSORT_API bool libsortDistribPlanDigits(const int64_t* counts, uint32_t nranks, uint32_t rounds, double growth,
                                          uint8_t* lut, int64_t* est);

/* The range digit of the multi-GPU rounds when the top 8 key bits leave the
 * keys in too few digits (csrc/distrib_plan.h range_digit; both engines use
 * it): over the ranks' smallest and largest keys [lo, hi] of a key_bits-bit
 * key (32 or 64), *bias = lo and *shift = max(0, bits(hi - lo) - 8), so every
 * key's digit (key - lo) >> shift is < 256.  Returns whether that digit splits
 * finer than the top digit (false when every key is equal).  Host only. */
LIBSORT_API bool libsortDistribRangeDigit(uint64_t lo, uint64_t hi, uint32_t key_bits, uint64_t* bias,
                                          uint32_t* shift);

/* Writes elements [first, first+n) of the populateInput stream of a fresh
 * process (state 0x4d595df4d0f33173) to device memory, by LCG skip-ahead. */
LIBSORT_API bool libsortPopulateDevice(uint32_t* d_out, size_t n, uint64_t first, void* stream);

/* Radix digit width used by the sorts (4 or 8 bits; default 8, or the
 * LIBSORT_DIGIT_BITS environment variable).  Returns the previous value, or
 * -1 if `bits` is unsupported. */
LIBSORT_API int libsortSetDigitBits(int bits);
LIBSORT_API int libsortGetDigitBits(void);

/* Pass algorithm: 0 = auto (default: tile offsets), 1 = onesweep (one kernel
 * per digit, decoupled look-back; n < 2^30, else tile offsets), 2 =
 * reduce-then-scan (upsweep + scan + downsweep), 3 = tile offsets (per-tile
 * counts + column scan + pass kernel without look-back; 4-bit digits count
 * the next pass inside the pass kernel).  Initial value from LIBSORT_ALGO
 * ("auto" / "onesweep" / "rts" / "tiles").  Returns the previous value, or -1
 * if `algo` is invalid. */
LIBSORT_API int libsortSetAlgorithm(int algo);

/* Full-width sorts (providedGpu, libsortSortKeysU32 with offset 0 / width 32,
 * libsortSortKeysRangeU32 over >= 20 bits, libsortSortPairsU32U32 and the
 * 64-bit key sorts at full width; 4- or 8-bit digits): 1 (default) = for
 * 2^27 <= n <= 2^28 + 2^24 keys (2^25 <= n for 64-bit keys) the MSD hybrid
 * (16 / digit-bits passes from the top digit down, then every bucket of keys
 * sharing the top 16 bits sorted on chip, stable; the host waits twice
 * inside the call for small read-backs while passes run, and the call returns
 * with the bucket sort queued like any other sort); 0 = always the LSD digit
 * passes; 2 = the hybrid for every
 * such sort of n >= 1024 keys (tests).  Initial value from LIBSORT_HYBRID.
 * Returns the previous value, or -1 if `mode` is invalid. */
LIBSORT_API int libsortSetHybrid(int mode);

/* The on-chip sort of the hybrid's buckets for 32-bit keys without values
 * (each bucket: the keys sharing their top 16 bits, sorted on their low 16
 * or fewer): 1 (default) = a counting sort in LDS -- 4096 cells by the top 12
 * of those bits, each holding a 3-bit count per value of the remaining 4
 * (the last 4-bit digit), one atomic per key, positions from the scanned cell
 * counts; also lets 2^30-key sorts take the hybrid (buckets of ~16K keys);
 * 0 = 4-bit LSD steps on chip (ballot ranks), and 2^30-key sorts take the
 * LSD passes.  Initial value from LIBSORT_BUCKET_COUNT.  Returns the previous
 * value, or -1 if `mode` is invalid. */
LIBSORT_API int libsortSetBucketMode(int mode);

/* Boundaries returned by gpuPartial / gpuPartialProfile / gpuPartialSort:
 * 0 (default) = for every group g the number of elements whose group is < g
 * (the exclusive prefix every reference caller and test expects:
 * localTest/tests.cpp:41-83, benchmark/pkg/sort/distrib.go:45-52,
 * faasTest/pylibsort/data.py:301-304); 1 = bit-for-bit the reference
 * SortState::GetBoundaries output (sort.cu:367-394), whose host fill leaves an
 * empty group 1 at 0 and overwrites a first non-empty group >= 2 with the
 * next group's start.  The two agree whenever group 1 is non-empty.  Initial
 * value from LIBSORT_BOUNDARIES ("reference" selects 1).  Returns the
 * previous mode, or -1 if `mode` is invalid. */
LIBSORT_API int libsortSetBoundaryMode(int mode);

/* Per-kernel timing with hipEvents on the launch stream.  Names: "tilecounts",
 * "colscan", "tilepass", "hybplan", "bucketsort", "whist", "onesweep",
 * "upsweep", "scan", "downsweep", "bounds", "histogram", "populate",
 * "segcopy".  libsortTimingFilter: record only the listed kernels
 * (comma-separated, e.g. "tilepass"); NULL or "" = all. */
LIBSORT_API void libsortTimingEnable(bool on);
LIBSORT_API void libsortTimingReset(void);
LIBSORT_API void libsortTimingFilter(const char* kernels);
/* Record only every `every`-th launch that passes the filter (counted from the
 * last reset; 0 or 1 = every launch).  A stride coprime to the launches of
 * one sort samples each of them in turn with fewer events in the stream. */
LIBSORT_API void libsortTimingSample(uint32_t every);
LIBSORT_API bool libsortTimingQuery(const char* kernel, uint64_t* launches, double* total_ms,
                                    uint64_t* total_keys);

/* Frees the cached per-device workspaces (they are otherwise kept for reuse). */
LIBSORT_API bool libsortReleaseWorkspace(void);

/* Last error message of the calling thread ("" if none). */
LIBSORT_API const char* libsortLastError(void);

/* Synchronises the current device; returns and clears its device-side error
 * word (bit 0: a look-back wait hit its spin bound).  0 = healthy. */
LIBSORT_API uint32_t libsortDeviceErrors(void);

#endif /* LIBSORT_MI355X_LIBSORT_H */
