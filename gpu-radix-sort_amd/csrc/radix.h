// radix.h -- internal interface between the C ABI (libsort_abi.cpp) and the
// HIP kernels / pass driver (radix_kernels.hip).  Not installed; the public
// surface is include/libsort.h.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#include <mutex>
#include <string>

namespace lsort {

// Tile geometry of the digit-pass kernels (DESIGN.md "Kernels").
constexpr int kBlock = 256;       // 4 waves of 64 lanes
constexpr int kItemsU32 = 16;     // keys per thread, u32 keys  -> 4096-key tiles
constexpr int kItemsU64 = 8;      // keys per thread, u64 keys  -> 2048-key tiles
constexpr int kScanBlock = 256;
constexpr int kScanItems = 16;
constexpr int kScanTile = kScanBlock * kScanItems;  // 4096 counters per scan tile
constexpr int kMaxSplit = 255;    // range partition: up to 256 buckets

// onesweep tiles and the layout of Workspace::os_small (uint32 words)
constexpr int kOsBlock = 512;  // 8192-key onesweep tiles (measured best for 8-bit digits)
constexpr int kOsItemsU32 = 16;
constexpr int kOsItemsU64 = 8;
constexpr int kOsWhist = 0;              // 8 windows x 256
constexpr int kOsGbase = 8 * 256;        // 16 passes x 256
constexpr int kOsCounters = kOsGbase + 16 * 256;  // 16 tile counters
constexpr int kOsErr = kOsCounters + 16;
constexpr int kOsSmallWords = kOsErr + 16;
constexpr int kOsZeroWords = kOsErr;     // memset per sort: histograms, bases, counters

struct NoValue {};

// Per-device cached state.  Every entry point holds `mu` while it uses it.
struct Workspace {
  int device = -1;
  int num_cus = 0;
  std::mutex mu;

  // reduce-then-scan counters: counts[digit][block] and its two-level scan
  uint32_t* counts = nullptr;
  uint32_t* scan_l1 = nullptr;
  uint32_t* scan_l2 = nullptr;
  size_t counts_cap = 0;  // elements
  size_t l2_cap = 0;      // elements

  // staging for the host-pointer ABI (providedGpu / gpuPartial)
  void* hbuf[2] = {nullptr, nullptr};
  size_t hbuf_cap = 0;  // bytes per buffer
  uint32_t* dbounds = nullptr;
  size_t dbounds_cap = 0;  // elements

  // segment tables for libsortSegmentCopyU32 (pinned staging + device copy)
  uint64_t* seg_dev = nullptr;
  uint64_t* seg_host = nullptr;
  size_t seg_cap = 0;  // uint64 elements
  hipEvent_t seg_evt = nullptr;

  // scratch for histogram partials
  uint32_t* hist_tmp = nullptr;
  size_t hist_tmp_cap = 0;

  hipStream_t stream = nullptr;  // used by the host-pointer ABI

  // pipelined host full sort (libsort_abi.cpp host_full_sort_pipelined): a
  // third key buffer, a copy stream, the plan block on the device (histogram,
  // partition table, chunk bucket starts, segment tables) and its pinned mirror
  void* pbuf = nullptr;
  size_t pbuf_cap = 0;  // bytes
  hipStream_t copy_stream = nullptr;
  uint32_t* plan_dev = nullptr;
  uint32_t* plan_host = nullptr;
  static constexpr size_t kPlanWords = 4096 + 1024 + 1024 + 3 * 2 * 1024;  // hist | lut | bounds | seg tables (u64)
  static constexpr int kPipeEvents = 64;
  hipEvent_t pipe_evt[kPipeEvents] = {};
  hipError_t ensure_pipeline(size_t bytes);

  // onesweep path: two look-back status buffers [tiles][RADIX] and a small
  // block: window histograms | per-pass digit bases | tile counters | error
  uint32_t* os_status[2] = {nullptr, nullptr};
  size_t os_status_cap = 0;  // words per buffer
  uint32_t* os_small = nullptr;
  int last_algo = 0;  // 1 = onesweep, 2 = reduce-then-scan, 3 = tile offsets (last sort)
  uint32_t* last_pass_counts = nullptr;  // tile path: the last pass's scanned count rows (gpuPartial boundaries)

  // tile-offset path: per-tile digit counts (two buffers) and chunk totals
  uint32_t* tc[2] = {nullptr, nullptr};
  size_t tc_cap = 0;  // words per buffer
  uint32_t* tb = nullptr;  // chunk prefixes B[chunks][RADIX], then the digit starts D[RADIX]
  size_t tb_cap = 0;  // words
  uint32_t* tticket = nullptr;  // last-arriver ticket of the column scan (zero between launches)
  // A table partition split in two calls (count + scan, then scatter): the
  // arguments of the count call, checked by the scatter call.  ensure_tiles()
  // (the start of every other tile-path operation) clears it.
  struct PartToken {
    const void* in;
    const void* vin;
    size_t n;
    const uint8_t* lut;  // null: the range digit (key - bias) >> shift
    int shift, nb;
    uint64_t bias;
    hipStream_t st;
    bool valid;
    bool operator==(const PartToken& o) const {
      return valid && o.valid && in == o.in && vin == o.vin && n == o.n && lut == o.lut && shift == o.shift &&
             nb == o.nb && bias == o.bias && st == o.st;
    }
  };
  PartToken part_pending{nullptr, nullptr, 0, nullptr, 0, 0, 0, nullptr, false};
  hipError_t ensure_tiles(size_t count_words, size_t chunk_words);

  // MSD hybrid (sort_hybrid_u32): tile tables, per-segment run bases and
  // child tables of two depths, counters; a pinned mirror for the host checks
  uint32_t* hyb = nullptr;
  size_t hyb_cap = 0;  // words
  uint32_t* hyb_host = nullptr;  // pinned, 512 words
  uint32_t hyb_seq = 0;          // the last sampler sequence number (hyb_host[511])
  hipEvent_t hyb_evt = nullptr;
  hipError_t ensure_hybrid(size_t words);

  // 8-bit digit passes: the next pass's digit of every key, one byte at the
  // key's output position (written by the pass, read by the next pass's count
  // kernel: 1 B per key instead of the key)
  uint8_t* dstream = nullptr;
  size_t dstream_cap = 0;  // bytes
  hipError_t ensure_dstream(size_t bytes);

  // MSD hybrid, reserved depth 0: the slices the depth-0 pass writes (the
  // keys plus each slice's sampled slack; rsv_capacity_bound(n) words)
  uint32_t* rsv = nullptr;
  size_t rsv_cap = 0;  // words
  hipError_t ensure_rsv(size_t words);

  hipError_t ensure_counts(size_t m);
  hipError_t ensure_hbuf(size_t bytes);
  hipError_t ensure_bounds(size_t m);
  hipError_t ensure_seg(size_t m);
  hipError_t ensure_onesweep(size_t status_words);
  void release();
};

// Returns the workspace of `device` (created on first use; never destroyed
// except by release()).  Thread-safe.
Workspace* workspace_for(int device);
void release_all_workspaces();

// Number of LSD passes for `width` bits at `bits` per digit.
inline int num_passes(int width, int bits) { return width <= 0 ? 0 : (width + bits - 1) / bits; }

// Stable LSD radix sort of bits [lo, hi) of the keys (values carried along).
// in may equal out; tmp must not alias out; tmp may alias in only when the
// pass count is odd (used by the host ABI to avoid a copy).  When d_bounds is
// non-null, it receives the 2^(hi-lo) group boundaries of gpuPartial.
// bias != 0: the digits are taken from key - bias (range-restricted sort of
// keys in [bias, bias + 2^hi); no boundaries).
// All work is enqueued on `stream`; nothing synchronises.
// range: the keys are known to lie in [bias, bias + 2^hi) (libsortSortKeysRangeU32), so the
// hi sorted bits determine a key and the MSD hybrid may serve the sort; span (when
// nonzero): they lie in [bias, bias + span), span <= 2^hi (sizes the hybrid's buckets).
hipError_t sort_u32(Workspace& ws, const uint32_t* in, uint32_t* out, uint32_t* tmp, size_t n,
                    int lo, int hi, int digit_bits, uint32_t* d_bounds, hipStream_t stream,
                    uint32_t bias = 0, bool range = false, uint64_t span = 0);
// Sort of pre-partitioned keys (a multi-GPU round's receive buffer, whose
// pieces arrive partitioned by the senders): piece p = in[off[p], off[p] +
// len[p]) of segment seg[p] (host arrays; np pieces in non-decreasing segment
// order, seg < nseg); the keys of segment s share the bits [bits, 32) of key -
// bias and those increase with s.  out (distinct from in and tmp) receives
// the n = sum(len) keys sorted; tmp: scratch of n keys.  The MSD hybrid
// starts from the pieces' own tiles (no gather, no pass over the top bits);
// small or skewed inputs are gathered and LSD-sorted; bits == 0 (every
// segment one value): the gather alone.
hipError_t sort_pieces_u32(Workspace& ws, const uint32_t* in, uint32_t* out, uint32_t* tmp, size_t n,
                           const uint64_t* off, const uint64_t* len, const uint32_t* seg, size_t np, uint32_t nseg,
                           int bits, int digit_bits, hipStream_t stream, uint32_t bias = 0);
// The same over 24-bit pieces (the multi-GPU exchange's "wire24" format):
// in16 / in8 hold each key's low 16 bits and bits 16..23 at the key's index,
// segment s's keys have top byte hi0 + s (bits = 24 below the segment).
hipError_t sort_pieces_planar_u32(Workspace& ws, const uint16_t* in16, const uint8_t* in8, uint32_t hi0,
                                  uint32_t* out, uint32_t* tmp, size_t n, const uint64_t* off, const uint64_t* len,
                                  const uint32_t* seg, size_t np, uint32_t nseg, int digit_bits, hipStream_t stream);
hipError_t sort_pairs_u32_u32(Workspace& ws, const uint32_t* kin, const uint32_t* vin,
                              uint32_t* kout, uint32_t* vout, uint32_t* ktmp, uint32_t* vtmp,
                              size_t n, int lo, int hi, int digit_bits, hipStream_t stream);
hipError_t sort_u64(Workspace& ws, const uint64_t* in, uint64_t* out, uint64_t* tmp, size_t n, int lo, int hi,
                    int digit_bits, hipStream_t stream);
hipError_t sort_pairs_u64_u64(Workspace& ws, const uint64_t* kin, const uint64_t* vin,
                              uint64_t* kout, uint64_t* vout, uint64_t* ktmp, uint64_t* vtmp,
                              size_t n, int lo, int hi, int digit_bits, hipStream_t stream);
hipError_t sort_pairs_u64_u32(Workspace& ws, const uint64_t* kin, const uint32_t* vin,
                              uint64_t* kout, uint32_t* vout, uint64_t* ktmp, uint32_t* vtmp,
                              size_t n, int lo, int hi, int digit_bits, hipStream_t stream);

// Pass algorithm: 0 = auto (tile offsets), 1 = onesweep (n < 2^30, else tile
// offsets), 2 = reduce-then-scan, 3 = tile offsets.  Initialised from LIBSORT_ALGO ("auto" / "onesweep" /
// "rts" / "tiles").
int get_algorithm();
int set_algorithm(int algo);  // returns the previous value, -1 if invalid
// MSD hybrid for full-width sorts: 0 = off, 1 = auto (2^27 <= n <= 2^28 +
// 2^24; 2^25 <= n for 64-bit keys), 2 = every full sort of n >= 1024 keys.
// LIBSORT_HYBRID.
int get_hybrid_mode();
int set_hybrid_mode(int mode);
int get_bucket_mode();  // 1 = counting placement in the hybrid's u32 bucket sort, 0 = 4-bit LSD steps
int set_bucket_mode(int mode);

// Host-side choice of the ping-pong pair for the host ABI: returns true when
// the result of a `passes`-pass sort started from hbuf[0] lands in hbuf[1].
inline bool host_result_in_second(int passes) { return (passes & 1) != 0; }

hipError_t histogram_u32(Workspace& ws, const uint32_t* keys, size_t n, int shift, int bits,
                         uint32_t* d_hist, hipStream_t stream);
hipError_t partition_u32(Workspace& ws, const uint32_t* in, uint32_t* out, size_t n,
                         const uint32_t* splitters, int nsplit, uint32_t* d_counts,
                         hipStream_t stream);
// Stable partition of `in` into `out` (in != out) by bucket = lut[key >>
// lut_shift] (lut: device, 1 << (32 - lut_shift) one-byte entries, 4-byte
// aligned, 20 <= lut_shift <= 30, entries < nbuckets <= 256); d_bounds (may
// be null) receives the nbuckets bucket starts.
// phase: kPartBoth (one call), or kPartCount (counts + scan + bounds; `out`
// unused) followed by kPartScatter (the pass, same in/lut/shift/nbuckets/
// stream, no other tile-path call on the workspace in between; d_bounds unused).
constexpr int kPartBoth = 0, kPartCount = 1, kPartScatter = 2;
hipError_t partition_lut_u32(Workspace& ws, const uint32_t* in, uint32_t* out, size_t n, const uint8_t* d_lut,
                             int lut_shift, int nbuckets, uint32_t* d_bounds, hipStream_t stream,
                             int phase = kPartBoth);
// The scatter phase of partition_lut_u32 (after its count call, lut_shift 24,
// 256 buckets) writing 24-bit planes instead of u32 keys: o16[i] = low 16
// bits, o8[i] = bits 16..23 of the key at partition position i (the top byte
// is the bucket).
hipError_t partition_lut_planar_u32(Workspace& ws, const uint32_t* in, uint16_t* o16, uint8_t* o8, size_t n,
                                   const uint8_t* d_lut, int lut_shift, int nbuckets, hipStream_t stream);
// The same for (u64 key, u32 value) pairs; bucket = lut[(key >> 32) >> lut_shift].
hipError_t partition_lut_pairs_u64_u32(Workspace& ws, const uint64_t* kin, const uint32_t* vin, uint64_t* kout,
                                       uint32_t* vout, size_t n, const uint8_t* d_lut, int lut_shift, int nbuckets,
                                       uint32_t* d_bounds, hipStream_t stream, int phase = kPartBoth);
// The same partitions by the 8-bit range digit (key - bias) >> shift (256
// buckets; keys in [bias, bias + 2^(shift + 8)), 0 <= shift <= 24 (u32) / 56
// (u64)): the multi-GPU rounds over a key range narrower than the top digit.
hipError_t partition_range_u32(Workspace& ws, const uint32_t* in, uint32_t* out, size_t n, uint32_t bias, int shift,
                               uint32_t* d_bounds, hipStream_t stream, int phase = kPartBoth);
hipError_t partition_range_pairs_u64_u32(Workspace& ws, const uint64_t* kin, const uint32_t* vin, uint64_t* kout,
                                         uint32_t* vout, size_t n, uint64_t bias, int shift, uint32_t* d_bounds,
                                         hipStream_t stream, int phase = kPartBoth);
// Smallest and largest key into d_mm[0], d_mm[1] (device; n == 0: ~0, 0).
hipError_t minmax_u32(Workspace& ws, const uint32_t* keys, size_t n, uint32_t* d_mm, hipStream_t stream);
hipError_t minmax_u64(Workspace& ws, const uint64_t* keys, size_t n, uint64_t* d_mm, hipStream_t stream);
// Segment copy with the table already on the device: d_tab = [src_off[nseg] |
// dst_off[nseg] | len[nseg]] (uint64), nseg <= 65535; maxlen = the longest
// segment (sizes the grid), total = sum of len (timing only).
hipError_t segment_copy_dev_u32(const uint32_t* src, uint32_t* dst, const uint64_t* d_tab, size_t nseg,
                                uint64_t maxlen, uint64_t total, hipStream_t stream);
hipError_t segment_copy_u32(Workspace& ws, const uint32_t* src, uint32_t* dst, size_t nseg,
                            const uint64_t* src_off, const uint64_t* dst_off, const uint64_t* len,
                            hipStream_t stream);
hipError_t populate_device(uint32_t* out, size_t n, uint64_t first, hipStream_t stream);
// delta-coded sorted runs (the msdz exchange): largest in-group gap, pack
// (w from the device word), unpack (w from the host), two-run merge
hipError_t delta_maxgap_u32(const uint32_t* keys, size_t n, uint32_t* d_maxgap, hipStream_t st);
hipError_t delta_pack_u32(const uint32_t* keys, size_t n, const uint32_t* d_maxgap, uint32_t* out, hipStream_t st);
hipError_t delta_unpack_u32(const uint32_t* in, size_t n, uint32_t w, uint32_t* keys, hipStream_t st);
hipError_t merge_u32(const uint32_t* a, size_t na, const uint32_t* b, size_t nb, uint32_t* out, hipStream_t st);

// Cross-stream ordering of a device's workspace (libsort_abi.cpp): a call on
// stream `st` first waits for the previous call's work on another stream;
// release records the point after this call's work.
bool ws_acquire_stream(int dev, hipStream_t st);
void ws_release_stream(int dev, hipStream_t st);

// ---- single-process multi-GPU sort (distrib.cpp) ----
constexpr unsigned kDistribLsd = 1u;       // the reference's BSP LSD rounds instead of the range rounds
constexpr unsigned kDistribCopy = 2u;      // exchanges as peer copies instead of RCCL
constexpr unsigned kDistribSelfRccl = 4u;  // a rank's own pieces through RCCL too (tests)
constexpr unsigned kDistribWire32 = 8u;    // 32-bit keys on the wire (default: 24-bit planes, top-digit rounds)
constexpr unsigned kDistribCoded = 16u;    // gap-coded rounds: sender sorts, coded exchange, receiver merges
// Rank r's shard d_in[r] (n_in[r] keys, on device devices[r]; devices may
// repeat) -> d_out[r] = keys [r*S, (r+1)*S) of the sorted whole, S =
// ceil(N/R); n_out[r] receives the count.  Synchronous.
// Bytes each rank sent to other ranks in the exchange rounds of the last
// distributed sort (own pieces and the re-cut excluded); false if none ran or
// nranks differs.
bool distrib_last_bytes(uint64_t* per_rank, int nranks);
// stage trace on stderr (libsortSetDistribTrace); returns the previous setting
int set_distrib_trace(int on);
// concurrency of the engine's compute and communication streams on devices[0]
// (two spinning kernels; ms[4] = their start / end times)
bool distrib_overlap_probe(const int* devices, int R, uint32_t spin_us, double* ms);
bool distrib_sort_u32(const int* devices, int R, const uint32_t* const* d_in, const size_t* n_in, uint32_t* const* d_out,
                      size_t* n_out, unsigned flags, int digit_bits);
// (u64 key, u32 payload) pairs, stable (configs[4]): the top-digit rounds on
// the key's top 8 bits; flags: kDistribCopy / kDistribSelfRccl.  Synchronous.
bool distrib_sort_pairs_u64_u32(const int* devices, int R, const uint64_t* const* d_kin, const uint32_t* const* d_vin,
                                const size_t* n_in, uint64_t* const* d_kout, uint32_t* const* d_vout, size_t* n_out,
                                unsigned flags, int digit_bits);
// Host-pointer form: h[0..len) is cut into R shards of ceil(len/R) keys,
// sorted across the ranks' devices and copied back in place.
bool distrib_sort_host_u32(uint32_t* h, size_t len, const int* devices, int R, unsigned flags, int digit_bits);
void distrib_release();

// ---- per-kernel timing (hipEvents on the launch stream) ----
bool timing_enabled();
void timing_enable(bool on);
void timing_reset();
// Records only the kernels named in `csv` ("tilepass,bucketsort"); null or "" = all.
void timing_filter(const char* csv);
void timing_sample(uint32_t every);
bool timing_query(const char* name, uint64_t* launches, double* total_ms, uint64_t* total_keys);
// Records a start event; returns a token (or -1 when timing is off).
int timing_start(const char* name, hipStream_t stream, uint64_t keys);
void timing_stop(int token, hipStream_t stream);

struct ScopedTimer {
  int tok;
  hipStream_t s;
  ScopedTimer(const char* name, hipStream_t st, uint64_t keys) : tok(timing_start(name, st, keys)), s(st) {}
  ~ScopedTimer() { timing_stop(tok, s); }
};

// ---- host PCG32 (utils.cu:65-80) ----
constexpr uint64_t kPcgInit = 0x4d595df4d0f33173ull;
constexpr uint64_t kPcgMult = 6364136223846793005ull;
constexpr uint64_t kPcgInc = 1442695040888963407ull;

// Error text of the calling thread.
void set_error(const std::string& msg);
const char* last_error();

}  // namespace lsort
