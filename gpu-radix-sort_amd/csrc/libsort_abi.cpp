// libsort_abi.cpp -- the C ABI of include/libsort.h: device pool, host-pointer
// entry points (reference invokers.cu / utils.cu), additive device-resident
// entry points, PCG32 host generator and the per-kernel timing registry.
//
// NOTE on return types: this TU includes libsort.h, so the compiler checks
// every entry point against its declaration (`bool` as in the reference,
// libsort/libsort.h:14-32).  ctypes callers (faasTest/pylibsort/sort.py:
// 101,118) never set `restype` and read the whole of eax, but a `bool`
// return only defines al (clang: `movb $1, %al`).  So each bool entry point
// is exported as an alias of an int-returning definition (LS_BOOL_ENTRY
// below): the machine code leaves 0 or 1 in the whole of eax
// (tests/test_abi_cpu.py::test_bool_exports_define_eax).
#include "libsort.h"

#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "boundaries.h"
#include "distrib_plan.h"
#include "radix.h"

#define LIBSORT_EXPORT extern "C" __attribute__((visibility("default")))
// An entry point that libsort.h declares `bool`: the exported symbol is an
// alias of an int-returning definition (result 0 or 1 in the whole of eax),
// declared here with the header's exact signature, so the compiler checks it
// against libsort.h and callers reading al (bool: cgo, C++) or eax (ctypes'
// default restype) both see 0/1.  Host-only TU (hipcc --offload-host-only).
#define LS_BOOL_ENTRY(name, ...)                                                                \
  extern "C" int name##_impl(__VA_ARGS__);                                                     \
  LIBSORT_EXPORT bool name(__VA_ARGS__) __attribute__((alias(#name "_impl")));                 \
  extern "C" int name##_impl(__VA_ARGS__)

namespace lsort {

// ---------------------------------------------------------------------------
// errors
// ---------------------------------------------------------------------------
static thread_local std::string t_last_error;

void set_error(const std::string& msg) {
  t_last_error = msg;
  fprintf(stderr, "libsort: %s\n", msg.c_str());
}
const char* last_error() { return t_last_error.c_str(); }

static bool hip_ok(hipError_t e, const char* what) {
  if (e == hipSuccess) return true;
  set_error(std::string(what) + ": " + hipGetErrorString(e));
  (void)hipGetLastError();  // clear the sticky-free error state
  return false;
}

// ---------------------------------------------------------------------------
// workspaces (one per device, created lazily, reused across calls)
// ---------------------------------------------------------------------------
static std::mutex g_ws_mu;
static std::vector<std::unique_ptr<Workspace>> g_ws;

Workspace* workspace_for(int device) {
  std::lock_guard<std::mutex> lk(g_ws_mu);
  if (device < 0) return nullptr;
  if ((size_t)device >= g_ws.size()) g_ws.resize(device + 1);
  if (!g_ws[device]) {
    auto ws = std::make_unique<Workspace>();
    ws->device = device;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess) cus = 256;
    ws->num_cus = cus > 0 ? cus : 256;
    int prev = -1;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(device);
    if (hipStreamCreateWithFlags(&ws->stream, hipStreamNonBlocking) != hipSuccess) ws->stream = nullptr;
    if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
    g_ws[device] = std::move(ws);
  }
  return g_ws[device].get();
}

void release_all_workspaces() {
  std::lock_guard<std::mutex> lk(g_ws_mu);
  for (auto& w : g_ws)
    if (w) {
      std::lock_guard<std::mutex> l2(w->mu);
      w->release();
    }
}

// Cross-stream ordering of one workspace: the counters live in device memory
// and are reused by every call, so a call on stream B waits for the last
// call's work on stream A.
struct WsOrder {
  hipEvent_t evt = nullptr;
  hipStream_t last = nullptr;
  bool used = false;
};
static std::mutex g_order_mu;
static std::vector<WsOrder> g_order;

bool ws_acquire_stream(int dev, hipStream_t st) {
  std::lock_guard<std::mutex> lk(g_order_mu);
  if ((size_t)dev >= g_order.size()) g_order.resize(dev + 1);
  WsOrder& o = g_order[dev];
  // device-scope release: the event only orders libsort's own kernels on two
  // streams of one device (no L2 write-back per call)
  if (!o.evt && !hip_ok(hipEventCreateWithFlags(&o.evt, hipEventDisableTiming | hipEventReleaseToDevice),
                        "hipEventCreate"))
    return false;
  if (o.used && o.last != st) return hip_ok(hipStreamWaitEvent(st, o.evt, 0), "hipStreamWaitEvent");
  return true;
}
void ws_release_stream(int dev, hipStream_t st) {
  std::lock_guard<std::mutex> lk(g_order_mu);
  WsOrder& o = g_order[dev];
  (void)hipEventRecord(o.evt, st);
  o.last = st;
  o.used = true;
}

// ---------------------------------------------------------------------------
// timing registry
// ---------------------------------------------------------------------------
struct TimingRec {
  std::string name;
  hipEvent_t a = nullptr, b = nullptr;
  uint64_t keys = 0;
};
static std::atomic<bool> g_timing_on{false};
static std::mutex g_tmu;
static std::vector<TimingRec> g_recs;  // [0, g_nrec) recorded since the last reset; the rest keep their events
static size_t g_nrec = 0;
static std::string g_filter;  // ",name,name," (empty: every kernel)
// record only every g_every-th launch that passes the filter (1: all); a
// stride coprime to the launches per sort rotates over them (bench.py: 5 over
// the 4 digit passes of a sort), so the timed region carries fewer events
static uint32_t g_every = 1, g_seen = 0;

bool timing_enabled() { return g_timing_on.load(std::memory_order_relaxed); }
void timing_enable(bool on) { g_timing_on.store(on); }

void timing_reset() {
  std::lock_guard<std::mutex> lk(g_tmu);
  g_nrec = 0;
  g_seen = 0;
}

void timing_sample(uint32_t every) {
  std::lock_guard<std::mutex> lk(g_tmu);
  g_every = every ? every : 1;
  g_seen = 0;
}

void timing_filter(const char* csv) {
  std::lock_guard<std::mutex> lk(g_tmu);
  g_filter = (csv && *csv) ? "," + std::string(csv) + "," : std::string();
}

int timing_start(const char* name, hipStream_t st, uint64_t keys) {
  if (!timing_enabled()) return -1;
  std::lock_guard<std::mutex> lk(g_tmu);
  if (!g_filter.empty() && g_filter.find("," + std::string(name) + ",") == std::string::npos) return -1;
  if (g_seen++ % g_every != 0) return -1;
  if (g_nrec == g_recs.size()) {
    // Timestamps only: no system-scope fence at record time.  A default
    // event writes back and invalidates L2 when it is recorded (~3 us each
    // between the kernels of a sort, and the pass kernel's L2-merged output
    // lines flushed early); these events are never used to order memory.
    TimingRec r;
    if (hipEventCreateWithFlags(&r.a, hipEventDisableSystemFence) != hipSuccess) return -1;
    if (hipEventCreateWithFlags(&r.b, hipEventDisableSystemFence) != hipSuccess) {
      (void)hipEventDestroy(r.a);
      return -1;
    }
    g_recs.push_back(r);
  }
  TimingRec& r = g_recs[g_nrec];
  r.name = name;
  r.keys = keys;
  if (hipEventRecord(r.a, st) != hipSuccess) return -1;
  return (int)g_nrec++;
}

void timing_stop(int tok, hipStream_t st) {
  if (tok < 0) return;
  std::lock_guard<std::mutex> lk(g_tmu);
  if ((size_t)tok >= g_nrec) return;
  (void)hipEventRecord(g_recs[tok].b, st);
}

bool timing_query(const char* name, uint64_t* launches, double* total_ms, uint64_t* total_keys) {
  std::lock_guard<std::mutex> lk(g_tmu);
  uint64_t cnt = 0, keys = 0;
  double ms = 0.0;
  for (size_t i = 0; i < g_nrec; ++i) {
    const TimingRec& r = g_recs[i];
    if (r.name != name) continue;
    if (hipEventSynchronize(r.b) != hipSuccess) return false;
    float t = 0.f;
    if (hipEventElapsedTime(&t, r.a, r.b) != hipSuccess) return false;
    ms += t;
    ++cnt;
    keys += r.keys;
  }
  if (launches) *launches = cnt;
  if (total_ms) *total_ms = ms;
  if (total_keys) *total_keys = keys;
  return true;
}

// ---------------------------------------------------------------------------
// device pool (utils.cu:10-61, utils.h:19-68)
// ---------------------------------------------------------------------------
class Semaphore {
 public:
  explicit Semaphore(int n) : count_(n) {}
  void down() {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return count_ > 0; });
    --count_;
  }
  void up() {
    std::lock_guard<std::mutex> lk(mu_);
    ++count_;
    cv_.notify_one();
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  int count_;
};

static std::mutex g_init_mu;
static int g_ndev = 0;
static std::atomic_flag* g_dev_locks = nullptr;
static Semaphore* g_dev_sem = nullptr;

// RAII reservation of one pool device; releases slot and flag on destruction.
class Reservation {
 public:
  ~Reservation() { release(); }
  bool reserve() {
    if (!g_dev_sem) {
      set_error("initLibSort() must be called before using the GPU entry points");
      return false;
    }
    g_dev_sem->down();
    for (int i = 0; i < g_ndev; ++i) {
      if (!g_dev_locks[i].test_and_set()) {
        hipError_t e = hipSetDevice(i);
        if (e != hipSuccess) {
          // the reference leaks the slot here (utils.cu:49-53); give it back
          g_dev_locks[i].clear();
          g_dev_sem->up();
          return hip_ok(e, "hipSetDevice");
        }
        dev_ = i;
        return true;
      }
    }
    g_dev_sem->up();
    set_error("failed to find an available device (pool invariant broken)");
    return false;
  }
  int device() const { return dev_; }

 private:
  void release() {
    if (dev_ >= 0) {
      g_dev_locks[dev_].clear();
      g_dev_sem->up();
      dev_ = -1;
    }
  }
  int dev_ = -1;
};

// RAII reservation of k pool devices for one multi-GPU call.  Multi-device
// reservations are serialised (two of them each holding part of the pool
// cannot wait on each other); single-device callers keep taking devices as
// they free up.
static std::mutex g_multi_mu;
class MultiReservation {
 public:
  ~MultiReservation() {
    for (int d : devs_) {
      g_dev_locks[d].clear();
      g_dev_sem->up();
    }
  }
  bool reserve(int k) {
    if (!g_dev_sem) {
      set_error("initLibSort() must be called before using the GPU entry points");
      return false;
    }
    if (k < 1 || k > g_ndev) {
      set_error("gpuDistribSort: ngpu must be in [1, " + std::to_string(g_ndev) + "] (the device pool)");
      return false;
    }
    std::lock_guard<std::mutex> lk(g_multi_mu);
    for (int j = 0; j < k; ++j) {
      g_dev_sem->down();
      int got = -1;
      for (int i = 0; i < g_ndev && got < 0; ++i)
        if (!g_dev_locks[i].test_and_set()) got = i;
      if (got < 0) {
        g_dev_sem->up();
        set_error("failed to find an available device (pool invariant broken)");
        return false;
      }
      devs_.push_back(got);
    }
    std::sort(devs_.begin(), devs_.end());
    return true;
  }
  const std::vector<int>& devices() const { return devs_; }

 private:
  std::vector<int> devs_;
};

// ---------------------------------------------------------------------------
// configuration
// ---------------------------------------------------------------------------
static int env_digit_bits() {
  const char* s = getenv("LIBSORT_DIGIT_BITS");
  if (!s) return 8;
  int b = atoi(s);
  return (b == 4 || b == 8) ? b : 8;
}
static std::atomic<int> g_digit_bits{env_digit_bits()};

static int env_algorithm() {
  const char* s = getenv("LIBSORT_ALGO");
  if (!s) return 0;
  switch (s[0]) {
    case 'o': case 'O': return 1;
    case 'r': case 'R': return 2;
    case 't': case 'T': return 3;
    default: return 0;
  }
}
static std::atomic<int> g_algorithm{env_algorithm()};

// gpuPartial boundaries: 0 = the exclusive prefix of group counts (what every
// reference caller and test expects, tests.cpp:41-83, distrib.go:45-52), 1 =
// the reference's GetBoundaries output bit for bit, quirk included
// (sort.cu:367-394; boundaries.h).  LIBSORT_BOUNDARIES=reference selects 1.
static int env_boundary_mode() {
  const char* s = getenv("LIBSORT_BOUNDARIES");
  return (s && (s[0] == 'r' || s[0] == 'R' || s[0] == '1')) ? 1 : 0;
}
static std::atomic<int> g_boundary_mode{env_boundary_mode()};

// MSD hybrid for full 32-bit key sorts (sort_hybrid_u32): 0 = off, 1 = auto
// (2^27 <= n <= 2^28 + 2^24), 2 = every full sort of n >= 1024 keys (tests).
// Initial value from LIBSORT_HYBRID (0 / 1 / 2; default 1).
static int env_hybrid() {
  const char* s = getenv("LIBSORT_HYBRID");
  return (s && s[0] >= '0' && s[0] <= '2') ? s[0] - '0' : 1;
}
static std::atomic<int> g_hybrid{env_hybrid()};
int get_hybrid_mode() { return g_hybrid.load(std::memory_order_relaxed); }
int set_hybrid_mode(int m) {
  if (m < 0 || m > 2) return -1;
  return g_hybrid.exchange(m);
}

// On-chip sort of the hybrid's buckets for 32-bit keys without values:
// 1 = the counting placement (12-bit cells + 4-bit residual counts), 0 = the
// 4-bit LSD steps.  Initial value from LIBSORT_BUCKET_COUNT (default 1).
static int env_bucket_mode() {
  const char* s = getenv("LIBSORT_BUCKET_COUNT");
  return (s && s[0] == '0') ? 0 : 1;
}
static std::atomic<int> g_bucket_mode{env_bucket_mode()};
int get_bucket_mode() { return g_bucket_mode.load(std::memory_order_relaxed); }
int set_bucket_mode(int m) {
  if (m < 0 || m > 1) return -1;
  return g_bucket_mode.exchange(m);
}

int get_algorithm() { return g_algorithm.load(std::memory_order_relaxed); }
int set_algorithm(int a) {
  if (a < 0 || a > 3) return -1;
  return g_algorithm.exchange(a);
}

// ---------------------------------------------------------------------------
// PCG32 host generator (utils.cu:65-80); state persists across calls
// ---------------------------------------------------------------------------
static std::mutex g_pcg_mu;
static uint64_t g_pcg_state = kPcgInit;

static inline uint32_t rotr32(uint32_t x, uint32_t r) { return (x >> r) | (x << ((0u - r) & 31u)); }

// ---------------------------------------------------------------------------
// host-pointer sorts
// ---------------------------------------------------------------------------
// Pipelined full sort of a host buffer (providedGpu).
// The host ABI is PCIe-bound (measured on the box, tools/pcie_probe: 1 GiB
// moves in ~19 ms each way, pageable and pinned alike, ~97 GB/s when both
// directions run at once), so the sort itself is hidden behind the two
// transfers:
//   1. H2D in kPipeChunks chunks on the copy stream; chunk c is partitioned
//      (stable, by a 12-bit top-bucket table -> kPipeGroups contiguous key
//      ranges) on the compute stream while chunk c+1 is in flight.  The table
//      comes from the histogram of chunk 0 (balance only; sizes are exact).
//   2. After the last chunk: one small D2H of the chunk bucket starts, then
//      per key range g (in key order): gather its chunk pieces into one
//      contiguous slice at its final position (segment copy), sort the slice
//      in place with the range-restricted sort (digits of key - lo), and D2H
//      it on the copy stream while range g+1 is gathered and sorted.
// Critical path: H2D + partition of the last chunk + gather/sort of range 0 +
// D2H, instead of H2D + whole sort + D2H.  Bit-identical result (a full sort
// is unique).
constexpr int kPipeChunks = 4, kPipeChunksMax = 16;   // LIBSORT_PIPE_CHUNKS
constexpr int kPipeGroups = 8, kPipeGroupsMax = 32;   // LIBSORT_PIPE_GROUPS (A/B knobs; tools/host_pipe_ab.py)
constexpr int kPlanBits = 12;
static_assert(kPipeChunksMax + kPipeGroupsMax <= Workspace::kPipeEvents, "events");
static_assert(3 * kPipeChunksMax * kPipeGroupsMax * 2 <= 3 * 2 * 1024, "segment tables");
static_assert(kPipeChunksMax * kPipeGroupsMax <= 1024, "chunk bucket starts");

static int env_int(const char* name, int dflt, int lo, int hi) {
  const char* s = getenv(name);
  if (!s) return dflt;
  const int v = atoi(s);
  return v < lo ? lo : v > hi ? hi : v;
}

static size_t env_pipeline_min() {
  const char* s = getenv("LIBSORT_HOST_PIPELINE_MIN");  // keys; 0 disables the pipeline
  if (!s) return (size_t)1 << 22;
  const long long v = atoll(s);
  return v <= 0 ? (size_t)-1 : (size_t)v;
}

// LIBSORT_PIPE_DEBUG=1: synchronise and check after every step (diagnostics).
static bool pipe_checkpoint(const char* step, hipStream_t a, hipStream_t b) {
  static const bool on = [] {
    const char* s = getenv("LIBSORT_PIPE_DEBUG");
    return s && s[0] == '1';
  }();
  if (!on) return true;
  hipError_t e1 = hipStreamSynchronize(a), e2 = hipStreamSynchronize(b);
  if (e1 != hipSuccess || e2 != hipSuccess) {
    fprintf(stderr, "libsort pipeline: fault after step %s: %s\n", step,
            hipGetErrorString(e1 != hipSuccess ? e1 : e2));
    return false;
  }
  fprintf(stderr, "libsort pipeline: ok after %s\n", step);
  return true;
}

static bool host_full_sort_pipelined(Workspace* ws, uint32_t* h, size_t len, int bits) {
  static const int NCH = env_int("LIBSORT_PIPE_CHUNKS", kPipeChunks, 1, kPipeChunksMax);
  static const int NG = env_int("LIBSORT_PIPE_GROUPS", kPipeGroups, 2, kPipeGroupsMax);
  hipStream_t st = ws->stream, cs = ws->copy_stream;
  uint32_t* b0 = static_cast<uint32_t*>(ws->hbuf[0]);
  uint32_t* b1 = static_cast<uint32_t*>(ws->hbuf[1]);
  uint32_t* b2 = static_cast<uint32_t*>(ws->pbuf);
  const size_t piece = ((len + NCH - 1) / NCH + 8191) & ~(size_t)8191;
  const int nch = (int)((len + piece - 1) / piece);
  // plan block layout (device and pinned mirror): hist[4096] | lut bytes[4096]
  // | chunk bucket starts[1024] | segment tables (uint64)
  uint32_t* d_hist = ws->plan_dev;
  uint8_t* d_lut = reinterpret_cast<uint8_t*>(ws->plan_dev + 4096);
  uint32_t* d_bnd = ws->plan_dev + 4096 + 1024;
  uint64_t* d_tab = reinterpret_cast<uint64_t*>(ws->plan_dev + 4096 + 2048);
  uint32_t* H = ws->plan_host;
  uint8_t* lut = reinterpret_cast<uint8_t*>(H + 4096);
  uint32_t* bnd = H + 4096 + 1024;
  uint64_t* tab = reinterpret_cast<uint64_t*>(H + 4096 + 2048);
  hipEvent_t* ev = ws->pipe_evt;
  uint64_t lo[kPipeGroupsMax], hi[kPipeGroupsMax];
  bool ok = true;
  for (int c = 0; ok && c < nch; ++c) {
    const size_t off = (size_t)c * piece, m = std::min(piece, len - off);
    ok = hip_ok(hipMemcpyAsync(b0 + off, h + off, m * sizeof(uint32_t), hipMemcpyHostToDevice, cs), "H2D chunk") &&
         hip_ok(hipEventRecord(ev[c], cs), "hipEventRecord") && hip_ok(hipStreamWaitEvent(st, ev[c], 0), "wait");
    if (ok && c == 0) {
      ok = hip_ok(histogram_u32(*ws, b0, m, 32 - kPlanBits, kPlanBits, d_hist, st), "plan histogram") &&
           hip_ok(hipMemcpyAsync(H, d_hist, 4096 * sizeof(uint32_t), hipMemcpyDeviceToHost, st), "D2H hist") &&
           hip_ok(hipStreamSynchronize(st), "hipStreamSynchronize");
      if (!ok) break;
      // contiguous bucket ranges of about equal (sampled) size, in key order
      uint64_t total = 0;
      for (int b = 0; b < 4096; ++b) total += H[b];
      uint64_t acc = 0;
      int prev = 0;
      for (int g = 0; g < NG; ++g) lo[g] = hi[g] = 0;
      for (int b = 0; b < 4096; ++b) {
        int g = total ? (int)((2 * acc + H[b]) * NG / (2 * total)) : 0;
        g = std::max(prev, std::min(g, NG - 1));
        if (hi[g] == 0) lo[g] = (uint64_t)b << (32 - kPlanBits);
        hi[g] = (uint64_t)(b + 1) << (32 - kPlanBits);
        lut[b] = (uint8_t)g;
        prev = g;
        acc += H[b];
      }
      ok = hip_ok(hipMemcpyAsync(d_lut, lut, 4096, hipMemcpyHostToDevice, st), "H2D plan") &&
           pipe_checkpoint("plan", st, cs);
    }
    if (ok)
      ok = hip_ok(partition_lut_u32(*ws, b0 + off, b1 + off, m, d_lut, 32 - kPlanBits, NG,
                                    d_bnd + c * NG, st),
                  "chunk partition") &&
           pipe_checkpoint("chunk partition", st, cs);
  }
  if (ok)
    ok = hip_ok(hipMemcpyAsync(bnd, d_bnd, (size_t)nch * NG * sizeof(uint32_t), hipMemcpyDeviceToHost, st),
                "D2H bucket starts") &&
         hip_ok(hipStreamSynchronize(st), "hipStreamSynchronize");
  if (!ok) {
    (void)hipStreamSynchronize(cs);
    (void)hipStreamSynchronize(st);
    return false;
  }
  uint64_t sz[kPipeChunksMax][kPipeGroupsMax], T[kPipeGroupsMax], G[kPipeGroupsMax], maxlen[kPipeGroupsMax];
  uint64_t run = 0;
  for (int g = 0; g < NG; ++g) {
    T[g] = maxlen[g] = 0;
    for (int c = 0; c < nch; ++c) {
      const uint64_t m = std::min(piece, len - (size_t)c * piece);
      const uint64_t end = g + 1 < NG ? bnd[c * NG + g + 1] : m;
      sz[c][g] = end - bnd[c * NG + g];
      T[g] += sz[c][g];
      maxlen[g] = std::max(maxlen[g], sz[c][g]);
    }
    G[g] = run;
    run += T[g];
  }
  for (int g = 0; g < NG; ++g) {
    uint64_t* t = tab + (size_t)g * 3 * nch;
    uint64_t dst = G[g];
    for (int c = 0; c < nch; ++c) {
      t[c] = (uint64_t)c * piece + bnd[c * NG + g];
      t[nch + c] = dst;
      t[2 * nch + c] = sz[c][g];
      dst += sz[c][g];
      // a malformed table would fault the gather: check it on the host
      if (t[c] + sz[c][g] > std::min<uint64_t>((uint64_t)(c + 1) * piece, len) || dst > len) {
        set_error("pipelined sort: inconsistent chunk bucket starts");
        return false;
      }
    }
  }
  if (run != len) {
    set_error("pipelined sort: bucket sizes do not add up");
    return false;
  }
  ok = hip_ok(hipMemcpyAsync(d_tab, tab, (size_t)NG * 3 * nch * sizeof(uint64_t), hipMemcpyHostToDevice, st),
              "H2D segment tables");
  // every range's gather + sort is queued before the first D2H (a pageable
  // D2H may hold the host thread until it is done)
  for (int g = 0; ok && g < NG; ++g) {
    if (!T[g]) continue;
    const uint64_t span = hi[g] - lo[g] - 1;
    int width = 0;
    while (width < 32 && (span >> width) != 0) ++width;
    ok = hip_ok(segment_copy_dev_u32(b1, b2, d_tab + (size_t)g * 3 * nch, nch, maxlen[g], T[g], st),
                "range gather") &&
         pipe_checkpoint("range gather", st, cs) &&
         hip_ok(sort_u32(*ws, b2 + G[g], b2 + G[g], b0 + G[g], T[g], 0, std::max(width, 1), bits, nullptr, st,
                         (uint32_t)lo[g]),
                "range sort") &&
         pipe_checkpoint("range sort", st, cs) &&
         hip_ok(hipEventRecord(ev[kPipeChunksMax + g], st), "hipEventRecord");
  }
  for (int g = 0; ok && g < NG; ++g) {
    if (!T[g]) continue;
    ok = hip_ok(hipStreamWaitEvent(cs, ev[kPipeChunksMax + g], 0), "wait") &&
         hip_ok(hipMemcpyAsync(h + G[g], b2 + G[g], T[g] * sizeof(uint32_t), hipMemcpyDeviceToHost, cs), "D2H range") &&
         pipe_checkpoint("D2H range", st, cs);
  }
  const bool synced = hip_ok(hipStreamSynchronize(cs), "hipStreamSynchronize") &&
                      hip_ok(hipStreamSynchronize(st), "hipStreamSynchronize");
  return ok && synced;
}

static bool host_sort(uint32_t* h, uint32_t* bounds, size_t len, uint32_t offset, uint32_t width,
                      bool partial) {
  Reservation res;
  if (!res.reserve()) return false;
  if (len > 0xffffffffull) {
    set_error("Input array length must be less than 2^32");
    return false;
  }
  if (partial) {
    if (width > 31 || offset > 32 || offset + width > 32) {
      set_error("gpuPartial: need width <= 31 and offset + width <= 32");
      return false;
    }
    if (!bounds) {
      set_error("gpuPartial: boundaries must not be NULL");
      return false;
    }
  }
  const uint32_t ngroups = partial ? (1u << width) : 0u;
  if (len == 0 || (partial && width == 0)) {
    if (partial) std::fill(bounds, bounds + ngroups, 0u);
    return true;
  }
  Workspace* ws = workspace_for(res.device());
  if (!ws) return false;
  std::lock_guard<std::mutex> lk(ws->mu);
  hipStream_t st = ws->stream;
  if (!ws_acquire_stream(ws->device, st)) return false;
  const int bits = g_digit_bits.load();
  const size_t bytes = len * sizeof(uint32_t);
  static const size_t pipe_min = env_pipeline_min();
  if (!partial && len >= pipe_min) {
    bool ok = hip_ok(ws->ensure_hbuf(bytes), "hipMalloc(keys)") &&
              hip_ok(ws->ensure_pipeline(bytes), "hipMalloc(pipeline)") &&
              host_full_sort_pipelined(ws, h, len, bits);
    ws_release_stream(ws->device, st);
    return ok;
  }
  const int lo = partial ? (int)offset : 0;
  const int hi = partial ? (int)(offset + width) : 32;
  const int P = num_passes(hi - lo, bits);
  bool ok = hip_ok(ws->ensure_hbuf(bytes), "hipMalloc(keys)");
  if (ok && partial) ok = hip_ok(ws->ensure_bounds(ngroups), "hipMalloc(boundaries)");
  if (ok) ok = hip_ok(hipMemcpyAsync(ws->hbuf[0], h, bytes, hipMemcpyHostToDevice, st), "H2D copy");
  uint32_t* b0 = static_cast<uint32_t*>(ws->hbuf[0]);
  uint32_t* b1 = static_cast<uint32_t*>(ws->hbuf[1]);
  // Odd pass count: hbuf0 -> hbuf1 first, result in hbuf1, hbuf0 is scratch.
  uint32_t* out = host_result_in_second(P) ? b1 : b0;
  uint32_t* tmp = host_result_in_second(P) ? b0 : b1;
  if (ok)
    ok = hip_ok(sort_u32(*ws, b0, out, tmp, len, lo, hi, bits, partial ? ws->dbounds : nullptr, st),
                "radix sort");
  if (ok) ok = hip_ok(hipMemcpyAsync(h, out, bytes, hipMemcpyDeviceToHost, st), "D2H copy");
  if (ok && partial)
    ok = hip_ok(hipMemcpyAsync(bounds, ws->dbounds, (size_t)ngroups * sizeof(uint32_t),
                               hipMemcpyDeviceToHost, st),
                "D2H boundaries");
  ws_release_stream(ws->device, st);
  if (ok) ok = hip_ok(hipStreamSynchronize(st), "hipStreamSynchronize");
  if (ok && partial && g_boundary_mode.load() == 1) reference_boundaries_from_prefix(bounds, ngroups, len);
  return ok;
}

static hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Runs fn(workspace) for the caller's current device with cross-stream
// ordering of the workspace.
template <typename Fn>
static bool with_current_ws(hipStream_t st, Fn fn) {
  int dev = -1;
  if (!hip_ok(hipGetDevice(&dev), "hipGetDevice")) return false;
  Workspace* ws = workspace_for(dev);
  if (!ws) {
    set_error("no workspace for current device");
    return false;
  }
  std::lock_guard<std::mutex> lk(ws->mu);
  if (!ws_acquire_stream(dev, st)) return false;
  bool ok = fn(*ws);
  ws_release_stream(dev, st);
  return ok;
}

}  // namespace lsort

using namespace lsort;

// ===========================================================================
// Part 1: reference ABI
// ===========================================================================
LS_BOOL_ENTRY(initLibSort, void) {
  std::lock_guard<std::mutex> lk(g_init_mu);
  if (g_dev_locks != nullptr) {
    set_error("attempted to initialize multiple times!");
    return 0;
  }
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess || n <= 0) {
    set_error(std::string("Failed to get device count: ") +
              (e != hipSuccess ? hipGetErrorString(e) : "no HIP device"));
    (void)hipGetLastError();
    return 0;
  }
  if (const char* s = getenv("LIBSORT_NGPU")) {
    int lim = atoi(s);
    if (lim > 0 && lim < n) n = lim;
  }
  g_ndev = n;
  g_dev_locks = new std::atomic_flag[n];
  for (int i = 0; i < n; ++i) g_dev_locks[i].clear();
  g_dev_sem = new Semaphore(n);
  return 1;
}

LS_BOOL_ENTRY(gpuPartial, uint32_t* h_in, uint32_t* boundaries, size_t h_in_len, uint32_t offset,
                              uint32_t width) {
  return host_sort(h_in, boundaries, h_in_len, offset, width, true) ? 1 : 0;
}

LS_BOOL_ENTRY(providedGpu, unsigned int* h_in, size_t len) {
  return host_sort(h_in, nullptr, len, 0, 32, false) ? 1 : 0;
}

LS_BOOL_ENTRY(providedCpu, unsigned int* in, size_t len) {
  std::sort(in, in + len);
  return 1;
}

LIBSORT_EXPORT void populateInput(uint32_t* arr, size_t nelem) {
  std::lock_guard<std::mutex> lk(g_pcg_mu);  // the reference state is unguarded (utils.cu:67)
  uint64_t state = g_pcg_state;
  for (size_t i = 0; i < nelem; ++i) {
    uint64_t x = state;
    const uint32_t count = (uint32_t)(x >> 59);
    state = x * kPcgMult + kPcgInc;
    x ^= x >> 18;
    arr[i] = rotr32((uint32_t)(x >> 27), count);
  }
  g_pcg_state = state;
}

LS_BOOL_ENTRY(gpuPartialProfile, uint32_t* h_in, uint32_t* boundaries, size_t h_in_len,
                                     uint32_t offset, uint32_t width) {
  roctxRangePush("gpuPartialProfile");
  int r = gpuPartial(h_in, boundaries, h_in_len, offset, width);
  roctxRangePop();
  return r;
}

LS_BOOL_ENTRY(providedGpuProfile, unsigned int* h_in, size_t h_in_len) {
  roctxRangePush("providedGpuProfile");
  int r = providedGpu(h_in, h_in_len);
  roctxRangePop();
  return r;
}

// ===========================================================================
// Part 2: additive API
// ===========================================================================
LS_BOOL_ENTRY(gpuFullSort, unsigned int* h_in, size_t len) { return providedGpu(h_in, len); }

LS_BOOL_ENTRY(gpuPartialSort, uint32_t* h_in, uint32_t* boundaries, size_t h_in_len, uint32_t offset,
                                  uint32_t width) {
  return gpuPartial(h_in, boundaries, h_in_len, offset, width);
}

static bool check_range(size_t n, uint32_t offset, uint32_t width, uint32_t keybits) {
  if (n > 0xffffffffull) {
    set_error("at most 2^32-1 elements per call");
    return false;
  }
  if (offset > keybits || width > keybits || offset + width > keybits) {
    set_error("bit range outside the key");
    return false;
  }
  return true;
}

LS_BOOL_ENTRY(libsortSortKeysU32, const uint32_t* d_in, uint32_t* d_out, uint32_t* d_tmp, size_t n,
                                      uint32_t offset, uint32_t width, uint32_t* d_boundaries,
                                      void* stream) {
  if (!check_range(n, offset, width, 32)) return 0;
  if (d_boundaries && width > 31) {
    set_error("boundaries need width <= 31");
    return 0;
  }
  if (n > 0 && (!d_in || !d_out || !d_tmp || d_tmp == d_out || (const uint32_t*)d_tmp == d_in)) {
    set_error("libsortSortKeysU32: need distinct d_tmp (d_in may equal d_out)");
    return 0;
  }
  hipStream_t st = as_stream(stream);
  return with_current_ws(st, [&](Workspace& ws) {
           return hip_ok(sort_u32(ws, d_in, d_out, d_tmp, n, (int)offset, (int)(offset + width),
                                  g_digit_bits.load(), d_boundaries, st),
                         "libsortSortKeysU32");
         })
             ? 1
             : 0;
}

LS_BOOL_ENTRY(libsortSortKeysRangeU32, const uint32_t* d_in, uint32_t* d_out, uint32_t* d_tmp, size_t n,
                                           uint32_t lo, uint64_t hi, void* stream) {
  if (hi <= (uint64_t)lo || hi > (1ull << 32)) {
    set_error("libsortSortKeysRangeU32: need lo < hi <= 2^32");
    return 0;
  }
  if (n > 0 && (!d_in || !d_out || !d_tmp || d_tmp == d_out || (const uint32_t*)d_tmp == d_in)) {
    set_error("libsortSortKeysRangeU32: need distinct d_tmp (d_in may equal d_out)");
    return 0;
  }
  // bits of the largest key - lo: keys are ordered by the low `width` bits of key - lo
  const uint64_t span = hi - lo - 1;
  int width = 0;
  while (width < 32 && (span >> width) != 0) ++width;
  hipStream_t st = as_stream(stream);
  return with_current_ws(st, [&](Workspace& ws) {
           return hip_ok(sort_u32(ws, d_in, d_out, d_tmp, n, 0, width, g_digit_bits.load(), nullptr, st, lo, true,
                                  hi - lo),
                         "libsortSortKeysRangeU32");
         })
             ? 1
             : 0;
}

LS_BOOL_ENTRY(libsortSortPiecesU32, const uint32_t* d_in, uint32_t* d_out, uint32_t* d_tmp, size_t n,
              const uint64_t* off, const uint64_t* len, const uint32_t* seg, size_t npieces, uint32_t nseg,
              uint32_t bits, void* stream) {
  if (n > 0 && (!d_in || !d_out || !d_tmp || d_out == d_in || d_tmp == d_out || (const uint32_t*)d_tmp == d_in ||
                !off || !len || !seg)) {
    set_error("libsortSortPiecesU32: need d_in, d_out, d_tmp distinct and the three piece tables");
    return 0;
  }
  hipStream_t st = as_stream(stream);
  return with_current_ws(st, [&](Workspace& ws) {
           return hip_ok(sort_pieces_u32(ws, d_in, d_out, d_tmp, n, off, len, seg, npieces, nseg, (int)bits,
                                         g_digit_bits.load(), st),
                         "libsortSortPiecesU32 (pieces in segment order, seg < nseg, lengths summing to n)");
         })
             ? 1
             : 0;
}

LS_BOOL_ENTRY(libsortSortPairsU64U32, const uint64_t* d_kin, const uint32_t* d_vin, uint64_t* d_kout,
                                          uint32_t* d_vout, uint64_t* d_ktmp, uint32_t* d_vtmp, size_t n,
                                          uint32_t offset, uint32_t width, void* stream) {
  if (!check_range(n, offset, width, 64)) return 0;
  if (n > 0 && (d_ktmp == d_kout || (const uint64_t*)d_ktmp == d_kin || d_vtmp == d_vout ||
                (const uint32_t*)d_vtmp == d_vin)) {
    set_error("libsortSortPairsU64U32: scratch buffers must not alias input/output");
    return 0;
  }
  hipStream_t st = as_stream(stream);
  return with_current_ws(st, [&](Workspace& ws) {
           return hip_ok(sort_pairs_u64_u32(ws, d_kin, d_vin, d_kout, d_vout, d_ktmp, d_vtmp, n,
                                            (int)offset, (int)(offset + width), g_digit_bits.load(), st),
                         "libsortSortPairsU64U32");
         })
             ? 1
             : 0;
}

LS_BOOL_ENTRY(libsortSortKeysU64, const uint64_t* d_in, uint64_t* d_out, uint64_t* d_tmp, size_t n,
                                      uint32_t offset, uint32_t width, void* stream) {
  if (!check_range(n, offset, width, 64)) return 0;
  if (n > 0 && (!d_in || !d_out || !d_tmp || d_tmp == d_out || (const uint64_t*)d_tmp == d_in)) {
    set_error("libsortSortKeysU64: need distinct d_tmp (d_in may equal d_out)");
    return 0;
  }
  hipStream_t st = as_stream(stream);
  return with_current_ws(st, [&](Workspace& ws) {
           return hip_ok(sort_u64(ws, d_in, d_out, d_tmp, n, (int)offset, (int)(offset + width),
                                  g_digit_bits.load(), st),
                         "libsortSortKeysU64");
         })
             ? 1
             : 0;
}

LS_BOOL_ENTRY(libsortSortPairsU64U64, const uint64_t* d_kin, const uint64_t* d_vin, uint64_t* d_kout,
                                          uint64_t* d_vout, uint64_t* d_ktmp, uint64_t* d_vtmp, size_t n,
                                          uint32_t offset, uint32_t width, void* stream) {
  if (!check_range(n, offset, width, 64)) return 0;
  if (n > 0 && (d_ktmp == d_kout || (const uint64_t*)d_ktmp == d_kin || d_vtmp == d_vout ||
                (const uint64_t*)d_vtmp == d_vin)) {
    set_error("libsortSortPairsU64U64: scratch buffers must not alias input/output");
    return 0;
  }
  hipStream_t st = as_stream(stream);
  return with_current_ws(st, [&](Workspace& ws) {
           return hip_ok(sort_pairs_u64_u64(ws, d_kin, d_vin, d_kout, d_vout, d_ktmp, d_vtmp, n,
                                            (int)offset, (int)(offset + width), g_digit_bits.load(), st),
                         "libsortSortPairsU64U64");
         })
             ? 1
             : 0;
}

LS_BOOL_ENTRY(libsortSortPairsU32U32, const uint32_t* d_kin, const uint32_t* d_vin, uint32_t* d_kout,
                                          uint32_t* d_vout, uint32_t* d_ktmp, uint32_t* d_vtmp, size_t n,
                                          uint32_t offset, uint32_t width, void* stream) {
  if (!check_range(n, offset, width, 32)) return 0;
  if (n > 0 && (d_ktmp == d_kout || (const uint32_t*)d_ktmp == d_kin || d_vtmp == d_vout ||
                (const uint32_t*)d_vtmp == d_vin)) {
    set_error("libsortSortPairsU32U32: scratch buffers must not alias input/output");
    return 0;
  }
  hipStream_t st = as_stream(stream);
  return with_current_ws(st, [&](Workspace& ws) {
           return hip_ok(sort_pairs_u32_u32(ws, d_kin, d_vin, d_kout, d_vout, d_ktmp, d_vtmp, n,
                                            (int)offset, (int)(offset + width), g_digit_bits.load(), st),
                         "libsortSortPairsU32U32");
         })
             ? 1
             : 0;
}

LS_BOOL_ENTRY(libsortHistogramU32, const uint32_t* d_keys, size_t n, uint32_t shift, uint32_t bits,
                                       uint32_t* d_hist, void* stream) {
  hipStream_t st = as_stream(stream);
  return with_current_ws(st, [&](Workspace& ws) {
           return hip_ok(histogram_u32(ws, d_keys, n, (int)shift, (int)bits, d_hist, st),
                         "libsortHistogramU32");
         })
             ? 1
             : 0;
}

LS_BOOL_ENTRY(libsortPartitionU32, const uint32_t* d_in, uint32_t* d_out, size_t n,
                                       const uint32_t* splitters, uint32_t nsplit, uint32_t* d_counts,
                                       void* stream) {
  if (nsplit > 0 && !splitters) {
    set_error("libsortPartitionU32: splitters must not be NULL");
    return 0;
  }
  if (n > 0 && (const uint32_t*)d_out == d_in) {
    set_error("libsortPartitionU32: out of place only");
    return 0;
  }
  hipStream_t st = as_stream(stream);
  return with_current_ws(st, [&](Workspace& ws) {
           return hip_ok(partition_u32(ws, d_in, d_out, n, splitters, (int)nsplit, d_counts, st),
                         "libsortPartitionU32");
         })
             ? 1
             : 0;
}

LS_BOOL_ENTRY(libsortPartitionLutU32, const uint32_t* d_in, uint32_t* d_out, size_t n, const uint8_t* d_lut,
                                          uint32_t lut_shift, uint32_t nbuckets, uint32_t* d_bounds,
                                          void* stream) {
  if (n > 0 && (const uint32_t*)d_out == d_in) {
    set_error("libsortPartitionLutU32: out of place only");
    return 0;
  }
  hipStream_t st = as_stream(stream);
  return with_current_ws(st, [&](Workspace& ws) {
           return hip_ok(partition_lut_u32(ws, d_in, d_out, n, d_lut, (int)lut_shift, (int)nbuckets, d_bounds, st),
                         "libsortPartitionLutU32");
         })
             ? 1
             : 0;
}

LS_BOOL_ENTRY(libsortPartitionLutU64U32, const uint64_t* d_kin, const uint32_t* d_vin, uint64_t* d_kout,
                                             uint32_t* d_vout, size_t n, const uint8_t* d_lut, uint32_t lut_shift,
                                             uint32_t nbuckets, uint32_t* d_bounds, void* stream) {
  hipStream_t st = as_stream(stream);
  return with_current_ws(st, [&](Workspace& ws) {
           return hip_ok(partition_lut_pairs_u64_u32(ws, d_kin, d_vin, d_kout, d_vout, n, d_lut, (int)lut_shift,
                                                     (int)nbuckets, d_bounds, st),
                         "libsortPartitionLutU64U32");
         })
             ? 1
             : 0;
}

LS_BOOL_ENTRY(libsortPartitionLutCountU32, const uint32_t* d_in, size_t n, const uint8_t* d_lut,
                                               uint32_t lut_shift, uint32_t nbuckets, uint32_t* d_bounds,
                                               void* stream) {
  hipStream_t st = as_stream(stream);
  return with_current_ws(st, [&](Workspace& ws) {
           return hip_ok(partition_lut_u32(ws, d_in, nullptr, n, d_lut, (int)lut_shift, (int)nbuckets, d_bounds, st,
                                           kPartCount),
                         "libsortPartitionLutCountU32");
         })
             ? 1
             : 0;
}

LS_BOOL_ENTRY(libsortPartitionLutScatterU32, const uint32_t* d_in, uint32_t* d_out, size_t n, const uint8_t* d_lut,
                                                 uint32_t lut_shift, uint32_t nbuckets, void* stream) {
  if (n > 0 && (const uint32_t*)d_out == d_in) {
    set_error("libsortPartitionLutScatterU32: out of place only");
    return 0;
  }
  hipStream_t st = as_stream(stream);
  return with_current_ws(st, [&](Workspace& ws) {
           return hip_ok(partition_lut_u32(ws, d_in, d_out, n, d_lut, (int)lut_shift, (int)nbuckets, nullptr, st,
                                           kPartScatter),
                         "libsortPartitionLutScatterU32 (needs the matching count call just before it)");
         })
             ? 1
             : 0;
}

LS_BOOL_ENTRY(libsortPartitionLutCountU64U32, const uint64_t* d_kin, const uint32_t* d_vin, size_t n,
                                                  const uint8_t* d_lut, uint32_t lut_shift, uint32_t nbuckets,
                                                  uint32_t* d_bounds, void* stream) {
  hipStream_t st = as_stream(stream);
  return with_current_ws(st, [&](Workspace& ws) {
           return hip_ok(partition_lut_pairs_u64_u32(ws, d_kin, d_vin, nullptr, nullptr, n, d_lut, (int)lut_shift,
                                                     (int)nbuckets, d_bounds, st, kPartCount),
                         "libsortPartitionLutCountU64U32");
         })
             ? 1
             : 0;
}

LS_BOOL_ENTRY(libsortPartitionLutScatterU64U32, const uint64_t* d_kin, const uint32_t* d_vin, uint64_t* d_kout,
                                                    uint32_t* d_vout, size_t n, const uint8_t* d_lut,
                                                    uint32_t lut_shift, uint32_t nbuckets, void* stream) {
  hipStream_t st = as_stream(stream);
  return with_current_ws(st, [&](Workspace& ws) {
           return hip_ok(partition_lut_pairs_u64_u32(ws, d_kin, d_vin, d_kout, d_vout, n, d_lut, (int)lut_shift,
                                                     (int)nbuckets, nullptr, st, kPartScatter),
                         "libsortPartitionLutScatterU64U32 (needs the matching count call just before it)");
         })
             ? 1
             : 0;
}

// The range-digit partitions (distrib.cpp's re-partition of narrow key
// ranges, exported for pylibsort.distrib): the table partitions' kernels
// with a BiasedDigit op.
static bool range_shift_ok(uint32_t shift, int key_bits, const char* who) {
  if ((int)shift > key_bits - 8) {
    set_error(std::string(who) + ": shift must be <= key bits - 8");
    return false;
  }
  return true;
}

LS_BOOL_ENTRY(libsortPartitionRangeCountU32, const uint32_t* d_in, size_t n, uint32_t bias, uint32_t shift,
              uint32_t* d_bounds, void* stream) {
  if (!range_shift_ok(shift, 32, "libsortPartitionRangeCountU32")) return 0;
  hipStream_t st = as_stream(stream);
  return with_current_ws(st, [&](Workspace& ws) {
           return hip_ok(partition_range_u32(ws, d_in, nullptr, n, bias, (int)shift, d_bounds, st, kPartCount),
                         "libsortPartitionRangeCountU32");
         })
             ? 1
             : 0;
}

LS_BOOL_ENTRY(libsortPartitionRangeScatterU32, const uint32_t* d_in, uint32_t* d_out, size_t n, uint32_t bias,
              uint32_t shift, void* stream) {
  if (!range_shift_ok(shift, 32, "libsortPartitionRangeScatterU32")) return 0;
  if (n > 0 && (const uint32_t*)d_out == d_in) {
    set_error("libsortPartitionRangeScatterU32: out of place only");
    return 0;
  }
  hipStream_t st = as_stream(stream);
  return with_current_ws(st, [&](Workspace& ws) {
           return hip_ok(partition_range_u32(ws, d_in, d_out, n, bias, (int)shift, nullptr, st, kPartScatter),
                         "libsortPartitionRangeScatterU32 (needs the matching count call just before it)");
         })
             ? 1
             : 0;
}

LS_BOOL_ENTRY(libsortPartitionRangeCountU64U32, const uint64_t* d_kin, const uint32_t* d_vin, size_t n,
              uint64_t bias, uint32_t shift, uint32_t* d_bounds, void* stream) {
  if (!range_shift_ok(shift, 64, "libsortPartitionRangeCountU64U32")) return 0;
  hipStream_t st = as_stream(stream);
  return with_current_ws(st, [&](Workspace& ws) {
           return hip_ok(partition_range_pairs_u64_u32(ws, d_kin, d_vin, nullptr, nullptr, n, bias, (int)shift,
                                                       d_bounds, st, kPartCount),
                         "libsortPartitionRangeCountU64U32");
         })
             ? 1
             : 0;
}

LS_BOOL_ENTRY(libsortPartitionRangeScatterU64U32, const uint64_t* d_kin, const uint32_t* d_vin, uint64_t* d_kout,
              uint32_t* d_vout, size_t n, uint64_t bias, uint32_t shift, void* stream) {
  if (!range_shift_ok(shift, 64, "libsortPartitionRangeScatterU64U32")) return 0;
  hipStream_t st = as_stream(stream);
  return with_current_ws(st, [&](Workspace& ws) {
           return hip_ok(partition_range_pairs_u64_u32(ws, d_kin, d_vin, d_kout, d_vout, n, bias, (int)shift, nullptr,
                                                       st, kPartScatter),
                         "libsortPartitionRangeScatterU64U32 (needs the matching count call just before it)");
         })
             ? 1
             : 0;
}

LS_BOOL_ENTRY(libsortMinMaxU32, const uint32_t* d_keys, size_t n, uint32_t* d_minmax, void* stream) {
  if (!d_minmax || (n > 0 && !d_keys)) {
    set_error("libsortMinMaxU32: bad arguments");
    return 0;
  }
  hipStream_t st = as_stream(stream);
  return with_current_ws(st, [&](Workspace& ws) {
           return hip_ok(minmax_u32(ws, d_keys, n, d_minmax, st), "libsortMinMaxU32");
         })
             ? 1
             : 0;
}

LS_BOOL_ENTRY(libsortMinMaxU64, const uint64_t* d_keys, size_t n, uint64_t* d_minmax, void* stream) {
  if (!d_minmax || (n > 0 && !d_keys)) {
    set_error("libsortMinMaxU64: bad arguments");
    return 0;
  }
  hipStream_t st = as_stream(stream);
  return with_current_ws(st, [&](Workspace& ws) {
           return hip_ok(minmax_u64(ws, d_keys, n, d_minmax, st), "libsortMinMaxU64");
         })
             ? 1
             : 0;
}

LS_BOOL_ENTRY(libsortSortPiecesRangeU32, const uint32_t* d_in, uint32_t* d_out, uint32_t* d_tmp, size_t n,
              const uint64_t* off, const uint64_t* len, const uint32_t* seg, size_t npieces, uint32_t nseg,
              uint32_t bits, uint32_t bias, void* stream) {
  if (n > 0 && (!d_in || !d_out || !d_tmp || d_out == d_in || d_tmp == d_out || (const uint32_t*)d_tmp == d_in ||
                !off || !len || !seg)) {
    set_error("libsortSortPiecesRangeU32: need d_in, d_out, d_tmp distinct and the three piece tables");
    return 0;
  }
  hipStream_t st = as_stream(stream);
  return with_current_ws(st, [&](Workspace& ws) {
           return hip_ok(sort_pieces_u32(ws, d_in, d_out, d_tmp, n, off, len, seg, npieces, nseg, (int)bits,
                                         g_digit_bits.load(), st, bias),
                         "libsortSortPiecesRangeU32 (pieces in segment order, seg < nseg, lengths summing to n)");
         })
             ? 1
             : 0;
}

LS_BOOL_ENTRY(libsortSegmentCopyU32, const uint32_t* d_src, uint32_t* d_dst, size_t nseg,
                                         const uint64_t* src_off, const uint64_t* dst_off,
                                         const uint64_t* len, void* stream) {
  hipStream_t st = as_stream(stream);
  return with_current_ws(st, [&](Workspace& ws) {
           return hip_ok(segment_copy_u32(ws, d_src, d_dst, nseg, src_off, dst_off, len, st),
                         "libsortSegmentCopyU32");
         })
             ? 1
             : 0;
}

LS_BOOL_ENTRY(libsortDeltaMaxGapU32, const uint32_t* d_keys, size_t n, uint32_t* d_maxgap, void* stream) {
  if (!d_maxgap || (n > 0 && !d_keys)) {
    set_error("libsortDeltaMaxGapU32: bad arguments");
    return 0;
  }
  return hip_ok(delta_maxgap_u32(d_keys, n, d_maxgap, as_stream(stream)), "libsortDeltaMaxGapU32") ? 1 : 0;
}

LS_BOOL_ENTRY(libsortDeltaPackU32, const uint32_t* d_keys, size_t n, const uint32_t* d_maxgap, uint32_t* d_out,
                                       void* stream) {
  if (!d_maxgap || (n > 0 && (!d_keys || !d_out))) {
    set_error("libsortDeltaPackU32: bad arguments");
    return 0;
  }
  return hip_ok(delta_pack_u32(d_keys, n, d_maxgap, d_out, as_stream(stream)), "libsortDeltaPackU32") ? 1 : 0;
}

LS_BOOL_ENTRY(libsortDeltaUnpackU32, const uint32_t* d_in, size_t n, uint32_t bits, uint32_t* d_keys,
                                         void* stream) {
  if (bits > 32 || (n > 0 && (!d_in || !d_keys))) {
    set_error("libsortDeltaUnpackU32: bad arguments");
    return 0;
  }
  return hip_ok(delta_unpack_u32(d_in, n, bits, d_keys, as_stream(stream)), "libsortDeltaUnpackU32") ? 1 : 0;
}

LS_BOOL_ENTRY(libsortMergeU32, const uint32_t* d_a, size_t na, const uint32_t* d_b, size_t nb, uint32_t* d_out,
                                   void* stream) {
  if ((na > 0 && !d_a) || (nb > 0 && !d_b) || (na + nb > 0 && !d_out) || (d_out && (d_out == d_a || d_out == d_b))) {
    set_error("libsortMergeU32: bad arguments (out must be distinct from both inputs)");
    return 0;
  }
  return hip_ok(merge_u32(d_a, na, d_b, nb, d_out, as_stream(stream)), "libsortMergeU32") ? 1 : 0;
}

LS_BOOL_ENTRY(libsortPopulateDevice, uint32_t* d_out, size_t n, uint64_t first, void* stream) {
  return hip_ok(populate_device(d_out, n, first, as_stream(stream)), "libsortPopulateDevice") ? 1 : 0;
}

LIBSORT_EXPORT int libsortSetDigitBits(int bits) {
  if (bits != 4 && bits != 8) return -1;
  return g_digit_bits.exchange(bits);
}

LIBSORT_EXPORT int libsortGetDigitBits(void) { return g_digit_bits.load(); }

LIBSORT_EXPORT int libsortSetAlgorithm(int algo) { return set_algorithm(algo); }
LIBSORT_EXPORT int libsortSetHybrid(int mode) { return set_hybrid_mode(mode); }
LIBSORT_EXPORT int libsortSetBucketMode(int mode) { return set_bucket_mode(mode); }

LIBSORT_EXPORT int libsortSetBoundaryMode(int mode) {
  if (mode != 0 && mode != 1) return -1;
  return g_boundary_mode.exchange(mode);
}

LIBSORT_EXPORT void libsortTimingEnable(bool on) { timing_enable(on); }
LIBSORT_EXPORT void libsortTimingReset(void) { timing_reset(); }
LIBSORT_EXPORT void libsortTimingFilter(const char* kernels) { timing_filter(kernels); }
LIBSORT_EXPORT void libsortTimingSample(uint32_t every) { timing_sample(every); }
LS_BOOL_ENTRY(libsortTimingQuery, const char* kernel, uint64_t* launches, double* total_ms,
                                      uint64_t* total_keys) {
  return timing_query(kernel, launches, total_ms, total_keys) ? 1 : 0;
}

LS_BOOL_ENTRY(libsortDistribPlanDigits, const int64_t* counts, uint32_t nranks, uint32_t rounds, double growth,
              uint8_t* lut, int64_t* est) {
  if (!counts || !lut || !est || nranks < 1 || rounds < 1 || (uint64_t)nranks * rounds > 256 || !(growth > 0.0)) {
    set_error("libsortDistribPlanDigits: need the tables, 1 <= nranks * rounds <= 256 and growth > 0");
    return 0;
  }
  std::vector<std::vector<uint64_t>> C(nranks, std::vector<uint64_t>(dplan::kTopDigits));
  for (uint32_t r = 0; r < nranks; ++r)
    for (int g = 0; g < dplan::kTopDigits; ++g) {
      const int64_t v = counts[(size_t)r * dplan::kTopDigits + g];
      if (v < 0) {
        set_error("libsortDistribPlanDigits: negative count");
        return 0;
      }
      C[r][g] = (uint64_t)v;
    }
  dplan::plan_digit_rounds(C, (int)rounds, growth, lut, est);
  return 1;
}

LS_BOOL_ENTRY(libsortDistribLastBytes, int nranks, uint64_t* per_rank) {
  if (nranks < 1 || !per_rank || !distrib_last_bytes(per_rank, nranks)) {
    set_error("libsortDistribLastBytes: no distributed sort over nranks ranks has run");
    return 0;
  }
  return 1;
}

LIBSORT_EXPORT int libsortSetDistribTrace(int on) { return set_distrib_trace(on ? 1 : 0); }

LS_BOOL_ENTRY(libsortDistribOverlapProbe, int nranks, const int* devices, uint32_t spin_us, double* ms) {
  if (nranks < 1 || !devices || !ms || spin_us == 0 || spin_us > 10000000u) {
    set_error("libsortDistribOverlapProbe: need nranks >= 1, devices, ms[4] and 0 < spin_us <= 10 s");
    return 0;
  }
  int ndev = 0;
  if (!hip_ok(hipGetDeviceCount(&ndev), "hipGetDeviceCount")) return 0;
  for (int r = 0; r < nranks; ++r)
    if (devices[r] < 0 || devices[r] >= ndev) {
      set_error("libsortDistribOverlapProbe: device out of range");
      return 0;
    }
  int prev = -1;
  (void)hipGetDevice(&prev);
  const bool ok = distrib_overlap_probe(devices, nranks, spin_us, ms);
  if (prev >= 0) (void)hipSetDevice(prev);
  return ok ? 1 : 0;
}

LS_BOOL_ENTRY(libsortDistribRangeDigit, uint64_t lo, uint64_t hi, uint32_t key_bits, uint64_t* bias,
              uint32_t* shift) {
  if (!bias || !shift || (key_bits != 32 && key_bits != 64)) {
    set_error("libsortDistribRangeDigit: need bias, shift and key_bits 32 or 64");
    return 0;
  }
  int sh = 0;
  const bool useful = dplan::range_digit(lo, hi, (int)key_bits, bias, &sh);
  *shift = (uint32_t)sh;
  return useful ? 1 : 0;
}

LS_BOOL_ENTRY(gpuDistribSort, uint32_t* h_in, size_t len, int ngpu) {
  MultiReservation res;
  if (!res.reserve(ngpu <= 0 ? g_ndev : ngpu)) return 0;
  if (len == 0) return 1;
  if (!h_in) {
    set_error("gpuDistribSort: h_in must not be NULL");
    return 0;
  }
  const std::vector<int>& d = res.devices();
  return distrib_sort_host_u32(h_in, len, d.data(), (int)d.size(), 0u, g_digit_bits.load()) ? 1 : 0;
}

LS_BOOL_ENTRY(libsortDistribSortU32, int nranks, const int* devices, const uint32_t* const* d_in,
                                         const size_t* n_in, uint32_t* const* d_out, size_t* n_out, uint32_t flags) {
  if (nranks < 1 || !devices || !d_in || !n_in || !d_out || !n_out) {
    set_error("libsortDistribSortU32: need nranks >= 1 and non-NULL tables");
    return 0;
  }
  if (flags & ~(kDistribLsd | kDistribCopy | kDistribSelfRccl | kDistribWire32 | kDistribCoded)) {
    set_error("libsortDistribSortU32: unknown flags");
    return 0;
  }
  int ndev = 0;
  if (!hip_ok(hipGetDeviceCount(&ndev), "hipGetDeviceCount")) return 0;
  for (int r = 0; r < nranks; ++r)
    if (devices[r] < 0 || devices[r] >= ndev) {
      set_error("libsortDistribSortU32: device out of range");
      return 0;
    }
  int prev = -1;
  (void)hipGetDevice(&prev);
  const bool ok = distrib_sort_u32(devices, nranks, d_in, n_in, d_out, n_out, flags, g_digit_bits.load());
  if (prev >= 0) (void)hipSetDevice(prev);
  return ok ? 1 : 0;
}

LS_BOOL_ENTRY(libsortDistribSortPairsU64U32, int nranks, const int* devices, const uint64_t* const* d_kin,
              const uint32_t* const* d_vin, const size_t* n_in, uint64_t* const* d_kout, uint32_t* const* d_vout,
              size_t* n_out, uint32_t flags) {
  if (nranks < 1 || !devices || !d_kin || !d_vin || !n_in || !d_kout || !d_vout || !n_out) {
    set_error("libsortDistribSortPairsU64U32: need nranks >= 1 and non-NULL tables");
    return 0;
  }
  if (flags & ~(kDistribCopy | kDistribSelfRccl)) {
    set_error("libsortDistribSortPairsU64U32: unknown flags (LSD rounds are for keys only)");
    return 0;
  }
  int ndev = 0;
  if (!hip_ok(hipGetDeviceCount(&ndev), "hipGetDeviceCount")) return 0;
  for (int r = 0; r < nranks; ++r)
    if (devices[r] < 0 || devices[r] >= ndev) {
      set_error("libsortDistribSortPairsU64U32: device out of range");
      return 0;
    }
  int prev = -1;
  (void)hipGetDevice(&prev);
  const bool ok = distrib_sort_pairs_u64_u32(devices, nranks, d_kin, d_vin, n_in, d_kout, d_vout, n_out, flags,
                                             g_digit_bits.load());
  if (prev >= 0) (void)hipSetDevice(prev);
  return ok ? 1 : 0;
}

LS_BOOL_ENTRY(libsortReleaseWorkspace, void) {
  distrib_release();
  release_all_workspaces();
  return 1;
}

LIBSORT_EXPORT const char* libsortLastError(void) { return last_error(); }

// Synchronises the current device and returns (then clears) the device-side
// error word of its workspace: bit 0 = a look-back spin hit its bound.
LIBSORT_EXPORT uint32_t libsortDeviceErrors(void) {
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess) return 0xffffffffu;
  Workspace* ws = workspace_for(dev);
  if (!ws) return 0xffffffffu;
  std::lock_guard<std::mutex> lk(ws->mu);
  if (!ws->os_small) return 0;
  uint32_t v = 0;
  if (hipDeviceSynchronize() != hipSuccess) return 0xffffffffu;
  if (hipMemcpy(&v, ws->os_small + kOsErr, sizeof(v), hipMemcpyDeviceToHost) != hipSuccess) return 0xffffffffu;
  if (v) (void)hipMemset(ws->os_small + kOsErr, 0, sizeof(uint32_t));
  return v;
}
