// distrib.cpp -- the multi-GPU sort behind the C ABI (libsort.h
// gpuDistribSort / libsortDistribSortU32): one process drives R ranks, one
// per GPU, over a single-process RCCL communicator (ncclCommInitAll over the
// ranks' devices, xGMI point-to-point), so C and Go callers reach the
// sharded sort without torch.distributed.
//
// Replaces the reference's distributed drivers, whose exchange goes through
// host memory (localTest/benchmarks.cpp:70-160, two std::async gpuPartial
// callers and a host shuffle) or files (benchmark/pkg/sort/distrib.go:90-179,
// GpuPartial workers, libsort.go:47-67).  Two schedules with the same final
// state -- rank r holds keys [r*S, (r+1)*S) of the sorted whole, S =
// ceil(N/R), the reference's equal re-cut (distrib.go:113):
//
//   top-digit rounds (default): per rank a stable partition by the top 8
//     key bits (the reference's gpuPartial(offset 24, width 8) building
//     block, split in a count and a scatter call) whose 256 exact bucket
//     counts go to the host while the scatter runs; ONE host plan of (rank,
//     round) digit ranges (distrib_plan.h plan_digit_rounds, the same plan
//     pylibsort.distrib runs); K exchange rounds issued up front on each
//     rank's communication stream; each round sorted into its slice of the
//     rank's output as soon as it has arrived, straight from the received
//     (source, digit) pieces (sort_pieces_u32: no gather, no pass over the
//     top digit), overlapping the later rounds' exchange -- the round sorts
//     of different devices are issued by one host thread per device, so one
//     device's host read-backs never hold another's; then the equal re-cut
//     moves the few surplus keys.  Falls back to the LSD rounds when one
//     digit range would overload a rank (identical decision for all).
//     (u64 key, u32 payload) pairs (configs[4], distrib_sort_pairs_u64_u32)
//     take the same rounds on the key's top 8 bits with a stable pair sort
//     per round.
//   LSD rounds (LIBSORT_DISTRIB_LSD): the reference's BSP semantics -- per
//     8-bit digit a stable local partial sort (gpuPartial on the device), the
//     bucket counts to the host, one exchange of contiguous slices and a
//     segment gather into bucket-major / rank-minor order; after every round
//     rank r holds exactly the reference's worker-r chunk.
//
// Ranks may share a device (tests on a one-GPU box): their work is then
// serialised on that device's streams and exchanges between them are device
// copies (RCCL refuses two ranks on one GPU).  LIBSORT_DISTRIB_COPY makes
// every exchange a peer copy (hipMemcpyPeerAsync) instead of RCCL.
//
// All host arithmetic lives in distrib_plan.h, which the CPU simulation test
// (tests/cpp/distrib_sim.cpp, under ASan/UBSan) runs against the oracle.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>  // types only: the functions are resolved with dlsym
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "distrib_plan.h"
#include "radix.h"

namespace lsort {

namespace {

bool ok_hip(hipError_t e, const char* what) {
  if (e == hipSuccess) return true;
  set_error(std::string("distributed sort: ") + what + ": " + hipGetErrorString(e));
  (void)hipGetLastError();
  return false;
}

// ---------------------------------------------------------------------------
// Stage trace (libsortSetDistribTrace / LIBSORT_DISTRIB_TRACE=1): one stderr
// line per stage, so that a multi-GPU run that hangs names the stage it
// stopped at.  While tracing, the round sorts wait on the
// host for their round's arrival and completion (serialised: diagnostics).
// ---------------------------------------------------------------------------
std::atomic<int> g_trace{[] {
  const char* e = getenv("LIBSORT_DISTRIB_TRACE");
  return e && e[0] == '1' ? 1 : 0;
}()};
std::mutex g_trace_mu;
std::chrono::steady_clock::time_point g_trace_t0 = std::chrono::steady_clock::now();

bool tracing() { return g_trace.load(std::memory_order_relaxed) != 0; }

__attribute__((format(printf, 1, 2))) void trace(const char* fmt, ...) {
  if (!tracing()) return;
  const double ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - g_trace_t0).count();
  std::lock_guard<std::mutex> lk(g_trace_mu);
  fprintf(stderr, "libsort distrib [%9.3f ms] ", ms);
  va_list ap;
  va_start(ap, fmt);
  vfprintf(stderr, fmt, ap);
  va_end(ap);
  fputc('\n', stderr);
  fflush(stderr);
}

void trace_start() { g_trace_t0 = std::chrono::steady_clock::now(); }

// ---------------------------------------------------------------------------
// RCCL, loaded on first use: libsort.so does not link it, so callers that
// never sort across GPUs do not load it.  An RCCL already in the process
// (torch's, in a Python process) is reused, otherwise the image's
// librccl.so.1 (LIBSORT_RCCL_PATH overrides).
// ---------------------------------------------------------------------------
struct Rccl {
  decltype(&ncclCommInitAll) commInitAll = nullptr;
  decltype(&ncclCommDestroy) commDestroy = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGroupStart) groupStart = nullptr;
  decltype(&ncclGroupEnd) groupEnd = nullptr;
  decltype(&ncclGetErrorString) errorString = nullptr;
  bool loaded = false;

  bool load() {
    if (loaded) return true;
    void* h = nullptr;
    if (const char* p = getenv("LIBSORT_RCCL_PATH")) h = dlopen(p, RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      set_error(std::string("distributed sort: cannot load RCCL: ") + dlerror());
      return false;
    }
#define LS_SYM(field, name)                                             \
  field = reinterpret_cast<decltype(field)>(dlsym(h, name));            \
  if (!field) {                                                         \
    set_error("distributed sort: RCCL lacks " name);                    \
    return false;                                                       \
  }
    LS_SYM(commInitAll, "ncclCommInitAll")
    LS_SYM(commDestroy, "ncclCommDestroy")
    LS_SYM(send, "ncclSend")
    LS_SYM(recv, "ncclRecv")
    LS_SYM(groupStart, "ncclGroupStart")
    LS_SYM(groupEnd, "ncclGroupEnd")
    LS_SYM(errorString, "ncclGetErrorString")
#undef LS_SYM
    loaded = true;
    return true;
  }
  bool ok(ncclResult_t r, const char* what) {
    if (r == ncclSuccess) return true;
    set_error(std::string("distributed sort: ") + what + ": " + errorString(r));
    return false;
  }
};
Rccl g_rccl;

// grow-only device buffer of one device
struct DBuf {
  void* p = nullptr;
  size_t cap = 0;  // bytes
  int dev = -1;
  bool ensure(int device, size_t bytes) {
    if (bytes <= cap && dev == device) return true;
    if (p) {
      (void)hipSetDevice(dev);
      (void)hipFree(p);
      p = nullptr;
      cap = 0;
    }
    const size_t want = std::max<size_t>(bytes + bytes / 16, 4096);  // slack: sizes vary call to call
    if (!ok_hip(hipSetDevice(device), "hipSetDevice") || !ok_hip(hipMalloc(&p, want), "hipMalloc")) return false;
    cap = want;
    dev = device;
    return true;
  }
  void release() {
    if (p) {
      (void)hipSetDevice(dev);
      (void)hipFree(p);
    }
    p = nullptr;
    cap = 0;
  }
  uint32_t* u32() const { return static_cast<uint32_t*>(p); }
};

constexpr int kMaxRounds = 4;
constexpr int kMaxParts = 2;  // partition parts per rank (partition_top)

struct DevState {
  int dev = -1;
  Workspace* ws = nullptr;
  hipStream_t st = nullptr;  // compute
  hipStream_t cs = nullptr;  // exchanges
  hipEvent_t ev_comm = nullptr, ev_comp = nullptr;
  DBuf lut;        // the identity table of the 256 top digits (partition by key >> 24)
  DBuf tmp, tmpv;  // round-sort scratch (keys; pair payloads)
};

struct RankState {
  int dev = -1;
  DevState* d = nullptr;
  DBuf bounds, part, pv, recv, rv, outb, ov, alt;  // pv / rv / ov: pair payloads
  DBuf mm;                                          // smallest and largest key (range partition)
  DBuf csend, crecv, mg, mtmp;                      // coded rounds: coded pieces out / in, largest gaps, merge levels
  DBuf hin, hout;  // staging of the host-pointer entry point
  uint64_t pn = 0;  // keys in `part` (24-bit planes: the 8-bit plane starts at byte 2 * pn)
  hipEvent_t ev_part = nullptr, ev_bounds = nullptr, ev_done = nullptr;
  hipEvent_t ev_part0 = nullptr;  // the first partition part written (two parts: partition_top)
  hipEvent_t ev_x[kMaxRounds] = {};
  hipEvent_t ev_c[kMaxRounds] = {};  // coded rounds: round i sorted and coded (largest gaps on the host)
};

struct Ctx {
  std::vector<int> devs;                       // device of each rank
  std::vector<std::unique_ptr<DevState>> uniq;  // one per distinct device
  std::vector<RankState> ranks;
  std::vector<ncclComm_t> comms;               // RCCL communicator of each rank (distinct devices only)
  uint32_t* h_bounds = nullptr;                // pinned: R x kMaxParts x 256 bucket starts
  uint64_t* h_mm = nullptr;                    // pinned: R x (min, max) keys
  uint32_t* h_mg = nullptr;                    // pinned: R x (R * kMaxRounds) largest gaps (coded rounds)
  bool distinct = false;
  std::vector<uint64_t> sent;                  // bytes each rank sent to others in the last sort

  ~Ctx() {
    for (ncclComm_t c : comms)
      if (c && g_rccl.loaded) (void)g_rccl.commDestroy(c);
    for (auto& r : ranks) {
      for (DBuf* b : {&r.bounds, &r.part, &r.pv, &r.recv, &r.rv, &r.outb, &r.ov, &r.alt, &r.mm, &r.hin, &r.hout,
                      &r.csend, &r.crecv, &r.mg, &r.mtmp})
        b->release();
      (void)hipSetDevice(r.dev);
      for (hipEvent_t e : {r.ev_part, r.ev_bounds, r.ev_done, r.ev_part0})
        if (e) (void)hipEventDestroy(e);
      for (hipEvent_t e : r.ev_x)
        if (e) (void)hipEventDestroy(e);
      for (hipEvent_t e : r.ev_c)
        if (e) (void)hipEventDestroy(e);
    }
    for (auto& u : uniq) {
      u->lut.release();
      u->tmp.release();
      u->tmpv.release();
      (void)hipSetDevice(u->dev);
      if (u->st) (void)hipStreamDestroy(u->st);
      if (u->cs) (void)hipStreamDestroy(u->cs);
      if (u->ev_comm) (void)hipEventDestroy(u->ev_comm);
      if (u->ev_comp) (void)hipEventDestroy(u->ev_comp);
    }
    if (h_bounds) (void)hipHostFree(h_bounds);
    if (h_mm) (void)hipHostFree(h_mm);
    if (h_mg) (void)hipHostFree(h_mg);
  }

  bool init(const std::vector<int>& d) {
    devs = d;
    const int R = (int)d.size();
    std::map<int, DevState*> by_dev;
    static const uint8_t kIdentity[dplan::kTopDigits] = {
#define LS_I4(x) x, x + 1, x + 2, x + 3
#define LS_I16(x) LS_I4(x), LS_I4(x + 4), LS_I4(x + 8), LS_I4(x + 12)
#define LS_I64(x) LS_I16(x), LS_I16(x + 16), LS_I16(x + 32), LS_I16(x + 48)
        LS_I64(0), LS_I64(64), LS_I64(128), LS_I64(192)
#undef LS_I64
#undef LS_I16
#undef LS_I4
    };
    for (int dev : d) {
      if (by_dev.count(dev)) continue;
      auto u = std::make_unique<DevState>();
      u->dev = dev;
      u->ws = workspace_for(dev);
      if (!u->ws || !ok_hip(hipSetDevice(dev), "hipSetDevice") ||
          !ok_hip(hipStreamCreateWithFlags(&u->st, hipStreamNonBlocking), "hipStreamCreate") ||
          !ok_hip(hipStreamCreateWithFlags(&u->cs, hipStreamNonBlocking), "hipStreamCreate") ||
          !ok_hip(hipEventCreateWithFlags(&u->ev_comm, hipEventDisableTiming), "hipEventCreate") ||
          !ok_hip(hipEventCreateWithFlags(&u->ev_comp, hipEventDisableTiming), "hipEventCreate") ||
          !u->lut.ensure(dev, dplan::kTopDigits) ||
          !ok_hip(hipMemcpy(u->lut.p, kIdentity, dplan::kTopDigits, hipMemcpyHostToDevice), "H2D digit table"))
        return false;
      by_dev[dev] = u.get();
      uniq.push_back(std::move(u));
    }
    distinct = (int)uniq.size() == R;
    ranks.resize(R);
    for (int r = 0; r < R; ++r) {
      RankState& s = ranks[r];
      s.dev = d[r];
      s.d = by_dev[d[r]];
      if (!ok_hip(hipSetDevice(s.dev), "hipSetDevice")) return false;
      for (hipEvent_t* e : {&s.ev_part, &s.ev_bounds, &s.ev_done, &s.ev_part0})
        if (!ok_hip(hipEventCreateWithFlags(e, hipEventDisableTiming), "hipEventCreate")) return false;
      for (hipEvent_t& e : s.ev_x)
        if (!ok_hip(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate")) return false;
      for (hipEvent_t& e : s.ev_c)
        if (!ok_hip(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate")) return false;
      if (!s.mg.ensure(s.dev, (size_t)R * kMaxRounds * sizeof(uint32_t))) return false;
      if (!s.bounds.ensure(s.dev, kMaxParts * dplan::kTopDigits * 4) || !s.mm.ensure(s.dev, 2 * sizeof(uint64_t)))
        return false;
    }
    return ok_hip(hipHostMalloc(&h_bounds, (size_t)R * kMaxParts * dplan::kTopDigits * sizeof(uint32_t), 0),
                  "hipHostMalloc") &&
           ok_hip(hipHostMalloc(&h_mm, (size_t)R * 2 * sizeof(uint64_t), 0), "hipHostMalloc") &&
           ok_hip(hipHostMalloc(&h_mg, (size_t)R * R * kMaxRounds * sizeof(uint32_t), 0), "hipHostMalloc");
  }

  bool ensure_comms() {
    if (!comms.empty()) return true;
    if (!g_rccl.load()) return false;
    comms.assign(devs.size(), nullptr);
    trace("RCCL: ncclCommInitAll over %zu devices", devs.size());
    const bool ok = g_rccl.ok(g_rccl.commInitAll(comms.data(), (int)devs.size(), devs.data()), "ncclCommInitAll");
    trace("RCCL: communicators %s", ok ? "ready" : "FAILED");
    return ok;
  }
};

std::mutex g_dist_mu;  // one distributed sort at a time (it holds several devices' workspaces)
std::unique_ptr<Ctx> g_ctx;

// Moves the pieces: rank p.src's src[p.src] + src_off -> rank p.dst's
// dst[p.dst] + dst_off (offsets and counts in elements of `esize` bytes: 4 or
// 8), on the communication streams.  A piece within one device is a device
// copy (unless self_rccl); across devices RCCL point-to-point (one group for
// the whole set) or, with `copy`, a peer copy pulled by the receiver.
bool move_pieces(Ctx& c, const std::vector<dplan::Piece>& ps, const std::vector<const void*>& src,
                 const std::vector<void*>& dst, size_t esize, bool use_rccl, bool self_rccl, bool count = true) {
  // (1- and 2-byte elements: the 24-bit key planes, sent as bytes)
  const ncclDataType_t dt = esize == 8 ? ncclUint64 : esize == 4 ? ncclUint32 : ncclUint8;
  const uint64_t per = esize >= 4 ? 1 : esize;  // RCCL elements per element
  auto at = [esize](const void* base, uint64_t off) { return static_cast<const char*>(base) + off * esize; };
  auto atw = [esize](void* base, uint64_t off) { return static_cast<char*>(base) + off * esize; };
  std::vector<const dplan::Piece*> net;
  if (c.sent.size() != c.ranks.size()) c.sent.assign(c.ranks.size(), 0);
  for (const dplan::Piece& p : ps) {
    if (!p.count) continue;
    RankState& a = c.ranks[p.src];
    RankState& b = c.ranks[p.dst];
    const size_t bytes = p.count * esize;
    if (count && p.src != p.dst) c.sent[p.src] += bytes;
    if (use_rccl && (p.src != p.dst || self_rccl)) {
      net.push_back(&p);
    } else if (a.dev == b.dev) {
      if (!ok_hip(hipSetDevice(b.dev), "hipSetDevice") ||
          !ok_hip(hipMemcpyAsync(atw(dst[p.dst], p.dst_off), at(src[p.src], p.src_off), bytes,
                                 hipMemcpyDeviceToDevice, b.d->cs),
                  "device copy"))
        return false;
    } else {
      if (!ok_hip(hipSetDevice(b.dev), "hipSetDevice") ||
          !ok_hip(hipMemcpyPeerAsync(atw(dst[p.dst], p.dst_off), b.dev, at(src[p.src], p.src_off), a.dev, bytes,
                                     b.d->cs),
                  "peer copy"))
        return false;
    }
  }
  if (net.empty()) return true;
  // RCCL point-to-point messages are cut into chunks of at most 256 MiB:
  // measured on the one-GPU box (RCCL 2.26.6, torch's build), a 2 GiB
  // self-send of u64 keys arrived intact only up to its first 1 GiB
  // (tools/debug_pairs.py); both sides post the chunks in the same order
  constexpr uint64_t kChunkBytes = 256ull << 20;
  const uint64_t chunk = kChunkBytes / esize;
  if (!g_rccl.ok(g_rccl.groupStart(), "ncclGroupStart")) return false;
  bool ok = true;
  for (const dplan::Piece* p : net) {
    RankState& a = c.ranks[p->src];
    RankState& b = c.ranks[p->dst];
    for (uint64_t o = 0; ok && o < p->count; o += chunk) {
      const uint64_t m = std::min(chunk, p->count - o);
      ok = g_rccl.ok(g_rccl.send(at(src[p->src], p->src_off + o), m * per, dt, p->dst, c.comms[p->src], a.d->cs),
                     "ncclSend") &&
           g_rccl.ok(g_rccl.recv(atw(dst[p->dst], p->dst_off + o), m * per, dt, p->src, c.comms[p->dst], b.d->cs),
                     "ncclRecv");
    }
  }
  return g_rccl.ok(g_rccl.groupEnd(), "ncclGroupEnd") && ok;
}

// Copy mode across devices: a peer copy is pulled on the RECEIVER's stream
// from the sender's buffer, so every compute stream waits for every device's
// communication stream before the buffers those copies read are rewritten.
bool compute_waits_all_comm(Ctx& c) {
  for (auto& u : c.uniq)
    if (!ok_hip(hipSetDevice(u->dev), "hipSetDevice") || !ok_hip(hipEventRecord(u->ev_comm, u->cs), "record"))
      return false;
  for (auto& u : c.uniq) {
    if (!ok_hip(hipSetDevice(u->dev), "hipSetDevice")) return false;
    for (auto& v : c.uniq)
      if (!ok_hip(hipStreamWaitEvent(u->st, v->ev_comm, 0), "wait")) return false;
  }
  return true;
}

// every communication stream waits for every rank's `ev` (cheap: R events)
bool comm_waits(Ctx& c, hipEvent_t RankState::*ev) {
  for (auto& u : c.uniq) {
    if (!ok_hip(hipSetDevice(u->dev), "hipSetDevice")) return false;
    for (auto& r : c.ranks)
      if (!ok_hip(hipStreamWaitEvent(u->cs, r.*ev, 0), "hipStreamWaitEvent")) return false;
  }
  return true;
}

bool sync_all(Ctx& c) {
  bool ok = true;
  for (auto& u : c.uniq) {
    ok = ok_hip(hipSetDevice(u->dev), "hipSetDevice") && ok_hip(hipStreamSynchronize(u->cs), "sync comm") &&
         ok_hip(hipStreamSynchronize(u->st), "sync compute") && ok;
  }
  return ok;
}

// The reference's BSP rounds (see the file comment).  cur: per-rank input.
bool run_lsd(Ctx& c, const std::vector<const uint32_t*>& in, const std::vector<uint64_t>& n_in,
             const std::vector<uint32_t*>& out, uint64_t S, int bits, bool use_rccl, bool self_rccl) {
  const int R = (int)c.ranks.size();
  constexpr int W = 8;
  uint64_t nmax = S;
  for (uint64_t n : n_in) nmax = std::max(nmax, n);
  for (auto& r : c.ranks)
    if (!r.part.ensure(r.dev, nmax * 4) || !r.recv.ensure(r.dev, nmax * 4) || !r.outb.ensure(r.dev, nmax * 4) ||
        !r.alt.ensure(r.dev, nmax * 4))
      return false;
  for (auto& u : c.uniq)
    if (!u->tmp.ensure(u->dev, nmax * 4)) return false;
  std::vector<const uint32_t*> cur(in);
  std::vector<uint64_t> n_cur(n_in);
  for (int step = 0; step < 32 / W; ++step) {
    // stable local partial sort by the step's digit (gpuPartial semantics)
    for (int r = 0; r < R; ++r) {
      RankState& s = c.ranks[r];
      if (!ok_hip(hipSetDevice(s.dev), "hipSetDevice")) return false;
      if (n_cur[r]) {
        ScopedTimer tm("lsdround", s.d->st, n_cur[r]);  // (the tests check which schedule ran)
        if (!ok_hip(sort_u32(*s.d->ws, cur[r], s.part.u32(), s.d->tmp.u32(), n_cur[r], step * W, step * W + W, bits,
                             s.bounds.u32(), s.d->st),
                    "local partial sort"))
          return false;
      } else if (!ok_hip(hipMemsetAsync(s.bounds.u32(), 0, 256 * 4, s.d->st), "memset")) {
        return false;
      }
      if (!ok_hip(hipMemcpyAsync(c.h_bounds + (size_t)r * 256, s.bounds.u32(), 256 * 4, hipMemcpyDeviceToHost,
                                 s.d->st),
                  "D2H bounds") ||
          !ok_hip(hipEventRecord(s.ev_part, s.d->st), "hipEventRecord"))
        return false;
    }
    trace("lsd step %d: local partial sorts issued", step);
    std::vector<std::vector<uint64_t>> C(R, std::vector<uint64_t>(256));
    for (int r = 0; r < R; ++r) {
      if (!ok_hip(hipEventSynchronize(c.ranks[r].ev_part), "hipEventSynchronize")) return false;
      const uint32_t* b = c.h_bounds + (size_t)r * 256;
      for (int g = 0; g < 256; ++g) C[r][g] = (g + 1 < 256 ? (uint64_t)b[g + 1] : n_cur[r]) - b[g];
    }
    dplan::LsdRound o = dplan::lsd_round(C, S);
    if (!comm_waits(c, &RankState::ev_part)) return false;
    std::vector<const void*> src(R);
    std::vector<void*> dst(R);
    for (int r = 0; r < R; ++r) {
      src[r] = c.ranks[r].part.p;
      dst[r] = c.ranks[r].recv.p;
    }
    trace("lsd step %d: bucket counts read, exchange of %zu pieces", step, o.pieces.size());
    if (!move_pieces(c, o.pieces, src, dst, 4, use_rccl, self_rccl)) return false;
    trace("lsd step %d: exchange issued", step);
    // gather into bucket-major / rank-minor order on the compute stream.
    // Every compute stream waits for EVERY device's communication stream: a
    // peer copy (copy mode across devices) is pulled on the receiver's stream
    // from the sender's `part`, which the sender's next partial sort rewrites
    // (write-after-read across devices).
    const bool last = step + 1 == 32 / W;
    if (!compute_waits_all_comm(c)) return false;
    for (int r = 0; r < R; ++r) {
      RankState& s = c.ranks[r];
      uint32_t* nxt = last ? out[r] : (step & 1 ? s.outb.u32() : s.alt.u32());
      if (!ok_hip(hipSetDevice(s.dev), "hipSetDevice") ||
          !ok_hip(segment_copy_u32(*s.d->ws, s.recv.u32(), nxt, o.seg_len[r].size(), o.seg_src[r].data(),
                                   o.seg_dst[r].data(), o.seg_len[r].data(), s.d->st),
                  "segment gather"))
        return false;
      cur[r] = nxt;
      n_cur[r] = o.n_next[r];
    }
    trace("lsd step %d: segment gathers issued", step);
  }
  return true;
}

}  // namespace

namespace {

// The context of this device list (rebuilt when the list changes); caller
// holds g_dist_mu.
Ctx* ctx_for(const int* devices, int R) {
  if (R < 1 || R > 64) {
    set_error("distributed sort: 1 <= ranks <= 64");
    return nullptr;
  }
  std::vector<int> devs(devices, devices + R);
  if (!g_ctx || g_ctx->devs != devs) {
    g_ctx.reset();
    auto c = std::make_unique<Ctx>();
    if (!c->init(devs)) return nullptr;
    g_ctx = std::move(c);
  }
  return g_ctx.get();
}

// Every involved workspace held (ascending device order) and its stream
// ordered after other callers' work, for the whole sort; release() syncs.
struct Hold {
  Ctx& c;
  std::vector<std::unique_lock<std::mutex>> locks;
  bool ok = true;
  explicit Hold(Ctx& cx) : c(cx) {
    std::vector<DevState*> order;
    for (auto& u : c.uniq) order.push_back(u.get());
    std::sort(order.begin(), order.end(), [](DevState* a, DevState* b) { return a->dev < b->dev; });
    for (DevState* u : order) locks.emplace_back(u->ws->mu);
    for (DevState* u : order)
      if (!ws_acquire_stream(u->dev, u->st)) ok = false;
  }
  bool finish(bool result) {
    trace("finish: waiting for every stream");
    const bool synced = sync_all(c);
    for (auto& u : c.uniq) ws_release_stream(u->dev, u->st);
    trace("done: %s", result && synced ? "ok" : last_error());
    return result && synced;
  }
};

// The partition digit of the rounds: the top 8 key bits (table partition with
// the identity table), or -- when those leave the keys in too few digits
// (a narrow key range: IDs, timestamps, keys below 2^26 at 8 ranks; ADVICE
// r03) -- the 8-bit digit (key - bias) >> shift over the populated range
// [bias = smallest key, largest key] (range partition).  Either way the
// digits are monotone in the key, so the rounds stay disjoint key ranges.
struct PartDigit {
  bool range = false;
  uint64_t bias = 0;
  int shift = dplan::kTopShift;  // keys of one digit share the bits above `shift` of key - bias
};

// Stable partition of every rank's keys (and payloads) by the digit `pd`
// into part (pv): the count call (per-tile counts + column scan) and the
// 256 bucket starts' copy to the host are queued first, then the scatter, so
// the host reads the counts while the data moves.  C[r][g] = rank r's keys
// in digit g.
// planar (keys, top digit): the scatter writes 24-bit planes into `part`
// (low 16 bits at byte 0, bits 16..23 at byte 2 * n): the top byte is the
// partition digit, which every receiver knows from its piece table, so the
// exchange moves 3 bytes per key instead of 4 (round 5).
// H = 2 parts (round 5): the rank's keys [0, cut) and
// [cut, n) (dplan::part_split) are partitioned one after the other into the
// same ranges of `part` (count, scatter, count, scatter), ev_part0 marks the
// first part written, and Cp[r * H + h] / first[r * H + h] are each part's
// digit counts and start, so the first part's exchange can run while the
// second is partitioned (run_digit_rounds).
template <typename K>
bool partition_top(Ctx& c, const std::vector<const K*>& in, const std::vector<const uint32_t*>* vin,
                   const std::vector<uint64_t>& n, std::vector<std::vector<uint64_t>>& C, const PartDigit& pd,
                   bool planar, int H, std::vector<std::vector<uint64_t>>& Cp, std::vector<uint64_t>& first) {
  const int R = (int)c.ranks.size();
  constexpr int NB = dplan::kTopDigits;
  first.assign((size_t)R * H, 0);
  for (int r = 0; r < R; ++r) {
    RankState& s = c.ranks[r];
    if (!ok_hip(hipSetDevice(s.dev), "hipSetDevice") || !s.part.ensure(s.dev, std::max<uint64_t>(n[r], 1) * sizeof(K)) ||
        (vin && !s.pv.ensure(s.dev, std::max<uint64_t>(n[r], 1) * 4)))
      return false;
    const uint8_t* lut = static_cast<const uint8_t*>(s.d->lut.p);
    Workspace& ws = *s.d->ws;
    s.pn = n[r];
    for (int h = 0; h < H; ++h) {
      const uint64_t a = H == 1 ? 0 : h == 0 ? 0 : dplan::part_split(n[r]);
      const uint64_t m = H == 1 ? n[r] : h == 0 ? dplan::part_split(n[r]) : n[r] - a;
      first[(size_t)r * H + h] = a;
      const K* ik = in[r] + a;
      const uint32_t* iv = vin ? (*vin)[r] + a : nullptr;
      uint32_t* const bnd = s.bounds.u32() + (size_t)h * NB;
      hipError_t e1, e2;
      if constexpr (sizeof(K) == 4) {
        e1 = pd.range ? partition_range_u32(ws, ik, nullptr, m, (uint32_t)pd.bias, pd.shift, bnd, s.d->st, kPartCount)
                      : partition_lut_u32(ws, ik, nullptr, m, lut, dplan::kTopShift, NB, bnd, s.d->st, kPartCount);
      } else {
        e1 = pd.range ? partition_range_pairs_u64_u32(ws, ik, iv, nullptr, nullptr, m, pd.bias, pd.shift, bnd, s.d->st,
                                                      kPartCount)
                      : partition_lut_pairs_u64_u32(ws, ik, iv, nullptr, nullptr, m, lut, dplan::kTopShift, NB, bnd,
                                                    s.d->st, kPartCount);
      }
      if (!ok_hip(e1, "partition counts") ||
          !ok_hip(hipMemcpyAsync(c.h_bounds + ((size_t)r * H + h) * NB, bnd, NB * 4, hipMemcpyDeviceToHost, s.d->st),
                  "D2H bucket starts") ||
          (h == H - 1 && !ok_hip(hipEventRecord(s.ev_bounds, s.d->st), "hipEventRecord")))
        return false;
      if constexpr (sizeof(K) == 4) {
        uint32_t* const ok = s.part.u32() + a;
        e2 = pd.range ? partition_range_u32(ws, ik, ok, m, (uint32_t)pd.bias, pd.shift, nullptr, s.d->st, kPartScatter)
             : planar ? partition_lut_planar_u32(ws, ik, static_cast<uint16_t*>(s.part.p) + a,
                                                 static_cast<uint8_t*>(s.part.p) + 2 * n[r] + a, m, lut,
                                                 dplan::kTopShift, NB, s.d->st)
                      : partition_lut_u32(ws, ik, ok, m, lut, dplan::kTopShift, NB, nullptr, s.d->st, kPartScatter);
      } else {
        uint64_t* const ok = static_cast<uint64_t*>(s.part.p) + a;
        e2 = pd.range ? partition_range_pairs_u64_u32(ws, ik, iv, ok, s.pv.u32() + a, m, pd.bias, pd.shift, nullptr,
                                                      s.d->st, kPartScatter)
                      : partition_lut_pairs_u64_u32(ws, ik, iv, ok, s.pv.u32() + a, m, lut, dplan::kTopShift, NB,
                                                    nullptr, s.d->st, kPartScatter);
      }
      if (!ok_hip(e2, "partition scatter")) return false;
      if (h == 0 && !ok_hip(hipEventRecord(s.ev_part0, s.d->st), "hipEventRecord")) return false;
    }
    if (!ok_hip(hipEventRecord(s.ev_part, s.d->st), "hipEventRecord")) return false;
  }
  trace("partition (%s digit%s, %d part%s): counts + scatter issued on %d ranks", pd.range ? "range" : "top",
        planar ? ", 24-bit planes" : "", H, H > 1 ? "s" : "", R);
  C.assign(R, std::vector<uint64_t>(NB, 0));
  Cp.assign((size_t)R * H, std::vector<uint64_t>(NB, 0));
  for (int r = 0; r < R; ++r) {
    if (!n[r]) continue;
    if (!ok_hip(hipEventSynchronize(c.ranks[r].ev_bounds), "hipEventSynchronize")) return false;
    for (int h = 0; h < H; ++h) {
      const size_t v = (size_t)r * H + h;
      const uint64_t m = (h + 1 < H ? first[v + 1] : n[r]) - first[v];  // (part h's keys)
      const uint32_t* b = c.h_bounds + v * NB;
      for (int g = 0; g < NB; ++g) {
        Cp[v][g] = m ? (g + 1 < NB ? (uint64_t)b[g + 1] : m) - b[g] : 0;
        C[r][g] += Cp[v][g];
      }
    }
  }
  trace("partition: bucket counts read");
  return true;
}

// The range digit over the keys of every rank: bias = the smallest key,
// shift = (bits of largest - smallest) - 8 (at least 0).  False on a HIP
// error; *useful = false when it would not split finer than the top digit
// (or all keys are equal).
template <typename K>
bool range_digit(Ctx& c, const std::vector<const K*>& in, const std::vector<uint64_t>& n, PartDigit& pd,
                 bool* useful) {
  const int R = (int)c.ranks.size();
  for (int r = 0; r < R; ++r) {
    RankState& s = c.ranks[r];
    if (!ok_hip(hipSetDevice(s.dev), "hipSetDevice")) return false;
    hipError_t e;
    if constexpr (sizeof(K) == 4)
      e = minmax_u32(*s.d->ws, in[r], n[r], s.mm.u32(), s.d->st);
    else
      e = minmax_u64(*s.d->ws, in[r], n[r], static_cast<uint64_t*>(s.mm.p), s.d->st);
    if (!ok_hip(e, "min/max") ||
        !ok_hip(hipMemcpyAsync(c.h_mm + 2 * (size_t)r, s.mm.p, 2 * sizeof(K), hipMemcpyDeviceToHost, s.d->st),
                "D2H min/max") ||
        !ok_hip(hipEventRecord(s.ev_bounds, s.d->st), "hipEventRecord"))
      return false;
  }
  uint64_t lo = ~0ull, hi = 0;
  for (int r = 0; r < R; ++r) {
    if (!ok_hip(hipEventSynchronize(c.ranks[r].ev_bounds), "hipEventSynchronize")) return false;
    if (!n[r]) continue;
    K mm[2];
    memcpy(mm, c.h_mm + 2 * (size_t)r, sizeof(mm));
    lo = std::min<uint64_t>(lo, mm[0]);
    hi = std::max<uint64_t>(hi, mm[1]);
  }
  // pd changes only when the range digit is used: a rejected one leaves the
  // top-digit partition's PartDigit for the rounds that follow
  PartDigit rd;
  rd.range = true;
  *useful = dplan::range_digit(lo, hi, 8 * (int)sizeof(K), &rd.bias, &rd.shift);
  if (*useful) pd = rd;
  return true;
}

// The rounds after the partition: every round's exchange issued up front on
// the communication streams, each round sorted into its slice of the rank's
// output as soon as it has arrived (keys: straight from the (source, digit)
// pieces; pairs: a stable pair sort, the pieces arriving in source order),
// then the equal re-cut into out (vout).
template <typename K>
bool run_digit_rounds(Ctx& c, const dplan::DigitPlan& p, const std::vector<K*>& out,
                      const std::vector<uint32_t*>* vout, bool use_rccl, bool self_rccl, int bits,
                      const PartDigit& pd, bool planar, int H) {
  const int R = (int)c.ranks.size(), K_ = p.K;
  const bool pairs = vout != nullptr;
  std::map<DevState*, uint64_t> round_max;
  for (int r = 0; r < R; ++r) {
    RankState& s = c.ranks[r];
    const uint64_t m = std::max<uint64_t>(p.n_recv[r], 1);
    if (!s.recv.ensure(s.dev, m * sizeof(K)) || !s.outb.ensure(s.dev, m * sizeof(K)) ||
        (pairs && (!s.rv.ensure(s.dev, m * 4) || !s.ov.ensure(s.dev, m * 4))))
      return false;
    for (int i = 0; i < K_; ++i)
      round_max[s.d] = std::max(round_max[s.d], p.roff[(size_t)r * (K_ + 1) + i + 1] - p.roff[(size_t)r * (K_ + 1) + i]);
  }
  for (auto& kv : round_max)
    if (!kv.first->tmp.ensure(kv.first->dev, std::max<uint64_t>(kv.second, 1) * sizeof(K)) ||
        (pairs && !kv.first->tmpv.ensure(kv.first->dev, std::max<uint64_t>(kv.second, 1) * 4)))
      return false;
  // (two parts: the first part's pieces wait for that part only)
  if (!comm_waits(c, H > 1 ? &RankState::ev_part0 : &RankState::ev_part)) return false;
  std::vector<const void*> src(R), vsrc(R);
  std::vector<void*> dst(R), vdst(R);
  for (int r = 0; r < R; ++r) {
    src[r] = c.ranks[r].part.p;
    dst[r] = c.ranks[r].recv.p;
    vsrc[r] = c.ranks[r].pv.p;
    vdst[r] = c.ranks[r].rv.p;
  }
  // planar: the 16-bit planes at the buffers' start, the 8-bit planes after
  // them (sender: 2 * its partition's keys; receiver: 2 * its received keys)
  std::vector<const void*> src8(R);
  std::vector<void*> dst8(R);
  if (planar)
    for (int r = 0; r < R; ++r) {
      src8[r] = static_cast<const char*>(c.ranks[r].part.p) + 2 * c.ranks[r].pn;
      dst8[r] = static_cast<char*>(c.ranks[r].recv.p) + 2 * p.n_recv[r];
    }
  // rounds inside the rank's output shard are sorted straight into it; the
  // others into outb, whose pieces move afterwards (dplan::place_rounds)
  const dplan::Placement pl = dplan::place_rounds(p.roff, p.n_recv, K_);
  // round i of every rank on device d, sorted as soon as it has arrived
  auto sort_round = [&](DevState& d, int i) -> bool {
    for (int r = 0; r < R; ++r) {
      RankState& s = c.ranks[r];
      if (s.d != &d) continue;
      const uint64_t a = p.roff[(size_t)r * (K_ + 1) + i], z = p.roff[(size_t)r * (K_ + 1) + i + 1];
      if (!ok_hip(hipStreamWaitEvent(d.st, s.ev_x[i], 0), "wait")) return false;
      if (tracing()) {
        if (!ok_hip(hipEventSynchronize(s.ev_x[i]), "hipEventSynchronize")) return false;
        trace("round %d rank %d: arrived (%llu keys)", i, r, (unsigned long long)(z - a));
      }
      if (z == a) continue;
      hipError_t e;
      const size_t q = (size_t)r * K_ + i;
      K* kdst = pl.direct[q] ? out[r] + pl.out_off[q] : static_cast<K*>(s.outb.p) + a;
      uint32_t* vdst = pairs ? (pl.direct[q] ? (*vout)[r] + pl.out_off[q] : s.ov.u32() + a) : nullptr;
      if constexpr (sizeof(K) == 4) {
        const uint32_t nsg = (uint32_t)(p.hi[(size_t)i * R + r] - p.lo[(size_t)i * R + r]);
        if (planar)
          e = sort_pieces_planar_u32(*d.ws, static_cast<const uint16_t*>(s.recv.p) + a,
                                     static_cast<const uint8_t*>(s.recv.p) + 2 * p.n_recv[r] + a,
                                     (uint32_t)p.lo[(size_t)i * R + r], kdst, d.tmp.u32(), z - a, p.p_off[q].data(),
                                     p.p_len[q].data(), p.p_seg[q].data(), p.p_off[q].size(), nsg, bits, d.st);
        else
          e = sort_pieces_u32(*d.ws, s.recv.u32() + a, kdst, d.tmp.u32(), z - a, p.p_off[q].data(),
                              p.p_len[q].data(), p.p_seg[q].data(), p.p_off[q].size(), nsg, pd.shift, bits, d.st,
                              (uint32_t)pd.bias);
      } else {
        e = sort_pairs_u64_u32(*d.ws, static_cast<uint64_t*>(s.recv.p) + a, s.rv.u32() + a, kdst, vdst,
                               static_cast<uint64_t*>(d.tmp.p), d.tmpv.u32(), z - a, 0, 64, bits, d.st);
      }
      if (!ok_hip(e, "round sort")) return false;
      if (tracing()) {
        if (!ok_hip(hipStreamSynchronize(d.st), "hipStreamSynchronize")) return false;
        trace("round %d rank %d: sorted", i, r);
      }
    }
    return true;
  };
  // Several devices: one host thread per device sorts its ranks' rounds, each
  // round as soon as this thread has issued that round's exchange (the round
  // sorts wait on the host for small read-backs; one device's waits must not
  // hold another device's issue -- ADVICE r02 -- and round 0's sorts need not
  // wait for the later rounds' exchange calls).  One device: inline, after
  // every exchange is issued.
  std::mutex mu;
  std::condition_variable cv;
  int issued = 0;
  bool stop = false;
  std::vector<std::string> err(c.uniq.size());
  std::vector<char> good(c.uniq.size(), 1);
  std::vector<std::thread> th;
  // (LIBSORT_DISTRIB_THREADS=1: the threaded path for one device too -- the
  // one-GPU test box's way into it)
  static const bool force_threads = [] {
    const char* e = getenv("LIBSORT_DISTRIB_THREADS");
    return e && e[0] == '1';
  }();
  const bool threaded = c.uniq.size() > 1 || force_threads;
  if (threaded)
    for (size_t u = 0; u < c.uniq.size(); ++u)
      th.emplace_back([&, u] {
        DevState& d = *c.uniq[u];
        bool ok = ok_hip(hipSetDevice(d.dev), "hipSetDevice");
        for (int i = 0; ok && i < K_; ++i) {
          {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return issued > i || stop; });
            if (issued <= i) break;  // the exchange failed
          }
          ok = sort_round(d, i);
        }
        if (!ok) {
          good[u] = 0;
          err[u] = last_error();
        }
      });
  // the pieces of round i that come from partition part `part` (-1: all)
  auto issue = [&](int i, int part) -> bool {
    std::vector<dplan::Piece> sel;
    const std::vector<dplan::Piece>* ps = &p.rounds[i];
    if (part >= 0) {
      for (const dplan::Piece& q : p.rounds[i])
        if (q.part == part) sel.push_back(q);
      ps = &sel;
    }
    return (planar ? move_pieces(c, *ps, src, dst, 2, use_rccl, self_rccl) &&
                         move_pieces(c, *ps, src8, dst8, 1, use_rccl, self_rccl)
                   : move_pieces(c, *ps, src, dst, sizeof(K), use_rccl, self_rccl)) &&
           (!pairs || move_pieces(c, *ps, vsrc, vdst, 4, use_rccl, self_rccl));
  };
  // round i has been issued: its arrival event, then its sorts may go
  auto issued_round = [&](int i) -> bool {
    trace("round %d: exchange issued (%zu pieces)", i, p.rounds[i].size());
    for (int r = 0; r < R; ++r) {
      RankState& s = c.ranks[r];
      if (!ok_hip(hipSetDevice(s.dev), "hipSetDevice") || !ok_hip(hipEventRecord(s.ev_x[i], s.d->cs), "record"))
        return false;
    }
    if (threaded) {
      std::lock_guard<std::mutex> lk(mu);
      issued = i + 1;
      cv.notify_all();
    }
    return true;
  };
  bool issue_ok = true;
  int next = 0;  // first round not issued yet
  if (H > 1) {
    // the first part of rounds 0 and 1 while the ranks partition their second
    // part (each link busy from the end of the first part's scatter: round 0
    // alone is shorter than the second scatter), then the second parts
    const int early = std::min(K_, 2);
    for (int i = 0; issue_ok && i < early; ++i) issue_ok = issue(i, 0);
    issue_ok = issue_ok && comm_waits(c, &RankState::ev_part);
    for (int i = 0; issue_ok && i < early; ++i) issue_ok = issue(i, 1) && issued_round(i);
    next = early;
  }
  for (int i = next; issue_ok && i < K_; ++i) issue_ok = issue(i, -1) && issued_round(i);
  if (threaded) {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
      cv.notify_all();
    }
    for (auto& t : th) t.join();
  }
  if (!issue_ok) return false;
  bool sorted = true;
  if (threaded) {
    for (size_t u = 0; u < good.size(); ++u)
      if (!good[u]) {
        set_error(err[u]);
        sorted = false;
      }
  } else {
    sorted = ok_hip(hipSetDevice(c.uniq[0]->dev), "hipSetDevice");
    for (int i = 0; sorted && i < K_; ++i) sorted = sort_round(*c.uniq[0], i);
  }
  if (!sorted) return false;
  // the equal re-cut: the pieces of the rounds that were not sorted in place
  for (int r = 0; r < R; ++r) {
    RankState& s = c.ranks[r];
    if (!ok_hip(hipSetDevice(s.dev), "hipSetDevice") || !ok_hip(hipEventRecord(s.ev_done, s.d->st), "record"))
      return false;
  }
  if (!comm_waits(c, &RankState::ev_done)) return false;
  const std::vector<dplan::Piece>& cut = pl.moves;
  trace("rounds sorted; re-cut of %zu pieces", cut.size());
  for (int r = 0; r < R; ++r) {
    src[r] = c.ranks[r].outb.p;
    dst[r] = out[r];
    vsrc[r] = c.ranks[r].ov.p;
    vdst[r] = pairs ? (*vout)[r] : nullptr;
  }
  // (the re-cut's few surplus keys are not counted in c.sent: the exchange
  // rounds' bytes are what the wire format changes)
  return move_pieces(c, cut, src, dst, sizeof(K), use_rccl, self_rccl, false) &&
         (!pairs || move_pieces(c, cut, vsrc, vdst, 4, use_rccl, self_rccl, false));
}

// ---------------------------------------------------------------------------
// Gap-coded rounds ("msdz"; the torch engine's pylibsort.distrib.sort_msdz,
// one engine for every world size).  The same partition
// and plan as run_digit_rounds, but the SENDER sorts: rank s sorts each of its
// outgoing (round i, destination d) pieces from its partition's digit pieces
// (sort_pieces_u32: the pieces are disjoint key ranges), codes every remote
// piece as 64-key groups of gaps (delta_pack_u32: a base word + 2w words per
// group, w = the bits of the piece's largest gap -- ~9.5 of 32 bits per key
// for uniform keys at 2^29 per rank), the host reads round i's largest gaps
// (exact coded sizes on both sides), the coded pieces cross the links, and
// the receiver decodes them (delta_unpack_u32) and merges its R sorted runs
// (merge_u32, pairwise levels) into its slice of the output; then the equal
// re-cut.  Fewer bytes on the wire (~0.3x), more GPU work (a merge level per
// doubling of R) -- for link-bound world sizes (2 GPUs: one xGMI link
// carries half of every shard).  Keys only, 32-bit partition (no planes).
// Per device one host thread issues its ranks' sender sorts of every round up
// front (the sorts' small host read-backs hold only that device), then each
// round's decode + merge once the exchange of that round is issued.
// ---------------------------------------------------------------------------
bool coded_rounds_on(int R, unsigned flags, bool rccl_between_gpus) {
  static const int env = [] {
    const char* e = getenv("LIBSORT_DISTRIB_CODED");
    return e && (e[0] == '0' || e[0] == '1') ? e[0] - '0' + 1 : 0;  // 0: auto, 1: off, 2: on
  }();
  if (flags & kDistribCoded) return true;
  if (env) return env == 2;
  return R == 2 && rccl_between_gpus;
}

bool run_coded_rounds(Ctx& c, const dplan::DigitPlan& p, const std::vector<std::vector<uint64_t>>& C,
                      const std::vector<uint32_t*>& out, bool use_rccl, bool self_rccl, int bits,
                      const PartDigit& pd) {
  const int R = (int)c.ranks.size(), K_ = p.K;
  const bool self_coded = use_rccl && self_rccl;
  auto remote = [&](int s, int d) { return s != d || self_coded; };
  // the coded layout (distrib_plan.h: digit starts, piece sizes M[s][i * R +
  // d], worst-case coded regions on both sides)
  const dplan::CodedPlan cp = dplan::coded_plan(p, C, self_coded);
  const auto& start = cp.start;
  const auto& M = cp.M;
  const auto& coff = cp.coff;
  const auto& cr_off = cp.cr_off;
  const auto& rcap = cp.rcap;
  std::map<DevState*, uint64_t> piece_max;
  for (int s = 0; s < R; ++s)
    for (int j = 0; j < R * K_; ++j) piece_max[c.ranks[s].d] = std::max(piece_max[c.ranks[s].d], M[s][j]);
  for (int r = 0; r < R; ++r) {
    RankState& s = c.ranks[r];
    const uint64_t m = std::max<uint64_t>(p.n_recv[r], 1);
    if (!s.alt.ensure(s.dev, std::max<uint64_t>(start[r][dplan::kTopDigits], 1) * 4) ||
        !s.csend.ensure(s.dev, std::max<uint64_t>(coff[r][(size_t)R * K_], 1) * 4) ||
        !s.crecv.ensure(s.dev, std::max<uint64_t>(rcap[r], 1) * 4) || !s.recv.ensure(s.dev, m * 4) ||
        !s.outb.ensure(s.dev, m * 4) || (R > 2 && !s.mtmp.ensure(s.dev, m * 4)))
      return false;
  }
  for (auto& kv : piece_max)
    if (!kv.first->tmp.ensure(kv.first->dev, std::max<uint64_t>(kv.second, 1) * 4)) return false;
  const dplan::Placement pl = dplan::place_rounds(p.roff, p.n_recv, K_);
  // the destination of rank r's round i (its output shard, or outb)
  auto round_dst = [&](int r, int i) -> uint32_t* {
    const size_t q = (size_t)r * K_ + i;
    return pl.direct[q] ? out[r] + pl.out_off[q] : c.ranks[r].outb.u32() + p.roff[(size_t)r * (K_ + 1) + i];
  };
  // a round whose only keys are the receiver's own piece: sorted straight
  // into its destination (no copy)
  auto only_self = [&](int r, int i) { return cp.self_only[(size_t)r * K_ + i] != 0; };
  uint32_t* const hmg = c.h_mg;
  const size_t mg_stride = (size_t)R * kMaxRounds;
  // sender side of rank r: sort, then code, every outgoing piece of round i
  auto send_round = [&](int r, int i) -> bool {
    RankState& s = c.ranks[r];
    DevState& d = *s.d;
    for (int dd = 0; dd < R; ++dd) {
      const size_t j = (size_t)i * R + dd;
      const uint64_t m = M[r][j];
      if (!m) continue;
      const int a = p.lo[j], b = p.hi[j];
      std::vector<uint64_t> offs, lens;
      std::vector<uint32_t> segs;
      for (int g = a; g < b; ++g) {
        offs.push_back(start[r][g] - start[r][a]);
        lens.push_back(C[r][g]);
        segs.push_back((uint32_t)(g - a));
      }
      uint32_t* const srt = (dd == r && only_self(r, i)) ? round_dst(r, i) : s.alt.u32() + start[r][a];
      if (!ok_hip(sort_pieces_u32(*d.ws, s.part.u32() + start[r][a], srt, d.tmp.u32(), m, offs.data(), lens.data(),
                                  segs.data(), offs.size(), (uint32_t)(b - a), pd.shift, bits, d.st,
                                  (uint32_t)pd.bias),
                  "sender round sort"))
        return false;
      if (remote(r, dd) &&
          (!ok_hip(delta_maxgap_u32(srt, m, s.mg.u32() + j, d.st), "largest gap") ||
           !ok_hip(delta_pack_u32(srt, m, s.mg.u32() + j, s.csend.u32() + coff[r][j], d.st), "gap coding")))
        return false;
    }
    return ok_hip(hipMemcpyAsync(hmg + (size_t)r * mg_stride + (size_t)i * R, s.mg.u32() + (size_t)i * R,
                                 (size_t)R * sizeof(uint32_t), hipMemcpyDeviceToHost, d.st),
                  "D2H largest gaps") &&
           ok_hip(hipEventRecord(s.ev_c[i], d.st), "hipEventRecord");
  };
  // receiver side of rank r, round i (after its exchange was issued): decode
  // the coded runs, merge them with the own piece into the round's destination
  auto merge_round = [&](int r, int i) -> bool {
    RankState& s = c.ranks[r];
    DevState& d = *s.d;
    if (!ok_hip(hipStreamWaitEvent(d.st, s.ev_x[i], 0), "wait")) return false;
    if (tracing()) {
      if (!ok_hip(hipEventSynchronize(s.ev_x[i]), "hipEventSynchronize")) return false;
      trace("round %d rank %d: arrived", i, r);
    }
    if (only_self(r, i)) return true;  // (sorted in place by the sender side)
    const uint64_t r0 = p.roff[(size_t)r * (K_ + 1) + i], r1 = p.roff[(size_t)r * (K_ + 1) + i + 1];
    if (r1 == r0) return true;
    std::vector<std::pair<const uint32_t*, uint64_t>> runs;
    uint64_t at = r0;
    for (int src = 0; src < R; ++src) {
      const size_t j = (size_t)i * R + r;
      const uint64_t m = M[src][j];
      if (!m) continue;
      if (!remote(src, r)) {
        runs.push_back({s.alt.u32() + start[r][p.lo[j]], m});
        continue;
      }
      const uint32_t w = dplan::gap_bits(hmg[(size_t)src * mg_stride + j]);
      if (!ok_hip(delta_unpack_u32(s.crecv.u32() + cr_off[r][(size_t)i * R + src], m, w, s.recv.u32() + at, d.st),
                  "gap decoding"))
        return false;
      runs.push_back({s.recv.u32() + at, m});
      at += m;
    }
    uint32_t* const dst = round_dst(r, i);
    // pairwise merge levels, ping-pong between mtmp and recv (the runs of a
    // level are consumed by the time the next level writes them)
    int level = 0;
    while (runs.size() > 2) {
      uint32_t* const buf = (level & 1) ? s.recv.u32() : s.mtmp.u32();
      std::vector<std::pair<const uint32_t*, uint64_t>> nxt;
      uint64_t o = r0;
      for (size_t k = 0; k + 1 < runs.size(); k += 2) {
        if (!ok_hip(merge_u32(runs[k].first, runs[k].second, runs[k + 1].first, runs[k + 1].second, buf + o, d.st),
                    "merge"))
          return false;
        nxt.push_back({buf + o, runs[k].second + runs[k + 1].second});
        o += runs[k].second + runs[k + 1].second;
      }
      if (runs.size() & 1) nxt.push_back(runs.back());
      runs.swap(nxt);
      ++level;
    }
    hipError_t e = runs.size() == 2 ? merge_u32(runs[0].first, runs[0].second, runs[1].first, runs[1].second, dst, d.st)
                                    : hipMemcpyAsync(dst, runs[0].first, runs[0].second * 4, hipMemcpyDeviceToDevice,
                                                     d.st);
    if (!ok_hip(e, "final merge")) return false;
    if (tracing()) {
      if (!ok_hip(hipStreamSynchronize(d.st), "hipStreamSynchronize")) return false;
      trace("round %d rank %d: decoded and merged (%zu runs)", i, r, runs.size());
    }
    return true;
  };
  // the exchange of round i: every sender's coded pieces, exact sizes from
  // the largest gaps the host read back (counted in c.sent: the coded bytes)
  auto exchange_round = [&](int i) -> bool {
    for (int r = 0; r < R; ++r)
      if (!ok_hip(hipEventSynchronize(c.ranks[r].ev_c[i]), "hipEventSynchronize")) return false;
    trace("round %d: sorted and coded on every rank", i);
    const std::vector<dplan::Piece> ps = dplan::coded_round_pieces(cp, i, hmg, mg_stride, self_coded);
    // every communication stream after every rank's round-i coding
    for (auto& u : c.uniq) {
      if (!ok_hip(hipSetDevice(u->dev), "hipSetDevice")) return false;
      for (auto& rk : c.ranks)
        if (!ok_hip(hipStreamWaitEvent(u->cs, rk.ev_c[i], 0), "hipStreamWaitEvent")) return false;
    }
    std::vector<const void*> src(R);
    std::vector<void*> dst(R);
    for (int r = 0; r < R; ++r) {
      src[r] = c.ranks[r].csend.p;
      dst[r] = c.ranks[r].crecv.p;
    }
    if (!move_pieces(c, ps, src, dst, 4, use_rccl, self_rccl)) return false;
    for (int r = 0; r < R; ++r) {
      RankState& s = c.ranks[r];
      if (!ok_hip(hipSetDevice(s.dev), "hipSetDevice") || !ok_hip(hipEventRecord(s.ev_x[i], s.d->cs), "record"))
        return false;
    }
    trace("round %d: coded exchange issued (%zu pieces)", i, ps.size());
    return true;
  };
  // Several devices (or LIBSORT_DISTRIB_THREADS=1): one host thread per
  // device -- its ranks' sender sorts of every round, then round by round
  // (once issued) their decode + merge; this thread issues the exchanges.
  static const bool force_threads = [] {
    const char* e = getenv("LIBSORT_DISTRIB_THREADS");
    return e && e[0] == '1';
  }();
  const bool threaded = c.uniq.size() > 1 || force_threads;
  std::mutex mu;
  std::condition_variable cv;
  int issued = 0;
  bool stop = false;
  std::vector<std::string> err(c.uniq.size());
  std::vector<char> good(c.uniq.size(), 1);
  // rounds whose sender sorts each device thread has issued (the issue loop
  // may wait on their events only after that: an event not recorded yet
  // would not hold it)
  std::vector<int> coded(c.uniq.size(), 0);
  auto device_work = [&](size_t u, bool wait_issue) -> bool {
    DevState& d = *c.uniq[u];
    if (!ok_hip(hipSetDevice(d.dev), "hipSetDevice")) return false;
    for (int i = 0; i < K_; ++i) {
      for (int r = 0; r < R; ++r)
        if (c.ranks[r].d == &d && !send_round(r, i)) return false;
      std::lock_guard<std::mutex> lk(mu);
      coded[u] = i + 1;
      cv.notify_all();
    }
    for (int i = 0; i < K_; ++i) {
      if (wait_issue) {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return issued > i || stop; });
        if (issued <= i) return true;  // the exchange failed (its error is reported)
      }
      for (int r = 0; r < R; ++r)
        if (c.ranks[r].d == &d && !merge_round(r, i)) return false;
    }
    return true;
  };
  bool issue_ok = true;
  if (threaded) {
    std::vector<std::thread> th;
    for (size_t u = 0; u < c.uniq.size(); ++u)
      th.emplace_back([&, u] {
        if (!device_work(u, true)) {
          good[u] = 0;
          err[u] = last_error();
          // (a device that failed its sorts never records their events:
          // stop the issue loop rather than wait for them)
          std::lock_guard<std::mutex> lk(mu);
          stop = true;
          cv.notify_all();
        }
      });
    // (the issue loop waits for events the device threads record: a failed
    // thread sets stop, checked between rounds)
    for (int i = 0; issue_ok && i < K_; ++i) {
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return stop || std::all_of(coded.begin(), coded.end(), [&](int k) { return k > i; }); });
        if (stop) break;
      }
      issue_ok = exchange_round(i);
      std::lock_guard<std::mutex> lk(mu);
      if (issue_ok) issued = i + 1;
      cv.notify_all();
    }
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
      cv.notify_all();
    }
    for (auto& t : th) t.join();
    for (size_t u = 0; u < good.size(); ++u)
      if (!good[u]) {
        set_error(err[u]);
        return false;
      }
    if (!issue_ok) return false;
  } else {
    // one device: every sender sort, then round by round exchange + merges
    DevState& d = *c.uniq[0];
    if (!ok_hip(hipSetDevice(d.dev), "hipSetDevice")) return false;
    for (int i = 0; i < K_; ++i)
      for (int r = 0; r < R; ++r)
        if (!send_round(r, i)) return false;
    for (int i = 0; i < K_; ++i) {
      if (!exchange_round(i) || !ok_hip(hipSetDevice(d.dev), "hipSetDevice")) return false;
      for (int r = 0; r < R; ++r)
        if (!merge_round(r, i)) return false;
    }
  }
  // the equal re-cut (as run_digit_rounds)
  for (int r = 0; r < R; ++r) {
    RankState& s = c.ranks[r];
    if (!ok_hip(hipSetDevice(s.dev), "hipSetDevice") || !ok_hip(hipEventRecord(s.ev_done, s.d->st), "record"))
      return false;
  }
  if (!comm_waits(c, &RankState::ev_done)) return false;
  trace("coded rounds merged; re-cut of %zu pieces", pl.moves.size());
  std::vector<const void*> src(R);
  std::vector<void*> dst(R);
  for (int r = 0; r < R; ++r) {
    src[r] = c.ranks[r].outb.p;
    dst[r] = out[r];
  }
  return move_pieces(c, pl.moves, src, dst, 4, use_rccl, self_rccl, false);
}


// distinct GPUs to overlap with the second part's partition; one otherwise
// (ranks sharing a GPU exchange by device copies, which two parts only double:
// +32 us of kernels per rank, 6.9 -> 7.7 ms in DESIGN.md 3d).
// The two-part gain comes from tools/msd_model.py and has not been measured
// across GPUs.  LIBSORT_DISTRIB_PARTS=1 / 2 forces one / two (tests, A/B).
int parts_for(int R, bool rccl_between_gpus) {
  static const int env = [] {
    const char* e = getenv("LIBSORT_DISTRIB_PARTS");
    return e && (e[0] == '1' || e[0] == '2') ? e[0] - '0' : 0;
  }();
  if (R <= 1) return 1;
  return env ? env : rccl_between_gpus ? kMaxParts : 1;
}

// Shared prologue of both entry points: sizes, the output shard counts.
bool check_sizes(int R, const size_t* n_in, std::vector<uint64_t>& n, uint64_t& N, size_t* n_out) {
  n.assign(R, 0);
  N = 0;
  for (int r = 0; r < R; ++r) {
    n[r] = n_in[r];
    N += n[r];
    if (n[r] > 0xffffffffull) {
      set_error("distributed sort: at most 2^32-1 keys per rank");
      return false;
    }
  }
  const uint64_t S = dplan::shard_size(N, R);
  if (S > 0xffffffffull) {
    set_error("distributed sort: at most 2^32-1 keys per output shard");
    return false;
  }
  for (int r = 0; r < R; ++r)
    n_out[r] = (size_t)(std::min<uint64_t>(N, (uint64_t)(r + 1) * S) - std::min<uint64_t>(N, (uint64_t)r * S));
  return true;
}

bool sort_device(Ctx& c, const uint32_t* const* d_in, const size_t* n_in, uint32_t* const* d_out, size_t* n_out,
                 unsigned flags, int bits) {
  const int R = (int)c.ranks.size();
  const bool copy = (flags & kDistribCopy) != 0 || !c.distinct;
  const bool self_rccl = (flags & kDistribSelfRccl) != 0 && !copy;
  trace_start();
  trace("sort u32: %d ranks on %zu devices, exchanges by %s, %d-bit digits, flags 0x%x", R, c.uniq.size(),
        copy ? "device/peer copies" : "RCCL", bits, flags);
  if (!copy && !c.ensure_comms()) return false;
  std::vector<uint64_t> n;
  uint64_t N = 0;
  if (!check_sizes(R, n_in, n, N, n_out)) return false;
  Hold hold(c);
  if (!hold.ok) return hold.finish(false);
  std::vector<const uint32_t*> in(d_in, d_in + R);
  std::vector<uint32_t*> out(d_out, d_out + R);
  c.sent.assign(R, 0);  // (before the empty return: libsortDistribLastBytes covers this call)
  if (N == 0) return hold.finish(true);
  const uint64_t S = dplan::shard_size(N, R);
  if (flags & kDistribLsd) return hold.finish(run_lsd(c, in, n, out, S, bits, !copy, self_rccl));
  const int K = std::max(1, std::min(kMaxRounds, 256 / R));
  std::vector<std::vector<uint64_t>> C;
  PartDigit pd;
  // 24-bit keys on the wire (top-digit rounds; LIBSORT_DISTRIB_WIRE24=0 or the
  // WIRE32 flag: 32-bit): planes from the partition scatter, read back by
  // the round sorts' reserved depth 0 (4-bit digits; 8-bit round sorts of
  // more than two segments could not take it and would unpack first)
  static const bool wire24_env = [] {
    const char* e = getenv("LIBSORT_DISTRIB_WIRE24");
    return !(e && e[0] == '0');
  }();
  // gap-coded rounds (kDistribCoded; by default at two ranks on two GPUs):
  // one partition part, 32-bit keys in the partition (the wire is coded)
  const bool coded = coded_rounds_on(R, flags, c.distinct && !copy);
  // (and R >= 3: the round sorts read planes only through the reserved depth
  // 0, which takes <= 32 segments; at R = 2 the rounds grow x1.2 over 128
  // digits per rank -- 24, 29, 34, 41 -- and the last two would unpack and
  // range-sort instead: 2^29 keys per rank sharing one GPU, 9.16 ms of GPU
  // work per rank against 7.07 ms with 32-bit words, gpurun_out/r06d)
  const bool planar = !coded && wire24_env && !(flags & kDistribWire32) && bits == 4 && R >= 3;
  const int H = coded ? 1 : parts_for(R, c.distinct && !copy);
  std::vector<std::vector<uint64_t>> Cp;
  std::vector<uint64_t> first;
  if (!partition_top<uint32_t>(c, in, nullptr, n, C, pd, planar, H, Cp, first)) return hold.finish(false);
  std::vector<uint8_t> lut(dplan::kTopDigits);
  std::vector<int64_t> est(R);
  dplan::plan_digit_rounds(C, K, 1.2, lut.data(), est.data());
  trace("plan: %d rounds per rank, %llu keys, largest rank %lld", K, (unsigned long long)N,
        (long long)*std::max_element(est.begin(), est.end()));
  if (dplan::msd_too_skewed(est.data(), R, N)) {
    trace("plan: too skewed for the top digit");
    // the top digit leaves the keys in too few digits: the 8-bit digit over
    // the populated key range, if that is finer; else (or still skewed) the
    // LSD rounds from the untouched input
    bool useful = false;
    if (!range_digit<uint32_t>(c, in, n, pd, &useful)) return hold.finish(false);
    if (useful) {  // (the range digit is not the top byte: 32-bit keys on the wire)
      if (!partition_top<uint32_t>(c, in, nullptr, n, C, pd, false, H, Cp, first)) return hold.finish(false);
      dplan::plan_digit_rounds(C, K, 1.2, lut.data(), est.data());
    }
    if (!useful || dplan::msd_too_skewed(est.data(), R, N)) {
      trace("plan: LSD rounds");
      return hold.finish(run_lsd(c, in, n, out, S, bits, !copy, self_rccl));
    }
  }
  if (coded) {
    trace("plan: gap-coded rounds");
    return hold.finish(run_coded_rounds(c, dplan::digit_plan_parts(Cp, 1, first, lut.data(), K), Cp, out, !copy,
                                        self_rccl, bits, pd));
  }
  return hold.finish(run_digit_rounds<uint32_t>(c, dplan::digit_plan_parts(Cp, H, first, lut.data(), K), out, nullptr,
                                                !copy, self_rccl, bits, pd, planar && !pd.range, H));
}

bool sort_device_pairs(Ctx& c, const uint64_t* const* d_kin, const uint32_t* const* d_vin, const size_t* n_in,
                       uint64_t* const* d_kout, uint32_t* const* d_vout, size_t* n_out, unsigned flags, int bits) {
  const int R = (int)c.ranks.size();
  const bool copy = (flags & kDistribCopy) != 0 || !c.distinct;
  const bool self_rccl = (flags & kDistribSelfRccl) != 0 && !copy;
  if (flags & kDistribLsd) {
    set_error("distributed pair sort: the LSD rounds are for keys only");
    return false;
  }
  trace_start();
  trace("sort pairs u64/u32: %d ranks on %zu devices, exchanges by %s, %d-bit digits", R, c.uniq.size(),
        copy ? "device/peer copies" : "RCCL", bits);
  if (!copy && !c.ensure_comms()) return false;
  std::vector<uint64_t> n;
  uint64_t N = 0;
  if (!check_sizes(R, n_in, n, N, n_out)) return false;
  Hold hold(c);
  if (!hold.ok) return hold.finish(false);
  c.sent.assign(R, 0);
  if (N == 0) return hold.finish(true);
  std::vector<const uint64_t*> kin(d_kin, d_kin + R);
  std::vector<const uint32_t*> vin(d_vin, d_vin + R);
  std::vector<uint64_t*> kout(d_kout, d_kout + R);
  std::vector<uint32_t*> vout(d_vout, d_vout + R);
  const int K = std::max(1, std::min(kMaxRounds, 256 / R));
  std::vector<std::vector<uint64_t>> C;
  PartDigit pd;
  const int H = parts_for(R, c.distinct && !copy);
  std::vector<std::vector<uint64_t>> Cp;
  std::vector<uint64_t> first;
  if (!partition_top<uint64_t>(c, kin, &vin, n, C, pd, false, H, Cp, first)) return hold.finish(false);
  std::vector<uint8_t> lut(dplan::kTopDigits);
  std::vector<int64_t> est(R);
  dplan::plan_digit_rounds(C, K, 1.2, lut.data(), est.data());
  if (dplan::msd_too_skewed(est.data(), R, N)) {
    // keys below 2^56, or sharing their top byte (IDs, timestamps): the 8-bit
    // digit over the populated key range.  Still skewed (few
    // distinct keys): no LSD fallback for pairs -- a heavy digit range
    // concentrates work on one rank, the result stays exact.
    bool useful = false;
    if (!range_digit<uint64_t>(c, kin, n, pd, &useful)) return hold.finish(false);
    if (useful) {
      if (!partition_top<uint64_t>(c, kin, &vin, n, C, pd, false, H, Cp, first)) return hold.finish(false);
      dplan::plan_digit_rounds(C, K, 1.2, lut.data(), est.data());
    }
  }
  return hold.finish(run_digit_rounds<uint64_t>(c, dplan::digit_plan_parts(Cp, H, first, lut.data(), K), kout, &vout,
                                                !copy, self_rccl, bits, pd, false, H));
}

}  // namespace

bool distrib_sort_u32(const int* devices, int R, const uint32_t* const* d_in, const size_t* n_in, uint32_t* const* d_out,
                      size_t* n_out, unsigned flags, int bits) {
  std::lock_guard<std::mutex> glk(g_dist_mu);
  Ctx* c = ctx_for(devices, R);
  return c && sort_device(*c, d_in, n_in, d_out, n_out, flags, bits);
}

bool distrib_sort_pairs_u64_u32(const int* devices, int R, const uint64_t* const* d_kin, const uint32_t* const* d_vin,
                                const size_t* n_in, uint64_t* const* d_kout, uint32_t* const* d_vout, size_t* n_out,
                                unsigned flags, int bits) {
  std::lock_guard<std::mutex> glk(g_dist_mu);
  Ctx* c = ctx_for(devices, R);
  return c && sort_device_pairs(*c, d_kin, d_vin, n_in, d_kout, d_vout, n_out, flags, bits);
}

bool distrib_sort_host_u32(uint32_t* h, size_t len, const int* devices, int R, unsigned flags, int bits) {
  std::lock_guard<std::mutex> glk(g_dist_mu);
  Ctx* c = ctx_for(devices, R);
  if (!c) return false;
  const uint64_t S = dplan::shard_size(len, R);
  if (S > 0xffffffffull) {
    set_error("distributed sort: at most 2^32-1 keys per GPU");
    return false;
  }
  std::vector<const uint32_t*> in(R);
  std::vector<uint32_t*> out(R);
  std::vector<size_t> n(R), n_out(R);
  // rank r's shard: keys [r*S, (r+1)*S) of the caller's array (the reference
  // cut, distrib.go:113), staged through the per-rank buffers
  for (int r = 0; r < R; ++r) {
    RankState& s = c->ranks[r];
    const uint64_t a = std::min<uint64_t>(len, (uint64_t)r * S), z = std::min<uint64_t>(len, (uint64_t)(r + 1) * S);
    n[r] = (size_t)(z - a);
    if (!s.hin.ensure(s.dev, std::max<uint64_t>(n[r], 1) * 4) || !s.hout.ensure(s.dev, std::max<uint64_t>(S, 1) * 4) ||
        !ok_hip(hipSetDevice(s.dev), "hipSetDevice") ||
        (n[r] && !ok_hip(hipMemcpyAsync(s.hin.p, h + a, n[r] * 4, hipMemcpyHostToDevice, s.d->st), "H2D shard")))
      return false;
    in[r] = s.hin.u32();
    out[r] = s.hout.u32();
  }
  if (!sort_device(*c, in.data(), n.data(), out.data(), n_out.data(), flags, bits)) return false;
  bool ok = true;
  for (int r = 0; ok && r < R; ++r) {
    RankState& s = c->ranks[r];
    ok = ok_hip(hipSetDevice(s.dev), "hipSetDevice") &&
         (!n_out[r] || ok_hip(hipMemcpyAsync(h + (uint64_t)r * S, s.hout.p, n_out[r] * 4, hipMemcpyDeviceToHost,
                                             s.d->st),
                              "D2H shard"));
  }
  return sync_all(*c) && ok;
}

bool distrib_last_bytes(uint64_t* per_rank, int nranks) {
  std::lock_guard<std::mutex> glk(g_dist_mu);
  if (!g_ctx || (int)g_ctx->sent.size() != nranks || !per_rank) return false;
  for (int r = 0; r < nranks; ++r) per_rank[r] = g_ctx->sent[r];
  return true;
}

int set_distrib_trace(int on) { return g_trace.exchange(on ? 1 : 0); }

namespace {
// one wave spinning on the constant-rate wall clock (s_memrealtime)
__global__ void k_spin(long long ticks, uint32_t* never) {
  const long long t0 = wall_clock64();
  uint32_t n = 0;
  while (wall_clock64() - t0 < ticks) ++n;
  if (n == 0xffffffffu && never) never[0] = n;  // (keeps the loop; never true)
}
}  // namespace

// do the engine's compute stream `st` and communication
// stream `cs` of devices[0] execute concurrently, in this process's exact
// stream set-up (torch's streams, the workspace streams, RCCL's)?  With
// GPU_MAX_HW_QUEUES = 4, HIP maps later streams onto shared hardware queues,
// and two streams on one in-order queue serialise -- an RCCL kernel waiting
// for its peer on cs would then hold the round sorts on st.  A spinning
// one-wave kernel on each stream; ms[0..3] = start / end on st, start / end
// on cs, in ms after a common event on st.
bool distrib_overlap_probe(const int* devices, int R, uint32_t spin_us, double* ms) {
  std::lock_guard<std::mutex> glk(g_dist_mu);
  Ctx* c = ctx_for(devices, R);
  if (!c) return false;
  DevState& d = *c->uniq[0];
  if (!ok_hip(hipSetDevice(d.dev), "hipSetDevice")) return false;
  int khz = 0;
  if (!ok_hip(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, d.dev), "hipDeviceGetAttribute"))
    return false;
  const long long ticks = (long long)spin_us * khz / 1000;
  hipEvent_t e[5] = {};
  bool ok = true;
  for (hipEvent_t& x : e) ok = ok && ok_hip(hipEventCreate(&x), "hipEventCreate");
  uint32_t* never = static_cast<uint32_t*>(d.lut.p);
  ok = ok && ok_hip(hipEventRecord(e[0], d.st), "record") && ok_hip(hipStreamWaitEvent(d.cs, e[0], 0), "wait") &&
       ok_hip(hipEventRecord(e[1], d.st), "record");
  if (ok) {
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, d.st, ticks, never);
    ok = ok_hip(hipGetLastError(), "spin on st") && ok_hip(hipEventRecord(e[2], d.st), "record") &&
         ok_hip(hipEventRecord(e[3], d.cs), "record");
  }
  if (ok) {
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, d.cs, ticks, never);
    ok = ok_hip(hipGetLastError(), "spin on cs") && ok_hip(hipEventRecord(e[4], d.cs), "record");
  }
  ok = ok && ok_hip(hipStreamSynchronize(d.st), "sync") && ok_hip(hipStreamSynchronize(d.cs), "sync");
  for (int i = 0; ok && i < 4; ++i) {
    float t = 0.f;
    ok = ok_hip(hipEventElapsedTime(&t, e[0], e[i + 1]), "hipEventElapsedTime");
    ms[i] = t;
  }
  for (hipEvent_t x : e)
    if (x) (void)hipEventDestroy(x);
  return ok;
}

void distrib_release() {
  std::lock_guard<std::mutex> glk(g_dist_mu);
  g_ctx.reset();
}

}  // namespace lsort
