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
//   range rounds (default): a sampled top-12-bit histogram per rank, ONE
//     host plan of (rank, round) key ranges (distrib_plan.h plan_rounds), one
//     stable table partition per rank (round-major, destination-minor), K
//     exchange rounds issued up front on each rank's communication stream,
//     and each round sorted into its slice of the rank's output on the
//     compute stream as soon as it has arrived (range-restricted LSD: digits
//     of key - lo), overlapping the later rounds' exchange; then the equal
//     re-cut moves the few surplus keys.  Falls back to the LSD rounds when
//     one key range would overload a rank (identical decision for all).
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
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <memory>
#include <mutex>
#include <string>
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

struct DevState {
  int dev = -1;
  Workspace* ws = nullptr;
  hipStream_t st = nullptr;  // compute
  hipStream_t cs = nullptr;  // exchanges
  hipEvent_t ev_comm = nullptr, ev_comp = nullptr;
  DBuf lut, tmp;
};

struct RankState {
  int dev = -1;
  DevState* d = nullptr;
  DBuf row, bounds, part, recv, outb, alt;
  DBuf hin, hout;  // staging of the host-pointer entry point
  hipEvent_t ev_part = nullptr, ev_bounds = nullptr, ev_done = nullptr;
  hipEvent_t ev_x[kMaxRounds] = {};
};

struct Ctx {
  std::vector<int> devs;                       // device of each rank
  std::vector<std::unique_ptr<DevState>> uniq;  // one per distinct device
  std::vector<RankState> ranks;
  std::vector<ncclComm_t> comms;               // RCCL communicator of each rank (distinct devices only)
  int64_t* h_rows = nullptr;                   // pinned: R x 4097 plan rows
  uint32_t* h_bounds = nullptr;                // pinned: R x 256 bucket starts
  bool distinct = false;

  ~Ctx() {
    for (ncclComm_t c : comms)
      if (c && g_rccl.loaded) (void)g_rccl.commDestroy(c);
    for (auto& r : ranks) {
      r.row.release();
      r.bounds.release();
      r.part.release();
      r.recv.release();
      r.outb.release();
      r.alt.release();
      r.hin.release();
      r.hout.release();
      (void)hipSetDevice(r.dev);
      for (hipEvent_t e : {r.ev_part, r.ev_bounds, r.ev_done})
        if (e) (void)hipEventDestroy(e);
      for (hipEvent_t e : r.ev_x)
        if (e) (void)hipEventDestroy(e);
    }
    for (auto& u : uniq) {
      u->lut.release();
      u->tmp.release();
      (void)hipSetDevice(u->dev);
      if (u->st) (void)hipStreamDestroy(u->st);
      if (u->cs) (void)hipStreamDestroy(u->cs);
      if (u->ev_comm) (void)hipEventDestroy(u->ev_comm);
      if (u->ev_comp) (void)hipEventDestroy(u->ev_comp);
    }
    if (h_rows) (void)hipHostFree(h_rows);
    if (h_bounds) (void)hipHostFree(h_bounds);
  }

  bool init(const std::vector<int>& d) {
    devs = d;
    const int R = (int)d.size();
    std::map<int, DevState*> by_dev;
    for (int dev : d) {
      if (by_dev.count(dev)) continue;
      auto u = std::make_unique<DevState>();
      u->dev = dev;
      u->ws = workspace_for(dev);
      if (!u->ws || !ok_hip(hipSetDevice(dev), "hipSetDevice") ||
          !ok_hip(hipStreamCreateWithFlags(&u->st, hipStreamNonBlocking), "hipStreamCreate") ||
          !ok_hip(hipStreamCreateWithFlags(&u->cs, hipStreamNonBlocking), "hipStreamCreate") ||
          !ok_hip(hipEventCreateWithFlags(&u->ev_comm, hipEventDisableTiming), "hipEventCreate") ||
          !ok_hip(hipEventCreateWithFlags(&u->ev_comp, hipEventDisableTiming), "hipEventCreate"))
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
      for (hipEvent_t* e : {&s.ev_part, &s.ev_bounds, &s.ev_done})
        if (!ok_hip(hipEventCreateWithFlags(e, hipEventDisableTiming), "hipEventCreate")) return false;
      for (hipEvent_t& e : s.ev_x)
        if (!ok_hip(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate")) return false;
      if (!s.row.ensure(s.dev, (dplan::kHistBins + 1) * sizeof(int64_t)) || !s.bounds.ensure(s.dev, 256 * 4))
        return false;
    }
    for (auto& u : uniq)
      if (!u->lut.ensure(u->dev, dplan::kHistBins)) return false;
    return ok_hip(hipHostMalloc(&h_rows, (size_t)R * (dplan::kHistBins + 1) * sizeof(int64_t), 0), "hipHostMalloc") &&
           ok_hip(hipHostMalloc(&h_bounds, (size_t)R * 256 * sizeof(uint32_t), 0), "hipHostMalloc");
  }

  bool ensure_comms() {
    if (!comms.empty()) return true;
    if (!g_rccl.load()) return false;
    comms.assign(devs.size(), nullptr);
    return g_rccl.ok(g_rccl.commInitAll(comms.data(), (int)devs.size(), devs.data()), "ncclCommInitAll");
  }
};

std::mutex g_dist_mu;  // one distributed sort at a time (it holds several devices' workspaces)
std::unique_ptr<Ctx> g_ctx;

// Moves the pieces: rank p.src's src[p.src] + src_off -> rank p.dst's
// dst[p.dst] + dst_off, on the communication streams.  A piece within one
// device is a device copy (unless self_rccl); across devices RCCL
// point-to-point (one group for the whole set) or, with `copy`, a peer copy
// pulled by the receiver.
bool move_pieces(Ctx& c, const std::vector<dplan::Piece>& ps, const std::vector<const uint32_t*>& src,
                 const std::vector<uint32_t*>& dst, bool use_rccl, bool self_rccl) {
  std::vector<const dplan::Piece*> net;
  for (const dplan::Piece& p : ps) {
    if (!p.count) continue;
    RankState& a = c.ranks[p.src];
    RankState& b = c.ranks[p.dst];
    const size_t bytes = p.count * sizeof(uint32_t);
    if (use_rccl && (p.src != p.dst || self_rccl)) {
      net.push_back(&p);
    } else if (a.dev == b.dev) {
      if (!ok_hip(hipSetDevice(b.dev), "hipSetDevice") ||
          !ok_hip(hipMemcpyAsync(dst[p.dst] + p.dst_off, src[p.src] + p.src_off, bytes, hipMemcpyDeviceToDevice,
                                 b.d->cs),
                  "device copy"))
        return false;
    } else {
      if (!ok_hip(hipSetDevice(b.dev), "hipSetDevice") ||
          !ok_hip(hipMemcpyPeerAsync(dst[p.dst] + p.dst_off, b.dev, src[p.src] + p.src_off, a.dev, bytes, b.d->cs),
                  "peer copy"))
        return false;
    }
  }
  if (net.empty()) return true;
  if (!g_rccl.ok(g_rccl.groupStart(), "ncclGroupStart")) return false;
  bool ok = true;
  for (const dplan::Piece* p : net) {
    RankState& a = c.ranks[p->src];
    RankState& b = c.ranks[p->dst];
    ok = ok && g_rccl.ok(g_rccl.send(src[p->src] + p->src_off, p->count, ncclUint32, p->dst, c.comms[p->src], a.d->cs),
                         "ncclSend") &&
         g_rccl.ok(g_rccl.recv(dst[p->dst] + p->dst_off, p->count, ncclUint32, p->src, c.comms[p->dst], b.d->cs),
                   "ncclRecv");
  }
  return g_rccl.ok(g_rccl.groupEnd(), "ncclGroupEnd") && ok;
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

int span_bits(uint64_t lo, uint64_t hi) {
  const uint64_t span = hi - lo - 1;
  int w = 0;
  while (w < 32 && (span >> w) != 0) ++w;
  return std::max(w, 1);
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
    std::vector<std::vector<uint64_t>> C(R, std::vector<uint64_t>(256));
    for (int r = 0; r < R; ++r) {
      if (!ok_hip(hipEventSynchronize(c.ranks[r].ev_part), "hipEventSynchronize")) return false;
      const uint32_t* b = c.h_bounds + (size_t)r * 256;
      for (int g = 0; g < 256; ++g) C[r][g] = (g + 1 < 256 ? (uint64_t)b[g + 1] : n_cur[r]) - b[g];
    }
    dplan::LsdRound o = dplan::lsd_round(C, S);
    if (!comm_waits(c, &RankState::ev_part)) return false;
    std::vector<const uint32_t*> src(R);
    std::vector<uint32_t*> dst(R);
    for (int r = 0; r < R; ++r) {
      src[r] = c.ranks[r].part.u32();
      dst[r] = c.ranks[r].recv.u32();
    }
    if (!move_pieces(c, o.pieces, src, dst, use_rccl, self_rccl)) return false;
    // gather into bucket-major / rank-minor order on the compute stream.
    // Every compute stream waits for EVERY device's communication stream: a
    // peer copy (copy mode across devices) is pulled on the receiver's stream
    // from the sender's `part`, which the sender's next partial sort rewrites
    // (write-after-read across devices).
    const bool last = step + 1 == 32 / W;
    for (auto& u : c.uniq)
      if (!ok_hip(hipSetDevice(u->dev), "hipSetDevice") || !ok_hip(hipEventRecord(u->ev_comm, u->cs), "record"))
        return false;
    for (auto& u : c.uniq) {
      if (!ok_hip(hipSetDevice(u->dev), "hipSetDevice")) return false;
      for (auto& v : c.uniq)
        if (!ok_hip(hipStreamWaitEvent(u->st, v->ev_comm, 0), "wait")) return false;
    }
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

bool sort_device(Ctx& c, const uint32_t* const* d_in, const size_t* n_in, uint32_t* const* d_out, size_t* n_out,
                 unsigned flags, int bits) {
  const int R = (int)c.ranks.size();
  const bool copy = (flags & kDistribCopy) != 0 || !c.distinct;
  const bool self_rccl = (flags & kDistribSelfRccl) != 0 && !copy;
  if (!copy && !c.ensure_comms()) return false;
  uint64_t N = 0;
  std::vector<uint64_t> n(R);
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
  for (int r = 0; r < R; ++r) n_out[r] = (size_t)(std::min<uint64_t>(N, (uint64_t)(r + 1) * S) -
                                                  std::min<uint64_t>(N, (uint64_t)r * S));
  // hold every involved workspace (ascending device order) for the whole sort
  std::vector<std::unique_lock<std::mutex>> locks;
  {
    std::vector<DevState*> order;
    for (auto& u : c.uniq) order.push_back(u.get());
    std::sort(order.begin(), order.end(), [](DevState* a, DevState* b) { return a->dev < b->dev; });
    for (DevState* u : order) locks.emplace_back(u->ws->mu);
    for (DevState* u : order)
      if (!ws_acquire_stream(u->dev, u->st)) return false;
  }
  auto finish = [&](bool ok) {
    const bool synced = sync_all(c);
    for (auto& u : c.uniq) ws_release_stream(u->dev, u->st);
    return ok && synced;
  };
  std::vector<const uint32_t*> in(d_in, d_in + R);
  std::vector<uint32_t*> out(d_out, d_out + R);
  if (N == 0) return finish(true);

  bool lsd = (flags & kDistribLsd) != 0;
  const int K = std::max(1, std::min(kMaxRounds, 256 / R));
  std::vector<uint8_t> lut(dplan::kHistBins);
  if (!lsd) {
    // 1. sampled top-12-bit histogram of every rank (every 16th 4096-key block)
    for (int r = 0; r < R; ++r) {
      RankState& s = c.ranks[r];
      int64_t* h = c.h_rows + (size_t)r * (dplan::kHistBins + 1);
      if (!ok_hip(hipSetDevice(s.dev), "hipSetDevice")) return finish(false);
      if (!n[r]) {
        memset(h, 0, (dplan::kHistBins + 1) * sizeof(int64_t));
        continue;
      }
      if (!ok_hip(plan_hist_u32(*s.d->ws, in[r], n[r], 12, 4096, 16, static_cast<int64_t*>(s.row.p), s.d->st),
                  "plan histogram") ||
          !ok_hip(hipMemcpyAsync(h, s.row.p, (dplan::kHistBins + 1) * sizeof(int64_t), hipMemcpyDeviceToHost, s.d->st),
                  "D2H plan row") ||
          !ok_hip(hipEventRecord(s.ev_bounds, s.d->st), "hipEventRecord"))
        return finish(false);
    }
    for (int r = 0; r < R; ++r)
      if (n[r] && !ok_hip(hipEventSynchronize(c.ranks[r].ev_bounds), "hipEventSynchronize")) return finish(false);
    // 2. the plan, once, on the host
    std::vector<int64_t> est(R);
    dplan::plan_rounds(c.h_rows, R, dplan::kHistBins + 1, K, 1.2, lut.data(), est.data());
    lsd = dplan::msd_too_skewed(est.data(), R, N);
  }
  if (lsd) return finish(run_lsd(c, in, n, out, S, 8, !copy, self_rccl));
  const int NB = R * K;
  // 3. table partition of every rank: counts + scan, bucket starts to the
  //    host, then the scatter (queued before the host waits for the starts)
  for (auto& u : c.uniq)
    if (!ok_hip(hipSetDevice(u->dev), "hipSetDevice") ||
        !ok_hip(hipMemcpyAsync(u->lut.p, lut.data(), dplan::kHistBins, hipMemcpyHostToDevice, u->st), "H2D plan"))
      return finish(false);
  for (int r = 0; r < R; ++r) {
    RankState& s = c.ranks[r];
    if (!ok_hip(hipSetDevice(s.dev), "hipSetDevice") || !s.part.ensure(s.dev, std::max<uint64_t>(n[r], 1) * 4))
      return finish(false);
    const uint8_t* dl = static_cast<const uint8_t*>(s.d->lut.p);
    if (n[r]) {
      if (!ok_hip(partition_lut_u32(*s.d->ws, in[r], nullptr, n[r], dl, dplan::kLutShift, NB, s.bounds.u32(), s.d->st,
                                    kPartCount),
                  "partition counts") ||
          !ok_hip(hipMemcpyAsync(c.h_bounds + (size_t)r * 256, s.bounds.p, NB * 4, hipMemcpyDeviceToHost, s.d->st),
                  "D2H bucket starts") ||
          !ok_hip(hipEventRecord(s.ev_bounds, s.d->st), "hipEventRecord") ||
          !ok_hip(partition_lut_u32(*s.d->ws, in[r], s.part.u32(), n[r], dl, dplan::kLutShift, NB, nullptr, s.d->st,
                                    kPartScatter),
                  "partition scatter"))
        return finish(false);
    }
    if (!ok_hip(hipEventRecord(s.ev_part, s.d->st), "hipEventRecord")) return finish(false);
  }
  std::vector<std::vector<uint64_t>> C(R, std::vector<uint64_t>(NB, 0));
  for (int r = 0; r < R; ++r) {
    if (!n[r]) continue;
    if (!ok_hip(hipEventSynchronize(c.ranks[r].ev_bounds), "hipEventSynchronize")) return finish(false);
    const uint32_t* b = c.h_bounds + (size_t)r * 256;
    for (int j = 0; j < NB; ++j) C[r][j] = (j + 1 < NB ? (uint64_t)b[j + 1] : n[r]) - b[j];
  }
  dplan::MsdPlan p = dplan::msd_plan(C, K);
  uint64_t round_max = 1;
  for (int r = 0; r < R; ++r) {
    RankState& s = c.ranks[r];
    if (!s.recv.ensure(s.dev, std::max<uint64_t>(p.n_recv[r], 1) * 4) ||
        !s.outb.ensure(s.dev, std::max<uint64_t>(p.n_recv[r], 1) * 4))
      return finish(false);
    for (int i = 0; i < K; ++i)
      round_max = std::max(round_max, p.roff[(size_t)r * (K + 1) + i + 1] - p.roff[(size_t)r * (K + 1) + i]);
  }
  for (auto& u : c.uniq)
    if (!u->tmp.ensure(u->dev, round_max * 4)) return finish(false);
  // 4. every round's exchange, issued now on the communication streams
  if (!comm_waits(c, &RankState::ev_part)) return finish(false);
  std::vector<const uint32_t*> src(R);
  std::vector<uint32_t*> dst(R);
  for (int r = 0; r < R; ++r) {
    src[r] = c.ranks[r].part.u32();
    dst[r] = c.ranks[r].recv.u32();
  }
  for (int i = 0; i < K; ++i) {
    if (!move_pieces(c, p.rounds[i], src, dst, !copy, self_rccl)) return finish(false);
    for (int r = 0; r < R; ++r) {
      RankState& s = c.ranks[r];
      if (!ok_hip(hipSetDevice(s.dev), "hipSetDevice") || !ok_hip(hipEventRecord(s.ev_x[i], s.d->cs), "record"))
        return finish(false);
    }
  }
  // 5. each round sorted into its slice as soon as it has arrived
  for (int i = 0; i < K; ++i)
    for (int r = 0; r < R; ++r) {
      RankState& s = c.ranks[r];
      const uint64_t a = p.roff[(size_t)r * (K + 1) + i], z = p.roff[(size_t)r * (K + 1) + i + 1];
      if (!ok_hip(hipSetDevice(s.dev), "hipSetDevice") || !ok_hip(hipStreamWaitEvent(s.d->st, s.ev_x[i], 0), "wait"))
        return finish(false);
      if (z == a) continue;
      uint64_t lo = 0, hi = 0;
      if (!dplan::group_range(lut.data(), i * R + r, &lo, &hi)) {
        set_error("distributed sort: round without a key range");
        return finish(false);
      }
      if (!ok_hip(sort_u32(*s.d->ws, s.recv.u32() + a, s.outb.u32() + a, s.d->tmp.u32(), z - a, 0,
                           span_bits(lo, hi), bits, nullptr, s.d->st, (uint32_t)lo, true, hi - lo),
                  "round sort"))
        return finish(false);
    }
  // 6. the equal re-cut into the caller's shards
  for (int r = 0; r < R; ++r) {
    RankState& s = c.ranks[r];
    if (!ok_hip(hipSetDevice(s.dev), "hipSetDevice") || !ok_hip(hipEventRecord(s.ev_done, s.d->st), "record"))
      return finish(false);
  }
  if (!comm_waits(c, &RankState::ev_done)) return finish(false);
  for (int r = 0; r < R; ++r) src[r] = c.ranks[r].outb.u32();
  return finish(move_pieces(c, dplan::recut_pieces(p.n_recv), src, out, !copy, self_rccl));
}

}  // namespace

bool distrib_sort_u32(const int* devices, int R, const uint32_t* const* d_in, const size_t* n_in, uint32_t* const* d_out,
                      size_t* n_out, unsigned flags, int bits) {
  std::lock_guard<std::mutex> glk(g_dist_mu);
  Ctx* c = ctx_for(devices, R);
  return c && sort_device(*c, d_in, n_in, d_out, n_out, flags, bits);
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

void distrib_release() {
  std::lock_guard<std::mutex> glk(g_dist_mu);
  g_ctx.reset();
}

}  // namespace lsort
