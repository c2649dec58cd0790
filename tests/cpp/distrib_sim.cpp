// distrib_sim.cpp -- CPU simulation of the single-process multi-GPU sort
// (gpu-radix-sort_amd/csrc/distrib.cpp) over R host "ranks": the SAME host
// arithmetic (csrc/distrib_plan.h: round plan, exchange pieces, LSD gather
// tables, equal re-cut) drives plain host copies, with the oracle's CPU
// restatements as the local operations.  Checked against the oracle
// (oracle/oracle.cpp, compiled in): the range rounds give std::sort cut into
// ceil(N/R) shards; the LSD rounds give, shard for shard, the reference BSP
// driver's output (oracle_distrib_bsp_u32: distrib.go:90-179).  Built and run
// with AddressSanitizer + UBSan by tests/test_distrib_plan_cpu.py.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <random>
#include <string>
#include <vector>

#include "../../oracle/oracle.cpp"
#include "distrib_plan.h"

using namespace lsort::dplan;
typedef std::vector<uint32_t> Vec;

static int g_fail = 0;
#define CHECK(c, ...)                                  \
  do {                                                 \
    if (!(c)) {                                        \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                    \
      fprintf(stderr, "\n");                           \
      ++g_fail;                                        \
      return false;                                    \
    }                                                  \
  } while (0)

static std::vector<Vec> split(const Vec& x, int R) {
  const uint64_t S = shard_size(x.size(), R);
  std::vector<Vec> out(R);
  for (int r = 0; r < R; ++r) {
    const size_t lo = std::min(x.size(), (size_t)(r * S)), hi = std::min(x.size(), (size_t)((r + 1) * S));
    out[r].assign(x.begin() + lo, x.begin() + hi);
  }
  return out;
}

static void apply(const std::vector<Piece>& ps, const std::vector<Vec>& src, std::vector<Vec>& dst) {
  for (const Piece& p : ps) memcpy(dst[p.dst].data() + p.dst_off, src[p.src].data() + p.src_off, p.count * 4);
}

// range rounds: full (unsampled) histograms, table partition, rounds, re-cut
static bool run_msd(const Vec& x, int R, int K, double growth) {
  std::vector<Vec> in = split(x, R);
  std::vector<int64_t> H((size_t)R * kHistBins, 0);
  for (int r = 0; r < R; ++r)
    for (uint32_t k : in[r]) H[(size_t)r * kHistBins + (k >> kLutShift)]++;
  std::vector<uint8_t> lut(kHistBins);
  std::vector<int64_t> est(R);
  plan_rounds(H.data(), R, kHistBins, K, growth, lut.data(), est.data());
  uint64_t tot = 0;
  for (int r = 0; r < R; ++r) tot += (uint64_t)est[r];
  CHECK(tot == x.size(), "est sum %llu != %zu", (unsigned long long)tot, x.size());
  for (int b = 1; b < kHistBins; ++b) {  // monotone (round, rank) groups
    const int c0 = lut[b - 1] % R * K + lut[b - 1] / R, c1 = lut[b] % R * K + lut[b] / R;
    CHECK(c1 >= c0, "plan not monotone at %d", b);
  }
  const int NB = R * K;
  std::vector<Vec> part(R);
  std::vector<std::vector<uint64_t>> C(R, std::vector<uint64_t>(NB, 0));
  for (int r = 0; r < R; ++r) {
    for (uint32_t k : in[r]) C[r][lut[k >> kLutShift]]++;
    std::vector<uint64_t> at(NB + 1, 0);
    for (int j = 0; j < NB; ++j) at[j + 1] = at[j] + C[r][j];
    part[r].resize(in[r].size());
    for (uint32_t k : in[r]) part[r][at[lut[k >> kLutShift]]++] = k;  // stable
  }
  MsdPlan p = msd_plan(C, K);
  std::vector<Vec> recv(R), out(R);
  for (int r = 0; r < R; ++r) {
    recv[r].assign(p.n_recv[r], 0xdeadbeefu);
    out[r].assign(p.n_recv[r], 0);
  }
  for (int i = 0; i < K; ++i) {
    apply(p.rounds[i], part, recv);
    for (int r = 0; r < R; ++r) {
      const uint64_t a = p.roff[(size_t)r * (K + 1) + i], z = p.roff[(size_t)r * (K + 1) + i + 1];
      if (z == a) continue;
      uint64_t lo, hi;
      CHECK(group_range(lut.data(), i * R + r, &lo, &hi), "round %d rank %d has keys but no range", i, r);
      for (uint64_t q = a; q < z; ++q) CHECK(recv[r][q] >= lo && recv[r][q] < hi, "key outside its round range");
      std::copy(recv[r].begin() + a, recv[r].begin() + z, out[r].begin() + a);
      std::sort(out[r].begin() + a, out[r].begin() + z);
    }
  }
  std::vector<Vec> fin(R);
  const uint64_t S = shard_size(x.size(), R);
  for (int r = 0; r < R; ++r) fin[r].assign(std::min<uint64_t>(S, x.size() - std::min<uint64_t>(x.size(), r * S)), 0);
  apply(recut_pieces(p.n_recv), out, fin);
  Vec want(x);
  std::sort(want.begin(), want.end());
  std::vector<Vec> ws = split(want, R);
  for (int r = 0; r < R; ++r) CHECK(fin[r] == ws[r], "msd shard %d differs (R=%d K=%d n=%zu)", r, R, K, x.size());
  return true;
}

// reference BSP rounds: stable 8-bit partial sort per rank, exchange, gather
static bool run_lsd(const Vec& x, int R, int width) {
  std::vector<Vec> cur = split(x, R);
  const uint64_t S = shard_size(x.size(), R);
  const size_t nb = (size_t)1 << width;
  for (int step = 0; step < 32 / width; ++step) {
    std::vector<std::vector<uint64_t>> C(R, std::vector<uint64_t>(nb, 0));
    for (int r = 0; r < R; ++r) {
      std::vector<uint32_t> b(nb);
      oracle_partial_u32(cur[r].data(), b.data(), cur[r].size(), step * width, width);
      for (size_t g = 0; g < nb; ++g) C[r][g] = (g + 1 < nb ? b[g + 1] : cur[r].size()) - b[g];
    }
    LsdRound o = lsd_round(C, S);
    std::vector<Vec> recv(R), nxt(R);
    for (int r = 0; r < R; ++r) {
      recv[r].assign(o.n_next[r], 0xdeadbeefu);
      nxt[r].assign(o.n_next[r], 0xdeadbeefu);
    }
    apply(o.pieces, cur, recv);
    for (int d = 0; d < R; ++d) {
      uint64_t covered = 0;
      for (size_t q = 0; q < o.seg_len[d].size(); ++q) {
        CHECK(o.seg_src[d][q] + o.seg_len[d][q] <= recv[d].size(), "segment src out of range");
        CHECK(o.seg_dst[d][q] + o.seg_len[d][q] <= nxt[d].size(), "segment dst out of range");
        memcpy(nxt[d].data() + o.seg_dst[d][q], recv[d].data() + o.seg_src[d][q], o.seg_len[d][q] * 4);
        covered += o.seg_len[d][q];
      }
      CHECK(covered == nxt[d].size(), "segments cover %llu of %zu", (unsigned long long)covered, nxt[d].size());
    }
    cur.swap(nxt);
  }
  Vec ref(x);
  std::vector<uint64_t> lens(R);
  oracle_distrib_bsp_u32(ref.data(), ref.size(), R, width, lens.data());
  std::vector<Vec> ws = split(ref, R);
  for (int r = 0; r < R; ++r) {
    CHECK(cur[r] == ws[r], "lsd shard %d differs from the reference BSP driver (R=%d n=%zu)", r, R, x.size());
    CHECK(lens[r] == cur[r].size(), "lsd shard %d length", r);
  }
  return true;
}

static Vec make(const std::string& kind, size_t n, uint64_t seed) {
  Vec x(n);
  std::mt19937_64 g(seed);
  if (kind == "pcg") {
    uint64_t st = oracle_pcg_initial_state();
    oracle_pcg_fill(x.data(), n, &st);
  } else if (kind == "dups") {
    for (auto& v : x) v = (uint32_t)(g() % 50);
  } else if (kind == "allequal") {
    std::fill(x.begin(), x.end(), 12345u);
  } else if (kind == "skewtop") {
    for (auto& v : x) v = (uint32_t)(g() % (1u << 20));
  } else if (kind == "sorted" || kind == "reverse") {
    for (auto& v : x) v = (uint32_t)g();
    std::sort(x.begin(), x.end());
    if (kind == "reverse") std::reverse(x.begin(), x.end());
  } else {  // "wide": full-range random
    for (auto& v : x) v = (uint32_t)g();
  }
  return x;
}

int main() {
  const char* kinds[] = {"pcg", "dups", "allequal", "skewtop", "sorted", "reverse", "wide"};
  const size_t sizes[] = {0, 1, 2, 7, 1111, 40001, 300007};
  int cases = 0;
  for (const char* k : kinds)
    for (size_t n : sizes)
      for (int R : {1, 2, 3, 5, 8}) {
        Vec x = make(k, n, n * 31 + R);
        for (int K : {1, 3, 4}) {
          run_msd(x, R, K, K == 4 ? 1.2 : 0.6);
          ++cases;
        }
        if (n <= 40001) {
          run_lsd(x, R, 8);
          ++cases;
        }
      }
  // R * K = 256 partition buckets (the table limit)
  run_msd(make("wide", 100003, 5), 2, 128, 1.2);
  ++cases;
  run_lsd(make("pcg", 4099, 0), 4, 4);
  ++cases;
  if (g_fail) {
    fprintf(stderr, "%d of %d cases failed\n", g_fail, cases);
    return 1;
  }
  printf("OK %d cases\n", cases);
  return 0;
}
