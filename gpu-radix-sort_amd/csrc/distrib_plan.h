// distrib_plan.h -- host arithmetic of the single-process multi-GPU sort
// (distrib.cpp): shard cut, round plan, exchange tables and rebalance.  Pure
// C++17 with no HIP types, so the same code is compiled into libsort.so and
// into the CPU simulation test (tests/cpp/distrib_sim.cpp, built with
// AddressSanitizer), which runs both schedules on host arrays against the
// oracle.
//
// Reference semantics (paths relative to the reference checkout):
//   - equal re-cut of the global order into chunks of ceil(N/R) keys:
//     benchmark/pkg/sort/distrib.go:113, helpers.go:94-121;
//   - BSP LSD rounds (global order per round: bucket-major, worker-minor):
//     distrib.go:119-176, localTest/benchmarks.cpp:91-143.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <cmath>
#include <vector>

namespace lsort {
namespace dplan {


// The reference's equal re-cut: S = ceil(N / R) keys per rank.
inline uint64_t shard_size(uint64_t N, int R) { return R > 0 ? (N + (uint64_t)R - 1) / (uint64_t)R : 0; }

// |[a, a + len) ∩ [d*S, (d+1)*S)| for every d (the last shard is open-ended,
// distrib.go:113 gives it the remainder), added into out[0..R).
inline void add_interval_counts(uint64_t a, uint64_t len, uint64_t S, int R, uint64_t* out) {
  if (!len || R <= 0) return;
  const uint64_t b = a + len;
  if (S == 0) {
    out[R - 1] += len;
    return;
  }
  uint64_t d0 = std::min<uint64_t>(a / S, (uint64_t)R - 1), d1 = std::min<uint64_t>((b - 1) / S, (uint64_t)R - 1);
  for (uint64_t d = d0; d <= d1; ++d) {
    const uint64_t lo = d * S, hi = (d + 1 == (uint64_t)R) ? UINT64_MAX : (d + 1) * S;
    out[d] += std::min(b, hi) - std::max(a, lo);
  }
}

// ---------------------------------------------------------------------------
// round plan ("msd"): contiguous bucket (top-digit) ranges -> (rank, round)
// ---------------------------------------------------------------------------
// H: R rows of ld >= bins int64 (per-rank key counts of `bins` top-bit
// buckets; the digit rounds pass the 256 exact top-8-bit counts).
// lut[b] = round * R + rank for bucket b; est[r] = keys of rank r.
// Bucket b's middle in rank coordinates x = (cum(b) - G(b)/2) / total * R
// gives rank floor(x); its round is the first i with x - rank < cw[i] (cw =
// normalised prefix of growth^i); rank * K + round is made monotone over the
// buckets (cumulative max).  The one plan both engines run (pylibsort.distrib
// through libsortDistribPlanDigits; tests/test_distrib_cpu.py checks it
// against a numpy restatement).
inline void plan_rounds(const int64_t* H, int R, size_t ld, int K, double growth, uint8_t* lut, int64_t* est,
                        int bins) {
  std::vector<double> cw(K);
  double acc = 0.0, p = 1.0;
  for (int i = 0; i < K; ++i) {
    cw[i] = acc + p;
    acc += p;
    p *= growth;
  }
  for (int i = 0; i < K; ++i) cw[i] /= acc;
  std::vector<uint64_t> G(bins, 0);
  uint64_t total = 0;
  for (int b = 0; b < bins; ++b) {
    for (int r = 0; r < R; ++r) G[b] += (uint64_t)H[(size_t)r * ld + b];
    total += G[b];
  }
  const double Td = total ? (double)total : 1.0;
  for (int r = 0; r < R; ++r) est[r] = 0;
  uint64_t cum = 0;
  uint32_t run = 0;
  for (int b = 0; b < bins; ++b) {
    cum += G[b];
    const double x = ((double)cum - (double)G[b] / 2.0) / Td * (double)R;
    int64_t rank = (int64_t)std::floor(x);
    rank = std::max<int64_t>(0, std::min<int64_t>(rank, R - 1));
    const double f = x - (double)rank;
    int rnd = 0;
    while (rnd < K && cw[rnd] <= f) ++rnd;
    rnd = std::min(rnd, K - 1);
    run = std::max(run, (uint32_t)(rank * K + rnd));
    const uint32_t rk = run / (uint32_t)K, rd = run % (uint32_t)K;
    lut[b] = (uint8_t)(rd * (uint32_t)R + rk);
    est[rk] += (int64_t)G[b];
  }
}

// Skew fallback of the digit rounds (identical on every rank): a rank
// would receive more than max_imbalance * S (+ one tile) keys.
inline bool msd_too_skewed(const int64_t* est, int R, uint64_t N, double max_imbalance = 1.5) {
  double hs = 0.0, mx = 0.0;
  for (int r = 0; r < R; ++r) {
    hs += (double)est[r];
    mx = std::max(mx, (double)est[r]);
  }
  if (!N || hs <= 0.0) return false;
  return mx * (double)N / hs > max_imbalance * (double)shard_size(N, R) + 4096.0;
}

// One piece of an exchange: `count` keys from rank `src` at element offset
// `src_off` of its send buffer to rank `dst` at `dst_off` of its receive
// buffer.
struct Piece {
  int src, dst;
  uint64_t src_off, dst_off, count;
  int part = 0;  // the sender's partition part it comes from (digit_plan_parts)
};

// ---------------------------------------------------------------------------
// top-digit rounds ("msd"): the exchange is planned on the EXACT counts of the
// top 8 key bits, which every rank has from its partition pass (a stable
// partition by the top digit, the reference's gpuPartial(offset 24, width 8)
// building block), so the receiver's pieces arrive partitioned by the digit
// and its round sort starts below it (sort_pieces_u32).
// ---------------------------------------------------------------------------
constexpr int kTopBits = 8;
constexpr int kTopDigits = 1 << kTopBits;  // 256
constexpr int kTopShift = 32 - kTopBits;   // digit = key >> 24

// C: R rows of 256 exact digit counts.  lut[g] = round * R + rank of digit g
// (plan_rounds over 256 bins: contiguous digit ranges, ~1/R of the keys per
// rank, rounds growing by `growth`); est[r] = keys rank r receives (exact).
inline void plan_digit_rounds(const std::vector<std::vector<uint64_t>>& C, int K, double growth, uint8_t* lut,
                              int64_t* est) {
  const int R = (int)C.size();
  std::vector<int64_t> H((size_t)R * kTopDigits);
  for (int r = 0; r < R; ++r)
    for (int g = 0; g < kTopDigits; ++g) H[(size_t)r * kTopDigits + g] = (int64_t)C[r][g];
  plan_rounds(H.data(), R, kTopDigits, K, growth, lut, est, kTopDigits);
}

// The range digit of the rounds when the top digit is too skewed: the 8-bit
// digit (key - lo) >> shift over the populated keys [lo, hi] of every rank,
// shift = bits(hi - lo) - 8 (at least 0), so every key's digit is < 256.
// Returns whether it splits finer than the top digit of a `key_bits`-bit key
// (false when every key is equal).
inline bool range_digit(uint64_t lo, uint64_t hi, int key_bits, uint64_t* bias, int* shift) {
  const uint64_t span = hi >= lo ? hi - lo : 0;
  int L = 0;
  while (L < 64 && (span >> L)) ++L;
  *bias = lo;
  *shift = std::max(0, L - kTopBits);
  return span > 0 && *shift < key_bits - kTopBits;
}

// Digit range [a, b) of group `code` (a == b: empty).  The table is monotone
// in rank * K + round over the digits, so each group's digits are contiguous.
inline void digit_range(const uint8_t* lut, int code, int* a, int* b) {
  int first = -1, last = -1;
  for (int g = 0; g < kTopDigits; ++g)
    if (lut[g] == code) {
      if (first < 0) first = g;
      last = g;
    }
  *a = first < 0 ? 0 : first;
  *b = first < 0 ? 0 : last + 1;
}

// The exchange and the receivers' piece tables.  Rank s's partition holds its
// keys in digit order (part_start[s][g] = start of digit g).  Round i sends
// rank s's digits [a, b) of group (d, i) to rank d, into d's receive buffer
// at roff[d][i] + (keys of the earlier sources): pieces in source order.  The
// round sort of rank d, round i sees piece (s, g) at offset src_base + (keys
// of s's digits a..g-1) -- listed digit-major, source-minor, segment g - a.
struct DigitPlan {
  int R = 0, K = 0;
  std::vector<int> lo, hi;                     // [R*K] digit range of group code i*R + d
  std::vector<uint64_t> roff;                  // [R][K+1]
  std::vector<uint64_t> n_recv;                // [R]
  std::vector<std::vector<Piece>> rounds;      // [K] exchange pieces
  // [R][K] the round sort's pieces (offsets within the round's receive region)
  std::vector<std::vector<uint64_t>> p_off, p_len;
  std::vector<std::vector<uint32_t>> p_seg;
};

// Parts (round 5): a rank may partition its keys in H
// parts one after the other (part h = its input keys [first[h], first[h+1]),
// stably partitioned into the same range of its send buffer), so that the
// exchange of the first part can start while the next is partitioned.  Cp
// holds R * H rows (row s * H + h: part h of rank s); lut comes from the
// rank totals.  A (rank, round) piece becomes one piece per part, in part
// order, so a receiver still gets every source's keys in input order (the
// pair sort's stability) and its round sort sees (source, part, digit)
// pieces.  H = 1 is digit_plan.
inline DigitPlan digit_plan_parts(const std::vector<std::vector<uint64_t>>& Cp, int H,
                                  const std::vector<uint64_t>& first, const uint8_t* lut, int K) {
  DigitPlan p;
  const int V = (int)Cp.size(), R = H > 0 ? V / H : 0;  // V: (rank, part) sources
  p.R = R;
  p.K = K;
  p.lo.assign((size_t)R * K, 0);
  p.hi.assign((size_t)R * K, 0);
  for (int c = 0; c < R * K; ++c) digit_range(lut, c, &p.lo[c], &p.hi[c]);
  // start[v][g]: digit g of source v in its rank's send buffer
  std::vector<std::vector<uint64_t>> start(V, std::vector<uint64_t>(kTopDigits + 1, 0));
  for (int v = 0; v < V; ++v) {
    start[v][0] = first.empty() ? 0 : first[v];
    for (int g = 0; g < kTopDigits; ++g) start[v][g + 1] = start[v][g] + Cp[v][g];
  }
  p.roff.assign((size_t)R * (K + 1), 0);
  p.n_recv.assign(R, 0);
  p.rounds.assign(K, {});
  p.p_off.assign((size_t)R * K, {});
  p.p_len.assign((size_t)R * K, {});
  p.p_seg.assign((size_t)R * K, {});
  for (int d = 0; d < R; ++d) {
    uint64_t run = 0;
    for (int i = 0; i < K; ++i) {
      p.roff[(size_t)d * (K + 1) + i] = run;
      const int a = p.lo[(size_t)i * R + d], b = p.hi[(size_t)i * R + d];
      std::vector<uint64_t> base(V, 0);
      uint64_t at = 0;
      for (int v = 0; v < V; ++v) {
        base[v] = at;
        const uint64_t m = start[v][b] - start[v][a];
        if (m) p.rounds[i].push_back(Piece{v / H, d, start[v][a], run + at, m, v % H});
        at += m;
      }
      const size_t q = (size_t)d * K + i;
      for (int g = a; g < b; ++g)
        for (int v = 0; v < V; ++v) {
          p.p_off[q].push_back(base[v] + (start[v][g] - start[v][a]));
          p.p_len[q].push_back(Cp[v][g]);
          p.p_seg[q].push_back((uint32_t)(g - a));
        }
      run += at;
    }
    p.roff[(size_t)d * (K + 1) + K] = run;
    p.n_recv[d] = run;
  }
  return p;
}

inline DigitPlan digit_plan(const std::vector<std::vector<uint64_t>>& C, const uint8_t* lut, int K) {
  return digit_plan_parts(C, 1, {}, lut, K);
}

// Where a rank's keys are cut into two partition parts: half, rounded down to
// whole 8192-key tiles (the second part's tiles stay 16-byte aligned for the
// count kernel's vector loads); 0 (one part) below two tiles.
inline uint64_t part_split(uint64_t n) { return (n / 2) & ~(uint64_t)8191; }

// The equal re-cut without copying what stays.  Rank r's sorted rounds hold
// global positions [G_r + roff[r][i], G_r + roff[r][i+1]) (G_r = keys of the
// ranks before it); its output shard is [min(N, r*S), min(N, (r+1)*S)).  A
// round that lies inside the shard is sorted straight into the output at
// out_off (direct); any other round is sorted into the rank's scratch at its
// roff, and `moves` carries its pieces to the shards they belong to (src_off
// in the rank's local order, dst_off in the destination shard).
struct Placement {
  std::vector<char> direct;       // [R][K]
  std::vector<uint64_t> out_off;  // [R][K]
  std::vector<Piece> moves;
};

inline Placement place_rounds(const std::vector<uint64_t>& roff, const std::vector<uint64_t>& n_recv, int K) {
  const int R = (int)n_recv.size();
  uint64_t N = 0;
  for (uint64_t x : n_recv) N += x;
  const uint64_t S = shard_size(N, R);
  auto cut = [&](int d) { return std::min<uint64_t>(N, (uint64_t)d * S); };
  Placement pl;
  pl.direct.assign((size_t)R * K, 0);
  pl.out_off.assign((size_t)R * K, 0);
  uint64_t G = 0;
  for (int r = 0; r < R; ++r) {
    const uint64_t s0 = cut(r), s1 = (r == R - 1) ? N : cut(r + 1);
    for (int i = 0; i < K; ++i) {
      const uint64_t a = G + roff[(size_t)r * (K + 1) + i], b = G + roff[(size_t)r * (K + 1) + i + 1];
      if (b == a) continue;
      const size_t q = (size_t)r * K + i;
      if (a >= s0 && b <= s1) {
        pl.direct[q] = 1;
        pl.out_off[q] = a - s0;
        continue;
      }
      for (int d = 0; d < R; ++d) {
        const uint64_t d0 = cut(d), d1 = (d == R - 1) ? N : cut(d + 1);
        const uint64_t x = std::max(a, d0), y = std::min(b, d1);
        if (y > x) pl.moves.push_back(Piece{r, d, x - G, x - d0, y - x});
      }
    }
    G += n_recv[r];
  }
  return pl;
}

// ---------------------------------------------------------------------------
// gap-coded rounds ("msdz", distrib.cpp run_coded_rounds): the same digit
// plan, but each sender sorts its (round, destination) pieces and sends them
// as 64-key groups of gaps -- one base word, then 2w words of w-bit gaps (w =
// the bits of the piece's largest gap; libsort.h libsortDeltaPackU32).
// ---------------------------------------------------------------------------
inline uint64_t delta_words(uint64_t n, uint32_t w) { return (n + 63) / 64 * (1 + 2 * (uint64_t)w); }
inline uint32_t gap_bits(uint32_t maxgap) {
  uint32_t b = 0;
  while (b < 32 && (maxgap >> b)) ++b;
  return b;
}

struct CodedPlan {
  int R = 0, K = 0;
  std::vector<std::vector<uint64_t>> start;   // [R][257]: digit g's start in rank s's partition
  std::vector<std::vector<uint64_t>> M;       // [R][R*K]: keys rank s sends in group i * R + d
  std::vector<std::vector<uint64_t>> coff;    // [R][R*K+1]: coded send regions (32-bit gaps: worst case)
  std::vector<std::vector<uint64_t>> cr_off;  // [R][R*K]: receiver d's coded region of (round i, source s) at i * R + s
  std::vector<uint64_t> rcap;                 // [R]: coded receive words (worst case)
  std::vector<char> self_only;                // [R*K] (rank r, round i) at r * K + i: only r's own piece, uncoded
};

// self_coded: a rank's own piece is coded and sent through the communicator
// too (one-rank RCCL tests); otherwise it stays put, uncoded.  Every layout is
// at worst-case (32-bit) widths, so no round depends on a later round's gaps.
inline CodedPlan coded_plan(const DigitPlan& p, const std::vector<std::vector<uint64_t>>& C, bool self_coded) {
  CodedPlan c;
  const int R = p.R, K = p.K;
  c.R = R;
  c.K = K;
  auto remote = [&](int s, int d) { return s != d || self_coded; };
  c.start.assign(R, std::vector<uint64_t>(kTopDigits + 1, 0));
  for (int s = 0; s < R; ++s)
    for (int g = 0; g < kTopDigits; ++g) c.start[s][g + 1] = c.start[s][g] + C[s][g];
  c.M.assign(R, std::vector<uint64_t>((size_t)R * K, 0));
  c.coff.assign(R, std::vector<uint64_t>((size_t)R * K + 1, 0));
  for (int s = 0; s < R; ++s)
    for (int j = 0; j < R * K; ++j) {
      c.M[s][j] = c.start[s][p.hi[j]] - c.start[s][p.lo[j]];
      c.coff[s][j + 1] = c.coff[s][j] + (remote(s, j % R) ? delta_words(c.M[s][j], 32) : 0);
    }
  c.cr_off.assign(R, std::vector<uint64_t>((size_t)R * K, 0));
  c.rcap.assign(R, 0);
  c.self_only.assign((size_t)R * K, 0);
  for (int d = 0; d < R; ++d) {
    uint64_t o = 0;
    for (int i = 0; i < K; ++i) {
      bool others = false;
      for (int s = 0; s < R; ++s) {
        const uint64_t m = c.M[s][(size_t)i * R + d];
        c.cr_off[d][(size_t)i * R + s] = o;
        if (remote(s, d)) o += delta_words(m, 32);
        if (s != d && m) others = true;
      }
      c.self_only[(size_t)d * K + i] = !others && !remote(d, d);
    }
    c.rcap[d] = o;
  }
  return c;
}

// The coded exchange of round i: maxgap[s * stride + i * R + d] = the largest
// gap of rank s's piece for d (read back after round i's coding).
inline std::vector<Piece> coded_round_pieces(const CodedPlan& c, int i, const uint32_t* maxgap, size_t stride,
                                             bool self_coded) {
  std::vector<Piece> ps;
  const int R = c.R;
  for (int s = 0; s < R; ++s)
    for (int d = 0; d < R; ++d) {
      const size_t j = (size_t)i * R + d;
      if ((s == d && !self_coded) || !c.M[s][j]) continue;
      ps.push_back(Piece{s, d, c.coff[s][j], c.cr_off[d][(size_t)i * R + s],
                         delta_words(c.M[s][j], gap_bits(maxgap[(size_t)s * stride + j]))});
    }
  return ps;
}

// ---------------------------------------------------------------------------
// BSP LSD round ("lsd", the reference's semantics)
// ---------------------------------------------------------------------------
// C[s][b] = keys of rank s in bucket b after its local stable partition
// (bucket starts from gpuPartial's boundaries).  The global order of the
// round is bucket-major, rank-minor; rank r receives positions [r*S,
// (r+1)*S).  Rank s's data for rank d is ONE contiguous slice of its
// partitioned shard (local order -> global position is monotone), so the
// exchange pieces are contiguous; the receiver then gathers its pieces into
// bucket-major order with the segment table `seg` (src offsets in its
// receive buffer, which holds the pieces in source-rank order).
struct LsdRound {
  std::vector<Piece> pieces;                       // send slices (src_off in the sender's shard, dst_off in recv)
  std::vector<uint64_t> n_next;                    // [R]: keys per rank after the round
  std::vector<std::vector<uint64_t>> seg_src, seg_dst, seg_len;  // [R]: gather table of each receiver
};

inline LsdRound lsd_round(const std::vector<std::vector<uint64_t>>& C, uint64_t S) {
  const int R = (int)C.size();
  const size_t nb = R ? C[0].size() : 0;
  LsdRound o;
  o.n_next.assign(R, 0);
  o.seg_src.assign(R, {});
  o.seg_dst.assign(R, {});
  o.seg_len.assign(R, {});
  // G[s][b]: global start of (s, b); L[s][b]: local start
  std::vector<std::vector<uint64_t>> G(R, std::vector<uint64_t>(nb)), L(R, std::vector<uint64_t>(nb));
  uint64_t g = 0;
  for (size_t b = 0; b < nb; ++b)
    for (int s = 0; s < R; ++s) {
      G[s][b] = g;
      g += C[s][b];
    }
  for (int s = 0; s < R; ++s) {
    uint64_t l = 0;
    for (size_t b = 0; b < nb; ++b) {
      L[s][b] = l;
      l += C[s][b];
    }
  }
  // walk the (s, b) runs cut at shard boundaries: fn(s, d, local start,
  // position in shard d, length)
  auto walk = [&](bool bucket_major, auto&& fn) {
    const size_t outer = bucket_major ? nb : (size_t)R, inner = bucket_major ? (size_t)R : nb;
    for (size_t x = 0; x < outer; ++x)
      for (size_t y = 0; y < inner; ++y) {
        const int s = (int)(bucket_major ? y : x);
        const size_t bk = bucket_major ? x : y;
        uint64_t a = G[s][bk], left = C[s][bk], la = L[s][bk];
        while (left) {
          const int d = S ? (int)std::min<uint64_t>(a / S, (uint64_t)R - 1) : R - 1;
          const uint64_t hi = (d == R - 1) ? a + left : std::min(a + left, (uint64_t)(d + 1) * S);
          const uint64_t m = hi - a;
          fn(s, d, la, a - (uint64_t)d * S, m);
          a += m;
          la += m;
          left -= m;
        }
      }
  };
  // send counts M[s][d] and where each slice starts in the sender's shard
  // (rank-major walk: for fixed s the local order is the global order)
  std::vector<std::vector<uint64_t>> M(R, std::vector<uint64_t>(R, 0)), first(R, std::vector<uint64_t>(R, UINT64_MAX));
  walk(false, [&](int s, int d, uint64_t la, uint64_t, uint64_t m) {
    if (first[s][d] == UINT64_MAX) first[s][d] = la;
    M[s][d] += m;
  });
  // receive buffer of d: the slices in source-rank order
  std::vector<std::vector<uint64_t>> base(R, std::vector<uint64_t>(R, 0));
  for (int d = 0; d < R; ++d) {
    uint64_t run = 0;
    for (int s = 0; s < R; ++s) {
      base[s][d] = run;
      run += M[s][d];
    }
    o.n_next[d] = run;
  }
  for (int s = 0; s < R; ++s)
    for (int d = 0; d < R; ++d)
      if (M[s][d]) o.pieces.push_back(Piece{s, d, first[s][d], base[s][d], M[s][d]});
  // gather tables in the round's global order (bucket-major, rank-minor)
  walk(true, [&](int s, int d, uint64_t la, uint64_t pos, uint64_t m) {
    o.seg_src[d].push_back(base[s][d] + (la - first[s][d]));
    o.seg_dst[d].push_back(pos);
    o.seg_len[d].push_back(m);
  });
  return o;
}

}  // namespace dplan
}  // namespace lsort
