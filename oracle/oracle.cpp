// oracle.cpp -- CPU restatement of the reference libsort path.  TEST
// INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and the
// cpu_baseline leg of bench.py as the checker.  The product (libsort.so)
// never links, loads or calls anything in oracle/.
//
// Parity is pinned by the reference's own outputs: the PCG32 golden words and
// sha256 table recorded from the reference utils.cu (committed
// as tests/golden/pcg_golden.json), and by the reference C++ harness
// localTest/{tests,benchmarks}.cpp compiled against libsort.so (oracle/_ref).
//
// Every function cites the reference code it restates (paths relative to the
// reference checkout).
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

// std::stable_sort / std::sort of large arrays on several host threads (the
// checker of the GPU tests sorts up to 2^28 elements; one thread took ~20 s
// per 2^27 pairs on the box): T contiguous chunks sorted each by the same std
// algorithm, then merged pairwise with std::merge, which keeps elements of the
// earlier chunk first among equals -- so the result is exactly the one-thread
// std::stable_sort (and, for keys only, std::sort) result.
namespace {
unsigned host_threads(size_t n) {
  if (n < ((size_t)1 << 20)) return 1;
  const unsigned h = std::thread::hardware_concurrency();
  return std::max(1u, std::min(16u, h ? h : 1u));
}

template <typename T, typename Cmp>
void par_sort(T* a, size_t n, Cmp cmp, bool stable) {
  const unsigned nt = host_threads(n);
  if (nt == 1) {
    if (stable) std::stable_sort(a, a + n, cmp); else std::sort(a, a + n, cmp);
    return;
  }
  std::vector<size_t> c(nt + 1);
  for (unsigned t = 0; t <= nt; ++t) c[t] = n * t / nt;
  std::vector<std::thread> th;
  for (unsigned t = 0; t < nt; ++t)
    th.emplace_back([&, t] {
      if (stable) std::stable_sort(a + c[t], a + c[t + 1], cmp); else std::sort(a + c[t], a + c[t + 1], cmp);
    });
  for (auto& x : th) x.join();
  std::vector<T> buf(n);
  T* src = a;
  T* dst = buf.data();
  for (unsigned w = 1; w < nt; w *= 2) {
    th.clear();
    for (unsigned i = 0; i < nt; i += 2 * w)
      th.emplace_back([&, i] {
        const size_t lo = c[i], mid = c[std::min(nt, i + w)], hi = c[std::min(nt, i + 2 * w)];
        std::merge(src + lo, src + mid, src + mid, src + hi, dst + lo, cmp);
      });
    for (auto& x : th) x.join();
    std::swap(src, dst);
  }
  if (src != a) std::copy(src, src + n, a);
}

// stable sort of (key, value) pairs by key, through packed records
template <typename K, typename V>
void stable_sort_kv(K* k, V* v, size_t n) {
  struct E {
    K k;
    V v;
  };
  std::vector<E> e(n);
  for (size_t i = 0; i < n; ++i) e[i] = E{k[i], v[i]};
  par_sort(e.data(), n, [](const E& x, const E& y) { return x.k < y.k; }, true);
  for (size_t i = 0; i < n; ++i) {
    k[i] = e[i].k;
    v[i] = e[i].v;
  }
}
}  // namespace

extern "C" {

// utils.cu:65-80 (populateInput): PCG32 XSH-RR.  `state` is in/out so the
// caller can reproduce the reference's process-wide persistence.
void oracle_pcg_fill(uint32_t* out, size_t n, uint64_t* state) {
  const uint64_t mult = 6364136223846793005ull, inc = 1442695040888963407ull;
  uint64_t s = *state;
  for (size_t i = 0; i < n; ++i) {
    uint64_t x = s;
    const unsigned count = (unsigned)(x >> 59);
    s = x * mult + inc;
    x ^= x >> 18;
    const uint32_t v = (uint32_t)(x >> 27);
    out[i] = (v >> count) | (v << ((0u - count) & 31u));
  }
  *state = s;
}

uint64_t oracle_pcg_initial_state(void) { return 0x4d595df4d0f33173ull; }  // utils.cu:67

// invokers.cu:68-71 (providedCpu): std::sort.
void oracle_sort_u32(uint32_t* a, size_t n) { par_sort(a, n, std::less<uint32_t>(), false); }

// The gpuPartial contract (invokers.cu:15-41 as checked by localTest/tests.cpp:
// 41-83 and benchmark/pkg/sort/testHelpers.go:411-448): stable partition by
// the group (x >> offset) & (2^width-1); bounds[g] = #elements with group < g.
// Restated as a counting sort.
void oracle_partial_u32(uint32_t* a, uint32_t* bounds, size_t n, uint32_t offset, uint32_t width) {
  const size_t ng = (size_t)1 << width;
  const uint32_t mask = (uint32_t)(ng - 1);
  std::vector<uint64_t> cnt(ng + 1, 0);
  for (size_t i = 0; i < n; ++i) cnt[((uint32_t)((uint64_t)a[i] >> offset) & mask) + 1]++;
  for (size_t g = 1; g <= ng; ++g) cnt[g] += cnt[g - 1];
  if (bounds)
    for (size_t g = 0; g < ng; ++g) bounds[g] = (uint32_t)cnt[g];
  std::vector<uint32_t> out(n);
  for (size_t i = 0; i < n; ++i) out[cnt[(uint32_t)((uint64_t)a[i] >> offset) & mask]++] = a[i];
  if (n) memcpy(a, out.data(), n * sizeof(uint32_t));
}

// Exact emulation of SortState::Step (sort.cu:322-346): for shift = offset,
// offset+2, ... < offset+width: gpu_radix_sort_local (sort.cu:29-184) on
// 128-key blocks (2-bit digit, per-block exclusive rank of each key within
// its digit, digit-major block sums d_block_sums[i*G+blk]), sum_scan_blelloch
// (scan.cu:165-250: exclusive scan of the 4G block sums), gpu_glbl_shuffle
// (sort.cu:186-213: out[scan[d*G+blk] + rank] = key).  An odd width covers one
// extra bit, exactly like the reference loop.
void oracle_ref_step_u32(uint32_t* a, size_t n, uint32_t offset, uint32_t width) {
  const size_t B = 128;  // MAX_BLOCK_SZ, sort.cu:5
  const size_t G = (n + B - 1) / B;
  std::vector<uint32_t> local(n), prefix(n), sums(4 * G), scan(4 * G), out(n);
  for (uint32_t shift = offset; shift < offset + width; shift += 2) {
    for (size_t blk = 0; blk < G; ++blk) {
      const size_t lo = blk * B, hi = std::min(n, lo + B);
      uint32_t c[4] = {0, 0, 0, 0};
      for (size_t i = lo; i < hi; ++i) {
        const uint32_t d = (a[i] >> shift) & 3u;
        prefix[i] = c[d]++;  // exclusive rank within digit
      }
      uint32_t start[4], run = 0;
      for (int d = 0; d < 4; ++d) {
        start[d] = run;
        run += c[d];
        sums[d * G + blk] = c[d];
      }
      // local shuffle: keys and their ranks to the locally sorted position
      std::vector<uint32_t> lk(hi - lo), lp(hi - lo);
      for (size_t i = lo; i < hi; ++i) {
        const uint32_t d = (a[i] >> shift) & 3u;
        const uint32_t pos = start[d] + prefix[i];
        lk[pos] = a[i];
        lp[pos] = prefix[i];
      }
      for (size_t i = lo; i < hi; ++i) {
        local[i] = lk[i - lo];
        prefix[i] = lp[i - lo];
      }
    }
    uint32_t run = 0;
    for (size_t i = 0; i < 4 * G; ++i) {
      scan[i] = run;
      run += sums[i];
    }
    for (size_t i = 0; i < n; ++i) {
      const uint32_t d = (local[i] >> shift) & 3u;
      out[scan[d * G + i / B] + prefix[i]] = local[i];
    }
    if (n) memcpy(a, out.data(), n * sizeof(uint32_t));
  }
}

// SortState::GetBoundaries (sort.cu:367-394) exactly, including its quirk:
// gpu_groups writes b[g(i)] = i where g(i) != g(i-1) over a zeroed array,
// then the host fills empty groups from the top down to group 2 only.
void oracle_ref_boundaries(const uint32_t* sorted, size_t n, uint32_t offset, uint32_t width,
                           uint32_t* b) {
  const size_t ng = (size_t)1 << width;
  const uint32_t mask = (uint32_t)(ng - 1);
  for (size_t g = 0; g < ng; ++g) b[g] = 0;
  for (size_t i = 0; i < n; ++i) {
    const size_t prev = i == 0 ? 0 : i - 1;
    const uint32_t g = (sorted[i] >> offset) & mask, pg = (sorted[prev] >> offset) & mask;
    if (g != pg) b[g] = (uint32_t)i;
  }
  uint32_t prev = (uint32_t)n;
  for (long long g = (long long)ng - 1; g > 1; --g) {
    if (b[g] == 0) b[g] = prev;
    prev = b[g];
  }
}

// localTest/benchmarks.cpp:70-160 (distribSort): two partitions of len/2 and
// len/2 + len%2 keys, each partial-sorted by one `width`-bit digit per step,
// then a host shuffle in bucket-major, partition-minor order.
void oracle_distrib_local_u32(uint32_t* data, size_t len, uint32_t width) {
  const size_t nb = (size_t)1 << width;
  const uint32_t nstep = 32 / width;
  const size_t p1len = len / 2, p2len = len / 2 + len % 2;
  std::vector<uint32_t> tmp(len), b1(nb), b2(nb);
  uint32_t* cur = data;
  uint32_t* next = tmp.data();
  for (uint32_t s = 0; s < nstep; ++s) {
    uint32_t* p1 = cur;
    uint32_t* p2 = cur + p1len;
    oracle_partial_u32(p1, b1.data(), p1len, s * width, width);
    oracle_partial_u32(p2, b2.data(), p2len, s * width, width);
    size_t slot = 0;
    for (size_t bkt = 0; bkt < nb; ++bkt) {
      const size_t l1 = (bkt == nb - 1 ? p1len : b1[bkt + 1]) - b1[bkt];
      const size_t l2 = (bkt == nb - 1 ? p2len : b2[bkt + 1]) - b2[bkt];
      memcpy(next + slot, p1 + b1[bkt], l1 * sizeof(uint32_t));
      slot += l1;
      memcpy(next + slot, p2 + b2[bkt], l2 * sizeof(uint32_t));
      slot += l2;
    }
    std::swap(cur, next);
  }
  if (cur != data) memcpy(data, cur, len * sizeof(uint32_t));
}

// benchmark/pkg/sort/distrib.go:90-179 (SortDistribFromArr) with the STRIDED
// BucketReader (helpers.go:67-121): per step, the previous outputs are read
// bucket-major / worker-minor and re-cut into chunks of ceil(N/nworker) keys
// (distrib.go:113); each worker partial-sorts its chunk by the step's digit.
// Writes the final per-worker output lengths to shard_lens (nworker entries);
// `a` receives the concatenation of the final outputs (read STRIDED).
void oracle_distrib_bsp_u32(uint32_t* a, size_t n, uint32_t nworker, uint32_t width, uint64_t* shard_lens) {
  const size_t nb = (size_t)1 << width;
  const uint32_t nstep = 32 / width;
  const size_t per = nworker ? (n + nworker - 1) / nworker : 0;
  // outputs[w] = (data, bucket boundaries) of worker w
  std::vector<std::vector<uint32_t>> out_data(1, std::vector<uint32_t>(a, a + n));
  std::vector<std::vector<uint32_t>> out_bounds(1, std::vector<uint32_t>(1, 0));
  size_t out_nb = 1;  // the raw input is one array with one part
  for (uint32_t s = 0; s < nstep; ++s) {
    // STRIDED read of the previous outputs: for each bucket, for each array
    std::vector<uint32_t> stream;
    stream.reserve(n);
    for (size_t b = 0; b < out_nb; ++b)
      for (size_t w = 0; w < out_data.size(); ++w) {
        const auto& d = out_data[w];
        const size_t lo = out_bounds[w][b];
        const size_t hi = b + 1 < out_nb ? out_bounds[w][b + 1] : d.size();
        stream.insert(stream.end(), d.begin() + lo, d.begin() + hi);
      }
    std::vector<std::vector<uint32_t>> nd(nworker);
    std::vector<std::vector<uint32_t>> nbnd(nworker, std::vector<uint32_t>(nb, 0));
    for (uint32_t w = 0; w < nworker; ++w) {
      const size_t lo = std::min(n, (size_t)w * per), hi = std::min(n, lo + per);
      nd[w].assign(stream.begin() + lo, stream.begin() + hi);
      oracle_partial_u32(nd[w].data(), nbnd[w].data(), nd[w].size(), s * width, width);
    }
    out_data.swap(nd);
    out_bounds.swap(nbnd);
    out_nb = nb;
  }
  // final STRIDED read (distrib.go:217-230)
  size_t k = 0;
  for (size_t b = 0; b < out_nb; ++b)
    for (size_t w = 0; w < out_data.size(); ++w) {
      const auto& d = out_data[w];
      const size_t lo = out_bounds[w][b];
      const size_t hi = b + 1 < out_nb ? out_bounds[w][b + 1] : d.size();
      for (size_t i = lo; i < hi; ++i) a[k++] = d[i];
    }
  if (shard_lens)
    for (size_t w = 0; w < out_data.size(); ++w) shard_lens[w] = out_data[w].size();
}

// Stable key/value sorts (BASELINE configs C5): std::stable_sort by key over
// the original order (par_sort above: per-chunk std::stable_sort + stable
// merges).  No reference function exists for KV; this is the definition of
// the result.
void oracle_stable_sort_kv64(uint64_t* k, uint32_t* v, size_t n) { stable_sort_kv(k, v, n); }

void oracle_stable_sort_kv32(uint32_t* k, uint32_t* v, size_t n) { stable_sort_kv(k, v, n); }

// 64-bit keys only / with 64-bit payloads (no
// reference function: std::sort defines the keys-only result, std::stable_sort
// by key over the original order the pair result).
void oracle_sort_u64(uint64_t* k, size_t n) { par_sort(k, n, std::less<uint64_t>(), false); }

void oracle_stable_sort_kv64v64(uint64_t* k, uint64_t* v, size_t n) { stable_sort_kv(k, v, n); }

// The sorted order of a keys-only array is fixed by how often each value
// occurs (std::sort, invokers.cu:68-71, has a unique result), so the sorted
// PCG stream at sizes std::sort cannot finish in seconds is restated as a
// counting sort: counts[v] = occurrences of v among elements [first,
// first+n) of the fresh-process populateInput stream (utils.cu:65-80),
// generated here (no key array is stored).  counts has 2^32 one-byte
// entries; returns the largest count (the caller rejects 255 = saturation).
uint32_t oracle_pcg_value_counts(uint8_t* counts, size_t n, uint64_t first) {
  const uint64_t mult = 6364136223846793005ull, inc = 1442695040888963407ull;
  // skip-ahead: state after `first` steps (LCG jump by squaring)
  uint64_t s = 0x4d595df4d0f33173ull, am = mult, ac = inc, m = 1, c = 0;
  for (uint64_t k = first; k; k >>= 1) {
    if (k & 1) {
      m *= am;
      c = c * am + ac;
    }
    ac = (am + 1) * ac;
    am *= am;
  }
  s = m * s + c;
  uint32_t mx = 0;
  for (size_t i = 0; i < n; ++i) {
    uint64_t x = s;
    const unsigned count = (unsigned)(x >> 59);
    s = x * mult + inc;
    x ^= x >> 18;
    const uint32_t v = (uint32_t)(x >> 27);
    const uint32_t key = (v >> count) | (v << ((0u - count) & 31u));
    const uint32_t q = counts[key];
    if (q < 255) counts[key] = (uint8_t)(q + 1);
    if (q + 1 > mx) mx = q + 1;
  }
  return mx;
}

}  // extern "C"
