// test_parallel.cpp -- native restatement of the reference's concurrency
// test (benchmark/pkg/sort/libsort_test.go:35-87, TestParallel: 16 callers
// of GpuFull on 4099 keys, then 16 of GpuPartial on 1021 keys at width 8,
// each phase within a 2 s timeout), calling libsort.so through include/
// libsort.h as a C/C++ (or cgo) caller does -- with the image's HIP runtime,
// not torch's.  Also: 8 concurrent gpuDistribSort callers mixed with
// single-device callers (the pool's multi-device reservation), and the
// reference's generator golden words.  Exit 0 = pass.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <future>
#include <thread>
#include <vector>

#include "libsort.h"

static std::atomic<int> g_fail{0};
#define EXPECT(c, ...)                                     \
  do {                                                     \
    if (!(c)) {                                            \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                        \
      fprintf(stderr, "\n");                               \
      g_fail++;                                            \
    }                                                      \
  } while (0)

static std::vector<uint32_t> inputs(size_t n) {
  std::vector<uint32_t> v(n);
  populateInput(v.data(), n);  // GenerateInputs (libsort.go / utils.cu:65-80)
  return v;
}

// TestLocal: GpuFull on 4099 keys, checked against std::sort
static void test_local() {
  std::vector<uint32_t> x = inputs(4099), ref = x;
  EXPECT(providedGpu(x.data(), x.size()), "providedGpu: %s", libsortLastError());
  std::sort(ref.begin(), ref.end());
  EXPECT(x == ref, "full sort differs");
}

// TestLocalPartial + checkPartial (testHelpers.go:411-448): 1021 keys, width 8
static void test_local_partial() {
  const int width = 8, nb = 1 << width;
  std::vector<uint32_t> x = inputs(1021), ref = x, b(nb);
  EXPECT(gpuPartial(x.data(), b.data(), x.size(), 0, width), "gpuPartial: %s", libsortLastError());
  std::stable_sort(ref.begin(), ref.end(), [](uint32_t a, uint32_t c) { return (a & 255u) < (c & 255u); });
  EXPECT(x == ref, "partial sort differs from the stable partition");
  size_t at = 0;
  for (int g = 0; g < nb; ++g) {
    EXPECT(b[g] == at, "boundary %d = %u, want %zu", g, b[g], at);
    while (at < x.size() && (int)(x[at] & 255u) == g) ++at;
  }
}

static void test_distrib(int ngpu, size_t n) {
  std::vector<uint32_t> x = inputs(n), ref = x;
  EXPECT(gpuDistribSort(x.data(), x.size(), ngpu), "gpuDistribSort: %s", libsortLastError());
  std::sort(ref.begin(), ref.end());
  EXPECT(x == ref, "distributed sort differs (n=%zu)", n);
}

template <typename Fn>
static bool run_parallel(const char* name, int k, Fn fn, double timeout_s) {
  std::vector<std::future<void>> fs;
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < k; ++i) fs.push_back(std::async(std::launch::async, [&, i] { fn(i); }));
  bool ok = true;
  for (auto& f : fs) {
    const auto left = std::chrono::duration<double>(timeout_s) - (std::chrono::steady_clock::now() - t0);
    if (f.wait_for(std::chrono::duration_cast<std::chrono::milliseconds>(left)) != std::future_status::ready) ok = false;
  }
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  printf("%s: %d callers, %.3f s%s\n", name, k, s, ok ? "" : " TIMEOUT");
  EXPECT(ok, "%s timed out (%.1f s limit)", name, timeout_s);
  return ok;
}

int main() {
  // the reference generator's first words (utils.cu:65-80)
  {
    std::vector<uint32_t> w = inputs(8);
    const uint32_t want[8] = {0x285594ea, 0x190ca349, 0xcbc42ff2, 0xd6508153,
                              0xc2a8052f, 0x0f55ac5f, 0xd6ff3e32, 0x4f46689c};
    EXPECT(memcmp(w.data(), want, sizeof(want)) == 0, "populateInput golden words");
  }
  if (!initLibSort()) {
    fprintf(stderr, "initLibSort failed: %s\n", libsortLastError());
    return 2;
  }
  EXPECT(!initLibSort(), "a second initLibSort must fail (utils.cu:14-17)");
  // warm the device (first-use allocation, code object load) outside the timed phases
  test_local();
  test_local_partial();
  test_distrib(1, 5000);
  const int nparallel = 16;  // libsort_test.go:37
  if (!run_parallel("Complete Sort", nparallel, [](int) { test_local(); }, 2.0)) return 1;
  if (!run_parallel("Partial Sort", nparallel, [](int) { test_local_partial(); }, 2.0)) return 1;
  // multi-device reservations mixed with single-device callers
  if (!run_parallel("Distributed + single", 8,
                    [](int i) {
                      if (i % 2)
                        test_distrib(1, 100003 + 17 * i);
                      else
                        test_local();
                    },
                    20.0))
    return 1;
  if (g_fail) {
    fprintf(stderr, "%d failures\n", g_fail.load());
    return 1;
  }
  printf("OK\n");
  return 0;
}
