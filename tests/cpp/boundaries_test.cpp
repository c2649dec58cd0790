// boundaries_test.cpp -- csrc/boundaries.h (the reference GetBoundaries
// result derived from the exclusive prefix, used by gpuPartial's
// reference mode) against the oracle's direct restatement of sort.cu:367-394
// (oracle_ref_boundaries) on many sorted inputs, including the cases where
// they differ (group 1 empty, first non-empty group >= 2).  Run under
// ASan/UBSan by tests/test_distrib_plan_cpu.py.
#include <stdio.h>

#include <algorithm>
#include <random>
#include <vector>

#include "../../oracle/oracle.cpp"
#include "boundaries.h"

int main() {
  std::mt19937_64 g(11);
  int fails = 0, cases = 0, differ = 0;
  for (int it = 0; it < 4000; ++it) {
    const int width = 1 + (int)(g() % 10);
    const uint32_t offset = (uint32_t)(g() % (33 - width));
    const size_t n = (size_t)(g() % 300);
    const uint32_t span = 1u + (uint32_t)(g() % (1u << width));  // few groups -> many empty ones
    const uint32_t skip = (uint32_t)(g() % 3);                    // often leave groups 0..1 empty
    std::vector<uint32_t> x(n);
    for (auto& v : x) {
      const uint64_t grp = std::min<uint64_t>(skip + g() % span, (1ull << width) - 1);
      v = (uint32_t)((grp << offset) | (g() & ((1ull << offset) - 1)));
    }
    std::vector<uint32_t> prefix(1u << width);
    oracle_partial_u32(x.data(), prefix.data(), n, offset, width);  // x is now the stable partition
    std::vector<uint32_t> want(1u << width), got(prefix);
    oracle_ref_boundaries(x.data(), n, offset, width, want.data());
    lsort::reference_boundaries_from_prefix(got.data(), got.size(), n);
    ++cases;
    if (got != want) {
      if (fails++ < 5) fprintf(stderr, "FAIL width %d offset %u n %zu\n", width, offset, n);
    }
    if (prefix != want) ++differ;
  }
  // SURVEY.md section 8a's two examples
  {
    uint32_t a[] = {4, 0, 7, 2, 0, 2}, p[4];
    oracle_partial_u32(a, p, 6, 0, 2);
    lsort::reference_boundaries_from_prefix(p, 4, 6);
    const uint32_t w[] = {0, 0, 3, 5};
    for (int i = 0; i < 4; ++i) fails += p[i] != w[i];
  }
  {
    uint32_t a[] = {2, 3, 2, 3}, p[4];
    oracle_partial_u32(a, p, 4, 0, 2);
    lsort::reference_boundaries_from_prefix(p, 4, 4);
    const uint32_t w[] = {0, 0, 2, 2};
    for (int i = 0; i < 4; ++i) fails += p[i] != w[i];
  }
  if (fails || differ == 0) {
    fprintf(stderr, "%d failures of %d cases (%d where the quirk shows)\n", fails, cases, differ);
    return 1;
  }
  printf("OK %d cases (%d where the reference differs from the exclusive prefix)\n", cases, differ);
  return 0;
}
