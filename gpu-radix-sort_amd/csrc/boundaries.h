// boundaries.h -- the reference's GetBoundaries result (quirk included) from
// the exclusive prefix of group counts.  Header-only host code, shared by
// libsort_abi.cpp (gpuPartial under LIBSORT_BOUNDARIES=reference /
// libsortSetBoundaryMode(1)) and the CPU test that checks it against the
// oracle's restatement of sort.cu:367-394.
//
// Reference (sort.cu:14-27 gpu_groups + sort.cu:367-394 GetBoundaries): over a
// zeroed array, b[g(i)] = i wherever g(i) != g(i-1) (i = 0 compares with
// itself, so the first non-empty group keeps 0); then the host walks g =
// ng-1 down to 2 and replaces every 0 by the value above it.  So an empty
// group >= 2 gets the next non-empty group's start (as the exclusive prefix
// does), but an empty group 1 keeps 0, and a FIRST non-empty group g0 >= 2
// (whose start is 0) is overwritten with the next non-empty group's start.
#pragma once

#include <stddef.h>
#include <stdint.h>

namespace lsort {

// prefix[g] = number of elements whose group is < g (what gpuPartial returns
// by default); n = element count.  Rewrites prefix into the reference's
// boundaries in place.
inline void reference_boundaries_from_prefix(uint32_t* b, size_t ngroups, uint64_t n) {
  if (ngroups == 0) return;
  // pass 1 (gpu_groups): non-empty groups keep their start, empty ones 0
  for (size_t g = 0; g < ngroups; ++g) {
    const uint64_t end = g + 1 < ngroups ? b[g + 1] : n;
    if (end == b[g]) b[g] = 0;
  }
  // pass 2 (host fill, sort.cu:384-391): from the top down to group 2
  uint32_t prev = (uint32_t)n;
  for (size_t g = ngroups - 1; g > 1; --g) {
    if (b[g] == 0) b[g] = prev;
    prev = b[g];
  }
}

}  // namespace lsort
