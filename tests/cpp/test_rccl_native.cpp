// test_rccl_native.cpp -- the C engine's RCCL path in a torch-free process
// (the RCCL C and Go callers load: /opt/rocm's librccl.so.1 on the image's
// HIP runtime): libsortDistribSortU32 over a one-device communicator with
// every piece sent through RCCL (LIBSORT_DISTRIB_SELF_RCCL), on configs[1]'s
// 2^28 keys of the reference stream (populateInput, utils.cu:65-80), and on
// 2^27 + 12345 keys.  Checked: each output sorted, and the same multiset as
// the input (sum, xor and sum of squares mod 2^64).  Plain device buffers
// from the HIP runtime, as a C caller would allocate them.  Exit 0 = pass.
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <vector>

#include "libsort.h"

struct Print {
  uint64_t sum = 0, x = 0, sq = 0;
  void add(uint32_t k) {
    sum += k;
    x ^= (uint64_t)k * 0x9E3779B97F4A7C15ull;
    sq += (uint64_t)k * k;
  }
  bool operator==(const Print& o) const { return sum == o.sum && x == o.x && sq == o.sq; }
};

static int run(size_t n) {
  std::vector<uint32_t> h(n);
  populateInput(h.data(), n);
  Print a;
  for (uint32_t k : h) a.add(k);
  uint32_t *d_in = nullptr, *d_out = nullptr;
  if (hipSetDevice(0) != hipSuccess || hipMalloc(&d_in, n * 4) != hipSuccess || hipMalloc(&d_out, n * 4) != hipSuccess ||
      hipMemcpy(d_in, h.data(), n * 4, hipMemcpyHostToDevice) != hipSuccess) {
    fprintf(stderr, "HIP setup failed\n");
    return 1;
  }
  const int dev = 0;
  const uint32_t* ins[1] = {d_in};
  uint32_t* outs[1] = {d_out};
  size_t n_in[1] = {n}, n_out[1] = {0};
  if (!libsortDistribSortU32(1, &dev, ins, n_in, outs, n_out, LIBSORT_DISTRIB_SELF_RCCL)) {
    fprintf(stderr, "libsortDistribSortU32: %s\n", libsortLastError());
    return 1;
  }
  if (n_out[0] != n || hipMemcpy(h.data(), d_out, n * 4, hipMemcpyDeviceToHost) != hipSuccess) {
    fprintf(stderr, "output size %zu / copy failed\n", n_out[0]);
    return 1;
  }
  Print b;
  size_t unsorted = 0;
  for (size_t i = 0; i < n; ++i) {
    b.add(h[i]);
    if (i && h[i - 1] > h[i]) ++unsorted;
  }
  (void)hipFree(d_in);
  (void)hipFree(d_out);
  printf("n=%zu through RCCL: %s, %zu descents\n", n, a == b ? "same multiset" : "MULTISET DIFFERS", unsorted);
  return (a == b && unsorted == 0) ? 0 : 1;
}

int main() {
  if (!initLibSort()) {
    fprintf(stderr, "initLibSort failed: %s\n", libsortLastError());
    return 2;
  }
  if (run((1u << 27) + 12345) || run(1u << 28)) return 1;
  printf("OK\n");
  return 0;
}
