// RCCL-only repro (no libsort): one device, a single-rank communicator
// (ncclCommInitAll), one grouped self send/recv of `count` uint64 elements,
// then the received buffer compared with the sent one on the host.  Used to
// pin whether RCCL itself corrupts large (> 1 GiB) self-sends, which the C
// engine works around by cutting messages into <= 256 MiB chunks
// (gpu-radix-sort_amd/csrc/distrib.cpp move_pieces).
//   hipcc -O2 -std=c++17 -o tools/rccl_selfsend tools/rccl_selfsend.cpp -ldl
//   tools/rccl_selfsend <librccl.so path> <log2 bytes> [chunks]
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__);          \
      return 3;                                                                        \
    }                                                                                  \
  } while (0)

__global__ void fill(uint64_t* p, uint64_t n, uint64_t salt) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = (i + 1) * 0x9E3779B97F4A7C15ull ^ salt;
}

__global__ void check(const uint64_t* a, const uint64_t* b, uint64_t n, unsigned long long* bad,
                      unsigned long long* first) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    if (a[i] != b[i]) {
      atomicAdd(bad, 1ull);
      atomicMin(first, (unsigned long long)i);
    }
}

int main(int argc, char** argv) {
  if (argc < 3) {
    printf("usage: %s <librccl.so> <log2 bytes> [chunks]\n", argv[0]);
    return 2;
  }
  void* h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    printf("dlopen %s: %s\n", argv[1], dlerror());
    return 2;
  }
  auto initAll = (decltype(&ncclCommInitAll))dlsym(h, "ncclCommInitAll");
  auto send = (decltype(&ncclSend))dlsym(h, "ncclSend");
  auto recv = (decltype(&ncclRecv))dlsym(h, "ncclRecv");
  auto gs = (decltype(&ncclGroupStart))dlsym(h, "ncclGroupStart");
  auto ge = (decltype(&ncclGroupEnd))dlsym(h, "ncclGroupEnd");
  auto ver = (decltype(&ncclGetVersion))dlsym(h, "ncclGetVersion");
  auto destroy = (decltype(&ncclCommDestroy))dlsym(h, "ncclCommDestroy");
  if (!initAll || !send || !recv || !gs || !ge || !ver || !destroy) {
    printf("missing RCCL symbols\n");
    return 2;
  }
  int v = 0;
  ver(&v);
  const uint64_t bytes = 1ull << atoi(argv[2]);
  const int chunks = argc > 3 ? atoi(argv[3]) : 1;
  const uint64_t n = bytes / 8;
  CK(hipSetDevice(0));
  uint64_t *src, *dst;
  unsigned long long* stat;
  CK(hipMalloc(&src, bytes));
  CK(hipMalloc(&dst, bytes));
  CK(hipMalloc(&stat, 16));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  ncclComm_t comm;
  int dev = 0;
  if (initAll(&comm, 1, &dev) != ncclSuccess) {
    printf("ncclCommInitAll failed\n");
    return 3;
  }
  int fails = 0;
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, st, src, n, (uint64_t)rep);
    CK(hipMemsetAsync(dst, 0xAB, bytes, st));
    const uint64_t per = (n + chunks - 1) / chunks;
    if (gs() != ncclSuccess) return 3;
    for (uint64_t o = 0; o < n; o += per) {
      const uint64_t m = per < n - o ? per : n - o;
      if (send(src + o, m, ncclUint64, 0, comm, st) != ncclSuccess || recv(dst + o, m, ncclUint64, 0, comm, st) != ncclSuccess) {
        printf("send/recv failed\n");
        return 3;
      }
    }
    if (ge() != ncclSuccess) return 3;
    unsigned long long init[2] = {0ull, ~0ull};
    CK(hipMemcpyAsync(stat, init, 16, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(check, dim3(4096), dim3(256), 0, st, src, dst, n, stat, stat + 1);
    unsigned long long res[2];
    CK(hipMemcpyAsync(res, stat, 16, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    printf("RCCL %d  %s  self send/recv of %llu MiB as %d message(s): %llu of %llu elements differ%s",
           v, argv[1], (unsigned long long)(bytes >> 20), chunks, res[0], (unsigned long long)n,
           res[0] ? "" : "\n");
    if (res[0]) {
      printf(", first at element %llu (byte %llu = %.3f GiB)\n", res[1], res[1] * 8, res[1] * 8.0 / (1 << 30));
      ++fails;
    }
  }
  destroy(comm);
  return fails ? 1 : 0;
}
