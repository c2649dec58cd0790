// pcie_probe -- host<->device transfer rates on the box, for the host-pointer
// ABI design (DESIGN.md §8 "host ABI"): pageable hipMemcpy, pinned hipMemcpy,
// both directions at once, and a chunked staging pipeline (CPU memcpy into
// pinned chunks overlapped with the DMA of the previous chunk).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -pthread -o tools/pcie_probe tools/pcie_probe.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void pmemcpy(void* dst, const void* src, size_t bytes, int threads) {
  if (threads <= 1) {
    memcpy(dst, src, bytes);
    return;
  }
  std::vector<std::thread> th;
  size_t per = (bytes / threads + 4095) & ~(size_t)4095;
  for (int t = 0; t < threads; ++t) {
    size_t a = std::min(bytes, per * t), b = std::min(bytes, per * (t + 1));
    if (a < b) th.emplace_back([=] { memcpy((char*)dst + a, (const char*)src + a, b - a); });
  }
  for (auto& x : th) x.join();
}

int main(int argc, char** argv) {
  const int lg = argc > 1 ? atoi(argv[1]) : 28;
  const size_t bytes = (size_t)4 << lg;
  char* d;
  CK(hipMalloc(&d, bytes));
  char* d2;
  CK(hipMalloc(&d2, bytes));
  char* hp = (char*)malloc(bytes);
  memset(hp, 1, bytes);
  char* hp2 = (char*)malloc(bytes);
  memset(hp2, 2, bytes);
  char* pin;
  CK(hipHostMalloc(&pin, bytes, 0));
  memset(pin, 3, bytes);
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  const double gb = bytes / 1e9;
  auto rep = [&](const char* what, double t, double mult = 1.0) {
    printf("%-48s %8.2f ms  %6.1f GB/s\n", what, t * 1e3, gb * mult / t);
  };
  for (int it = 0; it < 3; ++it) {
    double t0 = now();
    CK(hipMemcpy(d, hp, bytes, hipMemcpyHostToDevice));
    double t1 = now();
    CK(hipMemcpy(hp, d, bytes, hipMemcpyDeviceToHost));
    double t2 = now();
    CK(hipMemcpy(d, pin, bytes, hipMemcpyHostToDevice));
    double t3 = now();
    CK(hipMemcpy(pin, d, bytes, hipMemcpyDeviceToHost));
    double t4 = now();
    CK(hipMemcpyAsync(d, pin, bytes, hipMemcpyHostToDevice, s0));
    CK(hipMemcpyAsync(pin + 0, d2, bytes, hipMemcpyDeviceToHost, s1));
    CK(hipStreamSynchronize(s0));
    CK(hipStreamSynchronize(s1));
    double t5 = now();
    if (it == 0) continue;
    rep("pageable H2D", t1 - t0);
    rep("pageable D2H", t2 - t1);
    rep("pinned H2D", t3 - t2);
    rep("pinned D2H", t4 - t3);
    rep("pinned H2D + D2H concurrently (sum of bytes)", t5 - t4, 2.0);
  }
  // chunked staging: 4 pinned chunks, CPU memcpy of chunk i+1 overlapped with the DMA of chunk i
  for (size_t chunk : {(size_t)8 << 20, (size_t)32 << 20, (size_t)128 << 20}) {
    for (int thr : {1, 4, 8}) {
      const int NB = 4;
      hipEvent_t ev[NB];
      for (int i = 0; i < NB; ++i) CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
      double best_h2d = 1e9, best_d2h = 1e9;
      for (int it = 0; it < 3; ++it) {
        double t0 = now();
        size_t nch = (bytes + chunk - 1) / chunk;
        for (size_t c = 0; c < nch; ++c) {
          int b = c % NB;
          if (c >= NB) CK(hipEventSynchronize(ev[b]));
          size_t off = c * chunk, len = std::min(chunk, bytes - off);
          pmemcpy(pin + (size_t)b * chunk, hp + off, len, thr);
          CK(hipMemcpyAsync(d + off, pin + (size_t)b * chunk, len, hipMemcpyHostToDevice, s0));
          CK(hipEventRecord(ev[b], s0));
        }
        CK(hipStreamSynchronize(s0));
        double t1 = now();
        // D2H: DMA chunk c+1 while the CPU copies chunk c out of the pinned buffer
        for (size_t c = 0; c < std::min<size_t>(nch, NB); ++c) {
          size_t off = c * chunk, len = std::min(chunk, bytes - off);
          CK(hipMemcpyAsync(pin + (c % NB) * chunk, d + off, len, hipMemcpyDeviceToHost, s0));
          CK(hipEventRecord(ev[c % NB], s0));
        }
        for (size_t c = 0; c < nch; ++c) {
          int b = c % NB;
          CK(hipEventSynchronize(ev[b]));
          size_t off = c * chunk, len = std::min(chunk, bytes - off);
          pmemcpy(hp2 + off, pin + (size_t)b * chunk, len, thr);
          size_t cn = c + NB;
          if (cn < nch) {
            size_t offn = cn * chunk, lenn = std::min(chunk, bytes - offn);
            CK(hipMemcpyAsync(pin + (size_t)b * chunk, d + offn, lenn, hipMemcpyDeviceToHost, s0));
            CK(hipEventRecord(ev[b], s0));
          }
        }
        double t2 = now();
        if (it > 0) {
          best_h2d = std::min(best_h2d, t1 - t0);
          best_d2h = std::min(best_d2h, t2 - t1);
        }
      }
      if (memcmp(hp, hp2, bytes) != 0) printf("staged round trip MISMATCH\n");
      char name[96];
      snprintf(name, sizeof name, "staged H2D chunk %zu MiB, %d threads", chunk >> 20, thr);
      rep(name, best_h2d);
      snprintf(name, sizeof name, "staged D2H chunk %zu MiB, %d threads", chunk >> 20, thr);
      rep(name, best_d2h);
      for (int i = 0; i < NB; ++i) CK(hipEventDestroy(ev[i]));
    }
  }
  // host memcpy rate (pageable -> pageable) for scale
  for (int thr : {1, 4, 8, 16}) {
    double t0 = now();
    pmemcpy(hp2, hp, bytes, thr);
    double t1 = now();
    char name[64];
    snprintf(name, sizeof name, "host memcpy %d threads", thr);
    rep(name, t1 - t0);
  }
  return 0;
}
