// Allocation stalls after a large hipFree (round 5: bench.py's C3 leg took
// 5-7 s instead of 1.4 s whenever a phase before it had allocated and freed
// ~94 GiB; scripts/c3_after.py reproduces it with a plain torch allocation).
// This program frees F GiB and then times hipMalloc + first touch of 4-GiB
// buffers, right away or after a pause, to see whether the freed memory comes
// back slowly (e.g. while it is being cleared).
// Usage: alloc_stall <free GiB> <pause s> <allocs>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                 \
    }                                                                          \
  } while (0)

static double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

int main(int argc, char** argv) {
  const double fgib = argc > 1 ? atof(argv[1]) : 94.0;
  const double pause = argc > 2 ? atof(argv[2]) : 0.0;
  const int nalloc = argc > 3 ? atoi(argv[3]) : 12;
  const size_t chunk = 4ull << 30;
  CK(hipSetDevice(0));
  CK(hipFree(nullptr));
  if (fgib > 0) {
    void* big = nullptr;
    auto t = std::chrono::steady_clock::now();
    CK(hipMalloc(&big, (size_t)(fgib * (1ull << 30))));
    CK(hipMemset(big, 1, (size_t)(fgib * (1ull << 30))));
    CK(hipDeviceSynchronize());
    printf("alloc+touch %.1f GiB: %.1f ms\n", fgib, ms_since(t));
    t = std::chrono::steady_clock::now();
    CK(hipFree(big));
    printf("free: %.1f ms\n", ms_since(t));
  }
  if (pause > 0) std::this_thread::sleep_for(std::chrono::duration<double>(pause));
  std::vector<void*> bufs;
  double total = 0;
  for (int i = 0; i < nalloc; ++i) {
    void* p = nullptr;
    auto t = std::chrono::steady_clock::now();
    CK(hipMalloc(&p, chunk));
    const double a = ms_since(t);
    CK(hipMemset(p, 0, chunk));
    CK(hipDeviceSynchronize());
    const double b = ms_since(t);
    total += b;
    printf("alloc %2d (4 GiB): malloc %.1f ms, +touch %.1f ms\n", i, a, b);
    bufs.push_back(p);
  }
  printf("free %.0f GiB, pause %.1f s: %d x 4 GiB in %.1f ms\n", fgib, pause, nalloc, total);
  for (void* p : bufs) CK(hipFree(p));
  return 0;
}
