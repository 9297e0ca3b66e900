// Would chunked expand -> part2 staging read the coarse messages back from the
// 256-MB MALL (verdict r04, item 1(b))?  A chunk of S MB is written
// (k_expand's coarse-message writes), then G GB of random 128-B line reads
// stream through the memory system (k_expand's friends-row gathers for that
// chunk: ~3 GB of lines per 64 MB of messages at C5), then the chunk is read
// back (k_part2).  The read-back is timed against a cold read of a chunk the
// size of the MALL's many times over.
// Usage: mall_staging <chunk MB> <gather GB between>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(2);                                                                 \
    }                                                                          \
  } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

__global__ void k_write(uint4* p, uint64_t n, uint32_t salt) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = make_uint4((uint32_t)i ^ salt, salt, 1u, 2u);
}
__global__ void k_read(const uint4* p, uint64_t n, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = p[i];
    acc += v.x ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}
// random 16-B reads, one per 128-B line, `lines` of them
__global__ void k_gather(const uint4* tab, uint64_t nlines, uint64_t lines, uint32_t salt, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < lines; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t l = ((uint64_t)hash32((uint32_t)i * 2654435761u ^ salt) * nlines) >> 32;
    acc += tab[l * 8].x;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char** argv) {
  const double mb = argc > 1 ? atof(argv[1]) : 64;
  const double ggb = argc > 2 ? atof(argv[2]) : 3;
  const uint64_t n = (uint64_t)(mb * (1 << 20)) / 16, tab_bytes = 24ull << 30, nlines = tab_bytes / 128;
  const uint64_t glines = (uint64_t)(ggb * 1e9) / 128;
  uint4 *chunk = nullptr, *tab = nullptr, *cold = nullptr;
  uint32_t* out = nullptr;
  const uint64_t ncold = 8ull << 30 >> 4;  // 8 GiB of other chunks
  CK(hipMalloc(&chunk, n * 16));
  CK(hipMalloc(&tab, tab_bytes));
  CK(hipMalloc(&cold, ncold * 16));
  CK(hipMalloc(&out, 4));
  hipLaunchKernelGGL(k_write, dim3(8192), dim3(256), 0, 0, tab, tab_bytes / 16, 7u);
  hipLaunchKernelGGL(k_write, dim3(8192), dim3(256), 0, 0, cold, ncold, 9u);
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  auto timed = [&](auto&& f) {
    CK(hipEventRecord(a));
    f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms;
  };
  for (int rep = 0; rep < 3; ++rep) {
    // cold: the chunk written, then 8 GiB of other writes evict it
    hipLaunchKernelGGL(k_write, dim3(4096), dim3(256), 0, 0, chunk, n, rep);
    hipLaunchKernelGGL(k_write, dim3(8192), dim3(256), 0, 0, cold, ncold, rep + 100);
    const float tcold = timed([&] { hipLaunchKernelGGL(k_read, dim3(4096), dim3(256), 0, 0, chunk, n, out); });
    // warm: written, read back at once
    hipLaunchKernelGGL(k_write, dim3(4096), dim3(256), 0, 0, chunk, n, rep + 200);
    const float twarm = timed([&] { hipLaunchKernelGGL(k_read, dim3(4096), dim3(256), 0, 0, chunk, n, out); });
    // staged: written, G GB of random line reads, then read back
    hipLaunchKernelGGL(k_write, dim3(4096), dim3(256), 0, 0, chunk, n, rep + 300);
    const float tg = timed([&] { hipLaunchKernelGGL(k_gather, dim3(8192), dim3(256), 0, 0, tab, nlines, glines, rep, out); });
    const float tstaged = timed([&] { hipLaunchKernelGGL(k_read, dim3(4096), dim3(256), 0, 0, chunk, n, out); });
    printf("chunk %.0f MB: read back cold %.3f ms (%.0f GB/s), at once %.3f ms (%.0f GB/s), after %.1f GB of "
           "random lines (%.2f ms) %.3f ms (%.0f GB/s)\n",
           mb, tcold, n * 16 / (tcold * 1e6), twarm, n * 16 / (twarm * 1e6), ggb, tg, tstaged,
           n * 16 / (tstaged * 1e6));
  }
  return 0;
}
