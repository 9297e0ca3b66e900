// Micro-benchmark: random small-granule gathers/scatters from HBM on gfx950.
// Used to size the window engine: what a random 24-B friends
// row, a random 4-B word and a random 1-B degree cost chip-wide.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}

// each thread: R random rows of S u32 (row index hashed), sum to avoid DCE
template <int S>
__global__ void k_rows(const uint32_t* __restrict__ tab, uint64_t nrows, uint64_t nthreads, int R, uint32_t* out) {
  uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= nthreads) return;
  uint32_t acc = 0;
  for (int r = 0; r < R; ++r) {
    uint64_t row = ((uint64_t)hash32((uint32_t)tid * 2654435761u + r * 97u) * nrows) >> 32;
    const uint32_t* p = tab + row * S;
#pragma unroll
    for (int j = 0; j < S; ++j) acc += p[j];
  }
  if (acc == 0x12345678) out[0] = acc;
}

// sorted-sparse: thread i reads row (i * gap + jitter)
template <int S>
__global__ void k_rows_sorted(const uint32_t* __restrict__ tab, uint64_t nrows, uint64_t nthreads, uint32_t gap, uint32_t* out) {
  uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= nthreads) return;
  uint64_t row = tid * gap + (hash32((uint32_t)tid) % gap);
  if (row >= nrows) return;
  const uint32_t* p = tab + row * S;
  uint32_t acc = 0;
#pragma unroll
  for (int j = 0; j < S; ++j) acc += p[j];
  if (acc == 0x12345678) out[0] = acc;
}

__global__ void k_bytes(const uint8_t* __restrict__ tab, uint64_t n, uint64_t nthreads, int R, uint32_t* out) {
  uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= nthreads) return;
  uint32_t acc = 0;
  for (int r = 0; r < R; ++r) {
    uint64_t i = ((uint64_t)hash32((uint32_t)tid * 2654435761u + r * 97u) * n) >> 32;
    acc += tab[i];
  }
  if (acc == 0x12345678) out[0] = acc;
}

__global__ void k_scatter(uint32_t* tab, uint64_t n, uint64_t nthreads, int R) {
  uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= nthreads) return;
  for (int r = 0; r < R; ++r) {
    uint64_t i = ((uint64_t)hash32((uint32_t)tid * 2654435761u + r * 97u) * n) >> 32;
    tab[i] = (uint32_t)tid;
  }
}

__global__ void k_atomor(uint32_t* tab, uint64_t n, uint64_t nthreads, int R) {
  uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= nthreads) return;
  for (int r = 0; r < R; ++r) {
    uint64_t i = ((uint64_t)hash32((uint32_t)tid * 2654435761u + r * 97u) * n) >> 32;
    atomicOr(&tab[i], 1u << (tid & 31));
  }
}

__global__ void k_stream(const uint4* __restrict__ a, uint64_t n, uint32_t* out) {
  uint4 acc = {0, 0, 0, 0};
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint4 v = a[i]; acc.x += v.x; acc.y ^= v.y; acc.z += v.z; acc.w ^= v.w;
  }
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678) out[0] = 1;
}

int main() {
  const uint64_t nrows = 1000000000ull;
  uint32_t* tab; uint32_t* out;
  const size_t bytes = nrows * 8 * 4;  // room for stride 8
  CK(hipMalloc(&tab, bytes));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(tab, 1, bytes));
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  auto timeit = [&](const char* name, auto launch, double items, double bytes_alg) {
    launch(); hipDeviceSynchronize();
    hipEventRecord(e0); for (int i = 0; i < 3; ++i) launch(); hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 3;
    printf("%-40s %8.3f ms  %7.2f G items/s  %7.1f GB/s alg\n", name, ms, items / ms / 1e6, bytes_alg / ms / 1e6);
  };
  const uint64_t T = 64ull << 20; const int R = 4;  // 256M accesses
  const uint32_t blk = 256; const uint32_t grid = (uint32_t)((T + blk - 1) / blk);
  timeit("stream 16B/lane 16 GB", [&] { hipLaunchKernelGGL(k_stream, dim3(8192), dim3(256), 0, 0, (const uint4*)tab, (uint64_t)(16ull << 30) / 16, out); }, 1e9, 16.0 * (1ull << 30));
  timeit("random row S=1 (4B) 4GB", [&] { hipLaunchKernelGGL(k_rows<1>, dim3(grid), dim3(blk), 0, 0, tab, nrows, T, R, out); }, T * R, T * R * 4.0);
  timeit("random row S=6 (24B) 24GB", [&] { hipLaunchKernelGGL(k_rows<6>, dim3(grid), dim3(blk), 0, 0, tab, nrows, T, R, out); }, T * R, T * R * 24.0);
  timeit("random row S=8 (32B) 32GB", [&] { hipLaunchKernelGGL(k_rows<8>, dim3(grid), dim3(blk), 0, 0, tab, nrows, T, R, out); }, T * R, T * R * 32.0);
  timeit("random row S=6 in 240MB (MALL)", [&] { hipLaunchKernelGGL(k_rows<6>, dim3(grid), dim3(blk), 0, 0, tab, 10000000ull, T, R, out); }, T * R, T * R * 24.0);
  timeit("random byte 1GB", [&] { hipLaunchKernelGGL(k_bytes, dim3(grid), dim3(blk), 0, 0, (const uint8_t*)tab, nrows, T, R, out); }, T * R, T * R * 1.0);
  timeit("random byte 125MB (MALL)", [&] { hipLaunchKernelGGL(k_bytes, dim3(grid), dim3(blk), 0, 0, (const uint8_t*)tab, 125000000ull, T, R, out); }, T * R, T * R * 1.0);
  for (uint32_t gap : {1u, 2u, 4u, 8u, 16u, 64u}) {
    char nm[64]; snprintf(nm, 64, "sorted rows S=6 gap %u", gap);
    const uint64_t Tn = nrows / gap; const uint32_t g2 = (uint32_t)((Tn + blk - 1) / blk);
    timeit(nm, [&] { hipLaunchKernelGGL(k_rows_sorted<6>, dim3(g2), dim3(blk), 0, 0, tab, nrows, Tn, gap, out); }, Tn, Tn * 24.0);
  }
  timeit("random 4B store 4GB", [&] { hipLaunchKernelGGL(k_scatter, dim3(grid), dim3(blk), 0, 0, tab, nrows, T, R); }, T * R, T * R * 4.0);
  timeit("random 4B atomicOr 125MB", [&] { hipLaunchKernelGGL(k_atomor, dim3(grid), dim3(blk), 0, 0, tab, 31250000ull, T, R); }, T * R, T * R * 4.0);
  timeit("random 4B atomicOr 4GB", [&] { hipLaunchKernelGGL(k_atomor, dim3(grid), dim3(blk), 0, 0, tab, nrows, T, R); }, T * R, T * R * 4.0);
  return 0;
}
