// Does an uncached (or fine-grained) allocation cut the line traffic of a
// random 24-B row gather?  k_expand reads one friends row per firing node from
// the packed view (five 24-B rows per 128-B line, rows at 16-B aligned bases,
// one uint4 + one uint2 load); on coarse-grained memory every such read is a
// 128-B L2 fill from HBM (profiles/r03_fetch_calibration.json), ≈ 0.8 lines
// per row at N = 1e9.  If the L2 forwards sub-line requests for uncached
// memory, the same gather moves 32-64 B per row.
// Usage: uncached_gather <GiB> <mode: coarse|uncached|fine> [rows per thread]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

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

// row r of the packed view: line r / 5, offset 24 * (r % 5) rounded to 16 B
// (k_expand's layout: rows 0..4 at bytes 0, 24 -> 16+8, ...); here simply the
// 16-B aligned base 32 * (r % 4) inside a 128-B line of 4 rows -- one uint4 +
// one uint2 per row, as k_expand issues them
// LOADS: 1 = one uint4 (16 B), 2 = uint4 + uint2 (24 B, k_expand's), 3 = two uint4 (32 B)
template <int LOADS>
__global__ void k_gather(const uint4* __restrict__ tab, uint64_t nlines, uint32_t R, uint32_t* out) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  uint4 a[8], c[8];
  uint2 b[8];
  for (uint32_t r0 = 0; r0 < R; r0 += 8) {
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) {
      const uint32_t h = hash32((uint32_t)tid * 2654435761u + (r0 + k) * 97u);
      const uint64_t line = ((uint64_t)h * nlines) >> 32, slot = h & 3;
      const uint4* p = tab + line * 8 + slot * 2;
      a[k] = p[0];
      if (LOADS == 2) b[k] = *(const uint2*)(p + 1);
      if (LOADS == 3) c[k] = p[1];
    }
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) {
      acc += a[k].x ^ a[k].w;
      if (LOADS == 2) acc ^= b[k].y;
      if (LOADS == 3) acc ^= c[k].z;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// Lane pairs: lanes 2q and 2q+1 fetch the 32-B span of node 2q's row, then of
// node 2q+1's (each lane one uint4 per step, both halves of one line in one
// instruction: one L2 request per row), and swap halves with a DPP move so
// that each lane ends with its own node's row.
__device__ __forceinline__ uint32_t swap_pair(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
}
__global__ void k_gather_pair(const uint4* __restrict__ tab, uint64_t nlines, uint32_t R, uint32_t* out) {
  const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t odd = threadIdx.x & 1;
  uint32_t acc = 0;
  uint4 s0[8], s1[8];
  for (uint32_t r0 = 0; r0 < R; r0 += 8) {
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) {
      const uint32_t h = hash32((uint32_t)tid * 2654435761u + (r0 + k) * 97u);
      const uint64_t line = ((uint64_t)h * nlines) >> 32, slot = h & 3;
      const uint64_t mine = line * 8 + slot * 2;  // my row's first uint4
      const uint64_t other = ((uint64_t)swap_pair((uint32_t)(mine >> 32)) << 32) | swap_pair((uint32_t)mine);
      const uint64_t even_row = odd ? other : mine, odd_row = odd ? mine : other;
      s0[k] = tab[even_row + odd];  // step 0: the pair's even node, half `odd`
      s1[k] = tab[odd_row + odd];   // step 1: the pair's odd node
    }
#pragma unroll
    for (uint32_t k = 0; k < 8; ++k) {
      // even lane keeps s0 (its row's half 0) and needs the partner's s0 (half 1);
      // odd lane keeps s1 (its row's half 1) and needs the partner's s1 (half 0)
      const uint4 send = odd ? s0[k] : s1[k];
      uint4 got;
      got.x = swap_pair(send.x); got.y = swap_pair(send.y); got.z = swap_pair(send.z); got.w = swap_pair(send.w);
      const uint4 h0 = odd ? got : s0[k], h1 = odd ? s1[k] : got;
      acc += h0.x ^ h0.w ^ h1.y;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_fill(uint4* p, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = make_uint4((uint32_t)i, (uint32_t)(i >> 32), 7u, 9u);
}

int main(int argc, char** argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 25.6;
  const char* mode = argc > 2 ? argv[2] : "coarse";
  const uint32_t R = argc > 3 ? (uint32_t)atoi(argv[3]) : 64;
  const uint64_t bytes = (uint64_t)(gib * (1ull << 30)) & ~127ull, nlines = bytes / 128;
  uint4* tab = nullptr;
  if (!strcmp(mode, "coarse")) CK(hipMalloc(&tab, bytes));
  else if (!strcmp(mode, "uncached")) CK(hipExtMallocWithFlags((void**)&tab, bytes, hipDeviceMallocUncached));
  else CK(hipExtMallocWithFlags((void**)&tab, bytes, hipDeviceMallocFinegrained));
  uint32_t* out = nullptr;
  CK(hipMalloc(&out, 4));
  hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, tab, bytes / 16);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  const uint32_t threads = 256, blocks = 256 * 64;  // 4M threads
  const uint64_t rows = (uint64_t)threads * blocks * R;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int loads = 1; loads <= 4; ++loads)
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(e0));
      if (loads == 1) hipLaunchKernelGGL(k_gather<1>, dim3(blocks), dim3(threads), 0, 0, tab, nlines, R, out);
      if (loads == 2) hipLaunchKernelGGL(k_gather<2>, dim3(blocks), dim3(threads), 0, 0, tab, nlines, R, out);
      if (loads == 3) hipLaunchKernelGGL(k_gather<3>, dim3(blocks), dim3(threads), 0, 0, tab, nlines, R, out);
      if (loads == 4) hipLaunchKernelGGL(k_gather_pair, dim3(blocks), dim3(threads), 0, 0, tab, nlines, R, out);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("%s %.1f GiB, %s per row: %llu random rows in %.2f ms = %.3g rows/s (%.0f GB/s of 128-B lines)\n",
             mode, gib, loads == 1 ? "uint4" : loads == 2 ? "uint4+uint2" : loads == 3 ? "2 x uint4" : "lane pair 2 x uint4", (unsigned long long)rows, ms,
             rows / (ms * 1e-3), rows * 128.0 / (ms * 1e-3) / 1e9);
    }
  CK(hipFree(tab));
  return 0;
}
