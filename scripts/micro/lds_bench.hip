// Microbenchmark: random-address LDS operations on a k_resolve-sized bitmap
// (4096 words, 16 KB), two 512-thread workgroups per CU; addresses from one
// v_mad per op, so the ALU stays out of the way.
// Prints lane-operations per CU per ns for each form:
//   or_nr   ds_or_b32 (no return)      or_rtn  ds_or_rtn_b32
//   read    ds_read_b32                write   ds_write_b32
//   write8  ds_write_b8 (byte array)   add256  ds_add_rtn_u32 on 256 bins
//   read64  ds_read_b64                or_4    ds_or_b32 with 4 of 64 lanes active
//   seq     ds_read_b32, conflict-free (baseline)
// Usage: ./lds_bench [iters]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int kWords = 4096;

__device__ __forceinline__ uint32_t step(uint32_t x) {
  x ^= x << 13; x ^= x >> 17; x ^= x << 5;
  return x;
}

template <int MODE>
__global__ __launch_bounds__(512) void k_lds(uint32_t iters, uint32_t* out) {
  __shared__ uint32_t a[kWords];
  for (int i = threadIdx.x; i < kWords; i += 512) a[i] = 0;
  __syncthreads();
  // 8 independent LCG streams per lane: one v_mad per address, word index = top 12 bits
  uint32_t x[8], acc = 0;
#pragma unroll
  for (int u = 0; u < 8; ++u) x[u] = 0x9E3779B9u * (blockIdx.x * 4096 + threadIdx.x * 8 + u + 1);
  uint8_t* b = reinterpret_cast<uint8_t*>(a);
  for (uint32_t i = 0; i < iters; i += 8) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      x[u] = x[u] * 1664525u + 1013904223u;
      const uint32_t w = x[u] >> 20, bit = 1u << (x[u] & 31);
      if (MODE == 0) atomicOr(&a[w], bit);
      else if (MODE == 1) acc += atomicOr(&a[w], bit) & bit;
      else if (MODE == 2) acc += a[w];
      else if (MODE == 3) a[w] = x[u];
      else if (MODE == 4) b[x[u] >> 18] = 1;
      else if (MODE == 5) acc += atomicAdd(&a[w & 255], 1u);
      else if (MODE == 6) { const uint2 v = reinterpret_cast<const uint2*>(a)[w >> 1]; acc += v.x ^ v.y; }
      else if (MODE == 7) { if ((threadIdx.x & 15) == 0) atomicOr(&a[w], bit); }
      else if (MODE == 8) acc += a[(threadIdx.x & 63) + (w & ~63u)];  // conflict-free: one word per bank
    }
  }
  __syncthreads();
  if (acc == 0x12345u || a[threadIdx.x] == 0x12345u) out[0] = acc;
}

int main(int argc, char** argv) {
  const uint32_t iters = argc > 1 ? (uint32_t)atoi(argv[1]) : 8192;
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  uint32_t* out;
  (void)hipMalloc(&out, 4);
  const char* names[] = {"or_nr", "or_rtn", "read", "write", "write8", "add256", "read64", "or_4", "seq"};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int grid = 2 * cus;
  for (int mode = 0; mode < 9; ++mode) {
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipEventRecord(e0);
      switch (mode) {
        case 0: hipLaunchKernelGGL(k_lds<0>, dim3(grid), dim3(512), 0, 0, iters, out); break;
        case 1: hipLaunchKernelGGL(k_lds<1>, dim3(grid), dim3(512), 0, 0, iters, out); break;
        case 2: hipLaunchKernelGGL(k_lds<2>, dim3(grid), dim3(512), 0, 0, iters, out); break;
        case 3: hipLaunchKernelGGL(k_lds<3>, dim3(grid), dim3(512), 0, 0, iters, out); break;
        case 4: hipLaunchKernelGGL(k_lds<4>, dim3(grid), dim3(512), 0, 0, iters, out); break;
        case 5: hipLaunchKernelGGL(k_lds<5>, dim3(grid), dim3(512), 0, 0, iters, out); break;
        case 6: hipLaunchKernelGGL(k_lds<6>, dim3(grid), dim3(512), 0, 0, iters, out); break;
        case 7: hipLaunchKernelGGL(k_lds<7>, dim3(grid), dim3(512), 0, 0, iters, out); break;
        case 8: hipLaunchKernelGGL(k_lds<8>, dim3(grid), dim3(512), 0, 0, iters, out); break;
      }
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    const double ops_per_cu = 2.0 * 512 * iters;
    // wave-instructions per CU: ops / 64; cycles at 2.4 GHz
    printf("%-7s %8.3f ms  %6.2f lane-ops/CU/ns  %6.1f cycles per wave-instr (at 2.4 GHz)\n", names[mode], best,
           ops_per_cu / (best * 1e6), best * 1e-3 * 2.4e9 / (ops_per_cu / 64));
  }
  return 0;
}
