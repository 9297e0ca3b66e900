// Microbenchmark: random 64-bit atomicOr vs random 64-bit loads into a
// 125-MB bitset (the push-pull round's two kinds of random access), plus a
// random load + ballot-free store.  Usage: ./mb_random [nwords] [nops]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ uint32_t mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
  return (uint32_t)x;
}

__global__ void k_atomic(unsigned long long* b, uint64_t W, uint64_t ops, uint32_t salt) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ops; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t h = mix(i * 0x9E3779B97F4A7C15ull + salt);
    atomicOr(&b[h % W], 1ull << (h & 63));
  }
}
__global__ void k_load(const unsigned long long* b, uint64_t W, uint64_t ops, uint32_t salt, unsigned long long* out) {
  unsigned long long acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ops; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t h = mix(i * 0x9E3779B97F4A7C15ull + salt);
    acc += b[h % W];
  }
  if (acc == 0x1234567) out[0] = acc;
}
__global__ void k_load8(const unsigned long long* b, uint64_t W, uint64_t ops, uint32_t salt, unsigned long long* out) {
  // 8 independent loads per lane per iteration (more in flight)
  unsigned long long acc = 0;
  const uint64_t G = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ops / 8; i += G) {
    unsigned long long v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = b[mix((i * 8 + k) * 0x9E3779B97F4A7C15ull + salt) % W];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += v[k];
  }
  if (acc == 0x1234567) out[0] = acc;
}
// random byte stores into a byte-per-node array (N = 64 * W bytes): the
// alternative to atomicOr for idempotent "set node u" updates
__global__ void k_store_byte(unsigned char* a, uint64_t N, uint64_t ops, uint32_t salt) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < ops; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t h = mix(i * 0x9E3779B97F4A7C15ull + salt);
    a[((uint64_t)h * N) >> 32] = 1;
  }
}
__global__ void k_stream(const uint4* a, uint64_t n16, unsigned long long* out) {
  unsigned long long acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = a[i];
    acc += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x1234567) out[0] = acc;
}

int main(int argc, char** argv) {
  const uint64_t W = argc > 1 ? strtoull(argv[1], 0, 0) : 15625000ull;  // 1e9 bits
  const uint64_t ops = argc > 2 ? strtoull(argv[2], 0, 0) : 500000000ull;
  unsigned long long *b, *out;
  uint4* big;
  const uint64_t bigb = 8ull << 30;
  if (hipMalloc(&b, W * 8) || hipMalloc(&out, 8) || hipMalloc(&big, bigb)) return 1;
  (void)hipMemset(b, 0, W * 8);
  (void)hipMemset(big, 1, bigb);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  unsigned char* bytes = nullptr;
  if (hipMalloc(&bytes, W * 64)) return 1;
  (void)hipMemset(bytes, 0, W * 64);
  for (int rep = 0; rep < 2; ++rep) {
    float ms;
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k_store_byte, dim3(8192), dim3(256), 0, 0, bytes, W * 64, ops, rep);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("byte store %.3e ops in %7.2f ms = %.3e/s (1 B per node, %.2f GB array)\n", (double)ops, ms,
           ops / (ms * 1e-3), W * 64 / 1e9);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k_atomic, dim3(8192), dim3(256), 0, 0, b, W, ops, rep);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("atomicOr  %.3e ops in %7.2f ms = %.3e/s\n", (double)ops, ms, ops / (ms * 1e-3));
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k_load, dim3(8192), dim3(256), 0, 0, b, W, ops, rep, out);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("load      %.3e ops in %7.2f ms = %.3e/s\n", (double)ops, ms, ops / (ms * 1e-3));
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k_load8, dim3(4096), dim3(256), 0, 0, b, W, ops, rep, out);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("load x8   %.3e ops in %7.2f ms = %.3e/s\n", (double)ops, ms, ops / (ms * 1e-3));
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k_stream, dim3(8192), dim3(256), 0, 0, big, bigb / 16, out);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("stream    %.2f GB in %7.2f ms = %.2f TB/s\n", bigb / 1e9, ms, bigb / (ms * 1e-3) / 1e12);
  }
  return hipDeviceSynchronize() != hipSuccess;
}
