// Micro-benchmark: Philox4x32-10 on gfx950, mul_hi/mul_lo pairs (the
// compiler's default lowering) vs one v_mad_u64_u32 per product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__device__ __forceinline__ void mad64(uint32_t a, uint32_t b, uint32_t& hi, uint32_t& lo) {
  uint64_t p;
  asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(p) : "v"(a), "v"(b) : "vcc");
  hi = (uint32_t)(p >> 32);
  lo = (uint32_t)p;
}

template <int V>
__device__ __forceinline__ uint4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t h0, l0, h1, l1;
    if (V == 0) {
      h0 = __umulhi(0xD2511F53u, c0); l0 = 0xD2511F53u * c0;
      h1 = __umulhi(0xCD9E8D57u, c2); l1 = 0xCD9E8D57u * c2;
    } else {
      mad64(0xD2511F53u, c0, h0, l0);
      mad64(0xCD9E8D57u, c2, h1, l1);
    }
    const uint32_t n0 = h1 ^ c1 ^ k0, n2 = h0 ^ c3 ^ k1;
    c0 = n0; c1 = l1; c2 = n2; c3 = l0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return make_uint4(c0, c1, c2, c3);
}

template <int V>
__global__ void k_philox(uint32_t iters, uint32_t* out, uint32_t* chk) {
  uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (uint32_t i = 0; i < iters; ++i) {
    uint4 r = philox<V>(tid, i, 7, 0x3000000u, 0x5EED, 0);
    acc ^= r.x + r.y + r.z + r.w;
  }
  if (acc == 0x12345678) out[0] = acc;
  if (tid < 1024) chk[tid] = acc;
}

int main() {
  uint32_t *out, *c0, *c1; hipMalloc(&out, 64); hipMalloc(&c0, 4096); hipMalloc(&c1, 4096);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const uint32_t blocks = 256 * 32, thr = 256, iters = 1000;
  float ms[2];
  for (int v = 0; v < 2; ++v) {
    auto go = [&] {
      if (v == 0) hipLaunchKernelGGL(k_philox<0>, dim3(blocks), dim3(thr), 0, 0, iters, out, c0);
      else hipLaunchKernelGGL(k_philox<1>, dim3(blocks), dim3(thr), 0, 0, iters, out, c1);
    };
    go(); hipDeviceSynchronize();
    hipEventRecord(a); go(); hipEventRecord(b); hipEventSynchronize(b);
    hipEventElapsedTime(&ms[v], a, b);
    printf("philox4x32-10 variant %d: %.3f ms, %.2f G philox/s\n", v, ms[v], (double)blocks * thr * iters / ms[v] / 1e6);
  }
  uint32_t h0[1024], h1[1024];
  hipMemcpy(h0, c0, 4096, hipMemcpyDeviceToHost); hipMemcpy(h1, c1, 4096, hipMemcpyDeviceToHost);
  int bad = 0; for (int i = 0; i < 1024; ++i) bad += h0[i] != h1[i];
  printf("variants agree: %s\n", bad ? "NO" : "yes");
  return 0;
}
