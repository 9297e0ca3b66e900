// Micro-benchmark: Philox4x32-10 on gfx950 by product form and by the number
// of independent draws per thread (ILP):
//   V0 mul_hi + mul_lo (the compiler's lowering)
//   V1 v_mad_u64_u32 in inline asm with the carry in vcc (gs_rng.h, round 3)
//   V2 v_mad_u64_u32 in inline asm with the carry in an SGPR pair of its own
//      (no shared vcc: independent draws can interleave)
// Build: hipcc --offload-arch=gfx950 -O3 philox_bench3.hip -o philox_bench3
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

template <int V>
__device__ __forceinline__ void mul64(uint32_t a, uint32_t b, uint32_t& hi, uint32_t& lo) {
  if (V == 0) {
    hi = __umulhi(a, b);
    lo = a * b;
  } else if (V == 1) {
    uint64_t p;
    asm("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(p) : "v"(a), "v"(b) : "vcc");
    hi = (uint32_t)(p >> 32);
    lo = (uint32_t)p;
  } else {
    uint64_t p, c;
    asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(p), "=s"(c) : "v"(a), "v"(b));
    hi = (uint32_t)(p >> 32);
    lo = (uint32_t)p;
  }
}

template <int V>
__device__ __forceinline__ uint4 philox(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t h0, l0, h1, l1;
    mul64<V>(0xD2511F53u, c0, h0, l0);
    mul64<V>(0xCD9E8D57u, c2, h1, l1);
    const uint32_t n0 = h1 ^ c1 ^ k0, n2 = h0 ^ c3 ^ k1;
    c0 = n0; c1 = l1; c2 = n2; c3 = l0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return make_uint4(c0, c1, c2, c3);
}

template <int V, int ILP>
__global__ __launch_bounds__(256) void k_philox(uint32_t iters, uint32_t* out, uint32_t* chk) {
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (uint32_t i = 0; i < iters; i += ILP) {
#pragma unroll
    for (int j = 0; j < ILP; ++j) {
      const uint4 r = philox<V>(tid, i + j, 7, 0x3000000u, 0x5EED, 0);
      acc ^= r.x + r.y + r.z + r.w;
    }
  }
  if (acc == 0x12345678) out[0] = acc;
  if (tid < 1024) chk[tid] = acc;
}

template <int V, int ILP>
double run(uint32_t* out, uint32_t* chk, uint32_t blocks, uint32_t iters) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL((k_philox<V, ILP>), dim3(blocks), dim3(256), 0, 0, iters, out, chk);
  hipDeviceSynchronize();
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(a);
    hipLaunchKernelGGL((k_philox<V, ILP>), dim3(blocks), dim3(256), 0, 0, iters, out, chk);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  return (double)blocks * 256 * iters / best / 1e6;  // G philox/s
}

int main() {
  uint32_t *out, *c[12];
  hipMalloc(&out, 64);
  for (auto& p : c) hipMalloc(&p, 4096);
  const uint32_t iters = 960;
  for (uint32_t blocks : {1024u, 8192u}) {  // 4 and 32 waves... per CU (256 CUs)
    double g[12];
    g[0] = run<0, 1>(out, c[0], blocks, iters);
    g[1] = run<1, 1>(out, c[1], blocks, iters);
    g[2] = run<2, 1>(out, c[2], blocks, iters);
    g[3] = run<0, 2>(out, c[3], blocks, iters);
    g[4] = run<1, 2>(out, c[4], blocks, iters);
    g[5] = run<2, 2>(out, c[5], blocks, iters);
    g[6] = run<0, 4>(out, c[6], blocks, iters);
    g[7] = run<1, 4>(out, c[7], blocks, iters);
    g[8] = run<2, 4>(out, c[8], blocks, iters);
    printf("blocks %u (256 threads): G philox/s\n", blocks);
    for (int ilp = 0; ilp < 3; ++ilp)
      printf("  ILP %d: mulhi/lo %.1f  asm-vcc %.1f  asm-sgpr %.1f\n", 1 << ilp, g[3 * ilp], g[3 * ilp + 1],
             g[3 * ilp + 2]);
  }
  uint32_t h[12][1024];
  for (int v = 0; v < 9; ++v) hipMemcpy(h[v], c[v], 4096, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int v = 1; v < 9; ++v)
    for (int i = 0; i < 1024; ++i) bad += h[v][i] != h[(v / 3) * 3][i];
  printf("variants agree: %s\n", bad ? "NO" : "yes");
  return 0;
}
