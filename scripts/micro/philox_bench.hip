// Micro-benchmark: Philox4x32-10 throughput on gfx950 (the keyed RNG of
// gs_rng.h), and variants, to size the resolve kernel's compute floor.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../../gossip_simulator_amd/csrc/gs_rng.h"

__global__ void k_philox(uint32_t iters, uint32_t* out) {
  uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  for (uint32_t i = 0; i < iters; ++i) {
    gs::u32x4 r = gs::philox(tid, i, 7, 0x3000000u, 0x5EED, 0);
    acc ^= r.x + r.y + r.z + r.w;
  }
  if (acc == 0x12345678) out[0] = acc;
}

int main() {
  uint32_t* out; hipMalloc(&out, 64);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  const uint32_t blocks = 256 * 32, thr = 256, iters = 1000;
  hipLaunchKernelGGL(k_philox, dim3(blocks), dim3(thr), 0, 0, iters, out);
  hipDeviceSynchronize();
  hipEventRecord(a);
  hipLaunchKernelGGL(k_philox, dim3(blocks), dim3(thr), 0, 0, iters, out);
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  double n = (double)blocks * thr * iters;
  printf("philox4x32-10: %.3f ms, %.2f G philox/s\n", ms, n / ms / 1e6);
  return 0;
}
