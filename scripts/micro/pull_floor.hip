// Micro-benchmark: the floor of a receiver-driven ("pull") flood window at
// N = 1e9 (docs/DESIGN_NOTEBOOK.md 4.4.2).  A pull window makes every live receiver scan
// its in-edges (v, j) from the reverse table (rsrc u32 + rslot u8, as the
// push-pull engine's) and ask whether the in-neighbour v fires in the window
// and at which tick; only then can the sender-keyed drop digit be recomputed
// (Philox{v, t, j/4}).  This program times the scan alone, with nothing
// resolved and one u64 written per 64 receivers, so every real pull kernel
// is slower than what it reports:
//   mode 0  stream rsrc + rslot only (the table read, no lookups)
//   mode 1  + one random lookup per in-edge into the window's fire bitset
//           (N bits = 125 MB: fits the 256 MB Infinity Cache)
//   mode 2  mode 1 + for a firing v its fire tick (u8[N], random) and the
//           drop draw; kept receipts counted per tick in registers
//   mode 3  one random lookup per in-edge into the u8 fire-tick array instead
//           of the bitset, then as mode 2
// Synthetic table: in-degree 5 or 6 (rend(u) = floor(5.5 u), the C5 overlay's
// mean), sources uniform.  Fires: each node fires in the window with
// probability p at a uniform tick 0..9.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "../../gossip_simulator_amd/csrc/gs_rng.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

using gs::philox;
using gs::u32x4;

__host__ __device__ inline uint64_t rend(uint64_t u) { return (u * 11) >> 1; }

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}

__global__ void k_init_edges(uint32_t* rsrc, uint8_t* rslot, uint64_t E, uint32_t N) {
  for (uint64_t e = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; e < E; e += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t h = hash32((uint32_t)e ^ hash32((uint32_t)(e >> 32) + 0x9E3779B9u));
    rsrc[e] = (uint32_t)(((uint64_t)h * N) >> 32);
    rslot[e] = (uint8_t)((e % 6) | (5u << 4));
  }
}

// one thread per 64-node word: the word's fire bits and the nodes' fire ticks
__global__ void k_init_fire(uint8_t* ftick, unsigned long long* fbits, uint32_t N, uint32_t thr) {
  const uint64_t W = ((uint64_t)N + 63) / 64;
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < W; w += (uint64_t)gridDim.x * blockDim.x) {
    unsigned long long b = 0;
    for (uint32_t i = 0; i < 64; ++i) {
      const uint64_t v = w * 64 + i;
      if (v >= N) break;
      const uint32_t h = hash32((uint32_t)v * 2654435761u + 12345u);
      const bool f = h < thr;
      ftick[v] = f ? (uint8_t)(hash32(h) % 10u) : (uint8_t)0xFF;
      if (f) b |= 1ull << i;
    }
    fbits[w] = b;
  }
}

template <int MODE>
__global__ __launch_bounds__(256) void k_pull(const uint32_t* __restrict__ rsrc, const uint8_t* __restrict__ rslot,
                                              const unsigned long long* __restrict__ fbits,
                                              const uint8_t* __restrict__ ftick, uint32_t N, uint32_t t0,
                                              unsigned long long* __restrict__ out) {
  const uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool in = u < N;
  const uint64_t e0 = rend(u), e1 = in ? rend(u + 1) : e0;
  uint32_t v[6], x[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    const bool ok = e0 + k < e1;
    v[k] = ok ? rsrc[e0 + k] : 0u;
    x[k] = ok ? rslot[e0 + k] : 0u;
  }
  uint32_t acc = 0;
  if (MODE == 0) {
#pragma unroll
    for (int k = 0; k < 6; ++k) acc += (e0 + k < e1) ? (v[k] ^ x[k]) & 1u : 0u;
  } else {
    uint32_t tk[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      tk[k] = 0xFF;
      if (e0 + k < e1) {
        if (MODE == 3) tk[k] = ftick[v[k]];
        else if ((fbits[v[k] >> 6] >> (v[k] & 63)) & 1ull) tk[k] = MODE == 1 ? 0u : ftick[v[k]];
      }
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) {
      if (tk[k] == 0xFF) continue;
      if (MODE == 1) { acc += 1; continue; }
      const uint32_t j = x[k] & 15u;
      const u32x4 r = philox(v[k], t0 + tk[k], j >> 2, (3u << 24), 0x1234u, 0x5678u);
      uint32_t drop, crash;
      gs::drop_crash(gs::lane_of(r, j & 3), drop, crash);
      if (drop >= 10) acc += 1u << (3 * tk[k]);  // kept: a receipt at tick tk
    }
  }
  const unsigned long long b = __ballot(acc != 0);
  if ((threadIdx.x & 63) == 0 && in) out[u >> 6] = b;
}

int main(int argc, char** argv) {
  const uint32_t N = argc > 1 ? (uint32_t)atoll(argv[1]) : 1000000000u;
  const uint64_t E = rend(N), W = ((uint64_t)N + 63) / 64;
  uint32_t* rsrc; uint8_t* rslot; uint8_t* ftick; unsigned long long* fbits; unsigned long long* out;
  CK(hipMalloc(&rsrc, E * 4)); CK(hipMalloc(&rslot, E)); CK(hipMalloc(&ftick, N));
  CK(hipMalloc(&fbits, W * 8)); CK(hipMalloc(&out, W * 8));
  hipLaunchKernelGGL(k_init_edges, dim3(65536), dim3(256), 0, 0, rsrc, rslot, E, N);
  CK(hipDeviceSynchronize());
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  const double ps[] = {0.02, 0.10, 0.30};
  printf("N=%u E=%llu (in-edges, %.1f GB of rsrc+rslot)\n", N, (unsigned long long)E, E * 5.0 / 1e9);
  for (double p : ps) {
    hipLaunchKernelGGL(k_init_fire, dim3(16384), dim3(256), 0, 0, ftick, fbits, N, (uint32_t)(p * 4294967296.0));
    CK(hipDeviceSynchronize());
    for (int mode = 0; mode < 4; ++mode) {
      float best = 1e30f;
      for (int rep = 0; rep < 3; ++rep) {
        const dim3 g((N + 255) / 256);
        CK(hipEventRecord(a));
        if (mode == 0) hipLaunchKernelGGL(k_pull<0>, g, dim3(256), 0, 0, rsrc, rslot, fbits, ftick, N, 100u, out);
        if (mode == 1) hipLaunchKernelGGL(k_pull<1>, g, dim3(256), 0, 0, rsrc, rslot, fbits, ftick, N, 100u, out);
        if (mode == 2) hipLaunchKernelGGL(k_pull<2>, g, dim3(256), 0, 0, rsrc, rslot, fbits, ftick, N, 100u, out);
        if (mode == 3) hipLaunchKernelGGL(k_pull<3>, g, dim3(256), 0, 0, rsrc, rslot, fbits, ftick, N, 100u, out);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
      }
      printf("p=%.2f mode=%d  %.2f ms per window  (%.2f G in-edges/s, %.2f TB/s of table)\n", p, mode, best,
             E / (best * 1e6), E * 5.0 / (best * 1e9));
    }
  }
  return 0;
}
