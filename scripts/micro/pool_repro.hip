// Stream-ordered pool allocations at overlay sizes (verdict r04, Weak 5).
//
// Round 4 moved the overlay's buffers (gs_overlay.hip: one event bucket per
// ring block, the sort scratch, the emit list) from hipMalloc/hipFree to
// hipMallocAsync/hipFreeAsync and the N = 1e9 build then reported
// "too many overlay events at one node in one tick" (k_process saw a run of
// > 2^26 events with one destination: keys that no scatter wrote), while every
// smaller build (<= ~1.3 GB per bucket) stayed bit-exact.  This program
// replays the overlay's allocation pattern with nothing else: NB buckets of B
// bytes each, grown the way overlay_build grows them (allocate the new buffer,
// copy the filled prefix, free the old one), a scratch buffer swapped with a
// bucket as the radix sort's double buffer does, every buffer written with a
// pattern derived from (buffer id, generation, index) and checked after every
// step.  A check that fails names the buffer, the word and the allocation
// sizes: if pool memory aliases (or is shorter than requested), some buffer's
// words come back with another buffer's pattern.
//
// Usage: pool_repro <GiB per bucket> <buckets> [pool|malloc] [memcpy|kcopy] [nosync|sync]
//   kcopy: the regrow copies with a kernel instead of hipMemcpyAsync
//   sync:  hipStreamSynchronize after every allocation
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <utility>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));  \
      exit(2);                                                                  \
    }                                                                           \
  } while (0)

__device__ __forceinline__ uint64_t pat(uint32_t id, uint32_t gen, uint64_t i) {
  return ((uint64_t)id << 56) ^ ((uint64_t)gen << 48) ^ (i * 0x9E3779B97F4A7C15ull >> 16);
}

__global__ void k_copy(uint64_t* d, const uint64_t* s, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    d[i] = s[i];
}

__global__ void k_fill(uint64_t* p, uint64_t n, uint32_t id, uint32_t gen) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = pat(id, gen, i);
}

// bad[0] = mismatches, bad[1] = first bad index, bad[2] = the word found there
__global__ void k_check(const uint64_t* p, uint64_t n, uint32_t id, uint32_t gen, unsigned long long* bad) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t v = p[i];
    if (v != pat(id, gen, i)) {
      if (atomicAdd(&bad[0], 1ull) == 0) {
        bad[1] = i;
        bad[2] = v;
      }
    }
  }
}

struct Buf {
  uint64_t* p = nullptr;
  uint64_t words = 0;
  uint32_t id = 0, gen = 0;
};

static bool g_pool = true, g_kcopy = false, g_sync = false;
static hipStream_t g_st;

static void dalloc(Buf& b, uint64_t words) {
  if (g_pool) CK(hipMallocAsync((void**)&b.p, words * 8, g_st));
  else CK(hipMalloc((void**)&b.p, words * 8));
  if (g_sync) CK(hipStreamSynchronize(g_st));
  b.words = words;
}
static void dfree(Buf& b) {
  if (!b.p) return;
  if (g_pool) CK(hipFreeAsync(b.p, g_st));
  else { CK(hipStreamSynchronize(g_st)); CK(hipFree(b.p)); }
  b.p = nullptr;
  b.words = 0;
}

static unsigned long long* g_bad;
static int g_fail = 0;

static void fill(Buf& b, uint64_t n) {
  ++b.gen;
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, g_st, b.p, n, b.id, b.gen);
  CK(hipGetLastError());
}
static void check(const Buf& b, uint64_t n, const char* what) {
  CK(hipMemsetAsync(g_bad, 0, 24, g_st));
  hipLaunchKernelGGL(k_check, dim3(4096), dim3(256), 0, g_st, b.p, n, b.id, b.gen, g_bad);
  CK(hipGetLastError());
  unsigned long long h[3];
  CK(hipMemcpyAsync(h, g_bad, 24, hipMemcpyDeviceToHost, g_st));
  CK(hipStreamSynchronize(g_st));
  if (h[0]) {
    ++g_fail;
    printf("FAIL %s: buffer %u (%p, %llu words, gen %u): %llu bad words, first at %llu = %016llx (id %llu gen %llu)\n",
           what, b.id, (void*)b.p, (unsigned long long)b.words, b.gen, h[0], h[1], h[2], h[2] >> 56,
           (h[2] >> 48) & 255);
  }
}

int main(int argc, char** argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 5.0;
  const int nb = argc > 2 ? atoi(argv[2]) : 8;
  g_pool = !(argc > 3 && strcmp(argv[3], "malloc") == 0);
  g_kcopy = argc > 4 && strcmp(argv[4], "kcopy") == 0;
  g_sync = argc > 5 && strcmp(argv[5], "sync") == 0;
  CK(hipStreamCreate(&g_st));
  CK(hipMalloc(&g_bad, 24));
  if (g_pool) {
    hipMemPool_t pool;
    CK(hipDeviceGetDefaultMemPool(&pool, 0));
    uint64_t thr = ~0ull;  // keep freed memory in the pool (as the r04s build did)
    CK(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr));
  }
  const uint64_t words = (uint64_t)(gib * (1ull << 30)) / 8;
  printf("%s, %s, %s: %d buckets of %.2f GiB (%llu words)\n", g_pool ? "pool" : "malloc",
         g_kcopy ? "kernel copy" : "hipMemcpyAsync", g_sync ? "sync after alloc" : "no sync", nb, gib,
         (unsigned long long)words);
  std::vector<Buf> bk(nb);
  Buf scratch;
  scratch.id = 200;
  for (int i = 0; i < nb; ++i) {
    bk[i].id = (uint32_t)i;
    dalloc(bk[i], words / 2);  // tick 0: half size, grown below
    fill(bk[i], bk[i].words);
  }
  dalloc(scratch, words / 2);
  fill(scratch, scratch.words);
  for (int i = 0; i < nb; ++i) check(bk[i], bk[i].words, "initial");
  for (int round = 0; round < 3 && !g_fail; ++round) {
    for (int i = 0; i < nb; ++i) {
      // the regrow of gs_overlay.hip:549-556: new buffer, copy the filled prefix, free the old one
      Buf nbuf;
      nbuf.id = bk[i].id;
      nbuf.gen = bk[i].gen;
      const uint64_t keep = bk[i].words;
      dalloc(nbuf, bk[i].words + bk[i].words / 2 + 1);
      if (g_kcopy) {
        hipLaunchKernelGGL(k_copy, dim3(4096), dim3(256), 0, g_st, nbuf.p, bk[i].p, keep);
        CK(hipGetLastError());
      } else {
        CK(hipMemcpyAsync(nbuf.p, bk[i].p, keep * 8, hipMemcpyDeviceToDevice, g_st));
      }
      dfree(bk[i]);
      bk[i] = nbuf;
      check(bk[i], keep, "after regrow copy");
      fill(bk[i], bk[i].words);
    }
    // the sort's double buffer: grow scratch (free + allocate), use it, swap it with a bucket
    for (int i = 0; i < nb && !g_fail; ++i) {
      if (scratch.words < bk[i].words) {
        dfree(scratch);
        dalloc(scratch, bk[i].words + bk[i].words / 4);
      }
      scratch.id = bk[i].id;
      fill(scratch, scratch.words);
      std::swap(scratch, bk[i]);  // the sorted keys now live in the old scratch
      scratch.id = 200;
      fill(scratch, scratch.words);
      for (int j = 0; j < nb; ++j) check(bk[j], bk[j].words, "after swap");
      check(scratch, scratch.words, "scratch after swap");
    }
    printf("round %d done, %d failures\n", round, g_fail);
  }
  for (auto& b : bk) dfree(b);
  dfree(scratch);
  CK(hipStreamSynchronize(g_st));
  printf("%s\n", g_fail ? "POOL DEFECT REPRODUCED" : "no mismatch");
  return g_fail ? 1 : 0;
}
