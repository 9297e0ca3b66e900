// gs_rng.h -- keyed Philox4x32-10 streams shared by host and device code.
//
// Every rand.Intn call site of simulator.go becomes a pure function of
// (seed; kind, trial, tick, node, slot), so a decision does not depend on
// which lane, block, XCD or GPU makes it:
//   kind SENDER  simulator.go:240   ctr {0, 0, 0, .}            out[0] -> U_n
//   kind DELAY   simulator.go:167   ctr {v, t, 0, .}            out[0] -> U_(high-low)
//   kind DROP    simulator.go:172   ctr {v, t, j/4, .}          out[j%4] = r -> drop = U_100(r)
//                simulator.go:180   and the crash roll the message from sender v, fire tick t,
//                                   slot j carries: U_100(100 r mod 2^32) (drop_crash below)
//   kind PICK    simulator.go:97    ctr {v, 0, j, .}            out[0] -> U_n
//   kind OVDELAY simulator.go:153,160 ctr {u, t, k, .}          out[0] -> U_(high-low)
//   kind VICTIM  simulator.go:71    ctr {u, t, k, .}            out[0] -> U_deg
//   kind REPLACE simulator.go:86-88 ctr {u, t, k*64+a/4, .}     out[a%4] -> U_n
//   kind PUSHPULL (extension)        ctr {v, t, 0, .}            out[0] -> U_deg, out[1] -> U_100
//   kind ORDER   simulator.go:107-115 ctr {u, t, (g-1)/4, .}    out[(g-1)%4] -> U_(k-g+1): receipt
//                                   order, first_crash() below
// with counter word 3 = kind << 24 | trial.  U_m(r) = floor(r*m / 2^32).
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

namespace gs {

enum Kind : uint32_t {
  K_SENDER = 1, K_DELAY = 2, K_DROP = 3, K_CRASH = 4,  // K_CRASH: reserved (round 2's crash-roll stream)
  K_PICK = 5, K_OVDELAY = 6, K_VICTIM = 7, K_REPLACE = 8,
  K_PUSHPULL = 9,  // push-pull extension: peer pick + loss per (node, round)
  K_ORDER = 10     // receipt order of a (node, tick): first-crash position
};

struct u32x4 { uint32_t x, y, z, w; };

__host__ __device__ __forceinline__ uint32_t mulhi32(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umulhi(a, b);
#else
  return (uint32_t)(((uint64_t)a * b) >> 32);
#endif
}

// hi:lo of a * b.  On gfx950 one v_mad_u64_u32 instead of the v_mul_hi_u32 +
// v_mul_lo_u32 pair the compiler emits (Philox +24 %, scripts/micro/philox_bench2).
__host__ __device__ __forceinline__ void mul64(uint32_t a, uint32_t b, uint32_t& hi, uint32_t& lo) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint64_t p;
  asm("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(p) : "v"(a), "v"(b) : "vcc");
  hi = (uint32_t)(p >> 32);
  lo = (uint32_t)p;
#else
  const uint64_t p = (uint64_t)a * b;
  hi = (uint32_t)(p >> 32);
  lo = (uint32_t)p;
#endif
}

// Philox4x32-10 (Random123 round and key schedule).
__host__ __device__ __forceinline__ u32x4 philox(uint32_t c0, uint32_t c1, uint32_t c2,
                                                 uint32_t c3, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t h0, l0, h1, l1;
    mul64(0xD2511F53u, c0, h0, l0);
    mul64(0xCD9E8D57u, c2, h1, l1);
    const uint32_t n0 = h1 ^ c1 ^ k0, n2 = h0 ^ c3 ^ k1;
    c0 = n0; c1 = l1; c2 = n2; c3 = l0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return u32x4{c0, c1, c2, c3};
}

__host__ __device__ __forceinline__ uint32_t lane_of(const u32x4& v, uint32_t i) {
  return i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w;
}

__host__ __device__ __forceinline__ uint32_t uniform(uint32_t r, uint32_t m) {
  return mulhi32(r, m);
}

// RandomDrop (simulator.go:172) and the message's RandomCrash roll (:180)
// from ONE 32-bit draw r: the first two base-100 digits of r / 2^32,
// drop = floor(100 r / 2^32) and crash = floor(100 (100 r mod 2^32) / 2^32)
// = floor(10^4 r / 2^32) mod 100.  Each of the 10^4 pairs (drop, crash) is
// taken by floor(2^32 / 10^4) or one more of the 2^32 words, so the two are
// independent and uniform to within 2.4e-6 relative.
__host__ __device__ __forceinline__ void drop_crash(uint32_t r, uint32_t& drop, uint32_t& crash) {
  uint32_t hi, lo;
  mul64(r, 100u, hi, lo);
  drop = hi;
  crash = mulhi32(lo, 100u);
}

__host__ __device__ __forceinline__ uint32_t ctr3(uint32_t kind, uint32_t trial) {
  return (kind << 24) | (trial & 0xFFFFFFu);
}

struct Key {
  uint32_t k0, k1, trial;
};

__host__ __device__ __forceinline__ uint32_t draw0(const Key& k, uint32_t kind, uint32_t a,
                                                   uint32_t b, uint32_t c) {
  return philox(a, b, c, ctr3(kind, k.trial), k.k0, k.k1).x;
}

// Delay of a Broadcast/Makeup/Breakup in ticks (simulator.go:166-168); a
// delay below one tick runs as one tick.
__host__ __device__ __forceinline__ uint32_t fire_offset(int32_t low, uint32_t span, uint32_t r) {
  const int64_t d = (int64_t)low + (int64_t)uniform(r, span);
  return d < 1 ? 1u : (uint32_t)d;
}

// Rule A6 (simulator.go:107-123): the k receipts of node u at tick t are
// taken in a uniformly random order; each carries its own crash roll (kind
// CRASH, keyed by its sender), and `ones` of them (1 <= ones <= k) crash the
// node.  Returns the 1-based position of the first crashing receipt: draws
// U_(k-g+1)(r_g) < ones, g = 1, 2, ..., with r_g = Philox{u, t, (g-1)/4,
// c3order} lane (g-1)%4 (oracle/gsoracle.c or_first_crash).  k == 1 or
// ones == k needs no draw.
__host__ __device__ __forceinline__ uint32_t first_crash(uint32_t u, uint32_t t, uint32_t k, uint32_t ones,
                                                         uint32_t c3order, uint32_t k0, uint32_t k1) {
  if (k <= 1 || ones >= k) return 1;
  u32x4 r{0, 0, 0, 0};
  for (uint32_t g = 1;; ++g) {  // ends by g = k - ones + 1, where U_ones < ones
    if (((g - 1) & 3) == 0) r = philox(u, t, (g - 1) >> 2, c3order, k0, k1);
    if (uniform(lane_of(r, (g - 1) & 3), k - g + 1) < ones) return g;
  }
}

}  // namespace gs
