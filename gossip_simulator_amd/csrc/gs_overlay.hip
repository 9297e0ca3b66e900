// gs_overlay.hip -- overlay construction (simulator.go:62-106,127-164,214-235)
// as a tick-synchronous, sort-bucketed GPU protocol, processed in BLOCKS of
// ticks.
//
// An event sent at tick t arrives at t + off with off >= delay_low
// (simulator.go:172-176), so the events of the ticks [t, t + delay_low) are
// all known before any of them is processed, and a node's events of several
// such ticks can be replayed in one pass, tick by tick: its friends row is
// read and written once per block instead of once per tick (the row traffic
// -- every row of the table is touched in each tick of the burst -- is what
// bounds the build).  A block holds L ticks, L | 10 (the 10-tick windows of
// the stabilisation rule, simulator.go:222-234, end on block ends),
// L <= delay_low, L <= 2^TB.
//
// Events are u64 keys  dst << (B+1+TB) | tag << (B+1) | src << 1 | kind
// (kind 0 = makeup, 1 = breakup, B = bits of the id space, tag = the arrival
// tick's place in its block, TB = tag bits: 2B + 1 + TB <= 64), kept in one
// bucket per block of a ring of NB blocks.  A block:
//   1. radix-sort its bucket by destination (rocprim Onesweep) -> each node's
//      events contiguous;
//   2. one lane per destination (the first event of its run) orders the run
//      by (tag, src, kind) and replays it tick by tick -- the makeup /
//      breakup handler bodies -- with every draw keyed by (dst, tick,
//      ordinal k within the tick), so identical keys (identical messages)
//      commute;
//   3. each processed event emits at most one event (a breakup on eviction,
//      a makeup on replacement); a workgroup's emitted events are appended to
//      a compact list and counted per bucket, and a write scatter pass moves
//      them into their arrival blocks' buckets.
// Tick 0 is the needNewFriendCh burst: every node picks `fanout` friends
// (self -> id+1, simulator.go:97-101) and sends a makeup to each.
// Blocks of several ticks measured SLOWER than one tick per block (the row
// traffic halves, but the longer runs and fuller buckets cost more), so the
// default is L = 1; GS_OV_BLOCK=2|5|10 enables them (tests check every L).
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "gs_internal.h"
#include "gossip.h"

namespace gs {
namespace {

// Buckets in the overlay's ring of blocks: NB = ceil(R / L) + 2 <= kMaxRing
// (the scatter's and the process kernel's LDS histograms hold kMaxRing), so
// delayhigh <= kMaxRing - 2 at one tick per block
constexpr uint32_t kMaxRing = 1026;
constexpr uint32_t kScatterBlock = 256;
constexpr uint32_t kScatterIPT = 8;

struct OvParams {
  uint64_t n;                 // nodes per trial
  uint32_t fanout, fanin, stride, R, B;
  int32_t delay_low;
  uint32_t delay_span;
  Key key;
  // batched trials: trial i's node v has id i << tlog | v (tlog = 32: one trial)
  uint32_t tlog, tmask;
  // tick blocks: L ticks per block, TB tag bits, NB buckets in the ring
  uint32_t L, TB, NB;
  // per-bucket counters (counts, fill) lie fs words apart (GS_OV_FILL_STRIDE)
  uint32_t fs;
};

// Key node and counter word 3 of global id g (per-trial keys, gs_internal.h).
__device__ __forceinline__ uint32_t ov_draw(const OvParams& p, uint32_t kind, uint32_t g, uint32_t b,
                                            uint32_t c) {
  uint32_t node, c3;
  node_key(p.tlog, p.tmask, p.key, g, kind, node, c3);
  return philox(node, b, c, c3, p.key.k0, p.key.k1).x;
}

// An event arriving at tick a (>= 1): its key and its bucket.  (32-bit tick
// arithmetic: a 64-bit division is a long software sequence on the GPU, and
// the burst makes one key per friend slot.)
__device__ __forceinline__ uint64_t ev_key(const OvParams& p, uint32_t dst, uint32_t a, uint32_t src,
                                           uint32_t kind) {
  const uint32_t tag = (a - 1) % p.L;
  return ((uint64_t)dst << (p.B + 1 + p.TB)) | ((uint64_t)tag << (p.B + 1)) | ((uint64_t)src << 1) | kind;
}
__device__ __forceinline__ uint32_t ev_bucket(const OvParams& p, uint32_t a) {
  return ((a - 1) / p.L) % p.NB;
}

// Item sources for the bucket scatter -------------------------------------
struct PickSource {  // tick 0: item i = (trial i / (n*fanout), v, j = i % fanout)
  OvParams p;
  uint8_t* deg;
  uint32_t* ids;
  bool write_rows;
  __device__ __forceinline__ void get(uint64_t i, uint64_t& key, uint32_t& slot) const {
    const uint64_t per = p.n * p.fanout;
    const uint32_t tr = (uint32_t)(i / per);
    const uint64_t rem = i - (uint64_t)tr * per;
    const uint32_t v = (uint32_t)(rem / p.fanout), j = (uint32_t)(rem % p.fanout);
    const uint32_t tb = (uint32_t)((uint64_t)tr << p.tlog), gv = tb | v;
    uint32_t f = uniform(ov_draw(p, K_PICK, gv, 0, j), (uint32_t)p.n);       // :97
    if (f == v) f = (uint32_t)((f + 1) % p.n);                              // :98-100
    if (write_rows) {
      ids[(size_t)gv * p.stride + j] = tb | f;                              // :101
      if (j == 0) deg[gv] = (uint8_t)p.fanout;
    }
    // :102 Makeup, arriving at tick 0 + off
    const uint32_t a = fire_offset(p.delay_low, p.delay_span, ov_draw(p, K_OVDELAY, gv, 0, j));
    key = ev_key(p, tb | f, a, gv, 0u);
    slot = ev_bucket(p, a);
  }
  // the counting pass needs the bucket only: the delay draw, not the pick
  __device__ __forceinline__ uint32_t bucket_of(uint64_t i) const {
    const uint64_t per = p.n * p.fanout;
    const uint32_t tr = (uint32_t)(i / per);
    const uint64_t rem = i - (uint64_t)tr * per;
    const uint32_t v = (uint32_t)(rem / p.fanout), j = (uint32_t)(rem % p.fanout);
    const uint32_t gv = (uint32_t)((uint64_t)tr << p.tlog) | v;
    return ev_bucket(p, fire_offset(p.delay_low, p.delay_span, ov_draw(p, K_OVDELAY, gv, 0, j)));
  }
};

struct OutSource {  // events emitted by a processing block (a compact list)
  const uint64_t* out;
  const uint16_t* oslot;
  __device__ __forceinline__ void get(uint64_t i, uint64_t& key, uint32_t& slot) const {
    key = out[i];
    slot = oslot[i];
  }
  __device__ __forceinline__ uint32_t bucket_of(uint64_t i) const { return oslot[i]; }
};

// COUNT: counts[s] += items bound for bucket s.  WRITE: append them to bucket s.
// caps (WRITE, optional): bucket capacities; a workgroup whose reservation
// would pass one sets *ovf and writes none of that bucket's items (tick 0's
// planned buckets: the host then counts and writes again).
template <bool WRITE, class Src>
__global__ __launch_bounds__(kScatterBlock) void k_scatter(Src src, uint64_t nitems, uint32_t R, uint32_t fs,
                                                           unsigned long long* counts,
                                                           unsigned long long* fill,
                                                           uint64_t* const* buckets,
                                                           const unsigned long long* caps = nullptr,
                                                           uint32_t* ovf = nullptr) {
  __shared__ uint32_t s_hist[kMaxRing];
  __shared__ unsigned long long s_base[kMaxRing];
  for (uint32_t s = threadIdx.x; s < R; s += blockDim.x) s_hist[s] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kScatterBlock * kScatterIPT;
  uint64_t key[kScatterIPT];
  uint32_t slot[kScatterIPT], rank[kScatterIPT];
#pragma unroll
  for (uint32_t k = 0; k < kScatterIPT; ++k) {
    const uint64_t i = base + (uint64_t)k * kScatterBlock + threadIdx.x;
    slot[k] = 0xFFFFu;
    if (i < nitems) {
      if (WRITE) src.get(i, key[k], slot[k]);
      else slot[k] = src.bucket_of(i);
    }
    if (slot[k] != 0xFFFFu) rank[k] = atomicAdd(&s_hist[slot[k]], 1u);
  }
  __syncthreads();
  if (!WRITE) {
    for (uint32_t s = threadIdx.x; s < R; s += blockDim.x)
      if (s_hist[s]) atomicAdd(&counts[(size_t)s * fs], (unsigned long long)s_hist[s]);
    return;
  }
  for (uint32_t s = threadIdx.x; s < R; s += blockDim.x)
    if (s_hist[s]) {
      const unsigned long long b = atomicAdd(&fill[(size_t)s * fs], (unsigned long long)s_hist[s]);
      const bool over = caps && b + s_hist[s] > caps[s];
      if (over) atomicOr(ovf, 1u);
      s_base[s] = over ? ~0ull : b;
    }
  __syncthreads();
#pragma unroll
  for (uint32_t k = 0; k < kScatterIPT; ++k)
    if (slot[k] != 0xFFFFu && s_base[slot[k]] != ~0ull) buckets[slot[k]][s_base[slot[k]] + rank[k]] = key[k];
}

struct TickCounters {
  unsigned long long makeups, breakups, err;
};

// The block's sort: rocprim Onesweep, 8-bit digits (gfx950's default for
// 8-byte keys; 10-bit digits, 3 passes over a 30-bit destination instead of 4,
// measured no faster: profiles/r04j_overlay_ab.txt).
using OvRadix = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<512, 12>, rocprim::kernel_config<512, 12>, 8,
                                        rocprim::block_radix_rank_algorithm::match>>;

// Process a block: each thread takes kProcIPT event positions of the sorted
// bucket, and the first event of each destination's run (its destination
// differs from the previous key's) replays the run -- no head list.  The
// events a workgroup emits are gathered in LDS and appended with one
// reservation to the compact list (eout, eslot); a workgroup whose runs emit
// more than kEmitCap appends the rest one by one.
constexpr uint32_t kProcBlock = 256;
constexpr uint32_t kProcIPT = 4;
constexpr uint32_t kEmitCap = 1024;  // (10 KB of LDS: eight waves per SIMD, as the VGPRs allow)

// Wave-aggregated append among the ACTIVE lanes (divergent call sites).
__device__ __forceinline__ uint32_t active_append(uint32_t* n) {
  const unsigned long long act = __ballot(1);
  const uint32_t lane = threadIdx.x & 63, leader = (uint32_t)__ffsll((long long)act) - 1;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(n, (uint32_t)__popcll(act));
  base = __shfl(base, (int)leader, 64);
  return base + __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
}

// A friends row of 8 slots in registers: named members and selects only (an
// indexed array was left in scratch by the compiler).
struct Row8 {
  uint32_t v0, v1, v2, v3, v4, v5, v6, v7;
  // (the empty asm keeps the members in VGPRs: without it the select chains
  // were folded back into an indexed array in scratch)
  __device__ __forceinline__ void pin() {
    asm volatile("" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7));
  }
  __device__ __forceinline__ uint32_t get(uint32_t j) const {
    const bool b0 = j & 1, b1 = j & 2, b2 = j & 4;
    const uint32_t l0 = b0 ? v1 : v0, l1 = b0 ? v3 : v2, l2 = b0 ? v5 : v4, l3 = b0 ? v7 : v6;
    const uint32_t m0 = b1 ? l1 : l0, m1 = b1 ? l3 : l2;
    return b2 ? m1 : m0;
  }
  __device__ __forceinline__ void set(uint32_t j, uint32_t x) {
    v0 = j == 0 ? x : v0; v1 = j == 1 ? x : v1; v2 = j == 2 ? x : v2; v3 = j == 3 ? x : v3;
    v4 = j == 4 ? x : v4; v5 = j == 5 ? x : v5; v6 = j == 6 ? x : v6; v7 = j == 7 ? x : v7;
    pin();
  }
  // the first slot < d holding x, or d
  __device__ __forceinline__ uint32_t find(uint32_t x, uint32_t d) const {
    uint32_t i = d;
    i = (7 < d && v7 == x) ? 7 : i; i = (6 < d && v6 == x) ? 6 : i; i = (5 < d && v5 == x) ? 5 : i;
    i = (4 < d && v4 == x) ? 4 : i; i = (3 < d && v3 == x) ? 3 : i; i = (2 < d && v2 == x) ? 2 : i;
    i = (1 < d && v1 == x) ? 1 : i; i = (0 < d && v0 == x) ? 0 : i;
    return i;
  }
  // slots idx .. d-2 take their successors (removeFriend's shift)
  __device__ __forceinline__ void remove(uint32_t idx, uint32_t d) {
    v0 = (0 >= idx && 1 < d) ? v1 : v0; v1 = (1 >= idx && 2 < d) ? v2 : v1;
    v2 = (2 >= idx && 3 < d) ? v3 : v2; v3 = (3 >= idx && 4 < d) ? v4 : v3;
    v4 = (4 >= idx && 5 < d) ? v5 : v4; v5 = (5 >= idx && 6 < d) ? v6 : v5;
    v6 = (6 >= idx && 7 < d) ? v7 : v6;
    pin();
  }
};

// A run's keys, in LDS (the staged tile) or in global memory (a run that
// leaves the staged keys); local index 0 .. len-1.
struct LdsRun {
  uint64_t* s;
  __device__ __forceinline__ uint64_t get(uint32_t i) const { return s[i]; }
  __device__ __forceinline__ void set(uint32_t i, uint64_t v) const { s[i] = v; }
};
struct GlobalRun {
  uint64_t* g;
  __device__ __forceinline__ uint64_t get(uint32_t i) const { return g[i]; }
  __device__ __forceinline__ void set(uint32_t i, uint64_t v) const { g[i] = v; }
};

// One destination's run: ordered by (tag, src, kind) -- tick by tick, each
// tick's events in the order the handlers replay them (runs are short:
// insertion) -- and replayed against its friends row.  ROW8 (stride 8, the
// window engine's padded rows): the row was read into registers by the caller
// (two 16-B loads, with its degree d), is replayed there with unrolled
// selects and written back once -- instead of a dependent global load per
// slot of every linear search, shift and victim read.  Else in memory.
template <bool ROW8, class Run, class Emit>
__device__ __forceinline__ void ov_replay(const OvParams& p, uint64_t t0, Run run, uint32_t len, uint32_t u,
                                          uint8_t* deg, uint32_t* ids, Row8 r8, uint32_t d, Emit& emit,
                                          uint32_t& mk, uint32_t& bk, uint32_t& err) {
  const uint32_t sh = p.B + 1 + p.TB;  // destination field
  const uint64_t smask = (1ull << p.B) - 1, lmask = (1ull << sh) - 1;
  const uint32_t tagmask = (1u << p.TB) - 1;
  const uint32_t ul = u & p.tmask, tb = u & ~p.tmask;  // node within its trial, trial base
  for (uint32_t i = 1; i < len; ++i) {
    const uint64_t key = run.get(i);
    uint32_t j = i;
    for (; j > 0; --j) {
      const uint64_t prev = run.get(j - 1);
      if ((prev & lmask) <= (key & lmask)) break;
      run.set(j, prev);
    }
    run.set(j, key);
  }
  uint32_t* row = ids + (size_t)u * p.stride;
  uint32_t ptag = ~0u, k = 0;
  bool dirty = false;
#define RGET8(j) (r8.get(j))
#define RSET8(j, x) (r8.set((j), (x)), dirty = true)
  for (uint32_t i = 0; i < len; ++i) {
    const uint64_t key = run.get(i);
    const uint32_t src = (uint32_t)((key >> 1) & smask);
    const uint32_t tag = (uint32_t)(key >> (p.B + 1)) & tagmask;
    k = tag == ptag ? k + 1 : 0u;  // the ordinal restarts with each tick
    ptag = tag;
    const uint32_t t = (uint32_t)(t0 + tag);
    uint32_t emitted_dst = ~0u, emitted_kind = 0;
    if (k >= (1u << 26)) { err |= 2; continue; }
    if ((key & 1) == 0) {                                   // makeUpCh (:66-75)
      ++mk;
      if (d < p.fanin) {
        if (ROW8) RSET8(d, src); else row[d] = src;
        ++d;
      } else {
        const uint32_t pos = uniform(ov_draw(p, K_VICTIM, u, t, k), d);
        emitted_dst = ROW8 ? RGET8(pos) : row[pos];          // Breakup (:73)
        emitted_kind = 1;
        if (ROW8) RSET8(pos, src); else row[pos] = src;
      }
    } else {                                                // breakUpCh (:76-94)
      ++bk;
      uint32_t idx = 0;
      if (ROW8) {
        idx = r8.find(src, d);
      } else {
        while (idx < d && row[idx] != src) ++idx;
      }
      if (idx < d) {
        if (d > p.fanout) {                                 // removeFriend (:83)
          if (ROW8) {
            r8.remove(idx, d);
            dirty = true;
          } else {
            for (uint32_t q = idx; q + 1 < d; ++q) row[q] = row[q + 1];
          }
          --d;
        } else {                                            // replace (:86-91)
          uint32_t nf = 0, a = 0, kn, c3;
          node_key(p.tlog, p.tmask, p.key, u, K_REPLACE, kn, c3);
          for (; a < 256; ++a) {
            const u32x4 rr = philox(kn, t, (k << 6) | (a >> 2), c3, p.key.k0, p.key.k1);
            nf = uniform(lane_of(rr, a & 3), (uint32_t)p.n);
            if (nf != (src & p.tmask) && nf != ul) break;
          }
          nf |= tb;
          if (a == 256) {
            err |= 1;
          } else {
            if (ROW8) RSET8(idx, nf); else row[idx] = nf;
            emitted_dst = nf;                               // Makeup (:91)
            emitted_kind = 0;
          }
        }
      }
    }
    if (emitted_dst != ~0u) {
      const uint32_t a = t + fire_offset(p.delay_low, p.delay_span, ov_draw(p, K_OVDELAY, u, t, k));
      emit(ev_key(p, emitted_dst, a, u, emitted_kind), ev_bucket(p, a));
    }
  }
#undef RGET8
#undef RSET8
  if (ROW8 && dirty) {
    reinterpret_cast<uint4*>(row)[0] = make_uint4(r8.v0, r8.v1, r8.v2, r8.v3);
    reinterpret_cast<uint4*>(row)[1] = make_uint4(r8.v4, r8.v5, r8.v6, r8.v7);
  }
  deg[u] = (uint8_t)d;
}

// STAGED: the workgroup's 1024 key positions plus kProcLook more are read
// into LDS in one coalesced pass first; run heads, run ends and the runs'
// insertion sorts then work there.  STAGED 2 loads each run's row and degree
// just before its replay; STAGED 1 loads those of a thread's up to kProcIPT
// runs together first (more loads in flight, but 97 VGPRs: measured slower).
// Without it every run walks a chain of dependent global loads (its key, the
// key before it, each key to its end, the sort's re-reads, then the row): the
// burst ticks' waves spent 77 % of their cycles waiting
// (profiles/r05as_process_pmc.txt).  A run that leaves the staged keys is
// replayed from global memory.
constexpr uint32_t kProcLook = 64;
template <bool ROW8, uint32_t STAGED>  // STAGED 1: keys in LDS, rows batched; 2: keys in LDS only
__global__ __launch_bounds__(kProcBlock) void k_process(const OvParams p, uint64_t t0, uint64_t* keys, uint64_t m,
                                                        uint8_t* deg, uint32_t* ids, uint64_t* eout,
                                                        uint16_t* eslot, unsigned long long* ecount,
                                                        unsigned long long* counts, TickCounters* tc,
                                                        const uint32_t* skip) {
  if (skip && *skip) return;  // (the destination partition overflowed: the host sorts the tick)
  constexpr uint32_t kTile = kProcBlock * kProcIPT, kStage = STAGED ? kTile + kProcLook : 1;
  __shared__ uint64_t s_ev[kEmitCap];
  __shared__ uint16_t s_sl[kEmitCap];
  __shared__ uint32_t s_hist[kMaxRing];  // the workgroup's emitted events per bucket
  __shared__ uint64_t s_key[kStage + 1];  // STAGED: [0] = the key before the tile, [1 + i] = position base + i
  __shared__ uint32_t s_n, s_mk, s_bk, s_err;
  __shared__ unsigned long long s_base;
  const uint32_t tid = threadIdx.x;
  if (tid == 0) { s_n = 0; s_mk = 0; s_bk = 0; s_err = 0; }
  for (uint32_t q = tid; q < p.NB; q += kProcBlock) s_hist[q] = 0;
  const uint64_t base = (uint64_t)blockIdx.x * kTile;
  if (STAGED) {
    for (uint32_t i = tid; i < kStage; i += kProcBlock) {
      const uint64_t g = base + i;
      s_key[1 + i] = g < m ? keys[g] : 0ull;
    }
    if (tid == 0) s_key[0] = base > 0 ? keys[base - 1] : 0ull;
  }
  __syncthreads();
  uint32_t mk = 0, bk = 0, err = 0;
  auto emit = [&](uint64_t key, uint32_t slot) {
    const uint32_t at = active_append(&s_n);
    if (at < kEmitCap) {
      s_ev[at] = key;
      s_sl[at] = (uint16_t)slot;
    } else {
      const unsigned long long q = atomicAdd(ecount, 1ull);
      eout[q] = key;
      eslot[q] = (uint16_t)slot;
      atomicAdd(&counts[(size_t)slot * p.fs], 1ull);
    }
  };
  const uint32_t sh = p.B + 1 + p.TB;  // destination field
  auto load_row = [&](uint32_t u, Row8& r8) {
    const uint32_t* row = ids + (size_t)u * p.stride;
    const uint4 a = reinterpret_cast<const uint4*>(row)[0], b = reinterpret_cast<const uint4*>(row)[1];
    r8 = Row8{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    r8.pin();
  };
  if (STAGED) {
    // heads and run lengths from the staged keys (len 0: no run starts here;
    // glob: the run leaves the staged keys)
    uint32_t hu[kProcIPT], hlen[kProcIPT];
    bool glob[kProcIPT];
#pragma unroll
    for (uint32_t r = 0; r < kProcIPT; ++r) {
      const uint32_t pos = r * kProcBlock + tid;
      const uint64_t start = base + pos;
      hlen[r] = 0;
      glob[r] = false;
      hu[r] = 0;
      if (start < m) {
        const uint32_t u = (uint32_t)(s_key[1 + pos] >> sh);
        if (start == 0 || (uint32_t)(s_key[pos] >> sh) != u) {
          uint32_t len = 1;
          while (pos + len < kStage && start + len < m && (uint32_t)(s_key[1 + pos + len] >> sh) == u) ++len;
          glob[r] = pos + len == kStage && start + len < m;
          hu[r] = u;
          hlen[r] = len;
        }
      }
    }
    constexpr uint32_t NR = STAGED == 1 ? kProcIPT : 1;  // rows held at once
    Row8 r8[NR];
    uint32_t hd[NR];
    if (STAGED == 1) {
#pragma unroll
      for (uint32_t r = 0; r < NR; ++r) {
        r8[r] = Row8{};
        hd[r] = 0;
        if (hlen[r]) {
          if (ROW8) load_row(hu[r], r8[r]);
          hd[r] = deg[hu[r]];
        }
      }
    }
#pragma unroll
    for (uint32_t r = 0; r < kProcIPT; ++r) {
      if (!hlen[r]) continue;
      const uint32_t q = STAGED == 1 ? r : 0;
      if (STAGED != 1) {
        r8[q] = Row8{};
        if (ROW8) load_row(hu[r], r8[q]);
        hd[q] = deg[hu[r]];
      }
      const uint32_t pos = r * kProcBlock + tid;
      if (!glob[r]) {
        ov_replay<ROW8>(p, t0, LdsRun{&s_key[1 + pos]}, hlen[r], hu[r], deg, ids, r8[q], hd[q], emit, mk, bk, err);
      } else {
        const uint64_t start = base + pos;
        uint64_t end = start + hlen[r];
        while (end < m && (uint32_t)(keys[end] >> sh) == hu[r]) ++end;
        ov_replay<ROW8>(p, t0, GlobalRun{keys + start}, (uint32_t)(end - start), hu[r], deg, ids, r8[q], hd[q], emit,
                        mk, bk, err);
      }
    }
  } else {
    for (uint32_t r = 0; r < kProcIPT; ++r) {
      const uint64_t start = base + (uint64_t)r * kProcBlock + tid;
      if (start >= m) break;
      const uint32_t u = (uint32_t)(keys[start] >> sh);
      if (start > 0 && (uint32_t)(keys[start - 1] >> sh) == u) continue;  // not a run head
      uint64_t end = start + 1;
      while (end < m && (uint32_t)(keys[end] >> sh) == u) ++end;
      Row8 r8{};
      if (ROW8) load_row(u, r8);
      ov_replay<ROW8>(p, t0, GlobalRun{keys + start}, (uint32_t)(end - start), u, deg, ids, r8, (uint32_t)deg[u], emit,
                      mk, bk, err);
    }
  }
  if (mk) atomicAdd(&s_mk, mk);
  if (bk) atomicAdd(&s_bk, bk);
  if (err) atomicOr(&s_err, err);
  __syncthreads();
  const uint32_t n = min(s_n, kEmitCap);
  if (tid == 0) {
    if (n) s_base = atomicAdd(ecount, (unsigned long long)n);
    if (s_mk) atomicAdd(&tc->makeups, (unsigned long long)s_mk);
    if (s_bk) atomicAdd(&tc->breakups, (unsigned long long)s_bk);
    if (s_err) atomicOr(&tc->err, (unsigned long long)s_err);
  }
  __syncthreads();
  // the list, and the per-bucket counts the host sizes the buckets by (no
  // separate count pass over the list)
  for (uint32_t j = tid; j < n; j += kProcBlock) {
    eout[s_base + j] = s_ev[j];
    eslot[s_base + j] = s_sl[j];
    atomicAdd(&s_hist[s_sl[j]], 1u);
  }
  __syncthreads();
  for (uint32_t q = tid; q < p.NB; q += kProcBlock)
    if (s_hist[q]) atomicAdd(&counts[(size_t)q * p.fs], (unsigned long long)s_hist[q]);
}

// ---- destination partition of a dense tick (replaces the radix sort) -------
// k_process needs each destination's events contiguous, not the bucket in
// global destination order, so a dense tick is grouped in three passes:
//   P1 (k_ov_part<false>): the bucket -> coarse regions by dst >> (F + 8),
//      each coarse region in kOvSub sub-regions, one per XCD (tile t writes
//      sub-region t % 8: the reservation atomics of a region spread over 8
//      addresses -- one address per coarse region took P1 from 3.3 to 5.4 ms
//      per burst tick);
//   P2 (k_ov_part<true>):  each coarse sub-region -> its 256 fine regions by
//      dst >> F (F = kOvFineLog: 16,384 ids per fine bucket);
//   k_ov_scan:             the fine regions' fills -> compact offsets;
//   P3 (k_ov_fine):        each fine region counting-sorted by its 14-bit
//      local destination in LDS, written at its compact offset: k_process
//      gets exactly the tick's m keys (padded regions cost it 7 %).
// P1 and P2 are LDS counting sorts of 8192-key tiles over 256 digits written
// out as runs (≈ 32 keys, 256 B per run): two streaming passes where the
// Onesweep sort made four digit passes plus a histogram pass.  Region sizes
// are planned from the tick's event count and each fine bucket's share of
// the id space (the destinations are uniform over live ids); a region that
// would overflow sets a flag and the host sorts that tick with rocprim
// instead -- the bucket itself is only read, so the fallback starts from it.
// Within a destination the events come out in no particular order; k_process
// orders each run by (tag, src, kind) itself, so the result is the same.
constexpr uint32_t kOvFineLog = 14;
constexpr uint32_t kOvpBlock = 512, kOvpIPT = 16, kOvpTile = kOvpBlock * kOvpIPT;  // 8192 keys per tile
constexpr uint32_t kOvSub = 8;  // P1 sub-regions per coarse region (one per XCD: blockIdx % 8)
constexpr uint32_t kOvFineBlock = 1024, kOvFineIPT = 16;
constexpr uint32_t kOvFineMax = kOvFineBlock * kOvFineIPT;  // keys a fine region may hold (= 2^kOvFineLog)
static_assert(kOvFineMax == 1u << kOvFineLog, "one counter per local destination");

struct OvPart {
  const uint64_t* in;
  uint64_t* out;
  uint64_t m;                          // P1: the bucket's keys
  const unsigned long long* fstart;    // [nfb + 1] fine region starts; coarse region c = fine regions 256c ..
  unsigned long long* cfill;           // [ncb * kOvSub] coarse sub-region fills
  unsigned long long* ffill;           // [nfb] fine region fills
  const uint32_t* tprefix;             // [ncb * kOvSub + 1] P2 tiles per coarse sub-region (prefix)
  uint32_t* flag;                      // 1: a region overflowed
  uint32_t ncb, nfb, sh;               // coarse / fine regions, the key's destination shift
  const unsigned long long* cstart;    // [ncb * kOvSub + 1] coarse sub-region (c, x) starts in P1's output
};

// A wave's LDS counter increments, one atomic per DISTINCT digit: the lanes
// of the lowest pending lane's digit are ranked together (ballot + mbcnt)
// and leave, until none is pending.  A batched bucket is a sequence of
// single-trial chunks (each k_process workgroup appends its emitted events at
// once, ~100 per bucket, in no trial order), so a wave's 64 consecutive keys
// fall in one or two trials: the per-trial count pass took 70.7 -> 27.4 ms
// per two C3 builds with it (profiles/r06_c3_partition_experiments.txt).  Not for waves that hold
// several digits: in P2 (~8 fine regions per wave) it cost 60 -> 145 ms, and
// P1 was unchanged.
// Every lane of the wave calls it; returns the lane's rank among its digit's
// keys (0 for an invalid lane).
template <bool RET>
__device__ __forceinline__ uint32_t peel_rank(uint32_t* cnt, uint32_t d, bool valid) {
  const uint32_t lane = threadIdx.x & 63;
  uint32_t rank = 0;
  unsigned long long todo = __ballot(valid);
  while (todo) {
    const uint32_t leader = (uint32_t)__ffsll((long long)todo) - 1;
    const uint32_t ld = (uint32_t)__shfl((int)d, (int)leader, 64);
    const bool mine = valid && d == ld;
    const unsigned long long peers = __ballot(mine);
    uint32_t base = 0;
    if (lane == leader) {
      if (RET) base = atomicAdd(&cnt[ld], (uint32_t)__popcll(peers));
      else atomicAdd(&cnt[ld], (uint32_t)__popcll(peers));
    }
    if (RET) {
      base = (uint32_t)__shfl((int)base, (int)leader, 64);
      if (mine)
        rank = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(peers >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)peers, 0u));
    }
    todo &= ~peers;
  }
  return rank;
}

// P1's tile t writes sub-region t % kOvSub of each coarse region: (c, x) is
// [cstart[c * kOvSub + x], cstart[c * kOvSub + x + 1]).
__device__ __forceinline__ void ov_sub(const OvPart& a, uint32_t c, uint32_t x, unsigned long long& start,
                                       unsigned long long& cap) {
  const uint32_t r = c * kOvSub + x;
  start = a.cstart[r];
  cap = a.cstart[r + 1] - start;
}

__device__ __forceinline__ uint32_t block_exscan256(uint32_t v, uint32_t* s_ws) {
  // exclusive scan of v over threads 0..255 of the block (v = 0 elsewhere);
  // every thread calls it
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  uint32_t x = v;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63 && wv < 4) s_ws[wv] = x;
  __syncthreads();
  uint32_t before = 0;
  for (uint32_t q = 0; q < wv && q < 4; ++q) before += s_ws[q];
  __syncthreads();
  return before + x - v;
}

template <bool FINE>
__global__ __launch_bounds__(kOvpBlock) void k_ov_part(const OvPart a) {
  __shared__ uint64_t s_key[kOvpTile];
  __shared__ uint32_t s_cnt[256], s_off[256], s_ws[4], s_ovf;
  __shared__ unsigned long long s_gb[256];
  const uint32_t tid = threadIdx.x;
  uint64_t lo, hi;
  uint32_t dshift, dbase = 0, xsub = 0;
  if (!FINE) {
    lo = (uint64_t)blockIdx.x * kOvpTile;
    hi = min(a.m, lo + kOvpTile);
    dshift = kOvFineLog + 8;
    xsub = blockIdx.x % kOvSub;  // consecutive workgroups run on consecutive XCDs
  } else {
    // tile b of coarse sub-region r = c * kOvSub + x: tprefix[r] <= b < tprefix[r + 1]
    const uint32_t b = blockIdx.x;
    uint32_t l = 0, r = a.ncb * kOvSub;
    while (r - l > 1) {
      const uint32_t mid = (l + r) >> 1;
      if (a.tprefix[mid] <= b) l = mid; else r = mid;
    }
    unsigned long long st, cap;
    ov_sub(a, l / kOvSub, l % kOvSub, st, cap);
    lo = st + (uint64_t)(b - a.tprefix[l]) * kOvpTile;
    hi = min(st + min((unsigned long long)a.cfill[l], cap), lo + kOvpTile);  // (an overflowed P1 is discarded)
    dshift = kOvFineLog;
    dbase = (l / kOvSub) << 8;
  }
  if (lo >= hi) return;  // (uniform: an empty tail tile of a region)
  if (tid < 256) s_cnt[tid] = 0;
  if (tid == 0) s_ovf = 0;
  __syncthreads();
  const uint32_t n = (uint32_t)(hi - lo);
  uint64_t key[kOvpIPT];
  uint32_t rank[kOvpIPT];
#pragma unroll
  for (uint32_t j = 0; j < kOvpIPT; ++j) {
    const uint32_t i = j * kOvpBlock + tid;
    if (i < n) {
      key[j] = a.in[lo + i];
      const uint32_t d = (uint32_t)(key[j] >> (a.sh + dshift)) - dbase;
      rank[j] = atomicAdd(&s_cnt[d & 255], 1u);
      if (d > 255) s_ovf = 1;  // (not a destination of this region: corrupt input)
    }
  }
  __syncthreads();
  const uint32_t c = tid < 256 ? s_cnt[tid] : 0u;
  const uint32_t off = block_exscan256(c, s_ws);
  if (tid < 256) {
    s_off[tid] = off;
    if (c) {
      const uint32_t reg = dbase + tid;  // P1: coarse region; P2: fine region
      unsigned long long st, cap, *fill;
      if (FINE) {
        st = reg < a.nfb ? a.fstart[reg] : 0;
        cap = reg < a.nfb ? a.fstart[reg + 1] - st : 0;
        fill = &a.ffill[min(reg, a.nfb - 1)];
      } else {
        if (reg < a.ncb) ov_sub(a, reg, xsub, st, cap);
        else st = cap = 0;
        fill = &a.cfill[min(reg, a.ncb - 1) * kOvSub + xsub];
      }
      if (cap == 0) {
        s_ovf = 1;
      } else {
        const unsigned long long base = atomicAdd(fill, (unsigned long long)c);
        if (base + c > cap) s_ovf = 1;
        s_gb[tid] = st + base;
      }
    }
  }
  __syncthreads();
  if (s_ovf) {
    if (tid == 0) atomicOr(a.flag, 1u);
    return;
  }
#pragma unroll
  for (uint32_t j = 0; j < kOvpIPT; ++j) {
    const uint32_t i = j * kOvpBlock + tid;
    if (i < n) {
      const uint32_t d = ((uint32_t)(key[j] >> (a.sh + dshift)) - dbase) & 255;
      s_key[s_off[d] + rank[j]] = key[j];
    }
  }
  __syncthreads();
  for (uint32_t i = tid; i < n; i += kOvpBlock) {  // runs of one digit: consecutive addresses
    const uint64_t k = s_key[i];
    const uint32_t d = ((uint32_t)(k >> (a.sh + dshift)) - dbase) & 255;
    a.out[s_gb[d] + (i - s_off[d])] = k;
  }
}

// Batched trials: the tick's events per trial (trial = destination >> tlog),
// so the partition plan can follow each trial's own count -- trials drift
// apart after the burst, and a plan by node share alone overflowed on every
// dense C3 tick.  LDS histogram per workgroup (<= kOvMaxTrials), one global
// add per non-empty trial.
// It also counts the keys of every coarse sub-region (c = dst >> 22, x = the
// key's P1 tile % kOvSub) exactly: a batched bucket is made of single-trial
// runs (tick 0's picks written trial by trial, later ticks' emissions one
// k_process workgroup at a time), so the tiles' shares of a coarse region are
// far from even.
constexpr uint32_t kOvMaxTrials = 8192, kOvTrialBlock = 1024, kOvTrialGrid = 512;
__global__ __launch_bounds__(kOvTrialBlock) void k_ov_count(const uint64_t* keys, uint64_t m, uint32_t sh,
                                                            uint32_t tlog, uint32_t ntr, uint32_t ncb,
                                                            unsigned long long* tcnt, unsigned long long* cxcnt) {
  __shared__ uint32_t h[kOvMaxTrials];
  __shared__ uint32_t hc[256 * kOvSub];
  for (uint32_t i = threadIdx.x; i < ntr; i += kOvTrialBlock) h[i] = 0;
  for (uint32_t i = threadIdx.x; i < ncb * kOvSub; i += kOvTrialBlock) hc[i] = 0;
  __syncthreads();
  // block-uniform trip count (peel_rank: every lane of a wave takes part);
  // a wave's keys lie in one or two trials: one atomic per distinct counter
  for (uint64_t i0 = (uint64_t)blockIdx.x * kOvTrialBlock; i0 < m; i0 += (uint64_t)gridDim.x * kOvTrialBlock) {
    const uint64_t i = i0 + threadIdx.x;
    const bool in = i < m;
    const uint64_t dst = in ? keys[i] >> sh : 0ull;
    peel_rank<false>(h, min((uint32_t)(dst >> tlog), ntr - 1), in);
    const uint32_t c = min((uint32_t)(dst >> (kOvFineLog + 8)), ncb - 1), x = (uint32_t)(i / kOvpTile) % kOvSub;
    peel_rank<false>(hc, c * kOvSub + x, in);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < ntr; i += kOvTrialBlock)
    if (h[i]) atomicAdd(&tcnt[i], (unsigned long long)h[i]);
  for (uint32_t i = threadIdx.x; i < ncb * kOvSub; i += kOvTrialBlock)
    if (hc[i]) atomicAdd(&cxcnt[i], (unsigned long long)hc[i]);
}

// The fine regions' fills -> the exclusive prefix fbase[0..nfb] (one
// workgroup): P3 writes fine region f's keys at fbase[f], so k_process gets
// the tick's keys back to back, without the regions' unused tails.
constexpr uint32_t kOvScanBlock = 1024, kOvScanIPT = 8, kOvScanChunk = kOvScanBlock * kOvScanIPT;
__global__ __launch_bounds__(kOvScanBlock) void k_ov_scan(const unsigned long long* ffill, uint32_t nfb,
                                                          const unsigned long long* fstart,
                                                          unsigned long long* fbase) {
  // chunks of 8192 fills: coalesced loads into LDS, 8 consecutive per thread
  // scanned in registers, a block scan of the thread sums, coalesced stores;
  // the chunk total carries into the next chunk
  __shared__ unsigned long long s_v[kOvScanChunk];
  __shared__ unsigned long long s_ws[kOvScanBlock / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  unsigned long long carry = 0;
  for (uint32_t c0 = 0; c0 < nfb; c0 += kOvScanChunk) {
#pragma unroll
    for (uint32_t j = 0; j < kOvScanIPT; ++j) {
      const uint32_t f = c0 + j * kOvScanBlock + tid;
      // (an overflowed region is discarded with the tick)
      s_v[j * kOvScanBlock + tid] = f < nfb ? min(ffill[f], fstart[f + 1] - fstart[f]) : 0ull;
    }
    __syncthreads();
    unsigned long long v[kOvScanIPT], sum = 0;
#pragma unroll
    for (uint32_t j = 0; j < kOvScanIPT; ++j) {
      v[j] = s_v[tid * kOvScanIPT + j];
      sum += v[j];
    }
    unsigned long long x = sum;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const unsigned long long y = __shfl_up(x, d, 64);
      if (lane >= d) x += y;
    }
    if (lane == 63) s_ws[wv] = x;
    __syncthreads();
    unsigned long long run = carry + x - sum, total = 0;
    for (uint32_t q = 0; q < kOvScanBlock / 64; ++q) {
      if (q < wv) run += s_ws[q];
      total += s_ws[q];
    }
#pragma unroll
    for (uint32_t j = 0; j < kOvScanIPT; ++j) {
      s_v[tid * kOvScanIPT + j] = run;
      run += v[j];
    }
    __syncthreads();
#pragma unroll
    for (uint32_t j = 0; j < kOvScanIPT; ++j) {
      const uint32_t f = c0 + j * kOvScanBlock + tid;
      if (f < nfb) fbase[f] = s_v[j * kOvScanBlock + tid];
    }
    carry += total;
    __syncthreads();
  }
  if (tid == 0) fbase[nfb] = carry;
}

// P3: fine region f (in: P2's output) counting-sorted by local destination
// into out at fbase[f].  Keys stay in registers (16 per lane); counters,
// then offsets, are u16 pairs in u32 words.
__global__ __launch_bounds__(kOvFineBlock) void k_ov_fine(const uint64_t* in, uint64_t* out,
                                                          const unsigned long long* fstart,
                                                          const unsigned long long* ffill,
                                                          const unsigned long long* fbase, uint32_t sh) {
  __shared__ uint32_t s_c[kOvFineMax / 2];
  __shared__ uint32_t s_ws[kOvFineBlock / 64];
  const uint32_t f = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint64_t lo = fstart[f], cap = fstart[f + 1] - lo;
  const uint32_t n = (uint32_t)min((uint64_t)ffill[f], cap);  // (cap <= kOvFineMax: the host's plan)
  const uint64_t ob = fbase[f];
#pragma unroll
  for (uint32_t q = 0; q < kOvFineMax / 2 / kOvFineBlock; ++q) s_c[q * kOvFineBlock + tid] = 0;
  __syncthreads();
  uint64_t key[kOvFineIPT];
#pragma unroll
  for (uint32_t j = 0; j < kOvFineIPT; ++j) {
    const uint32_t i = j * kOvFineBlock + tid;
    if (i < n) {
      key[j] = in[lo + i];
      const uint32_t l = (uint32_t)(key[j] >> sh) & (kOvFineMax - 1);
      atomicAdd(&s_c[l >> 1], 1u << ((l & 1) << 4));
    }
  }
  __syncthreads();
  // exclusive scan over the 16,384 counters: thread t owns words 8t .. 8t + 7
  constexpr uint32_t W = kOvFineMax / 2 / kOvFineBlock;
  uint32_t sum = 0;
#pragma unroll
  for (uint32_t q = 0; q < W; ++q) {
    const uint32_t w = s_c[tid * W + q];
    sum += (w & 0xFFFFu) + (w >> 16);
  }
  uint32_t x = sum;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) s_ws[wv] = x;
  __syncthreads();
  uint32_t run = x - sum;
  for (uint32_t q = 0; q < wv; ++q) run += s_ws[q];
#pragma unroll
  for (uint32_t q = 0; q < W; ++q) {
    const uint32_t w = s_c[tid * W + q], c0 = w & 0xFFFFu;
    s_c[tid * W + q] = run | ((run + c0) << 16);
    run += c0 + (w >> 16);
  }
  __syncthreads();
  // each key takes the next place of its destination (the offsets count up:
  // a destination's half-word never carries into its neighbour's)
#pragma unroll
  for (uint32_t j = 0; j < kOvFineIPT; ++j) {
    const uint32_t i = j * kOvFineBlock + tid;
    if (i < n) {
      const uint32_t l = (uint32_t)(key[j] >> sh) & (kOvFineMax - 1), s = (l & 1) << 4;
      out[ob + ((atomicAdd(&s_c[l >> 1], 1u << s) >> s) & 0xFFFFu)] = key[j];
    }
  }
}

#define OVCHK(expr)                                                              \
  do {                                                                           \
    hipError_t e_ = (expr);                                                      \
    if (e_ != hipSuccess) {                                                      \
      snprintf(res->msg, sizeof(res->msg), "%s: %s", #expr, hipGetErrorString(e_)); \
      res->rc = GS_EDEVICE;                                                      \
      goto cleanup;                                                              \
    }                                                                            \
  } while (0)

using DevBuf = OverlayWork::Buf;

// Grown with 25 % headroom: a batched context rebuilds overlays batch after
// batch, and a regrow (hipFree + hipMalloc of GB-sized buckets) cost up to
// 1.7 s where the next batch's events outnumbered the first's by a little.
// (The stream-ordered pool allocator instead corrupted the N = 1e9 build:
// profiles/r04s_overlay_pool.txt.)
static void free_buf(DevBuf& b) {
  if (b.raw) (void)dev_free(b.raw);
  b.p = b.raw = nullptr;
  b.bytes = 0;
}
static hipError_t grow(DevBuf& b, size_t bytes, hipStream_t st) {
  (void)st;
  if (b.bytes >= bytes) return hipSuccess;
  const size_t nb = std::max(bytes + bytes / 4, b.bytes * 3 / 2);
  free_buf(b);
  hipError_t e = dev_malloc(&b.raw, nb + b.off);
  if (e == hipSuccess) {
    b.p = (char*)b.raw + b.off;
    b.bytes = nb;
  } else {
    b.raw = nullptr;
  }
  return e;
}

// The ring's buckets start at staggered offsets (slot s: s x 4352 B mod 64 KB;
// GS_OV_STAGGER=0: all at their allocation's base, A/B).  In one interleaved
// A/B P1 took 65 vs 84 ms per N = 1e9 build, but later runs spread 64-80 ms
// either way (profiles/r05ad_scatter_pmc.txt): kept as harmless, not as a
// measured win.  It was tried for the emitted events' scatter, whose burst
// ticks run 3 or 16 ms with the same requests, hits and misses (also with a
// 1-MB stagger): no change there.
static size_t ov_stagger(uint32_t s) {
  static const bool off = getenv("GS_OV_STAGGER") && atoi(getenv("GS_OV_STAGGER")) == 0;
  return off ? 0 : ((size_t)s * 4352u) % 65536u;
}

// The destination partition's plan for a tick of m events: fine region
// capacities from each fine bucket's share of the live ids (4 % + 6 sigma +
// 32 over its expected count -- the breakup waves after the burst are
// over-dispersed: at 1 % + 5 sigma five N = 1e9 ticks overflowed a fine
// region by up to 3 %; GS_OV_PART_SCALE replaces the 1.04, and one
// below 1 drops the slack -- the tests force the overflow fallback with it),
// coarse regions = 256 fine regions each.  False
// where the partition does not apply (a sparse tick: the radix sort's fixed
// cost is lower; a fine region beyond LDS; more than 256 coarse regions).
struct OvPlan {
  uint64_t nfb = 0, ncb = 0, total = 0, ctotal = 0, m = 0;
  double scale = 0;
  std::vector<unsigned long long> fstart;  // [nfb + 1]
  std::vector<uint32_t> tprefix;           // [ncb * kOvSub + 1]
  std::vector<unsigned long long> cstart;  // [ncb * kOvSub + 1] OvPart::cstart
};

// tcnt / cxcnt (batched trials, k_ov_count): the tick's events per trial and
// per coarse sub-region -- fine regions then follow their trial's count and
// the coarse sub-regions are exact.
static bool ov_plan(OvPlan& pl, uint64_t m, uint64_t n, uint32_t trials, uint32_t tlog, uint64_t ntot,
                    double scale, const unsigned long long* tcnt = nullptr,
                    const unsigned long long* cxcnt = nullptr) {
  const uint64_t nfb = (ntot + kOvFineMax - 1) >> kOvFineLog, ncb = (nfb + 255) / 256;
  if (nfb == 0 || ncb > 256 || m < 32 * nfb) return false;
  if (!tcnt && pl.m == m && pl.nfb == nfb && pl.scale == scale) return true;
  const uint64_t tmask = tlog >= 32 ? ~0ull : (1ull << tlog) - 1;
  const double live = (double)n * (trials > 1 ? trials : 1);
  pl.m = 0;
  pl.nfb = nfb;
  pl.ncb = ncb;
  pl.fstart.resize(nfb + 1);
  pl.tprefix.resize(ncb * kOvSub + 1);
  pl.cstart.resize(ncb * kOvSub + 1);
  uint64_t at = 0;
  for (uint64_t f = 0; f < nfb; ++f) {
    pl.fstart[f] = at;
    const uint64_t local = (f << kOvFineLog) & tmask;  // (tlog >= kOvFineLog: a fine bucket is in one trial)
    const uint64_t valid = local < n ? std::min<uint64_t>(kOvFineMax, n - local) : 0;
    if (!valid) continue;
    // batched: the fine bucket's trial's own count (tlog >= kOvFineLog)
    const double e = tcnt ? (double)tcnt[(f << kOvFineLog) >> tlog] * (double)valid / (double)n
                          : (double)m * (double)valid / live;
    const uint64_t cap = (uint64_t)std::ceil(scale >= 1.0 ? e * scale + 6.0 * std::sqrt(e) + 32.0 : e * scale);
    if (cap > kOvFineMax) return false;
    at += cap;
  }
  pl.fstart[nfb] = at;
  pl.total = at;
  // coarse sub-regions (c, x): P1's tile t (kOvpTile keys, the last one
  // short) writes sub-region t % kOvSub.  Exact counts when given; else the
  // coarse region's fine capacity split by the share of the bucket the tiles
  // of x hold (a single trial's bucket is well mixed)
  uint64_t share[kOvSub] = {};
  const uint64_t ntile = (m + kOvpTile - 1) / kOvpTile;
  for (uint32_t x = 0; x < kOvSub; ++x)
    for (uint64_t t = x; t < ntile; t += kOvSub) share[x] += std::min<uint64_t>(kOvpTile, m - t * kOvpTile);
  uint64_t cat = 0;
  uint32_t tiles = 0;  // P2's tiles per coarse sub-region
  for (uint64_t c = 0; c < ncb; ++c) {
    const uint64_t ccap = pl.fstart[std::min<uint64_t>((c + 1) * 256, nfb)] - pl.fstart[c * 256];
    for (uint32_t x = 0; x < kOvSub; ++x) {
      const uint64_t r = c * kOvSub + x;
      pl.cstart[r] = cat;
      pl.tprefix[r] = tiles;
      const uint64_t cx = cxcnt ? cxcnt[r] : (uint64_t)std::ceil((double)ccap * (double)share[x] / (double)m);
      cat += cx;
      tiles += (uint32_t)((cx + kOvpTile - 1) / kOvpTile);
    }
  }
  pl.cstart[ncb * kOvSub] = cat;
  pl.tprefix[ncb * kOvSub] = tiles;
  pl.ctotal = cat;
  pl.m = tcnt || cxcnt ? 0 : m;  // (a counted plan is not reused)
  pl.scale = scale;
  return true;
}

static uint32_t node_bits(uint64_t n) {
  uint32_t b = 1;
  while (b < 31 && (1ull << b) < n) ++b;
  return b;
}

}  // namespace

void overlay_free(OverlayWork* ws, hipStream_t st) {
  (void)st;
  if (!ws) return;
  for (auto& b : ws->bucket) free_buf(b);
  ws->bucket.clear();
  for (DevBuf* b : {&ws->scratch, &ws->outb, &ws->oslotb, &ws->cub_tmp, &ws->meta, &ws->fine, &ws->ovp}) free_buf(*b);
}

int overlay_build(uint64_t n, uint32_t trials, uint32_t tlog, int32_t fanout, int32_t fanin,
                  int32_t delay_low, int32_t delay_high, Key key, uint8_t* d_deg, uint32_t* d_ids,
                  uint32_t stride, uint64_t max_ticks, hipStream_t stream, OverlayWindowSink sink,
                  OverlayResult* res, OverlayWork* ws) {
  res->rc = GS_OK;
  res->final_tick = 0;
  res->msg[0] = 0;
  OvParams p;
  p.n = n;
  p.fanout = (uint32_t)fanout;
  p.fanin = (uint32_t)fanin;
  p.stride = stride;
  p.R = delay_high > 2 ? (uint32_t)delay_high : 2u;
  p.tlog = tlog;
  p.tmask = tlog >= 32 ? ~0u : (1u << tlog) - 1;
  const uint64_t ntot = trials > 1 ? (uint64_t)trials << tlog : n;  // id space
  p.B = node_bits(ntot);
  p.delay_low = delay_low;
  p.delay_span = (uint32_t)(delay_high - delay_low);
  p.key = key;
  if (p.R + 2 > kMaxRing) {
    res->rc = GS_EINVAL;
    snprintf(res->msg, sizeof(res->msg), "delayhigh %d exceeds the overlay ring limit %u",
             delay_high, kMaxRing - 2);
    return res->rc;
  }
  {
    // tick blocks: L | 10, L <= delay_low, L <= 2^TB with 2B + 1 + TB <= 64
    // default one tick per block: blocks of 2, 5 or 10 ticks measured slower
    // (profiles/r04q_overlay_blocks.txt); GS_OV_BLOCK raises the cap (read per
    // build: the tests switch it)
    const char* be = getenv("GS_OV_BLOCK");
    const uint32_t lmax = be ? (uint32_t)atoi(be) : 1u;
    const uint32_t tbmax = std::min<uint32_t>(4u, 63u - 2 * p.B);
    // a block's bucket stays below 2^31 events (the sort's item count): the
    // burst's n * fanout makeups spread over delayhigh - delaylow ticks
    const double burst = (double)n * p.fanout * (trials > 1 ? trials : 1);
    const double per_tick = burst / std::max<uint32_t>(p.delay_span, 1u);
    p.L = 1;
    for (uint32_t L : {10u, 5u, 2u}) {
      if (L <= lmax && (int32_t)L <= delay_low && L <= (1u << tbmax) && per_tick * L * 1.25 < 2147483647.0) {
        p.L = L;
        break;
      }
    }
    p.TB = 0;
    while ((1u << p.TB) < p.L) ++p.TB;
    // the ring: an event arrives at most delay_high - 1 ticks after it is sent
    p.NB = (p.R + p.L - 1) / p.L + 2;  // <= R + 2 <= kMaxRing (checked above)
  }
  const uint32_t NB = p.NB;
  // The per-bucket counters every workgroup of k_process and k_scatter adds
  // to (counts, fill) lie fs words apart (GS_OV_FILL_STRIDE, A/B).
  p.fs = getenv("GS_OV_FILL_STRIDE") ? std::max(1, atoi(getenv("GS_OV_FILL_STRIDE"))) : 1;
  const uint32_t fs = p.fs;
  // buffers live in the caller's workspace across builds (batched C3 builds
  // one overlay per batch; reallocating tens of GB per block was the cost)
  if (ws->bucket.size() < NB) ws->bucket.resize(NB);
  for (uint32_t s = 0; s < NB; ++s)
    if (!ws->bucket[s].raw) ws->bucket[s].off = ov_stagger(s);
  std::vector<DevBuf>& bucket = ws->bucket;
  std::vector<uint64_t> fill(NB, 0);
  DevBuf &scratch = ws->scratch, &outb = ws->outb, &oslotb = ws->oslotb, &cub_tmp = ws->cub_tmp,
         &meta = ws->meta, &fine = ws->fine, &ovp = ws->ovp;
  // the destination partition of dense ticks (GS_OV_SORT=1: the radix sort
  // for every tick, A/B)
  // Batched trials drift apart after the burst (one trial's wave of
  // breakups is another's lull), so a plan by node share overflowed on every
  // dense C3 tick (up to 16x a fine region's share): batched plans follow
  // each trial's own count of the tick's events and exact coarse sub-region
  // counts (k_ov_count).  That is exact but not faster for C3's batches
  // (overlay 559-566 vs 548-551 ms per 5,000-trial batch: the count pass, two
  // syncs and a 40,000-region plan per tick cost what the sort saves), so
  // batched builds sort unless GS_OV_PART_BATCHED=1 (the tests).
  const bool part_ok = !getenv("GS_OV_SORT") && (trials <= 1 || (getenv("GS_OV_PART_BATCHED") &&
                                                                  trials <= kOvMaxTrials));
  std::vector<unsigned long long> h_tcnt(trials > 1 ? trials : 0), h_cxcnt;
  const double part_scale = getenv("GS_OV_PART_SCALE") ? atof(getenv("GS_OV_PART_SCALE")) : 1.04;
  // rows of 8 slots replayed in registers (GS_OV_ROW8=0: slot by slot in memory, A/B)
  const bool row8 = stride == 8 && p.fanin <= 8 && !(getenv("GS_OV_ROW8") && atoi(getenv("GS_OV_ROW8")) == 0);
  // k_process with its keys staged in LDS and (2, the default) each run's row
  // loaded just before it is replayed or (1) the rows of a thread's runs loaded
  // together (97 VGPRs, 4 waves per SIMD: slower); 0: every key read from
  // global memory (A/B; profiles/r05au_process_staged_rows_ab.txt)
  const int staged = getenv("GS_OV_STAGED") ? atoi(getenv("GS_OV_STAGED")) : 2;
  OvPlan plan;
  uint32_t h_flag = 0;
  const int ov_debug = getenv("GS_OV_DEBUG") ? atoi(getenv("GS_OV_DEBUG")) : 0;
  ws->part_ticks = ws->sort_ticks = ws->part_fallbacks = ws->pick_fallbacks = 0;
  // meta layout: ptrs[NB] | nemit (64 B) | TickCounters | caps[NB] | ovf (64 B) | counts[NB * fs] | fill[NB * fs]
  uint64_t pending = 0, wm = 0, wb = 0;
  std::vector<unsigned long long> h_counts(NB), hfill(NB);
  std::vector<uint64_t*> h_ptrs(NB, nullptr);
  unsigned long long *d_counts = nullptr, *d_fill = nullptr, *d_nemit = nullptr;
  unsigned long long h_ne = 0;
  uint64_t** d_ptrs = nullptr;
  TickCounters* d_tc = nullptr;
  unsigned long long* d_caps = nullptr;  // tick 0's planned bucket capacities
  uint32_t* d_ovf = nullptr, h_ovf = 0;
  std::vector<unsigned long long> h_caps(NB, 0);
  TickCounters h_tc;
  const size_t head_bytes = (NB * 8 + 64 + sizeof(TickCounters) + NB * 8 + 64 + 255) / 256 * 256;
  const size_t meta_bytes = head_bytes + 2 * (size_t)NB * fs * 8;

  // host <-> device copies of the strided counters
  auto ctr_d2h = [&](unsigned long long* h, const unsigned long long* d) {
    return fs == 1 ? hipMemcpyAsync(h, d, NB * 8, hipMemcpyDeviceToHost, stream)
                   : hipMemcpy2DAsync(h, 8, d, (size_t)fs * 8, 8, NB, hipMemcpyDeviceToHost, stream);
  };
  auto ctr_h2d = [&](unsigned long long* d, const unsigned long long* h) {
    return fs == 1 ? hipMemcpyAsync(d, h, NB * 8, hipMemcpyHostToDevice, stream)
                   : hipMemcpy2DAsync(d, (size_t)fs * 8, h, 8, 8, NB, hipMemcpyHostToDevice, stream);
  };
  const size_t ctr_bytes = (size_t)NB * fs * 8;
  OVCHK(grow(meta, meta_bytes, stream));
  d_ptrs = (uint64_t**)meta.p;
  d_nemit = (unsigned long long*)(d_ptrs + NB);
  d_tc = (TickCounters*)((char*)d_nemit + 64);
  d_caps = (unsigned long long*)(d_tc + 1);
  d_ovf = (uint32_t*)(d_caps + NB);
  d_counts = (unsigned long long*)((char*)meta.p + head_bytes);
  d_fill = d_counts + (size_t)NB * fs;
  OVCHK(hipMemsetAsync(meta.p, 0, meta_bytes, stream));

  {
    // ---- tick 0: picks (count, size buckets, write) --------------------
    const uint64_t items = n * (uint64_t)p.fanout * (trials > 1 ? trials : 1);
    if (items) {
      PickSource src{p, d_deg, d_ids, false};
      const uint64_t per = (uint64_t)kScatterBlock * kScatterIPT;
      const uint64_t blocks = (items + per - 1) / per;
      // The picks' arrival buckets follow the delay draw alone: offset
      // low + o, o uniform over the span (fire_offset), so bucket b expects
      // items x P(b).  Buckets sized to that + 6 sigma + 1024 are written in
      // ONE pass; a bucket past its plan (or GS_OV_PICK_COUNT=1) falls back to
      // the exact count pass and the write again (the rows it writes are the
      // same both times).  The count pass was 38 ms of the N = 1e9 build.
      bool planned = !getenv("GS_OV_PICK_COUNT");
      if (planned) {
        std::vector<double> expct(NB, 0.0);
        const uint32_t span = std::max<uint32_t>(p.delay_span, 1u);
        for (uint32_t o = 0; o < span; ++o) {
          // words r with floor(r * span / 2^32) == o
          const double lo = std::ceil((double)o * 4294967296.0 / span), hi = std::ceil((double)(o + 1) * 4294967296.0 / span);
          const uint32_t a = fire_offset(p.delay_low, span, (uint32_t)std::min(lo, 4294967295.0));
          expct[((a - 1) / p.L) % NB] += (double)items * (hi - lo) / 4294967296.0;
        }
        // (GS_OV_PICK_SCALE < 1 shrinks the plan: the tests force the fallback with it)
        const double psc = getenv("GS_OV_PICK_SCALE") ? atof(getenv("GS_OV_PICK_SCALE")) : 1.0;
        for (uint32_t s = 0; s < NB; ++s) {
          h_caps[s] = expct[s] <= 0 ? 0ull
                      : psc < 1.0 ? (unsigned long long)(expct[s] * psc)
                                  : (unsigned long long)std::ceil(expct[s] + 6.0 * std::sqrt(expct[s]) + 1024.0);
        }
        for (uint32_t s = 0; s < NB; ++s) {
          OVCHK(grow(bucket[s], std::max<unsigned long long>(h_caps[s], 1) * 8, stream));
          h_ptrs[s] = (uint64_t*)bucket[s].p;
        }
        OVCHK(hipMemcpyAsync(d_ptrs, h_ptrs.data(), NB * 8, hipMemcpyHostToDevice, stream));
        OVCHK(hipMemcpyAsync(d_caps, h_caps.data(), NB * 8, hipMemcpyHostToDevice, stream));
        OVCHK(hipMemsetAsync(d_ovf, 0, 4, stream));
        src.write_rows = true;
        hipLaunchKernelGGL((k_scatter<true, PickSource>), dim3((uint32_t)blocks), dim3(kScatterBlock), 0, stream,
                           src, items, NB, fs, d_counts, d_fill, (uint64_t* const*)d_ptrs,
                           (const unsigned long long*)d_caps, d_ovf);
        OVCHK(hipGetLastError());
        OVCHK(ctr_d2h(h_counts.data(), d_fill));
        OVCHK(hipMemcpyAsync(&h_ovf, d_ovf, 4, hipMemcpyDeviceToHost, stream));
        OVCHK(hipStreamSynchronize(stream));
        if (h_ovf) {  // the exact path below, from empty buckets
          planned = false;
          ++ws->pick_fallbacks;
          if (ov_debug) fprintf(stderr, "[overlay] tick 0: a planned pick bucket overflowed; counting\n");
          OVCHK(hipMemsetAsync(d_fill, 0, ctr_bytes, stream));
        }
      }
      if (!planned) {
        src.write_rows = false;
        hipLaunchKernelGGL((k_scatter<false, PickSource>), dim3((uint32_t)blocks), dim3(kScatterBlock),
                           0, stream, src, items, NB, fs, d_counts, d_fill, (uint64_t* const*)d_ptrs);
        OVCHK(hipGetLastError());
        OVCHK(ctr_d2h(h_counts.data(), d_counts));
        OVCHK(hipStreamSynchronize(stream));
        for (uint32_t s = 0; s < NB; ++s) {
          OVCHK(grow(bucket[s], (fill[s] + h_counts[s]) * 8, stream));
          h_ptrs[s] = (uint64_t*)bucket[s].p;
        }
        OVCHK(hipMemcpyAsync(d_ptrs, h_ptrs.data(), NB * 8, hipMemcpyHostToDevice, stream));
        src.write_rows = true;
        hipLaunchKernelGGL((k_scatter<true, PickSource>), dim3((uint32_t)blocks), dim3(kScatterBlock),
                           0, stream, src, items, NB, fs, d_counts, d_fill, (uint64_t* const*)d_ptrs);
        OVCHK(hipGetLastError());
      }
      for (uint32_t s = 0; s < NB; ++s) { fill[s] += h_counts[s]; pending += h_counts[s]; }
      OVCHK(hipMemsetAsync(d_counts, 0, ctr_bytes, stream));
    } else if (ntot) {
      OVCHK(hipMemsetAsync(d_deg, 0, ntot, stream));
    }
  }

  for (uint64_t blk = 0;; ++blk) {
    const uint64_t t0 = blk * p.L + 1, tend = t0 + p.L - 1;  // the block's ticks
    if (t0 > max_ticks) {
      res->rc = GS_ELIVELOCK;
      snprintf(res->msg, sizeof(res->msg),
               "overlay did not stabilise within %llu ticks (fanin <= fanout livelocks, "
               "simulator.go:66-94)", (unsigned long long)max_ticks);
      goto cleanup;
    }
    const uint32_t s = (uint32_t)(blk % NB);
    const uint64_t m = fill[s];
    if (m) {
      if (m > 0x7FFFFFFFull) {
        res->rc = GS_EOVERFLOW;
        snprintf(res->msg, sizeof(res->msg), "%llu overlay events in one block exceed 2^31-1",
                 (unsigned long long)m);
        goto cleanup;
      }
      OVCHK(grow(outb, m * 8, stream));
      OVCHK(grow(oslotb, m * 2, stream));
      {
        uint64_t* keys = nullptr;
        uint64_t mproc = m;
        uint32_t* d_pflag = nullptr;  // the partition's overflow flag (k_process stands down on it)
        uint64_t p_ncb = 0, p_nfb = 0;
        unsigned long long* d_pcfill = nullptr;
        bool plan_ok = part_ok && m >= 32 * ((ntot + kOvFineMax - 1) >> kOvFineLog);
        const uint64_t ncb0 = (((ntot + kOvFineMax - 1) >> kOvFineLog) + 255) / 256;
        plan_ok = plan_ok && ncb0 <= 256;
        if (plan_ok && trials > 1) {  // the tick's events per trial and per coarse sub-region, for the plan
          const size_t nc = ncb0 * kOvSub;
          OVCHK(grow(ovp, (trials + nc) * 8 + 64, stream));
          unsigned long long* d_tcnt = (unsigned long long*)ovp.p;
          OVCHK(hipMemsetAsync(d_tcnt, 0, (trials + nc) * 8, stream));
          hipLaunchKernelGGL(k_ov_count, dim3(kOvTrialGrid), dim3(kOvTrialBlock), 0, stream,
                             (const uint64_t*)bucket[s].p, m, p.B + 1 + p.TB, tlog, trials, (uint32_t)ncb0, d_tcnt,
                             d_tcnt + trials);
          OVCHK(hipGetLastError());
          h_cxcnt.resize(nc);
          OVCHK(hipMemcpyAsync(h_tcnt.data(), d_tcnt, trials * 8, hipMemcpyDeviceToHost, stream));
          OVCHK(hipMemcpyAsync(h_cxcnt.data(), d_tcnt + trials, nc * 8, hipMemcpyDeviceToHost, stream));
          OVCHK(hipStreamSynchronize(stream));
        }
        if (plan_ok && ov_plan(plan, m, n, trials, tlog, ntot, part_scale, trials > 1 ? h_tcnt.data() : nullptr,
                               trials > 1 ? h_cxcnt.data() : nullptr)) {
          // P1 bucket -> fine.p (coarse regions), P2 -> scratch (fine
          // regions), P3 -> fine.p (sorted, padded); the bucket stays intact
          const uint64_t nfb = plan.nfb, ncb = plan.ncb;
          // each array on lines of its own: a line that holds both a region
          // fill (atomics, executed at the memory side) and plan words every
          // tile reads sends those reads to memory too (the bucket scatter's
          // pointer table beside its fills cost it 2.2x)
          auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
          const size_t b_fs = al((nfb + 1) * 8), b_fill = al((ncb * kOvSub + nfb) * 8),
                       b_tp = al((ncb * kOvSub + 1) * 4), b_cs = al((ncb * kOvSub + 1) * 8);
          OVCHK(grow(scratch, plan.total * 8, stream));
          OVCHK(grow(fine, std::max(plan.total, plan.ctotal) * 8, stream));
          OVCHK(grow(ovp, 2 * b_fs + b_cs + b_fill + b_tp + 256, stream));
          unsigned long long* d_fstart = (unsigned long long*)ovp.p;
          unsigned long long* d_fbase = (unsigned long long*)((char*)d_fstart + b_fs);
          unsigned long long* d_cstart = (unsigned long long*)((char*)d_fbase + b_fs);
          unsigned long long* d_cfill = (unsigned long long*)((char*)d_cstart + b_cs);
          uint32_t* d_tp = (uint32_t*)((char*)d_cfill + b_fill);
          uint32_t* d_flag = (uint32_t*)((char*)d_tp + b_tp);
          OVCHK(hipMemcpyAsync(d_fstart, plan.fstart.data(), (nfb + 1) * 8, hipMemcpyHostToDevice, stream));
          OVCHK(hipMemcpyAsync(d_cstart, plan.cstart.data(), (ncb * kOvSub + 1) * 8, hipMemcpyHostToDevice, stream));
          OVCHK(hipMemcpyAsync(d_tp, plan.tprefix.data(), (ncb * kOvSub + 1) * 4, hipMemcpyHostToDevice, stream));
          OVCHK(hipMemsetAsync(d_cfill, 0, b_fill, stream));
          OVCHK(hipMemsetAsync(d_flag, 0, 4, stream));
          OvPart a{(const uint64_t*)bucket[s].p, (uint64_t*)fine.p, m, d_fstart, d_cfill, d_cfill + ncb * kOvSub, d_tp,
                   d_flag, (uint32_t)ncb, (uint32_t)nfb, p.B + 1 + p.TB, (const unsigned long long*)d_cstart};
          hipLaunchKernelGGL((k_ov_part<false>), dim3((uint32_t)((m + kOvpTile - 1) / kOvpTile)), dim3(kOvpBlock),
                             0, stream, a);
          OVCHK(hipGetLastError());
          a.in = (const uint64_t*)fine.p;
          a.out = (uint64_t*)scratch.p;
          if (plan.tprefix[ncb * kOvSub]) {
            hipLaunchKernelGGL((k_ov_part<true>), dim3(plan.tprefix[ncb * kOvSub]), dim3(kOvpBlock), 0, stream, a);
            OVCHK(hipGetLastError());
          }
          hipLaunchKernelGGL(k_ov_scan, dim3(1), dim3(kOvScanBlock), 0, stream,
                             (const unsigned long long*)(d_cfill + ncb * kOvSub), (uint32_t)nfb,
                             (const unsigned long long*)d_fstart, d_fbase);
          OVCHK(hipGetLastError());
          hipLaunchKernelGGL(k_ov_fine, dim3((uint32_t)nfb), dim3(kOvFineBlock), 0, stream,
                             (const uint64_t*)scratch.p, (uint64_t*)fine.p, (const unsigned long long*)d_fstart,
                             (const unsigned long long*)(d_cfill + ncb * kOvSub), (const unsigned long long*)d_fbase,
                             p.B + 1 + p.TB);
          OVCHK(hipGetLastError());
          // no host round trip here: k_process reads the flag (a region
          // over its plan) and stands down; the tick's sync below sees it
          keys = (uint64_t*)fine.p;  // m keys (when no region overflowed)
          d_pflag = d_flag;
          p_ncb = ncb;
          p_nfb = nfb;
          d_pcfill = d_cfill;
        }
        for (;;) {
          if (!keys) {
            // by (destination, tag): each destination's run comes out tick by
            // tick, and the process kernel orders each tick's few events by
            // (src, kind) itself (sorting by destination only left runs of L
            // ticks to the insertion sort, in global memory: slower than the
            // TB extra radix bits)
            OVCHK(grow(scratch, m * 8, stream));
            rocprim::double_buffer<uint64_t> db((uint64_t*)bucket[s].p, (uint64_t*)scratch.p);
            const unsigned begin_bit = p.B + 1, end_bit = 2 * p.B + 1 + p.TB;
            size_t sort_bytes = 0;
            OVCHK(rocprim::radix_sort_keys<OvRadix>(nullptr, sort_bytes, db, (size_t)m, begin_bit, end_bit, stream));
            OVCHK(grow(cub_tmp, sort_bytes, stream));
            sort_bytes = cub_tmp.bytes;
            OVCHK(rocprim::radix_sort_keys<OvRadix>(cub_tmp.p, sort_bytes, db, (size_t)m, begin_bit, end_bit, stream));
            keys = db.current();
            if (db.current() != (uint64_t*)bucket[s].p) std::swap(bucket[s], scratch);
            ++ws->sort_ticks;
          }
          const uint64_t per = (uint64_t)kProcBlock * kProcIPT;
          const dim3 pgrid((uint32_t)((mproc + per - 1) / per));
          auto* pk = row8 ? (staged == 2 ? k_process<true, 2> : staged ? k_process<true, 1> : k_process<true, 0>)
                          : (staged == 2 ? k_process<false, 2> : staged ? k_process<false, 1> : k_process<false, 0>);
          hipLaunchKernelGGL(pk, pgrid, dim3(kProcBlock), 0, stream, p, t0, keys, mproc, d_deg, d_ids,
                             (uint64_t*)outb.p, (uint16_t*)oslotb.p, d_nemit, d_counts, d_tc,
                             (const uint32_t*)d_pflag);
          OVCHK(hipGetLastError());
          OVCHK(hipMemcpyAsync(&h_ne, d_nemit, 8, hipMemcpyDeviceToHost, stream));
          OVCHK(ctr_d2h(h_counts.data(), d_counts));
          OVCHK(hipMemcpyAsync(&h_tc, d_tc, sizeof(h_tc), hipMemcpyDeviceToHost, stream));
          OVCHK(hipMemsetAsync(d_nemit, 0, 8, stream));
          if (d_pflag) OVCHK(hipMemcpyAsync(&h_flag, d_pflag, 4, hipMemcpyDeviceToHost, stream));
          OVCHK(hipStreamSynchronize(stream));
          if (d_pflag && !h_flag) ++ws->part_ticks;
          if (!d_pflag || !h_flag) break;
          // a region overflowed its plan: k_process did nothing (its counters
          // are still zero); sort this tick from its intact bucket
          ++ws->part_fallbacks;
          if (ov_debug) {  // which level overflowed, by how much
            const uint64_t ncb = p_ncb, nfb = p_nfb;
            unsigned long long* d_cfill = d_pcfill;
            std::vector<unsigned long long> cf(ncb * kOvSub), ff(nfb);
            OVCHK(hipMemcpy(cf.data(), d_cfill, cf.size() * 8, hipMemcpyDeviceToHost));
            OVCHK(hipMemcpy(ff.data(), d_cfill + ncb * kOvSub, ff.size() * 8, hipMemcpyDeviceToHost));
            double worst_c = 0, worst_f = 0;
            uint64_t nc = 0, nf = 0;
            for (uint64_t c = 0; c < ncb; ++c) {
              for (uint32_t x = 0; x < kOvSub; ++x) {
                const uint64_t cap = plan.cstart[c * kOvSub + x + 1] - plan.cstart[c * kOvSub + x];
                const double r = cap ? (double)cf[c * kOvSub + x] / cap : 1e9;
                if (cf[c * kOvSub + x] > cap) ++nc;
                worst_c = std::max(worst_c, r);
              }
            }
            for (uint64_t f = 0; f < nfb; ++f) {
              const uint64_t cap = plan.fstart[f + 1] - plan.fstart[f];
              if (ff[f] > cap) ++nf;
              worst_f = std::max(worst_f, cap ? (double)ff[f] / cap : (ff[f] ? 1e9 : 0));
            }
            fprintf(stderr, "[overlay] tick %llu: m=%llu partition fallback: %llu coarse / %llu fine regions over, "
                    "worst fill/cap %.3f / %.3f\n", (unsigned long long)t0, (unsigned long long)m,
                    (unsigned long long)nc, (unsigned long long)nf, worst_c, worst_f);
          }
          keys = nullptr;
          d_pflag = nullptr;
        }
      }
      {
        // the emitted events (k_process counted them per bucket): grow, write
        const uint64_t nitems = h_ne;
        if (ov_debug > 1)
          fprintf(stderr, "[overlay] tick %llu: %llu events, %llu emitted, %llu makeups %llu breakups\n",
                  (unsigned long long)t0, (unsigned long long)m, (unsigned long long)nitems,
                  (unsigned long long)h_tc.makeups, (unsigned long long)h_tc.breakups);
        OutSource osrc{(const uint64_t*)outb.p, (const uint16_t*)oslotb.p};
        const uint64_t per = (uint64_t)kScatterBlock * kScatterIPT;
        const uint32_t blocks = (uint32_t)((nitems + per - 1) / per);
        if (h_tc.err) {
          res->rc = (h_tc.err & 1) ? GS_EREJECT : GS_EINVAL;
          snprintf(res->msg, sizeof(res->msg), (h_tc.err & 1)
                       ? "replacement-friend rejection exhausted (n too small, simulator.go:87-89)"
                       : "too many overlay events at one node in one tick");
          goto cleanup;
        }
        // The current bucket is consumed; emitted events never land in it
        // (they arrive >= delay_low >= L ticks later: a later block).
        fill[s] = 0;
        pending -= m;
        for (uint32_t q = 0; q < NB; ++q) {
          if (!h_counts[q]) continue;
          if (bucket[q].bytes < (fill[q] + h_counts[q]) * 8) {
            DevBuf nb;
            nb.off = bucket[q].off;
            OVCHK(grow(nb, (fill[q] + h_counts[q]) * 8 * 3 / 2, stream));
            if (fill[q])
              OVCHK(hipMemcpyAsync(nb.p, bucket[q].p, fill[q] * 8, hipMemcpyDeviceToDevice, stream));
            OVCHK(hipStreamSynchronize(stream));
            free_buf(bucket[q]);
            bucket[q] = nb;
          }
        }
        bool moved = false;
        for (uint32_t q = 0; q < NB; ++q) {
          if (h_ptrs[q] != (uint64_t*)bucket[q].p) moved = true;
          h_ptrs[q] = (uint64_t*)bucket[q].p;
        }
        if (moved) OVCHK(hipMemcpyAsync(d_ptrs, h_ptrs.data(), NB * 8, hipMemcpyHostToDevice, stream));
        // hfill is rewritten only after the next block's count sync, which
        // orders it after this copy: no host sync after the scatter
        hfill.assign(fill.begin(), fill.end());
        OVCHK(ctr_h2d(d_fill, hfill.data()));
        if (blocks) {
          hipLaunchKernelGGL((k_scatter<true, OutSource>), dim3(blocks), dim3(kScatterBlock), 0, stream, osrc,
                             nitems, NB, fs, d_counts, d_fill, (uint64_t* const*)d_ptrs);
          OVCHK(hipGetLastError());
        }
        for (uint32_t q = 0; q < NB; ++q) { fill[q] += h_counts[q]; pending += h_counts[q]; }
        wm += h_tc.makeups;
        wb += h_tc.breakups;
        OVCHK(hipMemsetAsync(d_counts, 0, ctr_bytes, stream));
        OVCHK(hipMemsetAsync(d_tc, 0, sizeof(TickCounters), stream));
      }
    }
    if (tend > max_ticks) continue;  // (the next block reports the livelock)
    if (tend % 10 == 0) {                                     // simulator.go:222-234
      if (wm == 0 && wb == 0 && pending == 0) {
        res->final_tick = tend;
        break;
      }
      if (sink.push) sink.push(sink.self, tend, wm, wb);
      wm = wb = 0;
    }
  }

cleanup:
  (void)hipStreamSynchronize(stream);
  return res->rc;
}

}  // namespace gs
