// gs_window.hip -- the broadcast round loop as a window pipeline without
// global random atomics (the "window engine").
//
// Why windows: a Broadcast() fires off = max(delaylow,1)..delayhigh-1 ticks
// after the receipt that triggered it (simulator.go:122,142,167), so every
// broadcast firing in ticks [t0, t0+L), L <= max(delaylow,1), is already
// scheduled when tick t0 starts.  The L ticks are processed together; the
// receipts of each tick are still resolved in tick order per node.
//
// Pipeline of one window:
//   units     fires per (fine bucket f, tick k), bucket-major; hipcub scan ->
//             firing index
//   groupmap  first unit of every 64-node group of firing indices
//   expand    one thread per firing node (Node.Broadcast, :141-147): row read
//             once, keyed RandomDrop per slot (one Philox per 4 slots), kept
//             targets counting-sorted in LDS by coarse bucket (target >> 22)
//             and written as coalesced runs into coarse regions sized from
//             the node share (+ margin); message = u_in_coarse | k << 22
//   plan      fine-bucket regions (16384 nodes) inside each coarse region,
//             sized from the coarse count (+ margin)
//   part2     one pass per coarse tile: LDS counting sort by fine digit,
//             coalesced runs into fine regions; message = u_in_fine | k << 14
//   resolve   one workgroup per fine bucket: received/crashed bits and u16
//             arrival counters in LDS; per tick, count then let one owner lane
//             per node replay ordinals 0..count-1 of the receive case
//             (:107-123); infections append to the fire list (slot, f) that
//             only this workgroup writes
// A region that overflows its estimated size is detected and the window's
// partition is redone with exact counts (expand and part2 are idempotent).
// Fire lists: fcount[R][nfine] + flist[R][nfine][16384] (u16 local ids).
#include <hipcub/hipcub.hpp>

#include <cstdlib>

#include "gossip.h"
#include "gs_internal.h"

namespace gs {
namespace {

constexpr uint32_t kExpandBlock = 256;
constexpr uint32_t kExpandNpt = 4;        // firing nodes per thread per round (rows <= 8)
constexpr uint32_t kResolveBlock = 512;
#ifndef GS_RESOLVE_WAVES
#define GS_RESOLVE_WAVES 4  // min waves per SIMD: two 512-thread workgroups per CU
#endif
// Messages: coarse = u_in_coarse | k << 22 | roll0 << 26; fine = loc | k << 14 |
// roll0 << 18, where roll0 is the receiver's crash roll for ordinal 0.
constexpr uint32_t kRoll0Coarse = kCoarseShift + 4;
constexpr uint32_t kRoll0Fine = kFineLog + 4;

// Device-driven windows (w.ctl set): the window being opened starts at
// ctl->tnext and may hold up to Lw ticks (none once the run has stopped, a
// partition overflowed -- the host then redoes that window -- or tend is
// reached; never past the next poll).  0 = nothing to do.
// Error bits that stop a window: an overflow (the host redoes the window), or
// in device-driven shard windows only kErrAbort (k_rtab: some shard's window
// overflowed; a fine overflow is re-partitioned in the window itself) --
// except a single in-process shard (w.solo), which stops on any overflow as
// the unsharded engine does.
__device__ __forceinline__ uint32_t stop_bits(const WinState& w) {
  return w.dd && !w.solo ? kErrAbort : (kErrCoarse | kErrFine | kErrAbort);
}
__device__ __forceinline__ bool win_abort(const WinState& w) {
  return (*w.err & stop_bits(w)) != 0;
}
// The window control block's first 32 bytes (t, L, tnext, tend, poll, pbase,
// stop, lmax) and the error word, all loaded before any is tested: a kernel
// of a window pays one load latency for them, not a chain of dependent ones.
struct CtlView {
  uint32_t t, L, tnext, tend, poll, pbase, stop, lmax, err;
};
__device__ __forceinline__ CtlView ctl_view(const WinState& w) {
  static_assert(offsetof(WinCtl, t) == 0 && offsetof(WinCtl, lmax) == 28, "WinCtl's first 32 bytes");
  const uint4* p = reinterpret_cast<const uint4*>(w.ctl);
  const uint4 a = p[0], b = p[1];
  const uint32_t e = *w.err;
  return CtlView{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, e};
}
// (The tests are selects, not early returns: a branch on the error word would
// let the compiler sink the control-block load behind it, two latencies.)
__device__ __forceinline__ uint32_t win_open(const WinState& w, uint32_t& t) {
  const CtlView c = ctl_view(w);
  t = c.tnext;
  const bool dead = (c.err & stop_bits(w)) || c.stop || t >= c.tend;
  uint32_t Lw = min(c.lmax, c.tend - t);
  if (c.poll) {
    const uint32_t P = c.pbase + c.poll * ((t - c.pbase + c.poll - 1) / c.poll);  // next poll tick
    Lw = min(Lw, P - t + 1);
  }
  return dead ? 0u : Lw;
}
// A kernel of an opened window: its start and length (0: skip the window).
__device__ __forceinline__ uint32_t win_live(const WinState& w, uint32_t& t0, uint32_t L) {
  if (!w.ctl) return w.abort_on_err && win_abort(w) ? 0u : L;  // shards: a window that overflowed is redone
  const CtlView c = ctl_view(w);
  t0 = c.t;
  // a guarded launch (the exact fine re-partition) runs only after an overflow
  const bool off = (c.err & stop_bits(w)) || (w.guard && !(c.err & kErrFine));
  return off ? 0u : c.L;
}

__device__ __forceinline__ uint32_t wave_sum32(uint32_t v) {
#pragma unroll
  for (uint32_t o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Exclusive scan of one u64 per thread over a 256-thread block (s: 4 words
// of LDS); returns the thread's prefix, *total the block's sum.  Block-uniform.
__device__ __forceinline__ unsigned long long block_exscan256_u64(unsigned long long v, unsigned long long* s,
                                                                   unsigned long long* total) {
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  unsigned long long x = v;
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s[wv] = x;
  __syncthreads();
  unsigned long long before = 0, all = 0;
#pragma unroll
  for (uint32_t q = 0; q < 4; ++q) {
    const unsigned long long t = s[q];
    if (q < wv) before += t;
    all += t;
  }
  __syncthreads();
  *total = all;
  return before + x - v;
}

// Units = (fine bucket f, tick k), bucket-major (u = f*Ls + k, Ls = the layout
// stride: L, or lmax for device-driven windows): the L fire lists of one
// bucket are expanded back to back, so friends-row lines that several ticks of
// the window share are fetched once into the XCD's L2.  usize = fires;
// tfires[k] = fires per tick (the window cut).  Also zeroes the window's
// counters (one launch instead of several memsets).
__device__ __forceinline__ void units_body(const WinState& w, uint32_t t0, uint32_t L) {
  __shared__ uint32_t s_t[kMaxWindow];
  uint32_t Ls = L;
  if (w.ctl) {
    L = win_open(w, t0);
    if (!L) return;
    Ls = w.lstride;
  }
  const uint32_t units = Ls * w.nfine;
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x, nth = gridDim.x * blockDim.x;
  // 256-bucket tiles: the L fcount rows are read coalesced (bucket fastest),
  // transposed in LDS and written bucket-major, coalesced.
  __shared__ uint32_t s_tile[256 * (kMaxWindow + 1)];
  uint32_t acc[kMaxWindow];
#pragma unroll
  for (uint32_t k = 0; k < kMaxWindow; ++k) acc[k] = 0;
  if (threadIdx.x < kMaxWindow) s_t[threadIdx.x] = 0;
  if (tid == 0) w.usize[units] = 0;
  __syncthreads();
  __shared__ uint32_t s_ts[kMaxWindow];  // this tile's fires per tick
  uint32_t slot[kMaxWindow];  // ring slot of tick t0 + k (uniform)
#pragma unroll
  for (uint32_t k = 0; k < kMaxWindow; ++k) slot[k] = k < L ? (t0 + k) % w.R : 0u;
  for (uint32_t f0 = blockIdx.x * 256; f0 < w.nfine; f0 += gridDim.x * 256) {
    const uint32_t f = f0 + threadIdx.x;
    if (threadIdx.x < kMaxWindow) s_ts[threadIdx.x] = 0;
    // all L loads in flight before the first use (one latency, not L)
    uint32_t cv[kMaxWindow];
#pragma unroll
    for (uint32_t k = 0; k < kMaxWindow; ++k)
      cv[k] = k < L && k < Ls && f < w.nfine ? w.fcount[(size_t)slot[k] * w.nfine + f] : 0u;
#pragma unroll
    for (uint32_t k = 0; k < kMaxWindow; ++k) {
      if (k < Ls) {
        s_tile[threadIdx.x * (kMaxWindow + 1) + k] = cv[k];
        acc[k] += cv[k];
      }
    }
    __syncthreads();
    // per-tile sums for the device-driven unit scan (k_cut, k_unitscan)
#pragma unroll
    for (uint32_t k = 0; k < kMaxWindow; ++k) {
      if (k < Ls) {
        const uint32_t c = wave_sum32(s_tile[threadIdx.x * (kMaxWindow + 1) + k]);
        if ((threadIdx.x & 63) == 0 && c) atomicAdd(&s_ts[k], c);
      }
    }
    __syncthreads();
    if (threadIdx.x < Ls) w.tsum[(size_t)(f0 >> 8) * kMaxWindow + threadIdx.x] = s_ts[threadIdx.x];
    const uint32_t nb = min(256u, w.nfine - f0), base = f0 * Ls;
    for (uint32_t i = threadIdx.x; i < nb * Ls; i += 256) {
      const uint32_t b = i / Ls, k = i - b * Ls;
      w.usize[base + i] = s_tile[b * (kMaxWindow + 1) + k];
    }
    __syncthreads();
  }
#pragma unroll
  for (uint32_t k = 0; k < kMaxWindow; ++k)
    if (acc[k]) atomicAdd(&s_t[k], acc[k]);
  __syncthreads();
  if (threadIdx.x < L && s_t[threadIdx.x]) atomicAdd(&w.tfires[threadIdx.x], (unsigned long long)s_t[threadIdx.x]);
  for (uint32_t i = tid; i < kRegions; i += nth) { w.chist[i] = 0; w.cfill[i] = 0; }
  for (uint32_t i = tid; i < w.nfine; i += nth) w.ffill[i] = 0;
  if (w.dd && tid == 0) {  // this shard's gathered row: flag word, buffer capacities
    w.cfill[kRegions] = 0;
    w.cfill[kRegions + 1] = w.ctl->fmsg_cap;
    w.cfill[kRegions + 2] = w.ctl->xs_cap;
    w.cfill[kRegions + 3] = w.ctl->xr_cap;
  }
  // host-driven windows clear the overflow flags here; device-driven and shard
  // windows keep them until the host has redone the window
  if (tid == 0 && !w.ctl && !w.abort_on_err) *w.err &= ~(kErrCoarse | kErrFine);
}
__global__ __launch_bounds__(256) void k_units(const WinState w, uint32_t t0, uint32_t L) { units_body(w, t0, L); }

// The device-driven shard windows of an in-process group launch each small
// per-shard kernel once for all M shards: shard blockIdx.y (or blockIdx.x for
// the one-block kernels) reads its window state from a device array.
__global__ __launch_bounds__(256) void k_units_m(const WinState* __restrict__ ws, uint32_t t0, uint32_t L) {
  units_body(ws[blockIdx.y], t0, L);
}

// Device-driven windows: the cut (as the host-driven engine makes it: a
// window holds whole ticks while its friend slots fit `budget`), the coarse
// region plan of the window's T friend slots, and the window's place in ctl.
// One block.
__device__ __forceinline__ void cut_body(const WinState& w, unsigned long long budget) {
  __shared__ unsigned long long s_sz[256];
  __shared__ unsigned long long s_T;
  __shared__ uint32_t s_go, s_L;
  WinCtl* c = w.ctl;
  const uint32_t b = threadIdx.x;  // 256 threads: thread b plans coarse bin b
  __shared__ unsigned long long s_tf[kMaxWindow];
  if (win_abort(w)) return;  // keep ctl: the host redoes the failed window
  uint32_t t = 0;
  const uint32_t Lw = win_open(w, t);
  // every load this kernel needs is issued up front (one latency, not a chain)
  const unsigned long long cap = c->cmsg_cap;
  __shared__ unsigned long long s_own[kMaxWindow];  // device-driven shards: this shard's fires per tick
  if (b < kMaxWindow) {
    if (w.dd) {  // the cut from every shard's gathered counts: the same window on every shard
      unsigned long long g = 0;
      for (uint32_t r = 0; r < w.G; ++r) g += w.gcnt[(size_t)r * kMaxWindow + b];
      s_tf[b] = g;
      s_own[b] = w.tfires[b];
    } else {
      s_tf[b] = w.tfires[b];
    }
  }
  unsigned long long ts[4][kMaxWindow];  // this thread's tiles' fires per tick
#pragma unroll
  for (uint32_t j = 0; j < 4; ++j)
#pragma unroll
    for (uint32_t k = 0; k < kMaxWindow; ++k)
      ts[j][k] = Lw && b * 4 + j < w.ncoarse ? w.tsum[(size_t)(b * 4 + j) * kMaxWindow + k] : 0ull;
  __syncthreads();
  if (b == 0) {
    s_go = Lw != 0;
    if (!Lw) {  // stopped or past tend: the rest of this window does nothing
      c->L = 0;
      c->Tn = 0;
    } else {
      uint32_t L = 1;
      unsigned long long Tn = s_tf[0];
      while (L < Lw && (Tn + s_tf[L]) * w.stride <= budget) Tn += s_tf[L++];
      if (w.dd) {  // this shard's own fires (its row is zeroed by k_unitscan, after every shard's cut)
        Tn = 0;
        for (uint32_t k = 0; k < L; ++k) Tn += s_own[k];
      } else {
        for (uint32_t k = 0; k < kMaxWindow; ++k) w.tfires[k] = 0;
      }
      c->t = t;
      c->L = L;
      s_L = L;
      c->tnext = t + L;
      c->Tn = Tn;
      // owner expand (shards): the plan of gs_api.cpp's plan_coarse_owner over
      // the longest row; unsharded: over the stride
      c->T = Tn * (w.owner ? w.slots : w.stride);
      s_T = c->T;
    }
  }
  __syncthreads();
  if (!s_go) return;
  {
    // firing index of each 256-bucket tile's first unit (ticks >= L count as
    // empty): k_unitscan finishes the scan inside the tiles (ncoarse <= 1024)
    const uint32_t L = s_L, nt = w.ncoarse;
    unsigned long long v[4], sum = 0;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
      v[j] = 0;
#pragma unroll
      for (uint32_t k = 0; k < kMaxWindow; ++k) v[j] += k < L ? ts[j][k] : 0ull;
      sum += v[j];
    }
    unsigned long long tot;
    unsigned long long pre = block_exscan256_u64(sum, &s_sz[0], &tot);
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
      const uint32_t tile = b * 4 + j;
      if (tile < nt) w.toff[tile] = pre;
      pre += v[j];
    }
    if (b == 0) w.toff[nt] = tot;
    __syncthreads();
  }
  // coarse regions: each sub-region gets 1/8 of its bin's node share of T,
  // plus 512 (plan_coarse on the host)
  unsigned long long sub = 0;
  if (!w.owner) {
    const unsigned long long lo = (unsigned long long)b << kCoarseShift;
    const unsigned long long hi = min((unsigned long long)w.n, lo + (1ull << kCoarseShift));
    const double xr = (double)kXRoundNodes * w.stride;  // one expand round's slots (kXRoundNodes)
    sub = b < w.ncoarse
              ? (unsigned long long)(((double)s_T / kCoarseSub + xr) * (double)(hi - lo) / (double)w.n) + 512
              : 0ull;
  } else {  // bin b = owner d * obins + 2^22-node chunk of d's range (plan_coarse_owner)
    const uint32_t d = b / w.obins, k = b % w.obins;
    unsigned long long cnt = 0;
    if (d < w.G) {
      const unsigned long long dlo = (unsigned long long)d * w.seg_per;
      const unsigned long long dhi = min(dlo + w.seg_per, (unsigned long long)w.nglob);
      const unsigned long long lo = dlo + ((unsigned long long)k << kCoarseShift);
      const unsigned long long hi = min(dhi, lo + (1ull << kCoarseShift));
      cnt = hi > lo ? hi - lo : 0ull;
    }
    const double xr = (double)kXRoundNodes * w.slots;
    sub = cnt ? (unsigned long long)(((double)s_T / kCoarseSub + xr) * (double)cnt / (double)w.nglob) + 512 : 0ull;
  }
  unsigned long long total;
  const unsigned long long base = block_exscan256_u64(sub * kCoarseSub, &s_sz[0], &total);
  if (total > cap) {  // the buffer is too small: no region at all, the host grows and redoes
    for (uint32_t x = 0; x < kCoarseSub; ++x) w.ccap[b * kCoarseSub + x] = 0;
    if (b == 0) {
      w.ccap[kRegions] = 0;
      atomicOr(w.err, kErrCoarse);
      if (w.dd) atomicOr(reinterpret_cast<unsigned int*>(&w.cfill[kRegions]), kErrCoarse);  // every shard stops
    }
    return;
  }
  for (uint32_t x = 0; x < kCoarseSub; ++x) w.ccap[b * kCoarseSub + x] = base + x * sub;
  if (b == 255) w.ccap[kRegions] = total;
}
__global__ __launch_bounds__(256) void k_cut(const WinState w, unsigned long long budget) { cut_body(w, budget); }
__global__ __launch_bounds__(256) void k_cut_m(const WinState* __restrict__ ws, unsigned long long budget) {
  cut_body(ws[blockIdx.x], budget);
}

// Device-driven windows: the unit scan inside each 256-bucket tile (thread =
// bucket, its Ls units contiguous; ticks >= L count as empty), offset by the
// tile's start from k_cut, and the group map of those units.  One block per
// tile.  (Host-driven windows: hipcub scan + k_groupmap.)
__device__ __forceinline__ void unitscan_body(const WinState& w) {
  __shared__ unsigned long long s_x[4];
  if (blockIdx.x >= w.ncoarse) return;  // shards of a group: the grid covers the largest
  uint32_t t0;
  const uint32_t L = win_live(w, t0, 0);
  if (!L) return;
  const uint32_t Ls = w.lstride, tile = blockIdx.x, f = tile * 256 + threadIdx.x;
  // device-driven shards: every shard's cut has read this shard's gathered
  // counts; its row restarts at 0 for the next window's k_units
  if (w.dd && tile == 0 && threadIdx.x < kMaxWindow) w.tfires[threadIdx.x] = 0;
  unsigned long long sz[kMaxWindow], sum = 0;
#pragma unroll
  for (uint32_t k = 0; k < kMaxWindow; ++k)  // all loads in flight, then the sum
    sz[k] = k < L && f < w.nfine ? w.usize[(size_t)f * Ls + k] : 0ull;
#pragma unroll
  for (uint32_t k = 0; k < kMaxWindow; ++k) sum += sz[k];
  unsigned long long tot;
  unsigned long long a = w.toff[tile] + block_exscan256_u64(sum, s_x, &tot);
  if (f >= w.nfine) return;
#pragma unroll
  for (uint32_t k = 0; k < kMaxWindow; ++k) {
    if (k >= Ls) break;
    const uint32_t u = f * Ls + k;
    w.unit_off[u] = a;
    const unsigned long long b = a + sz[k];
    for (unsigned long long q = (a + 63) >> 6; (q << 6) < b; ++q) w.gmap[q] = u;
    a = b;
  }
  if (f == w.nfine - 1) w.unit_off[(size_t)w.nfine * Ls] = a;
}
__global__ __launch_bounds__(256) void k_unitscan(const WinState w) { unitscan_body(w); }
__global__ __launch_bounds__(256) void k_unitscan_m(const WinState* __restrict__ ws) { unitscan_body(ws[blockIdx.y]); }

// gmap[q] = unit holding firing index 64*q.
__global__ void k_groupmap(const WinState w, uint32_t L) {
  if (w.ctl) {
    uint32_t t0;
    if (!win_live(w, t0, 0)) return;
    L = w.lstride;
  }
  const uint32_t units = L * w.nfine;
  for (uint32_t u = blockIdx.x * blockDim.x + threadIdx.x; u < units; u += gridDim.x * blockDim.x) {
    const unsigned long long a = w.unit_off[u], b = w.unit_off[u + 1];
    for (unsigned long long q = (a + 63) >> 6; (q << 6) < b; ++q) w.gmap[q] = u;
  }
}

// Unit of firing index g (gmap[q] = unit holding firing index 64*q) for a
// wave whose 64 lanes hold the 64 consecutive firing indices of group g0 / 64
// (g0 wave-uniform): the group's unit bounds are two scalar loads, and only a
// group that spans several units searches [gmap[q], gmap[q + 1]] per lane.
__device__ __forceinline__ uint32_t unit_of_wave(const WinState& w, unsigned long long g0, unsigned long long g,
                                                 unsigned long long Tn, uint32_t units) {
  const unsigned long long q = g0 >> 6;
  uint32_t lo = w.gmap[q];
  uint32_t hi = ((q + 1) << 6) < Tn ? w.gmap[q + 1] : units - 1;
  if (lo == hi) return lo;
  while (lo < hi) {
    const uint32_t mid = (lo + hi + 1) >> 1;
    if (w.unit_off[mid] <= g) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// Per-tick counters are added into one of kStatShards copies (by workgroup)
// and summed into the stats ring by k_stats_reduce / k_close: thousands of
// workgroups adding into the same few lines would serialise at the
// memory-side atomic unit (32 copies take a dense window's few hundred
// thousand adds at well under one per microsecond per address).
__device__ __forceinline__ unsigned long long* shard_row(const WinState& w, uint32_t k) {
  return w.sstats + ((size_t)(blockIdx.x & (kStatShards - 1)) * kMaxWindow + k) * kStatFields;
}

// GS_XSTAMPS builds (diagnostics, GS_STAMPS=1 at run time): wave 0 of every
// k_expand workgroup waits for everything it issued and adds the cycles since
// its last stamp to phase i (w.dbg[kXStamp0 + i]; i = 0 counts rounds).
#ifdef GS_XSTAMPS
__device__ __forceinline__ void xstamp(const WinState& w, unsigned long long& last, uint32_t i) {
  if (w.dbg && threadIdx.x < 64) {
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0 && i) atomicAdd(&w.dbg[kXStamp0 + i], t - last);
    if (threadIdx.x == 0 && i == 1) atomicAdd(&w.dbg[kXStamp0], 1ull);
    last = t;
  }
}
#define XSTAMP(i) xstamp(w, xlast, i)
#else
#define XSTAMP(i) ((void)0)
#endif

// Device-driven windows: the window's per-tick counters (stats ring, and
// staging slot `slot` for the host with the window's snapshot), the poll
// rule's running state and, at a poll tick, gs_run's stop rule
// (simulator.go:243-248: covered at float32 99 %; the engine also stops when
// nothing is pending or max_ticks has passed).  One block of 128 threads.
// Sum of stat shard field `i` (= tick * kStatFields + field) over the
// kStatShards copies, leaving them zeroed: lane group of kCloseLanes lanes
// per field, each lane kStatShards / kCloseLanes shards with all its loads
// in flight together.
constexpr uint32_t kCloseLanes = 8;
__device__ __forceinline__ unsigned long long stat_shard_sum(const WinState& w, uint32_t i, uint32_t part) {
  constexpr uint32_t kPer = kStatShards / kCloseLanes;
  unsigned long long x[kPer], sum = 0;
#pragma unroll
  for (uint32_t j = 0; j < kPer; ++j) x[j] = w.sstats[(size_t)(j * kCloseLanes + part) * kMaxWindow * kStatFields + i];
#pragma unroll
  for (uint32_t j = 0; j < kPer; ++j) {
    sum += x[j];
    if (x[j]) w.sstats[(size_t)(j * kCloseLanes + part) * kMaxWindow * kStatFields + i] = 0;
  }
#pragma unroll
  for (uint32_t o = 1; o < kCloseLanes; o <<= 1) sum += __shfl_xor(sum, o, 64);
  return sum;
}

__global__ void k_stats_reduce(const WinState w, uint32_t t0, uint32_t L) {  // as k_close's block
  if (w.abort_on_err && win_abort(w)) return;  // the redo of the window reduces them
  const uint32_t i = threadIdx.x / kCloseLanes, part = threadIdx.x % kCloseLanes;
  const uint32_t k = i / kStatFields, fld = i % kStatFields;
  if (k >= L) return;
  const unsigned long long sum = stat_shard_sum(w, i, part);
  if (part == 0 && sum) w.stats[(size_t)((t0 + k) % kStatSlots) * kStatFields + fld] += sum;
}

__global__ void k_close(const WinState w, uint32_t slot) {  // kMaxWindow * kStatFields * kCloseLanes threads
  __shared__ unsigned long long rows[kMaxWindow][kStatFields];
  WinCtl* c = w.ctl;
  unsigned long long* st = w.stage + (size_t)slot * kStageWords;
  uint32_t t0 = 0;
  const uint32_t L = win_live(w, t0, 0);
  const uint32_t i = threadIdx.x / kCloseLanes, part = threadIdx.x % kCloseLanes, tid = threadIdx.x;
  const uint32_t k = i / kStatFields, fld = i % kStatFields;
  if (k < L) {  // k is uniform over each lane group
    const unsigned long long sum = stat_shard_sum(w, i, part);
    if (part == 0) {
      rows[k][fld] = sum;
      w.stats[(size_t)((t0 + k) % kStatSlots) * kStatFields + fld] = sum;
      st[8 + k * kStatFields + fld] = sum;
    }
  }
  __syncthreads();
  if (tid != 0) return;
  uint32_t stop = c->stop;
  if (L) {
    for (uint32_t j = 0; j < L; ++j) {
      c->recv += rows[j][ST_RECV];
      c->crashed += rows[j][ST_CRASH];
      c->pending += rows[j][ST_SCHED] - rows[j][ST_FIRED];
    }
    const uint32_t tl = t0 + L - 1;  // windows never cross a poll tick
    if (c->poll && (tl - c->pbase) % c->poll == 0 && !stop) {
      if (c->recv >= c->cover) stop = 1 + GS_RUN_COVERED;
      else if (c->pending == 0) stop = 1 + GS_RUN_QUIESCENT;
      else if (tl >= c->max_ticks) stop = 1 + GS_RUN_MAX_TICKS;
      c->stop = stop;
    }
  }
  st[0] = t0;
  st[1] = L;
  st[2] = stop;
  st[3] = *w.err;
  st[4] = L ? c->Tn : 0;
}

template <uint32_t SLOTS>  // LDS message slots per round: block * nodes per thread * row length
struct ExpandLds {
  uint32_t sorted[SLOTS];
  uint8_t sbin[SLOTS];
  uint32_t cnt[256];
  uint32_t off[257];
  unsigned long long gbase[256];          // bin b's message p goes to gbase[b] + p
  unsigned long long cend[256];           // end of coarse region b (ccap[b + 1])
  uint32_t ovf;                           // a bin of this round overflowed its region
  unsigned long long acc[kMaxWindow][2];  // fired, sent per tick
};

__device__ __forceinline__ void block_scan256(uint32_t* cnt, uint32_t* off) {
  // exclusive scan of 256 counters by the first wave (4 per lane)
  if (threadIdx.x < 64) {
    const uint32_t l = threadIdx.x;
    const uint32_t a = cnt[4 * l], b = cnt[4 * l + 1], c = cnt[4 * l + 2], d = cnt[4 * l + 3];
    const uint32_t sum = a + b + c + d;
    uint32_t x = sum;
#pragma unroll
    for (uint32_t o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if (l >= o) x += y;
    }
    const uint32_t ex = x - sum;
    off[4 * l] = ex;
    off[4 * l + 1] = ex + a;
    off[4 * l + 2] = ex + a + b;
    off[4 * l + 3] = ex + a + b + c;
    if (l == 63) off[256] = x;
  }
}

// Batched trials: add (a, b) to fields (fa, fb) of row `key` of tstat
// (key = trial * kMaxWindow + tick, ~0u = nothing), one atomic pair per
// distinct key in the wave.  The wave's lanes usually share one key (firing
// indices are bucket-major, and a bucket belongs to one trial).
__device__ __forceinline__ void tstat_add(uint32_t* tstat, uint32_t key, uint32_t fa, uint32_t a,
                                          uint32_t fb, uint32_t b) {
  bool pend = key != ~0u;
  for (unsigned long long bal = __ballot(pend); bal; bal = __ballot(pend)) {
    const uint32_t lead = (uint32_t)__builtin_ctzll(bal);
    const uint32_t k0 = __shfl(key, lead, 64);
    const bool mine = pend && key == k0;
    const uint32_t sa = wave_sum32(mine ? a : 0u), sb = wave_sum32(mine ? b : 0u);
    if ((threadIdx.x & 63) == lead) {
      if (sa) atomicAdd(&tstat[(size_t)k0 * kTStatFields + fa], sa);
      if (sb) atomicAdd(&tstat[(size_t)k0 * kTStatFields + fb], sb);
    }
    pend = pend && !mine;
  }
}

// Packed view (rows <= 6 slots, stride 8): row v is the 24 bytes at byte
// 24 * (v mod 5) of 128-B line v / 5 (8 bytes of each line unused), so a
// line holds five rows instead of four and no row straddles two lines.
__device__ __forceinline__ uint64_t pk_byte(uint32_t v) {
  const uint32_t line = (uint32_t)(((uint64_t)v * 0xCCCCCCCDull) >> 34);  // v / 5 for every 32-bit v
  return (uint64_t)line * 128 + (v - line * 5) * 24;
}

// The packed view's rows of NPT nodes per lane, fetched by LANE PAIRS: lanes
// 2p and 2p+1 load the 32 bytes from the 16-B aligned base of lane 2p's row
// (one uint4 each: both halves of one 128-B line in one instruction, so one
// L2 request per row instead of two), then those of lane 2p+1's row, and swap
// halves with a DPP move.  A random 24-B row costs two requests fetched per
// lane (uint4 + uint2); by pairs the gather ran 1.87x faster
// (scripts/micro/uncached_gather.hip: 4.84e10 vs 2.58e10 rows/s,
// profiles/r05p_gather_pairs.txt).  Every lane of a wave takes part (a lane
// without a node fetches line 0 and drops it), so the call must not sit in
// lane-divergent code; a wave with no node at all skips the fetch uniformly.
__device__ __forceinline__ uint32_t dpp_swap_pair(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
}
template <uint32_t MAXS>
__device__ __forceinline__ void decode_pk_row(uint4 x, uint4 y, bool o8, uint32_t (&mm)[MAXS]) {
  mm[0] = o8 ? x.z : x.x;
  mm[1] = o8 ? x.w : x.y;
  mm[2] = o8 ? y.x : x.z;
  mm[3] = o8 ? y.y : x.w;
  mm[4 % MAXS] = o8 ? y.z : y.x;
  if (MAXS > 5) mm[5 % MAXS] = o8 ? y.w : y.y;
}
template <uint32_t MAXS, uint32_t NPT>
__device__ __forceinline__ void load_rows_pk_pairs(const WinState& w, const uint32_t (&vv)[NPT], const bool (&wlive)[NPT],
                                                   uint32_t (&mm)[NPT][MAXS]) {
  const uint32_t odd = threadIdx.x & 1;
  const uint4* pk = reinterpret_cast<const uint4*>(w.pk);
  uint4 s0[NPT], s1[NPT];
  uint32_t o8[NPT];
#pragma unroll
  for (uint32_t q = 0; q < NPT; ++q) {
    if (!wlive[q]) continue;  // (wave-uniform)
    const uint64_t b = vv[q] != ~0u ? pk_byte(vv[q]) : 0ull;
    o8[q] = (uint32_t)b & 8u;
    const uint32_t mine = (uint32_t)(b >> 4), other = dpp_swap_pair(mine);  // uint4 index of the base
    const uint32_t ev = odd ? other : mine, od = odd ? mine : other;
    s0[q] = pk[(size_t)ev + odd];  // the pair's even row, half `odd`
    s1[q] = pk[(size_t)od + odd];  // the pair's odd row, half `odd`
  }
#pragma unroll
  for (uint32_t q = 0; q < NPT; ++q) {
    if (!wlive[q]) continue;
    // the even lane holds its half 0 (s0) and the odd lane's half 0 (s1); the
    // odd lane the even lane's half 1 (s0) and its own half 1 (s1)
    const uint4 send = odd ? s0[q] : s1[q];
    uint4 got;
    got.x = dpp_swap_pair(send.x);
    got.y = dpp_swap_pair(send.y);
    got.z = dpp_swap_pair(send.z);
    got.w = dpp_swap_pair(send.w);
    if (vv[q] != ~0u) decode_pk_row<MAXS>(odd ? got : s0[q], odd ? s1[q] : got, o8[q] != 0, mm[q]);
  }
}

// Friends row of v into registers; slots past the list hold kEmptyMsg (rows
// are sealed by k_seal_rows, so the length byte is not read).
template <uint32_t MAXS>
__device__ __forceinline__ void load_row(const WinState& w, uint32_t v, uint32_t (&mm)[MAXS]) {
  const uint32_t S = w.stride;
  if (MAXS >= 5 && MAXS <= 6 && w.pk) {  // two 16-B loads from the row's 16-B aligned base
    const uint64_t b = pk_byte(v);
    const uint4* p = reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(w.pk) + (b & ~15ull));
    decode_pk_row<MAXS>(p[0], p[1], (b & 8) != 0, mm);  // (the row starts 8 bytes into the first load)
    return;
  }
  if ((S & 3) == 0 && S >= 8 && MAXS >= 5 && MAXS <= 8) {  // 16-B aligned rows: uint4 + uint2 / uint4
    const uint4 a = reinterpret_cast<const uint4*>(w.ids + (size_t)v * S)[0];
    mm[0] = a.x; mm[1] = a.y; mm[2] = a.z; mm[3] = a.w;
    if (MAXS > 4 && MAXS <= 6) {
      const uint2 b = reinterpret_cast<const uint2*>(w.ids + (size_t)v * S)[2];
      mm[4 % MAXS] = b.x;
      if (MAXS > 5) mm[5 % MAXS] = b.y;
    } else if (MAXS > 6) {
      const uint4 b = reinterpret_cast<const uint4*>(w.ids + (size_t)v * S)[1];
      mm[4 % MAXS] = b.x; mm[5 % MAXS] = b.y; mm[6 % MAXS] = b.z; mm[7 % MAXS] = b.w;
    }
  } else if ((S & 3) == 0 && MAXS > 8) {  // 16-B aligned longer rows: uint4 loads
    const uint4* row = reinterpret_cast<const uint4*>(w.ids + (size_t)v * S);
#pragma unroll
    for (uint32_t j = 0; j < MAXS; j += 4) {
      const uint4 x = j < S ? row[j / 4] : make_uint4(kEmptyMsg, kEmptyMsg, kEmptyMsg, kEmptyMsg);
      mm[j] = x.x;
      if (j + 1 < MAXS) mm[j + 1] = x.y;
      if (j + 2 < MAXS) mm[j + 2] = x.z;
      if (j + 3 < MAXS) mm[j + 3] = x.w;
    }
  } else if ((S & 1) == 0) {
    const uint2* row = reinterpret_cast<const uint2*>(w.ids + (size_t)v * S);
#pragma unroll
    for (uint32_t j = 0; j < MAXS; j += 2) {
      const uint2 x = 2 * j < 2 * S ? row[j / 2] : make_uint2(kEmptyMsg, kEmptyMsg);
      mm[j] = x.x;
      if (j + 1 < MAXS) mm[j + 1] = x.y;
    }
  } else {
    const uint32_t* row = w.ids + (size_t)v * S;
#pragma unroll
    for (uint32_t j = 0; j < MAXS; ++j) mm[j] = j < S ? row[j] : kEmptyMsg;
  }
}

// Coarse bin of target `t`; t becomes its index inside the bin.  Unsharded:
// bin = t >> 22.  Owner expand (node-range shards): the target's owner d (the
// shard whose range holds it: q = t >> 14 over seg_per >> 14, oseg_magic =
// floor((2^32 - 1) / oseg_q) never overestimates and is at most one below)
// and the 2^22-node chunk of d's range.
__device__ __forceinline__ uint32_t coarse_bin(const WinState& w, uint32_t& t) {
  if (!w.owner) {
    const uint32_t b = t >> kCoarseShift;
    t &= (1u << kCoarseShift) - 1;
    return b;
  }
  const uint32_t q = t >> kFineLog;
  uint32_t d = __umulhi(q, w.oseg_magic);
  if ((d + 1) * w.oseg_q <= q) ++d;
  const uint32_t off = t - d * w.seg_per;
  t = off & ((1u << kCoarseShift) - 1);
  return d * w.obins + (off >> kCoarseShift);
}

// Expand + coarse partition (Node.Broadcast, simulator.go:141-147).  Each
// thread takes NPT firing nodes per round; their rows are all in flight before
// any is used.  Kept targets are counting-sorted in LDS by coarse bucket and
// leave as coalesced runs, one global reservation per (round, bucket).
// WRITE=false only counts (exact fallback).
// XCD-aware round split: workgroups are dealt to the 8 XCDs round-robin
// (XCD = blockIdx & 7), so with a grid that is a multiple of 8 each XCD takes
// one contiguous eighth of the rounds, shared among its B/8 workgroups --
// fire lists of one bucket share friends-row lines in that XCD's L2, and the
// coarse sub-region (bin, blockIdx & 7) a workgroup writes receives an equal
// share of the window whatever the round count (a sparse window on a large
// fixed grid must not pile onto XCD 0).  Other grids: plain grid stride.
__device__ __forceinline__ void xcd_rounds(unsigned long long rounds, unsigned long long& beg,
                                           unsigned long long& end, unsigned long long& step) {
  const uint32_t B = gridDim.x;
  if ((B & 7) == 0) {
    const unsigned long long per = (rounds + 7) >> 3, x = blockIdx.x & 7;
    beg = x * per + (blockIdx.x >> 3);
    end = (x + 1) * per < rounds ? (x + 1) * per : rounds;
    step = B >> 3;
  } else {
    beg = blockIdx.x;
    end = rounds;
    step = B;
  }
}

template <bool WRITE, uint32_t MAXS, uint32_t NPT, uint32_t B>
__device__ __forceinline__ void expand_body(const WinState& w, uint32_t t0, uint32_t L, unsigned long long Tn,
                                            int add_stats) {
  __shared__ ExpandLds<B * NPT * MAXS> sm;
  const uint32_t tid = threadIdx.x;
  uint32_t Ls = L;  // unit layout stride
  if (w.ctl) {
    L = win_live(w, t0, 0);
    if (!L) return;
    Tn = w.ctl->Tn;
    Ls = w.lstride;
  }
  const uint32_t units = Ls * w.nfine;
  constexpr uint32_t per_round = B * NPT;
  if (tid < kMaxWindow * 2) (&sm.acc[0][0])[tid] = 0;
  static_assert(B % 256 == 0, "thread b < 256 owns coarse bin b");
  const bool binner = tid < 256;
  const uint32_t reg = (tid & 255) * kCoarseSub + (blockIdx.x & (kCoarseSub - 1));  // bin tid, this XCD's sub-region
  const unsigned long long cbase = w.ccap[reg], cend = w.ccap[reg + 1];
  if (binner) sm.cend[tid] = cend;
  const unsigned long long rounds = (Tn + per_round - 1) / per_round;
  unsigned long long rbeg, rend, rstep;
  xcd_rounds(rounds, rbeg, rend, rstep);
  // per-tick fired | sent << 16 of this thread's nodes (<= 1024 rounds per
  // workgroup, win_expand): registers, not same-address LDS atomics per node
  uint32_t accp[kBitTicks];
#pragma unroll
  for (uint32_t kx = 0; kx < kBitTicks; ++kx) accp[kx] = 0;
#ifdef GS_XSTAMPS
  unsigned long long xlast = 0;
  XSTAMP(0);
#endif
  for (unsigned long long rd = rbeg; rd < rend; rd += rstep) {
    if (binner) sm.cnt[tid] = 0;
    __syncthreads();
    if (tid == 0) sm.ovf = 0;
    XSTAMP(6);  // the previous round's write-out and this barrier
    uint32_t mm[NPT][MAXS], mt[NPT][MAXS];  // message, bin | rank << 8 (~0u = none)
    uint32_t vv[NPT], kk[NPT];
    bool wlive[NPT];  // the wave has a node in slot q (wave-uniform)
#pragma unroll
    for (uint32_t q = 0; q < NPT; ++q) {
      const unsigned long long g0 = rd * per_round + q * B + __builtin_amdgcn_readfirstlane(tid & ~63u);
      const unsigned long long g = g0 + (tid & 63);
      vv[q] = ~0u;
      kk[q] = 0;
      wlive[q] = g0 < Tn;
      if (g0 < Tn) {
        const uint32_t u = unit_of_wave(w, g0, g < Tn ? g : Tn - 1, Tn, units);
        if (g < Tn) {
        const uint32_t f = u / Ls, k = u - f * Ls;
        const uint32_t s = (t0 + k) % w.R;
        const uint32_t i = (uint32_t)(g - w.unit_off[u]);
        vv[q] = (f << kFineLog) + w.flist[((size_t)s * w.nfine + f) * kFineNodes + i];
        kk[q] = k;
        }
      }
    }
    XSTAMP(1);  // firing nodes looked up
#pragma unroll
    for (uint32_t q = 0; q < NPT; ++q) {
#pragma unroll
      for (uint32_t j = 0; j < MAXS; ++j) { mm[q][j] = kEmptyMsg; mt[q][j] = ~0u; }
    }
    if (MAXS >= 5 && MAXS <= 6 && w.pk && !w.nopair) {  // (uniform)
      load_rows_pk_pairs<MAXS, NPT>(w, vv, wlive, mm);  // all rows in flight
    } else {
#pragma unroll
      for (uint32_t q = 0; q < NPT; ++q)
        if (vv[q] != ~0u) load_row<MAXS>(w, vv[q], mm[q]);  // all rows in flight
    }
    XSTAMP(2);  // rows gathered
    uint32_t sentq[NPT];
#pragma unroll
    for (uint32_t q = 0; q < NPT; ++q) {
      sentq[q] = 0;
      if (vv[q] == ~0u) continue;
      const uint32_t v = vv[q], k = kk[q], t = t0 + k;
      uint32_t vn, c3drop;
      node_key(w.tlog, w.tmask, w.key, (uint64_t)w.base + v, K_DROP, vn, c3drop);
      uint32_t sent = 0;
#pragma unroll
      for (uint32_t jg = 0; jg < (MAXS + 3) / 4; ++jg) {
        if (mm[q][jg * 4] == kEmptyMsg) break;
        // :144, :172 and the messages' crash rolls (:180): one draw per slot
        const u32x4 r = philox(vn, t, jg, c3drop, w.key.k0, w.key.k1);
#pragma unroll
        for (uint32_t jj = 0; jj < 4; ++jj) {
          const uint32_t j = jg * 4 + jj;
          if (j >= MAXS) break;
          uint32_t dropd, crashd;
          drop_crash(lane_of(r, jj), dropd, crashd);
          if (mm[q][j] != kEmptyMsg && (int32_t)dropd >= w.kd) {  // kept: :145
            uint32_t loc = mm[q][j];
            const uint32_t bin = coarse_bin(w, loc);
            const uint32_t roll0 = (int32_t)crashd < w.kc;
            mt[q][j] = bin | (atomicAdd(&sm.cnt[bin], 1u) << 8);
            mm[q][j] = loc | (k << kCoarseShift) | (roll0 << kRoll0Coarse);
            ++sent;
          }
        }
      }
      sentq[q] = sent;
#pragma unroll
      for (uint32_t kx = 0; kx < kBitTicks; ++kx)
        if (kx == k) accp[kx] += 1u | (sent << 16);
    }
    if (WRITE && add_stats && w.tstat) {  // batched trials: fired/sent per (trial, tick)
#pragma unroll
      for (uint32_t q = 0; q < NPT; ++q) {
        const uint32_t key = vv[q] == ~0u ? ~0u : (uint32_t)((uint64_t)vv[q] >> w.tlog) * kMaxWindow + w.tofs + kk[q];
        tstat_add(w.tstat, key, TS_FIRED, 1u, TS_SENT, sentq[q]);
      }
    }
    XSTAMP(3);  // drop / crash draws and LDS ranks
    __syncthreads();
    if (!WRITE) {
      if (binner && sm.cnt[tid]) atomicAdd(&w.chist[reg], (unsigned long long)sm.cnt[tid]);
      continue;  // the next round's first barrier orders the reuse of sm.cnt
    }
    block_scan256(sm.cnt, sm.off);
    // thread b reserves bin b's run; the atomic's return latency overlaps the
    // LDS scatter below (which needs only off[] from the scan)
    const uint32_t mycnt = binner ? sm.cnt[tid] : 0u;
    unsigned long long at = 0;
    if (mycnt) at = atomicAdd(&w.cfill[reg], (unsigned long long)mycnt);
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < NPT; ++q)
#pragma unroll
      for (uint32_t j = 0; j < MAXS; ++j)
        if (mt[q][j] != ~0u) {
          const uint32_t bin = mt[q][j] & 255, p = sm.off[bin] + (mt[q][j] >> 8);
          sm.sorted[p] = mm[q][j];
          sm.sbin[p] = (uint8_t)bin;
        }
    if (mycnt) {
      if (at + mycnt > cend - cbase) {
        atomicOr(w.err, kErrCoarse);
        if (w.dd) atomicOr(reinterpret_cast<unsigned int*>(&w.cfill[kRegions]), kErrCoarse);  // every shard stops
        sm.ovf = 1;
      }
      sm.gbase[tid] = cbase + at - sm.off[tid];
    }
    XSTAMP(4);  // scan, reservation, LDS scatter (wave 0's part)
    __syncthreads();
    XSTAMP(5);  // waiting for the other waves
    const uint32_t total = sm.off[256];
    // two LDS reads per message; the region bound is checked only in a round
    // whose reservation overflowed (the window is then redone exactly)
    if (!sm.ovf) {
      for (uint32_t p = tid; p < total; p += B) w.cmsg[sm.gbase[sm.sbin[p]] + p] = sm.sorted[p];
    } else {
      for (uint32_t p = tid; p < total; p += B) {
        const uint32_t b = sm.sbin[p];
        const unsigned long long pos = sm.gbase[b] + p;
        if (pos < sm.cend[b]) w.cmsg[pos] = sm.sorted[p];
      }
    }
  }
  if (!WRITE || !add_stats) return;  // an exact redo must not count the window twice
#pragma unroll
  for (uint32_t kx = 0; kx < kBitTicks; ++kx) {
    if (kx >= L) continue;
    const uint32_t fired = wave_sum32(accp[kx] & 0xFFFFu), sent = wave_sum32(accp[kx] >> 16);
    if ((tid & 63) == 0) {
      if (fired) atomicAdd(&sm.acc[kx][0], (unsigned long long)fired);
      if (sent) atomicAdd(&sm.acc[kx][1], (unsigned long long)sent);
    }
  }
  __syncthreads();
  if (tid < L * 2) {
    const uint32_t k = tid >> 1, fld = tid & 1;
    const unsigned long long v = sm.acc[k][fld];
    unsigned long long* row = shard_row(w, k);
    if (v) atomicAdd(&row[fld ? ST_SENT : ST_FIRED], v);
    // every delivered send is a receipt; k_resolve subtracts the uncounted ones
    if (v && fld) atomicAdd(&row[ST_MSGS], v);
  }
}
template <bool WRITE, uint32_t MAXS, uint32_t NPT, uint32_t B = kExpandBlock>
__global__ __launch_bounds__(B) void k_expand(const WinState w, uint32_t t0, uint32_t L, unsigned long long Tn,
                                              int add_stats) {
  expand_body<WRITE, MAXS, NPT, B>(w, t0, L, Tn, add_stats);
}
// the shards of an in-process group (device-driven: each reads its Tn from its
// control block), a slice of the persistent grid each
template <bool WRITE, uint32_t MAXS, uint32_t NPT, uint32_t B = kExpandBlock>
__global__ __launch_bounds__(B) void k_expand_m(const WinState* __restrict__ ws, uint32_t L, int add_stats) {
  expand_body<WRITE, MAXS, NPT, B>(ws[blockIdx.y], 0u, L, 0ull, add_stats);
}

// The packed view of sealed stride-8 rows (pk_byte): slots 0..5 of row v.
__global__ void k_pack_rows(const uint32_t* ids, uint64_t n, uint32_t* pk) {
  for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n;
       v += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 a = reinterpret_cast<const uint4*>(ids + v * 8)[0];
    const uint2 b = reinterpret_cast<const uint2*>(ids + v * 8)[2];
    uint2* d = reinterpret_cast<uint2*>(reinterpret_cast<char*>(pk) + pk_byte((uint32_t)v));
    d[0] = make_uint2(a.x, a.y);
    d[1] = make_uint2(a.z, a.w);
    d[2] = b;
  }
}

// Slots past a node's friends list become kEmptyMsg (the window engine's
// expand reads rows without the length byte).
__global__ void k_seal_rows(const uint8_t* deg, uint32_t* ids, uint64_t n, uint32_t stride) {
  for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n;
       v += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t d = deg[v];
    for (uint32_t j = d; j < stride; ++j) ids[v * stride + j] = kEmptyMsg;
  }
}

// End of coarse region r, and its messages (the fill capped at its size).
__device__ __forceinline__ unsigned long long region_end(const WinState& w, uint32_t r) {
  return w.ccap_end ? w.ccap_end[r] : w.ccap[r + 1];
}
__device__ __forceinline__ unsigned long long region_fill(const WinState& w, uint32_t r) {
  const unsigned long long room = region_end(w, r) - w.ccap[r];
  return w.cfill[r] < room ? w.cfill[r] : room;
}

// Unsharded layouts deal k_part2's tiles by XCD: all tiles of coarse bin c
// go to XCD c & 7, so each fine region is written from one XCD's L2 (the
// runs of different tiles meet in whole lines there instead of in partial
// lines from eight L2s).  xcd_bin_pos(c) = the bin's place in that order.
__device__ __forceinline__ bool tiles_by_xcd(const WinState& w) {
  return w.csub == kCoarseSub && !w.csrc && !w.noxcd;
}
__device__ __forceinline__ uint32_t xcd_bin_pos(uint32_t c) { return (c & 7) * 32 + (c >> 3); }
__device__ __forceinline__ uint32_t xcd_bin_of(uint32_t pc) { return (pc & 31) * 8 + (pc >> 5); }

// Fine regions inside each coarse region: capacity per fine bucket of coarse
// c = cfill[c]*1.15/256 + 512 (fast path), or exact counts (fhist != null).
__device__ __forceinline__ void plan_body(const WinState& w, bool exact) {
  __shared__ unsigned long long s_base[257];
  __shared__ unsigned long long s_cap[256];
  __shared__ uint32_t s_tp[257];
  const uint32_t tid = threadIdx.x;  // 256 threads per block: thread c plans coarse bucket c
  if (w.ctl) {
    uint32_t t0;
    if (!win_live(w, t0, 0)) return;
  }
  // messages of bucket c = the fills of its csub sub-regions (capped at their
  // size); part2 tiles never cross a sub-region
  const uint32_t csub = w.csub;
  unsigned long long cnt = 0;
  uint32_t ntile = 0;
  unsigned long long fl[kCoarseSub];  // unsharded layout (csub = 8): the fills' loads in flight together
  if (csub == kCoarseSub) {
#pragma unroll
    for (uint32_t x = 0; x < kCoarseSub; ++x) fl[x] = region_fill(w, tid * kCoarseSub + x);
#pragma unroll
    for (uint32_t x = 0; x < kCoarseSub; ++x) {
      cnt += fl[x];
      ntile += (uint32_t)((fl[x] + kPartTile - 1) / kPartTile);
    }
  } else {
    for (uint32_t x = 0; x < csub && tid * csub + x < kRegions; ++x) {
      const unsigned long long f = region_fill(w, tid * csub + x);
      cnt += f;
      ntile += (uint32_t)((f + kPartTile - 1) / kPartTile);
    }
  }
  const bool live = tid < w.ncoarse;
  // the last coarse bucket may hold fewer than 256 fine buckets
  const uint32_t nf = live ? min(256u, w.nfine - tid * 256) : 1u;
  __shared__ unsigned long long s_x[4];
  s_cap[tid] = live ? (cnt + cnt / 8 + nf - 1) / nf + 512 : 0;
  unsigned long long tb, tt;
  // the bucket's nf fine regions (a partial last bucket's were counted as
  // 256 before: its plan outgrew the host's bound R + R/8 + 513 * 256 per
  // coarse bucket, and a shard window whose fine buffer was sized by that
  // bound overflowed every time -- r04aj)
  s_base[tid] = block_exscan256_u64(s_cap[tid] * nf, s_x, &tb);
  s_tp[tid] = (uint32_t)block_exscan256_u64(live ? ntile : 0u, s_x, &tt);
  if (tid == 0) { s_base[256] = tb; s_tp[256] = (uint32_t)tt; }
  __syncthreads();
  if (blockIdx.x == 0) {  // every region < kRegions is written (256 * csub >= kRegions)
    uint32_t a = s_tp[tid];
    if (tiles_by_xcd(w)) {
      // k_part2 deals the tiles of bin c to XCD c & 7: tprefix is in the
      // order (c & 7, c >> 3, sub-region), so XCD x's tiles are one run
      __shared__ uint32_t s_pt[256];
      const uint32_t pc = xcd_bin_pos(tid);
      s_pt[pc] = live ? ntile : 0u;
      __syncthreads();
      const uint32_t mine = s_pt[tid];
      unsigned long long tot;
      const uint32_t pre = (uint32_t)block_exscan256_u64(mine, s_x, &tot);
      s_pt[tid] = pre;
      __syncthreads();
      a = s_pt[pc];
#pragma unroll
      for (uint32_t x = 0; x < kCoarseSub; ++x) {
        w.tprefix[pc * kCoarseSub + x] = a;
        a += live ? (uint32_t)((fl[x] + kPartTile - 1) / kPartTile) : 0u;
      }
    } else if (csub == kCoarseSub) {
#pragma unroll
      for (uint32_t x = 0; x < kCoarseSub; ++x) {
        w.tprefix[tid * kCoarseSub + x] = a;
        a += live ? (uint32_t)((fl[x] + kPartTile - 1) / kPartTile) : 0u;
      }
    } else {
      for (uint32_t x = 0; x < csub && tid * csub + x < kRegions; ++x) {
        const uint32_t r = tid * csub + x;
        w.tprefix[r] = a;
        a += live ? (uint32_t)((region_fill(w, r) + kPartTile - 1) / kPartTile) : 0u;
      }
    }
    if (tid == 255) w.tprefix[kRegions] = s_tp[256];
  }
  if (exact) return;  // fstart comes from the exact count + scan instead
  // device-driven windows: regions past the buffer are empty, and the window
  // is flagged for the host to grow the buffer and redo it
  const unsigned long long cap = w.ctl ? w.ctl->fmsg_cap : ~0ull;
  if (w.tnodes) {
    // batched trials: a coarse bucket is whole trials of bpt fine buckets, the
    // first `full` of them full, one partial (rem nodes), the rest empty (ids
    // past the trial's n); a message stays in its trial, so a fine bucket's
    // share of the coarse count is its share of the nodes, not 1/256 (the
    // uniform share under-planned every full bucket by n / 2^tlog and sent most
    // dense windows of a C3 batch to the exact redo)
    const uint32_t bpt = 1u << (w.tlog - kFineLog);
    const uint32_t full = w.tnodes >> kFineLog, rem = w.tnodes & (kFineNodes - 1);
    __syncthreads();
    if (tid < w.ncoarse) {  // s_cap[c] = one trial's capacity in bucket c
      const uint32_t nf = min(256u, w.nfine - tid * 256);
      const unsigned long long nodes = (unsigned long long)(nf / bpt) * w.tnodes;
      const unsigned long long cf = (cnt * 9 * kFineNodes + 8 * nodes - 1) / (8 * nodes) + 512;
      const unsigned long long cr = rem ? (cnt * 9 * rem + 8 * nodes - 1) / (8 * nodes) + 512 : 0;
      s_cap[tid] = full * cf + cr;
      s_tp[tid] = (uint32_t)(nf / bpt);
      s_base[tid] = cf;  // (s_base is rebuilt below)
      fl[0] = cr;
    }
    __syncthreads();
    __shared__ unsigned long long s_cf[256], s_cr[256];
    if (tid < w.ncoarse) { s_cf[tid] = s_base[tid]; s_cr[tid] = fl[0]; }
    unsigned long long tb2;
    const unsigned long long btot = tid < w.ncoarse ? s_tp[tid] * s_cap[tid] : 0ull;
    __syncthreads();
    s_base[tid] = block_exscan256_u64(btot, s_x, &tb2);
    if (tid == 0) s_base[256] = tb2;
    __syncthreads();
    if (w.ctl && blockIdx.x == 0 && tid == 0 && s_base[w.ncoarse] > cap) atomicOr(w.err, kErrFine);
    for (uint32_t f = blockIdx.x * blockDim.x + tid; f <= w.nfine; f += gridDim.x * blockDim.x) {
      const uint32_t c = f >> 8, d = f & 255, q = d / bpt, j = d % bpt;
      const unsigned long long x =
          f == w.nfine ? s_base[w.ncoarse]
                       : s_base[c] + q * s_cap[c] + min(j, full) * s_cf[c] + (j > full ? s_cr[c] : 0ull);
      w.fstart[f] = x < cap ? x : cap;
    }
    return;
  }
  if (w.ctl && blockIdx.x == 0 && tid == 0 && s_base[w.ncoarse] > cap) atomicOr(w.err, kErrFine);
  for (uint32_t f = blockIdx.x * blockDim.x + tid; f <= w.nfine; f += gridDim.x * blockDim.x) {
    const uint32_t c = f >> 8, d = f & 255;
    const unsigned long long x = f == w.nfine ? s_base[w.ncoarse] : s_base[c] + d * s_cap[c];
    w.fstart[f] = x < cap ? x : cap;
  }
}
__global__ void k_plan(const WinState w, bool exact) { plan_body(w, exact); }
__global__ void k_plan_m(const WinState* __restrict__ ws, bool exact) { plan_body(ws[blockIdx.y], exact); }

// LDS counting sort of one tile by an 8-bit digit, then coalesced runs out.
#ifndef GS_PART_BLOCK
#define GS_PART_BLOCK 1024
#endif
constexpr uint32_t kPartBlock = GS_PART_BLOCK;  // threads per partition tile (16 messages each)
static_assert(kPartTile % kPartBlock == 0, "whole messages per thread");

// The tile holds coarse messages as they came: the fine digit (bits 14..21) is
// re-read at write-out, so there is no per-slot bin byte (64 KB: two tiles/CU).
struct TileSort {
  uint32_t buf[kPartTile];
  uint32_t cnt[256];
  uint32_t off[257];
  unsigned long long gbase[256];  // digit b's message p goes to gbase[b] + p
  unsigned long long gend[256];  // end of fine region b (fstart[c*256 + b + 1])
  uint32_t ovf;                  // a fine region of this tile overflowed
};

// part2: coarse tiles -> fine regions; message = u_in_fine | k << 14.
// SCATTER=false counts per fine bucket (exact fallback).
template <bool SCATTER>
__device__ __forceinline__ void part2_body(const WinState& w) {
  __shared__ TileSort ts;
  __shared__ uint32_t s_tp[kRegions + 1];
  const uint32_t tid = threadIdx.x;
  if (w.ctl) {
    uint32_t t0;
    if (!win_live(w, t0, 0)) return;
  }
  // a sparse window has few tiles: the workgroups past them leave before
  // staging the 8-KB tile prefix (the grid is sized for the densest window)
  const bool perm = tiles_by_xcd(w);
  uint32_t g0 = blockIdx.x, g1 = w.tprefix[kRegions], gstep = gridDim.x;
  if (perm && (gridDim.x & 7) == 0) {  // XCD x = blockIdx & 7 takes its bins' tiles
    const uint32_t x = blockIdx.x & 7;
    g0 = w.tprefix[x * 256] + (blockIdx.x >> 3);
    g1 = w.tprefix[(x + 1) * 256];
    gstep = gridDim.x >> 3;
  }
  if (g0 >= g1) return;
  for (uint32_t i = tid; i <= kRegions; i += kPartBlock) s_tp[i] = w.tprefix[i];
  __syncthreads();
  for (uint32_t g = g0; g < g1; g += gstep) {
    uint32_t lo = 0, hi = kRegions - 1;  // tile-order position rho: s_tp[rho] <= g < s_tp[rho+1]
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1) >> 1;
      if (s_tp[mid] <= g) lo = mid; else hi = mid - 1;
    }
    const uint32_t rho = lo;
    const uint32_t r = perm ? xcd_bin_of(rho / kCoarseSub) * kCoarseSub + rho % kCoarseSub : rho;
    const uint32_t c = r / w.csub;
    unsigned long long cb = w.ccap[r];
    const uint32_t* msrc = w.cmsg;  // the region's messages (a receive layout names their buffer)
    if (w.csrc) {
      msrc = w.csrc[cb >> kSrcShift];
      cb &= kSrcMask;
    }
    const unsigned long long ce = cb + region_fill(w, r);
    const unsigned long long base = cb + (unsigned long long)(g - s_tp[rho]) * kPartTile;
    if (tid < 256) ts.cnt[tid] = 0;
    __syncthreads();
    if (tid == 0) ts.ovf = 0;
    constexpr uint32_t kPer = kPartTile / kPartBlock;
    static_assert(kPartTile <= 65536 && kPer % 2 == 0, "two 16-bit ranks per register");
    uint32_t m[kPer], rank[kPer / 2] = {};
#pragma unroll
    for (uint32_t r = 0; r < kPer; ++r) {
      const unsigned long long x = base + r * kPartBlock + tid;
      // branch-free load (index clamped into the tile's region: base < ce)
      const uint32_t m1 = msrc[x < ce ? x : ce - 1];
      m[r] = x < ce ? m1 : kEmptyMsg;
    }
#pragma unroll
    for (uint32_t r = 0; r < kPer; ++r)
      if (m[r] != kEmptyMsg) rank[r / 2] |= atomicAdd(&ts.cnt[(m[r] >> kFineLog) & 255], 1u) << (16 * (r & 1));
    __syncthreads();
    if (!SCATTER) {
      if (tid < 256 && ts.cnt[tid]) atomicAdd(&w.fhist[c * 256 + tid], (unsigned long long)ts.cnt[tid]);
      __syncthreads();
      continue;
    }
    block_scan256(ts.cnt, ts.off);
    // thread b < 256 reserves fine bucket c*256+b's run; the atomic's return
    // latency overlaps the LDS scatter (which needs only off[] from the scan)
    const uint32_t mycnt = tid < 256 ? ts.cnt[tid] : 0u;
    const uint32_t myf = c * 256 + (tid & 255);
    unsigned long long at = 0, fb = 0, fe = 0;
    if (mycnt) {
      at = atomicAdd(&w.ffill[myf], (unsigned long long)mycnt);
      fb = w.fstart[myf];
      fe = w.fstart[myf + 1];
    }
    __syncthreads();
#pragma unroll
    for (uint32_t r = 0; r < kPer; ++r)
      if (m[r] != kEmptyMsg) {
        ts.buf[ts.off[(m[r] >> kFineLog) & 255] + ((rank[r / 2] >> (16 * (r & 1))) & 0xFFFFu)] = m[r];
        if ((m[r] >> kRoll0Coarse) & 1u) {  // a crash roll: its node is special in k_resolve
          const uint32_t v = (c << kCoarseShift) | (m[r] & ((1u << kCoarseShift) - 1));
          atomicOr(&w.rollw[v >> 5], 1u << (v & 31));
        }
      }
    if (mycnt) {
      if (at + mycnt > fe - fb) {
        atomicOr(w.err, kErrFine);
        ts.ovf = 1;
      }
      ts.gbase[tid] = fb + at - ts.off[tid];
      ts.gend[tid] = fe;
    }
    __syncthreads();
    const uint32_t total = ts.off[256];
    // two LDS reads per message; the region bound is checked only in a tile
    // whose reservation overflowed (the window is then redone exactly)
    if (!ts.ovf) {
      for (uint32_t p = tid; p < total; p += kPartBlock) {
        const uint32_t m1 = ts.buf[p];
        w.fmsg[ts.gbase[(m1 >> kFineLog) & 255] + p] = (m1 & (kFineNodes - 1)) | ((m1 >> kCoarseShift) << kFineLog);
      }
    } else {
      for (uint32_t p = tid; p < total; p += kPartBlock) {
        const uint32_t m1 = ts.buf[p], b = (m1 >> kFineLog) & 255;
        const unsigned long long pos = ts.gbase[b] + p;
        if (pos < ts.gend[b]) w.fmsg[pos] = (m1 & (kFineNodes - 1)) | ((m1 >> kCoarseShift) << kFineLog);
      }
    }
    __syncthreads();
  }
}
template <bool SCATTER>
__global__ __launch_bounds__(kPartBlock) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_part2(const WinState w) {
  part2_body<SCATTER>(w);
}
template <bool SCATTER>
__global__ __launch_bounds__(kPartBlock) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_part2_m(
    const WinState* __restrict__ ws) {
  part2_body<SCATTER>(ws[blockIdx.y]);
}

constexpr uint32_t kResolveMaxBuckets = 256;  // buckets one persistent workgroup may own
constexpr uint32_t kSmallMax = 256;           // buckets with <= this many receipts: k_resolve_small
#ifndef GS_SMALL_BLOCK
#define GS_SMALL_BLOCK 512
#endif
constexpr uint32_t kSmallBlock = GS_SMALL_BLOCK;  // k_resolve_small: 8 waves, one bucket each
#ifndef GS_ROLLED_BLOCK
#define GS_ROLLED_BLOCK 256
#endif
constexpr uint32_t kRolledBlock = GS_ROLLED_BLOCK;  // the rolled replay: 4 waves, one bucket each

// Bit-parallel resolve (k_resolve).  Three kinds of node in a window:
//   crashed before it: every receipt is uncounted (simulator.go:108), by tick;
//   ROLLED: live, and a receipt in the window carries a crash roll (k_part2
//     marks those nodes in w.rollw): the receipts are written to the bucket's
//     rolled list (w.rlmsg, w.rlcnt) and replayed exactly (rule A6) by
//     k_resolve_rolled after this kernel, sorted per wave like k_resolve_small;
//   plain: every receipt is counted and the first one informs the node
//     (:111, :117-121), so a bit per (tick, node) is the whole state.
// Per receipt: b1[k] |= bit (no-return LDS atomic) and a read of the word's
// (crashed, rolled) pair.  A bucket whose rolled list overflows takes the
// per-tick large path (resolve_tick), which reuses the same LDS for per-node
// counters.
constexpr uint32_t kBitWords = kFineNodes / 32;
struct ResolveLds {
  union {
    struct {                            // b1 .. dlist, then the infection list
      uint32_t b1[kBitTicks][kBitWords];
      uint2 cr0[kBitWords];             // per word: crashed before the window, a crash-roll
                                        // receipt in the window (from w.rollw)
    };
    struct {                            // large path
      uint32_t cnt[kFineNodes];         // per node at the current tick: arrivals | crash rolls << 16
      uint32_t recv[kBitWords];
      uint32_t crash[kBitWords];
      uint32_t nrecv[kBitWords];
      uint32_t ncrash[kBitWords];
    };
  };
  uint32_t fc[kWinMaxRing];         // fire-list lengths of this bucket, per ring slot
  uint32_t st[kMaxWindow][4];       // dead (not counted), recv, crash per tick: whole launch
  uint32_t dead[kMaxWindow];        // this bucket's receipts at nodes crashed before the window
  uint32_t blist[kResolveMaxBuckets];  // this workgroup's non-empty buckets
  unsigned long long bstart[kResolveMaxBuckets];  // their message region starts (fstart)
  uint32_t bcnt[kResolveMaxBuckets];   // their message counts (ffill)
  uint32_t ndup;
  uint32_t ninf;
  uint32_t err;
  uint32_t nb;
  uint32_t cls;
  unsigned long long stamp[2][kStampPhases];  // GS_STAMPS: [M >= 1024][phase] cycles (thread 0)
  unsigned long long tlast;
};  // ~72 KB: two workgroups per CU
static_assert(kBitTicks <= kMaxWindow, "window ticks fit the message format");
static_assert(sizeof(uint32_t) * kFineNodes <= sizeof(((ResolveLds*)0)->cnt), "the infection list fits");

// GS_STAMPS diagnostics: thread 0 adds the cycles since the last stamp to phase i.
__device__ __forceinline__ void stamp(const WinState& w, ResolveLds& sm, uint32_t i) {
  if (w.dbg && threadIdx.x == 0) {
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    if (i) sm.stamp[sm.cls][i] += t - sm.tlast;
    sm.tlast = t;
  }
}

// receipt (fine message): loc | k << 14 | roll0 << 18

// GS_RESOLVE_PROBE=1 (timing probe builds only, results differ): k_resolve's
// receipts phase skips the per-receipt (crashed, rolled) read, every node is
// plain -- the floor of the b1 atomics alone
#if defined(GS_RESOLVE_PROBE) && GS_RESOLVE_PROBE == 1
#define GS_RESOLVE_CR0(loc) make_uint2(0u, 0u)
#else
#define GS_RESOLVE_CR0(loc) sm.cr0[(loc) >> 5]
#endif

__device__ __forceinline__ uint32_t msg_loc(uint32_t m) { return m & (kFineNodes - 1); }
__device__ __forceinline__ uint32_t msg_tick(uint32_t m) { return (m >> kFineLog) & (kMaxWindow - 1); }

// The receive case of Node.Start (simulator.go:107-123) for node `loc` of the
// bucket with kk arrivals at tick t, `ones` of them carrying a crash roll
// (rule A6, first_crash).  (Large-bucket path.)
__device__ __forceinline__ void resolve_node(const WinState& w, ResolveLds& sm, uint32_t f,
                                             uint32_t loc, uint32_t kk, uint32_t ones, uint32_t t,
                                             uint32_t& cm, uint32_t& cr, uint32_t& cc, uint32_t& cs) {
  const uint32_t bit = 1u << (loc & 31), wi = loc >> 5;
  if (sm.crash[wi] & bit) return;                                  // :108 (not counted)
  const uint64_t g = (uint64_t)w.base + (f << kFineLog) + loc;
  uint32_t u, c3order;
  node_key(w.tlog, w.tmask, w.key, g, K_ORDER, u, c3order);
  const uint32_t pos = ones ? first_crash(u, t, kk, ones, c3order, w.key.k0, w.key.k1) : kk + 1;
  cm += pos <= kk ? pos : kk;                                      // :111
  if (pos > 1 && !(sm.recv[wi] & bit)) {                           // :117
    atomicOr(&sm.recv[wi], bit);                                   // :120
    ++cr;                                                          // :121
    // Broadcast() (:122, :141-142): fire at t + off
    uint32_t c3delay;
    node_key(w.tlog, w.tmask, w.key, g, K_DELAY, u, c3delay);
    const uint32_t off = fire_offset(w.delay_low, w.delay_span,
                                     philox(u, t, 0, c3delay, w.key.k0, w.key.k1).x);
    const uint32_t s = (t + off) % w.R;
    const uint32_t at = atomicAdd(&sm.fc[s], 1u);
    w.flist[((size_t)s * w.nfine + f) * kFineNodes + at] = (uint16_t)loc;
    ++cs;
  }
  if (pos <= kk) {                                                 // :112-115
    atomicOr(&sm.crash[wi], bit);
    ++cc;
  }
}

// One tick's receipts over messages m[lo, hi) (large buckets, streamed from
// global memory): count arrivals per node, then the lane whose atomicAnd takes
// a node's nonzero count resolves that node.
template <class Src>
__device__ __forceinline__ void resolve_tick(const WinState& w, ResolveLds& sm, uint32_t f,
                                             const Src& src, uint32_t lo, uint32_t hi, uint32_t k,
                                             uint32_t t) {
  const uint32_t tid = threadIdx.x;
  for (uint32_t p = lo + tid; p < hi; p += kResolveBlock) {
    const uint32_t m = src[p];
    if (msg_tick(m) != k) continue;
    const uint32_t old = atomicAdd(&sm.cnt[msg_loc(m)], 1u + (((m >> kRoll0Fine) & 1u) << 16));
    if ((old & 0xFFFFu) == 0xFFFFu) sm.err = 1;
  }
  __syncthreads();
  uint32_t arr = 0, cm = 0, cr = 0, cc = 0, cs = 0;
  for (uint32_t p = lo + tid; p < hi; p += kResolveBlock) {
    const uint32_t m = src[p];
    if (msg_tick(m) != k) continue;
    const uint32_t loc = msg_loc(m);
    const uint32_t kk = atomicExch(&sm.cnt[loc], 0u);
    arr += kk & 0xFFFFu;
    if (kk) resolve_node(w, sm, f, loc, kk & 0xFFFFu, kk >> 16, t, cm, cr, cc, cs);
  }
  if (arr != cm) atomicAdd(&sm.st[k][0], arr - cm);
  if (cr) atomicAdd(&sm.st[k][1], cr);
  if (cc) atomicAdd(&sm.st[k][2], cc);
  (void)cs;  // every infection schedules one Broadcast: ST_SCHED = ST_RECV
  __syncthreads();
}

__device__ __forceinline__ uint32_t lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
__device__ __forceinline__ uint32_t mbcnt(unsigned long long b) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
}

// Wave-aggregated append: one LDS atomic per wave, lanes with `take` get
// consecutive slots of the list whose fill counter is *n (all lanes active).
__device__ __forceinline__ uint32_t wave_append(uint32_t* n, bool take) {
  const unsigned long long bal = __ballot(take);
  uint32_t base = 0;
  if (bal && lane_id() == 0) base = atomicAdd(n, (uint32_t)__popcll(bal));
  return __builtin_amdgcn_readfirstlane(base) + mbcnt(bal);
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (uint32_t o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Adds the lanes' per-tick infection counts plus sm.st (dead, recv, crash) to
// the per-tick totals and, for a batched trial, to tstat[trial]; leaves them
// zeroed.  Block-uniform call.
// acc_ni[k / 2] holds tick k's count in bits 16 * (k & 1) (<= 32 per bucket,
// <= 256 buckets per lane).
__device__ __forceinline__ void flush_counts(const WinState& w, ResolveLds& sm, uint32_t (&acc_ni)[kBitTicks / 2],
                                             uint32_t L, uint32_t trial) {
#pragma unroll
  for (uint32_t k = 0; k < kBitTicks; ++k) {
    if (k >= L) continue;
    const uint32_t sr = wave_sum((acc_ni[k / 2] >> (16 * (k & 1))) & 0xFFFFu);
    if (lane_id() == 0 && sr) atomicAdd(&sm.st[k][1], sr);
  }
#pragma unroll
  for (uint32_t k = 0; k < kBitTicks / 2; ++k) acc_ni[k] = 0;
  __syncthreads();
  const uint32_t tid = threadIdx.x;
  if (tid < L * 3) {
    const uint32_t k = tid / 3, fld = tid - k * 3;
    const uint32_t v = sm.st[k][fld];
    // field 0 counts receipts that were NOT counted (:108, after a crash):
    // the expand added every delivered send to ST_MSGS
    unsigned long long* row = shard_row(w, k);
    if (v && fld == 0) atomicAdd(&row[ST_MSGS], 0ull - (unsigned long long)v);
    if (v && fld == 1) {
      atomicAdd(&row[ST_RECV], (unsigned long long)v);
      atomicAdd(&row[ST_SCHED], (unsigned long long)v);  // every infection schedules one Broadcast
    }
    if (v && fld == 2) atomicAdd(&row[ST_CRASH], (unsigned long long)v);
    if (v && trial != ~0u) atomicAdd(&w.tstat[((size_t)trial * kMaxWindow + w.tofs + k) * kTStatFields + TS_DEAD + fld], v);
    sm.st[k][fld] = 0;
  }
  __syncthreads();
}

// Persistent: workgroup g owns buckets g, g + G, g + 2G, ... (G = gridDim.x),
// resolves its non-empty ones in turn, and adds its per-tick counters once at
// the end.  Per bucket:
//   stage    thread w owns bit word w (32 nodes): its recv/crash words in
//            registers, spec = crashed | marked in rollw (cleared here), its
//            b1 words and chain head zeroed
//   receipts every receipt sets its (tick, node) bit in b1; receipts at
//            special nodes are listed, then chained under their word
//   ticks    thread w resolves its plain nodes with bit ops, tick by tick
//            (informed at the first receipt), then replays its special nodes'
//            (node, tick) groups in order (rule A6, first_crash); the
//            infections are Broadcast() (:122, :141)
// A bucket with more rolled receipts than kRolledCap takes the per-tick large path.
__device__ __forceinline__ void resolve_body(const WinState& w, uint32_t t0, uint32_t L) {
  __shared__ ResolveLds sm;
  const uint32_t tid = threadIdx.x, G = gridDim.x;
  L = win_live(w, t0, L);
  if (!L) return;
  static_assert(kBitWords == kResolveBlock, "one bit word per thread");
  static_assert(kWinMaxRing <= kResolveBlock, "one ring slot per thread");
  if (tid < kMaxWindow * 4) (&sm.st[0][0])[tid] = 0;
  if (tid == 0) { sm.nb = 0; sm.cls = 0; }
  if (tid < 2 * kStampPhases) (&sm.stamp[0][0])[tid] = 0;
  __syncthreads();
  {
    const uint32_t f = blockIdx.x + tid * G;
    const unsigned long long fl = tid < kResolveMaxBuckets && f < w.nfine ? w.ffill[f] : 0ull;
    const bool ne = fl > kSmallMax;  // small: k_resolve_small
    const uint32_t at = wave_append(&sm.nb, ne);
    if (ne) {
      // the bucket descriptors come from LDS later: a wait for them never waits
      // for the vector loads in flight (the next bucket's prefetch)
      sm.blist[at] = f;
      sm.bstart[at] = w.fstart[f];
      sm.bcnt[at] = (uint32_t)fl;
    }
  }
  __syncthreads();
  const uint32_t nb = sm.nb;
  stamp(w, sm, 0);
  uint32_t fB = 0, MB = 0;
  unsigned long long mbB = 0;
  auto next_bucket = [&](uint32_t j) { fB = sm.blist[j]; mbB = sm.bstart[j]; MB = sm.bcnt[j]; };
  if (nb > 0) next_bucket(0);
  uint32_t* rwg = (uint32_t*)w.recv;
  uint32_t* cwg = (uint32_t*)w.crash;
  // this lane's infections per tick over all its buckets
  uint32_t acc_ni[kBitTicks / 2];
#pragma unroll
  for (uint32_t k = 0; k < kBitTicks / 2; ++k) acc_ni[k] = 0;
  static_assert(kBitTicks % 2 == 0 && 32 * kResolveMaxBuckets < 65536, "two 16-bit counts per register");
  constexpr uint32_t kU = 8;  // loads in flight per lane
  constexpr uint32_t kBatch = kResolveBlock * kU;
  // messages p0 + u * kResolveBlock + tid of a bucket (gm, M): raw loads, valid
  // iff the index is < M (M >= 1); 32-bit byte offsets from the uniform base
  // (M < 2^28)
  auto ld = [&](const uint32_t* gm, uint32_t M, uint32_t p0, uint32_t (&m)[kU]) {
#pragma unroll
    for (uint32_t u = 0; u < kU; ++u) {
      const uint32_t p = p0 + u * kResolveBlock + tid;
      m[u] = *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(gm) + ((p < M ? p : M - 1) << 2));
    }
  };
  // the next bucket's state words and first batch of messages are loaded
  // while this bucket finishes (from the end of its receipts)
  uint32_t pm[kU], p_recv0 = 0, p_crash0 = 0, p_roll0 = 0, p_fcv = 0;
  bool p_in = false;
  auto prefetch = [&](uint32_t f, uint32_t M, unsigned long long mb) {
    const uint64_t wi = ((uint64_t)(f << kFineLog) >> 5) + tid;
    const bool in = wi < w.W * 2;
    // branch-free (clamped) loads, masked where they are used: a load in a
    // branch, or a select right after it, makes the compiler wait for it at
    // once, which serialises the prefetch with the rest of this bucket
    const uint64_t wc = in ? wi : w.W * 2 - 1;
    p_in = in;
    p_recv0 = rwg[wc];
    p_crash0 = cwg[wc];
    p_roll0 = w.rollw[wc];
    p_fcv = w.fcount[(size_t)(tid < w.R ? tid : 0u) * w.nfine + f];
    ld(w.fmsg + mb, M, 0, pm);
  };
  if (nb > 0) prefetch(fB, MB, mbB);
  for (uint32_t i = 0; i < nb; ++i) {
    const uint32_t f = fB, M = MB;
    const unsigned long long mb = mbB;
    const uint32_t node0 = f << kFineLog;
    const uint64_t wi = ((uint64_t)node0 >> 5) + tid;
    // Philox keys of the bucket's nodes: key node knode0 + local offset (a
    // bucket lies inside one trial), counter words c3order / c3delay
    uint32_t knode0, c3order;
    node_key(w.tlog, w.tmask, w.key, (uint64_t)w.base + node0, K_ORDER, knode0, c3order);
    const uint32_t c3delay = (c3order & 0xFFFFFFu) | (K_DELAY << 24);
    const bool in = wi < w.W * 2;
    const uint32_t recv0 = p_in ? p_recv0 : 0u, crash0 = p_in ? p_crash0 : 0u, roll0 = p_in ? p_roll0 : 0u;
    const uint32_t fcv = tid < w.R ? p_fcv : 0u;
    if (i + 1 < nb) next_bucket(i + 1);
    if (roll0) w.rollw[wi] = 0u;  // consumed: the next window starts clear
    const uint32_t rollw = roll0 & ~crash0;
#pragma unroll
    for (uint32_t k = 0; k < kBitTicks; ++k)
      if (k < L) sm.b1[k][tid] = 0;
    sm.cr0[tid] = make_uint2(crash0, rollw);
    if (tid < w.R) sm.fc[tid] = fcv;
    if (tid < kMaxWindow) sm.dead[tid] = 0;
    if (tid == 0) { sm.ndup = 0; sm.ninf = 0; sm.err = M >= (1u << 28) ? 3 : 0; sm.cls = M >= 1024 ? 1 : 0; }
    __syncthreads();
    stamp(w, sm, 1);
    // receipts: (tick, node) bits; uncounted receipts at crashed nodes by
    // tick (8-bit fields per lane, flushed every 31 batches); receipts at
    // rolled nodes listed.  The next batch's loads are issued before this
    // batch's LDS work.
    const uint32_t* gm = w.fmsg + mb;
    unsigned long long dlo = 0, dhi = 0;  // uncounted receipts, ticks 0..7 / 8..15
    auto flush_dead = [&]() {
      while (dlo) {
        const uint32_t b = __builtin_ctzll(dlo) >> 3;
        atomicAdd(&sm.dead[b], (uint32_t)(dlo >> (8 * b)) & 255u);
        dlo &= ~(255ull << (8 * b));
      }
      while (dhi) {
        const uint32_t b = __builtin_ctzll(dhi) >> 3;
        atomicAdd(&sm.dead[8 + b], (uint32_t)(dhi >> (8 * b)) & 255u);
        dhi &= ~(255ull << (8 * b));
      }
    };
    // one batch: receipts m[u] where VALID (a macro body: a lambda spills)
#define GS_RESOLVE_BATCH(m, VALID)                                                                \
    {                                                                                             \
      uint2 sp[kU];                                                                               \
      _Pragma("unroll") for (uint32_t u = 0; u < kU; ++u) {                                       \
        sp[u] = make_uint2(0, 0);                                                                 \
        if (VALID) {                                                                              \
          const uint32_t loc = msg_loc(m[u]);                                                     \
          atomicOr(&sm.b1[msg_tick(m[u])][loc >> 5], 1u << (loc & 31)); /* no return */         \
          sp[u] = GS_RESOLVE_CR0(loc);                                                            \
        }                                                                                         \
      }                                                                                           \
      uint32_t dm = 0; /* bit u: receipt u is at a rolled node */                                 \
      _Pragma("unroll") for (uint32_t u = 0; u < kU; ++u) {                                       \
        const uint32_t sh = msg_loc(m[u]) & 31, k = msg_tick(m[u]);                               \
        if ((sp[u].x >> sh) & 1u) { /* crashed before the window: not counted (:108) */           \
          if (k < 8) dlo += 1ull << (8 * k);                                                      \
          else dhi += 1ull << (8 * (k - 8));                                                      \
        }                                                                                         \
        if ((sp[u].y >> sh) & 1u) dm |= 1u << u;                                                  \
      }                                                                                           \
      if (nbat % 31 == 30) flush_dead();                                                          \
      const uint32_t nd = __popc(dm);                                                             \
      if (__ballot(nd != 0)) {                                                                    \
        uint32_t pre = 0, tot = 0; /* wave prefix of nd (<= 8) */                                 \
        _Pragma("unroll") for (uint32_t bb = 0; bb < 4; ++bb) {                                   \
          const unsigned long long bal = __ballot((nd >> bb) & 1u);                               \
          pre += mbcnt(bal) << bb;                                                                \
          tot += (uint32_t)__popcll(bal) << bb;                                                   \
        }                                                                                         \
        uint32_t base = 0;                                                                        \
        if (lane_id() == 0) base = atomicAdd(&sm.ndup, tot);                                      \
        uint32_t at = __builtin_amdgcn_readfirstlane(base) + pre;                                 \
        _Pragma("unroll") for (uint32_t u = 0; u < kU; ++u) if ((dm >> u) & 1u) {                 \
          if (at < kRolledCap) w.rlmsg[(size_t)f * kRolledCap + at] = m[u] & ((1u << 19) - 1);    \
          else sm.err = 3;                                                                        \
          ++at;                                                                                   \
        }                                                                                         \
      }                                                                                           \
    }
    {
      uint32_t m[kU];
#pragma unroll
      for (uint32_t u = 0; u < kU; ++u) m[u] = pm[u];
      for (uint32_t p0 = 0, nbat = 0; p0 < (sm.err == 3 ? 0u : M); p0 += kBatch, ++nbat) {
        uint32_t mn[kU];
        if (p0 + kBatch < M) ld(gm, M, p0 + kBatch, mn);
        GS_RESOLVE_BATCH(m, p0 + u * kResolveBlock + tid < M)
#pragma unroll
        for (uint32_t u = 0; u < kU; ++u) m[u] = mn[u];
      }
    }
#undef GS_RESOLVE_BATCH
    flush_dead();
    stamp(w, sm, 2);
    __syncthreads();
    if (i + 1 < nb) prefetch(fB, MB, mbB);
    // the rolled list goes to k_resolve_rolled (none on the large path)
    if (tid == 0) w.rlcnt[f] = sm.err == 3 ? 0u : min(sm.ndup, kRolledCap);
    stamp(w, sm, 3);
    uint32_t rw = recv0, cw = crash0;
    if (sm.err != 3) {
      if (tid < L && sm.dead[tid]) atomicAdd(&sm.st[tid][0], sm.dead[tid]);
      // plain nodes: informed at their first receipt, tick by tick
      uint32_t infk[kBitTicks], ninf = 0;  // infections per tick of this word
      const uint32_t plain = ~(crash0 | rollw);
#pragma unroll
      for (uint32_t k = 0; k < kBitTicks; ++k) {
        infk[k] = 0;
        if (k >= L) continue;
        const uint32_t infS = sm.b1[k][tid] & plain & ~rw;  // :117-121
        rw |= infS;
        infk[k] = infS;
      }
      stamp(w, sm, 4);
#pragma unroll
      for (uint32_t k = 0; k < kBitTicks; ++k) {
        const uint32_t ni = __popc(infk[k]);
        acc_ni[k / 2] += ni << (16 * (k & 1));
        ninf += ni;
      }
      stamp(w, sm, 5);
      __syncthreads();
      stamp(w, sm, 6);
      // Broadcast() of an infected node x = loc | tick << 14 (:122, :141-142):
      // fire at t + off
      auto bcast = [&](uint32_t x) {
        const uint32_t loc = msg_loc(x), t = t0 + msg_tick(x);
        const uint32_t off = fire_offset(w.delay_low, w.delay_span,
                                         philox(knode0 + loc, t, 0, c3delay, w.key.k0, w.key.k1).x);
        const uint32_t slot = (t + off) % w.R;
        const uint32_t pos = atomicAdd(&sm.fc[slot], 1u);
        w.flist[((size_t)slot * w.nfine + f) * kFineNodes + pos] = (uint16_t)loc;
      };
      // infection list (loc | tick << 14) over the bitmaps, dead from here on
      uint32_t* inf = &sm.cnt[0];
      {
        uint32_t pre = 0, tot = 0;
#pragma unroll
        for (uint32_t b = 0; b < 9; ++b) {  // ninf <= 32 * kBitTicks < 512
          const unsigned long long bal = __ballot((ninf >> b) & 1u);
          pre += mbcnt(bal) << b;
          tot += (uint32_t)__popcll(bal) << b;
        }
        uint32_t base = 0;
        if (tot && lane_id() == 0) base = atomicAdd(&sm.ninf, tot);
        uint32_t at = __builtin_amdgcn_readfirstlane(base) + pre;
#pragma unroll
        for (uint32_t k = 0; k < kBitTicks; ++k)
          for (uint32_t x = k < L ? infk[k] : 0u; x; x &= x - 1)
            inf[at++] = (tid * 32 + __builtin_ctz(x)) | (k << kFineLog);
      }
      __syncthreads();
      stamp(w, sm, 7);
      // the listed infections, spread over the block
      const uint32_t ni_all = sm.ninf;
      for (uint32_t q = tid; q < ni_all; q += kResolveBlock) bcast(inf[q]);
    } else {
      // large path: per-node counters, the messages streamed once per tick
      __syncthreads();
      uint4* c4 = reinterpret_cast<uint4*>(sm.cnt);
      for (uint32_t q = tid; q < kFineNodes / 4; q += kResolveBlock) c4[q] = make_uint4(0, 0, 0, 0);
      sm.recv[tid] = recv0;
      sm.crash[tid] = crash0;
      sm.nrecv[tid] = 0;
      sm.ncrash[tid] = 0;
      __syncthreads();
      for (uint32_t k = 0; k < L; ++k) resolve_tick(w, sm, f, gm, 0, M, k, t0 + k);
      rw = sm.recv[tid] | sm.nrecv[tid];
      cw = sm.crash[tid] | sm.ncrash[tid];
      if (tid == 0 && sm.err == 1) atomicOr(w.err, kErrArrivals);
    }
    __syncthreads();
    stamp(w, sm, 8);
    if (in) {
      if (rw != recv0) rwg[wi] = rw;
      if (cw != crash0) cwg[wi] = cw;
    }
    if (tid < w.R) w.fcount[(size_t)tid * w.nfine + f] = sm.fc[tid];
    stamp(w, sm, 9);
    if (w.dbg && tid == 0) sm.stamp[sm.cls][0] += 1;
    // batched trials: the bucket's counters go to its trial's rows (a bucket
    // lies inside one trial) as well as to the per-tick totals
    if (w.tstat) flush_counts(w, sm, acc_ni, L, (uint32_t)(((uint64_t)w.base + node0) >> w.tlog));
  }
  if (w.dbg && tid < 2 * kStampPhases) atomicAdd(&w.dbg[tid], (&sm.stamp[0][0])[tid]);
  if (!w.tstat) flush_counts(w, sm, acc_ni, L, ~0u);
}
__global__ __launch_bounds__(kResolveBlock, GS_RESOLVE_WAVES) void k_resolve(const WinState w, uint32_t t0, uint32_t L) {
  resolve_body(w, t0, L);
}
__global__ __launch_bounds__(kResolveBlock, GS_RESOLVE_WAVES) void k_resolve_m(const WinState* __restrict__ ws,
                                                                                uint32_t L) {
  resolve_body(ws[blockIdx.y], 0u, L);
}

// Small buckets (1..kSmallMax receipts in the window): one wave per bucket.
// In the sparse windows at the start and end of a broadcast nearly every
// bucket holds a few dozen or hundred receipts, and the bit-parallel
// k_resolve's fixed cost per bucket (512 bit words x L ticks, a chain of block
// barriers) is what the window pays.  Here a wave holds the bucket's
// receipts as E keys per lane (element lane*E + r in register r), sorts them
// by (node, tick, roll0) with a bitonic network (shuffles across lanes,
// swaps across registers), and the first element of every node's run replays
// the receive case (simulator.go:107-123, rule A6) along the run; infected
// nodes Broadcast() (:122, :141-142) into the bucket's fire lists.
// Instance E takes buckets with 64*(E/4) < M <= 64*E receipts (E = 1, 4);
// k_resolve takes the rest.  The launches touch disjoint buckets.
// The same body replays the rolled receipts k_resolve listed per bucket
// (k_resolve_rolled: the rolled nodes' receipts of a dense bucket, up to
// kRolledCap, E = 1, 4, 8 or 16); a rolled node is live when the window starts,
// and its recv/crash bits are untouched by k_resolve, so the replay is the
// same receive case from the same state.
template <uint32_t E, bool ROLLED>
__device__ __forceinline__ void resolve_small_bucket(const WinState& w, uint32_t t0, uint32_t L, uint32_t f,
                                                     const uint32_t* gm, unsigned long long M,
                                                     uint32_t (*st)[kMaxWindow][4], uint32_t* skw,
                                                     uint32_t* fcw);

// One launch for all sizes: each wave takes one bucket and the body by its
// receipt count (wave-uniform).
template <bool ROLLED>
__device__ __forceinline__ void resolve_small_body(const WinState& w, uint32_t t0, uint32_t L) {
  constexpr uint32_t kWaves = (ROLLED ? kRolledBlock : kSmallBlock) / 64;
  constexpr uint32_t kEmax = ROLLED ? 16 : 4;
  __shared__ uint32_t st[kWaves][kMaxWindow][4];  // per wave: dead (not counted), recv, crash per tick
  __shared__ uint32_t sk[kWaves][64 * kEmax];      // each wave's sorted keys
  __shared__ uint32_t fcw[kWaves][kWinMaxRing];    // each wave's bucket: fire-list lengths per ring slot
  const uint32_t tid = threadIdx.x, wv = tid >> 6;
  static_assert(kWaves * kMaxWindow * 4 == kWaves * 64, "one counter per thread");
  static_assert(kRolledCap == 64 * 16, "the rolled bodies cover 1..kRolledCap");
  const uint32_t f = __builtin_amdgcn_readfirstlane(blockIdx.x * kWaves + wv);
  // the bucket's size and start are loaded while the window check is in
  // flight (unused when the window is dead)
  unsigned long long M = 0;
  const uint32_t* gm = nullptr;
  if (f < w.nfine) {
    if (ROLLED) {
      M = w.rlcnt[f];
      gm = w.rlmsg + (size_t)f * kRolledCap;
    } else {
      M = w.ffill[f];
      gm = w.fmsg + w.fstart[f];
    }
  }
  L = win_live(w, t0, L);
  if (!L) return;
  (&st[0][0][0])[tid] = 0;
  __syncthreads();
  if (M > 0 && M <= 64) resolve_small_bucket<1, ROLLED>(w, t0, L, f, gm, M, st, sk[wv], fcw[wv]);
  else if (M > 64 && M <= 256) resolve_small_bucket<4, ROLLED>(w, t0, L, f, gm, M, st, sk[wv], fcw[wv]);
  else if (ROLLED && M > 256 && M <= 512)
    resolve_small_bucket<ROLLED ? 8 : 1, ROLLED>(w, t0, L, f, gm, M, st, sk[wv], fcw[wv]);
  else if (ROLLED && M > 512 && M <= kRolledCap)
    resolve_small_bucket<ROLLED ? 16 : 1, ROLLED>(w, t0, L, f, gm, M, st, sk[wv], fcw[wv]);
  if (ROLLED && M && (threadIdx.x & 63) == 0) w.rlcnt[f] = 0;  // consumed
  // device-driven windows: the window's fire lists of the buckets the body
  // did not take are consumed here (see resolve_small_bucket); k_resolve and
  // the rolled replay run after this kernel
  if (!ROLLED && w.ctl && !(M > 0 && M <= 256) && f < w.nfine && (threadIdx.x & 63) < L)
    w.fcount[(size_t)((t0 + (threadIdx.x & 63)) % w.R) * w.nfine + f] = 0;
  __syncthreads();
  if (tid < L * 3) {
    const uint32_t k = tid / 3, fld = tid - k * 3;
    uint32_t v = 0;
    for (uint32_t q = 0; q < kWaves; ++q) v += st[q][k][fld];
    unsigned long long* row = shard_row(w, k);
    if (v && fld == 0) atomicAdd(&row[ST_MSGS], 0ull - (unsigned long long)v);
    if (v && fld == 1) {
      atomicAdd(&row[ST_RECV], (unsigned long long)v);
      atomicAdd(&row[ST_SCHED], (unsigned long long)v);  // every infection schedules one Broadcast
    }
    if (v && fld == 2) atomicAdd(&row[ST_CRASH], (unsigned long long)v);
  }
}
template <bool ROLLED>
__global__ __launch_bounds__(ROLLED ? kRolledBlock : kSmallBlock) void k_resolve_small(const WinState w, uint32_t t0,
                                                                                       uint32_t L) {
  resolve_small_body<ROLLED>(w, t0, L);
}
template <bool ROLLED>
__global__ __launch_bounds__(ROLLED ? kRolledBlock : kSmallBlock) void k_resolve_small_m(
    const WinState* __restrict__ ws, uint32_t L) {
  resolve_small_body<ROLLED>(ws[blockIdx.y], 0u, L);
}

template <uint32_t E, bool ROLLED>
__device__ __forceinline__ void resolve_small_bucket(const WinState& w, uint32_t t0, uint32_t L, uint32_t f,
                                                     const uint32_t* gm, unsigned long long M,
                                                     uint32_t (*st)[kMaxWindow][4], uint32_t* skw,
                                                     uint32_t* fcw) {
  constexpr uint32_t N = 64 * E;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  {
    // the bucket's fire-list lengths, staged in this wave's LDS: infections
    // take their list positions with LDS atomics instead of same-address
    // global atomics (one wave owns the bucket)
    // device-driven windows: k_resolve_small, the first kernel to append to
    // the fire lists, consumes the window's (k_units counted them, k_expand
    // read them): ring slots t0 .. t0 + L - 1 restart at 0 in every bucket
    // before any infection of this window is appended (a short ring may
    // reuse them)
    const bool consume = !ROLLED && w.ctl;
    const uint32_t s0 = t0 % w.R;
    for (uint32_t s = lane; s < w.R; s += 64)
      fcw[s] = consume && (s + w.R - s0) % w.R < L ? 0u : w.fcount[(size_t)s * w.nfine + f];
    uint32_t knode0, c3order;  // keys of the bucket's nodes (one trial per bucket)
    node_key(w.tlog, w.tmask, w.key, (uint64_t)w.base + (f << kFineLog), K_ORDER, knode0, c3order);
    const uint32_t c3delay = (c3order & 0xFFFFFFu) | (K_DELAY << 24);
    // element i = lane * E + r in key[r] (lane-major: the bitonic stages with
    // j < E are register swaps, only those with j >= E shuffle across lanes)
    uint32_t key[E];  // loc << 5 | k << 1 | crash roll; ~0u sorts last
#pragma unroll
    for (uint32_t r = 0; r < E; ++r) {
      const uint32_t i = lane * E + r;
      key[r] = ~0u;
      if (i < M) {
        const uint32_t m = gm[i];
        key[r] = (msg_loc(m) << 5) | (msg_tick(m) << 1) | ((m >> kRoll0Fine) & 1u);
        // k_part2 marked the node of a crash roll for k_resolve: clear it here
        if (!ROLLED && ((m >> kRoll0Fine) & 1u)) w.rollw[((f << kFineLog) + msg_loc(m)) >> 5] = 0u;
      }
    }
#pragma unroll
    for (uint32_t k = 2; k <= N; k <<= 1)
#pragma unroll
      for (uint32_t j = k >> 1; j > 0; j >>= 1) {
        if (j >= E) {  // partner in lane ^ (j / E), same register
#pragma unroll
          for (uint32_t r = 0; r < E; ++r) {
            const uint32_t i = lane * E + r;
            const uint32_t o = __shfl_xor(key[r], j / E, 64);
            const bool keep_min = ((i & j) == 0) == ((i & k) == 0);
            key[r] = keep_min ? min(key[r], o) : max(key[r], o);
          }
        } else {  // partner in register r ^ j of this lane
#pragma unroll
          for (uint32_t r = 0; r < E; ++r) {
            if (r & j) continue;
            const bool up = ((lane * E + r) & k) == 0;
            const uint32_t a = key[r], b = key[r | j];
            key[r] = up ? min(a, b) : max(a, b);
            key[r | j] = up ? max(a, b) : min(a, b);
          }
        }
      }
#pragma unroll
    for (uint32_t r = 0; r < E; ++r) skw[lane * E + r] = key[r];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint32_t* rwg = (uint32_t*)w.recv;
    uint32_t* cwg = (uint32_t*)w.crash;
    bool any_inf = false;
    // run heads of this lane's elements
    uint32_t head = 0;
#pragma unroll
    for (uint32_t r = 0; r < E; ++r) {
      const uint32_t i = lane * E + r;
      if (key[r] != ~0u && !(i > 0 && (skw[i - 1] >> 5) == (key[r] >> 5))) head |= 1u << r;
    }
    // one run head at a time, keys re-read from LDS: the body (two Philox
    // draws) is emitted once, not E times (the E = 16 instance's unrolled
    // body outgrew the instruction cache)
#pragma unroll 1
    for (uint32_t r = 0; r < E; ++r) {
      if (!((head >> r) & 1u)) continue;
      const uint32_t i = lane * E + r;
      const uint32_t loc = skw[i] >> 5;
      const uint32_t wi = ((f << kFineLog) + loc) >> 5, bit = 1u << (loc & 31), u = knode0 + loc;
      const uint32_t cw = cwg[wi];
      bool rv = (rwg[wi] & bit) != 0, cr = (cw & bit) != 0, inf = false;
      uint32_t tinf = 0;
      for (uint32_t q = i; q < N;) {  // along the run, one (node, tick) group at a time
        const uint32_t e = skw[q];
        if ((e >> 5) != loc) break;  // (~0u never matches a loc)
        const uint32_t k = (e >> 1) & (kMaxWindow - 1), t = t0 + k;
        uint32_t c = 0, ones = 0;  // receipts, crash rolls among them
        for (; q < N && (skw[q] >> 1) == (e >> 1); ++q) {
          ++c;
          ones += skw[q] & 1u;
        }
        if (cr) {                                                   // :108 not counted
          atomicAdd(&st[wv][k][0], c);
          continue;
        }
        // rule A6: counted up to the first crash, informed if a receipt came first
        const uint32_t g = ones ? first_crash(u, t, c, ones, c3order, w.key.k0, w.key.k1) : c + 1;
        if (g > 1 && !rv) {                                         // :117-121
          rv = inf = true;
          tinf = t;
          atomicAdd(&st[wv][k][1], 1u);
        }
        if (g <= c) {                                               // :112-115
          cr = true;
          atomicAdd(&st[wv][k][2], 1u);
          if (c > g) atomicAdd(&st[wv][k][0], c - g);
        }
      }
      if (cr && !(cw & bit)) atomicOr(&cwg[wi], bit);
      if (inf) {  // Broadcast() (:122, :141-142): fire at tinf + off
        any_inf = true;
        atomicOr(&rwg[wi], bit);
        const uint32_t off = fire_offset(w.delay_low, w.delay_span,
                                         philox(u, tinf, 0, c3delay, w.key.k0, w.key.k1).x);
        const uint32_t slot = (tinf + off) % w.R;
        const uint32_t pos = atomicAdd(&fcw[slot], 1u);
        w.flist[((size_t)slot * w.nfine + f) * kFineNodes + pos] = (uint16_t)loc;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (__ballot(any_inf)) {
      for (uint32_t s = lane; s < w.R; s += 64) w.fcount[(size_t)s * w.nfine + f] = fcw[s];
    } else if (consume && lane < L) {
      w.fcount[(size_t)((t0 + lane) % w.R) * w.nfine + f] = 0;
    }
    if (w.tstat) {  // batched trials: this bucket's counters go to its trial's rows
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      if (lane < L * 3) {
        const uint32_t k = lane / 3, fld = lane - k * 3;
        const uint32_t v = st[wv][k][fld];
        const uint32_t trial = (uint32_t)(((uint64_t)w.base + (f << kFineLog)) >> w.tlog);
        if (v) atomicAdd(&w.tstat[((size_t)trial * kMaxWindow + w.tofs + k) * kTStatFields + TS_DEAD + fld], v);
      }
    }
  }
}

__global__ void k_schedule_win(const WinState w, uint32_t node, uint32_t t, uint32_t trials, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= trials) return;
  uint32_t local = node;
  if (trials > 1 || node == ~0u) {
    uint32_t v = node;
    if (node == ~0u) v = uniform(philox(0, 0, 0, ctr3(K_SENDER, w.key.trial + i), w.key.k0, w.key.k1).x, n);
    local = (i << w.tlog) | v;  // batched contexts have base 0
  }
  uint32_t kn, c3;
  node_key(w.tlog, w.tmask, w.key, (uint64_t)w.base + local, K_DELAY, kn, c3);
  const uint32_t off = fire_offset(w.delay_low, w.delay_span, philox(kn, t, 0, c3, w.key.k0, w.key.k1).x);
  const uint32_t s = (t + off) % w.R;
  const uint32_t f = local >> kFineLog;
  const uint32_t pos = atomicAdd(&w.fcount[(size_t)s * w.nfine + f], 1u);
  w.flist[((size_t)s * w.nfine + f) * kFineNodes + pos] = (uint16_t)(local & (kFineNodes - 1));
}

// ---- node-range shards (config C4) -----------------
// Shard r of G owns nodes [r * seg_per, min((r+1) * seg_per, N)) and their
// friend rows.  Every window it expands its OWN firing nodes with k_expand in
// owner mode: a kept message is binned by the shard that owns its target
// (bin = owner * obins + 2^22-node chunk of the owner's range), so the
// coarse regions of owner d are one contiguous block of the message buffer.
// k_pack moves the filled prefixes of each block that leaves the device or
// rank back to back; the blocks go to their owners (all-to-all); each shard
// then partitions (k_plan / k_part2 over the receive layout: G senders x 8
// sub-regions per bin, each region in its sender's buffer read in place or in
// the received blocks) and resolves its own buckets with the kernels above.  Keys are global ids, so the union
// over shards equals the unsharded run bit for bit.

// out[poff[r] ..] = the filled prefix of region r (< nreg), one region per
// blockIdx.x, blockIdx.y strided over it.
__global__ void k_pack(const WinState w, const unsigned long long* poff, uint32_t nreg, uint32_t* out) {
  const uint32_t r = blockIdx.x;
  if (r >= nreg || poff[r] == ~0ull) return;
  if (w.dd && (*w.err & kErrAbort)) return;  // device-driven shard window that some shard overflowed
  const unsigned long long f = region_fill(w, r);
  const uint32_t* src = w.cmsg + w.ccap[r];
  uint32_t* dst = out + poff[r];
  for (unsigned long long i = (unsigned long long)blockIdx.y * blockDim.x + threadIdx.x; i < f;
       i += (unsigned long long)gridDim.y * blockDim.x)
    dst[i] = src[i];
}

// Shards: the window's fire lists are consumed right after the expand (and
// its exact sender redo, which clears the coarse flag first); nothing later
// reads them -- a receive-side redo (receiver_redo) re-partitions and
// resolves the received messages only -- so the consume is unconditional.
__global__ void k_consume_sh(const WinState w, uint32_t t0, uint32_t L) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < L * w.nfine; i += gridDim.x * blockDim.x) {
    const uint32_t k = i / w.nfine, f = i - k * w.nfine;
    w.fcount[(size_t)((t0 + k) % w.R) * w.nfine + f] = 0;
  }
}

// Exclusive scan of one u64 per thread over a block of NW waves (s: NW words
// of LDS); returns the thread's prefix, *total the block's sum.  Block-uniform.
template <uint32_t NW>
__device__ __forceinline__ unsigned long long block_exscan_u64(unsigned long long v, unsigned long long* s,
                                                               unsigned long long* total) {
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  unsigned long long x = v;
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s[wv] = x;
  __syncthreads();
  unsigned long long before = 0, all = 0;
#pragma unroll
  for (uint32_t q = 0; q < NW; ++q) {
    const unsigned long long t = s[q];
    if (q < wv) before += t;
    all += t;
  }
  __syncthreads();
  *total = all;
  return before + x - v;
}

// ---- device-driven shard windows ------------------
// The host-driven shard window (gs_api.cpp shard_windows) reads every shard's
// fire counts and region fills on the host to cut the window and lay out the
// receive side.  Here the counts and fills are gathered into device buffers
// (RCCL all-gathers between ranks; the shards of one device share them), every
// shard cuts the same window (k_cut over the gathered counts) and computes its
// own receive layout (k_rtab), so a window needs no host round trip unless
// its blocks travel between ranks (the host then reads the block sizes for
// the grouped send / receive).

// Shard w.rank's receive layout from the gathered fills: the region starts,
// ends and fills of (bin c, sender s, sub-region x) at (c * G + s) * 8 + x, its
// own pack offsets, the source buffers and the window's received messages --
// what shard_exchange lays out on the host.  Every shard's row also carries
// its overflow flag and fine-buffer capacity: if any shard's expand overflowed
// a region estimate, or any shard would receive more messages than its fine
// buffer holds, every shard sets kErrAbort (the same decision everywhere,
// from the same gathered rows) and the host redoes the window host-driven.
// One block of 256 threads.
__device__ __forceinline__ void rtab_body(const WinState& w, unsigned long long* rtab,
                                          const unsigned long long* const* ccaps, const uint32_t* const* src,
                                          uint32_t nsrc, uint32_t travels) {
  __shared__ unsigned long long s_x[4];
  __shared__ unsigned long long s_R[256];
  __shared__ uint32_t s_abort;
  const uint32_t tid = threadIdx.x;
  uint32_t t0;
  if (!win_live(w, t0, 0)) return;
  const uint32_t G = w.G, me = w.rank, B8 = w.obins * kCoarseSub, nreg = G * B8;
  constexpr size_t K1 = kRegions + 1;
  // the f[8] staging below covers 8 regions per thread: nreg <= 8 * 256 =
  // kRegions, which ctx_setup's shard check (G * bins <= 256) guarantees; a
  // wider layout stops the window instead of dropping regions
  static_assert(kRegions == 8 * 256, "eight regions per thread");
  if (nreg > kRegions) {
    if (tid == 0) atomicOr(w.err, kErrAbort);
    return;
  }
  unsigned long long *rcap = rtab, *rend = rtab + K1, *rfill = rtab + 2 * K1, *mypoff = rtab + 3 * K1;
  s_R[tid] = 0;
  if (tid == 0) s_abort = 0;
  __syncthreads();
  uint32_t fl = 0;
  for (uint32_t s = tid; s < G; s += 256) fl |= (uint32_t)w.glay[(size_t)s * kDDRow + kRegions];
  if (fl & (kErrCoarse | kErrAbort)) atomicOr(&s_abort, 1u);
  for (uint32_t s = 0; s < G; ++s) {
    const unsigned long long* row = w.glay + (size_t)s * kDDRow;
    for (uint32_t r = tid; r < nreg; r += 256) {
      const unsigned long long f = row[r];
      if (f) atomicAdd(&s_R[r / B8], f);
    }
  }
  __syncthreads();
  for (uint32_t d = tid; d < G; d += 256) {  // shard d's fine plan bound (shard_receive's fcap) vs its buffer
    const unsigned long long lo = (unsigned long long)d * w.seg_per;
    const unsigned long long nd = min((unsigned long long)w.seg_per, (unsigned long long)w.nglob - lo);
    const unsigned long long ncd = (((nd + kFineNodes - 1) >> kFineLog) + 255) / 256;
    const unsigned long long R = s_R[d];
    if (R + R / 8 + ncd * 256 * 513 + 16 > w.glay[(size_t)d * kDDRow + kRegions + 1]) atomicOr(&s_abort, 2u);
  }
  __syncthreads();
  if (s_abort) {
    if (tid == 0) atomicOr(w.err, kErrAbort);
    return;
  }
  for (uint32_t rr = tid; rr < K1; rr += 256) {
    rcap[rr] = rend[rr] = rfill[rr] = 0;
    mypoff[rr] = ~0ull;
  }
  __syncthreads();
  // region (c, s, x) of the blocks for this shard: in place in sender s's
  // buffer (its region start), or in the received blocks at the sender's
  // block offset plus the fills before it inside the block
  const uint32_t in_src = travels ? 0u : G;
  const uint32_t per = (B8 + 255) / 256;  // <= 8 (B8 <= kRegions)
  unsigned long long in_s = 0, tot = 0;
  for (uint32_t s = 0; s < G; ++s) {
    const bool tr = travels && s != me;
    const unsigned long long* row = w.glay + (size_t)s * kDDRow + (size_t)me * B8;
    const unsigned long long* cc = ccaps[travels ? 0u : s] + (size_t)me * B8;
    unsigned long long f[8], sum = 0;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
      const uint32_t i = tid * per + j;
      f[j] = j < per && i < B8 ? row[i] : 0ull;
      sum += f[j];
    }
    unsigned long long btot;
    unsigned long long off = block_exscan_u64<4>(sum, s_x, &btot);
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
      const uint32_t i = tid * per + j;
      if (j >= per || i >= B8) continue;
      const uint32_t c = i / kCoarseSub, x = i % kCoarseSub;
      const size_t rr = ((size_t)c * G + s) * kCoarseSub + x;
      const unsigned long long at = tr ? ((unsigned long long)in_src << kSrcShift) | (in_s + off)
                                       : ((unsigned long long)(travels ? 1u : s) << kSrcShift) | cc[i];
      rcap[rr] = at;
      rend[rr] = at + f[j];
      rfill[rr] = f[j];
      off += f[j];
    }
    if (tr) in_s += btot;
    tot += btot;
  }
  if (travels) {  // this shard's own blocks that leave, back to back in region order (k_pack)
    const unsigned long long* row = w.glay + (size_t)me * kDDRow;
    const uint32_t per2 = (nreg + 255) / 256;
    unsigned long long f[8], sum = 0;
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
      const uint32_t r = tid * per2 + j;
      f[j] = j < per2 && r < nreg && r / B8 != me ? row[r] : 0ull;
      sum += f[j];
    }
    unsigned long long btot;
    unsigned long long off = block_exscan_u64<4>(sum, s_x, &btot);
#pragma unroll
    for (uint32_t j = 0; j < 8; ++j) {
      const uint32_t r = tid * per2 + j;
      if (j >= per2 || r >= nreg || r / B8 == me) continue;
      mypoff[r] = off;
      off += f[j];
    }
  }
  if (tid < nsrc) rtab[4 * K1 + tid] = (unsigned long long)(uintptr_t)src[tid];
  if (tid == 0) rtab[kRtabTotal] = tot;
}
__global__ __launch_bounds__(256) void k_rtab(const WinState w, unsigned long long* rtab,
                                              const unsigned long long* const* ccaps, const uint32_t* const* src,
                                              uint32_t nsrc, uint32_t travels) {
  rtab_body(w, rtab, ccaps, src, nsrc, travels);
}
// shard blockIdx.x's layout goes to its receive state's region table (wr.ccap)
__global__ __launch_bounds__(256) void k_rtab_m(const WinState* __restrict__ ws, const WinState* __restrict__ wr,
                                                const unsigned long long* const* ccaps, const uint32_t* const* src,
                                                uint32_t nsrc) {
  rtab_body(ws[blockIdx.x], const_cast<unsigned long long*>(wr[blockIdx.x].ccap), ccaps, src, nsrc, 0u);
}

// The exact fine re-partition of a device-driven shard window whose fine
// regions overflowed their estimates (kErrFine): the counts cleared (here),
// k_plan's tile prefix, k_part2's counting pass, the scan into fstart
// (k_fine_scan), k_part2's scatter.  Guarded launches (w.guard): they do
// nothing unless the shard's kErrFine is set; k_stats_dd clears it.
__device__ __forceinline__ void fine_zero_body(const WinState& w) {
  uint32_t t0;
  if (!win_live(w, t0, 0)) return;
  const uint32_t nh = w.ncoarse * 256 + 1;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < nh; i += gridDim.x * blockDim.x) {
    w.fhist[i] = 0;
    if (i < w.nfine) w.ffill[i] = 0;
  }
}
__global__ void k_fine_zero(const WinState w) { fine_zero_body(w); }
__global__ void k_fine_zero_m(const WinState* __restrict__ ws) { fine_zero_body(ws[blockIdx.y]); }

__device__ __forceinline__ void fine_scan_body(const WinState& w) {
  __shared__ unsigned long long s_x[16];
  uint32_t t0;
  if (!win_live(w, t0, 0)) return;
  const uint32_t n = w.nfine + 1, per = (n + 1023) / 1024, tid = threadIdx.x;
  unsigned long long sum = 0;
  for (uint32_t j = 0; j < per; ++j) {
    const uint32_t i = tid * per + j;
    if (i < n) sum += w.fhist[i];
  }
  unsigned long long tot;
  unsigned long long a = block_exscan_u64<16>(sum, s_x, &tot);
  for (uint32_t j = 0; j < per; ++j) {
    const uint32_t i = tid * per + j;
    if (i >= n) break;
    w.fstart[i] = a;
    a += w.fhist[i];
    if (i < w.nfine) w.ffill[i] = 0;
  }
}
__global__ __launch_bounds__(1024) void k_fine_scan(const WinState w) { fine_scan_body(w); }
__global__ __launch_bounds__(1024) void k_fine_scan_m(const WinState* __restrict__ ws) {
  fine_scan_body(ws[blockIdx.x]);
}

// The window's counters of this shard (its stat shards summed into w.wstat,
// zero rows past the window or in a stopped one) and its flags: kErrArrivals,
// an exact fine re-partition (kErrFine, cleared here), kErrAbort.  A single
// in-process shard (w.solo) closes its window here too (close_rows), one
// launch instead of two.
// kMaxWindow * kStatFields * kCloseLanes threads.
__device__ void close_rows(const WinState& w, const unsigned long long* rows, WinCtl* const* ctls, uint32_t n,
                           uint32_t slot);
__device__ __forceinline__ void stats_dd_body(const WinState& w, uint32_t slot) {
  __shared__ unsigned long long rows[kDDWStat];  // w.solo: closed here (no k_close_dd)
  const uint32_t tid = threadIdx.x;
  const CtlView c = ctl_view(w);
  const bool dead = (c.err & stop_bits(w)) != 0;
  const uint32_t L = dead || c.stop ? 0u : c.L;
  const uint32_t i = tid / kCloseLanes, part = tid % kCloseLanes, k = i / kStatFields;
  unsigned long long sum = 0;
  if (k < L) sum = stat_shard_sum(w, i, part);  // k is uniform over each lane group
  if (part == 0) {
    w.wstat[i] = sum;
    rows[i] = sum;
  }
  if (tid < 8) {
    constexpr uint32_t F = kMaxWindow * kStatFields;
    unsigned long long v = 0;
    if (tid == 0) v = (c.err & kErrArrivals) ? 1 : 0;
    if (tid == 1) v = !w.solo && (c.err & kErrFine) ? 1 : 0;
    if (tid == 2) v = dead ? 1 : 0;
    w.wstat[F + tid] = v;
    rows[F + tid] = v;
  }
  if (tid == 0 && !w.solo && (c.err & kErrFine)) atomicAnd(w.err, ~kErrFine);
  if (!w.solo) return;
  __syncthreads();
  WinCtl* const one[1] = {w.ctl};
  close_rows(w, rows, one, 1, slot);
}
__global__ void k_stats_dd(const WinState w, uint32_t slot) { stats_dd_body(w, slot); }
__global__ void k_stats_dd_m(const WinState* __restrict__ ws, uint32_t slot) { stats_dd_body(ws[blockIdx.x], slot); }

// The close of a device-driven shard window from its summed counter rows
// (F = kMaxWindow * kStatFields counters, then the flags): gs_run's poll rule
// (simulator.go:243-248, as k_close) on every shard's control block, and
// staging slot `slot` for the host.  Block-wide (tid 0 applies the rule).
__device__ void close_rows(const WinState& w, const unsigned long long* rows, WinCtl* const* ctls, uint32_t n,
                           uint32_t slot) {
  const uint32_t tid = threadIdx.x;
  constexpr uint32_t F = kMaxWindow * kStatFields;
  const WinCtl* c0 = ctls[0];
  const bool dead = rows[F + 2] != 0;
  const uint32_t t0 = c0->t, L = dead || c0->stop ? 0u : c0->L;
  unsigned long long* st = w.stage + (size_t)slot * kStageWords;
  for (uint32_t i = tid; i < F; i += blockDim.x) st[8 + i] = i / kStatFields < L ? rows[i] : 0ull;
  if (tid != 0) return;
  uint32_t stop = c0->stop;
  if (L) {
    unsigned long long recv = c0->recv, crashed = c0->crashed, pending = c0->pending;
    for (uint32_t j = 0; j < L; ++j) {
      recv += rows[j * kStatFields + ST_RECV];
      crashed += rows[j * kStatFields + ST_CRASH];
      pending += rows[j * kStatFields + ST_SCHED] - rows[j * kStatFields + ST_FIRED];
    }
    const uint32_t tl = t0 + L - 1;  // windows never cross a poll tick
    if (c0->poll && (tl - c0->pbase) % c0->poll == 0 && !stop) {
      if (recv >= c0->cover) stop = 1 + GS_RUN_COVERED;
      else if (pending == 0) stop = 1 + GS_RUN_QUIESCENT;
      else if (tl >= c0->max_ticks) stop = 1 + GS_RUN_MAX_TICKS;
    }
    for (uint32_t q = 0; q < n; ++q) {
      WinCtl* c = ctls[q];
      c->recv = recv;
      c->crashed = crashed;
      c->pending = pending;
      c->stop = stop;
    }
  }
  st[0] = t0;
  st[1] = L;
  st[2] = stop;
  st[3] = (dead ? kErrAbort : 0u) | (rows[F] ? kErrArrivals : 0u);
  st[4] = rows[F + 1];  // exact fine re-partitions in the window
}

// The close of a device-driven shard window: the window's global counters
// (the sum of the n shards' wstat: the group's shards, or this rank's own
// after the all-reduce), then close_rows.  One block of 128 threads.
__global__ __launch_bounds__(128) void k_close_dd(const WinState w, const unsigned long long* const* wstats,
                                                  WinCtl* const* ctls, uint32_t n, uint32_t slot) {
  __shared__ unsigned long long rows[kDDWStat];
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < kDDWStat; i += blockDim.x) {
    unsigned long long v = 0;
    for (uint32_t q = 0; q < n; ++q) v += wstats[q][i];
    rows[i] = v;
  }
  __syncthreads();
  close_rows(w, rows, ctls, n, slot);
}

}  // namespace

hipError_t win_rtab(const WinState& w, unsigned long long* rtab, const unsigned long long* const* ccaps,
                    const uint32_t* const* src, uint32_t nsrc, uint32_t travels, hipStream_t s) {
  hipLaunchKernelGGL(k_rtab, dim3(1), dim3(256), 0, s, w, rtab, ccaps, src, nsrc, travels);
  return hipGetLastError();
}

hipError_t win_fine_redo(const WinState& w, uint64_t T, hipStream_t s) {
  WinState g = w;
  g.guard = 1;
  (void)T;
  // small persistent grids: when nothing overflowed (nearly always) each launch
  // only reads the control block and leaves
  hipLaunchKernelGGL(k_fine_zero, dim3(64), dim3(256), 0, s, g);
  hipLaunchKernelGGL(k_plan, dim3(1), dim3(256), 0, s, g, true);
  hipLaunchKernelGGL(k_part2<false>, dim3(512), dim3(kPartBlock), 0, s, g);
  hipLaunchKernelGGL(k_fine_scan, dim3(1), dim3(1024), 0, s, g);
  hipLaunchKernelGGL(k_part2<true>, dim3(512), dim3(kPartBlock), 0, s, g);
  return hipGetLastError();
}

hipError_t win_stats_dd(const WinState& w, uint32_t slot, hipStream_t s) {
  hipLaunchKernelGGL(k_stats_dd, dim3(1), dim3(kMaxWindow * kStatFields * kCloseLanes), 0, s, w, slot);
  return hipGetLastError();
}

hipError_t win_close_dd(const WinState& w, const unsigned long long* const* wstats, WinCtl* const* ctls,
                        uint32_t n, uint32_t slot, hipStream_t s) {
  hipLaunchKernelGGL(k_close_dd, dim3(1), dim3(128), 0, s, w, wstats, ctls, n, slot);
  return hipGetLastError();
}

hipError_t win_units_g(const WinGroup& g, uint32_t L, hipStream_t s) {
  const uint32_t blocks = std::max<uint32_t>(std::min<uint32_t>((g.nfine_max + 255) / 256, 4096), 1);
  hipLaunchKernelGGL(k_units_m, dim3(blocks, g.M), dim3(256), 0, s, g.ws, 0u, L);
  return hipGetLastError();
}

hipError_t win_cut_g(const WinGroup& g, unsigned long long budget, hipStream_t s) {
  hipLaunchKernelGGL(k_cut_m, dim3(g.M), dim3(256), 0, s, g.ws, budget);
  return hipGetLastError();
}

hipError_t win_unitscan_g(const WinGroup& g, hipStream_t s) {
  hipLaunchKernelGGL(k_unitscan_m, dim3(std::max<uint32_t>(g.ncoarse_max, 1), g.M), dim3(256), 0, s, g.ws);
  return hipGetLastError();
}

hipError_t win_rtab_g(const WinGroup& g, const unsigned long long* const* ccaps, const uint32_t* const* src,
                      uint32_t nsrc, hipStream_t s) {
  hipLaunchKernelGGL(k_rtab_m, dim3(g.M), dim3(256), 0, s, g.ws, g.wr, ccaps, src, nsrc);
  return hipGetLastError();
}

hipError_t win_recv_g(const WinGroup& g, uint64_t T, hipStream_t s) {
  const uint32_t pblocks = std::min<uint32_t>((g.nfine_max + 1 + 255) / 256, 1024);
  hipLaunchKernelGGL(k_plan_m, dim3(pblocks, g.M), dim3(256), 0, s, g.wr, false);
  const uint64_t tiles = (T + kPartTile - 1) / kPartTile + 256;
  const uint32_t blocks = (uint32_t)(std::min<uint64_t>(tiles, 8192) + 7) & ~7u;
  hipLaunchKernelGGL(k_part2_m<true>, dim3(blocks, g.M), dim3(kPartBlock), 0, s, g.wr);
  // the guarded exact redo (win_fine_redo): each launch leaves at once unless
  // its shard's fine regions overflowed
  hipLaunchKernelGGL(k_fine_zero_m, dim3(64, g.M), dim3(256), 0, s, g.wg);
  hipLaunchKernelGGL(k_plan_m, dim3(1, g.M), dim3(256), 0, s, g.wg, true);
  hipLaunchKernelGGL(k_part2_m<false>, dim3(512, g.M), dim3(kPartBlock), 0, s, g.wg);
  hipLaunchKernelGGL(k_fine_scan_m, dim3(g.M), dim3(1024), 0, s, g.wg);
  hipLaunchKernelGGL(k_part2_m<true>, dim3(512, g.M), dim3(kPartBlock), 0, s, g.wg);
  return hipGetLastError();
}

hipError_t win_stats_dd_g(const WinGroup& g, uint32_t slot, hipStream_t s) {
  hipLaunchKernelGGL(k_stats_dd_m, dim3(g.M), dim3(kMaxWindow * kStatFields * kCloseLanes), 0, s, g.ws, slot);
  return hipGetLastError();
}

hipError_t win_units(const WinState& w, uint32_t t0, uint32_t L, hipStream_t s) {
  (void)L;
  const uint32_t blocks = std::max<uint32_t>(std::min<uint32_t>((w.nfine + 255) / 256, 4096), 1);
  hipLaunchKernelGGL(k_units, dim3(blocks), dim3(256), 0, s, w, t0, L);
  return hipGetLastError();
}

hipError_t win_cut(const WinState& w, unsigned long long budget, hipStream_t s) {
  hipLaunchKernelGGL(k_cut, dim3(1), dim3(256), 0, s, w, budget);
  return hipGetLastError();
}

hipError_t win_unitscan(const WinState& w, hipStream_t s) {
  hipLaunchKernelGGL(k_unitscan, dim3(w.ncoarse), dim3(256), 0, s, w);
  return hipGetLastError();
}

hipError_t win_close(const WinState& w, uint32_t slot, hipStream_t s) {
  hipLaunchKernelGGL(k_close, dim3(1), dim3(kMaxWindow * kStatFields * kCloseLanes), 0, s, w, slot);
  return hipGetLastError();
}

hipError_t win_scan_units(const WinState& w, uint32_t L, void* tmp, size_t& tmp_bytes, hipStream_t s) {
  return hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, (const unsigned long long*)w.usize,
                                          w.unit_off, (int)(L * w.nfine + 1), s);
}

hipError_t win_groupmap(const WinState& w, uint32_t L, hipStream_t s) {
  const uint32_t units = L * w.nfine;
  const uint32_t blocks = std::min<uint32_t>((units + 255) / 256, 4096);
  hipLaunchKernelGGL(k_groupmap, dim3(blocks ? blocks : 1), dim3(256), 0, s, w, L);
  return hipGetLastError();
}

// mode 0: count coarse buckets only; 1: write + per-tick stats; 2: write only
// k_expand's launch geometry for a window of Tn firing nodes: firing nodes per
// round, workgroup size, grid.  One source for win_expand and for the host's
// per-XCD region plan of batched trials (plan_coarse_trials, gs_api.cpp),
// which must know which sub-region each round writes (xcd_rounds).
uint32_t win_expand_geometry(const WinState& w, uint64_t Tn, uint32_t* per_round_out, uint32_t* bsz_out,
                             uint32_t* npt_out) {
  // rows of <= 6 (C5's fanin 6) and <= 8 slots: 4 nodes per thread; LDS holds
  // block * 4 * row slots, so 6-slot rows fit four workgroups per CU
  // GS_XNPT=2: two firing nodes per thread (experiment: LDS and VGPRs for 8 workgroups per CU)
  static const uint32_t npt = [] { const char* e = getenv("GS_XNPT"); return e && atoi(e) == 2 ? 2u : kExpandNpt; }();
  const uint32_t rs = w.slots;  // rows may be padded past the longest one
  // rows <= 6 (C5), 4 nodes per thread: 512-thread workgroups (2048 rows per
  // round, two per CU by LDS): the per-round scan, reservations and barriers
  // cost half as much per message and a bin's run per round doubles (~40
  // messages); 256 (four per CU) and 1024 (one per CU) measured slower
  // (GS_XBLOCK = 256 / 512 / 1024: A/B knob)
  static const uint32_t xb = [] {
    const char* e = getenv("GS_XBLOCK");
    const int v = e ? atoi(e) : 512;
    return v == 512 || v == 1024 ? (uint32_t)v : kExpandBlock;
  }();
  const uint32_t bsz = rs <= 6 && npt == kExpandNpt ? xb : kExpandBlock;
  const uint32_t per_round = rs <= 8 ? bsz * (rs <= 6 ? npt : kExpandNpt) : kExpandBlock;
  const uint64_t rounds = (Tn + per_round - 1) / per_round;
  // rows <= 8 slots: a persistent grid of four workgroups per CU (the LDS
  // holds four) whatever the window's size -- a sparse window then costs one
  // wave of workgroups, not several (GS_XGRID: A/B knob).  Longer rows (the
  // 20- and 32-slot instances fit more workgroups per CU): up to 8192.
  static const uint64_t cap = [] {
    const char* e = getenv("GS_XGRID");
    if (e) return (uint64_t)std::max(atoi(e), 8);
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      return (uint64_t)v * 4;
    return (uint64_t)1024;
  }();
  // (a thread counts fired | sent << 16 of its nodes in 16-bit halves: at most
  // 1024 rounds per workgroup, <= 4096 nodes and 32768 sends per thread)
  const uint64_t grid_cap = std::max<uint64_t>(rs <= 8 ? cap * kExpandBlock / bsz : 8192, (rounds + 1023) / 1024);
  const uint32_t blocks = (uint32_t)std::min<uint64_t>(rounds, grid_cap);
  if (per_round_out) *per_round_out = per_round;
  if (bsz_out) *bsz_out = bsz;
  if (npt_out) *npt_out = npt;
  return blocks;
}

hipError_t win_expand(const WinState& w, uint32_t t0, uint32_t L, uint64_t Tn, int mode,
                      hipStream_t s) {
  uint32_t per_round = 0, bsz = 0, npt = 0;
  const uint32_t blocks = win_expand_geometry(w, Tn, &per_round, &bsz, &npt);
  const uint32_t rs = w.slots;
  (void)per_round;
  const dim3 grid(blocks ? blocks : 1), blk(kExpandBlock);
  const unsigned long long tn = Tn;
  const int st = mode == 1 ? 1 : 0;
  if (rs <= 6 && npt == 2) {
    if (mode) hipLaunchKernelGGL((k_expand<true, 6, 2>), grid, blk, 0, s, w, t0, L, tn, st);
    else hipLaunchKernelGGL((k_expand<false, 6, 2>), grid, blk, 0, s, w, t0, L, tn, 0);
  } else if (rs <= 6 && bsz == 1024) {
    if (mode) hipLaunchKernelGGL((k_expand<true, 6, kExpandNpt, 1024>), grid, dim3(1024), 0, s, w, t0, L, tn, st);
    else hipLaunchKernelGGL((k_expand<false, 6, kExpandNpt, 1024>), grid, dim3(1024), 0, s, w, t0, L, tn, 0);
  } else if (rs <= 6 && bsz == 512) {
    if (mode) hipLaunchKernelGGL((k_expand<true, 6, kExpandNpt, 512>), grid, dim3(512), 0, s, w, t0, L, tn, st);
    else hipLaunchKernelGGL((k_expand<false, 6, kExpandNpt, 512>), grid, dim3(512), 0, s, w, t0, L, tn, 0);
  } else if (rs <= 6) {
    if (mode) hipLaunchKernelGGL((k_expand<true, 6, kExpandNpt>), grid, blk, 0, s, w, t0, L, tn, st);
    else hipLaunchKernelGGL((k_expand<false, 6, kExpandNpt>), grid, blk, 0, s, w, t0, L, tn, 0);
  } else if (rs <= 8) {
    if (mode) hipLaunchKernelGGL((k_expand<true, 8, kExpandNpt>), grid, blk, 0, s, w, t0, L, tn, st);
    else hipLaunchKernelGGL((k_expand<false, 8, kExpandNpt>), grid, blk, 0, s, w, t0, L, tn, 0);
  } else if (rs <= 20) {  // C4's 19-slot rows: a 25-KB LDS stage, six workgroups per CU
    if (mode) hipLaunchKernelGGL((k_expand<true, 20, 1>), grid, blk, 0, s, w, t0, L, tn, st);
    else hipLaunchKernelGGL((k_expand<false, 20, 1>), grid, blk, 0, s, w, t0, L, tn, 0);
  } else {
    if (mode) hipLaunchKernelGGL((k_expand<true, kWinMaxStride, 1>), grid, blk, 0, s, w, t0, L, tn, st);
    else hipLaunchKernelGGL((k_expand<false, kWinMaxStride, 1>), grid, blk, 0, s, w, t0, L, tn, 0);
  }
  return hipGetLastError();
}

hipError_t win_expand_g(const WinGroup& g, uint32_t L, hipStream_t s) {
  static const uint32_t cus = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      return (uint32_t)v;
    return 256u;
  }();
  const uint32_t rs = g.slots_max;
  // win_expand's persistent grid (rows <= 8: four 256-thread workgroups per
  // CU, or two of 512 for rows <= 6) split over the shards, a multiple of 8
  // per shard (blockIdx.x & 7 is the XCD); longer rows: 8192 per shard
  const uint32_t bsz = rs <= 6 ? 512u : kExpandBlock;
  const uint32_t total = rs <= 8 ? cus * 4 * kExpandBlock / bsz : 8192u * g.M;
  const uint32_t bx = std::max<uint32_t>(8, ((total + g.M - 1) / g.M + 7) & ~7u);
  const dim3 grid(bx, g.M);
  if (rs <= 6) hipLaunchKernelGGL((k_expand_m<true, 6, kExpandNpt, 512>), grid, dim3(512), 0, s, g.ws, L, 1);
  else if (rs <= 8) hipLaunchKernelGGL((k_expand_m<true, 8, kExpandNpt>), grid, dim3(kExpandBlock), 0, s, g.ws, L, 1);
  else if (rs <= 20) hipLaunchKernelGGL((k_expand_m<true, 20, 1>), grid, dim3(kExpandBlock), 0, s, g.ws, L, 1);
  else hipLaunchKernelGGL((k_expand_m<true, kWinMaxStride, 1>), grid, dim3(kExpandBlock), 0, s, g.ws, L, 1);
  return hipGetLastError();
}

hipError_t win_pack_rows(const uint32_t* ids, uint64_t n, uint32_t* pk, hipStream_t s) {
  const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(k_pack_rows, dim3((uint32_t)(blocks ? blocks : 1)), dim3(256), 0, s, ids, n, pk);
  return hipGetLastError();
}

hipError_t win_seal_rows(const uint8_t* deg, uint32_t* ids, uint64_t n, uint32_t stride,
                         hipStream_t s) {
  const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 8192);
  hipLaunchKernelGGL(k_seal_rows, dim3((uint32_t)(blocks ? blocks : 1)), dim3(256), 0, s, deg, ids, n,
                     stride);
  return hipGetLastError();
}

hipError_t win_plan(const WinState& w, bool exact, hipStream_t s) {
  const uint32_t blocks = std::min<uint32_t>((w.nfine + 1 + 255) / 256, 1024);
  hipLaunchKernelGGL(k_plan, dim3(blocks), dim3(256), 0, s, w, exact);
  return hipGetLastError();
}

hipError_t win_part2(const WinState& w, uint64_t T, bool scatter, hipStream_t s) {
  const uint64_t tiles = (T + kPartTile - 1) / kPartTile + 256;
  const uint32_t blocks = (uint32_t)(std::min<uint64_t>(tiles, 8192) + 7) & ~7u;  // a multiple of 8: tiles by XCD
  if (scatter) hipLaunchKernelGGL(k_part2<true>, dim3(blocks), dim3(kPartBlock), 0, s, w);
  else hipLaunchKernelGGL(k_part2<false>, dim3(blocks), dim3(kPartBlock), 0, s, w);
  return hipGetLastError();
}

hipError_t win_scan_fine(const WinState& w, void* tmp, size_t& tmp_bytes, hipStream_t s) {
  return hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, (const unsigned long long*)w.fhist,
                                          w.fstart, (int)(w.nfine + 1), s);
}

hipError_t win_resolve(const WinState& w, uint32_t t0, uint32_t L, hipStream_t s) {
  // persistent: two workgroups per CU (the LDS holds two), each owning <= 256 buckets
  static const uint32_t cus = [] {  // thread-safe one-time query (contexts may run in threads)
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      return (uint32_t)v;
    return 256u;
  }();
  static const uint32_t per_cu = [] { const char* e = getenv("GS_RESOLVE_PER_CU"); return e ? (uint32_t)std::max(atoi(e), 1) : 2u; }();  // A/B knob
  uint32_t G = std::min<uint32_t>(w.nfine, per_cu * cus);
  G = std::max<uint32_t>(G, (w.nfine + kResolveMaxBuckets - 1) / kResolveMaxBuckets);
  const uint32_t gs = (w.nfine + kSmallBlock / 64 - 1) / (kSmallBlock / 64);
  hipLaunchKernelGGL(k_resolve_small<false>, dim3(gs), dim3(kSmallBlock), 0, s, w, t0, L);
  static_assert(kSmallMax == 64 * 4, "the two bodies cover 1..kSmallMax");
  hipLaunchKernelGGL(k_resolve, dim3(G), dim3(kResolveBlock), 0, s, w, t0, L);
  // k_resolve_rolled: small blocks (the E = 16 key arrays take 4 KB per wave; blocks finish independently)
  hipLaunchKernelGGL(k_resolve_small<true>, dim3((w.nfine + kRolledBlock / 64 - 1) / (kRolledBlock / 64)),
                     dim3(kRolledBlock), 0, s, w, t0, L);
  return hipGetLastError();
}

hipError_t win_resolve_g(const WinGroup& g, uint32_t L, hipStream_t s) {
  static const uint32_t cus = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0)
      return (uint32_t)v;
    return 256u;
  }();
  // k_resolve's two workgroups per CU split over the shards (each still owns
  // <= kResolveMaxBuckets buckets of its shard)
  uint32_t G = std::min<uint32_t>(g.nfine_max, (2 * cus + g.M - 1) / g.M);
  G = std::max<uint32_t>(G, (g.nfine_max + kResolveMaxBuckets - 1) / kResolveMaxBuckets);
  const uint32_t gs = (g.nfine_max + kSmallBlock / 64 - 1) / (kSmallBlock / 64);
  hipLaunchKernelGGL(k_resolve_small_m<false>, dim3(gs, g.M), dim3(kSmallBlock), 0, s, g.wr, L);
  hipLaunchKernelGGL(k_resolve_m, dim3(G, g.M), dim3(kResolveBlock), 0, s, g.wr, L);
  hipLaunchKernelGGL(k_resolve_small_m<true>, dim3((g.nfine_max + kRolledBlock / 64 - 1) / (kRolledBlock / 64), g.M),
                     dim3(kRolledBlock), 0, s, g.wr, L);
  return hipGetLastError();
}

hipError_t win_stats_reduce(const WinState& w, uint32_t t0, uint32_t L, hipStream_t s) {
  hipLaunchKernelGGL(k_stats_reduce, dim3(1), dim3(kMaxWindow * kStatFields * kCloseLanes), 0, s, w, t0, L);
  return hipGetLastError();
}

hipError_t win_schedule(const WinState& w, uint32_t node, uint32_t tick, uint32_t trials, uint32_t n,
                        hipStream_t s) {
  hipLaunchKernelGGL(k_schedule_win, dim3((trials + 255) / 256), dim3(256), 0, s, w, node, tick, trials, n);
  return hipGetLastError();
}

hipError_t win_consume_sh(const WinState& w, uint32_t t0, uint32_t L, hipStream_t s) {
  const uint32_t blocks = std::min<uint32_t>((L * w.nfine + 255) / 256, 2048);
  hipLaunchKernelGGL(k_consume_sh, dim3(blocks ? blocks : 1), dim3(256), 0, s, w, t0, L);
  return hipGetLastError();
}

hipError_t win_pack(const WinState& w, const unsigned long long* poff, uint32_t nreg, uint32_t* out, hipStream_t s) {
  if (!nreg) return hipSuccess;
  hipLaunchKernelGGL(k_pack, dim3(nreg, 8), dim3(256), 0, s, w, poff, nreg, out);
  return hipGetLastError();
}

}  // namespace gs
