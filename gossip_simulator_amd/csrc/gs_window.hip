// gs_window.hip -- the broadcast round loop as a window pipeline without
// global random atomics (the "window engine").
//
// Why windows: a Broadcast() fires off = max(delaylow,1)..delayhigh-1 ticks
// after the receipt that triggered it (simulator.go:122,142,167), so every
// broadcast firing in ticks [t0, t0+L), L <= max(delaylow,1), is already
// scheduled when tick t0 starts.  The L ticks are processed together; the
// receipts of each tick are still resolved in tick order per node.
//
// Pipeline of one window (one launch each):
//   units   tasks per (tick k, fine bucket f) = fired(k,f) * stride
//   (scan)  hipcub exclusive sum -> a fixed output slot for every task
//   expand  for every firing node v and friend slot j: keyed RandomDrop
//           (:143-147); kept -> target id u into its task slot (no atomics,
//           coalesced), per-tick fired/sent counts, coarse histogram
//   part1   tiles of the expand output -> 256 coarse buckets (u >> 22),
//           LDS counting sort + one global reservation per (tile, bucket)
//   part2   per coarse bucket: count, scan, scatter into fine buckets
//           (16384 nodes each); message = u_in_fine | k << 14
//   resolve one workgroup per fine bucket: the bucket's received/crashed
//           bits and per-node arrival counters live in LDS; for each tick k
//           the arrivals are counted, then one owner lane per node replays
//           ordinals 0..count-1 of the receive case (:107-123) with keyed
//           crash rolls; infections append to the fire list of
//           (slot (t+off) mod R, f) -- a list only this workgroup writes.
// Fire lists: fcount[R][nfine] + flist[R][nfine][16384] (u16 local ids).
#include <hipcub/hipcub.hpp>

#include "gs_internal.h"

namespace gs {
namespace {

constexpr uint32_t kExpandBlock = 256;
constexpr uint32_t kResolveBlock = 512;
constexpr uint32_t kResolveMsgCap = 8192;

// Units = (tick k, fine bucket f); usize = fires.  Also zeroes the window's
// histograms (one launch instead of several memsets).
__global__ void k_units(const WinState w, uint32_t t0, uint32_t L) {
  const uint32_t units = L * w.nfine;
  const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x, nth = gridDim.x * blockDim.x;
  for (uint32_t u = tid; u <= units; u += nth) {
    if (u == units) { w.usize[u] = 0; continue; }
    const uint32_t k = u / w.nfine, f = u - k * w.nfine;
    const uint32_t s = (t0 + k) % w.R;
    w.usize[u] = w.fcount[(size_t)s * w.nfine + f];
  }
  for (uint32_t i = tid; i < 256; i += nth) w.chist[i] = 0;
  for (uint32_t i = tid; i <= w.ncoarse * 256; i += nth) w.fhist[i] = 0;
  for (uint32_t i = tid; i < w.nfine; i += nth) w.ffill[i] = 0;
}

// One lane per firing node (Node.Broadcast, simulator.go:141-147): its row is
// read once, one Philox block gives the drop rolls of 4 friend slots, and the
// node's `stride` output slots start at (firing index) * stride.  A wave
// walks kNodesPerWave consecutive firing nodes of the window.
constexpr uint32_t kNodesPerWave = 256;
__global__ __launch_bounds__(kExpandBlock) void k_expand(const WinState w, uint32_t t0, uint32_t L,
                                                         unsigned long long Tn) {
  __shared__ uint32_t s_hist[256];
  __shared__ unsigned long long s_acc[kMaxWindow][2];
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) s_hist[i] = 0;
  if (threadIdx.x < kMaxWindow * 2) (&s_acc[0][0])[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const uint32_t units = L * w.nfine;
  const uint32_t S = w.stride;
  const uint32_t c3drop = ctr3(K_DROP, w.key.trial);
  const unsigned long long* uo = w.unit_off;
  uint32_t one_bin = 0;  // messages when there is a single coarse bucket
  const unsigned long long nwaves = (Tn + kNodesPerWave - 1) / kNodesPerWave;
  for (unsigned long long gw = (unsigned long long)blockIdx.x * (kExpandBlock / 64) + wid; gw < nwaves;
       gw += (unsigned long long)gridDim.x * (kExpandBlock / 64)) {
    const unsigned long long start = gw * kNodesPerWave;
    // unit holding `start`: last u with uo[u] <= start (wave-uniform search)
    uint32_t lo = 0, hi = units;
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1) >> 1;
      if (uo[mid] <= start) lo = mid; else hi = mid - 1;
    }
    uint32_t u = lo;
    uint32_t cur_k = 0xFFFFFFFFu, sent = 0, fired = 0;
    for (uint32_t it = 0; it < kNodesPerWave / 64; ++it) {
      const unsigned long long g = start + it * 64 + lane;
      if (g >= Tn) break;
      while (uo[u + 1] <= g) ++u;  // empty units are skipped
      const uint32_t k = u / w.nfine, f = u - k * w.nfine;
      if (k != cur_k) {
        if (cur_k != 0xFFFFFFFFu) {
          if (sent) atomicAdd(&s_acc[cur_k][1], (unsigned long long)sent);
          if (fired) atomicAdd(&s_acc[cur_k][0], (unsigned long long)fired);
        }
        cur_k = k; sent = 0; fired = 0;
      }
      const uint32_t t = t0 + k;
      const uint32_t s = t % w.R;
      const uint32_t i = (uint32_t)(g - uo[u]);
      const uint32_t v = (f << kFineLog) + w.flist[((size_t)s * w.nfine + f) * kFineNodes + i];
      const uint32_t d = w.deg[v];
      const uint32_t* row = w.ids + (size_t)v * S;
      uint32_t* out = w.amsg + g * S;
      ++fired;
      for (uint32_t jg = 0; jg * 4 < S; ++jg) {
        u32x4 r{0, 0, 0, 0};
        if (jg * 4 < d) r = philox(v, t, jg, c3drop, w.key.k0, w.key.k1);   // :144, :172
#pragma unroll
        for (uint32_t jj = 0; jj < 4; ++jj) {
          const uint32_t j = jg * 4 + jj;
          if (j >= S) break;
          uint32_t msg = kEmptyMsg;
          if (j < d && (int32_t)uniform(lane_of(r, jj), 100u) >= w.kd) {
            msg = row[j];                                                    // :145
            ++sent;
            if (w.ncoarse == 1) ++one_bin;
            else atomicAdd(&s_hist[msg >> kCoarseShift], 1u);
          }
          out[j] = msg;
        }
      }
    }
    if (cur_k != 0xFFFFFFFFu) {
      if (sent) atomicAdd(&s_acc[cur_k][1], (unsigned long long)sent);
      if (fired) atomicAdd(&s_acc[cur_k][0], (unsigned long long)fired);
    }
  }
  if (one_bin) atomicAdd(&s_hist[0], one_bin);
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < 256; b += blockDim.x)
    if (s_hist[b]) atomicAdd(&w.chist[b], (unsigned long long)s_hist[b]);
  if (threadIdx.x < L * 2) {
    const uint32_t k = threadIdx.x >> 1, fld = threadIdx.x & 1;
    const unsigned long long v = s_acc[k][fld];
    if (v) atomicAdd(&w.stats[(size_t)((t0 + k) % kStatSlots) * kStatFields + (fld ? ST_SENT : ST_FIRED)], v);
  }
}

__global__ void k_coarse_scan(const WinState w) {
  __shared__ unsigned long long s[257];
  __shared__ uint32_t st[257];
  const uint32_t b = threadIdx.x;  // 256 threads
  s[b + 1] = w.chist[b];
  st[b + 1] = (uint32_t)((w.chist[b] + kPartTile - 1) / kPartTile);
  if (b == 0) { s[0] = 0; st[0] = 0; }
  __syncthreads();
  if (b == 0) {
    for (int i = 1; i <= 256; ++i) { s[i] += s[i - 1]; st[i] += st[i - 1]; }
  }
  __syncthreads();
  w.cbase[b] = s[b];
  w.tprefix[b] = st[b];
  w.cfill[b] = 0;
  if (b == 0) { w.cbase[256] = s[256]; w.tprefix[256] = st[256]; }
}

// LDS counting sort of one tile by an 8-bit digit, then coalesced runs out.
struct TileSort {
  uint32_t buf[kPartTile];
  uint8_t bin[kPartTile];
  uint32_t cnt[256];
  uint32_t off[257];
  unsigned long long gbase[256];
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

// part1: expand output -> coarse buckets; message = u_in_coarse | k << 22
__global__ __launch_bounds__(256) void k_part1(const WinState w, unsigned long long T, uint32_t L) {
  __shared__ TileSort ts;
  __shared__ unsigned long long s_kb[kMaxWindow + 1];
  const uint32_t tid = threadIdx.x;
  if (tid <= L) s_kb[tid] = w.unit_off[(size_t)tid * w.nfine] * w.stride;  // tick bounds in slots
  ts.cnt[tid] = 0;
  __syncthreads();
  const unsigned long long base = (unsigned long long)blockIdx.x * kPartTile;
  uint32_t m[kPartTile / 256], rank[kPartTile / 256];
  uint8_t bn[kPartTile / 256];
#pragma unroll
  for (uint32_t r = 0; r < kPartTile / 256; ++r) {
    const unsigned long long x = base + r * 256 + tid;
    bn[r] = 0;
    m[r] = kEmptyMsg;
    if (x < T) {
      const uint32_t u = w.amsg[x];
      if (u != kEmptyMsg) {
        uint32_t k = 0;
        while (k + 1 < L && s_kb[k + 1] <= x) ++k;
        bn[r] = (uint8_t)(u >> kCoarseShift);
        m[r] = (u & ((1u << kCoarseShift) - 1)) | (k << kCoarseShift);
        rank[r] = atomicAdd(&ts.cnt[bn[r]], 1u);
      }
    }
  }
  __syncthreads();
  block_scan256(ts.cnt, ts.off);
  if (ts.cnt[tid]) ts.gbase[tid] = w.cbase[tid] + atomicAdd(&w.cfill[tid], (unsigned long long)ts.cnt[tid]);
  __syncthreads();
#pragma unroll
  for (uint32_t r = 0; r < kPartTile / 256; ++r)
    if (m[r] != kEmptyMsg) {
      const uint32_t p = ts.off[bn[r]] + rank[r];
      ts.buf[p] = m[r];
      ts.bin[p] = bn[r];
    }
  __syncthreads();
  const uint32_t total = ts.off[256];
  for (uint32_t p = tid; p < total; p += 256) {
    const uint32_t b = ts.bin[p];
    w.cmsg[ts.gbase[b] + (p - ts.off[b])] = ts.buf[p];
  }
}

// part2: coarse bucket tiles -> fine buckets; message = u_in_fine | k << 14
template <bool SCATTER>
__global__ __launch_bounds__(256) void k_part2(const WinState w) {
  __shared__ TileSort ts;
  __shared__ uint32_t s_tp[257];
  const uint32_t tid = threadIdx.x;
  s_tp[tid] = w.tprefix[tid];
  if (tid == 0) s_tp[256] = w.tprefix[256];
  __syncthreads();
  const uint32_t ntiles = s_tp[256];
  for (uint32_t g = blockIdx.x; g < ntiles; g += gridDim.x) {
    uint32_t lo = 0, hi = 255;  // coarse bucket c: s_tp[c] <= g < s_tp[c+1]
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1) >> 1;
      if (s_tp[mid] <= g) lo = mid; else hi = mid - 1;
    }
    const uint32_t c = lo;
    const unsigned long long cb = w.cbase[c], ce = w.cbase[c + 1];
    const unsigned long long base = cb + (unsigned long long)(g - s_tp[c]) * kPartTile;
    ts.cnt[tid] = 0;
    __syncthreads();
    uint32_t m[kPartTile / 256], rank[kPartTile / 256];
    uint8_t bn[kPartTile / 256];
#pragma unroll
    for (uint32_t r = 0; r < kPartTile / 256; ++r) {
      const unsigned long long x = base + r * 256 + tid;
      m[r] = kEmptyMsg;
      bn[r] = 0;
      if (x < ce) {
        const uint32_t m1 = w.cmsg[x];
        bn[r] = (uint8_t)((m1 >> kFineLog) & 255);
        m[r] = (m1 & (kFineNodes - 1)) | ((m1 >> kCoarseShift) << kFineLog);
        rank[r] = atomicAdd(&ts.cnt[bn[r]], 1u);
      }
    }
    __syncthreads();
    if (!SCATTER) {
      if (ts.cnt[tid]) atomicAdd(&w.fhist[c * 256 + tid], (unsigned long long)ts.cnt[tid]);
      __syncthreads();
      continue;
    }
    block_scan256(ts.cnt, ts.off);
    if (ts.cnt[tid]) {
      const uint32_t f = c * 256 + tid;
      ts.gbase[tid] = w.fbase[f] + atomicAdd(&w.ffill[f], (unsigned long long)ts.cnt[tid]);
    }
    __syncthreads();
#pragma unroll
    for (uint32_t r = 0; r < kPartTile / 256; ++r)
      if (m[r] != kEmptyMsg) {
        const uint32_t p = ts.off[bn[r]] + rank[r];
        ts.buf[p] = m[r];
        ts.bin[p] = bn[r];
      }
    __syncthreads();
    const uint32_t total = ts.off[256];
    for (uint32_t p = tid; p < total; p += 256) {
      const uint32_t b = ts.bin[p];
      w.fmsg[ts.gbase[b] + (p - ts.off[b])] = ts.buf[p];
    }
    __syncthreads();
  }
}

struct ResolveLds {
  uint32_t recv[kFineNodes / 32];
  uint32_t crash[kFineNodes / 32];
  uint32_t cnt[kFineNodes / 2];  // two u16 arrival counters per word
  uint32_t fc[kWinMaxRing];      // fire-list lengths of this bucket, per ring slot
  uint32_t tcnt[kMaxWindow];     // messages per tick of the window
  uint32_t toff[kMaxWindow + 1];
  uint32_t st[kMaxWindow][4];    // msgs, recv, crash, sched per tick
  uint32_t err;
  uint32_t msg[kResolveMsgCap];  // the bucket's messages, sorted by tick
};

// The receive case of Node.Start (simulator.go:107-123) for node `loc` of the
// bucket with kk arrivals at tick t: ordinals 0..kk-1, keyed crash rolls.
__device__ __forceinline__ void resolve_node(const WinState& w, ResolveLds& sm, uint32_t f,
                                             uint32_t loc, uint32_t kk, uint32_t t, uint32_t c3crash,
                                             uint32_t& cm, uint32_t& cr, uint32_t& cc, uint32_t& cs) {
  const uint32_t u = (f << kFineLog) + loc, bit = 1u << (loc & 31), wi = loc >> 5;
  bool crashed = (sm.crash[wi] & bit) != 0;
  bool received = (sm.recv[wi] & bit) != 0;
  u32x4 r{0, 0, 0, 0};
  for (uint32_t i = 0; i < kk; ++i) {
    if (crashed) break;                                          // :108
    ++cm;                                                        // :111
    if (w.kc > 0) {
      if ((i & 3) == 0) r = philox(u, t, i >> 2, c3crash, w.key.k0, w.key.k1);
      if ((int32_t)uniform(lane_of(r, i & 3), 100u) < w.kc) {   // :112-115
        atomicOr(&sm.crash[wi], bit);
        ++cc;
        crashed = true;
        break;
      }
    }
    if (received) continue;                                      // :117
    atomicOr(&sm.recv[wi], bit);                                 // :120
    received = true;
    ++cr;                                                        // :121
    // Broadcast() (:122, :141-142): fire at t + off
    const uint32_t off = fire_offset(w.delay_low, w.delay_span, draw0(w.key, K_DELAY, u, t, 0));
    const uint32_t s = (t + off) % w.R;
    const uint32_t pos = atomicAdd(&sm.fc[s], 1u);
    w.flist[((size_t)s * w.nfine + f) * kFineNodes + pos] = (uint16_t)loc;
    ++cs;
  }
}

// One tick's receipts over messages m[lo, hi): count arrivals per node, then
// the lane whose atomicAnd takes a node's nonzero count resolves that node.
template <class Src>
__device__ __forceinline__ void resolve_tick(const WinState& w, ResolveLds& sm, uint32_t f,
                                             const Src& src, uint32_t lo, uint32_t hi, uint32_t k,
                                             bool filter, uint32_t t, uint32_t c3crash) {
  const uint32_t tid = threadIdx.x;
  for (uint32_t p = lo + tid; p < hi; p += kResolveBlock) {
    const uint32_t m = src[p];
    if (filter && (m >> kFineLog) != k) continue;
    const uint32_t loc = m & (kFineNodes - 1), sh = (loc & 1) * 16;
    const uint32_t old = atomicAdd(&sm.cnt[loc >> 1], 1u << sh);
    if (((old >> sh) & 0xFFFFu) == 0xFFFFu) sm.err = 1;
  }
  __syncthreads();
  uint32_t cm = 0, cr = 0, cc = 0, cs = 0;
  for (uint32_t p = lo + tid; p < hi; p += kResolveBlock) {
    const uint32_t m = src[p];
    if (filter && (m >> kFineLog) != k) continue;
    const uint32_t loc = m & (kFineNodes - 1), sh = (loc & 1) * 16;
    const uint32_t kk = (atomicAnd(&sm.cnt[loc >> 1], ~(0xFFFFu << sh)) >> sh) & 0xFFFFu;
    if (kk) resolve_node(w, sm, f, loc, kk, t, c3crash, cm, cr, cc, cs);
  }
  if (cm) atomicAdd(&sm.st[k][0], cm);
  if (cr) atomicAdd(&sm.st[k][1], cr);
  if (cc) atomicAdd(&sm.st[k][2], cc);
  if (cs) atomicAdd(&sm.st[k][3], cs);
  __syncthreads();
}

__global__ __launch_bounds__(kResolveBlock) void k_resolve(const WinState w, uint32_t t0, uint32_t L) {
  __shared__ ResolveLds sm;
  const uint32_t f = blockIdx.x, tid = threadIdx.x;
  const uint32_t node0 = f << kFineLog;
  const uint64_t wbase = (uint64_t)node0 >> 5;  // u32 word index of the bucket's bits
  const uint32_t* rg = (const uint32_t*)w.recv;
  const uint32_t* cg = (const uint32_t*)w.crash;
  const uint64_t nw32 = w.W * 2;
  for (uint32_t i = tid; i < kFineNodes / 32; i += kResolveBlock) {
    const bool in = wbase + i < nw32;
    sm.recv[i] = in ? rg[wbase + i] : 0u;
    sm.crash[i] = in ? cg[wbase + i] : 0u;
  }
  for (uint32_t i = tid; i < kFineNodes / 2; i += kResolveBlock) sm.cnt[i] = 0;
  for (uint32_t s = tid; s < w.R; s += kResolveBlock) sm.fc[s] = w.fcount[(size_t)s * w.nfine + f];
  if (tid < kMaxWindow * 4) (&sm.st[0][0])[tid] = 0;
  if (tid < kMaxWindow) sm.tcnt[tid] = 0;
  if (tid == 0) sm.err = 0;
  const unsigned long long mb = w.fbase[f];
  const uint32_t M = (uint32_t)(w.fbase[f + 1] - mb);
  const uint32_t* gm = w.fmsg + mb;
  const uint32_t c3crash = ctr3(K_CRASH, w.key.trial);
  __syncthreads();
  if (M <= kResolveMsgCap) {
    // counting sort of the bucket's messages by tick, into LDS
    for (uint32_t p = tid; p < M; p += kResolveBlock) atomicAdd(&sm.tcnt[gm[p] >> kFineLog], 1u);
    __syncthreads();
    if (tid == 0) {
      uint32_t a = 0;
      for (uint32_t k = 0; k < L; ++k) { sm.toff[k] = a; a += sm.tcnt[k]; sm.tcnt[k] = 0; }
      sm.toff[L] = a;
    }
    __syncthreads();
    for (uint32_t p = tid; p < M; p += kResolveBlock) {
      const uint32_t m = gm[p], k = m >> kFineLog;
      sm.msg[sm.toff[k] + atomicAdd(&sm.tcnt[k], 1u)] = m;
    }
    __syncthreads();
    for (uint32_t k = 0; k < L; ++k)
      resolve_tick(w, sm, f, sm.msg, sm.toff[k], sm.toff[k + 1], k, false, t0 + k, c3crash);
  } else {
    // large bucket: stream the messages from global memory once per pass
    for (uint32_t k = 0; k < L; ++k) resolve_tick(w, sm, f, gm, 0, M, k, true, t0 + k, c3crash);
  }
  uint32_t* rw = (uint32_t*)w.recv;
  uint32_t* cw = (uint32_t*)w.crash;
  for (uint32_t i = tid; i < kFineNodes / 32; i += kResolveBlock)
    if (wbase + i < nw32) { rw[wbase + i] = sm.recv[i]; cw[wbase + i] = sm.crash[i]; }
  for (uint32_t s = tid; s < w.R; s += kResolveBlock) w.fcount[(size_t)s * w.nfine + f] = sm.fc[s];
  if (tid < L * 4) {
    const uint32_t k = tid >> 2, fld = tid & 3;
    const uint32_t v = sm.st[k][fld];
    const uint32_t field = fld == 0 ? ST_MSGS : fld == 1 ? ST_RECV : fld == 2 ? ST_CRASH : ST_SCHED;
    if (v) atomicAdd(&w.stats[(size_t)((t0 + k) % kStatSlots) * kStatFields + field],
                     (unsigned long long)v);
  }
  if (tid == 0 && sm.err) atomicOr(w.err, 4u);
}

__global__ void k_schedule_one_win(const WinState w, uint32_t node, uint32_t t) {
  const uint32_t off = fire_offset(w.delay_low, w.delay_span, draw0(w.key, K_DELAY, node, t, 0));
  const uint32_t s = (t + off) % w.R;
  const uint32_t f = node >> kFineLog;
  const uint32_t pos = atomicAdd(&w.fcount[(size_t)s * w.nfine + f], 1u);
  w.flist[((size_t)s * w.nfine + f) * kFineNodes + pos] = (uint16_t)(node & (kFineNodes - 1));
}

}  // namespace

hipError_t win_units(const WinState& w, uint32_t t0, uint32_t L, hipStream_t s) {
  const uint32_t units = std::max<uint32_t>(L * w.nfine + 1, w.ncoarse * 256 + 1);
  const uint32_t blocks = std::min<uint32_t>((units + 255) / 256, 4096);
  hipLaunchKernelGGL(k_units, dim3(blocks), dim3(256), 0, s, w, t0, L);
  return hipGetLastError();
}

hipError_t win_expand(const WinState& w, uint32_t t0, uint32_t L, hipStream_t s, uint64_t Tn) {
  const uint64_t waves = (Tn + kNodesPerWave - 1) / kNodesPerWave;
  const uint32_t blocks = (uint32_t)std::min<uint64_t>((waves + 3) / 4, 16384);
  hipLaunchKernelGGL(k_expand, dim3(blocks ? blocks : 1), dim3(kExpandBlock), 0, s, w, t0, L,
                     (unsigned long long)Tn);
  return hipGetLastError();
}

hipError_t win_coarse_scan(const WinState& w, hipStream_t s) {
  hipLaunchKernelGGL(k_coarse_scan, dim3(1), dim3(256), 0, s, w);
  return hipGetLastError();
}

hipError_t win_part1(const WinState& w, uint64_t T, uint32_t L, hipStream_t s) {
  const uint64_t tiles = (T + kPartTile - 1) / kPartTile;
  hipLaunchKernelGGL(k_part1, dim3((uint32_t)tiles), dim3(256), 0, s, w, (unsigned long long)T, L);
  return hipGetLastError();
}

hipError_t win_part2(const WinState& w, uint64_t T, bool scatter, hipStream_t s) {
  const uint64_t tiles = (T + kPartTile - 1) / kPartTile + 256;
  const uint32_t blocks = (uint32_t)std::min<uint64_t>(tiles, 8192);
  if (scatter) hipLaunchKernelGGL(k_part2<true>, dim3(blocks), dim3(256), 0, s, w);
  else hipLaunchKernelGGL(k_part2<false>, dim3(blocks), dim3(256), 0, s, w);
  return hipGetLastError();
}

hipError_t win_resolve(const WinState& w, uint32_t t0, uint32_t L, hipStream_t s) {
  hipLaunchKernelGGL(k_resolve, dim3(w.nfine), dim3(kResolveBlock), 0, s, w, t0, L);
  return hipGetLastError();
}

hipError_t win_schedule_one(const WinState& w, uint32_t node, uint32_t tick, hipStream_t s) {
  hipLaunchKernelGGL(k_schedule_one_win, dim3(1), dim3(1), 0, s, w, node, tick);
  return hipGetLastError();
}

hipError_t win_scan_units(const WinState& w, uint32_t L, void* tmp, size_t& tmp_bytes, hipStream_t s) {
  return hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, (const unsigned long long*)w.usize,
                                          w.unit_off, (int)(L * w.nfine + 1), s);
}

hipError_t win_scan_fine(const WinState& w, void* tmp, size_t& tmp_bytes, hipStream_t s) {
  return hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, (const unsigned long long*)w.fhist,
                                          w.fbase, (int)(w.nfine + 1), s);
}

}  // namespace gs
