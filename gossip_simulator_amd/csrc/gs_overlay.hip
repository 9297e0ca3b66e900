// gs_overlay.hip -- overlay construction (simulator.go:62-106,127-164,214-235)
// as a tick-synchronous, sort-bucketed GPU protocol.
//
// Events are u64 keys  dst << (B+1) | src << 1 | kind  (kind 0 = makeup,
// 1 = breakup, B = bits of n-1), kept in one bucket per ring slot (arrival tick
// mod R).  A tick:
//   1. radix-sort the slot's keys (hipcub) -> each node's events contiguous,
//      ordered by (src, kind);
//   2. select segment heads (first event of each dst);
//   3. one lane per dst replays its events in order -- the makeup / breakup
//      handler bodies -- with every draw keyed by (dst, tick, ordinal k), so
//      identical keys (identical messages) commute;
//   4. each processed event emits at most one event (a breakup on eviction,
//      a makeup on replacement) into out[i]; a count pass sizes the buckets and
//      a scatter pass appends them with one global atomic per (block, slot).
// Tick 0 is the needNewFriendCh burst: every node picks `fanout` friends
// (self -> id+1, simulator.go:97-101) and sends a makeup to each.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "gs_internal.h"
#include "gossip.h"

namespace gs {
namespace {

constexpr uint64_t kEmpty = ~0ull;
constexpr uint32_t kMaxRing = 1024;
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
};

// Key node and counter word 3 of global id g (per-trial keys, gs_internal.h).
__device__ __forceinline__ uint32_t ov_draw(const OvParams& p, uint32_t kind, uint32_t g, uint32_t b,
                                            uint32_t c) {
  uint32_t node, c3;
  node_key(p.tlog, p.tmask, p.key, g, kind, node, c3);
  return philox(node, b, c, c3, p.key.k0, p.key.k1).x;
}

__device__ __forceinline__ uint64_t ev_key(uint32_t dst, uint32_t src, uint32_t kind, uint32_t B) {
  return ((uint64_t)dst << (B + 1)) | ((uint64_t)src << 1) | kind;
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
    key = ev_key(tb | f, gv, 0u, p.B);                                      // :102 Makeup
    slot = fire_offset(p.delay_low, p.delay_span, ov_draw(p, K_OVDELAY, gv, 0, j)) % p.R;
  }
};

struct OutSource {  // events emitted by a processing tick
  const uint64_t* out;
  const uint16_t* oslot;
  __device__ __forceinline__ void get(uint64_t i, uint64_t& key, uint32_t& slot) const {
    key = out[i];
    slot = key == kEmpty ? 0xFFFFu : oslot[i];
  }
};

// COUNT: counts[s] += items bound for s.  WRITE: append them to bucket s.
template <bool WRITE, class Src>
__global__ __launch_bounds__(kScatterBlock) void k_scatter(Src src, uint64_t nitems, uint32_t R,
                                                           unsigned long long* counts,
                                                           unsigned long long* fill,
                                                           uint64_t* const* buckets) {
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
    if (i < nitems) src.get(i, key[k], slot[k]);
    if (slot[k] != 0xFFFFu) rank[k] = atomicAdd(&s_hist[slot[k]], 1u);
  }
  __syncthreads();
  if (!WRITE) {
    for (uint32_t s = threadIdx.x; s < R; s += blockDim.x)
      if (s_hist[s]) atomicAdd(&counts[s], (unsigned long long)s_hist[s]);
    return;
  }
  for (uint32_t s = threadIdx.x; s < R; s += blockDim.x)
    if (s_hist[s]) s_base[s] = atomicAdd(&fill[s], (unsigned long long)s_hist[s]);
  __syncthreads();
#pragma unroll
  for (uint32_t k = 0; k < kScatterIPT; ++k)
    if (slot[k] != 0xFFFFu) buckets[slot[k]][s_base[slot[k]] + rank[k]] = key[k];
}

struct IsHead {
  const uint64_t* keys;
  uint32_t shift;
  __device__ __forceinline__ bool operator()(const int64_t i) const {
    return i == 0 || (keys[i] >> shift) != (keys[i - 1] >> shift);
  }
};

struct TickCounters {
  unsigned long long makeups, breakups, err;
};

// One lane per destination node: the makeup / breakup handlers in order.
__global__ __launch_bounds__(256) void k_process(const OvParams p, uint32_t t, uint64_t* keys,
                                                 uint64_t m, const int64_t* heads,
                                                 const int64_t* nheads, uint8_t* deg, uint32_t* ids,
                                                 uint64_t* out, uint16_t* oslot,
                                                 TickCounters* tc) {
  const int64_t H = *nheads;
  const int64_t h = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t mk = 0, bk = 0, err = 0;
  if (h < H) {
    const uint64_t start = (uint64_t)heads[h];
    const uint64_t end = (h + 1 < H) ? (uint64_t)heads[h + 1] : m;
    const uint32_t u = (uint32_t)(keys[start] >> (p.B + 1));
    const uint32_t ul = u & p.tmask, tb = u & ~p.tmask;  // node within its trial, trial base
    const uint64_t smask = (1ull << p.B) - 1;
    // the radix sort ordered the tick's events by destination only (its
    // passes over the B + 1 low bits are saved); this lane puts its
    // destination's run in (src, kind) order -- the order the handlers replay
    // -- by insertion (runs are a few events long in a random overlay)
    const uint64_t lmask = (2ull << p.B) - 1;
    for (uint64_t i = start + 1; i < end; ++i) {
      const uint64_t key = keys[i];
      uint64_t j = i;
      for (; j > start; --j) {
        const uint64_t prev = keys[j - 1];
        if ((prev & lmask) <= (key & lmask)) break;
        keys[j] = prev;
      }
      keys[j] = key;
    }
    uint32_t* row = ids + (size_t)u * p.stride;
    uint32_t d = deg[u];
    for (uint64_t i = start; i < end; ++i) {
      const uint64_t key = keys[i];
      const uint32_t src = (uint32_t)((key >> 1) & smask);
      const uint32_t k = (uint32_t)(i - start);
      uint64_t emitted = kEmpty;
      if (k >= (1u << 26)) { err |= 2; out[i] = kEmpty; continue; }
      if ((key & 1) == 0) {                                   // makeUpCh (:66-75)
        ++mk;
        if (d < p.fanin) {
          row[d++] = src;
        } else {
          const uint32_t pos = uniform(ov_draw(p, K_VICTIM, u, t, k), d);
          const uint32_t victim = row[pos];
          emitted = ev_key(victim, u, 1u, p.B);               // Breakup (:73)
          row[pos] = src;
        }
      } else {                                                // breakUpCh (:76-94)
        ++bk;
        uint32_t idx = 0;
        while (idx < d && row[idx] != src) ++idx;
        if (idx < d) {
          if (d > p.fanout) {                                 // removeFriend (:83)
            for (uint32_t q = idx; q + 1 < d; ++q) row[q] = row[q + 1];
            --d;
          } else {                                            // replace (:86-91)
            uint32_t nf = 0, a = 0, kn, c3;
            node_key(p.tlog, p.tmask, p.key, u, K_REPLACE, kn, c3);
            for (; a < 256; ++a) {
              const u32x4 r = philox(kn, t, (k << 6) | (a >> 2), c3, p.key.k0, p.key.k1);
              nf = uniform(lane_of(r, a & 3), (uint32_t)p.n);
              if (nf != (src & p.tmask) && nf != ul) break;
            }
            nf |= tb;
            if (a == 256) {
              err |= 1;
            } else {
              row[idx] = nf;
              emitted = ev_key(nf, u, 0u, p.B);               // Makeup (:91)
            }
          }
        }
      }
      out[i] = emitted;
      if (emitted != kEmpty)
        oslot[i] = (uint16_t)((t + fire_offset(p.delay_low, p.delay_span,
                                               ov_draw(p, K_OVDELAY, u, t, k))) % p.R);
    }
    deg[u] = (uint8_t)d;
  }
  // block reduction of the window counters
  __shared__ uint32_t s_mk, s_bk, s_err;
  if (threadIdx.x == 0) { s_mk = 0; s_bk = 0; s_err = 0; }
  __syncthreads();
  if (mk) atomicAdd(&s_mk, mk);
  if (bk) atomicAdd(&s_bk, bk);
  if (err) atomicOr(&s_err, err);
  __syncthreads();
  if (threadIdx.x == 0) {
    if (s_mk) atomicAdd(&tc->makeups, (unsigned long long)s_mk);
    if (s_bk) atomicAdd(&tc->breakups, (unsigned long long)s_bk);
    if (s_err) atomicOr(&tc->err, (unsigned long long)s_err);
  }
}

// Grouped variant (GS_OV_GROUP=1): the tick's events sorted by destination GROUP
// only (64 consecutive ids: 6 radix bits fewer), one wave per group, a lane per
// destination.  The group's events are staged in LDS (up to kOvStage; a larger
// group reads them from global memory), and each lane replays its own events
// in (src, kind, position) order by repeated minimum search over the group --
// the order k_process's insertion sort gives, identical keys in position
// order (they are identical messages, so the order among them is immaterial
// beyond the ordinal k).  The 64 lanes' rows are consecutive: the row reads
// and writes of a wave are coalesced instead of one line per destination.
constexpr uint32_t kOvGroupLog = 6;
constexpr uint32_t kOvWaves = 4;
constexpr uint32_t kOvStage = 1024;

__global__ __launch_bounds__(kOvWaves * 64) void k_process_g(const OvParams p, uint32_t t, const uint64_t* keys,
                                                             uint64_t m, const int64_t* heads,
                                                             const int64_t* nheads, uint8_t* deg, uint32_t* ids,
                                                             uint64_t* out, uint16_t* oslot, TickCounters* tc) {
  __shared__ uint64_t s_ev[kOvWaves][kOvStage];
  const int64_t H = *nheads;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t h = (int64_t)blockIdx.x * kOvWaves + wv;  // wave-uniform
  uint32_t mk = 0, bk = 0, err = 0;
  if (h < H) {
    const uint64_t start = (uint64_t)heads[h];
    const uint64_t end = (h + 1 < H) ? (uint64_t)heads[h + 1] : m;
    const uint32_t E = (uint32_t)(end - start);  // m < 2^31
    const uint32_t sh = p.B + 1;
    const uint32_t u = (uint32_t)(keys[start] >> (sh + kOvGroupLog)) << kOvGroupLog | lane;  // this lane's destination
    const bool staged = E <= kOvStage;
    uint64_t* ev = s_ev[wv];
    if (staged) {
      for (uint32_t i = lane; i < E; i += 64) ev[i] = keys[start + i];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    auto key_at = [&](uint32_t i) { return staged ? ev[i] : keys[start + i]; };
    uint32_t cnt = 0;
    for (uint32_t i = 0; i < E; ++i) cnt += (uint32_t)(key_at(i) >> sh) == u;
    if (cnt) {
      const uint32_t ul = u & p.tmask, tb = u & ~p.tmask;  // node within its trial, trial base
      const uint64_t smask = (1ull << p.B) - 1, lmask = (2ull << p.B) - 1;
      uint32_t* row = ids + (size_t)u * p.stride;
      uint32_t d = deg[u];
      uint64_t plow = 0;   // the last replayed event: (low key, position)
      uint32_t ppos = 0;
      for (uint32_t k = 0; k < cnt; ++k) {
        // the next event of u: the least (low key, position) after the last one
        uint64_t blow = ~0ull;
        uint32_t bpos = ~0u;
        for (uint32_t i = 0; i < E; ++i) {
          const uint64_t key = key_at(i);
          if ((uint32_t)(key >> sh) != u) continue;
          const uint64_t lo = key & lmask;
          const bool after = k == 0 || lo > plow || (lo == plow && i > ppos);
          if (after && (lo < blow || (lo == blow && i < bpos))) { blow = lo; bpos = i; }
        }
        plow = blow;
        ppos = bpos;
        const uint64_t i = start + bpos;
        const uint32_t src = (uint32_t)((blow >> 1) & smask);
        uint64_t emitted = kEmpty;
        if (k >= (1u << 26)) { err |= 2; out[i] = kEmpty; continue; }
        if ((blow & 1) == 0) {                                  // makeUpCh (:66-75)
          ++mk;
          if (d < p.fanin) {
            row[d++] = src;
          } else {
            const uint32_t pos = uniform(ov_draw(p, K_VICTIM, u, t, k), d);
            const uint32_t victim = row[pos];
            emitted = ev_key(victim, u, 1u, p.B);               // Breakup (:73)
            row[pos] = src;
          }
        } else {                                                // breakUpCh (:76-94)
          ++bk;
          uint32_t idx = 0;
          while (idx < d && row[idx] != src) ++idx;
          if (idx < d) {
            if (d > p.fanout) {                                 // removeFriend (:83)
              for (uint32_t q = idx; q + 1 < d; ++q) row[q] = row[q + 1];
              --d;
            } else {                                            // replace (:86-91)
              uint32_t nf = 0, a = 0, kn, c3;
              node_key(p.tlog, p.tmask, p.key, u, K_REPLACE, kn, c3);
              for (; a < 256; ++a) {
                const u32x4 r = philox(kn, t, (k << 6) | (a >> 2), c3, p.key.k0, p.key.k1);
                nf = uniform(lane_of(r, a & 3), (uint32_t)p.n);
                if (nf != (src & p.tmask) && nf != ul) break;
              }
              nf |= tb;
              if (a == 256) {
                err |= 1;
              } else {
                row[idx] = nf;
                emitted = ev_key(nf, u, 0u, p.B);               // Makeup (:91)
              }
            }
          }
        }
        out[i] = emitted;
        if (emitted != kEmpty)
          oslot[i] = (uint16_t)((t + fire_offset(p.delay_low, p.delay_span,
                                                 ov_draw(p, K_OVDELAY, u, t, k))) % p.R);
      }
      deg[u] = (uint8_t)d;
    }
  }
  __shared__ uint32_t s_mk, s_bk, s_err;
  if (threadIdx.x == 0) { s_mk = 0; s_bk = 0; s_err = 0; }
  __syncthreads();
  if (mk) atomicAdd(&s_mk, mk);
  if (bk) atomicAdd(&s_bk, bk);
  if (err) atomicOr(&s_err, err);
  __syncthreads();
  if (threadIdx.x == 0) {
    if (s_mk) atomicAdd(&tc->makeups, (unsigned long long)s_mk);
    if (s_bk) atomicAdd(&tc->breakups, (unsigned long long)s_bk);
    if (s_err) atomicOr(&tc->err, (unsigned long long)s_err);
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
static hipError_t grow(DevBuf& b, size_t bytes) {
  if (b.bytes >= bytes) return hipSuccess;
  const size_t nb = std::max(bytes + bytes / 4, b.bytes * 3 / 2);
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
  hipError_t e = hipMalloc(&b.p, nb);
  if (e == hipSuccess) b.bytes = nb;
  return e;
}

static uint32_t node_bits(uint64_t n) {
  uint32_t b = 1;
  while (b < 31 && (1ull << b) < n) ++b;
  return b;
}

}  // namespace

void overlay_free(OverlayWork* ws) {
  if (!ws) return;
  for (auto& b : ws->bucket)
    if (b.p) (void)hipFree(b.p);
  ws->bucket.clear();
  for (DevBuf* b : {&ws->scratch, &ws->outb, &ws->oslotb, &ws->heads, &ws->cub_tmp, &ws->meta}) {
    if (b->p) (void)hipFree(b->p);
    b->p = nullptr;
    b->bytes = 0;
  }
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
  if (p.R > kMaxRing) {
    res->rc = GS_EINVAL;
    snprintf(res->msg, sizeof(res->msg), "delayhigh %d exceeds the overlay ring limit %u",
             delay_high, kMaxRing);
    return res->rc;
  }
  const uint32_t R = p.R;
  // GS_OV_GROUP=1: k_process_g (A/B); default one lane per destination (k_process)
  static const bool group_env = [] { const char* e = getenv("GS_OV_GROUP"); return e && atoi(e) == 1; }();
  const bool grouped = group_env && p.B >= kOvGroupLog;
  // buffers live in the caller's workspace across builds (batched C3 builds
  // one overlay per batch; reallocating tens of GB per tick was the cost)
  if (ws->bucket.size() < R) ws->bucket.resize(R);
  std::vector<DevBuf>& bucket = ws->bucket;
  std::vector<uint64_t> fill(R, 0);
  DevBuf &scratch = ws->scratch, &outb = ws->outb, &oslotb = ws->oslotb, &heads = ws->heads,
         &cub_tmp = ws->cub_tmp, &meta = ws->meta;
  // meta layout: counts[R] | fill[R] | ptrs[R] | nheads | TickCounters
  uint64_t pending = 0, wm = 0, wb = 0;
  std::vector<unsigned long long> h_counts(R), hfill(R);
  std::vector<uint64_t*> h_ptrs(R, nullptr);
  unsigned long long *d_counts = nullptr, *d_fill = nullptr;
  uint64_t** d_ptrs = nullptr;
  int64_t* d_nheads = nullptr;
  TickCounters* d_tc = nullptr;
  TickCounters h_tc;
  const size_t meta_bytes = R * 8 * 3 + 64 + sizeof(TickCounters);

  OVCHK(grow(meta, meta_bytes));
  d_counts = (unsigned long long*)meta.p;
  d_fill = d_counts + R;
  d_ptrs = (uint64_t**)(d_fill + R);
  d_nheads = (int64_t*)(d_ptrs + R);
  d_tc = (TickCounters*)((char*)d_nheads + 64);
  OVCHK(hipMemsetAsync(meta.p, 0, meta_bytes, stream));

  {
    // ---- tick 0: picks (count, size buckets, write) --------------------
    const uint64_t items = n * (uint64_t)p.fanout * (trials > 1 ? trials : 1);
    if (items) {
      PickSource src{p, d_deg, d_ids, false};
      const uint64_t per = (uint64_t)kScatterBlock * kScatterIPT;
      const uint64_t blocks = (items + per - 1) / per;
      hipLaunchKernelGGL((k_scatter<false, PickSource>), dim3((uint32_t)blocks), dim3(kScatterBlock),
                         0, stream, src, items, R, d_counts, d_fill, (uint64_t* const*)d_ptrs);
      OVCHK(hipGetLastError());
      OVCHK(hipMemcpyAsync(h_counts.data(), d_counts, R * 8, hipMemcpyDeviceToHost, stream));
      OVCHK(hipStreamSynchronize(stream));
      for (uint32_t s = 0; s < R; ++s) {
        OVCHK(grow(bucket[s], (fill[s] + h_counts[s]) * 8));
        h_ptrs[s] = (uint64_t*)bucket[s].p;
      }
      OVCHK(hipMemcpyAsync(d_ptrs, h_ptrs.data(), R * 8, hipMemcpyHostToDevice, stream));
      src.write_rows = true;
      hipLaunchKernelGGL((k_scatter<true, PickSource>), dim3((uint32_t)blocks), dim3(kScatterBlock),
                         0, stream, src, items, R, d_counts, d_fill, (uint64_t* const*)d_ptrs);
      OVCHK(hipGetLastError());
      for (uint32_t s = 0; s < R; ++s) { fill[s] += h_counts[s]; pending += h_counts[s]; }
      OVCHK(hipMemsetAsync(d_counts, 0, R * 8, stream));
    } else if (ntot) {
      OVCHK(hipMemsetAsync(d_deg, 0, ntot, stream));
    }
  }

  for (uint64_t t = 1;; ++t) {
    if (t > max_ticks) {
      res->rc = GS_ELIVELOCK;
      snprintf(res->msg, sizeof(res->msg),
               "overlay did not stabilise within %llu ticks (fanin <= fanout livelocks, "
               "simulator.go:66-94)", (unsigned long long)max_ticks);
      goto cleanup;
    }
    const uint32_t s = (uint32_t)(t % R);
    const uint64_t m = fill[s];
    if (m) {
      if (m > 0x7FFFFFFFull) {
        res->rc = GS_EOVERFLOW;
        snprintf(res->msg, sizeof(res->msg), "%llu overlay events in one tick exceed 2^31-1",
                 (unsigned long long)m);
        goto cleanup;
      }
      OVCHK(grow(scratch, m * 8));
      OVCHK(grow(outb, m * 8));
      OVCHK(grow(oslotb, m * 2));
      OVCHK(grow(heads, m * 8));
      hipcub::DoubleBuffer<uint64_t> db((uint64_t*)bucket[s].p, (uint64_t*)scratch.p);
      // by destination group (grouped) or destination only (bits B+1 .. 2B):
      // the process kernel orders each destination's events by (src, kind)
      // itself
      const uint32_t glog = grouped ? kOvGroupLog : 0u;
      const int begin_bit = (int)(p.B + 1 + glog), end_bit = (int)(2 * p.B + 1);
      size_t sort_bytes = 0, sel_bytes = 0;
      OVCHK(hipcub::DeviceRadixSort::SortKeys(nullptr, sort_bytes, db, (int)m, begin_bit, end_bit, stream));
      IsHead pred{nullptr, p.B + 1 + glog};
      hipcub::CountingInputIterator<int64_t> it(0);
      OVCHK(hipcub::DeviceSelect::If(nullptr, sel_bytes, it, (int64_t*)heads.p, d_nheads, (int)m,
                                     pred, stream));
      OVCHK(grow(cub_tmp, std::max(sort_bytes, sel_bytes)));
      sort_bytes = cub_tmp.bytes;
      OVCHK(hipcub::DeviceRadixSort::SortKeys(cub_tmp.p, sort_bytes, db, (int)m, begin_bit, end_bit, stream));
      uint64_t* keys = db.Current();
      if (db.Current() != (uint64_t*)bucket[s].p) std::swap(bucket[s], scratch);
      pred.keys = keys;
      sel_bytes = cub_tmp.bytes;
      OVCHK(hipcub::DeviceSelect::If(cub_tmp.p, sel_bytes, it, (int64_t*)heads.p, d_nheads, (int)m,
                                     pred, stream));
      if (grouped) {
        const uint64_t ng = std::min<uint64_t>(m, (ntot >> kOvGroupLog) + 1);  // heads <= groups
        hipLaunchKernelGGL(k_process_g, dim3((uint32_t)((ng + kOvWaves - 1) / kOvWaves)), dim3(kOvWaves * 64), 0,
                           stream, p, (uint32_t)t, (const uint64_t*)keys, m, (const int64_t*)heads.p, d_nheads,
                           d_deg, d_ids, (uint64_t*)outb.p, (uint16_t*)oslotb.p, d_tc);
      } else {
        hipLaunchKernelGGL(k_process, dim3((uint32_t)((m + 255) / 256)), dim3(256), 0, stream, p,
                           (uint32_t)t, keys, m, (const int64_t*)heads.p, d_nheads, d_deg, d_ids,
                           (uint64_t*)outb.p, (uint16_t*)oslotb.p, d_tc);
      }
      OVCHK(hipGetLastError());
      OutSource osrc{(const uint64_t*)outb.p, (const uint16_t*)oslotb.p};
      const uint64_t per = (uint64_t)kScatterBlock * kScatterIPT;
      const uint32_t blocks = (uint32_t)((m + per - 1) / per);
      hipLaunchKernelGGL((k_scatter<false, OutSource>), dim3(blocks), dim3(kScatterBlock), 0, stream,
                         osrc, m, R, d_counts, d_fill, (uint64_t* const*)d_ptrs);
      OVCHK(hipGetLastError());
      OVCHK(hipMemcpyAsync(h_counts.data(), d_counts, R * 8, hipMemcpyDeviceToHost, stream));
      OVCHK(hipMemcpyAsync(&h_tc, d_tc, sizeof(h_tc), hipMemcpyDeviceToHost, stream));
      OVCHK(hipStreamSynchronize(stream));
      if (h_tc.err) {
        res->rc = (h_tc.err & 1) ? GS_EREJECT : GS_EINVAL;
        snprintf(res->msg, sizeof(res->msg), (h_tc.err & 1)
                     ? "replacement-friend rejection exhausted (n too small, simulator.go:87-89)"
                     : "too many overlay events at one node in one tick");
        goto cleanup;
      }
      // The current slot is consumed; emitted events never land in it.
      fill[s] = 0;
      pending -= m;
      bool moved = false;
      for (uint32_t q = 0; q < R; ++q) {
        if (!h_counts[q]) continue;
        if (bucket[q].bytes < (fill[q] + h_counts[q]) * 8) {
          DevBuf nb;
          OVCHK(grow(nb, (fill[q] + h_counts[q]) * 8 * 3 / 2));
          if (fill[q])
            OVCHK(hipMemcpyAsync(nb.p, bucket[q].p, fill[q] * 8, hipMemcpyDeviceToDevice, stream));
          OVCHK(hipStreamSynchronize(stream));
          (void)hipFree(bucket[q].p);
          bucket[q] = nb;
        }
      }
      for (uint32_t q = 0; q < R; ++q) {
        if (h_ptrs[q] != (uint64_t*)bucket[q].p) moved = true;
        h_ptrs[q] = (uint64_t*)bucket[q].p;
      }
      if (moved)
        OVCHK(hipMemcpyAsync(d_ptrs, h_ptrs.data(), R * 8, hipMemcpyHostToDevice, stream));
      {
        // hfill is rewritten only after the next tick's count sync, which
        // orders it after this copy: no host sync after the scatter
        hfill.assign(fill.begin(), fill.end());
        OVCHK(hipMemcpyAsync(d_fill, hfill.data(), R * 8, hipMemcpyHostToDevice, stream));
        hipLaunchKernelGGL((k_scatter<true, OutSource>), dim3(blocks), dim3(kScatterBlock), 0,
                           stream, osrc, m, R, d_counts, d_fill, (uint64_t* const*)d_ptrs);
        OVCHK(hipGetLastError());
      }
      for (uint32_t q = 0; q < R; ++q) { fill[q] += h_counts[q]; pending += h_counts[q]; }
      wm += h_tc.makeups;
      wb += h_tc.breakups;
      OVCHK(hipMemsetAsync(d_counts, 0, R * 8, stream));
      OVCHK(hipMemsetAsync(d_tc, 0, sizeof(TickCounters), stream));
    }
    if (t % 10 == 0) {                                        // simulator.go:222-234
      if (wm == 0 && wb == 0 && pending == 0) {
        res->final_tick = t;
        break;
      }
      if (sink.push) sink.push(sink.self, t, wm, wb);
      wm = wb = 0;
    }
  }

cleanup:
  (void)hipStreamSynchronize(stream);
  return res->rc;
}

}  // namespace gs
