// gs_broadcast.hip -- the broadcast round loop of simulator.go as gfx950 kernels.
//
// One tick (1 ms of simulated time) processes ring slot t mod R: every node
// whose Broadcast() delay expires at t (simulator.go:141-142) sends to each
// friend slot, dropping each send with the keyed RandomDrop (:143-147,
// :171-176); every receiver then runs the receive case of Node.Start
// (:107-123): crashed -> ignored; TotalMessage++; RandomCrash; first receipt
// -> received, TotalReceived++, Broadcast() (= schedule a fire bit at
// t + RandomNetworkDelay, :166-168).
//
// Work decomposition (per launch):
//   * only ACTIVE chunks (4096 nodes = 64 ring words) are visited: schedule()
//     appends a chunk to its slot's sharded list the first time the slot gets
//     a bit in it, so a tick costs O(frontier), not O(N);
//   * one wave per chunk: lane l loads ring word l (coalesced 512 B), the wave
//     compacts the set bits into an LDS list of firing nodes, then expands
//     (node, friend-slot) tasks 64 at a time so consecutive lanes read
//     consecutive ids of one friends row;
//   * counters are reduced wave -> LDS -> one atomic per block and field.
//
// Receipt semantics with crash% > 0 are made order-independent (DESIGN.md
// rule A6): pass COUNT sums the arrivals k at each node; pass RESOLVE lets the
// single lane whose atomicExch returns k > 0 replay ordinals 0..k-1 with the
// keyed crash rolls.  With crash% == 0 the FLOOD pass fuses delivery and
// infection into one atomicOr per delivered send.
#include "gs_internal.h"

namespace gs {

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Node.Broadcast() for node u infected at tick t: one delay per call
// (simulator.go:141-142), a fire bit in ring slot (t+off) mod R, and the
// chunk appended to that slot's active list on its first bit.
__device__ __forceinline__ void schedule(const DevState& st, uint32_t u, uint32_t t) {
  const uint32_t off = fire_offset(st.delay_low, st.delay_span, draw0(st.key, K_DELAY, u, t, 0));
  const uint32_t s = (t + off) % st.R;
  atomicOr(&st.ring[(size_t)s * st.W + (u >> 6)], 1ull << (u & 63));
  const uint32_t c = u >> kChunkNodesLog;
  uint32_t* fl = &st.cflag[(size_t)s * st.C + c];
  if (__hip_atomic_load(fl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u &&
      atomicExch(fl, 1u) == 0u) {
    const uint32_t sh = c & (kShards - 1);
    const uint32_t idx = atomicAdd(&st.ccount[(s * kShards + sh) * kCounterStride], 1u);
    st.clist[((size_t)s * kShards + sh) * st.CS + idx] = c;
  }
}

struct Counters {
  uint32_t v[6];
};

// Receive case of Node.Start for node u with k arrivals this tick, `ones` of
// them carrying a crash roll (simulator.go:107-123, rule A6: first_crash).
__device__ __forceinline__ void resolve_node(const DevState& st, uint32_t u, uint32_t k, uint32_t ones,
                                             uint32_t t, Counters& c) {
  const unsigned long long bit = 1ull << (u & 63);
  if (st.crash[u >> 6] & bit) return;                     // :108 (not counted)
  const uint32_t g = ones ? first_crash(u, t, k, ones, ctr3(K_ORDER, st.key.trial), st.key.k0, st.key.k1)
                          : k + 1;
  c.v[ST_MSGS] += g <= k ? g : k;                         // :111
  if (g > 1 && !(st.recv[u >> 6] & bit)) {                // :117
    atomicOr(&st.recv[u >> 6], bit);                      // :120
    c.v[ST_RECV]++;                                       // :121
    schedule(st, u, t);                                   // :122
    c.v[ST_SCHED]++;
  }
  if (g <= k) {                                           // :112-115
    atomicOr(&st.crash[u >> 6], bit);
    c.v[ST_CRASH]++;
  }
}

template <int MODE, bool CHECK_CRASHED>
__device__ __forceinline__ void process_chunk(const DevState& st, uint32_t t, uint32_t slot,
                                              uint32_t chunk, uint32_t* list, uint32_t lane,
                                              Counters& c) {
  const uint64_t wi = ((uint64_t)chunk << 6) + lane;
  unsigned long long* wp = &st.ring[(size_t)slot * st.W + wi];
  unsigned long long bits = wi < st.W ? *wp : 0ull;
  if (MODE != MODE_COUNT) {
    if (bits) *wp = 0ull;                                 // slot reused at t + R
    if (lane == 0) st.cflag[(size_t)slot * st.C + chunk] = 0u;
    if (chunk >= st.chunk_lo && chunk < st.chunk_hi) c.v[ST_FIRED] += __popcll(bits);
  }
  const uint32_t S = st.stride;
  const uint32_t node0 = (chunk << kChunkNodesLog) + (lane << 6);
  const uint32_t c3drop = ctr3(K_DROP, st.key.trial);
  while (__ballot(bits != 0ull)) {
    // Compact up to kListCap firing nodes of this chunk into LDS.
    const uint32_t cntb = __popcll(bits);
    uint32_t x = cntb;
#pragma unroll
    for (uint32_t d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d, 64);
      if (lane >= d) x += y;
    }
    const uint32_t total = __shfl(x, 63, 64);
    uint32_t pos = x - cntb;
    while (bits && pos < kListCap) {
      list[pos++] = node0 + (uint32_t)__builtin_ctzll(bits);
      bits &= bits - 1;
    }
    wave_sync();
    const uint32_t L = total < kListCap ? total : kListCap;
    const uint32_t tasks = L * S;
    for (uint32_t q = lane; q < tasks; q += kWave) {
      const uint32_t ni = __umulhi(q, st.stride_magic);
      const uint32_t j = q - ni * S;
      const uint32_t v = list[ni];
      if (j >= st.deg[v]) continue;
      // RandomDrop per friend slot (simulator.go:144, :172)
      const u32x4 r = philox(v, t, j >> 2, c3drop, st.key.k0, st.key.k1);
      uint32_t dropd, crashd;  // the drop draw and the message's crash roll (:180)
      drop_crash(lane_of(r, j & 3), dropd, crashd);
      if ((int32_t)dropd < st.kd) continue;
      const uint32_t u = st.ids[(size_t)v * S + j];        // GlobalView[id] (:145)
      if (u < st.lo || u >= st.hi) continue;               // another shard's target
      if (MODE == MODE_FLOOD) {
        c.v[ST_SENT]++;
        const unsigned long long bit = 1ull << (u & 63);
        if (CHECK_CRASHED && (st.crash[u >> 6] & bit)) continue;
        c.v[ST_MSGS]++;
        const unsigned long long old = atomicOr(&st.recv[u >> 6], bit);
        if (!(old & bit)) {
          c.v[ST_RECV]++;
          schedule(st, u, t);
          c.v[ST_SCHED]++;
        }
      } else if (MODE == MODE_COUNT) {
        c.v[ST_SENT]++;
        // the message's crash roll (:180), from its drop draw's second base-100 digit
        const uint32_t roll = (int32_t)crashd < st.kc;
        // receipts | crash rolls << 16: the receipt count is 16 bits, so the
        // 65536th arrival at one node in one tick is an overflow (GS_EOVERFLOW)
        const uint32_t old = atomicAdd(&st.cnt[u], 1u + (roll << 16));
        if ((old & 0xFFFFu) == 0xFFFFu) atomicOr(st.err, kErrArrivals);
      } else {
        const uint32_t k = atomicExch(&st.cnt[u], 0u);
        if (k) resolve_node(st, u, k & 0xFFFFu, k >> 16, t, c);
      }
    }
    wave_sync();
  }
}

template <int MODE, bool CHECK_CRASHED>
__global__ __launch_bounds__(kTickBlock) void k_tick(const DevState st, uint32_t t) {
  __shared__ uint32_t s_list[kTickBlock / kWave][kListCap];
  __shared__ uint32_t s_pref[kShards + 1];
  __shared__ unsigned long long s_red[kTickBlock / kWave][6];
  const uint32_t slot = t % st.R;
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (threadIdx.x < kShards)
    s_pref[threadIdx.x + 1] = st.ccount[(slot * kShards + threadIdx.x) * kCounterStride];
  __syncthreads();
  if (threadIdx.x == 0) {
    s_pref[0] = 0;
    for (uint32_t i = 0; i < kShards; ++i) s_pref[i + 1] += s_pref[i];
  }
  __syncthreads();
  // Sharded runs visit every chunk: the slot was overwritten by the frontier
  // all-gather, so this rank's active-chunk list does not cover it.
  const uint32_t total = st.sharded ? st.C : s_pref[kShards];
  Counters c{};
  const uint32_t wpb = kTickBlock / kWave;
  for (uint32_t g = blockIdx.x * wpb + wid; g < total; g += gridDim.x * wpb) {
    uint32_t chunk = g;
    if (!st.sharded) {
      uint32_t sh = 0;
      while (s_pref[sh + 1] <= g) ++sh;
      chunk = st.clist[((size_t)slot * kShards + sh) * st.CS + (g - s_pref[sh])];
    }
    process_chunk<MODE, CHECK_CRASHED>(st, t, slot, chunk, s_list[wid], lane, c);
  }
  // wave -> LDS -> one atomic per block and field
#pragma unroll
  for (int f = 0; f < 6; ++f) {
    unsigned long long x = c.v[f];
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
    if (lane == 0) s_red[wid][f] = x;
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    unsigned long long s = 0;
    for (uint32_t w = 0; w < wpb; ++w) s += s_red[w][threadIdx.x];
    if (s) atomicAdd(&st.stats[(size_t)(t % kStatSlots) * kStatFields + threadIdx.x], s);
  }
}

__global__ void k_slot_reset(uint32_t* ccount, uint32_t slot) {
  if (threadIdx.x < kShards) ccount[(slot * kShards + threadIdx.x) * kCounterStride] = 0u;
}

__global__ void k_schedule_one(const DevState st, uint32_t node, uint32_t tick) {
  if (threadIdx.x == 0 && blockIdx.x == 0) schedule(st, node, tick);
}

uint32_t tick_grid(const DevState& st) {
  const uint32_t wpb = kTickBlock / kWave;
  uint32_t g = (st.C + wpb - 1) / wpb;
  if (g > kTickGridMax) g = kTickGridMax;
  return g ? g : 1;
}

hipError_t launch_tick(const DevState& st, uint32_t tick, int mode, hipStream_t s) {
  const dim3 grid(tick_grid(st)), block(kTickBlock);
  switch (mode) {
    case MODE_FLOOD:
      if (st.check_crashed)
        hipLaunchKernelGGL((k_tick<MODE_FLOOD, true>), grid, block, 0, s, st, tick);
      else
        hipLaunchKernelGGL((k_tick<MODE_FLOOD, false>), grid, block, 0, s, st, tick);
      break;
    case MODE_COUNT:
      hipLaunchKernelGGL((k_tick<MODE_COUNT, false>), grid, block, 0, s, st, tick);
      break;
    default:
      hipLaunchKernelGGL((k_tick<MODE_RESOLVE, false>), grid, block, 0, s, st, tick);
      break;
  }
  return hipGetLastError();
}

hipError_t launch_slot_reset(const DevState& st, uint32_t slot, hipStream_t s) {
  hipLaunchKernelGGL(k_slot_reset, dim3(1), dim3(64), 0, s, st.ccount, slot);
  return hipGetLastError();
}

hipError_t launch_schedule_one(const DevState& st, uint32_t node, uint32_t tick, hipStream_t s) {
  hipLaunchKernelGGL(k_schedule_one, dim3(1), dim3(64), 0, s, st, node, tick);
  return hipGetLastError();
}

}  // namespace gs
