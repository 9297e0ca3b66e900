// gs_pushpull.hip -- push-pull gossip rounds (extension, config C5).
//
// The reference only floods (simulator.go:140-149: every receipt re-broadcasts
// to every friend).  Config C5 asks for push-pull gossip as well; it has no
// reference semantics, so the model is the one oracle/gsoracle.h states (and
// DESIGN.md section 4.5): one tick = one synchronous round; every live node v with a
// non-empty friends list draws r = Philox{v, t, 0, PUSHPULL}, calls
// u = friends[v][U_deg(r.x)], and the call is lost iff U_100(r.y) < kd
// (the -droprate quantisation of simulator.go:172).  With I = informed set at
// the start of the round: v in I pushes to u (u informed iff live); v not in I
// pulls from u in I.  Failed nodes (gs_set_failed) never call or answer.
//
// Layout: one lane per node, one wave per 64-bit word of the bitsets, so a
// wave's pulls land in its own word with one atomicOr of the ballot.  Pushes
// scatter into `next` (atomicOr, only when u is neither informed nor failed);
// `next` starts every round equal to `recv`, and k_pp_commit makes
// recv = next and counts the newly informed.  Per round at N = 1e9: the
// friends table is streamed once (a wave's 64 rows are contiguous), the
// 125-MB recv bitset is gathered once per call (Infinity-Cache resident).
// Word summaries (k_pp_summary, one bit per 64-node word, 2 MB each, L2
// resident) skip that gather where its answer is known: a pull from a word
// with no informed node fails, and a push into a word with no live
// uninformed node changes nothing (without a failed mask).  A second level
// (k_pp_summary2, one bit per 4096-node block, 61 KB at N = 1e9) sits in LDS
// in front of them, so the early and late rounds, where almost every call is
// decided by the summaries, cost the table stream only.
#include <algorithm>
#include <vector>

#include <hipcub/hipcub.hpp>

#include "gs_internal.h"

namespace gs {
namespace {

constexpr uint32_t kPPBlock = 256;

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (uint32_t o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Per-block sums of up to 3 counters into stats[slot][f0..], one atomic each.
template <uint32_t B = kPPBlock>
__device__ __forceinline__ void block_add(uint64_t* sh, const uint64_t (&v)[3], uint32_t nf,
                                          unsigned long long* row, const uint32_t (&fld)[3]) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid < 3 * (B / 64)) sh[tid] = 0;
  __syncthreads();
  for (uint32_t i = 0; i < nf; ++i) {
    const uint64_t s = wave_sum64(v[i]);
    if (lane == 0) sh[i * (B / 64) + wv] = s;
  }
  __syncthreads();
  if (tid < nf) {
    uint64_t s = 0;
    for (uint32_t k = 0; k < B / 64; ++k) s += sh[tid * (B / 64) + k];
    if (s) atomicAdd(&row[fld[tid]], (unsigned long long)s);
  }
}

// sumA bit w = recv word w has an informed node; sumB bit w = it has a node
// that is neither informed nor failed (bits past n count as such: the
// summary only ever skips work whose outcome it proves).
__global__ __launch_bounds__(kPPBlock) void k_pp_summary(const DevState s, unsigned long long* __restrict__ sumA,
                                                         unsigned long long* __restrict__ sumB, const PPCtl* ctl) {
  if (ctl && ctl->mode != PP_DENSE) return;
  const uint64_t Wr = (s.W + 63) & ~63ull;  // whole waves stay in the loop together
  for (uint64_t w = (uint64_t)blockIdx.x * kPPBlock + threadIdx.x; w < Wr;
       w += (uint64_t)gridDim.x * kPPBlock) {
    unsigned long long r = 0, f = ~0ull;
    if (w < s.W) { r = s.recv[w]; f = s.crash[w]; }
    const unsigned long long a = __ballot(r != 0), b = __ballot(w < s.W && (r | f) != ~0ull);
    if ((threadIdx.x & 63) == 0) { sumA[w >> 6] = a; sumB[w >> 6] = b; }
  }
}

// Each wave owns kPPU consecutive bitset words per pass and issues the loads
// of all of them phase by phase (state words + deg, then the friend id, then
// the peer word's summary, then the peer-word gathers), so kPPU independent
// dependency chains are in flight per wave: one word per pass left the launch
// bound by the chain's latency (8.8 ms per round with no gathers at all).
constexpr uint32_t kPPU = 8;

// Second level: bit j of sumA2/sumB2 = summary word j of sumA/sumB is non-zero.
__global__ __launch_bounds__(kPPBlock) void k_pp_summary2(const unsigned long long* __restrict__ sum1, uint64_t S1,
                                                          unsigned long long* __restrict__ sum2, uint64_t S2,
                                                          const PPCtl* ctl) {
  if (ctl && ctl->mode != PP_DENSE) return;
  const uint64_t Sr = (S1 + 63) & ~63ull;
  for (uint64_t j = (uint64_t)blockIdx.x * kPPBlock + threadIdx.x; j < Sr; j += (uint64_t)gridDim.x * kPPBlock) {
    const bool in = j < S1;
    const unsigned long long a = __ballot(in && sum1[j] != 0), b = __ballot(in && sum1[S1 + j] != 0);
    if ((threadIdx.x & 63) == 0) { sum2[j >> 6] = a; sum2[S2 + (j >> 6)] = b; }
  }
}

// The second-level summaries (2 x S2 words, 61 KB at N = 1e9) are staged in
// LDS when they fit (S2 > 0): a call whose peer's 4096-node block has no
// informed node (pull) or no live uninformed node (push) then skips the L2
// summary load too.  Persistent 1024-thread blocks, two per CU.
constexpr uint32_t kPPRoundBlock = 1024;
constexpr uint64_t kPPMaxS2 = 4000;  // 2 x 31.25 KB of dynamic LDS (under the 64 KB default)

__global__ __launch_bounds__(kPPRoundBlock) void k_pp_round(const DevState s,
                                                            unsigned long long* __restrict__ next,
                                                            const unsigned long long* __restrict__ sumA,
                                                            const unsigned long long* __restrict__ sumB,
                                                            const unsigned long long* __restrict__ sum2,
                                                            uint32_t S2, uint32_t t, const PPCtl* ctl,
                                                            const uint8_t* __restrict__ fmask) {
  __shared__ uint64_t sh[3 * (kPPRoundBlock / 64)];
  extern __shared__ unsigned long long l2sum[];  // [0,S2) A2, [S2,2*S2) B2
  if (ctl && ctl->mode != PP_DENSE) return;
  for (uint32_t j = threadIdx.x; j < 2 * S2; j += kPPRoundBlock) l2sum[j] = sum2[j];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t c3 = ctr3(K_PUSHPULL, s.key.trial);
  const bool cc = s.check_crashed;
  uint64_t fired = 0, sent = 0, msgs = 0;
  const uint64_t W = (s.n + 63) >> 6;
  const uint64_t wid = (uint64_t)blockIdx.x * (kPPRoundBlock / 64) + (threadIdx.x >> 6);
  const uint64_t step = (uint64_t)gridDim.x * (kPPRoundBlock / 64) * kPPU;
  for (uint64_t w0 = wid * kPPU; w0 < W; w0 += step) {  // wave-uniform
    unsigned long long Iw[kPPU], Fw[kPPU];
    uint32_t d[kPPU], u[kPPU], fm[kPPU];
    bool push[kPPU], kept[kPPU], sbit[kPPU];
#pragma unroll
    for (uint32_t i = 0; i < kPPU; ++i) {
      const uint64_t word = w0 + i, v = (word << 6) + lane;
      const bool inb = word < W;
      Iw[i] = inb ? s.recv[word] : 0ull;
      Fw[i] = inb ? s.crash[word] : ~0ull;
      d[i] = v < s.n ? s.deg[v] : 0u;
      fm[i] = fmask && v < s.n ? fmask[v] : 0u;
    }
#pragma unroll
    for (uint32_t i = 0; i < kPPU; ++i) {
      const uint64_t v = ((w0 + i) << 6) + lane;
      if ((Fw[i] >> lane) & 1) d[i] = 0;  // failed (or past the table): never calls
      push[i] = (Iw[i] >> lane) & 1;
      u[i] = 0;
      kept[i] = false;
      if (d[i] > 0) {
        const u32x4 r = philox((uint32_t)v, t, 0, c3, s.key.k0, s.key.k1);
        const uint32_t j = uniform(r.x, d[i]);
        u[i] = s.ids[v * s.stride + j];
        fm[i] = (fm[i] >> j) & 1;  // the picked friend is failed (fmask)
        kept[i] = (int32_t)uniform(r.y, 100u) >= s.kd;
      }
    }
    // summaries (L2 resident): push -> u's word has a live uninformed node;
    // pull -> u's word has an informed node.  A dropped call needs neither.
#pragma unroll
    for (uint32_t i = 0; i < kPPU; ++i) {
      sbit[i] = false;
      if (kept[i]) {
        const bool top = S2 == 0 || ((l2sum[(push[i] ? S2 : 0u) + (u[i] >> 18)] >> ((u[i] >> 12) & 63)) & 1);
        if (top) sbit[i] = ((push[i] ? sumB : sumA)[u[i] >> 12] >> ((u[i] >> 6) & 63)) & 1;
      }
    }
    unsigned long long Iu[kPPU], Cu[kPPU];
#pragma unroll
    for (uint32_t i = 0; i < kPPU; ++i) {
      // pulls gather the peer's word; a push needs no gather (its atomicOr
      // below is idempotent and returns nothing, so the wave does not wait)
      Iu[i] = (sbit[i] && !push[i]) ? s.recv[u[i] >> 6] : 0ull;
      // the failed-mask gather only when a mask was set (gs_set_failed) and
      // no per-node failed-slot mask replaces it
      Cu[i] = (cc && !fmask && kept[i] && push[i]) ? s.crash[u[i] >> 6]
              : (fm[i] ? (1ull << (u[i] & 63)) : 0ull);
    }
#pragma unroll
    for (uint32_t i = 0; i < kPPU; ++i) {
      const unsigned long long ubit = 1ull << (u[i] & 63);
      bool pulled = false;
      if (d[i] > 0) ++fired;
      if (kept[i]) {
        if (push[i]) {
          ++sent;
          if (!(Cu[i] & ubit)) {  // u live: delivered
            ++msgs;
            // sbit clear: every live node of u's word is informed already
            if (sbit[i]) atomicOr(&next[u[i] >> 6], ubit);
          }
        } else if (Iu[i] & ubit) {  // pull from an informed u (u informed => u live)
          ++sent;
          ++msgs;
          pulled = true;
        }
      }
      const unsigned long long bal = __ballot(pulled);
      if (lane == 0 && bal) atomicOr(&next[w0 + i], bal);
    }
  }
  const uint64_t v3[3] = {fired, sent, msgs};
  const uint32_t f3[3] = {ST_FIRED, ST_SENT, ST_MSGS};
  block_add<kPPRoundBlock>(sh, v3, 3, s.stats + (size_t)(t % kStatSlots) * kStatFields, f3);
}

// Bottom-up dense round (PPMode PP_BOTTOM, gs_internal.h).  Same draws,
// outcomes and counters as k_pp_round.  A wave owns ranges of kPPRange words
// (4096 nodes) and streams them a lane per node: an informed caller counts
// its push (sent; msgs unless fmask marks the picked friend failed) and reads
// nothing else; an uninformed live node joins the wave's LDS queue.  Each 64
// queued nodes are resolved together, a lane each: the pull (friend id + the
// friend's recv word) and the push receipts, found among the node's in-edges
// (v, j) -- v's pick is recomputed from the packed slot byte (no deg gather),
// and only a kept pick of slot j costs a gather of v's recv word.  So the
// dependent-load chain runs for full waves of uninformed nodes however few
// are left, and the range's newly informed gather in LDS and are stored, not
// OR'ed (the wave owns its words).
#ifndef GS_PPB
#define GS_PPB 8
#endif
constexpr uint32_t kPPB = GS_PPB;   // words loaded together while streaming
constexpr uint32_t kPPRange = 64;   // words per wave range (multiple of kPPB)
constexpr uint32_t kPPQ = 128;      // queue entries per wave (<= 63 left + 64 appended)
constexpr uint32_t kPPEdges = 4;    // in-edges loaded per batch
#ifndef GS_PPS_BLOCK
#define GS_PPS_BLOCK 1024
#endif
constexpr uint32_t kPPSBlock = GS_PPS_BLOCK;  // k_ppb_round / k_ppa_round workgroup
constexpr uint32_t kPPWaves = kPPSBlock / 64;
constexpr uint32_t kPPSGrid = 512 * 1024 / kPPSBlock;  // at most 8192 waves per launch

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Position of the k-th set bit of m (k < popc(m)).
__device__ __forceinline__ uint32_t nth_bit(unsigned long long m, uint32_t k) {
  uint32_t pos = 0, x = (uint32_t)m, c = (uint32_t)__popc(x);
  if (k >= c) { k -= c; x = (uint32_t)(m >> 32); pos = 32; }
  c = (uint32_t)__popc(x & 0xFFFFu);
  if (k >= c) { k -= c; x >>= 16; pos += 16; }
  c = (uint32_t)__popc(x & 0xFFu);
  if (k >= c) { k -= c; x >>= 8; pos += 8; }
  c = (uint32_t)__popc(x & 0xFu);
  if (k >= c) { k -= c; x >>= 4; pos += 4; }
  c = (uint32_t)__popc(x & 0x3u);
  if (k >= c) { k -= c; x >>= 2; pos += 2; }
  return pos + (k >= (x & 1u) ? 1u : 0u);
}

// The set bits of a wave's 64 words (lane l holds the mask of word l of the
// range), in node order, 64 at a time: f(cnt, off) runs wave-wide with lane
// j < cnt holding the node offset (word * 64 + bit) of the next bit.  A wave
// scan of the popcounts, then a binary search of the lane's word in LDS (pre:
// 64 u32, msk: 64 u64 of the wave) and the bit's rank inside it: the queue of
// a range is its nodes in order, so a 64-node batch touches few lines of the
// in-edge lists and of the degree bytes.
template <class F>
__device__ __forceinline__ void for_each_bit(unsigned long long m, uint32_t* pre, unsigned long long* msk, F&& f) {
  const uint32_t lane = threadIdx.x & 63, c = (uint32_t)__popcll(m);
  uint32_t x = c;
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
    if (lane >= o) x += y;
  }
  const uint32_t total = (uint32_t)__shfl((int)x, 63, 64);
  if (!total) return;
  pre[lane] = x - c;
  msk[lane] = m;
  wave_lds_sync();
  for (uint32_t p0 = 0; p0 < total; p0 += 64) {
    const uint32_t p = p0 + lane;
    uint32_t off = 0;
    if (p < total) {
      uint32_t lo = 0, hi = 63;  // the last word whose first bit ranks <= p
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (pre[mid] <= p) lo = mid; else hi = mid - 1;
      }
      off = (lo << 6) + nth_bit(msk[lo], p - pre[lo]);
    }
    f(min(64u, total - p0), off);
  }
  wave_lds_sync();  // pre / msk are reused by the next range
}

// Node u's in-edges [qb, qe): from the compact view (PPSparse::rend16 /
// rbase: the dense rounds read 2 B per node of it instead of 8 of rend, and
// they read it for most nodes) or from rend.
__device__ __forceinline__ void in_edges(const PPSparse& sp, uint64_t u, unsigned long long& qb,
                                         unsigned long long& qe) {
  if (sp.rend16) {
    const unsigned long long b = sp.rbase[u >> 6];
    qb = b + ((u & 63) ? (unsigned long long)sp.rend16[u - 1] : 0ull);
    qe = b + sp.rend16[u];
  } else {
    qb = u ? sp.rend[u - 1] : 0ull;
    qe = sp.rend[u];
  }
}

// Resolves queue entries [0, cnt) (cnt <= 64), one per lane.  Entry = node
// offset in the range (12 bits) | deg << 16.
__device__ __forceinline__ void ppb_resolve(const DevState& s, const PPSparse& sp, uint32_t t, uint32_t c3,
                                            const uint32_t* q, uint32_t cnt, uint64_t base,
                                            unsigned long long* nb, uint64_t& sent, uint64_t& msgs) {
  const uint32_t lane = threadIdx.x & 63;
  if (lane >= cnt) return;
  const uint32_t e = q[lane], loc = e & 0xFFFu, d = e >> 16;
  const uint64_t v = base + loc;  // local id (global s.gbase + v)
  unsigned long long qb, qe;
  in_edges(sp, v, qb, qe);
  bool pull = false;
  uint32_t u = 0;
  if (d > 0) {
    const u32x4 r = philox((uint32_t)(s.gbase + v), t, 0, c3, s.key.k0, s.key.k1);
    if ((int32_t)uniform(r.y, 100u) >= s.kd) {
      u = s.ids[v * s.stride + uniform(r.x, d)];
      pull = true;
    }
  }
  const unsigned long long Iu = pull ? s.grecv[u >> 6] : 0ull;  // u is a global id
  const bool pulled = pull && ((Iu >> (u & 63)) & 1);  // u informed => u live
  // a node its own pull informs needs no push receipt (sp.pullfirst: the
  // in-edge scan waits for the pull's two dependent loads, and skips)
  bool got = sp.pullfirst && pulled;
  for (unsigned long long q0 = qb; q0 < qe && !got; q0 += kPPEdges) {
    uint32_t src[kPPEdges], x[kPPEdges];
#pragma unroll
    for (uint32_t k = 0; k < kPPEdges; ++k) {
      const bool in = q0 + k < qe;
      src[k] = in ? sp.rsrc[q0 + k] : 0u;
      x[k] = in ? sp.rslot[q0 + k] : 0u;
    }
#pragma unroll
    for (uint32_t k = 0; k < kPPEdges; ++k) {
      if (q0 + k >= qe) break;
      const u32x4 r = philox(src[k], t, 0, c3, s.key.k0, s.key.k1);
      if (uniform(r.x, (x[k] >> 4) + 1) == (x[k] & 15u) && (int32_t)uniform(r.y, 100u) >= s.kd)
        got |= ((s.grecv[src[k] >> 6] >> (src[k] & 63)) & 1) != 0;
    }
  }
  if (pulled) {
    ++sent;
    ++msgs;
  }
  if (pulled || got) atomicOr(&nb[loc >> 6], 1ull << (loc & 63));
}

__global__ __launch_bounds__(kPPSBlock) void k_ppb_round(const DevState s, unsigned long long* __restrict__ next,
                                                             const PPSparse sp, uint32_t t) {
  __shared__ uint64_t sh[3 * kPPWaves];
  __shared__ uint32_t s_q[kPPWaves][kPPQ];
  __shared__ unsigned long long s_nb[kPPWaves][kPPRange];
  __shared__ uint32_t s_pre[kPPWaves][64];
  __shared__ unsigned long long s_msk[kPPWaves][64];
  if (sp.ctl->mode != PP_BOTTOM) return;
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t* q = s_q[wv];
  unsigned long long* nb = s_nb[wv];
  const uint32_t c3 = ctr3(K_PUSHPULL, s.key.trial);
  const uint8_t* __restrict__ fmask = sp.fmask;
  uint64_t fired = 0, sent = 0, msgs = 0;
  const uint64_t W = (s.n + 63) >> 6;
  const uint64_t nrange = (W + kPPRange - 1) / kPPRange;
  // every live node calls (no empty rows) and no failed-slot mask: an
  // informed caller's push needs only its loss draw (sent = delivered), so
  // its degree byte is not loaded -- in the late rounds, nearly every node's
  const bool nodeg = sp.ctl->nlive0 == 0 && !fmask && sp.nodeg;
  // GS_PPB_WORDS (A/B): 0 a lane per node throughout, 1 a lane per word, 2 a
  // lane per word where no word holds more than sp.word_maxu live uninformed
  // nodes (default; 64, i.e. always)
  const uint32_t ppb_words = sp.words;
  // lane-per-word ranges: every live node calls, and a failed-slot mask (if
  // any) has its has-a-failed-friend bits
  const bool wordok = sp.ctl->nlive0 == 0 && sp.nodeg && (!fmask || sp.fany);
  for (uint64_t rg = (uint64_t)blockIdx.x * kPPWaves + wv; rg < nrange; rg += (uint64_t)gridDim.x * kPPWaves) {
    const uint64_t w0 = rg * kPPRange, base = w0 << 6;
    nb[lane] = 0;
    uint32_t qn = 0;  // wave-uniform
    bool by_word = false;
    const uint64_t word = w0 + lane;
    unsigned long long mi = 0, mu = 0;
    if (wordok && ppb_words) {
      if (word < W) {
        const uint64_t left = s.n - (word << 6);
        const unsigned long long valid = left >= 64 ? ~0ull : ((1ull << left) - 1);
        const unsigned long long Iw = s.recv[word], Fw = s.crash[word];
        mi = Iw & ~Fw & valid;
        mu = ~Iw & ~Fw & valid;
      }
      uint32_t mx = (uint32_t)__popcll(mu);  // the most live uninformed nodes of one word
#pragma unroll
      for (uint32_t o = 32; o >= 1; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor(mx, o, 64));
      by_word = ppb_words == 1 || mx <= sp.word_maxu;
    }
    if (by_word) {
      // a lane per WORD of the range: an informed caller costs its loss draw
      // and a bit scan, no per-node load, ballot or queue step (the late
      // rounds, where nearly every caller is informed, are VALU-bound); the
      // range's live uninformed nodes are resolved 64 at a time in node order
      // (for_each_bit)
      fired += (uint64_t)(__popcll(mi) + __popcll(mu));  // nodeg: every live node calls
      const uint32_t vb = (uint32_t)(s.gbase + (word << 6));
      unsigned long long mf = fmask && word < W ? sp.fany[word] & mi : 0ull;
      uint32_t pushed = 0, dead = 0;
      while (mi) {
        const uint32_t b = (uint32_t)__builtin_ctzll(mi);
        mi &= mi - 1;
        const u32x4 r = philox(vb + b, t, 0, c3, s.key.k0, s.key.k1);
        pushed += (int32_t)uniform(r.y, 100u) >= s.kd ? 1u : 0u;
      }
      // callers with a failed friend (a push to it is sent, not delivered): a
      // second pass with their draws made again, so the loop above never waits
      // for a degree or mask byte (one of ~17 callers at 1 % failed, but in
      // nearly every step of a 64-lane wave)
      while (mf) {
        const uint32_t b = (uint32_t)__builtin_ctzll(mf);
        mf &= mf - 1;
        const uint64_t v = (word << 6) + b;
        const uint32_t fm = fmask[v], d = s.deg[v];
        const u32x4 r = philox(vb + b, t, 0, c3, s.key.k0, s.key.k1);
        if ((int32_t)uniform(r.y, 100u) >= s.kd) dead += (fm >> uniform(r.x, d)) & 1;
      }
      sent += pushed;
      msgs += pushed - dead;
      for_each_bit(mu, s_pre[wv], s_msk[wv], [&](uint32_t cnt, uint32_t off) {
        q[lane] = lane < cnt ? off | (uint32_t)s.deg[base + off] << 16 : 0u;
        wave_lds_sync();
        ppb_resolve(s, sp, t, c3, q, cnt, base, nb, sent, msgs);
        wave_lds_sync();
      });
    }
    for (uint32_t wi = 0; wi < kPPRange && !by_word; wi += kPPB) {
      unsigned long long Iw[kPPB];
      uint32_t d[kPPB], fm[kPPB];
      bool live[kPPB];
#pragma unroll
      for (uint32_t i = 0; i < kPPB; ++i) {
        const uint64_t word = w0 + wi + i, v = (word << 6) + lane;
        const bool inb = word < W;
        Iw[i] = inb ? s.recv[word] : ~0ull;
        const unsigned long long Fw = inb ? s.crash[word] : ~0ull;
        live[i] = v < s.n && !((Fw >> lane) & 1);
        d[i] = live[i] && !(nodeg && ((Iw[i] >> lane) & 1)) ? s.deg[v] : (live[i] ? 1u : 0u);
        fm[i] = fmask && live[i] ? fmask[v] : 0u;
      }
#pragma unroll
      for (uint32_t i = 0; i < kPPB; ++i) {
        const uint64_t v = ((w0 + wi + i) << 6) + lane;
        const bool inf = (Iw[i] >> lane) & 1;
        if (d[i] > 0) {
          ++fired;
          if (inf) {  // push: the receiver finds it
            const u32x4 r = philox((uint32_t)(s.gbase + v), t, 0, c3, s.key.k0, s.key.k1);
            if ((int32_t)uniform(r.y, 100u) >= s.kd) {
              ++sent;
              if (!((fm[i] >> uniform(r.x, d[i])) & 1)) ++msgs;
            }
          }
        }
        const bool enq = live[i] && !inf;
        const unsigned long long bal = __ballot(enq);
        if (enq) {
          const uint32_t at = qn + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
          q[at] = (uint32_t)(v - base) | d[i] << 16;
        }
        qn += (uint32_t)__popcll(bal);
        if (qn >= 64) {
          wave_lds_sync();
          ppb_resolve(s, sp, t, c3, q, 64, base, nb, sent, msgs);
          const uint32_t rest = qn - 64;
          const uint32_t keep = lane < rest ? q[64 + lane] : 0u;
          wave_lds_sync();
          if (lane < rest) q[lane] = keep;
          qn = rest;
        }
      }
    }
    wave_lds_sync();
    if (qn) ppb_resolve(s, sp, t, c3, q, qn, base, nb, sent, msgs);
    wave_lds_sync();
    const unsigned long long x = nb[lane];
    if (x && word < W) next[word] = s.recv[word] | x;
    wave_lds_sync();  // nb and q are reused by the next range
  }
  const uint64_t v3[3] = {fired, sent, msgs};
  const uint32_t f3[3] = {ST_FIRED, ST_SENT, ST_MSGS};
  block_add<kPPSBlock>(sh, v3, 3, s.stats + (size_t)(t % kStatSlots) * kStatFields, f3);
}

// Pull-answer round (PP_ANSWER): same draws, outcomes and counters as
// k_pp_round.  A wave streams ranges of kPPRange words, a lane per node, and
// queues its INFORMED nodes in LDS; each 64 queued nodes are resolved
// together, a lane each: the node's own call (a push, as top-down: one
// no-return atomicOr into its friend's word unless the friend is failed) and
// the pulls it answers -- its in-edges (v, j) whose caller v picks slot j
// (recomputed from the packed slot byte) and is not lost; only such an
// in-edge costs a gather of v's recv / failed words (v must be live and
// uninformed: its call is a pull from this informed node, counted here).
// Every live caller is counted as fired from ctl->ncallers.
// Node x is informed this round: appended to this workgroup's deferred list
// (the active lanes with `take`, one LDS atomic per wave and call), or, with
// no deferred buffers or a full list, an atomicOr into next.
__device__ __forceinline__ void pp_set(const PPSparse& sp, unsigned long long* __restrict__ next, bool take,
                                       uint32_t x, uint32_t* s_dn) {
  if (!sp.dset) {
    if (take) atomicOr(&next[x >> 6], 1ull << (x & 63));
    return;
  }
  const unsigned long long act = __ballot(1), bal = __ballot(take);
  if (!bal) return;
  const uint32_t lane = threadIdx.x & 63, leader = (uint32_t)__ffsll((long long)act) - 1;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(s_dn, (uint32_t)__popcll(bal));
  base = __shfl(base, (int)leader, 64);
  if (take) {
    const uint32_t pos = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
    if (pos < sp.dcap) sp.dset[(size_t)blockIdx.x * sp.dcap + pos] = x;
    else atomicOr(&next[x >> 6], 1ull << (x & 63));
  }
}

__device__ __forceinline__ void ppa_resolve(const DevState& s, const PPSparse& sp, uint32_t t, uint32_t c3,
                                            const uint32_t* q, uint32_t cnt, uint64_t base,
                                            unsigned long long* __restrict__ next, uint64_t& sent, uint64_t& msgs,
                                            uint32_t* s_dn) {
  const uint32_t lane = threadIdx.x & 63;
  if (lane >= cnt) return;
  const uint32_t e = q[lane], loc = e & 0xFFFu, d = e >> 16;
  const uint64_t u = base + loc;  // informed (so live)
  const bool cc = s.check_crashed;
  {  // u's own call: a push
    bool take = false;
    uint32_t w = 0;
    if (d > 0) {
      const u32x4 r = philox((uint32_t)(s.gbase + u), t, 0, c3, s.key.k0, s.key.k1);
      if ((int32_t)uniform(r.y, 100u) >= s.kd) {
        const uint32_t j = uniform(r.x, d);
        w = s.ids[u * s.stride + j];
        ++sent;
        const bool dead = sp.fmask ? ((sp.fmask[u] >> j) & 1) != 0
                                   : (cc && ((s.gcrash[w >> 6] >> (w & 63)) & 1));
        if (!dead) {
          ++msgs;
          take = true;
        }
      }
    }
#if defined(GS_PP_NOATOMIC)  // timing probe only: the round's sets are not made
    if (take && w == 0xFFFFFFFFu) next[0] = 1;
#elif defined(GS_PP_CHECKFIRST)  // an informed target's bit is set already (next starts as recv)
    if (take && !((s.grecv[w >> 6] >> (w & 63)) & 1)) atomicOr(&next[w >> 6], 1ull << (w & 63));
#else
    pp_set(sp, next, take, w, s_dn);
#endif
  }
  unsigned long long qb, qe;
  in_edges(sp, u, qb, qe);
  for (unsigned long long q0 = qb; q0 < qe; q0 += kPPEdges) {
    uint32_t src[kPPEdges], x[kPPEdges];
#pragma unroll
    for (uint32_t k = 0; k < kPPEdges; ++k) {
      const bool in = q0 + k < qe;
      src[k] = in ? sp.rsrc[q0 + k] : 0u;
      x[k] = in ? sp.rslot[q0 + k] : 0u;
    }
#pragma unroll
    for (uint32_t k = 0; k < kPPEdges; ++k) {
      bool take = false;
      if (q0 + k < qe) {
        const u32x4 r = philox(src[k], t, 0, c3, s.key.k0, s.key.k1);
        if (uniform(r.x, (x[k] >> 4) + 1) == (x[k] & 15u) && (int32_t)uniform(r.y, 100u) >= s.kd) {
          const unsigned long long vb = 1ull << (src[k] & 63);
          const bool iv = (s.grecv[src[k] >> 6] & vb) != 0;
          // v failed: its in-edge's bit (sp.rfail: a line the in-edge scan
          // reads anyway) instead of a gather of v's failed word
          const uint64_t q = q0 + k;
          const bool fv = cc && (sp.rfail ? ((sp.rfail[q >> 5] >> (q & 31)) & 1u) != 0
                                          : (s.gcrash[src[k] >> 6] & vb) != 0);
          if (!iv && !fv) {  // v's pull from this informed node succeeds
            ++sent;
            ++msgs;
            take = true;
          }
        }
      }
#if defined(GS_PP_NOATOMIC)
      if (take && src[k] == 0xFFFFFFFFu) next[0] = 1;
#else
      pp_set(sp, next, take, src[k], s_dn);
#endif
    }
  }
}

__global__ __launch_bounds__(kPPSBlock) void k_ppa_round(const DevState s, unsigned long long* __restrict__ next,
                                                             const PPSparse sp, uint32_t t) {
  __shared__ uint64_t sh[3 * kPPWaves];
  __shared__ uint32_t s_q[kPPWaves][kPPQ];
  __shared__ uint32_t s_dn;  // this workgroup's deferred sets
  __shared__ uint32_t s_pre[kPPWaves][64];
  __shared__ unsigned long long s_msk[kPPWaves][64];
  PPCtl* c = sp.ctl;
  if (c->mode != PP_ANSWER) return;
  static_assert(kPPSGrid <= kPPDLists, "one deferred list per workgroup");
  if (threadIdx.x == 0) s_dn = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t* q = s_q[wv];
  const uint32_t c3 = ctr3(K_PUSHPULL, s.key.trial);
  uint64_t sent = 0, msgs = 0;
  const uint64_t W = (s.n + 63) >> 6;
  const uint64_t nrange = (W + kPPRange - 1) / kPPRange;
  for (uint64_t rg = (uint64_t)blockIdx.x * kPPWaves + wv; rg < nrange; rg += (uint64_t)gridDim.x * kPPWaves) {
    const uint64_t w0 = rg * kPPRange, base = w0 << 6;
    uint32_t qn = 0;  // wave-uniform
    // a lane per WORD of the range where no word holds more than
    // sp.word_maxi informed nodes: the range's informed nodes are resolved 64
    // at a time in node order (for_each_bit), so a sparse range costs its
    // informed nodes / 64 batches instead of 64 word steps
    bool by_word = false;
    const uint64_t word = w0 + lane;
    unsigned long long mi = 0;
    if (sp.words) {
      mi = word < W ? s.recv[word] : 0ull;  // informed => live and in range
      uint32_t mx = (uint32_t)__popcll(mi);
#pragma unroll
      for (uint32_t o = 32; o >= 1; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor(mx, o, 64));
      by_word = sp.words == 1 || mx <= sp.word_maxi;
    }
    if (by_word)
      for_each_bit(mi, s_pre[wv], s_msk[wv], [&](uint32_t cnt, uint32_t off) {
        q[lane] = lane < cnt ? off | (uint32_t)s.deg[base + off] << 16 : 0u;
        wave_lds_sync();
        ppa_resolve(s, sp, t, c3, q, cnt, base, next, sent, msgs, &s_dn);
        wave_lds_sync();
      });
    for (uint32_t wi = 0; wi < kPPRange && !by_word; wi += kPPB) {
      unsigned long long Iw[kPPB];
      uint32_t d[kPPB];
#pragma unroll
      for (uint32_t i = 0; i < kPPB; ++i) {
        const uint64_t word = w0 + wi + i, v = (word << 6) + lane;
        Iw[i] = word < W ? s.recv[word] : 0ull;
        d[i] = ((Iw[i] >> lane) & 1) ? s.deg[v] : 0u;
      }
#pragma unroll
      for (uint32_t i = 0; i < kPPB; ++i) {
        const uint64_t v = ((w0 + wi + i) << 6) + lane;
        const bool enq = (Iw[i] >> lane) & 1;  // informed => live and in range
        const unsigned long long bal = __ballot(enq);
        if (enq) {
          const uint32_t at = qn + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
          q[at] = (uint32_t)(v - base) | d[i] << 16;
        }
        qn += (uint32_t)__popcll(bal);
        if (qn >= 64) {
          wave_lds_sync();
          ppa_resolve(s, sp, t, c3, q, 64, base, next, sent, msgs, &s_dn);
          const uint32_t rest = qn - 64;
          const uint32_t keep = lane < rest ? q[64 + lane] : 0u;
          wave_lds_sync();
          if (lane < rest) q[lane] = keep;
          qn = rest;
        }
      }
    }
    wave_lds_sync();
    if (qn) ppa_resolve(s, sp, t, c3, q, qn, base, next, sent, msgs, &s_dn);
    wave_lds_sync();
  }
  if (sp.dset) {
    __syncthreads();
    if (threadIdx.x == 0) sp.dcnt[blockIdx.x] = s_dn < sp.dcap ? s_dn : sp.dcap;
  }
  const uint64_t v3[3] = {blockIdx.x == 0 && threadIdx.x == 0 ? c->ncallers : 0ull, sent, msgs};
  const uint32_t f3[3] = {ST_FIRED, ST_SENT, ST_MSGS};
  block_add<kPPSBlock>(sh, v3, 3, s.stats + (size_t)(t % kStatSlots) * kStatFields, f3);
}

// ---- deferred sets: coarse and fine LDS partitions, then the bitmap OR ----
constexpr uint32_t kPPDTile = 16384;   // set targets per partition tile
constexpr uint32_t kPPDBlock = 1024;   // 16 per thread

// Exclusive scan of cnt[0..256) into off[0..257) by the first 256 threads
// (block-uniform call; every thread passes the barriers).
__device__ __forceinline__ void ppd_scan256(const uint32_t* cnt, uint32_t* off, uint32_t* s_w) {
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  uint32_t v = tid < 256 ? cnt[tid] : 0u, x = v;
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (tid < 256 && lane == 63) s_w[wv] = x;
  __syncthreads();
  if (tid < 256) {
    uint32_t pre = 0;
    for (uint32_t q = 0; q < wv; ++q) pre += s_w[q];
    off[tid] = pre + x - v;
    if (tid == 255) off[256] = pre + x;
  }
  __syncthreads();
}

// One partition pass: tiles of the `nsrc` input lists (list L holds
// min(fill[L], cap_in) targets at in + L * cap_in) are counting-sorted in LDS
// by the 8-bit digit (x >> shift) & 255 and leave as runs: coarse pass (shift
// 22) into region digit * 8 + (blockIdx & 7) of `out`, fine pass (shift 14)
// into fine bucket (region's bin) * 256 + digit; one reservation per (tile,
// digit); what does not fit its region is an atomicOr into next.
template <bool FINE>
__global__ __launch_bounds__(kPPDBlock) void k_ppd_part(const PPSparse sp, unsigned long long* __restrict__ next,
                                                        const uint32_t* in, const unsigned long long* fill,
                                                        uint32_t nsrc, uint64_t cap_in, uint32_t* out,
                                                        unsigned long long* ofill, uint64_t cap_out) {
  if (sp.ctl->mode != PP_ANSWER) return;
  __shared__ uint32_t buf[kPPDTile];
  __shared__ uint32_t cnt[256], off[257], s_w[4];
  __shared__ unsigned long long gb[256], ge[256];
  constexpr uint32_t kPer = kPPDTile / kPPDBlock;
  constexpr uint32_t shift = FINE ? 14 : 22;
  const uint32_t tid = threadIdx.x;
  const uint64_t nch = (cap_in + kPPDTile - 1) / kPPDTile;
  for (uint64_t tt = blockIdx.x; tt < nsrc * nch; tt += gridDim.x) {
    const uint32_t L = (uint32_t)(tt % nsrc);
    const uint64_t ch = tt / nsrc;
    const unsigned long long fl = fill[L];
    const uint64_t n = fl < cap_in ? fl : cap_in, b0 = ch * kPPDTile;
    if (b0 >= n) continue;  // block-uniform
    const uint32_t m = (uint32_t)min((uint64_t)kPPDTile, n - b0);
    if (tid < 256) cnt[tid] = 0;
    __syncthreads();
    uint32_t x[kPer], rk[kPer];
#pragma unroll
    for (uint32_t r = 0; r < kPer; ++r) {
      const uint32_t i = r * kPPDBlock + tid;
      x[r] = i < m ? in[L * cap_in + b0 + i] : ~0u;
      rk[r] = x[r] != ~0u ? atomicAdd(&cnt[(x[r] >> shift) & 255], 1u) : 0u;
    }
    __syncthreads();
    ppd_scan256(cnt, off, s_w);
    if (tid < 256 && cnt[tid]) {
      const uint64_t reg = FINE ? (uint64_t)(L / 8) * 256 + tid : (uint64_t)tid * 8 + (blockIdx.x & 7);
      const unsigned long long at = atomicAdd(&ofill[reg], (unsigned long long)cnt[tid]);
      gb[tid] = reg * cap_out + at - off[tid];
      ge[tid] = reg * cap_out + cap_out;
    }
#pragma unroll
    for (uint32_t r = 0; r < kPer; ++r)
      if (x[r] != ~0u) buf[off[(x[r] >> shift) & 255] + rk[r]] = x[r];
    __syncthreads();
    for (uint32_t p = tid; p < m; p += kPPDBlock) {
      const uint32_t v = buf[p], dg = (v >> shift) & 255;
      const unsigned long long pos = gb[dg] + p;
      if (pos < ge[dg]) out[pos] = FINE ? (v & ((1u << 14) - 1)) : v;
      else atomicOr(&next[v >> 6], 1ull << (v & 63));
    }
    __syncthreads();
  }
}

// One workgroup per 16384-node bucket f: its fine region's targets into an
// LDS bitmap, ORed into its 256 words of next (this workgroup alone writes
// them; the fallback atomics ran in the kernels before).
__global__ __launch_bounds__(256) void k_ppd_apply(const PPSparse sp, unsigned long long* __restrict__ next,
                                                   uint64_t W, uint32_t nfine) {
  if (sp.ctl->mode != PP_ANSWER) return;
  __shared__ uint32_t bm[512];
  const unsigned long long* ffill = sp.dcnt + kPPDLists + kPPDRegions;
  const uint32_t* fine = sp.dset + (size_t)kPPDLists * sp.dcap + (size_t)kPPDRegions * sp.ccap;
  for (uint32_t f = blockIdx.x; f < nfine; f += gridDim.x) {
    const unsigned long long fl = ffill[f];
    const uint32_t n = (uint32_t)(fl < sp.fcap ? fl : sp.fcap);
    if (!n) continue;  // block-uniform
    bm[threadIdx.x] = 0;
    bm[threadIdx.x + 256] = 0;
    __syncthreads();
    for (uint32_t p = threadIdx.x; p < n; p += 256) {
      const uint32_t loc = fine[(size_t)f * sp.fcap + p];
      atomicOr(&bm[loc >> 5], 1u << (loc & 31));
    }
    __syncthreads();
    const uint64_t w = (uint64_t)f * 256 + threadIdx.x;
    const unsigned long long v = (unsigned long long)bm[2 * threadIdx.x] |
                                 ((unsigned long long)bm[2 * threadIdx.x + 1] << 32);
    if (v && w < W) next[w] |= v;
    __syncthreads();
  }
}

// Shards: the round's mode, chosen by the host from the global informed count
// (the same on every shard: the replicated set), and the round counters.
__global__ void k_pp_set_mode(PPCtl* c, uint32_t mode) {
  c->mode = mode;
  c->nbottom += mode == PP_BOTTOM;
  c->nanswer += mode == PP_ANSWER;
}

// *out = popcount of words[0, n) (n = 0: *out = 0).
__global__ __launch_bounds__(kPPBlock) void k_pp_count(const unsigned long long* __restrict__ words,
                                                       unsigned long long n, unsigned long long* out) {
  __shared__ uint64_t sh[kPPBlock / 64];
  if (n == 0) {
    if (threadIdx.x == 0 && blockIdx.x == 0) *out = 0;
    return;
  }
  uint64_t c = 0;
  for (uint64_t w = (uint64_t)blockIdx.x * kPPBlock + threadIdx.x; w < n; w += (uint64_t)gridDim.x * kPPBlock)
    c += (uint64_t)__popcll(words[w]);
  const uint64_t ws = wave_sum64(c);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = ws;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t b = 0;
    for (uint32_t k = 0; k < kPPBlock / 64; ++k) b += sh[k];
    if (b) atomicAdd(out, (unsigned long long)b);
  }
}

// dst[w] |= src[i * words + w] for every slice i < nslices (the bits other
// shards set in this shard's range during a pull-answer round).
__global__ __launch_bounds__(kPPBlock) void k_pp_or_slices(unsigned long long* __restrict__ dst,
                                                           const unsigned long long* __restrict__ src,
                                                           uint32_t nslices, uint64_t words) {
  for (uint64_t w = (uint64_t)blockIdx.x * kPPBlock + threadIdx.x; w < words; w += (uint64_t)gridDim.x * kPPBlock) {
    unsigned long long x = dst[w];
    for (uint32_t i = 0; i < nslices; ++i) x |= src[(size_t)i * words + w];
    dst[w] = x;
  }
}

__global__ __launch_bounds__(kPPBlock) void k_pp_commit(const DevState s,
                                                        const unsigned long long* __restrict__ next,
                                                        uint32_t t, PPCtl* ctl) {
  __shared__ uint64_t sh[kPPBlock / 64];
  if (ctl && ctl->mode == PP_EARLY) return;
  uint64_t newly = 0;
  for (uint64_t w = (uint64_t)blockIdx.x * kPPBlock + threadIdx.x; w < s.W;
       w += (uint64_t)gridDim.x * kPPBlock) {
    const unsigned long long nx = next[w], old = s.recv[w];
    newly += (uint64_t)__popcll(nx & ~old);
    if (nx != old) s.recv[w] = nx;
  }
  const uint64_t ws = wave_sum64(newly);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = ws;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t b = 0;
    for (uint32_t k = 0; k < kPPBlock / 64; ++k) b += sh[k];
    if (b) {
      atomicAdd(&s.stats[(size_t)(t % kStatSlots) * kStatFields + ST_RECV], (unsigned long long)b);
      if (ctl) atomicAdd(&ctl->ninf, (unsigned long long)b);
    }
  }
}

// ---- sparse early rounds ------------------------------------------------------
// Round mode and the list bookkeeping (one block of kPPSegs threads): the
// previous early round's appends join the list unless a segment overflowed.
__global__ __launch_bounds__(kPPSegs) void k_pp_mode(PPCtl* c) {
  __shared__ unsigned long long sc[kPPSegs];
  const uint32_t tid = threadIdx.x;
  const bool was_early = c->mode == PP_EARLY;
  const bool ok = c->early_ok && !c->ovf;
  unsigned long long len = 0;
  if (tid < c->nseg) {
    len = c->segcnt[tid];
    c->seglen[tid] = len;
  }
  sc[tid] = len;
  __syncthreads();
  if (tid == 0) {
    unsigned long long a = 0;
    for (uint32_t k = 0; k < c->nseg; ++k) {
      c->segpre[k] = a;
      a += sc[k];
    }
    c->segpre[c->nseg] = a;
    const bool early = ok && c->ninf <= c->thr;
    c->mode = early ? PP_EARLY : c->ninf >= c->bthr ? PP_BOTTOM : c->ninf >= c->athr ? PP_ANSWER : PP_DENSE;
    c->nearly += c->mode == PP_EARLY;
    c->nbottom += c->mode == PP_BOTTOM;
    c->nanswer += c->mode == PP_ANSWER;
    if (!early) c->early_ok = 0;  // |I| only grows: the list is never needed again
    (void)was_early;
  }
}

// Appends v to the informed list when this lane's atomicOr on `next` set its
// bit first: one atomic per wave on segment blockIdx % nseg's counter (the
// lanes taking part may be any subset of the wave).
__device__ __forceinline__ void pp_append(PPCtl* c, uint32_t* ilist, uint32_t seg, unsigned long long cap,
                                          bool take, uint32_t v) {
  const unsigned long long bal = __ballot(take);
  if (!bal) return;
  const uint32_t lane = threadIdx.x & 63, lead = (uint32_t)__builtin_ctzll(bal);
  unsigned long long base = 0;
  if (lane == lead) base = atomicAdd(&c->segcnt[seg], (unsigned long long)__popcll(bal));
  base = __shfl(base, lead, 64);
  if (take) {
    const unsigned long long at =
        base + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0u));
    if (at < cap) ilist[(size_t)seg * cap + at] = v;
    else c->ovf = 1u;
  }
}

// One early round: lane per informed node u of the
// list.  u's own call is a push (u informed => live); every in-edge (v, j)
// of u whose caller v is live, uninformed, picks slot j and is not lost is a
// successful pull.  Same draws and counters as k_pp_round.
__global__ __launch_bounds__(kPPBlock) void k_ppe_round(const DevState s, unsigned long long* __restrict__ next,
                                                        PPSparse sp, uint32_t t) {
  __shared__ uint64_t sh[3 * (kPPBlock / 64)];
  __shared__ unsigned long long pre[kPPSegs + 1];
  PPCtl* c = sp.ctl;
  if (c->mode != PP_EARLY) return;
  const uint32_t nseg = c->nseg;
  const unsigned long long cap = c->seg_cap;
  for (uint32_t k = threadIdx.x; k <= nseg; k += kPPBlock) pre[k] = c->segpre[k];
  __syncthreads();
  const unsigned long long nl = pre[nseg];
  const uint32_t myseg = blockIdx.x % nseg;
  const uint32_t c3 = ctr3(K_PUSHPULL, s.key.trial);
  const bool cc = s.check_crashed, packed = pp_rslot_packed(s.stride);
  uint64_t sent = 0, msgs = 0;
  const uint64_t G = (uint64_t)gridDim.x * kPPBlock;
  const uint64_t nlr = (nl + 63) & ~63ull;  // whole waves iterate together (pp_append)
  for (uint64_t i = (uint64_t)blockIdx.x * kPPBlock + threadIdx.x; i < nlr; i += G) {
    const bool live = i < nl;
    uint32_t u = 0;
    if (live) {  // list index -> (segment, entry)
      uint32_t lo = 0, hi = nseg - 1;
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (pre[mid] <= i) lo = mid; else hi = mid - 1;
      }
      u = sp.ilist[(size_t)lo * cap + (i - pre[lo])];
    }
    // own call: push
    bool take = false;
    uint32_t w = 0;
    const uint32_t d = live ? s.deg[u] : 0u;
    if (d > 0) {
      const u32x4 r = philox(u, t, 0, c3, s.key.k0, s.key.k1);
      if ((int32_t)uniform(r.y, 100u) >= s.kd) {
        w = s.ids[(uint64_t)u * s.stride + uniform(r.x, d)];
        const unsigned long long wb = 1ull << (w & 63);
        ++sent;
        if (!(cc && (s.crash[w >> 6] & wb))) {  // w live: delivered
          ++msgs;
          if (!(s.recv[w >> 6] & wb)) take = !(atomicOr(&next[w >> 6], wb) & wb);
        }
      }
    }
    pp_append(c, sp.ilist, myseg, cap, take, w);
    // pulls from u: u's in-edges
    unsigned long long q = live ? (u ? sp.rend[u - 1] : 0ull) : 0ull;
    const unsigned long long e = live ? sp.rend[u] : 0ull;
    while (__ballot(q < e)) {
      bool tk = false;
      uint32_t v = 0;
      if (q < e) {
        v = sp.rsrc[q];
        const uint32_t x = sp.rslot[q];
        const uint32_t j = packed ? x & 15u : x;
        ++q;
        const unsigned long long vb = 1ull << (v & 63);
        // v informed: its own list entry pushes; v failed: never calls
        if (!(s.recv[v >> 6] & vb) && !(cc && (s.crash[v >> 6] & vb))) {
          const u32x4 r = philox(v, t, 0, c3, s.key.k0, s.key.k1);
          if (uniform(r.x, packed ? (x >> 4) + 1 : s.deg[v]) == j && (int32_t)uniform(r.y, 100u) >= s.kd) {
            ++sent;
            ++msgs;
            tk = !(atomicOr(&next[v >> 6], vb) & vb);
          }
        }
      }
      pp_append(c, sp.ilist, myseg, cap, tk, v);
    }
  }
  const uint64_t v3[3] = {blockIdx.x == 0 && threadIdx.x == 0 ? c->ncallers : 0ull, sent, msgs};
  const uint32_t f3[3] = {ST_FIRED, ST_SENT, ST_MSGS};
  block_add(sh, v3, 3, s.stats + (size_t)(t % kStatSlots) * kStatFields, f3);
}

// The early round's newly informed nodes join recv (next holds them already):
// from the list, or -- if a segment overflowed -- from the bitsets.
__global__ __launch_bounds__(kPPBlock) void k_ppe_commit(const DevState s, const unsigned long long* __restrict__ next,
                                                         PPSparse sp, uint32_t t) {
  __shared__ uint64_t sh[kPPBlock / 64];
  __shared__ unsigned long long s_b[kPPSegs], s_e[kPPSegs];
  PPCtl* c = sp.ctl;
  if (c->mode != PP_EARLY) return;
  const uint64_t G = (uint64_t)gridDim.x * kPPBlock, gid = (uint64_t)blockIdx.x * kPPBlock + threadIdx.x;
  uint64_t newly = 0;
  const bool ovf = c->ovf != 0;
  const uint32_t nseg = c->nseg;
  if (!ovf) {  // the segments' bounds staged once per block (a chain of 2 * nseg loads per thread before)
    for (uint32_t sg = threadIdx.x; sg < nseg; sg += kPPBlock) {
      s_b[sg] = c->seglen[sg];
      s_e[sg] = c->segcnt[sg];
    }
    __syncthreads();
  }
  if (ovf) {
    for (uint64_t w = gid; w < s.W; w += G) {
      const unsigned long long nx = next[w], old = s.recv[w];
      newly += (uint64_t)__popcll(nx & ~old);
      if (nx != old) s.recv[w] = nx;
    }
  } else {
    const unsigned long long cap = c->seg_cap;
    for (uint32_t sg = 0; sg < nseg; ++sg) {
      const unsigned long long b = s_b[sg], e = s_e[sg];
      for (uint64_t k = b + gid; k < e; k += G) {
        const uint32_t v = sp.ilist[(size_t)sg * cap + k];
        atomicOr(&s.recv[v >> 6], 1ull << (v & 63));
        ++newly;
      }
    }
  }
  const uint64_t ws = wave_sum64(newly);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = ws;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t b = 0;
    for (uint32_t k = 0; k < kPPBlock / 64; ++k) b += sh[k];
    if (b) {
      atomicAdd(&s.stats[(size_t)(t % kStatSlots) * kStatFields + ST_RECV], (unsigned long long)b);
      atomicAdd(&c->ninf, (unsigned long long)b);
    }
  }
}

// The counts of k_pp_callers, from an earlier count of the same table and mask.
__global__ void k_pp_set_callers(PPCtl* c, unsigned long long ncallers, unsigned long long nlive0) {
  c->ncallers = ncallers;
  c->nlive0 = nlive0;
}

// Live nodes with a non-empty row (each calls once per round).
__global__ __launch_bounds__(kPPBlock) void k_pp_callers(const DevState s, PPCtl* c) {
  uint64_t k = 0, z = 0;
  for (uint64_t v = (uint64_t)blockIdx.x * kPPBlock + threadIdx.x; v < s.n; v += (uint64_t)gridDim.x * kPPBlock) {
    const bool live = !((s.crash[v >> 6] >> (v & 63)) & 1);
    k += live && s.deg[v] > 0;
    z += live && s.deg[v] == 0;
  }
  k = wave_sum64(k);
  z = wave_sum64(z);
  if ((threadIdx.x & 63) == 0 && k) atomicAdd(&c->ncallers, (unsigned long long)k);
  if ((threadIdx.x & 63) == 0 && z) atomicAdd(&c->nlive0, (unsigned long long)z);
}

// ---- reverse table ------------------------------------------------------------
__global__ __launch_bounds__(kPPBlock) void k_rev_count(const DevState s, unsigned long long* cnt) {
  for (uint64_t v = (uint64_t)blockIdx.x * kPPBlock + threadIdx.x; v < s.n; v += (uint64_t)gridDim.x * kPPBlock) {
    const uint32_t d = s.deg[v];
    for (uint32_t j = 0; j < d; ++j) atomicAdd(&cnt[s.ids[v * s.stride + j]], 1ull);
  }
}

// After the exclusive scan rend[u] = start of u's in-edges; each fill bumps
// it, so it ends as the end of u's in-edges (= the start of u + 1's).
__global__ __launch_bounds__(kPPBlock) void k_rev_fill(const DevState s, unsigned long long* rend, uint32_t* rsrc,
                                                       uint8_t* rslot) {
  for (uint64_t v = (uint64_t)blockIdx.x * kPPBlock + threadIdx.x; v < s.n; v += (uint64_t)gridDim.x * kPPBlock) {
    const uint32_t d = s.deg[v];
    for (uint32_t j = 0; j < d; ++j) {
      const unsigned long long at = atomicAdd(&rend[s.ids[v * s.stride + j]], 1ull);
      rsrc[at] = (uint32_t)v;
      rslot[at] = (uint8_t)(pp_rslot_packed(s.stride) ? j | (d - 1) << 4 : j);
    }
  }
}

// fmask[v] bit j = ids[v][j] is failed: each failed node marks its in-edges.
__global__ __launch_bounds__(kPPBlock) void k_pp_fmask(const DevState s, const unsigned long long* rend,
                                                       const uint32_t* rsrc, const uint8_t* rslot, uint32_t* fm4) {
  for (uint64_t f = (uint64_t)blockIdx.x * kPPBlock + threadIdx.x; f < s.n; f += (uint64_t)gridDim.x * kPPBlock) {
    if (!((s.crash[f >> 6] >> (f & 63)) & 1)) continue;
    for (unsigned long long q = f ? rend[f - 1] : 0ull; q < rend[f]; ++q) {
      const uint32_t v = rsrc[q];
      atomicOr(&fm4[v >> 2], (1u << (rslot[q] & 15u)) << (8 * (v & 3)));  // stride <= 8: packed
    }
  }
}

// Exact stop test (gs_run): out += edges (v, friends[v][j]) over which a call
// could still change the informed set -- v live and informed with a live
// uninformed friend (push), or v live and uninformed with an informed friend
// (pull).  Zero means no later round can inform anyone.  Run only when a poll
// window informed nobody new.
__global__ __launch_bounds__(kPPBlock) void k_pp_live_edges(const DevState s, uint32_t* out) {
  uint32_t cnt = 0;
  for (uint64_t v = (uint64_t)blockIdx.x * kPPBlock + threadIdx.x; v < s.n; v += (uint64_t)gridDim.x * kPPBlock) {
    const unsigned long long bit = 1ull << (v & 63);
    if (s.crash[v >> 6] & bit) continue;
    const bool iv = (s.recv[v >> 6] & bit) != 0;
    const uint32_t d = s.deg[v];
    for (uint32_t j = 0; j < d; ++j) {
      const uint32_t u = s.ids[v * s.stride + j];  // global id
      const unsigned long long ub = 1ull << (u & 63);
      const bool iu = (s.grecv[u >> 6] & ub) != 0, fu = (s.gcrash[u >> 6] & ub) != 0;
      if (iv ? (!iu && !fu) : iu) { ++cnt; break; }
    }
  }
  const uint32_t w = wave_sum64(cnt);
  if ((threadIdx.x & 63) == 0 && w) atomicAdd(out, w);
}

// ---- node-range shards ----------------------------------------------------------
// In-edge counts of the targets in [lo, hi) over the full table (cnt indexed
// by target - lo), then the fill (rend ends as the end of each target's edges).
__global__ __launch_bounds__(kPPBlock) void k_rev_count_range(const uint8_t* deg, const uint32_t* ids, uint64_t n,
                                                              uint32_t stride, uint64_t lo, uint64_t hi,
                                                              unsigned long long* cnt) {
  for (uint64_t v = (uint64_t)blockIdx.x * kPPBlock + threadIdx.x; v < n; v += (uint64_t)gridDim.x * kPPBlock) {
    const uint32_t d = deg[v];
    for (uint32_t j = 0; j < d; ++j) {
      const uint32_t u = ids[v * stride + j];
      if (u >= lo && u < hi) atomicAdd(&cnt[u - lo], 1ull);
    }
  }
}

__global__ __launch_bounds__(kPPBlock) void k_rev_fill_range(const uint8_t* deg, const uint32_t* ids, uint64_t n,
                                                             uint32_t stride, uint64_t lo, uint64_t hi,
                                                             unsigned long long* rend, uint32_t* rsrc,
                                                             uint8_t* rslot) {
  for (uint64_t v = (uint64_t)blockIdx.x * kPPBlock + threadIdx.x; v < n; v += (uint64_t)gridDim.x * kPPBlock) {
    const uint32_t d = deg[v];
    for (uint32_t j = 0; j < d; ++j) {
      const uint32_t u = ids[v * stride + j];
      if (u < lo || u >= hi) continue;
      const unsigned long long at = atomicAdd(&rend[u - lo], 1ull);
      rsrc[at] = (uint32_t)v;
      rslot[at] = (uint8_t)(pp_rslot_packed(stride) ? j | (d - 1) << 4 : j);
    }
  }
}

// fmask[v] bit j = friend j of own caller v is failed (replicated failed set).
// rfail bit q: in-edge q's caller rsrc[q] is failed (the pull-answer rounds'
// answer test; rfail zeroed before).  Built from the failed callers' side: a
// thread per failed-set word, and for each failed caller v and slot j the
// in-edge (v, j) is found in friend w's short in-list (a pass over every
// in-edge with a gather of its caller's failed word took 175 ms at N = 1e9).
// In-lists longer than this are not scanned per failed caller (the scan is
// the friend's whole in-list, so a hub listed by many failed callers would
// cost quadratically): k_pp_rfail_hubs walks them once instead.
constexpr uint32_t kRfailScan = 64;

// *hub = 1 when some failed caller has a friend whose in-list is longer than
// kRfailScan: only then does k_pp_rfail_hubs walk the in-lists (ADVICE r05:
// it read every rend entry, ~8 GB at N = 1e9, whether or not a hub existed).
__global__ __launch_bounds__(kPPBlock) void k_pp_rfail(const DevState s, const unsigned long long* __restrict__ rend,
                                                       const uint32_t* __restrict__ rsrc,
                                                       const uint8_t* __restrict__ rslot, uint32_t* __restrict__ rfail,
                                                       uint32_t* __restrict__ hub) {
  for (uint64_t wd = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; wd < s.W;
       wd += (uint64_t)gridDim.x * blockDim.x) {
    for (unsigned long long m = s.crash[wd]; m; m &= m - 1) {
      const uint64_t v = (wd << 6) + (uint64_t)__builtin_ctzll(m);
      if (v >= s.n) break;
      const uint32_t d = s.deg[v];
      for (uint32_t j = 0; j < d; ++j) {
        const uint32_t w = s.ids[v * s.stride + j];
        const unsigned long long qb = w ? rend[w - 1] : 0ull, qe = rend[w];
        if (qe - qb > kRfailScan) {  // a hub: k_pp_rfail_hubs
          if (!*hub) atomicOr(hub, 1u);
          continue;
        }
        for (unsigned long long q = qb; q < qe; ++q)
          if (rsrc[q] == (uint32_t)v && (rslot[q] & 15u) == j) {
            atomicOr(&rfail[q >> 5], 1u << (q & 31));
            break;
          }
      }
    }
  }
}

// The in-edges of every node with more than kRfailScan of them: one wave per
// such node walks its in-list once and marks the edges whose caller failed
// (linear in the hubs' in-degrees).
__global__ __launch_bounds__(kPPBlock) void k_pp_rfail_hubs(const DevState s, const unsigned long long* __restrict__ rend,
                                                            const uint32_t* __restrict__ rsrc,
                                                            uint32_t* __restrict__ rfail,
                                                            const uint32_t* __restrict__ hub) {
  if (!*hub) return;  // no failed caller lists a hub
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  for (uint64_t w0 = wave * 64; w0 < s.n; w0 += nwaves * 64) {
    // the wave's 64 candidate nodes, one per lane; then each hub among them in turn
    const uint64_t w = w0 + lane;
    const unsigned long long qe = w < s.n ? rend[w] : 0ull, qb = w < s.n && w ? rend[w - 1] : 0ull;
    for (unsigned long long hubs = __ballot(w < s.n && qe - qb > kRfailScan); hubs; hubs &= hubs - 1) {
      const uint32_t h = (uint32_t)__builtin_ctzll(hubs);
      const unsigned long long hb = __shfl(qb, h, 64), he = __shfl(qe, h, 64);
      for (unsigned long long q = hb + lane; q < he; q += 64) {
        const uint32_t v = rsrc[q];
        if ((s.crash[v >> 6] >> (v & 63)) & 1ull) atomicOr(&rfail[q >> 5], 1u << (q & 31));
      }
    }
  }
}

// fany bit v: node v has a failed friend (fmask[v] != 0): the lane-per-word
// bottom-up ranges read a node's degree and mask byte only then.  A thread
// per 64-node word.
__global__ __launch_bounds__(kPPBlock) void k_pp_fmask_any(const uint8_t* __restrict__ fmask, uint64_t n,
                                                           unsigned long long* __restrict__ fany) {
  const uint64_t W = (n + 63) >> 6;
  for (uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; w < W; w += (uint64_t)gridDim.x * blockDim.x) {
    unsigned long long bits = 0;
    for (uint32_t b = 0; b < 64; ++b) {
      const uint64_t v = (w << 6) + b;
      if (v < n && fmask[v]) bits |= 1ull << b;
    }
    fany[w] = bits;
  }
}

__global__ __launch_bounds__(kPPBlock) void k_pp_fmask_rows(const DevState s, uint8_t* fmask) {
  for (uint64_t v = (uint64_t)blockIdx.x * kPPBlock + threadIdx.x; v < s.n; v += (uint64_t)gridDim.x * kPPBlock) {
    const uint32_t d = s.deg[v];
    uint32_t m = 0;
    for (uint32_t j = 0; j < d; ++j) {
      const uint32_t u = s.ids[v * s.stride + j];
      if ((s.gcrash[u >> 6] >> (u & 63)) & 1) m |= 1u << j;
    }
    fmask[v] = (uint8_t)m;
  }
}

// Sender (simulator.go:239-241 for the flood model): informed at begin unless
// failed; flag[0] = 1 if it was informed.  ctl (zeroed, ncallers counted):
// the informed list starts as the sender.
__global__ void k_pp_seed(const DevState s, unsigned long long* next, uint32_t node, uint32_t* flag, PPSparse sp,
                          unsigned long long thr, unsigned long long bthr, unsigned long long athr) {
  const unsigned long long bit = 1ull << (node & 63);
  const bool ok = node != ~0u && !(s.crash[node >> 6] & bit);  // ~0u: the sender is another shard's
  if (ok) {
    s.recv[node >> 6] |= bit;
    next[node >> 6] |= bit;
  }
  *flag = ok ? 1u : 0u;
  if (sp.ctl) {  // ctl was zeroed: the list is segment 0 = {sender}
    PPCtl* c = sp.ctl;
    c->ninf = ok ? 1 : 0;
    c->thr = thr;
    c->bthr = bthr;
    c->athr = athr;
    c->nseg = (uint32_t)(s.n >> 12 < kPPSegs ? (s.n >> 12 ? s.n >> 12 : 1) : kPPSegs);
    c->seg_cap = (s.n + c->nseg - 1) / c->nseg;
    c->mode = PP_DENSE;
    c->early_ok = sp.ilist ? 1 : 0;  // shards keep no informed list: never sparse
    c->segcnt[0] = ok ? 1 : 0;
    if (ok && sp.ilist) sp.ilist[0] = node;
  }
}


// ---- reverse table by partitioning (pp_rev_build_part) ----------------------
// The in-edges (v, j) -> u of the whole table, without a random atomic per
// edge (k_rev_count + k_rev_fill make two, 0.85 s at N = 1e9): a histogram of
// the targets' 2^22-node coarse bins (exact coarse regions), a coarse
// partition of the edges as 8-byte records (u mod 2^22 | v << 22 | slot byte
// << 53), a fine partition of each coarse region by the 16384-node bucket,
// and one workgroup per bucket that counts its targets' in-edges in LDS, writes
// their rend and places rsrc / rslot.  The order of a node's in-list is free
// (every use of the reverse table is order-independent, as with the atomic
// fill).
constexpr uint32_t kRvShift = 22;            // coarse bin = u >> 22
constexpr uint32_t kRvBins = 512;            // n < 2^31
constexpr uint32_t kRvBlock = 1024;
constexpr uint32_t kRvRows = 2 * kRvBlock;   // rows per coarse-pass round
constexpr uint32_t kRvTile = 16 * kRvBlock;  // records per fine-pass tile

__device__ __forceinline__ uint8_t rv_slot_byte(uint32_t stride, uint32_t j, uint32_t d) {
  return (uint8_t)(pp_rslot_packed(stride) ? j | (d - 1) << 4 : j);
}

// The compact view of rend (PPSparse::rend16 / rbase): one thread per node.
__global__ __launch_bounds__(kPPBlock) void k_rv_compact(const unsigned long long* __restrict__ rend, uint64_t n,
                                                         uint16_t* __restrict__ rend16,
                                                         unsigned long long* __restrict__ rbase, uint32_t* ovf) {
  for (uint64_t u = (uint64_t)blockIdx.x * kPPBlock + threadIdx.x; u < n; u += (uint64_t)gridDim.x * kPPBlock) {
    const uint64_t w = u >> 6;
    const unsigned long long b = w ? rend[(w << 6) - 1] : 0ull;
    if ((u & 63) == 0) rbase[w] = b;
    const unsigned long long d = rend[u] - b;
    if (d > 0xFFFFull) atomicOr(ovf, 1u);
    rend16[u] = (uint16_t)d;
  }
}

__global__ __launch_bounds__(kRvBlock) void k_rv_hist(const DevState s, unsigned long long* chist) {
  __shared__ uint32_t h[kRvBins];
  for (uint32_t b = threadIdx.x; b < kRvBins; b += kRvBlock) h[b] = 0;
  __syncthreads();
  for (uint64_t v = (uint64_t)blockIdx.x * kRvBlock + threadIdx.x; v < s.n; v += (uint64_t)gridDim.x * kRvBlock) {
    const uint32_t d = s.deg[v];
    for (uint32_t j = 0; j < d; ++j) atomicAdd(&h[s.ids[v * s.stride + j] >> kRvShift], 1u);
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < kRvBins; b += kRvBlock)
    if (h[b]) atomicAdd(&chist[b], (unsigned long long)h[b]);
}

// Rounds of kRvRows rows: count per coarse bin in LDS, one reservation per
// (round, bin), then every record to its bin's run (the rows re-read from L2).
// One pass covers the coarse bins [blo, bhi) (edges to other bins are
// skipped; cstart / cfill are indexed by bin - blo): a build in several passes
// bounds the temporaries (pp_rev_build_part).
__global__ __launch_bounds__(kRvBlock) void k_rv_coarse(const DevState s, const unsigned long long* __restrict__ cstart,
                                                        unsigned long long* __restrict__ cfill,
                                                        unsigned long long* __restrict__ rec, uint32_t blo,
                                                        uint32_t bhi) {
  __shared__ uint32_t cnt[kRvBins], off[kRvBins];
  __shared__ unsigned long long gb[kRvBins];
  const uint32_t tid = threadIdx.x;
  const uint64_t rounds = (s.n + kRvRows - 1) / kRvRows;
  for (uint64_t r = blockIdx.x; r < rounds; r += gridDim.x) {
    for (uint32_t b = tid; b < kRvBins; b += kRvBlock) { cnt[b] = 0; off[b] = 0; }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < 2; ++k) {
      const uint64_t v = r * kRvRows + k * kRvBlock + tid;
      if (v >= s.n) continue;
      const uint32_t d = s.deg[v];
      for (uint32_t j = 0; j < d; ++j) {
        const uint32_t b = s.ids[v * s.stride + j] >> kRvShift;
        if (b >= blo && b < bhi) atomicAdd(&cnt[b], 1u);
      }
    }
    __syncthreads();
    for (uint32_t b = tid; b < kRvBins; b += kRvBlock)
      if (cnt[b]) gb[b] = cstart[b - blo] + atomicAdd(&cfill[b - blo], (unsigned long long)cnt[b]);
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < 2; ++k) {
      const uint64_t v = r * kRvRows + k * kRvBlock + tid;
      if (v >= s.n) continue;
      const uint32_t d = s.deg[v];
      for (uint32_t j = 0; j < d; ++j) {
        const uint32_t u = s.ids[v * s.stride + j], b = u >> kRvShift;
        if (b < blo || b >= bhi) continue;
        const unsigned long long pos = gb[b] + atomicAdd(&off[b], 1u);
        rec[pos] = (u & ((1u << kRvShift) - 1)) | (v << kRvShift) |
                   ((unsigned long long)rv_slot_byte(s.stride, j, d) << 53);
      }
    }
    __syncthreads();
  }
}

// Tiles of a coarse region -> its fine regions (bits 14..21 of u): LDS counts,
// one reservation per (tile, bucket), records placed by offset atomics.  A
// fine region past its planned capacity sets *ovf (the build falls back).
__global__ __launch_bounds__(kRvBlock) void k_rv_fine(const unsigned long long* __restrict__ rec,
                                                      const unsigned long long* __restrict__ cstart,
                                                      const unsigned long long* __restrict__ cend,
                                                      const uint32_t* __restrict__ tpre, uint32_t nbins,
                                                      const unsigned long long* __restrict__ fstart,
                                                      unsigned long long* __restrict__ ffill,
                                                      unsigned long long* __restrict__ frec, uint32_t* ovf) {
  __shared__ uint32_t cnt[256], off[256];
  __shared__ unsigned long long gb[256], ge[256];
  __shared__ uint32_t s_tp[kRvBins + 1];
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i <= nbins; i += kRvBlock) s_tp[i] = tpre[i];
  __syncthreads();
  const uint32_t ntiles = s_tp[nbins];
  for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    uint32_t lo = 0, hi = nbins - 1;
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1) >> 1;
      if (s_tp[mid] <= t) lo = mid; else hi = mid - 1;
    }
    const uint32_t c = lo;
    const unsigned long long b0 = cstart[c] + (unsigned long long)(t - s_tp[c]) * kRvTile, be = cend[c];
    if (tid < 256) { cnt[tid] = 0; off[tid] = 0; }
    __syncthreads();
    unsigned long long r[kRvTile / kRvBlock];
#pragma unroll
    for (uint32_t k = 0; k < kRvTile / kRvBlock; ++k) {
      const unsigned long long i = b0 + k * kRvBlock + tid;
      r[k] = i < be ? rec[i] : ~0ull;
      if (r[k] != ~0ull) atomicAdd(&cnt[(r[k] >> 14) & 255], 1u);
    }
    __syncthreads();
    if (tid < 256 && cnt[tid]) {
      const size_t fb = (size_t)c * 256 + tid;
      gb[tid] = fstart[fb] + atomicAdd(&ffill[fb], (unsigned long long)cnt[tid]);
      ge[tid] = fstart[fb + 1];
      if (gb[tid] + cnt[tid] > ge[tid]) atomicOr(ovf, 1u);
    }
    __syncthreads();
#pragma unroll
    for (uint32_t k = 0; k < kRvTile / kRvBlock; ++k)
      if (r[k] != ~0ull) {
        const uint32_t d = (r[k] >> 14) & 255;
        const unsigned long long pos = gb[d] + atomicAdd(&off[d], 1u);
        if (pos < ge[d]) frec[pos] = r[k];
      }
    __syncthreads();
  }
}

// One workgroup per 16384-node bucket: in-degree counts in LDS, the bucket's
// rend (end of each node's in-edges), then rsrc / rslot in place.
__global__ __launch_bounds__(kRvBlock) void k_rv_final(const unsigned long long* __restrict__ frec,
                                                       const unsigned long long* __restrict__ fstart,
                                                       const unsigned long long* __restrict__ ffill,
                                                       const unsigned long long* __restrict__ bbase, uint64_t n,
                                                       unsigned long long* __restrict__ rend, uint32_t* __restrict__ rsrc,
                                                       uint8_t* __restrict__ rslot, uint32_t fb0) {
  __shared__ uint32_t cnt[16384];
  __shared__ unsigned long long s_x[kRvBlock / 64];
  // bucket b of the table = bucket blockIdx.x of this pass's arrays
  const uint32_t tid = threadIdx.x, b = fb0 + blockIdx.x;
  const unsigned long long M = ffill[blockIdx.x], f0 = fstart[blockIdx.x], ob = bbase[blockIdx.x];
  for (uint32_t i = tid; i < 16384; i += kRvBlock) cnt[i] = 0;
  __syncthreads();
  for (unsigned long long i = tid; i < M; i += kRvBlock) atomicAdd(&cnt[frec[f0 + i] & 16383], 1u);
  __syncthreads();
  // exclusive offsets: 16 consecutive counters per thread
  uint32_t loc[16], sum = 0;
#pragma unroll
  for (uint32_t k = 0; k < 16; ++k) { loc[k] = cnt[tid * 16 + k]; sum += loc[k]; }
  const uint32_t lane = tid & 63, wv = tid >> 6;
  uint32_t x = sum;
#pragma unroll
  for (uint32_t o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_x[wv] = x;
  __syncthreads();
  uint32_t before = 0;
  for (uint32_t q = 0; q < wv; ++q) before += (uint32_t)s_x[q];
  uint32_t a = before + x - sum;
#pragma unroll
  for (uint32_t k = 0; k < 16; ++k) {
    const uint64_t u = (uint64_t)b * 16384 + tid * 16 + k;
    cnt[tid * 16 + k] = a;
    a += loc[k];
    if (u < n) rend[u] = ob + a;  // the end of u's in-edges
  }
  __syncthreads();
  for (unsigned long long i = tid; i < M; i += kRvBlock) {
    const unsigned long long rc = frec[f0 + i];
    const unsigned long long at = ob + atomicAdd(&cnt[rc & 16383], 1u);
    rsrc[at] = (uint32_t)((rc >> kRvShift) & 0x7FFFFFFFull);
    rslot[at] = (uint8_t)(rc >> 53);
  }
}
}  // namespace

// Every context sets grecv / gcrash (ctx_setup: = recv / crash; push-pull
// shards: the replicated sets); a launch without them would fault.
inline bool pp_state_ok(const DevState& s) { return s.recv && s.crash && s.grecv && s.gcrash; }

hipError_t pp_round(const DevState& s, unsigned long long* next, unsigned long long* sum, uint32_t t,
                    bool l2_only_flag, const PPSparse& sp, hipStream_t st) {
  if (!pp_state_ok(s) || !next) return hipErrorInvalidValue;
  if (sp.ctl) {
    hipLaunchKernelGGL(k_pp_mode, dim3(1), dim3(kPPSegs), 0, st, sp.ctl);
    // early rounds: the list grows at most ~(1 + in-degree)-fold per round;
    // a fixed grid, idle blocks leave at once
    hipLaunchKernelGGL(k_ppe_round, dim3(2048), dim3(kPPBlock), 0, st, s, next, sp, t);
  }
  unsigned long long* sumA = sum;
  unsigned long long* sumB = sum + pp_summary_words(s.W);
  const uint32_t sblocks = (uint32_t)std::min<uint64_t>((s.W + kPPBlock - 1) / kPPBlock, 4096);
  hipLaunchKernelGGL(k_pp_summary, dim3(sblocks), dim3(kPPBlock), 0, st, s, sumA, sumB, sp.ctl);
  const uint64_t S1 = pp_summary_words(s.W), S2 = pp_summary2_words(s.W);
  unsigned long long* sum2 = sum + 2 * S1;
  const uint32_t s2blocks = (uint32_t)std::min<uint64_t>((S1 + kPPBlock - 1) / kPPBlock, 1024);
  hipLaunchKernelGGL(k_pp_summary2, dim3(s2blocks), dim3(kPPBlock), 0, st, sum, S1, sum2, S2, sp.ctl);
  // 0: no LDS stage, every call checks L2 (N > ~1.02e9; GS_FLAG_PP_L2_ONLY
  // forces it so the parity tests cover that path at small N)
  const bool l2_only = S2 > kPPMaxS2 || l2_only_flag;
  const uint32_t S2l = l2_only ? 0u : (uint32_t)S2;
  const uint64_t groups = (s.W + kPPU - 1) / kPPU;  // one wave per kPPU words
  const uint32_t blocks =
      (uint32_t)std::min<uint64_t>((groups + kPPRoundBlock / 64 - 1) / (kPPRoundBlock / 64), 512);
  hipLaunchKernelGGL(k_pp_round, dim3(blocks), dim3(kPPRoundBlock), (size_t)2 * S2l * 8, st, s, next, sumA,
                     sumB, sum2, S2l, t, (const PPCtl*)sp.ctl, sp.fmask);
  if (sp.ctl) {  // no-op unless the round is bottom-up
    const uint64_t nrange = (s.W + kPPRange - 1) / kPPRange;
    const uint32_t bblocks = (uint32_t)std::min<uint64_t>((nrange + kPPWaves - 1) / kPPWaves, kPPSGrid);
    hipLaunchKernelGGL(k_ppb_round, dim3(bblocks), dim3(kPPSBlock), 0, st, s, next, sp, t);
    if (sp.dset) {
      const uint32_t nfine = (uint32_t)((s.n + 16383) >> 14);
      (void)hipMemsetAsync(sp.dcnt, 0, ((size_t)kPPDLists + kPPDRegions + nfine) * 8, st);
    }
    hipLaunchKernelGGL(k_ppa_round, dim3(bblocks), dim3(kPPSBlock), 0, st, s, next, sp, t);
    if (sp.dset) {  // no-ops unless the round is pull-answer
      const uint32_t nfine = (uint32_t)((s.n + 16383) >> 14);
      uint32_t* coarse = sp.dset + (size_t)kPPDLists * sp.dcap;
      uint32_t* fine = coarse + (size_t)kPPDRegions * sp.ccap;
      unsigned long long* cfill = sp.dcnt + kPPDLists;
      hipLaunchKernelGGL(k_ppd_part<false>, dim3(1024), dim3(kPPDBlock), 0, st, sp, next, sp.dset, sp.dcnt,
                         bblocks, sp.dcap, coarse, cfill, sp.ccap);
      hipLaunchKernelGGL(k_ppd_part<true>, dim3(1024), dim3(kPPDBlock), 0, st, sp, next, coarse, cfill,
                         kPPDRegions, sp.ccap, fine, cfill + kPPDRegions, sp.fcap);
      hipLaunchKernelGGL(k_ppd_apply, dim3(std::min<uint32_t>(nfine, 8192)), dim3(256), 0, st, sp, next, s.W, nfine);
    }
  }
  return hipGetLastError();
}

hipError_t pp_commit(const DevState& s, const unsigned long long* next, uint32_t t, const PPSparse& sp,
                     hipStream_t st) {
  const uint32_t blocks = (uint32_t)std::min<uint64_t>((s.W + kPPBlock - 1) / kPPBlock, 2048);
  hipLaunchKernelGGL(k_pp_commit, dim3(blocks), dim3(kPPBlock), 0, st, s, next, t, sp.ctl);
  if (sp.ctl) hipLaunchKernelGGL(k_ppe_commit, dim3(1024), dim3(kPPBlock), 0, st, s, next, sp, t);
  return hipGetLastError();
}

hipError_t pp_live_edges(const DevState& s, uint32_t* out, hipStream_t st) {
  if (!pp_state_ok(s)) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(out, 0, 4, st);
  if (e != hipSuccess) return e;
  const uint32_t blocks = (uint32_t)std::min<uint64_t>((s.n + kPPBlock - 1) / kPPBlock, 8192);
  hipLaunchKernelGGL(k_pp_live_edges, dim3(blocks), dim3(kPPBlock), 0, st, s, out);
  return hipGetLastError();
}

hipError_t pp_seed(const DevState& s, unsigned long long* next, uint32_t node, uint32_t* flag,
                   const PPSparse& sp, unsigned long long thr, unsigned long long bthr, unsigned long long athr,
                   const unsigned long long* callers, hipStream_t st) {
  if (sp.ctl) {
    hipError_t e = hipMemsetAsync(sp.ctl, 0, sizeof(PPCtl), st);
    if (e != hipSuccess) return e;
    if (callers) {
      hipLaunchKernelGGL(k_pp_set_callers, dim3(1), dim3(1), 0, st, sp.ctl, callers[0], callers[1]);
    } else {
      const uint32_t blocks = (uint32_t)std::min<uint64_t>((s.n + kPPBlock - 1) / kPPBlock, 4096);
      hipLaunchKernelGGL(k_pp_callers, dim3(blocks), dim3(kPPBlock), 0, st, s, sp.ctl);
    }
  }
  hipLaunchKernelGGL(k_pp_seed, dim3(1), dim3(1), 0, st, s, next, node, flag, sp, thr, bthr, athr);
  return hipGetLastError();
}

size_t pp_rev_scan_bytes(uint64_t n) {
  size_t bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (unsigned long long*)nullptr,
                                         (unsigned long long*)nullptr, (int)(n + 1));
  return bytes;
}

hipError_t pp_rev_build(const DevState& s, unsigned long long* rend, uint32_t* rsrc, uint8_t* rslot, void* tmp,
                        size_t tmp_bytes, hipStream_t st) {
  hipError_t e = hipMemsetAsync(rend, 0, (s.n + 1) * 8, st);
  if (e != hipSuccess) return e;
  const uint32_t blocks = (uint32_t)std::min<uint64_t>((s.n + kPPBlock - 1) / kPPBlock, 8192);
  hipLaunchKernelGGL(k_rev_count, dim3(blocks), dim3(kPPBlock), 0, st, s, rend);
  e = hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, rend, rend, (int)(s.n + 1), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_rev_fill, dim3(blocks), dim3(kPPBlock), 0, st, s, rend, rsrc, rslot);
  return hipGetLastError();
}

// The reverse table by partitioning (the k_rv_* kernels above): host-paced
// (a few small read-backs per pass).  The coarse bins are taken in passes of
// consecutive bins whose temporaries (8-B records: the coarse copy, then the
// fine regions, ~17 B per edge) fit the largest block the device allocator can
// give without returning cached memory to the driver (gs_devmem_largest): one
// pass when memory allows, more after other contexts left their blocks cached
// (every pass streams the table again, ~8 ms per pass at N = 1e9, where a
// hipMalloc right after large hipFrees stalled for seconds: DESIGN.md section
// 9).  GS_PP_REV_PASSES=k (read per call) forces k passes.  An error (no
// memory even for one bin, or a fine region past its planned size on a skewed
// table) leaves the outputs unspecified: the caller then builds with
// pp_rev_build.
hipError_t pp_rev_compact(const unsigned long long* rend, uint64_t n, uint16_t* rend16, unsigned long long* rbase,
                          uint32_t* ovf, hipStream_t st) {
  if (!n) return hipSuccess;
  const uint64_t blocks = std::min<uint64_t>((n + kPPBlock - 1) / kPPBlock, 8192);
  hipLaunchKernelGGL(k_rv_compact, dim3((uint32_t)blocks), dim3(kPPBlock), 0, st, rend, n, rend16, rbase, ovf);
  return hipGetLastError();
}

hipError_t pp_rev_build_part(const DevState& s, unsigned long long* rend, uint32_t* rsrc, uint8_t* rslot,
                             hipStream_t st, uint32_t* passes_out) {
  if (!s.n || s.n >= (1ull << 31)) return hipErrorInvalidValue;
  const uint64_t n = s.n, nbins = (n + (1ull << kRvShift) - 1) >> kRvShift, nbf = (n + 16383) >> 14;
  // small device arrays: chist[512] | cstart[513] | cend[512] | fstart[nbf+1] | ffill[nbf] | bbase[nbf] | tpre[513] | ovf
  const size_t small = 8 * (512 + 513 + 512 + (nbf + 1) + nbf + nbf) + 4 * 513 + 64;
  char* sm = nullptr;
  hipError_t e = dev_malloc(&sm, small);
  if (e != hipSuccess) return e;
  unsigned long long* d_chist = (unsigned long long*)sm;
  unsigned long long* d_cstart = d_chist + 512;
  unsigned long long* d_cend = d_cstart + 513;
  unsigned long long* d_fstart = d_cend + 512;
  unsigned long long* d_ffill = d_fstart + nbf + 1;
  unsigned long long* d_bbase = d_ffill + nbf;
  uint32_t* d_tpre = (uint32_t*)(d_bbase + nbf);
  uint32_t* d_ovf = d_tpre + 513;
  unsigned long long* tmp = nullptr;
  std::vector<unsigned long long> h(512, 0), cs(513, 0), fsz(nbf, 0), need(nbins, 0);
  uint32_t ovf = 0;
  const uint32_t grid = 512;
  auto done = [&](hipError_t r) {
    (void)hipStreamSynchronize(st);
    if (tmp) (void)dev_free(tmp);
    (void)dev_free(sm);
    return r;
  };
#define RV(x)                          \
  do {                                 \
    hipError_t e_ = (x);               \
    if (e_ != hipSuccess) return done(e_); \
  } while (0)
  RV(hipMemsetAsync(sm, 0, small, st));
  hipLaunchKernelGGL(k_rv_hist, dim3(grid), dim3(kRvBlock), 0, st, s, d_chist);
  RV(hipGetLastError());
  RV(hipMemcpyAsync(h.data(), d_chist, 512 * 8, hipMemcpyDeviceToHost, st));
  RV(hipStreamSynchronize(st));
  // exact coarse regions; a fine region planned at 1.125 x its node share of
  // its coarse region + 1024; need[c] = bin c's records in both copies
  for (uint64_t c = 0; c < nbins; ++c) {
    cs[c + 1] = cs[c] + h[c];
    const uint64_t nf = std::min<uint64_t>(256, nbf - c * 256);
    const uint64_t nodes_c = std::min<uint64_t>(1ull << kRvShift, n - (c << kRvShift));
    need[c] = h[c];
    for (uint64_t d = 0; d < nf; ++d) {
      const uint64_t fb = c * 256 + d, nodes_b = std::min<uint64_t>(16384, n - fb * 16384);
      const unsigned long long share = (unsigned long long)((double)h[c] * nodes_b / nodes_c);
      fsz[fb] = share + share / 8 + 1024;
      need[c] += fsz[fb];
    }
  }
  const unsigned long long E = cs[nbins];
  // passes of consecutive bins: forced count, or as many bins as fit the
  // largest block the allocator can give
  std::vector<uint32_t> cut{0};
  {
    const char* fp = getenv("GS_PP_REV_PASSES");
    const uint64_t forced = fp ? (uint64_t)std::max(atoi(fp), 1) : 0;
    if (forced) {
      const uint64_t per = (nbins + forced - 1) / forced;
      for (uint64_t c = per; c < nbins; c += per) cut.push_back((uint32_t)c);
    } else {
      const uint64_t cap = gs_devmem_largest() / 8;
      uint64_t acc = 0;
      for (uint64_t c = 0; c < nbins; ++c) {
        if (need[c] > cap) return done(hipErrorOutOfMemory);  // not even one bin: the atomic build
        if (acc + need[c] > cap) {
          cut.push_back((uint32_t)c);
          acc = 0;
        }
        acc += need[c];
      }
    }
    cut.push_back((uint32_t)nbins);
  }
  const size_t P = cut.size() - 1;
  if (passes_out) *passes_out = (uint32_t)P;
  unsigned long long rec_max = 1, frec_max = 1;
  for (size_t p = 0; p < P; ++p) {
    unsigned long long r = 0, f = 0;
    for (uint32_t c = cut[p]; c < cut[p + 1]; ++c) {
      r += h[c];
      f += need[c] - h[c];
    }
    rec_max = std::max(rec_max, r);
    frec_max = std::max(frec_max, f);
  }
  // one block for both copies: it fits the extent the plan was made for
  RV(dev_malloc(&tmp, (rec_max + frec_max) * 8));
  unsigned long long* rec = tmp;
  unsigned long long* frec = tmp + rec_max;
  for (size_t p = 0; p < P; ++p) {
    const uint32_t blo = cut[p], bhi = cut[p + 1], nb = bhi - blo;
    const uint64_t fb0 = (uint64_t)blo * 256, fb1 = std::min<uint64_t>((uint64_t)bhi * 256, nbf), nfl = fb1 - fb0;
    std::vector<unsigned long long> csl(nb + 1, 0), cel(nb, 0), fsl(nfl + 1, 0), ffl(nfl, 0), bbl(nfl, 0);
    std::vector<uint32_t> tpl(nb + 1, 0);
    for (uint32_t c = 0; c < nb; ++c) {
      csl[c + 1] = csl[c] + h[blo + c];
      cel[c] = csl[c + 1];
      tpl[c + 1] = tpl[c] + (uint32_t)((h[blo + c] + kRvTile - 1) / kRvTile);
    }
    for (uint64_t i = 0; i < nfl; ++i) fsl[i + 1] = fsl[i] + fsz[fb0 + i];
    RV(hipMemcpyAsync(d_cstart, csl.data(), (nb + 1) * 8, hipMemcpyHostToDevice, st));
    RV(hipMemcpyAsync(d_cend, cel.data(), nb * 8, hipMemcpyHostToDevice, st));
    RV(hipMemcpyAsync(d_fstart, fsl.data(), (nfl + 1) * 8, hipMemcpyHostToDevice, st));
    RV(hipMemcpyAsync(d_tpre, tpl.data(), (nb + 1) * 4, hipMemcpyHostToDevice, st));
    RV(hipMemsetAsync(d_ffill, 0, nfl * 8, st));
    unsigned long long* d_cfill = d_chist;  // reused: the fills of the coarse pass
    RV(hipMemsetAsync(d_cfill, 0, 512 * 8, st));
    const uint64_t rounds = (n + kRvRows - 1) / kRvRows;
    hipLaunchKernelGGL(k_rv_coarse, dim3((uint32_t)std::min<uint64_t>(rounds, grid)), dim3(kRvBlock), 0, st, s,
                       d_cstart, d_cfill, rec, blo, bhi);
    RV(hipGetLastError());
    if (tpl[nb]) {
      hipLaunchKernelGGL(k_rv_fine, dim3(std::min<uint32_t>(tpl[nb], grid)), dim3(kRvBlock), 0, st, rec, d_cstart,
                         d_cend, d_tpre, nb, d_fstart, d_ffill, frec, d_ovf);
      RV(hipGetLastError());
    }
    RV(hipMemcpyAsync(ffl.data(), d_ffill, nfl * 8, hipMemcpyDeviceToHost, st));
    RV(hipMemcpyAsync(&ovf, d_ovf, 4, hipMemcpyDeviceToHost, st));
    RV(hipStreamSynchronize(st));
    if (ovf) return done(hipErrorInvalidValue);  // a skewed table: the atomic build
    bbl[0] = cs[blo];  // every in-edge of the earlier buckets lies in the earlier bins
    for (uint64_t b = 1; b < nfl; ++b) bbl[b] = bbl[b - 1] + ffl[b - 1];
    RV(hipMemcpyAsync(d_bbase, bbl.data(), nfl * 8, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_rv_final, dim3((uint32_t)nfl), dim3(kRvBlock), 0, st, frec, d_fstart, d_ffill, d_bbase, n,
                       rend, rsrc, rslot, (uint32_t)fb0);
    RV(hipGetLastError());
    RV(hipStreamSynchronize(st));  // this pass's host arrays and the temporaries are reused
  }
  RV(hipMemcpyAsync(rend + n, &E, 8, hipMemcpyHostToDevice, st));
#undef RV
  return done(hipSuccess);
}

hipError_t pp_fmask_build(const DevState& s, const unsigned long long* rend, const uint32_t* rsrc,
                          const uint8_t* rslot, uint8_t* fmask, hipStream_t st) {
  hipError_t e = hipMemsetAsync(fmask, 0, (s.n + 3) & ~3ull, st);
  if (e != hipSuccess) return e;
  const uint32_t blocks = (uint32_t)std::min<uint64_t>((s.n + kPPBlock - 1) / kPPBlock, 8192);
  hipLaunchKernelGGL(k_pp_fmask, dim3(blocks), dim3(kPPBlock), 0, st, s, rend, rsrc, rslot, (uint32_t*)fmask);
  return hipGetLastError();
}

size_t pp_rev_range_scan_bytes(uint64_t n) { return pp_rev_scan_bytes(n); }

hipError_t pp_rev_count_range(const uint8_t* deg, const uint32_t* ids, uint64_t nfull, uint32_t stride, uint64_t lo,
                              uint64_t hi, unsigned long long* rend, void* tmp, size_t tmp_bytes, hipStream_t st) {
  const uint64_t n = hi - lo;
  hipError_t e = hipMemsetAsync(rend, 0, (n + 1) * 8, st);
  if (e != hipSuccess) return e;
  const uint32_t blocks = (uint32_t)std::min<uint64_t>((nfull + kPPBlock - 1) / kPPBlock, 8192);
  hipLaunchKernelGGL(k_rev_count_range, dim3(blocks), dim3(kPPBlock), 0, st, deg, ids, nfull, stride, lo, hi, rend);
  return hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, rend, rend, (int)(n + 1), st);
}

hipError_t pp_rev_fill_range(const uint8_t* deg, const uint32_t* ids, uint64_t nfull, uint32_t stride, uint64_t lo,
                             uint64_t hi, unsigned long long* rend, uint32_t* rsrc, uint8_t* rslot, hipStream_t st) {
  const uint32_t blocks = (uint32_t)std::min<uint64_t>((nfull + kPPBlock - 1) / kPPBlock, 8192);
  hipLaunchKernelGGL(k_rev_fill_range, dim3(blocks), dim3(kPPBlock), 0, st, deg, ids, nfull, stride, lo, hi, rend,
                     rsrc, rslot);
  return hipGetLastError();
}

hipError_t pp_rfail_build(const DevState& s, const unsigned long long* rend, const uint32_t* rsrc,
                          const uint8_t* rslot, uint32_t* rfail, hipStream_t st) {
  const uint64_t NW = (s.n * s.stride + 31) >> 5;  // at most; word NW + 1 is the hub flag
  uint32_t* hub = rfail + NW + 1;
  hipError_t e = hipMemsetAsync(rfail, 0, (NW + 2) * 4, st);
  if (e != hipSuccess) return e;
  const uint32_t blocks = (uint32_t)std::min<uint64_t>((s.W + kPPBlock - 1) / kPPBlock, 8192);
  hipLaunchKernelGGL(k_pp_rfail, dim3(blocks ? blocks : 1), dim3(kPPBlock), 0, st, s, rend, rsrc, rslot, rfail, hub);
  const uint32_t hblocks = (uint32_t)std::min<uint64_t>((s.n + 64 * (kPPBlock / 64) - 1) / (64 * (kPPBlock / 64)), 4096);
  hipLaunchKernelGGL(k_pp_rfail_hubs, dim3(hblocks ? hblocks : 1), dim3(kPPBlock), 0, st, s, rend, rsrc, rfail, hub);
  return hipGetLastError();
}

hipError_t pp_fmask_any(const uint8_t* fmask, uint64_t n, unsigned long long* fany, hipStream_t st) {
  const uint64_t W = (n + 63) >> 6;
  const uint32_t blocks = (uint32_t)std::min<uint64_t>((W + kPPBlock - 1) / kPPBlock, 8192);
  hipLaunchKernelGGL(k_pp_fmask_any, dim3(blocks), dim3(kPPBlock), 0, st, fmask, n, fany);
  return hipGetLastError();
}

hipError_t pp_fmask_rows(const DevState& s, uint8_t* fmask, hipStream_t st) {
  if (!pp_state_ok(s) || !fmask) return hipErrorInvalidValue;
  const uint32_t blocks = (uint32_t)std::min<uint64_t>((s.n + kPPBlock - 1) / kPPBlock, 8192);
  hipLaunchKernelGGL(k_pp_fmask_rows, dim3(blocks), dim3(kPPBlock), 0, st, s, fmask);
  return hipGetLastError();
}

hipError_t pp_round_shard(const DevState& s, unsigned long long* next, unsigned long long* gnext, uint32_t t,
                          const PPSparse& sp, uint32_t mode, hipStream_t st) {
  if (!pp_state_ok(s) || !next || !sp.ctl || !sp.rend || !sp.rsrc || !sp.rslot || (s.check_crashed && !sp.fmask) ||
      (mode == PP_ANSWER && !gnext) || (mode != PP_ANSWER && mode != PP_BOTTOM))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_pp_set_mode, dim3(1), dim3(1), 0, st, sp.ctl, mode);
  const uint64_t nrange = (s.W + kPPRange - 1) / kPPRange;
  const uint32_t bblocks = (uint32_t)std::min<uint64_t>((nrange + kPPWaves - 1) / kPPWaves, kPPSGrid);
  if (mode == PP_BOTTOM)
    hipLaunchKernelGGL(k_ppb_round, dim3(bblocks ? bblocks : 1), dim3(kPPSBlock), 0, st, s, next, sp, t);
  else
    hipLaunchKernelGGL(k_ppa_round, dim3(bblocks ? bblocks : 1), dim3(kPPSBlock), 0, st, s, gnext, sp, t);
  return hipGetLastError();
}

hipError_t pp_count(const unsigned long long* words, uint64_t nwords, unsigned long long* out, hipStream_t st) {
  hipLaunchKernelGGL(k_pp_count, dim3(1), dim3(1), 0, st, words, 0ull, out);  // zero the total
  const uint32_t blocks = (uint32_t)std::min<uint64_t>((nwords + kPPBlock - 1) / kPPBlock, 2048);
  hipLaunchKernelGGL(k_pp_count, dim3(blocks ? blocks : 1), dim3(kPPBlock), 0, st, words, nwords, out);
  return hipGetLastError();
}

hipError_t pp_or_slices(unsigned long long* dst, const unsigned long long* src, uint32_t nslices, uint64_t words,
                        hipStream_t st) {
  const uint32_t blocks = (uint32_t)std::min<uint64_t>((words + kPPBlock - 1) / kPPBlock, 2048);
  hipLaunchKernelGGL(k_pp_or_slices, dim3(blocks ? blocks : 1), dim3(kPPBlock), 0, st, dst, src, nslices, words);
  return hipGetLastError();
}

}  // namespace gs
