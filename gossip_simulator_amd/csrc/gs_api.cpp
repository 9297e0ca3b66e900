// gs_api.cpp -- the C ABI of libgossip_hip.so (include/gossip.h).
//
// Owns one HIP device + stream per context and the HBM-resident state of
// gs_internal.h.  Replaces the reference's main() body (simulator.go:207-253):
// allocation (:208-212), overlay (:214-235), broadcast and polling (:237-253).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gossip.h"
#include "gs_internal.h"

using namespace gs;

struct gs_ctx {
  gs_params p{};
  int dev = 0;
  hipStream_t stream = nullptr;  // where device work is issued (own, or gs_set_stream's)
  hipStream_t own = nullptr;     // the context's own stream
  std::string err;
  DevState st{};
  uint8_t* d_deg = nullptr;
  uint32_t* d_ids = nullptr;
  void* d_state = nullptr;  // one allocation for recv/crash/ring/cflag/clist/ccount/stats
  uint32_t* d_cnt = nullptr;
  uint32_t* d_err = nullptr;
  unsigned long long* d_failed = nullptr;  // pre-failed mask, re-applied by gs_reset
  size_t state_bytes = 0;
  unsigned long long* h_stats = nullptr;  // pinned, kStatSlots * kStatFields
  bool peers = false, begun = false, failed = false;
  uint64_t t = 0, fired = 0, sent = 0, msgs = 0, recv = 0, crashed = 0, pending = 0;
  std::vector<hipEvent_t> ev;
  gs_timing timing{};
  // push-pull extension (gs_pushpull.hip)
  bool pp = false;
  unsigned long long* d_next = nullptr;  // informed set being built (state block)
  unsigned long long* d_ppsum = nullptr;  // push-pull word summaries (state block)
  uint32_t* d_flag = nullptr;
  // window engine (gs_window.hip)
  bool win = false;
  WinState ws{};
  void* d_win = nullptr;      // fcount + small per-window buffers
  void* d_flist = nullptr;    // [R][nfine][16384] u16
  size_t fcount_bytes = 0;
  struct Buf { void* p = nullptr; size_t bytes = 0; } gmap, cmsg, fmsg, tmp;
  unsigned long long* h_cap = nullptr;  // pinned [257] coarse region plan
  unsigned long long* h_misc = nullptr; // pinned scratch (counts, flags)
};

namespace {

int fail(gs_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

bool grow(gs_ctx::Buf& b, size_t bytes) {
  if (b.bytes >= bytes) return true;
  const size_t nb = std::max(bytes, b.bytes + b.bytes / 4);
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.bytes = 0;
  if (hipMalloc(&b.p, nb) != hipSuccess) return false;
  b.bytes = nb;
  return true;
}

// Window-engine buffers.  Sizes at n = 1e9, R = 20: flist 40 GB (two bytes
// per node per ring slot), fcount 4.9 MB; message buffers grow on demand.
int alloc_window(gs_ctx* c) {
  const DevState& s = c->st;
  WinState& w = c->ws;
  w.n = s.n;
  w.W = s.W;
  w.nfine = (uint32_t)((s.n + kFineNodes - 1) >> kFineLog);
  w.ncoarse = (w.nfine + 255) / 256;
  w.R = s.R;
  w.delay_low = s.delay_low;
  w.delay_span = s.delay_span;
  w.kd = s.kd;
  w.kc = s.kc;
  w.key = s.key;
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t units = (size_t)kMaxWindow * w.nfine + 1;
  const size_t b_fc = al((size_t)w.R * w.nfine * 4), b_units = al(units * 8),
               b_small = al(256 * 8) * 3 + al(257 * 4) + al(257 * 8) + al(kMaxWindow * 8),
               b_fhist = al(((size_t)w.ncoarse * 256 + 1) * 8), b_fbase = al(((size_t)w.nfine + 1) * 8),
               b_ffill = al((size_t)w.nfine * 8),
               b_sst = al((size_t)kStatShards * kMaxWindow * kStatFields * 8);
  const size_t total = b_fc + 2 * b_units + b_small + b_fhist + b_fbase + b_ffill + b_sst;
  if (hipMalloc(&c->d_win, total) != hipSuccess)
    return fail(c, GS_ENOMEM, "cannot allocate window-engine buffers");
  const size_t flist = (size_t)w.R * w.nfine * kFineNodes * 2;
  if (hipMalloc(&c->d_flist, flist) != hipSuccess)
    return fail(c, GS_ENOMEM, "cannot allocate " + std::to_string(flist >> 20) + " MiB of fire lists");
  char* q = (char*)c->d_win;
  w.fcount = (uint32_t*)q; q += b_fc;
  w.usize = (unsigned long long*)q; q += b_units;
  w.unit_off = (unsigned long long*)q; q += b_units;
  w.chist = (unsigned long long*)q; q += al(256 * 8);
  w.cfill = (unsigned long long*)q; q += al(256 * 8);
  w.ccap = (unsigned long long*)q; q += al(257 * 8);
  w.tprefix = (uint32_t*)q; q += al(257 * 4);
  w.tfires = (unsigned long long*)q;
  q = (char*)c->d_win + b_fc + 2 * b_units + b_small;
  w.fhist = (unsigned long long*)q; q += b_fhist;
  w.fstart = (unsigned long long*)q; q += b_fbase;
  w.ffill = (unsigned long long*)q; q += b_ffill;
  w.sstats = (unsigned long long*)q; q += b_sst;
  w.dbg = nullptr;
  if (getenv("GS_STAMPS") && hipMalloc(&w.dbg, 2 * kStampPhases * 8) == hipSuccess)
    (void)hipMemset(w.dbg, 0, 2 * kStampPhases * 8);
  w.flist = (uint16_t*)c->d_flist;
  c->fcount_bytes = (size_t)w.R * w.nfine * 4;
  if (hipMemsetAsync(c->d_win, 0, total, c->stream) != hipSuccess)
    return fail(c, GS_EDEVICE, "memset of window buffers failed");
  if (hipHostMalloc((void**)&c->h_cap, 257 * 8) != hipSuccess ||
      hipHostMalloc((void**)&c->h_misc, 512 * 8) != hipSuccess)
    return fail(c, GS_ENOMEM, "cannot allocate pinned window buffers");
  return GS_OK;
}

// Coarse region plan: bucket c gets its node share of the window's T friend
// slots (a kept send is at most one slot) plus 4096, or exactly `exact[c]`.
void plan_coarse(gs_ctx* c, uint64_t T, const unsigned long long* exact) {
  const WinState& w = c->ws;
  unsigned long long a = 0;
  for (uint32_t b = 0; b < 256; ++b) {
    c->h_cap[b] = a;
    if (b >= w.ncoarse) continue;
    if (exact) { a += exact[b]; continue; }
    const uint64_t lo = (uint64_t)b << kCoarseShift;
    const uint64_t hi = std::min<uint64_t>(w.n, lo + (1ull << kCoarseShift));
    a += (unsigned long long)((long double)T * (long double)(hi - lo) / (long double)w.n) + 4096;
  }
  c->h_cap[256] = a;
}

void refresh_window(gs_ctx* c) {
  WinState& w = c->ws;
  w.deg = c->st.deg;
  w.ids = c->st.ids;
  w.recv = c->st.recv;
  w.crash = c->st.crash;
  w.stats = c->st.stats;
  w.err = c->d_err;
  w.stride = c->st.stride;
  w.stride_magic = c->st.stride_magic;
}

#define CK(c, expr)                                                                   \
  do {                                                                                \
    hipError_t e_ = (expr);                                                           \
    if (e_ != hipSuccess)                                                             \
      return fail((c), GS_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

uint32_t ring_slots(const gs_params& p) { return p.delay_high > 2 ? (uint32_t)p.delay_high : 2u; }

int check_params(const gs_params* p, std::string& why) {
  if (!p) { why = "params is NULL"; return GS_EINVAL; }
  if (p->n == 0) { why = "n must be >= 1 (simulator.go:240 panics on rand.Intn(0))"; return GS_EINVAL; }
  if (p->n > 0x7FFFFFFFull) { why = "n must be < 2^31"; return GS_EINVAL; }
  if (p->delay_high <= p->delay_low) {
    why = "delayhigh must exceed delaylow (simulator.go:167 panics on rand.Intn(<=0))";
    return GS_EINVAL;
  }
  if (p->fanout < 0 || p->fanin < 0 || p->fanout > 255 || p->fanin > 255) {
    why = "fanout/fanin must be in [0, 255]";
    return GS_EINVAL;
  }
  if (ring_slots(*p) > 4096) { why = "delayhigh must be <= 4096"; return GS_EINVAL; }
  if (p->model > GS_MODEL_PUSHPULL) { why = "model must be GS_MODEL_FLOOD or GS_MODEL_PUSHPULL"; return GS_EINVAL; }
  if (p->model == GS_MODEL_PUSHPULL && !(p->node_lo == 0 && (p->node_hi == 0 || p->node_hi == p->n))) {
    why = "push-pull runs are not node-range sharded (shard trials instead)";
    return GS_EINVAL;
  }
  return GS_OK;
}

void refresh_state(gs_ctx* c) {
  DevState& s = c->st;
  s.deg = c->d_deg;
  s.ids = c->d_ids;
  if (c->win) refresh_window(c);
}

int set_stride(gs_ctx* c, uint32_t stride) {
  if (stride < 2 || stride > 255) return fail(c, GS_EINVAL, "row stride must be in [2, 255]");
  if (c->win && stride > kWinMaxStride)
    return fail(c, GS_EINVAL, "rows longer than 32 need GS_FLAG_TICK_ENGINE (or fanin > 32 at create)");
  c->st.stride = stride;
  c->st.stride_magic = (uint32_t)((1ull << 32) / stride + 1);
  if (c->win) refresh_window(c);
  return GS_OK;
}

int alloc_table(gs_ctx* c, uint32_t stride) {
  if (c->d_deg) (void)hipFree(c->d_deg);
  if (c->d_ids) (void)hipFree(c->d_ids);
  c->d_deg = nullptr;
  c->d_ids = nullptr;
  const uint64_t n = c->p.n;
  if (hipMalloc(&c->d_deg, n) != hipSuccess || hipMalloc(&c->d_ids, n * stride * 4ull) != hipSuccess)
    return fail(c, GS_ENOMEM, "cannot allocate the peer table on the device");
  int rc = set_stride(c, stride);
  if (rc) return rc;
  refresh_state(c);
  return GS_OK;
}

__global__ void k_validate_peers(const uint8_t* deg, const uint32_t* ids, uint64_t n,
                                 uint32_t stride, uint32_t* err) {
  for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n;
       v += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t d = deg[v];
    if (d > stride) { atomicOr(err, 1u); continue; }
    for (uint32_t j = 0; j < d; ++j)
      if (ids[v * stride + j] >= n) atomicOr(err, 2u);
  }
}

int validate_table(gs_ctx* c) {
  CK(c, hipMemsetAsync(c->d_err, 0, 4, c->stream));
  const uint64_t blocks = std::min<uint64_t>((c->p.n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_validate_peers, dim3((uint32_t)blocks), dim3(256), 0, c->stream, c->d_deg,
                     c->d_ids, c->p.n, c->st.stride, c->d_err);
  CK(c, hipGetLastError());
  uint32_t e = 0;
  CK(c, hipMemcpyAsync(&e, c->d_err, 4, hipMemcpyDeviceToHost, c->stream));
  CK(c, hipStreamSynchronize(c->stream));
  if (e & 1) return fail(c, GS_EINVAL, "a friends-list length exceeds the row stride");
  if (e & 2) return fail(c, GS_EINVAL, "a friend id is >= n");
  return GS_OK;
}

// The window engine reads friend rows without the length byte: slots past a
// node's list are set to kEmptyMsg on the device copy.
int seal_rows(gs_ctx* c) {
  if (!c->win) return GS_OK;
  CK(c, win_seal_rows(c->d_deg, c->d_ids, c->p.n, c->st.stride, c->stream));
  CK(c, hipStreamSynchronize(c->stream));
  return GS_OK;
}

bool covered(uint64_t recv, uint64_t n) {
  // simulator.go:246-248, in float32
  volatile float a = (float)recv, b = (float)n;
  volatile float pct = a / b;
  return pct >= 0.99f;
}

}  // namespace

extern "C" {

int gs_version(void) { return GS_ABI_VERSION; }

const char* gs_strerror(int code) {
  switch (code) {
    case GS_OK: return "ok";
    case GS_EINVAL: return "invalid argument";
    case GS_ELIVELOCK: return "overlay livelock";
    case GS_EREJECT: return "replacement rejection exhausted";
    case GS_ENOMEM: return "out of memory";
    case GS_EDEVICE: return "HIP device error";
    case GS_EOVERFLOW: return "counter overflow";
    default: return "unknown error";
  }
}

const char* gs_last_error(const gs_ctx* c) { return c ? c->err.c_str() : "NULL context"; }

int gs_create(const gs_params* params, gs_ctx** out) {
  if (!out) return GS_EINVAL;
  *out = nullptr;
  std::string why;
  int rc = check_params(params, why);
  if (rc) {
    fprintf(stderr, "gs_create: %s\n", why.c_str());
    return rc;
  }
  gs_ctx* c = new gs_ctx();
  c->p = *params;
  c->dev = params->device;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    fprintf(stderr, "gs_create: no HIP device visible (libgossip_hip needs an MI355X)\n");
    delete c;
    return GS_EDEVICE;
  }
  if (c->dev < 0 || c->dev >= ndev) {
    fprintf(stderr, "gs_create: device %d out of range (%d visible)\n", c->dev, ndev);
    delete c;
    return GS_EDEVICE;
  }
  hipDeviceProp_t prop;
  if (hipSetDevice(c->dev) != hipSuccess || hipGetDeviceProperties(&prop, c->dev) != hipSuccess ||
      strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    fprintf(stderr, "gs_create: device %d is not gfx950 (%s)\n", c->dev, prop.gcnArchName);
    delete c;
    return GS_EDEVICE;
  }
  if (hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return GS_EDEVICE;
  }
  c->stream = c->own;
  DevState& s = c->st;
  {
    uint64_t lo = c->p.node_lo, hi = c->p.node_hi;
    if (lo == 0 && hi == 0) hi = c->p.n;
    if (lo > hi || hi > c->p.n || ((lo & 4095) && lo != c->p.n) ||
        ((hi & 4095) && hi != c->p.n)) {
      fprintf(stderr, "gs_create: node range [%llu, %llu) must be 4096-aligned within [0, n]\n",
              (unsigned long long)lo, (unsigned long long)hi);
      gs_destroy(c);
      return GS_EINVAL;
    }
    s.lo = (uint32_t)lo;
    s.hi = (uint32_t)hi;
    s.chunk_lo = (uint32_t)(lo >> kChunkNodesLog);
    s.chunk_hi = (uint32_t)((hi + (1ull << kChunkNodesLog) - 1) >> kChunkNodesLog);
    s.sharded = !(lo == 0 && hi == c->p.n);
  }
  s.n = c->p.n;
  s.W = (s.n + 63) / 64;
  s.C = (uint32_t)((s.n + (1ull << kChunkNodesLog) - 1) >> kChunkNodesLog);
  s.CS = (s.C + kShards - 1) / kShards;
  s.R = ring_slots(c->p);
  s.delay_low = c->p.delay_low;
  s.delay_span = (uint32_t)(c->p.delay_high - c->p.delay_low);
  s.kd = gs_threshold(c->p.drop_rate);
  s.kc = gs_threshold(c->p.crash_rate);
  s.key = Key{(uint32_t)c->p.seed, (uint32_t)(c->p.seed >> 32), c->p.trial};
  // Engine: the window engine (gs_window.hip) unless the run is node-range
  // sharded (per-tick frontier exchange) or its ring is too long for LDS.
  // Push-pull has its own round kernels (gs_pushpull.hip).
  c->pp = c->p.model == GS_MODEL_PUSHPULL;
  c->win = !c->pp && !s.sharded && s.R <= kWinMaxRing && !(c->p.flags & GS_FLAG_TICK_ENGINE) &&
           (uint32_t)std::max(c->p.fanout, c->p.fanin) <= kWinMaxStride;
  // One state allocation, 256-B aligned sub-buffers; everything before
  // `stats` is per-broadcast state that gs_reset clears.
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const bool tick = !c->win && !c->pp;
  const size_t b_next = c->pp ? al(s.W * 8) + al(pp_summary_total_words(s.W) * 8) : 0;
  const size_t b_bits = al(s.W * 8), b_ring = tick ? al((size_t)s.R * s.W * 8) : 0,
               b_cflag = tick ? al((size_t)s.R * s.C * 4) : 0,
               b_clist = tick ? al((size_t)s.R * kShards * s.CS * 4) : 0,
               b_ccount = tick ? al((size_t)s.R * kShards * kCounterStride * 4) : 0,
               b_stats = al((size_t)kStatSlots * kStatFields * 8);
  const size_t total = 2 * b_bits + b_next + b_ring + b_cflag + b_clist + b_ccount + b_stats + 256;
  c->state_bytes = total;
  if (hipMalloc(&c->d_state, total) != hipSuccess) {
    fprintf(stderr, "gs_create: cannot allocate %zu bytes of device state\n", total);
    gs_destroy(c);
    return GS_ENOMEM;
  }
  char* q = (char*)c->d_state;
  s.recv = (unsigned long long*)q; q += b_bits;
  s.crash = (unsigned long long*)q; q += b_bits;
  c->d_next = b_next ? (unsigned long long*)q : nullptr;
  c->d_ppsum = b_next ? (unsigned long long*)(q + al(s.W * 8)) : nullptr;
  q += b_next;
  s.ring = (unsigned long long*)q; q += b_ring;
  s.cflag = (uint32_t*)q; q += b_cflag;
  s.clist = (uint32_t*)q; q += b_clist;
  s.ccount = (uint32_t*)q; q += b_ccount;
  s.stats = (unsigned long long*)q; q += b_stats;
  c->d_err = (uint32_t*)q;
  c->d_flag = c->d_err + 1;
  if (tick && s.kc > 0) {
    if (hipMalloc(&c->d_cnt, s.n * 4) != hipSuccess) {
      fprintf(stderr, "gs_create: cannot allocate arrival counters\n");
      gs_destroy(c);
      return GS_ENOMEM;
    }
  }
  s.cnt = c->d_cnt;
  if (c->win) {
    rc = alloc_window(c);
    if (rc) {
      fprintf(stderr, "gs_create: %s\n", c->err.c_str());
      gs_destroy(c);
      return rc;
    }
  }
  if (hipMemsetAsync(c->d_state, 0, total, c->stream) != hipSuccess ||
      (c->d_cnt && hipMemsetAsync(c->d_cnt, 0, s.n * 4, c->stream) != hipSuccess) ||
      hipHostMalloc((void**)&c->h_stats, (size_t)kStatSlots * kStatFields * 8) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess) {
    gs_destroy(c);
    return GS_EDEVICE;
  }
  *out = c;
  return GS_OK;
}

void gs_destroy(gs_ctx* c) {
  if (!c) return;
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->ws.dbg) {
    unsigned long long h[2 * kStampPhases];
    if (hipMemcpy(h, c->ws.dbg, sizeof h, hipMemcpyDeviceToHost) == hipSuccess)
      for (int cls = 0; cls < 2; ++cls) {  // k_resolve phases (GS_STAMPS=1), thread 0 of every workgroup
        const unsigned long long* d = h + cls * kStampPhases;
        if (!d[0]) continue;
        fprintf(stderr, "[stamps] k_resolve %s: %llu buckets, mean kcycles per bucket per phase:",
                cls ? "M>=1024" : "M<1024", d[0]);
        for (uint32_t i = 1; i < kStampPhases; ++i) fprintf(stderr, " %.2f", d[i] * 1e-3 / d[0]);
        fprintf(stderr, "\n");
      }
    (void)hipFree(c->ws.dbg);
  }
  for (hipEvent_t e : c->ev) (void)hipEventDestroy(e);
  if (c->d_deg) (void)hipFree(c->d_deg);
  if (c->d_ids) (void)hipFree(c->d_ids);
  if (c->d_state) (void)hipFree(c->d_state);
  if (c->d_cnt) (void)hipFree(c->d_cnt);
  if (c->d_failed) (void)hipFree(c->d_failed);
  if (c->d_win) (void)hipFree(c->d_win);
  if (c->d_flist) (void)hipFree(c->d_flist);
  for (gs_ctx::Buf* b : {&c->gmap, &c->cmsg, &c->fmsg, &c->tmp})
    if (b->p) (void)hipFree(b->p);
  if (c->h_cap) (void)hipHostFree(c->h_cap);
  if (c->h_misc) (void)hipHostFree(c->h_misc);
  if (c->h_stats) (void)hipHostFree(c->h_stats);
  if (c->own) (void)hipStreamDestroy(c->own);
  delete c;
}

int gs_load_peers(gs_ctx* c, const uint8_t* deg, const uint32_t* ids, uint32_t stride) {
  if (!c || !deg || !ids || stride == 0 || stride > 255) return fail(c, GS_EINVAL, "bad peer table");
  if (c->begun) return fail(c, GS_EINVAL, "peers must be loaded before gs_broadcast_begin");
  CK(c, hipSetDevice(c->dev));
  const uint32_t S = stride < 2 ? 2 : stride;
  int rc = alloc_table(c, S);
  if (rc) return rc;
  const uint64_t n = c->p.n;
  CK(c, hipMemcpyAsync(c->d_deg, deg, n, hipMemcpyHostToDevice, c->stream));
  if (S == stride) {
    CK(c, hipMemcpyAsync(c->d_ids, ids, n * S * 4, hipMemcpyHostToDevice, c->stream));
    CK(c, hipStreamSynchronize(c->stream));
  } else {
    std::vector<uint32_t> tmp(n * S, 0);
    for (uint64_t v = 0; v < n; ++v) tmp[v * S] = ids[v];
    CK(c, hipMemcpyAsync(c->d_ids, tmp.data(), n * S * 4, hipMemcpyHostToDevice, c->stream));
    CK(c, hipStreamSynchronize(c->stream));
  }
  rc = validate_table(c);
  if (rc) return rc;
  rc = seal_rows(c);
  if (rc) return rc;
  c->peers = true;
  return GS_OK;
}

int gs_load_peers_device(gs_ctx* c, const void* d_deg, const void* d_ids, uint32_t stride) {
  if (!c || !d_deg || !d_ids || stride < 2 || stride > 255)
    return fail(c, GS_EINVAL, "bad device peer table (stride must be in [2,255])");
  if (c->begun) return fail(c, GS_EINVAL, "peers must be loaded before gs_broadcast_begin");
  CK(c, hipSetDevice(c->dev));
  int rc = alloc_table(c, stride);
  if (rc) return rc;
  CK(c, hipMemcpyAsync(c->d_deg, d_deg, c->p.n, hipMemcpyDeviceToDevice, c->stream));
  CK(c, hipMemcpyAsync(c->d_ids, d_ids, c->p.n * stride * 4ull, hipMemcpyDeviceToDevice, c->stream));
  rc = validate_table(c);
  if (rc) return rc;
  rc = seal_rows(c);
  if (rc) return rc;
  c->peers = true;
  return GS_OK;
}

int gs_read_peers(gs_ctx* c, uint8_t* deg, uint32_t* ids, uint32_t* stride_out) {
  if (!c || !c->peers) return fail(c, GS_EINVAL, "no peer table");
  if (stride_out) *stride_out = c->st.stride;
  CK(c, hipSetDevice(c->dev));
  if (deg) CK(c, hipMemcpyAsync(deg, c->d_deg, c->p.n, hipMemcpyDeviceToHost, c->stream));
  if (ids)
    CK(c, hipMemcpyAsync(ids, c->d_ids, c->p.n * c->st.stride * 4ull, hipMemcpyDeviceToHost, c->stream));
  CK(c, hipStreamSynchronize(c->stream));
  return GS_OK;
}

namespace {
struct WinSink {
  gs_window* win;
  size_t cap, n;
  static void push(void* self, uint64_t tick, uint64_t mk, uint64_t bk) {
    WinSink* w = (WinSink*)self;
    if (w->win && w->n < w->cap) w->win[w->n] = gs_window{tick, mk, bk};
    ++w->n;
  }
};
}  // namespace

int gs_build_overlay(gs_ctx* c, uint64_t max_ticks, gs_window* win, size_t cap, size_t* nwin,
                     uint64_t* final_tick) {
  if (!c) return GS_EINVAL;
  if (c->begun) return fail(c, GS_EINVAL, "overlay must be built before gs_broadcast_begin");
  CK(c, hipSetDevice(c->dev));
  const uint32_t fo = (uint32_t)c->p.fanout, fi = (uint32_t)c->p.fanin;
  uint32_t stride = fo > fi ? fo : fi;
  if (stride < 2) stride = 2;
  int rc = alloc_table(c, stride);
  if (rc) return rc;
  CK(c, hipMemsetAsync(c->d_ids, 0, c->p.n * stride * 4ull, c->stream));
  CK(c, hipMemsetAsync(c->d_deg, 0, c->p.n, c->stream));
  WinSink ws{win, cap, 0};
  OverlayResult res;
  const auto t0 = std::chrono::steady_clock::now();
  rc = overlay_build(c->p.n, c->p.fanout, c->p.fanin, c->p.delay_low, c->p.delay_high, c->st.key,
                     c->d_deg, c->d_ids, stride, max_ticks, c->stream,
                     OverlayWindowSink{&WinSink::push, &ws}, &res);
  c->timing.overlay_ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  if (nwin) *nwin = ws.n;
  if (final_tick) *final_tick = res.final_tick;
  if (rc) return fail(c, rc, res.msg);
  rc = seal_rows(c);
  if (rc) return rc;
  c->peers = true;
  return GS_OK;
}

int gs_set_failed(gs_ctx* c, const uint64_t* words, size_t nwords) {
  if (!c || !words || nwords < c->st.W) return fail(c, GS_EINVAL, "mask needs ceil(n/64) words");
  if (c->begun) return fail(c, GS_EINVAL, "failure mask must be set before gs_broadcast_begin");
  CK(c, hipSetDevice(c->dev));
  std::vector<uint64_t> w(words, words + c->st.W);
  if (c->p.n & 63) w[c->st.W - 1] &= (1ull << (c->p.n & 63)) - 1;
  if (!c->d_failed && hipMalloc(&c->d_failed, c->st.W * 8) != hipSuccess)
    return fail(c, GS_ENOMEM, "cannot allocate the failure mask");
  CK(c, hipMemcpyAsync(c->d_failed, w.data(), c->st.W * 8, hipMemcpyHostToDevice, c->stream));
  CK(c, hipMemcpyAsync(c->st.crash, c->d_failed, c->st.W * 8, hipMemcpyDeviceToDevice, c->stream));
  CK(c, hipStreamSynchronize(c->stream));
  c->failed = true;
  c->st.check_crashed = 1;
  return GS_OK;
}

int gs_broadcast_begin(gs_ctx* c, int64_t sender) {
  if (!c) return GS_EINVAL;
  if (!c->peers) return fail(c, GS_EINVAL, "load peers or build the overlay first");
  if (c->begun) return fail(c, GS_EINVAL, "broadcast already begun");
  uint64_t s = sender < 0 ? uniform(draw0(c->st.key, K_SENDER, 0, 0, 0), (uint32_t)c->p.n)
                          : (uint64_t)sender;
  if (s >= c->p.n) return fail(c, GS_EINVAL, "sender out of range");
  CK(c, hipSetDevice(c->dev));
  if (c->pp) {  // push-pull: the sender is informed (unless failed)
    CK(c, pp_seed(c->st, c->d_next, (uint32_t)s, c->d_flag, c->stream));
    uint32_t ok = 0;
    CK(c, hipMemcpyAsync(&ok, c->d_flag, 4, hipMemcpyDeviceToHost, c->stream));
    CK(c, hipStreamSynchronize(c->stream));
    c->t = 0;
    c->recv = c->pending = ok;
    c->begun = true;
    return GS_OK;
  }
  const bool mine = s >= c->st.lo && s < c->st.hi;  // only the sender's owner schedules it
  if (mine && c->win) CK(c, win_schedule_one(c->ws, (uint32_t)s, 0, c->stream));
  else if (mine) CK(c, launch_schedule_one(c->st, (uint32_t)s, 0, c->stream));
  CK(c, hipStreamSynchronize(c->stream));
  c->t = 0;
  c->pending = mine ? 1 : 0;
  c->begun = true;
  return GS_OK;
}

int gs_set_stream(gs_ctx* c, void* hip_stream) {
  if (!c) return GS_EINVAL;
  CK(c, hipStreamSynchronize(c->stream));
  c->stream = hip_stream ? (hipStream_t)hip_stream : c->own;
  return GS_OK;
}

int gs_frontier_export(gs_ctx* c, uint64_t tick, void* dst, uint64_t word_lo, uint64_t nwords) {
  if (!c || !dst || word_lo + nwords > c->st.W) return fail(c, GS_EINVAL, "bad frontier range");
  if (!nwords) return GS_OK;
  const size_t slot = (size_t)(tick % c->st.R);
  CK(c, hipMemcpyAsync(dst, c->st.ring + slot * c->st.W + word_lo, nwords * 8,
                       hipMemcpyDeviceToDevice, c->stream));
  return GS_OK;
}

int gs_frontier_import(gs_ctx* c, uint64_t tick, const void* src) {
  if (!c || !src) return fail(c, GS_EINVAL, "bad frontier source");
  const size_t slot = (size_t)(tick % c->st.R);
  CK(c, hipMemcpyAsync(c->st.ring + slot * c->st.W, src, c->st.W * 8, hipMemcpyDeviceToDevice,
                       c->stream));
  return GS_OK;
}

// Window engine: ticks [t0, t0 + n) as windows of <= min(max(delaylow,1),16)
// ticks (gs_window.hip).  One host sync per window reads its task count.
static int run_windows(gs_ctx* c, uint64_t t0, uint32_t n, bool timing) {
  WinState& w = c->ws;
  const uint32_t Lmax = std::min<uint32_t>(std::max<int32_t>(c->p.delay_low, 1), kBitTicks);
  uint32_t done = 0, widx = 0;
  std::vector<std::pair<uint32_t, uint32_t>> evs;
  // Receipts per fine bucket are ~density * 16384 whatever N is; a window whose
  // slots would overflow k_resolve's LDS message buffer on average is cut short.
  const uint64_t slot_budget = (uint64_t)w.nfine * kWinSlotsPerBucket;
  while (done < n) {
    const uint32_t Lw = std::min(Lmax, n - done);
    const uint32_t t = (uint32_t)(t0 + done);
    auto units = [&](uint32_t Lu) -> int {
      CK(c, hipMemsetAsync(w.tfires, 0, kMaxWindow * 8, c->stream));
      CK(c, win_units(w, t, Lu, c->stream));
      size_t need = 0;
      CK(c, win_scan_units(w, Lu, nullptr, need, c->stream));
      if (!grow(c->tmp, need)) return fail(c, GS_ENOMEM, "cannot allocate scan scratch");
      need = c->tmp.bytes;
      CK(c, win_scan_units(w, Lu, c->tmp.p, need, c->stream));
      CK(c, hipMemcpyAsync(c->h_misc, w.tfires, kMaxWindow * 8, hipMemcpyDeviceToHost, c->stream));
      CK(c, hipStreamSynchronize(c->stream));
      return GS_OK;
    };
    if (int rc = units(Lw)) return rc;
    // fires per tick -> the window's length under the slot budget
    uint32_t L = 1;
    unsigned long long Tn = c->h_misc[0];  // broadcasts firing in the window
    while (L < Lw && (Tn + c->h_misc[L]) * w.stride <= slot_budget) Tn += c->h_misc[L++];
    // units are bucket-major: a cut window is laid out again for its L ticks
    if (L < Lw)
      if (int rc = units(L)) return rc;
    const unsigned long long T = Tn * w.stride;  // friend slots of the firing nodes
    plan_coarse(c, T, nullptr);
    const uint64_t fcap = T + T / 8 + (uint64_t)w.ncoarse * 256 * 513 + 16;
    if (!grow(c->gmap, ((Tn + 63) / 64 + 1) * 4) || !grow(c->cmsg, (c->h_cap[256] + 16) * 4) ||
        !grow(c->fmsg, fcap * 4))
      return fail(c, GS_ENOMEM, "cannot allocate " + std::to_string(T) + " window messages");
    w.gmap = (uint32_t*)c->gmap.p;
    w.cmsg = (uint32_t*)c->cmsg.p;
    w.fmsg = (uint32_t*)c->fmsg.p;
    if (timing)
      while (c->ev.size() < (size_t)(widx + 1) * 5) {
        hipEvent_t ev;
        CK(c, hipEventCreate(&ev));
        c->ev.push_back(ev);
      }
    hipEvent_t* e = timing ? &c->ev[(size_t)widx * 5] : nullptr;
    if (T) {
      CK(c, hipMemcpyAsync(w.ccap, c->h_cap, 257 * 8, hipMemcpyHostToDevice, c->stream));
      CK(c, win_groupmap(w, L, c->stream));
      if (e) CK(c, hipEventRecord(e[0], c->stream));
      CK(c, win_expand(w, t, L, Tn, 1, c->stream));
      if (e) CK(c, hipEventRecord(e[1], c->stream));
      CK(c, win_plan(w, false, c->stream));
      CK(c, win_part2(w, T, true, c->stream));
      if (e) CK(c, hipEventRecord(e[2], c->stream));
      // regions sized from estimates: check, and redo exactly on overflow
      CK(c, hipMemcpyAsync(c->h_misc, c->d_err, 4, hipMemcpyDeviceToHost, c->stream));
      CK(c, hipStreamSynchronize(c->stream));
      uint32_t err = (uint32_t)c->h_misc[0];
      if (err & kErrCoarse) {
        CK(c, hipMemsetAsync(w.chist, 0, 256 * 8, c->stream));
        CK(c, win_expand(w, t, L, Tn, 0, c->stream));
        CK(c, hipMemcpyAsync(c->h_misc, w.chist, 256 * 8, hipMemcpyDeviceToHost, c->stream));
        CK(c, hipStreamSynchronize(c->stream));
        plan_coarse(c, T, c->h_misc);
        CK(c, hipMemcpyAsync(w.ccap, c->h_cap, 257 * 8, hipMemcpyHostToDevice, c->stream));
        CK(c, hipMemsetAsync(w.cfill, 0, 256 * 8, c->stream));
        CK(c, win_expand(w, t, L, Tn, 2, c->stream));
        CK(c, win_plan(w, false, c->stream));
        err = kErrFine;  // the fine regions must be redone as well
      }
      if (err & kErrFine) {
        CK(c, hipMemsetAsync(w.fhist, 0, ((size_t)w.ncoarse * 256 + 1) * 8, c->stream));
        CK(c, win_plan(w, true, c->stream));
        CK(c, win_part2(w, T, false, c->stream));
        size_t need2 = 0;
        CK(c, win_scan_fine(w, nullptr, need2, c->stream));
        if (!grow(c->tmp, need2)) return fail(c, GS_ENOMEM, "cannot allocate scan scratch");
        need2 = c->tmp.bytes;
        CK(c, win_scan_fine(w, c->tmp.p, need2, c->stream));
        CK(c, hipMemsetAsync(w.ffill, 0, (size_t)w.nfine * 8, c->stream));
        CK(c, win_part2(w, T, true, c->stream));
        ++c->timing.exact_redos;
      }
    } else if (e) {
      CK(c, hipEventRecord(e[0], c->stream));
      CK(c, hipEventRecord(e[1], c->stream));
      CK(c, hipEventRecord(e[2], c->stream));
    }
    // the window's fire lists are consumed: later ticks t + R may reuse the slots
    const uint32_t s0 = t % w.R;
    const uint32_t first = std::min(L, w.R - s0);
    CK(c, hipMemsetAsync(w.fcount + (size_t)s0 * w.nfine, 0, (size_t)first * w.nfine * 4, c->stream));
    if (first < L) CK(c, hipMemsetAsync(w.fcount, 0, (size_t)(L - first) * w.nfine * 4, c->stream));
    if (e) CK(c, hipEventRecord(e[3], c->stream));
    if (T) CK(c, win_resolve(w, t, L, c->stream));
    if (T) CK(c, win_stats_reduce(w, t, L, c->stream));
    if (e) {
      CK(c, hipEventRecord(e[4], c->stream));
      evs.emplace_back(widx * 5, T ? 1u : 0u);
    }
    ++widx;
    done += L;
  }
  if (timing) {
    CK(c, hipStreamSynchronize(c->stream));
    for (auto& pr : evs) {
      hipEvent_t* e = &c->ev[pr.first];
      float ms = 0;
      CK(c, hipEventElapsedTime(&ms, e[0], e[1]));
      c->timing.expand_ms += ms;
      c->timing.deliver_ms += ms;
      CK(c, hipEventElapsedTime(&ms, e[1], e[2]));
      c->timing.part_ms += ms;
      c->timing.deliver_ms += ms;
      CK(c, hipEventElapsedTime(&ms, e[3], e[4]));
      c->timing.resolve_ms += ms;
      c->timing.deliver_launches += pr.second;
      c->timing.resolve_launches += pr.second;
      c->timing.windows += 1;
    }
  }
  uint32_t err = 0;
  CK(c, hipMemcpyAsync(&err, c->d_err, 4, hipMemcpyDeviceToHost, c->stream));
  CK(c, hipStreamSynchronize(c->stream));
  if (err & 4) return fail(c, GS_EOVERFLOW, "too many arrivals at one node in one tick");
  return GS_OK;
}

int gs_step(gs_ctx* c, uint32_t ticks, gs_tick_stats* out) {
  if (!c) return GS_EINVAL;
  if (!c->begun) return fail(c, GS_EINVAL, "gs_broadcast_begin first");
  CK(c, hipSetDevice(c->dev));
  const bool timing = (c->p.flags & GS_FLAG_TIMING) != 0;
  const bool flood = c->st.kc == 0;
  uint32_t done = 0;
  while (done < ticks) {
    const uint32_t batch = std::min<uint32_t>(ticks - done, kStatSlots);
    const uint64_t t0 = c->t + 1;
    // zero this batch's stats entries (ring-indexed)
    const uint32_t i0 = (uint32_t)(t0 % kStatSlots);
    const uint32_t first = std::min<uint32_t>(batch, kStatSlots - i0);
    CK(c, hipMemsetAsync(c->st.stats + (size_t)i0 * kStatFields, 0, (size_t)first * kStatFields * 8,
                         c->stream));
    if (first < batch)
      CK(c, hipMemsetAsync(c->st.stats, 0, (size_t)(batch - first) * kStatFields * 8, c->stream));
    const uint32_t nev = timing && !c->win ? batch * (flood || c->pp ? 2 : 4) : 0;
    while (c->ev.size() < nev) {
      hipEvent_t e;
      CK(c, hipEventCreate(&e));
      c->ev.push_back(e);
    }
    if (c->win) {
      int rc = run_windows(c, t0, batch, timing);
      if (rc) return rc;
    }
    for (uint32_t i = 0; i < batch && c->pp; ++i) {  // push-pull rounds
      const uint32_t tt = (uint32_t)(t0 + i);
      hipEvent_t* e = timing ? &c->ev[(size_t)i * 2] : nullptr;
      if (e) CK(c, hipEventRecord(e[0], c->stream));
      CK(c, pp_round(c->st, c->d_next, c->d_ppsum, tt, c->stream));
      if (e) CK(c, hipEventRecord(e[1], c->stream));
      CK(c, pp_commit(c->st, c->d_next, tt, c->stream));
    }
    for (uint32_t i = 0; i < batch && !c->win && !c->pp; ++i) {
      const uint32_t tt = (uint32_t)(t0 + i);
      hipEvent_t* e = timing ? &c->ev[(size_t)i * (flood ? 2 : 4)] : nullptr;
      if (e) CK(c, hipEventRecord(e[0], c->stream));
      CK(c, launch_tick(c->st, tt, flood ? MODE_FLOOD : MODE_COUNT, c->stream));
      if (e) CK(c, hipEventRecord(e[1], c->stream));
      if (!flood) {
        if (e) CK(c, hipEventRecord(e[2], c->stream));
        CK(c, launch_tick(c->st, tt, MODE_RESOLVE, c->stream));
        if (e) CK(c, hipEventRecord(e[3], c->stream));
      }
      CK(c, launch_slot_reset(c->st, tt % c->st.R, c->stream));
    }
    CK(c, hipMemcpyAsync(c->h_stats + (size_t)i0 * kStatFields, c->st.stats + (size_t)i0 * kStatFields,
                         (size_t)first * kStatFields * 8, hipMemcpyDeviceToHost, c->stream));
    if (first < batch)
      CK(c, hipMemcpyAsync(c->h_stats, c->st.stats, (size_t)(batch - first) * kStatFields * 8,
                           hipMemcpyDeviceToHost, c->stream));
    CK(c, hipStreamSynchronize(c->stream));
    if (timing && !c->win) {
      for (uint32_t i = 0; i < batch; ++i) {
        hipEvent_t* e = &c->ev[(size_t)i * (flood || c->pp ? 2 : 4)];
        float ms = 0;
        CK(c, hipEventElapsedTime(&ms, e[0], e[1]));
        c->timing.deliver_ms += ms;
        c->timing.deliver_launches++;
        if (!flood && !c->pp) {
          CK(c, hipEventElapsedTime(&ms, e[2], e[3]));
          c->timing.resolve_ms += ms;
          c->timing.resolve_launches++;
        }
      }
    }
    for (uint32_t i = 0; i < batch; ++i) {
      const unsigned long long* s = c->h_stats + (size_t)((t0 + i) % kStatSlots) * kStatFields;
      c->t = t0 + i;
      c->fired += s[ST_FIRED];
      c->sent += s[ST_SENT];
      c->msgs += s[ST_MSGS];
      c->recv += s[ST_RECV];
      c->crashed += s[ST_CRASH];
      // push-pull: every informed node keeps calling
      c->pending = c->pp ? c->recv : c->pending + s[ST_SCHED] - s[ST_FIRED];
      if (out) {
        gs_tick_stats& o = out[done + i];
        o.tick = c->t;
        o.fired = s[ST_FIRED];
        o.sent = s[ST_SENT];
        o.messages = s[ST_MSGS];
        o.received = c->recv;
        o.crashed = c->crashed;
        o.pending = c->pending;
      }
    }
    done += batch;
  }
  return GS_OK;
}

int gs_run(gs_ctx* c, uint32_t poll, uint64_t max_ticks, gs_tick_stats* out, size_t cap,
           size_t* nout, int32_t* status) {
  if (!c || poll == 0) return fail(c, GS_EINVAL, "poll must be >= 1");
  size_t k = 0;
  int32_t st = GS_RUN_MAX_TICKS;
  for (;;) {
    const uint64_t f0 = c->fired, s0 = c->sent, m0 = c->msgs, r0 = c->recv;
    int rc = gs_step(c, poll, nullptr);
    if (rc) return rc;
    if (out && k < cap)
      out[k] = gs_tick_stats{c->t, c->fired - f0, c->sent - s0, c->msgs - m0, c->recv, c->crashed,
                             c->pending};
    ++k;
    if (covered(c->recv, c->p.n)) { st = GS_RUN_COVERED; break; }
    // push-pull: informed nodes call forever, so a poll window that informs
    // nobody new (or an empty informed set) ends the run instead
    if (c->pending == 0 || (c->pp && c->recv == r0)) { st = GS_RUN_QUIESCENT; break; }
    if (c->t >= max_ticks) { st = GS_RUN_MAX_TICKS; break; }
  }
  if (nout) *nout = k;
  if (status) *status = st;
  return GS_OK;
}

int gs_totals(gs_ctx* c, gs_tick_stats* out) {
  if (!c || !out) return GS_EINVAL;
  *out = gs_tick_stats{c->t, c->fired, c->sent, c->msgs, c->recv, c->crashed, c->pending};
  return GS_OK;
}

int gs_read_received(gs_ctx* c, uint64_t* words, size_t nwords) {
  if (!c || !words || nwords < c->st.W) return fail(c, GS_EINVAL, "need ceil(n/64) words");
  CK(c, hipSetDevice(c->dev));
  CK(c, hipMemcpyAsync(words, c->st.recv, c->st.W * 8, hipMemcpyDeviceToHost, c->stream));
  CK(c, hipStreamSynchronize(c->stream));
  return GS_OK;
}

int gs_read_crashed(gs_ctx* c, uint64_t* words, size_t nwords) {
  if (!c || !words || nwords < c->st.W) return fail(c, GS_EINVAL, "need ceil(n/64) words");
  CK(c, hipSetDevice(c->dev));
  CK(c, hipMemcpyAsync(words, c->st.crash, c->st.W * 8, hipMemcpyDeviceToHost, c->stream));
  CK(c, hipStreamSynchronize(c->stream));
  return GS_OK;
}

int gs_timing_get(gs_ctx* c, gs_timing* out) {
  if (!c || !out) return GS_EINVAL;
  *out = c->timing;
  return GS_OK;
}

int gs_set_flags(gs_ctx* c, uint32_t flags) {
  if (!c) return GS_EINVAL;
  c->p.flags = flags;
  return GS_OK;
}

int gs_reset(gs_ctx* c) {
  if (!c) return GS_EINVAL;
  CK(c, hipSetDevice(c->dev));
  // everything in the state block except the stats ring and error word
  CK(c, hipMemsetAsync(c->d_state, 0, (char*)c->st.stats - (char*)c->d_state, c->stream));
  if (c->d_cnt) CK(c, hipMemsetAsync(c->d_cnt, 0, c->p.n * 4, c->stream));
  if (c->win) CK(c, hipMemsetAsync(c->ws.fcount, 0, c->fcount_bytes, c->stream));
  if (c->failed)
    CK(c, hipMemcpyAsync(c->st.crash, c->d_failed, c->st.W * 8, hipMemcpyDeviceToDevice, c->stream));
  CK(c, hipStreamSynchronize(c->stream));
  c->t = c->fired = c->sent = c->msgs = c->recv = c->crashed = c->pending = 0;
  c->begun = false;
  return GS_OK;
}

void gs_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  const u32x4 r = philox(ctr[0], ctr[1], ctr[2], ctr[3], key[0], key[1]);
  out[0] = r.x; out[1] = r.y; out[2] = r.z; out[3] = r.w;
}

}  // extern "C"
