// gs_api.cpp -- the C ABI of libgossip_hip.so (include/gossip.h).
//
// Replaces the reference's main() body (simulator.go:207-253): allocation
// (:208-212), overlay (:214-235), broadcast and polling (:237-253).  Four
// kinds of context sit behind the same calls:
//   plain    one device, one stream, one trial (window / tick / push-pull engine)
//   batched  one device, `trials` independent trials laid out at trial << tlog
//            and run by the window engine at once (config C3)
//   shard    one node range [lo, hi) of one broadcast (config C4): a member of a
//            group, or one rank of a multi-process run (RCCL inside)
//   group    gs_create_multi: shards or trial batches over several devices
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "gossip.h"
#include "gs_comm.h"
#include "gs_internal.h"

using namespace gs;

namespace {

struct Buf {
  void* p = nullptr;
  size_t bytes = 0;
};

// One trial's running counters and its stopping snapshot (gs_run's rule).
struct TrialAcc {
  uint64_t fired = 0, sent = 0, msgs = 0, recv = 0, crash = 0, sched = 0, tick99 = 0;
  int32_t status = GS_RUN_RUNNING;
  gs_trial_stats snap{};
};

}  // namespace

struct gs_ctx {
  gs_params p{};
  int dev = 0;
  hipStream_t stream = nullptr;  // where device work is issued (own, or gs_set_stream's)
  hipStream_t own = nullptr;     // the context's own stream
  std::string err;
  DevState st{};
  uint8_t* d_deg = nullptr;
  uint32_t* d_ids = nullptr;
  uint32_t tab_stride = 0;  // row stride d_ids was allocated for
  uint32_t* d_pk = nullptr;  // k_expand's packed view of the sealed rows (expand_view)
  size_t pk_bytes = 0;
  uint64_t pk_ver = ~0ull;   // table_ver the packed view was built from
  uint32_t row_slots = 0;   // longest row when rows are padded past it (0: the stride)
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
  bool pp = false, pp_l2_only = false;
  unsigned long long* d_next = nullptr;  // informed set being built (state block)
  unsigned long long* d_ppsum = nullptr;  // push-pull word summaries (state block)
  uint32_t* d_flag = nullptr;
  // sparse early rounds (PPSparse): reverse table, informed list, failed-slot
  // mask, round control; rebuilt when the table (table_ver) or the failure
  // mask (fail_ver) changes
  Buf pp_rend, pp_rsrc, pp_rslot, pp_ilist, pp_fmask, pp_scan, pp_ctlb;
  Buf pp_rfail;  // push-pull: failed-caller bit per in-edge (with pp_fmask)
  Buf pp_dset, pp_dcnt;  // deferred sets of the pull-answer rounds (PPSparse::dset)
  Buf pp_rend16;         // the compact view of pp_rend: rend16 [n] u16, then rbase [n/64 + 1] u64, then a flag
  bool rend16_ok = false;  // the view fits (no 64-node block with more than 65,535 in-edges)
  uint64_t table_ver = 0, fail_ver = 0, rev_ver = ~0ull, fm_tver = ~0ull, fm_fver = ~0ull;
  // push-pull: live callers and live empty rows of (cl_tver, cl_fver) (pp_seed_ctx)
  uint64_t cl_tver = ~0ull, cl_fver = ~0ull;
  unsigned long long cl_counts[2] = {0, 0};
  PPSparse sp{};
  // window engine (gs_window.hip)
  bool win = false;
  WinState ws{};
  void* d_win = nullptr;      // fcount + small per-window buffers
  void* d_flist = nullptr;    // [R][nfine][16384] u16
  void* d_rlmsg = nullptr;    // [nfine][kRolledCap] k_resolve's rolled receipts
  size_t fcount_bytes = 0;
  Buf gmap, cmsg, fmsg, tmp;
  unsigned long long* h_cap = nullptr;  // pinned [257] coarse region plan
  unsigned long long* h_misc = nullptr; // pinned scratch (counts, flags): misc_words words
  size_t misc_words = 0;                // >= kRegions and >= G * kMaxWindow (gathered fire counts)
  uint32_t* h_err = nullptr;            // pinned copy of the error word (shard windows)
  // device-driven windows (run_async)
  WinCtl* d_ctl = nullptr;
  unsigned long long* d_stage = nullptr;  // [kSlots][kStageWords]
  unsigned long long* h_stage = nullptr;  // pinned, mapped: d_stage is its device address
  std::vector<hipEvent_t> wev;            // one per staging slot
  bool async_off = false;                 // GS_SYNC_WINDOWS=1: host-driven windows only (A/B tests)
  bool winlog = false;                    // GS_WINLOG=1: one stderr line per device-driven window
  // trials: `trials` per context (batched when > 1), ids trial << tlog | node
  uint32_t trials = 1, tlog = 32;
  uint64_t ntot = 0;                    // nodes in this context's id space
  uint32_t* d_tstat = nullptr;          // [trials][kMaxWindow][kTStatFields]
  uint32_t* h_tstat = nullptr;          // pinned copy
  std::vector<TrialAcc> tacc;
  // node-range shard (config C4)
  bool shard = false;
  uint32_t G = 1, rank = 0;
  uint64_t lo = 0, hi = 0, seg_per = 0;
  // owner expand: the receive layout of a window ([4][kRegions + 1]: region
  // starts, ends, fills; the pack offsets of this shard's own send blocks),
  // pinned host copy, and the receive-side WinState (kept for an exact redo)
  unsigned long long* d_rtab = nullptr;
  unsigned long long* h_rtab = nullptr;
  WinState wr{};
  uint64_t rtotal = 0;                  // messages received in the window
  Buf xsend, xrecv;                     // multi-process: packed send blocks, received blocks
  unsigned long long* d_gcounts = nullptr;  // multi-process: [G][16] gathered fires per tick
  unsigned long long* d_glay = nullptr;     // multi-process: [G][kRegions + 1] gathered region fills + error word
  unsigned long long* h_glay = nullptr;     // pinned copy
  ncclComm_t comm = nullptr;
  // multi-process exchange done by the caller (gs_create_rank_exchange)
  gs_exchange hx{};
  bool has_hx = false;
  char* h_xbuf = nullptr;               // pinned staging of the host exchanges
  size_t h_xbytes = 0;
  // push-pull node-range shard: the informed / failed sets by global id
  // (G * segw words; shared by the members on one device, owned by a rank);
  // st.recv / st.crash are this shard's slice of them
  bool pp_shard = false, own_ig = false;
  bool aborted = false;                 // a rank whose exchange failed (RCCL communicator aborted)
  unsigned long long* d_ig = nullptr;
  unsigned long long* d_fg = nullptr;
  // pull-answer rounds of push-pull shards: the round's informed set being
  // built, by global id (shared like d_ig); a rank's staging for the bits the
  // other ranks set in its range ([G][segw] words)
  unsigned long long* d_gn = nullptr;
  unsigned long long* d_gst = nullptr;
  bool pp_answer = false;               // the current broadcast's sharded rounds still run pull-answer
  bool pp_gn_ok = false;                // d_gn holds the replicated set (set at the first sharded round)
  uint64_t segw = 0;
  // push-pull shards: the replica -- an unsharded push-pull context over the
  // full table on this device (shared by the device's members; owned by the
  // group, or by the rank) whose informed / failed sets ARE the replicated
  // ones: it runs the sparse early rounds, identically on every device and
  // rank, with no exchange (section 6.3 of DESIGN.md)
  gs_ctx* rep = nullptr;
  bool own_rep = false;
  bool rep_live = false;                // the current broadcast's rounds still run on the replicas
  uint32_t rep_rounds = 0;              // rounds run on the replicas since the broadcast began
  // group (gs_create_multi)
  bool group = false, gtrials = false;
  std::vector<gs_ctx*> mem;
  std::vector<int> gdevs;               // distinct devices, first-use order
  std::vector<int> gdev_of;             // member -> index into gdevs
  std::vector<Buf> gbuf;                // per distinct device: its members' send blocks, then blocks from other devices
  std::vector<hipEvent_t> gev_c, gev_x; // per member: its part of an exchange done; per device: copies done
  std::vector<unsigned long long*> gig, gfg, ggn;  // push-pull shards: per distinct device, the replicated sets
  std::vector<gs_ctx*> greps;           // push-pull shards: per distinct device, the replica
  OverlayWork ovw;                      // overlay builder buffers, kept between builds
  // device-driven shard windows (dd_run; the group's or the rank's): gathered
  // fire counts [G][kMaxWindow] and region rows [G][kDDRow], each member's
  // window counters [M][kDDWStat] and control block, the pointer tables the
  // kernels read (region starts [M], sources [M + 1], counters [M], control
  // blocks [M]); pinned copy of the gathered rows for ranks whose blocks travel
  void* dd_mem = nullptr;
  unsigned long long* dd_gcnt = nullptr;
  unsigned long long* dd_glay = nullptr;
  unsigned long long* dd_wstat = nullptr;
  WinCtl* dd_ctl = nullptr;
  void** dd_ptrs = nullptr;
  void** h_ddptrs = nullptr;            // pinned staging of dd_ptrs
  WinState* dd_wsm = nullptr;           // in-process group: the members' window states [3][M] (WinGroup)
  unsigned long long* h_ddlay = nullptr;
};

namespace {

int fail(gs_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

// gs_timing's device-memory fields: the library's process-wide figures
void fill_devmem(gs_timing* out) {
  DevMemStats d;
  gs_devmem_stats(&d);
  out->alloc_ms = d.alloc_ms;
  out->largest_alloc_ms = d.largest_alloc_ms;
  out->free_ms = d.free_ms;
  out->alloc_calls = d.hip_allocs;
  out->alloc_cache_hits = d.cache_hits;
  out->cached_bytes = d.cached_bytes;
}

bool grow(Buf& b, size_t bytes) {
  if (b.bytes >= bytes) return true;
  const size_t nb = std::max(bytes, b.bytes + b.bytes / 4);
  if (b.p) (void)dev_free(b.p);
  b.p = nullptr;
  b.bytes = 0;
  if (dev_malloc(&b.p, nb) != hipSuccess) return false;
  b.bytes = nb;
  return true;
}

#define CK(c, expr)                                                                   \
  do {                                                                                \
    hipError_t e_ = (expr);                                                           \
    if (e_ != hipSuccess)                                                             \
      return fail((c), GS_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

#define NCK(c, expr)                                                                  \
  do {                                                                                \
    ncclResult_t r_ = (expr);                                                         \
    if (r_ != ncclSuccess)                                                            \
      return fail((c), GS_EDEVICE, std::string(#expr) + ": " + rccl_error((int)r_));  \
  } while (0)

#define RC(expr)              \
  do {                        \
    int rc_ = (expr);         \
    if (rc_) return rc_;      \
  } while (0)


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
  w.base = (uint32_t)c->lo;
  w.tlog = c->tlog;
  w.tmask = c->tlog >= 32 ? ~0u : (1u << c->tlog) - 1;
  // a batched context's fine buckets are whole-trial runs of 2^(tlog-14) with
  // the last ones of each trial partly or wholly past its n nodes
  w.tnodes = c->trials > 1 && c->tlog <= kCoarseShift && !c->shard ? (uint32_t)c->p.n : 0u;
  w.G = c->G;
  w.rank = c->rank;
  w.seg_per = (uint32_t)c->seg_per;
  w.csub = kCoarseSub;
  w.noxcd = getenv("GS_PART2_NOXCD") ? 1u : 0u;  // A/B knob: k_part2 tiles in region order
  {
    const char* xp = getenv("GS_XPAIR");  // A/B knob: 0 = k_expand's packed rows fetched per lane
    w.nopair = xp && atoi(xp) == 0 ? 1u : 0u;
  }
  w.ccap_end = nullptr;
  w.csrc = nullptr;
  if (c->shard) {  // owner expand (k_expand's coarse_bin)
    w.owner = 1;
    w.obins = 256 / c->G;
    w.oseg_q = (uint32_t)(c->seg_per >> kFineLog);
    w.oseg_magic = 0xFFFFFFFFu / w.oseg_q;
    if (dev_malloc(&c->d_rtab, kRtabWords * 8) != hipSuccess ||
        hipHostMalloc((void**)&c->h_rtab, kRtabWords * 8) != hipSuccess)
      return fail(c, GS_ENOMEM, "cannot allocate the shard's receive layout");
  }
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t units = (size_t)kMaxWindow * w.nfine + 1;
  const size_t b_fc = al((size_t)w.R * w.nfine * 4), b_units = al(units * 8),
               b_small = al(kRegions * 8) * 2 + al((kRegions + 1) * 8) + al((kRegions + 1) * 4) + al(kMaxWindow * 8),
               b_fhist = al(((size_t)w.ncoarse * 256 + 1) * 8), b_fbase = al(((size_t)w.nfine + 1) * 8),
               b_ffill = al((size_t)w.nfine * 8),
               b_sst = al((size_t)kStatShards * kMaxWindow * kStatFields * 8),
               b_rlcnt = al((size_t)w.nfine * 4),
               b_tsum = al((size_t)w.ncoarse * kMaxWindow * 8) + al(((size_t)w.ncoarse + 1) * 8);
  const size_t total = b_fc + 2 * b_units + b_small + b_fhist + b_fbase + b_ffill + b_sst + b_rlcnt + b_tsum;
  if (dev_malloc(&c->d_win, total) != hipSuccess)
    return fail(c, GS_ENOMEM, "cannot allocate window-engine buffers");
  const size_t flist = (size_t)w.R * w.nfine * kFineNodes * 2;
  if (dev_malloc(&c->d_flist, flist) != hipSuccess)
    return fail(c, GS_ENOMEM, "cannot allocate " + std::to_string(flist >> 20) + " MiB of fire lists");
  char* q = (char*)c->d_win;
  w.fcount = (uint32_t*)q; q += b_fc;
  w.usize = (unsigned long long*)q; q += b_units;
  w.unit_off = (unsigned long long*)q; q += b_units;
  w.chist = (unsigned long long*)q; q += al(kRegions * 8);
  w.cfill = (unsigned long long*)q; q += al(kRegions * 8);
  w.ccap = (unsigned long long*)q; q += al((kRegions + 1) * 8);
  w.tprefix = (uint32_t*)q; q += al((kRegions + 1) * 4);
  w.tfires = (unsigned long long*)q;
  q = (char*)c->d_win + b_fc + 2 * b_units + b_small;
  w.fhist = (unsigned long long*)q; q += b_fhist;
  w.fstart = (unsigned long long*)q; q += b_fbase;
  w.ffill = (unsigned long long*)q; q += b_ffill;
  w.sstats = (unsigned long long*)q; q += b_sst;
  w.rlcnt = (uint32_t*)q; q += b_rlcnt;
  w.tsum = (unsigned long long*)q; q += al((size_t)w.ncoarse * kMaxWindow * 8);
  w.toff = (unsigned long long*)q; q += al(((size_t)w.ncoarse + 1) * 8);
  if (dev_malloc(&c->d_rlmsg, (size_t)w.nfine * kRolledCap * 4) != hipSuccess)
    return fail(c, GS_ENOMEM, "cannot allocate the rolled-receipt lists");
  w.rlmsg = (uint32_t*)c->d_rlmsg;
  w.dbg = nullptr;
  if (getenv("GS_STAMPS") && dev_malloc(&w.dbg, kDbgWords * 8) == hipSuccess)
    (void)hipMemset(w.dbg, 0, kDbgWords * 8);
  w.flist = (uint16_t*)c->d_flist;
  c->fcount_bytes = (size_t)w.R * w.nfine * 4;
  if (hipMemsetAsync(c->d_win, 0, total, c->stream) != hipSuccess)
    return fail(c, GS_EDEVICE, "memset of window buffers failed");
  c->misc_words = std::max<size_t>(4096, (size_t)c->G * kMaxWindow + 64);
  if (hipHostMalloc((void**)&c->h_cap, (kRegions + 1) * 8) != hipSuccess ||
      hipHostMalloc((void**)&c->h_misc, c->misc_words * 8) != hipSuccess ||
      hipHostMalloc((void**)&c->h_err, 64) != hipSuccess)
    return fail(c, GS_ENOMEM, "cannot allocate pinned window buffers");
  if (c->trials > 1) {
    const size_t tb = (size_t)c->trials * kMaxWindow * kTStatFields * 4;
    if (dev_malloc((void**)&c->d_tstat, tb) != hipSuccess ||
        hipHostMalloc((void**)&c->h_tstat, tb) != hipSuccess)
      return fail(c, GS_ENOMEM, "cannot allocate per-trial counters");
    w.tstat = c->d_tstat;
  }
  return GS_OK;
}

// Coarse region plan: each of bin b's 8 sub-regions gets 1/8 of the bin's
// node share of the window's T message bound plus 512, or exactly
// `exact[region]` (region = bin * 8 + sub).
void plan_coarse(gs_ctx* c, uint64_t T, const unsigned long long* exact) {
  const WinState& w = c->ws;
  unsigned long long a = 0;
  for (uint32_t b = 0; b < 256; ++b) {
    const uint64_t lo = (uint64_t)b << kCoarseShift;
    const uint64_t hi = std::min<uint64_t>(w.n, lo + (1ull << kCoarseShift));
    const double xr = (double)kXRoundNodes * w.stride;  // one expand round's slots (gs_internal.h)
    const unsigned long long sub =
        b < w.ncoarse ? (unsigned long long)(((double)T / kCoarseSub + xr) * (double)(hi - lo) / (double)w.n) + 512
                      : 0ull;
    for (uint32_t x = 0; x < kCoarseSub; ++x) {
      const uint32_t r = b * kCoarseSub + x;
      c->h_cap[r] = a;
      if (b >= w.ncoarse) continue;
      a += exact ? exact[r] : sub;
    }
  }
  c->h_cap[kRegions] = a;
}

// Batched trials (trials > 1, tlog <= kCoarseShift): a message never leaves
// its sender's trial, so it lands in the sender's coarse bin, and the
// sub-region it goes to is the XCD whose rounds expanded the sender
// (xcd_rounds in gs_window.hip).  fb[b] = the first firing index of bin b
// (bins are contiguous in the bucket-major unit order), fb[ncoarse] = Tn.
// Region (b, x) gets an exact upper bound -- the window's firing nodes of bin
// b in XCD x's rounds, times the row length -- so it never overflows: the
// node-share estimate of plan_coarse assumed targets spread over every bin
// and overflowed almost every window of a C3 batch (each then expanded three
// times: estimate, count, redo).
void plan_coarse_trials(gs_ctx* c, const unsigned long long* fb, unsigned long long Tn) {
  const WinState& w = c->ws;
  uint32_t per_round = 0;
  const uint32_t blocks = win_expand_geometry(w, Tn, &per_round, nullptr, nullptr);
  const unsigned long long rounds = (Tn + per_round - 1) / per_round;
  const bool by_xcd = blocks && (blocks & 7) == 0;
  const unsigned long long per = (rounds + 7) >> 3;
  std::vector<unsigned long long> cap(kRegions, 0);
  for (uint32_t b = 0; b < w.ncoarse; ++b) {
    const unsigned long long lo = fb[b], hi = fb[b + 1];
    for (unsigned long long r = lo / per_round; lo < hi && r * per_round < hi; ++r) {
      const unsigned long long a = std::max(lo, r * per_round), e = std::min(hi, (r + 1) * per_round);
      const uint32_t x = by_xcd ? (uint32_t)std::min<unsigned long long>(r / per, 7) : (uint32_t)((r % blocks) & 7);
      cap[b * kCoarseSub + x] += (e - a) * w.slots;
    }
  }
  unsigned long long a = 0;
  for (uint32_t r = 0; r < kRegions; ++r) {
    c->h_cap[r] = a;
    a += cap[r] ? cap[r] + 16 : 0;
  }
  c->h_cap[kRegions] = a;
}

void refresh_window(gs_ctx* c) {
  WinState& w = c->ws;
  w.deg = c->st.deg;
  w.ids = c->st.ids;
  w.recv = c->st.recv;
  w.crash = c->st.crash;
  w.rollw = c->st.rollw;
  w.stats = c->st.stats;
  w.err = c->d_err;
  w.stride = c->st.stride;
  w.slots = c->row_slots && c->row_slots < c->st.stride ? c->row_slots : c->st.stride;
  w.stride_magic = c->st.stride_magic;
  w.abort_on_err = c->shard ? 1u : 0u;
}

uint32_t ring_slots(const gs_params& p) { return p.delay_high > 2 ? (uint32_t)p.delay_high : 2u; }

uint32_t ceil_log2(uint64_t x) {
  uint32_t b = 0;
  while ((1ull << b) < x) ++b;
  return b;
}

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
  if (p->trials > 1 && p->model != GS_MODEL_FLOOD) {
    why = "batched trials run the flood model (the reference's)";
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

// Nodes of the table this context loads: a shard loads the whole (replicated)
// table and keeps its partition.
uint64_t table_n(const gs_ctx* c) { return c->shard ? c->p.n : c->ntot; }

int alloc_table(gs_ctx* c, uint32_t stride) {
  const uint64_t n = table_n(c);
  if (!(c->d_deg && c->d_ids && c->tab_stride == stride)) {  // same shape: reuse (batch after batch)
    if (c->d_deg) (void)dev_free(c->d_deg);
    if (c->d_ids) (void)dev_free(c->d_ids);
    c->d_deg = nullptr;
    c->d_ids = nullptr;
    c->tab_stride = 0;
    if (dev_malloc(&c->d_deg, n) != hipSuccess || dev_malloc(&c->d_ids, n * stride * 4ull) != hipSuccess)
      return fail(c, GS_ENOMEM, "cannot allocate the peer table on the device");
    c->tab_stride = stride;
  }
  RC(set_stride(c, stride));
  refresh_state(c);
  return GS_OK;
}

__global__ void k_validate_peers(const uint8_t* deg, const uint32_t* ids, uint64_t n, uint64_t bound,
                                 uint32_t stride, uint32_t* err) {
  for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < n;
       v += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t d = deg[v];
    if (d > stride) { atomicOr(err, 1u); continue; }
    for (uint32_t j = 0; j < d; ++j)
      if (ids[v * stride + j] >= bound) atomicOr(err, 2u);
  }
}

int validate_table(gs_ctx* c, const uint8_t* deg, const uint32_t* ids, uint64_t n, uint64_t bound) {
  CK(c, hipMemsetAsync(c->d_err, 0, 4, c->stream));
  const uint64_t blocks = std::min<uint64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_validate_peers, dim3((uint32_t)blocks), dim3(256), 0, c->stream, deg, ids, n, bound,
                     c->st.stride, c->d_err);
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
int seal_rows(gs_ctx* c, const uint8_t* deg, uint32_t* ids, uint64_t n) {
  ++c->table_ver;  // every table change ends here
  if (!c->win) return GS_OK;
  CK(c, win_seal_rows(deg, ids, n, c->st.stride, c->stream));
  CK(c, hipStreamSynchronize(c->stream));
  return GS_OK;
}

// k_expand's packed view of the sealed rows (stride 8, rows <= 6 slots: C5's
// fanin 6): five 24-B rows per 128-B line instead of four 32-B ones, built
// once per table version (k_pack_rows, outside any timed step), about 0.8 of
// the table's bytes beside it.  Other shapes -- and GS_NO_PACK=1, an A/B
// knob -- read the table itself.  Called before every window run.
int expand_view(gs_ctx* c) {
  static const bool off = getenv("GS_NO_PACK") != nullptr;
  if (!c->win || c->pp || off || c->st.stride != 8 || c->ws.slots > 6 || !c->d_ids) {
    c->ws.pk = nullptr;
    return GS_OK;
  }
  if (c->pk_ver != c->table_ver || !c->d_pk) {
    const uint64_t rows = c->ntot, bytes = (rows + 4) / 5 * 128;
    if (c->pk_bytes < bytes) {
      if (c->d_pk) (void)dev_free(c->d_pk);
      c->d_pk = nullptr;
      c->pk_bytes = 0;
      if (dev_malloc(&c->d_pk, bytes) != hipSuccess) {  // no room: expand reads the table itself
        (void)hipGetLastError();
        c->d_pk = nullptr;
        c->ws.pk = nullptr;
        return GS_OK;
      }
      c->pk_bytes = bytes;
    }
    CK(c, win_pack_rows(c->d_ids, rows, c->d_pk, c->stream));
    c->pk_ver = c->table_ver;
  }
  c->ws.pk = c->d_pk;
  return GS_OK;
}

// Shard c keeps the sealed rows of its own nodes [lo, hi) (copied from the
// full table `deg` / `ids` of stride S on c's device): owner expand reads
// only the rows of its own firing nodes.
int own_rows(gs_ctx* c, const uint8_t* deg, const uint32_t* ids, uint32_t S, uint32_t row_slots, hipStream_t st) {
  const uint64_t n = c->ntot;
  if (c->d_deg) (void)dev_free(c->d_deg);
  if (c->d_ids) (void)dev_free(c->d_ids);
  c->d_deg = nullptr;
  c->d_ids = nullptr;
  c->tab_stride = 0;  // not the full-table shape: the next load reallocates
  if (dev_malloc(&c->d_deg, n) != hipSuccess || dev_malloc(&c->d_ids, n * S * 4ull) != hipSuccess)
    return fail(c, GS_ENOMEM, "cannot allocate the shard's rows");
  RC(set_stride(c, S));
  c->row_slots = row_slots;
  refresh_state(c);
  CK(c, hipMemcpyAsync(c->d_deg, deg + c->lo, n, hipMemcpyDeviceToDevice, st));
  CK(c, hipMemcpyAsync(c->d_ids, ids + c->lo * S, n * S * 4ull, hipMemcpyDeviceToDevice, st));
  CK(c, hipStreamSynchronize(st));
  ++c->table_ver;
  return GS_OK;
}

bool covered(uint64_t recv, uint64_t n) {
  // simulator.go:246-248, in float32
  volatile float a = (float)recv, b = (float)n;
  volatile float pct = a / b;
  return pct >= 0.99f;
}

int ctx_setup(gs_ctx* c, const gs_params* params, int device, bool shard, uint32_t G, uint32_t rank,
              std::string& why) {
  c->p = *params;
  c->p.device = device;
  c->dev = device;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    why = "no HIP device visible (libgossip_hip needs an MI355X)";
    return GS_EDEVICE;
  }
  if (c->dev < 0 || c->dev >= ndev) {
    why = "device " + std::to_string(c->dev) + " out of range (" + std::to_string(ndev) + " visible)";
    return GS_EDEVICE;
  }
  hipDeviceProp_t prop;
  if (hipSetDevice(c->dev) != hipSuccess || hipGetDeviceProperties(&prop, c->dev) != hipSuccess ||
      strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    why = "device " + std::to_string(c->dev) + " is not gfx950";
    return GS_EDEVICE;
  }
  if (hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
    why = "cannot create a stream";
    return GS_EDEVICE;
  }
  c->stream = c->own;
  DevState& s = c->st;
  const uint32_t stride0 = (uint32_t)std::max(c->p.fanout, c->p.fanin);
  c->pp = c->p.model == GS_MODEL_PUSHPULL;
  c->pp_l2_only = (c->p.flags & GS_FLAG_PP_L2_ONLY) != 0;
  c->trials = std::max<uint32_t>(1, c->p.trials);
  c->ntot = c->p.n;
  if (c->trials > 1) {
    c->tlog = std::max<uint32_t>(kFineLog, ceil_log2(c->p.n));
    c->ntot = (uint64_t)c->trials << c->tlog;
    if (c->ntot > 0x7FFFFFFFull) {
      why = "trials x 2^ceil(log2 n) must be < 2^31 (batch fewer trials per context)";
      return GS_EINVAL;
    }
  }
  c->shard = shard;
  c->G = G;
  c->rank = rank;
  if (shard) {
    if (c->pp && !pp_rslot_packed(stride0)) {
      why = "push-pull node-range shards need rows of at most 16 slots (bottom-up rounds)";
      return GS_EINVAL;
    }
    c->seg_per = (((c->p.n + G - 1) / G) + kFineNodes - 1) & ~(uint64_t)(kFineNodes - 1);
    if ((uint64_t)(G - 1) * c->seg_per >= c->p.n) {
      why = "n = " + std::to_string(c->p.n) + " is too small for " + std::to_string(G) +
            " shards of whole 16384-node buckets";
      return GS_EINVAL;
    }
    c->pp_shard = c->pp;
    c->segw = c->seg_per / 64;
    c->lo = rank * c->seg_per;
    c->hi = std::min<uint64_t>(c->lo + c->seg_per, c->p.n);
    c->ntot = c->hi - c->lo;
  }
  s.lo = 0;
  s.hi = (uint32_t)c->ntot;
  s.n = c->ntot;
  s.W = (s.n + 63) / 64;
  s.C = (uint32_t)((s.n + (1ull << kChunkNodesLog) - 1) >> kChunkNodesLog);
  s.CS = (s.C + kShards - 1) / kShards;
  s.chunk_lo = 0;
  s.chunk_hi = s.C;
  s.sharded = 0;
  s.R = ring_slots(c->p);
  s.delay_low = c->p.delay_low;
  s.delay_span = (uint32_t)(c->p.delay_high - c->p.delay_low);
  s.kd = gs_threshold(c->p.drop_rate);
  s.kc = gs_threshold(c->p.crash_rate);
  s.key = Key{(uint32_t)c->p.seed, (uint32_t)(c->p.seed >> 32), c->p.trial};
  // Engine: the window engine unless the ring is too long for LDS, rows are
  // wider than 32 or the tick engine is forced; push-pull has its own kernels.
  // (its coarse partition has 256 bins of 2^22 nodes: at most 2^30 nodes per context)
  c->win = !c->pp && s.R <= kWinMaxRing && !(c->p.flags & GS_FLAG_TICK_ENGINE) && stride0 <= kWinMaxStride &&
           s.n <= (1ull << (kCoarseShift + 8));
  if ((c->trials > 1 || (shard && !c->pp)) && !c->win) {
    why = "batched trials and node-range shards run on the window engine (delayhigh <= 256, "
          "fanout/fanin <= 32, no GS_FLAG_TICK_ENGINE, at most 2^30 nodes per context or shard)";
    return GS_EINVAL;
  }
  // owner expand: every shard's range fits its 256 / G coarse bins of 2^22 nodes
  // and a group's received blocks take source index G of the receive layout's
  // 8-bit source field (kSrcShift): G <= 255
  static_assert(kSrcShift + 8 == 64, "8-bit source index in the receive layout");
  if (shard && !c->pp && (G > 255 || ((c->seg_per + (1ull << kCoarseShift) - 1) >> kCoarseShift) > 256 / G)) {
    why = "flood node-range shards: each of the G <= 255 shards' ranges must fit 256 / G bins of 2^22 nodes "
          "(n up to about 2^30)";
    return GS_EINVAL;
  }
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
  const size_t b_roll = c->win ? b_bits : 0;
  const size_t total = 2 * b_bits + b_roll + b_next + b_ring + b_cflag + b_clist + b_ccount + b_stats + 256;
  c->state_bytes = total;
  if (dev_malloc(&c->d_state, total) != hipSuccess) {
    why = "cannot allocate " + std::to_string(total) + " bytes of device state";
    return GS_ENOMEM;
  }
  char* q = (char*)c->d_state;
  s.recv = (unsigned long long*)q; q += b_bits;
  s.crash = (unsigned long long*)q; q += b_bits;
  s.rollw = b_roll ? (uint32_t*)q : nullptr; q += b_roll;
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
  s.err = c->d_err;
  s.grecv = s.recv;  // a push-pull shard points these at the replicated sets (attach_pp_sets)
  s.gcrash = s.crash;
  s.gbase = 0;
  if (tick && s.kc > 0 && dev_malloc(&c->d_cnt, s.n * 4) != hipSuccess) {
    why = "cannot allocate arrival counters";
    return GS_ENOMEM;
  }
  s.cnt = c->d_cnt;
  if (c->win) {
    int rc = alloc_window(c);
    if (rc) { why = c->err; return rc; }
  }
  c->tacc.assign(c->trials, TrialAcc{});
  c->async_off = getenv("GS_SYNC_WINDOWS") != nullptr;
  c->winlog = getenv("GS_WINLOG") != nullptr;
  if (hipMemsetAsync(c->d_state, 0, total, c->stream) != hipSuccess ||
      (c->d_cnt && hipMemsetAsync(c->d_cnt, 0, s.n * 4, c->stream) != hipSuccess) ||
      hipHostMalloc((void**)&c->h_stats, (size_t)kStatSlots * kStatFields * 8) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess) {
    why = "device initialisation failed";
    return GS_EDEVICE;
  }
  return GS_OK;
}

void destroy_one(gs_ctx* c) {
  if (!c) return;
  for (gs_ctx* m : c->mem) destroy_one(m);
  if (c->group) {
    for (size_t i = 0; i < c->gdevs.size() && i < c->gbuf.size(); ++i)
      if (c->gbuf[i].p) {
        (void)hipSetDevice(c->gdevs[i]);
        (void)dev_free(c->gbuf[i].p);
      }
    for (size_t i = 0; i < c->gdevs.size(); ++i) {
      (void)hipSetDevice(c->gdevs[i]);
      if (i < c->gig.size() && c->gig[i]) (void)dev_free(c->gig[i]);
      if (i < c->gfg.size() && c->gfg[i]) (void)dev_free(c->gfg[i]);
      if (i < c->ggn.size() && c->ggn[i]) (void)dev_free(c->ggn[i]);
    }
    for (hipEvent_t e : c->gev_c) (void)hipEventDestroy(e);
    for (hipEvent_t e : c->gev_x) (void)hipEventDestroy(e);
    for (gs_ctx* r : c->greps) destroy_one(r);
    if (!c->gdevs.empty()) (void)hipSetDevice(c->gdevs[0]);
    if (c->dd_mem) (void)dev_free(c->dd_mem);
    for (void* ptr : {(void*)c->h_stage, (void*)c->h_ddlay, (void*)c->h_ddptrs})
      if (ptr) (void)hipHostFree(ptr);
    for (hipEvent_t e : c->wev) (void)hipEventDestroy(e);
    delete c;
    return;
  }
  if (c->own_rep) destroy_one(c->rep);
  (void)hipSetDevice(c->dev);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->comm && rccl().ok) (void)rccl().comm_destroy(c->comm);
  if (c->ws.dbg) {
    unsigned long long h[kDbgWords];
    if (hipMemcpy(h, c->ws.dbg, sizeof h, hipMemcpyDeviceToHost) == hipSuccess && h[kXStamp0]) {
      const double r = 1e-3 / h[kXStamp0];  // k_expand phases (GS_XSTAMPS builds)
      fprintf(stderr, "[stamps] k_expand: %llu rounds (wave 0), mean kcycles per round: lookup %.2f rows %.2f "
              "draws %.2f scan+scatter %.2f barrier %.2f writeout %.2f\n", h[kXStamp0], h[kXStamp0 + 1] * r,
              h[kXStamp0 + 2] * r, h[kXStamp0 + 3] * r, h[kXStamp0 + 4] * r, h[kXStamp0 + 5] * r, h[kXStamp0 + 6] * r);
    }
    if (hipMemcpy(h, c->ws.dbg, sizeof h, hipMemcpyDeviceToHost) == hipSuccess)
      for (int cls = 0; cls < 2; ++cls) {  // k_resolve phases (GS_STAMPS=1), thread 0 of every workgroup
        const unsigned long long* d = h + cls * kStampPhases;
        if (!d[0]) continue;
        fprintf(stderr, "[stamps] k_resolve %s: %llu buckets, mean kcycles per bucket per phase:",
                cls ? "M>=1024" : "M<1024", d[0]);
        for (uint32_t i = 1; i < kStampPhases; ++i) fprintf(stderr, " %.2f", d[i] * 1e-3 / d[0]);
        fprintf(stderr, "\n");
      }
    (void)dev_free(c->ws.dbg);
  }
  for (hipEvent_t e : c->ev) (void)hipEventDestroy(e);
  overlay_free(&c->ovw, c->stream);
  if (c->own_ig) {
    if (c->d_ig) (void)dev_free(c->d_ig);
    if (c->d_fg) (void)dev_free(c->d_fg);
    if (c->d_gn) (void)dev_free(c->d_gn);
    if (c->d_gst) (void)dev_free(c->d_gst);
  }
  if (c->h_xbuf) (void)hipHostFree(c->h_xbuf);
  if (c->d_pk) (void)dev_free(c->d_pk);
  for (void* ptr : {(void*)c->d_deg, (void*)c->d_ids, c->d_state, (void*)c->d_cnt, (void*)c->d_failed, c->d_win,
                    c->d_flist, c->d_rlmsg, (void*)c->d_tstat, (void*)c->d_rtab, (void*)c->d_gcounts,
                    (void*)c->d_glay})
    if (ptr) (void)dev_free(ptr);
  for (Buf* b : {&c->gmap, &c->cmsg, &c->fmsg, &c->tmp, &c->xsend, &c->xrecv, &c->pp_rend, &c->pp_rsrc,
                 &c->pp_rslot, &c->pp_ilist, &c->pp_fmask, &c->pp_scan, &c->pp_ctlb, &c->pp_dset, &c->pp_dcnt, &c->pp_rfail,
                 &c->pp_rend16})
    if (b->p) (void)dev_free(b->p);
  for (void* ptr : {(void*)c->h_cap, (void*)c->h_misc, (void*)c->h_err, (void*)c->h_stats, (void*)c->h_tstat,
                    (void*)c->h_stage, (void*)c->h_rtab, (void*)c->h_glay})
    if (ptr) (void)hipHostFree(ptr);
  if (c->d_ctl) (void)dev_free(c->d_ctl);  // (d_stage maps h_stage)
  if (c->dd_mem) (void)dev_free(c->dd_mem);
  for (void* ptr : {(void*)c->h_ddlay, (void*)c->h_ddptrs})
    if (ptr) (void)hipHostFree(ptr);
  for (hipEvent_t e : c->wev) (void)hipEventDestroy(e);
  if (c->own) (void)hipStreamDestroy(c->own);
  delete c;
}

int create_one(const gs_params* params, int device, bool shard, uint32_t G, uint32_t rank, gs_ctx** out) {
  std::string why;
  int rc = check_params(params, why);
  if (!rc) {
    gs_ctx* c = new gs_ctx();
    rc = ctx_setup(c, params, device, shard, G, rank, why);
    if (!rc) {
      *out = c;
      return GS_OK;
    }
    destroy_one(c);
  }
  fprintf(stderr, "gs_create: %s\n", why.c_str());
  return rc;
}

// Runs f(member) for every member, one host thread each (members on several
// devices, or several trial batches on one, overlap); first error wins.
template <class F>
int par_members(gs_ctx* g, F f) {
  std::vector<int> rcs(g->mem.size(), 0);
  std::vector<std::thread> th;
  for (size_t i = 0; i < g->mem.size(); ++i)
    th.emplace_back([&, i] {
      (void)hipSetDevice(g->mem[i]->dev);
      rcs[i] = f(g->mem[i]);
    });
  for (auto& t : th) t.join();
  for (size_t i = 0; i < rcs.size(); ++i)
    if (rcs[i]) return fail(g, rcs[i], "member " + std::to_string(i) + ": " + g->mem[i]->err);
  return GS_OK;
}

// Host copies of the broadcast counters a gs_ctx keeps: for a group, the
// group's own fields; members and ranks keep theirs.
void reset_counters(gs_ctx* c) {
  c->t = c->fired = c->sent = c->msgs = c->recv = c->crashed = c->pending = 0;
  for (TrialAcc& a : c->tacc) a = TrialAcc{};
}

// ---- multi-process exchange ----------------------------------
// A rank context exchanges through RCCL (gs_create_rank) or the caller's host
// callbacks (gs_create_rank_exchange); both are stream-ordered on c->stream.
bool is_rank(const gs_ctx* c) { return c->comm != nullptr || c->has_hx; }

bool grow_pinned(gs_ctx* c, size_t bytes) {
  if (c->h_xbytes >= bytes) return true;
  const size_t nb = std::max(bytes, c->h_xbytes + c->h_xbytes / 4);
  if (c->h_xbuf) (void)hipHostFree(c->h_xbuf);
  c->h_xbuf = nullptr;
  c->h_xbytes = 0;
  if (hipHostMalloc((void**)&c->h_xbuf, nb) != hipSuccess) return false;
  c->h_xbytes = nb;
  return true;
}

// In place: rank r's `bytes` at dbuf + r * bytes go to every rank.
int x_all_gather(gs_ctx* c, void* dbuf, size_t bytes) {
  if (c->comm) {
    NCK(c, rccl().all_gather((char*)dbuf + (size_t)c->rank * bytes, dbuf, bytes, ncclUint8, c->comm, c->stream));
    return GS_OK;
  }
  if (!grow_pinned(c, ((size_t)c->G + 1) * bytes)) return fail(c, GS_ENOMEM, "cannot allocate exchange staging");
  char* send = c->h_xbuf + (size_t)c->G * bytes;
  CK(c, hipMemcpyAsync(send, (char*)dbuf + (size_t)c->rank * bytes, bytes, hipMemcpyDeviceToHost, c->stream));
  CK(c, hipStreamSynchronize(c->stream));
  if (c->hx.all_gather(c->hx.user, send, c->h_xbuf, bytes))
    return fail(c, GS_EDEVICE, "the exchange's all_gather callback failed");
  CK(c, hipMemcpyAsync(dbuf, c->h_xbuf, (size_t)c->G * bytes, hipMemcpyHostToDevice, c->stream));
  CK(c, hipStreamSynchronize(c->stream));
  return GS_OK;
}

// In place: element-wise sum of `count` u64 over the ranks.
int x_all_reduce(gs_ctx* c, unsigned long long* dbuf, size_t count) {
  if (c->comm) {
    NCK(c, rccl().all_reduce(dbuf, dbuf, count, ncclUint64, ncclSum, c->comm, c->stream));
    return GS_OK;
  }
  if (!grow_pinned(c, count * 8)) return fail(c, GS_ENOMEM, "cannot allocate exchange staging");
  CK(c, hipMemcpyAsync(c->h_xbuf, dbuf, count * 8, hipMemcpyDeviceToHost, c->stream));
  CK(c, hipStreamSynchronize(c->stream));
  if (c->hx.all_reduce_sum_u64(c->hx.user, (uint64_t*)c->h_xbuf, count))
    return fail(c, GS_EDEVICE, "the exchange's all_reduce_sum_u64 callback failed");
  CK(c, hipMemcpyAsync(dbuf, c->h_xbuf, count * 8, hipMemcpyHostToDevice, c->stream));
  CK(c, hipStreamSynchronize(c->stream));
  return GS_OK;
}

// A rank whose collective failed is torn down so that the other ranks' RCCL
// calls fail instead of waiting for it (and torchrun-style launchers end the
// job when this process exits with the error).
int abort_rank(gs_ctx* c, int rc) {
  if (rc && is_rank(c)) c->aborted = true;
  if (rc && c->comm && rccl().ok && rccl().comm_abort) {
    (void)rccl().comm_abort(c->comm);
    c->comm = nullptr;
  }
  return rc;
}

// Push-pull shard c uses the replicated informed / failed sets ig / fg
// (G * segw words each): its own nodes are words [rank * segw, ...).
void attach_pp_sets(gs_ctx* c, unsigned long long* ig, unsigned long long* fg, unsigned long long* gn) {
  c->d_ig = ig;
  c->d_fg = fg;
  c->d_gn = gn;
  DevState& s = c->st;
  s.grecv = ig;
  s.gcrash = fg;
  s.gbase = c->lo;
  s.recv = ig + (size_t)c->rank * c->segw;
  s.crash = fg + (size_t)c->rank * c->segw;
}

int alloc_pp_sets(gs_ctx* c, uint64_t words, unsigned long long** ig, unsigned long long** fg,
                  unsigned long long** gn);
int make_replica(const gs_params* params, int dev, unsigned long long* ig, unsigned long long* fg, gs_ctx** out);

// The rest of a rank context once its exchange is set: gathered fire counts
// (flood) or its own replicated sets (push-pull).
int finish_rank(gs_ctx* c, gs_ctx** out) {
  (void)hipSetDevice(c->dev);
  if (dev_malloc(&c->d_gcounts, (size_t)c->G * kMaxWindow * 8 + (size_t)kMaxWindow * 8) != hipSuccess ||
      (!c->pp_shard && (dev_malloc(&c->d_glay, (size_t)c->G * (kRegions + 1) * 8) != hipSuccess ||
                        hipHostMalloc((void**)&c->h_glay, (size_t)c->G * (kRegions + 1) * 8) != hipSuccess))) {
    destroy_one(c);
    return GS_ENOMEM;
  }
  if (c->pp_shard) {
    unsigned long long *ig = nullptr, *fg = nullptr, *gn = nullptr, *gst = nullptr;
    if (alloc_pp_sets(c, (uint64_t)c->G * c->segw, &ig, &fg, &gn) ||
        alloc_pp_sets(c, (uint64_t)c->G * c->segw, &gst, nullptr, nullptr)) {
      fprintf(stderr, "gs_create_rank: %s\n", c->err.c_str());
      for (unsigned long long* q : {ig, fg, gn, gst})
        if (q) (void)dev_free(q);
      destroy_one(c);
      return GS_ENOMEM;
    }
    c->own_ig = true;
    c->d_gst = gst;
    attach_pp_sets(c, ig, fg, gn);
    if (make_replica(&c->p, c->dev, ig, fg, &c->rep)) {
      destroy_one(c);
      return GS_ENOMEM;
    }
    c->own_rep = c->rep != nullptr;
  }
  *out = c;
  return GS_OK;
}

// Allocates and zeroes up to three bitsets of `words` words (null outputs are
// skipped): the replicated informed / failed sets and the pull-answer set.
int alloc_pp_sets(gs_ctx* c, uint64_t words, unsigned long long** ig, unsigned long long** fg,
                  unsigned long long** gn) {
  for (unsigned long long** q : {ig, fg, gn}) {
    if (!q) continue;
    *q = nullptr;
    if (dev_malloc(q, words * 8) != hipSuccess)
      return fail(c, GS_ENOMEM, "cannot allocate the replicated informed / failed sets");
    CK(c, hipMemsetAsync(*q, 0, words * 8, c->stream));
  }
  CK(c, hipStreamSynchronize(c->stream));
  return GS_OK;
}

// The replica of push-pull shards on device `dev` (gs_ctx::rep): an unsharded
// push-pull context whose informed / failed sets are the replicated ig / fg.
// It gets the full table at load time (partition_pp).  GS_PP_NO_REPLICA=1:
// none (every round runs sharded bottom-up; A/B and memory-tight runs).
int make_replica(const gs_params* params, int dev, unsigned long long* ig, unsigned long long* fg, gs_ctx** out) {
  *out = nullptr;
  if (getenv("GS_PP_NO_REPLICA")) return GS_OK;
  gs_params rp = *params;
  rp.trials = 1;
  gs_ctx* r = nullptr;
  RC(create_one(&rp, dev, false, 1, 0, &r));
  r->st.recv = r->st.grecv = ig;
  r->st.crash = r->st.gcrash = fg;
  r->st.gbase = 0;
  *out = r;
  return GS_OK;
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
  return create_one(params, params ? params->device : 0, false, 1, 0, out);
}

int gs_create_multi(const gs_params* params, const int* devices, int ndev, gs_ctx** out) {
  if (!out || !params || !devices || ndev < 1) return GS_EINVAL;
  *out = nullptr;
  gs_ctx* g = new gs_ctx();
  g->group = true;
  g->p = *params;
  g->dev = devices[0];
  g->trials = std::max<uint32_t>(1, params->trials);
  g->gtrials = g->trials > 1;
  if (g->gtrials && (uint32_t)ndev > g->trials) ndev = (int)g->trials;
  for (int i = 0; i < ndev; ++i) {
    gs_params mp = *params;
    gs_ctx* m = nullptr;
    int rc;
    if (g->gtrials) {  // trials [t0, t1) on member i
      const uint32_t t0 = (uint32_t)((uint64_t)g->trials * i / ndev), t1 = (uint32_t)((uint64_t)g->trials * (i + 1) / ndev);
      mp.trial = params->trial + t0;
      mp.trials = t1 - t0;
      rc = create_one(&mp, devices[i], false, 1, 0, &m);
    } else {
      rc = create_one(&mp, devices[i], true, (uint32_t)ndev, (uint32_t)i, &m);
    }
    if (rc) {
      destroy_one(g);
      return rc;
    }
    g->mem.push_back(m);
    auto it = std::find(g->gdevs.begin(), g->gdevs.end(), devices[i]);
    if (it == g->gdevs.end()) {
      g->gdevs.push_back(devices[i]);
      g->gdev_of.push_back((int)g->gdevs.size() - 1);
    } else {
      g->gdev_of.push_back((int)(it - g->gdevs.begin()));
    }
  }
  g->gbuf.resize(g->gdevs.size());
  g->pp = params->model == GS_MODEL_PUSHPULL;
  if (g->pp && !g->gtrials) {  // push-pull shards: one pair of replicated sets per device
    g->gig.assign(g->gdevs.size(), nullptr);
    g->gfg.assign(g->gdevs.size(), nullptr);
    g->ggn.assign(g->gdevs.size(), nullptr);
    for (size_t d = 0; d < g->gdevs.size(); ++d) {
      std::vector<gs_ctx*> ms;
      for (size_t i = 0; i < g->mem.size(); ++i)
        if ((size_t)g->gdev_of[i] == d) ms.push_back(g->mem[i]);
      (void)hipSetDevice(g->gdevs[d]);
      if (alloc_pp_sets(ms[0], (uint64_t)g->mem.size() * ms[0]->segw, &g->gig[d], &g->gfg[d], &g->ggn[d])) {
        fprintf(stderr, "gs_create_multi: %s\n", ms[0]->err.c_str());
        destroy_one(g);
        return GS_ENOMEM;
      }
      for (gs_ctx* m : ms) attach_pp_sets(m, g->gig[d], g->gfg[d], g->ggn[d]);
      gs_ctx* r = nullptr;
      if (make_replica(params, g->gdevs[d], g->gig[d], g->gfg[d], &r)) {
        destroy_one(g);
        return GS_ENOMEM;
      }
      g->greps.push_back(r);
      for (gs_ctx* m : ms) m->rep = r;
    }
  }
  for (size_t i = 0; i < g->mem.size(); ++i) {
    hipEvent_t e;
    (void)hipSetDevice(g->mem[i]->dev);
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
      destroy_one(g);
      return GS_EDEVICE;
    }
    g->gev_c.push_back(e);
  }
  for (size_t d = 0; d < g->gdevs.size(); ++d) {
    hipEvent_t e;
    (void)hipSetDevice(g->gdevs[d]);
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
      destroy_one(g);
      return GS_EDEVICE;
    }
    g->gev_x.push_back(e);
  }
  g->tacc.assign(g->gtrials ? 0 : 1, TrialAcc{});
  *out = g;
  return GS_OK;
}

int gs_comm_unique_id(uint8_t id[GS_COMM_ID_BYTES]) {
  if (!id) return GS_EINVAL;
  const Rccl& r = rccl();
  if (!r.ok) {
    fprintf(stderr, "gs_comm_unique_id: %s\n", r.why.c_str());
    return GS_EDEVICE;
  }
  ncclUniqueId u;
  if (r.get_unique_id(&u) != ncclSuccess) return GS_EDEVICE;
  static_assert(sizeof(ncclUniqueId) == GS_COMM_ID_BYTES, "RCCL unique id size");
  memcpy(id, &u, GS_COMM_ID_BYTES);
  return GS_OK;
}

int gs_create_rank(const gs_params* params, int device, int nranks, int rank, const uint8_t* id, gs_ctx** out) {
  if (!out || !params || nranks < 1 || rank < 0 || rank >= nranks) return GS_EINVAL;
  *out = nullptr;
  const uint32_t T = std::max<uint32_t>(1, params->trials);
  if (T > 1) {  // this rank's share of the trials, no communication
    gs_params mp = *params;
    const uint32_t t0 = (uint32_t)((uint64_t)T * rank / nranks), t1 = (uint32_t)((uint64_t)T * (rank + 1) / nranks);
    if (t1 == t0) {
      fprintf(stderr, "gs_create_rank: %u trials leave rank %d none\n", T, rank);
      return GS_EINVAL;
    }
    mp.trial = params->trial + t0;
    mp.trials = t1 - t0;
    return create_one(&mp, device, false, 1, 0, out);
  }
  if (!id) return GS_EINVAL;
  const Rccl& r = rccl();
  if (!r.ok) {
    fprintf(stderr, "gs_create_rank: %s\n", r.why.c_str());
    return GS_EDEVICE;
  }
  gs_ctx* c = nullptr;
  int rc = create_one(params, device, true, (uint32_t)nranks, (uint32_t)rank, &c);
  if (rc) return rc;
  ncclUniqueId u;
  memcpy(&u, id, GS_COMM_ID_BYTES);
  (void)hipSetDevice(device);
  ncclResult_t nr = r.comm_init_rank(&c->comm, nranks, u, rank);
  if (nr != ncclSuccess) {
    fprintf(stderr, "gs_create_rank: ncclCommInitRank: %s\n", rccl_error((int)nr).c_str());
    c->comm = nullptr;
    destroy_one(c);
    return GS_EDEVICE;
  }
  return finish_rank(c, out);
}

int gs_create_rank_exchange(const gs_params* params, int device, int nranks, int rank, const gs_exchange* ex,
                            gs_ctx** out) {
  if (!out || !params || !ex || !ex->all_gather || !ex->all_reduce_sum_u64 || nranks < 1 || rank < 0 ||
      rank >= nranks)
    return GS_EINVAL;
  if (params->model == GS_MODEL_FLOOD && std::max<uint32_t>(1, params->trials) == 1 && !ex->all_to_allv) {
    fprintf(stderr, "gs_create_rank_exchange: flood shards need the all_to_allv callback\n");
    return GS_EINVAL;
  }
  *out = nullptr;
  if (std::max<uint32_t>(1, params->trials) > 1) return gs_create_rank(params, device, nranks, rank, nullptr, out);
  gs_ctx* c = nullptr;
  int rc = create_one(params, device, true, (uint32_t)nranks, (uint32_t)rank, &c);
  if (rc) return rc;
  c->hx = *ex;
  c->has_hx = true;
  return finish_rank(c, out);
}

int gs_shard_info(const gs_ctx* c, uint32_t index, uint32_t* nshards, uint64_t* lo, uint64_t* hi) {
  if (!c) return GS_EINVAL;
  const bool sg = c->group && !c->gtrials;
  const uint32_t ns = sg ? (uint32_t)c->mem.size() : c->shard ? c->G : 1u;
  if (nshards) *nshards = ns;
  if (index >= ns) return GS_EINVAL;
  const gs_ctx* s = sg ? c->mem[0] : c;
  uint64_t a = 0, b = c->p.n;
  if (s->shard) {
    a = std::min<uint64_t>(index * s->seg_per, c->p.n);
    b = std::min<uint64_t>(a + s->seg_per, c->p.n);
  }
  if (lo) *lo = a;
  if (hi) *hi = b;
  return GS_OK;
}

void gs_destroy(gs_ctx* c) { destroy_one(c); }

}  // extern "C"

// ---------------------------------------------------------------------------
// Peer tables
// ---------------------------------------------------------------------------
namespace {

// Uploads a host table into `c`'s table buffers (c = a plain/batched context,
// or the device leader of shards) and validates it.
int upload_table(gs_ctx* c, const uint8_t* deg, const uint32_t* ids, uint32_t stride) {
  CK(c, hipSetDevice(c->dev));
  const uint32_t S = stride < 2 ? 2 : stride;
  c->row_slots = 0;  // injected rows are used as given
  RC(alloc_table(c, S));
  const uint64_t n = table_n(c);
  if (c->trials > 1) {  // trial tables back to back -> the padded id space
    const uint64_t np = c->p.n, per = 1ull << c->tlog;
    std::vector<uint8_t> hd(n, 0);
    std::vector<uint32_t> hi(n * S, 0);
    for (uint32_t t = 0; t < c->trials; ++t)
      for (uint64_t v = 0; v < np; ++v) {
        const uint64_t src = t * np + v, dst = t * per + v;
        const uint32_t d = deg[src];
        if (d > stride) return fail(c, GS_EINVAL, "a friends-list length exceeds the row stride");
        hd[dst] = (uint8_t)d;
        for (uint32_t j = 0; j < d; ++j) {
          const uint32_t x = ids[src * stride + j];
          if (x >= np) return fail(c, GS_EINVAL, "a friend id is >= n");
          hi[dst * S + j] = (uint32_t)(t * per) | x;
        }
      }
    CK(c, hipMemcpyAsync(c->d_deg, hd.data(), n, hipMemcpyHostToDevice, c->stream));
    CK(c, hipMemcpyAsync(c->d_ids, hi.data(), n * S * 4, hipMemcpyHostToDevice, c->stream));
    CK(c, hipStreamSynchronize(c->stream));
    return GS_OK;
  }
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
  return validate_table(c, c->d_deg, c->d_ids, n, c->p.n);
}

// Push-pull shards: each member keeps the rows of its own nodes (its callers)
// and the reverse table of its own nodes (in-edges from every caller), built
// from the leader's full table, which is then dropped.
int partition_pp(gs_ctx* leader, const std::vector<gs_ctx*>& ms) {
  uint8_t* fdeg = leader->d_deg;
  uint32_t* fids = leader->d_ids;
  const uint32_t S = leader->st.stride, slots = leader->row_slots;
  const uint64_t N = leader->p.n;
  leader->d_deg = nullptr;
  leader->d_ids = nullptr;
  leader->tab_stride = 0;
  int rc = GS_OK;
  for (gs_ctx* m : ms) {
    const uint64_t n = m->ntot;
    if (m->d_deg) (void)dev_free(m->d_deg);
    if (m->d_ids) (void)dev_free(m->d_ids);
    m->d_deg = nullptr;
    m->d_ids = nullptr;
    if (dev_malloc(&m->d_deg, n) != hipSuccess || dev_malloc(&m->d_ids, n * S * 4ull) != hipSuccess) {
      rc = fail(m, GS_ENOMEM, "cannot allocate the shard's rows");
      break;
    }
    m->tab_stride = 0;  // not the full-table shape: the next load reallocates
    if ((rc = set_stride(m, S))) break;
    refresh_state(m);
    if (hipMemcpyAsync(m->d_deg, fdeg + m->lo, n, hipMemcpyDeviceToDevice, leader->stream) != hipSuccess ||
        hipMemcpyAsync(m->d_ids, fids + m->lo * S, n * S * 4ull, hipMemcpyDeviceToDevice, leader->stream) !=
            hipSuccess) {
      rc = fail(m, GS_EDEVICE, "copying the shard's rows failed");
      break;
    }
    // reverse table of [lo, hi): count + scan, then size the edge arrays
    const size_t scan = pp_rev_range_scan_bytes(n);
    if (!grow(m->pp_rend, (n + 1) * 8) || !grow(m->pp_scan, scan + 256) || !grow(m->pp_ctlb, sizeof(PPCtl))) {
      rc = fail(m, GS_ENOMEM, "cannot allocate the shard's reverse table");
      break;
    }
    unsigned long long* rend = (unsigned long long*)m->pp_rend.p;
    if (pp_rev_count_range(fdeg, fids, N, S, m->lo, m->hi, rend, m->pp_scan.p, m->pp_scan.bytes, leader->stream) !=
        hipSuccess) {
      rc = fail(m, GS_EDEVICE, "counting the shard's in-edges failed");
      break;
    }
    unsigned long long E = 0;
    if (hipMemcpyAsync(&E, rend + n, 8, hipMemcpyDeviceToHost, leader->stream) != hipSuccess ||
        hipStreamSynchronize(leader->stream) != hipSuccess) {
      rc = fail(m, GS_EDEVICE, "reading the shard's in-edge count failed");
      break;
    }
    if (!grow(m->pp_rsrc, std::max<uint64_t>(E, 1) * 4) || !grow(m->pp_rslot, std::max<uint64_t>(E, 1))) {
      rc = fail(m, GS_ENOMEM, "cannot allocate the shard's in-edges");
      break;
    }
    if (pp_rev_fill_range(fdeg, fids, N, S, m->lo, m->hi, rend, (uint32_t*)m->pp_rsrc.p, (uint8_t*)m->pp_rslot.p,
                          leader->stream) != hipSuccess ||
        hipStreamSynchronize(leader->stream) != hipSuccess) {
      rc = fail(m, GS_EDEVICE, "filling the shard's in-edges failed");
      break;
    }
    ++m->table_ver;
    m->rev_ver = m->table_ver;
    m->fm_tver = ~0ull;
    m->peers = true;
  }
  gs_ctx* r = ms[0]->rep;
  if (r && rc == GS_OK) {  // the full table stays on the device as the replica's
    if (r->d_deg) (void)dev_free(r->d_deg);
    if (r->d_ids) (void)dev_free(r->d_ids);
    r->d_deg = fdeg;
    r->d_ids = fids;
    r->tab_stride = S;
    r->row_slots = slots;
    if ((rc = set_stride(r, S))) return fail(leader, rc, r->err);
    refresh_state(r);
    ++r->table_ver;
    r->peers = true;
    return GS_OK;
  }
  (void)dev_free(fdeg);
  (void)dev_free(fids);
  return rc;
}

// Shards: partition every member on the leader's device from the leader's
// sealed table, then drop the replicated table.
int partition_from(gs_ctx* leader, const std::vector<gs_ctx*>& ms) {
  if (leader->pp_shard) return partition_pp(leader, ms);
  uint8_t* fdeg = leader->d_deg;
  uint32_t* fids = leader->d_ids;
  const uint32_t S = leader->st.stride, slots = leader->row_slots;
  leader->d_deg = nullptr;  // own_rows must not free the full table it copies from
  leader->d_ids = nullptr;
  int rc = GS_OK;
  for (gs_ctx* m : ms) {
    if ((rc = own_rows(m, fdeg, fids, S, slots, leader->stream))) break;
    m->peers = true;
  }
  (void)dev_free(fdeg);
  (void)dev_free(fids);
  return rc;
}

// Members sharing device d (group) or just c.
std::vector<gs_ctx*> on_device(gs_ctx* g, size_t d) {
  std::vector<gs_ctx*> v;
  for (size_t i = 0; i < g->mem.size(); ++i)
    if ((size_t)g->gdev_of[i] == d) v.push_back(g->mem[i]);
  return v;
}

}  // namespace

extern "C" {

int gs_load_peers(gs_ctx* c, const uint8_t* deg, const uint32_t* ids, uint32_t stride) {
  if (!c || !deg || !ids || stride == 0 || stride > 255) return fail(c, GS_EINVAL, "bad peer table");
  if (c->begun) return fail(c, GS_EINVAL, "peers must be loaded before gs_broadcast_begin");
  if (c->group && c->gtrials) {
    uint64_t off = 0;
    for (gs_ctx* m : c->mem) {
      RC(gs_load_peers(m, deg + off * c->p.n, ids + off * c->p.n * stride, stride) ? fail(c, GS_EINVAL, m->err) : 0);
      off += m->trials;
    }
    c->peers = true;
    return GS_OK;
  }
  if (c->group) {
    for (size_t d = 0; d < c->gdevs.size(); ++d) {
      std::vector<gs_ctx*> ms = on_device(c, d);
      int rc = upload_table(ms[0], deg, ids, stride);
      if (!rc) rc = seal_rows(ms[0], ms[0]->d_deg, ms[0]->d_ids, c->p.n);
      if (!rc) rc = partition_from(ms[0], ms);
      if (rc) return fail(c, rc, ms[0]->err);
    }
    c->peers = true;
    return GS_OK;
  }
  RC(upload_table(c, deg, ids, stride));
  RC(seal_rows(c, c->d_deg, c->d_ids, table_n(c)));
  if (c->shard) RC(partition_from(c, {c}));
  c->peers = true;
  return GS_OK;
}

int gs_load_peers_device(gs_ctx* c, const void* d_deg, const void* d_ids, uint32_t stride) {
  if (!c || !d_deg || !d_ids || stride < 2 || stride > 255)
    return fail(c, GS_EINVAL, "bad device peer table (stride must be in [2,255])");
  if (c->begun) return fail(c, GS_EINVAL, "peers must be loaded before gs_broadcast_begin");
  if (c->group || c->trials > 1)
    return fail(c, GS_EINVAL, "device tables load into one-device, one-trial contexts");
  CK(c, hipSetDevice(c->dev));
  c->row_slots = 0;
  RC(alloc_table(c, stride));
  const uint64_t n = table_n(c);
  CK(c, hipMemcpyAsync(c->d_deg, d_deg, n, hipMemcpyDeviceToDevice, c->stream));
  CK(c, hipMemcpyAsync(c->d_ids, d_ids, n * stride * 4ull, hipMemcpyDeviceToDevice, c->stream));
  RC(validate_table(c, c->d_deg, c->d_ids, n, c->p.n));
  RC(seal_rows(c, c->d_deg, c->d_ids, n));
  if (c->shard) RC(partition_from(c, {c}));
  c->peers = true;
  return GS_OK;
}

int gs_read_peers(gs_ctx* c, uint8_t* deg, uint32_t* ids, uint32_t* stride_out) {
  if (!c || !c->peers) return fail(c, GS_EINVAL, "no peer table");
  if (c->group && c->gtrials) {
    uint32_t s = 0;
    uint64_t off = 0;
    for (gs_ctx* m : c->mem) {
      if (gs_read_peers(m, deg ? deg + off * c->p.n : nullptr, nullptr, &s)) return fail(c, GS_EINVAL, m->err);
      if (ids && gs_read_peers(m, nullptr, ids + off * c->p.n * s, &s)) return fail(c, GS_EINVAL, m->err);
      off += m->trials;
    }
    if (stride_out) *stride_out = s;
    return GS_OK;
  }
  if (c->group || c->shard)
    return fail(c, GS_EINVAL, "a sharded context keeps only its partition of the table");
  const uint32_t S = c->st.stride, So = c->row_slots && c->row_slots < S ? c->row_slots : S;
  if (stride_out) *stride_out = So;
  CK(c, hipSetDevice(c->dev));
  if (c->trials > 1) {  // padded id space -> trial tables back to back, local ids
    const uint64_t np = c->p.n, per = 1ull << c->tlog;
    std::vector<uint8_t> hd(c->ntot);
    std::vector<uint32_t> hi;
    CK(c, hipMemcpyAsync(hd.data(), c->d_deg, c->ntot, hipMemcpyDeviceToHost, c->stream));
    if (ids) {
      hi.resize(c->ntot * S);
      CK(c, hipMemcpyAsync(hi.data(), c->d_ids, c->ntot * S * 4ull, hipMemcpyDeviceToHost, c->stream));
    }
    CK(c, hipStreamSynchronize(c->stream));
    for (uint32_t t = 0; t < c->trials; ++t)
      for (uint64_t v = 0; v < np; ++v) {
        const uint64_t src = t * per + v, dst = t * np + v;
        if (deg) deg[dst] = hd[src];
        if (ids)
          for (uint32_t j = 0; j < So; ++j) {
            const uint32_t x = hi[src * S + j];
            ids[dst * So + j] = x == kEmptyMsg ? x : (x & ((uint32_t)per - 1));
          }
      }
    return GS_OK;
  }
  if (deg) CK(c, hipMemcpyAsync(deg, c->d_deg, c->p.n, hipMemcpyDeviceToHost, c->stream));
  if (ids && So == S) CK(c, hipMemcpyAsync(ids, c->d_ids, c->p.n * S * 4ull, hipMemcpyDeviceToHost, c->stream));
  if (ids && So != S)  // padded rows: the first So slots of each
    CK(c, hipMemcpy2DAsync(ids, So * 4ull, c->d_ids, S * 4ull, So * 4ull, c->p.n, hipMemcpyDeviceToHost, c->stream));
  CK(c, hipStreamSynchronize(c->stream));
  return GS_OK;
}

}  // extern "C"

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

// The overlay of c's table_n(c) nodes (all trials of a batched context) into
// c's table buffers.
int overlay_into(gs_ctx* c, uint64_t max_ticks, gs_window* win, size_t cap, size_t* nwin, uint64_t* final_tick) {
  CK(c, hipSetDevice(c->dev));
  const uint32_t fo = (uint32_t)c->p.fanout, fi = (uint32_t)c->p.fanin;
  uint32_t stride = fo > fi ? fo : fi;
  if (stride < 2) stride = 2;
  // Window engine: rows of 5..7 slots are padded to 8 (32 B, 16-B aligned):
  // a row never straddles two 128-B lines and k_expand gathers it with one
  // uint4 + one uint2 load instead of three uint2 loads (C5: 67.3 -> 66.3 ms
  // per broadcast).  gs_read_peers returns the unpadded rows.
  // Rows of 9..31 slots (C4: fanin 19) are padded to a multiple of 4: 16-B
  // aligned rows gathered with uint4 loads.
  c->row_slots = 0;
  if (c->win && stride > 4 && stride < 8) {
    c->row_slots = stride;
    stride = 8;
  } else if (c->win && stride > 8 && (stride & 3)) {
    c->row_slots = stride;
    stride = (stride + 3) & ~3u;
  }
  RC(alloc_table(c, stride));
  const uint64_t n = table_n(c);
  CK(c, hipMemsetAsync(c->d_ids, 0, n * stride * 4ull, c->stream));
  CK(c, hipMemsetAsync(c->d_deg, 0, n, c->stream));
  WinSink ws{win, cap, 0};
  OverlayResult res;
  const auto t0 = std::chrono::steady_clock::now();
  const int rc = overlay_build(c->p.n, c->trials, c->tlog, c->p.fanout, c->p.fanin, c->p.delay_low,
                               c->p.delay_high, c->st.key, c->d_deg, c->d_ids, stride, max_ticks, c->stream,
                               OverlayWindowSink{&WinSink::push, &ws}, &res, &c->ovw);
  c->timing.overlay_ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  c->timing.ov_part_ticks = c->ovw.part_ticks;
  c->timing.ov_sort_ticks = c->ovw.sort_ticks;
  c->timing.ov_part_fallbacks = c->ovw.part_fallbacks;
  if (nwin) *nwin = ws.n;
  if (final_tick) *final_tick = res.final_tick;
  // batched contexts rebuild per batch (gs_set_trial): keep the workspace
  if (c->trials <= 1) overlay_free(&c->ovw, c->stream);
  if (rc) return fail(c, rc, res.msg);
  return seal_rows(c, c->d_deg, c->d_ids, n);
}
}  // namespace

extern "C" {

int gs_build_overlay(gs_ctx* c, uint64_t max_ticks, gs_window* win, size_t cap, size_t* nwin,
                     uint64_t* final_tick) {
  if (!c) return GS_EINVAL;
  if (c->begun) return fail(c, GS_EINVAL, "overlay must be built before gs_broadcast_begin");
  if (c->group && c->gtrials) {
    std::vector<uint64_t> ft(c->mem.size(), 0);
    std::vector<size_t> nw(c->mem.size(), 0);
    std::vector<gs_ctx*>& ms = c->mem;
    RC(par_members(c, [&](gs_ctx* m) {
      const size_t i = (size_t)(std::find(ms.begin(), ms.end(), m) - ms.begin());
      return gs_build_overlay(m, max_ticks, i == 0 ? win : nullptr, i == 0 ? cap : 0, &nw[i], &ft[i]);
    }));
    if (nwin) *nwin = nw[0];
    if (final_tick) *final_tick = *std::max_element(ft.begin(), ft.end());
    c->timing.overlay_ms = c->mem[0]->timing.overlay_ms;
    c->peers = true;
    return GS_OK;
  }
  if (c->group) {
    for (size_t d = 0; d < c->gdevs.size(); ++d) {
      std::vector<gs_ctx*> ms = on_device(c, d);
      int rc = overlay_into(ms[0], max_ticks, d == 0 ? win : nullptr, d == 0 ? cap : 0,
                            d == 0 ? nwin : nullptr, d == 0 ? final_tick : nullptr);
      if (!rc) rc = partition_from(ms[0], ms);
      if (rc) return fail(c, rc, ms[0]->err);
    }
    c->timing.overlay_ms = c->mem[0]->timing.overlay_ms;
    c->peers = true;
    return GS_OK;
  }
  RC(overlay_into(c, max_ticks, win, cap, nwin, final_tick));
  if (c->shard) RC(partition_from(c, {c}));
  c->peers = true;
  return GS_OK;
}

int gs_set_failed(gs_ctx* c, const uint64_t* words, size_t nwords) {
  if (!c || !words || nwords < (c->p.n + 63) / 64) return fail(c, GS_EINVAL, "mask needs ceil(n/64) words");
  if (c->begun) return fail(c, GS_EINVAL, "failure mask must be set before gs_broadcast_begin");
  if (c->trials > 1) return fail(c, GS_EINVAL, "failure masks are not supported for batched trials");
  if (c->group) {
    for (gs_ctx* m : c->mem)
      if (gs_set_failed(m, words, nwords)) return fail(c, GS_EINVAL, m->err);
    c->failed = true;
    return GS_OK;
  }
  CK(c, hipSetDevice(c->dev));
  if (c->pp_shard) {  // the replicated failed set: every word (k_ppb_round reads the callers' friends)
    if (c->st.stride > 8) return fail(c, GS_EINVAL, "push-pull shards take a failure mask with rows <= 8 slots");
    const uint64_t Wg = (c->p.n + 63) / 64;
    std::vector<uint64_t> w(words, words + Wg);
    if (c->p.n & 63) w[Wg - 1] &= (1ull << (c->p.n & 63)) - 1;
    CK(c, hipMemcpyAsync(c->d_fg, w.data(), Wg * 8, hipMemcpyHostToDevice, c->stream));
    CK(c, hipStreamSynchronize(c->stream));
    c->failed = true;
    c->st.check_crashed = 1;
    ++c->fail_ver;
    if (c->rep) {  // the replica reads the same replicated failed set
      c->rep->failed = true;
      c->rep->st.check_crashed = 1;
      ++c->rep->fail_ver;
    }
    return GS_OK;
  }
  const uint64_t W = c->st.W, w0 = c->lo / 64;  // this context's words (a shard's own range)
  std::vector<uint64_t> w(words + w0, words + w0 + W);
  if (c->ntot & 63) w[W - 1] &= (1ull << (c->ntot & 63)) - 1;
  if (!c->d_failed && dev_malloc(&c->d_failed, W * 8) != hipSuccess)
    return fail(c, GS_ENOMEM, "cannot allocate the failure mask");
  CK(c, hipMemcpyAsync(c->d_failed, w.data(), W * 8, hipMemcpyHostToDevice, c->stream));
  CK(c, hipMemcpyAsync(c->st.crash, c->d_failed, W * 8, hipMemcpyDeviceToDevice, c->stream));
  CK(c, hipStreamSynchronize(c->stream));
  c->failed = true;
  c->st.check_crashed = 1;
  ++c->fail_ver;
  return GS_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Broadcast
// ---------------------------------------------------------------------------
namespace {

// Is local node `u` of c crashed (a pre-failed mask)?
int is_failed(gs_ctx* c, uint64_t u, bool* out) {
  *out = false;
  if (!c->failed) return GS_OK;
  unsigned long long w = 0;
  CK(c, hipMemcpyAsync(&w, c->st.crash + u / 64, 8, hipMemcpyDeviceToHost, c->stream));
  CK(c, hipStreamSynchronize(c->stream));
  *out = (w >> (u & 63)) & 1;
  return GS_OK;
}

uint64_t keyed_sender(const gs_ctx* c) {
  return uniform(draw0(c->st.key, K_SENDER, 0, 0, 0), (uint32_t)c->p.n);  // simulator.go:240
}

// Schedules the global sender s if c owns it (and it is live); *sched = 1 if so.
int begin_one(gs_ctx* c, uint64_t s, uint32_t* sched) {
  *sched = 0;
  CK(c, hipSetDevice(c->dev));
  if (c->trials > 1) {  // every trial's sender (:240 per trial when s == ~0)
    CK(c, win_schedule(c->ws, (uint32_t)s, 0, c->trials, (uint32_t)c->p.n, c->stream));
    CK(c, hipStreamSynchronize(c->stream));
    *sched = c->trials;
    return GS_OK;
  }
  if (s < c->lo || s >= (c->shard ? c->hi : c->p.n)) return GS_OK;  // another shard's node
  const uint64_t u = s - c->lo;
  bool dead = false;
  RC(is_failed(c, u, &dead));
  if (dead) return GS_OK;  // a failed sender never broadcasts
  if (c->win) CK(c, win_schedule(c->ws, (uint32_t)u, 0, 1, (uint32_t)c->p.n, c->stream));
  else CK(c, launch_schedule_one(c->st, (uint32_t)u, 0, c->stream));
  CK(c, hipStreamSynchronize(c->stream));
  *sched = 1;
  return GS_OK;
}

// Push-pull sparse-round buffers: the reverse table
// once per peer table, the failed-slot mask once per (table, failure mask),
// the informed list and round control.  GS_FLAG_PP_DENSE, or buffers that do
// not fit, leave the dense rounds only (same results).
// The failed-slot mask buffer: fmask bytes [n] (8-aligned), then the fany
// bitset [ceil(n / 64)] (pp_fmask_any).
size_t fmask_bytes(uint64_t n) { return ((n + 7) & ~7ull) + ((n + 63) >> 6) * 8; }
unsigned long long* fmask_any(gs_ctx* c) {
  return (unsigned long long*)((char*)c->pp_fmask.p + ((c->st.n + 7) & ~7ull));
}

// pp_seed on context c's state and stream: the live callers are counted
// once per (table, failure mask) version and reused after (a pass over the
// 1e9 degree bytes was 0.76 ms of every push-pull broadcast_begin).  Leaves
// the stream synchronized.
int pp_seed_ctx(gs_ctx* c, unsigned long long* next, uint32_t node, unsigned long long thr, unsigned long long bthr,
                unsigned long long athr) {
  const bool known = c->sp.ctl && c->cl_tver == c->table_ver && c->cl_fver == c->fail_ver;
  CK(c, pp_seed(c->st, next, node, c->d_flag, c->sp, thr, bthr, athr, known ? c->cl_counts : nullptr, c->stream));
  if (c->sp.ctl && !known) {
    CK(c, hipMemcpyAsync(&c->cl_counts[0], &c->sp.ctl->ncallers, 8, hipMemcpyDeviceToHost, c->stream));
    CK(c, hipMemcpyAsync(&c->cl_counts[1], &c->sp.ctl->nlive0, 8, hipMemcpyDeviceToHost, c->stream));
    CK(c, hipStreamSynchronize(c->stream));
    c->cl_tver = c->table_ver;
    c->cl_fver = c->fail_ver;
  }
  CK(c, hipStreamSynchronize(c->stream));
  return GS_OK;
}

int pp_prepare(gs_ctx* c) {
  c->sp = PPSparse{};
  static const bool load_deg = [] { const char* e = getenv("GS_PP_NODEG"); return e && atoi(e) == 0; }();  // A/B
  c->sp.nodeg = load_deg ? 0u : 1u;
  // k_ppb_round's ranges: 2 = a lane per word where few nodes are uninformed
  // (default), 1 = always, 0 = never (GS_PPB_WORDS, A/B)
  static const uint32_t words = [] { const char* e = getenv("GS_PPB_WORDS"); return e ? (uint32_t)std::min(std::max(atoi(e), 0), 2) : 2u; }();
  c->sp.words = words;
  static const uint32_t maxu = [] { const char* e = getenv("GS_PPB_WORD_MAXU"); return e ? (uint32_t)std::max(atoi(e), 0) : 64u; }();
  c->sp.word_maxu = maxu;
  static const uint32_t maxi = [] { const char* e = getenv("GS_PPA_WORD_MAXI"); return e ? (uint32_t)std::max(atoi(e), 0) : 64u; }();
  c->sp.word_maxi = maxi;
  static const uint32_t pullfirst = [] { const char* e = getenv("GS_PPB_PULLFIRST"); return e && !atoi(e) ? 0u : 1u; }();
  c->sp.pullfirst = pullfirst;
  if (c->pp_shard) {  // bottom-up rounds only: the partition built the reverse table
    c->sp.ctl = (PPCtl*)c->pp_ctlb.p;
    c->sp.rend = (const unsigned long long*)c->pp_rend.p;
    c->sp.rsrc = (const uint32_t*)c->pp_rsrc.p;
    c->sp.rslot = (const uint8_t*)c->pp_rslot.p;
    if (c->failed) {
      if (c->fm_tver != c->table_ver || c->fm_fver != c->fail_ver) {
        if (!grow(c->pp_fmask, fmask_bytes(c->st.n))) return fail(c, GS_ENOMEM, "cannot allocate the failed-slot mask");
        CK(c, pp_fmask_rows(c->st, (uint8_t*)c->pp_fmask.p, c->stream));
        CK(c, pp_fmask_any((const uint8_t*)c->pp_fmask.p, c->st.n, fmask_any(c), c->stream));
        c->fm_tver = c->table_ver;
        c->fm_fver = c->fail_ver;
      }
      c->sp.fmask = (const uint8_t*)c->pp_fmask.p;
      c->sp.fany = fmask_any(c);
    }
    return GS_OK;
  }
  if (c->p.flags & GS_FLAG_PP_DENSE) return GS_OK;
  const DevState& s = c->st;
  const uint64_t n = s.n, E = n * s.stride;
  const auto t0 = std::chrono::steady_clock::now();
  bool built = false;
  if (c->rev_ver != c->table_ver) {
    const size_t scan = pp_rev_scan_bytes(n);
    if (!grow(c->pp_rend, (n + 1) * 8) || !grow(c->pp_rsrc, E * 4) || !grow(c->pp_rslot, E) ||
        !grow(c->pp_scan, scan + 256) || !grow(c->pp_ilist, (n + kPPSegs) * 4) || !grow(c->pp_ctlb, sizeof(PPCtl))) {
      (void)hipGetLastError();
      return GS_OK;  // dense rounds only
    }
    // by partitioning (GS_PP_REV_ATOMIC=1: the atomic count + fill, A/B);
    // the atomic build also takes what the partition cannot (memory, skew)
    // (both switches read per call, so tests can force either path)
    const bool rev_atomic = getenv("GS_PP_REV_ATOMIC") != nullptr;
    bool part = false;
    uint32_t passes = 0;
    if (!rev_atomic) {
      part = pp_rev_build_part(s, (unsigned long long*)c->pp_rend.p, (uint32_t*)c->pp_rsrc.p,
                               (uint8_t*)c->pp_rslot.p, c->stream, &passes) == hipSuccess;
      if (!part) (void)hipGetLastError();
    }
    if (!part)
      CK(c, pp_rev_build(s, (unsigned long long*)c->pp_rend.p, (uint32_t*)c->pp_rsrc.p, (uint8_t*)c->pp_rslot.p,
                         c->pp_scan.p, c->pp_scan.bytes, c->stream));
    c->timing.pp_rev_part = part ? passes : 0;
    c->rev_ver = c->table_ver;
    c->fm_tver = ~0ull;
    built = true;
    // the dense rounds' compact view of rend (2.1 B per node instead of 8)
    c->rend16_ok = false;
    const size_t r16 = (n * 2 + 255) / 256 * 256, rb = ((n >> 6) + 1) * 8;
    if (grow(c->pp_rend16, r16 + rb + 8)) {
      char* base = (char*)c->pp_rend16.p;
      uint32_t* ovf = (uint32_t*)(base + r16 + rb);
      uint32_t h_ovf = 1;
      CK(c, hipMemsetAsync(ovf, 0, 4, c->stream));
      CK(c, pp_rev_compact((const unsigned long long*)c->pp_rend.p, n, (uint16_t*)base,
                           (unsigned long long*)(base + r16), ovf, c->stream));
      CK(c, hipMemcpyAsync(&h_ovf, ovf, 4, hipMemcpyDeviceToHost, c->stream));
      CK(c, hipStreamSynchronize(c->stream));
      c->rend16_ok = h_ovf == 0;
    } else {
      (void)hipGetLastError();  // rend only
    }
  }
  c->sp.ctl = (PPCtl*)c->pp_ctlb.p;
  c->sp.ilist = (uint32_t*)c->pp_ilist.p;
  c->sp.rend = (const unsigned long long*)c->pp_rend.p;
  c->sp.rsrc = (const uint32_t*)c->pp_rsrc.p;
  c->sp.rslot = (const uint8_t*)c->pp_rslot.p;
  // (GS_PP_REND16=0: the dense rounds read rend, A/B; read per call)
  if (c->rend16_ok && !(getenv("GS_PP_REND16") && atoi(getenv("GS_PP_REND16")) == 0)) {
    const size_t r16 = (n * 2 + 255) / 256 * 256;
    c->sp.rend16 = (const uint16_t*)c->pp_rend16.p;
    c->sp.rbase = (const unsigned long long*)((const char*)c->pp_rend16.p + r16);
  }
  // the pull-answer rounds' deferred sets (n <= 2^30; GS_PP_NODEFER=1: atomics, A/B):
  // lists, coarse and fine regions for 0.6 n sets each (more fall back to atomicOr)
  if (!getenv("GS_PP_NODEFER") && n <= (1ull << 30) && pp_rslot_packed(s.stride)) {
    const uint64_t nfine = (n + 16383) >> 14, want = n * 3 / 5;
    const uint64_t dcap = std::max<uint64_t>(4096, (want + kPPDLists - 1) / kPPDLists);
    const uint64_t ccap = std::max<uint64_t>(4096, (want + kPPDRegions - 1) / kPPDRegions), fcap = 16384;
    const size_t elems = (size_t)kPPDLists * dcap + (size_t)kPPDRegions * ccap + (size_t)nfine * fcap;
    if (grow(c->pp_dset, elems * 4) && grow(c->pp_dcnt, ((size_t)kPPDLists + kPPDRegions + nfine) * 8)) {
      c->sp.dset = (uint32_t*)c->pp_dset.p;
      c->sp.dcnt = (unsigned long long*)c->pp_dcnt.p;
      c->sp.dcap = dcap;
      c->sp.ccap = ccap;
      c->sp.fcap = fcap;
    } else {
      (void)hipGetLastError();  // atomics
    }
  }
  if (c->failed && s.stride <= 8) {  // the dense rounds read fmask instead of gathering failed words
    if (c->fm_tver != c->table_ver || c->fm_fver != c->fail_ver) {
      if (!grow(c->pp_fmask, fmask_bytes(n))) {
        (void)hipGetLastError();
        return GS_OK;
      }
      CK(c, pp_fmask_build(s, c->sp.rend, c->sp.rsrc, c->sp.rslot, (uint8_t*)c->pp_fmask.p, c->stream));
      CK(c, pp_fmask_any((const uint8_t*)c->pp_fmask.p, n, fmask_any(c), c->stream));
      // (optional: without it the answer test gathers the caller's failed word)
      if (grow(c->pp_rfail, ((n * s.stride + 31) >> 5) * 4 + 8))  // + the hub flag word
        CK(c, pp_rfail_build(s, c->sp.rend, c->sp.rsrc, c->sp.rslot, (uint32_t*)c->pp_rfail.p, c->stream));
      else
        (void)hipGetLastError();
      c->fm_tver = c->table_ver;
      c->fm_fver = c->fail_ver;
      built = true;
    }
    c->sp.fmask = (const uint8_t*)c->pp_fmask.p;
    c->sp.fany = fmask_any(c);
    c->sp.rfail = c->pp_rfail.p && !getenv("GS_PP_NORFAIL") ? (const uint32_t*)c->pp_rfail.p : nullptr;
  }
  if (built) {
    CK(c, hipStreamSynchronize(c->stream));
    c->timing.prep_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  return GS_OK;
}

// Early rounds while |I| <= n >> shift (GS_PP_SHIFT, default 8, for tuning).
uint32_t pp_shift() {
  const char* e = getenv("GS_PP_SHIFT");
  const int v = e ? atoi(e) : 8;
  return (uint32_t)std::min(std::max(v, 0), 63);
}

// Dense rounds run bottom-up once |I| >= n * GS_PP_BOTTOM256 / 256 (default
// 96), when the reverse table has packed slots and the failed mask (if any)
// has fmask.
unsigned long long pp_bottom_thr(const gs_ctx* c) {
  const bool can = c->sp.ctl && pp_rslot_packed(c->st.stride) && (!c->failed || c->sp.fmask);
  if (!can || (c->p.flags & GS_FLAG_PP_TOPDOWN)) return ~0ull;
  if (c->p.flags & GS_FLAG_PP_BOTTOM) return 0;
  const char* e = getenv("GS_PP_BOTTOM256");
  const unsigned long long k = (unsigned long long)std::min(std::max(e ? atoi(e) : 96, 0), 256);
  return k == 256 ? ~0ull : (unsigned long long)(((unsigned __int128)c->st.n * k) >> 8);
}

// ---- push-pull node-range shards (SURVEY.md 8(e)2 for config C5) -------------
// Every shard owns nodes [lo, hi): their rows (calls) and their in-edges
// (pushes they receive), and a replicated copy of the informed set by global
// id.  A round is bottom-up on the own nodes against the replicated set
// (k_ppb_round: same draws and counters as the unsharded rounds, so the union
// equals the unsharded run bit for bit); then the shards exchange their own
// informed words: events only between members that share a device's arrays,
// peer copies between devices, an all-gather between ranks.
int pp_exchange(gs_ctx* acc, const std::vector<gs_ctx*>& ms) {
  if (!acc->group) return x_all_gather(acc, acc->d_ig, acc->segw * 8);
  const bool multi = acc->gdevs.size() > 1;
  for (size_t i = 0; i < ms.size(); ++i) {
    CK(ms[i], hipSetDevice(ms[i]->dev));
    CK(ms[i], hipEventRecord(acc->gev_c[i], ms[i]->stream));
  }
  if (multi) {
    for (size_t d = 0; d < acc->gdevs.size(); ++d) {
      gs_ctx* L = nullptr;
      for (size_t i = 0; i < ms.size() && !L; ++i)
        if ((size_t)acc->gdev_of[i] == d) L = ms[i];
      CK(L, hipSetDevice(L->dev));
      for (size_t j = 0; j < ms.size(); ++j) {
        const size_t dj = (size_t)acc->gdev_of[j];
        if (dj == d) continue;
        CK(L, hipStreamWaitEvent(L->stream, acc->gev_c[j], 0));
        const size_t off = (size_t)ms[j]->rank * ms[j]->segw;
        CK(L, hipMemcpyPeerAsync(acc->gig[d] + off, L->dev, acc->gig[dj] + off, ms[j]->dev, ms[j]->segw * 8,
                                 L->stream));
      }
      CK(L, hipEventRecord(acc->gev_x[d], L->stream));
    }
  }
  for (size_t i = 0; i < ms.size(); ++i) {
    gs_ctx* m = ms[i];
    CK(m, hipSetDevice(m->dev));
    for (size_t j = 0; j < ms.size(); ++j)
      if (j != i && acc->gdev_of[j] == acc->gdev_of[i]) CK(m, hipStreamWaitEvent(m->stream, acc->gev_c[j], 0));
    if (multi) CK(m, hipStreamWaitEvent(m->stream, acc->gev_x[acc->gdev_of[i]], 0));
  }
  return GS_OK;
}

std::vector<gs_ctx*> shards_of(gs_ctx* c) { return c->group ? c->mem : std::vector<gs_ctx*>{c}; }

// The replicas of a push-pull shard group (one per device) or rank (one).
std::vector<gs_ctx*> replicas_of(gs_ctx* c) {
  std::vector<gs_ctx*> v;
  if (c->group) {
    for (gs_ctx* r : c->greps)
      if (r) v.push_back(r);
  } else if (c->rep) {
    v.push_back(c->rep);
  }
  return v;
}

// Members sharing a device share its informed set: no member may commit its
// round's new bits into it while another member's round still reads it.
int pp_barrier(gs_ctx* acc, const std::vector<gs_ctx*>& ms) {
  if (!acc->group) return GS_OK;
  for (size_t i = 0; i < ms.size(); ++i) {
    CK(ms[i], hipSetDevice(ms[i]->dev));
    CK(ms[i], hipEventRecord(acc->gev_c[i], ms[i]->stream));
  }
  for (size_t i = 0; i < ms.size(); ++i) {
    CK(ms[i], hipSetDevice(ms[i]->dev));
    for (size_t j = 0; j < ms.size(); ++j)
      if (j != i && acc->gdev_of[j] == acc->gdev_of[i])
        CK(ms[i], hipStreamWaitEvent(ms[i]->stream, acc->gev_c[j], 0));
  }
  return GS_OK;
}

uint32_t pp_shift();

// The unsharded engine's bottom-up threshold (pp_bottom_thr) for n nodes.
unsigned long long pp_bottom_thr_n(const gs_ctx* c, uint64_t n) {
  if (c->p.flags & GS_FLAG_PP_BOTTOM) return 0;
  const char* e = getenv("GS_PP_BOTTOM256");
  const unsigned long long k = (unsigned long long)std::min(std::max(e ? atoi(e) : 96, 0), 256);
  return k == 256 ? ~0ull : (unsigned long long)(((unsigned __int128)n * k) >> 8);
}

// A rank's pull-answer round set bits in other ranks' ranges of its d_gn:
// slice p goes to rank p (all-to-all), and the slices this rank receives are
// ORed into its own slice before the commit.
int pp_answer_exchange(gs_ctx* c) {
  const uint32_t G = c->G, me = c->rank;
  const uint64_t sw = c->segw;
  unsigned long long* own = c->d_gn + (size_t)me * sw;
  if (c->comm) {
    const Rccl& r = rccl();
    NCK(c, r.group_start());
    for (uint32_t p = 0; p < G; ++p) {
      if (p == me) continue;
      NCK(c, r.send(c->d_gn + (size_t)p * sw, sw, ncclUint64, (int)p, c->comm, c->stream));
      NCK(c, r.recv(c->d_gst + (size_t)p * sw, sw, ncclUint64, (int)p, c->comm, c->stream));
    }
    NCK(c, r.group_end());
  } else {
    if (!grow_pinned(c, (size_t)2 * G * sw * 8)) return fail(c, GS_ENOMEM, "cannot allocate exchange staging");
    char* hs = c->h_xbuf;
    char* hr = c->h_xbuf + (size_t)G * sw * 8;
    std::vector<size_t> sb(G, sw * 8), rb(G, sw * 8);
    sb[me] = rb[me] = 0;
    // send blocks back to back in rank order without this rank's own slice
    size_t at = 0;
    for (uint32_t p = 0; p < G; ++p)
      if (p != me) {
        CK(c, hipMemcpyAsync(hs + at, c->d_gn + (size_t)p * sw, sw * 8, hipMemcpyDeviceToHost, c->stream));
        at += sw * 8;
      }
    CK(c, hipStreamSynchronize(c->stream));
    if (c->hx.all_to_allv(c->hx.user, hs, sb.data(), hr, rb.data()))
      return fail(c, GS_EDEVICE, "the exchange's all_to_allv callback failed");
    at = 0;
    for (uint32_t p = 0; p < G; ++p)
      if (p != me) {
        CK(c, hipMemcpyAsync(c->d_gst + (size_t)p * sw, hr + at, sw * 8, hipMemcpyHostToDevice, c->stream));
        at += sw * 8;
      }
  }
  CK(c, pp_or_slices(own, c->d_gst, G, sw, c->stream));  // the own slot of d_gst stays zero
  return GS_OK;
}

// simulator.go:239-241 for the push-pull extension: the owner informs the
// sender (unless failed), every shard resets its round control; the replicas
// (if any) start the broadcast's sparse early rounds.
int pp_shard_begin(gs_ctx* acc, uint64_t sender) {
  std::vector<gs_ctx*> ms = shards_of(acc);
  unsigned long long informed = 0;
  acc->rep_live = false;
  acc->rep_rounds = 0;
  std::vector<gs_ctx*> reps = replicas_of(acc);
  bool sparse = !reps.empty();
  for (gs_ctx* r : reps) {
    CK(r, hipSetDevice(r->dev));
    if (int rc = pp_prepare(r)) return fail(acc, rc, r->err);
    if (!r->sp.ctl || !r->sp.ilist) sparse = false;  // no sparse-round buffers: the shards run every round
  }
  if (sparse)
    for (gs_ctx* r : reps) {
      CK(r, hipSetDevice(r->dev));
      CK(r, hipMemsetAsync(r->d_next, 0, r->st.W * 8, r->stream));
      RC(pp_seed_ctx(r, r->d_next, (uint32_t)sender, r->st.n >> pp_shift(), ~0ull, ~0ull));
    }
  acc->rep_live = sparse;
  acc->pp_gn_ok = false;
  // pull-answer sharded rounds: between ranks (their bits in other ranks' ranges
  // move by an all-to-all) or among the shards of one device (one shared set);
  // shards over several devices of one group run bottom-up only
  const bool onedev = !acc->group || acc->gdevs.size() == 1;
  bool answer = onedev && !getenv("GS_PP_SHARD_BOTTOM") && (!acc->has_hx || acc->hx.all_to_allv);
  for (gs_ctx* m : ms) answer = answer && m->d_gn && (!m->failed || m->sp.fmask);
  acc->pp_answer = answer;
  for (gs_ctx* m : ms) {
    CK(m, hipSetDevice(m->dev));
    if (int rc = pp_prepare(m)) return fail(acc, rc, m->err);
    const uint32_t node = sender >= m->lo && sender < m->hi ? (uint32_t)(sender - m->lo) : ~0u;
    RC(pp_seed_ctx(m, m->d_next, node, 0ull, 0ull, ~0ull));
    uint32_t ok = 0;
    CK(m, hipMemcpyAsync(&ok, m->d_flag, 4, hipMemcpyDeviceToHost, m->stream));
    CK(m, hipStreamSynchronize(m->stream));
    informed += ok;
    reset_counters(m);
    m->begun = true;
  }
  if (!acc->group) {  // every rank learns whether the owner informed the sender
    unsigned long long* d = acc->d_gcounts;
    CK(acc, hipMemcpyAsync(d, &informed, 8, hipMemcpyHostToDevice, acc->stream));
    if (int rc = x_all_reduce(acc, d, 1)) return abort_rank(acc, rc);
    CK(acc, hipMemcpyAsync(&informed, d, 8, hipMemcpyDeviceToHost, acc->stream));
    CK(acc, hipStreamSynchronize(acc->stream));
  }
  if (int rc = pp_exchange(acc, ms)) return abort_rank(acc, rc);
  acc->recv = acc->pending = informed;
  acc->begun = true;
  return GS_OK;
}

void account_tick(gs_ctx* c, uint64_t tick, const unsigned long long* s, gs_tick_stats* o);

int pp_shard_step(gs_ctx* acc, uint32_t ticks, gs_tick_stats* out) {
  std::vector<gs_ctx*> ms = shards_of(acc);
  std::vector<gs_ctx*> reps = replicas_of(acc);
  std::vector<unsigned long long> sum(kStatFields);
  uint32_t done = 0;
  while (done < ticks) {
    const uint32_t batch = std::min<uint32_t>(ticks - done, kStatSlots);
    const uint64_t t0 = acc->t + 1;
    const uint32_t i0 = (uint32_t)(t0 % kStatSlots);
    const uint32_t first = std::min<uint32_t>(batch, kStatSlots - i0);
    for (gs_ctx* m : ms) {
      CK(m, hipSetDevice(m->dev));
      CK(m, hipMemsetAsync(m->st.stats + (size_t)i0 * kStatFields, 0, (size_t)first * kStatFields * 8, m->stream));
      if (first < batch)
        CK(m, hipMemsetAsync(m->st.stats, 0, (size_t)(batch - first) * kStatFields * 8, m->stream));
    }
    for (gs_ctx* r : reps) {
      CK(r, hipSetDevice(r->dev));
      CK(r, hipMemsetAsync(r->st.stats + (size_t)i0 * kStatFields, 0, (size_t)first * kStatFields * 8, r->stream));
      if (first < batch)
        CK(r, hipMemsetAsync(r->st.stats, 0, (size_t)(batch - first) * kStatFields * 8, r->stream));
    }
    for (uint32_t i = 0; i < batch; ++i) {
      const uint32_t tt = (uint32_t)(t0 + i);
      if (acc->rep_live) {
        // is this round a sparse early round on the replicas (k_pp_mode's test)?
        gs_ctx* r0 = reps[0];
        PPCtl h;
        CK(r0, hipSetDevice(r0->dev));
        CK(r0, hipMemcpyAsync(&h, r0->sp.ctl, offsetof(PPCtl, segcnt), hipMemcpyDeviceToHost, r0->stream));
        CK(r0, hipStreamSynchronize(r0->stream));
        if (h.early_ok && !h.ovf && h.ninf <= h.thr) {
          // every replica runs the same round: the replicated sets stay equal with no exchange
          for (gs_ctx* r : reps) {
            CK(r, hipSetDevice(r->dev));
            CK(r, pp_round(r->st, r->d_next, r->d_ppsum, tt, r->pp_l2_only, r->sp, r->stream));
            CK(r, pp_commit(r->st, r->d_next, tt, r->sp, r->stream));
          }
          for (gs_ctx* r : reps) {
            CK(r, hipSetDevice(r->dev));
            CK(r, hipStreamSynchronize(r->stream));
          }
          // the round's counters, once: the group's first member / rank 0
          if (acc->group || acc->rank == 0) {
            const size_t row = (size_t)(tt % kStatSlots) * kStatFields;
            CK(ms[0], hipSetDevice(ms[0]->dev));
            CK(ms[0], hipMemcpyAsync(ms[0]->st.stats + row, r0->st.stats + row, kStatFields * 8,
                                     hipMemcpyDeviceToDevice, ms[0]->stream));
          }
          ++acc->rep_rounds;
          continue;
        }
        acc->rep_live = false;  // the shards take over
      }
      if (!acc->pp_gn_ok) {  // the round's set starts as the replicated set (per device / rank)
        std::vector<int> done(acc->group ? acc->gdevs.size() : 1, 0);
        for (size_t i = 0; i < ms.size(); ++i) {
          gs_ctx* m = ms[i];
          const int d = acc->group ? acc->gdev_of[i] : 0;
          if (done[d]) continue;
          done[d] = 1;
          CK(m, hipSetDevice(m->dev));
          CK(m, hipMemcpyAsync(m->d_gn, m->d_ig, (size_t)m->G * m->segw * 8, hipMemcpyDeviceToDevice, m->stream));
        }
        RC(pp_barrier(acc, ms));
        acc->pp_gn_ok = true;
      }
      uint32_t mode = PP_BOTTOM;
      if (acc->pp_answer) {  // pull-answer until |I| >= the unsharded engine's bottom-up threshold
        gs_ctx* m0 = ms[0];  // every shard's copy of the replicated set is the same
        unsigned long long* cnt = (unsigned long long*)(m0->d_err + 4);
        unsigned long long ninf = 0;
        CK(m0, hipSetDevice(m0->dev));
        CK(m0, pp_count(m0->d_ig, (uint64_t)m0->G * m0->segw, cnt, m0->stream));
        CK(m0, hipMemcpyAsync(&ninf, cnt, 8, hipMemcpyDeviceToHost, m0->stream));
        CK(m0, hipStreamSynchronize(m0->stream));
        if (ninf >= pp_bottom_thr_n(acc, acc->p.n)) acc->pp_answer = false;
        else mode = PP_ANSWER;
      }
      for (gs_ctx* m : ms) {
        CK(m, hipSetDevice(m->dev));
        CK(m, pp_round_shard(m->st, m->d_gn + (size_t)m->rank * m->segw, m->d_gn, tt, m->sp, mode, m->stream));
      }
      RC(pp_barrier(acc, ms));
      if (mode == PP_ANSWER && !acc->group)  // the bits this rank set in other ranks' ranges go to their owners
        if (int rc = pp_answer_exchange(acc)) return abort_rank(acc, rc);
      for (gs_ctx* m : ms) {
        CK(m, hipSetDevice(m->dev));
        CK(m, pp_commit(m->st, m->d_gn + (size_t)m->rank * m->segw, tt, m->sp, m->stream));
      }
      if (int rc = pp_exchange(acc, ms)) return abort_rank(acc, rc);
    }
    for (gs_ctx* m : ms) {
      CK(m, hipSetDevice(m->dev));
      unsigned long long* a = m->st.stats + (size_t)i0 * kStatFields;
      if (is_rank(m)) {  // the global per-round counters on every rank
        if (int rc = x_all_reduce(m, a, (size_t)first * kStatFields)) return abort_rank(m, rc);
        if (first < batch)
          if (int rc = x_all_reduce(m, m->st.stats, (size_t)(batch - first) * kStatFields)) return abort_rank(m, rc);
      }
      CK(m, hipMemcpyAsync(m->h_stats + (size_t)i0 * kStatFields, a, (size_t)first * kStatFields * 8,
                           hipMemcpyDeviceToHost, m->stream));
      if (first < batch)
        CK(m, hipMemcpyAsync(m->h_stats, m->st.stats, (size_t)(batch - first) * kStatFields * 8,
                             hipMemcpyDeviceToHost, m->stream));
    }
    for (gs_ctx* m : ms) {
      CK(m, hipSetDevice(m->dev));
      CK(m, hipStreamSynchronize(m->stream));
    }
    for (uint32_t i = 0; i < batch; ++i) {
      const size_t row = (size_t)((t0 + i) % kStatSlots) * kStatFields;
      for (uint32_t f = 0; f < kStatFields; ++f) {
        sum[f] = 0;
        for (gs_ctx* m : ms) sum[f] += m->h_stats[row + f];
      }
      account_tick(acc, t0 + i, sum.data(), out ? &out[done + i] : nullptr);
    }
    done += batch;
  }
  return GS_OK;
}

// Dense rounds below the bottom-up threshold run pull-answer (informed nodes
// answer the pulls among their in-edges) once |I| >= n * GS_PP_ANSWER256 / 256
// (default 0: every such round; 256 = never, the top-down rounds), when the
// reverse table has packed slots and the failed mask (if any) has fmask.
unsigned long long pp_answer_thr(const gs_ctx* c) {
  const bool can = c->sp.ctl && pp_rslot_packed(c->st.stride) && (!c->failed || c->sp.fmask);
  if (!can || (c->p.flags & GS_FLAG_PP_TOPDOWN)) return ~0ull;
  if (c->p.flags & GS_FLAG_PP_ANSWER) return 0;
  const char* e = getenv("GS_PP_ANSWER256");
  const unsigned long long k = (unsigned long long)std::min(std::max(e ? atoi(e) : 0, 0), 256);
  return k == 256 ? ~0ull : (unsigned long long)(((unsigned __int128)c->st.n * k) >> 8);
}

}  // namespace

extern "C" {

int gs_broadcast_begin(gs_ctx* c, int64_t sender) {
  if (!c) return GS_EINVAL;
  if (c->aborted) return fail(c, GS_EDEVICE, "this rank's exchange failed earlier; the run is over");
  if (!c->peers) return fail(c, GS_EINVAL, "load peers or build the overlay first");
  if (c->begun) return fail(c, GS_EINVAL, "broadcast already begun");
  if (sender >= 0 && (uint64_t)sender >= c->p.n) return fail(c, GS_EINVAL, "sender out of range");
  reset_counters(c);
  if (c->group && c->gtrials) {
    for (gs_ctx* m : c->mem)
      if (gs_broadcast_begin(m, sender)) return fail(c, GS_EINVAL, m->err);
    c->pending = c->trials;
    c->begun = true;
    return GS_OK;
  }
  const bool batched = c->trials > 1;
  const uint64_t s = sender >= 0 ? (uint64_t)sender : batched ? ~0ull : keyed_sender(c->group ? c->mem[0] : c);
  if (c->pp && (c->group || c->pp_shard)) return pp_shard_begin(c, s);
  if (c->pp) {  // push-pull: the sender is informed (unless failed)
    CK(c, hipSetDevice(c->dev));
    RC(pp_prepare(c));
    const uint64_t n = c->st.n;
    const unsigned long long thr = (c->p.flags & GS_FLAG_PP_EARLY) ? n : (n >> pp_shift());
    RC(pp_seed_ctx(c, c->d_next, (uint32_t)s, thr, pp_bottom_thr(c), pp_answer_thr(c)));
    uint32_t ok = 0;
    CK(c, hipMemcpyAsync(&ok, c->d_flag, 4, hipMemcpyDeviceToHost, c->stream));
    CK(c, hipStreamSynchronize(c->stream));
    c->recv = c->pending = ok;
    c->begun = true;
    return GS_OK;
  }
  uint64_t scheduled = 0;
  if (c->group) {
    for (gs_ctx* m : c->mem) {
      reset_counters(m);
      uint32_t k = 0;
      if (int rc = begin_one(m, s, &k)) return fail(c, rc, m->err);
      scheduled += k;
      m->begun = true;
    }
  } else {
    uint32_t k = 0;
    RC(begin_one(c, s, &k));
    scheduled = k;
    if (is_rank(c)) {  // every rank learns whether the owner scheduled the sender
      unsigned long long* d = c->d_gcounts;  // scratch
      unsigned long long h = scheduled;
      CK(c, hipMemcpyAsync(d, &h, 8, hipMemcpyHostToDevice, c->stream));
      if (int rc = x_all_reduce(c, d, 1)) return abort_rank(c, rc);
      CK(c, hipMemcpyAsync(&h, d, 8, hipMemcpyDeviceToHost, c->stream));
      CK(c, hipStreamSynchronize(c->stream));
      scheduled = h;
    }
  }
  c->pending = scheduled;
  for (TrialAcc& a : c->tacc) a.sched = 0;
  c->begun = true;
  return GS_OK;
}

int gs_set_stream(gs_ctx* c, void* hip_stream) {
  if (!c) return GS_EINVAL;
  if (c->group || is_rank(c)) return fail(c, GS_EINVAL, "multi-device contexts keep their own streams");
  CK(c, hipSetDevice(c->dev));
  CK(c, hipStreamSynchronize(c->stream));
  c->stream = hip_stream ? (hipStream_t)hip_stream : c->own;
  return GS_OK;
}

int gs_memory_stats(gs_timing* out) {
  if (!out) return GS_EINVAL;
  *out = gs_timing{};
  fill_devmem(out);
  return GS_OK;
}

int gs_trim(int device, size_t* released) {
  const size_t b = gs_devmem_trim(device);
  if (released) *released = b;
  return GS_OK;
}

}  // extern "C"

namespace {

// Window engine: ticks [t0, t0 + n) as windows of <= min(max(delaylow,1),10)
// ticks (gs_window.hip).  One host sync per window reads its task count.
int run_windows(gs_ctx* c, uint64_t t0, uint32_t n, bool timing, uint64_t tchunk) {
  RC(expand_view(c));
  WinState& w = c->ws;
  const uint32_t Lmax = std::min<uint32_t>(std::max<int32_t>(c->p.delay_low, 1), kBitTicks);
  uint32_t done = 0, widx = 0;
  std::vector<std::pair<uint32_t, uint32_t>> evs;
  // Receipts per fine bucket are ~density * 16384 whatever N is; a window whose
  // slots would overflow k_resolve's LDS message buffer on average is cut short.
  const uint64_t slot_budget = (uint64_t)w.nfine * kWinSlotsPerBucket;
  // batched trials: each coarse bin's first firing index comes back with the
  // window's fire counts (plan_coarse_trials)
  const bool trial_plan = c->trials > 1 && c->tlog <= kCoarseShift && !c->shard;
  while (done < n) {
    const uint32_t Lw = std::min(Lmax, n - done);
    const uint32_t t = (uint32_t)(t0 + done);
    w.tofs = (uint32_t)(t - tchunk);
    auto units = [&](uint32_t Lu) -> int {
      CK(c, hipMemsetAsync(w.tfires, 0, kMaxWindow * 8, c->stream));
      CK(c, win_units(w, t, Lu, c->stream));
      size_t need = 0;
      CK(c, win_scan_units(w, Lu, nullptr, need, c->stream));
      if (!grow(c->tmp, need)) return fail(c, GS_ENOMEM, "cannot allocate scan scratch");
      need = c->tmp.bytes;
      CK(c, win_scan_units(w, Lu, c->tmp.p, need, c->stream));
      CK(c, hipMemcpyAsync(c->h_misc, w.tfires, kMaxWindow * 8, hipMemcpyDeviceToHost, c->stream));
      if (trial_plan)
        CK(c, hipMemcpy2DAsync(c->h_misc + kMaxWindow, 8, w.unit_off, (size_t)256 * Lu * 8, 8, w.ncoarse,
                               hipMemcpyDeviceToHost, c->stream));
      CK(c, hipStreamSynchronize(c->stream));
      return GS_OK;
    };
    RC(units(Lw));
    // fires per tick -> the window's length under the slot budget
    uint32_t L = 1;
    unsigned long long Tn = c->h_misc[0];  // broadcasts firing in the window
    while (L < Lw && (Tn + c->h_misc[L]) * w.stride <= slot_budget) Tn += c->h_misc[L++];
    // units are bucket-major: a cut window is laid out again for its L ticks
    if (L < Lw) RC(units(L));
    const unsigned long long T = Tn * w.stride;  // friend slots of the firing nodes
    if (trial_plan && Tn) {
      // batched trials: exact per-(bin, XCD) bounds from the bins' first firing
      // indices (unit_off at every 256 * L-th unit, copied by units())
      std::vector<unsigned long long> fb(c->h_misc + kMaxWindow, c->h_misc + kMaxWindow + w.ncoarse);
      fb.push_back(Tn);
      plan_coarse_trials(c, fb.data(), Tn);
    } else {
      plan_coarse(c, T, nullptr);
    }
    const uint64_t fcap = T + T / 8 + (uint64_t)w.ncoarse * 256 * 513 + 16;
    if (!grow(c->gmap, ((Tn + 63) / 64 + 1) * 4) || !grow(c->cmsg, (c->h_cap[kRegions] + 16) * 4) ||
        !grow(c->fmsg, (fcap + 16) * 4))  // buf_cap(fmsg) >= fcap (the device-driven windows' bound)
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
      CK(c, hipMemcpyAsync(w.ccap, c->h_cap, (kRegions + 1) * 8, hipMemcpyHostToDevice, c->stream));
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
        ++c->timing.coarse_redos;
        CK(c, hipMemsetAsync(w.chist, 0, kRegions * 8, c->stream));
        CK(c, win_expand(w, t, L, Tn, 0, c->stream));
        CK(c, hipMemcpyAsync(c->h_misc, w.chist, kRegions * 8, hipMemcpyDeviceToHost, c->stream));
        CK(c, hipStreamSynchronize(c->stream));
        plan_coarse(c, T, c->h_misc);
        CK(c, hipMemcpyAsync(w.ccap, c->h_cap, (kRegions + 1) * 8, hipMemcpyHostToDevice, c->stream));
        CK(c, hipMemsetAsync(w.cfill, 0, kRegions * 8, c->stream));
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

// ---- device-driven windows ----------------------------------------------------
// The unsharded one-trial window engine runs gs_step / gs_run without a host
// round trip per window: k_cut makes the window cut and coarse plan on the
// device, k_close applies gs_run's poll rule there, every kernel reads the
// window from ctl, and the host enqueues window i before it reads window
// i-1's results (staging slot + event), so the GPU never waits on it.  A
// partition overflow (skewed targets, or a message buffer too small) makes
// every later kernel a no-op; the host then finishes with run_windows, which
// redoes that window exactly and grows the buffers.
constexpr uint32_t kSlots = 4;

bool async_ok(const gs_ctx* c) {
  return c->win && !c->pp && !c->shard && !c->group && c->trials == 1 && !c->async_off &&
         !(c->p.flags & GS_FLAG_TIMING);
}

uint64_t cover_threshold(uint64_t n) {  // smallest r with covered(r, n)
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) / 2;
    if (covered(mid, n)) hi = mid; else lo = mid + 1;
  }
  return lo;
}

int async_setup(gs_ctx* c) {
  if (!c->d_ctl) {
    CK(c, dev_malloc(&c->d_ctl, sizeof(WinCtl)));
    // k_close writes each window's results straight into pinned host memory
    // (no copy launch per window); d_stage is its device address
    CK(c, hipHostMalloc((void**)&c->h_stage, (size_t)kSlots * kStageWords * 8,
                        hipHostMallocMapped | hipHostMallocPortable));
    CK(c, hipHostGetDevicePointer((void**)&c->d_stage, c->h_stage, 0));
    for (uint32_t i = 0; i < kSlots; ++i) {
      hipEvent_t e;
      CK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
      c->wev.push_back(e);
    }
  }
  // the message buffers keep the size the windows so far needed: a window
  // that needs more is flagged and redone host-driven, which grows them
  if (!grow(c->gmap, ((c->ntot + 1 + 63) / 64 + 1) * 4) || !grow(c->cmsg, 64) || !grow(c->fmsg, 64))
    return fail(c, GS_ENOMEM, "cannot allocate the window message buffers");
  return GS_OK;
}

// Ticks c->t+1 .. tend-1, or (poll > 0) until gs_run's rule stops the run at a
// poll.  on_tick(tick, row) sees every tick's counters in order.  *stop gets
// 1 + GS_RUN_* if a poll stopped the run; *fallback = true if a window
// overflowed (the caller continues host-driven from c->t).
template <class OnTick>
int run_async(gs_ctx* c, uint64_t tend, uint32_t poll, uint64_t max_ticks, OnTick on_tick, uint32_t* stop,
              bool* fallback) {
  *stop = 0;
  *fallback = false;
  RC(async_setup(c));
  RC(expand_view(c));
  WinState w = c->ws;
  w.ctl = c->d_ctl;
  w.stage = c->d_stage;
  w.lstride = std::min<uint32_t>(std::max<int32_t>(c->p.delay_low, 1), kBitTicks);
  w.gmap = (uint32_t*)c->gmap.p;
  w.cmsg = (uint32_t*)c->cmsg.p;
  w.fmsg = (uint32_t*)c->fmsg.p;
  WinCtl h{};
  h.tnext = (uint32_t)(c->t + 1);
  h.tend = (uint32_t)std::min<uint64_t>(tend, 0xFFFFFFFFull);
  h.poll = poll;
  h.pbase = (uint32_t)c->t;
  h.lmax = w.lstride;
  h.recv = c->recv;
  h.crashed = c->crashed;
  h.pending = c->pending;
  h.cover = cover_threshold(c->p.n);
  h.max_ticks = max_ticks;
  h.cmsg_cap = c->cmsg.bytes / 4 > 16 ? c->cmsg.bytes / 4 - 16 : 0;
  h.fmsg_cap = c->fmsg.bytes / 4 > 16 ? c->fmsg.bytes / 4 - 16 : 0;
  CK(c, hipMemcpyAsync(c->d_ctl, &h, sizeof h, hipMemcpyHostToDevice, c->stream));
  CK(c, hipMemsetAsync(w.tfires, 0, kMaxWindow * 8, c->stream));
  const uint64_t budget = (uint64_t)w.nfine * kWinSlotsPerBucket;
  // launch sizes: grid-stride kernels, sized for the dense windows
  const uint64_t Tn_bound = std::min<uint64_t>(c->ntot + 1, 4096ull * 1024),
                 T_bound = std::min<uint64_t>((c->ntot + 1) * w.stride, 2048ull * 16384);
  auto enqueue = [&](uint32_t slot) -> int {
    // units (+ tile sums) -> cut (+ tile offsets) -> unit scan and group map
    // inside the tiles; the rolled replay consumes the window's fire lists
    CK(c, win_units(w, 0, w.lstride, c->stream));
    CK(c, win_cut(w, budget, c->stream));
    CK(c, win_unitscan(w, c->stream));
    CK(c, win_expand(w, 0, w.lstride, Tn_bound, 1, c->stream));
    CK(c, win_plan(w, false, c->stream));
    CK(c, win_part2(w, T_bound, true, c->stream));
    CK(c, win_resolve(w, 0, w.lstride, c->stream));
    CK(c, win_close(w, slot, c->stream));
    CK(c, hipEventRecord(c->wev[slot], c->stream));
    return GS_OK;
  };
  // window i-1's results: 0 = go on, 1 = finished (the enqueued window i is a no-op)
  auto absorb = [&](uint32_t slot, int* what) -> int {
    CK(c, hipEventSynchronize(c->wev[slot]));
    const unsigned long long* st = c->h_stage + (size_t)slot * kStageWords;
    const uint32_t t0 = (uint32_t)st[0], L = (uint32_t)st[1];
    *what = 0;
    if (st[3] & (kErrCoarse | kErrFine)) {  // overflow: later windows did nothing
      *fallback = true;
      *what = 1;
      return GS_OK;
    }
    if (c->winlog) fprintf(stderr, "[win] t0=%u L=%u Tn=%llu stop=%llu\n", t0, L, st[4], st[2]);
    for (uint32_t k = 0; k < L; ++k) on_tick((uint64_t)t0 + k, st + 8 + (size_t)k * kStatFields);
    if (st[2]) *stop = (uint32_t)st[2];
    if (st[2] || L == 0 || (uint64_t)t0 + L >= tend) *what = 1;
    return GS_OK;
  };
  RC(enqueue(0));
  for (uint32_t i = 1;; ++i) {
    RC(enqueue(i % kSlots));
    int what = 0;
    RC(absorb((i - 1) % kSlots, &what));
    if (what) break;
  }
  CK(c, hipStreamSynchronize(c->stream));
  if (*fallback) {  // undo what the failed window left: its partial counters and flags
    uint32_t e = 0;
    CK(c, hipMemcpy(&e, c->d_err, 4, hipMemcpyDeviceToHost));
    e &= ~(kErrCoarse | kErrFine);
    CK(c, hipMemcpy(c->d_err, &e, 4, hipMemcpyHostToDevice));
    CK(c, hipMemsetAsync(c->ws.sstats, 0, (size_t)kStatShards * kMaxWindow * kStatFields * 8, c->stream));
    CK(c, hipMemsetAsync(c->ws.tfires, 0, kMaxWindow * 8, c->stream));
    CK(c, hipStreamSynchronize(c->stream));
  }
  uint32_t err = 0;
  CK(c, hipMemcpy(&err, c->d_err, 4, hipMemcpyDeviceToHost));
  if (err & kErrArrivals) return fail(c, GS_EOVERFLOW, "too many arrivals at one node in one tick");
  return GS_OK;
}

// ---- node-range shards ------------------------------------------------------
// One window for shards `ms` (all shards of a group, or this rank's one shard
// with an exchange), SURVEY.md section 8(e)2 -- owner expand:
//   1. each shard counts its fires per tick; the counts are gathered, so every
//      shard cuts the same window (host sync 1);
//   2. each shard expands its OWN firing nodes (its own friend rows), binning
//      every kept message by the shard that owns its target;
//   3. the region fills and error words are gathered (host sync 2); a shard
//      whose size estimate overflowed redoes its expand with exact counts;
//   4. each shard packs the filled prefixes of its regions into one block per
//      destination, and the blocks move to their owners (device copies, RCCL
//      grouped send/recv, or the caller's all_to_allv);
//   5. each shard partitions and resolves the messages it received.
// Per shard, the expand reads 1/G of the window's rows and the resolve owns
// 1/G of the buckets, so the work per shard shrinks with G.
int sync_all(const std::vector<gs_ctx*>& ms) {
  for (gs_ctx* m : ms) {
    CK(m, hipSetDevice(m->dev));
    CK(m, hipStreamSynchronize(m->stream));
  }
  return GS_OK;
}

// A shard that cannot allocate a window buffer marks its error word
// (kErrNoMem) and keeps taking part in the window's collectives; every rank
// sees the mark at the next gather (counts, layouts, or the end-of-step
// check) and returns GS_ENOMEM there, so no rank waits on a peer that left.
int mark_nomem(gs_ctx* m, const std::string& what) {
  uint32_t e = 0;
  CK(m, hipMemcpyAsync(&e, m->d_err, 4, hipMemcpyDeviceToHost, m->stream));
  CK(m, hipStreamSynchronize(m->stream));
  e |= kErrNoMem;
  CK(m, hipMemcpyAsync(m->d_err, &e, 4, hipMemcpyHostToDevice, m->stream));
  CK(m, hipStreamSynchronize(m->stream));
  m->err = what;
  return GS_OK;
}

// Fire counts of the window's units and their scan; with gather, tfires
// (fires per tick, plus this shard's partition-overflow flag in slot 15) is
// gathered: every rank's into d_gcounts, or the member's into its h_misc.
constexpr uint32_t kFlagSlot = kMaxWindow - 1;
static_assert(kFlagSlot >= kBitTicks, "the flag slot is past the window's ticks");

int shard_units(gs_ctx* m, uint32_t t, uint32_t Lu, bool gather) {
  WinState& w = m->ws;
  CK(m, hipSetDevice(m->dev));
  CK(m, hipMemsetAsync(w.tfires, 0, kMaxWindow * 8, m->stream));
  CK(m, hipMemcpyAsync(w.tfires + kFlagSlot, m->d_err, 4, hipMemcpyDeviceToDevice, m->stream));
  CK(m, win_units(w, t, Lu, m->stream));
  size_t need = 0;
  CK(m, win_scan_units(w, Lu, nullptr, need, m->stream));
  if (!grow(m->tmp, need)) {
    RC(mark_nomem(m, "cannot allocate scan scratch"));
    CK(m, hipMemcpyAsync(w.tfires + kFlagSlot, m->d_err, 4, hipMemcpyDeviceToDevice, m->stream));
  } else {
    need = m->tmp.bytes;
    CK(m, win_scan_units(w, Lu, m->tmp.p, need, m->stream));
  }
  if (!gather) return GS_OK;
  if (is_rank(m)) {
    CK(m, hipMemcpyAsync(m->d_gcounts + (size_t)m->rank * kMaxWindow, w.tfires, kMaxWindow * 8,
                         hipMemcpyDeviceToDevice, m->stream));
    RC(x_all_gather(m, m->d_gcounts, kMaxWindow * 8));
    CK(m, hipMemcpyAsync(m->h_misc, m->d_gcounts, (size_t)m->G * kMaxWindow * 8, hipMemcpyDeviceToHost,
                         m->stream));
  } else {
    CK(m, hipMemcpyAsync(m->h_misc, w.tfires, kMaxWindow * 8, hipMemcpyDeviceToHost, m->stream));
  }
  return GS_OK;
}

// Serial shard pipelines (GS_SHARD_SERIAL=1, in-process shards): each shard's
// phases run alone on the device, so GS_FLAG_TIMING measures one shard's
// device time per window (bench.py's in-process scaling proxy).
bool shard_serial() { return getenv("GS_SHARD_SERIAL") != nullptr; }

// A shard window the host keeps until the next window's count sync has shown
// that no shard's receive-side partition overflowed.
struct ShardWin {
  uint32_t t = 0, L = 0;
  bool live = false;
};

// Coarse plan of shard c's outgoing messages (owner expand): bin b = d *
// obins + k holds the targets in chunk k (2^22 nodes) of shard d's range;
// each of its 8 sub-regions gets 1/8 of the chunk's node share of T plus 512,
// or exactly `exact[region]`.  Bins past G * obins and empty chunks get none.
void plan_coarse_owner(gs_ctx* c, uint64_t T, const unsigned long long* exact) {
  const WinState& w = c->ws;
  const uint64_t N = c->p.n;
  unsigned long long a = 0;
  for (uint32_t b = 0; b < 256; ++b) {
    const uint32_t d = b / w.obins, k = b % w.obins;
    uint64_t cnt = 0;
    if (d < w.G) {
      const uint64_t dlo = (uint64_t)d * c->seg_per, dhi = std::min<uint64_t>(dlo + c->seg_per, N);
      const uint64_t lo = dlo + ((uint64_t)k << kCoarseShift);
      const uint64_t hi = std::min<uint64_t>(dhi, lo + (1ull << kCoarseShift));
      cnt = hi > lo ? hi - lo : 0;
    }
    const double xr = (double)kXRoundNodes * w.slots;  // one expand round's slots (gs_internal.h)
    const unsigned long long sub =
        cnt ? (unsigned long long)(((double)T / kCoarseSub + xr) * (double)cnt / (double)N) + 512 : 0;
    for (uint32_t x = 0; x < kCoarseSub; ++x) {
      const uint32_t r = b * kCoarseSub + x;
      c->h_cap[r] = a;
      if (cnt) a += exact ? exact[r] : sub;
    }
  }
  c->h_cap[kRegions] = a;
}

int shard_events(gs_ctx* m, size_t k) {
  while (m->ev.size() < k) {
    hipEvent_t ev;
    CK(m, hipEventCreate(&ev));
    m->ev.push_back(ev);
  }
  return GS_OK;
}

// Step 2 on shard m: expand its Tn own fires of window [t, t + L).
int shard_expand(gs_ctx* m, uint32_t t, uint32_t L, uint64_t Tn, bool timing) {
  WinState& w = m->ws;
  CK(m, hipSetDevice(m->dev));
  plan_coarse_owner(m, Tn * w.slots, nullptr);
  if (!grow(m->cmsg, (m->h_cap[kRegions] + 16) * 4) || !grow(m->gmap, ((Tn + 63) / 64 + 1) * 4))
    return mark_nomem(m, "cannot allocate " + std::to_string(m->h_cap[kRegions]) + " window messages");
  w.cmsg = (uint32_t*)m->cmsg.p;
  w.gmap = (uint32_t*)m->gmap.p;
  w.tofs = 0;
  CK(m, hipMemcpyAsync(w.ccap, m->h_cap, (kRegions + 1) * 8, hipMemcpyHostToDevice, m->stream));
  CK(m, win_groupmap(w, L, m->stream));
  if (timing) {
    RC(shard_events(m, 7));
    CK(m, hipEventRecord(m->ev[0], m->stream));
  }
  CK(m, win_expand(w, t, L, Tn, 1, m->stream));
  if (timing) CK(m, hipEventRecord(m->ev[1], m->stream));
  return GS_OK;
}

// Step 3: lay[s * (kRegions + 1) + r] = shard s's fill of region r, and
// lay[s * (kRegions + 1) + kRegions] = its error word.
int gather_layouts(const std::vector<gs_ctx*>& ms, std::vector<unsigned long long>& lay) {
  gs_ctx* m0 = ms[0];
  const size_t K1 = kRegions + 1;
  lay.assign((size_t)m0->G * K1, 0);
  if (is_rank(m0)) {
    gs_ctx* m = m0;
    unsigned long long* mine = m->d_glay + (size_t)m->rank * K1;
    CK(m, hipMemcpyAsync(mine, m->ws.cfill, kRegions * 8, hipMemcpyDeviceToDevice, m->stream));
    CK(m, hipMemsetAsync(mine + kRegions, 0, 8, m->stream));
    CK(m, hipMemcpyAsync(mine + kRegions, m->d_err, 4, hipMemcpyDeviceToDevice, m->stream));
    RC(x_all_gather(m, m->d_glay, K1 * 8));
    CK(m, hipMemcpyAsync(m->h_glay, m->d_glay, (size_t)m->G * K1 * 8, hipMemcpyDeviceToHost, m->stream));
    CK(m, hipStreamSynchronize(m->stream));
    std::copy(m->h_glay, m->h_glay + (size_t)m->G * K1, lay.begin());
    return GS_OK;
  }
  for (gs_ctx* m : ms) {
    CK(m, hipSetDevice(m->dev));
    CK(m, hipMemcpyAsync(m->h_misc, m->ws.cfill, kRegions * 8, hipMemcpyDeviceToHost, m->stream));
    CK(m, hipMemcpyAsync(m->h_err, m->d_err, 4, hipMemcpyDeviceToHost, m->stream));
  }
  RC(sync_all(ms));
  for (gs_ctx* m : ms) {
    std::copy(m->h_misc, m->h_misc + kRegions, lay.begin() + (size_t)m->rank * K1);
    lay[(size_t)m->rank * K1 + kRegions] = *m->h_err;
  }
  return GS_OK;
}

// Clears the partition-overflow flags of m's error word (host round trip).
int clear_part_flags(gs_ctx* m) {
  uint32_t e = 0;
  CK(m, hipMemcpyAsync(&e, m->d_err, 4, hipMemcpyDeviceToHost, m->stream));
  CK(m, hipStreamSynchronize(m->stream));
  e &= ~(kErrCoarse | kErrFine);
  CK(m, hipMemcpyAsync(m->d_err, &e, 4, hipMemcpyHostToDevice, m->stream));
  return GS_OK;
}

// Shard m's expand overflowed a region estimate: count its messages per
// region, plan exactly and write them again (the stats were added by the
// first pass).  Rank-local.
int sender_redo(gs_ctx* m, uint32_t t, uint32_t L, uint64_t Tn) {
  WinState& w = m->ws;
  CK(m, hipSetDevice(m->dev));
  RC(clear_part_flags(m));
  CK(m, hipMemsetAsync(w.chist, 0, kRegions * 8, m->stream));
  CK(m, hipMemsetAsync(w.cfill, 0, kRegions * 8, m->stream));
  CK(m, win_expand(w, t, L, Tn, 0, m->stream));
  CK(m, hipMemcpyAsync(m->h_misc, w.chist, kRegions * 8, hipMemcpyDeviceToHost, m->stream));
  CK(m, hipStreamSynchronize(m->stream));
  plan_coarse_owner(m, Tn * w.slots, m->h_misc);
  if (!grow(m->cmsg, (m->h_cap[kRegions] + 16) * 4)) return mark_nomem(m, "cannot allocate the window messages");
  w.cmsg = (uint32_t*)m->cmsg.p;
  CK(m, hipMemcpyAsync(w.ccap, m->h_cap, (kRegions + 1) * 8, hipMemcpyHostToDevice, m->stream));
  CK(m, win_expand(w, t, L, Tn, 2, m->stream));
  ++m->timing.exact_redos;
  return GS_OK;
}

// A rank's local allocation result made collective: every rank returns
// GS_ENOMEM if any rank could not allocate (one u64 all-reduce).
int agree_ok(gs_ctx* m, bool ok, const char* what) {
  unsigned long long* d = m->d_gcounts + (size_t)m->G * kMaxWindow;  // scratch
  m->h_misc[8] = ok ? 0ull : 1ull;
  CK(m, hipMemcpyAsync(d, &m->h_misc[8], 8, hipMemcpyHostToDevice, m->stream));
  RC(x_all_reduce(m, d, 1));
  CK(m, hipMemcpyAsync(&m->h_misc[9], d, 8, hipMemcpyDeviceToHost, m->stream));
  CK(m, hipStreamSynchronize(m->stream));
  if (m->h_misc[9]) return fail(m, GS_ENOMEM, ok ? std::string("another rank: ") + what : std::string(what));
  return GS_OK;
}

// Step 4: moves every block to its owner and sets each shard's receive
// layout (m->wr, m->rtotal).  A block that stays on its device (in-process
// shards of one device; a rank's block to itself) is read in place from its
// sender's message buffer; the others are packed (filled prefixes back to
// back) and sent: peer copies between devices, RCCL grouped send / receive
// or the caller's all_to_allv between ranks.  Destination d's block of a
// sender is its regions [d * obins * 8, (d + 1) * obins * 8).
int shard_exchange(gs_ctx* acc, const std::vector<gs_ctx*>& ms, const std::vector<unsigned long long>& lay,
                   bool timing) {
  gs_ctx* m0 = ms[0];
  const uint32_t G = m0->G, B8 = m0->ws.obins * kCoarseSub, nreg = G * B8;
  const size_t K1 = kRegions + 1;
  const bool rank = is_rank(m0);
  // a group's members are its shards in rank order
  auto travels = [&](uint32_t s, uint32_t d) { return rank ? s != d : acc->gdev_of[s] != acc->gdev_of[d]; };
  // poff[s][r]: offset of region r in sender s's packed output (~0: stays in place);
  // blk[s][d]: messages of sender s for destination d
  std::vector<unsigned long long> poff((size_t)G * K1, ~0ull), blk((size_t)G * G, 0), ptot(G, 0);
  for (uint32_t s = 0; s < G; ++s) {
    unsigned long long a = 0;
    for (uint32_t r = 0; r < nreg; ++r) {
      const uint32_t d = r / B8;
      const unsigned long long f = lay[(size_t)s * K1 + r];
      blk[(size_t)s * G + d] += f;
      if (!travels(s, d)) continue;
      poff[(size_t)s * K1 + r] = a;
      a += f;
    }
    ptot[s] = a;
  }
  auto bstart = [&](uint32_t s, uint32_t d) { return poff[(size_t)s * K1 + (size_t)d * B8]; };
  auto bsize = [&](uint32_t s, uint32_t d) { return blk[(size_t)s * G + d]; };
  // where each receiver finds the blocks that travel to it: in[i][s]; pack destinations pout[i]
  std::vector<std::vector<unsigned long long>> in(ms.size(), std::vector<unsigned long long>(G, 0));
  std::vector<uint32_t*> inbuf(ms.size(), nullptr), pout(ms.size(), nullptr);
  if (rank) {
    gs_ctx* m = m0;
    const uint32_t me = m->rank;
    unsigned long long rsum = 0;
    for (uint32_t s = 0; s < G; ++s)
      if (s != me) { in[0][s] = rsum; rsum += bsize(s, me); }
    // every rank learns whether every rank has its buffers before any sends
    const bool ok = grow(m->xsend, (ptot[me] + 16) * 4) && grow(m->xrecv, (rsum + 16) * 4);
    RC(agree_ok(m, ok, "cannot allocate the exchange buffers"));
    inbuf[0] = (uint32_t*)m->xrecv.p;
    pout[0] = (uint32_t*)m->xsend.p;
  } else {
    // device D's buffer: its members' packed outputs, then the blocks its
    // members receive from members on other devices
    std::vector<unsigned long long> dtot(acc->gdevs.size(), 0), O(ms.size(), 0);
    for (size_t i = 0; i < ms.size(); ++i) {
      const int D = acc->gdev_of[i];
      O[i] = dtot[D];
      dtot[D] += ptot[i];
    }
    for (size_t i = 0; i < ms.size(); ++i)
      for (uint32_t s = 0; s < G; ++s)
        if (travels(s, (uint32_t)i)) {
          const int D = acc->gdev_of[i];
          in[i][s] = dtot[D];
          dtot[D] += bsize(s, (uint32_t)i);
        }
    for (size_t D = 0; D < acc->gdevs.size(); ++D) {
      if (!dtot[D]) continue;
      CK(acc, hipSetDevice(acc->gdevs[D]));
      if (!grow(acc->gbuf[D], (dtot[D] + 16) * 4)) return fail(acc, GS_ENOMEM, "cannot allocate the exchange buffers");
    }
    for (size_t i = 0; i < ms.size(); ++i) {
      inbuf[i] = (uint32_t*)acc->gbuf[acc->gdev_of[i]].p;
      pout[i] = inbuf[i] ? inbuf[i] + O[i] : nullptr;
    }
  }
  // receive layouts (region = bin * (G * 8) + sender * 8 + sub), pack offsets, sources
  for (size_t i = 0; i < ms.size(); ++i) {
    gs_ctx* m = ms[i];
    const uint32_t d = m->rank;
    unsigned long long* rcap = m->h_rtab;
    unsigned long long* rend = rcap + K1;
    unsigned long long* rfill = rend + K1;
    unsigned long long* mypoff = rfill + K1;
    const uint32_t** src = (const uint32_t**)(mypoff + K1);
    std::fill(m->h_rtab, m->h_rtab + kRtabWords, 0ull);
    // sources: rank: 0 = received blocks, 1 = own buffer; group: s = member s's buffer, G = received blocks
    const uint32_t in_src = rank ? 0u : G;
    if (rank) {
      src[0] = inbuf[i];
      src[1] = m->ws.cmsg;
    } else {
      for (uint32_t s = 0; s < G; ++s) src[s] = travels(s, d) ? nullptr : ms[s]->ws.cmsg;
      src[G] = inbuf[i];
    }
    unsigned long long tot = 0;
    for (uint32_t c = 0; c < m->ws.obins; ++c)
      for (uint32_t s = 0; s < G; ++s)
        for (uint32_t x = 0; x < kCoarseSub; ++x) {
          const size_t rr = ((size_t)c * G + s) * kCoarseSub + x, sr = (size_t)d * B8 + c * kCoarseSub + x;
          const unsigned long long f = lay[(size_t)s * K1 + sr];
          unsigned long long at;
          if (!travels(s, d))  // in place: the sender's own region start
            at = ((unsigned long long)(rank ? 1u : s) << kSrcShift) | (rank ? m : ms[s])->h_cap[sr];
          else
            at = ((unsigned long long)in_src << kSrcShift) | (in[i][s] + poff[(size_t)s * K1 + sr] - bstart(s, d));
          rcap[rr] = at;
          rend[rr] = at + f;
          rfill[rr] = f;
          tot += f;
        }
    std::copy(poff.begin() + (size_t)d * K1, poff.begin() + (size_t)(d + 1) * K1, mypoff);
    m->rtotal = tot;
    WinState& wr = m->wr;
    wr = m->ws;
    wr.cmsg = nullptr;
    wr.csrc = (const uint32_t* const*)(m->d_rtab + 4 * K1);
    wr.ccap = m->d_rtab;
    wr.ccap_end = m->d_rtab + K1;
    wr.cfill = m->d_rtab + 2 * K1;
    wr.csub = G * kCoarseSub;
    CK(m, hipSetDevice(m->dev));
    CK(m, hipMemcpyAsync(m->d_rtab, m->h_rtab, kRtabWords * 8, hipMemcpyHostToDevice, m->stream));
    if (timing) CK(m, hipEventRecord(m->ev[2], m->stream));
    if (ptot[d]) CK(m, win_pack(m->ws, m->d_rtab + 3 * K1, nreg, pout[i], m->stream));
    if (timing) CK(m, hipEventRecord(m->ev[3], m->stream));
    if (!rank) CK(m, hipEventRecord(acc->gev_c[i], m->stream));
    if (shard_serial() && !rank) CK(m, hipStreamSynchronize(m->stream));
  }
  if (rank) {
    gs_ctx* m = m0;
    const uint32_t me = m->rank;
    if (m->comm) {
      const Rccl& r = rccl();
      NCK(m, r.group_start());
      for (uint32_t p = 0; p < G; ++p) {
        if (p == me) continue;
        if (bsize(me, p))
          NCK(m, r.send(pout[0] + bstart(me, p), bsize(me, p), ncclUint32, (int)p, m->comm, m->stream));
        if (bsize(p, me))
          NCK(m, r.recv(inbuf[0] + in[0][p], bsize(p, me), ncclUint32, (int)p, m->comm, m->stream));
      }
      NCK(m, r.group_end());
    } else {
      unsigned long long rsum = 0;
      std::vector<size_t> sb(G, 0), rb(G, 0);
      for (uint32_t p = 0; p < G; ++p)
        if (p != me) {
          sb[p] = bsize(me, p) * 4;
          rb[p] = bsize(p, me) * 4;
          rsum += bsize(p, me);
        }
      RC(agree_ok(m, grow_pinned(m, (ptot[me] + rsum) * 4 + 16), "cannot allocate exchange staging"));
      char* hs = m->h_xbuf;
      char* hr = m->h_xbuf + ptot[me] * 4;
      CK(m, hipMemcpyAsync(hs, pout[0], ptot[me] * 4, hipMemcpyDeviceToHost, m->stream));
      CK(m, hipStreamSynchronize(m->stream));
      if (m->hx.all_to_allv(m->hx.user, hs, sb.data(), hr, rb.data()))
        return fail(m, GS_EDEVICE, "the exchange's all_to_allv callback failed");
      CK(m, hipMemcpyAsync(inbuf[0], hr, rsum * 4, hipMemcpyHostToDevice, m->stream));
      CK(m, hipStreamSynchronize(m->stream));
    }
    return GS_OK;
  }
  // group: blocks from other devices are copied in once their senders packed
  // them (blocks on the same device were complete at the layout sync)
  for (size_t i = 0; i < ms.size(); ++i) {
    gs_ctx* m = ms[i];
    CK(m, hipSetDevice(m->dev));
    for (uint32_t s = 0; s < G; ++s) {
      if (!travels(s, (uint32_t)i) || !bsize(s, (uint32_t)i)) continue;
      CK(m, hipStreamWaitEvent(m->stream, acc->gev_c[s], 0));
      CK(m, hipMemcpyPeerAsync(inbuf[i] + in[i][s], m->dev, pout[s] + bstart(s, (uint32_t)i), ms[s]->dev,
                               bsize(s, (uint32_t)i) * 4, m->stream));
    }
  }
  return GS_OK;
}

// Step 5 on shard m: partition and resolve the received messages.
int shard_receive(gs_ctx* m, const ShardWin& sw, bool timing) {
  WinState& wr = m->wr;
  CK(m, hipSetDevice(m->dev));
  const uint64_t R = m->rtotal;
  const uint64_t fcap = R + R / 8 + (uint64_t)wr.ncoarse * 256 * 513 + 16;
  // (+16: buf_cap's slack -- k_rtab checks the next device-driven window's
  // bound against buf_cap, so a buffer grown to exactly fcap aborted it)
  if (!grow(m->fmsg, (fcap + 16) * 4))  // nothing resolved: every rank stops at the next gather
    return mark_nomem(m, "cannot allocate " + std::to_string(R) + " received messages");
  wr.fmsg = m->ws.fmsg = (uint32_t*)m->fmsg.p;
  if (timing) CK(m, hipEventRecord(m->ev[4], m->stream));
  CK(m, win_plan(wr, false, m->stream));
  CK(m, win_part2(wr, R, true, m->stream));
  if (timing) CK(m, hipEventRecord(m->ev[5], m->stream));
  CK(m, win_resolve(wr, sw.t, sw.L, m->stream));
  CK(m, win_stats_reduce(wr, sw.t, sw.L, m->stream));
  if (timing) {
    CK(m, hipEventRecord(m->ev[6], m->stream));
    CK(m, hipStreamSynchronize(m->stream));
    float ex = 0, pk = 0, p2 = 0, rs = 0;
    CK(m, hipEventElapsedTime(&ex, m->ev[0], m->ev[1]));
    CK(m, hipEventElapsedTime(&pk, m->ev[2], m->ev[3]));
    CK(m, hipEventElapsedTime(&p2, m->ev[4], m->ev[5]));
    CK(m, hipEventElapsedTime(&rs, m->ev[5], m->ev[6]));
    m->timing.expand_ms += ex;
    m->timing.part_ms += pk + p2;
    m->timing.deliver_ms += ex + pk + p2;
    m->timing.resolve_ms += rs;
    m->timing.deliver_launches += 1;
    m->timing.resolve_launches += 1;
    m->timing.windows += 1;
  }
  return GS_OK;
}

// Shard m's receive-side partition of window sw overflowed: partition the
// received messages (still in place) again with exact counts and resolve.
int receiver_redo(gs_ctx* m, const ShardWin& sw) {
  WinState& wr = m->wr;
  CK(m, hipSetDevice(m->dev));
  RC(clear_part_flags(m));
  const uint64_t R = m->rtotal;
  CK(m, hipMemsetAsync(wr.ffill, 0, (size_t)wr.nfine * 8, m->stream));
  CK(m, hipMemsetAsync(wr.fhist, 0, ((size_t)wr.ncoarse * 256 + 1) * 8, m->stream));
  CK(m, win_plan(wr, true, m->stream));
  CK(m, win_part2(wr, R, false, m->stream));
  size_t need = 0;
  CK(m, win_scan_fine(wr, nullptr, need, m->stream));
  if (!grow(m->tmp, need)) return mark_nomem(m, "cannot allocate scan scratch");
  need = m->tmp.bytes;
  CK(m, win_scan_fine(wr, m->tmp.p, need, m->stream));
  CK(m, hipMemsetAsync(wr.ffill, 0, (size_t)wr.nfine * 8, m->stream));
  CK(m, win_part2(wr, R, true, m->stream));
  CK(m, win_resolve(wr, sw.t, sw.L, m->stream));
  CK(m, win_stats_reduce(wr, sw.t, sw.L, m->stream));
  ++m->timing.exact_redos;
  return GS_OK;
}

int shard_windows(gs_ctx* acc, const std::vector<gs_ctx*>& ms, uint64_t t0, uint32_t n, bool timing) {
  gs_ctx* m0 = ms[0];
  const uint32_t G = m0->G;
  const uint64_t N = m0->p.n;
  const uint32_t stride = m0->ws.stride;
  const uint32_t Lmax = std::min<uint32_t>(std::max<int32_t>(m0->p.delay_low, 1), kBitTicks);
  const uint64_t slot_budget = ((N + kFineNodes - 1) >> kFineLog) * (uint64_t)kWinSlotsPerBucket;
  const size_t K1 = kRegions + 1;
  std::vector<unsigned long long> cnt((size_t)G * kMaxWindow), lay;
  ShardWin prev;
  uint32_t done = 0;
  // 1. fire counts per tick (every shard's, gathered) and every shard's
  //    overflow flag of the previous window
  auto counts = [&](uint32_t t, uint32_t Lw) -> int {
    for (gs_ctx* m : ms) RC(shard_units(m, t, Lw, true));
    RC(sync_all(ms));
    for (uint32_t r = 0; r < G; ++r)
      for (uint32_t k = 0; k < kMaxWindow; ++k)
        cnt[(size_t)r * kMaxWindow + k] = is_rank(m0) ? m0->h_misc[(size_t)r * kMaxWindow + k] : ms[r]->h_misc[k];
    return GS_OK;
  };
  auto flagged = [&]() {
    for (uint32_t r = 0; r < G; ++r)
      if (cnt[(size_t)r * kMaxWindow + kFlagSlot] & (kErrCoarse | kErrFine)) return true;
    return false;
  };
  while (done < n) {
    const uint32_t Lw = std::min(Lmax, n - done);
    const uint32_t t = (uint32_t)(t0 + done);
    RC(counts(t, Lw));
    for (uint32_t r = 0; r < G; ++r)  // a shard could not allocate: every shard stops here
      if (cnt[(size_t)r * kMaxWindow + kFlagSlot] & kErrNoMem)
        return fail(acc, GS_ENOMEM, "shard " + std::to_string(r) + " could not allocate a window buffer");
    if (flagged()) {  // a shard's previous window overflowed its receive partition: it redoes it, then all count again
      for (uint32_t r = 0; r < G; ++r) {
        if (!(cnt[(size_t)r * kMaxWindow + kFlagSlot] & (kErrCoarse | kErrFine))) continue;
        for (gs_ctx* m : ms)
          if (m->rank == r) RC(receiver_redo(m, prev));
      }
      RC(counts(t, Lw));
    }
    auto F = [&](uint32_t k) {
      unsigned long long s = 0;
      for (uint32_t r = 0; r < G; ++r) s += cnt[(size_t)r * kMaxWindow + k];
      return s;
    };
    // the same cut on every shard (global counts), as the unsharded engine would
    uint32_t L = 1;
    unsigned long long Tn = F(0);
    while (L < Lw && (Tn + F(L)) * stride <= slot_budget) Tn += F(L++);
    if (L < Lw)
      for (gs_ctx* m : ms) RC(shard_units(m, t, L, false));
    std::vector<unsigned long long> own(G, 0);
    unsigned long long Ftot = 0;
    for (uint32_t r = 0; r < G; ++r) {
      for (uint32_t k = 0; k < L; ++k) own[r] += cnt[(size_t)r * kMaxWindow + k];
      Ftot += own[r];
    }
    ShardWin sw;
    sw.t = t;
    sw.L = L;
    sw.live = Ftot > 0;
    if (Ftot) {
      // 2. expand own fires
      for (gs_ctx* m : ms) {
        RC(shard_expand(m, t, L, own[m->rank], timing));
        if (shard_serial() && !is_rank(m)) CK(m, hipStreamSynchronize(m->stream));
      }
      // 3. fills and overflow flags; exact redo of an overflowed expand
      RC(gather_layouts(ms, lay));
      auto nomem = [&]() {
        for (uint32_t r = 0; r < G; ++r)
          if (lay[(size_t)r * K1 + kRegions] & kErrNoMem) return true;
        return false;
      };
      if (nomem()) return fail(acc, GS_ENOMEM, "a shard could not allocate its window messages");
      bool redo = false;
      for (uint32_t r = 0; r < G; ++r)
        if (lay[(size_t)r * K1 + kRegions] & kErrCoarse) {
          redo = true;
          for (gs_ctx* m : ms)
            if (m->rank == r) RC(sender_redo(m, t, L, own[r]));
        }
      if (redo) {
        RC(gather_layouts(ms, lay));
        if (nomem()) return fail(acc, GS_ENOMEM, "a shard could not allocate its window messages");
      }
      for (gs_ctx* m : ms) {
        CK(m, hipSetDevice(m->dev));
        CK(m, win_consume_sh(m->ws, t, L, m->stream));
      }
      // 4. pack and move the blocks; 5. partition and resolve what arrived
      RC(shard_exchange(acc, ms, lay, timing));
      for (gs_ctx* m : ms) {
        RC(shard_receive(m, sw, timing));
        if (shard_serial() && !is_rank(m)) CK(m, hipStreamSynchronize(m->stream));
      }
    } else {
      for (gs_ctx* m : ms) {
        CK(m, hipSetDevice(m->dev));
        CK(m, win_consume_sh(m->ws, t, L, m->stream));
      }
    }
    prev = sw;
    done += L;
  }
  // the last window's overflow check (rank-local: the redo needs no exchange)
  for (gs_ctx* m : ms) {
    CK(m, hipSetDevice(m->dev));
    CK(m, hipMemcpyAsync(m->h_err, m->d_err, 4, hipMemcpyDeviceToHost, m->stream));
  }
  RC(sync_all(ms));
  for (gs_ctx* m : ms)
    if (*m->h_err & (kErrCoarse | kErrFine)) {
      RC(receiver_redo(m, prev));
      CK(m, hipMemcpyAsync(m->h_err, m->d_err, 4, hipMemcpyDeviceToHost, m->stream));
      CK(m, hipStreamSynchronize(m->stream));
    }
  // the errors no gather has carried yet (a receipt count overflow, a shard
  // that could not allocate its received messages): every rank returns the
  // same code at the same point (one u64 all-reduce per rank)
  unsigned long long bad = 0;
  for (gs_ctx* m : ms) bad |= *m->h_err & (kErrArrivals | kErrNoMem);
  if (is_rank(m0)) {
    unsigned long long* d = m0->d_gcounts + (size_t)G * kMaxWindow;  // scratch: [arrivals, nomem]
    m0->h_misc[8] = (bad & kErrArrivals) ? 1 : 0;
    m0->h_misc[9] = (bad & kErrNoMem) ? 1 : 0;
    CK(m0, hipMemcpyAsync(d, &m0->h_misc[8], 16, hipMemcpyHostToDevice, m0->stream));
    RC(x_all_reduce(m0, d, 2));
    CK(m0, hipMemcpyAsync(&m0->h_misc[10], d, 16, hipMemcpyDeviceToHost, m0->stream));
    CK(m0, hipStreamSynchronize(m0->stream));
    bad = (m0->h_misc[10] ? kErrArrivals : 0u) | (m0->h_misc[11] ? kErrNoMem : 0u);
  }
  if (bad & kErrNoMem) return fail(acc, GS_ENOMEM, "a shard could not allocate its received messages");
  if (bad & kErrArrivals) return fail(acc, GS_EOVERFLOW, "too many arrivals at one node in one tick");
  return GS_OK;
}

// Per-tick host bookkeeping shared by every flood/push-pull context: c's
// cumulative counters and (one trial) its TrialAcc.
void account_tick(gs_ctx* c, uint64_t tick, const unsigned long long* s, gs_tick_stats* o) {
  c->t = tick;
  c->fired += s[ST_FIRED];
  c->sent += s[ST_SENT];
  c->msgs += s[ST_MSGS];
  c->recv += s[ST_RECV];
  c->crashed += s[ST_CRASH];
  // push-pull: every informed node keeps calling
  c->pending = c->pp ? c->recv : c->pending + s[ST_SCHED] - s[ST_FIRED];
  if (c->tacc.size() == 1 && c->trials == 1) {
    TrialAcc& a = c->tacc[0];
    a.fired = c->fired; a.sent = c->sent; a.msgs = c->msgs; a.recv = c->recv; a.crash = c->crashed;
    if (!a.tick99 && covered(a.recv, c->p.n)) a.tick99 = tick;
  }
  if (o) *o = gs_tick_stats{c->t, s[ST_FIRED], s[ST_SENT], s[ST_MSGS], c->recv, c->crashed, c->pending};
}

// ---- device-driven shard windows -------------------
// The shards of one device (a group on one GPU, one stream) or one rank run
// their windows without a host round trip: every shard's fire counts and
// region fills are gathered into device buffers (the shards of a device share
// them; ranks all-gather them with RCCL), k_cut makes the same window cut on
// every shard, k_rtab lays out each shard's receive side, a fine-region
// overflow is re-partitioned exactly inside the window, and k_close_dd applies
// gs_run's poll rule to the global counters.  The host enqueues window i
// before it reads window i-1's staged counters.  A rank whose blocks travel
// to other ranks (G > 1) waits once per window: the grouped send / receive
// needs the block sizes on the host.  A window in which any shard overflowed
// a region estimate or its buffers is stopped on every shard before anything
// is consumed or resolved (kErrAbort), and the host redoes it host-driven.
bool dd_ok(const gs_ctx* acc, const std::vector<gs_ctx*>& ms) {
  if ((acc->p.flags & GS_FLAG_TIMING) || getenv("GS_SYNC_WINDOWS") || shard_serial()) return false;
  const gs_ctx* m0 = ms[0];
  if (m0->pp || !m0->win || !m0->shard) return false;
  if (acc->group) return !acc->gtrials && acc->gdevs.size() == 1;  // one device: one stream, blocks read in place
  return is_rank(acc);
}

// GS_WINLOG=1: one stderr line per device-driven shard window (and its aborts)
bool dd_log() {
  static const bool on = getenv("GS_WINLOG") != nullptr;
  return on;
}

int dd_setup(gs_ctx* acc, const std::vector<gs_ctx*>& ms) {
  gs_ctx* m0 = ms[0];
  const uint32_t G = m0->G, M = (uint32_t)ms.size();
  CK(acc, hipSetDevice(m0->dev));
  if (!acc->dd_mem) {
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t b1 = al((size_t)G * kMaxWindow * 8), b2 = al((size_t)G * kDDRow * 8),
                 b3 = al((size_t)M * kDDWStat * 8), b4 = al((size_t)M * sizeof(WinCtl)),
                 b5 = al((size_t)(4 * M + 2) * sizeof(void*)), b6 = al((size_t)3 * M * sizeof(WinState));
    CK(acc, dev_malloc(&acc->dd_mem, b1 + b2 + b3 + b4 + b5 + b6));
    char* q = (char*)acc->dd_mem;
    acc->dd_gcnt = (unsigned long long*)q; q += b1;
    acc->dd_glay = (unsigned long long*)q; q += b2;
    acc->dd_wstat = (unsigned long long*)q; q += b3;
    acc->dd_ctl = (WinCtl*)q; q += b4;
    acc->dd_ptrs = (void**)q; q += b5;
    acc->dd_wsm = (WinState*)q;
    CK(acc, hipHostMalloc((void**)&acc->h_ddptrs, (size_t)(4 * M + 2) * sizeof(void*)));
    if (is_rank(acc) && G > 1) CK(acc, hipHostMalloc((void**)&acc->h_ddlay, (size_t)G * kDDRow * 8));
  }
  if (!acc->h_stage) {
    CK(acc, hipHostMalloc((void**)&acc->h_stage, (size_t)kSlots * kStageWords * 8,
                          hipHostMallocMapped | hipHostMallocPortable));
    CK(acc, hipHostGetDevicePointer((void**)&acc->d_stage, acc->h_stage, 0));
    for (uint32_t i = 0; i < kSlots; ++i) {
      hipEvent_t e;
      CK(acc, hipEventCreateWithFlags(&e, hipEventDisableTiming));
      acc->wev.push_back(e);
    }
  }
  return GS_OK;
}

// Elements a buffer holds for the window kernels (16 of slack, as run_async).
unsigned long long buf_cap(const Buf& b) { return b.bytes / 4 > 16 ? b.bytes / 4 - 16 : 0; }

// Windows from acc->t + 1 until tend (exclusive), or (poll > 0) until the poll
// rule stops the run; on_tick(tick, row) sees every tick's global counters in
// order; *stop = 1 + GS_RUN_* if the poll rule stopped the run; *fallback =
// true if a window was stopped by an overflow (nothing of it consumed or
// resolved: the caller redoes it and goes on host-driven from acc->t).
template <class OnTick>
int dd_run(gs_ctx* acc, const std::vector<gs_ctx*>& ms, uint64_t tend, uint32_t poll, uint64_t max_ticks,
           OnTick on_tick, uint32_t* stop, bool* fallback) {
  *stop = 0;
  *fallback = false;
  RC(dd_setup(acc, ms));
  gs_ctx* m0 = ms[0];
  const uint32_t G = m0->G, M = (uint32_t)ms.size();
  const bool rank = is_rank(m0), travel = rank && G > 1;
  // one in-process shard: its send layout is its receive layout, so the
  // window runs as the unsharded engine's does (no k_rtab, overflows stop the
  // window) -- the G = 1 case of bench.py's sharded flood
  const bool solo = !rank && G == 1 && M == 1;
  const size_t K1 = kRegions + 1;
  hipStream_t st = m0->stream;
  CK(acc, hipSetDevice(m0->dev));
  // the members' own streams (begin, reset, the packed row view) are done
  // before their windows run on m0's stream
  for (gs_ctx* m : ms)
    if (m != m0) CK(acc, hipStreamSynchronize(m->stream));
  const uint32_t Lmax = std::min<uint32_t>(std::max<int32_t>(m0->p.delay_low, 1), kBitTicks);
  const uint64_t N = m0->p.n;
  const unsigned long long budget = ((N + kFineNodes - 1) >> kFineLog) * (unsigned long long)kWinSlotsPerBucket;
  const uint32_t B8 = m0->ws.obins * kCoarseSub, nreg = G * B8;
  // the message buffers keep the size the windows so far needed (an overflow
  // is redone host-driven, which grows them); the group map holds every fire
  bool ok = true;
  for (gs_ctx* m : ms)
    ok = ok && grow(m->gmap, ((m->ntot + 1 + 63) / 64 + 1) * 4) && grow(m->cmsg, 64) && grow(m->fmsg, 64);
  if (rank) RC(agree_ok(m0, ok, "cannot allocate the window message buffers"));
  else if (!ok) return fail(acc, GS_ENOMEM, "cannot allocate the window message buffers");
  // pointer tables: region starts (k_rtab's in-place regions), the receive
  // layout's sources, the members' counters and control blocks
  void** hp = acc->h_ddptrs;
  const uint32_t nsrc = rank ? 2u : M + 1;
  void** d_ccaps = acc->dd_ptrs;
  void** d_src = acc->dd_ptrs + M;
  void** d_wst = acc->dd_ptrs + 2 * M + 1;
  void** d_ctls = acc->dd_ptrs + 3 * M + 1;
  for (uint32_t i = 0; i < M; ++i) {
    hp[i] = ms[i]->ws.ccap;
    hp[2 * M + 1 + i] = acc->dd_wstat + (size_t)i * kDDWStat;
    hp[3 * M + 1 + i] = acc->dd_ctl + i;
  }
  if (rank) {
    hp[M] = m0->xrecv.p;
    hp[M + 1] = m0->cmsg.p;
  } else {
    for (uint32_t i = 0; i < M; ++i) hp[M + i] = ms[i]->cmsg.p;
    hp[2 * M] = nullptr;
  }
  CK(acc, hipMemcpyAsync(acc->dd_ptrs, hp, (size_t)(4 * M + 2) * sizeof(void*), hipMemcpyHostToDevice, st));
  // control blocks: the same window state on every member
  std::vector<WinCtl> hc(M);
  for (uint32_t i = 0; i < M; ++i) {
    WinCtl& h = hc[i];
    h = WinCtl{};
    h.tnext = (uint32_t)(acc->t + 1);
    h.tend = (uint32_t)std::min<uint64_t>(tend, 0xFFFFFFFFull);
    h.poll = poll;
    h.pbase = (uint32_t)acc->t;
    h.lmax = Lmax;
    h.recv = acc->recv;
    h.crashed = acc->crashed;
    h.pending = acc->pending;
    h.cover = cover_threshold(N);
    h.max_ticks = max_ticks;
    h.cmsg_cap = buf_cap(ms[i]->cmsg);
    h.fmsg_cap = buf_cap(ms[i]->fmsg);
    h.xs_cap = buf_cap(ms[i]->xsend);
    h.xr_cap = buf_cap(ms[i]->xrecv);
  }
  CK(acc, hipMemcpyAsync(acc->dd_ctl, hc.data(), (size_t)M * sizeof(WinCtl), hipMemcpyHostToDevice, st));
  CK(acc, hipMemsetAsync(acc->dd_gcnt, 0, (size_t)G * kMaxWindow * 8, st));
  // the members' window states (send side, and the receive side as
  // shard_exchange lays it out)
  std::vector<WinState> ws(M), wr(M);
  std::vector<uint64_t> tn_bound(M);
  for (uint32_t i = 0; i < M; ++i) {
    gs_ctx* m = ms[i];
    WinState w = m->ws;
    w.ctl = acc->dd_ctl + i;
    w.stage = acc->d_stage;
    w.lstride = Lmax;
    w.dd = 1;
    w.guard = 0;
    w.abort_on_err = 0;
    w.gcnt = acc->dd_gcnt;
    w.glay = acc->dd_glay;
    w.tfires = acc->dd_gcnt + (size_t)m->rank * kMaxWindow;
    w.cfill = acc->dd_glay + (size_t)m->rank * kDDRow;
    w.wstat = acc->dd_wstat + (size_t)i * kDDWStat;
    w.nglob = N;
    w.solo = solo ? 1u : 0u;
    w.gmap = (uint32_t*)m->gmap.p;
    w.cmsg = (uint32_t*)m->cmsg.p;
    w.fmsg = (uint32_t*)m->fmsg.p;
    ws[i] = w;
    if (solo) {
      wr[i] = w;
      tn_bound[i] = std::min<uint64_t>(m->ntot + 1, 4096ull * 1024);
      continue;
    }
    WinState r = w;
    r.cmsg = nullptr;
    r.csrc = (const uint32_t* const*)(m->d_rtab + 4 * K1);
    r.ccap = m->d_rtab;
    r.ccap_end = m->d_rtab + K1;
    r.cfill = m->d_rtab + 2 * K1;
    r.csub = G * kCoarseSub;
    wr[i] = r;
    tn_bound[i] = std::min<uint64_t>(m->ntot + 1, 4096ull * 1024);
  }
  const uint64_t T_bound = 2048ull * 16384;
  // an in-process group launches each small per-shard kernel once for all its
  // shards (WinGroup; GS_DD_GROUP=0: one launch per shard, the A/B baseline)
  static const bool group_env = [] { const char* e = getenv("GS_DD_GROUP"); return !(e && atoi(e) == 0); }();
  const bool grouped = !rank && M > 1 && group_env;
  std::vector<WinState> wall;
  WinGroup grp{};
  if (grouped) {
    wall.reserve(3 * M);
    wall.insert(wall.end(), ws.begin(), ws.end());
    wall.insert(wall.end(), wr.begin(), wr.end());
    for (uint32_t i = 0; i < M; ++i) {
      wall.push_back(wr[i]);
      wall.back().guard = 1;
    }
    CK(acc, hipMemcpyAsync(acc->dd_wsm, wall.data(), wall.size() * sizeof(WinState), hipMemcpyHostToDevice, st));
    grp.ws = acc->dd_wsm;
    grp.wr = acc->dd_wsm + M;
    grp.wg = acc->dd_wsm + 2 * M;
    grp.M = M;
    for (uint32_t i = 0; i < M; ++i) {
      grp.nfine_max = std::max(grp.nfine_max, ws[i].nfine);
      grp.ncoarse_max = std::max(grp.ncoarse_max, ws[i].ncoarse);
      grp.slots_max = std::max(grp.slots_max, ws[i].slots);
    }
  }
  // ranks whose blocks travel: the block sizes, from the gathered rows
  auto bsize = [&](uint32_t s, uint32_t d) {
    unsigned long long a = 0;
    for (uint32_t r = d * B8; r < (d + 1) * B8; ++r) a += acc->h_ddlay[(size_t)s * kDDRow + r];
    return a;
  };
  // one window: 0 = enqueued up to its close, 1 = stopped at the block
  // exchange (the window is dead: stopped, or aborted -> *aborted)
  auto enqueue = [&](uint32_t slot, bool* aborted) -> int {
    *aborted = false;
    if (grouped) {
      CK(acc, win_units_g(grp, Lmax, st));
      CK(acc, win_cut_g(grp, budget, st));
      CK(acc, win_unitscan_g(grp, st));
    } else {
      for (uint32_t i = 0; i < M; ++i) CK(acc, win_units(ws[i], 0, Lmax, st));
      if (rank) RC(x_all_gather(m0, acc->dd_gcnt, kMaxWindow * 8));
      for (uint32_t i = 0; i < M; ++i) CK(acc, win_cut(ws[i], budget, st));
      for (uint32_t i = 0; i < M; ++i) CK(acc, win_unitscan(ws[i], st));
    }
    if (grouped) CK(acc, win_expand_g(grp, Lmax, st));
    for (uint32_t i = 0; i < M && !grouped; ++i) CK(acc, win_expand(ws[i], 0, Lmax, tn_bound[i], 1, st));
    if (rank) RC(x_all_gather(m0, acc->dd_glay, kDDRow * 8));
    if (grouped)
      CK(acc, win_rtab_g(grp, (const unsigned long long* const*)d_ccaps, (const uint32_t* const*)d_src, nsrc, st));
    for (uint32_t i = 0; i < M && !solo && !grouped; ++i)
      CK(acc, win_rtab(ws[i], ms[i]->d_rtab, (const unsigned long long* const*)d_ccaps, (const uint32_t* const*)d_src,
                       nsrc, rank ? 1u : 0u, st));
    if (travel) {
      // the window's one host wait: block sizes for the grouped send / receive
      gs_ctx* m = m0;
      const uint32_t me = m->rank;
      CK(acc, hipMemcpyAsync(acc->h_ddlay, acc->dd_glay, (size_t)G * kDDRow * 8, hipMemcpyDeviceToHost, st));
      CK(acc, hipMemcpyAsync(m->h_err, m->d_err, 4, hipMemcpyDeviceToHost, st));
      CK(acc, hipMemcpyAsync(m->h_misc, acc->dd_ctl, 32, hipMemcpyDeviceToHost, st));
      CK(acc, hipStreamSynchronize(st));
      const uint32_t* hc0 = (const uint32_t*)m->h_misc;  // WinCtl t, L, tnext, tend, poll, pbase, stop, lmax
      if (*m->h_err & kErrAbort) { *aborted = true; return 1; }
      if (hc0[1] == 0 || hc0[6]) return 1;  // stopped or past the end: the same on every rank
      // every rank's send / receive needs against its buffers (their
      // capacities travel in the gathered rows): a rank that must grow them
      // does, and then every rank learns whether every rank could
      std::vector<unsigned long long> ptot(G, 0), rsum(G, 0);
      for (uint32_t s = 0; s < G; ++s)
        for (uint32_t d = 0; d < G; ++d)
          if (s != d) {
            const unsigned long long b = bsize(s, d);
            ptot[s] += b;
            rsum[d] += b;
          }
      bool any_grow = false;
      for (uint32_t s = 0; s < G; ++s) {
        const unsigned long long* row = acc->h_ddlay + (size_t)s * kDDRow;
        if (ptot[s] > row[kRegions + 2] || rsum[s] > row[kRegions + 3]) any_grow = true;
      }
      if (any_grow) {
        const void* old_recv = m->xrecv.p;
        const bool ok = grow(m->xsend, (ptot[me] + 16) * 4) && grow(m->xrecv, (rsum[me] + 16) * 4);
        unsigned long long* d = m->d_gcounts + (size_t)G * kMaxWindow;  // scratch
        m->h_misc[8] = ok ? 0ull : 1ull;
        CK(acc, hipMemcpyAsync(d, &m->h_misc[8], 8, hipMemcpyHostToDevice, st));
        RC(x_all_reduce(m, d, 1));
        CK(acc, hipMemcpyAsync(&m->h_misc[9], d, 8, hipMemcpyDeviceToHost, st));
        CK(acc, hipStreamSynchronize(st));
        if (m->h_misc[9]) return fail(acc, GS_ENOMEM, "a rank cannot allocate its exchange buffers");
        WinCtl* c = acc->dd_ctl;
        m->h_misc[10] = buf_cap(m->xsend);
        m->h_misc[11] = buf_cap(m->xrecv);
        CK(acc, hipMemcpyAsync(&c->xs_cap, &m->h_misc[10], 16, hipMemcpyHostToDevice, st));
        if (m->xrecv.p != old_recv) {  // the receive layout's source 0 (k_rtab wrote the old address)
          m->h_misc[12] = (unsigned long long)(uintptr_t)m->xrecv.p;
          CK(acc, hipMemcpyAsync(m->d_rtab + 4 * K1, &m->h_misc[12], 8, hipMemcpyHostToDevice, st));
          hp[M] = m->xrecv.p;
          CK(acc, hipMemcpyAsync(&d_src[0], &hp[M], sizeof(void*), hipMemcpyHostToDevice, st));
        }
        CK(acc, hipStreamSynchronize(st));  // the pinned words above are reused next window
      }
      CK(acc, win_pack(ws[0], m->d_rtab + 3 * K1, nreg, (uint32_t*)m->xsend.p, st));
      // block of sender s for destination d: after s's blocks for d' < d (its packed output)
      auto bstart = [&](uint32_t s, uint32_t d) {
        unsigned long long a = 0;
        for (uint32_t d2 = 0; d2 < d; ++d2)
          if (d2 != s) a += bsize(s, d2);
        return a;
      };
      std::vector<unsigned long long> in(G, 0);
      unsigned long long rs = 0;
      for (uint32_t s = 0; s < G; ++s)
        if (s != me) { in[s] = rs; rs += bsize(s, me); }
      uint32_t* xs = (uint32_t*)m->xsend.p;
      uint32_t* xr = (uint32_t*)m->xrecv.p;
      if (m->comm) {
        const Rccl& r = rccl();
        NCK(acc, r.group_start());
        for (uint32_t p = 0; p < G; ++p) {
          if (p == me) continue;
          if (bsize(me, p)) NCK(acc, r.send(xs + bstart(me, p), bsize(me, p), ncclUint32, (int)p, m->comm, st));
          if (bsize(p, me)) NCK(acc, r.recv(xr + in[p], bsize(p, me), ncclUint32, (int)p, m->comm, st));
        }
        NCK(acc, r.group_end());
      } else {
        std::vector<size_t> sb(G, 0), rb(G, 0);
        for (uint32_t p = 0; p < G; ++p)
          if (p != me) { sb[p] = bsize(me, p) * 4; rb[p] = bsize(p, me) * 4; }
        RC(agree_ok(m, grow_pinned(m, (ptot[me] + rs) * 4 + 16), "cannot allocate exchange staging"));
        char* hs = m->h_xbuf;
        char* hr = m->h_xbuf + ptot[me] * 4;
        CK(acc, hipMemcpyAsync(hs, xs, ptot[me] * 4, hipMemcpyDeviceToHost, st));
        CK(acc, hipStreamSynchronize(st));
        if (m->hx.all_to_allv(m->hx.user, hs, sb.data(), hr, rb.data()))
          return fail(acc, GS_EDEVICE, "the exchange's all_to_allv callback failed");
        CK(acc, hipMemcpyAsync(xr, hr, rs * 4, hipMemcpyHostToDevice, st));
        CK(acc, hipStreamSynchronize(st));
      }
    }
    if (grouped) {
      CK(acc, win_recv_g(grp, T_bound, st));
      CK(acc, win_resolve_g(grp, Lmax, st));
      CK(acc, win_stats_dd_g(grp, slot, st));
    } else {
      for (uint32_t i = 0; i < M; ++i) {
        CK(acc, win_plan(wr[i], false, st));
        CK(acc, win_part2(wr[i], T_bound, true, st));
        if (!solo) CK(acc, win_fine_redo(wr[i], T_bound, st));
        CK(acc, win_resolve(wr[i], 0, Lmax, st));
        CK(acc, win_stats_dd(ws[i], slot, st));
      }
    }
    if (rank) RC(x_all_reduce(m0, acc->dd_wstat, kDDWStat));
    if (!solo)  // (one in-process shard: k_stats_dd closed the window)
      CK(acc, win_close_dd(ws[0], (const unsigned long long* const*)d_wst, (WinCtl* const*)d_ctls, M, slot, st));
    CK(acc, hipEventRecord(acc->wev[slot], st));
    return 0;
  };
  bool eoverflow = false;
  // window i-1's results: 0 = go on, 1 = finished
  auto absorb = [&](uint32_t slot, int* what) -> int {
    CK(acc, hipEventSynchronize(acc->wev[slot]));
    const unsigned long long* sg = acc->h_stage + (size_t)slot * kStageWords;
    const uint32_t t0 = (uint32_t)sg[0], L = (uint32_t)sg[1];
    *what = 0;
    if (sg[3] & kErrAbort) {
      if (dd_log()) fprintf(stderr, "[dd] window at t0=%u aborted: redone host-driven\n", t0);
      ++m0->timing.dd_fallbacks;
      *fallback = true;
      *what = 1;
      return GS_OK;
    }
    if (dd_log()) fprintf(stderr, "[dd] t0=%u L=%u stop=%llu redos=%llu\n", t0, L, sg[2], sg[4]);
    m0->timing.exact_redos += sg[4];
    for (uint32_t k = 0; k < L; ++k) on_tick((uint64_t)t0 + k, sg + 8 + (size_t)k * kStatFields);
    if (sg[3] & kErrArrivals) eoverflow = true;
    if (sg[2]) *stop = (uint32_t)sg[2];
    if (sg[2] || L == 0 || (uint64_t)t0 + L >= tend || eoverflow) *what = 1;
    return GS_OK;
  };
  bool ab = false;
  int e0 = 0;
  RC((e0 = enqueue(0, &ab), e0 < 0 ? e0 : 0));
  if (e0 == 1) {
    *fallback = ab;
  } else {
    for (uint32_t i = 1;; ++i) {
      const int e = enqueue(i % kSlots, &ab);
      if (e < 0) return e;
      int what = 0;
      RC(absorb((i - 1) % kSlots, &what));
      if (what) break;
      if (e == 1) {  // window i stopped at its exchange (it staged nothing)
        *fallback = ab;
        break;
      }
    }
  }
  CK(acc, hipStreamSynchronize(st));
  if (*fallback) {  // undo what the stopped window left: its expand's counters, the flags
    for (gs_ctx* m : ms) {
      CK(acc, hipMemsetAsync(m->ws.sstats, 0, (size_t)kStatShards * kMaxWindow * kStatFields * 8, st));
      CK(acc, hipMemcpyAsync(m->h_err, m->d_err, 4, hipMemcpyDeviceToHost, st));
      CK(acc, hipStreamSynchronize(st));
      if (dd_log()) {  // the window's cut and coarse plan (plan 0: k_cut found the buffer too small)
        const size_t i = (size_t)(std::find(ms.begin(), ms.end(), m) - ms.begin());
        WinCtl h1{};
        unsigned long long plan = 0;
        CK(acc, hipMemcpy(&h1, acc->dd_ctl + i, sizeof(WinCtl), hipMemcpyDeviceToHost));
        CK(acc, hipMemcpy(&plan, m->ws.ccap + kRegions, 8, hipMemcpyDeviceToHost));
        fprintf(stderr, "[dd] shard %u flags %#x t=%u L=%u Tn=%llu T=%llu cmsg_cap=%llu plan=%llu\n", m->rank,
                *m->h_err, h1.t, h1.L, h1.Tn, h1.T, h1.cmsg_cap, plan);
      }
      *m->h_err &= ~(kErrCoarse | kErrFine | kErrAbort);
      CK(acc, hipMemcpyAsync(m->d_err, m->h_err, 4, hipMemcpyHostToDevice, st));
    }
    CK(acc, hipStreamSynchronize(st));
  }
  if (eoverflow) return fail(acc, GS_EOVERFLOW, "too many arrivals at one node in one tick");
  return GS_OK;
}

// Sharded step: `acc` keeps the global counters (the group, or the rank).
int shard_step(gs_ctx* acc, const std::vector<gs_ctx*>& ms, uint32_t ticks, gs_tick_stats* out) {
  const bool timing = (acc->p.flags & GS_FLAG_TIMING) != 0;
  for (gs_ctx* m : ms) {
    CK(m, hipSetDevice(m->dev));
    RC(expand_view(m));
  }
  if (dd_ok(acc, ms) && ticks > 0) {  // device-driven windows
    uint32_t stop = 0, k = 0;
    bool fallback = false;
    RC(dd_run(acc, ms, acc->t + ticks + 1, 0, ~0ull,
              [&](uint64_t tick, const unsigned long long* row) {
                account_tick(acc, tick, row, out ? &out[k] : nullptr);
                ++k;
              },
              &stop, &fallback));
    if (!fallback) return GS_OK;
    ticks -= k;  // a window overflowed: it and the rest host-driven
    if (out) out += k;
  }
  std::vector<unsigned long long> sum(kStatFields);
  uint32_t done = 0;
  while (done < ticks) {
    const uint32_t batch = std::min<uint32_t>(ticks - done, kStatSlots);
    const uint64_t t0 = acc->t + 1;
    const uint32_t i0 = (uint32_t)(t0 % kStatSlots);
    const uint32_t first = std::min<uint32_t>(batch, kStatSlots - i0);
    for (gs_ctx* m : ms) {
      CK(m, hipSetDevice(m->dev));
      CK(m, hipMemsetAsync(m->st.stats + (size_t)i0 * kStatFields, 0, (size_t)first * kStatFields * 8, m->stream));
      if (first < batch)
        CK(m, hipMemsetAsync(m->st.stats, 0, (size_t)(batch - first) * kStatFields * 8, m->stream));
    }
    RC(shard_windows(acc, ms, t0, batch, timing));
    for (gs_ctx* m : ms) {
      CK(m, hipSetDevice(m->dev));
      unsigned long long* a = m->st.stats + (size_t)i0 * kStatFields;
      if (is_rank(m)) {  // the global per-tick counters on every rank
        RC(x_all_reduce(m, a, (size_t)first * kStatFields));
        if (first < batch) RC(x_all_reduce(m, m->st.stats, (size_t)(batch - first) * kStatFields));
      }
      CK(m, hipMemcpyAsync(m->h_stats + (size_t)i0 * kStatFields, a, (size_t)first * kStatFields * 8,
                           hipMemcpyDeviceToHost, m->stream));
      if (first < batch)
        CK(m, hipMemcpyAsync(m->h_stats, m->st.stats, (size_t)(batch - first) * kStatFields * 8,
                             hipMemcpyDeviceToHost, m->stream));
    }
    RC(sync_all(ms));
    for (uint32_t i = 0; i < batch; ++i) {
      const size_t row = (size_t)((t0 + i) % kStatSlots) * kStatFields;
      for (uint32_t f = 0; f < kStatFields; ++f) {
        sum[f] = 0;
        for (gs_ctx* m : ms) sum[f] += m->h_stats[row + f];
      }
      account_tick(acc, t0 + i, sum.data(), out ? &out[done + i] : nullptr);
    }
    done += batch;
  }
  return GS_OK;
}

// Batched trials: fold one chunk's per-trial counters (h_tstat, `nt` ticks
// from tick t0) into the trials' running totals.
void account_trials(gs_ctx* c, uint64_t t0, uint32_t nt) {
  for (uint32_t tr = 0; tr < c->trials; ++tr) {
    TrialAcc& a = c->tacc[tr];
    for (uint32_t k = 0; k < nt; ++k) {
      const uint32_t* r = c->h_tstat + ((size_t)tr * kMaxWindow + k) * kTStatFields;
      a.fired += r[TS_FIRED];
      a.sent += r[TS_SENT];
      a.msgs += (uint64_t)r[TS_SENT] - r[TS_DEAD];
      a.recv += r[TS_RECV];
      a.sched += r[TS_RECV];  // every infection schedules one Broadcast
      a.crash += r[TS_CRASH];
      if (!a.tick99 && covered(a.recv, c->p.n)) a.tick99 = t0 + k;
    }
  }
}

}  // namespace

extern "C" {

int gs_step(gs_ctx* c, uint32_t ticks, gs_tick_stats* out) {
  if (!c) return GS_EINVAL;
  if (c->aborted) return fail(c, GS_EDEVICE, "this rank's exchange failed earlier; the run is over");
  if (!c->begun) return fail(c, GS_EINVAL, "gs_broadcast_begin first");
  if (c->group && c->gtrials) {
    std::vector<std::vector<gs_tick_stats>> rows(c->mem.size(), std::vector<gs_tick_stats>(ticks));
    std::vector<gs_ctx*>& ms = c->mem;
    RC(par_members(c, [&](gs_ctx* m) {
      const size_t i = (size_t)(std::find(ms.begin(), ms.end(), m) - ms.begin());
      return gs_step(m, ticks, rows[i].data());
    }));
    std::vector<unsigned long long> s(kStatFields);
    for (uint32_t k = 0; k < ticks; ++k) {
      std::fill(s.begin(), s.end(), 0ull);
      uint64_t pend = 0;
      for (auto& r : rows) {
        s[ST_FIRED] += r[k].fired;
        s[ST_SENT] += r[k].sent;
        s[ST_MSGS] += r[k].messages;
        pend += r[k].pending;
      }
      uint64_t recv = 0, cr = 0;
      for (auto& r : rows) { recv += r[k].received; cr += r[k].crashed; }
      c->t = rows[0][k].tick;
      c->fired += s[ST_FIRED]; c->sent += s[ST_SENT]; c->msgs += s[ST_MSGS];
      c->recv = recv; c->crashed = cr; c->pending = pend;
      if (out) out[k] = gs_tick_stats{c->t, s[ST_FIRED], s[ST_SENT], s[ST_MSGS], recv, cr, pend};
    }
    return GS_OK;
  }
  if (c->pp && (c->group || c->pp_shard)) return pp_shard_step(c, ticks, out);
  if (c->group) return shard_step(c, c->mem, ticks, out);
  if (c->shard) return abort_rank(c, shard_step(c, {c}, ticks, out));
  CK(c, hipSetDevice(c->dev));
  if (async_ok(c) && ticks > 0) {  // device-driven windows
    uint32_t stop = 0, k = 0;
    bool fallback = false;
    RC(run_async(c, c->t + ticks + 1, 0, ~0ull,
                 [&](uint64_t tick, const unsigned long long* row) {
                   account_tick(c, tick, row, out ? &out[k] : nullptr);
                   ++k;
                 },
                 &stop, &fallback));
    if (!fallback) return GS_OK;
    ticks -= k;  // a window overflowed: the rest host-driven (it redoes that window exactly)
    if (out) out += k;
  }
  const bool timing = (c->p.flags & GS_FLAG_TIMING) != 0;
  const bool flood = c->st.kc == 0;
  const bool batched = c->trials > 1;
  uint32_t done = 0;
  while (done < ticks) {
    // batched trials: chunks of <= kMaxWindow ticks (the per-trial counter rows)
    const uint32_t batch = std::min<uint32_t>(ticks - done, batched ? kMaxWindow : kStatSlots);
    const uint64_t t0 = c->t + 1;
    // zero this batch's stats entries (ring-indexed)
    const uint32_t i0 = (uint32_t)(t0 % kStatSlots);
    const uint32_t first = std::min<uint32_t>(batch, kStatSlots - i0);
    CK(c, hipMemsetAsync(c->st.stats + (size_t)i0 * kStatFields, 0, (size_t)first * kStatFields * 8,
                         c->stream));
    if (first < batch)
      CK(c, hipMemsetAsync(c->st.stats, 0, (size_t)(batch - first) * kStatFields * 8, c->stream));
    if (batched)
      CK(c, hipMemsetAsync(c->d_tstat, 0, (size_t)c->trials * kMaxWindow * kTStatFields * 4, c->stream));
    const uint32_t nev = timing && !c->win ? batch * (flood || c->pp ? 2 : 4) : 0;
    while (c->ev.size() < nev) {
      hipEvent_t e;
      CK(c, hipEventCreate(&e));
      c->ev.push_back(e);
    }
    if (c->win) RC(run_windows(c, t0, batch, timing, t0));
    for (uint32_t i = 0; i < batch && c->pp; ++i) {  // push-pull rounds
      const uint32_t tt = (uint32_t)(t0 + i);
      hipEvent_t* e = timing ? &c->ev[(size_t)i * 2] : nullptr;
      if (e) CK(c, hipEventRecord(e[0], c->stream));
      CK(c, pp_round(c->st, c->d_next, c->d_ppsum, tt, c->pp_l2_only, c->sp, c->stream));
      CK(c, pp_commit(c->st, c->d_next, tt, c->sp, c->stream));
      if (e) CK(c, hipEventRecord(e[1], c->stream));
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
    if (batched)
      CK(c, hipMemcpyAsync(c->h_tstat, c->d_tstat, (size_t)c->trials * kMaxWindow * kTStatFields * 4,
                           hipMemcpyDeviceToHost, c->stream));
    CK(c, hipStreamSynchronize(c->stream));
    if (!c->win && !c->pp && !flood) {  // the tick engine's 16-bit receipt counts (MODE_COUNT)
      uint32_t err = 0;
      CK(c, hipMemcpy(&err, c->d_err, 4, hipMemcpyDeviceToHost));
      if (err & kErrArrivals) return fail(c, GS_EOVERFLOW, "too many arrivals at one node in one tick");
    }
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
      account_tick(c, t0 + i, s, out ? &out[done + i] : nullptr);
    }
    if (batched) account_trials(c, t0, batch);
    done += batch;
  }
  return GS_OK;
}

}  // extern "C"

namespace {

void snap_trial(const gs_ctx* c, uint32_t tr, int32_t status) {
  TrialAcc& a = const_cast<gs_ctx*>(c)->tacc[tr];
  a.status = status;
  a.snap = gs_trial_stats{(uint64_t)c->p.trial + tr, a.tick99, c->t, a.fired, a.sent, a.msgs, a.recv,
                          a.crash, status, 0};
}

// Push-pull's exact stop: can any call still change the informed set?
int pp_stalled(gs_ctx* c, bool* stalled) {
  *stalled = true;
  if (c->st.kd >= 100) return GS_OK;  // every call is lost (simulator.go:172 quantisation)
  if (c->group || c->pp_shard) {  // shards: their own callers' edges against the replicated sets, summed
    unsigned long long live = 0;
    for (gs_ctx* m : shards_of(c)) {
      CK(m, hipSetDevice(m->dev));
      CK(m, pp_live_edges(m->st, m->d_err + 2, m->stream));
      uint32_t h = 0;
      CK(m, hipMemcpyAsync(&h, m->d_err + 2, 4, hipMemcpyDeviceToHost, m->stream));
      CK(m, hipStreamSynchronize(m->stream));
      live += h;
    }
    if (!c->group) {
      unsigned long long* d = c->d_gcounts;
      CK(c, hipMemcpyAsync(d, &live, 8, hipMemcpyHostToDevice, c->stream));
      if (int rc = x_all_reduce(c, d, 1)) return abort_rank(c, rc);
      CK(c, hipMemcpyAsync(&live, d, 8, hipMemcpyDeviceToHost, c->stream));
      CK(c, hipStreamSynchronize(c->stream));
    }
    *stalled = live == 0;
    return GS_OK;
  }
  unsigned long long live = 0;
  CK(c, pp_live_edges(c->st, c->d_err + 2, c->stream));
  uint32_t h = 0;
  CK(c, hipMemcpyAsync(&h, c->d_err + 2, 4, hipMemcpyDeviceToHost, c->stream));
  CK(c, hipStreamSynchronize(c->stream));
  live = h;
  *stalled = live == 0;
  return GS_OK;
}

}  // namespace

extern "C" {

int gs_run(gs_ctx* c, uint32_t poll, uint64_t max_ticks, gs_tick_stats* out, size_t cap,
           size_t* nout, int32_t* status) {
  if (!c || poll == 0) return fail(c, GS_EINVAL, "poll must be >= 1");
  if (c->group && c->gtrials) {  // every batch runs its own trials to their stops
    std::vector<int32_t> sts(c->mem.size(), 0);
    std::vector<gs_ctx*>& ms = c->mem;
    RC(par_members(c, [&](gs_ctx* m) {
      const size_t i = (size_t)(std::find(ms.begin(), ms.end(), m) - ms.begin());
      return gs_run(m, poll, max_ticks, nullptr, 0, nullptr, &sts[i]);
    }));
    gs_tick_stats tot{};
    uint64_t recv = 0, cr = 0, t = 0, pend = 0;
    c->fired = c->sent = c->msgs = 0;
    for (gs_ctx* m : ms) {
      c->fired += m->fired; c->sent += m->sent; c->msgs += m->msgs;
      recv += m->recv; cr += m->crashed; pend += m->pending; t = std::max(t, m->t);
    }
    c->t = t; c->recv = recv; c->crashed = cr; c->pending = pend;
    tot = gs_tick_stats{t, c->fired, c->sent, c->msgs, recv, cr, pend};
    if (out && cap) out[0] = tot;
    if (nout) *nout = 1;
    if (status) *status = *std::max_element(sts.begin(), sts.end());
    return GS_OK;
  }
  size_t k = 0;
  int32_t st = GS_RUN_MAX_TICKS;
  const bool trials = c->trials > 1 && !c->group;
  const bool flood = !c->pp;
  const uint64_t pbase = c->t;
  uint64_t f0 = c->fired, s0 = c->sent, m0 = c->msgs;
  if (!c->pp && !c->gtrials && (c->group || c->shard) && dd_ok(c, shards_of(c))) {
    // device-driven shard windows: the poll rule runs on the device (k_close_dd)
    if (c->aborted) return fail(c, GS_EDEVICE, "this rank's exchange failed earlier; the run is over");
    if (!c->begun) return fail(c, GS_EINVAL, "gs_broadcast_begin first");
    std::vector<gs_ctx*> ms = shards_of(c);
    for (gs_ctx* m : ms) {
      CK(m, hipSetDevice(m->dev));
      RC(expand_view(m));
    }
    uint32_t stop = 0;
    bool fallback = false;
    const int rc = dd_run(c, ms, ~0ull, poll, max_ticks,
                          [&](uint64_t tick, const unsigned long long* row) {
                            account_tick(c, tick, row, nullptr);
                            if ((tick - pbase) % poll) return;
                            if (out && k < cap)
                              out[k] = gs_tick_stats{c->t, c->fired - f0, c->sent - s0, c->msgs - m0, c->recv,
                                                     c->crashed, c->pending};
                            ++k;
                            f0 = c->fired; s0 = c->sent; m0 = c->msgs;
                          },
                          &stop, &fallback);
    if (rc) return c->group ? rc : abort_rank(c, rc);
    if (!fallback) {
      st = stop ? (int32_t)stop - 1 : GS_RUN_MAX_TICKS;
      if (c->tacc.size() == 1) snap_trial(c, 0, st);
      if (nout) *nout = k;
      if (status) *status = st;
      return GS_OK;
    }
  } else if (async_ok(c)) {  // device-driven windows: the poll rule runs on the device (k_close)
    uint32_t stop = 0;
    bool fallback = false;
    RC(run_async(c, ~0ull, poll, max_ticks,
                 [&](uint64_t tick, const unsigned long long* row) {
                   account_tick(c, tick, row, nullptr);
                   if ((tick - pbase) % poll) return;
                   if (out && k < cap)
                     out[k] = gs_tick_stats{c->t, c->fired - f0, c->sent - s0, c->msgs - m0, c->recv,
                                            c->crashed, c->pending};
                   ++k;
                   f0 = c->fired; s0 = c->sent; m0 = c->msgs;
                 },
                 &stop, &fallback));
    if (!fallback) {
      st = stop ? (int32_t)stop - 1 : GS_RUN_MAX_TICKS;
      snap_trial(c, 0, st);
      if (nout) *nout = k;
      if (status) *status = st;
      return GS_OK;
    }
  }
  for (;;) {
    const uint64_t r0 = c->recv;
    // one poll (the first may finish a poll the device-driven windows began)
    RC(gs_step(c, (uint32_t)(poll - (c->t - pbase) % poll), nullptr));
    if (out && k < cap)
      out[k] = gs_tick_stats{c->t, c->fired - f0, c->sent - s0, c->msgs - m0, c->recv, c->crashed, c->pending};
    ++k;
    f0 = c->fired; s0 = c->sent; m0 = c->msgs;
    if (trials) {  // each trial stops at its own poll (simulator.go:243-251 per process)
      uint32_t running = 0;
      for (uint32_t tr = 0; tr < c->trials; ++tr) {
        TrialAcc& a = c->tacc[tr];
        if (a.status != GS_RUN_RUNNING) continue;
        const uint64_t pend = 1 + a.sched - a.fired;
        if (covered(a.recv, c->p.n)) snap_trial(c, tr, GS_RUN_COVERED);
        else if (pend == 0) snap_trial(c, tr, GS_RUN_QUIESCENT);
        else if (c->t >= max_ticks) snap_trial(c, tr, GS_RUN_MAX_TICKS);
        else ++running;
      }
      if (running == 0) {
        st = GS_RUN_COVERED;
        for (const TrialAcc& a : c->tacc) st = std::max(st, a.status);
        break;
      }
      continue;
    }
    if (covered(c->recv, c->p.n)) { st = GS_RUN_COVERED; break; }
    if (flood && c->pending == 0) { st = GS_RUN_QUIESCENT; break; }
    if (!flood && c->recv == r0) {  // push-pull: a window that informed nobody new
      bool stalled = false;
      RC(pp_stalled(c, &stalled));
      if (stalled) { st = GS_RUN_QUIESCENT; break; }
    }
    if (c->t >= max_ticks) { st = GS_RUN_MAX_TICKS; break; }
  }
  if (!trials && c->tacc.size() == 1) snap_trial(c, 0, st);
  if (nout) *nout = k;
  if (status) *status = st;
  return GS_OK;
}

int gs_trial_results(gs_ctx* c, gs_trial_stats* out, size_t cap, size_t* nout) {
  if (!c) return GS_EINVAL;
  size_t k = 0;
  auto one = [&](const gs_ctx* x) {
    for (size_t i = 0; i < x->tacc.size(); ++i, ++k) {
      if (!out || k >= cap) continue;
      const TrialAcc& a = x->tacc[i];
      if (a.status != GS_RUN_RUNNING) {
        out[k] = a.snap;
      } else {
        out[k] = gs_trial_stats{(uint64_t)x->p.trial + i, a.tick99, x->t, a.fired, a.sent, a.msgs, a.recv,
                                a.crash, GS_RUN_RUNNING, 0};
      }
    }
  };
  if (c->group && c->gtrials) for (gs_ctx* m : c->mem) one(m);
  else one(c);
  if (nout) *nout = k;
  return GS_OK;
}

int gs_totals(gs_ctx* c, gs_tick_stats* out) {
  if (!c || !out) return GS_EINVAL;
  *out = gs_tick_stats{c->t, c->fired, c->sent, c->msgs, c->recv, c->crashed, c->pending};
  return GS_OK;
}

}  // extern "C"

namespace {

// Bitset `which` (0 = received, 1 = crashed) of context c into words: a
// shard's own words at their global positions, batched trials trial-major.
int read_bits(gs_ctx* c, int which, uint64_t* words, size_t nwords) {
  const uint64_t Wn = (c->p.n + 63) / 64;
  if (c->group && c->gtrials) {  // every member's trials, back to back: the caller's buffer holds them all
    if (nwords < Wn * c->trials) return fail(c, GS_EINVAL, "need ceil(n/64) words per trial");
    uint64_t off = 0;
    for (gs_ctx* m : c->mem) {
      if (read_bits(m, which, words + off * Wn, nwords - off * Wn)) return fail(c, GS_EINVAL, m->err);
      off += m->trials;
    }
    return GS_OK;
  }
  if (c->group) {
    std::fill(words, words + Wn, 0ull);
    std::vector<uint64_t> tmp(Wn);
    for (gs_ctx* m : c->mem) {
      if (read_bits(m, which, tmp.data(), Wn)) return fail(c, GS_EINVAL, m->err);
      for (uint64_t i = 0; i < Wn; ++i) words[i] |= tmp[i];
    }
    return GS_OK;
  }
  if (nwords < Wn * c->trials) return fail(c, GS_EINVAL, "need ceil(n/64) words per trial");
  CK(c, hipSetDevice(c->dev));
  const unsigned long long* src = which ? c->st.crash : c->st.recv;
  if (c->trials > 1) {
    CK(c, hipMemcpy2DAsync(words, Wn * 8, src, ((size_t)1 << c->tlog) / 8, Wn * 8, c->trials,
                           hipMemcpyDeviceToHost, c->stream));
  } else if (c->shard) {
    std::fill(words, words + Wn, 0ull);
    CK(c, hipMemcpyAsync(words + c->lo / 64, src, c->st.W * 8, hipMemcpyDeviceToHost, c->stream));
  } else {
    CK(c, hipMemcpyAsync(words, src, c->st.W * 8, hipMemcpyDeviceToHost, c->stream));
  }
  CK(c, hipStreamSynchronize(c->stream));
  return GS_OK;
}

}  // namespace

extern "C" {

int gs_read_received(gs_ctx* c, uint64_t* words, size_t nwords) {
  if (!c || !words || nwords < (c->p.n + 63) / 64) return fail(c, GS_EINVAL, "need ceil(n/64) words");
  return read_bits(c, 0, words, nwords);
}

int gs_read_crashed(gs_ctx* c, uint64_t* words, size_t nwords) {
  if (!c || !words || nwords < (c->p.n + 63) / 64) return fail(c, GS_EINVAL, "need ceil(n/64) words");
  return read_bits(c, 1, words, nwords);
}

int gs_timing_get(gs_ctx* c, gs_timing* out) {
  if (!c || !out) return GS_EINVAL;
  *out = c->group ? c->mem[0]->timing : c->timing;  // a group: its first member's kernels
  if (c->group) out->overlay_ms = c->timing.overlay_ms;
  out->pp_early_rounds = out->pp_bottom_rounds = out->pp_answer_rounds = 0;
  gs_ctx* pc = c->group ? c->mem[0] : c;  // a group: its first shard's rounds (all shards run the same modes)
  if (c->pp && pc->sp.ctl && c->begun) {
    CK(pc, hipSetDevice(pc->dev));
    PPCtl h;
    CK(pc, hipMemcpyAsync(&h, pc->sp.ctl, offsetof(PPCtl, segcnt), hipMemcpyDeviceToHost, pc->stream));
    CK(pc, hipStreamSynchronize(pc->stream));
    out->pp_early_rounds = h.nearly;
    out->pp_bottom_rounds = h.nbottom;
    out->pp_answer_rounds = h.nanswer;
  }
  if (c->pp && c->begun) out->pp_early_rounds += c->rep_rounds;  // shards: the replicas' sparse rounds
  fill_devmem(out);
  return GS_OK;
}

int gs_shard_timing(gs_ctx* c, uint32_t index, gs_timing* out) {
  if (!c || !out) return GS_EINVAL;
  if (!c->group) return index == 0 ? gs_timing_get(c, out) : fail(c, GS_EINVAL, "no such shard");
  if (index >= c->mem.size()) return fail(c, GS_EINVAL, "no such shard");
  *out = c->mem[index]->timing;
  fill_devmem(out);
  return GS_OK;
}

int gs_set_trial(gs_ctx* c, uint32_t trial) {
  if (!c) return GS_EINVAL;
  if (c->begun) return fail(c, GS_EINVAL, "gs_reset before gs_set_trial");
  if (c->group) {
    uint32_t t = trial;
    for (gs_ctx* m : c->mem) {
      RC(gs_set_trial(m, c->gtrials ? t : trial) ? fail(c, GS_EINVAL, m->err) : 0);
      t += m->trials;
    }
    c->p.trial = trial;
    c->peers = false;
    return GS_OK;
  }
  c->p.trial = trial;
  c->st.key.trial = trial;
  c->ws.key.trial = trial;
  c->peers = false;  // the overlay of the new trials is still to be built (or loaded)
  reset_counters(c);
  return GS_OK;
}

int gs_set_flags(gs_ctx* c, uint32_t flags) {
  if (!c) return GS_EINVAL;
  c->p.flags = flags;
  for (gs_ctx* m : c->mem) m->p.flags = flags;
  return GS_OK;
}

int gs_reset(gs_ctx* c) {
  if (!c) return GS_EINVAL;
  for (gs_ctx* m : c->mem) RC(gs_reset(m) ? fail(c, GS_EDEVICE, m->err) : 0);
  if (!c->group) {
    CK(c, hipSetDevice(c->dev));
    // everything in the state block except the stats ring, then the error
    // word (a broadcast that overflowed -- kErrArrivals, or a partition flag
    // -- leaves the context usable; table validation reports at load time)
    CK(c, hipMemsetAsync(c->d_state, 0, (char*)c->st.stats - (char*)c->d_state, c->stream));
    if (c->d_err) CK(c, hipMemsetAsync(c->d_err, 0, 4, c->stream));
    if (c->d_cnt) CK(c, hipMemsetAsync(c->d_cnt, 0, c->st.n * 4, c->stream));
    if (c->win) CK(c, hipMemsetAsync(c->ws.fcount, 0, c->fcount_bytes, c->stream));
    if (c->failed && !c->pp_shard)
      CK(c, hipMemcpyAsync(c->st.crash, c->d_failed, c->st.W * 8, hipMemcpyDeviceToDevice, c->stream));
    if (c->pp_shard)  // this shard's slice of the replicated informed set
      CK(c, hipMemsetAsync(c->st.recv, 0, c->st.W * 8, c->stream));
    CK(c, hipStreamSynchronize(c->stream));
  }
  reset_counters(c);
  c->begun = false;
  return GS_OK;
}

void gs_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  const u32x4 r = philox(ctr[0], ctr[1], ctr[2], ctr[3], key[0], key[1]);
  out[0] = r.x; out[1] = r.y; out[2] = r.z; out[3] = r.w;
}

}  // extern "C"
