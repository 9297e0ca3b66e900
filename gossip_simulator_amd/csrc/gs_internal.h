// gs_internal.h -- device-state layout shared by the broadcast and overlay
// translation units and the C-ABI implementation.
//
// HBM layout for one broadcast (N nodes, W = ceil(N/64) words, R ring slots):
//   deg     u8 [N]              friends-list length   (simulator.go:45)
//   ids     u32[N * stride]     friends rows          (simulator.go:45)
//   recv    u64[W]              received bitset       (simulator.go:38)
//   crash   u64[W]              crashed bitset        (simulator.go:39)
//   ring    u64[R][W]           fire ring: slot s holds every Broadcast whose
//                               time.After(delay) expires at a tick = s mod R
//                               (simulator.go:141-142)
//   cflag   u32[R][C]           1 if chunk c (4096 nodes = 64 words) of slot s
//                               has a pending fire bit
//   clist   u32[R][32][CS]      active chunks of slot s, 32 shards (c mod 32)
//   ccount  u32[R][32 * 16]     shard fill counters, one 64-B line each
//   cnt     u32[N]              per-tick arrival counts (only if crash% > 0)
//   stats   u64[4096][8]        per-tick counters, ring-indexed by tick
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

#include <vector>

#include "gs_devmem.h"
#include "gs_rng.h"

namespace gs {

constexpr uint32_t kWave = 64;
constexpr uint32_t kChunkNodesLog = 12;  // 4096 nodes = 64 words per chunk
constexpr uint32_t kChunkWords = 64;
constexpr uint32_t kShards = 32;
constexpr uint32_t kCounterStride = 16;  // u32s between shard counters (64 B)
constexpr uint32_t kStatFields = 8;
constexpr uint32_t kStatSlots = 4096;
constexpr uint32_t kListCap = 1024;      // per-wave LDS list of firing nodes
constexpr uint32_t kTickBlock = 256;
constexpr uint32_t kTickGridMax = 2048;

enum Stat : uint32_t {
  ST_FIRED = 0, ST_SENT = 1, ST_MSGS = 2, ST_RECV = 3, ST_CRASH = 4, ST_SCHED = 5,
  ST_ERR = 6, ST_RSVD = 7
};

// Tick kernel modes.
enum Mode : int {
  MODE_FLOOD = 0,    // crash% == 0: deliver + infect fused, one atomicOr per send
  MODE_COUNT = 1,    // crash% > 0, pass 1: count arrivals per node
  MODE_RESOLVE = 2   // crash% > 0, pass 2: one owner per node runs the ordinals
};

struct DevState {
  const uint8_t* deg;
  const uint32_t* ids;
  unsigned long long* recv;
  unsigned long long* crash;
  uint32_t* rollw;         // window engine: crash-roll marks of the window (cleared by k_resolve)
  uint32_t* cnt;
  unsigned long long* ring;
  uint32_t* cflag;
  uint32_t* clist;
  uint32_t* ccount;
  unsigned long long* stats;
  uint32_t* err;           // error word (kErrArrivals: a 16-bit receipt count overflowed)
  // Push-pull node-range shards: the informed and failed sets by GLOBAL node id
  // (replicated on every shard, exchanged each round); recv / crash above are
  // this shard's own slice of them, local node i = global gbase + i.  Every
  // other context: grecv = recv, gcrash = crash, gbase = 0.
  unsigned long long* grecv;
  unsigned long long* gcrash;
  uint64_t gbase;
  uint64_t n, W;
  uint32_t C, CS, R, stride;
  uint32_t stride_magic;   // floor(2^32 / stride) + 1: exact q/stride for q < 2^18
  int32_t delay_low;
  uint32_t delay_span;
  int32_t kd, kc;
  int32_t check_crashed;   // FLOOD mode: a pre-failed mask is present
  int32_t sharded;         // node-range sharding: visit every chunk (the slot was all-gathered)
  uint32_t lo, hi;         // owned node range
  uint32_t chunk_lo, chunk_hi;  // owned chunks [lo/4096, ceil(hi/4096))
  Key key;
};

// ---- window engine (gs_window.hip) --------------------------------------
// Fires scheduled at tick t land at t + off with off >= max(delaylow, 1), so
// the firing sets of the next L = min(max(delaylow,1), 16) ticks are known
// before any of them is processed: a WINDOW of L ticks is expanded,
// partitioned by target bucket and resolved in one pass.
constexpr uint32_t kFineLog = 14;               // 16384 nodes per fine bucket
constexpr uint32_t kFineNodes = 1u << kFineLog;
constexpr uint32_t kCoarseShift = kFineLog + 8; // 256 fine buckets per coarse bucket
constexpr uint32_t kMaxWindow = 16;             // tick offset in 4 bits
// Coarse regions: each of the 256 coarse bins has kCoarseSub sub-regions, one
// per XCD (a block writes the sub-region of blockIdx % 8): the reservation
// atomics of a bin spread over 8 addresses, and the runs written into one
// sub-region meet in one XCD's L2.
constexpr uint32_t kCoarseSub = 8;
constexpr uint32_t kRegions = 256 * kCoarseSub;
constexpr uint32_t kWinMaxRing = 256;
constexpr uint32_t kWinMaxStride = 32;          // friends-row length the window engine takes
constexpr uint32_t kEmptyMsg = 0xFFFFFFFFu;
constexpr uint32_t kSrcShift = 56;                        // receive layout: source index of a region
constexpr unsigned long long kSrcMask = (1ull << kSrcShift) - 1;
#ifndef GS_PART_TILE
#define GS_PART_TILE 16384
#endif
constexpr uint32_t kPartTile = GS_PART_TILE;    // messages per partition tile (runs of ~64 per fine bucket)
constexpr uint32_t kRolledCap = 1024;           // rolled receipts per bucket k_resolve lists (more: its large path)
constexpr uint32_t kBitTicks = 10;              // window length k_resolve's per-tick bitmaps hold
// Coarse sub-region estimates: k_expand deals its rounds to the XCDs in 8
// contiguous runs of ceil(rounds / 8), so one XCD's sub-region of a bin can
// hold one round more than an eighth of the bin's share: at most this many
// firing nodes per round (512 threads x 4) times the row length, times the
// bin's node share, is added to every sub-region (small windows, small N)
constexpr uint32_t kXRoundNodes = 2048;
constexpr uint32_t kWinSlotsPerBucket = 1u << 16;  // window cut: friend slots per fine bucket
                                                // (bounds the message buffers, not LDS)

// Device-driven window loop (gs_run / gs_step of an unsharded one-trial
// context): the window's start, length and the poll rule's counters live on
// the device, so the host enqueues windows without waiting for any of them.
struct WinCtl {
  uint32_t t, L, tnext, tend;        // window start, length; next start; first tick not run
  uint32_t poll, pbase, stop, lmax;  // polls at pbase + k*poll (0: none); 1 + GS_RUN_* once stopped
  unsigned long long Tn, T;          // broadcasts firing in the window, their friend slots
  unsigned long long recv, crashed, pending, cover, max_ticks;  // poll rule state
  unsigned long long cmsg_cap, fmsg_cap;  // message buffer capacities (elements)
  unsigned long long xs_cap, xr_cap;      // device-driven shard windows of ranks: send / receive block buffers
};
constexpr uint32_t kStageWords = 8 + 16 * 8;  // per-window staging: snapshot + per-tick rows

struct WinState {
  const uint8_t* deg;
  const uint32_t* ids;
  unsigned long long* recv;
  unsigned long long* crash;
  uint32_t* rollw;               // [2W] nodes with a crash-roll receipt in the window (k_part2 -> k_resolve)
  uint32_t* rlmsg;               // [nfine][kRolledCap] receipts at rolled nodes (k_resolve -> k_resolve_rolled)
  uint32_t* rlcnt;               // [nfine] their counts (zeroed by the consumer)
  unsigned long long* stats;
  uint32_t* err;
  uint32_t* fcount;              // [R][nfine] fire-list lengths
  uint16_t* flist;               // [R][nfine][16384] local ids of firing nodes
  unsigned long long* usize;     // [L*nfine + 1] fires per unit (bucket f, tick k), u = f*L + k
  unsigned long long* unit_off;  // [L*nfine + 1] exclusive scan of usize
  unsigned long long* tfires;    // [kMaxWindow] fires per tick of the window (host-zeroed)
  uint32_t* gmap;                // [ceil(fires/64)] unit of every 64th firing index
  const uint32_t* pk;            // rows <= 6 slots: the sealed rows packed 5 per 128-B line, or null
  uint32_t noxcd;                // 1: k_part2 tiles in region order (GS_PART2_NOXCD=1, A/B); else dealt by XCD
  uint32_t nopair;               // 1: k_expand's packed rows fetched per lane (GS_XPAIR=0, A/B); else by lane pairs
  uint32_t* cmsg;                // coarse regions: u_in_coarse | k << 22
  uint32_t* fmsg;                // fine regions:   u_in_fine   | k << 14
  unsigned long long* chist;     // [kRegions] exact coarse region counts (fallback)
  unsigned long long* ccap;      // [kRegions + 1] coarse region starts, region = bin * csub + sub
  const unsigned long long* ccap_end;  // [kRegions] region ends (null: ccap[r + 1])
  unsigned long long* cfill;     // [kRegions] coarse region fill
  uint32_t* tprefix;             // [kRegions + 1] part2 tiles per coarse region (prefix)
  unsigned long long* fhist;     // [ncoarse*256 + 1] exact fine counts (fallback)
  unsigned long long* fstart;    // [nfine + 1] fine region starts
  unsigned long long* ffill;     // [nfine] fine region fill
  unsigned long long* tsum;      // [ncoarse][kMaxWindow] fires per (256-bucket tile, tick) (k_units)
  unsigned long long* toff;      // [ncoarse + 1] device-driven windows: firing index of each tile's first unit (k_cut)
  unsigned long long* sstats;    // [kStatShards][kMaxWindow][kStatFields] per-window partial counters
  unsigned long long* dbg;       // diagnostic phase stamps (GS_STAMPS=1), else null
  // batched trials: [trials][kMaxWindow][kTStatFields] per-window counters of every
  // trial (null for a single-trial context)
  uint32_t* tstat;
  uint32_t tofs;                 // tstat row of the window's first tick (ticks since the rows were zeroed)
  WinCtl* ctl;                   // device-driven windows (null: the host passes t0 / L)
  unsigned long long* stage;     // [slots][kStageWords] per-window results for the host (device-driven)
  uint32_t lstride;              // unit layout stride: units u = f * lstride + k
  uint32_t slots;                // longest row in use (<= stride: rows may be padded for 16-B loads)
  // Regions per coarse bin: kCoarseSub, or G * kCoarseSub in a shard's receive
  // layout (region = bin * csub + sender * kCoarseSub + sub)
  uint32_t csub;
  // receive layout: region starts / ends carry a source in bits 56..63, the
  // buffer csrc[source] their offsets index (a sender's own message buffer,
  // read in place, or the blocks received from other devices / ranks);
  // null: every region indexes cmsg
  const uint32_t* const* csrc;
  // node-range shard (owner expand): k_expand bins a kept message by its
  // target's owner d and the 2^22-node chunk of d's range, bin = d * obins +
  // chunk, message = target - d's first node within the chunk
  uint32_t owner;                // 1: bin by owner
  uint32_t obins;                // bins per owner (256 / G)
  uint32_t oseg_q, oseg_magic;   // seg_per >> 14 and ceil(2^32 / oseg_q): owner d of a target
  uint32_t abort_on_err;         // host-driven shard windows: an overflowed window's later kernels skip
  uint32_t G, rank;              // shards, this shard's index
  uint32_t seg_per;              // nodes per shard (shard r owns [r*seg_per, ...))
  // Device-driven shard windows (dd = 1; section 6.6 of DESIGN.md): every
  // shard's per-tick fire counts are gathered in gcnt ([G][kMaxWindow], this
  // shard's row is tfires) and its region fills, overflow flags and fine
  // buffer capacity in glay ([G][kDDRow], this shard's row is cfill), so each
  // shard cuts the same window and computes its receive layout on the device.
  // Only kErrAbort (set by k_rtab when any shard overflowed) stops a window;
  // kErrFine makes the receive side re-partition exactly in the same window
  // (the guard kernels run only then).
  uint32_t dd;
  uint32_t guard;                // 1: this launch runs only if the shard's kErrFine is set
  uint32_t solo;                 // device-driven single in-process shard: its send layout is its
                                 // receive layout (no k_rtab, no in-window fine redo); any
                                 // overflow stops the window and the host redoes it
  unsigned long long* gcnt;
  unsigned long long* glay;
  unsigned long long* wstat;     // [kMaxWindow][kStatFields] the window's counters (this shard's, then global)
  uint64_t nglob;                // nodes of the whole broadcast
  uint64_t n, W;
  uint32_t nfine, ncoarse, R, stride, stride_magic;
  int32_t delay_low;
  uint32_t delay_span;
  int32_t kd, kc;
  // Philox node keys: a node's global id is g = base + local id; batched trials lay
  // trial i's nodes out at i << tlog, so the key node is g & tmask and the key
  // trial is key.trial + (g >> tlog) (tlog = 32: one trial)
  uint32_t base;
  uint32_t tlog, tmask;
  uint32_t tnodes;  // batched trials: nodes per trial (k_plan's fine estimate); 0: one trial
  Key key;
};
constexpr uint32_t kStatShards = 32;  // per-window counter copies (k_close reads them all: 32 KB)
constexpr uint32_t kStampPhases = 10;
constexpr uint32_t kXStamp0 = 2 * kStampPhases;  // k_expand phases (GS_XSTAMPS builds) after k_resolve's
constexpr uint32_t kDbgWords = kXStamp0 + 8;
// per-trial window counters (batched trials)
enum TStat : uint32_t { TS_FIRED = 0, TS_SENT = 1, TS_DEAD = 2, TS_RECV = 3, TS_CRASH = 4 };
constexpr uint32_t kTStatFields = 8;

// Key (node, counter word 3) of global id g for a draw of `kind`.
__host__ __device__ __forceinline__ void node_key(uint32_t tlog, uint32_t tmask, const Key& key,
                                                  uint64_t g, uint32_t kind, uint32_t& node,
                                                  uint32_t& c3) {
  node = (uint32_t)(g & tmask);
  c3 = ctr3(kind, key.trial + (uint32_t)(g >> tlog));
}

constexpr uint32_t kErrArrivals = 4;  // > 65535 arrivals at one node in one tick (both engines)
constexpr uint32_t kErrCoarse = 8;    // a coarse region overflowed its estimate
constexpr uint32_t kErrFine = 16;     // a fine region overflowed its estimate
constexpr uint32_t kErrAbort = 32;    // device-driven shard windows: a shard's window overflowed, every shard stops
constexpr uint32_t kErrNoMem = 64;    // host-driven shard windows: a shard could not allocate (every rank returns)
// device-driven shard windows: a row of glay = kRegions fills, the flag word
// (kErrCoarse), the capacities (elements) of the shard's fine buffer and, for
// ranks, of its send / receive block buffers
constexpr uint32_t kDDRow = kRegions + 4;
constexpr uint32_t kDDWStat = kMaxWindow * kStatFields + 8;  // wstat words: rows, then flags (kErrArrivals, redos)
// A shard's receive layout (gs_ctx::d_rtab): region starts, ends, fills, its
// own pack offsets ([kRegions + 1] each), then the source buffers (<= 257
// pointers), the window's received messages in the last word.
constexpr size_t kRtabWords = 4 * (kRegions + 1) + 260;
constexpr size_t kRtabTotal = kRtabWords - 1;

hipError_t win_units(const WinState& w, uint32_t t0, uint32_t L, hipStream_t s);
// device-driven windows (w.ctl set, w.lstride = ctl->lmax)
hipError_t win_cut(const WinState& w, unsigned long long budget, hipStream_t s);
hipError_t win_unitscan(const WinState& w, hipStream_t s);
hipError_t win_close(const WinState& w, uint32_t slot, hipStream_t s);
hipError_t win_scan_units(const WinState& w, uint32_t L, void* tmp, size_t& tmp_bytes, hipStream_t s);
hipError_t win_groupmap(const WinState& w, uint32_t L, hipStream_t s);
hipError_t win_expand(const WinState& w, uint32_t t0, uint32_t L, uint64_t Tn, int mode,
                      hipStream_t s);
// win_expand's grid for Tn firing nodes (returned) and firing nodes per round
uint32_t win_expand_geometry(const WinState& w, uint64_t Tn, uint32_t* per_round, uint32_t* bsz,
                             uint32_t* npt);
hipError_t win_plan(const WinState& w, bool exact, hipStream_t s);
hipError_t win_scan_fine(const WinState& w, void* tmp, size_t& tmp_bytes, hipStream_t s);
hipError_t win_part2(const WinState& w, uint64_t T, bool scatter, hipStream_t s);
hipError_t win_resolve(const WinState& w, uint32_t t0, uint32_t L, hipStream_t s);
hipError_t win_pack_rows(const uint32_t* ids, uint64_t n, uint32_t* pk, hipStream_t s);
hipError_t win_seal_rows(const uint8_t* deg, uint32_t* ids, uint64_t n, uint32_t stride,
                         hipStream_t s);
hipError_t win_stats_reduce(const WinState& w, uint32_t t0, uint32_t L, hipStream_t s);
// node-range shards
hipError_t win_consume_sh(const WinState& w, uint32_t t0, uint32_t L, hipStream_t s);
// device-driven shard windows (w.dd): the receive layout of shard w.rank from
// the gathered fills (rtab as gs_api.cpp's shard_exchange lays it out;
// ccaps[s] = sender s's region starts, in place unless `travels`; src[] the
// layout's source buffers); the exact fine re-partition guarded by kErrFine;
// the window's counters into w.wstat; the close over the G shards' wstat
// (wstats / ctls: the group's shards, or this rank's own after the
// all-reduce) with gs_run's poll rule and the host staging slot.
hipError_t win_rtab(const WinState& w, unsigned long long* rtab, const unsigned long long* const* ccaps,
                    const uint32_t* const* src, uint32_t nsrc, uint32_t travels, hipStream_t s);
hipError_t win_fine_redo(const WinState& w, uint64_t T, hipStream_t s);
hipError_t win_stats_dd(const WinState& w, uint32_t slot, hipStream_t s);  // w.solo: also closes
// The M device-driven shard windows of an in-process group (one device): each
// small per-shard kernel is one launch for all M (the window states in device
// memory: send side ws, receive side wr, wr with guard = 1 for the fine redo)
struct WinGroup {
  const WinState* ws;
  const WinState* wr;
  const WinState* wg;
  uint32_t M;
  uint32_t nfine_max;
  uint32_t ncoarse_max;
  uint32_t slots_max;  // the longest row (k_expand's variant)
};
hipError_t win_units_g(const WinGroup& g, uint32_t L, hipStream_t s);
hipError_t win_cut_g(const WinGroup& g, unsigned long long budget, hipStream_t s);
hipError_t win_unitscan_g(const WinGroup& g, hipStream_t s);
hipError_t win_rtab_g(const WinGroup& g, const unsigned long long* const* ccaps, const uint32_t* const* src,
                      uint32_t nsrc, hipStream_t s);
// k_plan + k_part2 scatter of every shard's receive side, then the guarded
// exact fine redo (win_fine_redo)
hipError_t win_recv_g(const WinGroup& g, uint64_t T, hipStream_t s);
hipError_t win_stats_dd_g(const WinGroup& g, uint32_t slot, hipStream_t s);
// k_expand (mode 1: write + per-tick stats) and the resolve of every shard,
// each shard on a 1/M slice of the persistent grid
hipError_t win_expand_g(const WinGroup& g, uint32_t L, hipStream_t s);
hipError_t win_resolve_g(const WinGroup& g, uint32_t L, hipStream_t s);
hipError_t win_close_dd(const WinState& w, const unsigned long long* const* wstats, WinCtl* const* ctls,
                        uint32_t n, uint32_t slot, hipStream_t s);
// Copies the first min(cfill[r], room) messages of every region r < nreg from
// w.cmsg to out + poff[r] (the all-to-all's send blocks, back to back);
// regions with poff[r] = ~0 stay where they are.
hipError_t win_pack(const WinState& w, const unsigned long long* poff, uint32_t nreg, uint32_t* out, hipStream_t s);
// Schedule local node `node` (batched: in every trial; ~0u: each trial's keyed sender) at `tick`.
hipError_t win_schedule(const WinState& w, uint32_t node, uint32_t tick, uint32_t trials, uint32_t n,
                        hipStream_t s);

// Push-pull extension (gs_pushpull.hip): one round per tick; `next` is the
// informed set being built (equal to recv at the start of every round).
// sum = pp_summary_total_words(W) words: the round's word summaries, one bit
// per 64-node word (A: any informed, B: any live uninformed) and a second
// level with one bit per summary word (rebuilt by pp_round).
inline uint64_t pp_summary_words(uint64_t W) { return (W + 63) / 64; }
inline uint64_t pp_summary2_words(uint64_t W) { return (pp_summary_words(W) + 63) / 64; }
inline uint64_t pp_summary_total_words(uint64_t W) { return 2 * pp_summary_words(W) + 2 * pp_summary2_words(W); }
//
// Sparse early rounds: while |I| <= thr the round walks the informed list
// instead of streaming the table -- each informed u makes its own call, and
// the uninformed callers that pull from u are found among u's in-edges
// (reverse table: in-edges (v, j) with ids[v*stride + j] = u, of node u at
// [u ? rend[u-1] : 0, rend[u])).  The round's mode is decided on the device
// (k_pp_mode) from PPCtl, so rounds stay queued without host syncs.
// Dense rounds come in two directions.  Top-down (PP_DENSE, k_pp_round):
// every informed caller's push is an atomicOr into its friend's word.
// Bottom-up (PP_BOTTOM, k_ppb_round), once ninf > bthr: an uninformed live
// node u finds the pushes it receives among its in-edges (v, j) -- v's keyed
// pick is slot j, the call is kept and v is informed -- so the round issues no
// global atomic and an informed caller reads no friend id at all.  Once
// ninf >= bthr (dense rounds only: the early test comes first).  Needs the
// reverse table with packed slots (stride <= 16) and, with a failure mask,
// fmask (stride <= 8).
// Pull-answer (PP_ANSWER, k_ppa_round), for the middle rounds between the
// sparse and the bottom-up ones (ninf >= athr): informed nodes answer the
// pulls -- an informed u scans its in-edges (v, j) and informs v when v's pick
// is slot j, kept, and v is live and uninformed -- so the uninformed callers'
// random gathers of their picks' words (most of which fail) are not made;
// informed callers push as in the top-down round.
enum PPMode : uint32_t { PP_DENSE = 0, PP_EARLY = 1, PP_BOTTOM = 2, PP_ANSWER = 3 };
// rslot entries: slot j in bits 0..3 and deg(v) - 1 in bits 4..7 when
// stride <= 16 (the caller's pick needs no deg[v] gather), else j alone.
__host__ __device__ inline bool pp_rslot_packed(uint32_t stride) { return stride <= 16; }
// The informed list is kPPSegs segments of seg_cap entries; workgroup b
// appends to segment b % nseg (one counter per segment: a single append
// counter saturated at ~1e8 atomics/s).  A full segment sets ovf: the round
// still commits exactly (from the bitsets) and later rounds are dense.
constexpr uint32_t kPPSegs = 256;
struct PPCtl {
  unsigned long long ninf;      // |I|: informed nodes (all modes)
  unsigned long long thr;       // early rounds while ninf <= thr
  unsigned long long bthr;      // dense rounds bottom-up once ninf >= bthr (0: always, ~0: never)
  unsigned long long athr;      // other dense rounds pull-answer once ninf >= athr (~0: never, top-down)
  unsigned long long ncallers;  // live nodes with a non-empty row: calls per round
  unsigned long long nlive0;    // live nodes with an empty row (0: every live node calls)
  unsigned long long seg_cap;   // entries per segment
  uint32_t nseg;                // segments in use (<= kPPSegs)
  uint32_t mode;                // PPMode of the current round
  uint32_t early_ok;            // the informed list is complete (never re-entered)
  uint32_t ovf;                 // a segment overflowed this round
  uint32_t nearly, nbottom;     // rounds run sparse / bottom-up since the broadcast began (gs_timing)
  uint32_t nanswer, pad_;       // rounds run pull-answer
  unsigned long long segcnt[kPPSegs];      // entries in segment s (incl. this round's appends)
  unsigned long long seglen[kPPSegs];      // entries at the start of this round
  unsigned long long segpre[kPPSegs + 1];  // prefix of seglen: list index -> segment
};
struct PPSparse {
  PPCtl* ctl;                   // null: dense rounds only
  uint32_t* ilist;              // [nseg][seg_cap] informed nodes, per segment in order of informing
  const unsigned long long* rend;  // [n] end of node u's in-edges
  // the dense rounds' compact view of rend (null: read rend): node u's in-edges
  // end at rbase[u >> 6] + rend16[u] and start at rbase[u >> 6] (u % 64 == 0)
  // or rbase[u >> 6] + rend16[u - 1] -- 2.1 B per node instead of 8
  const uint16_t* rend16;       // [n]
  const unsigned long long* rbase;  // [ceil(n / 64)] start of node 64w's in-edges
  const uint32_t* rsrc;         // [E] caller v of each in-edge
  const uint8_t* rslot;         // [E] its slot j
  const uint8_t* fmask;         // [n] bit j: friend j is failed (stride <= 8 and a mask set), else null
  const unsigned long long* fany;  // [W] bit v: fmask[v] != 0 (with fmask), else null
  const uint32_t* rfail;        // [ceil(E / 32)] bit q: in-edge q's caller is failed (with fmask, unsharded), else null
  // Deferred sets of the pull-answer rounds (unsharded contexts, n <= 2^30;
  // null: atomicOr): the round's "x is informed" updates go to per-block
  // lists ([kPPDLists][dcap]), a coarse LDS partition by x >> 22 into
  // [kPPDRegions][ccap], a fine one into [nfine][fcap] by x >> 14, then one
  // workgroup per 16384-node bucket ORs them into `next` from an LDS bitmap:
  // streamed writes instead of random atomics.  A full list or region falls
  // back to atomicOr for what does not fit.  dcnt: the fills (lists, coarse
  // regions, fine regions), zeroed before every round.
  uint32_t* dset;
  unsigned long long* dcnt;
  uint64_t dcap, ccap, fcap;
  // bottom-up rounds: an informed caller's degree byte is not loaded when
  // every live node calls and no failed-slot mask is set (GS_PP_NODEG=0: load)
  uint32_t nodeg;
  uint32_t pullfirst;  // bottom-up: skip the in-edge scan of a node whose own pull succeeded (GS_PPB_PULLFIRST=0: scan, A/B)
  uint32_t word_maxi;  // k_ppa_round (words != 0): a range goes by word if no word holds more informed nodes
  uint32_t word_maxu;  // words == 2: a range goes by word if no word holds more live uninformed nodes
  uint32_t words;  // k_ppb_round with nodeg: 2 a lane per bitset word in ranges with few uninformed nodes, 1 always, 0 never
};
constexpr uint32_t kPPDLists = 512;    // = k_ppa_round's grid (kPPSGrid)
constexpr uint32_t kPPDRegions = 2048; // 256 coarse bins x 8 (XCD) sub-regions
hipError_t pp_round(const DevState& s, unsigned long long* next, unsigned long long* sum, uint32_t t,
                    bool l2_only, const PPSparse& sp, hipStream_t st);
hipError_t pp_live_edges(const DevState& s, uint32_t* out, hipStream_t st);
hipError_t pp_commit(const DevState& s, const unsigned long long* next, uint32_t t, const PPSparse& sp,
                     hipStream_t st);
// Sender informed unless failed; flag = 1 if informed.  Also initialises ctl
// with the live callers and the live nodes with an empty row: counted (a pass
// over deg and the failed mask) when callers is null, else callers[0..1] as
// counted before for the same table and mask.
hipError_t pp_seed(const DevState& s, unsigned long long* next, uint32_t node, uint32_t* flag,
                   const PPSparse& sp, unsigned long long thr, unsigned long long bthr, unsigned long long athr,
                   const unsigned long long* callers, hipStream_t st);
// Reverse table: rend must hold n + 1 words of scratch-free u64 space; tmp /
// tmp_bytes the hipcub scan workspace (pp_rev_scan_bytes).
size_t pp_rev_scan_bytes(uint64_t n);
hipError_t pp_rev_build(const DevState& s, unsigned long long* rend, uint32_t* rsrc, uint8_t* rslot, void* tmp,
                        size_t tmp_bytes, hipStream_t st);
// The same table by partitioning the edges (no random atomic per edge;
// temporaries ~17 B per edge, in as many passes over the coarse bins as the
// device allocator's largest block needs; *passes_out = the passes).  An
// error leaves the outputs unspecified (pp_rev_build then builds them).
// rend16 / rbase (PPSparse) from rend; *ovf = 1 where a 64-node block's
// in-edges pass 65,535 (the view is then not used)
hipError_t pp_rev_compact(const unsigned long long* rend, uint64_t n, uint16_t* rend16, unsigned long long* rbase,
                          uint32_t* ovf, hipStream_t st);
hipError_t pp_rev_build_part(const DevState& s, unsigned long long* rend, uint32_t* rsrc, uint8_t* rslot,
                             hipStream_t st, uint32_t* passes_out);
// fmask from the reverse table and the failed mask (stride <= 8).
hipError_t pp_fmask_build(const DevState& s, const unsigned long long* rend, const uint32_t* rsrc,
                          const uint8_t* rslot, uint8_t* fmask, hipStream_t st);
// Node-range shards of a push-pull run (SURVEY.md 8(e)2 for the C5 extension):
// every round is bottom-up on the shard's own nodes [gbase, gbase + n) against
// the replicated informed set (grecv), which the shards all-gather before
// each round.  Reverse table of the targets in [lo, hi) from the full table
// (deg/ids of nfull nodes; rend indexed by target - lo, rsrc global callers).
// (count + scan: rend[0..n] = exclusive prefix, rend[n] = the range's in-edges;
// then the fill, which leaves rend[i] = the end of target lo + i's edges)
size_t pp_rev_range_scan_bytes(uint64_t n);
hipError_t pp_rev_count_range(const uint8_t* deg, const uint32_t* ids, uint64_t nfull, uint32_t stride, uint64_t lo,
                              uint64_t hi, unsigned long long* rend, void* tmp, size_t tmp_bytes, hipStream_t st);
hipError_t pp_rev_fill_range(const uint8_t* deg, const uint32_t* ids, uint64_t nfull, uint32_t stride, uint64_t lo,
                             uint64_t hi, unsigned long long* rend, uint32_t* rsrc, uint8_t* rslot, hipStream_t st);
// fmask of the shard's own callers from their rows and the replicated failed set.
hipError_t pp_fmask_rows(const DevState& s, uint8_t* fmask, hipStream_t st);
// fany bit v = (fmask[v] != 0), W = ceil(n / 64) words.
hipError_t pp_fmask_any(const uint8_t* fmask, uint64_t n, unsigned long long* fany, hipStream_t st);
// rfail bit q = (rsrc[q] is failed), q < rend[n - 1].
hipError_t pp_rfail_build(const DevState& s, const unsigned long long* rend, const uint32_t* rsrc,
                          const uint8_t* rslot, uint32_t* rfail, hipStream_t st);
// One sharded round in `mode` (PP_BOTTOM: k_ppb_round into next, the shard's
// own words; PP_ANSWER: k_ppa_round into gnext, a bitset by global id whose
// bits in other shards' ranges go to their owners); commit with pp_commit.
hipError_t pp_round_shard(const DevState& s, unsigned long long* next, unsigned long long* gnext, uint32_t t,
                          const PPSparse& sp, uint32_t mode, hipStream_t st);
// *out = popcount(words[0, nwords)) (stream-ordered).
hipError_t pp_count(const unsigned long long* words, uint64_t nwords, unsigned long long* out, hipStream_t st);
// dst[w] |= src[i * words + w] for i < nslices.
hipError_t pp_or_slices(unsigned long long* dst, const unsigned long long* src, uint32_t nslices, uint64_t words,
                        hipStream_t st);

// Launchers (gs_broadcast.hip).
hipError_t launch_tick(const DevState& st, uint32_t tick, int mode, hipStream_t s);
hipError_t launch_slot_reset(const DevState& st, uint32_t slot, hipStream_t s);
hipError_t launch_schedule_one(const DevState& st, uint32_t node, uint32_t tick, hipStream_t s);
uint32_t tick_grid(const DevState& st);

// Overlay builder (gs_overlay.hip).
struct OverlayResult {
  uint64_t final_tick;
  int rc;  // GS_* code
  char msg[160];
};
struct OverlayWindowSink {
  void (*push)(void* self, uint64_t tick, uint64_t makeups, uint64_t breakups);
  void* self;
};
// Device buffers the overlay builder keeps between builds (one per context).
struct OverlayWork {
  // p = raw + off: a bucket's data starts `off` bytes into its allocation
  // (staggered per ring slot, see gs_overlay.hip)
  struct Buf { void* p = nullptr; size_t bytes = 0; void* raw = nullptr; size_t off = 0; };
  std::vector<Buf> bucket;  // per arrival slot
  Buf scratch, outb, oslotb, cub_tmp, meta;
  Buf fine, ovp;            // destination partition of the dense ticks: regions, plan + fills
  uint64_t part_ticks = 0, sort_ticks = 0, part_fallbacks = 0;  // of the last build
  uint64_t pick_fallbacks = 0;  // the last build's tick-0 plan overflowed (then counted)
};
void overlay_free(OverlayWork* ws, hipStream_t st);
// n = nodes per trial; trials > 1 builds every trial's overlay at once in the
// id space trial << tlog | node (tlog = 32 for one trial).
int overlay_build(uint64_t n, uint32_t trials, uint32_t tlog, int32_t fanout, int32_t fanin,
                  int32_t delay_low, int32_t delay_high, Key key, uint8_t* d_deg, uint32_t* d_ids,
                  uint32_t stride, uint64_t max_ticks, hipStream_t stream, OverlayWindowSink sink,
                  OverlayResult* res, OverlayWork* ws);

}  // namespace gs
