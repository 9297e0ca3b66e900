/*
 * gossip.h -- C ABI of libgossip_hip.so, the MI355X (gfx950) engine for the
 * broadcast round loop of go-distributed/gossip_simulator (simulator.go).
 *
 * The reference has no FFI/plugin seam: it is one Go `package main`.  This ABI
 * is the seam a maintainer adds behind its `main` (simulator.go:207-253); each
 * entry point names the reference code it replaces.  A cgo binding is shown in
 * INTEGRATION.md.
 *
 * Conventions
 *  - return 0 on success, <0 on error (GS_E*); message via gs_last_error().
 *  - all caller buffers are caller-owned and copied during the call; nothing
 *    is retained across calls (cgo pointer rules).
 *  - one gs_ctx is single-threaded.  gs_create gives one HIP device and one
 *    stream; gs_create_multi spreads one context over several devices (or
 *    several shards of one device) and gs_create_rank makes one shard of a
 *    multi-process (RCCL) run -- every other call is the same for all three.
 *  - node ids are uint32 (n <= 2^31-1); friend rows are uint32[stride] with a
 *    uint8 length per node (a friends list is at most 255 long).
 *  - every random decision is drawn from Philox4x32-10 keyed by
 *    (seed; kind, trial, tick, node, slot) -- see DESIGN.md "Tick model".
 */
#ifndef GOSSIP_H
#define GOSSIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GS_ABI_VERSION 6

enum {
  GS_OK = 0,
  GS_EINVAL = -1,     /* bad parameter or call order                          */
  GS_ELIVELOCK = -2,  /* overlay never stabilised (fanin <= fanout livelock)  */
  GS_EREJECT = -3,    /* replacement-friend rejection exhausted (n <= 2)      */
  GS_ENOMEM = -4,     /* host or device allocation failed                     */
  GS_EDEVICE = -5,    /* HIP runtime error / no gfx950 device                 */
  GS_EOVERFLOW = -6   /* a counter exceeded its range                         */
};

/* Flags (gs_params.flags). */
#define GS_FLAG_TIMING 1u /* time every tick kernel with HIP events (gs_timing) */
#define GS_FLAG_TICK_ENGINE 2u /* force the per-tick atomic engine (default: window engine) */
#define GS_FLAG_PP_L2_ONLY 4u  /* push-pull: skip the LDS-staged second-level summaries (the path
                                * N > ~1.02e9 takes); read at gs_create, for tests */
#define GS_FLAG_PP_DENSE 8u    /* push-pull: every round streams the whole table (no reverse
                                * table, no sparse early rounds); same results, for tests */
#define GS_FLAG_PP_EARLY 16u   /* push-pull: sparse early rounds at any informed count (default:
                                * while |I| <= n/256); same results, for tests */
#define GS_FLAG_PP_TOPDOWN 32u /* push-pull: dense rounds always push by atomics (default: bottom-up,
                                * receivers scan their in-edges, once |I| >= 96n/256); same results */
#define GS_FLAG_PP_BOTTOM 64u  /* push-pull: every dense round bottom-up; same results, for tests */
#define GS_FLAG_PP_ANSWER 128u /* push-pull: every dense round below the bottom-up threshold pull-answer
                                * (informed nodes answer the pulls among their in-edges; the default
                                * does too unless GS_PP_ANSWER256 is set); same results, for tests */

/* Dissemination model (gs_params.model). */
#define GS_MODEL_FLOOD 0u    /* the reference: every receipt re-broadcasts to all friends (simulator.go:107-149) */
#define GS_MODEL_PUSHPULL 1u /* extension (config C5), no reference counterpart: one synchronous
                              * round per tick; each live node calls one Philox-picked friend,
                              * informed callers push, uninformed callers pull; -droprate loses
                              * calls, -crashrate is unused, gs_set_failed masks nodes
                              * (oracle/gsoracle.h) */

/* simulator.go:11-20 (Parameters) + the additive -seed/-trial knobs. */
typedef struct gs_params {
  uint64_t n;          /* -n          simulator.go:187                       */
  int32_t fanout;      /* -fanout     simulator.go:188                       */
  int32_t fanin;       /* -fanin      simulator.go:189 (default 6, see :189) */
  int32_t delay_low;   /* -delaylow   simulator.go:190 (ms = ticks)          */
  int32_t delay_high;  /* -delayhigh  simulator.go:191                       */
  double drop_rate;    /* -droprate   simulator.go:192 -> int(rate*100) %    */
  double crash_rate;   /* -crashrate  simulator.go:193 -> int(rate*100) %    */
  uint64_t seed;       /* Philox key                                          */
  uint32_t trial;      /* Philox counter word 3, low 24 bits                  */
  int32_t device;      /* HIP device ordinal                                  */
  uint32_t flags;      /* GS_FLAG_*                                           */
  uint32_t model;      /* GS_MODEL_* (0 = the reference's push flooding)      */
  /* Batched independent trials (config C3): trials trial .. trial+trials-1 of n
   * nodes each, run at once (one overlay, one broadcast per trial, keyed by
   * its trial number exactly as a one-trial context).  0 or 1 = one trial.
   * The reference runs one trial per process (simulator.go:207-253). */
  uint32_t trials;
  uint32_t reserved0_;
  uint64_t reserved_[5];
} gs_params;

/* One tick (1 ms) of the broadcast phase; the reference exposes these as the
 * int32 atomics of simulator.go:26-31, read by main's poll loop (:243-253). */
typedef struct gs_tick_stats {
  uint64_t tick;      /* simulated ms since Broadcast() (:239-241)            */
  uint64_t fired;     /* Broadcast goroutines whose delay expired (:142)     */
  uint64_t sent;      /* friend slots not dropped = delivered sends (:144-145)*/
  uint64_t messages;  /* TotalMessage increments (:111)                      */
  uint64_t received;  /* TotalReceived, cumulative (:121)                    */
  uint64_t crashed;   /* TotalCrashed, cumulative (:114)                     */
  uint64_t pending;   /* broadcasts scheduled, not yet fired                  */
} gs_tick_stats;

/* One 10-ms poll window of overlay construction (simulator.go:222-234). */
typedef struct gs_window {
  uint64_t tick;      /* end of the window (ms)                               */
  uint64_t makeups;   /* MakeUps  in the window (:67)                         */
  uint64_t breakups;  /* BreakUps in the window (:77)                         */
} gs_window;

/* Device time spent in the broadcast kernels (GS_FLAG_TIMING), from HIP
 * events on the context's stream.  Tick engine: deliver = the per-tick
 * delivery kernel, resolve = its second (kc > 0) pass.  Window engine:
 * deliver = expand + partition (expand_ms + part_ms), resolve = k_resolve. */
typedef struct gs_timing {
  double deliver_ms;       /* sum over launches of the delivery kernel(s)    */
  double resolve_ms;       /* sum over launches of the resolve kernel        */
  uint64_t deliver_launches;
  uint64_t resolve_launches;
  double overlay_ms;       /* wall time of the last gs_build_overlay          */
  double expand_ms;        /* window engine: k_expand (row gather + coarse partition) */
  double part_ms;          /* window engine: k_plan + k_part2 (fine partition)        */
  uint64_t windows;        /* window engine: windows processed                */
  uint64_t exact_redos;    /* window engine: windows re-partitioned exactly   */
  double prep_ms;          /* push-pull: wall time of the last reverse-table / failed-slot-mask
                            * build (at gs_broadcast_begin, once per table / failure mask) */
  uint64_t pp_early_rounds;  /* push-pull: rounds of this broadcast run sparse (informed list)   */
  uint64_t pp_bottom_rounds; /* push-pull: dense rounds of this broadcast run bottom-up          */
  uint64_t pp_answer_rounds; /* push-pull: dense rounds of this broadcast run pull-answer        */
  uint64_t dd_fallbacks;     /* device-driven shard windows stopped by an overflow and redone
                              * host-driven (cumulative; a buffer that fits makes it stop growing) */
  uint64_t pp_rev_part;      /* push-pull: the passes of the last reverse table's partition build
                              * (>= 1), or 0 if the atomic count + fill built it (GS_PP_REV_ATOMIC, or a
                              * fallback) */
  uint64_t ov_part_ticks;    /* last overlay build: ticks grouped by the destination partition     */
  uint64_t ov_sort_ticks;    /* last overlay build: ticks grouped by the radix sort (sparse ticks,
                              * GS_OV_SORT=1, or a partition fallback)                              */
  uint64_t ov_part_fallbacks; /* last overlay build: partition plans that overflowed (then sorted) */
  /* Device memory, process-wide and cumulative since the library was loaded (every
   * context shares the library's cache of large blocks; see gs_trim).  The reference
   * allocates its nodes once per process (simulator.go:208-212). */
  double alloc_ms;           /* wall time inside hipMalloc                                      */
  double largest_alloc_ms;   /* the longest single hipMalloc                                    */
  double free_ms;            /* wall time inside hipFree and the cache's idle waits             */
  uint64_t alloc_calls;      /* hipMalloc calls                                                 */
  uint64_t alloc_cache_hits; /* device buffers served from the cache (no hipMalloc)             */
  uint64_t cached_bytes;     /* bytes the cache holds free now                                  */
  uint64_t coarse_redos;     /* window engine, host-driven windows: windows whose k_expand overflowed
                              * a coarse region estimate and ran again from exact counts (cumulative) */
} gs_timing;

/* gs_run status */
enum { GS_RUN_COVERED = 0, GS_RUN_QUIESCENT = 1, GS_RUN_MAX_TICKS = 2, GS_RUN_RUNNING = -1 };

/* One trial's outcome (batched trials, or the one trial of any flood context):
 * the counters at the poll that stopped it under gs_run's rule -- what the
 * reference prints at :252-253 -- plus the first tick it was covered. */
typedef struct gs_trial_stats {
  uint64_t trial;     /* trial number (Philox counter word 3)                 */
  uint64_t tick_99;   /* first tick with float32(recv)/float32(n) >= 0.99, else 0 */
  uint64_t tick;      /* tick of the stopping poll (or the last tick run)     */
  uint64_t fired, sent, messages, received, crashed;  /* cumulative at `tick` */
  int32_t status;     /* GS_RUN_* (GS_RUN_RUNNING: not stopped yet)          */
  int32_t reserved_;
} gs_trial_stats;

typedef struct gs_ctx gs_ctx;

int gs_version(void);
const char* gs_strerror(int code);

/* Replaces simulator.go:186-212 (flag globals, GlobalView/NewNode allocation).
 * Validates params exactly as the reference would fail: n == 0 (:240 panics),
 * delay_high <= delay_low (:167 panics).  One device (params.device). */
int gs_create(const gs_params* params, gs_ctx** out);

/* ---- multi-GPU (no reference counterpart: the reference runs every node as
 * a goroutine of one process, simulator.go:214-217) ----
 * One context over ndev devices (entries may repeat: several shards or trial
 * batches on one GPU).  params.trials > 1: the trials are split over the
 * devices and run with no communication.  Otherwise ONE broadcast whose node
 * range is split into ndev shards (config C4): every window each shard
 * expands its own firing nodes and hands every other shard the messages
 * addressed to its nodes (an all-to-all: device-to-device copies), then
 * resolves its own nodes; counters are summed.  Results are bit-identical to
 * gs_create's. */
int gs_create_multi(const gs_params* params, const int* devices, int ndev, gs_ctx** out);
/* Multi-process (one process per GPU): rank 0 calls gs_comm_unique_id and
 * ships the GS_COMM_ID_BYTES bytes to every rank; each rank calls
 * gs_create_rank.  A flood run is then node-range sharded over the ranks with
 * an RCCL all-to-all of each window's messages (grouped send/recv, after an
 * all-gather of the fire counts and the message layout) and an RCCL sum per
 * gs_step (every rank's
 * gs_step/gs_run/gs_totals return the global counters); a push-pull run
 * (rows <= 16 slots) is node-range sharded with an all-gather of the informed
 * set's owned words per round; params.trials > 1 gives each rank its share of
 * the trials (no communication, id may be NULL).  gs_create_multi splits both
 * models the same way over its devices. */
#define GS_COMM_ID_BYTES 128
int gs_comm_unique_id(uint8_t id[GS_COMM_ID_BYTES]);
int gs_create_rank(const gs_params* params, int device, int nranks, int rank,
                   const uint8_t* id, gs_ctx** out);
/* The same with the exchange done by the caller instead of RCCL (MPI, a
 * torch.distributed group, a test harness): every rank calls it with the same
 * nranks and its own rank, and the callbacks move HOST bytes between the
 * ranks -- all_gather: `bytes` from every rank into recv (nranks * bytes,
 * rank-major; send is this rank's part); all_reduce_sum_u64: element-wise sum
 * over the ranks of count uint64, in place; all_to_allv (flood runs): rank r
 * gets send_bytes[r] bytes of send (the blocks lie back to back in rank
 * order) and recv receives recv_bytes[r] bytes from every rank r, back to back
 * in rank order.  All return 0 on success and are called by every rank in the
 * same order.  Unlike every other argument the struct is kept: user and the
 * callbacks must stay valid until gs_destroy. */
typedef struct gs_exchange {
  void* user;
  int (*all_gather)(void* user, const void* send, void* recv, size_t bytes);
  int (*all_reduce_sum_u64)(void* user, uint64_t* buf, size_t count);
  int (*all_to_allv)(void* user, const void* send, const size_t* send_bytes, void* recv,
                     const size_t* recv_bytes);
} gs_exchange;
int gs_create_rank_exchange(const gs_params* params, int device, int nranks, int rank, const gs_exchange* ex,
                            gs_ctx** out);
/* Nodes [lo, hi) owned by shard `index` of a context (index < *nshards);
 * an unsharded context is one shard [0, n). */
int gs_shard_info(const gs_ctx* ctx, uint32_t index, uint32_t* nshards, uint64_t* lo, uint64_t* hi);
void gs_destroy(gs_ctx* ctx);
const char* gs_last_error(const gs_ctx* ctx);

/* Injects a peer table in place of the overlay (the `friends` slices,
 * simulator.go:45,58).  deg[n] uint8, ids[n*stride] uint32 row-major.
 * Host buffers; copied.  Batched trials: trials tables back to back
 * (deg[trials*n], ids[trials*n*stride], ids local to their trial).  A sharded
 * context keeps only each shard's partition (gs_read_peers then fails). */
int gs_load_peers(gs_ctx* ctx, const uint8_t* deg, const uint32_t* ids, uint32_t stride);
/* Same, from device-resident buffers (copied device-to-device). */
int gs_load_peers_device(gs_ctx* ctx, const void* d_deg, const void* d_ids, uint32_t stride);
/* Copies the current table out (stride = max(fanout, fanin) after an overlay). */
int gs_read_peers(gs_ctx* ctx, uint8_t* deg, uint32_t* ids, uint32_t* stride_out);

/* Replaces simulator.go:62-106,127-164 (makeup/breakup handlers, Makeup,
 * Breakup, removeFriend) and the stabilisation loop :214-235, on the GPU.
 * Writes one gs_window per non-final poll (up to cap; *nwin gets the total)
 * and the stabilising poll's tick.  GS_ELIVELOCK after max_ticks. */
int gs_build_overlay(gs_ctx* ctx, uint64_t max_ticks, gs_window* win, size_t cap,
                     size_t* nwin, uint64_t* final_tick);

/* Pre-failed node mask (extension, config C5): words[ceil(n/64)], set bits
 * are crash-stopped before the broadcast: they never count nor forward, and
 * a failed sender does not broadcast (both models).  Not for batched trials. */
int gs_set_failed(gs_ctx* ctx, const uint64_t* words, size_t nwords);

/* Replaces simulator.go:239-241.  sender < 0 draws it from the keyed stream
 * like rand.Intn(len(GlobalView)) (per trial when batched).  The sender is NOT
 * marked received. */
int gs_broadcast_begin(gs_ctx* ctx, int64_t sender);
/* Advances `ticks` ticks of the receive/broadcast actors (simulator.go:107-123,
 * 140-149, 166-184); out[i] (may be NULL) gets each tick's stats. */
int gs_step(gs_ctx* ctx, uint32_t ticks, gs_tick_stats* out);
/* Replaces the poll loop simulator.go:243-251: steps `poll` ticks at a time
 * until float32(received)/float32(n) >= 0.99 at a poll (GS_RUN_COVERED), no
 * broadcast is pending (GS_RUN_QUIESCENT; the reference would spin forever;
 * push-pull: no call can change the informed set any more -- no live
 * informed node has a live uninformed friend and no live uninformed node has
 * an informed friend, or every call is dropped), or max_ticks.  out (may be
 * NULL) receives one gs_tick_stats per poll.  Batched trials: each trial
 * stops at its own poll (gs_trial_results); the run ends when all have. */
int gs_run(gs_ctx* ctx, uint32_t poll, uint64_t max_ticks, gs_tick_stats* out,
           size_t cap, size_t* nout, int32_t* status);
/* Cumulative totals so far (tick, fired/sent/messages summed). */
int gs_totals(gs_ctx* ctx, gs_tick_stats* out);

/* Per-trial outcomes, trials in order (cap entries; *nout gets the count). */
int gs_trial_results(gs_ctx* ctx, gs_trial_stats* out, size_t cap, size_t* nout);

/* Bitset dumps for per-round parity: words[ceil(n/64)], bit v of word v/64
 * (batched trials: trials x ceil(n/64) words, trial-major).  A rank of a
 * multi-process run fills only the words of the nodes it owns (others 0). */
int gs_read_received(gs_ctx* ctx, uint64_t* words, size_t nwords);
int gs_read_crashed(gs_ctx* ctx, uint64_t* words, size_t nwords);

int gs_timing_get(gs_ctx* ctx, gs_timing* out);
/* The same for shard `index` of a sharded (or batched) context's members;
 * index 0 of a one-device context is gs_timing_get. */
int gs_shard_timing(gs_ctx* ctx, uint32_t index, gs_timing* out);
/* Renumber the context's trial(s) to trial .. trial+trials-1 (Philox
 * counter word 3) between runs, keeping its device buffers: the overlay must
 * be built or loaded again before gs_broadcast_begin (config C3 runs batch
 * after batch in one context this way). */
int gs_set_trial(gs_ctx* ctx, uint32_t trial);
/* Replace gs_params.flags (e.g. toggle GS_FLAG_TIMING between runs). */
int gs_set_flags(gs_ctx* ctx, uint32_t flags);
/* Return to the state before gs_broadcast_begin: clears received/crashed,
 * the fire ring and the counters; keeps the peer table and failure mask
 * (a fresh process in the reference, simulator.go:207). */
int gs_reset(gs_ctx* ctx);

/* Run all later device work of a one-device context on `hip_stream` (a
 * hipStream_t owned by the caller); NULL restores the context's own stream. */
int gs_set_stream(gs_ctx* ctx, void* hip_stream);
/* Device-memory cache.  Device buffers of >= 64 MiB come from a process-wide
 * cache: a destroyed context's blocks (or a rebuilt table's temporaries) stay
 * mapped and serve the next context's requests, so a process that creates
 * context after context does not hand tens of GB back to the driver and ask
 * for them again (first allocations after large frees ran seconds slow on
 * some MI355X boxes).  gs_trim returns every free cached
 * block of `device` (-1: all devices) to the driver; *released (may be NULL)
 * gets the bytes.  The cache also trims itself before a hipMalloc the device
 * has no room for.  GS_DEVMEM_CACHE=0 in the environment disables it.  The
 * reference allocates once per process (simulator.go:208-212). */
int gs_trim(int device, size_t* released);
/* The device-memory fields of a gs_timing, alloc_ms .. cached_bytes, without a
 * context; every other field is zero. */
int gs_memory_stats(gs_timing* out);

/* ---- host-only helpers for the reference's stdout contract ------------- */
/* Go fmt %v of a float32 (strconv 'g', -1, 32), e.g. 99.61 or 9.9999994e-08
 * (simulator.go:247).  Returns the length written (NUL-terminated). */
size_t gs_format_float32(float x, char* buf, size_t cap);
/* Go fmt %v of a float64 (flag echo, simulator.go:199). */
size_t gs_format_float64(double x, char* buf, size_t cap);
/* Go time.Duration.String() of `ns` nanoseconds, e.g. 1.5s, 120ms, 1m0s. */
size_t gs_format_duration(int64_t ns, char* buf, size_t cap);
/* Go int(rate*100) (simulator.go:172,180), clamped to [0,100]. */
int32_t gs_threshold(double rate);
/* Philox4x32-10 (for replay tooling and tests). */
void gs_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);

#ifdef __cplusplus
}
#endif
#endif
