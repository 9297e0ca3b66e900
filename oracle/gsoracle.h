/*
 * gsoracle.h -- CPU restatement of go-distributed/gossip_simulator's broadcast
 * round loop and overlay protocol.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is part of the product:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it, and only as the checker / CPU baseline.  The product path
 * (gossip_simulator_amd/, libgossip_hip.so, gossip_sim) never links it.
 *
 * Parity status: UNPINNED by the reference.  The reference (simulator.go, Go,
 * no go.mod) has no tests, golden vectors or fixtures, and no Go toolchain
 * exists in this image, so it cannot be built or run (oracle/_ref is empty by
 * necessity; see DESIGN.md section "Oracle").  This restatement is pinned instead by
 * hand-derived known answers (tests/test_oracle_*.py): Philox KATs checked
 * against rocRAND's philox4x32_10 engine, BFS layers on ring/complete graphs,
 * drop=1.0, sender echo, Go's int(rate*100) quantisation, float32 99 %
 * thresholds; and statistically against the event-driven Go-like model
 * or_refsim() below.
 *
 * Two models live here:
 *   1. The tick model (or_overlay, or_engine_*): 1 tick = 1 ms, every random
 *      decision drawn from Philox4x32-10 keyed by (seed; trial, tick, node,
 *      slot).  This is the bit-exact spec the HIP engine must reproduce.
 *   2. or_refsim: an event-driven restatement that follows simulator.go more
 *      literally -- one sequential RNG stream consumed in processing order,
 *      events in a time-ordered FIFO queue -- used for KS tests of the
 *      rounds-to-coverage distribution ("native RNG" check).
 */
#ifndef GSORACLE_H
#define GSORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Philox stream kinds (counter word 3 = kind << 24 | trial). */
enum {
  OR_K_SENDER = 1,  /* simulator.go:240  rand.Intn(len(GlobalView))          */
  OR_K_DELAY = 2,   /* simulator.go:167  RandomNetworkDelay, per Broadcast    */
  OR_K_DROP = 3,    /* simulator.go:172  RandomDrop, per friend slot; the same
                     * draw's second base-100 digit is the message's RandomCrash
                     * roll (:180), or_drop_crash                               */
  OR_K_CRASH = 4,   /* reserved (round 2's separate crash-roll stream)          */
  OR_K_PICK = 5,    /* simulator.go:97   new-friend pick                      */
  OR_K_OVDELAY = 6, /* simulator.go:153,160 Breakup/Makeup delay              */
  OR_K_VICTIM = 7,  /* simulator.go:71   victim slot                          */
  OR_K_REPLACE = 8, /* simulator.go:86-89 replacement friend (rejection)      */
  OR_K_PUSHPULL = 9, /* push-pull extension: peer pick + loss, per (node, round) */
  OR_K_ORDER = 10    /* simulator.go:107-115 receipt order: position of the first
                      * crashing message among a (node, tick)'s receipts        */
};

/* or_engine_step / om_engine_step: more than 65535 arrivals at one node in one
 * tick overflow the 16-bit receipt count the engines pack (the HIP engine
 * returns GS_EOVERFLOW for the same input). */
#define OR_EOVERFLOW (-6)

/* Dissemination models (or_params.model). */
enum {
  OR_MODEL_FLOOD = 0,    /* the reference: push flooding (simulator.go:107-149)  */
  OR_MODEL_PUSHPULL = 1  /* extension (config C5), no reference counterpart      */
};

typedef struct or_params {
  uint64_t n;          /* -n         simulator.go:187 */
  int32_t fanout;      /* -fanout    simulator.go:188 */
  int32_t fanin;       /* -fanin     simulator.go:189 */
  int32_t delay_low;   /* -delaylow  simulator.go:190 */
  int32_t delay_high;  /* -delayhigh simulator.go:191 */
  double drop_rate;    /* -droprate  simulator.go:192 */
  double crash_rate;   /* -crashrate simulator.go:193 */
  uint64_t seed;       /* Philox key (additive flag -seed) */
  uint32_t trial;      /* Philox counter word 3 low 24 bits */
  uint32_t model;      /* OR_MODEL_* */
} or_params;

typedef struct or_tick_stats {
  uint64_t tick;
  uint64_t fired;    /* broadcasts whose delay expired this tick          */
  uint64_t sent;     /* friend slots not dropped (delivered sends)         */
  uint64_t messages; /* TotalMessage increments (simulator.go:111)         */
  uint64_t received; /* TotalReceived after this tick (cumulative, :121)   */
  uint64_t crashed;  /* TotalCrashed after this tick (cumulative, :114)    */
  uint64_t pending;  /* broadcasts scheduled but not yet fired             */
} or_tick_stats;

typedef struct or_window {
  uint64_t tick;     /* end tick of the 10-tick window (simulator.go:223) */
  uint64_t makeups;  /* MakeUps in the window  (simulator.go:67)          */
  uint64_t breakups; /* BreakUps in the window (simulator.go:77)          */
} or_window;

/* Go quantisation int(rate*100) (simulator.go:172,180), clamped to [0,100]. */
int32_t or_threshold(double rate);
/* Philox4x32-10, Random123 constants. */
void or_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
/* Receipt order (rule A6): the 1-based position of the first crashing
 * message when k receipts of node u at tick t, `ones` of them with a crash
 * roll (1 <= ones <= k), are taken in a uniformly random order -- sequential
 * draws U_{k-g+1} < ones from Philox{u, t, (g-1)/4, ORDER}, lane (g-1)%4.
 * k == 1 or ones == k needs no draw (position 1). */
uint32_t or_first_crash(const uint32_t key[2], uint32_t trial, uint32_t u, uint32_t t, uint32_t k,
                        uint32_t ones);
/* floor(r * m / 2^32): the uniform-in-[0,m) map shared with the HIP engine. */
uint32_t or_uniform(uint32_t r, uint32_t m);
/* RandomDrop (simulator.go:172) and the message's RandomCrash roll (:180)
 * from one draw r: drop = floor(100 r / 2^32), crash = floor(100 (100 r mod
 * 2^32) / 2^32) -- the first two base-100 digits of r / 2^32 (each of the
 * 10^4 pairs is taken by floor(2^32 / 10^4) or one more of the 2^32 words). */
void or_drop_crash(uint32_t r, uint32_t* drop, uint32_t* crash);
/* Sender chosen as simulator.go:240 does, from the keyed stream. */
uint64_t or_pick_sender(const or_params* p);

/* ---- overlay (simulator.go:62-106,127-164,214-235) ---------------------- */
/* deg[n], ids[n*fanin] (row stride = fanin).  Returns 0, or <0 on error:
 *  -1 bad params, -2 livelock (max_ticks exceeded; reference never
 *  stabilises when fanin <= fanout), -3 replacement rejection exhausted,
 *  -4 out of memory.  *final_tick = tick of the stabilising poll. */
int or_overlay(const or_params* p, uint8_t* deg, uint32_t* ids, or_window* win,
               size_t wcap, size_t* nwin, uint64_t max_ticks,
               uint64_t* final_tick);

/* ---- broadcast tick engine (simulator.go:107-123,140-149,237-253) ------- */
/* model OR_MODEL_PUSHPULL (extension; the reference only floods): one tick is
 * one synchronous round.  Every live node v with a non-empty friends list
 * draws r = Philox{v, t, 0, PUSHPULL}: peer u = friends[U_deg(r.x)], call lost
 * iff U_100(r.y) < int(droprate*100).  With I = the informed set at the start
 * of the round: v in I pushes to u (sent; delivered and u informed iff u is
 * live); v not in I pulls from u in I (sent, delivered, v informed).  Failed
 * nodes (or_engine_set_failed) never call, answer or become informed; the
 * crash rate is not used.  The sender is informed at begin (if live).
 * Per tick: fired = calls, sent = rumour transmissions not lost, messages =
 * those delivered to a live node, received = |I|, pending = |I|. */
typedef struct or_engine or_engine;
or_engine* or_engine_new(const or_params* p, const uint8_t* deg,
                         const uint32_t* ids, uint32_t stride);
void or_engine_free(or_engine* e);
/* sender < 0 -> keyed pick (simulator.go:240). */
int or_engine_begin(or_engine* e, int64_t sender);
/* Advance `ticks` ticks; out[i] = stats of each tick. */
int or_engine_step(or_engine* e, uint32_t ticks, or_tick_stats* out);
int or_engine_read_received(const or_engine* e, uint64_t* words, size_t nwords);
int or_engine_read_crashed(const or_engine* e, uint64_t* words, size_t nwords);
/* Pre-failed node mask (C5 extension): words of ceil(n/64); set bits crash-stop. */
int or_engine_set_failed(or_engine* e, const uint64_t* words, size_t nwords);
uint64_t or_engine_tick(const or_engine* e);
/* Node-range sharding (config C4): this engine owns nodes [lo, hi).  Every
 * rank evaluates every firing node of the (all-gathered) fire slot with the
 * same keyed draws, but only counts fired nodes it owns and only delivers to
 * targets it owns, so the union over ranks equals the unsharded run. */
int or_engine_set_range(or_engine* e, uint64_t lo, uint64_t hi);
/* Fire-ring slot that tick `tick` will process: copy out / overwrite. */
int or_engine_get_slot(const or_engine* e, uint64_t tick, uint64_t* words, size_t nwords);
int or_engine_set_slot(or_engine* e, uint64_t tick, const uint64_t* words, size_t nwords);

/* ---- event-driven Go-like model with a sequential RNG -------------------- */
typedef struct or_refsim_result {
  uint64_t tick_99;       /* first ms at which TotalReceived >= 99 % (float32 rule) */
  uint64_t poll_99;       /* first 10-ms poll that sees it (simulator.go:243-248)   */
  uint64_t messages;      /* TotalMessage at poll_99                                */
  uint64_t crashed;       /* TotalCrashed at poll_99                                */
  uint64_t received;      /* TotalReceived at poll_99                               */
  uint64_t sent;          /* kept sends up to poll_99                               */
  uint64_t overlay_ticks; /* ms until no overlay message remains in flight          */
  uint64_t deg_hist[256]; /* friends-list length histogram                          */
  int32_t reached;        /* 1 if 99 % was reached before the queue drained         */
  int32_t pad_;
} or_refsim_result;
int or_refsim(const or_params* p, uint64_t rng_seed, uint64_t max_ms,
              or_refsim_result* r);
/* Same, broadcast only, over an injected table. */
int or_refsim_broadcast(const or_params* p, const uint8_t* deg,
                        const uint32_t* ids, uint32_t stride,
                        uint64_t rng_seed, uint64_t max_ms,
                        or_refsim_result* r);

#ifdef __cplusplus
}
#endif
#endif
