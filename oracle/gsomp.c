/*
 * gsomp.c -- all-core (OpenMP) CPU port of the tick engine in gsoracle.c.
 *
 * TEST INFRASTRUCTURE ONLY, like everything under oracle/: bench.py's
 * cpu_baseline leg times it on the GPU box's host cores, and tests/ check
 * it against the single-thread restatement.  Same tick model, same keyed
 * Philox draws (simulator.go:107-123 receive, :140-149 broadcast, :166-184
 * delay/drop/crash), so its per-tick counters and bitsets equal
 * or_engine_step's bit for bit whatever the thread count:
 *   phase A (parallel over the fire slot's words): every firing node draws
 *     its drops and its messages' crash rolls and counts one arrival (and its
 *     roll) per kept send (atomic add); the first arrival at a node lists it
 *     in the thread's touched list;
 *   phase B (parallel over the touched nodes): rule A6 -- k receipts, their
 *     crash rolls and the keyed first-crash position -- then Broadcast() of
 *     the newly received (atomic OR into the fire ring).
 * Flood model only (the reference's); no node-range sharding.
 */
#include <omp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "gsoracle.h"

typedef struct om_engine {
  or_params p;
  uint64_t n, W;
  uint32_t stride, R, key[2];
  int32_t kd, kc;
  uint8_t* deg;
  uint32_t* ids;
  uint64_t *received, *crashed, *ring;
  uint32_t* cnt;
  uint32_t** touched;  /* per thread */
  uint64_t* tcap;      /* per thread capacity */
  int nth;
  uint64_t t, recv, crashed_cnt, pending;
  int begun;
} om_engine;

static inline uint32_t c3of(int kind, uint32_t trial) { return ((uint32_t)kind << 24) | (trial & 0xFFFFFFu); }

static inline void draw4(const uint32_t key[2], uint32_t a, uint32_t b, uint32_t c, int kind, uint32_t trial,
                         uint32_t out[4]) {
  uint32_t ctr[4] = {a, b, c, c3of(kind, trial)};
  or_philox(ctr, key, out);
}

static inline uint32_t fire_offset(const or_params* p, uint32_t r) {
  int64_t d = (int64_t)p->delay_low + (int64_t)or_uniform(r, (uint32_t)(p->delay_high - p->delay_low));
  return d < 1 ? 1u : (uint32_t)d;
}

#define BIT(a, i) (((a)[(i) >> 6] >> ((i) & 63)) & 1ull)

void om_engine_free(om_engine* e) {
  if (!e) return;
  free(e->deg); free(e->ids); free(e->received); free(e->crashed); free(e->ring); free(e->cnt);
  if (e->touched)
    for (int i = 0; i < e->nth; ++i) free(e->touched[i]);
  free(e->touched); free(e->tcap);
  free(e);
}

om_engine* om_engine_new(const or_params* p, const uint8_t* deg, const uint32_t* ids, uint32_t stride,
                         int nthreads) {
  if (!p || p->n == 0 || p->n > 0x7FFFFFFFull || p->delay_high <= p->delay_low || p->model != OR_MODEL_FLOOD ||
      stride == 0 || stride > 255)
    return NULL;
  om_engine* e = (om_engine*)calloc(1, sizeof(om_engine));
  if (!e) return NULL;
  e->p = *p;
  e->n = p->n;
  e->W = (p->n + 63) / 64;
  e->stride = stride;
  e->R = p->delay_high > 2 ? (uint32_t)p->delay_high : 2u;
  e->kd = or_threshold(p->drop_rate);
  e->kc = or_threshold(p->crash_rate);
  e->key[0] = (uint32_t)p->seed;
  e->key[1] = (uint32_t)(p->seed >> 32);
  e->nth = nthreads > 0 ? nthreads : omp_get_max_threads();
  e->deg = (uint8_t*)malloc(e->n);
  e->ids = (uint32_t*)malloc(e->n * stride * sizeof(uint32_t));
  e->received = (uint64_t*)calloc(e->W, 8);
  e->crashed = (uint64_t*)calloc(e->W, 8);
  e->ring = (uint64_t*)calloc((size_t)e->R * e->W, 8);
  e->cnt = (uint32_t*)calloc(e->n, 4);
  e->touched = (uint32_t**)calloc(e->nth, sizeof(uint32_t*));
  e->tcap = (uint64_t*)calloc(e->nth, 8);
  if (!e->deg || !e->ids || !e->received || !e->crashed || !e->ring || !e->cnt || !e->touched || !e->tcap) {
    om_engine_free(e);
    return NULL;
  }
  int bad = 0;
#pragma omp parallel for num_threads(e->nth) schedule(static) reduction(| : bad)
  for (uint64_t v = 0; v < e->n; ++v) {
    if (deg[v] > stride) bad = 1;
    e->deg[v] = deg[v];
    for (uint32_t j = 0; j < stride; ++j) {
      const uint32_t x = ids[v * stride + j];
      if (j < deg[v] && x >= e->n) bad = 1;
      e->ids[v * stride + j] = j < deg[v] ? x : 0;
    }
  }
  for (int i = 0; i < e->nth && !bad; ++i) {  /* grown on demand */
    e->tcap[i] = e->n / e->nth + 4096;
    e->touched[i] = (uint32_t*)malloc(e->tcap[i] * 4);
    if (!e->touched[i]) bad = 1;
  }
  if (bad) {
    om_engine_free(e);
    return NULL;
  }
  return e;
}

static void schedule(om_engine* e, uint32_t v, uint64_t t) {
  uint32_t r[4];
  draw4(e->key, v, (uint32_t)t, 0, OR_K_DELAY, e->p.trial, r);
  const uint32_t off = fire_offset(&e->p, r[0]);
  __atomic_fetch_or(&e->ring[((t + off) % e->R) * e->W + (v >> 6)], 1ull << (v & 63), __ATOMIC_RELAXED);
}

int om_engine_begin(om_engine* e, int64_t sender) {
  if (!e || e->begun) return -1;
  const uint64_t s = sender < 0 ? or_pick_sender(&e->p) : (uint64_t)sender;
  if (s >= e->n) return -1;
  e->t = 0;
  if (!BIT(e->crashed, s)) {
    schedule(e, (uint32_t)s, 0);
    e->pending = 1;
  }
  e->begun = 1;
  return 0;
}

int om_engine_step(om_engine* e, uint32_t ticks, or_tick_stats* out) {
  if (!e || !e->begun) return -1;
  for (uint32_t s = 0; s < ticks; ++s) {
    const uint64_t t = ++e->t;
    uint64_t* ring = e->ring + (t % e->R) * e->W;
    uint64_t fired = 0, sent = 0, msgs = 0, nrecv = 0, ncrash = 0;
    int ovf = 0;
#pragma omp parallel num_threads(e->nth) reduction(+ : fired, sent, msgs, nrecv, ncrash) reduction(| : ovf)
    {
      const int me = omp_get_thread_num();
      uint32_t* tl = e->touched[me];
      uint64_t nt = 0, cap = e->tcap[me];
      /* phase A: Broadcast goroutines whose time.After expired (:142-147) */
#pragma omp for schedule(dynamic, 256)
      for (uint64_t w = 0; w < e->W; ++w) {
        uint64_t bits = ring[w];
        if (!bits) continue;
        ring[w] = 0;
        while (bits) {
          const uint32_t v = (uint32_t)(w * 64 + (uint64_t)__builtin_ctzll(bits));
          bits &= bits - 1;
          ++fired;
          const uint32_t d = e->deg[v];
          const uint32_t* row = e->ids + (uint64_t)v * e->stride;
          uint32_t rnd[4] = {0, 0, 0, 0};
          for (uint32_t j = 0; j < d; ++j) {
            if ((j & 3) == 0) draw4(e->key, v, (uint32_t)t, j >> 2, OR_K_DROP, e->p.trial, rnd);
            uint32_t drop, crash;  /* the drop draw and the message's crash roll (:180) */
            or_drop_crash(rnd[j & 3], &drop, &crash);
            if ((int32_t)drop < e->kd) continue;                         /* :144, :172 */
            const uint32_t u = row[j];                                   /* :145 */
            ++sent;
            const uint32_t roll = (int32_t)crash < e->kc;                /* :180 */
            const uint32_t old = __atomic_fetch_add(&e->cnt[u], 1u + (roll << 16), __ATOMIC_RELAXED);
            if ((old & 0xFFFFu) == 0xFFFFu) ovf = 1;  /* 16-bit receipt count: GS_EOVERFLOW */
            if (old == 0) {
              if (nt == cap) {
                cap *= 2;
                uint32_t* g = (uint32_t*)realloc(tl, cap * 4);
                if (!g) abort();
                tl = g;
                e->touched[me] = g;
                e->tcap[me] = cap;
              }
              tl[nt++] = u;
            }
          }
        }
      }
      /* implicit barrier: every arrival is counted */
      /* phase B: the receive case per touched node (:107-123, rule A6) */
      for (uint64_t i = 0; i < nt; ++i) {
        const uint32_t u = tl[i];
        const uint32_t k = e->cnt[u] & 0xFFFFu, ones = e->cnt[u] >> 16;
        e->cnt[u] = 0;
        const uint64_t bit = 1ull << (u & 63);
        if (__atomic_load_n(&e->crashed[u >> 6], __ATOMIC_RELAXED) & bit) continue;   /* :108 */
        const uint32_t g = ones ? or_first_crash(e->key, e->p.trial, u, (uint32_t)t, k, ones) : k + 1;
        msgs += g <= k ? g : k;                                                       /* :111 */
        if (g > 1 && !(__atomic_load_n(&e->received[u >> 6], __ATOMIC_RELAXED) & bit)) {  /* :117 */
          __atomic_fetch_or(&e->received[u >> 6], bit, __ATOMIC_RELAXED);             /* :120 */
          ++nrecv;                                                                    /* :121 */
          schedule(e, u, t);                                                          /* :122 */
        }
        if (g <= k) {                                                                 /* :112-115 */
          __atomic_fetch_or(&e->crashed[u >> 6], bit, __ATOMIC_RELAXED);
          ++ncrash;
        }
      }
    }
    if (ovf) return OR_EOVERFLOW;  /* >= 65536 arrivals at one node in one tick */
    e->recv += nrecv;
    e->crashed_cnt += ncrash;
    e->pending = e->pending - fired + nrecv;
    if (out) {
      out[s].tick = t; out[s].fired = fired; out[s].sent = sent; out[s].messages = msgs;
      out[s].received = e->recv; out[s].crashed = e->crashed_cnt; out[s].pending = e->pending;
    }
  }
  return 0;
}

int om_engine_read_received(const om_engine* e, uint64_t* words, size_t nwords) {
  if (!e || nwords < e->W) return -1;
  memcpy(words, e->received, e->W * 8);
  return 0;
}

int om_engine_read_crashed(const om_engine* e, uint64_t* words, size_t nwords) {
  if (!e || nwords < e->W) return -1;
  memcpy(words, e->crashed, e->W * 8);
  return 0;
}

int om_engine_set_failed(om_engine* e, const uint64_t* words, size_t nwords) {
  if (!e || nwords < e->W || e->begun) return -1;
  for (uint64_t w = 0; w < e->W; ++w) e->crashed[w] |= words[w];
  if (e->n & 63) e->crashed[e->W - 1] &= (1ull << (e->n & 63)) - 1;
  return 0;
}

int om_threads(const om_engine* e) { return e ? e->nth : 0; }
