/*
 * gsoracle.c -- CPU restatement of go-distributed/gossip_simulator.
 *
 * TEST INFRASTRUCTURE ONLY (see gsoracle.h).  Parity with the reference is
 * UNPINNED by reference artefacts (none exist; no Go toolchain here); the
 * restatement is pinned by hand-derived known answers in tests/.
 *
 * Every function cites the simulator.go lines it restates.  The tick model is
 * the bit-exact specification of the HIP engine (DESIGN.md section "Tick model").
 */
#include "gsoracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* Philox4x32-10 (Salmon et al., SC'11; Random123 constants).                */
/* ------------------------------------------------------------------------ */
#define PH_M0 0xD2511F53u
#define PH_M1 0xCD9E8D57u
#define PH_W0 0x9E3779B9u
#define PH_W1 0xBB67AE85u

void or_philox(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
  uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
  uint32_t k0 = key[0], k1 = key[1];
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)PH_M0 * c0;
    uint64_t p1 = (uint64_t)PH_M1 * c2;
    uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
    uint32_t n1 = (uint32_t)p1;
    uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
    uint32_t n3 = (uint32_t)p0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += PH_W0; k1 += PH_W1;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

uint32_t or_uniform(uint32_t r, uint32_t m) {
  return (uint32_t)(((uint64_t)r * (uint64_t)m) >> 32);
}

void or_drop_crash(uint32_t r, uint32_t* drop, uint32_t* crash) {
  const uint64_t x = (uint64_t)r * 100u;
  *drop = (uint32_t)(x >> 32);
  *crash = or_uniform((uint32_t)x, 100);
}

uint32_t or_first_crash(const uint32_t key[2], uint32_t trial, uint32_t u, uint32_t t, uint32_t k,
                        uint32_t ones) {
  if (k <= 1 || ones >= k) return 1;
  uint32_t rnd[4] = {0, 0, 0, 0};
  for (uint32_t g = 1;; ++g) {  /* ends by g = k - ones + 1, where U_ones < ones */
    if (((g - 1) & 3) == 0) {
      uint32_t ctr[4] = {u, t, (g - 1) >> 2, ((uint32_t)OR_K_ORDER << 24) | (trial & 0xFFFFFFu)};
      or_philox(ctr, key, rnd);
    }
    if (or_uniform(rnd[(g - 1) & 3], k - g + 1) < ones) return g;
  }
}

/* Go: int(rate*100) -- float64 multiply, truncation toward zero
 * (simulator.go:172,180).  0.001 -> 0, 0.1 -> 10, 0.29 -> 28. */
int32_t or_threshold(double rate) {
  double x = rate * 100.0;
  if (x != x) return 0;
  if (x >= 100.0) return 100;
  if (x <= 0.0) return 0;
  return (int32_t)x; /* C conversion truncates toward zero, like Go */
}

static inline uint32_t c3of(int kind, uint32_t trial) {
  return ((uint32_t)kind << 24) | (trial & 0xFFFFFFu);
}

static inline uint32_t draw(const uint32_t key[2], uint32_t a, uint32_t b,
                            uint32_t c, int kind, uint32_t trial, int lane) {
  uint32_t ctr[4] = {a, b, c, c3of(kind, trial)};
  uint32_t out[4];
  or_philox(ctr, key, out);
  return out[lane];
}

static inline void keyof(const or_params* p, uint32_t key[2]) {
  key[0] = (uint32_t)p->seed;
  key[1] = (uint32_t)(p->seed >> 32);
}

/* simulator.go:240  senderPos := rand.Intn(len(GlobalView)) */
uint64_t or_pick_sender(const or_params* p) {
  uint32_t key[2];
  keyof(p, key);
  return or_uniform(draw(key, 0, 0, 0, OR_K_SENDER, p->trial, 0), (uint32_t)p->n);
}

/* simulator.go:166-168  DelayLow + rand.Intn(DelayHigh-DelayLow), in ticks;
 * a delay below one tick is executed as one tick ("delays"). */
static inline uint32_t fire_offset(const or_params* p, uint32_t r) {
  int64_t d = (int64_t)p->delay_low +
              (int64_t)or_uniform(r, (uint32_t)(p->delay_high - p->delay_low));
  return d < 1 ? 1u : (uint32_t)d;
}

static inline uint32_t ring_size(const or_params* p) {
  return p->delay_high > 2 ? (uint32_t)p->delay_high : 2u;
}

static int check_params(const or_params* p) {
  if (p->n == 0 || p->n > 0x7FFFFFFFull) return -1;     /* :240 panics at n=0 */
  if (p->delay_high <= p->delay_low) return -1;          /* :167 Intn(<=0) panics */
  if (p->fanin < 0 || p->fanout < 0) return -1;
  if (p->fanin > 255 || p->fanout > 255) return -1;
  if (p->model > OR_MODEL_PUSHPULL) return -1;
  return 0;
}

static inline int f32_covered(uint64_t recv, uint64_t n) {
  /* simulator.go:246-248: float32(TotalReceived)/float32(N) >= 0.99 */
  volatile float a = (float)recv;
  volatile float b = (float)n;
  volatile float pct = a / b;
  return pct >= 0.99f;
}

/* ======================================================================== */
/* Overlay: tick-synchronous makeup/breakup protocol.                        */
/* ======================================================================== */
typedef struct { uint64_t* a; size_t n, cap; } u64vec;

static int vpush(u64vec* v, uint64_t x) {
  if (v->n == v->cap) {
    size_t nc = v->cap ? v->cap * 2 : 1024;
    uint64_t* na = (uint64_t*)realloc(v->a, nc * sizeof(uint64_t));
    if (!na) return -4;
    v->a = na; v->cap = nc;
  }
  v->a[v->n++] = x;
  return 0;
}

static int cmp_u64(const void* x, const void* y) {
  uint64_t a = *(const uint64_t*)x, b = *(const uint64_t*)y;
  return a < b ? -1 : a > b;
}

static uint32_t node_bits(uint64_t n) {
  uint32_t b = 1;
  while (b < 31 && (1ull << b) < n) ++b;
  return b;
}

/* Event key: dst-major, then src, then kind (0 = makeup, 1 = breakup).
 * Identical keys are identical messages, and every draw is keyed by the
 * processing ordinal, so their relative order cannot change the outcome. */
#define EV_MAKEUP 0u
#define EV_BREAKUP 1u

int or_overlay(const or_params* p, uint8_t* deg, uint32_t* ids, or_window* win,
               size_t wcap, size_t* nwin, uint64_t max_ticks,
               uint64_t* final_tick) {
  if (check_params(p)) return -1;
  const uint64_t n = p->n;
  const uint32_t fanout = (uint32_t)p->fanout, fanin = (uint32_t)p->fanin;
  const uint32_t stride = fanout > fanin ? fanout : fanin;
  const uint32_t R = ring_size(p);
  const uint32_t B = node_bits(n);
  const uint64_t src_mask = (1ull << B) - 1;
  uint32_t key[2];
  keyof(p, key);
  if (nwin) *nwin = 0;
  if (final_tick) *final_tick = 0;

  u64vec* slot = (u64vec*)calloc(R, sizeof(u64vec));
  if (!slot) return -4;
  int rc = 0;
  uint64_t pending = 0;

  /* Tick 0 -- simulator.go:95-106 (needNewFriendCh), executed by every node
   * before any makeup can arrive (delays >= 1 tick). */
  for (uint64_t v = 0; v < n; ++v) {
    for (uint32_t j = 0; j < fanout; ++j) {
      uint32_t f = or_uniform(draw(key, (uint32_t)v, 0, j, OR_K_PICK, p->trial, 0),
                              (uint32_t)n);
      if (f == v) f = (uint32_t)((f + 1) % n);          /* :98-100 */
      ids[v * stride + j] = f;                           /* :101    */
      uint32_t off = fire_offset(p, draw(key, (uint32_t)v, 0, j, OR_K_OVDELAY, p->trial, 0));
      uint64_t ev = ((uint64_t)f << (B + 1)) | (v << 1) | EV_MAKEUP; /* :102 */
      if ((rc = vpush(&slot[off % R], ev))) goto done;
      ++pending;
    }
    deg[v] = (uint8_t)fanout;
  }

  uint64_t wm = 0, wb = 0;
  size_t nw = 0;
  for (uint64_t t = 1;; ++t) {
    if (t > max_ticks) { rc = -2; goto done; }
    u64vec* s = &slot[t % R];
    if (s->n) {
      qsort(s->a, s->n, sizeof(uint64_t), cmp_u64);
      size_t m = s->n;
      pending -= m;
      uint64_t prev_dst = ~0ull;
      uint32_t k = 0;
      for (size_t e = 0; e < m; ++e) {
        uint64_t ev = s->a[e];
        uint32_t u = (uint32_t)(ev >> (B + 1));
        uint32_t src = (uint32_t)((ev >> 1) & src_mask);
        uint32_t kind = (uint32_t)(ev & 1);
        if (u != prev_dst) { prev_dst = u; k = 0; } else { ++k; }
        if (k >= (1u << 26)) { rc = -1; goto done; }
        uint32_t* row = ids + (uint64_t)u * stride;
        uint32_t d = deg[u];
        if (kind == EV_MAKEUP) {                         /* simulator.go:66-75 */
          ++wm;
          if (d < fanin) {
            row[d] = src;
            deg[u] = (uint8_t)(d + 1);
          } else {
            uint32_t pos = or_uniform(draw(key, u, (uint32_t)t, k, OR_K_VICTIM, p->trial, 0), d);
            uint32_t victim = row[pos];
            uint32_t off = fire_offset(p, draw(key, u, (uint32_t)t, k, OR_K_OVDELAY, p->trial, 0));
            uint64_t nev = ((uint64_t)victim << (B + 1)) | ((uint64_t)u << 1) | EV_BREAKUP;
            if ((rc = vpush(&slot[(t + off) % R], nev))) goto done;
            ++pending;
            row[pos] = src;
          }
        } else {                                         /* simulator.go:76-94 */
          ++wb;
          uint32_t i = 0;
          while (i < d && row[i] != src) ++i;
          if (i == d) continue;                          /* not a friend: ignored */
          if (d > fanout) {                              /* :80-84 removeFriend  */
            memmove(row + i, row + i + 1, (size_t)(d - i - 1) * sizeof(uint32_t));
            deg[u] = (uint8_t)(d - 1);
          } else {                                       /* :86-91 replace       */
            uint32_t nf = 0;
            uint32_t a = 0;
            for (; a < 256; ++a) {
              nf = or_uniform(draw(key, u, (uint32_t)t, (k << 6) | (a >> 2), OR_K_REPLACE,
                                   p->trial, (int)(a & 3)),
                              (uint32_t)n);
              if (nf != src && nf != u) break;
            }
            if (a == 256) { rc = -3; goto done; }
            row[i] = nf;
            uint32_t off = fire_offset(p, draw(key, u, (uint32_t)t, k, OR_K_OVDELAY, p->trial, 0));
            uint64_t nev = ((uint64_t)nf << (B + 1)) | ((uint64_t)u << 1) | EV_MAKEUP;
            if ((rc = vpush(&slot[(t + off) % R], nev))) goto done;
            ++pending;
          }
        }
      }
      /* Emitted events never land in this slot (1 <= off < R). */
      s->n = 0;
    }
    if (t % 10 == 0) {                                   /* simulator.go:222-234 */
      if (wm == 0 && wb == 0 && pending == 0) {
        if (final_tick) *final_tick = t;
        break;
      }
      if (win && nw < wcap) {
        win[nw].tick = t; win[nw].makeups = wm; win[nw].breakups = wb;
      }
      ++nw;
      wm = wb = 0;
    }
  }
  if (nwin) *nwin = nw;
done:
  for (uint32_t i = 0; i < R; ++i) free(slot[i].a);
  free(slot);
  return rc;
}

/* ======================================================================== */
/* Broadcast tick engine.                                                    */
/* ======================================================================== */
struct or_engine {
  or_params p;
  uint64_t n, W;
  uint32_t stride, R;
  int32_t kd, kc;
  uint32_t key[2];
  uint8_t* deg;
  uint32_t* ids;
  uint64_t *received, *crashed, *ring;
  uint32_t* cnt;
  uint32_t* touched;
  uint64_t t, recv, crashed_cnt, pending;
  uint64_t lo, hi; /* owned node range (node-range sharding) */
  int begun;
};

or_engine* or_engine_new(const or_params* p, const uint8_t* deg,
                         const uint32_t* ids, uint32_t stride) {
  if (check_params(p)) return NULL;
  if (stride == 0 || stride > 255) return NULL;
  or_engine* e = (or_engine*)calloc(1, sizeof(or_engine));
  if (!e) return NULL;
  e->p = *p;
  e->n = p->n;
  e->W = (p->n + 63) / 64;
  e->stride = stride;
  e->R = ring_size(p);
  e->kd = or_threshold(p->drop_rate);
  e->kc = or_threshold(p->crash_rate);
  e->lo = 0;
  e->hi = p->n;
  keyof(p, e->key);
  e->deg = (uint8_t*)malloc(e->n);
  e->ids = (uint32_t*)malloc(e->n * stride * sizeof(uint32_t));
  e->received = (uint64_t*)calloc(e->W, 8);
  e->crashed = (uint64_t*)calloc(e->W, 8);
  e->ring = (uint64_t*)calloc((size_t)e->R * e->W, 8);
  e->cnt = (uint32_t*)calloc(e->n, 4);
  e->touched = (uint32_t*)malloc(e->n * 4);
  if (!e->deg || !e->ids || !e->received || !e->crashed || !e->ring || !e->cnt || !e->touched) {
    or_engine_free(e);
    return NULL;
  }
  for (uint64_t v = 0; v < e->n; ++v) {
    if (deg[v] > stride) { or_engine_free(e); return NULL; }
    e->deg[v] = deg[v];
    for (uint32_t j = 0; j < stride; ++j) {
      uint32_t x = ids[v * stride + j];
      if (j < deg[v] && x >= e->n) { or_engine_free(e); return NULL; }
      e->ids[v * stride + j] = j < deg[v] ? x : 0;
    }
  }
  return e;
}

void or_engine_free(or_engine* e) {
  if (!e) return;
  free(e->deg); free(e->ids); free(e->received); free(e->crashed);
  free(e->ring); free(e->cnt); free(e->touched);
  free(e);
}

#define BIT(a, i) (((a)[(i) >> 6] >> ((i) & 63)) & 1ull)
#define SETBIT(a, i) ((a)[(i) >> 6] |= 1ull << ((i) & 63))

/* Node.Broadcast (simulator.go:140-142): one delay per call. */
static void schedule(or_engine* e, uint32_t v, uint64_t t) {
  uint32_t off = fire_offset(&e->p, draw(e->key, v, (uint32_t)t, 0, OR_K_DELAY, e->p.trial, 0));
  SETBIT(e->ring + ((t + off) % e->R) * e->W, v);
  ++e->pending;
}

int or_engine_begin(or_engine* e, int64_t sender) {
  if (!e || e->begun) return -1;
  uint64_t s = sender < 0 ? or_pick_sender(&e->p) : (uint64_t)sender;
  if (s >= e->n) return -1;
  e->t = 0;
  if (e->p.model == OR_MODEL_PUSHPULL) {
    if (e->lo != 0 || e->hi != e->n) return -1;  /* not sharded */
    if (!BIT(e->crashed, s)) {                    /* a failed sender informs nobody */
      SETBIT(e->received, s);
      e->recv = 1;
    }
    e->pending = e->recv;
    e->begun = 1;
    return 0;
  }
  /* only the owner of the sender schedules it (simulator.go:241; the sender
   * is NOT marked received); a pre-failed sender (extension) never broadcasts */
  if (s >= e->lo && s < e->hi && !BIT(e->crashed, s)) schedule(e, (uint32_t)s, 0);
  e->begun = 1;
  return 0;
}

int or_engine_set_failed(or_engine* e, const uint64_t* words, size_t nwords) {
  if (!e || nwords < e->W) return -1;
  for (uint64_t w = 0; w < e->W; ++w) e->crashed[w] |= words[w];
  if (e->n & 63) e->crashed[e->W - 1] &= (1ull << (e->n & 63)) - 1;
  return 0;
}

/* Push-pull extension: one synchronous round per tick (see gsoracle.h).  The
 * next informed set is built from the round's starting set only, so the
 * result does not depend on the order nodes are visited in. */
static int pushpull_step(or_engine* e, uint32_t ticks, or_tick_stats* out) {
  uint64_t* next = (uint64_t*)malloc(e->W * 8);
  if (!next) return -1;
  for (uint32_t s = 0; s < ticks; ++s) {
    uint64_t t = ++e->t;
    uint64_t fired = 0, sent = 0, msgs = 0;
    memcpy(next, e->received, e->W * 8);
    for (uint64_t v = 0; v < e->n; ++v) {
      uint32_t d = e->deg[v];
      if (BIT(e->crashed, v) || d == 0) continue;
      uint32_t ctr[4] = {(uint32_t)v, (uint32_t)t, 0, c3of(OR_K_PUSHPULL, e->p.trial)}, rnd[4];
      or_philox(ctr, e->key, rnd);
      uint32_t u = e->ids[v * e->stride + or_uniform(rnd[0], d)];
      int kept = (int32_t)or_uniform(rnd[1], 100) >= e->kd;
      ++fired;
      if (BIT(e->received, v)) {              /* push */
        if (!kept) continue;
        ++sent;
        if (BIT(e->crashed, u)) continue;
        ++msgs;
        SETBIT(next, u);
      } else if (BIT(e->received, u)) {       /* pull (u informed => u live) */
        if (!kept) continue;
        ++sent;
        ++msgs;
        SETBIT(next, v);
      }
    }
    for (uint64_t w = 0; w < e->W; ++w) {
      e->recv += (uint64_t)__builtin_popcountll(next[w] & ~e->received[w]);
      e->received[w] = next[w];
    }
    e->pending = e->recv;
    if (out) {
      out[s].tick = t; out[s].fired = fired; out[s].sent = sent;
      out[s].messages = msgs; out[s].received = e->recv;
      out[s].crashed = e->crashed_cnt; out[s].pending = e->pending;
    }
  }
  free(next);
  return 0;
}

int or_engine_step(or_engine* e, uint32_t ticks, or_tick_stats* out) {
  if (!e || !e->begun) return -1;
  if (e->p.model == OR_MODEL_PUSHPULL) return pushpull_step(e, ticks, out);
  for (uint32_t s = 0; s < ticks; ++s) {
    uint64_t t = ++e->t;
    uint64_t* ring = e->ring + (t % e->R) * e->W;
    uint64_t fired = 0, sent = 0, msgs = 0;
    uint64_t nt = 0;
    /* Broadcast goroutines whose time.After expired (simulator.go:142-147). */
    for (uint64_t w = 0; w < e->W; ++w) {
      uint64_t bits = ring[w];
      if (!bits) continue;
      ring[w] = 0;
      while (bits) {
        uint32_t v = (uint32_t)(w * 64 + (uint64_t)__builtin_ctzll(bits));
        bits &= bits - 1;
        if (v >= e->lo && v < e->hi) ++fired;
        uint32_t d = e->deg[v];
        const uint32_t* row = e->ids + (uint64_t)v * e->stride;
        uint32_t rnd[4] = {0, 0, 0, 0};
        for (uint32_t j = 0; j < d; ++j) {
          if ((j & 3) == 0) {
            uint32_t ctr[4] = {v, (uint32_t)t, j >> 2, c3of(OR_K_DROP, e->p.trial)};
            or_philox(ctr, e->key, rnd);
          }
          uint32_t drop, crash;  /* the drop draw and the message's crash roll (:180) */
          or_drop_crash(rnd[j & 3], &drop, &crash);
          if ((int32_t)drop < e->kd) continue;                         /* :144,:172 */
          uint32_t u = row[j];                                         /* :145 */
          if (u < e->lo || u >= e->hi) continue;  /* another rank's target */
          ++sent;
          const uint32_t roll = (int32_t)crash < e->kc;
          if (e->cnt[u] == 0) e->touched[nt++] = u;
          /* receipts | crash rolls << 16: a 16-bit count, so >= 65536 arrivals at
           * one node in one tick is an overflow (the engine returns GS_EOVERFLOW) */
          if ((e->cnt[u] & 0xFFFFu) == 0xFFFFu) return OR_EOVERFLOW;
          e->cnt[u] += 1u + (roll << 16);
        }
      }
    }
    e->pending -= fired;
    /* Receipts (simulator.go:107-123), rule A6: the k messages of a tick are
     * taken in a uniformly random order; each is counted (:111) and rolls
     * its own crash (:112-115), the first that does not crash informs the
     * node (:117-122), and the node stops at the first crash.  So only k, the
     * number of crash rolls among them and the keyed first-crash position
     * matter -- not who sent what, nor the order atomics arrive in. */
    for (uint64_t i = 0; i < nt; ++i) {
      uint32_t u = e->touched[i];
      const uint32_t k = e->cnt[u] & 0xFFFFu, ones = e->cnt[u] >> 16;
      e->cnt[u] = 0;
      if (BIT(e->crashed, u)) continue;                          /* :108 */
      const uint32_t g = ones ? or_first_crash(e->key, e->p.trial, u, (uint32_t)t, k, ones) : k + 1;
      msgs += g <= k ? g : k;                                    /* :111 */
      if (g > 1 && !BIT(e->received, u)) {                       /* :117 */
        SETBIT(e->received, u);                                  /* :120 */
        ++e->recv;                                               /* :121 */
        schedule(e, u, t);                                       /* :122 */
      }
      if (g <= k) {                                              /* :112-115 */
        SETBIT(e->crashed, u);
        ++e->crashed_cnt;
      }
    }
    if (out) {
      out[s].tick = t; out[s].fired = fired; out[s].sent = sent;
      out[s].messages = msgs; out[s].received = e->recv;
      out[s].crashed = e->crashed_cnt; out[s].pending = e->pending;
    }
  }
  return 0;
}

int or_engine_read_received(const or_engine* e, uint64_t* words, size_t nwords) {
  if (!e || nwords < e->W) return -1;
  memcpy(words, e->received, e->W * 8);
  return 0;
}

int or_engine_read_crashed(const or_engine* e, uint64_t* words, size_t nwords) {
  if (!e || nwords < e->W) return -1;
  memcpy(words, e->crashed, e->W * 8);
  return 0;
}

uint64_t or_engine_tick(const or_engine* e) { return e ? e->t : 0; }

int or_engine_set_range(or_engine* e, uint64_t lo, uint64_t hi) {
  if (!e || e->begun || lo > hi || hi > e->n) return -1;
  e->lo = lo;
  e->hi = hi;
  return 0;
}

int or_engine_get_slot(const or_engine* e, uint64_t tick, uint64_t* words, size_t nwords) {
  if (!e || nwords < e->W) return -1;
  memcpy(words, e->ring + (tick % e->R) * e->W, e->W * 8);
  return 0;
}

int or_engine_set_slot(or_engine* e, uint64_t tick, const uint64_t* words, size_t nwords) {
  if (!e || nwords < e->W) return -1;
  memcpy(e->ring + (tick % e->R) * e->W, words, e->W * 8);
  return 0;
}

/* ======================================================================== */
/* or_refsim: event-driven, sequential-RNG restatement (Go-like).            */
/* ======================================================================== */
typedef struct { uint64_t s[4]; } xoshiro;

static uint64_t splitmix(uint64_t* x) {
  uint64_t z = (*x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static void xo_seed(xoshiro* r, uint64_t seed) {
  for (int i = 0; i < 4; ++i) r->s[i] = splitmix(&seed);
}
static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
static uint64_t xo_next(xoshiro* r) {
  uint64_t* s = r->s;
  uint64_t res = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
  s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t;
  s[3] = rotl(s[3], 45);
  return res;
}
/* rand.Intn(m) stand-in: unbiased enough for m << 2^32 (one sequential stream). */
static uint32_t intn(xoshiro* r, uint32_t m) {
  return (uint32_t)(((xo_next(r) >> 32) * (uint64_t)m) >> 32);
}

enum { RS_MAKEUP = 0, RS_BREAKUP = 1, RS_FIRE = 2, RS_RECV = 3 };
typedef struct { uint64_t time, seq; uint32_t dst, src; uint32_t type; } rs_ev;
typedef struct { rs_ev* a; size_t n, cap; uint64_t seq; } rs_heap;

static inline int ev_less(const rs_ev* x, const rs_ev* y) {
  return x->time < y->time || (x->time == y->time && x->seq < y->seq);
}
static int hpush(rs_heap* h, uint64_t time, uint32_t type, uint32_t dst, uint32_t src) {
  if (h->n == h->cap) {
    size_t nc = h->cap ? h->cap * 2 : 4096;
    rs_ev* na = (rs_ev*)realloc(h->a, nc * sizeof(rs_ev));
    if (!na) return -4;
    h->a = na; h->cap = nc;
  }
  rs_ev e = {time, h->seq++, dst, src, type};
  size_t i = h->n++;
  while (i > 0) {
    size_t par = (i - 1) / 2;
    if (!ev_less(&e, &h->a[par])) break;
    h->a[i] = h->a[par];
    i = par;
  }
  h->a[i] = e;
  return 0;
}
static rs_ev hpop(rs_heap* h) {
  rs_ev top = h->a[0];
  rs_ev last = h->a[--h->n];
  size_t i = 0;
  for (;;) {
    size_t l = 2 * i + 1, r = l + 1, m = i;
    const rs_ev* best = &last;
    if (l < h->n && ev_less(&h->a[l], best)) { m = l; best = &h->a[l]; }
    if (r < h->n && ev_less(&h->a[r], best)) { m = r; }
    if (m == i) break;
    h->a[i] = h->a[m];
    i = m;
  }
  if (h->n) h->a[i] = last;
  return top;
}

static uint64_t rs_delay(const or_params* p, xoshiro* rng) {
  int64_t d = (int64_t)p->delay_low + (int64_t)intn(rng, (uint32_t)(p->delay_high - p->delay_low));
  return d < 1 ? 1u : (uint64_t)d;
}

/* Overlay with the reference's handler bodies (simulator.go:66-106). */
static int rs_overlay(const or_params* p, xoshiro* rng, uint8_t* deg, uint32_t* ids,
                      uint32_t stride, uint64_t max_ms, uint64_t* end_ms) {
  const uint64_t n = p->n;
  const uint32_t fanout = (uint32_t)p->fanout, fanin = (uint32_t)p->fanin;
  rs_heap h = {0};
  int rc = 0;
  for (uint64_t v = 0; v < n; ++v) {
    deg[v] = 0;
    while (deg[v] < fanout) {
      uint32_t f = intn(rng, (uint32_t)n);
      if (f == v) f = (uint32_t)((f + 1) % n);
      ids[v * stride + deg[v]] = f;
      deg[v]++;
      if ((rc = hpush(&h, rs_delay(p, rng), RS_MAKEUP, f, (uint32_t)v))) goto out;
    }
  }
  uint64_t now = 0;
  while (h.n) {
    rs_ev e = hpop(&h);
    now = e.time;
    if (now > max_ms) { rc = -2; goto out; }
    uint32_t u = e.dst, src = e.src, d = deg[u];
    uint32_t* row = ids + (uint64_t)u * stride;
    if (e.type == RS_MAKEUP) {
      if (d < fanin) { row[d] = src; deg[u] = (uint8_t)(d + 1); }
      else {
        uint32_t pos = intn(rng, d);
        uint32_t victim = row[pos];
        if ((rc = hpush(&h, now + rs_delay(p, rng), RS_BREAKUP, victim, u))) goto out;
        row[pos] = src;
      }
    } else {
      uint32_t i = 0;
      while (i < d && row[i] != src) ++i;
      if (i == d) continue;
      if (d > fanout) {
        memmove(row + i, row + i + 1, (size_t)(d - i - 1) * 4);
        deg[u] = (uint8_t)(d - 1);
      } else {
        uint32_t nf, a = 0;
        do { nf = intn(rng, (uint32_t)n); } while ((nf == src || nf == u) && ++a < 100000);
        if (a >= 100000) { rc = -3; goto out; }
        row[i] = nf;
        if ((rc = hpush(&h, now + rs_delay(p, rng), RS_MAKEUP, nf, u))) goto out;
      }
    }
  }
  if (end_ms) *end_ms = now;
out:
  free(h.a);
  return rc;
}

static int rs_broadcast(const or_params* p, xoshiro* rng, const uint8_t* deg,
                        const uint32_t* ids, uint32_t stride, uint64_t max_ms,
                        or_refsim_result* r) {
  const uint64_t n = p->n;
  const int32_t kd = or_threshold(p->drop_rate), kc = or_threshold(p->crash_rate);
  uint8_t* st = (uint8_t*)calloc(n, 1); /* bit0 received, bit1 crashed */
  if (!st) return -4;
  rs_heap h = {0};
  int rc = 0;
  uint64_t recv = 0, crashed = 0, msgs = 0, sent = 0;
  r->reached = 0;
  uint32_t s = intn(rng, (uint32_t)n);                        /* :240 */
  if ((rc = hpush(&h, rs_delay(p, rng), RS_FIRE, s, s))) goto out; /* :241,:142 */
  int have99 = 0;
  while (h.n) {
    if (have99 && h.a[0].time > r->poll_99) break;
    rs_ev e = hpop(&h);
    if (e.time > max_ms) break;
    if (e.type == RS_FIRE) {                                  /* :143-147 */
      uint32_t v = e.dst;
      for (uint32_t j = 0; j < deg[v]; ++j) {
        if ((int32_t)intn(rng, 100) < kd) continue;
        ++sent;
        if ((rc = hpush(&h, e.time, RS_RECV, ids[(uint64_t)v * stride + j], v))) goto out;
      }
    } else {                                                  /* :107-123 */
      uint32_t u = e.dst;
      if (st[u] & 2) continue;
      ++msgs;
      if ((int32_t)intn(rng, 100) < kc) { st[u] |= 2; ++crashed; continue; }
      if (st[u] & 1) continue;
      st[u] |= 1;
      ++recv;
      if ((rc = hpush(&h, e.time + rs_delay(p, rng), RS_FIRE, u, u))) goto out;
      if (!have99 && f32_covered(recv, n)) {
        have99 = 1;
        r->tick_99 = e.time;
        r->poll_99 = ((e.time + 9) / 10) * 10;
        if (r->poll_99 == 0) r->poll_99 = 10;
      }
    }
  }
  r->reached = have99;
  r->messages = msgs; r->crashed = crashed; r->received = recv; r->sent = sent;
out:
  free(st);
  free(h.a);
  return rc;
}

int or_refsim_broadcast(const or_params* p, const uint8_t* deg,
                        const uint32_t* ids, uint32_t stride,
                        uint64_t rng_seed, uint64_t max_ms,
                        or_refsim_result* r) {
  if (check_params(p) || !r) return -1;
  memset(r, 0, sizeof(*r));
  xoshiro rng;
  xo_seed(&rng, rng_seed);
  for (uint64_t v = 0; v < p->n; ++v) r->deg_hist[deg[v]]++;
  return rs_broadcast(p, &rng, deg, ids, stride, max_ms, r);
}

int or_refsim(const or_params* p, uint64_t rng_seed, uint64_t max_ms,
              or_refsim_result* r) {
  if (check_params(p) || !r) return -1;
  memset(r, 0, sizeof(*r));
  const uint32_t stride = p->fanout > p->fanin ? (uint32_t)p->fanout : (uint32_t)p->fanin;
  uint8_t* deg = (uint8_t*)calloc(p->n, 1);
  uint32_t* ids = (uint32_t*)calloc(p->n * (stride ? stride : 1), 4);
  if (!deg || !ids) { free(deg); free(ids); return -4; }
  xoshiro rng;
  xo_seed(&rng, rng_seed);
  int rc = rs_overlay(p, &rng, deg, ids, stride ? stride : 1, max_ms, &r->overlay_ticks);
  if (rc == 0) {
    for (uint64_t v = 0; v < p->n; ++v) r->deg_hist[deg[v]]++;
    rc = rs_broadcast(p, &rng, deg, ids, stride ? stride : 1, max_ms, r);
  }
  free(deg);
  free(ids);
  return rc;
}
