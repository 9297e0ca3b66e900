/*
 * relabel_estimate.c -- verdict r05 item 1(a): how many 128-B packed-row lines
 * does k_expand fetch per broadcast under the identity node order, and how many
 * under a graph-local order?  CPU only, built on the oracle's tick model
 * (oracle/gsoracle.c, test infrastructure), so the fire ticks are exactly the
 * engine's.
 *
 *   gcc -O2 -std=gnu11 -o /tmp/relabel_estimate scripts/relabel_estimate.c \
 *       oracle/gsoracle.c -lm && /tmp/relabel_estimate 10000000
 *
 * Model of the fetch: k_expand reads firing node v's row from packed line
 * pos(v) / 5 (five 24-B rows per 128-B line); within one window a line is
 * fetched once (bucket-major units keep a window's re-touches in L2), across
 * windows once per window that fires one of its rows (the 25.6-GB view does
 * not survive in L2/MALL between windows).  So lines fetched = sum over
 * windows of the distinct lines holding a firing row.  The same count is made
 * for the 4-B orig-id lookups (32 per line) a relabelled engine would need at
 * fire time (Philox drop key) and at infection time (delay key).
 *
 * simulator.go:140-149 is the friend loop whose row this gathers.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../oracle/gsoracle.h"

#define NOTICK 0xFFFFFFFFu

static uint32_t n_g;

/* distinct (line, window) pairs for events (node -> window) under order pos */
static uint64_t lines_touched(const uint32_t* win, const uint32_t* pos, uint32_t per_line,
                              uint32_t nwin) {
  uint64_t nl = (n_g + per_line - 1) / per_line;
  /* last window stamp per line; events processed window by window */
  uint32_t* stamp = malloc(nl * sizeof(uint32_t));
  for (uint64_t i = 0; i < nl; ++i) stamp[i] = NOTICK;
  /* bucket the nodes by window */
  uint64_t* cnt = calloc(nwin + 1, sizeof(uint64_t));
  for (uint32_t v = 0; v < n_g; ++v)
    if (win[v] != NOTICK) cnt[win[v] + 1]++;
  for (uint32_t w = 0; w < nwin; ++w) cnt[w + 1] += cnt[w];
  uint32_t* byw = malloc((size_t)cnt[nwin] * sizeof(uint32_t));
  uint64_t* fill = malloc((nwin + 1) * sizeof(uint64_t));
  memcpy(fill, cnt, (nwin + 1) * sizeof(uint64_t));
  for (uint32_t v = 0; v < n_g; ++v)
    if (win[v] != NOTICK) byw[fill[win[v]]++] = v;
  uint64_t total = 0;
  for (uint32_t w = 0; w < nwin; ++w)
    for (uint64_t i = cnt[w]; i < cnt[w + 1]; ++i) {
      uint64_t l = pos[byw[i]] / per_line;
      if (stamp[l] != w) { stamp[l] = w; ++total; }
    }
  free(stamp); free(cnt); free(byw); free(fill);
  return total;
}

int main(int argc, char** argv) {
  uint64_t n = argc > 1 ? strtoull(argv[1], 0, 10) : 10000000ull;
  n_g = (uint32_t)n;
  or_params p = {0};
  p.n = n; p.fanout = 5; p.fanin = 6; p.delay_low = 10; p.delay_high = 20;
  p.drop_rate = 0.1; p.crash_rate = 0.01; p.seed = 0x5EED; p.trial = 0; p.model = 0;
  uint32_t stride = 6;
  uint8_t* deg = malloc(n);
  uint32_t* ids = malloc(n * stride * sizeof(uint32_t));
  or_window wbuf[4096]; size_t nw = 0; uint64_t ft = 0;
  int rc = or_overlay(&p, deg, ids, wbuf, 4096, &nw, 100000, &ft);
  if (rc) { fprintf(stderr, "overlay rc %d\n", rc); return 1; }
  fprintf(stderr, "overlay done (tick %llu)\n", (unsigned long long)ft);

  or_engine* e = or_engine_new(&p, deg, ids, stride);
  if (!e || or_engine_begin(e, -1)) { fprintf(stderr, "engine\n"); return 1; }
  size_t W = (n + 63) / 64;
  uint64_t* slot = malloc(W * 8);
  uint64_t* recv = calloc(W, 8);
  uint64_t* prev = calloc(W, 8);
  uint32_t* fire = malloc(n * 4);
  uint32_t* inf = malloc(n * 4);
  for (uint64_t i = 0; i < n; ++i) fire[i] = inf[i] = NOTICK;
  uint64_t fired = 0;
  uint32_t lastw = 0;
  for (uint32_t it = 0; it < 2000; ++it) {
    uint64_t t = or_engine_tick(e) + 1;
    or_engine_get_slot(e, t, slot, W);
    for (size_t w = 0; w < W; ++w)
      for (uint64_t b = slot[w]; b; b &= b - 1) {
        uint64_t v = w * 64 + __builtin_ctzll(b);
        if (fire[v] == NOTICK) fire[v] = (uint32_t)(t / 10); else fire[v] = fire[v]; /* fires once */
        ++fired;
        lastw = (uint32_t)(t / 10);
      }
    or_tick_stats st;
    if (or_engine_step(e, 1, &st)) break;
    or_engine_read_received(e, recv, W);
    for (size_t w = 0; w < W; ++w)
      for (uint64_t b = recv[w] & ~prev[w]; b; b &= b - 1)
        inf[w * 64 + __builtin_ctzll(b)] = (uint32_t)(st.tick / 10);
    memcpy(prev, recv, W * 8);
    if (st.pending == 0) break;
  }
  uint32_t nwin = lastw + 3;
  fprintf(stderr, "fired %llu over %u windows\n", (unsigned long long)fired, nwin);
  /* fire histogram */
  uint64_t* h = calloc(nwin, 8);
  for (uint64_t v = 0; v < n; ++v) if (fire[v] != NOTICK) h[fire[v]]++;
  printf("fires per window (%% of fired):");
  for (uint32_t w = 0; w < nwin; ++w) if (h[w]) printf(" %u:%.1f", w, 100.0 * h[w] / fired);
  printf("\n");

  /* orders */
  uint32_t* pos_id = malloc(n * 4);
  for (uint64_t v = 0; v < n; ++v) pos_id[v] = (uint32_t)v;

  /* greedy groups of 5: v, its unplaced friends, then their unplaced friends */
  uint32_t* pos_g = malloc(n * 4);
  for (uint64_t v = 0; v < n; ++v) pos_g[v] = NOTICK;
  uint64_t next = 0, filler = 0;
  for (uint64_t v = 0; v < n; ++v) {
    if (pos_g[v] != NOTICK) continue;
    uint32_t grp[5]; int g = 0;
    grp[g++] = (uint32_t)v; pos_g[v] = (uint32_t)next++;
    for (int q = 0; q < g && g < 5; ++q) {
      uint32_t u = grp[q];
      for (uint32_t j = 0; j < deg[u] && g < 5; ++j) {
        uint32_t f = ids[(uint64_t)u * stride + j];
        if (pos_g[f] == NOTICK) { pos_g[f] = (uint32_t)next++; grp[g++] = f; }
      }
    }
    while (g < 5 && next % 5) { /* pad the line with the next unplaced ids */
      while (filler < n && pos_g[filler] != NOTICK) ++filler;
      if (filler >= n) break;
      pos_g[filler] = (uint32_t)next++; ++g;
    }
  }

  /* BFS order from node 0 over the friend rows */
  uint32_t* pos_b = malloc(n * 4);
  for (uint64_t v = 0; v < n; ++v) pos_b[v] = NOTICK;
  uint32_t* q = malloc(n * 4);
  uint64_t qh = 0, qt = 0; next = 0;
  for (uint64_t s = 0; s < n; ++s) {
    if (pos_b[s] != NOTICK) continue;
    pos_b[s] = (uint32_t)next++; q[qt++] = (uint32_t)s;
    while (qh < qt) {
      uint32_t u = q[qh++];
      for (uint32_t j = 0; j < deg[u]; ++j) {
        uint32_t f = ids[(uint64_t)u * stride + j];
        if (pos_b[f] == NOTICK) { pos_b[f] = (uint32_t)next++; q[qt++] = f; }
      }
    }
  }

  /* upper bound: sorted by fire window (per-broadcast; not buildable) */
  uint32_t* pos_s = malloc(n * 4);
  {
    uint64_t* c = calloc(nwin + 2, 8);
    for (uint64_t v = 0; v < n; ++v) c[(fire[v] == NOTICK ? nwin : fire[v]) + 1]++;
    for (uint32_t w = 0; w <= nwin; ++w) c[w + 1] += c[w];
    for (uint64_t v = 0; v < n; ++v) pos_s[v] = (uint32_t)c[fire[v] == NOTICK ? nwin : fire[v]]++;
    free(c);
  }

  struct { const char* name; uint32_t* pos; } ord[] = {
      {"identity", pos_id}, {"greedy friend groups", pos_g}, {"BFS from node 0", pos_b},
      {"sorted by fire window (bound)", pos_s}};
  printf("| order | row lines fetched | rows per line | vs identity | orig lookups at fire (32/line) | at infection |\n");
  printf("|---|---|---|---|---|---|\n");
  uint64_t base = 0;
  for (int o = 0; o < 4; ++o) {
    uint64_t L = lines_touched(fire, ord[o].pos, 5, nwin);
    uint64_t Lf = lines_touched(fire, ord[o].pos, 32, nwin);
    uint64_t Li = lines_touched(inf, ord[o].pos, 32, nwin);
    if (!o) base = L;
    printf("| %s | %llu | %.3f | %.3f | %llu | %llu |\n", ord[o].name, (unsigned long long)L,
           (double)fired / L, (double)L / base, (unsigned long long)Lf, (unsigned long long)Li);
  }

  /* Forward staging (identity order): when window w fetches line l, copy the
   * co-resident rows already scheduled for window w + 1 (infected in w - 1,
   * fire in w + 1: the only rows whose fire window is known at w's expand)
   * into a dense per-window buffer; window w + 1 fetches l only for rows not
   * staged.  Costs 28 B written + 28 B read per staged row (row + id). */
  {
    uint64_t nl = (n + 4) / 5;
    uint8_t* staged = calloc(n, 1);
    uint32_t* stamp = malloc(nl * 4);
    for (uint64_t i = 0; i < nl; ++i) stamp[i] = NOTICK;
    uint64_t fetched = 0, nstaged = 0;
    for (uint32_t w = 0; w < nwin; ++w) {
      for (uint64_t v = 0; v < n; ++v) {
        if (fire[v] != w || staged[v]) continue;
        uint64_t l = v / 5;
        if (stamp[l] == w) continue;
        stamp[l] = w; ++fetched;
        for (uint64_t r = l * 5; r < l * 5 + 5 && r < n; ++r)
          if (fire[r] == w + 1 && inf[r] + 1 == w && !staged[r]) { staged[r] = 1; ++nstaged; }
      }
    }
    printf("forward staging: lines fetched %llu (%.3f of identity), rows staged %llu; "
           "bytes %.1f MB vs identity %.1f MB\n",
           (unsigned long long)fetched, (double)fetched / base, (unsigned long long)nstaged,
           (fetched * 128.0 + nstaged * 56.0) / 1e6, base * 128.0 / 1e6);
  }
  return 0;
}
