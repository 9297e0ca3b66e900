/* abi_test.c -- a plain C (gcc, C99) client of include/gossip.h: what a cgo
 * host (go/simulator_hip.go) does, without Go.  Built and run by
 * tests/test_c_abi.py.
 *
 *   abi_test cpu   error paths that need no GPU (bad parameters, NULL
 *                  arguments, formatting helpers); with no GPU visible,
 *                  gs_create must fail with GS_EDEVICE, not crash
 *   abi_test gpu   create -> load_peers -> broadcast_begin -> step ->
 *                  read_received on a ring (exact BFS layers, simulator.go
 *                  :140-149 with no loss), the call-order errors, gs_run, and
 *                  the same ring through gs_create_multi with 1 and 2 shards
 *                  on device 0 (bit-identical received sets)
 * Exit status 0 = pass; every failed check prints one line. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gossip.h"

static int failures = 0;
#define CHECK(cond, ...)                                  \
  do {                                                    \
    if (!(cond)) {                                        \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                       \
      fprintf(stderr, "\n");                              \
      ++failures;                                         \
    }                                                     \
  } while (0)

static gs_params ring_params(uint64_t n) {
  gs_params p;
  memset(&p, 0, sizeof p);
  p.n = n;
  p.fanout = 2;
  p.fanin = 2;
  p.delay_low = 3;
  p.delay_high = 4; /* constant 3-ms hop */
  p.drop_rate = 0.0;
  p.crash_rate = 0.0;
  p.seed = 7;
  return p;
}

static int cpu_checks(void) {
  gs_ctx* c = NULL;
  gs_params p = ring_params(1000);
  CHECK(gs_version() == GS_ABI_VERSION, "gs_version %d", gs_version());
  CHECK(gs_create(NULL, &c) == GS_EINVAL && c == NULL, "NULL params");
  CHECK(gs_create(&p, NULL) == GS_EINVAL, "NULL out");
  p.n = 0; /* simulator.go:240 panics on rand.Intn(0) */
  CHECK(gs_create(&p, &c) == GS_EINVAL, "n = 0 accepted");
  p = ring_params(1000);
  p.delay_high = p.delay_low; /* :167 panics on rand.Intn(0) */
  CHECK(gs_create(&p, &c) == GS_EINVAL, "delayhigh == delaylow accepted");
  p = ring_params(1000);
  p.model = 7;
  CHECK(gs_create(&p, &c) == GS_EINVAL, "bad model accepted");
  p = ring_params(1000);
  p.trials = 4;
  p.model = GS_MODEL_PUSHPULL;
  CHECK(gs_create(&p, &c) == GS_EINVAL, "batched push-pull accepted");
  p = ring_params(1000);
  int rc = gs_create(&p, &c); /* no GPU here: a clean device error */
  CHECK(rc == GS_EDEVICE && c == NULL, "gs_create without a GPU returned %d", rc);
  int devs[1] = {0};
  CHECK(gs_create_multi(&p, devs, 0, &c) == GS_EINVAL, "ndev = 0 accepted");
  CHECK(gs_create_rank(&p, 0, 2, 2, NULL, &c) == GS_EINVAL, "rank >= nranks accepted");
  char buf[64];
  gs_format_float32(99.61f, buf, sizeof buf);
  CHECK(strcmp(buf, "99.61") == 0, "format_float32 %s", buf);
  gs_format_duration(1500000000LL, buf, sizeof buf);
  CHECK(strcmp(buf, "1.5s") == 0, "format_duration %s", buf);
  CHECK(gs_threshold(0.29) == 28 && gs_threshold(0.001) == 0, "Go int(rate*100)");
  CHECK(gs_last_error(NULL) != NULL, "gs_last_error(NULL)");
  gs_destroy(NULL);
  /* the device-memory cache without a device: nothing cached, nothing to trim */
  gs_timing mt;
  CHECK(gs_memory_stats(NULL) == GS_EINVAL, "gs_memory_stats(NULL)");
  CHECK(gs_memory_stats(&mt) == GS_OK && mt.cached_bytes == 0 && mt.deliver_ms == 0.0, "gs_memory_stats");
  size_t released = 1;
  CHECK(gs_trim(-1, &released) == GS_OK && released == 0, "gs_trim on an empty cache");
  CHECK(gs_trim(0, NULL) == GS_OK, "gs_trim(0, NULL)");
  return failures;
}

/* ring: friends v-1, v+1; sender s; after h hops (3 ticks each) exactly the
 * nodes at ring distance 1..h are received, plus the sender from hop 2 on
 * (the echo, simulator.go:117-122). */
static int ring_run(gs_ctx* c, uint64_t n, const char* what) {
  uint8_t* deg = malloc(n);
  uint32_t* ids = malloc(n * 2 * sizeof(uint32_t));
  uint64_t W = (n + 63) / 64;
  uint64_t* words = malloc(W * 8);
  for (uint64_t v = 0; v < n; ++v) {
    deg[v] = 2;
    ids[2 * v] = (uint32_t)((v + n - 1) % n);
    ids[2 * v + 1] = (uint32_t)((v + 1) % n);
  }
  CHECK(gs_broadcast_begin(c, 5) == GS_EINVAL, "%s: begin before peers", what);
  CHECK(gs_step(c, 1, NULL) == GS_EINVAL, "%s: step before begin", what);
  CHECK(gs_load_peers(c, deg, ids, 2) == GS_OK, "%s: load_peers: %s", what, gs_last_error(c));
  CHECK(gs_broadcast_begin(c, (int64_t)n) == GS_EINVAL, "%s: sender out of range", what);
  const uint64_t s = 17;
  CHECK(gs_broadcast_begin(c, (int64_t)s) == GS_OK, "%s: begin: %s", what, gs_last_error(c));
  CHECK(gs_broadcast_begin(c, (int64_t)s) == GS_EINVAL, "%s: second begin", what);
  for (int h = 1; h <= 12; ++h) {
    gs_tick_stats st[3];
    CHECK(gs_step(c, 3, st) == GS_OK, "%s: step: %s", what, gs_last_error(c));
    CHECK(gs_read_received(c, words, W) == GS_OK, "%s: read_received", what);
    for (uint64_t v = 0; v < n; ++v) {
      const uint64_t d1 = (v + n - s) % n, d2 = (s + n - v) % n, d = d1 < d2 ? d1 : d2;
      const int want = (d >= 1 && d <= (uint64_t)h) || (d == 0 && h >= 2);
      const int got = (int)((words[v / 64] >> (v % 64)) & 1);
      if (got != want) {
        CHECK(0, "%s: hop %d node %llu got %d want %d", what, h, (unsigned long long)v, got, want);
        h = 99;
        break;
      }
    }
  }
  gs_tick_stats polls[64];
  size_t np = 0;
  int32_t status = -9;
  /* a ring needs ~n/2 hops to cover: the poll loop stops at max_ticks */
  CHECK(gs_run(c, 10, 200, polls, 64, &np, &status) == GS_OK, "%s: run", what);
  CHECK(status == GS_RUN_MAX_TICKS && np == 17 && polls[np - 1].tick == 206, "%s: run status %d, %zu polls",
        what, status, np);
  CHECK(polls[np - 1].received == 2 * (206 / 3) + 1, "%s: received %llu after 206 ticks", what,
        (unsigned long long)polls[np - 1].received);
  gs_trial_stats tr;
  size_t nt = 0;
  CHECK(gs_trial_results(c, &tr, 1, &nt) == GS_OK && nt == 1 && tr.status == GS_RUN_MAX_TICKS &&
            tr.tick == 206 && tr.received == polls[np - 1].received && tr.tick_99 == 0,
        "%s: trial results", what);
  free(deg);
  free(ids);
  free(words);
  return failures;
}

static int gpu_checks(void) {
  const uint64_t n = 40000;
  gs_params p = ring_params(n);
  gs_ctx* c = NULL;
  int rc = gs_create(&p, &c);
  CHECK(rc == GS_OK, "gs_create: %d", rc);
  if (rc) return failures;
  ring_run(c, n, "gs_create");
  CHECK(gs_reset(c) == GS_OK, "reset");
  gs_destroy(c);
  for (int g = 1; g <= 2; ++g) {
    int devs[2] = {0, 0};
    rc = gs_create_multi(&p, devs, g, &c);
    CHECK(rc == GS_OK, "gs_create_multi(%d): %d", g, rc);
    if (rc) continue;
    uint32_t ns = 0;
    uint64_t lo = 0, hi = 0;
    CHECK(gs_shard_info(c, (uint32_t)g - 1, &ns, &lo, &hi) == GS_OK && ns == (uint32_t)g && hi == n,
          "shard_info");
    CHECK(gs_read_peers(c, NULL, NULL, NULL) == GS_EINVAL, "read_peers on a sharded context");
    ring_run(c, n, g == 1 ? "multi(1)" : "multi(2)");
    gs_destroy(c);
  }
  /* the destroyed contexts' large blocks are cached; gs_trim hands them back */
  gs_timing mt;
  CHECK(gs_memory_stats(&mt) == GS_OK && mt.alloc_calls > 0, "gs_memory_stats after runs");
  size_t released = 0;
  CHECK(gs_trim(-1, &released) == GS_OK, "gs_trim");
  CHECK(gs_memory_stats(&mt) == GS_OK && mt.cached_bytes == 0, "cache empty after gs_trim (%llu bytes left)",
        (unsigned long long)mt.cached_bytes);
  return failures;
}

int main(int argc, char** argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: %s cpu|gpu\n", argv[0]);
    return 2;
  }
  if (!strcmp(argv[1], "cpu")) cpu_checks();
  else gpu_checks();
  if (failures) fprintf(stderr, "%d check(s) failed\n", failures);
  else printf("abi_test %s: ok\n", argv[1]);
  return failures ? 1 : 0;
}
