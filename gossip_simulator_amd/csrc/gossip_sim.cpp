// gossip_sim -- drop-in for `go run simulator.go` on an MI355X.
//
// Same seven flags, defaults and stdout lines as simulator.go:186-253, driven
// through the C ABI (include/gossip.h).  Durations are SIMULATED time
// (1 tick = 1 ms, the unit of simulator.go:167) printed with Go's
// time.Duration format; wall-clock figures go to stderr.  Additive flags
// (-seed -trial -device -peers -maxticks) are not echoed in the parameter
// block, so stdout keeps the reference's shape.
#include <chrono>
#include <cinttypes>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "gossip.h"

namespace {

struct Flag {
  const char* name;
  const char* type;  // Go UnquoteUsage type name
  const char* usage;
  std::string defv;  // Go default as printed
  bool echo;         // part of the reference's flag set (echoed, :197-204)
  std::string val;
};

std::vector<Flag> g_flags;
const char* g_prog = "gossip_sim";

Flag* find(const std::string& name) {
  for (auto& f : g_flags)
    if (name == f.name) return &f;
  return nullptr;
}

std::string gofloat(double x) {
  char b[64];
  gs_format_float64(x, b, sizeof(b));
  return b;
}

void usage() {  // flag.PrintDefaults, lexical order
  fprintf(stderr, "Usage of %s:\n", g_prog);
  std::map<std::string, Flag*> sorted;
  for (auto& f : g_flags) sorted[f.name] = &f;
  for (auto& kv : sorted) {
    Flag* f = kv.second;
    std::string b = std::string("  -") + f->name;
    if (f->type[0]) b += std::string(" ") + f->type;
    b += (b.size() <= 4) ? "\t" : "\n    \t";
    b += f->usage;
    const bool zero = f->defv == "0" || f->defv.empty();
    if (!zero) {
      if (!strcmp(f->type, "string")) b += " (default \"" + f->defv + "\")";
      else b += " (default " + f->defv + ")";
    }
    fprintf(stderr, "%s\n", b.c_str());
  }
}

[[noreturn]] void die_usage(const std::string& msg) {
  fprintf(stderr, "%s\n", msg.c_str());
  usage();
  exit(2);
}

bool parse_int(const std::string& s, long long& out) {  // strconv.ParseInt(s, 0, 64)
  std::string t;
  for (char ch : s) if (ch != '_') t.push_back(ch);
  if (t.empty()) return false;
  char* end = nullptr;
  errno = 0;
  out = strtoll(t.c_str(), &end, 0);
  return errno == 0 && end && *end == 0;
}

bool parse_float(const std::string& s, double& out) {
  if (s.empty()) return false;
  char* end = nullptr;
  out = strtod(s.c_str(), &end);
  return end && *end == 0;
}

// Go flag.Parse semantics (ExitOnError): -name=v, -name v, --name; stops at
// the first non-flag or after "--"; -h/-help prints usage and exits 0.
void parse(int argc, char** argv) {
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    if (a.size() < 2 || a[0] != '-') break;
    if (a == "--") break;
    std::string body = a.substr(a[1] == '-' ? 2 : 1);
    if (body.empty() || body[0] == '-' || body[0] == '=')
      die_usage("bad flag syntax: " + a);
    std::string name = body, value;
    bool has = false;
    const size_t eq = body.find('=');
    if (eq != std::string::npos) { name = body.substr(0, eq); value = body.substr(eq + 1); has = true; }
    Flag* f = find(name);
    if (!f) {
      if (name == "h" || name == "help") { usage(); exit(0); }
      die_usage("flag provided but not defined: -" + name);
    }
    if (!has) {
      if (i + 1 >= argc) die_usage("flag needs an argument: -" + name);
      value = argv[++i];
    }
    if (!strcmp(f->type, "int") || !strcmp(f->type, "uint")) {
      long long v;
      if (!parse_int(value, v) || (!strcmp(f->type, "uint") && v < 0))
        die_usage("invalid value \"" + value + "\" for flag -" + name + ": parse error");
      f->val = std::to_string(v);
    } else if (!strcmp(f->type, "float")) {
      double v;
      if (!parse_float(value, v))
        die_usage("invalid value \"" + value + "\" for flag -" + name + ": parse error");
      f->val = gofloat(v);
    } else {
      f->val = value;
    }
  }
}

long long ival(const char* n) { return strtoll(find(n)->val.c_str(), nullptr, 10); }
double fval(const char* n) { return strtod(find(n)->val.c_str(), nullptr); }

std::string dur_ms(uint64_t ticks) {
  char b[64];
  gs_format_duration((int64_t)ticks * 1000000ll, b, sizeof(b));
  return b;
}

int die(gs_ctx* c, int rc, const char* what) {
  fprintf(stderr, "%s: %s failed: %s (%s)\n", g_prog, what, gs_strerror(rc),
          c ? gs_last_error(c) : "");
  if (c) gs_destroy(c);
  return 1;
}

// Injected peer table (DESIGN.md "peer-table file"): "GSPEERS1", u64 n,
// u32 stride, u32 reserved, u8 deg[n], pad to 4, u32 ids[n*stride].
bool load_peers_file(const std::string& path, uint64_t n, std::vector<uint8_t>& deg,
                     std::vector<uint32_t>& ids, uint32_t& stride) {
  FILE* f = fopen(path.c_str(), "rb");
  if (!f) { fprintf(stderr, "%s: cannot open %s\n", g_prog, path.c_str()); return false; }
  char magic[8];
  uint64_t fn = 0;
  uint32_t hdr[2] = {0, 0};
  bool ok = fread(magic, 1, 8, f) == 8 && !memcmp(magic, "GSPEERS1", 8) &&
            fread(&fn, 8, 1, f) == 1 && fread(hdr, 4, 2, f) == 2;
  if (ok && fn != n) {
    fprintf(stderr, "%s: %s holds n=%" PRIu64 ", but -n is %" PRIu64 "\n", g_prog, path.c_str(), fn, n);
    ok = false;
  }
  stride = hdr[0];
  if (ok) {
    deg.resize(n);
    ok = fread(deg.data(), 1, n, f) == n;
    const size_t pad = (4 - (n & 3)) & 3;
    char p[4];
    if (ok && pad) ok = fread(p, 1, pad, f) == pad;
    ids.resize(n * stride);
    if (ok) ok = fread(ids.data(), 4, n * stride, f) == n * stride;
  }
  fclose(f);
  if (!ok) fprintf(stderr, "%s: %s is not a valid peer table\n", g_prog, path.c_str());
  return ok;
}

}  // namespace

int main(int argc, char** argv) {
  g_prog = argv[0];
  // simulator.go:187-193 (fanin's default is Fanout+1 evaluated before Parse: 6)
  g_flags = {
      {"n", "int", "total number of nodes", "50000", true, "50000"},
      {"fanout", "int", "fanout", "5", true, "5"},
      {"fanin", "int", "fanin", "6", true, "6"},
      {"delaylow", "int", "delay low (ms)", "10", true, "10"},
      {"delayhigh", "int", "delay high (ms)", "20", true, "20"},
      {"droprate", "float", "message drop rate", "0.1", true, "0.1"},
      {"crashrate", "float", "machine crash rate", "0.001", true, "0.001"},
      {"seed", "uint", "Philox key for every random decision", "1", false, "1"},
      {"trial", "uint", "Philox trial index", "0", false, "0"},
      {"device", "int", "HIP device ordinal", "0", false, "0"},
      {"gpus", "int", "node-range shards over devices device .. device+gpus-1 (one process)", "1", false,
       "1"},
      {"peers", "string", "injected peer-table file (skips overlay construction)", "", false, ""},
      {"model", "string", "dissemination model: flood (the reference) or pushpull (extension)",
       "flood", false, "flood"},
      {"maxticks", "int", "give up after this many simulated ms per phase", "10000000", false,
       "10000000"},
  };
  parse(argc, argv);

  printf("=== Parameters ===\n");                              // :197-204
  {
    std::map<std::string, Flag*> sorted;
    for (auto& f : g_flags) if (f.echo) sorted[f.name] = &f;
    for (auto& kv : sorted) {
      printf("%s=%s", kv.first.c_str(), kv.second->val.c_str());
      if (kv.first == "delaylow" || kv.first == "delayhigh") printf("ms");
      printf("\n");
    }
  }
  fflush(stdout);

  gs_params p{};
  p.n = (uint64_t)ival("n");
  p.fanout = (int32_t)ival("fanout");
  p.fanin = (int32_t)ival("fanin");
  p.delay_low = (int32_t)ival("delaylow");
  p.delay_high = (int32_t)ival("delayhigh");
  p.drop_rate = fval("droprate");
  p.crash_rate = fval("crashrate");
  p.seed = strtoull(find("seed")->val.c_str(), nullptr, 10);
  p.trial = (uint32_t)strtoull(find("trial")->val.c_str(), nullptr, 10);
  p.device = (int32_t)ival("device");
  const std::string model = find("model")->val;
  if (model != "flood" && model != "pushpull") {
    fprintf(stderr, "invalid value \"%s\" for flag -model: want flood or pushpull\n", model.c_str());
    return 2;
  }
  p.model = model == "pushpull" ? GS_MODEL_PUSHPULL : GS_MODEL_FLOOD;
  const uint64_t max_ticks = (uint64_t)ival("maxticks");
  if (ival("n") <= 0) {
    fprintf(stderr, "panic: invalid argument to Intn\n");  // simulator.go:240 with N=0
    return 2;
  }
  gs_ctx* c = nullptr;
  int rc;
  const int64_t gpus = ival("gpus");
  if (gpus > 1) {
    std::vector<int> devs;
    for (int64_t i = 0; i < gpus; ++i) devs.push_back((int)(p.device + i));
    rc = gs_create_multi(&p, devs.data(), (int)gpus, &c);
  } else {
    rc = gs_create(&p, &c);
  }
  if (rc) return die(nullptr, rc, "gs_create");

  printf("\n=== Constructing Overlay ===\n");                   // :219
  const auto w0 = std::chrono::steady_clock::now();
  const std::string peers = find("peers")->val;
  uint64_t stab = 0;
  if (!peers.empty()) {
    std::vector<uint8_t> deg;
    std::vector<uint32_t> ids;
    uint32_t stride = 0;
    if (!load_peers_file(peers, p.n, deg, ids, stride)) { gs_destroy(c); return 1; }
    rc = gs_load_peers(c, deg.data(), ids.data(), stride);
    if (rc) return die(c, rc, "gs_load_peers");
    stab = 10;  // one empty poll window: nothing to construct
  } else {
    std::vector<gs_window> win(1 << 16);
    size_t nwin = 0;
    rc = gs_build_overlay(c, max_ticks, win.data(), win.size(), &nwin, &stab);
    if (rc) return die(c, rc, "gs_build_overlay");
    for (size_t i = 0; i < nwin && i < win.size(); ++i)     // :230
      printf("break %" PRIu64 " makeup %" PRIu64 " elasped %s\n", win[i].breakups, win[i].makeups,
             dur_ms(win[i].tick).c_str());
  }
  printf("--- Took %s to stabilize ---\n\n", dur_ms(stab).c_str()); // :235
  const double ov_wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - w0).count();

  printf("=== Broadcast one message ===\n");                    // :237
  fflush(stdout);
  const auto b0 = std::chrono::steady_clock::now();
  rc = gs_broadcast_begin(c, -1);                               // :239-241
  if (rc) return die(c, rc, "gs_broadcast_begin");
  // gs_run is the poll loop (:243-251) with the engine's stop rule: one row
  // per 10-ms poll, printed in the reference's format
  std::vector<gs_tick_stats> polls((size_t)std::min<uint64_t>(max_ticks / 10 + 2, 1u << 20));
  size_t npoll = 0;
  int32_t status = GS_RUN_MAX_TICKS;
  rc = gs_run(c, 10, max_ticks, polls.data(), polls.size(), &npoll, &status);
  if (rc) return die(c, rc, "gs_run");
  for (size_t i = 0; i < npoll && i < polls.size(); ++i) {
    const float percent = (float)polls[i].received / (float)p.n;
    char pb[64];
    gs_format_float32(percent * 100.0f, pb, sizeof(pb));
    printf("%s%% covered, took %s\n", pb, dur_ms(polls[i].tick).c_str());
  }
  gs_tick_stats tot{};
  gs_totals(c, &tot);
  const double bc_wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - b0).count();
  if (status != GS_RUN_COVERED) {
    fflush(stdout);
    fprintf(stderr, "%s: %s before 99%% coverage (the reference would poll forever)\n", g_prog,
            status == GS_RUN_QUIESCENT ? "no broadcast left in flight" : "-maxticks reached");
    gs_destroy(c);
    return 3;
  }
  printf("--- Took %s to get 99%% ---\n\n", dur_ms(tot.tick).c_str());  // :252
  printf("Total message %" PRIu64 " Total Crashed %" PRIu64 "\n", tot.messages, tot.crashed); // :253
  fflush(stdout);
  fprintf(stderr,
          "[gossip_sim] wall: overlay %.3f s, broadcast %.3f s; %" PRIu64
          " delivered sends -> %.3e msgs/s\n",
          ov_wall, bc_wall, tot.sent, bc_wall > 0 ? (double)tot.sent / bc_wall : 0.0);
  gs_destroy(c);
  return 0;
}
