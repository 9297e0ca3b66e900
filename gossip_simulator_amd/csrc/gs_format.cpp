// gs_format.cpp -- Go's fmt %v / flag / time.Duration formatting, so the CLI
// prints the reference's stdout lines byte-for-byte in shape
// (simulator.go:197-204, 230, 235, 247, 252, 253).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "gossip.h"

namespace {

// Shortest decimal digits that round-trip (strconv 'g', -1): returns digits
// (no leading zeros) and dp = decimal-point position (value = 0.d1d2.. * 10^dp).
template <bool F32>
void shortest(double x, std::string& digits, int& dp) {
  char buf[64];
  const int maxp = F32 ? 9 : 17;
  for (int p = 1; p <= maxp; ++p) {
    snprintf(buf, sizeof(buf), "%.*e", p - 1, x);
    bool ok;
    if (F32) ok = strtof(buf, nullptr) == (float)x;
    else ok = strtod(buf, nullptr) == x;
    if (ok || p == maxp) break;
  }
  // buf = d.ddddde[+-]XX
  const char* e = strchr(buf, 'e');
  int exp10 = atoi(e + 1);
  digits.clear();
  for (const char* c = buf; c < e; ++c)
    if (*c >= '0' && *c <= '9') digits.push_back(*c);
  while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
  dp = exp10 + 1;
}

// strconv.FormatFloat(x, 'g', -1, bits) as used by fmt %v and flag.Value.
template <bool F32>
std::string go_g(double x) {
  if (std::isnan(x)) return "NaN";
  if (std::isinf(x)) return x > 0 ? "+Inf" : "-Inf";
  std::string out;
  if (std::signbit(x)) { out.push_back('-'); x = -x; }
  if (x == 0) return out + "0";
  std::string d;
  int dp;
  shortest<F32>(x, d, dp);
  const int nd = (int)d.size();
  const int exp = dp - 1;
  if (exp < -4 || exp >= 6) {  // shortest: eprec = 6 (strconv/ftoa.go)
    out.push_back(d[0]);
    if (nd > 1) { out.push_back('.'); out.append(d, 1, std::string::npos); }
    char eb[16];
    snprintf(eb, sizeof(eb), "e%c%02d", exp < 0 ? '-' : '+', exp < 0 ? -exp : exp);
    return out + eb;
  }
  if (dp <= 0) {
    out += "0.";
    out.append((size_t)(-dp), '0');
    out += d;
  } else if (dp >= nd) {
    out += d;
    out.append((size_t)(dp - nd), '0');
  } else {
    out.append(d, 0, (size_t)dp);
    out.push_back('.');
    out.append(d, (size_t)dp, std::string::npos);
  }
  return out;
}

size_t emit(const std::string& s, char* buf, size_t cap) {
  if (buf && cap) {
    size_t k = s.size() < cap - 1 ? s.size() : cap - 1;
    memcpy(buf, s.data(), k);
    buf[k] = 0;
  }
  return s.size();
}

// fmtFrac: fraction of v/10^prec without trailing zeros (time/time.go).
void frac(std::string& tail, uint64_t& v, int prec) {
  bool print = false;
  std::string f;
  for (int i = 0; i < prec; ++i) {
    const uint64_t digit = v % 10;
    print = print || digit != 0;
    if (print) f.insert(f.begin(), (char)('0' + digit));
    v /= 10;
  }
  if (print) tail = "." + f + tail;
}

}  // namespace

extern "C" size_t gs_format_float32(float x, char* buf, size_t cap) {
  return emit(go_g<true>((double)x), buf, cap);
}

extern "C" size_t gs_format_float64(double x, char* buf, size_t cap) {
  return emit(go_g<false>(x), buf, cap);
}

// time.Duration.String()
extern "C" size_t gs_format_duration(int64_t ns, char* buf, size_t cap) {
  uint64_t u = ns < 0 ? (uint64_t)(-(ns + 1)) + 1 : (uint64_t)ns;
  std::string s;
  if (u < 1000000000ull) {
    if (u == 0) return emit("0s", buf, cap);
    std::string tail;
    int prec;
    if (u < 1000ull) { prec = 0; tail = "ns"; }
    else if (u < 1000000ull) { prec = 3; tail = "\xC2\xB5s"; }
    else { prec = 6; tail = "ms"; }
    frac(tail, u, prec);
    s = std::to_string(u) + tail;
  } else {
    std::string tail = "s";
    frac(tail, u, 9);
    s = std::to_string(u % 60) + tail;
    u /= 60;
    if (u > 0) {
      s = std::to_string(u % 60) + "m" + s;
      u /= 60;
      if (u > 0) s = std::to_string(u) + "h" + s;
    }
  }
  if (ns < 0) s = "-" + s;
  return emit(s, buf, cap);
}

// Go int(rate*100) (simulator.go:172,180): float64 product, truncation.
extern "C" int32_t gs_threshold(double rate) {
  const double x = rate * 100.0;
  if (x != x) return 0;
  if (x >= 100.0) return 100;
  if (x <= 0.0) return 0;
  return (int32_t)x;
}
