// gs_devmem.cpp -- process-wide cache of large device blocks (gs_devmem.h).
//
// Layout: every block >= kCacheMin comes from a slab (one hipMalloc).  A slab
// is cut into extents, each used or free; free extents are indexed by size per
// device for best fit.  An allocation takes the smallest free extent that fits
// and splits off the rest; a free coalesces with free neighbours of the same
// slab, so a slab whose extents are all free is one extent again and can be
// trimmed.  Only when no free extent fits is a new slab mapped; if the device
// lacks the room beside the cache, fully free slabs are trimmed first, largest
// first, as many as the request needs.
#include "gs_devmem.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <iterator>
#include <map>
#include <mutex>
#include <vector>

namespace {

constexpr size_t kCacheMin = 64ull << 20;  // smaller blocks: plain hipMalloc / hipFree
constexpr size_t kGran = 2ull << 20;
// device memory left to the rest of the process (RCCL's buffers, torch, a
// small hipMalloc): a new slab is mapped only with this much beside it, and a
// free that leaves the device with less returns cached slabs until it has it
constexpr size_t kMargin = 8ull << 30;

bool logging() {
  static const bool on = getenv("GS_DEVMEM_LOG") != nullptr;
  return on;
}

struct Ext {
  size_t size;
  int slab;
  bool used;
};
struct Slab {
  char* base;
  size_t size;
  int device;
  size_t used;
};

struct Cache {
  std::mutex mu;
  std::map<char*, Ext> ext;                            // every extent, by address
  std::map<int, std::multimap<size_t, char*>> freeix;  // device -> free extents by size
  std::vector<Slab> slab;                              // size 0 = returned to the driver
  DevMemStats st{};
};

Cache& cache() {
  static Cache* c = new Cache;  // never destroyed: frees may run at process exit
  return *c;
}

bool enabled() {
  static const bool on = [] {
    const char* s = getenv("GS_DEVMEM_CACHE");
    return !(s && atoi(s) == 0);
  }();
  return on;
}

double now_ms() {
  using namespace std::chrono;
  return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

hipError_t timed_malloc(Cache& c, void** p, size_t bytes) {
  const double t0 = now_ms();
  const hipError_t e = hipMalloc(p, bytes);
  const double dt = now_ms() - t0;
  std::lock_guard<std::mutex> g(c.mu);
  c.st.alloc_ms += dt;
  if (dt > c.st.largest_alloc_ms) c.st.largest_alloc_ms = dt;
  ++c.st.hip_allocs;
  if (logging() && bytes >= (1ull << 30))  // GS_DEVMEM_LOG: every hipMalloc of >= 1 GiB
    fprintf(stderr, "[devmem] hipMalloc %.2f GiB: %.1f ms%s (cached free %.2f GiB, mapped %.2f GiB)\n",
            bytes / 1073741824.0, dt, e == hipSuccess ? "" : " FAILED", c.st.cached_bytes / 1073741824.0,
            c.st.mapped_bytes / 1073741824.0);
  return e;
}

void unindex(Cache& c, int dev, char* b, size_t size) {
  auto& fi = c.freeix[dev];
  auto r = fi.equal_range(size);
  for (auto it = r.first; it != r.second; ++it)
    if (it->second == b) {
      fi.erase(it);
      return;
    }
}

// caller holds c.mu; returns the slabs to hipFree (done outside the lock).
// Fully free slabs of `device` (-1: all) worth at least `want` bytes (~0: all
// of them): the smallest single slab that covers `want` if there is one, else
// the largest first -- as few bytes back to the driver as the request needs.
std::vector<char*> collect_trim(Cache& c, int device, size_t want = ~(size_t)0) {
  std::vector<size_t> idx;
  for (size_t i = 0; i < c.slab.size(); ++i) {
    const Slab& s = c.slab[i];
    if (s.size && !s.used && (device < 0 || s.device == device)) idx.push_back(i);
  }
  std::sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return c.slab[a].size > c.slab[b].size; });
  if (want != ~(size_t)0) {
    for (size_t k = idx.size(); k-- > 0;)  // ascending sizes
      if (c.slab[idx[k]].size >= want) {
        idx = {idx[k]};
        break;
      }
  }
  std::vector<char*> out;
  size_t got = 0;
  for (size_t i : idx) {
    if (got >= want) break;
    Slab& s = c.slab[i];
    unindex(c, s.device, s.base, s.size);  // a free slab is one extent
    c.ext.erase(s.base);
    c.st.cached_bytes -= s.size;
    c.st.mapped_bytes -= s.size;
    out.push_back(s.base);
    got += s.size;
    s.size = 0;
  }
  return out;
}

void release(Cache& c, const std::vector<char*>& blocks) {
  for (char* b : blocks) {
    const double t0 = now_ms();
    (void)hipFree(b);
    std::lock_guard<std::mutex> g(c.mu);
    c.st.free_ms += now_ms() - t0;
  }
  if (logging() && !blocks.empty()) fprintf(stderr, "[devmem] returned %zu cached slab(s) to the driver\n", blocks.size());
}

}  // namespace

namespace {
// Best-fit from the free extents of `dev` (caller holds c.mu).  With `picky`,
// an extent more than 4x the request (and more than 1 GiB over it) is left
// alone: a small buffer carved out of a big free slab pins the slab, which can
// then never be returned to the driver when a big request needs the room.
char* take_cached(Cache& c, int dev, size_t need, bool picky) {
  auto& fi = c.freeix[dev];
  auto it = fi.lower_bound(need);
  if (it == fi.end()) return nullptr;
  if (picky && it->first > 4 * need && it->first - need > (1ull << 30)) return nullptr;
  char* b = it->second;
  fi.erase(it);
  Ext& x = c.ext[b];
  if (x.size - need >= kGran) {  // split: the tail stays free
    c.ext[b + need] = Ext{x.size - need, x.slab, false};
    fi.emplace(x.size - need, b + need);
    x.size = need;
  }
  x.used = true;
  c.slab[x.slab].used += x.size;
  c.st.cached_bytes -= x.size;
  ++c.st.cache_hits;
  return b;
}
}  // namespace

hipError_t gs_dev_malloc(void** p, size_t bytes) {
  if (!p) return hipErrorInvalidValue;
  Cache& c = cache();
  if (!enabled() || bytes < kCacheMin) return timed_malloc(c, p, bytes);
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  const size_t need = (bytes + kGran - 1) & ~(kGran - 1);
  {
    std::lock_guard<std::mutex> g(c.mu);
    if (char* b = take_cached(c, dev, need, true)) {
      *p = b;
      return hipSuccess;
    }
  }
  // a new slab; make room beside the cache first if the device lacks it
  // (only as much as the request needs: a hipMalloc right after large
  // hipFrees is what stalls)
  size_t freeb = 0, totalb = 0;
  if (hipMemGetInfo(&freeb, &totalb) == hipSuccess && freeb < need + kMargin) {
    std::vector<char*> t;
    {
      std::lock_guard<std::mutex> g(c.mu);
      t = collect_trim(c, dev, need + kMargin - freeb);
    }
    release(c, t);
  }
  void* q = nullptr;
  e = timed_malloc(c, &q, need);
  if (e != hipSuccess) {
    // no room: any cached extent that fits, however big; then every fully free
    // slab back to the driver and one more try
    (void)hipGetLastError();
    std::vector<char*> t;
    {
      std::lock_guard<std::mutex> g(c.mu);
      if (char* b = take_cached(c, dev, need, false)) {
        *p = b;
        return hipSuccess;
      }
      t = collect_trim(c, dev);
    }
    if (t.empty()) return e;
    release(c, t);
    e = timed_malloc(c, &q, need);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      std::lock_guard<std::mutex> g(c.mu);
      if (char* b = take_cached(c, dev, need, false)) {  // (another thread freed one meanwhile)
        *p = b;
        return hipSuccess;
      }
      return e;
    }
  }
  std::lock_guard<std::mutex> g(c.mu);
  c.slab.push_back(Slab{(char*)q, need, dev, need});
  c.ext[(char*)q] = Ext{need, (int)c.slab.size() - 1, true};
  c.st.mapped_bytes += need;
  *p = q;
  return hipSuccess;
}

namespace {
// After a free: keep kMargin of device memory for the rest of the process
// (hipFree'd memory comes back slowly, so only what the margin needs).
void keep_headroom(int dev) {
  Cache& c = cache();
  int cur = 0;
  (void)hipGetDevice(&cur);
  if (cur != dev) (void)hipSetDevice(dev);
  size_t freeb = 0, totalb = 0;
  if (hipMemGetInfo(&freeb, &totalb) == hipSuccess && freeb < kMargin) {
    std::vector<char*> t;
    {
      std::lock_guard<std::mutex> g(c.mu);
      t = collect_trim(c, dev, kMargin - freeb);
    }
    release(c, t);
  }
  if (cur != dev) (void)hipSetDevice(cur);
}
}  // namespace

hipError_t gs_dev_free(void* p) {
  if (!p) return hipSuccess;
  Cache& c = cache();
  int sdev = -1;
  {
    std::lock_guard<std::mutex> g(c.mu);
    auto it = c.ext.find((char*)p);
    if (it != c.ext.end() && it->second.used) sdev = c.slab[it->second.slab].device;
  }
  if (sdev < 0) {  // not a cached block
    const double t0 = now_ms();
    const hipError_t e = hipFree(p);
    std::lock_guard<std::mutex> g(c.mu);
    c.st.free_ms += now_ms() - t0;
    return e;
  }
  // hipFree's contract: the block is idle before anyone can reuse it
  const double t0 = now_ms();
  int cur = 0;
  (void)hipGetDevice(&cur);
  if (cur != sdev) (void)hipSetDevice(sdev);
  const hipError_t se = hipDeviceSynchronize();
  if (cur != sdev) (void)hipSetDevice(cur);
  {
    std::lock_guard<std::mutex> g(c.mu);
    c.st.free_ms += now_ms() - t0;
    auto it = c.ext.find((char*)p);
    if (it == c.ext.end() || !it->second.used) return hipErrorInvalidValue;  // freed twice
    Ext x = it->second;
    Slab& s = c.slab[x.slab];
    s.used -= x.size;
    c.st.cached_bytes += x.size;
    char* b = (char*)p;
    auto& fi = c.freeix[s.device];
    // coalesce with the next extent of the same slab
    auto nx = std::next(it);
    if (nx != c.ext.end() && !nx->second.used && nx->second.slab == x.slab && b + x.size == nx->first) {
      unindex(c, s.device, nx->first, nx->second.size);
      x.size += nx->second.size;
      c.ext.erase(nx);
    }
    // and with the previous one
    bool merged = false;
    if (it != c.ext.begin()) {
      auto pv = std::prev(it);
      if (!pv->second.used && pv->second.slab == x.slab && pv->first + pv->second.size == b) {
        unindex(c, s.device, pv->first, pv->second.size);
        pv->second.size += x.size;
        c.ext.erase(it);
        fi.emplace(pv->second.size, pv->first);
        merged = true;
      }
    }
    if (!merged) {
      it->second = Ext{x.size, x.slab, false};
      fi.emplace(x.size, b);
    }
  }
  keep_headroom(sdev);
  return se;
}


void gs_devmem_stats(DevMemStats* out) {
  if (!out) return;
  Cache& c = cache();
  std::lock_guard<std::mutex> g(c.mu);
  *out = c.st;
}

size_t gs_devmem_largest() {
  Cache& c = cache();
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  size_t freeb = 0, totalb = 0, best = 0;
  if (hipMemGetInfo(&freeb, &totalb) == hipSuccess && freeb > kMargin) best = freeb - kMargin;
  if (!enabled()) return best;
  std::lock_guard<std::mutex> g(c.mu);
  auto it = c.freeix.find(dev);
  if (it != c.freeix.end() && !it->second.empty()) best = std::max(best, it->second.rbegin()->first);
  return best;
}

size_t gs_devmem_trim(int device) {
  Cache& c = cache();
  std::vector<char*> t;
  size_t bytes = 0;
  {
    std::lock_guard<std::mutex> g(c.mu);
    const uint64_t before = c.st.mapped_bytes;
    t = collect_trim(c, device);
    bytes = (size_t)(before - c.st.mapped_bytes);
  }
  release(c, t);
  return bytes;
}
