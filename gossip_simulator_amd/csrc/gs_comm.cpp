// gs_comm.cpp -- RCCL entry points for multi-process node-range shards,
// resolved with dlopen at first use, so libgossip_hip.so loads (and every
// single-process path runs) on hosts without RCCL.  When the process already
// holds librccl.so.1 (PyTorch ships one), that copy is reused: one RCCL
// instance per process.
#include <dlfcn.h>

#include <mutex>
#include <string>

#include "gs_comm.h"

namespace gs {

static Rccl g_rccl;
static std::once_flag g_once;

const Rccl& rccl() {
  std::call_once(g_once, [] {
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      g_rccl.why = std::string("cannot load librccl.so.1: ") + dlerror();
      return;
    }
    bool ok = true;
    auto sym = [&](const char* name) {
      void* f = dlsym(h, name);
      if (!f) ok = false;
      return f;
    };
    g_rccl.get_unique_id = (decltype(g_rccl.get_unique_id))sym("ncclGetUniqueId");
    g_rccl.comm_init_rank = (decltype(g_rccl.comm_init_rank))sym("ncclCommInitRank");
    g_rccl.comm_destroy = (decltype(g_rccl.comm_destroy))sym("ncclCommDestroy");
    g_rccl.comm_abort = (decltype(g_rccl.comm_abort))sym("ncclCommAbort");
    g_rccl.all_gather = (decltype(g_rccl.all_gather))sym("ncclAllGather");
    g_rccl.all_reduce = (decltype(g_rccl.all_reduce))sym("ncclAllReduce");
    g_rccl.send = (decltype(g_rccl.send))sym("ncclSend");
    g_rccl.recv = (decltype(g_rccl.recv))sym("ncclRecv");
    g_rccl.group_start = (decltype(g_rccl.group_start))sym("ncclGroupStart");
    g_rccl.group_end = (decltype(g_rccl.group_end))sym("ncclGroupEnd");
    g_rccl.error_string = (decltype(g_rccl.error_string))sym("ncclGetErrorString");
    g_rccl.ok = ok;
    if (!ok) g_rccl.why = "librccl.so.1 lacks an entry point this engine needs";
  });
  return g_rccl;
}

std::string rccl_error(int rc) {
  const Rccl& r = rccl();
  if (r.ok && r.error_string) return r.error_string((ncclResult_t)rc);
  return "RCCL error " + std::to_string(rc);
}

}  // namespace gs
