// gs_comm.h -- the RCCL calls a multi-process node-range shard makes
// (all-gather of each window's fire counts and message
// layout, an all-to-all of its messages as grouped send/recv, sum of the
// per-tick counters).  RCCL has no bitwise-OR reduction, so nothing here ORs.
#pragma once
#include <rccl/rccl.h>

#include <string>

namespace gs {

struct Rccl {
  bool ok = false;
  std::string why;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

const Rccl& rccl();
std::string rccl_error(int rc);

}  // namespace gs
