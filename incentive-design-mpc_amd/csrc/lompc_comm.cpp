// lompc_comm.cpp — the extension's own RCCL communicator (C-ABI in include/lompc_amd.h).
//
// The reference runs every LoMPC of a price iteration in one process (price_solver.py:203-209);
// the sharded engine splits each partition's EVs across one process per GPU, and the only
// exchange of an iteration is the per-set reduction record the price step consumes (sum of w,
// max A_bar error, sums of cost / price0 / counts — price_solver.py:205-214, the aggregate demand
// of charging_station.py:356-366).  With a communicator attached to a plan
// (lompc_plan_set_comm) every run closes its sets into one packed record, all-gathers it over
// xGMI and combines the ranks' records in rank order on the device (lompc_plan.hip, k_combine):
// the collective is issued on the plan's stream by the C++ price loop itself, so a sharded price
// iteration has no Python in it.
//
// RCCL is resolved with dlopen at the first communicator: when PyTorch-ROCm is loaded, its
// librccl.so.1 is the copy already in the process (same soname) and is reused; otherwise the
// system library is loaded.  The library itself has no link-time dependency on RCCL.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <string.h>

#include <mutex>

#include "lompc_ctx.hpp"

namespace {

struct RcclApi {
  void* h = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  bool ok = false;
};

RcclApi g_api;
std::once_flag g_once;

void load_api() {
  for (const char* name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"}) {
    g_api.h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
    if (g_api.h) break;
  }
  if (!g_api.h) return;
  g_api.get_unique_id = (decltype(g_api.get_unique_id))dlsym(g_api.h, "ncclGetUniqueId");
  g_api.init_rank = (decltype(g_api.init_rank))dlsym(g_api.h, "ncclCommInitRank");
  g_api.destroy = (decltype(g_api.destroy))dlsym(g_api.h, "ncclCommDestroy");
  g_api.all_gather = (decltype(g_api.all_gather))dlsym(g_api.h, "ncclAllGather");
  g_api.error_string = (decltype(g_api.error_string))dlsym(g_api.h, "ncclGetErrorString");
  g_api.ok = g_api.get_unique_id && g_api.init_rank && g_api.destroy && g_api.all_gather && g_api.error_string;
}

bool api() {
  std::call_once(g_once, load_api);
  return g_api.ok;
}

}  // namespace

int lq_comm_allgather(lompc_comm* c, const double* send, double* recv, size_t count, hipStream_t st) {
  const ncclResult_t r = g_api.all_gather(send, recv, count, ncclFloat64, (ncclComm_t)c->nccl, st);
  if (r != ncclSuccess) {
    c->err = std::string("ncclAllGather: ") + g_api.error_string(r);
    return LOMPC_ERR_HIP;
  }
  return LOMPC_OK;
}

extern "C" {

int lompc_comm_get_unique_id(unsigned char* id) {
  if (!id) return LOMPC_ERR_INVALID_ARG;
  if (!api()) return LOMPC_ERR_UNSUPPORTED;
  static_assert(sizeof(ncclUniqueId) == LOMPC_COMM_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId u;
  if (g_api.get_unique_id(&u) != ncclSuccess) return LOMPC_ERR_HIP;
  memcpy(id, &u, sizeof(u));
  return LOMPC_OK;
}

int lompc_comm_create(const unsigned char* id, int nranks, int rank, int device, lompc_comm** out) {
  if (!out) return LOMPC_ERR_INVALID_ARG;
  *out = nullptr;
  if (!id || nranks < 1 || rank < 0 || rank >= nranks || device < 0) return LOMPC_ERR_INVALID_ARG;
  if (!api()) return LOMPC_ERR_UNSUPPORTED;
  if (hipSetDevice(device) != hipSuccess) return LOMPC_ERR_HIP;
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  ncclComm_t comm = nullptr;
  if (g_api.init_rank(&comm, nranks, u, rank) != ncclSuccess) return LOMPC_ERR_HIP;  // collective over the ranks
  lompc_comm* c = new lompc_comm();
  c->nccl = comm;
  c->nranks = nranks;
  c->rank = rank;
  c->device = device;
  *out = c;
  return LOMPC_OK;
}

int lompc_comm_destroy(lompc_comm* c) {
  if (!c) return LOMPC_OK;
  int rc = LOMPC_OK;
  if (c->nccl) {
    (void)hipSetDevice(c->device);
    if (g_api.destroy((ncclComm_t)c->nccl) != ncclSuccess) rc = LOMPC_ERR_HIP;
  }
  delete c;
  return rc;
}

}  // extern "C"
