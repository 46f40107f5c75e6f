// comm.hip -- the eval all-gather over RCCL behind the C-ABI (include/ogbx.h).
//
// Reference: impls/main.py:226-258 (per-task success means over all
// evaluation workers).  The counters are int64[num_tasks, 2] per rank
// (eval.hip); ncclAllGather over xGMI collects them on every rank.
//
// RCCL is bound at run time with dlopen/dlsym: a process that already holds a
// librccl.so.1 (PyTorch bundles one) must not load a second copy, and hosts
// that never evaluate across ranks do not need RCCL at all.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstring>
#include <string>

#include "common.h"

struct ogbx_comm {
  ncclComm_t comm = nullptr;
  int32_t world = 0, rank = 0, device = 0;
};

namespace {

struct Rccl {
  decltype(&ncclGetUniqueId) get_id = nullptr;
  decltype(&ncclCommInitRank) init = nullptr;
  decltype(&ncclAllGather) allgather = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclGetErrorString) err = nullptr;
  std::string why;
  bool ok() const { return get_id && init && allgather && destroy && err; }
};

const Rccl& rccl() {
  static const Rccl r = [] {
    Rccl x;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);  // the copy already in the process
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
      const char* e = dlerror();
      x.why = std::string("librccl.so.1 not found: ") + (e ? e : "");
      return x;
    }
    x.get_id = reinterpret_cast<decltype(x.get_id)>(dlsym(h, "ncclGetUniqueId"));
    x.init = reinterpret_cast<decltype(x.init)>(dlsym(h, "ncclCommInitRank"));
    x.allgather = reinterpret_cast<decltype(x.allgather)>(dlsym(h, "ncclAllGather"));
    x.destroy = reinterpret_cast<decltype(x.destroy)>(dlsym(h, "ncclCommDestroy"));
    x.err = reinterpret_cast<decltype(x.err)>(dlsym(h, "ncclGetErrorString"));
    if (!x.ok()) x.why = "librccl.so.1 lacks an nccl* entry point";
    return x;
  }();
  return r;
}

}  // namespace

using namespace ogbx;

#define OGBX_RCCL(call, what)                                                        \
  do {                                                                               \
    const ncclResult_t _r = (call);                                                  \
    if (_r != ncclSuccess) return fail(OGBX_EDEVICE, std::string(what) + ": " + rccl().err(_r)); \
  } while (0)

extern "C" {

ogbx_status ogbx_comm_unique_id(uint8_t* id) {
  OGBX_CHECK(id, OGBX_EINVAL, "ogbx_comm_unique_id: null argument");
  OGBX_CHECK(rccl().ok(), OGBX_EDEVICE, rccl().why);
  ncclUniqueId uid;
  static_assert(sizeof(uid) == OGBX_COMM_ID_BYTES, "RCCL unique id size");
  OGBX_RCCL(rccl().get_id(&uid), "ncclGetUniqueId");
  std::memcpy(id, &uid, sizeof(uid));
  return OGBX_OK;
}

ogbx_status ogbx_comm_create(const uint8_t* id, int32_t world_size, int32_t rank, int32_t device,
                             ogbx_comm_t* out) {
  OGBX_CHECK(id && out, OGBX_EINVAL, "ogbx_comm_create: null argument");
  *out = nullptr;
  OGBX_CHECK(world_size >= 1 && rank >= 0 && rank < world_size, OGBX_EINVAL, "ogbx_comm_create: bad rank");
  OGBX_CHECK(rccl().ok(), OGBX_EDEVICE, rccl().why);
  ogbx_status st = use_device(device);
  if (st != OGBX_OK) return st;
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  auto* c = new ogbx_comm();
  c->world = world_size, c->rank = rank, c->device = device;
  const ncclResult_t r = rccl().init(&c->comm, world_size, uid, rank);
  if (r != ncclSuccess) {
    delete c;
    return fail(OGBX_EDEVICE, std::string("ncclCommInitRank: ") + rccl().err(r));
  }
  *out = c;
  return OGBX_OK;
}

ogbx_status ogbx_comm_destroy(ogbx_comm_t c) {
  if (!c) return OGBX_OK;
  if (c->comm && rccl().ok()) (void)rccl().destroy(c->comm);
  delete c;
  return OGBX_OK;
}

ogbx_status ogbx_eval_allgather(ogbx_comm_t c, const int64_t* local, int64_t count, int64_t* all,
                                void* stream) {
  OGBX_CHECK(c && c->comm && local && all && count >= 0, OGBX_EINVAL, "ogbx_eval_allgather: bad argument");
  if (count == 0) return OGBX_OK;
  OGBX_HIP(hipSetDevice(c->device));
  OGBX_RCCL(rccl().allgather(local, all, (size_t)count, ncclInt64, c->comm, (hipStream_t)stream),
            "ncclAllGather");
  return OGBX_OK;
}

}  // extern "C"
