// RCCL communicator behind the C-ABI (fr_comm_init / fr_allreduce_f32).
//
// The reference is single-process (utils/configurator.py:110-114 pins one device), so these
// exports are new: they let a host that binds only the C-ABI (no torch.distributed) run the
// multi-GPU exchange steps of engine/sharded.py and engine/dist.py -- the per-layer item
// all-reduce and the dense-gradient all-reduce (float sums, in place) and the row all-gather --
// over RCCL on xGMI, stream-ordered on the caller's HIP stream like every other export.
//
// RCCL is resolved at run time, not linked: the process's already-loaded copy is reused when
// there is one (PyTorch-ROCm maps its own librccl.so.1; two RCCL instances in one process would
// each set up their own proxies and channels), else librccl.so.1 from the ROCm install.  The
// library therefore loads on hosts without RCCL; the comm calls then return FR_ENOTSUP.
#include <dlfcn.h>

#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include "fr_host.h"
#include "fr_engine.h"

namespace {

struct Rccl {
  void* handle = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  std::string why;
};

Rccl& rccl() {
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    const char* names[] = {"librccl.so.1", "librccl.so"};
    for (const char* n : names) {  // a copy the process already mapped (PyTorch-ROCm's)
      r.handle = dlopen(n, RTLD_NOW | RTLD_NOLOAD | RTLD_GLOBAL);
      if (r.handle) break;
    }
    if (!r.handle) r.handle = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!r.handle) r.handle = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!r.handle) {
      const char* e = dlerror();
      r.why = std::string("RCCL not loadable: ") + (e ? e : "?");
      return;
    }
    auto sym = [&](const char* s) { return dlsym(r.handle, s); };
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(sym("ncclGetUniqueId"));
    r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(sym("ncclCommInitRank"));
    r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(sym("ncclAllReduce"));
    r.all_gather = reinterpret_cast<decltype(r.all_gather)>(sym("ncclAllGather"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(sym("ncclCommDestroy"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(sym("ncclGetErrorString"));
    if (!r.get_unique_id || !r.comm_init_rank || !r.all_reduce || !r.all_gather || !r.comm_destroy) {
      r.why = "RCCL library lacks an entry point";
      r.handle = nullptr;
    }
  });
  return r;
}

int nccl_fail(const char* what, ncclResult_t rc) {
  Rccl& r = rccl();
  return fr::fail(FR_EHIP, std::string(what) + ": RCCL error " + std::to_string(static_cast<int>(rc)) + " (" +
                               (r.error_string ? r.error_string(rc) : "?") + ")");
}

struct Comm {
  ncclComm_t comm;
  int rank, world;
};

}  // namespace

extern "C" int fr_comm_available(void) { return rccl().handle != nullptr ? 1 : 0; }

extern "C" int64_t fr_comm_unique_id_bytes(void) { return NCCL_UNIQUE_ID_BYTES; }

extern "C" int fr_comm_unique_id(void* out, int64_t out_bytes) {
  Rccl& r = rccl();
  if (!r.handle) return fr::fail(FR_ENOTSUP, "fr_comm_unique_id: " + r.why);
  FR_REQUIRE(out != nullptr && out_bytes >= NCCL_UNIQUE_ID_BYTES, "need a 128-byte buffer");
  ncclUniqueId id;
  ncclResult_t rc = r.get_unique_id(&id);
  if (rc != ncclSuccess) return nccl_fail("fr_comm_unique_id", rc);
  std::memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
  return FR_OK;
}

extern "C" int fr_comm_init(int rank, int world, const void* unique_id, void** comm) {
  Rccl& r = rccl();
  if (!r.handle) return fr::fail(FR_ENOTSUP, "fr_comm_init: " + r.why);
  FR_REQUIRE(unique_id != nullptr && comm != nullptr, "null argument");
  FR_REQUIRE(world >= 1 && rank >= 0 && rank < world, "rank / world out of range");
  ncclUniqueId id;
  std::memcpy(id.internal, unique_id, NCCL_UNIQUE_ID_BYTES);
  Comm* c = new Comm{nullptr, rank, world};
  ncclResult_t rc = r.comm_init_rank(&c->comm, world, id, rank);  // on the calling thread's device
  if (rc != ncclSuccess) {
    delete c;
    return nccl_fail("fr_comm_init", rc);
  }
  *comm = c;
  return FR_OK;
}

extern "C" int fr_allreduce_f32(void* comm, float* buf, int64_t n, void* stream) {
  Rccl& r = rccl();
  if (!r.handle) return fr::fail(FR_ENOTSUP, "fr_allreduce_f32: " + r.why);
  FR_REQUIRE(comm != nullptr && n >= 0 && (buf != nullptr || n == 0), "bad argument");
  if (n == 0) return FR_OK;
  Comm* c = static_cast<Comm*>(comm);
  ncclResult_t rc = r.all_reduce(buf, buf, static_cast<size_t>(n), ncclFloat32, ncclSum, c->comm,
                                 static_cast<hipStream_t>(stream));
  return rc == ncclSuccess ? FR_OK : nccl_fail("fr_allreduce_f32", rc);
}

extern "C" int fr_allgather_f32(void* comm, const float* send, float* recv, int64_t n, void* stream) {
  Rccl& r = rccl();
  if (!r.handle) return fr::fail(FR_ENOTSUP, "fr_allgather_f32: " + r.why);
  FR_REQUIRE(comm != nullptr && n >= 0 && ((send != nullptr && recv != nullptr) || n == 0), "bad argument");
  if (n == 0) return FR_OK;
  Comm* c = static_cast<Comm*>(comm);
  ncclResult_t rc = r.all_gather(send, recv, static_cast<size_t>(n), ncclFloat32, c->comm,
                                 static_cast<hipStream_t>(stream));
  return rc == ncclSuccess ? FR_OK : nccl_fail("fr_allgather_f32", rc);
}

extern "C" int fr_comm_destroy(void* comm) {
  if (comm == nullptr) return FR_OK;
  Rccl& r = rccl();
  Comm* c = static_cast<Comm*>(comm);
  ncclResult_t rc = r.handle ? r.comm_destroy(c->comm) : ncclSuccess;
  delete c;
  return rc == ncclSuccess ? FR_OK : nccl_fail("fr_comm_destroy", rc);
}
