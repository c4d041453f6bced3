// Inter-rank exchange: RCCL (dlopen'ed) or host callbacks.  See pgo_comm.h.
#include "pgo_comm.h"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstdlib>
#include <cstring>

namespace pgo {
namespace {

// RCCL entry points, resolved once.  dlopen("librccl.so.1") by soname first:
// when PyTorch has already loaded its own RCCL (same soname) the process keeps
// one RCCL instance; otherwise ROCm's copy is loaded.
struct Rccl {
  bool tried = false, ok = false;
  std::string why;
  decltype(&::ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&::ncclCommInitRank) init_rank = nullptr;
  decltype(&::ncclCommDestroy) destroy = nullptr;
  decltype(&::ncclAllGather) all_gather = nullptr;
  decltype(&::ncclBroadcast) broadcast = nullptr;
  decltype(&::ncclGetErrorString) error_string = nullptr;
  decltype(&::ncclGroupStart) group_start = nullptr;
  decltype(&::ncclGroupEnd) group_end = nullptr;
};

Rccl& rccl() {
  static Rccl r;
  if (r.tried) return r;
  r.tried = true;
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h) {
    const char* e = dlerror();
    r.why = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
    return r;
  }
#define PGO_SYM(field, name)                                              \
  r.field = reinterpret_cast<decltype(r.field)>(dlsym(h, name));          \
  if (!r.field) {                                                         \
    r.why = std::string("librccl.so.1 lacks ") + name;                    \
    return r;                                                             \
  }
  PGO_SYM(get_unique_id, "ncclGetUniqueId")
  PGO_SYM(init_rank, "ncclCommInitRank")
  PGO_SYM(destroy, "ncclCommDestroy")
  PGO_SYM(all_gather, "ncclAllGather")
  PGO_SYM(broadcast, "ncclBroadcast")
  PGO_SYM(error_string, "ncclGetErrorString")
  PGO_SYM(group_start, "ncclGroupStart")
  PGO_SYM(group_end, "ncclGroupEnd")
#undef PGO_SYM
  r.ok = true;
  return r;
}

int nccl_fail(ncclResult_t e, const char* what, std::string* err) {
  *err = std::string(what) + ": " + rccl().error_string(e);
  return PGO_E_COMM;
}

int hip_fail(hipError_t e, const char* what, std::string* err) {
  *err = std::string(what) + ": " + hipGetErrorString(e);
  return PGO_E_HIP;
}

}  // namespace

int comm_unique_id(void* out, size_t cap, std::string* err) {
  Rccl& r = rccl();
  if (!r.ok) {
    *err = r.why;
    return PGO_E_COMM;
  }
  if (!out || cap < sizeof(ncclUniqueId)) {
    *err = "unique id buffer smaller than NCCL_UNIQUE_ID_BYTES";
    return PGO_E_ARG;
  }
  ncclUniqueId id;
  const ncclResult_t e = r.get_unique_id(&id);
  if (e != ncclSuccess) return nccl_fail(e, "ncclGetUniqueId", err);
  std::memcpy(out, &id, sizeof(id));
  return (int)sizeof(id);
}

int comm_init_rccl(Comm* c, const void* uid, size_t uid_bytes, int rank, int size, std::string* err) {
  Rccl& r = rccl();
  if (!r.ok) {
    *err = r.why;
    return PGO_E_COMM;
  }
  if (!uid || uid_bytes != sizeof(ncclUniqueId) || size < 1 || rank < 0 || rank >= size) {
    *err = "bad RCCL unique id, rank or size";
    return PGO_E_ARG;
  }
  ncclUniqueId id;
  std::memcpy(&id, uid, sizeof(id));
  ncclComm_t comm = nullptr;
  const ncclResult_t e = r.init_rank(&comm, size, id, rank);
  if (e != ncclSuccess) return nccl_fail(e, "ncclCommInitRank", err);
  double* buf = nullptr;
  const hipError_t he = hipMalloc((void**)&buf, sizeof(double) * kMaxGather * (size_t)size);
  if (he != hipSuccess) {
    r.destroy(comm);
    return hip_fail(he, "hipMalloc(all-gather buffer)", err);
  }
  comm_free(c);
  c->rank = rank;
  c->size = size;
  c->host = false;
  c->nccl = comm;
  c->d_gather = buf;
  return PGO_OK;
}

int comm_init_host(Comm* c, const pgo_host_comm* hc, std::string* err) {
  if (!hc || !hc->allgather || !hc->broadcast || hc->size < 1 || hc->rank < 0 || hc->rank >= hc->size) {
    *err = "pgo_host_comm needs allgather, broadcast and 0 <= rank < size";
    return PGO_E_ARG;
  }
  comm_free(c);
  c->rank = hc->rank;
  c->size = hc->size;
  c->host = true;
  c->hc = *hc;
  return PGO_OK;
}

void comm_free(Comm* c) {
  if (c->nccl && rccl().ok) rccl().destroy(static_cast<ncclComm_t>(c->nccl));
  if (c->d_gather) (void)hipFree(c->d_gather);
  *c = Comm();
}

// PGO_COMM_FORCE_COLLECTIVES=1: a one-rank RCCL communicator still goes
// through ncclAllGather / ncclBroadcast (instead of the local shortcuts), so
// the collective path and its slot arithmetic run on a one-GPU box
bool force_collectives(const Comm* c) {
  if (!c->nccl) return false;
  const char* v = getenv("PGO_COMM_FORCE_COLLECTIVES");
  return v && v[0] == '1';
}

int comm_allgather(Comm* c, const double* mine, int count, double* all, hipStream_t s, std::string* err) {
  if (c->size == 1 && !force_collectives(c)) {
    std::memcpy(all, mine, sizeof(double) * count);
    return PGO_OK;
  }
  if (c->host) {
    if (c->hc.allgather(c->hc.ctx, mine, all, sizeof(double) * count) != 0) {
      *err = "host all-gather callback failed";
      return PGO_E_COMM;
    }
    return PGO_OK;
  }
  if (count > kMaxGather) {
    *err = "all-gather of more than kMaxGather doubles per rank";
    return PGO_E_ARG;
  }
  // in place: rank r's slice of the receive buffer is its send buffer
  double* slot = c->d_gather + (size_t)count * c->rank;
  hipError_t he = hipMemcpyAsync(slot, mine, sizeof(double) * count, hipMemcpyHostToDevice, s);
  if (he != hipSuccess) return hip_fail(he, "all-gather upload", err);
  const ncclResult_t e = rccl().all_gather(slot, c->d_gather, count, ncclFloat64,
                                          static_cast<ncclComm_t>(c->nccl), s);
  if (e != ncclSuccess) return nccl_fail(e, "ncclAllGather", err);
  he = hipMemcpyAsync(all, c->d_gather, sizeof(double) * count * c->size, hipMemcpyDeviceToHost, s);
  if (he != hipSuccess) return hip_fail(he, "all-gather download", err);
  he = hipStreamSynchronize(s);
  if (he != hipSuccess) return hip_fail(he, "all-gather", err);
  return PGO_OK;
}

int comm_allgather_device(Comm* c, const void* send, void* recv, size_t bytes, hipStream_t s, std::string* err) {
  hipError_t he;
  if (c->size == 1 && !force_collectives(c)) {
    he = hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, s);
    return he == hipSuccess ? PGO_OK : hip_fail(he, "all-gather copy", err);
  }
  if (c->host) {   // stage through host memory, the caller's all-gather, back
    c->stage.resize(bytes * (c->size + 1));
    char* mine = c->stage.data() + bytes * c->size;
    he = hipMemcpyAsync(mine, send, bytes, hipMemcpyDeviceToHost, s);
    if (he == hipSuccess) he = hipStreamSynchronize(s);
    if (he != hipSuccess) return hip_fail(he, "all-gather download", err);
    if (c->hc.allgather(c->hc.ctx, mine, c->stage.data(), bytes) != 0) {
      *err = "host all-gather callback failed";
      return PGO_E_COMM;
    }
    he = hipMemcpyAsync(recv, c->stage.data(), bytes * c->size, hipMemcpyHostToDevice, s);
    if (he == hipSuccess) he = hipStreamSynchronize(s);
    return he == hipSuccess ? PGO_OK : hip_fail(he, "all-gather upload", err);
  }
  const ncclResult_t e = rccl().all_gather(send, recv, bytes, ncclUint8, static_cast<ncclComm_t>(c->nccl), s);
  if (e != ncclSuccess) return nccl_fail(e, "ncclAllGather", err);
  return PGO_OK;
}

int comm_broadcast_device(Comm* c, void* dptr, size_t bytes, int root, hipStream_t s, std::string* err) {
  if ((c->size == 1 && !force_collectives(c)) || bytes == 0) return PGO_OK;
  hipError_t he;
  if (c->host) {
    c->stage.resize(bytes);
    if (c->rank == root) {
      he = hipMemcpyAsync(c->stage.data(), dptr, bytes, hipMemcpyDeviceToHost, s);
      if (he == hipSuccess) he = hipStreamSynchronize(s);
      if (he != hipSuccess) return hip_fail(he, "broadcast download", err);
    }
    if (c->hc.broadcast(c->hc.ctx, c->stage.data(), bytes, root) != 0) {
      *err = "host broadcast callback failed";
      return PGO_E_COMM;
    }
    if (c->rank != root) {
      he = hipMemcpyAsync(dptr, c->stage.data(), bytes, hipMemcpyHostToDevice, s);
      if (he == hipSuccess) he = hipStreamSynchronize(s);
      if (he != hipSuccess) return hip_fail(he, "broadcast upload", err);
    }
    return PGO_OK;
  }
  const ncclResult_t e = rccl().broadcast(dptr, dptr, bytes, ncclUint8, root, static_cast<ncclComm_t>(c->nccl), s);
  if (e != ncclSuccess) return nccl_fail(e, "ncclBroadcast", err);
  he = hipStreamSynchronize(s);
  if (he != hipSuccess) return hip_fail(he, "broadcast", err);
  return PGO_OK;
}

int comm_broadcast_device_async(Comm* c, void* dptr, size_t bytes, int root, hipStream_t s, std::string* err) {
  if ((c->size == 1 && !force_collectives(c)) || bytes == 0 || c->host)
    return comm_broadcast_device(c, dptr, bytes, root, s, err);   // (the host transport synchronises anyway)
  const ncclResult_t e = rccl().broadcast(dptr, dptr, bytes, ncclUint8, root, static_cast<ncclComm_t>(c->nccl), s);
  return e == ncclSuccess ? PGO_OK : nccl_fail(e, "ncclBroadcast", err);
}

int comm_group(Comm* c, int begin, std::string* err) {
  if (c->host || !c->nccl || (c->size == 1 && !force_collectives(c))) return PGO_OK;
  const ncclResult_t e = begin ? rccl().group_start() : rccl().group_end();
  return e == ncclSuccess ? PGO_OK : nccl_fail(e, begin ? "ncclGroupStart" : "ncclGroupEnd", err);
}

}  // namespace pgo
