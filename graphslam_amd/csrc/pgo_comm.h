// Inter-rank exchange of the multi-GPU path (internal to libpgo.so).
//
// The data-path exchanges of the multi-GPU modes: speculative
// lambda search -- per lambda round an all-gather of every rank's try outcome
// (4 doubles) and a broadcast of the accepted candidate values (N double4) from
// the rank that computed them; partitioned factorisation -- per factorisation
// an all-gather of the subtree roots' update matrices / vectors and one of the
// subtrees' solutions.  Two transports behind one interface:
//   * RCCL (librccl.so.1 resolved at run time with dlopen; device buffers, the
//     handle's HIP stream) -- xGMI between the GPUs of one node;
//   * host callbacks (pgo_host_comm) -- the caller's own transport on host
//     buffers (gloo in the tests, where two ranks share one GPU or run on CPU).
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "pgo.h"

namespace pgo {

constexpr int kMaxGather = 64;       // doubles per rank in one all-gather

struct Comm {
  int rank = 0, size = 1;
  bool host = false;                 // host callbacks (else RCCL)
  pgo_host_comm hc{};
  void* nccl = nullptr;              // ncclComm_t
  double* d_gather = nullptr;        // [kMaxGather * size] device all-gather buffer (RCCL)
  std::vector<char> stage;           // host staging of device broadcasts (host transport)
};

// ncclGetUniqueId through the run-time loaded RCCL; returns the id size or < 0
int comm_unique_id(void* out, size_t cap, std::string* err);
// ncclCommInitRank on the current device (collective over all ranks)
int comm_init_rccl(Comm* c, const void* uid, size_t uid_bytes, int rank, int size, std::string* err);
int comm_init_host(Comm* c, const pgo_host_comm* hc, std::string* err);
void comm_free(Comm* c);

// all[size * count] = every rank's mine[count] in rank order (host buffers);
// the RCCL transport stages through device memory on `s` and synchronises it
int comm_allgather(Comm* c, const double* mine, int count, double* all, hipStream_t s, std::string* err);
// device buffer dptr[bytes] of rank `root` -> every rank (in place); returns
// after the data has arrived (stream synchronised)
int comm_broadcast_device(Comm* c, void* dptr, size_t bytes, int root, hipStream_t s, std::string* err);

// as comm_broadcast_device, but the RCCL transport only enqueues it on s (the
// distributed top's panel broadcasts, stream ordered with the kernels around
// them); inside comm_group(c, 1) ... comm_group(c, 0) several broadcasts form one
// RCCL group (ncclGroupStart / ncclGroupEnd; no-op on the host transport)
int comm_broadcast_device_async(Comm* c, void* dptr, size_t bytes, int root, hipStream_t s, std::string* err);
int comm_group(Comm* c, int begin, std::string* err);

// device all-gather: recv[size * bytes] = every rank's send[bytes], rank order;
// RCCL: enqueued on s (ncclAllGather over xGMI); host transport: staged and
// synchronised (the partitioned factorisation's exchanges)
int comm_allgather_device(Comm* c, const void* send, void* recv, size_t bytes, hipStream_t s, std::string* err);

// PGO_COMM_FORCE_COLLECTIVES=1 on an RCCL communicator: exchanges run even at size 1
bool force_collectives(const Comm* c);
}  // namespace pgo
