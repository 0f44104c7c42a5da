// Native stream-ordered communicator over RCCL.
//
// torch's ProcessGroupNCCL runs every collective on its own internal stream: an event on the
// caller's stream, a wait on the NCCL stream, the collective, and on wait() an event back. For the
// small per-iteration collectives of the iterative algorithms (k-means' k*f + k sums, moment
// triples, argmin keys) that bookkeeping is a large part of the cost, and it keeps the step from
// being captured in a HIP graph. This communicator issues the RCCL call directly on the CALLER's
// stream: the collective is ordered with the kernels around it like any other kernel, with no
// extra events or host syncs.
//
// The RCCL library is the instance torch already loaded (its path is passed in and re-opened with
// RTLD_NOLOAD), so both communicators share one RCCL runtime. Functions are resolved with dlsym;
// nothing here links against RCCL at build time.
#include "common.h"

#include <dlfcn.h>
#include <string.h>

namespace {

typedef int rcclResult;  // ncclResult_t
typedef void* rcclComm;  // ncclComm_t
struct rcclUniqueId { char internal[128]; };

struct Rccl {
  void* handle = nullptr;
  rcclResult (*GetUniqueId)(rcclUniqueId*) = nullptr;
  rcclResult (*CommInitRank)(rcclComm*, int, rcclUniqueId, int) = nullptr;
  rcclResult (*CommDestroy)(rcclComm) = nullptr;
  rcclResult (*CommAbort)(rcclComm) = nullptr;
  rcclResult (*CommGetAsyncError)(rcclComm, rcclResult*) = nullptr;
  rcclResult (*AllReduce)(const void*, void*, size_t, int, int, rcclComm, hipStream_t) = nullptr;
  rcclResult (*AllGather)(const void*, void*, size_t, int, rcclComm, hipStream_t) = nullptr;
  rcclResult (*Broadcast)(const void*, void*, size_t, int, int, rcclComm, hipStream_t) = nullptr;
  rcclResult (*ReduceScatter)(const void*, void*, size_t, int, int, rcclComm, hipStream_t) = nullptr;
  rcclResult (*Send)(const void*, size_t, int, int, rcclComm, hipStream_t) = nullptr;
  rcclResult (*Recv)(void*, size_t, int, int, rcclComm, hipStream_t) = nullptr;
  rcclResult (*GroupStart)() = nullptr;
  rcclResult (*GroupEnd)() = nullptr;
};

Rccl g_rccl;

template <typename F>
bool sym(F& f, const char* name) {
  f = (F)dlsym(g_rccl.handle, name);
  return f != nullptr;
}

// ncclDataType_t codes: int8 0, uint8 1, int32 2, uint32 3, int64 4, uint64 5, fp16 6, fp32 7,
// fp64 8, bf16 9. ncclRedOp_t: sum 0, prod 1, max 2, min 3.
constexpr int kUint8 = 1;

}  // namespace

// 0 on success; the library at ``path`` must already be loaded (torch's copy) or loadable.
HA_EXPORT int ha_comm_load(const char* path) {
  if (g_rccl.handle) return HA_OK;
  void* h = dlopen(path, RTLD_NOW | RTLD_NOLOAD);
  if (!h) h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
  if (!h) return HA_UNSUPPORTED;
  g_rccl.handle = h;
  bool ok = sym(g_rccl.GetUniqueId, "ncclGetUniqueId") && sym(g_rccl.CommInitRank, "ncclCommInitRank") &&
            sym(g_rccl.CommDestroy, "ncclCommDestroy") && sym(g_rccl.CommAbort, "ncclCommAbort") &&
            sym(g_rccl.CommGetAsyncError, "ncclCommGetAsyncError") && sym(g_rccl.AllReduce, "ncclAllReduce") &&
            sym(g_rccl.AllGather, "ncclAllGather") && sym(g_rccl.Broadcast, "ncclBroadcast") &&
            sym(g_rccl.ReduceScatter, "ncclReduceScatter") && sym(g_rccl.Send, "ncclSend") &&
            sym(g_rccl.Recv, "ncclRecv") && sym(g_rccl.GroupStart, "ncclGroupStart") &&
            sym(g_rccl.GroupEnd, "ncclGroupEnd");
  if (!ok) {
    g_rccl.handle = nullptr;
    return HA_UNSUPPORTED;
  }
  return HA_OK;
}

HA_EXPORT int ha_comm_unique_id(char* out128) {
  if (!g_rccl.handle) return HA_UNSUPPORTED;
  rcclUniqueId id;
  if (g_rccl.GetUniqueId(&id) != 0) return HA_LAUNCH;
  memcpy(out128, id.internal, 128);
  return HA_OK;
}

HA_EXPORT int ha_comm_init(const char* id128, int nranks, int rank, void** comm_out) {
  if (!g_rccl.handle) return HA_UNSUPPORTED;
  if (nranks < 1 || rank < 0 || rank >= nranks) return HA_BAD_ARG;
  rcclUniqueId id;
  memcpy(id.internal, id128, 128);
  rcclComm c = nullptr;
  const rcclResult r = g_rccl.CommInitRank(&c, nranks, id, rank);
  if (r != 0) return 100 + r;
  *comm_out = c;
  return HA_OK;
}

HA_EXPORT int ha_comm_destroy(void* comm, int abort_) {
  if (!g_rccl.handle || !comm) return HA_BAD_ARG;
  return (abort_ ? g_rccl.CommAbort(comm) : g_rccl.CommDestroy(comm)) == 0 ? HA_OK : HA_LAUNCH;
}

// the communicator's asynchronous error (0 = none), for the watchdog
HA_EXPORT int ha_comm_async_error(void* comm) {
  rcclResult e = 0;
  if (!g_rccl.handle || !comm) return -1;
  if (g_rccl.CommGetAsyncError(comm, &e) != 0) return -1;
  return e;
}

HA_EXPORT int ha_comm_allreduce(void* comm, const void* send, void* recv, int64_t count, int dtype, int op,
                                void* stream) {
  if (!g_rccl.handle || !comm || count < 0) return HA_BAD_ARG;
  const rcclResult r = g_rccl.AllReduce(send, recv, (size_t)count, dtype, op, comm, (hipStream_t)stream);
  return r == 0 ? HA_OK : 100 + r;
}

HA_EXPORT int ha_comm_allgather(void* comm, const void* send, void* recv, int64_t count, int dtype, void* stream) {
  if (!g_rccl.handle || !comm || count < 0) return HA_BAD_ARG;
  const rcclResult r = g_rccl.AllGather(send, recv, (size_t)count, dtype, comm, (hipStream_t)stream);
  return r == 0 ? HA_OK : 100 + r;
}

// recv (recvcount elements) = this rank's block of the reduction of send (nranks x recvcount)
HA_EXPORT int ha_comm_reducescatter(void* comm, const void* send, void* recv, int64_t recvcount, int dtype, int op,
                                    void* stream) {
  if (!g_rccl.handle || !comm || recvcount < 0) return HA_BAD_ARG;
  const rcclResult r = g_rccl.ReduceScatter(send, recv, (size_t)recvcount, dtype, op, comm, (hipStream_t)stream);
  return r == 0 ? HA_OK : 100 + r;
}

HA_EXPORT int ha_comm_broadcast(void* comm, void* buf, int64_t count, int dtype, int root, void* stream) {
  if (!g_rccl.handle || !comm || count < 0) return HA_BAD_ARG;
  const rcclResult r = g_rccl.Broadcast(buf, buf, (size_t)count, dtype, root, comm, (hipStream_t)stream);
  return r == 0 ? HA_OK : 100 + r;
}

// personalised exchange of raw bytes: to rank q ``send_bytes[q]`` bytes at ``send + send_off[q]``,
// from rank r ``recv_bytes[r]`` bytes into ``recv + recv_off[r]``, as one RCCL group of p sends
// and p receives on the caller's stream (the local block is a device copy).
HA_EXPORT int ha_comm_alltoallv(void* comm, int nranks, int rank, const void* send, const int64_t* send_bytes,
                                const int64_t* send_off, void* recv, const int64_t* recv_bytes,
                                const int64_t* recv_off, void* stream) {
  if (!g_rccl.handle || !comm) return HA_BAD_ARG;
  hipStream_t s = (hipStream_t)stream;
  const char* sb = (const char*)send;
  char* rb = (char*)recv;
  if (send_bytes[rank] != recv_bytes[rank]) return HA_BAD_ARG;
  if (send_bytes[rank] > 0 &&
      hipMemcpyAsync(rb + recv_off[rank], sb + send_off[rank], (size_t)send_bytes[rank], hipMemcpyDeviceToDevice, s) !=
          hipSuccess)
    return HA_LAUNCH;
  if (g_rccl.GroupStart() != 0) return HA_LAUNCH;
  // every enqueue is checked; the group is always closed (an open group would swallow the next
  // collective), and the first failure is returned as 100 + the RCCL code
  rcclResult first = 0;
  for (int k = 1; k < nranks; ++k) {
    // pairwise schedule: at step k send to rank+k, receive from rank-k (every link busy both ways)
    const int to = (rank + k) % nranks, from = (rank - k + nranks) % nranks;
    if (send_bytes[to] > 0) {
      const rcclResult r = g_rccl.Send(sb + send_off[to], (size_t)send_bytes[to], kUint8, to, comm, s);
      if (r != 0 && first == 0) first = r;
    }
    if (recv_bytes[from] > 0) {
      const rcclResult r = g_rccl.Recv(rb + recv_off[from], (size_t)recv_bytes[from], kUint8, from, comm, s);
      if (r != 0 && first == 0) first = r;
    }
  }
  const rcclResult e = g_rccl.GroupEnd();
  if (first != 0) return 100 + first;
  return e == 0 ? HA_OK : 100 + e;
}
