// Native RCCL communicator: a thin C ABI over librccl for the
// data-parallel learner's collectives on explicit HIP streams, plus the
// communicator abort that failure recovery needs (§5.3).
//
// The library is not linked: apex_comm_load() dlopen()s the librccl the process
// already uses (torch's bundled copy, found with RTLD_NOLOAD first) so exactly one
// RCCL instance lives in the process; every entry point is resolved with dlsym.
// The unique id is created on rank 0 (apex_comm_unique_id) and exchanged by the
// caller (torch.distributed broadcast / store), then every rank calls
// apex_comm_init(nranks, id, rank) with its HIP device current.
//
// Collectives enqueue on the stream they are given, so they are captured by a HIP
// graph like any kernel (the learner's DP step is one captured graph).
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstring>

#define APEX_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

struct Api {
  void* handle = nullptr;
  ncclResult_t (*get_version)(int*) = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*comm_abort)(ncclComm_t) = nullptr;
  ncclResult_t (*comm_async_error)(ncclComm_t, ncclResult_t*) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*reduce_scatter)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                                 hipStream_t) = nullptr;
  ncclResult_t (*comm_count)(const ncclComm_t, int*) = nullptr;
  ncclResult_t (*comm_user_rank)(const ncclComm_t, int*) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
};

Api g;

template <typename F>
bool sym(F& f, const char* name) {
  f = reinterpret_cast<F>(dlsym(g.handle, name));
  return f != nullptr;
}

constexpr int kNotLoaded = 1000;   // beyond ncclResult_t's range

}  // namespace

// 0 on success; `path` = the librccl.so to use (nullptr: "librccl.so" from the
// loader path).  Idempotent.
APEX_EXPORT int apex_comm_load(const char* path) {
  if (g.handle != nullptr) return 0;
  const char* p = path != nullptr ? path : "librccl.so";
  void* h = dlopen(p, RTLD_NOW | RTLD_NOLOAD);          // the copy already in the process
  if (h == nullptr) h = dlopen(p, RTLD_NOW | RTLD_LOCAL);
  if (h == nullptr) return kNotLoaded;
  g.handle = h;
  bool ok = sym(g.get_version, "ncclGetVersion") && sym(g.get_unique_id, "ncclGetUniqueId") &&
            sym(g.comm_init_rank, "ncclCommInitRank") && sym(g.comm_destroy, "ncclCommDestroy") &&
            sym(g.comm_abort, "ncclCommAbort") && sym(g.comm_async_error, "ncclCommGetAsyncError") &&
            sym(g.error_string, "ncclGetErrorString") && sym(g.all_reduce, "ncclAllReduce") &&
            sym(g.all_gather, "ncclAllGather") && sym(g.broadcast, "ncclBroadcast") &&
            sym(g.group_start, "ncclGroupStart") && sym(g.group_end, "ncclGroupEnd") &&
            sym(g.reduce_scatter, "ncclReduceScatter") && sym(g.comm_count, "ncclCommCount") &&
            sym(g.comm_user_rank, "ncclCommUserRank");
  if (!ok) {
    g = Api{};
    return kNotLoaded;
  }
  return 0;
}

APEX_EXPORT int apex_comm_version() {
  int v = 0;
  if (g.get_version == nullptr || g.get_version(&v) != ncclSuccess) return -1;
  return v;
}

APEX_EXPORT const char* apex_comm_error_string(int rc) {
  if (rc == kNotLoaded) return "librccl not loaded (apex_comm_load)";
  if (g.error_string == nullptr) return "unknown";
  return g.error_string(static_cast<ncclResult_t>(rc));
}

// out: NCCL_UNIQUE_ID_BYTES (128) bytes
APEX_EXPORT int apex_comm_unique_id(char* out) {
  if (g.get_unique_id == nullptr) return kNotLoaded;
  ncclUniqueId id;
  const ncclResult_t r = g.get_unique_id(&id);
  if (r == ncclSuccess) std::memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
  return static_cast<int>(r);
}

APEX_EXPORT int apex_comm_id_bytes() { return NCCL_UNIQUE_ID_BYTES; }

// a communicator for `rank` of `nranks` on the current HIP device (blocks until
// every rank has joined)
APEX_EXPORT int apex_comm_init(void** comm_out, int nranks, const char* id_bytes, int rank) {
  if (g.comm_init_rank == nullptr) return kNotLoaded;
  if (comm_out == nullptr || id_bytes == nullptr || nranks < 1 || rank < 0 || rank >= nranks)
    return static_cast<int>(ncclInvalidArgument);
  ncclUniqueId id;
  std::memcpy(id.internal, id_bytes, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c = nullptr;
  const ncclResult_t r = g.comm_init_rank(&c, nranks, id, rank);
  *comm_out = r == ncclSuccess ? static_cast<void*>(c) : nullptr;
  return static_cast<int>(r);
}

APEX_EXPORT int apex_comm_all_reduce(void* comm, const void* send, void* recv, size_t count, int dtype, int op,
                                     void* stream) {
  if (g.all_reduce == nullptr) return kNotLoaded;
  return static_cast<int>(g.all_reduce(send, recv, count, static_cast<ncclDataType_t>(dtype),
                                       static_cast<ncclRedOp_t>(op), static_cast<ncclComm_t>(comm),
                                       static_cast<hipStream_t>(stream)));
}

// recv = concatenation over ranks of `sendcount` elements each
APEX_EXPORT int apex_comm_all_gather(void* comm, const void* send, void* recv, size_t sendcount, int dtype,
                                     void* stream) {
  if (g.all_gather == nullptr) return kNotLoaded;
  return static_cast<int>(g.all_gather(send, recv, sendcount, static_cast<ncclDataType_t>(dtype),
                                       static_cast<ncclComm_t>(comm), static_cast<hipStream_t>(stream)));
}

// recv = this rank's `recvcount`-element chunk of the reduction of send (W x recvcount)
APEX_EXPORT int apex_comm_reduce_scatter(void* comm, const void* send, void* recv, size_t recvcount, int dtype,
                                         int op, void* stream) {
  if (g.reduce_scatter == nullptr) return kNotLoaded;
  return static_cast<int>(g.reduce_scatter(send, recv, recvcount, static_cast<ncclDataType_t>(dtype),
                                           static_cast<ncclRedOp_t>(op), static_cast<ncclComm_t>(comm),
                                           static_cast<hipStream_t>(stream)));
}

// the rank count / this rank as the communicator itself sees them (bench.py reports
// them next to WORLD_SIZE: a world RCCL never formed cannot hide behind the env)
APEX_EXPORT int apex_comm_count(void* comm, int* count, int* rank) {
  if (g.comm_count == nullptr || g.comm_user_rank == nullptr) return kNotLoaded;
  ncclResult_t r = g.comm_count(static_cast<ncclComm_t>(comm), count);
  if (r != ncclSuccess) return static_cast<int>(r);
  return static_cast<int>(g.comm_user_rank(static_cast<ncclComm_t>(comm), rank));
}

APEX_EXPORT int apex_comm_broadcast(void* comm, const void* send, void* recv, size_t count, int dtype, int root,
                                    void* stream) {
  if (g.broadcast == nullptr) return kNotLoaded;
  return static_cast<int>(g.broadcast(send, recv, count, static_cast<ncclDataType_t>(dtype), root,
                                      static_cast<ncclComm_t>(comm), static_cast<hipStream_t>(stream)));
}

APEX_EXPORT int apex_comm_group_start() { return g.group_start ? static_cast<int>(g.group_start()) : kNotLoaded; }
APEX_EXPORT int apex_comm_group_end() { return g.group_end ? static_cast<int>(g.group_end()) : kNotLoaded; }

// the communicator's asynchronous error state (ncclSuccess while healthy)
APEX_EXPORT int apex_comm_async_error(void* comm) {
  if (g.comm_async_error == nullptr) return kNotLoaded;
  ncclResult_t e = ncclSuccess;
  const ncclResult_t r = g.comm_async_error(static_cast<ncclComm_t>(comm), &e);
  return static_cast<int>(r != ncclSuccess ? r : e);
}

// abort: outstanding collectives are cancelled, the communicator is freed (a rank
// whose peer died must not block in teardown)
APEX_EXPORT int apex_comm_abort(void* comm) {
  if (g.comm_abort == nullptr) return kNotLoaded;
  return static_cast<int>(g.comm_abort(static_cast<ncclComm_t>(comm)));
}

APEX_EXPORT int apex_comm_destroy(void* comm) {
  if (g.comm_destroy == nullptr) return kNotLoaded;
  return static_cast<int>(g.comm_destroy(static_cast<ncclComm_t>(comm)));
}
