// Thin RCCL binding (SURVEY.md §2.3 "Comm backend", §5.8): communicators built from a unique id
// that the caller exchanges (Python: a torch.distributed object collective over any group),
// every collective enqueued on the CALLER's HIP stream -- the compute stream, a dedicated comm
// stream with events, or a stream being captured into a HIP graph -- with no work object, host
// callback or extra stream hop in between.
//
// RCCL is resolved at run time, never linked: the copy the process already has (PyTorch's
// bundled librccl, found with RTLD_NOLOAD) is preferred, else the one named by the caller or
// /opt/rocm/lib/librccl.so.1 -- so one process never holds two RCCL copies with two sets of
// proxy threads and topology state.
//
// Failure: pk_rccl_async_error polls ncclCommGetAsyncError without blocking;
// pk_rccl_abort tears a communicator down even while a collective of it is hung, so a watchdog
// can fail the process instead of waiting forever.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstring>
#include <mutex>

#define PK_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

struct Api {
  decltype(&ncclGetVersion) get_version = nullptr;
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) init_rank = nullptr;
  decltype(&ncclCommDestroy) destroy = nullptr;
  decltype(&ncclCommAbort) abort = nullptr;
  decltype(&ncclCommGetAsyncError) async_error = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclAllGather) all_gather = nullptr;
  decltype(&ncclReduceScatter) reduce_scatter = nullptr;
  decltype(&ncclBroadcast) broadcast = nullptr;
  decltype(&ncclSend) send = nullptr;
  decltype(&ncclRecv) recv = nullptr;
  decltype(&ncclGroupStart) group_start = nullptr;
  decltype(&ncclGroupEnd) group_end = nullptr;
};

Api g_api;
void* g_handle = nullptr;
std::mutex g_mu;
char g_path[512] = {0};

template <class F>
bool resolve(void* h, const char* name, F& fn) {
  fn = reinterpret_cast<F>(dlsym(h, name));
  return fn != nullptr;
}

bool load_from(void* h) {
  Api a;
  bool ok = resolve(h, "ncclGetVersion", a.get_version) && resolve(h, "ncclGetUniqueId", a.get_unique_id) &&
            resolve(h, "ncclCommInitRank", a.init_rank) && resolve(h, "ncclCommDestroy", a.destroy) &&
            resolve(h, "ncclCommAbort", a.abort) && resolve(h, "ncclCommGetAsyncError", a.async_error) &&
            resolve(h, "ncclGetErrorString", a.error_string) && resolve(h, "ncclAllReduce", a.all_reduce) &&
            resolve(h, "ncclAllGather", a.all_gather) && resolve(h, "ncclReduceScatter", a.reduce_scatter) &&
            resolve(h, "ncclBroadcast", a.broadcast) && resolve(h, "ncclSend", a.send) &&
            resolve(h, "ncclRecv", a.recv) && resolve(h, "ncclGroupStart", a.group_start) &&
            resolve(h, "ncclGroupEnd", a.group_end);
  if (ok) g_api = a;
  return ok;
}

bool loaded() { return g_handle != nullptr; }

// Element-type codes shared with parallel/rccl.py: 0 bf16, 1 fp32, 2 int32, 3 uint8 (bytes), 4 fp16, 5 int64.
bool dtype_of(int code, ncclDataType_t* t) {
  switch (code) {
    case 0: *t = ncclBfloat16; return true;
    case 1: *t = ncclFloat32; return true;
    case 2: *t = ncclInt32; return true;
    case 3: *t = ncclUint8; return true;
    case 4: *t = ncclFloat16; return true;
    case 5: *t = ncclInt64; return true;
    default: return false;
  }
}

size_t dtype_bytes(ncclDataType_t t) {
  switch (t) {
    case ncclBfloat16:
    case ncclFloat16: return 2;
    case ncclFloat32:
    case ncclInt32: return 4;
    case ncclInt64: return 8;
    default: return 1;
  }
}

// Reduction codes: 0 sum, 1 max, 2 min.
bool op_of(int code, ncclRedOp_t* op) {
  switch (code) {
    case 0: *op = ncclSum; return true;
    case 1: *op = ncclMax; return true;
    case 2: *op = ncclMin; return true;
    default: return false;
  }
}

// Return convention: 0 ok, -1 bad argument / RCCL not loaded, otherwise the ncclResult_t code.
constexpr int kBadArg = -1;

}  // namespace

// Load RCCL: the copy already in the process first (RTLD_NOLOAD), else `path` (may be null),
// else /opt/rocm/lib/librccl.so.1.  Idempotent.  Returns 0 when the API is usable.
PK_EXPORT int pk_rccl_load(const char* path) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (loaded()) return 0;
  const char* resident[] = {"librccl.so", "librccl.so.1"};
  for (const char* n : resident) {
    void* h = dlopen(n, RTLD_NOW | RTLD_NOLOAD);
    if (h != nullptr && load_from(h)) {
      g_handle = h;
      std::snprintf(g_path, sizeof(g_path), "%s (resident)", n);
      return 0;
    }
    if (h != nullptr) dlclose(h);
  }
  const char* cands[] = {path, "/opt/rocm/lib/librccl.so.1"};
  for (const char* p : cands) {
    if (p == nullptr || p[0] == 0) continue;
    void* h = dlopen(p, RTLD_NOW | RTLD_GLOBAL);
    if (h != nullptr && load_from(h)) {
      g_handle = h;
      std::snprintf(g_path, sizeof(g_path), "%s", p);
      return 0;
    }
    if (h != nullptr) dlclose(h);
  }
  return kBadArg;
}

PK_EXPORT const char* pk_rccl_library() { return g_path; }

PK_EXPORT int pk_rccl_version() {
  if (!loaded()) return kBadArg;
  int v = 0;
  return g_api.get_version(&v) == ncclSuccess ? v : kBadArg;
}

PK_EXPORT const char* pk_rccl_error_string(int rc) {
  if (rc == kBadArg) return "bad argument or RCCL not loaded";
  if (!loaded()) return "RCCL not loaded";
  return g_api.error_string(static_cast<ncclResult_t>(rc));
}

PK_EXPORT int pk_rccl_unique_id_size() { return NCCL_UNIQUE_ID_BYTES; }

PK_EXPORT int pk_rccl_unique_id(void* out) {
  if (!loaded() || out == nullptr) return kBadArg;
  ncclUniqueId id;
  const ncclResult_t r = g_api.get_unique_id(&id);
  if (r == ncclSuccess) std::memcpy(out, &id, sizeof(id));
  return r;
}

// Blocking: every rank of the communicator must call it (on its own device, set by the caller).
PK_EXPORT int pk_rccl_init(void** comm_out, const void* id, int nranks, int rank) {
  if (!loaded() || comm_out == nullptr || id == nullptr || nranks < 1 || rank < 0 || rank >= nranks) return kBadArg;
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  ncclComm_t c = nullptr;
  const ncclResult_t r = g_api.init_rank(&c, nranks, uid, rank);
  *comm_out = r == ncclSuccess ? c : nullptr;
  return r;
}

PK_EXPORT int pk_rccl_destroy(void* comm) {
  if (!loaded() || comm == nullptr) return kBadArg;
  return g_api.destroy(static_cast<ncclComm_t>(comm));
}

PK_EXPORT int pk_rccl_abort(void* comm) {
  if (!loaded() || comm == nullptr) return kBadArg;
  return g_api.abort(static_cast<ncclComm_t>(comm));
}

// Non-blocking health poll: the communicator's asynchronous error (0 = none).
PK_EXPORT int pk_rccl_async_error(void* comm) {
  if (!loaded() || comm == nullptr) return kBadArg;
  ncclResult_t e = ncclSuccess;
  const ncclResult_t r = g_api.async_error(static_cast<ncclComm_t>(comm), &e);
  return r != ncclSuccess ? r : e;
}

PK_EXPORT int pk_rccl_all_reduce(void* comm, const void* send, void* recv, size_t count, int dtype, int op,
                                 hipStream_t stream) {
  ncclDataType_t t;
  ncclRedOp_t o;
  if (!loaded() || comm == nullptr || !dtype_of(dtype, &t) || !op_of(op, &o)) return kBadArg;
  return g_api.all_reduce(send, recv, count, t, o, static_cast<ncclComm_t>(comm), stream);
}

// recv = the ranks' `count`-element send buffers concatenated in rank order.
PK_EXPORT int pk_rccl_all_gather(void* comm, const void* send, void* recv, size_t count, int dtype,
                                 hipStream_t stream) {
  ncclDataType_t t;
  if (!loaded() || comm == nullptr || !dtype_of(dtype, &t)) return kBadArg;
  return g_api.all_gather(send, recv, count, t, static_cast<ncclComm_t>(comm), stream);
}

// recv (`count` elements) = this rank's block of the element-wise reduction of the send buffers.
PK_EXPORT int pk_rccl_reduce_scatter(void* comm, const void* send, void* recv, size_t count, int dtype, int op,
                                     hipStream_t stream) {
  ncclDataType_t t;
  ncclRedOp_t o;
  if (!loaded() || comm == nullptr || !dtype_of(dtype, &t) || !op_of(op, &o)) return kBadArg;
  return g_api.reduce_scatter(send, recv, count, t, o, static_cast<ncclComm_t>(comm), stream);
}

PK_EXPORT int pk_rccl_broadcast(void* comm, const void* send, void* recv, size_t count, int dtype, int root,
                                hipStream_t stream) {
  ncclDataType_t t;
  if (!loaded() || comm == nullptr || !dtype_of(dtype, &t)) return kBadArg;
  return g_api.broadcast(send, recv, count, t, root, static_cast<ncclComm_t>(comm), stream);
}

// Variable all-to-all (EP dispatch / combine): rank r sends send[sdispl[j] : sdispl[j] + scount[j]]
// to rank j and receives rcount[j] elements from rank j at recv + rdispl[j] (counts and
// displacements in elements, host arrays of nranks entries).  One RCCL group of point-to-point
// transfers, so every peer pair moves over its own xGMI link concurrently.
PK_EXPORT int pk_rccl_all_to_allv(void* comm, const void* send, const size_t* scount, const size_t* sdispl,
                                  void* recv, const size_t* rcount, const size_t* rdispl, int nranks, int dtype,
                                  hipStream_t stream) {
  ncclDataType_t t;
  if (!loaded() || comm == nullptr || !dtype_of(dtype, &t) || nranks < 1) return kBadArg;
  const size_t eb = dtype_bytes(t);
  const auto c = static_cast<ncclComm_t>(comm);
  ncclResult_t r = g_api.group_start();
  if (r != ncclSuccess) return r;
  for (int j = 0; j < nranks && r == ncclSuccess; ++j) {
    if (scount[j] > 0)
      r = g_api.send(static_cast<const char*>(send) + sdispl[j] * eb, scount[j], t, j, c, stream);
    if (r == ncclSuccess && rcount[j] > 0)
      r = g_api.recv(static_cast<char*>(recv) + rdispl[j] * eb, rcount[j], t, j, c, stream);
  }
  const ncclResult_t e = g_api.group_end();
  return r != ncclSuccess ? r : e;
}
