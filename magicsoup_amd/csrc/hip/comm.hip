// Native RCCL communicator of the domain-decomposed world (magicsoup_amd.parallel.comm.RcclComm).
//
// The strip decomposition talks to at most two peers (the ranks owning the rows above and below)
// plus a handful of tiny all-reduces per step (integrator exit flags, diffusion mass totals). Going
// through torch.distributed costs tens of microseconds of host time per call (work objects, events,
// a side stream); here every collective is one C++ call that enqueues RCCL work on the caller's
// current HIP stream, ordered with the kernels around it, no host synchronisation.
//
// The RCCL library is the one PyTorch already loaded (its librccl.so, found by path and opened with
// RTLD_NOLOAD first), so the process holds a single RCCL runtime; the communicator is our own
// (ncclCommInitRank over a unique id that Python broadcasts through the bootstrap process group).
// Only the API declarations of <rccl/rccl.h> are used; nothing links against librccl.
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <chrono>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <string>
#include <vector>

#include "hip_common.h"

namespace msd {

namespace {

struct Rccl {
  void* lib = nullptr;
  decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&ncclCommInitRank) CommInitRank = nullptr;
  decltype(&ncclCommDestroy) CommDestroy = nullptr;
  decltype(&ncclCommAbort) CommAbort = nullptr;
  decltype(&ncclCommGetAsyncError) CommGetAsyncError = nullptr;
  decltype(&ncclGetErrorString) GetErrorString = nullptr;
  decltype(&ncclAllReduce) AllReduce = nullptr;
  decltype(&ncclSend) Send = nullptr;
  decltype(&ncclRecv) Recv = nullptr;
  decltype(&ncclGroupStart) GroupStart = nullptr;
  decltype(&ncclGroupEnd) GroupEnd = nullptr;
  decltype(&ncclGetVersion) GetVersion = nullptr;
};

Rccl g_rccl;
std::mutex g_rccl_mu;

template <class F>
void sym(void* lib, const char* name, F& out) {
  out = reinterpret_cast<F>(dlsym(lib, name));
  if (!out) throw std::runtime_error(std::string("rccl: missing symbol ") + name);
}

const Rccl& api() {
  if (!g_rccl.lib) throw std::runtime_error("rccl: library not loaded (call rccl_load first)");
  return g_rccl;
}

void check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) {
    const char* msg = g_rccl.GetErrorString ? g_rccl.GetErrorString(r) : "?";
    throw std::runtime_error(std::string("rccl: ") + what + " failed: " + msg);
  }
}

ncclComm_t C_(uintptr_t c) {
  if (!c) throw std::invalid_argument("rccl: null communicator");
  return reinterpret_cast<ncclComm_t>(c);
}

}  // namespace

// Resolve the RCCL entry points from `path` (PyTorch's librccl.so). Returns the RCCL version code.
int rccl_load(const std::string& path) {
  std::lock_guard<std::mutex> lk(g_rccl_mu);
  if (!g_rccl.lib) {
    void* h = dlopen(path.c_str(), RTLD_NOW | RTLD_NOLOAD);
    if (!h) h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (!h) throw std::runtime_error(std::string("rccl: cannot open ") + path + ": " + dlerror());
    Rccl r;
    r.lib = h;
    sym(h, "ncclGetUniqueId", r.GetUniqueId);
    sym(h, "ncclCommInitRank", r.CommInitRank);
    sym(h, "ncclCommDestroy", r.CommDestroy);
    sym(h, "ncclCommAbort", r.CommAbort);
    sym(h, "ncclCommGetAsyncError", r.CommGetAsyncError);
    sym(h, "ncclGetErrorString", r.GetErrorString);
    sym(h, "ncclAllReduce", r.AllReduce);
    sym(h, "ncclSend", r.Send);
    sym(h, "ncclRecv", r.Recv);
    sym(h, "ncclGroupStart", r.GroupStart);
    sym(h, "ncclGroupEnd", r.GroupEnd);
    sym(h, "ncclGetVersion", r.GetVersion);
    g_rccl = r;
  }
  int v = 0;
  check(g_rccl.GetVersion(&v), "ncclGetVersion");
  return v;
}

std::string rccl_unique_id() {
  ncclUniqueId id;
  check(api().GetUniqueId(&id), "ncclGetUniqueId");
  return std::string(id.internal, NCCL_UNIQUE_ID_BYTES);
}

// New communicator of `nranks` ranks on the current HIP device (every rank calls this with the same id).
uintptr_t rccl_init(const std::string& uid, int nranks, int rank) {
  if (uid.size() != NCCL_UNIQUE_ID_BYTES) throw std::invalid_argument("rccl_init: unique id must be 128 bytes");
  if (nranks < 1 || rank < 0 || rank >= nranks) throw std::invalid_argument("rccl_init: bad rank / size");
  ncclUniqueId id;
  std::copy(uid.begin(), uid.end(), id.internal);
  ncclComm_t comm = nullptr;
  check(api().CommInitRank(&comm, nranks, id, rank), "ncclCommInitRank");
  return reinterpret_cast<uintptr_t>(comm);
}

void rccl_destroy(uintptr_t comm, bool abort) {
  if (!comm) return;
  if (abort) check(api().CommAbort(C_(comm)), "ncclCommAbort");
  else check(api().CommDestroy(C_(comm)), "ncclCommDestroy");
}

// "" when healthy, else the asynchronous error of the communicator (e.g. a peer failed).
std::string rccl_async_error(uintptr_t comm) {
  ncclResult_t r = ncclSuccess;
  check(api().CommGetAsyncError(C_(comm), &r), "ncclCommGetAsyncError");
  return r == ncclSuccess ? std::string() : std::string(api().GetErrorString(r));
}

// Wait for the work queued on `stream` while polling the communicators for asynchronous errors
// (a dead peer leaves an RCCL kernel waiting forever: a plain hipStreamSynchronize would hang).
// Returns "" when the stream drained; otherwise every communicator in `comms` is aborted (its
// kernels are released, the handles become unusable) and the reason is returned: the RCCL error,
// or "timeout" after `timeout_s` seconds. `event` (optional): wait for that event instead of the
// whole stream (a deferred read-back that must not wait for work queued after it).
std::string rccl_guarded_wait(const std::vector<uintptr_t>& comms, uintptr_t stream, double timeout_s,
                              uintptr_t event) {
  const Rccl& r = api();
  hipStream_t s = S_(stream);
  hipEvent_t ev = reinterpret_cast<hipEvent_t>(event);
  const auto t0 = std::chrono::steady_clock::now();
  std::string why;
  for (long long it = 0;; ++it) {
    const hipError_t q = ev ? msd::event_query(ev) : msd::stream_query(s);
    if (q == hipSuccess) return std::string();
    if (q != hipErrorNotReady) MS_HIP_CHECK(q);
    // errors are polled every 256 queries (~tens of microseconds): the common case (a healthy job
    // waiting for its own kernels) stays a tight query loop
    if ((it & 255) == 255) {
      for (uintptr_t c : comms) {
        if (!c) continue;
        ncclResult_t e = ncclSuccess;
        if (r.CommGetAsyncError(C_(c), &e) != ncclSuccess || (e != ncclSuccess && e != ncclInProgress)) {
          why = std::string("rccl: asynchronous error: ") + r.GetErrorString(e);
          break;
        }
      }
      if (!why.empty()) break;
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (el > timeout_s) {
        why = "timeout";
        break;
      }
      std::this_thread::yield();
    }
  }
  for (uintptr_t c : comms)
    if (c) (void)r.CommAbort(C_(c));
  return why;
}

// In-place all-reduce of `count` elements. dtype: 0 int32, 1 float32, 2 float64, 3 int64;
// op: 0 sum, 1 max, 2 min.
void rccl_allreduce(uintptr_t comm, uintptr_t buf, long long count, int dtype, int op, uintptr_t stream) {
  static const ncclDataType_t kT[] = {ncclInt32, ncclFloat32, ncclFloat64, ncclInt64};
  static const ncclRedOp_t kO[] = {ncclSum, ncclMax, ncclMin};
  if (dtype < 0 || dtype > 3 || op < 0 || op > 2) throw std::invalid_argument("rccl_allreduce: bad dtype / op");
  if (count <= 0) return;
  batch_flush();  // (the kernels recorded before it run first)
  void* p = reinterpret_cast<void*>(buf);
  check(api().AllReduce(p, p, (size_t)count, kT[dtype], kO[op], C_(comm), S_(stream)), "ncclAllReduce");
}

// One grouped neighbour exchange of byte buffers: send_up -> rank `up` (which receives it as its
// recv_down), send_down -> rank `down` (its recv_up). Sizes of 0 skip an operation; the protocol
// guarantees the matching side skips too. Sends and receives to one peer match in issue order, so
// up == down (two ranks) and up == down == self (one rank) work as well.
void rccl_exchange(uintptr_t comm, int up, int down, uintptr_t send_up, long long n_send_up, uintptr_t send_down,
                   long long n_send_down, uintptr_t recv_down, long long n_recv_down, uintptr_t recv_up,
                   long long n_recv_up, uintptr_t stream) {
  const Rccl& r = api();
  ncclComm_t c = C_(comm);
  hipStream_t s = S_(stream);
  if (n_send_up + n_send_down + n_recv_down + n_recv_up == 0) return;
  batch_flush();  // (the kernels recorded before it run first)
  check(r.GroupStart(), "ncclGroupStart");
  try {
    if (n_send_up > 0) check(r.Send(reinterpret_cast<void*>(send_up), (size_t)n_send_up, ncclUint8, up, c, s), "ncclSend");
    if (n_send_down > 0)
      check(r.Send(reinterpret_cast<void*>(send_down), (size_t)n_send_down, ncclUint8, down, c, s), "ncclSend");
    if (n_recv_down > 0)
      check(r.Recv(reinterpret_cast<void*>(recv_down), (size_t)n_recv_down, ncclUint8, down, c, s), "ncclRecv");
    if (n_recv_up > 0) check(r.Recv(reinterpret_cast<void*>(recv_up), (size_t)n_recv_up, ncclUint8, up, c, s), "ncclRecv");
  } catch (...) {
    r.GroupEnd();
    throw;
  }
  check(r.GroupEnd(), "ncclGroupEnd");
}

}  // namespace msd
