// Pooled HIP events for the host-side ordering of the op layer (stream joins, pending genome-pipeline
// calls): one native call per record / wait / query instead of torch.cuda.Event + current_stream(),
// which resolve the device in Python (~10 us per call on the step's critical host path).
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>

#include <chrono>
#include <cstdint>
#include <mutex>
#include <vector>

#include "hip_common.h"
#include "bind_util.h"

namespace py = pybind11;

namespace msd {
namespace {
std::mutex g_ev_mu;
std::vector<hipEvent_t> g_ev_free;
std::vector<hipEvent_t> g_ev_all;
}  // namespace

uintptr_t ev_acquire() {
  std::lock_guard<std::mutex> lk(g_ev_mu);
  if (!g_ev_free.empty()) {
    hipEvent_t e = g_ev_free.back();
    g_ev_free.pop_back();
    return reinterpret_cast<uintptr_t>(e);
  }
  hipEvent_t e = nullptr;
  MS_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  g_ev_all.push_back(e);
  return reinterpret_cast<uintptr_t>(e);
}

void ev_release(uintptr_t e) {
  if (!e) return;
  std::lock_guard<std::mutex> lk(g_ev_mu);
  g_ev_free.push_back(reinterpret_cast<hipEvent_t>(e));
}

void ev_record(uintptr_t e, uintptr_t stream) {
  MS_HIP_CHECK(msd::event_record(reinterpret_cast<hipEvent_t>(e), reinterpret_cast<hipStream_t>(stream)));
}

// `stream` waits (device-side) for the work recorded in `e`
void ev_wait(uintptr_t stream, uintptr_t e) {
  MS_HIP_CHECK(msd::stream_wait_event(reinterpret_cast<hipStream_t>(stream), reinterpret_cast<hipEvent_t>(e), 0));
}

bool ev_query(uintptr_t e) {
  const hipError_t r = msd::event_query(reinterpret_cast<hipEvent_t>(e));
  if (r == hipErrorNotReady) return false;
  MS_HIP_CHECK(r);
  return true;
}

// Host wait for an event. hipEventSynchronize spins only briefly and then blocks on an interrupt:
// the op layer's waits (a kill_divide waiting for the previous genome chain, a flush for a
// division's count) last 0.1-0.3 ms, and the thread woke tens of microseconds after the event, with
// the step's next launches behind it. Spinning on the event (query + pause) for up to kSpinNs first
// returns within a microsecond of the completion; longer waits still block (set_event_spin(0): block
// at once).
static int g_ev_spin = 1;
void set_event_spin(int on) { g_ev_spin = on; }
void ev_sync(uintptr_t e) {
  hipEvent_t ev = reinterpret_cast<hipEvent_t>(e);
  if (g_ev_spin) {
    constexpr int64_t kSpinNs = 20'000'000;  // 20 ms
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned it = 0;; ++it) {
      const hipError_t r = msd::event_query(ev);
      if (r == hipSuccess) return;
      if (r != hipErrorNotReady) MS_HIP_CHECK(r);
      __builtin_ia32_pause();
      if ((it & 255u) == 255u &&
          std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count() > kSpinNs)
        break;
    }
  }
  MS_HIP_CHECK(msd::event_synchronize(ev));
}

// `dst` waits for everything issued to `src` so far (a fresh pooled event in between)
void stream_join(uintptr_t dst, uintptr_t src) {
  if (dst == src) return;
  const uintptr_t e = ev_acquire();
  ev_record(e, src);
  ev_wait(dst, e);
  ev_release(e);  // (re-recording later is fine: the wait already captured this record)
}

void release_events() {
  std::lock_guard<std::mutex> lk(g_ev_mu);
  for (hipEvent_t e : g_ev_all) MS_HIP_CHECK(hipEventDestroy(e));
  g_ev_all.clear();
  g_ev_free.clear();
}

void bind_events(py::module_& m) {
  msd::gdef(m, "ev_acquire", &ev_acquire);
  msd::gdef(m, "ev_release", &ev_release);
  msd::gdef(m, "ev_record", &ev_record);
  msd::gdef(m, "ev_wait", &ev_wait);
  msd::gdef(m, "ev_query", &ev_query);
  msd::gdef(m, "ev_sync", &ev_sync, py::call_guard<py::gil_scoped_release>());
  msd::gdef(m, "set_event_spin", &set_event_spin, "1: host event waits spin before blocking (0: block at once)");
  msd::gdef(m, "stream_join", &stream_join);
}

}  // namespace msd
