// Kernel launches of the device core, optionally batched into hipGraphs.
//
// Every launcher issues its kernels as `kl(kernel, grid, block, lds, stream)(args...)` instead of the
// triple-chevron syntax: by default one hipLaunchKernel, exactly what the chevrons compile to. With
// batching on (MS_GRAPH_BATCH=1 or set_graph_batch(True)), every call from Python into the module
// (BatchGuard, installed by gdef() on each binding) records its launches instead and issues them as
// ONE hipGraphLaunch when it returns, or earlier, before anything else goes to a stream (memset /
// copy / event / RCCL / synchronisation: the wrappers below flush first). A recorded sequence is
// instantiated once per distinct kernel sequence and replayed with its arguments and grids updated
// in place (hipGraphExecKernelNodeSetParams for the nodes that changed).
//
// Measured (profiles/r6/graph_batch): the host issue cost drops from ~3 to ~1 us per kernel
// (scripts/lab/launch_lab.hip: 17 kernels 11.6-15 us vs 52 us direct; updates while earlier launches
// of the graph are still queued leave those untouched, 3400 nodes checked; a graph on one stream
// still runs next to another stream's kernel), and a bench step's genome chain issues 15 us faster --
// but whole steps run 2-7 % SLOWER batched (in-process A/B, alternating blocks of steps in one world:
// flagship 0.829 vs 0.813 ms, the flagship as one strip 1.09 vs 1.02, the N = 8 proxy 0.385 vs
// 0.366), so direct launches stay the default: on the device a graph's kernel nodes run slower
// than the same kernels launched directly with the host ahead (8 write / read-back pairs of a 2 MiB
// buffer: 4.85 vs 4.20 us per pair, launch_lab_l2.log), which outweighs the host saving wherever the
// step is device-bound. Results are bit-identical either way
// (test_graph_batched_launches_match_direct_launches).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <tuple>
#include <utility>

namespace msd {

// ---------------------------------------------------------------- batch state (launch.hip)
void batch_enter();
void batch_exit(bool flush_now);  // flush_now false: leaving by an exception (best effort, no throw)
void batch_flush();               // issue what is recorded (no-op outside a batch / when empty)
bool batch_recording();           // inside a batch, batching enabled
void batch_record(const void* f, dim3 g, dim3 b, unsigned lds, hipStream_t st, void** args, const size_t* sizes,
                  const size_t* aligns, int nargs);

// One call from Python: kernels recorded while it runs go out as one graph when it returns.
struct BatchGuard {
  bool done = false;
  BatchGuard() { batch_enter(); }
  void finish() {
    done = true;
    batch_exit(true);
  }
  ~BatchGuard() {
    if (!done) batch_exit(false);
  }
  BatchGuard(const BatchGuard&) = delete;
  BatchGuard& operator=(const BatchGuard&) = delete;
};

template <class... P>
struct KLaunch {
  void (*f)(P...);
  dim3 g, b;
  unsigned lds;
  hipStream_t st;

  template <class... A>
  void operator()(A&&... a) const {
    static_assert(sizeof...(A) == sizeof...(P), "kernel argument count");
    if ((size_t)g.x * g.y * g.z == 0) return;  // (an empty grid launches nothing)
    if constexpr (sizeof...(P) == 0) {
      std::tuple<> t;
      issue(t, std::index_sequence<>{});
    } else {
      std::tuple<P...> t(std::forward<A>(a)...);
      issue(t, std::index_sequence_for<P...>{});
    }
  }

 private:
  template <size_t... I>
  void issue(std::tuple<P...>& t, std::index_sequence<I...>) const {
    constexpr int n = (int)sizeof...(P);
    void* ptrs[n > 0 ? n : 1] = {static_cast<void*>(&std::get<I>(t))...};
    if (batch_recording()) {
      const size_t sizes[n > 0 ? n : 1] = {sizeof(P)...};
      const size_t aligns[n > 0 ? n : 1] = {alignof(P)...};
      batch_record(reinterpret_cast<const void*>(f), g, b, lds, st, ptrs, sizes, aligns, n);
      return;
    }
    const hipError_t e = hipLaunchKernel(reinterpret_cast<const void*>(f), g, b, ptrs, lds, st);
    (void)e;  // (reported by the launcher's MS_LAUNCH_CHECK, as for a chevron launch)
  }
};

template <class... P>
inline KLaunch<P...> kl(void (*f)(P...), dim3 g, dim3 b, size_t lds, hipStream_t st) {
  return KLaunch<P...>{f, g, b, (unsigned)lds, st};
}

// ---------------------------------------------------------------- stream operations (flush first)
inline hipError_t memset_async(void* p, int v, size_t n, hipStream_t s) {
  batch_flush();
  return hipMemsetAsync(p, v, n, s);
}
inline hipError_t memcpy_async(void* d, const void* src, size_t n, hipMemcpyKind k, hipStream_t s) {
  batch_flush();
  return hipMemcpyAsync(d, src, n, k, s);
}
inline hipError_t event_record(hipEvent_t e, hipStream_t s) {
  batch_flush();
  return hipEventRecord(e, s);
}
inline hipError_t stream_wait_event(hipStream_t s, hipEvent_t e, unsigned flags) {
  batch_flush();
  return hipStreamWaitEvent(s, e, flags);
}
inline hipError_t stream_synchronize(hipStream_t s) {
  batch_flush();
  return hipStreamSynchronize(s);
}
inline hipError_t stream_query(hipStream_t s) {
  batch_flush();
  return hipStreamQuery(s);
}
inline hipError_t event_query(hipEvent_t e) {
  batch_flush();
  return hipEventQuery(e);
}
inline hipError_t event_synchronize(hipEvent_t e) {
  batch_flush();
  return hipEventSynchronize(e);
}
inline hipError_t device_synchronize() {
  batch_flush();
  return hipDeviceSynchronize();
}
inline hipError_t dev_malloc(void** p, size_t n) {
  batch_flush();
  return hipMalloc(p, n);
}
inline hipError_t dev_free(void* p) {
  batch_flush();  // (a recorded kernel may still use it)
  return hipFree(p);
}
inline hipError_t flushed_coop_launch(const void* f, dim3 g, dim3 b, void** args, unsigned lds, hipStream_t s) {
  batch_flush();
  return hipLaunchCooperativeKernel(f, g, b, args, lds, s);
}
inline hipError_t dev_memset(void* p, int v, size_t n) {
  batch_flush();
  return hipMemset(p, v, n);
}

}  // namespace msd
