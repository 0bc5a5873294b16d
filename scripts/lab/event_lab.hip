// Cost of a cross-stream dependency on this stack (not part of the package): stream A runs a long
// kernel, stream B a short one whose completion event A waits for (already complete by the time A
// reaches the wait), then A runs a short kernel. Under `rocprofv3 --kernel-trace` the gap between
// the long kernel's end and the next kernel's start is the price of the wait; the same sequence
// without the wait is the baseline.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/lab/event_lab.hip -o event_lab.bin
//   rocprofv3 --kernel-trace --stats -d out -o run --output-format csv -- ./event_lab.bin
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                          \
    }                                                                                        \
  } while (0)

// ~`cycles` of busy waiting per wave (s_memtime ticks at a fixed rate)
__global__ void k_long(long long cycles, int* out) {
  const long long t0 = __builtin_readcyclecounter();
  while (__builtin_readcyclecounter() - t0 < cycles) {
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) out[0] = 1;
}
__global__ void k_mark_a(int* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) out[1] = 1;
}
__global__ void k_side(int* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) out[2] = 1;
}
__global__ void k_next_wait(int* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) out[3] = 1;
}
__global__ void k_next_plain(int* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) out[4] = 1;
}

int main() {
  int* d;
  CK(hipMalloc(&d, 64));
  hipStream_t a, b;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
  hipEvent_t e;
  CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  const long long cyc = 200000;  // ~100-200 us
  for (int it = 0; it < 30; ++it) {
    // with a wait on an event recorded on stream b long before stream a reaches it
    k_long<<<256, 64, 0, a>>>(cyc, d);
    k_side<<<1, 64, 0, b>>>(d);
    CK(hipEventRecord(e, b));
    k_mark_a<<<1, 64, 0, a>>>(d);
    CK(hipStreamWaitEvent(a, e, 0));
    k_next_wait<<<1, 64, 0, a>>>(d);
    CK(hipStreamSynchronize(a));
    CK(hipStreamSynchronize(b));
    // the same without the wait
    k_long<<<256, 64, 0, a>>>(cyc, d);
    k_mark_a<<<1, 64, 0, a>>>(d);
    k_next_plain<<<1, 64, 0, a>>>(d);
    CK(hipStreamSynchronize(a));
  }
  std::printf("done\n");
  return 0;
}
