// Host cost of kernel launches on this stack (not part of the package): back-to-back launches of an
// empty kernel with small / 256-byte arguments, and the same 17-kernel sequence as a hipGraph.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/lab/launch_lab.hip -o launch_lab.bin && ./launch_lab.bin
#include <hip/hip_runtime.h>

#include <chrono>
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

struct Big {
  unsigned long long w[32];
};
__global__ void k_small(int* p, int v) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && v == -12345) *p = v;
}
__global__ void k_big(Big b) {
  if (threadIdx.x == 0 && blockIdx.x == 0 && b.w[3] == 12345ull) *reinterpret_cast<int*>(b.w[0]) = 1;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  int* d;
  CK(hipMalloc(&d, 4));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  Big b{};
  b.w[0] = reinterpret_cast<unsigned long long>(d);
  for (int i = 0; i < 100; ++i) k_small<<<1, 64, 0, s>>>(d, i);
  CK(hipStreamSynchronize(s));
  const int N = 2000;
  for (int grid : {1, 256, 4096}) {
    double t0 = now_us();
    for (int i = 0; i < N; ++i) k_small<<<grid, 256, 0, s>>>(d, i);
    double t1 = now_us();
    CK(hipStreamSynchronize(s));
    double t2 = now_us();
    for (int i = 0; i < N; ++i) k_big<<<grid, 256, 0, s>>>(b);
    double t3 = now_us();
    CK(hipStreamSynchronize(s));
    std::printf("{\"grid\": %d, \"launch_small_us\": %.2f, \"launch_256B_us\": %.2f}\n", grid, (t1 - t0) / N,
                (t3 - t2) / N);
  }
  // a 17-kernel sequence captured once, launched as a graph
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int i = 0; i < 17; ++i) k_big<<<64, 256, 0, s>>>(b);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int i = 0; i < 20; ++i) CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  const int M = 300;
  double t0 = now_us();
  for (int i = 0; i < M; ++i) CK(hipGraphLaunch(ge, s));
  double t1 = now_us();
  CK(hipStreamSynchronize(s));
  double t2 = now_us();
  for (int i = 0; i < M; ++i)
    for (int j = 0; j < 17; ++j) k_big<<<64, 256, 0, s>>>(b);
  double t3 = now_us();
  CK(hipStreamSynchronize(s));
  double t4 = now_us();
  std::printf("{\"graph17_launch_us\": %.2f, \"direct17_us\": %.2f, \"graph17_device_us\": %.2f, \"direct17_device_us\": %.2f}\n",
              (t1 - t0) / M, (t3 - t2) / M, (t2 - t0) / M, (t4 - t2) / M);
  return 0;
}
