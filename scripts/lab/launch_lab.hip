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
// writes its own (slot, value) after a short spin: a graph updated while earlier launches of it are
// still queued must not show them the later arguments
__global__ void k_rec(int* out, int slot, int val, int spin) {
  long long t0 = clock64();
  while (clock64() - t0 < spin) {
  }
  if (threadIdx.x == 0) atomicAdd(out + slot, val);
}
// producer / consumer pair over a buffer that fits the L2: is a graph's data still in the cache
__global__ void k_write(float* x, int n, float v) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) x[i] = v + (float)i;
}
__global__ void k_read(const float* x, int n, float* out) {
  float a = 0.0f;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) a += x[i];
  if (a == -1.0f) *out = a;
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
  // every node's arguments and grid changed before each launch (hipGraphExecKernelNodeSetParams)
  {
    size_t nn = 0;
    CK(hipGraphGetNodes(g, nullptr, &nn));
    hipGraphNode_t nodes[64];
    CK(hipGraphGetNodes(g, nodes, &nn));
    hipKernelNodeParams kp[64];
    for (size_t j = 0; j < nn; ++j) CK(hipGraphKernelNodeGetParams(nodes[j], &kp[j]));
    Big bb[64];
    void* argp[64][1];
    double u0 = now_us();
    for (int i = 0; i < M; ++i) {
      for (size_t j = 0; j < nn; ++j) {
        bb[j] = b;
        bb[j].w[5] = (unsigned long long)(i * 64 + j);
        argp[j][0] = &bb[j];
        kp[j].kernelParams = argp[j];
        kp[j].gridDim = dim3(64 + (i & 1), 1, 1);
        CK(hipGraphExecKernelNodeSetParams(ge, nodes[j], &kp[j]));
      }
      CK(hipGraphLaunch(ge, s));
    }
    double u1 = now_us();
    CK(hipStreamSynchronize(s));
    double u2 = now_us();
    std::printf("{\"graph17_setparams_launch_us\": %.2f, \"graph17_setparams_device_us\": %.2f}\n", (u1 - u0) / M,
                (u2 - u0) / M);
  }
  // a graph whose kernels read their arguments from a device block refreshed by a captured
  // host-to-device copy from pinned memory (one memcpy node + 17 kernels)
  {
    Big* hb;
    Big* db;
    CK(hipHostMalloc(&hb, sizeof(Big), 0));
    CK(hipMalloc(&db, sizeof(Big)));
    *hb = b;
    hipGraph_t g2;
    hipGraphExec_t ge2;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    CK(hipMemcpyAsync(db, hb, sizeof(Big), hipMemcpyHostToDevice, s));
    for (int i = 0; i < 17; ++i) k_small<<<64, 256, 0, s>>>(reinterpret_cast<int*>(db), i);
    CK(hipStreamEndCapture(s, &g2));
    CK(hipGraphInstantiate(&ge2, g2, nullptr, nullptr, 0));
    for (int i = 0; i < 20; ++i) CK(hipGraphLaunch(ge2, s));
    CK(hipStreamSynchronize(s));
    double v0 = now_us();
    for (int i = 0; i < M; ++i) {
      CK(hipGraphLaunch(ge2, s));
      CK(hipStreamSynchronize(s));  // (the pinned block is rewritten for the next launch)
      hb->w[5] = i;
    }
    double v1 = now_us();
    std::printf("{\"graph_memcpy17_launch_sync_us\": %.2f}\n", (v1 - v0) / M);
    double w0 = now_us();
    for (int i = 0; i < M; ++i) {
      for (int j = 0; j < 17; ++j) k_big<<<64, 256, 0, s>>>(b);
      CK(hipStreamSynchronize(s));
    }
    double w1 = now_us();
    std::printf("{\"direct17_sync_us\": %.2f}\n", (w1 - w0) / M);
  }
  // correctness of in-flight updates: 200 launches of a 17-node graph, every node's arguments
  // changed before each launch, the device ~20 us behind per node
  {
    const int L = 200, K = 17;
    int* out;
    CK(hipMalloc(&out, L * K * sizeof(int)));
    CK(hipMemset(out, 0, L * K * sizeof(int)));
    hipGraph_t g3;
    hipGraphExec_t ge3;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int j = 0; j < K; ++j) k_rec<<<4, 64, 0, s>>>(out, 0, 0, 1);
    CK(hipStreamEndCapture(s, &g3));
    CK(hipGraphInstantiate(&ge3, g3, nullptr, nullptr, 0));
    size_t nn = 0;
    CK(hipGraphGetNodes(g3, nullptr, &nn));
    hipGraphNode_t nodes[64];
    CK(hipGraphGetNodes(g3, nodes, &nn));
    hipKernelNodeParams kp;
    CK(hipGraphKernelNodeGetParams(nodes[0], &kp));
    int spin = 20000;
    double t0 = now_us();
    for (int i = 0; i < L; ++i) {
      for (size_t j = 0; j < nn; ++j) {
        int slot = i * K + (int)j, val = slot + 1;
        void* a[4] = {&out, &slot, &val, &spin};
        kp.kernelParams = a;
        kp.gridDim = dim3(1 + (i % 4), 1, 1);
        CK(hipGraphExecKernelNodeSetParams(ge3, nodes[j], &kp));
      }
      CK(hipGraphLaunch(ge3, s));
    }
    double t1 = now_us();
    CK(hipStreamSynchronize(s));
    double t2 = now_us();
    int* h = (int*)std::malloc(L * K * sizeof(int));
    CK(hipMemcpy(h, out, L * K * sizeof(int), hipMemcpyDeviceToHost));
    int bad = 0;
    for (int i = 0; i < L; ++i)
      for (int j = 0; j < K; ++j) {
        const int x = i * K + j;
        if (h[x] != (x + 1) * (1 + (i % 4))) ++bad;
      }
    std::printf("{\"inflight_update_bad_slots\": %d, \"of\": %d, \"host_us_per_launch\": %.2f, \"device_us_per_launch\": %.2f}\n",
                bad, L * K, (t1 - t0) / L, (t2 - t0) / L);
  }
  // L2 reuse inside a graph: 8 x (write 2 MiB, read it back) as direct launches and as one graph,
  // device time from events with the host far ahead (a 2 ms spin first)
  {
    const int n = 512 * 1024;
    float *x, *o;
    CK(hipMalloc(&x, n * sizeof(float)));
    CK(hipMalloc(&o, sizeof(float)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipGraph_t g5;
    hipGraphExec_t ge5;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    for (int j = 0; j < 8; ++j) {
      k_write<<<256, 256, 0, s>>>(x, n, (float)j);
      k_read<<<256, 256, 0, s>>>(x, n, o);
    }
    CK(hipStreamEndCapture(s, &g5));
    CK(hipGraphInstantiate(&ge5, g5, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge5, s));
    CK(hipStreamSynchronize(s));
    for (int mode = 0; mode < 2; ++mode) {
      float best = 1e9f, tot = 0.0f;
      for (int rep = 0; rep < 20; ++rep) {
        k_rec<<<1, 64, 0, s>>>(o ? reinterpret_cast<int*>(o) : nullptr, 0, 0, 2100 * 2000);
        CK(hipEventRecord(e0, s));
        for (int r2 = 0; r2 < 4; ++r2) {
          if (mode == 0) {
            for (int j = 0; j < 8; ++j) {
              k_write<<<256, 256, 0, s>>>(x, n, (float)j);
              k_read<<<256, 256, 0, s>>>(x, n, o);
            }
          } else {
            CK(hipGraphLaunch(ge5, s));
          }
        }
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0.0f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = ms < best ? ms : best;
        tot += ms;
      }
      std::printf("{\"l2_pairs_%s_us_per_pair\": %.2f, \"mean\": %.2f}\n", mode == 0 ? "direct" : "graph",
                  best * 1e3f / 32.0f, tot / 20.0f * 1e3f / 32.0f);
    }
  }
  // concurrency across streams: a 300 us kernel on stream A, then 3 short kernels on stream B --
  // directly and as a graph -- and the host time until B's event completes
  {
    hipStream_t sa, sb;
    CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    int* o;
    CK(hipMalloc(&o, 64 * sizeof(int)));
    hipEvent_t eb;
    CK(hipEventCreateWithFlags(&eb, hipEventDisableTiming));
    hipGraph_t g4;
    hipGraphExec_t ge4;
    CK(hipStreamBeginCapture(sb, hipStreamCaptureModeGlobal));
    for (int j = 0; j < 3; ++j) k_rec<<<1, 64, 0, sb>>>(o, j, 1, 1000);
    CK(hipStreamEndCapture(sb, &g4));
    CK(hipGraphInstantiate(&ge4, g4, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge4, sb));
    CK(hipDeviceSynchronize());
    const int spin_a = 300 * 2100;  // ~300 us at ~2.1 GHz
    for (int mode = 0; mode < 2; ++mode) {
      double tot = 0.0;
      for (int rep = 0; rep < 20; ++rep) {
        k_rec<<<1, 64, 0, sa>>>(o, 10, 1, spin_a);
        double t0 = now_us();
        if (mode == 0) {
          for (int j = 0; j < 3; ++j) k_rec<<<1, 64, 0, sb>>>(o, j, 1, 1000);
        } else {
          CK(hipGraphLaunch(ge4, sb));
        }
        CK(hipEventRecord(eb, sb));
        while (hipEventQuery(eb) == hipErrorNotReady) {
        }
        tot += now_us() - t0;
        CK(hipDeviceSynchronize());
      }
      std::printf("{\"cross_stream_%s_us\": %.1f}\n", mode == 0 ? "direct" : "graph", tot / 20);
    }
  }
  return 0;
}
