// Stand-alone bandwidth lab for the diffusion stencil (not part of the package): times a float4 copy
// (the HBM roofline of a read + write stream) and variants of the 9-point wrap-around stencil on an
// m x S x S fp32 map, so load policy, rows in flight, band height and grid size can be A/B'd in
// seconds without the framework around them.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/lab/stencil_lab.hip -o build/stencil_lab
//   build/stencil_lab [S=4096] [m=14] [iters=20]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ float4 ld4(const float* p) {
  f4 q;
  if constexpr (NT) q = __builtin_nontemporal_load(reinterpret_cast<const f4*>(p));
  else q = *reinterpret_cast<const f4*>(p);
  return make_float4(q.x, q.y, q.z, q.w);
}
template <bool NT>
__device__ __forceinline__ float ld1(const float* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NTS>
__device__ __forceinline__ void st4(float* p, float4 v) {
  const f4 q = {v.x, v.y, v.z, v.w};
  if constexpr (NTS) __builtin_nontemporal_store(q, reinterpret_cast<f4*>(p));
  else *reinterpret_cast<f4*>(p) = q;
}

template <bool NT, bool NTS>
__global__ void __launch_bounds__(256) copy_kernel(const float* __restrict__ in, float* __restrict__ out, size_t n4) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256)
    st4<NTS>(out + 4 * i, ld4<NT>(in + 4 * i));
}

// each block copies one contiguous chunk, U float4 loads in flight per lane
template <int U>
__global__ void __launch_bounds__(256) copy_chunk_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                         size_t n4, size_t per_block) {
  const size_t lo = (size_t)blockIdx.x * per_block, hi = lo + per_block < n4 ? lo + per_block : n4;
  for (size_t i0 = lo + threadIdx.x; i0 < hi; i0 += 256 * U) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = i0 + (size_t)u * 256;
      if (i < hi) v[u] = ld4<false>(in + 4 * i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t i = i0 + (size_t)u * 256;
      if (i < hi) st4<true>(out + 4 * i, v[u]);
    }
  }
}
// grid-stride with U loads in flight
template <int U>
__global__ void __launch_bounds__(256) copy_u_kernel(const float* __restrict__ in, float* __restrict__ out, size_t n4) {
  const size_t step = (size_t)gridDim.x * 256;
  for (size_t i0 = (size_t)blockIdx.x * 256 + threadIdx.x; i0 < n4; i0 += step * U) {
    float4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) if (i0 + u * step < n4) v[u] = ld4<false>(in + 4 * (i0 + u * step));
#pragma unroll
    for (int u = 0; u < U; ++u) if (i0 + u * step < n4) st4<true>(out + 4 * (i0 + u * step), v[u]);
  }
}
__global__ void __launch_bounds__(256) read_kernel(const float* __restrict__ in, size_t n4, float* __restrict__ sink) {
  float acc = 0.0f;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    const float4 v = ld4<false>(in + 4 * i);
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 12345.678f) sink[0] = acc;
}
__global__ void __launch_bounds__(256) write_kernel(float* __restrict__ out, size_t n4) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256)
    st4<true>(out + 4 * i, make_float4(1.f, 2.f, 3.f, 4.f));
}

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// One wave: 256 columns (4 per lane) x a band of BAND rows, sliding down with the 3x3 window in
// registers; DEPTH rows of loads in flight ahead of the row being computed (a register ring).
// Tiles (column strip, group of 4 bands, molecule), x fastest; grid-stride over tiles.
struct Row {
  float4 v;
  float el, er;
};
template <bool NT, bool NTS, int DEPTH, int BAND, int HALO = 1, bool SUMS = true, bool WIDE = false>
__global__ void __launch_bounds__(256) stencil_kernel(const float* __restrict__ in, float* __restrict__ out, int S,
                                                      int m, float a, float b, double* __restrict__ part) {
  // WIDE: the 4 waves of a block take 4 adjacent column strips of the same band (a 4 KB row segment
  // per block row); else 4 consecutive bands of one strip
  const int gx = WIDE ? S / 1024 : S / 256, gy = WIDE ? S / BAND : (S / BAND + 3) / 4, ntiles = gx * gy * m;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  double before = 0.0, after = 0.0;
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int bx = tile % gx, by = (tile / gx) % gy, mol = tile / (gx * gy);
    const int y0 = WIDE ? (bx * 4 + wv) * 256 + lane * 4 : bx * 256 + lane * 4;
    const bool need_l = lane == 0, need_r = lane == 63;
    const int yl = y0 == 0 ? S - 1 : y0 - 1, yr = y0 + 4 >= S ? 0 : y0 + 4;
    const float* src = in + (size_t)mol * S * S;
    float* dst = out + (size_t)mol * S * S;
    const int o0 = WIDE ? by * BAND : (by * 4 + wv) * BAND;
    if (o0 >= S) continue;
    const int o1 = min(S, o0 + BAND);
    auto fetch = [&](int o, Row& r) {
      const int x = o < 0 ? o + S : (o >= S ? o - S : o);
      const float* p = src + (size_t)x * S;
      r.v = ld4<NT>(p + y0);
      if constexpr (HALO == 1) {
        r.el = need_l ? ld1<NT>(p + yl) : 0.0f;
        r.er = need_r ? ld1<NT>(p + yr) : 0.0f;
      } else if constexpr (HALO == 2) {  // one load instruction: lane 0 the left, lane 63 the right column
        const float e = (need_l || need_r) ? ld1<NT>(p + (need_l ? yl : yr)) : 0.0f;
        r.el = e;
        r.er = e;
      } else if constexpr (HALO == 3) {  // branch-free: every lane loads (the inner lanes their own column)
        const float e = ld1<NT>(p + (need_l ? yl : (need_r ? yr : y0)));
        r.el = e;
        r.er = e;
      } else {
        r.el = r.er = 0.0f;
      }
    };
    auto hs = [&](const Row& r, float h[4], float v[4], float& L, float& R) {
      v[0] = r.v.x, v[1] = r.v.y, v[2] = r.v.z, v[3] = r.v.w;
      const float up = __shfl_up(v[3], 1), dn = __shfl_down(v[0], 1);
      L = need_l ? r.el : up;
      R = need_r ? r.er : dn;
      h[0] = L + v[0] + v[1];
      h[1] = v[0] + v[1] + v[2];
      h[2] = v[1] + v[2] + v[3];
      h[3] = v[2] + v[3] + R;
    };
    Row ring[DEPTH + 1];
    Row rp, rc;
    fetch(o0 - 1, rp);
    fetch(o0, rc);
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) fetch(min(o0 + 1 + d, o1), ring[d]);
    float hp[4], hc[4], vp[4], vc[4], Lc, Rc, Lp, Rp;
    hs(rp, hp, vp, Lp, Rp);
    hs(rc, hc, vc, Lc, Rc);
    auto step = [&](int o, int u) {
      // ring slot u holds row o + u + 1; refill slot (u + DEPTH) % (DEPTH + 1) with row o + u + 1 + DEPTH
      fetch(min(o + u + 1 + DEPTH, o1), ring[(u + DEPTH) % (DEPTH + 1)]);
      float hn[4], vn[4], Ln, Rn;
      hs(ring[u], hn, vn, Ln, Rn);
      const float lft[4] = {Lc, vc[0], vc[1], vc[2]}, rgt[4] = {vc[1], vc[2], vc[3], Rc};
      float res[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) res[j] = b * vc[j] + a * (hp[j] + hn[j] + lft[j] + rgt[j]);
      st4<NTS>(dst + (size_t)(o + u) * S + y0, make_float4(res[0], res[1], res[2], res[3]));
      if constexpr (SUMS) {
        before += (double)((vc[0] + vc[1]) + (vc[2] + vc[3]));
        after += (double)((res[0] + res[1]) + (res[2] + res[3]));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) hp[j] = hc[j], hc[j] = hn[j], vc[j] = vn[j];
      Lc = Ln, Rc = Rn;
    };
    int o = o0;
    // whole ring turns without guards (exact vmcnt waits), then the guarded tail
    for (; o + DEPTH + 1 <= o1; o += DEPTH + 1) {
#pragma unroll
      for (int u = 0; u <= DEPTH; ++u) step(o, u);
    }
    if (o < o1) {
#pragma unroll
      for (int u = 0; u <= DEPTH; ++u)
        if (o + u < o1) step(o, u);
    }
  }
  before = wsum(before);
  after = wsum(after);
  if (lane == 0) {
    part[(blockIdx.x * 4 + wv) * 2] = before;
    part[(blockIdx.x * 4 + wv) * 2 + 1] = after;
  }
}

static float time_it(int iters, const std::function<void()>& f) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < iters; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3f / iters;
}

int main(int argc, char** argv) {
  const int S = argc > 1 ? std::atoi(argv[1]) : 4096, m = argc > 2 ? std::atoi(argv[2]) : 14;
  const int iters = argc > 3 ? std::atoi(argv[3]) : 20;
  const size_t n = (size_t)m * S * S;
  float *x, *y;
  double* part;
  CK(hipMalloc(&x, n * 4));
  CK(hipMalloc(&y, n * 4 + ((size_t)64 << 20)));
  CK(hipMalloc(&part, (size_t)1 << 24));
  {
    std::vector<float> h(n);
    for (size_t i = 0; i < n; ++i) h[i] = (float)((i * 2654435761u) % 1000) * 1e-3f;
    CK(hipMemcpy(x, h.data(), n * 4, hipMemcpyHostToDevice));
  }
  const double bytes = 2.0 * n * 4;
  auto report = [&](const char* name, int blocks, float us) {
    std::printf("{\"kernel\": \"%s\", \"blocks\": %d, \"us\": %.1f, \"TBps\": %.3f}\n", name, blocks, us,
                bytes / us * 1e-6);
    std::fflush(stdout);
  };
  const int mode = argc > 4 ? std::atoi(argv[4]) : 0;
  if (mode == 0 || mode == 1) {
    auto rep1 = [&](const char* nm, int blocks, float us, double by) {
      std::printf("{\"kernel\": \"%s\", \"blocks\": %d, \"us\": %.1f, \"TBps\": %.3f}\n", nm, blocks, us, by / us * 1e-6);
      std::fflush(stdout);
    };
    for (int blocks : {256, 512, 1024, 2048}) {
      rep1("read", blocks, time_it(iters, [&] { read_kernel<<<blocks, 256>>>(x, n / 4, reinterpret_cast<float*>(part)); }), n * 4.0);
      rep1("write", blocks, time_it(iters, [&] { write_kernel<<<blocks, 256>>>(y, n / 4); }), n * 4.0);
      report("copy", blocks, time_it(iters, [&] { copy_kernel<false, true><<<blocks, 256>>>(x, y, n / 4); }));
      report("copy_u4", blocks, time_it(iters, [&] { copy_u_kernel<4><<<blocks, 256>>>(x, y, n / 4); }));
      const size_t pb = (n / 4 + blocks - 1) / blocks;
      report("copy_chunk_u1", blocks, time_it(iters, [&] { copy_chunk_kernel<1><<<blocks, 256>>>(x, y, n / 4, pb); }));
      report("copy_chunk_u4", blocks, time_it(iters, [&] { copy_chunk_kernel<4><<<blocks, 256>>>(x, y, n / 4, pb); }));
    }
    // destination skewed against the source by 1 MiB + 4 KiB (channel / bank aliasing of the two streams)
    float* y2 = y + (((size_t)1 << 18) + 1024);
    const size_t n2 = n - (((size_t)1 << 18) + 1024);
    for (int blocks : {1024}) {
      const double by = 2.0 * n2 * 4;
      auto r2 = [&](const char* nm, float us) {
        std::printf("{\"kernel\": \"%s\", \"blocks\": %d, \"us\": %.1f, \"TBps\": %.3f}\n", nm, blocks, us, by / us * 1e-6);
      };
      r2("copy_skew", time_it(iters, [&] { copy_kernel<false, true><<<blocks, 256>>>(x, y2, n2 / 4); }));
      const size_t pb = (n2 / 4 + blocks - 1) / blocks;
      r2("copy_chunk_u4_skew", time_it(iters, [&] { copy_chunk_kernel<4><<<blocks, 256>>>(x, y2, n2 / 4, pb); }));
    }
  }
  if (mode == 1) return 0;
  if (mode == 6) {
    const float a = 0.1f, b = 0.2f;
    const size_t skew = argc > 5 ? (size_t)std::atoll(argv[5]) : ((size_t)2 << 20) + 8192;
    float* yy = y + skew / 4;
#define R7(D, BAND)                                                                                          \
    for (int g : {512, 768, 1024, 0}) {                                                                     \
      const int tiles = (S / 256) * ((S / BAND + 3) / 4) * m, gg = g ? std::min(g, tiles) : tiles;          \
      char nm[64];                                                                                           \
      std::snprintf(nm, sizeof nm, "h3_d%d_b%d", D, BAND);                                                   \
      report(nm, gg, time_it(iters, [&] { stencil_kernel<false, true, D, BAND, 3, true, false><<<gg, 256>>>(x, yy, S, m, a, b, part); })); \
    }
    R7(2, 64) R7(3, 64) R7(4, 64) R7(2, 128) R7(3, 128) R7(5, 64) R7(2, 48) R7(3, 96)
    return 0;
  }
  if (mode == 5) {
    const float a = 0.1f, b = 0.2f;
    float* yy = y + (((size_t)2 << 20) + 8192) / 4;
    const int t32 = (S / 256) * ((S / 32 + 3) / 4) * m, t16 = (S / 256) * ((S / 16 + 3) / 4) * m;
#define R6(NM, D, BAND, G)                                                                                 \
    report(NM, G, time_it(iters, [&] { stencil_kernel<false, true, D, BAND, 3, true, false><<<G, 256>>>(x, yy, S, m, a, b, part); }));
    for (int rep = 0; rep < 2; ++rep) {
      R6("h3_d1_b32_1024", 1, 32, 1024)
      R6("h3_d2_b32_1024", 2, 32, 1024)
      R6("h3_d3_b32_1024", 3, 32, 1024)
      R6("h3_d2_b32_512", 2, 32, 512)
      R6("h3_d4_b32_512", 4, 32, 512)
      R6("h3_d4_b32_256", 4, 32, 256)
      R6("h3_d2_b32_all", 2, 32, t32)
      R6("h3_d1_b16_all", 1, 16, t16)
      R6("h3_d2_b16_all", 2, 16, t16)
      R6("h3_d2_b64_768", 2, 64, 768)
    }
    return 0;
  }
  if (mode == 4) {
    const float a = 0.1f, b = 0.2f;
    float* yy = y + (((size_t)2 << 20) + 8192) / 4;
#define R5(NM, D, BAND, G)                                                                                 \
    report(NM, G, time_it(iters, [&] { stencil_kernel<false, true, D, BAND, 1, true, false><<<G, 256>>>(x, yy, S, m, a, b, part); }));
    for (int rep = 0; rep < 2; ++rep) {
      R5("d1_b32_256", 1, 32, 256)
      R5("d2_b32_256", 2, 32, 256)
      R5("d4_b32_256", 4, 32, 256)
      R5("d1_b32_512", 1, 32, 512)
      R5("d2_b32_512", 2, 32, 512)
      R5("d3_b32_512", 3, 32, 512)
      R5("d4_b64_512", 4, 64, 512)
      R5("d2_b64_768", 2, 64, 768)
      R5("d1_b32_1024", 1, 32, 1024)
    }
    return 0;
  }
  if (mode == 3) {
    const float a = 0.1f, b = 0.2f;
    float* yy = y + (((size_t)2 << 20) + 8192) / 4;
    const int t32 = (S / 256) * ((S / 32 + 3) / 4) * m, t16 = (S / 256) * ((S / 16 + 3) / 4) * m;
#define R3(NM, HALO, SUMS, BAND, G)                                                                                 \
    report(NM, G, time_it(iters, [&] { stencil_kernel<false, true, 1, BAND, HALO, SUMS><<<G, 256>>>(x, yy, S, m, a, b, part); }));
#define R4(NM, BAND, G)                                                                                 \
    report(NM, G, time_it(iters, [&] { stencil_kernel<false, true, 1, BAND, 1, true, true><<<G, 256>>>(x, yy, S, m, a, b, part); }));
    for (int rep = 0; rep < 2; ++rep) {
      R4("wide_b32_1024", 32, 1024)
      R4("wide_b32_2048", 32, 2048)
      R4("wide_b32_all", 32, t32)
      R4("wide_b16_1024", 16, 1024)
      R4("wide_b16_all", 16, t16)
      R4("wide_b64_1024", 64, 1024)
      R4("wide_b64_all", 64, t32 / 2)
      R4("wide_b128_all", 128, t32 / 4)
    }
    for (int rep = 0; rep < 1; ++rep) {
      R3("b32_halo1_sums", 1, true, 32, 1024)
      R3("b32_halo2_sums", 2, true, 32, 1024)
      R3("b32_halo0_sums", 0, true, 32, 1024)
      R3("b32_halo1_nosums", 1, false, 32, 1024)
      R3("b32_halo0_nosums", 0, false, 32, 1024)
      R3("b16all_halo1_sums", 1, true, 16, t16)
      R3("b16all_halo2_sums", 2, true, 16, t16)
      R3("b16all_halo0_nosums", 0, false, 16, t16)
      R3("b32all_halo2_sums", 2, true, 32, t32)
    }
    return 0;
  }
  if (mode == 2) {  // skew of the destination against the source (bytes)
    const float a = 0.1f, b = 0.2f;
    for (size_t skew : {(size_t)0, (size_t)4096, (size_t)65536, (size_t)1 << 20, ((size_t)1 << 20) + 4096,
                        ((size_t)2 << 20) + 8192, ((size_t)32 << 20) + 4096, (size_t)256 + 4096 * 3}) {
      float* yy = y + skew / 4;
      char nm[96];
      std::snprintf(nm, sizeof nm, "copy_skew%zu", skew);
      report(nm, 1024, time_it(iters, [&] { copy_kernel<false, true><<<1024, 256>>>(x, yy, n / 4); }));
      std::snprintf(nm, sizeof nm, "copy512_skew%zu", skew);
      report(nm, 512, time_it(iters, [&] { copy_kernel<false, true><<<512, 256>>>(x, yy, n / 4); }));
      std::snprintf(nm, sizeof nm, "stencil_b32_skew%zu", skew);
      report(nm, 1024, time_it(iters, [&] { stencil_kernel<false, true, 1, 32><<<1024, 256>>>(x, yy, S, m, a, b, part); }));
      const int t16 = (S / 256) * ((S / 16 + 3) / 4) * m;
      std::snprintf(nm, sizeof nm, "stencil_b16_all_skew%zu", skew);
      report(nm, t16, time_it(iters, [&] { stencil_kernel<false, true, 1, 16><<<t16, 256>>>(x, yy, S, m, a, b, part); }));
    }
    return 0;
  }
  const float a = 0.1f, b = 0.2f;
#define RUN(NT, NTS, D, B)                                                                                   \
  for (int blocks : {1024, 2048, 0}) {                                                                      \
    const int tiles = (S / 256) * ((S / B + 3) / 4) * m, g = blocks ? std::min(blocks, tiles) : tiles;      \
    char nm[96];                                                                                             \
    std::snprintf(nm, sizeof nm, "stencil_nt%d_nts%d_depth%d_band%d", NT, NTS, D, B);                        \
    report(nm, g, time_it(iters, [&] { stencil_kernel<NT, NTS, D, B><<<g, 256>>>(x, y, S, m, a, b, part); })); \
  }
  RUN(false, true, 1, 32)
  RUN(true, true, 1, 32)
  RUN(false, false, 1, 32)
  RUN(false, true, 2, 32)
  RUN(true, true, 2, 32)
  RUN(false, true, 3, 32)
  RUN(false, true, 1, 64)
  RUN(true, true, 2, 64)
  RUN(false, true, 1, 16)
  CK(hipFree(x));
  CK(hipFree(y));
  CK(hipFree(part));
  return 0;
}
