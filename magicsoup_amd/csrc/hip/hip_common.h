// Device-side helpers shared by the gfx950 kernels of magicsoup_amd._hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdexcept>
#include <string>

#include "launch.h"
#include "ms_common.h"

#define MS_HIP_CHECK(expr)                                                                  \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    if (_e != hipSuccess)                                                                   \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__));                  \
  } while (0)

#define MS_LAUNCH_CHECK() MS_HIP_CHECK(hipGetLastError())

namespace msd {

template <class T>
inline T* P_(uintptr_t p) {
  return reinterpret_cast<T*>(p);
}
inline hipStream_t S_(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }
inline unsigned cdiv(long long a, long long b) { return (unsigned)((a + b - 1) / b); }

// ---------------------------------------------------------------- Philox4x32-10 counter RNG
struct Philox {
  uint32_t c0, c1, c2, c3, k0, k1;
  __device__ __forceinline__ Philox(uint64_t seed, uint64_t stream, uint32_t item)
      : c0(item), c1((uint32_t)stream), c2((uint32_t)(stream >> 32)), c3(0),
        k0((uint32_t)seed), k1((uint32_t)(seed >> 32)) {}
  __device__ __forceinline__ uint4 next() {
    uint32_t x0 = c0, x1 = c1, x2 = c2, x3 = c3, a = k0, b = k1;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      const uint64_t p0 = (uint64_t)0xD2511F53u * x0;
      const uint64_t p1 = (uint64_t)0xCD9E8D57u * x2;
      const uint32_t y0 = (uint32_t)(p1 >> 32) ^ x1 ^ a;
      const uint32_t y2 = (uint32_t)(p0 >> 32) ^ x3 ^ b;
      x1 = (uint32_t)p1;
      x3 = (uint32_t)p0;
      x0 = y0;
      x2 = y2;
      a += 0x9E3779B9u;
      b += 0xBB67AE85u;
    }
    ++c3;
    return make_uint4(x0, x1, x2, x3);
  }
  // 4 uniforms are cached per block of output
  uint4 buf;
  int have = 0;
  __device__ __forceinline__ uint32_t u32() {
    if (have == 0) {
      buf = next();
      have = 4;
    }
    --have;
    return have == 3 ? buf.x : have == 2 ? buf.y : have == 1 ? buf.z : buf.w;
  }
  // uniform in [0, 1)
  __device__ __forceinline__ float uniform() { return (u32() >> 8) * (1.0f / 16777216.0f); }
  __device__ __forceinline__ double uniform_d() {
    const uint64_t hi = u32(), lo = u32();
    return ((hi << 21) ^ (lo >> 11)) * (1.0 / 9007199254740992.0);
  }
  // uniform integer in [0, n)
  __device__ __forceinline__ uint32_t below(uint32_t n) { return (uint32_t)(((uint64_t)u32() * n) >> 32); }
  __device__ __forceinline__ uint64_t below64(uint64_t n) {
    const uint64_t r = ((uint64_t)u32() << 32) | u32();
    return r % n;
  }
};

// Poisson(lambda) sample: inversion for small lambda, rounded normal approximation above 30.
__device__ __forceinline__ long long poisson(Philox& rng, double lam) {
  if (!(lam > 0.0)) return 0;
  if (lam < 30.0) {
    const double u = rng.uniform_d();
    // k = 0 iff u <= exp(-lam) >= 1 - lam: below 1 - lam (less a few ulps for the rounding of both
    // sides) the answer is 0 without the exp -- the same draw, for all but ~lam of the calls (the
    // genome pipeline draws per neighbour slot at lam ~ 1e-4)
    if (u <= (1.0 - lam) - 1e-15) return 0;
    double p = exp(-lam), cum = p;
    long long k = 0;
    while (u > cum && k < 1000) {
      ++k;
      p *= lam / (double)k;
      cum += p;
    }
    return k;
  }
  // Box-Muller normal
  const double u1 = fmax(rng.uniform_d(), 1e-300), u2 = rng.uniform_d();
  const double z = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
  const long long k = (long long)floor(lam + sqrt(lam) * z + 0.5);
  return k < 0 ? 0 : k;
}

// ---------------------------------------------------------------- genome pool
// GPU genomes live in one byte pool (models/strings.py PoolArena): cell i's genome is the lens[i]
// bytes at pool + off[i], allocations 16-byte aligned and never written again (new genomes take new
// space, so cells can share a genome). An allocation is an atomic bump of the device counter `top`;
// -1 when the pool is full (the caller raises a flag; the host collects or grows the pool).
// (an empty genome takes 16 bytes too: every allocation has an offset of its own)
__device__ __forceinline__ long long pool_alloc(unsigned long long* top, long long cap, int len) {
  const unsigned long long sz = ((unsigned long long)(len > 1 ? len : 1) + 15ull) & ~15ull;
  const unsigned long long o = atomicAdd(top, sz);
  return (long long)(o + sz) <= cap ? (long long)o : -1;
}

// The pool as kernel launchers take it (filled from Python: PoolArena.args()).
struct GenomePoolArgs {
  uintptr_t pool = 0, off = 0, top = 0, failed = 0;  // bytes, per-cell offsets, bump counter, error word
  long long cap = 0;                                 // pool bytes
};

// ---------------------------------------------------------------- wave helpers
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

}  // namespace msd
