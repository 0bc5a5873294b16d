// Recombination of two genomes (semantics of rust/mutations.rs:78-154), shared by the arena
// kernels (mutations.hip) and the strip-boundary recombination (dist.hip).
#pragma once
#include "hip_common.h"

namespace msd {

constexpr uint64_t kApplyStream = 0x6A09E667F3BCC909ull;

constexpr int kFloydMax = 32;

// k distinct sorted positions in [0, n): Floyd's algorithm + insertion sort (k <= kFloydMax).
__device__ __forceinline__ void floyd_sorted(Philox& rng, int n, int k, int* pos) {
  int cnt = 0;
  for (int j = n - k; j < n; ++j) {
    int t = (int)rng.below((uint32_t)(j + 1));
    for (int q = 0; q < cnt; ++q)
      if (pos[q] == t) {
        t = j;
        break;
      }
    pos[cnt++] = t;
  }
  for (int a = 1; a < cnt; ++a) {
    const int v = pos[a];
    int b = a - 1;
    while (b >= 0 && pos[b] > v) {
      pos[b + 1] = pos[b];
      --b;
    }
    pos[b + 1] = v;
  }
}

// Cooperative copy of src[a, b) to dst[w, ...) by the 64 lanes of a wave (clipped at cap). Parts
// start at any byte, so the lanes copy bytes, eight loads in flight per lane: a long evolving run's
// recombined pairs of 10^5 nt spent ~270 us in one load-store round trip per 64 bytes.
__device__ __forceinline__ void wave_copy(const uint8_t* src, int a, int b, uint8_t* dst, int w, int cap, int lane) {
  constexpr int U = 8;
  const int e = min(b, a + max(cap - w, 0));  // (bytes landing at or past cap are dropped)
  uint8_t* d = dst + (w - a);
  int t = a + lane;
  for (; t + 64 * (U - 1) < e; t += 64 * U) {
    uint8_t v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = src[t + 64 * u];
#pragma unroll
    for (int u = 0; u < U; ++u) d[t + 64 * u] = v[u];
  }
  for (; t < e; t += 64) d[t] = src[t];
}

// Recombine genomes sa[0, n0) and sb[0, n1) with kk strand breaks: cut both strands at kk sorted
// positions, shuffle the kk + 2 parts and split them at a random index into two new genomes o0 / o1
// (w0 / w1 bytes, clipped at out_width). One wavefront: lane 0 plans the parts (LDS `lparts` for up
// to kFloydMax cuts, else `parts_g` with room for kk + 2 entries of 3 ints), then all lanes copy.
// The RNG stream is (seed, call ^ kApplyStream, item): the same inputs give the same outputs on any
// rank, which the strip-boundary recombination relies on.
__device__ __forceinline__ void rec_pair_apply(const uint8_t* sa, int n0, const uint8_t* sb, int n1, int kk,
                                               uint64_t seed, uint64_t call, uint32_t item, int32_t* parts_g,
                                               int32_t* lparts, int* meta, uint8_t* o0, uint8_t* o1, int out_width,
                                               int& w0_out, int& w1_out) {
  const int lane = threadIdx.x;
  const int nb = n0 + n1;
  const uint32_t i = item;
  int32_t* pt = kk <= kFloydMax ? lparts : parts_g;
  if (lane == 0) {
    int need = kk;
    Philox rng(seed, call ^ kApplyStream, (uint32_t)i);
    int np = 0;
    auto push = [&](int src, int a0, int a1) {
      pt[3 * np] = src; pt[3 * np + 1] = a0; pt[3 * np + 2] = a1; ++np;
    };
    if (need <= kFloydMax) {
      int cuts[kFloydMax];
      floyd_sorted(rng, nb, need, cuts);
      int start = 0, q = 0;
      for (; q < need && cuts[q] < n0; ++q) {
        push(0, start, cuts[q]);
        start = cuts[q];
      }
      push(0, start, n0);
      start = 0;
      for (; q < need; ++q) {
        push(1, start, cuts[q] - n0);
        start = cuts[q] - n0;
      }
      push(1, start, n1);
    } else {
      int start = 0, src = 0;
      for (int t = 0; t < nb; ++t) {
        if (t == n0) {  // close the last part of strand a
          push(0, start, n0);
          start = 0;
          src = 1;
        }
        if (need > 0 && rng.below((uint32_t)(nb - t)) < (uint32_t)need) {
          --need;
          const int pos = src == 0 ? t : t - n0;
          push(src, start, pos);
          start = pos;
        }
      }
      if (n0 == nb) {  // strand b empty: close strand a here
        push(0, start, n0);
        start = 0;
      }
      push(1, start, n1);
    }
    // Fisher-Yates shuffle of the parts
    for (int q = np - 1; q > 0; --q) {
      const int r = (int)rng.below((uint32_t)(q + 1));
      for (int f = 0; f < 3; ++f) {
        const int32_t tmp = pt[3 * q + f];
        pt[3 * q + f] = pt[3 * r + f];
        pt[3 * r + f] = tmp;
      }
    }
    meta[0] = np;
    meta[1] = (int)rng.below((uint32_t)np);
  }
  __syncthreads();
  const int np = meta[0], split = meta[1];
  int w0 = 0, w1 = 0;
  for (int q = 0; q < np; ++q) {
    const uint8_t* src = pt[3 * q] == 0 ? sa : sb;
    const int a0 = pt[3 * q + 1], a1 = pt[3 * q + 2];
    if (q < split) {
      wave_copy(src, a0, a1, o0, w0, out_width, lane);
      w0 += a1 - a0;
    } else {
      wave_copy(src, a0, a1, o1, w1, out_width, lane);
      w1 += a1 - a0;
    }
  }
  w0_out = w0;
  w1_out = w1;
}

}  // namespace msd
