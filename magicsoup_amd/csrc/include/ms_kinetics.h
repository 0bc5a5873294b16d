// Single-source kinetics math shared by the OpenMP host path and the HIP kernels.
//
// Reference semantics: python/magicsoup/kinetics.py:521-625 (parameter build) and :725-918
// (integrator); the constants match kinetics.py:9-13. The integrator's global early exit
// (kinetics.py:846, `torch.any` over ALL cells) is reproduced exactly without per-iteration grid
// synchronisation: each cell computes its full 4-iteration trajectory, records which iterations
// still had an impactful correction (a 4-bit mask OR-reduced over all cells), and keeps the five
// candidate states; the reduced mask then selects, for every cell, the state at which the reference
// loop would have returned.
#pragma once
#include <math.h>
#include <stdint.h>

#include "ms_common.h"

namespace ms {

constexpr float kEps = 1e-36f;
constexpr float kMax = 1e36f;
constexpr float kMin = -1e36f;
constexpr int kEqIters = 4;
constexpr int kSnap = kEqIters + 1;
constexpr float kUpper = 1.5f;
constexpr float kLower = (float)(1.0 / 1.5);

MS_HD bool f_isnan(float x) { return x != x; }
MS_HD bool f_isinf(float x) { return x == INFINITY || x == -INFINITY; }

// x^n for small integer n (n < 0 -> 1 / x^|n|), matching powf on the values the simulator produces.
MS_HD float ipow(float x, int n) {
  int e = n < 0 ? -n : n;
  float r = 1.0f, b = x;
  while (e) {
    if (e & 1) r *= b;
    b *= b;
    e >>= 1;
  }
  return n < 0 ? 1.0f / r : r;
}

// reference _multiply_signals post-processing: NaN -> 0, negative -> 0, Inf -> MAX
MS_HD float clean_prod(float xx) {
  if (f_isnan(xx) || xx < 0.0f) return 0.0f;
  if (f_isinf(xx)) return kMax;
  return xx;
}

// Mean over the finite-flagged entries; NaN (-> 0 after nan_to_num) if none.
struct NanMean {
  float sum = 0.0f;
  int n = 0;
  MS_HD void add(float v) {
    if (!f_isnan(v)) {
      sum += v;
      ++n;
    }
  }
  MS_HD float value0() const { return n > 0 ? sum / (float)n : 0.0f; }
};

}  // namespace ms
