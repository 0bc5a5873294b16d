// gfx950 kernels for the world map and cell geometry:
//   * diffusion: LDS-tiled 3x3 stencil per molecule plane with an optional fused pre-scale (a
//     pending degrade_molecules), per-tile double partial sums of the mass before and after, a
//     per-molecule reduction and a correction + clamp pass writing back in place (reference
//     world.py:627-649 semantics);
//   * permeation and map degradation (world.py:651-678);
//   * placement: random free-pixel claims (spawn / add / reposition) and neighbour candidate picks
//     for division / movement (conflicts resolved by list priority on the host side);
//   * neighbour pairs via a pixel -> cell index map (O(n) instead of the reference's O(n^2)).
//
// Geometry: a map is R x C pixels per molecule plane. Cells live in rows [r_lo, r_hi). A
// single-GPU world is R = C = map_size, r_lo = 0, r_hi = R with the x axis wrapping. A strip of a
// domain-decomposed world (magicsoup_amd.parallel) has one halo row above and below its owned rows
// (R = H + 2, r_lo = 1, r_hi = H + 1, no x wrap: the halo rows hold the neighbours' boundary rows).
// The y axis always wraps (columns are never split).
#include "hip_common.h"

namespace msd {

struct Geom {
  int R, C, r_lo, r_hi, wrap;
  __device__ __forceinline__ int xup(int x) const { return (wrap && x == 0) ? R - 1 : x - 1; }
  __device__ __forceinline__ int xdn(int x) const { return (wrap && x == R - 1) ? 0 : x + 1; }
  __device__ __forceinline__ int yl(int y) const { return y == 0 ? C - 1 : y - 1; }
  __device__ __forceinline__ int yr(int y) const { return y == C - 1 ? 0 : y + 1; }
};

constexpr int kTW = 64;   // tile width  (y, contiguous)
constexpr int kTH = 32;   // tile height (x)
constexpr int kRows = 4;  // thread rows per block (block = kTW x kRows = 256 threads)

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// grid: (ceil(C/kTW), ceil(H/kTH), m) over the owned rows; out = b*x + a*sum(neighbours) on
// pre-scaled inputs, written to the same pixel of `out`.
__global__ void __launch_bounds__(kTW* kRows) diffuse_stencil_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                                     const float* __restrict__ wa, const float* __restrict__ wb,
                                                                     const float* __restrict__ scale, Geom g,
                                                                     double* __restrict__ partials) {
  __shared__ float tile[kTH + 2][kTW + 2 + 1];
  __shared__ double red[2][kRows * kTW / 64];
  const int mol = blockIdx.z;
  const int H = g.r_hi - g.r_lo;
  const int y0 = blockIdx.x * kTW, o0 = blockIdx.y * kTH;  // o = owned-row offset
  const size_t plane = (size_t)g.R * g.C;
  const float* src = in + (size_t)mol * plane;
  const float sc = scale ? scale[mol] : 1.0f;
  const int tid = threadIdx.y * kTW + threadIdx.x;

  for (int i = tid; i < (kTH + 2) * (kTW + 2); i += kTW * kRows) {
    const int r = i / (kTW + 2), cc = i - r * (kTW + 2);
    const int o = o0 + r - 1;   // -1 .. kTH (owned-row offset)
    const int yy = y0 + cc - 1;  // -1 .. kTW
    float v = 0.0f;
    if (o <= H && yy <= g.C) {
      int x = g.r_lo + o;  // r_lo - 1 .. r_hi
      if (x < 0) x += g.R;  // only with wrap (r_lo = 0)
      if (x >= g.R) x -= g.R;
      const int y = yy < 0 ? yy + g.C : (yy >= g.C ? yy - g.C : yy);
      v = src[(size_t)x * g.C + y] * sc;
    }
    tile[r][cc] = v;
  }
  __syncthreads();

  const float a = wa[mol], b = wb[mol];
  double before = 0.0, after = 0.0;
  const int ty = threadIdx.x, gy = y0 + ty;
  float* dst = out + (size_t)mol * plane;
  if (gy < g.C) {
    for (int r = threadIdx.y; r < kTH; r += kRows) {
      const int o = o0 + r;
      if (o >= H) break;
      const int lr = r + 1, lc = ty + 1;
      const float c0 = tile[lr][lc];
      const float ns = tile[lr - 1][lc - 1] + tile[lr - 1][lc] + tile[lr - 1][lc + 1] + tile[lr][lc - 1] +
                       tile[lr][lc + 1] + tile[lr + 1][lc - 1] + tile[lr + 1][lc] + tile[lr + 1][lc + 1];
      const float v = b * c0 + a * ns;
      dst[(size_t)(g.r_lo + o) * g.C + gy] = v;
      before += c0;
      after += v;
    }
  }
  before = wave_sum(before);
  after = wave_sum(after);
  const int wid = tid >> 6;
  if ((tid & 63) == 0) {
    red[0][wid] = before;
    red[1][wid] = after;
  }
  __syncthreads();
  if (tid == 0) {
    double sb = 0.0, sa = 0.0;
    for (int w = 0; w < kRows * kTW / 64; ++w) {
      sb += red[0][w];
      sa += red[1][w];
    }
    const size_t tiles = (size_t)gridDim.x * gridDim.y;
    const size_t t = (size_t)blockIdx.y * gridDim.x + blockIdx.x;
    partials[((size_t)mol * tiles + t) * 2] = sb;
    partials[((size_t)mol * tiles + t) * 2 + 1] = sa;
  }
}

// one block per molecule: totals[mol] = (sum before, sum after) of this map's owned rows
__global__ void __launch_bounds__(256) diffuse_reduce_kernel(const double* partials, int tiles, double* totals) {
  __shared__ double sb[4], sa[4];
  const int mol = blockIdx.x;
  double b = 0.0, a = 0.0;
  for (int t = threadIdx.x; t < tiles; t += blockDim.x) {
    b += partials[((size_t)mol * tiles + t) * 2];
    a += partials[((size_t)mol * tiles + t) * 2 + 1];
  }
  b = wave_sum(b);
  a = wave_sum(a);
  if ((threadIdx.x & 63) == 0) {
    sb[threadIdx.x >> 6] = b;
    sa[threadIdx.x >> 6] = a;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    totals[2 * mol] = sb[0] + sb[1] + sb[2] + sb[3];
    totals[2 * mol + 1] = sa[0] + sa[1] + sa[2] + sa[3];
  }
}

// map[owned rows] = max(tmp + (before - after) / n_pix, 0); each plane's owned rows are one
// contiguous range of `span` floats starting at r_lo * C. float4-vectorised when aligned.
__global__ void __launch_bounds__(256) diffuse_correct_kernel(const float* __restrict__ tmp, float* __restrict__ map,
                                                              const double* __restrict__ totals, double n_pix,
                                                              long long plane, long long start, long long span, int m) {
  const long long total = span * m;
  const bool vec = (start % 4 == 0) && (span % 4 == 0) && (plane % 4 == 0);
  if (vec) {
    const long long s4 = span / 4;
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < s4 * m; i += (long long)gridDim.x * blockDim.x) {
      const int mol = (int)(i / s4);
      const float c = (float)((totals[2 * mol] - totals[2 * mol + 1]) / n_pix);
      const long long o = (long long)mol * plane + start + (i - (long long)mol * s4) * 4;
      float4 v = *reinterpret_cast<const float4*>(tmp + o);
      v.x = fmaxf(v.x + c, 0.0f);
      v.y = fmaxf(v.y + c, 0.0f);
      v.z = fmaxf(v.z + c, 0.0f);
      v.w = fmaxf(v.w + c, 0.0f);
      *reinterpret_cast<float4*>(map + o) = v;
    }
  } else {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
      const int mol = (int)(i / span);
      const float c = (float)((totals[2 * mol] - totals[2 * mol + 1]) / n_pix);
      const long long o = (long long)mol * plane + start + (i - (long long)mol * span);
      map[o] = fmaxf(tmp[o] + c, 0.0f);
    }
  }
}

// map *= f[mol] (standalone degradation of the map)
__global__ void __launch_bounds__(256) scale_planes_kernel(float* map, const float* f, long long plane, int m) {
  const long long total = plane * m;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x)
    map[i] *= f[i / plane];
}

// Division bookkeeping after the rows were cloned (reference world.py:446-473): parent and child
// share the parent's molecules half-half, both get divisions + 1 and lifetime 0. One thread per
// (pair, molecule); molecule 0 threads also do the scalar fields.
__global__ void __launch_bounds__(256) split_cells_kernel(int k, int m, const int64_t* parents, const int64_t* children,
                                                          float* cell_mols, int32_t* divisions, int32_t* lifetimes) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)k * m) return;
  const int i = (int)(t / m), j = (int)(t - (long long)i * m);
  const long long p = parents[i], c = children[i];
  const float h = cell_mols[p * m + j] * 0.5f;
  cell_mols[p * m + j] = h;
  cell_mols[c * m + j] = h;
  if (j == 0) {
    const int32_t d = divisions[p] + 1;
    divisions[p] = d;
    divisions[c] = d;
    lifetimes[p] = 0;
    lifetimes[c] = 0;
  }
}

// Killed cells spill their molecules onto their pixel and free it (reference world.py:520-530);
// new cells take half of their pixel's molecules (world.py:326-331). One thread per
// (cell, molecule); pixels are distinct, so no atomics.
__global__ void __launch_bounds__(256) spill_free_kernel(int k, int m, const int64_t* idxs, const int32_t* pos, int C,
                                                         long long plane, const float* cell_mols, float* map,
                                                         uint8_t* cell_map) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)k * m) return;
  const int i = (int)(t / m), j = (int)(t - (long long)i * m);
  const long long c = idxs[i];
  const long long pix = (long long)pos[2 * c] * C + pos[2 * c + 1];
  map[j * plane + pix] += cell_mols[c * m + j];
  if (j == 0) cell_map[pix] = 0;
}

__global__ void __launch_bounds__(256) spill_free_mask_kernel(int n, int m, const uint8_t* dead, const int32_t* pos,
                                                              int C, long long plane, const float* cell_mols,
                                                              float* map, uint8_t* cell_map) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)n * m) return;
  const int c = (int)(t / m), j = (int)(t - (long long)c * m);
  if (!dead[c]) return;
  const long long pix = (long long)pos[2 * c] * C + pos[2 * c + 1];
  map[j * plane + pix] += cell_mols[(long long)c * m + j];
  if (j == 0) cell_map[pix] = 0;
}

__global__ void __launch_bounds__(256) pickup_kernel(int k, int m, const int64_t* idxs, const int32_t* pos, int C,
                                                     long long plane, float* cell_mols, float* map) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)k * m) return;
  const int i = (int)(t / m), j = (int)(t - (long long)i * m);
  const long long c = idxs[i];
  const long long pix = (long long)pos[2 * c] * C + pos[2 * c + 1];
  const float half = map[j * plane + pix] * 0.5f;
  cell_mols[c * m + j] += half;
  map[j * plane + pix] -= half;
}

// exchange between cells and their pixels, one thread per (cell, molecule)
__global__ void __launch_bounds__(256) permeate_kernel(int c, int m, Geom g, const int32_t* pos, const float* perm,
                                                       float* cell_mols, float* map) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)c * m) return;
  const int cell = (int)(t / m), i = (int)(t - (long long)cell * m);
  const float p = perm[i];
  if (p == 0.0f) return;
  const size_t o = (size_t)i * g.R * g.C + (size_t)pos[2 * cell] * g.C + pos[2 * cell + 1];
  const float xi = cell_mols[t], xe = map[o];
  const float di = xi * p, de = xe * p;
  cell_mols[t] = xi + (de - di);
  map[o] = xe + (di - de);
}

// ---------------------------------------------------------------- placement
// Claim k uniformly random free pixels of the owned rows by rejection: atomically set the pixel's
// byte in the (4-byte padded) bool occupancy map; out[i] = pixel or -1 after `attempts` misses.
__global__ void __launch_bounds__(256) claim_free_kernel(int k, Geom g, uint8_t* cell_map, uint64_t seed, uint64_t call,
                                                         int attempts, long long* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= k) return;
  Philox rng(seed, call, (uint32_t)i);
  const long long base = (long long)g.r_lo * g.C, n_pix = (long long)(g.r_hi - g.r_lo) * g.C;
  long long got = -1;
  for (int t = 0; t < attempts; ++t) {
    const long long pix = base + (long long)rng.below64((uint64_t)n_pix);
    if (cell_map[pix]) continue;
    unsigned* word = reinterpret_cast<unsigned*>(cell_map + (pix & ~3ll));
    const unsigned bit = 1u << (8 * (pix & 3));
    const unsigned old = atomicOr(word, bit);
    if (!(old & (0xFFu << (8 * (pix & 3))))) {
      got = pix;
      break;
    }
  }
  out[i] = got;
}

// Moore neighbours in the reference order (w,n),(w,y),(w,s),(x,n),(x,s),(e,n),(e,y),(e,s) as
// pixel indices; duplicates (tiny maps) removed. Returns the count.
__device__ __forceinline__ int moore(int x, int y, const Geom& g, long long* nb) {
  const int w = g.xup(x), e = g.xdn(x), n = g.yl(y), s = g.yr(y);
  const int xs[8] = {w, w, w, x, x, e, e, e}, ys[8] = {n, y, s, n, s, n, y, s};
  int cnt = 0;
  for (int k = 0; k < 8; ++k) {
    const long long p = (long long)xs[k] * g.C + ys[k];
    bool dup = false;
    for (int q = 0; q < cnt; ++q) dup |= nb[q] == p;
    if (!dup) nb[cnt++] = p;
  }
  return cnt;
}

// For each pending cell pick a uniformly random free Moore neighbour (cand = pixel) or report
// that none is free (cand = -1). Halo-row pixels are candidates too (the caller arbitrates them
// with the owning rank).
__global__ void __launch_bounds__(256) pick_neighbour_kernel(int k, const int64_t* cells, const int32_t* pos, Geom g,
                                                             const uint8_t* cell_map, const uint8_t* pending,
                                                             uint64_t seed, uint64_t call, long long* cand) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= k) return;
  if (!pending[i]) {
    cand[i] = -1;
    return;
  }
  const int c = (int)cells[i];
  long long nb[8], fr[8];
  const int cnt = moore(pos[2 * c], pos[2 * c + 1], g, nb);
  int nf = 0;
  for (int q = 0; q < cnt; ++q)
    if (!cell_map[nb[q]]) fr[nf++] = nb[q];
  if (nf == 0) {
    cand[i] = -1;
    return;
  }
  Philox rng(seed, call, (uint32_t)i);
  cand[i] = fr[rng.below((uint32_t)nf)];
}

// Device-resolved placement rounds (divide / move): in a round every pending cell bids for a
// random free Moore neighbour with atomicMin(claim[pixel], list position); the lowest list position
// wins each pixel (the reference places cells in list order, rust/world.rs:59-146), losers retry
// next round against the updated occupancy. `claim` is an int32 per pixel kept at INT_MAX between
// rounds: the winner resets its pixel (a loser reading the reset value still sees "not mine").
// Cells without any free neighbour drop out. No host synchronisation between rounds.
constexpr int kNoClaim = 0x7FFFFFFF;

__global__ void __launch_bounds__(256) place_bid_kernel(int k, const int64_t* cells, const int32_t* pos, Geom g,
                                                        const uint8_t* cell_map, uint8_t* pending, uint64_t seed,
                                                        uint64_t call, long long* cand, int* claim) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= k || !pending[i]) return;
  const int c = (int)cells[i];
  long long nb[8], fr[8];
  const int cnt = moore(pos[2 * c], pos[2 * c + 1], g, nb);
  int nf = 0;
  for (int q = 0; q < cnt; ++q)
    if (!cell_map[nb[q]]) fr[nf++] = nb[q];
  if (nf == 0) {
    pending[i] = 0;
    cand[i] = -1;
    return;
  }
  Philox rng(seed, call, (uint32_t)i);
  const long long px = fr[rng.below((uint32_t)nf)];
  cand[i] = px;
  atomicMin(claim + px, i);
}

__global__ void __launch_bounds__(256) place_resolve_kernel(int k, const int64_t* cells, const int32_t* pos, Geom g,
                                                            bool vacate, uint8_t* cell_map, uint8_t* pending,
                                                            const long long* cand, int* claim, long long* result) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= k || !pending[i]) return;
  const long long px = cand[i];
  if (px < 0 || claim[px] != i) return;
  claim[px] = kNoClaim;
  cell_map[px] = 1;
  result[i] = px;
  pending[i] = 0;
  // a move into a halo row is committed only after the owning rank accepts it: keep the pixel
  const int x = (int)(px / g.C);
  if (vacate && (g.wrap || (x >= g.r_lo && x < g.r_hi))) {
    const int c = (int)cells[i];
    cell_map[(size_t)pos[2 * c] * g.C + pos[2 * c + 1]] = 0;
  }
}

// ---------------------------------------------------------------- neighbours
__global__ void __launch_bounds__(256) index_map_kernel(int c, const int32_t* pos, int C, int32_t* idx_map, bool clear) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= c) return;
  idx_map[(size_t)pos[2 * i] * C + pos[2 * i + 1]] = clear ? -1 : i;
}

__global__ void __launch_bounds__(256) neighbor_pairs_kernel(int nf, const int64_t* from, const int32_t* pos, Geom g,
                                                             const int32_t* idx_map, const uint8_t* in_from,
                                                             const uint8_t* in_to, int* counter, int cap,
                                                             int64_t* pairs) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nf) return;
  const int c = (int)from[i];
  long long nb[8];
  const int cnt = moore(pos[2 * c], pos[2 * c + 1], g, nb);
  for (int q = 0; q < cnt; ++q) {
    const int o = idx_map[nb[q]];
    if (o < 0 || o == c || !in_to[o]) continue;
    if (in_from[o] && in_to[c] && o < c) continue;  // found from the other side
    const int slot = atomicAdd(counter, 1);
    if (slot < cap) pairs[slot] = c < o ? ((int64_t)c << 32) | o : ((int64_t)o << 32) | c;
  }
}

// All neighbour pairs of all cells in fixed slots: slot c*8 + q holds (c << 32) | o for the q-th
// Moore neighbour o > c of cell c, else -1. Deterministic order (cell-major, reference neighbour
// order), no atomics, no counter read-back.
__global__ void __launch_bounds__(256) neighbor_slots_kernel(int n, const int32_t* pos, Geom g, const int32_t* idx_map,
                                                             int64_t* keys) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  long long nb[8];
  const int cnt = moore(pos[2 * c], pos[2 * c + 1], g, nb);
  for (int q = 0; q < 8; ++q) {
    int64_t key = -1;
    if (q < cnt) {
      const int o = idx_map[nb[q]];
      if (o > c) key = ((int64_t)c << 32) | o;
    }
    keys[(size_t)c * 8 + q] = key;
  }
}

// ---------------------------------------------------------------- host launchers
static Geom geom(int R, int C, int r_lo, int r_hi, int wrap) {
  if (R <= 0 || C <= 0 || r_lo < 0 || r_hi > R || r_lo >= r_hi) throw std::invalid_argument("bad map geometry");
  if (!wrap && (r_lo < 1 || r_hi > R - 1)) throw std::invalid_argument("a non-wrapping strip needs halo rows");
  return Geom{R, C, r_lo, r_hi, wrap};
}

// Stencil + per-molecule (before, after) totals of the owned rows. The caller (optionally after
// an all-reduce of `totals` over ranks) runs diffuse_correct.
void diffuse_stencil(int m, int R, int C, int r_lo, int r_hi, int wrap, uintptr_t map, uintptr_t tmp, uintptr_t wa,
                     uintptr_t wb, uintptr_t scale, uintptr_t partials, uintptr_t totals, uintptr_t stream) {
  if (m <= 0) return;
  const Geom g = geom(R, C, r_lo, r_hi, wrap);
  hipStream_t st = S_(stream);
  const dim3 grid(cdiv(C, kTW), cdiv(r_hi - r_lo, kTH), m), block(kTW, kRows);
  diffuse_stencil_kernel<<<grid, block, 0, st>>>(P_<float>(map), P_<float>(tmp), P_<float>(wa), P_<float>(wb),
                                                 scale ? P_<float>(scale) : nullptr, g, P_<double>(partials));
  MS_LAUNCH_CHECK();
  diffuse_reduce_kernel<<<m, 256, 0, st>>>(P_<double>(partials), (int)(grid.x * grid.y), P_<double>(totals));
  MS_LAUNCH_CHECK();
}

void diffuse_correct(int m, int R, int C, int r_lo, int r_hi, uintptr_t map, uintptr_t tmp, uintptr_t totals,
                     double n_pix, uintptr_t stream) {
  if (m <= 0) return;
  const long long plane = (long long)R * C, start = (long long)r_lo * C, span = (long long)(r_hi - r_lo) * C;
  const unsigned g = std::min<long long>(cdiv(span * m / 4 + 1, 256), 4096);
  diffuse_correct_kernel<<<g, 256, 0, S_(stream)>>>(P_<float>(tmp), P_<float>(map), P_<double>(totals), n_pix, plane,
                                                    start, span, m);
  MS_LAUNCH_CHECK();
}

size_t diffuse_partials_len(int m, int C, int H) { return (size_t)cdiv(C, kTW) * cdiv(H, kTH) * m * 2; }

void scale_planes(int m, long long plane, uintptr_t map, uintptr_t f, uintptr_t stream) {
  if (m <= 0 || plane <= 0) return;
  const unsigned g = std::min<long long>(cdiv(plane * m, 256), 4096);
  scale_planes_kernel<<<g, 256, 0, S_(stream)>>>(P_<float>(map), P_<float>(f), plane, m);
  MS_LAUNCH_CHECK();
}

void spill_free(int k, int m, uintptr_t idxs, uintptr_t pos, int R, int C, uintptr_t cell_mols, uintptr_t map,
                uintptr_t cell_map, uintptr_t stream) {
  if (k <= 0 || m <= 0) return;
  spill_free_kernel<<<cdiv((long long)k * m, 256), 256, 0, S_(stream)>>>(
      k, m, P_<int64_t>(idxs), P_<int32_t>(pos), C, (long long)R * C, P_<float>(cell_mols), P_<float>(map),
      P_<uint8_t>(cell_map));
  MS_LAUNCH_CHECK();
}

void spill_free_mask(int n, int m, uintptr_t dead, uintptr_t pos, int R, int C, uintptr_t cell_mols, uintptr_t map,
                     uintptr_t cell_map, uintptr_t stream) {
  if (n <= 0 || m <= 0) return;
  spill_free_mask_kernel<<<cdiv((long long)n * m, 256), 256, 0, S_(stream)>>>(
      n, m, P_<uint8_t>(dead), P_<int32_t>(pos), C, (long long)R * C, P_<float>(cell_mols), P_<float>(map),
      P_<uint8_t>(cell_map));
  MS_LAUNCH_CHECK();
}

void pickup(int k, int m, uintptr_t idxs, uintptr_t pos, int R, int C, uintptr_t cell_mols, uintptr_t map,
            uintptr_t stream) {
  if (k <= 0 || m <= 0) return;
  pickup_kernel<<<cdiv((long long)k * m, 256), 256, 0, S_(stream)>>>(k, m, P_<int64_t>(idxs), P_<int32_t>(pos), C,
                                                                     (long long)R * C, P_<float>(cell_mols),
                                                                     P_<float>(map));
  MS_LAUNCH_CHECK();
}

void split_cells(int k, int m, uintptr_t parents, uintptr_t children, uintptr_t cell_mols, uintptr_t divisions,
                 uintptr_t lifetimes, uintptr_t stream) {
  if (k <= 0 || m <= 0) return;
  split_cells_kernel<<<cdiv((long long)k * m, 256), 256, 0, S_(stream)>>>(
      k, m, P_<int64_t>(parents), P_<int64_t>(children), P_<float>(cell_mols), P_<int32_t>(divisions),
      P_<int32_t>(lifetimes));
  MS_LAUNCH_CHECK();
}

void permeate(int c, int m, int R, int C, uintptr_t pos, uintptr_t perm, uintptr_t cell_mols, uintptr_t map,
              uintptr_t stream) {
  if (c <= 0 || m <= 0) return;
  const Geom g{R, C, 0, R, 1};
  permeate_kernel<<<cdiv((long long)c * m, 256), 256, 0, S_(stream)>>>(c, m, g, P_<int32_t>(pos), P_<float>(perm),
                                                                       P_<float>(cell_mols), P_<float>(map));
  MS_LAUNCH_CHECK();
}

void claim_free(int k, int R, int C, int r_lo, int r_hi, uintptr_t cell_map, uint64_t seed, uint64_t call,
                int attempts, uintptr_t out, uintptr_t stream) {
  if (k <= 0) return;
  const Geom g = geom(R, C, r_lo, r_hi, 1);
  claim_free_kernel<<<cdiv(k, 256), 256, 0, S_(stream)>>>(k, g, P_<uint8_t>(cell_map), seed, call, attempts,
                                                           P_<long long>(out));
  MS_LAUNCH_CHECK();
}

void pick_neighbour(int k, uintptr_t cells, uintptr_t pos, int R, int C, int r_lo, int r_hi, int wrap,
                    uintptr_t cell_map, uintptr_t pending, uint64_t seed, uint64_t call, uintptr_t cand,
                    uintptr_t stream) {
  if (k <= 0) return;
  const Geom g = geom(R, C, r_lo, r_hi, wrap);
  pick_neighbour_kernel<<<cdiv(k, 256), 256, 0, S_(stream)>>>(k, P_<int64_t>(cells), P_<int32_t>(pos), g,
                                                               P_<uint8_t>(cell_map), P_<uint8_t>(pending), seed, call,
                                                               P_<long long>(cand));
  MS_LAUNCH_CHECK();
}

void place_rounds(int k, uintptr_t cells, uintptr_t pos, int R, int C, int r_lo, int r_hi, int wrap, bool vacate,
                  uintptr_t cell_map, uintptr_t pending, uintptr_t cand, uintptr_t claim, uintptr_t result, int rounds,
                  uint64_t seed, uint64_t call, uintptr_t stream) {
  if (k <= 0) return;
  const Geom g = geom(R, C, r_lo, r_hi, wrap);
  const unsigned grid = cdiv(k, 256);
  for (int r = 0; r < rounds; ++r) {
    place_bid_kernel<<<grid, 256, 0, S_(stream)>>>(k, P_<int64_t>(cells), P_<int32_t>(pos), g, P_<uint8_t>(cell_map),
                                                   P_<uint8_t>(pending), seed, call + ((uint64_t)r << 48), P_<long long>(cand),
                                                   P_<int>(claim));
    MS_LAUNCH_CHECK();
    place_resolve_kernel<<<grid, 256, 0, S_(stream)>>>(k, P_<int64_t>(cells), P_<int32_t>(pos), g, vacate,
                                                       P_<uint8_t>(cell_map), P_<uint8_t>(pending),
                                                       P_<long long>(cand), P_<int>(claim), P_<long long>(result));
    MS_LAUNCH_CHECK();
  }
}

void index_map(int c, uintptr_t pos, int C, uintptr_t idx_map, bool clear, uintptr_t stream) {
  if (c <= 0) return;
  index_map_kernel<<<cdiv(c, 256), 256, 0, S_(stream)>>>(c, P_<int32_t>(pos), C, P_<int32_t>(idx_map), clear);
  MS_LAUNCH_CHECK();
}

void neighbor_slots(int n, uintptr_t pos, int R, int C, int r_lo, int r_hi, int wrap, uintptr_t idx_map, uintptr_t keys,
                    uintptr_t stream) {
  if (n <= 0) return;
  const Geom g = geom(R, C, r_lo, r_hi, wrap);
  neighbor_slots_kernel<<<cdiv(n, 256), 256, 0, S_(stream)>>>(n, P_<int32_t>(pos), g, P_<int32_t>(idx_map),
                                                               P_<int64_t>(keys));
  MS_LAUNCH_CHECK();
}

void neighbor_pairs(int nf, uintptr_t from, uintptr_t pos, int R, int C, int r_lo, int r_hi, int wrap, uintptr_t idx_map,
                    uintptr_t in_from, uintptr_t in_to, uintptr_t counter, int cap, uintptr_t pairs, uintptr_t stream) {
  if (nf <= 0) return;
  const Geom g = geom(R, C, r_lo, r_hi, wrap);
  neighbor_pairs_kernel<<<cdiv(nf, 256), 256, 0, S_(stream)>>>(nf, P_<int64_t>(from), P_<int32_t>(pos), g,
                                                               P_<int32_t>(idx_map), P_<uint8_t>(in_from),
                                                               P_<uint8_t>(in_to), P_<int>(counter), cap,
                                                               P_<int64_t>(pairs));
  MS_LAUNCH_CHECK();
}

}  // namespace msd
