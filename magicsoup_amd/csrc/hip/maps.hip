// gfx950 molecule-map physics: diffusion stencil + mass correction, degradation, permeation and the
// cell <-> pixel exchanges of spawn / kill (reference world.py:326-331, 520-530, 627-678).
//
// The map may be stored as fp32 (default), bf16 or fp16 (opt-in, BASELINE's large-map configs);
// every kernel computes in fp32 and the diffusion mass totals in fp64.
//
// Diffusion stencil: one wavefront owns 64 columns and a band of rows and slides down the band
// with the 3x3 window in registers -- every map value is loaded once per band (plus one halo row
// above and below), left/right neighbours come from lane shuffles, only the two edge lanes load
// their outer column. No LDS, no workgroup barriers; the per-wave before/after sums are reduced
// per block into fp64 partials.
#include "hip_common.h"
#include "map_types.h"

namespace msd {

struct MGeom {
  int R, C, r_lo, r_hi, wrap;
};

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// ---------------------------------------------------------------- diffusion
constexpr int kBand = 32;  // rows per wavefront band
constexpr int kWaves = 4;  // wavefronts per block (adjacent 64-column strips)

// grid: (ceil(C / (64 kWaves)), ceil(H / kBand), m). out = b*x + a*sum(8 neighbours) of the
// pre-scaled input over the owned rows of the band; fp64 before/after partial sums per block.
template <class T>
__global__ void __launch_bounds__(64 * kWaves) diffuse_stencil_kernel(const T* __restrict__ in, T* __restrict__ out,
                                                                      const float* __restrict__ wa,
                                                                      const float* __restrict__ wb,
                                                                      const float* __restrict__ scale,
                                                                      const float* __restrict__ corr, MGeom g,
                                                                      double* __restrict__ partials) {
  __shared__ double red[2][kWaves];
  const int mol = blockIdx.z;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int H = g.r_hi - g.r_lo;
  const int y = (blockIdx.x * kWaves + wv) * 64 + lane;
  const bool col = y < g.C;
  const int yl = y == 0 ? g.C - 1 : y - 1, yr = y + 1 >= g.C ? y + 1 - g.C : y + 1;
  // a neighbour comes from the adjacent lane unless it is outside this wave's valid columns
  const bool own_l = lane > 0 && y - 1 >= 0, own_r = lane < 63 && y + 1 < g.C;
  const size_t plane = (size_t)g.R * g.C;
  const T* src = in + (size_t)mol * plane;
  T* dst = out + (size_t)mol * plane;
  const float sc = scale ? scale[mol] : 1.0f;
  const float a = wa[mol], b = wb[mol];
  const int o0 = blockIdx.y * kBand, o1 = min(H, o0 + kBand);

  auto row_of = [&](int o) {  // owned-row offset -> map row (halo / wrap)
    int x = g.r_lo + o;
    if (x < 0) x += g.R;
    if (x >= g.R) x -= g.R;
    return x;
  };
  // v: centre, l/r: horizontal neighbours, h = l + v + r, for rows o-1 (p), o (c), o+1 (n)
  auto load = [&](int o, float& v, float& l, float& r) {
    const size_t base = (size_t)row_of(o) * g.C;
    v = col ? corr_in(ld(src + base + y), corr, mol) * sc : 0.0f;
    const float vl = __shfl_up(v, 1), vr = __shfl_down(v, 1);
    l = own_l ? vl : (col ? corr_in(ld(src + base + yl), corr, mol) * sc : 0.0f);
    r = own_r ? vr : (col ? corr_in(ld(src + base + yr), corr, mol) * sc : 0.0f);
  };
  float vp, lp, rp, vc, lc, rc;
  load(o0 - 1, vp, lp, rp);
  load(o0, vc, lc, rc);
  float hp = lp + vp + rp, hc = lc + vc + rc;
  double before = 0.0, after = 0.0;
  for (int o = o0; o < o1; ++o) {
    float vn, ln, rn;
    load(o + 1, vn, ln, rn);
    const float hn = ln + vn + rn;
    const float ns = hp + hn + lc + rc;
    const float v = b * vc + a * ns;
    if (col) {
      st(dst + (size_t)row_of(o) * g.C + y, v);
      before += vc;
      after += v;
    }
    hp = hc;
    vc = vn;
    lc = ln;
    rc = rn;
    hc = hn;
  }
  before = wave_sum_d(before);
  after = wave_sum_d(after);
  if (lane == 0) {
    red[0][wv] = before;
    red[1][wv] = after;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double sb = 0.0, sa = 0.0;
    for (int w = 0; w < kWaves; ++w) {
      sb += red[0][w];
      sa += red[1][w];
    }
    const size_t tiles = (size_t)gridDim.x * gridDim.y;
    const size_t t = (size_t)blockIdx.y * gridDim.x + blockIdx.x;
    partials[((size_t)mol * tiles + t) * 2] = sb;
    partials[((size_t)mol * tiles + t) * 2 + 1] = sa;
  }
}

// Vector variant for C % 4 == 0 (every practical map): a lane owns 4 adjacent columns (one
// 16 B / 8 B access per row), a wave 256 columns; the 4 waves of a block take 4 consecutive bands
// of the same column strip. While row o is computed, the load of row o + 2 is in flight (row o + 1
// arrived in the previous iteration): one row load per wave ahead. A variant with two row loads in
// flight was measured and not kept (docs/performance.md, "Diffusion").
// Tiles: (ceil(C / 256), ceil(ceil(H / kBand) / 4), m), x fastest; a 1-D grid of `gridDim.x`
// blocks walks them in steps of the grid (one tile per block when the grid is the tile count). A
// smaller grid leaves workgroup slots free on every CU, so the side stream's short pipeline kernels
// (deferred genome chains, World._flush_deferred) start at once instead of waiting for stencil
// workgroups to retire (set_stencil_blocks).
constexpr int kVBand = 64;     // rows per wave band of the vector stencils (default)
constexpr int kMinVBand = 16;  // the narrowest band set_stencil_band accepts
// rows per wave band (set_stencil_band; 0 = the default 64): a band re-reads one halo row above and
// below it, so taller bands read less but leave fewer tiles per block of the grid-stride launch.
// With the branch-free ring (band_loop) 64 rows win at every map type: 4096^2 x 14, diffuse step
// fp32 0.391 (32 rows, 1 row ahead, 1024 blocks) -> 0.357 ms (64 rows, 2 ahead, 768 blocks), bf16 /
// fp16 0.212 / 0.220 -> 0.196 / 0.199 ms (3 ahead) (profiles/r5/stencil_ring.txt).
static int g_vband = kVBand;
void set_stencil_band(int b) { g_vband = b <= 0 ? kVBand : (b < kMinVBand ? kMinVBand : (b > 256 ? 256 : b)); }
static int stencil_band(int, int, int, int, int) { return g_vband; }

// The rows of a wave's band: row_step(o, raw row o + 1) for o in [o0, o1); `first` holds raw row
// o0 + 1 on entry. PF = 0: one raw row ahead, fetched into `spare` under a branch and copied (the
// register copy waits for the loads at the end of the same row). PF >= 1: PF rows ahead in a ring of
// PF + 1 raw buffers, unrolled by the ring size so every buffer is a fixed register set: a row's
// loads are only waited for by the step that uses them, PF steps later. Rows past the band are
// clamped to o1 (the halo row below it, already the last row the PF = 0 loop loads). Whole turns of
// the ring run without a branch (and the fetches themselves are branch-free): the compiler's vmcnt
// waits only count exactly across straight-line code, so a guard per row made every step wait for
// all but the newest loads and the ring collapsed to one row in flight (scripts/lab/stencil_lab.hip:
// 4096^2 x 14 fp32, 360 -> 328-333 us at 3 rows ahead, 64-row bands, 512-768 blocks).
template <int PF, class Raw, class Fetch, class Step>
__device__ __forceinline__ void band_loop(int o0, int o1, Raw& first, Raw& spare, Fetch&& fetch, Step&& row_step) {
  if constexpr (PF == 0) {
    for (int o = o0; o < o1; ++o) {
      if (o + 2 <= o1) fetch(o + 2, spare);
      row_step(o, first);
      first = spare;
    }
  } else {
    constexpr int NB = PF + 1;
    Raw ring[NB];
    ring[0] = first;
#pragma unroll
    for (int d = 1; d < PF; ++d) fetch(min(o0 + 1 + d, o1), ring[d]);
    int o = o0;
    for (; o + NB <= o1; o += NB) {
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        fetch(min(o + u + 1 + PF, o1), ring[(u + PF) % NB]);
        row_step(o + u, ring[u]);
      }
    }
    if (o < o1) {  // the band's last partial turn
#pragma unroll
      for (int u = 0; u < NB; ++u) {
        if (o + u < o1) {
          fetch(min(o + u + 1 + PF, o1), ring[(u + PF) % NB]);
          row_step(o + u, ring[u]);
        }
      }
    }
  }
}
// FULL: every lane's columns exist (C a multiple of the wave's columns): no per-lane store branch
template <class T, int PF, bool FULL = false>
__global__ void __launch_bounds__(256) diffuse_stencil4_kernel(const T* __restrict__ in, T* __restrict__ out,
                                                               const float* __restrict__ wa,
                                                               const float* __restrict__ wb,
                                                               const float* __restrict__ scale,
                                                               const float* __restrict__ corr, MGeom g,
                                                               double* __restrict__ partials, int gx, int gy,
                                                               int ntiles, int vband) {
  __shared__ double red[2][4];
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
  const int bx = tile % gx, by = (tile / gx) % gy, mol = tile / (gx * gy);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int H = g.r_hi - g.r_lo;
  const int y0 = bx * 256 + lane * 4;
  const bool col = FULL || y0 < g.C;
  const bool need_l = lane == 0 && col, need_r = col && (lane == 63 || y0 + 4 >= g.C);
  const int yl = y0 == 0 ? g.C - 1 : y0 - 1, yr = y0 + 4 >= g.C ? 0 : y0 + 4;
  const size_t plane = (size_t)g.R * g.C;
  const T* src = in + (size_t)mol * plane;
  T* dst = out + (size_t)mol * plane;
  const float sc = scale ? scale[mol] : 1.0f;
  const float a = wa[mol], b = wb[mol];
  const int o0 = (by * 4 + wv) * vband, o1 = min(H, o0 + vband);

  auto row_of = [&](int o) {
    int x = g.r_lo + o;
    if (x < 0) x += g.R;
    if (x >= g.R) x -= g.R;
    return x;
  };
  struct Raw {  // raw bits: converted in finish(), so a prefetched row's loads stay in flight
    uint32_t v[4], el, er;
  };
  // branch-free (see band_loop): every lane loads -- a lane past the last column its strip's first
  // columns, zeroed after; the halo loads of the inner lanes their own first column (the same line)
  const int yc = col ? y0 : bx * 256;
  auto fetch = [&](int o, Raw& r) {
    const size_t base = (size_t)row_of(o) * g.C;
    if constexpr (sizeof(T) == 4) {
      const uint4 q = *reinterpret_cast<const uint4*>(src + base + yc);
      r.v[0] = q.x, r.v[1] = q.y, r.v[2] = q.z, r.v[3] = q.w;
    } else {
      const uint2 q = *reinterpret_cast<const uint2*>(src + base + yc);
      r.v[0] = q.x & 0xFFFFu, r.v[1] = q.x >> 16, r.v[2] = q.y & 0xFFFFu, r.v[3] = q.y >> 16;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) r.v[j] = col ? r.v[j] : 0u;
    if constexpr (FULL) {
      // every strip is whole: only lane 0 needs a left and only lane 63 a right edge value, so
      // one edge load per row serves both (a third fewer load instructions per row)
      r.el = ld_bits(src + base + (need_l ? yl : (need_r ? yr : yc)));
    } else {
      r.el = ld_bits(src + base + (need_l ? yl : yc));
      r.er = ld_bits(src + base + (need_r ? yr : yc));
    }
  };
  // scaled values of the row plus the left neighbour of column y0 and the right one of y0 + 3
  auto finish = [&](const Raw& r, float v[4], float& L, float& Rn) {
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = corr_in(from_bits<T>(r.v[j]), corr, mol) * sc;
    const float up = __shfl_up(v[3], 1), dn = __shfl_down(v[0], 1);
    // (both edge values computed by every lane and selected: no branch, see band_loop)
    const float el = corr_in(from_bits<T>(r.el), corr, mol) * sc;
    const float er = FULL ? el : corr_in(from_bits<T>(r.er), corr, mol) * sc;
    L = need_l ? el : up;
    Rn = need_r ? er : dn;
  };
  auto hsum = [](const float v[4], float L, float Rn, float h[4]) {
    h[0] = L + v[0] + v[1];
    h[1] = v[0] + v[1] + v[2];
    h[2] = v[1] + v[2] + v[3];
    h[3] = v[2] + v[3] + Rn;
  };

  // mass sums in fp64 per row: fp32 sums per band were tried (round 4) and rejected -- their
  // rounding scales with the largest concentrations of a species, and the correction spreads it
  // over every pixel, so a decomposed map no longer matched the single-process one to 1e-4
  // (tests/test_gpu_distributed.py); the two fp64 adds per row are not what bounds the kernel
  double before = 0.0, after = 0.0;
  if (o0 < H) {
    Raw rp, rc, rn, rn2;
    fetch(o0 - 1, rp);
    fetch(o0, rc);
    fetch(o0 + 1, rn);
    float vp[4], Lp, Rp, vc[4], Lc, Rc, hp[4], hc[4];
    finish(rp, vp, Lp, Rp);
    finish(rc, vc, Lc, Rc);
    hsum(vp, Lp, Rp, hp);
    hsum(vc, Lc, Rc, hc);
    // row o from rows o - 1, o (in registers) and the raw row o + 1 (see band_loop)
    auto row_step = [&](int o, const Raw& r_next) {
      float vn[4], Ln, Rn, hn[4];
      finish(r_next, vn, Ln, Rn);
      hsum(vn, Ln, Rn, hn);
      float res[4];
      const float lft[4] = {Lc, vc[0], vc[1], vc[2]}, rgt[4] = {vc[1], vc[2], vc[3], Rc};
#pragma unroll
      for (int j = 0; j < 4; ++j) res[j] = b * vc[j] + a * (hp[j] + hn[j] + lft[j] + rgt[j]);
      if (col) {
        st4_stream(dst + (size_t)row_of(o) * g.C + y0, res);
        before += (double)((vc[0] + vc[1]) + (vc[2] + vc[3]));
        after += (double)((res[0] + res[1]) + (res[2] + res[3]));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        hp[j] = hc[j];
        hc[j] = hn[j];
        vc[j] = vn[j];
      }
      Lc = Ln;
      Rc = Rn;
    };
    band_loop<PF>(o0, o1, rn, rn2, fetch, row_step);
  }
  before = wave_sum_d(before);
  after = wave_sum_d(after);
  if (lane == 0) {
    red[0][wv] = before;
    red[1][wv] = after;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const size_t tiles = (size_t)gx * gy;
    const size_t t = (size_t)by * gx + bx;
    partials[((size_t)mol * tiles + t) * 2] = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
    partials[((size_t)mol * tiles + t) * 2 + 1] = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
  }
  __syncthreads();  // red is refilled by the next tile
  }
}

// Eight columns per lane (C % 8 == 0): a wave covers 512 columns with 16 B accesses only (fp32:
// two per row, bf16 / fp16: one, converted with packed instructions), so every wave keeps twice the
// bytes of the 4-column kernel in flight per row and half the instructions per byte -- the
// 4-column kernel reached ~5 TB/s on fp32 and stayed issue-bound on the 2-byte types. Same tiling
// (4 waves = 4 consecutive 32-row bands of one column strip), same one-row-ahead prefetch, same
// fp64 partials (the 8 values of a row are summed in fp32 first, as pairs of 4).
// FULL: every lane's columns exist (C a multiple of the wave's columns): no per-lane store branch
template <class T, int PF, bool FULL = false>
__global__ void __launch_bounds__(256) diffuse_stencil8_kernel(const T* __restrict__ in, T* __restrict__ out,
                                                               const float* __restrict__ wa,
                                                               const float* __restrict__ wb,
                                                               const float* __restrict__ scale,
                                                               const float* __restrict__ corr, MGeom g,
                                                               double* __restrict__ partials, int gx, int gy,
                                                               int ntiles, int vband) {
  __shared__ double red[2][4];
  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int bx = tile % gx, by = (tile / gx) % gy, mol = tile / (gx * gy);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int H = g.r_hi - g.r_lo;
    const int y0 = bx * 512 + lane * 8;
    const bool col = FULL || y0 < g.C;
    const bool need_l = lane == 0 && col, need_r = col && (lane == 63 || y0 + 8 >= g.C);
    const int yl = y0 == 0 ? g.C - 1 : y0 - 1, yr = y0 + 8 >= g.C ? 0 : y0 + 8;
    const size_t plane = (size_t)g.R * g.C;
    const T* src = in + (size_t)mol * plane;
    T* dst = out + (size_t)mol * plane;
    const float sc = scale ? scale[mol] : 1.0f;
    const float a = wa[mol], b = wb[mol];
    const bool has_c = corr != nullptr;
    const float cm = has_c ? corr[mol] : 0.0f;
    const int o0 = (by * 4 + wv) * vband, o1 = min(H, o0 + vband);

    auto row_of = [&](int o) {
      int x = g.r_lo + o;
      if (x < 0) x += g.R;
      if (x >= g.R) x -= g.R;
      return x;
    };
    struct Raw {  // raw bits: converted in finish(), so a prefetched row's loads stay in flight
      Bits8<T> v;
      uint32_t el, er;
    };
    const int yc = col ? y0 : bx * 512;
    auto fetch = [&](int o, Raw& r) {  // (branch-free, as in diffuse_stencil4_kernel)
      const size_t base = (size_t)row_of(o) * g.C;
      ld8_bits(src + base + yc, r.v);
#pragma unroll
      for (int i = 0; i < (int)(sizeof(r.v.q) / sizeof(uint4)); ++i) {
        r.v.q[i].x = col ? r.v.q[i].x : 0u;
        r.v.q[i].y = col ? r.v.q[i].y : 0u;
        r.v.q[i].z = col ? r.v.q[i].z : 0u;
        r.v.q[i].w = col ? r.v.q[i].w : 0u;
      }
      if constexpr (FULL) {  // (one edge load per row, see diffuse_stencil4_kernel)
        r.el = ld_bits(src + base + (need_l ? yl : (need_r ? yr : yc)));
      } else {
        r.el = ld_bits(src + base + (need_l ? yl : yc));
        r.er = ld_bits(src + base + (need_r ? yr : yc));
      }
    };
    auto cin = [&](float raw) { return (has_c ? fmaxf(raw + cm, 0.0f) : raw) * sc; };
    auto finish = [&](const Raw& r, float v[8], float& L, float& Rn) {
      cvt8(r.v, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = cin(v[j]);
      const float up = __shfl_up(v[7], 1), dn = __shfl_down(v[0], 1);
      const float el = cin(from_bits<T>(r.el)), er = FULL ? el : cin(from_bits<T>(r.er));  // (selected: no branch)
      L = need_l ? el : up;
      Rn = need_r ? er : dn;
    };
    auto hsum = [](const float v[8], float L, float Rn, float h[8]) {
      h[0] = L + v[0] + v[1];
#pragma unroll
      for (int j = 1; j < 7; ++j) h[j] = v[j - 1] + v[j] + v[j + 1];
      h[7] = v[6] + v[7] + Rn;
    };

    double before = 0.0, after = 0.0;
    if (o0 < H) {
      Raw rp, rc, rn, rn2;
      fetch(o0 - 1, rp);
      fetch(o0, rc);
      fetch(o0 + 1, rn);
      float vp[8], Lp, Rp, vc[8], Lc, Rc, hp[8], hc[8];
      finish(rp, vp, Lp, Rp);
      finish(rc, vc, Lc, Rc);
      hsum(vp, Lp, Rp, hp);
      hsum(vc, Lc, Rc, hc);
      // (as diffuse_stencil4_kernel, see band_loop)
      auto row_step = [&](int o, const Raw& r_next) {
        float vn[8], Ln, Rn, hn[8];
        finish(r_next, vn, Ln, Rn);
        hsum(vn, Ln, Rn, hn);
        float res[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float lft = j == 0 ? Lc : vc[j - 1], rgt = j == 7 ? Rc : vc[j + 1];
          res[j] = b * vc[j] + a * (hp[j] + hn[j] + lft + rgt);
        }
        if (col) {
          st8_stream(dst + (size_t)row_of(o) * g.C + y0, res);
          before += (double)((vc[0] + vc[1]) + (vc[2] + vc[3])) + (double)((vc[4] + vc[5]) + (vc[6] + vc[7]));
          after += (double)((res[0] + res[1]) + (res[2] + res[3])) + (double)((res[4] + res[5]) + (res[6] + res[7]));
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          hp[j] = hc[j];
          hc[j] = hn[j];
          vc[j] = vn[j];
        }
        Lc = Ln;
        Rc = Rn;
      };
      band_loop<PF>(o0, o1, rn, rn2, fetch, row_step);
    }
    before = wave_sum_d(before);
    after = wave_sum_d(after);
    if (lane == 0) {
      red[0][wv] = before;
      red[1][wv] = after;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const size_t tiles = (size_t)gx * gy;
      const size_t t = (size_t)by * gx + bx;
      partials[((size_t)mol * tiles + t) * 2] = (red[0][0] + red[0][1]) + (red[0][2] + red[0][3]);
      partials[((size_t)mol * tiles + t) * 2 + 1] = (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]);
    }
    __syncthreads();  // red is refilled by the next tile
  }
}

// one block per molecule: totals[mol] = (sum before, sum after) over the owned rows
// (corr_out: also the new per-species correction of a single-process map, (before - after) / n_pix,
// which otherwise takes a diffuse_corr launch after the totals were all-reduced)
__global__ void __launch_bounds__(256) diffuse_reduce_kernel(const double* partials, int tiles, double* totals,
                                                             bool accumulate, float* corr_out, double n_pix) {
  __shared__ double sb[4], sa[4];
  const int mol = blockIdx.x;
  double b = 0.0, a = 0.0;
  for (int t = threadIdx.x; t < tiles; t += blockDim.x) {
    b += partials[((size_t)mol * tiles + t) * 2];
    a += partials[((size_t)mol * tiles + t) * 2 + 1];
  }
  b = wave_sum_d(b);
  a = wave_sum_d(a);
  if ((threadIdx.x & 63) == 0) {
    sb[threadIdx.x >> 6] = b;
    sa[threadIdx.x >> 6] = a;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const double b4 = sb[0] + sb[1] + sb[2] + sb[3], a4 = sa[0] + sa[1] + sa[2] + sa[3];
    const double tb = accumulate ? totals[2 * mol] + b4 : b4, ta = accumulate ? totals[2 * mol + 1] + a4 : a4;
    totals[2 * mol] = tb;
    totals[2 * mol + 1] = ta;
    if (corr_out) corr_out[mol] = (float)((tb - ta) / n_pix);  // (as diffuse_corr_kernel)
  }
}

// diffuse_reduce_kernel over a strip's three stencil launches at once (diffuse_strip): the interior
// rows' partials (`ti` tiles per molecule) and the two boundary rows' (`gx` tiles per molecule each,
// launch b at offset b * gx * m); totals overwritten
__global__ void __launch_bounds__(256) diffuse_reduce_strip_kernel(const double* pi, int ti, const double* pb, int gx,
                                                                   int m, double* totals) {
  __shared__ double sb[4], sa[4];
  const int mol = blockIdx.x;
  double b = 0.0, a = 0.0;
  for (int t = threadIdx.x; t < ti; t += blockDim.x) {
    b += pi[((size_t)mol * ti + t) * 2];
    a += pi[((size_t)mol * ti + t) * 2 + 1];
  }
  for (int t = threadIdx.x; t < 2 * gx; t += blockDim.x) {
    const double* p = pb + (size_t)(t / gx) * gx * m * 2 + ((size_t)mol * gx + t % gx) * 2;
    b += p[0];
    a += p[1];
  }
  b = wave_sum_d(b);
  a = wave_sum_d(a);
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

// Deferred correction: instead of a second full pass map = max(tmp + (before - after) / n_pix, 0),
// only the per-species constant is computed; the stencil output becomes the map (buffer swap) with
// the constant pending, and every later reader applies max(raw + corr, 0) (corr_in) -- the next
// stencil, the pixel gathers of the integrator / permeation / pickup / spill, or one full apply
// when the map is accessed from Python. Saves a read + write of the whole map per step.
__global__ void diffuse_corr_kernel(const double* __restrict__ totals, int m, double n_pix, float* __restrict__ corr) {
  const int mol = blockIdx.x * blockDim.x + threadIdx.x;
  if (mol < m) corr[mol] = (float)((totals[2 * mol] - totals[2 * mol + 1]) / n_pix);
}

// map = max(map + corr, 0) * f (pending correction and / or degradation; either may be null)
template <class T>
__global__ void __launch_bounds__(256) apply_pending_kernel(T* map, const float* corr, const float* f, long long plane,
                                                            int m) {
  const long long total = plane * m;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const int mol = (int)(i / plane);
    float v = corr_in(ld(map + i), corr, mol);
    if (f) v *= f[mol];
    st(map + i, v);
  }
}

// map[owned rows] = max(tmp + (before - after) / n_pix, 0); a plane's owned rows are one
// contiguous range of `span` values starting at r_lo * C. 4 values per thread and iteration.
template <class T>
__global__ void __launch_bounds__(256) diffuse_correct_kernel(const T* __restrict__ tmp, T* __restrict__ map,
                                                              const double* __restrict__ totals, double n_pix,
                                                              long long plane, long long start, long long span, int m) {
  const long long s4 = (span + 3) / 4;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < s4 * m;
       i += (long long)gridDim.x * blockDim.x) {
    const int mol = (int)(i / s4);
    const float c = (float)((totals[2 * mol] - totals[2 * mol + 1]) / n_pix);
    const long long q = (i - (long long)mol * s4) * 4;
    const long long o = (long long)mol * plane + start + q;
    if (q + 4 <= span && (o % 4) == 0) {
      float v[4];
      ld4(tmp + o, v);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = fmaxf(v[j] + c, 0.0f);
      st4(map + o, v);
    } else {
      for (long long e = 0; e < 4 && q + e < span; ++e) st(map + o + e, fmaxf(ld(tmp + o + e) + c, 0.0f));
    }
  }
}

// map *= f[mol] (standalone degradation of the map)
template <class T>
__global__ void __launch_bounds__(256) scale_planes_kernel(T* map, const float* f, long long plane, int m) {
  const long long total = plane * m;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x)
    st(map + i, ld(map + i) * f[i / plane]);
}

// cell_molecules (rows, m) *= f[mol] (the cells' share of degrade_molecules: torch's mul_ with the
// factor row broadcast, one fp32 product per entry)
__global__ void __launch_bounds__(256) scale_rows_kernel(float* x, const float* f, long long total, int m) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x)
    x[i] = x[i] * f[i % m];
}

// x[i] += v (increment_cell_lifetimes)
__global__ void __launch_bounds__(256) add_i32_kernel(int32_t* x, long long n, int v) {
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    x[i] += v;
}

// ---------------------------------------------------------------- cell <-> pixel exchanges
// Killed cells spill their molecules onto their pixel and free it; new cells take half of their
// pixel's molecules. One thread per (cell, molecule); pixels are distinct, so no atomics.
template <class T>
__global__ void __launch_bounds__(256) spill_free_kernel(int k, int m, const int64_t* idxs, const uint8_t* dead,
                                                         const int32_t* pos, int C, long long plane,
                                                         const float* cell_mols, T* map, uint8_t* cell_map,
                                                         const float* corr) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)k * m) return;
  const int i = (int)(t / m), j = (int)(t - (long long)i * m);
  long long c = i;
  if (idxs) c = idxs[i];
  else if (!dead[c]) return;
  const long long pix = (long long)pos[2 * c] * C + pos[2 * c + 1];
  T* p = map + j * plane + pix;
  st(p, corr_out(corr_in(ld(p), corr, j) + cell_mols[c * m + j], corr, j));
  if (j == 0) cell_map[pix] = 0;
}

// The kill / divide thresholds of kill_divide_where (fast.hip threshold_masks_kernel: kill below
// `kill_below` or with probability `kill_p`, divide above `divide_above` paying `cost`) fused with
// the killed cells' spill onto their pixels (spill_free_kernel). Thread (cell i, molecule j), as the
// spill, whole cells per workgroup (blockDim = m * cells per block): every thread of a cell derives
// its kill decision (same value, same Philox draw) before the barrier, after which j == 0 writes
// the masks and the payment (a paying cell survives, so no spill reads the paid molecule).
// One launch less in the step.
template <class T>
__global__ void __launch_bounds__(256) threshold_spill_kernel(int n, int m, int mol, float kill_below, float divide_above,
                                                              float cost, float kill_p, uint64_t seed, uint64_t call,
                                                              float* mols, uint8_t* kill, uint8_t* divide,
                                                              const int32_t* pos, int C, long long plane, T* map,
                                                              uint8_t* cell_map, const float* corr) {
  // (more molecules than threads: one cell per workgroup, molecules strided over the threads)
  const int cpb = max(1, (int)blockDim.x / m), jstep = cpb == 1 ? (int)blockDim.x : m;
  const int i = blockIdx.x * cpb + (cpb == 1 ? 0 : (int)threadIdx.x / m);
  const int j = cpb == 1 ? (int)threadIdx.x : (int)threadIdx.x % m;
  const bool live = (cpb == 1 || (int)threadIdx.x < cpb * m) && i < n && j < m;
  float* x = mols + (size_t)i * m + mol;
  const float v = live ? *x : 0.0f;
  bool k = v < kill_below;
  if (kill_p > 0.0f) {
    Philox rng(seed, call, (uint32_t)i);
    k |= rng.uniform() < kill_p;
  }
  __syncthreads();  // every thread of the cell has read the molecule before j == 0 pays from it
  if (!live) return;
  if (j == 0) {
    const bool d = !k && v > divide_above;
    if (d) *x = v - cost;
    kill[i] = k;
    divide[i] = d;
  }
  if (k) {
    const long long pix = (long long)pos[2 * i] * C + pos[2 * i + 1];
    for (int jj = j; jj < m; jj += jstep) {
      T* p = map + jj * plane + pix;
      st(p, corr_out(corr_in(ld(p), corr, jj) + mols[(size_t)i * m + jj], corr, jj));
    }
    if (j == 0) cell_map[pix] = 0;
  }
}

template <class T>
__global__ void __launch_bounds__(256) pickup_kernel(int k, int m, const int64_t* idxs, const int32_t* pos, int C,
                                                     long long plane, float* cell_mols, T* map, const float* corr) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)k * m) return;
  const int i = (int)(t / m), j = (int)(t - (long long)i * m);
  const long long c = idxs[i];
  const long long pix = (long long)pos[2 * c] * C + pos[2 * c + 1];
  T* p = map + j * plane + pix;
  const float x = corr_in(ld(p), corr, j);
  const float half = x * 0.5f;
  cell_mols[c * m + j] += half;
  st(p, corr_out(x - half, corr, j));
}

// exchange between cells and their pixels (reference world.py:651-665), one thread per
// (cell, molecule)
template <class T>
__global__ void __launch_bounds__(256) permeate_kernel(int c, int m, long long plane, int C, const int32_t* pos,
                                                       const float* perm, float* cell_mols, T* map, const float* corr) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)c * m) return;
  const int cell = (int)(t / m), i = (int)(t - (long long)cell * m);
  const float p = perm[i];
  if (p == 0.0f) return;
  T* q = map + (size_t)i * plane + (size_t)pos[2 * cell] * C + pos[2 * cell + 1];
  const float xi = cell_mols[t], xe = corr_in(ld(q), corr, i);
  const float di = xi * p, de = xe * p;
  cell_mols[t] = xi + (de - di);
  st(q, corr_out(xe + (di - de), corr, i));
}

// ---------------------------------------------------------------- health scan
// flags |= 1 << shift for a non-finite value, 2 << shift for a negative one, over `planes` planes
// of `span` values each (plane stride `stride`). One wave ballot per 64 values, one atomic per block.
template <class T>
__global__ void __launch_bounds__(256) health_kernel(const T* __restrict__ x, int planes, long long span,
                                                     long long stride, int shift, int* flags) {
  __shared__ int blk;
  if (threadIdx.x == 0) blk = 0;
  __syncthreads();
  int f = 0;
  const long long total = (long long)planes * span;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long pl = i / span;
    const float v = ld(x + pl * stride + (i - pl * span));
    f |= (isfinite(v) ? 0 : 1) | (v < 0.0f ? 2 : 0);
  }
  if (__ballot(f & 1)) f |= 1;
  if (__ballot(f & 2)) f |= 2;
  if ((threadIdx.x & 63) == 0 && f) atomicOr(&blk, f);
  __syncthreads();
  if (threadIdx.x == 0 && blk) atomicOr(flags, blk << shift);
}

// ---------------------------------------------------------------- host launchers
static MGeom mgeom(int R, int C, int r_lo, int r_hi, int wrap) {
  if (R <= 0 || C <= 0 || r_lo < 0 || r_hi > R || r_lo >= r_hi) throw std::invalid_argument("bad map geometry");
  if (!wrap && (r_lo < 1 || r_hi > R - 1)) throw std::invalid_argument("a non-wrapping strip needs halo rows");
  return MGeom{R, C, r_lo, r_hi, wrap};
}

// dispatch a templated launch on the map storage type
#define MS_MAP_DISPATCH(dtype, LAUNCH)                                   \
  switch (dtype) {                                                       \
    case kF32: { using T = float; LAUNCH; } break;                       \
    case kBF16: { using T = bf16_t; LAUNCH; } break;                     \
    case kF16: { using T = _Float16; LAUNCH; } break;                    \
    default: throw std::invalid_argument("unknown molecule map dtype");  \
  }

// stencil variant (set_stencil_vec; 0 = auto): 8 columns per lane for 2-byte maps (4096^2 x 14:
// bf16 0.35 -> 0.27-0.31 ms, fp16 0.35 -> 0.31 ms), 4 for fp32 (0.37 ms; the 8-column variant
// measured 0.40-0.43: one 16 B access per row and lane is already enough in flight there,
// profiles/r3/diffuse_bench_4096.jsonl); 1 when C % 4 != 0
static int g_stencil_vec = 0;
void set_stencil_vec(int v) { g_stencil_vec = v; }
static bool use_vec8(int C, int dtype) {
  const int v = g_stencil_vec ? g_stencil_vec : (dtype == kF32 ? 4 : 8);
  return v >= 8 && C % 8 == 0;
}
static bool use_vec4(int C) { return (g_stencil_vec == 0 || g_stencil_vec >= 4) && C % 4 == 0; }

// rows in flight ahead of the vector stencils' current row (band_loop; set_stencil_prefetch, -1 =
// auto: 2 for fp32 maps, 3 for 2-byte maps). Round 3 measured the rings slower than one row ahead
// (profiles/r3/stencil_pf/) -- their per-row guards and branchy edge loads made the compiler wait for
// every load at each row, so they never had more than one row in flight; branch-free whole turns do.
static int g_stencil_pf = -1;
void set_stencil_prefetch(int pf) { g_stencil_pf = pf < -1 ? -1 : (pf > 3 ? 3 : pf); }
static int stencil_pf(int dtype) { return g_stencil_pf >= 0 ? g_stencil_pf : (dtype == kF32 ? 2 : 3); }
// launch LAUNCH with the compile-time prefetch distance PF (and the map type T of MS_MAP_DISPATCH)
#define MS_PF_DISPATCH1(pf, LAUNCH)                                 \
  switch (pf) {                                                     \
    case 0: { constexpr int PF = 0; LAUNCH; } break;                \
    case 1: { constexpr int PF = 1; LAUNCH; } break;                \
    case 2: { constexpr int PF = 2; LAUNCH; } break;                \
    default: { constexpr int PF = 3; LAUNCH; } break;               \
  }
// (and FULL: whether every lane of every strip has its columns, see diffuse_stencil4_kernel)
#define MS_PF_DISPATCH(pf, full, LAUNCH)                                            \
  if (full) { constexpr bool FULL = true; MS_PF_DISPATCH1(pf, LAUNCH) }             \
  else { constexpr bool FULL = false; MS_PF_DISPATCH1(pf, LAUNCH) }

// Blocks of the vector stencil launch (0: one per tile). 256 CUs x 2 workgroups (2 waves per SIMD)
// with 2-3 rows in flight per wave keep the stencil within 1 % of its full-grid time alone (diffuse
// step 0.361 vs 0.357 ms at 768 blocks) and leave the most room to the genome chain it runs next to
// on the side stream, whose latency-bound kernels are the step's other critical path: flagship 300
// timed steps 1178 / 1178 steps/s at 512 blocks, 1100-1122 at 768, 1166-1168 with round 4's one row
// in flight at 1024 (profiles/r5/stencil_blocks_flagship.txt). Round 4 (one row in flight): stencil
// 378 / side chain done 100 us after it at 1024 blocks; 427 / 75 at 896; 500 at 512.
static int g_stencil_blocks = 256 * 2;
void set_stencil_blocks(int n) { g_stencil_blocks = std::max(0, n); }

size_t diffuse_partials_len(int m, int C, int H) {
  // (the largest layout of any variant: the variant may be switched between calls)
  // (sized for the narrowest band set_stencil_band allows)
  const size_t v8 = (size_t)cdiv(C, 512) * cdiv(cdiv(H, kMinVBand), 4) * m * 2;
  const size_t v4 = (size_t)cdiv(C, 256) * cdiv(cdiv(H, kMinVBand), 4) * m * 2;
  const size_t v1 = (size_t)cdiv(C, 64 * kWaves) * cdiv(H, kBand) * m * 2;
  return std::max(v8, std::max(v4, v1));
}

// the stencil launch of diffuse_stencil (partials per tile, no reduce); returns the tiles per molecule
static int stencil_launch(int m, int R, int C, int r_lo, int r_hi, int wrap, uintptr_t map, uintptr_t tmp,
                          uintptr_t wa, uintptr_t wb, uintptr_t scale, uintptr_t corr, uintptr_t partials, int dtype,
                          uintptr_t stream) {
  const MGeom g = mgeom(R, C, r_lo, r_hi, wrap);
  hipStream_t st_ = S_(stream);
  const int H = r_hi - r_lo;
  const bool v8 = use_vec8(C, dtype), v4 = !v8 && use_vec4(C);
  const int vband = stencil_band(C, H, m, v8 ? 512 : 256, g_stencil_blocks);
  const dim3 grid = v8   ? dim3(cdiv(C, 512), cdiv(cdiv(H, vband), 4), m)
                    : v4 ? dim3(cdiv(C, 256), cdiv(cdiv(H, vband), 4), m)
                         : dim3(cdiv(C, 64 * kWaves), cdiv(H, kBand), m);
  if (v8) {
    const int ntiles = (int)(grid.x * grid.y * grid.z);
    const int blocks = g_stencil_blocks > 0 ? std::min(ntiles, g_stencil_blocks) : ntiles;
    MS_MAP_DISPATCH(dtype, MS_PF_DISPATCH(stencil_pf(dtype), C % 512 == 0, (msd::kl(diffuse_stencil8_kernel<T, PF, FULL>, blocks, 256, 0, st_)(
                               P_<T>(map), P_<T>(tmp), P_<float>(wa), P_<float>(wb), scale ? P_<float>(scale) : nullptr,
                               corr ? P_<float>(corr) : nullptr, g, P_<double>(partials), (int)grid.x, (int)grid.y,
                               ntiles, vband))));
  } else if (v4) {
    const int ntiles = (int)(grid.x * grid.y * grid.z);
    const int blocks = g_stencil_blocks > 0 ? std::min(ntiles, g_stencil_blocks) : ntiles;
    MS_MAP_DISPATCH(dtype, MS_PF_DISPATCH(stencil_pf(dtype), C % 256 == 0, (msd::kl(diffuse_stencil4_kernel<T, PF, FULL>, blocks, 256, 0, st_)(
                               P_<T>(map), P_<T>(tmp), P_<float>(wa), P_<float>(wb), scale ? P_<float>(scale) : nullptr,
                               corr ? P_<float>(corr) : nullptr, g, P_<double>(partials), (int)grid.x, (int)grid.y,
                               ntiles, vband))));
  } else {
    MS_MAP_DISPATCH(dtype, (msd::kl(diffuse_stencil_kernel<T>, grid, 64 * kWaves, 0, st_)(
                               P_<T>(map), P_<T>(tmp), P_<float>(wa), P_<float>(wb), scale ? P_<float>(scale) : nullptr,
                               corr ? P_<float>(corr) : nullptr, g, P_<double>(partials))));
  }
  MS_LAUNCH_CHECK();
  return (int)(grid.x * grid.y);
}

void diffuse_stencil(int m, int R, int C, int r_lo, int r_hi, int wrap, uintptr_t map, uintptr_t tmp, uintptr_t wa,
                     uintptr_t wb, uintptr_t scale, uintptr_t corr, uintptr_t partials, uintptr_t totals, int dtype,
                     int accumulate, uintptr_t stream, uintptr_t corr_out, double n_pix) {
  // rows [r_lo, r_hi) of the map; `accumulate`: add this launch's mass totals to `totals` (a strip's
  // stencil split into interior rows, issued while the halo rows are exchanged, and boundary rows)
  if (m <= 0 || r_hi <= r_lo) return;
  const int tiles = stencil_launch(m, R, C, r_lo, r_hi, wrap, map, tmp, wa, wb, scale, corr, partials, dtype, stream);
  msd::kl(diffuse_reduce_kernel, m, 256, 0, S_(stream))(P_<double>(partials), tiles, P_<double>(totals), accumulate != 0,
                                                   corr_out ? P_<float>(corr_out) : nullptr, n_pix);
  MS_LAUNCH_CHECK();
}

// The two boundary rows r_lo and r_hi - 1 of a strip (after its halo rows arrived; the interior rows
// r_lo + 1 .. r_hi - 2 were computed by a diffuse_stencil launch issued before the exchange): one
// single-row stencil launch each, partials side by side, one reduce adding to `totals`.
// the two single-row launches of diffuse_boundary; returns the tiles per molecule and launch
static int boundary_launch(int m, int R, int C, int r_lo, int r_hi, uintptr_t map, uintptr_t tmp, uintptr_t wa,
                           uintptr_t wb, uintptr_t scale, uintptr_t corr, uintptr_t partials, int dtype,
                           uintptr_t stream) {
  hipStream_t st_ = S_(stream);
  const bool v8 = use_vec8(C, dtype), v4 = !v8 && use_vec4(C);
  const int gx = v8 ? cdiv(C, 512) : v4 ? cdiv(C, 256) : cdiv(C, 64 * kWaves);
  const int tiles = gx * m;  // per row (grid.y = 1 for a single row)
  for (int b = 0; b < 2; ++b) {
    const int row = b == 0 ? r_lo : r_hi - 1;
    const MGeom g = mgeom(R, C, row, row + 1, 0);
    double* part = P_<double>(partials) + (size_t)b * tiles * 2;
    if (v8) {
      MS_MAP_DISPATCH(dtype, MS_PF_DISPATCH(stencil_pf(dtype), C % 512 == 0, (msd::kl(diffuse_stencil8_kernel<T, PF, FULL>, tiles, 256, 0, st_)(
                                 P_<T>(map), P_<T>(tmp), P_<float>(wa), P_<float>(wb), scale ? P_<float>(scale) : nullptr,
                                 corr ? P_<float>(corr) : nullptr, g, part, gx, 1, tiles, kVBand))));
    } else if (v4) {
      MS_MAP_DISPATCH(dtype, MS_PF_DISPATCH(stencil_pf(dtype), C % 256 == 0, (msd::kl(diffuse_stencil4_kernel<T, PF, FULL>, tiles, 256, 0, st_)(
                                 P_<T>(map), P_<T>(tmp), P_<float>(wa), P_<float>(wb), scale ? P_<float>(scale) : nullptr,
                                 corr ? P_<float>(corr) : nullptr, g, part, gx, 1, tiles, kVBand))));
    } else {
      MS_MAP_DISPATCH(dtype, (msd::kl(diffuse_stencil_kernel<T>, dim3(gx, 1, m), 64 * kWaves, 0, st_)(
                                 P_<T>(map), P_<T>(tmp), P_<float>(wa), P_<float>(wb), scale ? P_<float>(scale) : nullptr,
                                 corr ? P_<float>(corr) : nullptr, g, part)));
    }
    MS_LAUNCH_CHECK();
  }
  return gx;
}

void diffuse_boundary(int m, int R, int C, int r_lo, int r_hi, uintptr_t map, uintptr_t tmp, uintptr_t wa,
                      uintptr_t wb, uintptr_t scale, uintptr_t corr, uintptr_t partials, uintptr_t totals, int dtype,
                      uintptr_t stream) {
  if (m <= 0 || r_hi - r_lo < 2) throw std::invalid_argument("diffuse_boundary: a strip of at least 2 rows");
  hipStream_t st_ = S_(stream);
  const int gx = boundary_launch(m, R, C, r_lo, r_hi, map, tmp, wa, wb, scale, corr, partials, dtype, stream);
  const int tiles = gx * m;
  // partials of both launches: (mol, tile) pairs, launch b at offset b * tiles; reduce them as one
  // (2 * gx)-tile layout per molecule requires mol-major order, so reduce each launch and accumulate
  msd::kl(diffuse_reduce_kernel, m, 256, 0, st_)(P_<double>(partials), gx, P_<double>(totals), true, nullptr, 1.0);
  MS_LAUNCH_CHECK();
  msd::kl(diffuse_reduce_kernel, m, 256, 0, st_)(P_<double>(partials) + (size_t)tiles * 2, gx, P_<double>(totals), true, nullptr, 1.0);
  MS_LAUNCH_CHECK();
}

size_t diffuse_boundary_partials_len(int m, int C) { return (size_t)4 * cdiv(C, 64) * m; }

void halo_pack(int m, int C, int H, int elem, uintptr_t map, uintptr_t send_up, uintptr_t send_dn, uintptr_t stream);
void halo_unpack(int m, int C, int H, int elem, uintptr_t map, uintptr_t from_up, uintptr_t from_dn, uintptr_t stream);
void rccl_exchange(uintptr_t comm, int up, int down, uintptr_t send_up, long long n_send_up, uintptr_t send_down,
                   long long n_send_down, uintptr_t recv_down, long long n_recv_down, uintptr_t recv_up,
                   long long n_recv_up, uintptr_t stream);
void rccl_allreduce(uintptr_t comm, uintptr_t buf, long long count, int dtype, int op, uintptr_t stream);
void stream_join(uintptr_t dst, uintptr_t src);
void diffuse_corr(int m, uintptr_t totals, double n_pix, uintptr_t corr, uintptr_t stream);

// One diffusion step of a strip of a decomposed world over the native RCCL communicator, in one call:
// the halo rows travel on `halo_stream` (pack, exchange, unpack) while the interior rows' stencil runs
// on `stream`; then the two boundary rows, one reduce of the three launches' partials, the all-reduce
// (SUM) of the mass totals and the new correction. Same kernels as ops/hip_ops.py diffuse (split path).
void diffuse_strip(int m, int R, int C, int r_lo, int r_hi, uintptr_t map, uintptr_t tmp, uintptr_t wa, uintptr_t wb,
                   uintptr_t scale, uintptr_t corr, uintptr_t partials, uintptr_t partials_b, uintptr_t totals,
                   uintptr_t new_corr, double n_pix, int dtype, uintptr_t comm, int up, int down, uintptr_t halo_bufs,
                   uintptr_t halo_stream, uintptr_t stream) {
  const int H = r_hi - r_lo;
  if (m <= 0 || H < 3 || r_lo != 1 || R != r_hi + 1) throw std::invalid_argument("diffuse_strip: not a strip of >= 3 rows");
  const int elem = dtype == kF32 ? 4 : 2;
  const long long plane_b = (long long)m * C * elem;  // one halo row of every species, bytes
  const uintptr_t s_up = halo_bufs, s_dn = halo_bufs + plane_b, r_dn = halo_bufs + 2 * plane_b,
                  r_up = halo_bufs + 3 * plane_b;
  stream_join(halo_stream, stream);
  halo_pack(m, C, H, elem, map, s_up, s_dn, halo_stream);
  rccl_exchange(comm, up, down, s_up, plane_b, s_dn, plane_b, r_dn, plane_b, r_up, plane_b, halo_stream);
  halo_unpack(m, C, H, elem, map, r_up, r_dn, halo_stream);
  const int ti = stencil_launch(m, R, C, r_lo + 1, r_hi - 1, 0, map, tmp, wa, wb, scale, corr, partials, dtype, stream);
  stream_join(stream, halo_stream);
  const int gx = boundary_launch(m, R, C, r_lo, r_hi, map, tmp, wa, wb, scale, corr, partials_b, dtype, stream);
  msd::kl(diffuse_reduce_strip_kernel, m, 256, 0, S_(stream))(P_<double>(partials), ti, P_<double>(partials_b), gx, m,
                                                         P_<double>(totals));
  MS_LAUNCH_CHECK();
  rccl_allreduce(comm, totals, 2ll * m, 2 /* float64 */, 0 /* sum */, stream);
  diffuse_corr(m, totals, n_pix, new_corr, stream);
}

void diffuse_correct(int m, int R, int C, int r_lo, int r_hi, uintptr_t map, uintptr_t tmp, uintptr_t totals,
                     double n_pix, int dtype, uintptr_t stream) {
  if (m <= 0) return;
  const long long plane = (long long)R * C, start = (long long)r_lo * C, span = (long long)(r_hi - r_lo) * C;
  const unsigned g = std::min<long long>(cdiv((span + 3) / 4 * m, 256), 8192);
  MS_MAP_DISPATCH(dtype, (msd::kl(diffuse_correct_kernel<T>, g, 256, 0, S_(stream))(P_<T>(tmp), P_<T>(map),
                                                                               P_<double>(totals), n_pix, plane,
                                                                               start, span, m)));
  MS_LAUNCH_CHECK();
}

void diffuse_corr(int m, uintptr_t totals, double n_pix, uintptr_t corr, uintptr_t stream) {
  if (m <= 0) return;
  msd::kl(diffuse_corr_kernel, cdiv(m, 64), 64, 0, S_(stream))(P_<double>(totals), m, n_pix, P_<float>(corr));
  MS_LAUNCH_CHECK();
}

// Per-species totals of the owned rows [r_lo, r_hi) of a map in float64, as a reader sees it (the
// pending correction and degradation applied on the fly, nothing written): one block per (species,
// chunk of rows) writes a partial, atomically added into out[mol] (zeroed by the caller). A read
// of the map instead of the full read + write of apply_pending (World.molecule_totals).
template <class T>
__global__ void __launch_bounds__(256) map_totals_kernel(const T* __restrict__ map, int R, int C, int r_lo, int r_hi,
                                                         const float* corr, const float* f, double* out) {
  const int mol = blockIdx.y;
  const long long plane = (long long)R * C;
  const long long lo = (long long)r_lo * C, hi = (long long)r_hi * C;
  double acc = 0.0;
  const float sc = f ? f[mol] : 1.0f;
  for (long long i = lo + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < hi; i += (long long)gridDim.x * blockDim.x)
    acc += (double)(corr_in(ld(map + mol * plane + i), corr, mol) * sc);
  acc = wave_sum_d(acc);
  __shared__ double sh[4];
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(out + mol, (sh[0] + sh[1]) + (sh[2] + sh[3]));
}

void map_totals(int m, int R, int C, int r_lo, int r_hi, uintptr_t map, uintptr_t corr, uintptr_t f, int dtype,
                uintptr_t out, uintptr_t stream) {
  if (m <= 0 || r_hi <= r_lo) return;
  const long long px = (long long)(r_hi - r_lo) * C;
  const dim3 g((unsigned)std::max<long long>(1, std::min<long long>(cdiv(px, 256 * 8), 512)), (unsigned)m);
  MS_MAP_DISPATCH(dtype, (msd::kl(map_totals_kernel<T>, g, 256, 0, S_(stream))(
                             P_<T>(map), R, C, r_lo, r_hi, corr ? P_<float>(corr) : nullptr,
                             f ? P_<float>(f) : nullptr, P_<double>(out))));
  MS_LAUNCH_CHECK();
}

void apply_pending(int m, long long plane, uintptr_t map, uintptr_t corr, uintptr_t f, int dtype, uintptr_t stream) {
  if (m <= 0 || plane <= 0 || (!corr && !f)) return;
  const unsigned g = std::min<long long>(cdiv(plane * m, 256), 8192);
  MS_MAP_DISPATCH(dtype, (msd::kl(apply_pending_kernel<T>, g, 256, 0, S_(stream))(
                             P_<T>(map), corr ? P_<float>(corr) : nullptr, f ? P_<float>(f) : nullptr, plane, m)));
  MS_LAUNCH_CHECK();
}

void health_scan(int planes, long long span, long long stride, uintptr_t x, int dtype, int shift, uintptr_t flags,
                 uintptr_t stream) {
  if (planes <= 0 || span <= 0) return;
  const unsigned g = std::min<long long>(cdiv((long long)planes * span, 256), 4096);
  MS_MAP_DISPATCH(dtype, (msd::kl(health_kernel<T>, g, 256, 0, S_(stream))(P_<T>(x), planes, span, stride, shift,
                                                                        P_<int>(flags))));
  MS_LAUNCH_CHECK();
}

void scale_planes(int m, long long plane, uintptr_t map, uintptr_t f, int dtype, uintptr_t stream) {
  if (m <= 0 || plane <= 0) return;
  const unsigned g = std::min<long long>(cdiv(plane * m, 256), 8192);
  MS_MAP_DISPATCH(dtype, (msd::kl(scale_planes_kernel<T>, g, 256, 0, S_(stream))(P_<T>(map), P_<float>(f), plane, m)));
  MS_LAUNCH_CHECK();
}

void scale_rows(long long rows, int m, uintptr_t x, uintptr_t f, uintptr_t stream) {
  if (rows <= 0 || m <= 0) return;
  const unsigned g = std::min<long long>(cdiv(rows * m, 256), 4096);
  msd::kl(scale_rows_kernel, g, 256, 0, S_(stream))(P_<float>(x), P_<float>(f), rows * m, m);
  MS_LAUNCH_CHECK();
}

void add_i32(long long n, uintptr_t x, int v, uintptr_t stream) {
  if (n <= 0) return;
  const unsigned g = std::min<long long>(cdiv(n, 256), 4096);
  msd::kl(add_i32_kernel, g, 256, 0, S_(stream))(P_<int32_t>(x), n, v);
  MS_LAUNCH_CHECK();
}

void spill_free(int k, int m, uintptr_t idxs, uintptr_t pos, int R, int C, uintptr_t cell_mols, uintptr_t map,
                uintptr_t cell_map, int dtype, uintptr_t corr, uintptr_t stream) {
  if (k <= 0 || m <= 0) return;
  MS_MAP_DISPATCH(dtype, (msd::kl(spill_free_kernel<T>, cdiv((long long)k * m, 256), 256, 0, S_(stream))(
                             k, m, P_<int64_t>(idxs), nullptr, P_<int32_t>(pos), C, (long long)R * C,
                             P_<float>(cell_mols), P_<T>(map), P_<uint8_t>(cell_map), P_<float>(corr))));
  MS_LAUNCH_CHECK();
}

void threshold_spill(int n, int m, int mol, float kill_below, float divide_above, float cost, float kill_p, uint64_t seed,
                     uint64_t call, uintptr_t mols, uintptr_t kill, uintptr_t divide, uintptr_t pos, int R, int C,
                     uintptr_t map, uintptr_t cell_map, int dtype, uintptr_t corr, uintptr_t stream) {
  if (n <= 0 || m <= 0) return;
  const int cpb = std::max(1, 256 / m);
  MS_MAP_DISPATCH(dtype, (msd::kl(threshold_spill_kernel<T>, cdiv(n, cpb), cpb == 1 ? 256 : cpb * m, 0, S_(stream))(
                             n, m, mol, kill_below, divide_above, cost, kill_p, seed, call, P_<float>(mols),
                             P_<uint8_t>(kill), P_<uint8_t>(divide), P_<int32_t>(pos), C, (long long)R * C, P_<T>(map),
                             P_<uint8_t>(cell_map), P_<float>(corr))));
  MS_LAUNCH_CHECK();
}

void spill_free_mask(int n, int m, uintptr_t dead, uintptr_t pos, int R, int C, uintptr_t cell_mols, uintptr_t map,
                     uintptr_t cell_map, int dtype, uintptr_t corr, uintptr_t stream) {
  if (n <= 0 || m <= 0) return;
  MS_MAP_DISPATCH(dtype, (msd::kl(spill_free_kernel<T>, cdiv((long long)n * m, 256), 256, 0, S_(stream))(
                             n, m, nullptr, P_<uint8_t>(dead), P_<int32_t>(pos), C, (long long)R * C,
                             P_<float>(cell_mols), P_<T>(map), P_<uint8_t>(cell_map), P_<float>(corr))));
  MS_LAUNCH_CHECK();
}

// spawn_cells without a host round trip: the new cells' pixels from spawn_claims (world.hip:
// deterministic priority rounds), then one thread per new cell j (row n0 + j): position, lifetime 0,
// divisions 0, half of the pixel's molecules (the pixel keeps the other half, as pickup) and a random
// 12-character label.
constexpr int kLabelLen = 12;
__global__ void __launch_bounds__(256) spawn_init_kernel(int k, int R, int C, const long long* result, uint64_t seed,
                                                         uint64_t call, long long n0, int m, int32_t* pos,
                                                         int32_t* lifetimes, int32_t* divisions, float* cell_mols,
                                                         void* map, int dtype, const float* corr, uint8_t* labels,
                                                         int label_w, int32_t* label_lens, int* failed) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= k) return;
  const long long got = result[j];
  const long long c = n0 + j;
  if (got < 0) {  // more new cells than free pixels: the caller's count was wrong
    atomicOr(failed, 1);
    return;
  }
  Philox rng(seed, call ^ 0x9E3779B97F4A7C15ull, (uint32_t)j);  // (the labels' stream)
  const int x = (int)(got / C), y = (int)(got - (long long)(got / C) * C);
  pos[2 * c] = x;
  pos[2 * c + 1] = y;
  lifetimes[c] = 0;
  divisions[c] = 0;
  const long long plane = (long long)R * C;
  for (int q = 0; q < m; ++q) {
    const size_t px = (size_t)q * plane + got;
    const float v = corr_in(ld_map(map, px, dtype), corr, q);
    const float half = v * 0.5f;
    cell_mols[c * m + q] = half;
    st_map(map, px, corr_out(v - half, corr, q), dtype);
  }
  const char* abc = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789";
  uint8_t* lab = labels + (size_t)c * label_w;
  for (int i = 0; i < label_w; ++i) lab[i] = i < kLabelLen ? (uint8_t)abc[rng.below(62)] : 0;
  label_lens[c] = kLabelLen;
}

void spawn_claims(int k, int C, int r_lo, int r_hi, uintptr_t cell_map, uintptr_t claim, uintptr_t cand,
                  uintptr_t result, uint64_t seed, uint64_t call, uintptr_t failed, hipStream_t s);  // world.hip

void pool_write(int k, int L_in, uintptr_t rows, uintptr_t lens, uintptr_t dst, long long n0, uintptr_t pool,
                uintptr_t off, uintptr_t top, long long cap, uintptr_t out_lens, uintptr_t failed, uintptr_t stream);

void spawn_dev(int k, int R, int C, int r_lo, int r_hi, uintptr_t cell_map, uint64_t seed, uint64_t call,
               long long n0, int m, uintptr_t pos, uintptr_t lifetimes, uintptr_t divisions, uintptr_t cell_mols,
               uintptr_t map, int dtype, uintptr_t corr, uintptr_t labels, int label_w, uintptr_t label_lens,
               int L_in, uintptr_t rows, uintptr_t lens, uintptr_t pool, uintptr_t off, uintptr_t top,
               long long pool_cap, uintptr_t arena_lens, uintptr_t failed, uintptr_t pool_failed, uintptr_t claim,
               uintptr_t cand, uintptr_t result, uintptr_t stream) {
  if (k <= 0) return;
  if (R <= 0 || C <= 0 || r_lo < 0 || r_hi > R || r_lo >= r_hi) throw std::invalid_argument("spawn_dev: bad geometry");
  if (label_w < kLabelLen) throw std::invalid_argument("spawn_dev: label rows too narrow");
  if (!claim || !cand || !result) throw std::invalid_argument("spawn_dev: claim map and scratch required");
  hipStream_t s = S_(stream);
  spawn_claims(k, C, r_lo, r_hi, cell_map, claim, cand, result, seed, call, failed, s);
  msd::kl(spawn_init_kernel, cdiv(k, 256), 256, 0, s)(k, R, C, P_<long long>(result), seed, call, n0, m, P_<int32_t>(pos),
                                                 P_<int32_t>(lifetimes), P_<int32_t>(divisions), P_<float>(cell_mols),
                                                 P_<void>(map), dtype, corr ? P_<float>(corr) : nullptr,
                                                 P_<uint8_t>(labels), label_w, P_<int32_t>(label_lens), P_<int>(failed));
  MS_LAUNCH_CHECK();
  // the genomes into fresh pool space (pool.hip)
  pool_write(k, L_in, rows, lens, 0, n0, pool, off, top, pool_cap, arena_lens, pool_failed, stream);
}

// Save / restore the state an enzymatic_activity changes: cell molecules and the raw map values
// (no pending correction applied) of the cells' pixels, as (n, 2m) floats (bf16 / fp16 storage
// round-trips exactly through float). Lets the World issue the activity before pending parameter
// rebuilds are confirmed and undo it in the rare case one had to be redone on the host.
__global__ void __launch_bounds__(256) cell_state_io_kernel(int n, int m, const int32_t* pos, int C, long long plane,
                                                            void* map, int dtype, float* cell_mols, float* buf,
                                                            int restore) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)n * m) return;
  const int i = (int)(t / m), j = (int)(t - (long long)i * m);
  const size_t px = (size_t)pos[2 * i] * C + pos[2 * i + 1] + (size_t)j * plane;
  float* row = buf + (size_t)i * 2 * m;
  if (restore) {
    cell_mols[(size_t)i * m + j] = row[j];
    st_map(map, px, row[m + j], dtype);
  } else {
    row[j] = cell_mols[(size_t)i * m + j];
    row[m + j] = ld_map(map, px, dtype);
  }
}

void cell_state_io(int n, int m, uintptr_t pos, int R, int C, uintptr_t map, int dtype, uintptr_t cell_mols,
                   uintptr_t buf, bool restore, uintptr_t stream) {
  if (n <= 0 || m <= 0) return;
  msd::kl(cell_state_io_kernel, cdiv((long long)n * m, 256), 256, 0, S_(stream))(
      n, m, P_<int32_t>(pos), C, (long long)R * C, P_<void>(map), dtype, P_<float>(cell_mols), P_<float>(buf),
      restore ? 1 : 0);
  MS_LAUNCH_CHECK();
}

void pickup(int k, int m, uintptr_t idxs, uintptr_t pos, int R, int C, uintptr_t cell_mols, uintptr_t map, int dtype,
            uintptr_t corr, uintptr_t stream) {
  if (k <= 0 || m <= 0) return;
  MS_MAP_DISPATCH(dtype, (msd::kl(pickup_kernel<T>, cdiv((long long)k * m, 256), 256, 0, S_(stream))(
                             k, m, P_<int64_t>(idxs), P_<int32_t>(pos), C, (long long)R * C, P_<float>(cell_mols),
                             P_<T>(map), P_<float>(corr))));
  MS_LAUNCH_CHECK();
}

void permeate(int c, int m, int R, int C, uintptr_t pos, uintptr_t perm, uintptr_t cell_mols, uintptr_t map, int dtype,
              uintptr_t corr, uintptr_t stream) {
  if (c <= 0 || m <= 0) return;
  MS_MAP_DISPATCH(dtype, (msd::kl(permeate_kernel<T>, cdiv((long long)c * m, 256), 256, 0, S_(stream))(
                             c, m, (long long)R * C, C, P_<int32_t>(pos), P_<float>(perm), P_<float>(cell_mols),
                             P_<T>(map), P_<float>(corr))));
  MS_LAUNCH_CHECK();
}

}  // namespace msd
