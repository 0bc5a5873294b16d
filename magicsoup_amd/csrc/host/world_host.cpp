// Host (OpenMP) world geometry and map physics for the CPU plumbing path.
//
// Neighbour search, division and movement placement follow rust/world.rs:9-146 but replace the
// O(n) `positions.contains` scans with an O(1) occupancy lookup (a dense bitmap of the map and a
// hash of occupied pixels -> cell index). The diffusion stencil / mass correction follow
// python/magicsoup/world.py:627-665 and 948-984.
//
// Geometry (same as csrc/hip/world.hip): R x C pixels, cells in rows [r_lo, r_hi), the x axis wraps
// for a whole map; a strip of a domain-decomposed world has halo rows 0 and R-1 and does not wrap.
#include <omp.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <string_view>

#include "host_common.h"

namespace ms_host {

using iarr = py::array_t<int32_t, py::array::c_style>;
using farr = py::array_t<float, py::array::c_style>;
using barr = py::array_t<uint8_t, py::array::c_style>;

namespace {

struct Grid {
  int64_t R, C;
  bool wrap;
  std::vector<uint64_t> bits;
  Grid(int64_t R_, int64_t C_, bool w) : R(R_), C(C_), wrap(w), bits((size_t)((R_ * C_ + 63) / 64), 0ull) {}
  int64_t key(int64_t x, int64_t y) const { return x * C + y; }
  bool get(int64_t k) const { return (bits[(size_t)(k >> 6)] >> (k & 63)) & 1ull; }
  void set(int64_t k, bool v) {
    if (v) bits[(size_t)(k >> 6)] |= 1ull << (k & 63);
    else bits[(size_t)(k >> 6)] &= ~(1ull << (k & 63));
  }
  // reference neighbour order (rust/util.rs:30-46): (w,n),(w,y),(w,s),(x,n),(x,s),(e,n),(e,y),(e,s),
  // duplicates removed (tiny maps). Without wrap, x +- 1 stays inside the halo rows.
  int nghbhd(int64_t x, int64_t y, int64_t* out) const {
    const int64_t e = wrap ? (x + 1) % R : x + 1, w = wrap ? (x - 1 + R) % R : x - 1;
    const int64_t s = (y + 1) % C, n = (y - 1 + C) % C;
    const int64_t v[8][2] = {{w, n}, {w, y}, {w, s}, {x, n}, {x, s}, {e, n}, {e, y}, {e, s}};
    int cnt = 0;
    for (int i = 0; i < 8; ++i) {
      const int64_t k = key(v[i][0], v[i][1]);
      bool dup = false;
      for (int q = 0; q < cnt; ++q) dup |= out[q] == k;
      if (!dup) out[cnt++] = k;
    }
    return cnt;
  }
};

void check_geom(int64_t R, int64_t C, int64_t r_lo, int64_t r_hi, bool wrap) {
  if (R <= 0 || C <= 0 || r_lo < 0 || r_hi > R || r_lo >= r_hi) throw std::invalid_argument("bad map geometry");
  if (!wrap && (r_lo < 1 || r_hi > R - 1)) throw std::invalid_argument("a non-wrapping strip needs halo rows");
}

// pick among free neighbours; shared by division and movement. `occ_extra` marks occupied halo
// pixels (from the neighbour ranks) in addition to the cells' own positions.
py::tuple place(iarr cell_idxs, iarr positions, int64_t R, int64_t C, int64_t r_lo, int64_t r_hi, bool wrap,
                py::object halo_occ, bool vacate) {
  check_geom(R, C, r_lo, r_hi, wrap);
  const int32_t* pos = positions.data();
  const int n_all = (int)positions.shape(0), n = (int)cell_idxs.size();
  const int32_t* ci = cell_idxs.data();
  Grid occ(R, C, wrap);
  for (int i = 0; i < n_all; ++i) occ.set(occ.key(pos[2 * i], pos[2 * i + 1]), true);
  if (!halo_occ.is_none()) {
    // (R, C) uint8 occupancy of the strip: the halo rows (neighbours' boundary rows) and pixels of
    // the owned boundary rows reserved for a neighbour's claims (strip protocol: value 2)
    barr h = halo_occ.cast<barr>();
    const uint8_t* hp = h.data();
    for (int64_t px = 0; px < R * C; ++px)
      if (hp[px]) occ.set(px, true);
  }
  auto rng = item_engine(next_call_seed(), 0);
  std::vector<int32_t> who, npos;
  for (int i = 0; i < n; ++i) {
    const int32_t c = ci[i];
    const int64_t x = pos[2 * c], y = pos[2 * c + 1];
    int64_t nb[8], fr[8];
    const int cnt = occ.nghbhd(x, y, nb);
    int nf = 0;
    for (int q = 0; q < cnt; ++q)
      if (!occ.get(nb[q])) fr[nf++] = nb[q];
    if (nf == 0) continue;
    std::uniform_int_distribution<int> pick(0, nf - 1);
    const int64_t k = fr[pick(rng)];
    // a move into a halo row is committed only after the owning rank accepts it: keep the pixel
    if (vacate && (wrap || (k / C >= r_lo && k / C < r_hi))) occ.set(occ.key(x, y), false);
    occ.set(k, true);
    who.push_back(c);
    npos.push_back((int32_t)(k / C));
    npos.push_back((int32_t)(k % C));
  }
  iarr p((py::ssize_t)who.size());
  std::copy(who.begin(), who.end(), p.mutable_data());
  iarr q({(py::ssize_t)who.size(), (py::ssize_t)2});
  std::copy(npos.begin(), npos.end(), q.mutable_data());
  return py::make_tuple(p, q);
}

}  // namespace

// All unique neighbour pairs (a < b) between `from` cells and `to` cells (Chebyshev distance 1).
// Returns an int32 array (k, 2) sorted lexicographically.
iarr get_neighbors(iarr from_idxs, iarr to_idxs, iarr positions, int64_t R, int64_t C, bool wrap) {
  const int32_t* pos = positions.data();
  const int nf = (int)from_idxs.size(), nt = (int)to_idxs.size();
  const int32_t *fi = from_idxs.data(), *ti = to_idxs.data();
  std::unordered_map<int64_t, std::vector<int32_t>> at;  // pixel -> to-cells on it
  at.reserve((size_t)nt * 2);
  for (int i = 0; i < nt; ++i) {
    const int32_t c = ti[i];
    at[(int64_t)pos[2 * c] * C + pos[2 * c + 1]].push_back(c);
  }
  Grid g(1, C, wrap);
  g.R = R;
  std::vector<std::pair<int32_t, int32_t>> pairs;
  for (int i = 0; i < nf; ++i) {
    const int32_t c = fi[i];
    int64_t keys[9];
    int cnt = g.nghbhd(pos[2 * c], pos[2 * c + 1], keys);
    // the cell's own pixel can hold further to-cells only if positions were set by hand
    keys[cnt++] = (int64_t)pos[2 * c] * C + pos[2 * c + 1];
    std::sort(keys, keys + cnt);
    const int64_t* kend = std::unique(keys, keys + cnt);
    for (const int64_t* k = keys; k != kend; ++k) {
      auto it = at.find(*k);
      if (it == at.end()) continue;
      for (int32_t o : it->second)
        if (o != c) pairs.push_back({std::min(c, o), std::max(c, o)});
    }
  }
  std::sort(pairs.begin(), pairs.end());
  pairs.erase(std::unique(pairs.begin(), pairs.end()), pairs.end());
  iarr out({(py::ssize_t)pairs.size(), (py::ssize_t)2});
  int32_t* o = out.mutable_data();
  for (size_t i = 0; i < pairs.size(); ++i) {
    o[2 * i] = pairs[i].first;
    o[2 * i + 1] = pairs[i].second;
  }
  return out;
}

// Division placement (rust/world.rs:59-97): in list order, each dividing cell claims a uniformly
// random free Moore neighbour not claimed by an earlier child. Returns (parents, child positions).
py::tuple divide_cells(iarr cell_idxs, iarr positions, int64_t R, int64_t C, int64_t r_lo, int64_t r_hi, bool wrap,
                       py::object halo_occ) {
  return place(cell_idxs, positions, R, C, r_lo, r_hi, wrap, halo_occ, false);
}

// Movement (rust/world.rs:102-146): non-moving cells are obstacles; moving cells, in list order,
// hop to a uniformly random free Moore neighbour. Returns (moved cell idxs, new positions).
py::tuple move_cells(iarr cell_idxs, iarr positions, int64_t R, int64_t C, int64_t r_lo, int64_t r_hi, bool wrap,
                     py::object halo_occ) {
  return place(cell_idxs, positions, R, C, r_lo, r_hi, wrap, halo_occ, true);
}

// Diffusion stencil over the owned rows of an (m, R, C) map into `out` (same shape; only owned
// rows written): b*x + a*sum(8 neighbours) on inputs pre-scaled by `scale`. Returns per-molecule
// (sum before, sum after) of the owned rows, accumulated in double.
py::array_t<double> diffuse_stencil(farr mol_map, farr out, std::vector<float> a_w, std::vector<float> b_w,
                                    std::vector<float> scale, int64_t r_lo, int64_t r_hi, bool wrap) {
  const int m = (int)mol_map.shape(0);
  const int64_t R = mol_map.shape(1), C = mol_map.shape(2);
  check_geom(R, C, r_lo, r_hi, wrap);
  if ((int)a_w.size() != m || (int)b_w.size() != m || (int)scale.size() != m)
    throw std::invalid_argument("one weight pair / scale per molecule");
  const float* base = mol_map.data();
  float* dst = out.mutable_data();
  py::array_t<double> totals({(py::ssize_t)m, (py::ssize_t)2});
  double* tot = totals.mutable_data();
  py::gil_scoped_release nogil;
  for (int mi = 0; mi < m; ++mi) {
    const float* x = base + (size_t)mi * R * C;
    float* o = dst + (size_t)mi * R * C;
    const float a = a_w[mi], b = b_w[mi], sc = scale[mi];
    double before = 0.0, after = 0.0;
#pragma omp parallel for reduction(+ : before, after) schedule(static)
    for (int64_t i = r_lo; i < r_hi; ++i) {
      const int64_t im = wrap ? (i - 1 + R) % R : i - 1, ip = wrap ? (i + 1) % R : i + 1;
      for (int64_t j = 0; j < C; ++j) {
        const int64_t jm = (j - 1 + C) % C, jp = (j + 1) % C;
        const float c0 = x[i * C + j] * sc;
        const float nsum = x[im * C + jm] * sc + x[im * C + j] * sc + x[im * C + jp] * sc + x[i * C + jm] * sc +
                           x[i * C + jp] * sc + x[ip * C + jm] * sc + x[ip * C + j] * sc + x[ip * C + jp] * sc;
        const float v = b * c0 + a * nsum;
        o[i * C + j] = v;
        before += c0;
        after += v;
      }
    }
    tot[2 * mi] = before;
    tot[2 * mi + 1] = after;
  }
  return totals;
}

// map[owned] = max(out + (before - after) / n_pix, 0)
void diffuse_correct(farr mol_map, farr out, py::array_t<double, py::array::c_style> totals, double n_pix,
                     int64_t r_lo, int64_t r_hi) {
  const int m = (int)mol_map.shape(0);
  const int64_t R = mol_map.shape(1), C = mol_map.shape(2);
  float* x = mol_map.mutable_data();
  const float* o = out.data();
  const double* tot = totals.data();
  py::gil_scoped_release nogil;
  for (int mi = 0; mi < m; ++mi) {
    const float corr = (float)((tot[2 * mi] - tot[2 * mi + 1]) / n_pix);
    const size_t base = (size_t)mi * R * C;
#pragma omp parallel for schedule(static)
    for (int64_t k = r_lo * C; k < r_hi * C; ++k) {
      const float v = o[base + k] + corr;
      x[base + k] = v < 0.0f ? 0.0f : v;
    }
  }
}

// Strings concatenated in `joined` (lengths `lens`) -> zero-padded rows (n, width): the bulk upload
// format of the genome / label arenas (models/strings.py pack_strings), one pass instead of a
// Python slice assignment per string.
barr pack_rows(py::bytes joined, iarr lens, int64_t width) {
  std::string_view buf = joined;
  const int64_t n = lens.shape(0);
  const int32_t* L = lens.data();
  std::vector<int64_t> off((size_t)n + 1, 0);
  for (int64_t i = 0; i < n; ++i) {
    if (L[i] < 0 || L[i] > width) throw std::invalid_argument("pack_rows: a string is longer than the row width");
    off[(size_t)i + 1] = off[(size_t)i] + L[i];
  }
  if (off[(size_t)n] != (int64_t)buf.size()) throw std::invalid_argument("pack_rows: lengths do not add up");
  barr out({n, width});
  uint8_t* o = out.mutable_data();
  const char* src = buf.data();
  {
    py::gil_scoped_release nogil;
#pragma omp parallel for schedule(static) if (n > 256)
    for (int64_t i = 0; i < n; ++i) {
      uint8_t* row = o + i * width;
      std::memcpy(row, src + off[(size_t)i], (size_t)L[i]);
      std::memset(row + L[i], 0, (size_t)(width - L[i]));
    }
  }
  return out;
}

// The inverse of pack_rows: the first lens[i] bytes of every row, concatenated (one buffer the
// caller decodes once and slices into strings).
py::bytes unpack_rows(barr rows, iarr lens) {
  if (rows.ndim() != 2 || lens.shape(0) != rows.shape(0)) throw std::invalid_argument("unpack_rows: shapes");
  const int64_t n = rows.shape(0), w = rows.shape(1);
  const int32_t* L = lens.data();
  std::vector<int64_t> off((size_t)n + 1, 0);
  for (int64_t i = 0; i < n; ++i) {
    if (L[i] < 0 || L[i] > w) throw std::invalid_argument("unpack_rows: a length exceeds the row width");
    off[(size_t)i + 1] = off[(size_t)i] + L[i];
  }
  std::string out((size_t)off[(size_t)n], '\0');
  const uint8_t* src = rows.data();
  char* dst = out.data();
  {
    py::gil_scoped_release nogil;
#pragma omp parallel for schedule(static) if (n > 256)
    for (int64_t i = 0; i < n; ++i) std::memcpy(dst + off[(size_t)i], src + i * w, (size_t)L[i]);
  }
  return py::bytes(out);
}

void bind_world(py::module_& m) {
  m.def("unpack_rows", &unpack_rows, "first lens[i] bytes of every uint8 row, concatenated");
  m.def("pack_rows", &pack_rows, "concatenated strings + lengths -> zero-padded uint8 rows (n, width)");
  m.def("get_neighbors", &get_neighbors);
  m.def("divide_cells", &divide_cells);
  m.def("move_cells", &move_cells);
  m.def("diffuse_stencil", &diffuse_stencil);
  m.def("diffuse_correct", &diffuse_correct);
}

}  // namespace ms_host
