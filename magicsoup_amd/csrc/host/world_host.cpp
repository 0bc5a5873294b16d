// Host (OpenMP) world geometry and map physics for the CPU plumbing path.
//
// Neighbour search, division and movement placement follow rust/world.rs:9-146 but replace the
// O(n) `positions.contains` scans with an O(1) occupancy lookup (a dense bitmap of the torus and a
// hash of occupied pixels -> cell index). The diffusion stencil / mass correction follow
// python/magicsoup/world.py:627-665 and 948-984.
#include <omp.h>

#include <algorithm>
#include <cmath>
#include <stdexcept>

#include "host_common.h"

namespace ms_host {

using iarr = py::array_t<int32_t, py::array::c_style>;
using farr = py::array_t<float, py::array::c_style>;

namespace {

struct Torus {
  int64_t m;
  std::vector<uint64_t> bits;
  explicit Torus(int64_t m_) : m(m_), bits((size_t)((m_ * m_ + 63) / 64), 0ull) {}
  int64_t key(int64_t x, int64_t y) const { return x * m + y; }
  bool get(int64_t x, int64_t y) const {
    const int64_t k = key(x, y);
    return (bits[(size_t)(k >> 6)] >> (k & 63)) & 1ull;
  }
  void set(int64_t x, int64_t y, bool v) {
    const int64_t k = key(x, y);
    if (v) bits[(size_t)(k >> 6)] |= 1ull << (k & 63);
    else bits[(size_t)(k >> 6)] &= ~(1ull << (k & 63));
  }
  // reference neighbour order (rust/util.rs:30-46): (w,n),(w,y),(w,s),(x,n),(x,s),(e,n),(e,y),(e,s)
  void nghbhd(int64_t x, int64_t y, int64_t out[8][2]) const {
    const int64_t e = (x + 1) % m, w = (x - 1 + m) % m, s = (y + 1) % m, n = (y - 1 + m) % m;
    const int64_t v[8][2] = {{w, n}, {w, y}, {w, s}, {x, n}, {x, s}, {e, n}, {e, y}, {e, s}};
    for (int i = 0; i < 8; ++i) {
      out[i][0] = v[i][0];
      out[i][1] = v[i][1];
    }
  }
};

}  // namespace

// All unique neighbour pairs (a < b) between `from` cells and `to` cells (Chebyshev distance 1 on
// the torus). Returns an int32 array (k, 2) sorted lexicographically.
iarr get_neighbors(iarr from_idxs, iarr to_idxs, iarr positions, int64_t map_size) {
  const int32_t* pos = positions.data();
  const int nf = (int)from_idxs.size(), nt = (int)to_idxs.size();
  const int32_t *fi = from_idxs.data(), *ti = to_idxs.data();
  std::unordered_map<int64_t, std::vector<int32_t>> at;  // pixel -> to-cells on it
  at.reserve((size_t)nt * 2);
  for (int i = 0; i < nt; ++i) {
    const int32_t c = ti[i];
    at[(int64_t)pos[2 * c] * map_size + pos[2 * c + 1]].push_back(c);
  }
  std::vector<std::pair<int32_t, int32_t>> pairs;
  Torus tor(1);
  tor.m = map_size;
  for (int i = 0; i < nf; ++i) {
    const int32_t c = fi[i];
    int64_t nb[8][2];
    tor.nghbhd(pos[2 * c], pos[2 * c + 1], nb);
    // the cell's own pixel can hold further to-cells only if positions were set by hand
    int64_t keys[9];
    for (int k = 0; k < 8; ++k) keys[k] = nb[k][0] * map_size + nb[k][1];
    keys[8] = (int64_t)pos[2 * c] * map_size + pos[2 * c + 1];
    std::sort(keys, keys + 9);
    const int64_t* kend = std::unique(keys, keys + 9);
    for (const int64_t* k = keys; k != kend; ++k) {
      auto it = at.find(*k);
      if (it == at.end()) continue;
      for (int32_t o : it->second) {
        if (o == c) continue;
        pairs.push_back({std::min(c, o), std::max(c, o)});
      }
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
py::tuple divide_cells(iarr cell_idxs, iarr positions, int64_t map_size) {
  const int32_t* pos = positions.data();
  const int n_all = (int)positions.shape(0), n = (int)cell_idxs.size();
  const int32_t* ci = cell_idxs.data();
  Torus occ(map_size);
  for (int i = 0; i < n_all; ++i) occ.set(pos[2 * i], pos[2 * i + 1], true);
  auto rng = item_engine(next_call_seed(), 0);
  std::vector<int32_t> parents, cpos;
  for (int i = 0; i < n; ++i) {
    const int32_t c = ci[i];
    int64_t nb[8][2];
    occ.nghbhd(pos[2 * c], pos[2 * c + 1], nb);
    int64_t free_[8][2];
    int nfree = 0;
    for (int k = 0; k < 8; ++k) {
      if (occ.get(nb[k][0], nb[k][1])) continue;
      bool dup = false;  // tiny maps repeat neighbours
      for (int q = 0; q < nfree; ++q) dup |= free_[q][0] == nb[k][0] && free_[q][1] == nb[k][1];
      if (dup) continue;
      free_[nfree][0] = nb[k][0];
      free_[nfree][1] = nb[k][1];
      ++nfree;
    }
    if (nfree == 0) continue;
    std::uniform_int_distribution<int> pick(0, nfree - 1);
    const int k = pick(rng);
    occ.set(free_[k][0], free_[k][1], true);
    parents.push_back(c);
    cpos.push_back((int32_t)free_[k][0]);
    cpos.push_back((int32_t)free_[k][1]);
  }
  iarr p((py::ssize_t)parents.size());
  std::copy(parents.begin(), parents.end(), p.mutable_data());
  iarr q({(py::ssize_t)parents.size(), (py::ssize_t)2});
  std::copy(cpos.begin(), cpos.end(), q.mutable_data());
  return py::make_tuple(p, q);
}

// Movement (rust/world.rs:102-146): non-moving cells are obstacles; moving cells, in list order,
// hop to a uniformly random free Moore neighbour. Returns (moved cell idxs, new positions).
py::tuple move_cells(iarr cell_idxs, iarr positions, int64_t map_size) {
  const int32_t* pos = positions.data();
  const int n_all = (int)positions.shape(0), n = (int)cell_idxs.size();
  const int32_t* ci = cell_idxs.data();
  Torus occ(map_size);
  for (int i = 0; i < n_all; ++i) occ.set(pos[2 * i], pos[2 * i + 1], true);
  auto rng = item_engine(next_call_seed(), 0);
  std::vector<int32_t> moved, npos;
  for (int i = 0; i < n; ++i) {
    const int32_t c = ci[i];
    const int64_t x = pos[2 * c], y = pos[2 * c + 1];
    int64_t nb[8][2];
    occ.nghbhd(x, y, nb);
    int64_t free_[8][2];
    int nfree = 0;
    for (int k = 0; k < 8; ++k) {
      if (occ.get(nb[k][0], nb[k][1])) continue;
      bool dup = false;
      for (int q = 0; q < nfree; ++q) dup |= free_[q][0] == nb[k][0] && free_[q][1] == nb[k][1];
      if (dup) continue;
      free_[nfree][0] = nb[k][0];
      free_[nfree][1] = nb[k][1];
      ++nfree;
    }
    if (nfree == 0) continue;
    std::uniform_int_distribution<int> pick(0, nfree - 1);
    const int k = pick(rng);
    occ.set(x, y, false);
    occ.set(free_[k][0], free_[k][1], true);
    moved.push_back(c);
    npos.push_back((int32_t)free_[k][0]);
    npos.push_back((int32_t)free_[k][1]);
  }
  iarr p((py::ssize_t)moved.size());
  std::copy(moved.begin(), moved.end(), p.mutable_data());
  iarr q({(py::ssize_t)moved.size(), (py::ssize_t)2});
  std::copy(npos.begin(), npos.end(), q.mutable_data());
  return py::make_tuple(p, q);
}

// One diffusion step of the molecule map (m, S, S) in place: 3x3 circular stencil with weights
// (a neighbours, b centre) per molecule, then the reference's global mass correction
// (before - after) / S^2 and clamp at 0. Sums are accumulated in double.
void diffuse(farr mol_map, std::vector<float> a_w, std::vector<float> b_w) {
  const int m = (int)mol_map.shape(0);
  const int64_t S = mol_map.shape(1);
  if (mol_map.shape(2) != S) throw std::invalid_argument("molecule map must be square");
  if ((int)a_w.size() != m || (int)b_w.size() != m) throw std::invalid_argument("one weight pair per molecule");
  float* base = mol_map.mutable_data();
  py::gil_scoped_release nogil;
  std::vector<float> out((size_t)(S * S));
  for (int mi = 0; mi < m; ++mi) {
    float* x = base + (size_t)mi * S * S;
    const float a = a_w[mi], b = b_w[mi];
    if (a == 0.0f && b == 1.0f) continue;  // identity kernel: conv, sums and correction are no-ops
    double before = 0.0, after = 0.0;
#pragma omp parallel for reduction(+ : before, after) schedule(static)
    for (int64_t i = 0; i < S; ++i) {
      const int64_t im = (i - 1 + S) % S, ip = (i + 1) % S;
      for (int64_t j = 0; j < S; ++j) {
        const int64_t jm = (j - 1 + S) % S, jp = (j + 1) % S;
        const float nsum = x[im * S + jm] + x[im * S + j] + x[im * S + jp] + x[i * S + jm] + x[i * S + jp] +
                           x[ip * S + jm] + x[ip * S + j] + x[ip * S + jp];
        const float v = b * x[i * S + j] + a * nsum;
        out[(size_t)(i * S + j)] = v;
        before += x[i * S + j];
        after += v;
      }
    }
    const float corr = (float)((before - after) / (double)(S * S));
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < S * S; ++k) {
      const float v = out[(size_t)k] + corr;
      x[k] = v < 0.0f ? 0.0f : v;
    }
  }
}

void bind_world(py::module_& m) {
  m.def("get_neighbors", &get_neighbors);
  m.def("divide_cells", &divide_cells);
  m.def("move_cells", &move_cells);
  m.def("diffuse", &diffuse);
}

}  // namespace ms_host
