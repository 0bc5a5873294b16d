// Host (OpenMP) point mutations and recombinations (reference rust/mutations.rs:11-154).
//
// Per work item an independent mt19937_64 is derived from the call seed and the item index, so
// results are reproducible for a given ms.set_seed() and independent of the thread schedule.
#include <omp.h>

#include <algorithm>
#include <deque>
#include <string_view>

#include "host_common.h"

namespace ms_host {

namespace {

const char kNts[4] = {'A', 'C', 'T', 'G'};

// k distinct sorted positions in [0, n) (Floyd's algorithm; k <= n).
std::vector<int64_t> sample_sorted(std::mt19937_64& rng, int64_t n, int64_t k) {
  std::vector<int64_t> out;
  out.reserve(k);
  if (k * 4 >= n) {  // dense: partial shuffle
    std::vector<int64_t> all(n);
    for (int64_t i = 0; i < n; ++i) all[i] = i;
    for (int64_t i = 0; i < k; ++i) {
      std::uniform_int_distribution<int64_t> d(i, n - 1);
      std::swap(all[i], all[d(rng)]);
    }
    out.assign(all.begin(), all.begin() + k);
  } else {
    std::vector<int64_t> chosen;
    chosen.reserve(k);
    for (int64_t j = n - k; j < n; ++j) {
      std::uniform_int_distribution<int64_t> d(0, j);
      int64_t t = d(rng);
      if (std::find(chosen.begin(), chosen.end(), t) != chosen.end()) t = j;
      chosen.push_back(t);
    }
    out = std::move(chosen);
  }
  std::sort(out.begin(), out.end());
  return out;
}

int64_t poisson(std::mt19937_64& rng, double lam) {
  if (!(lam > 0.0)) return 0;
  std::poisson_distribution<int64_t> d(lam);
  return d(rng);
}

// Number of mutations drawn for a sequence of length len (the first draw of mutate_one).
int64_t draw_mutations(std::mt19937_64& rng, int64_t len, double p) {
  if (len < 1) return 0;
  return std::min(poisson(rng, p * (double)len), len);
}

// Apply k >= 1 drawn point mutations to one sequence.
void apply_mutations(std::string& seq, int64_t k, std::mt19937_64& rng, double p_indel, double p_del) {
  const int64_t len = (int64_t)seq.size();
  std::vector<int64_t> pos = sample_sorted(rng, len, k);
  std::bernoulli_distribution indel(p_indel), del(p_del);
  std::uniform_int_distribution<int> nt(0, 3);
  int64_t offset = 0;
  for (int64_t idx : pos) {
    const int64_t at = idx + offset;
    if (indel(rng)) {
      if (del(rng)) {
        seq.erase((size_t)at, 1);
        offset -= 1;
      } else {
        seq.insert(seq.begin() + at, kNts[nt(rng)]);
        offset += 1;
      }
    } else {
      seq[(size_t)at] = kNts[nt(rng)];
    }
  }
}

// Apply point mutations to one sequence; returns false if no mutation was drawn.
bool mutate_one(std::string& seq, std::mt19937_64& rng, double p, double p_indel, double p_del) {
  const int64_t k = draw_mutations(rng, (int64_t)seq.size(), p);
  if (k < 1) return false;
  apply_mutations(seq, k, rng, p_indel, p_del);
  return true;
}

// Recombine one pair; returns false if no strand break was drawn.
bool recombine_one(std::string_view s0, std::string_view s1, std::mt19937_64& rng, double p,
                   std::string& o0, std::string& o1) {
  const int64_t n0 = (int64_t)s0.size(), n1 = (int64_t)s1.size(), nb = n0 + n1;
  if (nb < 1) return false;
  int64_t k = poisson(rng, p * (double)nb);
  if (k < 1) return false;
  k = std::min(k, nb);
  std::vector<int64_t> cuts = sample_sorted(rng, nb, k);
  std::vector<std::pair<const std::string_view*, std::pair<int64_t, int64_t>>> parts;
  parts.reserve(k + 2);
  int64_t i = 0;
  for (int64_t c : cuts)
    if (c < n0) {
      parts.push_back({&s0, {i, c}});
      i = c;
    }
  parts.push_back({&s0, {i, n0}});
  i = 0;
  for (int64_t c : cuts)
    if (c >= n0) {
      parts.push_back({&s1, {i, c - n0}});
      i = c - n0;
    }
  parts.push_back({&s1, {i, n1}});
  std::shuffle(parts.begin(), parts.end(), rng);
  std::uniform_int_distribution<size_t> split(0, parts.size() - 1);
  const size_t s = split(rng);
  o0.clear();
  o1.clear();
  for (size_t j = 0; j < parts.size(); ++j) {
    auto& pr = parts[j];
    std::string& dst = j < s ? o0 : o1;
    dst.append(pr.first->substr((size_t)pr.second.first, (size_t)(pr.second.second - pr.second.first)));
  }
  return true;
}

}  // namespace

// Borrowed views of Python str items: a compact str's UTF-8 buffer is read in place (no copy; the
// caller's list keeps the objects alive for the call), anything else is converted into `owned`.
std::string_view seq_view(PyObject* o, std::deque<std::string>& owned) {
  if (PyUnicode_Check(o)) {
    Py_ssize_t n = 0;
    const char* d = PyUnicode_AsUTF8AndSize(o, &n);
    if (d == nullptr) throw py::error_already_set();
    return {d, (size_t)n};
  }
  owned.push_back(py::reinterpret_borrow<py::object>(o).cast<std::string>());
  return owned.back();
}

// list[str] -> list[(str, idx)] of mutated sequences (reference _lib.point_mutations). Only the
// sequences that draw a mutation are copied: at p ~ 1e-6 that is a few in 10k.
py::list point_mutations(const py::list& seqs, double p, double p_indel, double p_del) {
  const int n = (int)seqs.size();
  std::deque<std::string> owned;
  std::vector<std::string_view> v(n);
  for (int i = 0; i < n; ++i) v[i] = seq_view(PyList_GET_ITEM(seqs.ptr(), i), owned);
  std::vector<std::string> res(n);
  std::vector<uint8_t> hit(n, 0);
  const uint64_t cs = next_call_seed();
  {
    py::gil_scoped_release nogil;
#pragma omp parallel for schedule(static, 256)
    for (int i = 0; i < n; ++i) {
      auto rng = item_engine(cs, (uint64_t)i);
      const int64_t k = draw_mutations(rng, (int64_t)v[i].size(), p);
      if (k < 1) continue;
      res[i].assign(v[i]);
      apply_mutations(res[i], k, rng, p_indel, p_del);
      hit[i] = 1;
    }
  }
  py::list out;
  for (int i = 0; i < n; ++i)
    if (hit[i]) out.append(py::make_tuple(res[i], i));
  return out;
}

// list[(str, str)] -> list[(str, str, idx)] (reference _lib.recombinations); inputs are read in place.
py::list recombinations(const py::list& pairs, double p) {
  const int n = (int)pairs.size();
  std::deque<std::string> owned;
  std::vector<std::string_view> a(n), b(n);
  for (int i = 0; i < n; ++i) {
    PyObject* t = PyList_GET_ITEM(pairs.ptr(), i);
    if (PyTuple_Check(t) && PyTuple_GET_SIZE(t) == 2) {
      a[i] = seq_view(PyTuple_GET_ITEM(t, 0), owned);
      b[i] = seq_view(PyTuple_GET_ITEM(t, 1), owned);
    } else {
      py::sequence sq = py::reinterpret_borrow<py::sequence>(t);
      if (sq.size() != 2) throw py::value_error("recombinations: every item must be a pair of sequences");
      owned.push_back(sq[0].cast<std::string>());
      a[i] = owned.back();
      owned.push_back(sq[1].cast<std::string>());
      b[i] = owned.back();
    }
  }
  std::vector<std::string> oa(n), ob(n);
  std::vector<uint8_t> hit(n, 0);
  const uint64_t cs = next_call_seed();
  {
    py::gil_scoped_release nogil;
#pragma omp parallel for schedule(static, 256)
    for (int i = 0; i < n; ++i) {
      auto rng = item_engine(cs, (uint64_t)i);
      hit[i] = recombine_one(a[i], b[i], rng, p, oa[i], ob[i]);
    }
  }
  py::list out;
  for (int i = 0; i < n; ++i)
    if (hit[i]) out.append(py::make_tuple(oa[i], ob[i], i));
  return out;
}

// Arena form used by the CPU World path: mutate rows of a [n, L] byte arena in place where the new
// length fits, and report (mutated row ids, new lengths, rows that overflowed L as (id, bytes)).
py::tuple point_mutations_arena(py::array_t<uint8_t, py::array::c_style> arena,
                                py::array_t<int32_t, py::array::c_style> lengths, double p, double p_indel,
                                double p_del) {
  const int n = (int)arena.shape(0);
  const int64_t L = arena.shape(1);
  uint8_t* a = arena.mutable_data();
  int32_t* lens = lengths.mutable_data();
  std::vector<uint8_t> hit(n, 0);
  std::vector<std::string> overflow(n);
  const uint64_t cs = next_call_seed();
  {
    py::gil_scoped_release nogil;
#pragma omp parallel for schedule(static, 256)
    for (int i = 0; i < n; ++i) {
      auto rng = item_engine(cs, (uint64_t)i);
      // cheap rejection first: most genomes draw zero mutations
      std::string s(reinterpret_cast<const char*>(a + i * L), (size_t)lens[i]);
      if (!mutate_one(s, rng, p, p_indel, p_del)) continue;
      hit[i] = 1;
      if ((int64_t)s.size() <= L) {
        std::copy(s.begin(), s.end(), a + i * L);
        lens[i] = (int32_t)s.size();
      } else {
        overflow[i] = std::move(s);
      }
    }
  }
  std::vector<int32_t> ids;
  py::list ovf;
  for (int i = 0; i < n; ++i) {
    if (!hit[i]) continue;
    ids.push_back(i);
    if (!overflow[i].empty()) ovf.append(py::make_tuple(i, py::bytes(overflow[i])));
  }
  py::array_t<int32_t> out_ids((py::ssize_t)ids.size());
  std::copy(ids.begin(), ids.end(), out_ids.mutable_data());
  return py::make_tuple(out_ids, ovf);
}

void bind_mutations(py::module_& m) {
  m.def("point_mutations", &point_mutations, py::arg("seqs"), py::arg("p"), py::arg("p_indel"), py::arg("p_del"));
  m.def("recombinations", &recombinations, py::arg("seq_pairs"), py::arg("p"));
  m.def("point_mutations_arena", &point_mutations_arena);
}

}  // namespace ms_host
