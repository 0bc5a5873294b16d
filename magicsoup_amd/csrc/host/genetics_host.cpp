// Host (OpenMP) genome translation: the CPU counterpart of hip/genetics.hip, sharing the MS_HD scan
// in ms_common.h. Exposes the reference-compatible list outputs (rust/lib.rs:57-118) and dense token
// arrays for the parameter builder.
#include <omp.h>

#include <stdexcept>

#include "host_common.h"

namespace ms_host {

namespace {
std::atomic<uint64_t> g_seed{0x5EEDF00Dull};
std::atomic<uint64_t> g_calls{0};
}  // namespace

uint64_t next_call_seed() { return splitmix64(g_seed.load() + 0x9E37ull * (g_calls.fetch_add(1) + 1)); }
void set_seed(uint64_t seed) {
  g_seed.store(seed);
  g_calls.store(0);
}
// (seed, calls drawn): the whole state of the host streams, for checkpoints
std::pair<uint64_t, uint64_t> get_rng_state() { return {g_seed.load(), g_calls.load()}; }
void set_rng_state(uint64_t seed, uint64_t calls) {
  g_seed.store(seed);
  g_calls.store(calls);
}

int seq_index(const std::string& s) {
  int v = 0;
  for (char c : s) v = (v << 2) | ms::nt_code(static_cast<uint8_t>(c));
  return v;
}

HostTables::HostTables(const std::vector<std::string>& start_codons,
                       const std::vector<std::string>& stop_codons,
                       const std::unordered_map<std::string, int>& domain_map,
                       const std::unordered_map<std::string, int>& one_codon_map,
                       const std::unordered_map<std::string, int>& two_codon_map, int dom_size,
                       int dom_type_size) {
  if (dom_type_size <= 0 || dom_type_size > ms::kMaxDomTypeNts)
    throw std::invalid_argument("dom_type_size must be in 1..9 nucleotides");
  dom_type.assign(size_t(1) << (2 * dom_type_size), 0);
  two_codon.assign(4096, 0);
  for (int i = 0; i < 64; ++i) is_start[i] = is_stop[i] = one_codon[i] = 0;
  t.is_start = is_start;
  t.is_stop = is_stop;
  t.one_codon = one_codon;
  for (auto& c : start_codons) {
    if (c.size() != 3) throw std::invalid_argument("start codons must have 3 nucleotides");
    is_start[seq_index(c)] = 1;
  }
  for (auto& c : stop_codons) {
    if (c.size() != 3) throw std::invalid_argument("stop codons must have 3 nucleotides");
    is_stop[seq_index(c)] = 1;
  }
  for (auto& kv : domain_map)
    if ((int)kv.first.size() == dom_type_size) dom_type[seq_index(kv.first)] = (uint8_t)kv.second;
  for (auto& kv : one_codon_map)
    if (kv.first.size() == 3) one_codon[seq_index(kv.first)] = (uint8_t)kv.second;
  for (auto& kv : two_codon_map)
    if (kv.first.size() == 6) two_codon[seq_index(kv.first)] = (uint16_t)kv.second;
  t.dom_type = dom_type.data();
  t.two_codon = two_codon.data();
  t.dom_size = dom_size;
  t.dom_type_size = dom_type_size;
}

namespace {

struct Dom {
  int t, i0, i1, i2, i3, start, end;
};
struct Prot {
  std::vector<Dom> doms;
  int cds_start, cds_end;
  bool is_fwd;
};

// Collects whole proteins for the list-returning API.
struct ListVisitor {
  std::vector<Prot>* out;
  Prot cur;
  void begin(int s, int e, bool fwd) {
    cur.doms.clear();
    cur.cds_start = s;
    cur.cds_end = e;
    cur.is_fwd = fwd;
  }
  void domain(int t, int i0, int i1, int i2, int i3, int s, int e) { cur.doms.push_back({t, i0, i1, i2, i3, s, e}); }
  void end(bool keep) {
    if (keep) out->push_back(cur);
  }
};

py::list proteins_to_py(const std::vector<Prot>& prots) {
  py::list out;
  for (auto& p : prots) {
    py::list doms;
    for (auto& d : p.doms)
      doms.append(py::make_tuple(py::make_tuple(d.t, d.i0, d.i1, d.i2, d.i3), d.start, d.end));
    out.append(py::make_tuple(doms, p.cds_start, p.cds_end, p.is_fwd));
  }
  return out;
}

std::vector<std::string> to_strings(const py::list& genomes) {
  std::vector<std::string> v;
  v.reserve(genomes.size());
  for (auto g : genomes) v.push_back(g.cast<std::string>());
  return v;
}

}  // namespace

// list[str] -> list[list[ProteinSpecType]] (reference _lib.translate_genomes)
py::list translate_genomes(const HostTables& T, const py::list& genomes) {
  std::vector<std::string> seqs = to_strings(genomes);
  const int n = (int)seqs.size();
  std::vector<std::vector<Prot>> res(n);
  {
    py::gil_scoped_release nogil;
#pragma omp parallel for schedule(dynamic, 16)
    for (int i = 0; i < n; ++i) {
      ListVisitor v{&res[i], {}};
      ms::translate_genome(reinterpret_cast<const uint8_t*>(seqs[i].data()), (int)seqs[i].size(), T.t, v);
    }
  }
  py::list out;
  for (int i = 0; i < n; ++i) out.append(proteins_to_py(res[i]));
  return out;
}

// Dense translation of a packed genome arena for the parameter builder: returns
// (tokens int32 [n, P, D, 5], n_prots int32 [n]). P, D are the maxima over the batch (>= 1).
py::tuple translate_tokens(const HostTables& T, py::array_t<uint8_t, py::array::c_style> arena,
                           py::array_t<int32_t, py::array::c_style> lengths) {
  if (arena.ndim() != 2) throw std::invalid_argument("arena must be 2D [n, L]");
  const int n = (int)arena.shape(0);
  const int64_t L = arena.shape(1);
  if (lengths.size() < n) throw std::invalid_argument("lengths too short");
  const uint8_t* a = arena.data();
  const int32_t* lens = lengths.data();
  std::vector<int32_t> nprots(n), ndoms(n);
  {
    py::gil_scoped_release nogil;
#pragma omp parallel for schedule(dynamic, 16)
    for (int i = 0; i < n; ++i) {
      ms::CountVisitor c;
      ms::translate_genome(a + i * L, lens[i], T.t, c);
      nprots[i] = c.n_prots;
      ndoms[i] = c.max_doms;
    }
  }
  int P = 1, D = 1;
  for (int i = 0; i < n; ++i) {
    P = std::max(P, nprots[i]);
    D = std::max(D, ndoms[i]);
  }
  py::array_t<int32_t> tokens({(py::ssize_t)n, (py::ssize_t)P, (py::ssize_t)D, (py::ssize_t)5});
  py::array_t<int32_t> np_out(n);
  int32_t* tk = tokens.mutable_data();
  std::fill(tk, tk + (size_t)n * P * D * 5, 0);
  {
    py::gil_scoped_release nogil;
#pragma omp parallel for schedule(dynamic, 16)
    for (int i = 0; i < n; ++i) {
      ms::TokenVisitor v{tk + (size_t)i * P * D * 5, P, D};
      ms::translate_genome(a + i * L, lens[i], T.t, v);
    }
  }
  std::copy(nprots.begin(), nprots.end(), np_out.mutable_data());
  return py::make_tuple(tokens, np_out);
}

// ---- reference-compatible single-purpose helpers (rust/lib.rs:57-92) ----

py::list get_coding_regions(const std::string& seq, int min_cds_size, const std::vector<std::string>& starts,
                            const std::vector<std::string>& stops, bool is_fwd) {
  uint8_t is_start[64] = {0}, is_stop[64] = {0};
  for (auto& c : starts) is_start[seq_index(c)] = 1;
  for (auto& c : stops) is_stop[seq_index(c)] = 1;
  py::list out;
  const int n = (int)seq.size();
  if (n < min_cds_size || n < 3) return out;
  ms::FwdSeq q{reinterpret_cast<const uint8_t*>(seq.data())};
  int last_stop[3] = {-1, -1, -1};
  for (int i = 0; i + 3 <= n; ++i) {
    const int c = ms::codon_at(q, i);
    if (is_start[c] || !is_stop[c]) continue;
    const int f = i % 3, j = i + 3;
    for (int p = i - 3; p > last_stop[f]; p -= 3)
      if (is_start[ms::codon_at(q, p)] && j - p >= min_cds_size) out.append(py::make_tuple(p, j, is_fwd));
    last_stop[f] = i;
  }
  return out;
}

py::list extract_domains(const std::string& genome, const std::vector<std::tuple<int, int, bool>>& cdss,
                         int dom_size, int dom_type_size,
                         const std::unordered_map<std::string, int>& dom_type_map,
                         const std::unordered_map<std::string, int>& one_codon_map,
                         const std::unordered_map<std::string, int>& two_codon_map) {
  HostTables T({}, {}, dom_type_map, one_codon_map, two_codon_map, dom_size, dom_type_size);
  std::vector<Prot> prots;
  ListVisitor v{&prots, {}};
  ms::FwdSeq q{reinterpret_cast<const uint8_t*>(genome.data())};
  for (auto& cds : cdss) {
    v.begin(std::get<0>(cds), std::get<1>(cds), std::get<2>(cds));
    bool keep = ms::extract_domains(q, std::get<0>(cds), std::get<1>(cds), T.t, v);
    v.end(keep);
  }
  return proteins_to_py(prots);
}

std::string reverse_complement(const std::string& seq) {
  std::string out;
  out.reserve(seq.size());
  for (auto it = seq.rbegin(); it != seq.rend(); ++it) {
    switch (*it) {
      case 'A': out.push_back('T'); break;
      case 'T': out.push_back('A'); break;
      case 'C': out.push_back('G'); break;
      case 'G': out.push_back('C'); break;
      default: break;  // non-nucleotide characters are dropped
    }
  }
  return out;
}

void bind_genetics(py::module_& m) {
  py::class_<HostTables>(m, "TranslationTables")
      .def(py::init<const std::vector<std::string>&, const std::vector<std::string>&,
                    const std::unordered_map<std::string, int>&, const std::unordered_map<std::string, int>&,
                    const std::unordered_map<std::string, int>&, int, int>(),
           py::arg("start_codons"), py::arg("stop_codons"), py::arg("domain_map"), py::arg("one_codon_map"),
           py::arg("two_codon_map"), py::arg("dom_size"), py::arg("dom_type_size"))
      .def("translate_genomes", &translate_genomes, py::arg("genomes"))
      .def("translate_tokens", &translate_tokens, py::arg("arena"), py::arg("lengths"))
      .def("luts", [](const HostTables& T) {
        // (is_start[64], is_stop[64], one_codon[64], dom_type[4^k], two_codon[4096]) for device upload
        py::array_t<uint8_t> st(64), sp(64), oc(64);
        std::copy(T.t.is_start, T.t.is_start + 64, st.mutable_data());
        std::copy(T.t.is_stop, T.t.is_stop + 64, sp.mutable_data());
        std::copy(T.t.one_codon, T.t.one_codon + 64, oc.mutable_data());
        py::array_t<uint8_t> dt(T.dom_type.size());
        std::copy(T.dom_type.begin(), T.dom_type.end(), dt.mutable_data());
        py::array_t<int16_t> tc(T.two_codon.size());
        std::copy(T.two_codon.begin(), T.two_codon.end(), reinterpret_cast<uint16_t*>(tc.mutable_data()));
        return py::make_tuple(st, sp, oc, dt, tc);
      })
      .def_property_readonly("dom_size", [](const HostTables& T) { return T.t.dom_size; })
      .def_property_readonly("dom_type_size", [](const HostTables& T) { return T.t.dom_type_size; });
  m.def("get_coding_regions", &get_coding_regions);
  m.def("extract_domains", &extract_domains);
  m.def("reverse_complement", &reverse_complement);
  m.def("set_seed", &set_seed, "Seed the host RNG streams (mutations, placement).");
  m.def("get_rng_state", &get_rng_state, "(seed, calls) of the host RNG streams");
  m.def("set_rng_state", &set_rng_state, "restore a get_rng_state() value");
}

}  // namespace ms_host
