// Native checkpoint IO: the reference's cells.fasta (python/magicsoup/world.py:813-819 writes
// ">{idx} {label}\n{genome}" entries joined by "\n"; :853-866 parses them back) straight from / to
// packed byte buffers -- the genomes and labels back to back plus their lengths, the layout the
// device pool hands out (strings.py PoolArena.packed) -- without one Python string per cell.
//
// fasta_write appends one block of entries (a rank's shard when a decomposed world's checkpoint is
// assembled: the first entry of a later block is preceded by the "\n" separator). fasta_parse reads
// a whole file with the reference's rules: split at every '>', strip each entry, skip empty ones;
// the label is the second whitespace-separated word of the first line, the genome the second line.
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <string_view>
#include <vector>

#include "host_common.h"

namespace ms_host {

using larr = py::array_t<int64_t, py::array::c_style>;
using u8arr = py::array_t<uint8_t, py::array::c_style>;

namespace {

std::vector<int64_t> offsets(const larr& lens, size_t total, const char* what) {
  const int64_t n = lens.shape(0);
  const int64_t* L = lens.data();
  std::vector<int64_t> off((size_t)n + 1, 0);
  for (int64_t i = 0; i < n; ++i) {
    if (L[i] < 0) throw std::invalid_argument(std::string(what) + ": negative length");
    off[(size_t)i + 1] = off[(size_t)i] + L[i];
  }
  if ((size_t)off[(size_t)n] != total) throw std::invalid_argument(std::string(what) + ": lengths do not add up");
  return off;
}

inline bool is_space(char c) { return c == ' ' || c == '\n' || c == '\t' || c == '\r' || c == '\v' || c == '\f'; }

}  // namespace

// Writes entries idx0 .. idx0 + n - 1 to `path` (mode "w" unless `append`); `lead_sep`: start with
// the "\n" that separates this block from entries already in the file. Returns the bytes written.
int64_t fasta_write(const std::string& path, int64_t idx0, u8arr genomes, larr glens, u8arr labels, larr llens,
                    bool append, bool lead_sep) {
  const int64_t n = glens.shape(0);
  if (llens.shape(0) != n) throw std::invalid_argument("fasta_write: genome and label counts differ");
  const auto go = offsets(glens, (size_t)genomes.size(), "fasta_write genomes");
  const auto lo = offsets(llens, (size_t)labels.size(), "fasta_write labels");
  const char* g = reinterpret_cast<const char*>(genomes.data());
  const char* l = reinterpret_cast<const char*>(labels.data());
  FILE* fh = std::fopen(path.c_str(), append ? "ab" : "wb");
  if (!fh) throw std::runtime_error("fasta_write: cannot open " + path);
  int64_t written = 0;
  {
    py::gil_scoped_release nogil;
    // entries are formatted into a buffer of ~4 MB and written in one call each
    std::string buf;
    buf.reserve(size_t(4) << 20);
    char num[32];
    for (int64_t i = 0; i < n; ++i) {
      if (i > 0 || lead_sep) buf.push_back('\n');
      const int k = std::snprintf(num, sizeof(num), ">%lld ", (long long)(idx0 + i));
      buf.append(num, (size_t)k);
      buf.append(l + lo[(size_t)i], (size_t)(lo[(size_t)i + 1] - lo[(size_t)i]));
      buf.push_back('\n');
      buf.append(g + go[(size_t)i], (size_t)(go[(size_t)i + 1] - go[(size_t)i]));
      if (buf.size() >= (size_t(4) << 20) || i == n - 1) {
        written += (int64_t)std::fwrite(buf.data(), 1, buf.size(), fh);
        buf.clear();
      }
    }
  }
  const bool bad = std::ferror(fh) != 0;
  std::fclose(fh);
  if (bad) throw std::runtime_error("fasta_write: write error on " + path);
  return written;
}

// (genome bytes, genome lengths, label bytes, label lengths) of every entry of a cells.fasta
py::tuple fasta_parse(const std::string& path) {
  FILE* fh = std::fopen(path.c_str(), "rb");
  if (!fh) throw std::runtime_error("fasta_parse: cannot open " + path);
  std::string text;
  {
    std::fseek(fh, 0, SEEK_END);
    const long sz = std::ftell(fh);
    std::fseek(fh, 0, SEEK_SET);
    text.resize(sz > 0 ? (size_t)sz : 0);
    if (sz > 0 && std::fread(text.data(), 1, (size_t)sz, fh) != (size_t)sz) {
      std::fclose(fh);
      throw std::runtime_error("fasta_parse: read error on " + path);
    }
    std::fclose(fh);
  }
  std::vector<char> gb, lb;
  std::vector<int64_t> gl, ll;
  {
    py::gil_scoped_release nogil;
    gb.reserve(text.size());
    const std::string_view all(text);
    size_t pos = 0;
    while (pos <= all.size()) {
      size_t next = all.find('>', pos);
      if (next == std::string_view::npos) next = all.size();
      std::string_view e = all.substr(pos, next - pos);
      pos = next + 1;
      size_t a = 0, b = e.size();
      while (a < b && is_space(e[a])) ++a;
      while (b > a && is_space(e[b - 1])) --b;
      e = e.substr(a, b - a);
      if (e.empty()) continue;
      const size_t nl = e.find('\n');
      const std::string_view head = e.substr(0, nl);
      // the second whitespace-separated word of the header (Python str.split())
      std::string_view label;
      {
        size_t i = 0, word = 0;
        while (i < head.size()) {
          while (i < head.size() && is_space(head[i])) ++i;
          const size_t s = i;
          while (i < head.size() && !is_space(head[i])) ++i;
          if (i > s) {
            if (word == 1) {
              label = head.substr(s, i - s);
              break;
            }
            ++word;
          }
        }
      }
      std::string_view seq;
      if (nl != std::string_view::npos) {
        const std::string_view rest = e.substr(nl + 1);
        seq = rest.substr(0, rest.find('\n'));
      }
      gb.insert(gb.end(), seq.begin(), seq.end());
      gl.push_back((int64_t)seq.size());
      lb.insert(lb.end(), label.begin(), label.end());
      ll.push_back((int64_t)label.size());
    }
  }
  u8arr g((py::ssize_t)gb.size()), l((py::ssize_t)lb.size());
  if (!gb.empty()) std::memcpy(g.mutable_data(), gb.data(), gb.size());
  if (!lb.empty()) std::memcpy(l.mutable_data(), lb.data(), lb.size());
  larr glo((py::ssize_t)gl.size()), llo((py::ssize_t)ll.size());
  if (!gl.empty()) std::memcpy(glo.mutable_data(), gl.data(), gl.size() * sizeof(int64_t));
  if (!ll.empty()) std::memcpy(llo.mutable_data(), ll.data(), ll.size() * sizeof(int64_t));
  return py::make_tuple(g, glo, l, llo);
}

void bind_io(py::module_& m) {
  m.def("fasta_write", &fasta_write, py::arg("path"), py::arg("idx0"), py::arg("genomes"), py::arg("glens"),
        py::arg("labels"), py::arg("llens"), py::arg("append") = false, py::arg("lead_sep") = false,
        "write '>{idx} {label}\\n{genome}' entries joined by '\\n' from packed bytes");
  m.def("fasta_parse", &fasta_parse, "cells.fasta -> (genome bytes, genome lens, label bytes, label lens)");
}

}  // namespace ms_host
