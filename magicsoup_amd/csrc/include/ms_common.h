// Shared host/device definitions for the magicsoup_amd native core.
//
// This header is compiled twice: by g++ into the OpenMP host module (_host) and by hipcc for gfx950
// into the device module (_hip). Everything marked MS_HD is single-source between the two, so the
// CPU plumbing path and the GPU path run the same genome-translation logic.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define MS_HD __host__ __device__ __forceinline__
#else
#define MS_HD inline
#endif

namespace ms {

// Nucleotides are stored as ASCII bytes. (c >> 1) & 3 maps A,C,T,G -> 0,1,2,3 and complementing is
// an XOR with 2 (A<->T, C<->G). Codon index = 16*n0 + 4*n1 + n2.
MS_HD int nt_code(uint8_t c) { return (c >> 1) & 3; }
MS_HD int nt_comp(int code) { return code ^ 2; }

constexpr int kCodon = 3;
constexpr int kMaxDomTypeNts = 9;  // n_dom_type_codons <= 3 -> LUT of 4^9 entries at most

// Translation lookup tables (see models/genetics.py for how they are derived from a Genetics object).
struct TransTables {
  const uint8_t* is_start;      // 64 entries
  const uint8_t* is_stop;       // 64 entries
  const uint8_t* one_codon;     // 64 entries: 1-codon token (1..61), 0 for stop codons
  const uint8_t* dom_type;      // 4^dom_type_size entries: 0 none, 1 catalytic, 2 transporter, 3 regulatory
  const uint16_t* two_codon;    // 4096 entries: 2-codon token (1..3904), 0 if the first codon is a stop
  int dom_size;                 // nts per domain
  int dom_type_size;            // nts of the domain-type prefix
};

// Forward-strand view of a genome.
struct FwdSeq {
  const uint8_t* s;
  MS_HD int code(int i) const { return nt_code(s[i]); }
};

// Reverse-complement view: position i of the reverse complement without materialising it.
struct RevSeq {
  const uint8_t* s;
  int n;
  MS_HD int code(int i) const { return nt_comp(nt_code(s[n - 1 - i])); }
};

template <class Seq>
MS_HD int codon_at(const Seq& q, int i) {
  return (q.code(i) << 4) | (q.code(i + 1) << 2) | q.code(i + 2);
}

template <class Seq>
MS_HD int kmer_at(const Seq& q, int i, int k) {
  int v = 0;
  for (int j = 0; j < k; ++j) v = (v << 2) | q.code(i + j);
  return v;
}

// Extract the domains of one CDS [cds_start, cds_end) in parsing direction (reference
// rust/genetics.rs:58-123). Calls vis.domain(type, i0, i1, i2, i3, start, end) with CDS-relative
// offsets and returns whether the protein has at least one non-regulatory domain.
template <class Seq, class Vis>
MS_HD bool extract_domains(const Seq& q, int cds_start, int cds_end, const TransTables& T, Vis& vis) {
  const int n = cds_end - cds_start;
  const int ds = T.dom_size, dts = T.dom_type_size;
  bool useful = false;
  int i = 0;
  while (i + ds <= n) {
    const int s0 = cds_start + i;
    const int t = T.dom_type[kmer_at(q, s0, dts)];
    if (t != 0) {
      const int a = s0 + dts;
      const int i0 = T.one_codon[codon_at(q, a)];
      const int i1 = T.one_codon[codon_at(q, a + 3)];
      const int i2 = T.one_codon[codon_at(q, a + 6)];
      const int i3 = T.two_codon[(codon_at(q, a + 9) << 6) | codon_at(q, a + 12)];
      if (t != 3) useful = true;
      vis.domain(t, i0, i1, i2, i3, i, i + ds);
      i += ds;
    } else {
      i += kCodon;
    }
  }
  return useful;
}

// Scan one strand for coding regions and translate them (reference rust/genetics.rs:13-50 + 141-175).
//
// A CDS runs from a start codon to the first in-frame stop codon (stop included). A stop codon closes
// every start of its frame seen since that frame's previous stop, latest start first (the
// reference's stack pop order); CDSs shorter than dom_size are dropped. This is the stack-free
// formulation: at stop q we walk back over frame positions until the frame's previous stop.
//
// vis.begin(cds_start, cds_end, is_fwd) / vis.domain(...) / vis.end(keep) are called per CDS; keep is
// false for proteins without a catalytic or transporter domain.
template <class Seq, class Vis>
MS_HD void scan_strand(const Seq& q, int n, const TransTables& T, bool is_fwd, Vis& vis) {
  if (n < T.dom_size || n < kCodon) return;
  int last_stop[3] = {-1, -1, -1};
  for (int i = 0; i + kCodon <= n; ++i) {
    const int c = codon_at(q, i);
    if (T.is_start[c] || !T.is_stop[c]) continue;
    const int f = i % kCodon;
    const int j = i + kCodon;
    for (int p = i - kCodon; p > last_stop[f]; p -= kCodon) {
      if (!T.is_start[codon_at(q, p)]) continue;
      if (j - p < T.dom_size) continue;
      vis.begin(p, j, is_fwd);
      const bool keep = extract_domains(q, p, j, T, vis);
      vis.end(keep);
    }
    last_stop[f] = i;
  }
}

// Translate a genome: forward strand first, then its reverse complement.
template <class Vis>
MS_HD void translate_genome(const uint8_t* s, int n, const TransTables& T, Vis& vis) {
  FwdSeq f{s};
  scan_strand(f, n, T, true, vis);
  RevSeq r{s, n};
  scan_strand(r, n, T, false, vis);
}

// Visitor that only counts proteins and the largest domain count (first translation pass).
struct CountVisitor {
  int n_prots = 0;
  int max_doms = 0;
  int cur = 0;
  MS_HD void begin(int, int, bool) { cur = 0; }
  MS_HD void domain(int, int, int, int, int, int, int) { ++cur; }
  MS_HD void end(bool keep) {
    if (keep) {
      ++n_prots;
      if (cur > max_doms) max_doms = cur;
    }
  }
};

// Visitor writing dense tokens [P][D][5] for one genome (second translation pass). Domains of a
// dropped protein are overwritten by the next protein (slots are zero-filled beforehand).
struct TokenVisitor {
  int32_t* tok;  // this genome's [P][D][5] block, zero-initialised
  int P, D;
  int n_prots = 0;
  int cur = 0;
  MS_HD void begin(int, int, bool) { cur = 0; }
  MS_HD void domain(int t, int i0, int i1, int i2, int i3, int, int) {
    if (n_prots < P && cur < D) {
      int32_t* d = tok + ((size_t)n_prots * D + cur) * 5;
      d[0] = t; d[1] = i0; d[2] = i1; d[3] = i2; d[4] = i3;
    }
    ++cur;
  }
  MS_HD void end(bool keep) {
    if (keep) {
      ++n_prots;
    } else if (n_prots < P) {
      for (int k = 0; k < cur && k < D; ++k) {
        int32_t* d = tok + ((size_t)n_prots * D + k) * 5;
        d[0] = d[1] = d[2] = d[3] = d[4] = 0;
      }
    }
  }
};

}  // namespace ms
