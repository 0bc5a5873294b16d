// gfx950 genome translation over the device genome arena.
//
// One thread per (genome, strand) runs the single-source scan of ms_common.h (the same code the
// OpenMP host path runs): pass 1 counts proteins and domains, pass 2 writes dense tokens
// (n, P, D, 5); reverse-strand proteins are placed after the forward-strand ones of their genome,
// which reproduces the reference's protein order (rust/genetics.rs:151-175).
#include "hip_common.h"

namespace msd {

struct DevTables {
  ms::TransTables t;
};

__global__ void __launch_bounds__(256) translate_count_kernel(int n, const int64_t* rows, const uint8_t* arena, int width,
                                                              const int32_t* lens, DevTables T, int32_t* nprot,
                                                              int32_t* ndom) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 2 * n) return;
  const int g = t >> 1, strand = t & 1;
  const int64_t r = rows[g];
  const uint8_t* s = arena + (size_t)r * width;
  const int L = lens[r];
  ms::CountVisitor v;
  if (strand == 0) {
    ms::FwdSeq q{s};
    ms::scan_strand(q, L, T.t, true, v);
  } else {
    ms::RevSeq q{s, L};
    ms::scan_strand(q, L, T.t, false, v);
  }
  nprot[t] = v.n_prots;
  ndom[t] = v.max_doms;
}

__global__ void __launch_bounds__(256) translate_write_kernel(int n, const int64_t* rows, const uint8_t* arena, int width,
                                                              const int32_t* lens, DevTables T, const int32_t* nprot,
                                                              int P, int D, int32_t* tokens) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 2 * n) return;
  const int g = t >> 1, strand = t & 1;
  const int64_t r = rows[g];
  const uint8_t* s = arena + (size_t)r * width;
  const int L = lens[r];
  const int off = strand == 0 ? 0 : nprot[2 * g];
  ms::TokenVisitor v{tokens + ((size_t)g * P + off) * D * 5, P - off, D};
  if (strand == 0) {
    ms::FwdSeq q{s};
    ms::scan_strand(q, L, T.t, true, v);
  } else {
    ms::RevSeq q{s, L};
    ms::scan_strand(q, L, T.t, false, v);
  }
}

static DevTables make_tables(const std::vector<uint8_t>& is_start, const std::vector<uint8_t>& is_stop,
                             const std::vector<uint8_t>& one_codon, uintptr_t dom_type, uintptr_t two_codon,
                             int dom_size, int dom_type_size) {
  if (is_start.size() != 64 || is_stop.size() != 64 || one_codon.size() != 64)
    throw std::invalid_argument("codon LUTs must have 64 entries");
  DevTables T{};
  for (int i = 0; i < 64; ++i) {
    T.t.is_start[i] = is_start[i];
    T.t.is_stop[i] = is_stop[i];
    T.t.one_codon[i] = one_codon[i];
  }
  T.t.dom_type = P_<uint8_t>(dom_type);
  T.t.two_codon = P_<uint16_t>(two_codon);
  T.t.dom_size = dom_size;
  T.t.dom_type_size = dom_type_size;
  return T;
}

void translate_count(int n, uintptr_t rows, uintptr_t arena, int width, uintptr_t lens, const std::vector<uint8_t>& st,
                     const std::vector<uint8_t>& sp, const std::vector<uint8_t>& oc, uintptr_t dom_type,
                     uintptr_t two_codon, int dom_size, int dom_type_size, uintptr_t nprot, uintptr_t ndom,
                     uintptr_t stream) {
  if (n <= 0) return;
  DevTables T = make_tables(st, sp, oc, dom_type, two_codon, dom_size, dom_type_size);
  translate_count_kernel<<<cdiv(2ll * n, 256), 256, 0, S_(stream)>>>(n, P_<int64_t>(rows), P_<uint8_t>(arena), width,
                                                                     P_<int32_t>(lens), T, P_<int32_t>(nprot),
                                                                     P_<int32_t>(ndom));
  MS_LAUNCH_CHECK();
}

void translate_write(int n, uintptr_t rows, uintptr_t arena, int width, uintptr_t lens, const std::vector<uint8_t>& st,
                     const std::vector<uint8_t>& sp, const std::vector<uint8_t>& oc, uintptr_t dom_type,
                     uintptr_t two_codon, int dom_size, int dom_type_size, uintptr_t nprot, int P, int D,
                     uintptr_t tokens, uintptr_t stream) {
  if (n <= 0) return;
  DevTables T = make_tables(st, sp, oc, dom_type, two_codon, dom_size, dom_type_size);
  translate_write_kernel<<<cdiv(2ll * n, 256), 256, 0, S_(stream)>>>(n, P_<int64_t>(rows), P_<uint8_t>(arena), width,
                                                                     P_<int32_t>(lens), T, P_<int32_t>(nprot), P, D,
                                                                     P_<int32_t>(tokens));
  MS_LAUNCH_CHECK();
}

}  // namespace msd
