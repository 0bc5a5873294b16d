// Device genome pipeline issued from C++ (magicsoup_amd/ops/genome_pipeline.py).
//
// mutate_cells() / recombinate_cells() over all cells run a fixed chain of ~15 dependent kernels
// whose item counts stay on the device (draws -> selection -> apply -> arena commit -> translation
// -> fresh parameter rows -> parameter build -> status). Issuing that chain from Python cost more
// host time than the whole chain takes on the GPU (~180 us vs ~40 us at 6k cells), which is what a
// rank of a multi-GPU job waits on. Here Python fills three small descriptor objects (arena and
// counters, kinetics storage + LUTs, translation LUTs) and makes one call; the launches, scratch
// layout and status slot are handled in C++.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <tuple>

#include "hip_common.h"
#include "params.h"
#include "bind_util.h"

namespace py = pybind11;

namespace msd {

// ---- launchers defined in the other translation units
void rec_slots(int n, uintptr_t pos, int R, int C, int r_lo, int r_hi, int wrap, uintptr_t idx_map, uintptr_t lens,
               uintptr_t lw_word, double p, uint64_t seed, uint64_t call, int kcap, uintptr_t gflags,
               uintptr_t opflags, uintptr_t keys, uintptr_t k, uintptr_t sel, uintptr_t out_dev, int cap,
               uintptr_t cand, uintptr_t stream, uintptr_t na, uintptr_t nb);
void select_indices_dev(long long n, int kind, uintptr_t src, uintptr_t vals, uintptr_t sel, uintptr_t rest,
                        uintptr_t out_dev, uintptr_t stream);
void cap_skip(uintptr_t dn, int cap, uintptr_t gflags, uintptr_t opflags, uintptr_t stream);
int status_write(uintptr_t dcnt, uintptr_t opflags, uintptr_t d_rows, uintptr_t cnt, uintptr_t stream);
void gather_dev(int cap, uintptr_t dn, uintptr_t idx, uintptr_t src, uintptr_t dst, uintptr_t stream);
void translate_fused(int n, uintptr_t rows, uintptr_t arena, uintptr_t off, int width, uintptr_t lens, uintptr_t luts,
                     uintptr_t dom_type, int dt_entries, uintptr_t two_codon, int dom_size, int dom_type_size,
                     uintptr_t nprot, uintptr_t ndom, int P, int D, uintptr_t tokens, uintptr_t long_list,
                     uintptr_t long_count, uintptr_t dn, uintptr_t stream);
void translate_fused_long(int lcap, uintptr_t rows, uintptr_t arena, uintptr_t off, int width, uintptr_t lens,
                          uintptr_t luts,
                          uintptr_t dom_type, int dt_entries, uintptr_t two_codon, int dom_size, int dom_type_size,
                          uintptr_t nprot, uintptr_t ndom, int P, int D, uintptr_t tokens, uintptr_t long_list,
                          uintptr_t gslot, uintptr_t dn, uintptr_t stream);
size_t translate_slot_bytes(int width);
void build_params(int n, int P, int D, int Pt, int s, uintptr_t tokens, uintptr_t rows, uintptr_t vmax_w, int nw,
                  uintptr_t km_w, int nk, uintptr_t signs, int nsg, uintptr_t hills, int nh, uintptr_t RM,
                  uintptr_t TM, uintptr_t EM, int nv, uintptr_t energies, float abs_temp, float gas, uintptr_t N,
                  uintptr_t Nf, uintptr_t Nb, uintptr_t A, uintptr_t Kmr, uintptr_t Kmf, uintptr_t Kmb,
                  uintptr_t Vmax, uintptr_t Ke, uintptr_t nprot, uintptr_t W, uintptr_t Q, uintptr_t overflow,
                  uintptr_t dn, uintptr_t roff, uintptr_t stream);
int translate_lds_max();  // genetics.hip: the longest genome of the LDS translation pass
void mut_count_select(int n, uintptr_t lens, double p, uint64_t seed, uint64_t call, uintptr_t k, int kcap,
                      uintptr_t gflags, uintptr_t opflags, uintptr_t sel, uintptr_t out_dev, int cap, uintptr_t cand,
                      uintptr_t stream, uintptr_t na, uintptr_t nb);
void mut_count(int n, uintptr_t rows, uintptr_t lens, double p, uint64_t seed, uint64_t call, uintptr_t k, int kcap,
               uintptr_t gflags, uintptr_t opflags, uintptr_t stream);
void mut_apply(int nsel, uintptr_t dn, uintptr_t sel, uintptr_t rows, uintptr_t arena, uintptr_t off, uintptr_t lens,
               uintptr_t k, double p_indel, double p_del, uint64_t seed, uint64_t call, uintptr_t out, int out_width,
               uintptr_t out_len, uintptr_t stream);
void rec_count_keys(int n, uintptr_t keys, uintptr_t lens, double p, uint64_t seed, uint64_t call, uintptr_t k,
                    uintptr_t tot, int kcap, uintptr_t gflags, uintptr_t opflags, uintptr_t stream,
                    uintptr_t lw_word);
void rec_apply(int nsel, uintptr_t dn, uintptr_t sel, uintptr_t pairs, uintptr_t keys, uintptr_t arena, uintptr_t off,
               uintptr_t lens, uintptr_t k, uint64_t seed, uint64_t call, uintptr_t parts, int parts_cap, uintptr_t out,
               int out_width, uintptr_t out_len, uintptr_t out_rows, uintptr_t stream);
void arena_scatter(int k, uintptr_t dn, int dn_mul, uintptr_t rows, uintptr_t src, int src_width, uintptr_t src_len,
                   uintptr_t pool, uintptr_t off, uintptr_t top, long long pool_cap, int width, uintptr_t lens,
                   uintptr_t mark, uint64_t gen, uintptr_t flags, uintptr_t gflags, uintptr_t opflags,
                   uintptr_t stream);

void select_indices_capped(long long n, int kind, uintptr_t src, uintptr_t sel, uintptr_t out_dev, int cap,
                           uintptr_t gflags, uintptr_t opflags, uintptr_t stream);
void arena_scatter_app(int k, uintptr_t dn, int dn_mul, uintptr_t rows, uintptr_t src, int src_width, uintptr_t src_len,
                       uintptr_t pool, uintptr_t off, uintptr_t top, long long pool_cap, int width, uintptr_t lens,
                       uintptr_t mark, uint64_t gen, uintptr_t gflags, uintptr_t opflags, uintptr_t cand,
                       uintptr_t stream);
int* append_counter(hipStream_t s);
void sel_sort(uintptr_t cand, int* cnt, int cap, uintptr_t sel, uintptr_t out_dev, uintptr_t gflags, uintptr_t opflags,
              hipStream_t s, uintptr_t gather);
int sel_sort_cap();
extern int g_mut_append;

std::pair<long long*, int> status_slot();
long long* status_bad_dev(int slot);
int status_bad_cap();

// ---- fused small steps of the rebuild chain
// token rows of the live items cleared and the long-genome counter reset, one launch
__global__ void __launch_bounds__(256) gp_zero_kernel(int cap, const int* dn, long long row, int32_t* buf,
                                                      int32_t* long_count) {
  if (blockIdx.x == 0 && threadIdx.x == 0) *long_count = 0;
  const long long total = (long long)min(*dn, cap) * row;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x)
    buf[i] = 0;
}

// One workgroup: proteome-shape checks, fresh parameter records (params.h: each cell's proteins
// as consecutive records from the bump counter *rtop, which the kinetics storage owns) and the
// call's status {rebuilt, op flags, record counter, count} into its pinned slot. A cell whose
// records do not fit below rec_cap keeps its old ones and is flagged for a host rebuild. A cell
// whose proteome outgrew the token slots (more than Pcap proteins or Dcap domains in one), or whose
// long genome found no global translation slot, is built from what fit and listed in the call's
// pinned overflow list {count, cell...} for a host rebuild of just those cells (kFlagPartialBit);
// a list that overflows falls back to the whole call (kFlagTranslateBit).
constexpr int kFlagTranslateBit = 1, kFlagRowsBit = 4, kFlagPartialBit = 32;  // select.hip DevFlag
__global__ void __launch_bounds__(1024) gp_check_assign_kernel(int cap, int lcap, const int* dn, const int32_t* counts,
                                                               const int32_t* ndom, const int32_t* long_list,
                                                               const int32_t* long_count, int32_t* per, int Pcap,
                                                               int Dcap, const int64_t* cells, int64_t* slot,
                                                               long long* rtop, long long rec_cap, int64_t* roff,
                                                               int* opflags, const int* stat_cnt, long long* status,
                                                               long long* bad, int bad_cap) {
  __shared__ int nbad;
  const int n = min(*dn, cap);
  if (threadIdx.x == 0) {
    nbad = 0;
    if (*dn > cap) atomicOr(opflags, 2);  // kFlagCapacity
  }
  __syncthreads();
  for (int j = threadIdx.x; j < n; j += blockDim.x) {
    const int p = counts[2 * j] + counts[2 * j + 1];
    if (p > Pcap || ndom[2 * j] > Dcap || ndom[2 * j + 1] > Dcap) {
      const int b = atomicAdd(&nbad, 1);
      if (b < bad_cap) bad[1 + b] = cells[j];
    }
    per[j] = p < Pcap ? p : Pcap;
  }
  // (long genomes past the global slots: not translated, their counts are stale)
  for (int i = lcap + threadIdx.x; i < min(*long_count, n); i += blockDim.x) {
    const int b = atomicAdd(&nbad, 1);
    if (b < bad_cap) bad[1 + b] = cells[long_list[i]];
  }
  __syncthreads();
  if (threadIdx.x == 0 && nbad > 0) atomicOr(opflags, nbad > bad_cap ? kFlagTranslateBit : kFlagPartialBit);
  assign_records_block(n, per, cells, slot, rtop, rec_cap, Pcap, roff, opflags, kFlagRowsBit);
  __syncthreads();
  if (threadIdx.x == 0) {
    bad[0] = min(nbad, bad_cap);
    status[0] = *dn;
    status[1] = __hip_atomic_load(opflags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    status[2] = *rtop;
    status[3] = *stat_cnt;
  }
}

// ---- descriptors filled from Python
struct GpArena {  // genome pool + the pipeline's device counters
  uintptr_t data = 0, lens = 0, off = 0, top = 0;  // pool bytes, per-cell lengths / offsets, bump counter
  long long pool_cap = 0;
  int width = 0, n = 0;  // width: the genome length bound of the call's scratch (PoolArena.width)
  uintptr_t cnt = 0, cnt2 = 0, opflags = 0, gflags = 0, d_rows = 0;
};
struct GpGen {  // translation LUTs (Genetics.device_luts)
  uintptr_t small = 0, dom_type = 0, two_codon = 0;
  int dt_entries = 0, dom_size = 0, dom_type_size = 0;
};
struct GpKin {  // ragged parameter records (params.h) + token LUTs + the cell -> records map
  uintptr_t Kmr = 0, W = 0, Q = 0, overflow = 0, slot = 0, rtop = 0;
  int P = 0, s = 0;
  long long rec_cap = 0;
  uintptr_t vmax = 0, km = 0, signs = 0, hills = 0, react = 0, trnsp = 0, eff = 0, energies = 0;
  int nw = 0, nk = 0, nsg = 0, nh = 0, nv = 0;
  float abs_temp = 0.f, gas = 0.f;
};

namespace {
constexpr int kSelI32Pos = 2, kSelSet = 0;

// bump allocator over one scratch blob (256-byte aligned pieces)
struct Carve {
  uintptr_t base;
  size_t off = 0;
  explicit Carve(uintptr_t b) : base(b) {}
  uintptr_t take(size_t bytes) {
    off = (off + 255) & ~size_t(255);
    const uintptr_t p = base + off;
    off += bytes;
    return p;
  }
};

// genomes longer than the LDS translation slots handled per call (global-memory slots, each sized
// for the call's length bound: at most 1 GiB of them -- a long evolving run's bound of 10^6 nt makes
// a slot 40 MB); the long genomes past them are listed for the host rebuild (gp_check_assign_kernel)
int long_cap(int cap, int width) {
  const size_t sb = std::max<size_t>(1, translate_slot_bytes(width));
  return (int)std::max<size_t>(1, std::min<size_t>(std::min(cap, 1024), (size_t(1) << 30) / sb));
}

// translation + fresh rows + parameter build for cells[:*dcnt]
size_t rebuild_bytes(int cap, int P, int dcap, int width) {
  Carve c(0);
  c.take((size_t)long_cap(cap, width) * translate_slot_bytes(width));  // long-genome slots
  c.take(8 * (size_t)cap);                        // counts (2 per cell)
  c.take(8 * (size_t)cap);                        // ndom
  c.take(4 * (size_t)cap);                        // long list
  c.take(16);                                     // long count
  c.take(4 * (size_t)cap);                        // proteins per cell
  c.take(8 * (size_t)cap);                        // record offsets
  c.take(4 * (size_t)cap * P * dcap * 5);         // tokens
  return c.off + 256;
}

// returns the status slot (written by the check / assign launch; final once the chain completed)
int rebuild(int cap, uintptr_t cells, uintptr_t dcnt, const GpArena& a, const GpGen& g, const GpKin& k, int dcap,
            Carve& c, uintptr_t stat_cnt, hipStream_t s) {
  const uintptr_t st = reinterpret_cast<uintptr_t>(s);
  const int lcap = long_cap(cap, a.width);
  const uintptr_t gslot = c.take((size_t)lcap * translate_slot_bytes(a.width));
  const uintptr_t counts = c.take(8 * (size_t)cap), ndom = c.take(8 * (size_t)cap);
  const uintptr_t long_list = c.take(4 * (size_t)cap), long_count = c.take(16);
  const uintptr_t per = c.take(4 * (size_t)cap), roff = c.take(8 * (size_t)cap);
  const uintptr_t tokens = c.take(4 * (size_t)cap * k.P * dcap * 5);
  const long long row = (long long)k.P * dcap * 5;
  const unsigned gz = (unsigned)std::max<long long>(1, std::min<long long>(cdiv((long long)cap * row, 256), 1024));
  msd::kl(gp_zero_kernel, gz, 256, 0, s)(cap, P_<int>(dcnt), row, P_<int32_t>(tokens), P_<int32_t>(long_count));
  MS_LAUNCH_CHECK();
  translate_fused(cap, cells, a.data, a.off, a.width, a.lens, g.small, g.dom_type, g.dt_entries, g.two_codon, g.dom_size,
                  g.dom_type_size, counts, ndom, k.P, dcap, tokens, long_list, long_count, dcnt, st);
  if (a.width > translate_lds_max())  // genomes longer than the LDS slots: second pass over the queued ones
    translate_fused_long(lcap, cells, a.data, a.off, a.width, a.lens, g.small, g.dom_type, g.dt_entries, g.two_codon,
                         g.dom_size, g.dom_type_size, counts, ndom, k.P, dcap, tokens, long_list, gslot, long_count,
                         st);
  auto sl = status_slot();
  msd::kl(gp_check_assign_kernel, 1, 1024, 0, s)(cap, lcap, P_<int>(dcnt), P_<int32_t>(counts), P_<int32_t>(ndom),
                                            P_<int32_t>(long_list), P_<int32_t>(long_count), P_<int32_t>(per), k.P,
                                            dcap, P_<int64_t>(cells), P_<int64_t>(k.slot), P_<long long>(k.rtop),
                                            k.rec_cap, P_<int64_t>(roff), P_<int>(a.opflags), P_<int>(stat_cnt),
                                            sl.first, status_bad_dev(sl.second), status_bad_cap());
  MS_LAUNCH_CHECK();
  build_params(cap, k.P, dcap, k.P, k.s, tokens, 0, k.vmax, k.nw, k.km, k.nk, k.signs, k.nsg, k.hills, k.nh,
               k.react, k.trnsp, k.eff, k.nv, k.energies, k.abs_temp, k.gas, 0, 0, 0, 0, k.Kmr, 0, 0, 0, 0, per, k.W, k.Q,
               k.overflow, dcnt, roff, st);
  return sl.second;
}
}  // namespace

// The recombination's commit and the list of its changed cells: the winning result rows (the last
// result per cell) committed and their cells listed in result order -- appended by the commit and
// sorted + gathered in one launch (sel_sort), or (more result rows than the sort holds, or the
// append paths off) the `won` flags, their selection and a gather.
void commit_rec_results(int nr, uintptr_t dn, int dn_mul, uintptr_t out_rows, uintptr_t out, int out_w,
                        uintptr_t out_len, const GpArena& a, int L, uintptr_t mark, uint64_t gen, uintptr_t won,
                        uintptr_t q, uintptr_t cells, uintptr_t stream) {
  if (g_mut_append && nr <= sel_sort_cap()) {
    arena_scatter_app(nr, dn, dn_mul, out_rows, out, out_w, out_len, a.data, a.off, a.top, a.pool_cap, L, a.lens, mark,
                      gen, a.gflags, a.opflags, q, stream);
    hipStream_t s = S_(stream);
    sel_sort(q, append_counter(s), nr, cells, a.cnt2, 0, 0, s, out_rows);
    return;
  }
  arena_scatter(nr, dn, dn_mul, out_rows, out, out_w, out_len, a.data, a.off, a.top, a.pool_cap, L, a.lens, mark, gen,
                won, a.gflags, a.opflags, stream);
  select_indices_dev(nr, kSelSet, won, 0, q, 0, a.cnt2, stream);
  gather_dev(nr, a.cnt2, q, out_rows, cells, stream);
}

// Scratch bytes of one call (the caller passes a blob of at least this size; the blob must stay
// untouched until the call was reconciled: it holds the results a replay may re-commit).
size_t gp_blob_bytes(int kind, int n, int cap, int P, int L, int dcap, int kcap, int extra_rows) {
  Carve c(0);
  if (kind == 2) return rebuild_bytes(cap, P, dcap, L) + 512;  // rebuild of listed cells (L: arena width)
  if (kind == 0) {  // mutations
    const int out_w = (L + kcap + 15) / 16 * 16;
    c.take(4 * (size_t)n);                 // k
    c.take(8 * (size_t)n);                 // sel
    c.take((size_t)cap * out_w);           // out
    c.take(4 * (size_t)cap);               // out_len
    c.take(8 * (size_t)cap);               // appended draws (mutations.hip mut_count_select)
    return c.off + rebuild_bytes(cap, P, dcap, L) + 512;
  }
  // recombinations: cap = pairs capacity
  const int nr = 2 * cap + extra_rows, out_w = 2 * L;
  c.take(4 * 8 * (size_t)n);               // k per slot
  c.take(8 * 8 * (size_t)n);               // sel
  c.take((size_t)nr * out_w);              // out
  c.take(4 * (size_t)nr);                  // out_len
  c.take(8 * (size_t)nr);                  // out_rows
  c.take(4 * (size_t)cap * (kcap + 2) * 3);  // parts
  c.take((size_t)nr);                      // won
  c.take(8 * (size_t)nr);                  // q
  c.take(8 * (size_t)nr);                  // cells
  c.take(8 * (size_t)cap);                 // thinned-draw candidates (world.hip rec_slots)
  return c.off + rebuild_bytes(nr, P, dcap, L) + 512;
}

// Offsets of the pieces a reconcile may need: mutations {sel, out, out_len}; recombinations
// {out_rows, out, out_len, cells}.
py::dict gp_layout(int kind, int n, int cap, int L, int kcap, int extra_rows) {
  Carve c(0);
  py::dict d;
  if (kind == 0) {
    const int out_w = (L + kcap + 15) / 16 * 16;
    c.take(4 * (size_t)n);
    d["sel"] = c.take(8 * (size_t)n);
    d["out"] = c.take((size_t)cap * out_w);
    d["out_len"] = c.take(4 * (size_t)cap);
    d["out_w"] = out_w;
    return d;
  }
  const int nr = 2 * cap + extra_rows, out_w = 2 * L;
  c.take(4 * 8 * (size_t)n);
  c.take(8 * 8 * (size_t)n);
  d["out"] = c.take((size_t)nr * out_w);
  d["out_len"] = c.take(4 * (size_t)nr);
  d["out_rows"] = c.take(8 * (size_t)nr);
  c.take(4 * (size_t)cap * (kcap + 2) * 3);
  c.take((size_t)nr);
  c.take(8 * (size_t)nr);
  d["cells"] = c.take(8 * (size_t)nr);
  d["out_w"] = out_w;
  d["nr"] = nr;
  return d;
}

// Per-call counter setup in one launch: op flags cleared; with a fresh chain (nothing pending) the
// chain flags too and the device row counter set to the host's row count.
__global__ void gp_begin_kernel(int* opflags, int* gflags, long long* d_rows, long long nrows, int fresh) {
  *opflags = 0;
  if (fresh) {
    *gflags = 0;
    if (nrows >= 0) *d_rows = nrows;  // (-1: the counter is the kinetics' record counter, kept)
  }
}

void gp_begin(const GpArena& a, bool fresh, long long nrows, uintptr_t stream) {
  msd::kl(gp_begin_kernel, 1, 1, 0, S_(stream))(P_<int>(a.opflags), P_<int>(a.gflags), P_<long long>(a.d_rows), nrows,
                                           fresh ? 1 : 0);
  MS_LAUNCH_CHECK();
}

// mutate_cells() over all n genomes; returns the pinned status slot {rebuilt, flags, row counter, selected}.
int gp_mutate(const GpArena& a, const GpGen& g, const GpKin& k, double p, double p_indel, double p_del, uint64_t seed,
              uint64_t call, int cap, int kcap, int dcap, uintptr_t blob, uintptr_t stream) {
  hipStream_t s = S_(stream);
  const int n = a.n, L = a.width;
  Carve c(blob);
  const uintptr_t kk = c.take(4 * (size_t)n), sel = c.take(8 * (size_t)n);
  const int out_w = (L + kcap + 15) / 16 * 16;
  const uintptr_t out = c.take((size_t)cap * out_w), out_len = c.take(4 * (size_t)cap);
  const uintptr_t cand = c.take(8 * (size_t)cap);
  mut_count_select(n, a.lens, p, seed, call, kk, kcap, a.gflags, a.opflags, sel, a.cnt, cap, cand, stream, 0, 0);
  mut_apply(cap, a.cnt, sel, 0, a.data, a.off, a.lens, kk, p_indel, p_del, seed, call, out, out_w, out_len, stream);
  arena_scatter(cap, a.cnt, 1, sel, out, out_w, out_len, a.data, a.off, a.top, a.pool_cap, L, a.lens, 0, 0, 0,
                a.gflags, a.opflags, stream);
  return rebuild(cap, sel, a.cnt, a, g, k, dcap, c, a.cnt, s);
}

// recombinate_cells() over neighbour slot keys (8 per cell); `extra` (optional Python object with
// .rows and .apply(pair_count, out, out_w, out_len, out_rows, nres)) appends strip-boundary results.
// keys: the neighbour slot keys (8n int64); with `nbr` = (positions, R, C, r_lo, r_hi, wrap, index
// map, longest-genome word of index_map_lmax) they are computed here, fused with the draws and the selection count (world.hip rec_slots),
// otherwise read.
int gp_recombine(const GpArena& a, const GpGen& g, const GpKin& k, uintptr_t keys, py::object nbr, double p,
                 uint64_t seed, uint64_t call, int cap, int kcap, int dcap, uintptr_t mark, uint64_t gen,
                 py::object extra, uintptr_t nres, uintptr_t blob, uintptr_t stream) {
  hipStream_t s = S_(stream);
  const int n = a.n, L = a.width;
  const int xr = extra.is_none() ? 0 : extra.attr("rows").cast<int>();
  const int nr = 2 * cap + xr, out_w = 2 * L, parts_cap = kcap + 2;
  Carve c(blob);
  const uintptr_t kk = c.take(4 * 8 * (size_t)n), sel = c.take(8 * 8 * (size_t)n);
  const uintptr_t out = c.take((size_t)nr * out_w), out_len = c.take(4 * (size_t)nr), out_rows = c.take(8 * (size_t)nr);
  const uintptr_t parts = c.take(4 * (size_t)cap * parts_cap * 3);
  const uintptr_t won = c.take((size_t)nr), q = c.take(8 * (size_t)nr), cells = c.take(8 * (size_t)nr);
  const uintptr_t cand = c.take(8 * (size_t)cap);
  if (!nbr.is_none()) {
    const auto t = nbr.cast<std::tuple<uintptr_t, int, int, int, int, int, uintptr_t, uintptr_t>>();
    rec_slots(n, std::get<0>(t), std::get<1>(t), std::get<2>(t), std::get<3>(t), std::get<4>(t), std::get<5>(t),
              std::get<6>(t), a.lens, std::get<7>(t), p, seed, call, kcap, a.gflags, a.opflags, keys, kk, sel, a.cnt,
              cap, cand, stream, 0, 0);
  } else {
    rec_count_keys(8 * n, keys, a.lens, p, seed, call, kk, 0, kcap, a.gflags, a.opflags, stream, 0);
    select_indices_capped(8ll * n, kSelI32Pos, kk, sel, a.cnt, cap, a.gflags, a.opflags, stream);
  }
  rec_apply(cap, a.cnt, sel, 0, keys, a.data, a.off, a.lens, kk, seed, call, parts, parts_cap, out, out_w, out_len,
            out_rows, stream);
  if (xr) {
    extra.attr("apply")(a.cnt, out, out_w, out_len, out_rows, nres);
  }
  // (a0, b0, a1, b1, ..., extra rows): the last result per cell wins (reference update order)
  commit_rec_results(nr, xr ? nres : a.cnt, xr ? 1 : 2, out_rows, out, out_w, out_len, a, L, mark, gen, won, q, cells,
                     stream);
  return rebuild(nr, cells, a.cnt2, a, g, k, dcap, c, xr ? nres : a.cnt, s);
}

// Translation + fresh rows + parameter build of cells[:*cnt] (cnt <= cap; e.g. spawned cells or
// cells that arrived from another rank); returns the status slot.
int gp_rebuild(const GpArena& a, const GpGen& g, const GpKin& k, uintptr_t cells, uintptr_t cnt, int cap, int dcap,
               uintptr_t blob, uintptr_t stream) {
  if (cap <= 0) throw std::invalid_argument("gp_rebuild: empty");
  Carve c(blob);
  return rebuild(cap, cells, cnt, a, g, k, dcap, c, cnt, S_(stream));
}

// ---- recombinate_cells() + mutate_cells() as one chain (the reference loop calls them back to
// back, performance/run_simulation.py:92-93): the recombination is applied and committed, the point
// mutations are drawn over the recombined genomes and committed, and the union of the changed cells
// is translated and built ONCE (a cell's parameters are a function of its final genome). Against two
// separate calls this drops one translation + build (and its zero / check launches) from the side
// stream, which is what the next activity waits for.

// union list: recombined cells, then mutated ones (a cell in both is built twice into two fresh rows
// from the same final genome; either row is right), then the cells [arr0, arr0 + narr) (a strip's
// arrivals of the division before, whose parameters are built here instead of by a rebuild chain of
// their own) + the parts' status {pairs, rec flags, mutated, mut flags} into a pinned slot
__global__ void __launch_bounds__(256) gp_union_kernel(int ucap, int mcap, const int* rec_cnt, const int64_t* rec_cells,
                                                       const int* mut_cnt, const int64_t* mut_sel, long long arr0,
                                                       int narr, int64_t* cells, int* cnt_u, const int* rec_pairs,
                                                       const int* rec_opflags, const int* mut_opflags,
                                                       long long* parts_status, const unsigned long long* top,
                                                       long long* top_host) {
  const int cr = *rec_cnt, cm = min(*mut_cnt, mcap);
  const int nr = min(cr, ucap - narr), nm = min(cm, ucap - narr - nr);
  for (int j = threadIdx.x; j < nr; j += blockDim.x) cells[j] = rec_cells[j];
  for (int j = threadIdx.x; j < nm; j += blockDim.x) cells[nr + j] = mut_sel[j];
  for (int j = threadIdx.x; j < narr; j += blockDim.x) cells[nr + nm + j] = arr0 + j;
  if (threadIdx.x == 0) {
    cnt_u[0] = nr + nm + narr;
    parts_status[0] = *rec_pairs;
    parts_status[1] = __hip_atomic_load(rec_opflags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    parts_status[2] = *mut_cnt;
    parts_status[3] = __hip_atomic_load(mut_opflags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // the pool's bump counter after the chain's last allocation, mirrored into mapped host memory:
    // the host tightens its upper bound of it at the next reconcile without a read-back
    if (top_host)
      __hip_atomic_store(top_host, (long long)__hip_atomic_load(top, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ void gp_begin3_kernel(int* f0, int* f1, int* f2, int* gflags, long long* d_rows, long long nrows, int fresh) {
  *f0 = 0;
  *f1 = 0;
  *f2 = 0;
  if (fresh) {
    *gflags = 0;
    if (nrows >= 0) *d_rows = nrows;  // (-1: the counter is the kinetics' record counter, kept)
  }
}

size_t gp_evolve_union_bytes(int ucap, int P, int dcap, int L) {
  Carve c(0);
  c.take(8 * (size_t)ucap);  // union cells
  c.take(16);                // union count
  return c.off + rebuild_bytes(ucap, P, dcap, L) + 512;
}

// ar / am / au: the recombination's, the mutation's and the union rebuild's counters (the arena
// fields are the same in all three). `extra` / `nres`: strip-boundary recombination results of a
// decomposed world, appended after the local pairs' results (as in gp_recombine; the parts status
// then counts result rows instead of pairs). `arr0` / `narr`: cells whose parameters are built with
// the union (a strip's arrivals, magicsoup_amd/parallel/dist_world.py _divide_phase_b). `nd_a` /
// `nd_b`: device words whose sum is the cell count, `ar.n` its bound (World._chain_bound), or 0. Returns
// (union status slot {count, flags, row counter, count}, parts status slot {pairs or result rows, rec
// flags, mutated, mut flags}).
std::pair<int, int> gp_evolve(const GpArena& ar, const GpArena& am, const GpArena& au, const GpGen& g, const GpKin& k,
                              uintptr_t keys, py::object nbr, double p_rec, uint64_t seed_r, uint64_t call_r, int pcap,
                              double p, double p_indel, double p_del, uint64_t seed_m, uint64_t call_m, int mcap,
                              int kcap, int dcap, uintptr_t mark, uint64_t gen, uintptr_t blob_r, uintptr_t blob_m,
                              uintptr_t blob_u, bool fresh, long long nrows, py::object extra, uintptr_t nres,
                              long long arr0, int narr, uintptr_t nd_a, uintptr_t nd_b, uintptr_t top_host,
                              uintptr_t stream) {
  hipStream_t s = S_(stream);
  if (narr < 0) throw std::invalid_argument("gp_evolve: negative arrival count");
  const int n = ar.n, L = ar.width;
  const int xr = extra.is_none() ? 0 : extra.attr("rows").cast<int>();
  if (xr && !nres) throw std::invalid_argument("gp_evolve: boundary rows need the result-row counter");
  msd::kl(gp_begin3_kernel, 1, 1, 0, s)(P_<int>(ar.opflags), P_<int>(am.opflags), P_<int>(au.opflags), P_<int>(ar.gflags),
                                   P_<long long>(ar.d_rows), nrows, fresh ? 1 : 0);
  MS_LAUNCH_CHECK();
  // recombination (gp_recombine's layout of blob_r, without its rebuild)
  const int nr = 2 * pcap + xr, out_w = 2 * L, parts_cap = kcap + 2;
  Carve cr(blob_r);
  const uintptr_t kk = cr.take(4 * 8 * (size_t)n), sel = cr.take(8 * 8 * (size_t)n);
  const uintptr_t out = cr.take((size_t)nr * out_w), out_len = cr.take(4 * (size_t)nr), out_rows = cr.take(8 * (size_t)nr);
  const uintptr_t parts = cr.take(4 * (size_t)pcap * parts_cap * 3);
  const uintptr_t won = cr.take((size_t)nr), q = cr.take(8 * (size_t)nr), cells = cr.take(8 * (size_t)nr);
  const uintptr_t cand = cr.take(8 * (size_t)pcap);
  const auto t = nbr.cast<std::tuple<uintptr_t, int, int, int, int, int, uintptr_t, uintptr_t>>();
  rec_slots(n, std::get<0>(t), std::get<1>(t), std::get<2>(t), std::get<3>(t), std::get<4>(t), std::get<5>(t),
            std::get<6>(t), ar.lens, std::get<7>(t), p_rec, seed_r, call_r, kcap, ar.gflags, ar.opflags, keys, kk, sel,
            ar.cnt, pcap, cand, stream, nd_a, nd_b);
  rec_apply(pcap, ar.cnt, sel, 0, keys, ar.data, ar.off, ar.lens, kk, seed_r, call_r, parts, parts_cap, out, out_w,
            out_len, out_rows, stream);
  if (xr) extra.attr("apply")(ar.cnt, out, out_w, out_len, out_rows, nres);
  commit_rec_results(nr, xr ? nres : ar.cnt, xr ? 1 : 2, out_rows, out, out_w, out_len, ar, L, mark, gen, won, q, cells,
                     stream);
  // point mutations over the recombined genomes (gp_mutate's layout of blob_m, without its rebuild)
  Carve cm(blob_m);
  const uintptr_t mk = cm.take(4 * (size_t)n), msel = cm.take(8 * (size_t)n);
  const int mout_w = (L + kcap + 15) / 16 * 16;
  const uintptr_t mout = cm.take((size_t)mcap * mout_w), mout_len = cm.take(4 * (size_t)mcap);
  const uintptr_t mcand = cm.take(8 * (size_t)mcap);
  mut_count_select(n, am.lens, p, seed_m, call_m, mk, kcap, am.gflags, am.opflags, msel, am.cnt, mcap, mcand, stream,
                   nd_a, nd_b);
  mut_apply(mcap, am.cnt, msel, 0, am.data, am.off, am.lens, mk, p_indel, p_del, seed_m, call_m, mout, mout_w, mout_len,
            stream);
  arena_scatter(mcap, am.cnt, 1, msel, mout, mout_w, mout_len, am.data, am.off, am.top, am.pool_cap, L, am.lens, 0, 0,
                0, am.gflags, am.opflags,
                stream);
  // union of the changed cells -> one translation + build
  const int ucap = nr + mcap + narr;
  Carve cu(blob_u);
  const uintptr_t ucells = cu.take(8 * (size_t)ucap), ucnt = cu.take(16);
  auto ps = status_slot();
  msd::kl(gp_union_kernel, 1, 256, 0, s)(ucap, mcap, P_<int>(ar.cnt2), P_<int64_t>(cells), P_<int>(am.cnt),
                                    P_<int64_t>(msel), arr0, narr, P_<int64_t>(ucells), P_<int>(ucnt),
                                    P_<int>(xr ? nres : ar.cnt),
                                    P_<int>(ar.opflags), P_<int>(am.opflags), ps.first,
                                    P_<unsigned long long>(ar.top), top_host ? P_<long long>(top_host) : nullptr);
  MS_LAUNCH_CHECK();
  const int slot_u = rebuild(ucap, ucells, ucnt, au, g, k, dcap, cu, ucnt, s);
  return {slot_u, ps.second};
}

void bind_gp(py::module_& m) {
  msd::gdef(m, "gp_evolve", &gp_evolve, "device-pipeline recombinate_cells() + mutate_cells() with one rebuild (no sync)");
  msd::gdef(m, "gp_evolve_union_bytes", &gp_evolve_union_bytes);
  // a pinned, device-mapped int64 (host pointer, device pointer) and its host-side read / write
  msd::gdef(m, "mapped_i64", []() {
    long long* h = nullptr;
    long long* d = nullptr;
    MS_HIP_CHECK(hipHostMalloc((void**)&h, sizeof(long long), hipHostMallocMapped | hipHostMallocCoherent));
    MS_HIP_CHECK(hipHostGetDevicePointer((void**)&d, h, 0));
    *h = -1;
    return std::make_pair(reinterpret_cast<uintptr_t>(h), reinterpret_cast<uintptr_t>(d));
  });
  msd::gdef(m, "mapped_i64_read", [](uintptr_t h) {
    return __atomic_load_n(reinterpret_cast<long long*>(h), __ATOMIC_ACQUIRE);
  });
  msd::gdef(m, "mapped_i64_write", [](uintptr_t h, long long v) {
    __atomic_store_n(reinterpret_cast<long long*>(h), v, __ATOMIC_RELEASE);
  });
  py::class_<GpArena>(m, "GpArena", py::module_local())
      .def(py::init<>())
      .def_readwrite("data", &GpArena::data).def_readwrite("lens", &GpArena::lens)
      .def_readwrite("off", &GpArena::off).def_readwrite("top", &GpArena::top)
      .def_readwrite("pool_cap", &GpArena::pool_cap)
      .def_readwrite("width", &GpArena::width).def_readwrite("n", &GpArena::n)
      .def_readwrite("cnt", &GpArena::cnt).def_readwrite("cnt2", &GpArena::cnt2)
      .def_readwrite("opflags", &GpArena::opflags).def_readwrite("gflags", &GpArena::gflags)
      .def_readwrite("d_rows", &GpArena::d_rows);
  py::class_<GpGen>(m, "GpGen", py::module_local())
      .def(py::init<>())
      .def_readwrite("small", &GpGen::small).def_readwrite("dom_type", &GpGen::dom_type)
      .def_readwrite("two_codon", &GpGen::two_codon).def_readwrite("dt_entries", &GpGen::dt_entries)
      .def_readwrite("dom_size", &GpGen::dom_size).def_readwrite("dom_type_size", &GpGen::dom_type_size);
  py::class_<GpKin>(m, "GpKin", py::module_local())
      .def(py::init<>())
      .def_readwrite("Kmr", &GpKin::Kmr)
      .def_readwrite("W", &GpKin::W).def_readwrite("Q", &GpKin::Q).def_readwrite("overflow", &GpKin::overflow)
      .def_readwrite("slot", &GpKin::slot).def_readwrite("rtop", &GpKin::rtop).def_readwrite("P", &GpKin::P)
      .def_readwrite("s", &GpKin::s)
      .def_readwrite("rec_cap", &GpKin::rec_cap).def_readwrite("vmax", &GpKin::vmax).def_readwrite("km", &GpKin::km)
      .def_readwrite("signs", &GpKin::signs).def_readwrite("hills", &GpKin::hills)
      .def_readwrite("react", &GpKin::react).def_readwrite("trnsp", &GpKin::trnsp).def_readwrite("eff", &GpKin::eff)
      .def_readwrite("energies", &GpKin::energies).def_readwrite("nw", &GpKin::nw).def_readwrite("nk", &GpKin::nk)
      .def_readwrite("nsg", &GpKin::nsg).def_readwrite("nh", &GpKin::nh).def_readwrite("nv", &GpKin::nv)
      .def_readwrite("abs_temp", &GpKin::abs_temp).def_readwrite("gas", &GpKin::gas);
  msd::gdef(m, "gp_begin", &gp_begin);
  msd::gdef(m, "gp_blob_bytes", &gp_blob_bytes);
  msd::gdef(m, "gp_layout", &gp_layout);
  msd::gdef(m, "gp_mutate", &gp_mutate, "device-pipeline point mutations over all genomes (one call, no sync)");
  msd::gdef(m, "gp_recombine", &gp_recombine, "device-pipeline recombinations over neighbour slot keys (one call, no sync)");
  msd::gdef(m, "gp_rebuild", &gp_rebuild, "device-pipeline translation + parameter build of listed cells (no sync)");
}

}  // namespace msd
