// pybind11 entry point of the gfx950 device module magicsoup_amd._hip.
//
// Tensors cross as raw device pointers (uintptr_t) together with the caller's current HIP stream,
// so launches are ordered with PyTorch's work on that stream and can be captured into hipGraphs.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <atomic>
#include <string>
#include <tuple>
#include <vector>

#include "hip_common.h"
#include "bind_util.h"

namespace py = pybind11;

namespace msd {
void split_cells(int k, int m, uintptr_t parents, uintptr_t children, uintptr_t cell_mols, uintptr_t divisions,
                 uintptr_t lifetimes, uintptr_t stream);
void place_rounds(int k, uintptr_t cells, uintptr_t pos, int R, int C, int r_lo, int r_hi, int wrap, bool vacate,
                  uintptr_t cell_map, uintptr_t pending, uintptr_t cand, uintptr_t claim, uintptr_t result, int rounds,
                  uint64_t seed, uint64_t call, uintptr_t stream);
void place_rounds_mask(int n, uintptr_t mask, uintptr_t pos, int R, int C, int r_lo, int r_hi, int wrap, bool vacate,
                       uintptr_t cell_map, uintptr_t pending, uintptr_t cand, uintptr_t claim, uintptr_t result,
                       int rounds, uint64_t seed, uint64_t call, uintptr_t stream);
void set_coop_blocks(int n);
void set_overflow_blocks(int n);
void set_place_tail(int on);
void set_stencil_vec(int v);
void set_stencil_prefetch(int pf);
void set_stencil_band(int b);
void set_stencil_blocks(int n);
void set_place_mode(int mode);
int place_error_take();
void neighbor_slots(int n, uintptr_t pos, int R, int C, int r_lo, int r_hi, int wrap, uintptr_t idx_map, uintptr_t keys,
                    uintptr_t stream);
void rec_count_keys(int n, uintptr_t keys, uintptr_t lens, double p, uint64_t seed, uint64_t call, uintptr_t k,
                    uintptr_t tot, int kcap, uintptr_t gflags, uintptr_t opflags, uintptr_t stream,
                    uintptr_t lw_word);
// maps.hip
size_t diffuse_partials_len(int m, int C, int H);
void diffuse_stencil(int m, int R, int C, int r_lo, int r_hi, int wrap, uintptr_t map, uintptr_t tmp, uintptr_t wa,
                     uintptr_t wb, uintptr_t scale, uintptr_t corr, uintptr_t partials, uintptr_t totals, int dtype, int accumulate,
                     uintptr_t stream, uintptr_t corr_out, double n_pix);
void diffuse_corr(int m, uintptr_t totals, double n_pix, uintptr_t corr, uintptr_t stream);
void diffuse_boundary(int m, int R, int C, int r_lo, int r_hi, uintptr_t map, uintptr_t tmp, uintptr_t wa,
                      uintptr_t wb, uintptr_t scale, uintptr_t corr, uintptr_t partials, uintptr_t totals, int dtype,
                      uintptr_t stream);
size_t diffuse_boundary_partials_len(int m, int C);
void diffuse_strip(int m, int R, int C, int r_lo, int r_hi, uintptr_t map, uintptr_t tmp, uintptr_t wa, uintptr_t wb,
                   uintptr_t scale, uintptr_t corr, uintptr_t partials, uintptr_t partials_b, uintptr_t totals,
                   uintptr_t new_corr, double n_pix, int dtype, uintptr_t comm, int up, int down, uintptr_t halo_bufs,
                   uintptr_t halo_stream, uintptr_t stream);
void apply_pending(int m, long long plane, uintptr_t map, uintptr_t corr, uintptr_t f, int dtype, uintptr_t stream);
void map_totals(int m, int R, int C, int r_lo, int r_hi, uintptr_t map, uintptr_t corr, uintptr_t f, int dtype,
                uintptr_t out, uintptr_t stream);
void diffuse_correct(int m, int R, int C, int r_lo, int r_hi, uintptr_t map, uintptr_t tmp, uintptr_t totals,
                     double n_pix, int dtype, uintptr_t stream);
void scale_planes(int m, long long plane, uintptr_t map, uintptr_t f, int dtype, uintptr_t stream);
void scale_rows(long long rows, int m, uintptr_t x, uintptr_t f, uintptr_t stream);
std::vector<unsigned long long> int_prof_read(bool reset);
void add_i32(long long n, uintptr_t x, int v, uintptr_t stream);
void health_scan(int planes, long long span, long long stride, uintptr_t x, int dtype, int shift, uintptr_t flags,
                 uintptr_t stream);
void spill_free(int k, int m, uintptr_t idxs, uintptr_t pos, int R, int C, uintptr_t cell_mols, uintptr_t map,
                uintptr_t cell_map, int dtype, uintptr_t corr, uintptr_t stream);
void spill_free_mask(int n, int m, uintptr_t dead, uintptr_t pos, int R, int C, uintptr_t cell_mols, uintptr_t map,
                     uintptr_t cell_map, int dtype, uintptr_t corr, uintptr_t stream);
void pickup(int k, int m, uintptr_t idxs, uintptr_t pos, int R, int C, uintptr_t cell_mols, uintptr_t map, int dtype,
            uintptr_t corr, uintptr_t stream);
void cell_state_io(int n, int m, uintptr_t pos, int R, int C, uintptr_t map, int dtype, uintptr_t cell_mols,
                   uintptr_t buf, bool restore, uintptr_t stream);
void spawn_dev(int k, int R, int C, int r_lo, int r_hi, uintptr_t cell_map, uint64_t seed, uint64_t call,
               long long n0, int m, uintptr_t pos, uintptr_t lifetimes, uintptr_t divisions, uintptr_t cell_mols,
               uintptr_t map, int dtype, uintptr_t corr, uintptr_t labels, int label_w, uintptr_t label_lens,
               int L_in, uintptr_t rows, uintptr_t lens, uintptr_t pool, uintptr_t off, uintptr_t top,
               long long pool_cap, uintptr_t arena_lens, uintptr_t failed, uintptr_t pool_failed, uintptr_t claim,
               uintptr_t cand, uintptr_t result, uintptr_t stream);
void permeate(int c, int m, int R, int C, uintptr_t pos, uintptr_t perm, uintptr_t cell_mols, uintptr_t map, int dtype,
              uintptr_t corr, uintptr_t stream);
void gather_rows(int n, uintptr_t dn, uintptr_t src_rows, uintptr_t dst_rows,
                 const std::vector<std::tuple<uintptr_t, uintptr_t, long long, long long, long long, uintptr_t>>& descs,
                 uintptr_t stream);
// kinetics.hip
bool integrate_spec_ok(int s, int nparts);
int integrate_dist(int c, int P, int s, int m, int R, int C, uintptr_t W, uintptr_t Q, uintptr_t Kmr,
                   uintptr_t cell_mols, uintptr_t molmap, uintptr_t positions, uintptr_t snap_a, uintptr_t snap_b,
                   uintptr_t masks, const std::vector<float>& trims, int n_iters, uintptr_t prow, uintptr_t lists,
                   int map_dtype, uintptr_t map_corr, uintptr_t spec_buf, uintptr_t save_buf, uintptr_t comm,
                   uintptr_t stream);
void release_select_buffers();
void release_dist_buffers();
void release_world_buffers();
void release_kinetics_streams();
void release_events();
void bind_events(py::module_& m);
// Exit path (registered with Python's atexit by ops/native.py): drain the device and free the
// process-wide pinned / device buffers and streams of the extension while the HIP runtime (and a
// profiler's interception layer, which finalises in the C exit handlers after Python's) is intact.
void release_static() {
  MS_HIP_CHECK(msd::device_synchronize());
  release_select_buffers();
  release_dist_buffers();
  release_world_buffers();
  release_kinetics_streams();
  release_events();
}
int integrate(int c, int P, int s, int m, int R, int C, uintptr_t W, uintptr_t Q, uintptr_t Kmr, uintptr_t cell_mols,
              uintptr_t molmap, uintptr_t positions, uintptr_t X_io, uintptr_t snap_a, uintptr_t snap_b,
              uintptr_t masks, const std::vector<float>& trims, int n_iters, int part_begin, int part_end,
              bool scatter, uintptr_t prow, uintptr_t lists, int map_dtype, uintptr_t map_corr, uintptr_t spec_buf,
              uintptr_t save_buf, int dist_stage, uintptr_t stream);
void build_params(int n, int P, int D, int Pt, int s, uintptr_t tokens, uintptr_t rows, uintptr_t vmax_w, int nw,
                  uintptr_t km_w, int nk, uintptr_t signs, int nsg, uintptr_t hills, int nh, uintptr_t RM,
                  uintptr_t TM, uintptr_t EM, int nv, uintptr_t energies, float abs_temp, float gas, uintptr_t N,
                  uintptr_t Nf, uintptr_t Nb, uintptr_t A, uintptr_t Kmr, uintptr_t Kmf, uintptr_t Kmb,
                  uintptr_t Vmax, uintptr_t Ke, uintptr_t nprot, uintptr_t W, uintptr_t Q, uintptr_t overflow,
                  uintptr_t dn, uintptr_t roff, uintptr_t stream);
void assign_records(int n, uintptr_t dn, uintptr_t nprot, uintptr_t cells, uintptr_t slot, uintptr_t rtop,
                    long long rcap, int width, uintptr_t roff, uintptr_t flags, uintptr_t stream);
void records_to_dense(int n, int P, int s, uintptr_t slot, uintptr_t W, uintptr_t Q, uintptr_t Kmr, uintptr_t Wd,
                      uintptr_t Qd, uintptr_t Kmrd, uintptr_t stream);
void records_move(int n, int s, uintptr_t slot, uintptr_t new_off, uintptr_t W, uintptr_t Q, uintptr_t Kmr,
                  uintptr_t W2, uintptr_t Q2, uintptr_t Kmr2, uintptr_t slot_out, uintptr_t stream);
void pack_params(long long items, int s, uintptr_t N, uintptr_t Nf, uintptr_t Nb, uintptr_t A, uintptr_t Vmax,
                 uintptr_t Kmf, uintptr_t Kmb, uintptr_t Ke, uintptr_t W, uintptr_t Q, uintptr_t overflow,
                 uintptr_t stream);
// world.hip
void claim_free(int k, int R, int C, int r_lo, int r_hi, uintptr_t cell_map, uint64_t seed, uint64_t call,
                int attempts, uintptr_t out, uintptr_t stream);
void index_map(int c, uintptr_t pos, int C, uintptr_t idx_map, bool clear, uintptr_t stream);
void index_map_lmax(int c, uintptr_t pos, int C, uintptr_t idx_map, uintptr_t lens, uintptr_t word, uint64_t gen,
                    uintptr_t na, uintptr_t nb, uintptr_t stream);
int sel_sort_cap();
void neighbor_pairs_sorted(int n, uintptr_t pos, int R, int C, int r_lo, int r_hi, int wrap, uintptr_t idx_map,
                           uintptr_t in_from, uintptr_t in_to, uintptr_t keys, uintptr_t stream);

// genetics.hip
void translate_count(int n, uintptr_t rows, uintptr_t arena, uintptr_t off, int width, uintptr_t lens, uintptr_t luts,
                     uintptr_t dom_type, int dt_entries, uintptr_t two_codon, int dom_size, int dom_type_size,
                     uintptr_t nprot, uintptr_t ndom, uintptr_t list, uintptr_t gslot, uintptr_t long_list,
                     uintptr_t long_count, uintptr_t dn, uintptr_t stream);
void translate_write(int n, uintptr_t rows, uintptr_t arena, uintptr_t off, int width, uintptr_t lens, uintptr_t luts,
                     uintptr_t dom_type, int dt_entries, uintptr_t two_codon, int dom_size, int dom_type_size,
                     uintptr_t nprot, int P, int D, uintptr_t tokens, uintptr_t list, uintptr_t gslot,
                     uintptr_t dn, uintptr_t stream);
void translate_fused(int n, uintptr_t rows, uintptr_t arena, uintptr_t off, int width, uintptr_t lens, uintptr_t luts,
                     uintptr_t dom_type, int dt_entries, uintptr_t two_codon, int dom_size, int dom_type_size,
                     uintptr_t nprot, uintptr_t ndom, int P, int D, uintptr_t tokens, uintptr_t long_list,
                     uintptr_t long_count, uintptr_t dn, uintptr_t stream);
size_t translate_slot_bytes(int width);
void set_integrate_mode(int mode);
void set_rec_thinning(int on);
void set_spl2_waves(int w);
void set_rescue_mode(int m);
int rescue_error_take();
int lb_error_take();
// mutations.hip
void mut_count(int n, uintptr_t rows, uintptr_t lens, double p, uint64_t seed, uint64_t call, uintptr_t k, int kcap,
               uintptr_t gflags, uintptr_t opflags, uintptr_t stream);
void mut_apply(int nsel, uintptr_t dn, uintptr_t sel, uintptr_t rows, uintptr_t arena, uintptr_t off, uintptr_t lens,
               uintptr_t k, double p_indel, double p_del, uint64_t seed, uint64_t call, uintptr_t out, int out_width,
               uintptr_t out_len, uintptr_t stream);
void rec_count(int n, uintptr_t pairs, uintptr_t lens, double p, uint64_t seed, uint64_t call, uintptr_t k,
               uintptr_t stream);
void rec_apply(int nsel, uintptr_t dn, uintptr_t sel, uintptr_t pairs, uintptr_t keys, uintptr_t arena, uintptr_t off,
               uintptr_t lens, uintptr_t k, uint64_t seed, uint64_t call, uintptr_t parts, int parts_cap, uintptr_t out,
               int out_width, uintptr_t out_len, uintptr_t out_rows, uintptr_t stream);
void arena_scatter(int k, uintptr_t dn, int dn_mul, uintptr_t rows, uintptr_t src, int src_width, uintptr_t src_len,
                   uintptr_t pool, uintptr_t off, uintptr_t top, long long pool_cap, int width, uintptr_t lens,
                   uintptr_t mark, uint64_t gen, uintptr_t flags, uintptr_t gflags, uintptr_t opflags,
                   uintptr_t stream);
int divide_mask_dev(int n, uintptr_t mask, uintptr_t pos, int R, int C, int r_lo, int r_hi, int wrap, uintptr_t cell_map,
                    uintptr_t pending, uintptr_t cand, uintptr_t claim, uintptr_t result, int rounds, uint64_t seed,
                    uint64_t call, uintptr_t wins, uintptr_t dcount, long long n0, int m, uintptr_t par,
                    uintptr_t cell_mols, uintptr_t divisions, uintptr_t lifetimes, uintptr_t stream);
void divide_commit_list(int k, uintptr_t par, uintptr_t npos, long long n0, int n_exp, uintptr_t exp, int m,
                        uintptr_t pos, uintptr_t cell_mols, uintptr_t divisions, uintptr_t lifetimes, uintptr_t stream);
void place_collect(int k, uintptr_t wins, uintptr_t cells, uintptr_t result, int C, uintptr_t par, uintptr_t npos,
                   uintptr_t stream);
// select.hip
void select_indices_dev(long long n, int kind, uintptr_t src, uintptr_t vals, uintptr_t sel, uintptr_t rest,
                        uintptr_t out_dev, uintptr_t stream);
void gather_dev(int cap, uintptr_t dn, uintptr_t idx, uintptr_t src, uintptr_t dst, uintptr_t stream);
int count_to_host(uintptr_t dcount, uintptr_t stream);
int select_indices_async(long long n, int kind, uintptr_t src, uintptr_t sel, uintptr_t rest, uintptr_t out_dev,
                         uintptr_t stream);
int select_indices_async_pay(long long n, int kind, uintptr_t src, uintptr_t sel, uintptr_t rest, uintptr_t out_dev,
                             uintptr_t pay_src, uintptr_t pay_dst, uintptr_t stream);
void set_select_single_pass(int on, int items);
void cap_skip(uintptr_t dn, int cap, uintptr_t gflags, uintptr_t opflags, uintptr_t stream);
int status_write(uintptr_t dcnt, uintptr_t opflags, uintptr_t d_rows, uintptr_t cnt, uintptr_t stream);
std::tuple<long long, long long, long long, long long> status_read(int slot);
std::vector<long long> status_bad_read(int slot);
std::pair<uintptr_t, uintptr_t> mapped_flag();
int mapped_flag_read(uintptr_t host);
std::tuple<long long, long long, long long, long long> stream_sync_read(int slot, uintptr_t stream);
std::tuple<int, int, int> translate_stats(int n, uintptr_t counts, uintptr_t ndom, uintptr_t long_count, uintptr_t per,
                                          uintptr_t stream);
std::pair<long long, int> select_indices(long long n, int kind, uintptr_t src, uintptr_t vals, uintptr_t sel,
                                         uintptr_t rest, uintptr_t stream);
// comm.hip
int rccl_load(const std::string& path);
std::string rccl_unique_id();
uintptr_t rccl_init(const std::string& uid, int nranks, int rank);
void rccl_destroy(uintptr_t comm, bool abort);
std::string rccl_async_error(uintptr_t comm);
std::string rccl_guarded_wait(const std::vector<uintptr_t>& comms, uintptr_t stream, double timeout_s,
                              uintptr_t event);
void rccl_allreduce(uintptr_t comm, uintptr_t buf, long long count, int dtype, int op, uintptr_t stream);
void rccl_exchange(uintptr_t comm, int up, int down, uintptr_t send_up, long long n_send_up, uintptr_t send_down,
                   long long n_send_down, uintptr_t recv_down, long long n_recv_down, uintptr_t recv_up,
                   long long n_recv_up, uintptr_t stream);
// dist.hip
void strip_marks(int C, int H, uintptr_t cell_map, int k, uintptr_t cells, uintptr_t mask, uintptr_t pos, uintptr_t up,
                 uintptr_t dn, uintptr_t stream);
void strip_reserve(int C, int H, uintptr_t from_up, uintptr_t from_dn, uintptr_t cell_map, uintptr_t stream);
void strip_clear(int C, int H, uintptr_t cell_map, uintptr_t stream);
void set_split_single(int on);
void place_split(int k, uintptr_t result, uintptr_t cells, int C, int H, uintptr_t par, uintptr_t npos, uintptr_t counts,
                 uintptr_t hdr_up, uintptr_t hdr_dn, int lw, int gw, int m, uintptr_t stream);
long long rec_record_bytes(int m, int lw, int gw);
void rec_pack(int k_up, int k_dn, uintptr_t par_up, uintptr_t pos_up, uintptr_t par_dn, uintptr_t pos_dn,
              uintptr_t mols, uintptr_t pos, uintptr_t life, uintptr_t div, const GenomePoolArgs& gp, uintptr_t glen,
              int gw, uintptr_t ldata, uintptr_t llen, int lw, int m, bool child, uintptr_t out_up, uintptr_t out_dn,
              uintptr_t stream);
void rec_unpack(int n0, int k_up, uintptr_t in_up, int up_lw, int up_gw, int k_dn, uintptr_t in_dn, int dn_lw,
                int dn_gw, int C, int H, uintptr_t mols, uintptr_t pos, uintptr_t life, uintptr_t div,
                const GenomePoolArgs& gp, uintptr_t glen, int gw, uintptr_t ldata, uintptr_t llen, int lw, int m,
                uintptr_t cell_map, uintptr_t stream);
void halo_pack(int m, int C, int H, int elem, uintptr_t map, uintptr_t send_up, uintptr_t send_dn, uintptr_t stream);
void halo_unpack(int m, int C, int H, int elem, uintptr_t map, uintptr_t from_up, uintptr_t from_dn, uintptr_t stream);
void xb_prep(int C, int H, int n, uintptr_t pos, uintptr_t idx_map, uintptr_t lens, int width, uintptr_t len_up,
             uintptr_t len_dn, uintptr_t own1, uintptr_t ownH, uintptr_t stream);
void xb_begin(int C, int H, int n, uintptr_t pos, uintptr_t idx_map, uintptr_t glens, uintptr_t gdata, uintptr_t goff,
              int width,
              uintptr_t lens, uintptr_t own, int E, int slot_w, double p, int kcap, uint64_t seed_dn, uint64_t seed_up,
              uint64_t call, uintptr_t evbuf, uintptr_t slots, uintptr_t comm, int up, int down, uintptr_t stream);
void xb_events(int C, int E, int slot_w, double p, int kcap, uint64_t seed_dn, uint64_t seed_up, uint64_t call,
               uintptr_t mine_dn, uintptr_t from_dn, uintptr_t mine_up, uintptr_t from_up, uintptr_t own1,
               uintptr_t ownH, uintptr_t arena, uintptr_t off, uintptr_t evbuf, uintptr_t slots_dn, uintptr_t slots_up,
               uintptr_t stream);
void xb_apply(int C, int E, int slot_w, uint64_t seed_dn, uint64_t seed_up, uint64_t call, uintptr_t evbuf,
              uintptr_t slots_dn, uintptr_t slots_up, uintptr_t recv_dn, uintptr_t recv_up, uintptr_t parts,
              int parts_cap, uintptr_t pair_count, uintptr_t out, int out_width, uintptr_t out_len,
              uintptr_t out_rows, uintptr_t other, uintptr_t nres, uintptr_t stream);
void bind_gp(py::module_& m);
void bind_pool(py::module_& m);
void bind_fast(py::module_& m);
void bind_launch(py::module_& m);
}  // namespace msd

namespace {
std::atomic<uint64_t> g_seed{0xC0FFEE1234ull};
std::atomic<uint64_t> g_call{0};
}  // namespace

PYBIND11_MODULE(_hip, m) {
  m.doc() = "magicsoup_amd gfx950 (MI355X) device kernels";
  msd::gdef(m, "set_seed", [](uint64_t s) {
    g_seed.store(s);
    g_call.store(0);
  });
  msd::gdef(m, "next_call", []() { return py::make_tuple(g_seed.load(), g_call.fetch_add(1) + 1); },
        "(seed, call) for a fresh Philox stream family");
  msd::gdef(m, "get_rng_state", []() { return py::make_tuple(g_seed.load(), g_call.load()); },
        "(seed, calls drawn) of the device Philox streams");
  msd::gdef(m, "set_rng_state", [](uint64_t s, uint64_t c) {
    g_seed.store(s);
    g_call.store(c);
  }, "restore a get_rng_state() value");
  msd::gdef(m, "device_arch", []() {
    hipDeviceProp_t p;
    int dev = 0;
    MS_HIP_CHECK(hipGetDevice(&dev));
    MS_HIP_CHECK(hipGetDeviceProperties(&p, dev));
    return std::string(p.gcnArchName);
  });
  msd::gdef(m, "integrate", &msd::integrate);
  msd::gdef(m, "integrate_spec_ok", &msd::integrate_spec_ok);
  msd::gdef(m, "integrate_dist", &msd::integrate_dist);
  msd::gdef(m, "release_static", &msd::release_static);
  msd::bind_events(m);
  msd::bind_launch(m);
  msd::gdef(m, "build_params", &msd::build_params);
  msd::gdef(m, "assign_records", &msd::assign_records, "ragged parameter records for built cells (one workgroup scan)");
  msd::gdef(m, "records_to_dense", &msd::records_to_dense, "dense (n, P, s) view of the ragged parameter records");
  msd::gdef(m, "records_move", &msd::records_move, "collection: every cell's records to an exclusive-scan offset");
  msd::gdef(m, "pack_params", &msd::pack_params);
  msd::gdef(m, "diffuse_stencil", &msd::diffuse_stencil);
  msd::gdef(m, "diffuse_correct", &msd::diffuse_correct);
  msd::gdef(m, "diffuse_corr", &msd::diffuse_corr);
  msd::gdef(m, "diffuse_boundary", &msd::diffuse_boundary);
  msd::gdef(m, "diffuse_boundary_partials_len", &msd::diffuse_boundary_partials_len);
  msd::gdef(m, "diffuse_strip", &msd::diffuse_strip);
  msd::gdef(m, "map_totals", &msd::map_totals, "per-species float64 totals of owned map rows (pending corr / scale applied)");
  msd::gdef(m, "apply_pending", &msd::apply_pending);
  msd::gdef(m, "diffuse_partials_len", &msd::diffuse_partials_len);
  msd::gdef(m, "scale_planes", &msd::scale_planes);
  msd::gdef(m, "int_prof_read", &msd::int_prof_read, "register integrator phase cycles (lab builds with -DMS_INT_PROF; empty otherwise)");
  msd::gdef(m, "scale_rows", &msd::scale_rows, "x (rows, m) *= f[col] in place (fp32)");
  msd::gdef(m, "add_i32", &msd::add_i32, "x[:n] += v in place (int32)");
  msd::gdef(m, "health_scan", &msd::health_scan);
  msd::gdef(m, "gather_rows", &msd::gather_rows);
  msd::gdef(m, "neighbor_slots", &msd::neighbor_slots);
  msd::gdef(m, "rec_count_keys", &msd::rec_count_keys);
  msd::gdef(m, "spill_free", &msd::spill_free);
  msd::gdef(m, "pickup", &msd::pickup);
  msd::gdef(m, "spill_free_mask", &msd::spill_free_mask);
  msd::gdef(m, "place_rounds", &msd::place_rounds);
  msd::gdef(m, "place_rounds_mask", &msd::place_rounds_mask, "cooperative placement over cells selected by a mask");
  msd::gdef(m, "set_place_tail", &msd::set_place_tail, "1: single-launch placement with one grid barrier + a one-workgroup tail of the later rounds");
  msd::gdef(m, "set_overflow_blocks", &msd::set_overflow_blocks, "workgroups of the integrator's strided overflow-list launch");
  msd::gdef(m, "set_coop_blocks", &msd::set_coop_blocks, "workgroups of the cooperative placement (A/B)");
  msd::gdef(m, "set_stencil_vec", &msd::set_stencil_vec, "diffusion stencil columns per lane: 8 (default), 4 or 1");
  msd::gdef(m, "set_stencil_prefetch", &msd::set_stencil_prefetch, "rows the vector stencils load ahead (-1 auto, 0-3)");
  msd::gdef(m, "set_stencil_band", &msd::set_stencil_band, "rows per wave band of the vector stencils (16-256; 0 = the default 64)");
  msd::gdef(m, "set_stencil_blocks", &msd::set_stencil_blocks, "blocks of the vector diffusion stencil (0: one per tile)");
  msd::gdef(m, "set_place_mode", &msd::set_place_mode, "0 single-launch placement, ordinary launch (default), 1 multi-launch rounds, 2 single launch as a cooperative launch");
  msd::gdef(m, "place_error_take", &msd::place_error_take,
        "1 if a cooperative placement's grid barrier timed out since the last call (clears the flag)");
  msd::gdef(m, "split_cells", &msd::split_cells);
  msd::gdef(m, "permeate", &msd::permeate);
  msd::gdef(m, "claim_free", &msd::claim_free);
  msd::gdef(m, "index_map", &msd::index_map);
  msd::gdef(m, "index_map_lmax", &msd::index_map_lmax, "index map + the longest genome into a (gen << 32 | length) word");
  msd::gdef(m, "sel_sort_cap", &msd::sel_sort_cap, "capacity of the append + sort selections of the genome pipeline");
  msd::gdef(m, "neighbor_pairs_sorted", &msd::neighbor_pairs_sorted, "unique neighbour pairs in (a, b)-sorted slots");
  msd::gdef(m, "translate_count", &msd::translate_count);
  msd::gdef(m, "translate_write", &msd::translate_write);
  msd::gdef(m, "translate_fused", &msd::translate_fused);
  msd::gdef(m, "set_spl2_waves", &msd::set_spl2_waves, "waves per SIMD of the wide chemistries' narrow launch (2-4)");
  msd::gdef(m, "set_select_single_pass", &msd::set_select_single_pass, py::arg("on"), py::arg("items") = 0,
        "1: selections of <= 4M items in one launch (tile counts tagged + summed); 0: count + write passes; items: per thread of its tiles (1, 4, 16; 0 keeps)");
  msd::gdef(m, "set_rec_thinning", &msd::set_rec_thinning, "1: recombination (thinned) and mutation draws appended + sorted (0: count + selection passes)");
  msd::gdef(m, "set_rescue_mode", &msd::set_rescue_mode, "1: one launch behind the speculative integrator (0: separate)");
  msd::gdef(m, "lb_error_take", &msd::lb_error_take, "1 if a single-pass selection's look-back spin timed out");
  msd::gdef(m, "rescue_error_take", &msd::rescue_error_take, "1 if the integrator rescue launch's grid barrier timed out");
  msd::gdef(m, "set_integrate_mode", &msd::set_integrate_mode, "binned integrator launches: 0 serial, 1 concurrent, 2 concurrent + strided wide bin");
  msd::gdef(m, "translate_slot_bytes", &msd::translate_slot_bytes);
  msd::gdef(m, "mut_count", &msd::mut_count);
  msd::gdef(m, "mut_apply", &msd::mut_apply);
  msd::gdef(m, "rec_count", &msd::rec_count);
  msd::gdef(m, "rec_apply", &msd::rec_apply);
  msd::gdef(m, "arena_scatter", &msd::arena_scatter);
  msd::gdef(m, "place_collect", &msd::place_collect);
  msd::gdef(m, "divide_commit_list", &msd::divide_commit_list, "division commit with a host count (+ exporting parents)");
  msd::gdef(m, "cell_state_io", &msd::cell_state_io, "save / restore cell molecules + raw pixel values under the cells");
  msd::gdef(m, "spawn_dev", &msd::spawn_dev, "spawn_cells without a sync: claim pixels, init rows, pick up molecules, labels, genomes");
  msd::gdef(m, "divide_mask_dev", &msd::divide_mask_dev,
        "divide_cells over a mask: placement, winner compaction and commit issued without a sync; returns the status slot");
  msd::gdef(m, "translate_stats", &msd::translate_stats,
        "(max proteins, max domains, long genomes) of a translate count pass; synchronises the stream");
  msd::gdef(m, "select_indices_dev", &msd::select_indices_dev);
  msd::gdef(m, "gather_dev", &msd::gather_dev);
  msd::gdef(m, "cap_skip", &msd::cap_skip, "pipeline capacity guard: count > cap -> no-op call replayed by the host");
  msd::gdef(m, "select_indices_async", &msd::select_indices_async,
        "compaction with the count on the device and in a pinned status slot (returned); no sync");
  msd::gdef(m, "select_indices_async_pay", &msd::select_indices_async_pay,
        "select_indices_async plus pay_dst[k] = pay_src[sel[k]] (zeros past the count)");
  msd::gdef(m, "count_to_host", &msd::count_to_host, "device {count, max} -> pinned ring slot (returns the slot)");
  msd::gdef(m, "status_write", &msd::status_write, "pipeline status -> pinned ring slot (returns the slot)");
  msd::gdef(m, "status_read", &msd::status_read);
  msd::gdef(m, "status_bad_read", &msd::status_bad_read);
  msd::gdef(m, "mapped_flag", &msd::mapped_flag, "a zeroed int in mapped pinned memory: (host pointer, device pointer)");
  msd::gdef(m, "mapped_flag_read", &msd::mapped_flag_read);
  msd::gdef(m, "stream_sync_read", &msd::stream_sync_read, "synchronise a stream, then read a pinned status slot");
  msd::gdef(m, "rccl_load", &msd::rccl_load, "resolve RCCL from a loaded librccl.so path; returns its version");
  msd::gdef(m, "rccl_unique_id", [](){ return py::bytes(msd::rccl_unique_id()); });
  msd::gdef(m, "rccl_init", [](py::bytes uid, int nranks, int rank) { return msd::rccl_init(std::string(uid), nranks, rank); });
  msd::gdef(m, "rccl_destroy", &msd::rccl_destroy);
  msd::gdef(m, "rccl_async_error", &msd::rccl_async_error);
  msd::gdef(m, "rccl_guarded_wait", &msd::rccl_guarded_wait, py::call_guard<py::gil_scoped_release>(), py::arg("comms"),
        py::arg("stream"), py::arg("timeout_s"), py::arg("event") = 0,
        "wait for a stream (or one event on it) while polling RCCL errors; aborts the communicators on error / "
        "timeout");
  msd::gdef(m, "rccl_allreduce", &msd::rccl_allreduce, "in-place all-reduce on a stream (dtype 0 i32 1 f32 2 f64 3 i64; op 0 sum 1 max 2 min)");
  msd::gdef(m, "rccl_exchange", &msd::rccl_exchange, "grouped byte send/recv with the up / down neighbours on a stream");
  msd::gdef(m, "strip_marks", &msd::strip_marks, "boundary-row bytes (1 occupied, 3 dividing) for the strip neighbours");
  msd::gdef(m, "strip_reserve", &msd::strip_reserve, "halo occupancy + reservations from the neighbours' marks");
  msd::gdef(m, "strip_clear", &msd::strip_clear);
  msd::gdef(m, "place_split", &msd::place_split, "placement winners split into local / up / down (device counts + headers)");
  msd::gdef(m, "set_split_single", &msd::set_split_single, "1: place_split as one single-pass launch (0: count + write)");
  msd::gdef(m, "rec_record_bytes", &msd::rec_record_bytes);
  msd::gdef(m, "rec_pack", &msd::rec_pack);
  msd::gdef(m, "rec_unpack", &msd::rec_unpack);
  msd::gdef(m, "halo_pack", &msd::halo_pack);
  msd::gdef(m, "halo_unpack", &msd::halo_unpack);
  msd::gdef(m, "xb_prep", &msd::xb_prep);
  msd::gdef(m, "xb_events", &msd::xb_events, "strip-boundary recombination events (one workgroup, both boundaries)");
  msd::gdef(m, "xb_begin", &msd::xb_begin);
  msd::gdef(m, "xb_apply", &msd::xb_apply);
  msd::bind_fast(m);
  msd::bind_gp(m);
  msd::bind_pool(m);
  msd::gdef(m, "select_indices", &msd::select_indices,
        "(count, max) of an order-preserving compaction; synchronises the stream");
}
