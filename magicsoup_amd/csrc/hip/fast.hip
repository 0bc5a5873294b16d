// Host-floor fast paths of the steady-state World operations (GPU worlds).
//
// A strong-scaled rank of the flagship (4096^2 / 50k cells over 8 GPUs: ~6k cells per rank) spends
// its step on the host, not on the device: every operation used to rebuild its launch descriptors
// in Python (views, dtype checks, descriptor tuples, scratch lookups) before the few launches it
// issues. Here the buffers an operation touches live in one FastWorld descriptor, built once from
// the World's capacity buffers and rebuilt only when one of them is reallocated (capacity growth,
// a wider genome arena: magicsoup_amd.models.world.World._fast_world); an operation is then one C++
// call. Compactions gather into spare buffers and copy back (a few MB at most) instead of swapping,
// so buffer addresses stay fixed between reallocations and the prebuilt row plans stay valid.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <stdexcept>
#include <vector>

#include "rows.h"
#include "bind_util.h"

namespace msd {

void threshold_spill(int n, int m, int mol, float kill_below, float divide_above, float cost, float kill_p, uint64_t seed,
                     uint64_t call, uintptr_t mols, uintptr_t kill, uintptr_t divide, uintptr_t pos, int R, int C,
                     uintptr_t map, uintptr_t cell_map, int dtype, uintptr_t corr, uintptr_t stream);
void spill_free_mask(int n, int m, uintptr_t dead, uintptr_t pos, int R, int C, uintptr_t cell_mols, uintptr_t map,
                     uintptr_t cell_map, int dtype, uintptr_t corr, uintptr_t stream);
int select_indices_async(long long n, int kind, uintptr_t src, uintptr_t sel, uintptr_t rest, uintptr_t out_dev,
                         uintptr_t stream);
int select_indices_async_pay(long long n, int kind, uintptr_t src, uintptr_t sel, uintptr_t rest, uintptr_t out_dev,
                             uintptr_t pay_src, uintptr_t pay_dst, uintptr_t stream);
int divide_mask_dev(int n, uintptr_t mask, uintptr_t pos, int R, int C, int r_lo, int r_hi, int wrap, uintptr_t cell_map,
                    uintptr_t pending, uintptr_t cand, uintptr_t claim, uintptr_t result, int rounds, uint64_t seed,
                    uint64_t call, uintptr_t wins, uintptr_t dcount, long long n0, int m, uintptr_t par,
                    uintptr_t cell_mols, uintptr_t divisions, uintptr_t lifetimes, uintptr_t stream);
int divide_mask_dev_at(int n, uintptr_t mask, uintptr_t pos, int R, int C, int r_lo, int r_hi, int wrap,
                       uintptr_t cell_map, uintptr_t pending, uintptr_t cand, uintptr_t claim, uintptr_t result,
                       int rounds, uint64_t seed, uint64_t call, uintptr_t wins, uintptr_t dcount, long long n0,
                       uintptr_t n0_dev, int m, uintptr_t par, uintptr_t cell_mols, uintptr_t divisions,
                       uintptr_t lifetimes, uintptr_t stream);

struct FastWorld {
  // local map geometry (a strip of a decomposed world: halo rows, no wrap)
  int R = 0, C = 0, r_lo = 0, r_hi = 0, wrap = 1, m = 0;
  long long cap = 0;  // rows every per-cell buffer below holds
  // per-cell columns (molecules f32 (cap, m), positions i32 (cap, 2), lifetimes, divisions) + spares
  uintptr_t mols = 0, pos = 0, life = 0, div = 0, mols_sp = 0, pos_sp = 0, life_sp = 0, div_sp = 0;
  // genomes: per-cell pool offsets (int64) + int32 lengths and their spares (the bytes stay where they
  // are: compaction and cloning move offsets only; records read / write the pool `gpool`); labels:
  // rows of `l_width` bytes + int32 lengths + spares
  uintptr_t g_off = 0, g_lens = 0, g_off_sp = 0, g_lens_sp = 0;
  GenomePoolArgs gpool{};
  uintptr_t l_data = 0, l_lens = 0, l_data_sp = 0, l_lens_sp = 0;
  int l_width = 0;
  uintptr_t slot = 0, slot_sp = 0;  // kinetics cell -> parameter row map (int64)
  uintptr_t cell_map = 0;           // occupancy bytes (4-byte padded)
  // scratch, `cap` entries each (claim: R * C)
  uintptr_t sel = 0, dcount = 0, pending = 0, cand = 0, result = 0, wins = 0, par = 0, claim = 0, dcount2 = 0;
  uintptr_t dmask = 0;  // (cap bytes) the division mask of kill_divide, compacted with the survivors
  int rounds = 8;
  // prebuilt row plans: compaction into the spares, copy back, children cloned from parents
  RowArgs fwd{}, back{}, clone{};
  bool ready = false;

  void finalize() {
    if (cap <= 0 || !mols || !pos || !life || !div || !g_off || !gpool.pool || !l_data || !slot || !cell_map)
      throw std::invalid_argument("FastWorld: incomplete descriptor");
    if (!mols_sp || !pos_sp || !life_sp || !div_sp || !g_off_sp || !l_data_sp || !slot_sp)
      throw std::invalid_argument("FastWorld: missing spare buffers");
    const long long mb = 4ll * m;
    std::vector<RowDescTuple> f = {
        {mols, mols_sp, mb, mb, mb, 0},
        {pos, pos_sp, 8, 8, 8, 0},
        {life, life_sp, 4, 4, 4, 0},
        {div, div_sp, 4, 4, 4, 0},
        {g_off, g_off_sp, 8, 8, 8, 0},
        {g_lens, g_lens_sp, 4, 4, 4, 0},
        {l_data, l_data_sp, l_width, l_width, l_width, l_lens},
        {l_lens, l_lens_sp, 4, 4, 4, 0},
        {slot, slot_sp, 8, 8, 8, 0},
    };
    std::vector<RowDescTuple> b;
    for (const auto& t : f) {
      const auto& [s, d, ss, ds, rb, lp] = t;
      // copy back: the spare's lengths bound the used bytes of a copied arena row
      const uintptr_t l = lp == l_lens ? l_lens_sp : 0;
      b.emplace_back(d, s, ds, ss, rb, l);
    }
    std::vector<RowDescTuple> c = {
        {g_off, g_off, 8, 8, 8, 0},
        {g_lens, g_lens, 4, 4, 4, 0},
        {l_data, l_data, l_width, l_width, l_width, l_lens},
        {l_lens, l_lens, 4, 4, 4, 0},
        {slot, slot, 8, 8, 8, 0},
    };
    fwd = make_row_args(f);
    back = make_row_args(b);
    clone = make_row_args(c);
    ready = true;
  }
};

// kill_cells over a uint8 mask of the n cells: spill + free the dead cells' pixels (unless the
// caller did, `spill` false), order-preserving
// compaction of every per-cell buffer (device survivor count), copy back. Returns the pinned status
// slot of the survivor count (hip_ops.wait_count).
int fast_kill(const FastWorld& f, int n, uintptr_t mask, uintptr_t map, int mdt, uintptr_t corr, bool spill,
              uintptr_t stream) {
  if (!f.ready) throw std::invalid_argument("fast_kill: descriptor not finalized");
  if (n <= 0 || n > f.cap) throw std::invalid_argument("fast_kill: cell count outside the capacity");
  hipStream_t s = S_(stream);
  if (spill) spill_free_mask(n, f.m, mask, f.pos, f.R, f.C, f.mols, map, f.cell_map, mdt, corr, stream);
  const int slot = select_indices_async(n, 1 /* clear */, mask, f.sel, 0, f.dcount, stream);
  const int* dn = P_<int>(f.dcount);
  launch_row_args(f.fwd, n, dn, P_<int64_t>(f.sel), nullptr, 0, s);
  launch_row_args(f.back, n, dn, nullptr, nullptr, 0, s);
  return slot;
}

// divide_cells over a uint8 mask of the n cells: placement, winner compaction and the commit of the
// children's rows n.. (world.hip divide_mask_dev), then the genome / label / parameter-row entries
// cloned from the parents, all against the device winner count. Parents go to `par`. Returns the
// pinned status slot of the winner count.
int fast_divide(const FastWorld& f, int n, uintptr_t mask, uint64_t seed, uint64_t call, uintptr_t stream) {
  if (!f.ready) throw std::invalid_argument("fast_divide: descriptor not finalized");
  if (n <= 0 || 2ll * n > f.cap) throw std::invalid_argument("fast_divide: 2 x cell count exceeds the capacity");
  const int slot = divide_mask_dev(n, mask, f.pos, f.R, f.C, f.r_lo, f.r_hi, f.wrap, f.cell_map, f.pending, f.cand,
                                   f.claim, f.result, f.rounds, seed, call, f.wins, f.dcount2, n, f.m, f.par, f.mols,
                                   f.div, f.life, stream);
  launch_row_args(f.clone, n, P_<int>(f.dcount2), P_<int64_t>(f.par), nullptr, n, S_(stream));
  return slot;
}

// The division mask (over the n cells before the kill) compacted with the survivors: dmask[i] =
// mask[sel[i]] for the dn survivors, 0 up to n (the rows past the survivors are stale).
__global__ void __launch_bounds__(256) compact_mask_kernel(int n, const int* dn, const int64_t* sel, const uint8_t* mask,
                                                           uint8_t* dmask) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  dmask[i] = i < *dn ? mask[sel[i]] : (uint8_t)0;
}

// Threshold masks of the reference loop's kill / replicate step (performance/run_simulation.py:80-92)
// in one pass over the cells: a cell dies if its molecule `mol` is below `kill_below` (or, with
// probability `kill_p`, at random: a chemostat dilution), a surviving cell with more than
// `divide_above` pays `cost` of it and divides.
__global__ void __launch_bounds__(256) threshold_masks_kernel(int n, int m, int mol, float kill_below, float divide_above,
                                                              float cost, float kill_p, uint64_t seed, uint64_t call,
                                                              float* mols, uint8_t* kill, uint8_t* divide) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float* x = mols + (size_t)i * m + mol;
  const float v = *x;
  bool k = v < kill_below;
  if (kill_p > 0.0f) {
    Philox rng(seed, call, (uint32_t)i);
    k |= rng.uniform() < kill_p;
  }
  const bool d = !k && v > divide_above;
  if (d) *x = v - cost;
  kill[i] = k;
  divide[i] = d;
}

// kill_cells(kill) then divide_cells(divide restricted to the survivors) without a synchronisation
// in between: the kill as fast_kill, the division mask compacted with the survivors, the division
// over it with the children appended after the device survivor count (rows dn..). Both masks are
// uint8 over the same n cells. Returns the status slots of the survivor count and of the winner
// count; the population is their sum.
static std::pair<int, int> kill_divide_impl(const FastWorld& f, int n, uintptr_t kill, uintptr_t divide, uintptr_t map,
                                            int mdt, uintptr_t corr, uint64_t seed, uint64_t call, uintptr_t stream,
                                            bool spilled) {
  if (!f.ready) throw std::invalid_argument("fast_kill_divide: descriptor not finalized");
  if (n <= 0 || 2ll * n > f.cap) throw std::invalid_argument("fast_kill_divide: 2 x cell count exceeds the capacity");
  if (!f.dmask) throw std::invalid_argument("fast_kill_divide: no mask scratch");
  hipStream_t s = S_(stream);
  if (!spilled) spill_free_mask(n, f.m, kill, f.pos, f.R, f.C, f.mols, map, f.cell_map, mdt, corr, stream);
  // the survivors, and with them the division mask compacted (dmask[k] = divide[sel[k]], zeros past
  // the survivor count) in the same single-pass selection
  const int slot_k = select_indices_async_pay(n, 1 /* clear */, kill, f.sel, 0, f.dcount, divide, f.dmask, stream);
  const int* dn = P_<int>(f.dcount);
  launch_row_args(f.fwd, n, dn, P_<int64_t>(f.sel), nullptr, 0, s);
  launch_row_args(f.back, n, dn, nullptr, nullptr, 0, s);
  const int slot_d = divide_mask_dev_at(n, f.dmask, f.pos, f.R, f.C, f.r_lo, f.r_hi, f.wrap, f.cell_map, f.pending,
                                        f.cand, f.claim, f.result, f.rounds, seed, call, f.wins, f.dcount2, 0, f.dcount,
                                        f.m, f.par, f.mols, f.div, f.life, stream);
  launch_row_args(f.clone, n, P_<int>(f.dcount2), P_<int64_t>(f.par), nullptr, 0, s, dn);
  return {slot_k, slot_d};
}

std::pair<int, int> fast_kill_divide(const FastWorld& f, int n, uintptr_t kill, uintptr_t divide, uintptr_t map,
                                     int mdt, uintptr_t corr, uint64_t seed, uint64_t call, uintptr_t stream) {
  return kill_divide_impl(f, n, kill, divide, map, mdt, corr, seed, call, stream, false);
}

// The threshold masks alone (a decomposed world's strips: their division is a collective protocol)
void fast_threshold_masks(const FastWorld& f, int n, int mol, float kill_below, float divide_above, float cost,
                          float kill_p, uint64_t seed, uint64_t call, uintptr_t kill, uintptr_t divide,
                          uintptr_t stream) {
  if (!f.ready) throw std::invalid_argument("fast_threshold_masks: descriptor not finalized");
  if (n <= 0 || mol < 0 || mol >= f.m) throw std::invalid_argument("fast_threshold_masks: bad cell count or molecule");
  msd::kl(threshold_masks_kernel, cdiv(n, 256), 256, 0, S_(stream))(n, f.m, mol, kill_below, divide_above, cost, kill_p, seed,
                                                                  call, P_<float>(f.mols), P_<uint8_t>(kill),
                                                                  P_<uint8_t>(divide));
  MS_LAUNCH_CHECK();
}

// A mask over the n cells before the last fast_kill compacted with its survivors (f.sel, f.dcount)
void fast_compact_mask(const FastWorld& f, int n, uintptr_t mask, uintptr_t out, uintptr_t stream) {
  if (!f.ready || n <= 0) throw std::invalid_argument("fast_compact_mask: descriptor / count");
  msd::kl(compact_mask_kernel, cdiv(n, 256), 256, 0, S_(stream))(n, P_<int>(f.dcount), P_<int64_t>(f.sel), P_<uint8_t>(mask),
                                                               P_<uint8_t>(out));
  MS_LAUNCH_CHECK();
}

// fast_kill_divide with the masks from threshold_masks_kernel (written to kill / divide, uint8 n)
std::pair<int, int> fast_kill_divide_where(const FastWorld& f, int n, int mol, float kill_below, float divide_above,
                                           float cost, float kill_p, uint64_t mseed, uint64_t mcall, uintptr_t kill,
                                           uintptr_t divide, uintptr_t map, int mdt, uintptr_t corr, uint64_t seed,
                                           uint64_t call, uintptr_t stream) {
  if (!f.ready) throw std::invalid_argument("fast_kill_divide_where: descriptor not finalized");
  if (n <= 0 || mol < 0 || mol >= f.m) throw std::invalid_argument("fast_kill_divide_where: bad cell count or molecule");
  if (n > f.cap / 2) throw std::invalid_argument("fast_kill_divide: 2 x cell count exceeds the capacity");
  // the masks and the killed cells' spill in one launch (maps.hip threshold_spill_kernel)
  threshold_spill(n, f.m, mol, kill_below, divide_above, cost, kill_p, mseed, mcall, f.mols, kill, divide, f.pos, f.R,
                  f.C, map, f.cell_map, mdt, corr, stream);
  return kill_divide_impl(f, n, kill, divide, map, mdt, corr, seed, call, stream, true);
}

// ---- the strip protocol of a decomposed world's divide_cells over a mask (parallel/dist_world.py),
// its neighbour exchanges issued here on the native RCCL communicator `comm` (comm.hip)
void strip_marks(int C, int H, uintptr_t cell_map, int k, uintptr_t cells, uintptr_t mask, uintptr_t pos, uintptr_t up,
                 uintptr_t dn, uintptr_t stream);
void strip_reserve(int C, int H, uintptr_t from_up, uintptr_t from_dn, uintptr_t cell_map, uintptr_t stream);
void strip_clear(int C, int H, uintptr_t cell_map, uintptr_t stream);
void place_rounds_mask(int n, uintptr_t mask, uintptr_t pos, int R, int C, int r_lo, int r_hi, int wrap, bool vacate,
                       uintptr_t cell_map, uintptr_t pending, uintptr_t cand, uintptr_t claim, uintptr_t result,
                       int rounds, uint64_t seed, uint64_t call, uintptr_t stream);
void place_split(int k, uintptr_t result, uintptr_t cells, int C, int H, uintptr_t par, uintptr_t npos, uintptr_t counts,
                 uintptr_t hdr_up, uintptr_t hdr_dn, int lw, int gw, int m, uintptr_t stream);
void rec_pack(int k_up, int k_dn, uintptr_t par_up, uintptr_t pos_up, uintptr_t par_dn, uintptr_t pos_dn,
              uintptr_t mols, uintptr_t pos, uintptr_t life, uintptr_t div, const GenomePoolArgs& gp, uintptr_t glen,
              int gw, uintptr_t ldata, uintptr_t llen, int lw, int m, bool child, uintptr_t out_up, uintptr_t out_dn,
              uintptr_t stream);
void rec_unpack(int n0, int k_up, uintptr_t in_up, int up_lw, int up_gw, int k_dn, uintptr_t in_dn, int dn_lw,
                int dn_gw, int C, int H, uintptr_t mols, uintptr_t pos, uintptr_t life, uintptr_t div,
                const GenomePoolArgs& gp, uintptr_t glen, int gw, uintptr_t ldata, uintptr_t llen, int lw, int m,
                uintptr_t cell_map, uintptr_t stream);
void divide_commit_list(int k, uintptr_t par, uintptr_t npos, long long n0, int n_exp, uintptr_t exp, int m,
                        uintptr_t pos, uintptr_t cell_mols, uintptr_t divisions, uintptr_t lifetimes, uintptr_t stream);
void rccl_exchange(uintptr_t comm, int up, int down, uintptr_t send_up, long long n_send_up, uintptr_t send_down,
                   long long n_send_down, uintptr_t recv_down, long long n_recv_down, uintptr_t recv_up,
                   long long n_recv_up, uintptr_t stream);

static long long rec_bytes(int m, int lw, int gw) { return 4ll * (5 + m) + lw + gw; }

__global__ void fill_i64_kernel(int64_t* dst, const int64_t* val, int k) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < k) dst[i] = *val;
}

// Phase A (up to the one synchronisation): boundary marks -> exchange -> reservations of the
// neighbours' dividing cells -> placement over the mask -> winners split by destination (local /
// upper halo / lower halo: par3 / npos3 at offsets 0, n, 2n) with the record headers -> header
// exchange. st (int32[20]): counts [0:3], headers to up [4:8] / down [8:12], from up [12:16] / down
// [16:20]. marks: 4 C bytes. host_st (optional, pinned host memory): st is copied there at the end,
// so the host reads it after an event instead of with a stream-synchronising read-back.
void fast_dist_divide_a(const FastWorld& f, int n, uintptr_t mask, uintptr_t comm, int up, int down, uint64_t seed,
                        uint64_t call, uintptr_t marks, uintptr_t par3, uintptr_t npos3, uintptr_t st, int lw, int gw,
                        uintptr_t host_st, uintptr_t stream) {
  if (!f.ready) throw std::invalid_argument("fast_dist_divide_a: descriptor not finalized");
  if (n <= 0 || n > f.cap) throw std::invalid_argument("fast_dist_divide_a: cell count outside the capacity");
  if (f.wrap || f.r_lo != 1 || f.R != f.r_hi + 1) throw std::invalid_argument("fast_dist_divide_a: not a strip");
  const int C = f.C, H = f.r_hi - f.r_lo;
  const uintptr_t s_up = marks, s_dn = marks + C, r_dn = marks + 2 * (size_t)C, r_up = marks + 3 * (size_t)C;
  strip_marks(C, H, f.cell_map, n, 0, mask, f.pos, s_up, s_dn, stream);
  rccl_exchange(comm, up, down, s_up, C, s_dn, C, r_dn, C, r_up, C, stream);
  strip_reserve(C, H, r_up, r_dn, f.cell_map, stream);
  place_rounds_mask(n, mask, f.pos, f.R, C, f.r_lo, f.r_hi, 0, false, f.cell_map, f.pending, f.cand, f.claim, f.result,
                    f.rounds, seed, call, stream);
  place_split(n, f.result, 0, C, H, par3, npos3, st, st + 16, st + 32, lw, gw, f.m, stream);
  rccl_exchange(comm, up, down, st + 16, 16, st + 32, 16, st + 64, 16, st + 48, 16, stream);
  if (host_st)
    MS_HIP_CHECK(msd::memcpy_async(reinterpret_cast<void*>(host_st), reinterpret_cast<const void*>(st),
                                20 * sizeof(int32_t), hipMemcpyDeviceToHost, S_(stream)));
}

// The strip's kill / replicate step up to the division's one synchronisation, with no wait for the
// kill's survivor count: threshold masks + the killed cells' spill (one launch), the survivors
// selected with the division mask compacted alongside (zeros past the survivor count), every
// per-cell buffer compacted, then phase A over all n rows -- rows past the survivors carry a zero
// mask, so they take no part in the marks (the occupancy marks come from the cell map), the
// placement or the split. Indices, draws and order are those of the eager kill followed by phase A
// over the survivors. Returns the pinned status slot of the survivor count; phase B then runs with
// n0 = that count and kk = n (the par3 / npos3 offsets).
int fast_dist_kill_divide_a(const FastWorld& f, int n, int mol, float kill_below, float divide_above, float cost,
                            float kill_p, uint64_t mseed, uint64_t mcall, uintptr_t kill, uintptr_t divide,
                            uintptr_t map, int mdt, uintptr_t corr, uintptr_t comm, int up, int down, uint64_t seed,
                            uint64_t call, uintptr_t marks, uintptr_t par3, uintptr_t npos3, uintptr_t st, int lw,
                            int gw, uintptr_t host_st, uintptr_t stream) {
  if (!f.ready) throw std::invalid_argument("fast_dist_kill_divide_a: descriptor not finalized");
  if (n <= 0 || n > f.cap) throw std::invalid_argument("fast_dist_kill_divide_a: cell count outside the capacity");
  if (mol < 0 || mol >= f.m) throw std::invalid_argument("fast_dist_kill_divide_a: molecule index");
  if (!f.dmask) throw std::invalid_argument("fast_dist_kill_divide_a: no mask scratch");
  hipStream_t s = S_(stream);
  threshold_spill(n, f.m, mol, kill_below, divide_above, cost, kill_p, mseed, mcall, f.mols, kill, divide, f.pos, f.R,
                  f.C, map, f.cell_map, mdt, corr, stream);
  const int slot = select_indices_async_pay(n, 1 /* clear */, kill, f.sel, 0, f.dcount, divide, f.dmask, stream);
  const int* dn = P_<int>(f.dcount);
  launch_row_args(f.fwd, n, dn, P_<int64_t>(f.sel), nullptr, 0, s);
  launch_row_args(f.back, n, dn, nullptr, nullptr, 0, s);
  fast_dist_divide_a(f, n, f.dmask, comm, up, down, seed, call, marks, par3, npos3, st, lw, gw, host_st, stream);
  return slot;
}

// Phase B (after the synchronisation, counts known): child records of the exporting parents packed
// and exchanged, local children committed as rows n0.. (positions, halved molecules, divisions,
// lifetimes; exporters halved too) with their genome / label / parameter-row entries cloned, the
// arrivals unpacked as rows n0 + n_loc.. (their parameter rows: the all-zero row `zero_row` until
// the caller's rebuild), the halo rows cleared. The descriptor has room for every row.
void fast_dist_divide_b(const FastWorld& f, long long n0, uintptr_t comm, int up, int down, uintptr_t par3,
                        uintptr_t npos3, int kk, int n_loc, int n_up, int n_dn, int lw, int gw, uintptr_t out,
                        uintptr_t in, int in_up, int up_lw, int up_gw, int in_dn, int dn_lw, int dn_gw,
                        uintptr_t zero_row, uintptr_t stream) {
  if (!f.ready) throw std::invalid_argument("fast_dist_divide_b: descriptor not finalized");
  if (n0 + n_loc + in_up + in_dn > f.cap) throw std::invalid_argument("fast_dist_divide_b: capacity");
  const int C = f.C, H = f.r_hi - f.r_lo, m = f.m;
  const uintptr_t par_up = par3 + 8ull * kk, par_dn = par3 + 16ull * kk;
  const uintptr_t pos_up = npos3 + 8ull * kk, pos_dn = npos3 + 16ull * kk;
  const long long B = rec_bytes(m, lw, gw);
  const uintptr_t out_up = out, out_dn = out + (size_t)n_up * B;
  rec_pack(n_up, n_dn, par_up, pos_up, par_dn, pos_dn, f.mols, f.pos, f.life, f.div, f.gpool, f.g_lens, gw, f.l_data,
           f.l_lens, f.l_width, m, true, out_up, out_dn, stream);
  const long long b_up = in_up * rec_bytes(m, up_lw, up_gw), b_dn = in_dn * rec_bytes(m, dn_lw, dn_gw);
  const uintptr_t rin_up = in, rin_dn = in + (size_t)b_up;
  rccl_exchange(comm, up, down, out_up, n_up * B, out_dn, n_dn * B, rin_dn, b_dn, rin_up, b_up, stream);
  hipStream_t s = S_(stream);
  divide_commit_list(n_loc, par3, npos3, n0, n_up, par_up, m, f.pos, f.mols, f.div, f.life, stream);
  if (n_dn) divide_commit_list(0, 0, 0, n0, n_dn, par_dn, m, f.pos, f.mols, f.div, f.life, stream);
  if (n_loc) launch_row_args(f.clone, n_loc, nullptr, P_<int64_t>(par3), nullptr, n0, s);
  const int k_in = in_up + in_dn;
  if (k_in) {
    rec_unpack((int)(n0 + n_loc), in_up, rin_up, up_lw, up_gw, in_dn, rin_dn, dn_lw, dn_gw, C, H, f.mols, f.pos, f.life,
               f.div, f.gpool, f.g_lens, std::max(up_gw, dn_gw), f.l_data, f.l_lens, f.l_width, m, f.cell_map,
               stream);
    msd::kl(fill_i64_kernel, cdiv(k_in, 256), 256, 0, s)(P_<int64_t>(f.slot) + n0 + n_loc, P_<int64_t>(zero_row), k_in);
    MS_LAUNCH_CHECK();
  }
  strip_clear(C, H, f.cell_map, stream);
}

void bind_fast(pybind11::module_& m) {
  namespace py = pybind11;
  py::class_<FastWorld>(m, "FastWorld", py::module_local())
      .def(py::init<>())
      .def_readwrite("R", &FastWorld::R)
      .def_readwrite("C", &FastWorld::C)
      .def_readwrite("r_lo", &FastWorld::r_lo)
      .def_readwrite("r_hi", &FastWorld::r_hi)
      .def_readwrite("wrap", &FastWorld::wrap)
      .def_readwrite("m", &FastWorld::m)
      .def_readwrite("cap", &FastWorld::cap)
      .def_readwrite("mols", &FastWorld::mols)
      .def_readwrite("pos", &FastWorld::pos)
      .def_readwrite("life", &FastWorld::life)
      .def_readwrite("div", &FastWorld::div)
      .def_readwrite("mols_sp", &FastWorld::mols_sp)
      .def_readwrite("pos_sp", &FastWorld::pos_sp)
      .def_readwrite("life_sp", &FastWorld::life_sp)
      .def_readwrite("div_sp", &FastWorld::div_sp)
      .def_readwrite("g_off", &FastWorld::g_off)
      .def_readwrite("g_lens", &FastWorld::g_lens)
      .def_readwrite("g_off_sp", &FastWorld::g_off_sp)
      .def_readwrite("g_lens_sp", &FastWorld::g_lens_sp)
      .def_readwrite("gpool", &FastWorld::gpool)
      .def_readwrite("l_data", &FastWorld::l_data)
      .def_readwrite("l_lens", &FastWorld::l_lens)
      .def_readwrite("l_data_sp", &FastWorld::l_data_sp)
      .def_readwrite("l_lens_sp", &FastWorld::l_lens_sp)
      .def_readwrite("l_width", &FastWorld::l_width)
      .def_readwrite("slot", &FastWorld::slot)
      .def_readwrite("slot_sp", &FastWorld::slot_sp)
      .def_readwrite("cell_map", &FastWorld::cell_map)
      .def_readwrite("sel", &FastWorld::sel)
      .def_readwrite("dcount", &FastWorld::dcount)
      .def_readwrite("pending", &FastWorld::pending)
      .def_readwrite("cand", &FastWorld::cand)
      .def_readwrite("result", &FastWorld::result)
      .def_readwrite("wins", &FastWorld::wins)
      .def_readwrite("par", &FastWorld::par)
      .def_readwrite("claim", &FastWorld::claim)
      .def_readwrite("dcount2", &FastWorld::dcount2)
      .def_readwrite("dmask", &FastWorld::dmask)
      .def_readwrite("rounds", &FastWorld::rounds)
      .def("finalize", &FastWorld::finalize);
  msd::gdef(m, "fast_kill", &fast_kill, "kill_cells(mask) in one call (status slot of the survivor count)");
  msd::gdef(m, "fast_divide", &fast_divide, "divide_cells(mask) in one call (status slot of the winner count)");
  msd::gdef(m, "fast_threshold_masks", &fast_threshold_masks, "threshold kill / replicate masks (and the payment)");
  msd::gdef(m, "fast_compact_mask", &fast_compact_mask, "a mask compacted with the last fast_kill's survivors");
  msd::gdef(m, "fast_kill_divide_where", &fast_kill_divide_where,
        "threshold kill / replicate masks + fast_kill_divide in one call (status slots of both counts)");
  msd::gdef(m, "fast_kill_divide", &fast_kill_divide,
        "kill_cells(kill) + divide_cells(divide & survivors) in one call (status slots of both counts)");
  msd::gdef(m, "fast_dist_divide_a", &fast_dist_divide_a, "strip divide protocol up to the synchronisation");
  msd::gdef(m, "fast_dist_divide_b", &fast_dist_divide_b, "strip divide protocol after the synchronisation");
  msd::gdef(m, "fast_dist_kill_divide_a", &fast_dist_kill_divide_a,
        "strip kill / replicate step up to the division's synchronisation (status slot of the survivor count)");
}

}  // namespace msd
