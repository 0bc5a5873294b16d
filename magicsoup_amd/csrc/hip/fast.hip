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

#include <algorithm>
#include <stdexcept>
#include <vector>

#include "rows.h"

namespace msd {

void spill_free_mask(int n, int m, uintptr_t dead, uintptr_t pos, int R, int C, uintptr_t cell_mols, uintptr_t map,
                     uintptr_t cell_map, int dtype, uintptr_t corr, uintptr_t stream);
int select_indices_async(long long n, int kind, uintptr_t src, uintptr_t sel, uintptr_t rest, uintptr_t out_dev,
                         uintptr_t stream);
int divide_mask_dev(int n, uintptr_t mask, uintptr_t pos, int R, int C, int r_lo, int r_hi, int wrap, uintptr_t cell_map,
                    uintptr_t pending, uintptr_t cand, uintptr_t claim, uintptr_t result, int rounds, uint64_t seed,
                    uint64_t call, uintptr_t wins, uintptr_t dcount, long long n0, int m, uintptr_t par,
                    uintptr_t cell_mols, uintptr_t divisions, uintptr_t lifetimes, uintptr_t stream);

struct FastWorld {
  // local map geometry (a strip of a decomposed world: halo rows, no wrap)
  int R = 0, C = 0, r_lo = 0, r_hi = 0, wrap = 1, m = 0;
  long long cap = 0;  // rows every per-cell buffer below holds
  // per-cell columns (molecules f32 (cap, m), positions i32 (cap, 2), lifetimes, divisions) + spares
  uintptr_t mols = 0, pos = 0, life = 0, div = 0, mols_sp = 0, pos_sp = 0, life_sp = 0, div_sp = 0;
  // genome / label arenas (rows of `width` bytes + int32 lengths) + spares of the same shape
  uintptr_t g_data = 0, g_lens = 0, g_data_sp = 0, g_lens_sp = 0;
  uintptr_t l_data = 0, l_lens = 0, l_data_sp = 0, l_lens_sp = 0;
  int g_width = 0, l_width = 0;
  uintptr_t slot = 0, slot_sp = 0;  // kinetics cell -> parameter row map (int64)
  uintptr_t cell_map = 0;           // occupancy bytes (4-byte padded)
  // scratch, `cap` entries each (claim: R * C)
  uintptr_t sel = 0, dcount = 0, pending = 0, cand = 0, result = 0, wins = 0, par = 0, claim = 0, dcount2 = 0;
  int rounds = 8;
  // prebuilt row plans: compaction into the spares, copy back, children cloned from parents
  RowArgs fwd{}, back{}, clone{};
  bool ready = false;

  void finalize() {
    if (cap <= 0 || !mols || !pos || !life || !div || !g_data || !l_data || !slot || !cell_map)
      throw std::invalid_argument("FastWorld: incomplete descriptor");
    if (!mols_sp || !pos_sp || !life_sp || !div_sp || !g_data_sp || !l_data_sp || !slot_sp)
      throw std::invalid_argument("FastWorld: missing spare buffers");
    const long long mb = 4ll * m;
    std::vector<RowDescTuple> f = {
        {mols, mols_sp, mb, mb, mb, 0},
        {pos, pos_sp, 8, 8, 8, 0},
        {life, life_sp, 4, 4, 4, 0},
        {div, div_sp, 4, 4, 4, 0},
        {g_data, g_data_sp, g_width, g_width, g_width, g_lens},
        {g_lens, g_lens_sp, 4, 4, 4, 0},
        {l_data, l_data_sp, l_width, l_width, l_width, l_lens},
        {l_lens, l_lens_sp, 4, 4, 4, 0},
        {slot, slot_sp, 8, 8, 8, 0},
    };
    std::vector<RowDescTuple> b;
    for (const auto& t : f) {
      const auto& [s, d, ss, ds, rb, lp] = t;
      // copy back: the spare's lengths bound the used bytes of a copied arena row
      const uintptr_t l = lp == g_lens ? g_lens_sp : (lp == l_lens ? l_lens_sp : 0);
      b.emplace_back(d, s, ds, ss, rb, l);
    }
    std::vector<RowDescTuple> c = {
        {g_data, g_data, g_width, g_width, g_width, g_lens},
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
      .def_readwrite("g_data", &FastWorld::g_data)
      .def_readwrite("g_lens", &FastWorld::g_lens)
      .def_readwrite("g_data_sp", &FastWorld::g_data_sp)
      .def_readwrite("g_lens_sp", &FastWorld::g_lens_sp)
      .def_readwrite("l_data", &FastWorld::l_data)
      .def_readwrite("l_lens", &FastWorld::l_lens)
      .def_readwrite("l_data_sp", &FastWorld::l_data_sp)
      .def_readwrite("l_lens_sp", &FastWorld::l_lens_sp)
      .def_readwrite("g_width", &FastWorld::g_width)
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
      .def_readwrite("rounds", &FastWorld::rounds)
      .def("finalize", &FastWorld::finalize);
  m.def("fast_kill", &fast_kill, "kill_cells(mask) in one call (status slot of the survivor count)");
  m.def("fast_divide", &fast_divide, "divide_cells(mask) in one call (status slot of the winner count)");
}

}  // namespace msd
