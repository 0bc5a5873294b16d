// gfx950 kinetics kernels: fused signal integrator (World.enzymatic_activity) and the fused
// parameter builder (Kinetics.set_cell_params).
//
// Integrator mapping (see ms_kinetics.h for the exact-global-exit scheme):
//   * G lanes (32 or 64) of a wavefront own one cell; a 256-thread workgroup holds 256/G cells.
//     A cell never spans waves, so phases are separated by wave-level LDS fences, not workgroup
//     barriers: the waves of a block progress independently.
//   * The cell's active proteins (Vmax' != 0) are compacted with a ballot prefix; their
//     stoichiometry rows are staged once per part into LDS as packed int8x4 words (N, Nf, Nb, A),
//     row stride padded to an odd word count so both access patterns are bank-conflict free:
//       - protein phase: lane = protein, loops over that protein's non-zero signals (a sparse
//         index list built once per part: proteins touch a handful of the s signals);
//       - signal phase:  lane = signal, loops over proteins (consumption sums, X updates).
//   * All 4 equilibrium iterations run unconditionally; the 5 candidate states go to a snapshot
//     buffer and every cell ORs its "still correcting" bits into one word per part. The next part
//     (or the final scatter) picks the state where the reference's global `torch.any` loop stops.
//   3 part launches + 1 scatter launch per enzymatic_activity; no grid barriers, no host syncs.
#include <algorithm>
#include <unordered_map>

#include "hip_common.h"
#include "params.h"
#include "map_types.h"
#include "ms_kinetics.h"

namespace msd {

constexpr int kBlock = 256;
// Canonical summation order of the per-signal sums over a cell's active proteins (consumption, the
// candidate states): chunks of kChunk proteins in ascending order, each summed in ascending protein
// order -- the first chunk from the initial value (X0_j, or 0 for the consumption), the others from
// 0 -- and the chunk sums added to the running total in ascending chunk order. For cells with at most
// kChunk active proteins this is the plain ascending sum. Every path (LDS staging, register lanes,
// multi-group cells, the host core) sums this way, so all of them agree bit for bit, and a cell with
// many proteins can be split over several lane groups (one chunk each) without changing results.
// A candidate-state term is one fused multiply-add, fma(n_kj, w_k, sum), for every active protein
// (n_kj == 0 included: a NaN velocity turns the cell's every signal into NaN, as the reference's
// X0 + (N * V).sum(1) does, kinetics.py:759-763).
constexpr int kChunk = 32;
constexpr int kNarrowP = 12;  // LDS protein slots of the narrow integrator launch
constexpr int kWideBlocksPerCU = 2;  // resident blocks per CU of the strided wide launch
constexpr int kMaxParts = 4;  // speculative mode: 4 parts x 4 iterations in one 16-bit flag set
// binned launch mode (set_integrate_mode, for A/B on one state: scripts/lab/integrator_bench.py):
// bit 0: the wide launch on a side stream next to the narrow one (else serial, wide first); bit 1:
// the wide bin on a small strided grid (else a full grid); bit 2: 16-lane groups for the narrow
// launch. Measured at 4096^2 / 50k (3 parts, 4 iterations): serial 532 us, concurrent 558 us,
// 16-lane 590 us -- the kernel is VALU-throughput bound (37M wave instructions per launch, ~60 %
// of the SIMDs' issue capacity), so overlapping the bins only adds contention. Serial is default.
// bit 3: legacy LDS-staged path; bit 4: register path with cells sorted by active-protein count;
// bits 5 / 6: see the launcher; bit 7: no speculative all-parts launch (any of bits 3-7 disables it);
// bit 8: the speculative register launches store their final states in the snapshot for the
// write-back kernel instead of writing the world directly.
static int g_integrate_mode = 0;
// side stream + fork / join events of the legacy binned LDS launches (mode bit 0), created on first use
static hipStream_t g_lds_side = nullptr;
static hipEvent_t g_lds_fork = nullptr, g_lds_join = nullptr;
void release_kinetics_streams() {
  if (g_lds_side) MS_HIP_CHECK(hipStreamDestroy(g_lds_side));
  if (g_lds_fork) MS_HIP_CHECK(hipEventDestroy(g_lds_fork));
  if (g_lds_join) MS_HIP_CHECK(hipEventDestroy(g_lds_join));
  g_lds_side = nullptr;
  g_lds_fork = g_lds_join = nullptr;
}
void set_integrate_mode(int mode) { g_integrate_mode = mode; }

struct IntegrateArgs {
  int c, P, s;
  const int32_t* W;           // (rows, P, s) packed int8x4 stoichiometry words (N, Nf, Nb, A)
  const float4* Q;            // (rows, P)    (Vmax, Kmf, Kmb, Ke)
  const float* Kmr;           // (rows, P, s)
  const float* snap_prev;     // (c, kSnap, s) previous part's candidates (part 0: the gathered X)
  const unsigned* mask_prev;  // previous part's 4 iteration flags
  int n_iters_prev;
  float* snap_out;            // (c, kSnap, s)
  unsigned* mask_out;         // this part's 4 iteration flags (0/1, MAX-reducible across ranks)
  float trim;
  int n_iters;
  int slot_words;             // LDS words per cell slot
  int sp;                     // padded LDS row stride (odd)
  const int64_t* prow;        // cell -> parameter storage row (nullptr: identity)
  const int32_t* list;        // item -> cell (nullptr: identity)
  const int32_t* count;       // number of items in `list` (device)
  int Ps;                     // LDS protein capacity of a slot (>= active proteins of listed cells)
  // Speculative all-parts mode of the register path (spec_parts > 0, see integrate()): part p + 1
  // starts from part p's last candidate, i.e. it assumes the reference's global loop ran all n_iters
  // iterations of every part; part p's bits go to bit 4p + it of the speculative flag words, the
  // final state to slot n_iters of snap_out, and no other candidate is stored.
  int spec_parts;
  float trims[kMaxParts];
  int prelisted;              // cells with more than G active proteins are on another list: skip them
  int32_t* ovf_list;          // cells whose non-zeros / exponents do not fit this launch go here ...
  int32_t* ovf_count;
  unsigned* unfit;            // ... or, without a list, set this flag (the speculation is void)
  // LDS-path fallback launches: return at once when the speculation held (flags spec_check[0 ..
  // 4 * spec_n) all set up to n_iters, unfit word spec_check[4 * spec_n] clear); the last part's
  // launch then copies the speculative flags over the regular ones (the write-back reads those)
  const unsigned* spec_check;
  int spec_n;
  unsigned* copy_to;
  int spec_prev;              // LDS path: start from candidate n_iters_prev of snap_prev (no mask)
  // Speculative register launches: the final state goes straight to the world (cell molecules and
  // the pixels under the cells, or the explicit X) instead of snap_out; the write-back kernel then
  // only covers the LDS-list cells, or everything again if the speculation did not hold.
  int wb;
  float* wb_cm;
  void* wb_map;
  const float* wb_corr;
  const int32_t* wb_pos;
  float* wb_x;
  int wb_m, wb_R, wb_C, wb_dtype;
  // LDS-path slots in global memory instead (a proteome whose slot exceeds the 160 KiB of LDS; see
  // lds_slots): block b's slots start at gslots + b * gslot_stride * slot_words
  int* gslots = nullptr;
  int gslot_stride = 0;
};

// a.trims[q] without dynamic indexing (a dynamically indexed kernel-argument array is copied to
// scratch memory: the speculative register kernels spilled there)
__device__ __forceinline__ float trim_of(const IntegrateArgs& a, int q) {
  static_assert(kMaxParts == 4, "trim_of selects among 4 parts");
  return q == 0 ? a.trims[0] : (q == 1 ? a.trims[1] : (q == 2 ? a.trims[2] : a.trims[3]));
}

// Did the speculative all-parts launch hold? (every part ran all n_iters iterations and every cell
// was integrated)
__device__ __forceinline__ bool spec_held(const unsigned* w, int nparts, int n_iters) {
  if (w[ms::kEqIters * nparts]) return false;
  for (int p = 0; p < nparts; ++p)
    for (int it = 0; it < n_iters; ++it)
      if (!w[ms::kEqIters * p + it]) return false;
  return true;
}

__device__ __forceinline__ int stop_iter(const unsigned* flags, int n_iters) {
  for (int it = 0; it < n_iters; ++it)
    if (!flags[it]) return it;
  return n_iters;
}

__device__ __forceinline__ int w_n(int w) { return (int)(int8_t)(w & 0xFF); }
__device__ __forceinline__ int w_nf(int w) { return (w >> 8) & 0xFF; }
__device__ __forceinline__ int w_nb(int w) { return (w >> 16) & 0xFF; }
__device__ __forceinline__ int w_a(int w) { return (int)(int8_t)((w >> 24) & 0xFF); }

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// OR the "still correcting" bits (bit b -> flag word b: 4 per part) wave -> block -> at most one
// atomic per block and bit, skipped once the flag is set (tens of thousands of same-address atomics
// would serialise in one L2 channel)
__device__ __forceinline__ void or_block_bits(unsigned bits, unsigned* mask_out) {
  __shared__ unsigned wave_bits[kBlock / 64];
  for (int o = 32; o > 0; o >>= 1) bits |= __shfl_xor(bits, o);
  if ((threadIdx.x & 63) == 0) wave_bits[threadIdx.x >> 6] = bits;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned b = 0u;
    for (int w = 0; w < (int)(blockDim.x + 63) / 64; ++w) b |= wave_bits[w];
    for (int i = 0; i < ms::kEqIters * kMaxParts; ++i)
      if ((b & (1u << i)) && __hip_atomic_load(mask_out + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u)
        atomicOr(mask_out + i, 1u);
  }
}

// One cell (list item `item`) per G-lane group; ORs the cell's "still correcting" bits into `bits`.
template <int G>
__device__ __forceinline__ void integrate_item(const IntegrateArgs& a, int* smem, int item, unsigned& bits) {
  const int slot = threadIdx.x / G, lane = threadIdx.x % G;
  const bool valid0 = a.list ? item < *a.count : item < a.c;
  const int cell0 = valid0 ? (a.list ? a.list[item] : item) : 0;
  const bool valid = valid0 && (unsigned)cell0 < (unsigned)a.c;  // (a list entry is a cell index)
  const int cell = valid ? cell0 : 0;
  const int P = a.P, s = a.s, SP = a.sp, Ps = a.Ps;
  size_t pbase;  // the cell's first parameter record (params.h) ...
  int pc;        // ... and its proteins (records past them: absent, i.e. inactive)
  prot_range(a.prow, cell, P, valid, pbase, pc);

  int* words = (a.gslots ? a.gslots + (size_t)blockIdx.x * a.gslot_stride * a.slot_words : smem) +
               (size_t)slot * a.slot_words;
  int* act = words + Ps * SP;
  float* V = reinterpret_cast<float*>(act + Ps);
  float* Va = V + Ps;
  float* F = Va + Ps;
  float* kmf = F + Ps;
  float* kmb = kmf + Ps;
  float* ke = kmb + Ps;
  int* flg = reinterpret_cast<int*>(ke + Ps);
  float* X0 = reinterpret_cast<float*>(flg + Ps);
  float* Xc = X0 + s;
  float* fs = Xc + s;
  int* na_p = reinterpret_cast<int*>(fs + s);
  int* nnz = na_p + 1;                                       // (Ps,) non-zero signals per protein
  uint8_t* nzj = reinterpret_cast<uint8_t*>(nnz + Ps);        // (Ps, s) their indices

  // ---- 1. load X0: the selected candidate of the previous part (part 0: the gathered X)
  if (valid) {
    const int k = a.spec_prev ? a.n_iters_prev : stop_iter(a.mask_prev, a.n_iters_prev);
    const float* src = a.snap_prev + ((size_t)cell * ms::kSnap + k) * s;
    for (int j = lane; j < s; j += G) X0[j] = src[j];
  }

  // ---- 2. compact active proteins (Vmax' != 0) in ascending order with a ballot prefix
  {
    const int gbase = (threadIdx.x & 63) - lane;  // first lane of this group inside the wave
    int na = 0;
    for (int p0 = 0; p0 < P; p0 += G) {
      const int p = p0 + lane;
      float4 q = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
      if (p < pc) q = a.Q[pbase + p];
      const float vm = q.x * a.trim;
      const bool on = p < pc && !(vm <= 0.0f);  // NaN stays active (propagates like the reference)
      const unsigned long long bal = __ballot(on);
      unsigned long long gm;
      if constexpr (G == 64) gm = bal;
      else gm = (bal >> gbase) & ((1ull << G) - 1ull);
      const int rank = __popcll(gm & ((1ull << lane) - 1ull));
      if (on && na + rank < Ps) {
        const int k = na + rank;
        act[k] = p;
        kmf[k] = q.y;
        kmb[k] = q.z;
        ke[k] = q.w;
        V[k] = vm > 0.0f || vm != vm ? vm : 0.0f;  // temporarily holds Vmax'
      }
      na += __popcll(gm);
    }
    if (lane == 0) *na_p = na < Ps ? na : Ps;
  }
  wave_lds_sync();
  const int na = valid ? *na_p : 0;

  // ---- 3. stage the packed stoichiometry rows of the active proteins -- lanes over signals, up to
  //         8 rows (8 independent loads per lane) in flight per batch, no index division -- and
  //         each row's non-zero signals in ascending order from one wave ballot per row
  for (int j0 = 0; j0 < s; j0 += G) {
    const int j = j0 + lane;
    for (int k0 = 0; k0 < na; k0 += 8) {
      int w[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + u;
        w[u] = (k < na && j < s) ? a.W[(pbase + act[k]) * s + j] : 0;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + u;
        if (k < na && j < s) words[k * SP + j] = w[u];
      }
    }
  }
  wave_lds_sync();
  {
    const int gbase = (threadIdx.x & 63) - lane;  // first lane of this group inside the wave
    for (int k = 0; k < na; ++k) {                 // group-uniform trip count
      int cnt = 0;
      for (int j0 = 0; j0 < s; j0 += G) {
        const int j = j0 + lane;
        const bool on = j < s && words[k * SP + j] != 0;
        const unsigned long long bal = __ballot(on);
        unsigned long long gm;
        if constexpr (G == 64) gm = bal;
        else gm = (bal >> gbase) & ((1ull << G) - 1ull);
        if (on) nzj[k * s + cnt + __popcll(gm & ((1ull << lane) - 1ull))] = (uint8_t)j;
        cnt += __popcll(gm);
      }
      if (lane == 0) nnz[k] = cnt;
    }
  }
  wave_lds_sync();

  // ---- 4. velocities (protein phase)
  for (int k = lane; k < na; k += G) {
    const int* wr = words + k * SP;
    const float* kmr = a.Kmr + (pbase + act[k]) * s;
    const uint8_t* nz = nzj + k * s;
    const int cnt = nnz[k];
    float xf = 1.0f, xb = 1.0f, ar = 1.0f;
    bool anyf = false, anyb = false;
    for (int q = 0; q < cnt; ++q) {
      const int j = nz[q];
      const int w = wr[j];
      const int nf = w_nf(w), nb = w_nb(w), av = w_a(w);
      const float x = X0[j];
      if (nf > 0) {
        xf *= ms::ipow(x, nf);
        anyf = true;
      }
      if (nb > 0) {
        xb *= ms::ipow(x, nb);
        anyb = true;
      }
      if (av != 0) {
        float r = ms::ipow(x, av);
        r = r / (r + kmr[j]);
        if (ms::f_isnan(r)) r = 1.0f;
        ar *= r;
      }
    }
    float kf = ms::clean_prod(xf) / kmf[k];
    if (!anyf) kf = 0.0f;
    if (ms::f_isinf(kf)) kf = ms::kMax;
    float kb = ms::clean_prod(xb) / kmb[k];
    if (!anyb) kb = 0.0f;
    if (ms::f_isinf(kb)) kb = ms::kMax;
    if (ms::f_isinf(ar)) ar = ms::kMax;
    const float acat = (kf - kb) / (1.0f + kf + kb);
    float v = acat * V[k] * ar;
    v = v < ms::kMin ? ms::kMin : (v > ms::kMax ? ms::kMax : v);
    V[k] = v;
  }
  wave_lds_sync();

  // ---- 5. consumption per signal and the negative-concentration factors (signal phase; sums in the
  //         canonical chunk order, see kChunk)
  for (int j = lane; j < s; j += G) {
    float cons = 0.0f;
    for (int k0 = 0; k0 < na; k0 += kChunk) {
      const int k1 = min(k0 + kChunk, na);
      float part = 0.0f;
      for (int k = k0; k < k1; ++k) {
        const float nv = (float)w_n(words[k * SP + j]) * V[k];
        if (nv < 0.0f) part += -nv;
      }
      cons = k0 == 0 ? part : cons + part;
    }
    const float f = X0[j] / cons;
    fs[j] = f > 1.0f ? 1.0f : f;
  }
  wave_lds_sync();

  // ---- 6. per-protein limiting factor (protein phase)
  for (int k = lane; k < na; k += G) {
    const int* wr = words + k * SP;
    const float v = V[k];
    const uint8_t* nz = nzj + k * s;
    const int cnt = nnz[k];
    float fmin = 1.0f;
    bool nan = false;
    for (int q = 0; q < cnt; ++q) {
      const int j = nz[q];
      const int n = w_n(wr[j]);
      if ((float)n * v < 0.0f) {
        const float f = fs[j];
        if (ms::f_isnan(f)) nan = true;
        else if (f < fmin) fmin = f;
      }
    }
    Va[k] = v * (nan ? NAN : fmin);
    F[k] = 1.0f;
    flg[k] = (v > 0.0f ? 1 : 0) | (fabsf(v) > 0.1f ? 2 : 0);
  }
  wave_lds_sync();

  // ---- 7. X1 (signal phase), candidate 0
  // X0_j + sum_k n_kj * w_k over the active proteins in the canonical chunk order
  auto chunk_sum = [&](int j, auto&& w_of) {
    float x = X0[j];
    for (int k0 = 0; k0 < na; k0 += kChunk) {
      const int k1 = min(k0 + kChunk, na);
      float part = k0 == 0 ? x : 0.0f;
      for (int k = k0; k < k1; ++k) {
        const int n = w_n(words[k * SP + j]);
        part = fmaf((float)n, w_of(k), part);
      }
      x = k0 == 0 ? part : x + part;
    }
    return x;
  };
  float* snap = a.snap_out + (size_t)(valid ? cell : 0) * ms::kSnap * s;
  for (int j = lane; j < s; j += G) {
    float x = chunk_sum(j, [&](int k) { return Va[k]; });
    x = x < 0.0f ? 0.0f : x;
    Xc[j] = x;
    if (valid) snap[j] = x;
  }
  wave_lds_sync();

  // ---- 8. equilibrium damping trajectory
  float inc = 0.5f;
  const int gbase8 = (threadIdx.x & 63) - lane;  // first lane of this group inside the wave
  for (int it = 0; it < a.n_iters; ++it, inc *= 0.5f) {
    bool changed = false;
    bool cb = false;  // this cell has an impactful correction at iteration it
    for (int k = lane; k < na; k += G) {
      const int* wr = words + k * SP;
      const uint8_t* nz = nzj + k * s;
      const int cnt = nnz[k];
      float pf = 1.0f, pb = 1.0f;
      bool anyf = false, anyb = false;
      for (int q = 0; q < cnt; ++q) {
        const int j = nz[q];
        const int w = wr[j];
        const int nf = w_nf(w), nb = w_nb(w);
        if (nf > 0) {
          pf *= ms::ipow(Xc[j], nf);
          anyf = true;
        }
        if (nb > 0) {
          pb *= ms::ipow(Xc[j], nb);
          anyb = true;
        }
      }
      pf = anyf ? ms::clean_prod(pf) : 0.0f;
      pb = anyb ? ms::clean_prod(pb) : 0.0f;
      float Q = pb / pf;
      if (ms::f_isnan(Q)) Q = 1.0f;
      else Q = Q < ms::kEps ? ms::kEps : (Q > ms::kMax ? ms::kMax : Q);
      const float qke = Q / ke[k];
      const bool fwd = flg[k] & 1, imp = flg[k] & 2;
      const float f0 = F[k];
      bool low = fwd ? (qke < ms::kLower) : (qke > ms::kUpper);
      if (fwd && f0 == 1.0f) low = false;
      bool high = fwd ? (qke > ms::kUpper) : (qke < ms::kLower);
      if (!fwd && f0 == 0.0f) high = false;
      if ((low || high) && imp) {
        bits |= 1u << it;
        cb = true;
      }
      float f = f0;
      if (high) f -= inc;
      if (low) f += inc;
      f = f > 1.0f ? 1.0f : (f < 0.0f ? 0.0f : f);
      changed |= f != f0;
      F[k] = f;
    }
    wave_lds_sync();
    {
      // per-cell fixed point: with no factor changed, this and every later iteration reproduce the
      // current state bit for bit (same F, same X, same decisions), so the remaining candidates are
      // copies of it and the iterations are skipped. The later iterations would also repeat this
      // one's decisions, so an impactful correction that changed nothing (a backward reaction whose
      // factor is capped at 1) keeps the reference's global loop running: its bit is carried forward.
      const unsigned long long bal = __ballot(changed);
      unsigned long long gm;
      if constexpr (G == 64) gm = bal;
      else gm = (bal >> gbase8) & ((1ull << G) - 1ull);
      if (gm == 0ull) {
        unsigned long long cgm = __ballot(cb);
        if constexpr (G != 64) cgm = (cgm >> gbase8) & ((1ull << G) - 1ull);
        if (cgm) bits |= ((1u << a.n_iters) - 1u) & ~((2u << it) - 1u);
        for (int it2 = it + 1; it2 <= a.n_iters; ++it2) {
          float* sn2 = snap + (size_t)it2 * s;
          for (int j = lane; j < s; j += G)
            if (valid) sn2[j] = Xc[j];
        }
        break;
      }
    }
    float* sn = snap + (size_t)(it + 1) * s;
    for (int j = lane; j < s; j += G) {
      float x = chunk_sum(j, [&](int k) { return Va[k] * F[k]; });
      x = x < 0.0f ? 0.0f : x;
      Xc[j] = x;
      if (valid) sn[j] = x;
    }
    wave_lds_sync();
  }
}

// kStride: grid-stride over groups of cells with a block-uniform trip count (the wide bin runs on
// a small grid next to the narrow launch); otherwise one group per block.
template <int G, bool kStride>
__global__ void __launch_bounds__(kBlock) integrate_part_kernel(IntegrateArgs a) {
  extern __shared__ __attribute__((aligned(16))) int smem[];
  const int cps = blockDim.x / G, slot = threadIdx.x / G;
  if (a.spec_check && spec_held(a.spec_check, a.spec_n, a.n_iters)) {
    // the speculative launch held: nothing to redo (the last part hands its flags over)
    if (a.copy_to && blockIdx.x == 0 && (int)threadIdx.x < ms::kEqIters * a.spec_n)
      a.copy_to[threadIdx.x] = a.spec_check[threadIdx.x];
    return;
  }
  unsigned bits = 0u;
  if constexpr (kStride) {
    const int limit = a.list ? *a.count : a.c;
    for (int base = (int)blockIdx.x * cps; base < limit; base += (int)gridDim.x * cps) {
      integrate_item<G>(a, smem, base + slot, bits);
      wave_lds_sync();
    }
  } else {
    integrate_item<G>(a, smem, (int)blockIdx.x * cps + slot, bits);
  }

  // ---- 9. OR the "still correcting" bits
  or_block_bits(bits, a.mask_out);
}

// Speculative all-parts mode for the cells no register launch can take (more than 64 active proteins,
// more than 2 * kNzReg non-zeros, large exponents): every listed cell runs all parts on the LDS path
// (integrate_item), part p > 0 starting from part p - 1's candidate n_iters, in place in snap_out
// (a cell's group reads its own previous output before writing any candidate); part p's bits go to
// flag words 4p.. (a.mask_out). a.snap_prev holds the input (slot 0), a.trims the parts' trims.
template <int G>
__global__ void __launch_bounds__(kBlock) integrate_spec_lds_kernel(IntegrateArgs a) {
  extern __shared__ __attribute__((aligned(16))) int smem[];
  const int cps = blockDim.x / G, slot = threadIdx.x / G;
  unsigned bits = 0u;
  const int limit = *a.count;
  for (int base = (int)blockIdx.x * cps; base < limit; base += (int)gridDim.x * cps) {
    for (int part = 0; part < a.spec_parts; ++part) {
      IntegrateArgs ap = a;
      ap.trim = trim_of(a, part);
      ap.spec_prev = part > 0;
      ap.snap_prev = part > 0 ? a.snap_out : a.snap_prev;
      unsigned b = 0u;
      integrate_item<G>(ap, smem, base + slot, b);
      bits |= b << (ms::kEqIters * part);
      wave_lds_sync();
    }
  }
  or_block_bits(bits, a.mask_out);
}

// ---------------------------------------------------------------------------------------------
// Register-resident integrator (the default for s <= 64): G lanes own one cell and every lane plays
// two roles -- lane j is signal j (X0_j, the current X_j and the column n_{0..na-1, j} of the
// stoichiometry, packed int8 in registers) and lane k is active protein k (velocity, damping factor,
// Ke / direction flags and its first kNzReg non-zero signals in registers). The roles exchange
// values through two small LDS arrays: protein lanes publish one float each (read back by the
// signal lanes as 16-byte broadcasts, four proteins per load) and signal lanes publish X_j (gathered
// by the protein lanes, all loads independent). Entries past a protein's non-zero count are zero
// words, which leave every product unchanged, so the protein loops run branch-free to the wave's
// largest count. Every sum and product runs in the same order as integrate_item (ascending protein
// / ascending signal), so both paths give bit-identical results (scripts/lab/integrator_bench.py). A
// cell with more than G active proteins is appended (part 0) to the wide list and integrated by
// integrate_item with all P protein slots.
constexpr int kNzReg = 16;  // non-zero signals per protein in the LDS lists (more: the cell goes wide)
constexpr int kNzWide = 2 * kNzReg;  // the same for the 64-lane launch of the wide list

// LDS row strides of the per-protein non-zero lists: NZ entry words + 1 and NZ index bytes + 4 (an
// odd number of words). Protein lanes read entry q of their own row in lock step, so with a stride
// of NZ words (a multiple of the bank count's divisors) all lanes of a wave hit 64 / NZ banks: 16-
// to 32-way bank conflicts on every entry read (profiles/r3/wide/pmc_wide_integrator_stencil.txt:
// 2.47 M per dispatch). An odd stride spreads the lanes over all banks.
template <int NZ>
constexpr int ent_stride() { return NZ + 1; }
template <int NZ>
constexpr int jl_stride() { return NZ + 4; }

// LDS words per cell slot of the register-resident integrator (SPL signals per lane: s <= SPL * G)
template <int G, int NZ, int SPL = 1>
constexpr int fast_slot_words() {
  return G * ent_stride<NZ>() /*entry words*/ + G * jl_stride<NZ>() / 4 /*entry signal indices*/ +
         3 * G /*cnt, act, pub*/ + SPL * G /*X*/;
}

template <int G>
__device__ __forceinline__ unsigned long long group_ballot(bool b) {
  const unsigned long long bal = __ballot(b);
  if constexpr (G == 64) return bal;
  else return (threadIdx.x & 32) ? (bal >> 32) : (bal & 0xFFFFFFFFull);
}

__device__ __forceinline__ int wave_max(int v) {
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
  return v;
}

// ms::ipow for |n| < 8 without branches: the same multiplications in the same order
__device__ __forceinline__ float ipow_small(float x, int n) {
  const int e = n < 0 ? -n : n;
  float r = 1.0f, b = x;
  r = (e & 1) ? r * b : r;
  b = b * b;
  r = (e & 2) ? r * b : r;
  b = b * b;
  r = (e & 4) ? r * b : r;
  return n < 0 ? 1.0f / r : r;
}

// A protein's non-zero entry in 16 bits: signal j, forward / backward exponents. SPL == 1 (s <= 64):
// j 6 bits, nf / nb 5 bits (< 32); SPL == 2 (s <= 128): j 7 bits, nf / nb 4 bits (< 16: a larger
// exponent sends the cell to the LDS path, which has no such limit).
template <int SPL>
struct E16 {
  static constexpr int kJ = SPL == 1 ? 6 : 7, kN = SPL == 1 ? 5 : 4;
  static constexpr int kMaxExp = 1 << kN;
  __device__ static int pack(int j, int nf, int nb) { return j | (nf << kJ) | (nb << (kJ + kN)); }
  __device__ static int j(int e) { return e & ((1 << kJ) - 1); }
  __device__ static int nf(int e) { return (e >> kJ) & ((1 << kN) - 1); }
  __device__ static int nb(int e) { return (e >> (kJ + kN)) & ((1 << kN) - 1); }
};

// Register-resident integration of one cell (see above). SPL = 2 (the wide chemistries, s <= 128):
// lane l plays signals l and l + G; the per-signal sums still run over proteins in ascending order
// and a protein's products over its non-zero signals in ascending signal order (half 0 before half
// 1), exactly as integrate_item, so all paths stay bit-identical.
// Multi-group cells (NG > 1, G == 32, SPL == 1): the NG groups of a block share ONE cell. Group g holds
// active proteins [g * G, g * G + G) -- one canonical chunk (kChunk == G) -- with the same register
// and LDS layout as a single-group cell; the per-signal sums are formed per chunk and combined across
// the groups through LDS in ascending chunk order (the canonical order, so the results are those of
// every other path bit for bit). A cell with up to NG * G active proteins then runs as G-protein
// chains plus one block barrier per signal pass, instead of one 64-lane chain (or an LDS-path chain)
// over all of them. The cross-group words need no LDS of their own (the block keeps the narrow
// launch's 6 blocks per CU): each group publishes its votes in the padding words of its slot's
// entry-index rows (bytes NZ .. JS of a row are never written) and its chunk sums in the entry-index
// bytes (jl) past those rows' votes, which are dead once the protein lanes hold their entries in
// registers.
template <int NZ>
constexpr int vote_word(int v) { return (v * jl_stride<NZ>() + NZ) / 4; }  // row v's pad
constexpr int kMgSumWord = 16;  // first jl word of the chunk-sum buffers (past the vote rows 0..2)

// Phase timing of the register integrator (lab builds only: -DMS_INT_PROF, scripts/lab/int_prof.py):
// cycles per phase of the first cell of a launch, summed over launches, read by int_prof_read().
#ifdef MS_INT_PROF
__device__ unsigned long long g_int_prof[64];
#define MS_PROBE(id)                                                   \
  do {                                                                 \
    if (item == 0 && lane == 0 && grp == 0) {                          \
      const unsigned long long t_ = clock64();                         \
      g_int_prof[id] += t_ - prof_t;                                   \
      prof_t = t_;                                                     \
    }                                                                  \
  } while (0)
#else
#define MS_PROBE(id) \
  do {               \
  } while (0)
#endif

template <int G, int NZ, bool kSpec = false, int SPL = 1, int NG = 1>
__device__ __forceinline__ void integrate_item_fast(const IntegrateArgs& a, int* smem, int item, unsigned& bits,
                                                    int32_t* wide_list, int32_t* wide_count) {
  using EP = E16<SPL>;
  static_assert(NG == 1 || (G == kChunk && SPL == 1 && kSpec && NG * G <= kBlock),
                "multi-group cells: 32-lane groups, one signal per lane, speculative launches");
  static_assert(G == kChunk || G == 2 * kChunk, "a group covers one or two canonical chunks");
  const int slot = threadIdx.x / G, lane = threadIdx.x % G;
  const int grp = NG > 1 ? slot : 0;  // this group's chunk of the cell's active proteins
#ifdef MS_INT_PROF
  unsigned long long prof_t = clock64();
#endif
  const bool listed0 = a.list ? item < *a.count : item < a.c;
  const int cell0 = listed0 ? (a.list ? a.list[item] : item) : 0;
  const bool listed = listed0 && (unsigned)cell0 < (unsigned)a.c;  // (a list entry is a cell index)
  const int cell = listed ? cell0 : 0;
  const int P = a.P, s = a.s;
  size_t pbase;  // the cell's parameter records (params.h)
  int pc;
  prot_range(a.prow, cell, P, listed, pbase, pc);
  // wave-uniform bound of the protein scan (its ballots need every lane of the wave)
  const int pc_w = __builtin_amdgcn_readfirstlane(wave_max(pc));

  constexpr int ES = ent_stride<NZ>(), JS = jl_stride<NZ>();
  constexpr int SW = fast_slot_words<G, NZ, SPL>();
  int* ents = smem + slot * SW;                                  // (G, ES) words of the non-zeros
  uint8_t* jl = reinterpret_cast<uint8_t*>(ents + G * ES);  // (G, JS) bytes: their signal indices
  int* cnts = ents + G * ES + G * JS / 4;                    // (G,) non-zero signals per protein
  int* act = cnts + G;                                           // (G,) protein slot of active protein k
  float* pub = reinterpret_cast<float*>(act + G);                // (G,) protein -> signal: V_k / Va_k * F_k
  float* Xs = pub + G;                                           // (SPL * G,) signal -> protein: X_j / factor
  int pass = 0;                                                  // multi-group: chunk-sum buffer parity

  // ---- 1. X0 of this lane's signals (independent of the compaction, issued first)
  float x0[SPL];
  {
    const int k = listed ? stop_iter(a.mask_prev, a.n_iters_prev) : 0;
#pragma unroll
    for (int h = 0; h < SPL; ++h) {
      const int j = lane + h * G;
      x0[h] = (listed && j < s) ? a.snap_prev[((size_t)cell * ms::kSnap + k) * s + j] : 0.0f;
    }
  }

  MS_PROBE(0);
  // ---- 2. active proteins (Vmax' != 0, NaN included) in ascending order; group grp keeps entries
  //         [grp * G, grp * G + G) of the compacted list
  constexpr bool spec = kSpec;
  const int nparts = spec ? a.spec_parts : 1;
  int na = 0;
  bool trim_diff = false;  // speculative mode: every part must see the same active set
  for (int p0 = 0; p0 < pc_w; p0 += G) {
    const int p = p0 + lane;
    float vmax = 0.0f;
    if (p < pc) vmax = a.Q[pbase + p].x;
    const float vm = vmax * (spec ? a.trims[0] : a.trim);
    const bool on = p < pc && !(vm <= 0.0f);
    for (int q = 1; q < nparts; ++q) trim_diff |= on != (p < pc && !(vmax * trim_of(a, q) <= 0.0f));
    const unsigned long long gm = group_ballot<G>(on);
    const int k = na + __popcll(gm & ((1ull << lane) - 1ull)) - grp * G;
    if (on && k >= 0 && k < G) act[k] = p;
    na += __popcll(gm);
  }
  bool fits = na <= NG * G;
  wave_lds_sync();
  const int nac = fits ? min(max(na - grp * G, 0), G) : 0;  // this group's active proteins
  // wave-uniform bound of the protein loops (both groups of a wave), in an SGPR: scalar loop exits
  const int na_w = __builtin_amdgcn_readfirstlane(wave_max(nac));

  MS_PROBE(1);
  // ---- 3. this lane's signals' stoichiometry columns (int8 n per protein, packed in registers) and
  //         the per-protein non-zero lists (one ballot per protein and half), 8 rows of loads in flight
  int npk[SPL][G / 4];
#pragma unroll
  for (int h = 0; h < SPL; ++h)
#pragma unroll
    for (int i = 0; i < G / 4; ++i) npk[h][i] = 0;
  bool wide_ok = true;  // every protein has <= NZ non-zeros and exponents below the entry limit
#pragma unroll
  for (int k0 = 0; k0 < G; k0 += 8) {
    if (k0 >= na_w) break;
    int w[SPL][8];
#pragma unroll
    for (int h = 0; h < SPL; ++h)
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + u, j = lane + h * G;
        w[h][u] = (k < nac && listed && j < s) ? a.W[(pbase + act[k]) * s + j] : 0;
      }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int k = k0 + u;
      int base = 0;
#pragma unroll
      for (int h = 0; h < SPL; ++h) {
        npk[h][k >> 2] |= (w[h][u] & 0xFF) << (8 * (k & 3));
        const bool on = w[h][u] != 0;
        const unsigned long long gm = group_ballot<G>(on);
        const int r = base + __popcll(gm & ((1ull << lane) - 1ull));
        if (on && r < NZ) {
          ents[k * ES + r] = w[h][u];
          jl[k * JS + r] = (uint8_t)(lane + h * G);
        }
        base += __popcll(gm);
        wide_ok &= w_nf(w[h][u]) < EP::kMaxExp && w_nb(w[h][u]) < EP::kMaxExp;
      }
      if (lane == 0 && k < nac) cnts[k] = base;
      wide_ok &= base <= NZ;
    }
  }
  MS_PROBE(2);
  bool nz_ok = group_ballot<G>(!wide_ok) == 0ull;
  // multi-group: word v of group g's votes (a pad word of its slot's entry-index rows)
  auto vote = [&](int g, int v) -> int& { return smem[g * SW + G * ES + vote_word<NZ>(v)]; };
  if constexpr (NG > 1) {
    static_assert(JS - NZ >= 4 && vote_word<NZ>(2) < kMgSumWord, "vote words must be row padding");
    // the cell fits only if every group's proteins do (one block-wide vote)
    if (lane == 0) vote(grp, 0) = nz_ok ? 1 : 0;
    __syncthreads();
#pragma unroll
    for (int g = 0; g < NG; ++g) nz_ok &= vote(g, 0) != 0;
  }
  // (multi-group: one report per cell, from group 0)
  const bool reporter = listed && lane == 0 && grp == 0;
  if (!spec) {
    fits = fits && nz_ok;
    if (!fits && reporter && wide_list) wide_list[atomicAdd(wide_count, 1)] = cell;
  } else if (reporter) {
    // too many active proteins: skipped when the cell is on the wide list already (prelisted);
    // otherwise, and with too many non-zeros / large exponents, the cell goes to the overflow list
    // (the next, wider launch), without one the speculation is void; so is a cell whose active set
    // differs between parts (a Vmax' underflowing to 0)
    if (!(!fits && a.prelisted) && (!fits || !nz_ok)) {
      if (a.ovf_list) a.ovf_list[atomicAdd(a.ovf_count, 1)] = cell;
      else __hip_atomic_store(a.unfit, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (spec) {
    if (listed && group_ballot<G>(trim_diff) != 0ull && lane == 0)
      __hip_atomic_store(a.unfit, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    fits = fits && nz_ok;
  }
  const bool valid = listed && fits;
  bool sig[SPL];
#pragma unroll
  for (int h = 0; h < SPL; ++h) sig[h] = valid && lane + h * G < s && grp == 0;  // (the writer of the cell)
  const bool prot = valid && lane < nac;
  const int nchunks = valid ? (na + kChunk - 1) / kChunk : 0;  // (multi-group: uniform over the block)
#pragma unroll
  for (int h = 0; h < SPL; ++h) Xs[lane + h * G] = x0[h];
  wave_lds_sync();

  // protein lane: constants, and its non-zeros as 16-bit (signal, nf, nb) registers for the
  // damping iterations (velocity and limiting factor read the full words from LDS once per part)
  float vraw = 0.0f, kmf = 1.0f, kmb = 1.0f, ke = 1.0f;
  int pk = 0, cnt = 0;
  int e16[NZ / 2];
#pragma unroll
  for (int q = 0; q < NZ / 2; ++q) e16[q] = 0;
  bool small = true;  // all exponents < 8: branch-free powers
  bool both = false;  // an entry with forward and backward exponents (a signal consumed and produced)
  bool allo = false;  // an allosteric entry (a != 0)
  int nfs_p = 0, nbs_p = 0;  // any forward / backward exponent of this protein
  if (prot) {
    pk = act[lane];
    const float4 q4 = a.Q[pbase + pk];
    vraw = q4.x;
    kmf = q4.y;
    kmb = q4.z;
    ke = q4.w;
    cnt = cnts[lane];
    const int* jw = reinterpret_cast<const int*>(jl + lane * JS);
#pragma unroll
    for (int q = 0; q < NZ; ++q) {
      if (q < cnt) {
        const int w = ents[lane * ES + q];
        const int j = (jw[q >> 2] >> (8 * (q & 3))) & 0xFF;
        const int e = EP::pack(j, w_nf(w), w_nb(w));
        e16[q >> 1] |= e << (16 * (q & 1));
        small &= w_nf(w) < 8 && w_nb(w) < 8 && w_a(w) < 8 && w_a(w) > -8;
        both |= w_nf(w) > 0 && w_nb(w) > 0;
        allo |= w_a(w) != 0;
        nfs_p |= w_nf(w);
        nbs_p |= w_nb(w);
      }
    }
  }
  const int cnt_w = __builtin_amdgcn_readfirstlane(wave_max(cnt));
  const bool small_w = __ballot(!small) == 0ull;
  const bool one_w = __ballot(both) == 0ull;  // every entry has one exponent: one power per entry
  const bool allo_w = __ballot(allo) != 0ull;  // any allosteric entry in the wave (else no word reads)
#define MS_E(q) ((e16[(q) >> 1] >> (16 * ((q) & 1))) & 0xFFFF)
  auto pw = [&](float x, int n) { return small_w ? ipow_small(x, n) : ms::ipow(x, n); };

  // signal lane, half h: acc[h] (the initial value) + sum over this group's proteins k (ascending) of
  // op(n_kj, pub[k]), four proteins per LDS load, in the canonical chunk order: a 64-lane group sums
  // its second chunk (proteins 32..63) separately and adds it after the first. Multi-group cells
  // then combine the groups' chunk sums (combine below).
  auto signal_pass = [&](float (&acc)[SPL], auto&& op) {
    float part[SPL];
#pragma unroll
    for (int h = 0; h < SPL; ++h) part[h] = 0.0f;
    // the stoichiometry bytes are loop-invariant over the parts and damping iterations: without this
    // (empty) redefinition LICM hoists all G * SPL sign-extended n's out of the loops, into registers
    // (128 of them for SPL == 2: 296 B/lane of scratch at 4 waves, 204 in the flagship's fused launch)
#pragma unroll
    for (int h = 0; h < SPL; ++h)
#pragma unroll
      for (int i = 0; i < G / 4; ++i) asm volatile("" : "+v"(npk[h][i]));
#pragma unroll
    for (int k0 = 0; k0 < G; k0 += 4) {
      if (k0 >= na_w) break;
      const float4 b4 = *reinterpret_cast<const float4*>(pub + k0);
      const float bv[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = k0 + u;
#pragma unroll
        for (int h = 0; h < SPL; ++h) {
          const int n = (int)(int8_t)(npk[h][k >> 2] >> (8 * (k & 3)));
          if (k < kChunk) op(acc[h], n, bv[u]);
          else op(part[h], n, bv[u]);
        }
      }
    }
    if constexpr (G > kChunk) {
      if (nac > kChunk) {
#pragma unroll
        for (int h = 0; h < SPL; ++h) acc[h] += part[h];
      }
    }
  };
  // multi-group: group g's chunk sum (group 0's includes the initial value) -> the cell's sum, read by
  // every group from the others' slots in ascending chunk order (double-buffered by pass parity: a
  // group writing pass i + 2 has passed pass i + 1's barrier, so every group has read pass i)
  auto combine = [&](float (&x)[SPL]) {
    if constexpr (NG > 1) {
      constexpr int kJlWords = G * JS / 4;
      static_assert(kMgSumWord + 2 * G <= kJlWords, "chunk-sum buffers must fit the entry-index bytes");
      const int off = kMgSumWord + (pass & 1) * G + lane;
      reinterpret_cast<float*>(jl)[off] = x[0];
      __syncthreads();
      float t = x[0];
      if (grp != 0) t = reinterpret_cast<const float*>(smem + G * ES)[off];
      for (int g = 1; g < nchunks; ++g) t += reinterpret_cast<const float*>(smem + g * SW + G * ES)[off];
      x[0] = t;
      ++pass;
    }
  };
  // multi-group: a predicate over the cell's protein lanes (one block barrier); else over the group
  auto cell_any = [&](bool b, int word) {
    if constexpr (NG > 1) {
      const bool gb = group_ballot<G>(b) != 0ull;  // (all lanes: a ballot under lane == 0 sees one lane)
      if (lane == 0) vote(grp, 1 + word) = gb ? 1 : 0;
      __syncthreads();
      int any = 0;
#pragma unroll
      for (int g = 0; g < NG; ++g) any |= vote(g, 1 + word);
      return any != 0;
    } else {
      return group_ballot<G>(b) != 0ull;
    }
  };

  // parts: one (the launch's trim), or all of them in the speculative mode; x0 / Xs carry the state
  float* snap = a.snap_out + (size_t)(valid ? cell : 0) * ms::kSnap * s;
  float xc[SPL];
#pragma unroll
  for (int h = 0; h < SPL; ++h) xc[h] = x0[h];
  MS_PROBE(3);
  for (int part = 0; part < nparts; ++part) {
  const float vm = vraw * (spec ? trim_of(a, part) : a.trim);
  const float vmx = prot && (vm > 0.0f || vm != vm) ? vm : 0.0f;
  const int bsh = spec ? ms::kEqIters * part : 0;  // this part's bits
  // ---- 4. velocity (protein lane; entries past the count are zero words: no effect)
  float v = 0.0f;
  {
    const float* kmr = a.Kmr + (pbase + pk) * s;
    float xf = 1.0f, xb = 1.0f, ar = 1.0f;
#pragma unroll
    for (int q = 0; q < NZ; ++q) asm volatile("" : "+v"(e16[q >> 1]));  // (no hoisting, see signal_pass)
#pragma unroll
    for (int q = 0; q < NZ; ++q) {
      if (q < cnt_w) {
        const int e = MS_E(q);
        const int j = EP::j(e), nf = EP::nf(e), nb = EP::nb(e);
        const float x = Xs[j];
        if (one_w) {  // (as in the damping loop: the entry's one power)
          const float p = pw(x, nf | nb);
          xf = nf > 0 ? xf * p : xf;
          xb = nb > 0 ? xb * p : xb;
        } else {
          xf = nf > 0 ? xf * pw(x, nf) : xf;
          xb = nb > 0 ? xb * pw(x, nb) : xb;
        }
        if (allo_w) {  // (the allosteric exponent is in the full word only)
          const int av = w_a(q < cnt ? ents[lane * ES + q] : 0);
          if (av != 0) {
            float r = pw(x, av);
            r = r / (r + kmr[j]);
            if (ms::f_isnan(r)) r = 1.0f;
            ar *= r;
          }
        }
      }
    }
    if (prot) {
      float kf = ms::clean_prod(xf) / kmf;
      if (nfs_p == 0) kf = 0.0f;
      if (ms::f_isinf(kf)) kf = ms::kMax;
      float kb = ms::clean_prod(xb) / kmb;
      if (nbs_p == 0) kb = 0.0f;
      if (ms::f_isinf(kb)) kb = ms::kMax;
      if (ms::f_isinf(ar)) ar = ms::kMax;
      const float acat = (kf - kb) / (1.0f + kf + kb);
      v = acat * vmx * ar;
      v = v < ms::kMin ? ms::kMin : (v > ms::kMax ? ms::kMax : v);
    }
  }
  pub[lane] = v;
  wave_lds_sync();

  MS_PROBE(4);
  // ---- 5. consumption per signal -> negative-concentration factor (signal lane)
  {
    float cons[SPL];
#pragma unroll
    for (int h = 0; h < SPL; ++h) cons[h] = 0.0f;
    signal_pass(cons, [](float& acc, int n, float vk) {
      // (acc - min(nv, 0): the sum of the consumptions -nv > 0, bit for bit; a NaN nv adds nothing)
      acc -= fminf((float)n * vk, 0.0f);
    });
    combine(cons);
#pragma unroll
    for (int h = 0; h < SPL; ++h) {
      const float f = x0[h] / cons[h];
      Xs[lane + h * G] = f > 1.0f ? 1.0f : f;  // Xs holds the factors until candidate 0 exists
    }
  }
  wave_lds_sync();

  MS_PROBE(5);
  // ---- 6. per-protein limiting factor (protein lane)
  float va = 0.0f, F = 1.0f;
  int flg = 0;
  {
    float fmin = 1.0f;
    bool nan = false;
#pragma unroll
    for (int q = 0; q < NZ; ++q) {
      if (q < cnt_w) {
        const int w = q < cnt ? ents[lane * ES + q] : 0;
        if ((float)w_n(w) * v < 0.0f) {
          const float f = Xs[EP::j(MS_E(q))];
          if (ms::f_isnan(f)) nan = true;
          else if (f < fmin) fmin = f;
        }
      }
    }
    if (prot) {
      va = v * (nan ? NAN : fmin);
      flg = (v > 0.0f ? 1 : 0) | (fabsf(v) > 0.1f ? 2 : 0);
    }
  }
  pub[lane] = va;
  wave_lds_sync();

  MS_PROBE(6);
  // ---- 7. candidate 0 (signal lane)
  auto advance = [&]() {  // X0 + sum_k n_k * pub_k (canonical order), clamped at 0
    float x[SPL];
#pragma unroll
    for (int h = 0; h < SPL; ++h) x[h] = grp == 0 ? x0[h] : 0.0f;  // (multi-group: chunk 0 starts from X0)
    signal_pass(x, [](float& acc, int n, float b) {
      acc = fmaf((float)n, b, acc);
    });
    combine(x);
#pragma unroll
    for (int h = 0; h < SPL; ++h) xc[h] = x[h] < 0.0f ? 0.0f : x[h];
  };
  advance();
#pragma unroll
  for (int h = 0; h < SPL; ++h) {
    if (sig[h] && !spec) snap[lane + h * G] = xc[h];
    Xs[lane + h * G] = xc[h];
  }
  wave_lds_sync();

  MS_PROBE(7);
  // ---- 8. equilibrium damping trajectory
  float inc = 0.5f;
  for (int it = 0; it < a.n_iters; ++it, inc *= 0.5f) {
    bool changed = false, cb = false;
#pragma unroll
    for (int q = 0; q < NZ / 2; ++q) asm volatile("" : "+v"(e16[q]));  // (the same for the entry fields)
    {
      float pf = 1.0f, pb = 1.0f;
#pragma unroll
      for (int q = 0; q < NZ; ++q) {
        if (q < cnt_w) {
          const int e = MS_E(q);
          const int nf = EP::nf(e), nb = EP::nb(e);
          const float x = Xs[EP::j(e)];
          if (one_w) {  // (nf == 0 or nb == 0: x^(nf | nb) is the one power the entry needs)
            const float p = pw(x, nf | nb);
            pf = nf > 0 ? pf * p : pf;
            pb = nb > 0 ? pb * p : pb;
          } else {
            pf = nf > 0 ? pf * pw(x, nf) : pf;
            pb = nb > 0 ? pb * pw(x, nb) : pb;
          }
        }
      }
      if (prot) {
        pf = nfs_p ? ms::clean_prod(pf) : 0.0f;
        pb = nbs_p ? ms::clean_prod(pb) : 0.0f;
        float Q = pb / pf;
        if (ms::f_isnan(Q)) Q = 1.0f;
        else Q = Q < ms::kEps ? ms::kEps : (Q > ms::kMax ? ms::kMax : Q);
        const float qke = Q / ke;
        const bool fwd = flg & 1, imp = flg & 2;
        const float f0 = F;
        bool low = fwd ? (qke < ms::kLower) : (qke > ms::kUpper);
        if (fwd && f0 == 1.0f) low = false;
        bool high = fwd ? (qke > ms::kUpper) : (qke < ms::kLower);
        if (!fwd && f0 == 0.0f) high = false;
        cb = (low || high) && imp;
        if (cb) bits |= 1u << (bsh + it);
        float f = f0;
        if (high) f -= inc;
        if (low) f += inc;
        f = f > 1.0f ? 1.0f : (f < 0.0f ? 0.0f : f);
        changed = f != f0;
        F = f;
      }
    }
    if (!cell_any(changed, 0)) {
      // per-cell fixed point (see integrate_item): the remaining candidates are copies, and an
      // impactful correction that changed nothing repeats in every remaining iteration
      if (cell_any(cb, 1)) bits |= (((1u << a.n_iters) - 1u) & ~((2u << it) - 1u)) << bsh;
      if (!spec)
        for (int it2 = it + 1; it2 <= a.n_iters; ++it2)
#pragma unroll
          for (int h = 0; h < SPL; ++h)
            if (sig[h]) snap[(size_t)it2 * s + lane + h * G] = xc[h];
      break;
    }
    pub[lane] = va * F;
    wave_lds_sync();  // the protein lanes of this wave finished reading Xs, published Va * F
    advance();
#pragma unroll
    for (int h = 0; h < SPL; ++h) {
      if (sig[h] && !spec) snap[(size_t)(it + 1) * s + lane + h * G] = xc[h];
      Xs[lane + h * G] = xc[h];
    }
    wave_lds_sync();
  }
#pragma unroll
  for (int h = 0; h < SPL; ++h) x0[h] = xc[h];  // the next part starts from this part's last candidate
  MS_PROBE(8);
  }
  if (spec) {
#pragma unroll
    for (int h = 0; h < SPL; ++h) {
      if (!sig[h]) continue;
      const int j = lane + h * G;
      if (!a.wb) {
        snap[(size_t)a.n_iters * s + j] = xc[h];
      } else if (a.wb_x) {
        a.wb_x[(size_t)cell * s + j] = xc[h];
      } else if (j < a.wb_m) {
        a.wb_cm[(size_t)cell * a.wb_m + j] = xc[h];
      } else {
        const size_t pix = (size_t)a.wb_pos[2 * cell] * a.wb_C + a.wb_pos[2 * cell + 1];
        st_map(a.wb_map, (size_t)(j - a.wb_m) * a.wb_R * a.wb_C + pix, corr_out(xc[h], a.wb_corr, j - a.wb_m),
               a.wb_dtype);
      }
    }
  }
  MS_PROBE(9);
#ifdef MS_INT_PROF
  if (item == 0 && lane == 0 && grp == 0) g_int_prof[63] += 1;
#endif
#undef MS_E
}

// kStrided: a list launch of unknown length (a.count on the device) on a small grid; each block
// walks the list in steps of the whole grid (the bound is block-uniform, so every wave runs the
// same number of items and the wave-wide ballots / reductions inside stay convergent)
#ifndef MS_SPL2_WAVES
#define MS_SPL2_WAVES 4  // waves per SIMD the two-signals-per-lane launches are compiled for
#endif
template <int G, int NZ, bool kStrided, bool kSpec = false, int SPL = 1>
__global__ void __launch_bounds__(kBlock, G == 32 ? 6 : (NZ == kNzReg ? (SPL == 2 ? MS_SPL2_WAVES : 4) : 1)) integrate_fast_kernel(IntegrateArgs a, int32_t* wide_list,
                                                                int32_t* wide_count) {
  extern __shared__ __attribute__((aligned(16))) int smem[];
  unsigned bits = 0u;
  const int cpb = (int)blockDim.x / G;
  if constexpr (kStrided) {
    const int n = *a.count;
    for (int base = (int)blockIdx.x * cpb; base < n; base += (int)gridDim.x * cpb) {
      wave_lds_sync();  // the previous item's LDS reads are done before its slot is refilled
      integrate_item_fast<G, NZ, kSpec, SPL>(a, smem, base + (int)threadIdx.x / G, bits, wide_list, wide_count);
    }
  } else {
    integrate_item_fast<G, NZ, kSpec, SPL>(a, smem, (int)blockIdx.x * cpb + (int)threadIdx.x / G, bits, wide_list,
                                           wide_count);
  }
  or_block_bits(bits, a.mask_out);
}

// The narrow cells of the speculative all-parts launch on their own, compiled for W waves per SIMD
// (A/B of the occupancy / register-spill trade: at 6 waves the path spills, at 5 it does not).
template <int W>
__global__ void __launch_bounds__(kBlock, W) integrate_narrow_spec_kernel(IntegrateArgs a) {
  extern __shared__ __attribute__((aligned(16))) int smem[];
  unsigned bits = 0u;
  integrate_item_fast<32, kNzReg, true>(a, smem, (int)blockIdx.x * (kBlock / 32) + (int)threadIdx.x / 32, bits, nullptr,
                                         nullptr);
  or_block_bits(bits, a.mask_out);
}

// The two-signals-per-lane narrow cells (s <= 128: the wide chemistries) of the speculative launch,
// compiled for W waves per SIMD: the path needs ~256 VGPRs to run without spills (316 B/lane of
// scratch at 4 waves, 208 at 3, 44 at 2), so occupancy and spills trade (set_spl2_waves).
template <int W>
__global__ void __launch_bounds__(kBlock, W) integrate_spl2_spec_kernel(const IntegrateArgs* __restrict__ args) {
  extern __shared__ __attribute__((aligned(16))) int smem[];
  const IntegrateArgs& a = args[0];  // (device memory, as integrate_spec_fused_kernel)
  unsigned bits = 0u;
  integrate_item_fast<64, kNzReg, true, 2>(a, smem, (int)blockIdx.x * (kBlock / 64) + (int)threadIdx.x / 64, bits,
                                           nullptr, nullptr);
  or_block_bits(bits, a.mask_out);
}
static int g_spl2_waves = 4;
void set_spl2_waves(int w) { g_spl2_waves = w <= 2 ? 2 : (w >= 4 ? 4 : 3); }

// Parts >= 1 of the register path with the wide list (known from part 0) in the same launch: the
// first `nwb` blocks walk the wide list with two 64-lane slots each (integrate_item_fast<64,
// kNzWide>, the rest of the block idles), the others take the cells as integrate_fast_kernel<G>.
// A wide cell's integration is a long dependency chain (~30 us on its own); at the front of the
// grid it runs under the narrow blocks instead of after them. Cells that do not fit the 64-lane
// slots either are skipped here (part 0 listed them for the LDS launch).
template <int G, bool kSpec = false, int W = 6>
__global__ void __launch_bounds__(kBlock, W) integrate_fused_kernel(IntegrateArgs a, IntegrateArgs aw, int nwb) {
  extern __shared__ __attribute__((aligned(16))) int smem[];
  static_assert(2 * fast_slot_words<64, kNzWide>() <= (kBlock / G) * fast_slot_words<G, kNzReg>(),
                "two wide slots must fit the narrow block's LDS");
  unsigned bits = 0u;
  if ((int)blockIdx.x < nwb) {
    if (threadIdx.x < 128) {
      const int n = *aw.count;  // block-uniform bound: both waves run the same number of items
      for (int base = (int)blockIdx.x * 2; base < n; base += nwb * 2) {
        wave_lds_sync();
        integrate_item_fast<64, kNzWide, kSpec>(aw, smem, base + (int)threadIdx.x / 64, bits, nullptr, nullptr);
      }
    }
  } else {
    integrate_item_fast<G, kNzReg, kSpec>(a, smem, ((int)blockIdx.x - nwb) * (kBlock / G) + (int)threadIdx.x / G, bits,
                                   nullptr, nullptr);
  }
  or_block_bits(bits, a.mask_out);
}

// The speculative all-parts launch for the 32-lane chemistries (s <= 32): every block first takes
// cells of the wide list (more than 32 active proteins, listed by gather_bin_kernel), strided over
// the whole grid, each as ONE multi-group cell (the block's 8 groups: up to 256 active proteins, one
// canonical chunk per group), then its own 8 narrow cells. A grown population's wide cells thus run
// at the front of the grid with as many blocks as there are such cells, each as 32-protein chains,
// under the narrow cells' throughput work instead of after it. Cells that fit neither role (too
// many proteins or non-zeros, large exponents) go to the overflow lists for the launches behind.
// (not inlined: the wide role's second copy of integrate_item_fast has a register allocation of its
// own instead of adding its uniform values to the narrow path's -- 498 -> 76 SGPR spills with the
// argument blocks in memory, below)
__device__ __attribute__((noinline)) void integrate_wide_cells(const IntegrateArgs& aw, int* smem, unsigned& bits) {
  const int nw = *aw.count;  // (block-uniform: the multi-group cell's barriers need every wave)
  for (int item = (int)blockIdx.x; item < nw; item += (int)gridDim.x) {
    integrate_item_fast<32, kNzReg, true, 1, kBlock / 32>(aw, smem, item, bits, nullptr, nullptr);
    __syncthreads();  // the cell's slots and votes are reused by the next item
  }
}

// The two argument blocks (narrow, wide) are read from device memory (args[0], args[1]: written by
// the input kernel before it, gather_bin_kernel) instead of being passed by value: by-value blocks
// were loaded into SGPRs at the kernel start and spilled (498 SGPR spills, 84 B/lane of scratch at
// the 80-VGPR cap); through a pointer the fields are loaded where they are used.
template <int W>
__global__ void __launch_bounds__(kBlock, W) integrate_spec_fused_kernel(const IntegrateArgs* __restrict__ args) {
  extern __shared__ __attribute__((aligned(16))) int smem[];
  const IntegrateArgs& a = args[0];
  const IntegrateArgs& aw = args[1];
  constexpr int kGroups = kBlock / 32;
  unsigned bits = 0u;
  if ((int)blockIdx.x < *aw.count) integrate_wide_cells(aw, smem, bits);
  integrate_item_fast<32, kNzReg, true>(a, smem, (int)blockIdx.x * kGroups + (int)threadIdx.x / 32, bits, nullptr,
                                        nullptr);
  or_block_bits(bits, a.mask_out);
}

// Everything behind the speculative fused launch of a single-process world in two launches (the
// 32-lane chemistries; decomposed worlds all-reduce flags between these stages and keep the separate
// launches). Usually every list is empty and the speculation held: each block reads a few words and
// writes nothing back -- two launches instead of the five that used to return at once plus the
// write-back. The grid is co-resident (at most one block per CU, like the placement's cooperative
// launch), so phases that feed each other are separated by a software grid barrier, taken only when
// the phase before had work:
//   A. (a launch of its own before this one: inlined here, its 64-lane registers spilled) the narrow
//      launch's overflow list (at most 32 active proteins, more non-zeros / large exponents) on
//      64-lane slots with 2 * kNzReg non-zeros; what these cannot take goes on to list B;
//   B. the cells no register path took, all parts on the LDS path (cps cells per block);
//   C. only if the speculation failed (some part's reference loop ended early for the whole
//      population, or a cell was unfit): the exact per-part LDS integration of every cell, a grid
//      barrier after each part (part p + 1 starts from part p's candidate the global flags select);
//   D. the write-back: the list-B cells' final states when the speculation held (the register paths
//      wrote theirs), every cell's selected candidate when it did not.
struct RescueArgs {
  IntegrateArgs lb;      // phase B (list wl3 / count wc3, LDS slots of slot_words)
  IntegrateArgs fb;      // phase C, part 0 (the later parts differ in the fields below)
  const float* fb_snap_prev[kMaxParts];
  const unsigned* fb_mask_prev[kMaxParts];
  float* fb_snap_out[kMaxParts];
  unsigned* fb_mask_out[kMaxParts];
  int cps;               // LDS-path cells per block
  int nparts, n_iters;
  const unsigned* sflags;  // speculative flags (4 per part) + unfit word
  unsigned* masks;       // regular per-part flags (the host reads these)
  unsigned* barrier;     // grid-barrier counter (zeroed by the input kernel)
  unsigned* err_host;    // barrier timeout (mapped host word), optional
  int* wide_reset;       // the wide-list count, zeroed for the next call
  int all_from_snap;     // the register launches left their final states in snap_spec (mode bit 8)
  // write-back
  int c, s, m, R, C, map_dtype;
  const float* snap_spec;  // where the speculative LDS path left its final states (slot n_iters)
  const float* snap_last;  // the exact path's last part
  const int32_t* positions;
  float* cell_mols;
  void* molmap;
  const float* corr;
  float* X_out;
};

// v[q] of a kernel-argument array without dynamic indexing (that copies the array to scratch)
template <class T>
__device__ __forceinline__ T sel4(const T (&v)[kMaxParts], int q) {
  static_assert(kMaxParts == 4, "sel4 selects among 4 parts");
  return q == 0 ? v[0] : (q == 1 ? v[1] : (q == 2 ? v[2] : v[3]));
}

__device__ void rescue_barrier(unsigned* ctr, unsigned& phase, unsigned* err_host) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();  // this block's stores (snapshots, outputs) reach agent scope before the arrival
    const unsigned target = (++phase) * gridDim.x;
    atomicAdd(ctr, 1u);
    for (long long spin = 0; __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target; ++spin) {
      if (spin > (1ll << 24)) {  // a grid that is not co-resident: report instead of hanging
        if (err_host) __hip_atomic_store(err_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    __threadfence();  // the other blocks' stores are visible to this CU's waves
  }
  __syncthreads();
}

__device__ __forceinline__ void rescue_store(const RescueArgs& r, int cell, int j, float x) {
  if (r.X_out) {
    r.X_out[(size_t)cell * r.s + j] = x;
  } else if (j < r.m) {
    r.cell_mols[(size_t)cell * r.m + j] = x;
  } else {
    const size_t pix = (size_t)r.positions[2 * cell] * r.C + r.positions[2 * cell + 1];
    st_map(r.molmap, (size_t)(j - r.m) * r.R * r.C + pix, corr_out(x, r.corr, j - r.m), r.map_dtype);
  }
}

__global__ void __launch_bounds__(kBlock, 1) integrate_rescue_kernel(RescueArgs r) {
  extern __shared__ __attribute__((aligned(16))) int smem[];
  unsigned phase = 0;
  unsigned bits = 0u;
  // ---- B (list A ran in the launch before: its 64-lane path in this kernel spilled ~1 KB per lane)
  const int cB = *r.lb.count;
  const int slot = (int)threadIdx.x / 32;
  if (cB > 0) {
    for (int base = (int)blockIdx.x * r.cps; base < cB; base += (int)gridDim.x * r.cps) {
      if (slot < r.cps) {
        for (int part = 0; part < r.nparts; ++part) {
          IntegrateArgs ap = r.lb;
          ap.trim = trim_of(r.lb, part);
          ap.spec_prev = part > 0;
          ap.snap_prev = part > 0 ? r.lb.snap_out : r.lb.snap_prev;
          unsigned b = 0u;
          integrate_item<32>(ap, smem, base + slot, b);
          bits |= b << (ms::kEqIters * part);
          wave_lds_sync();
        }
      }
      __syncthreads();  // (slots are refilled by the next items)
    }
    or_block_bits(bits, r.lb.mask_out);
    bits = 0u;
    rescue_barrier(r.barrier, phase, r.err_host);  // (flags and snapshots for the verdict / write-back)
  }
  const bool held = spec_held(r.sflags, r.nparts, r.n_iters);
  const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x, nth = (long long)gridDim.x * blockDim.x;
  if (held) {
    // the regular flags are the speculative ones (the host reads those)
    if (blockIdx.x == 0 && (int)threadIdx.x < ms::kEqIters * r.nparts) r.masks[threadIdx.x] = r.sflags[threadIdx.x];
    // ---- D (held): list-B cells (or every cell, all_from_snap), candidate n_iters of the
    //      speculative snapshots
    const long long nb = r.all_from_snap ? r.c : cB;
    for (long long t = tid; t < nb * r.s; t += nth) {
      const int i = (int)(t / r.s), j = (int)(t - (long long)i * r.s);
      const int cell = r.all_from_snap ? i : r.lb.list[i];
      if ((unsigned)cell >= (unsigned)r.c) continue;
      rescue_store(r, cell, j, r.snap_spec[((size_t)cell * ms::kSnap + r.n_iters) * r.s + j]);
    }
  } else {
    // ---- C: the exact per-part path over every cell
    for (int part = 0; part < r.nparts; ++part) {
      IntegrateArgs f = r.fb;
      f.snap_prev = sel4(r.fb_snap_prev, part);
      f.mask_prev = sel4(r.fb_mask_prev, part);
      f.snap_out = sel4(r.fb_snap_out, part);
      f.mask_out = sel4(r.fb_mask_out, part);
      f.trim = trim_of(r.fb, part);
      for (int base = (int)blockIdx.x * r.cps; base < r.c; base += (int)gridDim.x * r.cps) {
        if (slot < r.cps) integrate_item<32>(f, smem, base + slot, bits);
        __syncthreads();
      }
      or_block_bits(bits, f.mask_out);
      bits = 0u;
      rescue_barrier(r.barrier, phase, r.err_host);  // (part + 1 selects by these global flags)
    }
    // ---- D (not held): every cell's selected candidate of the last part
    const int k = stop_iter(r.masks + ms::kEqIters * (r.nparts - 1), r.n_iters);
    for (long long t = tid; t < (long long)r.c * r.s; t += nth) {
      const int cell = (int)(t / r.s), j = (int)(t - (long long)cell * r.s);
      rescue_store(r, cell, j, r.snap_last[((size_t)cell * ms::kSnap + k) * r.s + j]);
    }
  }
  if (tid == 0) r.wide_reset[0] = 0;  // (the wide-list count, for the next call)
}

static int g_rescue_mode = 1;  // 0: the separate launches (A/B)
void set_rescue_mode(int m) { g_rescue_mode = m; }
// workgroups of the strided 64-lane overflow-list launch (its length is only known on the device)
static unsigned g_ovf_blocks = 64;
void set_overflow_blocks(int n) { g_ovf_blocks = (unsigned)std::max(1, std::min(n, 4096)); }
static unsigned g_rescue_blocks = 0;  // co-resident grid: one block per CU
static unsigned* g_rescue_err = nullptr;
static unsigned* g_rescue_err_dev = nullptr;
int rescue_error_take() {
  if (!g_rescue_err) return 0;
  return __atomic_exchange_n(g_rescue_err, 0u, __ATOMIC_ACQ_REL) ? 1 : 0;
}

// Split the cells by their number of active proteins (Vmax > 0 or NaN; the same set for every part
// since all trims are positive): cells with at most `pn` go to the narrow list (small LDS slots,
// high occupancy), the others to the wide list (slots for all P proteins). List order does not
// matter: cells are independent and the iteration flags are OR-reduced.
__global__ void __launch_bounds__(256) bin_cells_kernel(int c, int P, int pn, const float4* Q, const int64_t* prow,
                                                        int32_t* lists, int32_t* counts) {
  const int cell = blockIdx.x * blockDim.x + threadIdx.x;
  if (cell >= c) return;
  size_t r;
  int pc;
  prot_range(prow, cell, P, true, r, pc);
  int na = 0;
  for (int p = 0; p < pc; ++p) na += !(Q[r + p].x <= 0.0f);
  if (na <= pn) lists[atomicAdd(counts, 1)] = cell;
  else lists[c + atomicAdd(counts + 1, 1)] = cell;
}

// Final state -> cell_molecules and the molecule-map pixels under the cells.
__global__ void __launch_bounds__(kBlock) integrate_scatter_kernel(int c, int s, int m, int R, int C, const float* snap,
                                                                   const unsigned* mask, int n_iters,
                                                                   const int32_t* positions, float* cell_mols,
                                                                   void* molmap, int map_dtype, const float* corr,
                                                                   float* X_out, unsigned* reset,
                                                                   const unsigned* spec_flags, int spec_n,
                                                                   const int32_t* lds_list, const int32_t* lds_count) {
  const long long t0 = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (reset && t0 == 0) reset[0] = 0u;  // the speculative path's wide-list count, for the next call
  // grid-stride (a bounded grid): after a speculation that held, the register launches wrote their
  // cells already and only the LDS-list cells are left, usually none
  const bool held = spec_flags && spec_held(spec_flags, spec_n, n_iters);
  const long long total = (long long)(held ? *lds_count : c) * s;
  const int k = stop_iter(mask, n_iters);
  for (long long t = t0; t < total; t += (long long)gridDim.x * blockDim.x) {
    int cell = (int)(t / s);
    const int j = (int)(t - (long long)cell * s);
    if (held) {
      cell = lds_list[cell];
      if ((unsigned)cell >= (unsigned)c) continue;
    }
    const float x = snap[((size_t)cell * ms::kSnap + k) * s + j];
    if (X_out) {
      X_out[(size_t)cell * s + j] = x;
    } else if (j < m) {
      cell_mols[(size_t)cell * m + j] = x;
    } else {
      const size_t pix = (size_t)positions[2 * cell] * C + positions[2 * cell + 1];
      st_map(molmap, (size_t)(j - m) * R * C + pix, corr_out(x, corr, j - m), map_dtype);
    }
  }
}

// X (c, s) -> snapshot slot 0 with an all-zero mask, so a part kernel can start from an explicit X.
// Both input kernels also clear the launch's flag words (zero[0..nz)) and the wide-list counter
// (zero_wc, optional) from block 0: no separate memset launches before part 0.
constexpr int kSortBuckets = 34;  // active-protein counts 0..32, and "more" (the wide bin)

__device__ __forceinline__ void clear_words(unsigned* zero, int nz, int32_t* zero_wc) {
  if (blockIdx.x == 0) {
    if ((int)threadIdx.x < nz) zero[threadIdx.x] = 0u;
    if (threadIdx.x == 0 && zero_wc) {
      zero_wc[0] = 0;
      zero_wc[-1] = 0;  // the second-level wide count (cells the 64-lane fast launch cannot take)
    }
    // the active-protein sort's histogram and cursors follow the wide-list counter
    if (zero_wc && (int)threadIdx.x < 2 * kSortBuckets) zero_wc[1 + threadIdx.x] = 0;
  }
}

// Active proteins per cell (Vmax > 0 or NaN: the set every part integrates, all trims being
// positive) into a histogram; with the scatter below, the register-resident launches take the cells
// in order of that count, so the two cells sharing a wave have similar protein / non-zero counts
// and the wave-uniform loop bounds (the larger of the two) waste fewer lanes (mode bit 4; measured
// slower, see the launcher).
__global__ void __launch_bounds__(256) na_hist_kernel(int c, int P, const float4* Q, const int64_t* prow,
                                                      uint8_t* na_out, int32_t* hist, int32_t* total) {
  __shared__ int h[kSortBuckets];
  if (blockIdx.x == 0 && threadIdx.x == 0) *total = c;
  if ((int)threadIdx.x < kSortBuckets) h[threadIdx.x] = 0;
  __syncthreads();
  const int cell = blockIdx.x * blockDim.x + threadIdx.x;
  if (cell < c) {
    size_t r;
    int pc;
    prot_range(prow, cell, P, true, r, pc);
    int na = 0;
    for (int p = 0; p < pc; ++p) na += !(Q[r + p].x <= 0.0f);
    const int b = na > 32 ? 33 : na;
    na_out[cell] = (uint8_t)b;
    atomicAdd(&h[b], 1);
  }
  __syncthreads();
  if ((int)threadIdx.x < kSortBuckets && h[threadIdx.x]) atomicAdd(hist + threadIdx.x, h[threadIdx.x]);
}

__global__ void __launch_bounds__(256) na_scatter_kernel(int c, const uint8_t* na, const int32_t* hist, int32_t* cursor,
                                                         int32_t* order) {
  __shared__ int base[kSortBuckets];
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int b = 0; b < kSortBuckets; ++b) {
      base[b] = acc;
      acc += hist[b];
    }
  }
  __syncthreads();
  const int cell = blockIdx.x * blockDim.x + threadIdx.x;
  if (cell >= c) return;
  const int b = na[cell];
  order[base[b] + atomicAdd(cursor + b, 1)] = cell;
}

__global__ void load_x_kernel(int c, int s, const float* X, float* snap, unsigned* zero, int nz, int32_t* zero_wc) {
  clear_words(zero, nz, zero_wc);
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)c * s) return;
  const int cell = (int)(t / s), j = (int)(t - (long long)cell * s);
  snap[(size_t)cell * ms::kSnap * s + j] = X[t];
}

// Part 0 input: X = (cell molecules | molecules of the cell's pixel) -> candidate 0 of `snap`.
// A flat, full-occupancy gather, so the random pixel reads (one per species plane) are not on the
// LDS-limited integrator's critical path.
__global__ void __launch_bounds__(kBlock) gather_x_kernel(int c, int s, int m, int R, int C, const float* cell_mols,
                                                          const void* molmap, int map_dtype, const float* corr,
                                                          const int32_t* positions, float* snap, unsigned* zero,
                                                          int nz, int32_t* zero_wc) {
  clear_words(zero, nz, zero_wc);
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)c * s) return;
  const int cell = (int)(t / s), j = (int)(t - (long long)cell * s);
  float x;
  if (j < m) {
    x = cell_mols[(size_t)cell * m + j];
  } else {
    const size_t pix = (size_t)positions[2 * cell] * C + positions[2 * cell + 1];
    x = corr_in(ld_map(molmap, (size_t)(j - m) * R * C + pix, map_dtype), corr, j - m);
  }
  snap[(size_t)cell * ms::kSnap * s + j] = x;
}

// Input of the speculative all-parts path: X (the explicit X, or gathered from the world
// like gather_x_kernel) -> candidate 0 of `snap`, one 32-lane group per cell; the cells with more
// than 32 active proteins go to the wide list (count wide[0], zero on entry: the write-back kernel
// resets it) for the front blocks of the speculative launch. Block 0 clears the launch's flag words
// and the speculative flags + unfit word (wide[4 ..]).
// G = 64 (s in 33..128): 64 lanes per cell, each lane loads signals lane, lane + 64; no wide list
// (the register launches pass cells they cannot take on to the next level themselves).
template <int G>
__global__ void __launch_bounds__(kBlock) gather_bin_kernel(int c, int s, int m, int R, int C, int P,
                                                            const float* X, const float* cell_mols,
                                                            const void* molmap, int map_dtype, const float* corr,
                                                            const int32_t* positions, const float4* Q,
                                                            const int64_t* prow, float trim0, float* snap,
                                                            int32_t* wide_list, unsigned* wide, unsigned* zero,
                                                            int nz, int32_t* zero_wc, float* save, int nparts,
                                                            bool void_spec, IntegrateArgs pa, IntegrateArgs pw,
                                                            IntegrateArgs* args_out) {
  clear_words(zero, nz, zero_wc);
  // (the register launch's argument blocks into device memory: see integrate_spec_fused_kernel)
  if (args_out && blockIdx.x == 0 && threadIdx.x == 0) {
    args_out[0] = pa;
    args_out[1] = pw;
  }
  // (void_spec, mode bit 9, for tests: the unfit word starts set, so the exact launches run)
  if (blockIdx.x == 0 && threadIdx.x < ms::kEqIters * kMaxParts + 1)
    wide[4 + threadIdx.x] = (void_spec && threadIdx.x == ms::kEqIters * nparts) ? 1u : 0u;
  if (blockIdx.x == 0 && threadIdx.x == 0) wide[1] = 0u;  // (the rescue launch's grid-barrier counter)
  const int lane = threadIdx.x & (G - 1);
  const int cell = (int)blockIdx.x * (kBlock / G) + (int)threadIdx.x / G;
  const bool ok = cell < c;
  for (int j = lane; ok && j < s; j += G) {
    float x;
    if (X) {
      x = X[(size_t)cell * s + j];
    } else if (j < m) {
      x = cell_mols[(size_t)cell * m + j];
      if (save) save[(size_t)cell * s + j] = x;
    } else {
      const size_t pix = (size_t)positions[2 * cell] * C + positions[2 * cell + 1];
      const float raw = ld_map(molmap, (size_t)(j - m) * R * C + pix, map_dtype);
      if (save) save[(size_t)cell * s + j] = raw;  // cell_state_io layout: (molecules | raw pixels)
      x = corr_in(raw, corr, j - m);
    }
    snap[(size_t)cell * ms::kSnap * s + j] = x;
  }
  if constexpr (G == 64) return;
  size_t r;
  int pc;
  prot_range(prow, cell, P, ok, r, pc);
  const int pc_w = __builtin_amdgcn_readfirstlane(wave_max(pc));  // (uniform bound: the ballots)
  int na = 0;
  for (int p0 = 0; p0 < pc_w; p0 += 32) {
    const int p = p0 + lane;
    const bool on = p < pc && !(Q[r + p].x * trim0 <= 0.0f);
    na += __popcll(group_ballot<32>(on));
  }
  if (ok && lane == 0 && na > 32) wide_list[atomicAdd(reinterpret_cast<int*>(wide), 1)] = cell;
}

__device__ __forceinline__ int pack_word(int n, int nf, int nb, int av, int* overflow) {
  // (the flag lives in mapped host memory: a plain system-scope store, read by the host directly)
  if (n < -128 || n > 127 || nf < 0 || nf > 255 || nb < 0 || nb > 255 || av < -128 || av > 127)
    __hip_atomic_store(overflow, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return (n & 0xFF) | ((nf & 0xFF) << 8) | ((nb & 0xFF) << 16) | ((av & 0xFF) << 24);
}

// Integrator layout of the parameters: W (rows, P, s) int8x4 words, Q (rows, P) float4. Rebuilt
// from the API tensors after they were written from the host side; the fused parameter build
// writes both layouts directly.
__global__ void __launch_bounds__(kBlock) pack_params_kernel(long long items, int s, const int32_t* N,
                                                             const int32_t* Nf, const int32_t* Nb, const int32_t* A,
                                                             const float* Vmax, const float* Kmf, const float* Kmb,
                                                             const float* Ke, int32_t* W, float4* Q, int* overflow) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= items * s) return;
  W[t] = pack_word(N[t], Nf[t], Nb[t], A[t], overflow);
  if (t % s == 0) {
    const long long o = t / s;
    Q[o] = make_float4(Vmax[o], Kmf[o], Kmb[o], Ke[o]);
  }
}

// ---------------------------------------------------------------------------------------------
// Parameter build: one thread per (row, protein slot). Semantics in kinetics_host.cpp.
struct BuildArgs {
  int n, P, D, Pt, s;
  const int32_t* tokens;  // (n, P, D, 5)
  const int32_t* rows;    // (n,)
  const int32_t* nprot;   // (n,) proteins per row (0: the row is unset, all params 0) or nullptr
  const float *vmax_w, *km_w;
  const int32_t *signs, *hills, *RM, *TM, *EM;
  int nw, nk, nsg, nh, nv;
  const float* energies;
  float abs_temp, gas;
  int32_t *N, *Nf, *Nb, *A;
  float *Kmr, *Kmf, *Kmb, *Vmax, *Ke;
  int32_t* W;  // integrator layout (optional: nullptr skips it)
  float4* Q;
  int* overflow;
  const int* dn;  // optional device row count (<= n; n is then the capacity)
  // ragged storage (params.h): the first record of item ci (-1: nothing to write), its proteins
  // nprot[ci] are records roff[ci] + p; the padding proteins get no records (rows / Pt unused)
  const int64_t* roff;
};

__device__ __forceinline__ int lut(int t, int lim) { return (t >= 0 && t < lim) ? t : 0; }

// One G-lane group per (row, protein slot); lanes over signals j. Each lane folds the protein's
// domains for its signals (stoichiometry, effector Hill sums, Kmr means), the group reduces the
// energy change for Ke, and lane 0 writes the per-protein scalars. The energy sum is accumulated in
// double (integer N times float energies: exact, hence order-independent) so host and device agree
// bit for bit.
template <int G>
__device__ __forceinline__ void build_group(const BuildArgs& b, long long grp, int lane) {
  const int ci = (int)(grp / b.Pt), p = (int)(grp - (long long)ci * b.Pt);
  size_t o2;
  if (b.roff) {
    const long long ro = b.roff[ci];
    if (ro < 0 || p >= (b.nprot ? b.nprot[ci] : b.P)) return;  // no records / a padding protein
    o2 = (size_t)ro + p;
  } else {
    if (b.rows[ci] < 0) return;  // no row assigned
    o2 = (size_t)b.rows[ci] * b.Pt + p;
  }
  const size_t o3 = o2 * b.s;
  const int32_t* pt = b.tokens + ((size_t)ci * b.P + (p < b.P ? p : 0)) * b.D * 5;
  // (b.full: the eight unpacked parameter tensors are held too; compact storage has W / Q / Kmr only)
  if (b.nprot && b.nprot[ci] == 0) {  // empty proteome: unset_cell_params semantics (all zero)
    for (int j = lane; j < b.s; j += G) {
      if (b.N) {
        b.N[o3 + j] = 0;
        b.Nf[o3 + j] = 0;
        b.Nb[o3 + j] = 0;
        b.A[o3 + j] = 0;
      }
      b.Kmr[o3 + j] = 0.0f;
      if (b.W) b.W[o3 + j] = 0;
    }
    if (lane == 0) {
      if (b.Ke) {
        b.Ke[o2] = 0.0f;
        b.Kmf[o2] = 0.0f;
        b.Kmb[o2] = 0.0f;
        b.Vmax[o2] = 0.0f;
      }
      if (b.Q) b.Q[o2] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
    return;
  }
  int nd = p < b.P ? b.D : 0;
  while (nd > 0 && pt[(nd - 1) * 5] == 0) --nd;  // trailing empty domain slots

  double E = 0.0;
  for (int j = lane; j < b.s; j += G) {
    int n = 0, nf = 0, nb = 0, av = 0, kc = 0;
    float ks = 0.0f;
    for (int d = 0; d < nd; ++d) {
      const int32_t* dm = pt + d * 5;
      const int ty = dm[0];
      if (ty == 0) continue;
      const int sgn = b.signs[lut(dm[3], b.nsg)];
      const int vi = lut(dm[4], b.nv);
      if (ty == 3) {
        const int e = b.EM[(size_t)vi * b.s + j];
        if (e == 0) continue;
        av += e * sgn * b.hills[lut(dm[1], b.nh)];
        const float kv = (float)e * b.km_w[lut(dm[2], b.nk)];
        if (!ms::f_isnan(kv) && kv != 0.0f) {
          ks += kv;
          ++kc;
        }
      } else {
        const int v = (ty == 1 ? b.RM : b.TM)[(size_t)vi * b.s + j];
        const int ndv = v * sgn;
        n += ndv;
        if (ndv < 0) nf += -ndv;
        if (ndv > 0) nb += ndv;
      }
    }
    if (b.N) {
      b.N[o3 + j] = n;
      b.Nf[o3 + j] = nf;
      b.Nb[o3 + j] = nb;
      b.A[o3 + j] = av;
    }
    if (b.W) b.W[o3 + j] = pack_word(n, nf, nb, av, b.overflow);
    // (x^a by multiplications, as the host build: device and host powf differ in the last bit)
    b.Kmr[o3 + j] = ms::ipow(kc > 0 ? ks / (float)kc : 0.0f, av);
    E += (double)n * (double)b.energies[j];
  }
  for (int o = G / 2; o > 0; o >>= 1) E += __shfl_xor(E, o, G);
  if (lane != 0) return;
  ms::NanMean vm, km;
  for (int d = 0; d < nd; ++d) {
    const int32_t* dm = pt + d * 5;
    if (dm[0] == 0 || dm[0] == 3) continue;
    vm.add(b.vmax_w[lut(dm[1], b.nw)]);
    km.add(b.km_w[lut(dm[2], b.nk)]);
  }
  // (the float exponent as before, evaluated in double and rounded once: device and host expf differ
  // in the last bit for ~1 in 10^4 proteins, the double results round to the same float)
  float kev = (float)exp((double)(-(float)E / b.abs_temp / b.gas));
  kev = kev < ms::kEps ? ms::kEps : (kev > ms::kMax ? ms::kMax : kev);
  const float kmn = km.value0();
  float kmfv = kev >= 1.0f ? kmn : kmn / kev;
  float kmbv = kev >= 1.0f ? kmn * kev : kmn;
  kmfv = kmfv < ms::kEps ? ms::kEps : (kmfv > ms::kMax ? ms::kMax : kmfv);
  kmbv = kmbv < ms::kEps ? ms::kEps : (kmbv > ms::kMax ? ms::kMax : kmbv);
  const float vmv = vm.value0();
  if (b.Ke) {
    b.Ke[o2] = kev;
    b.Kmf[o2] = kmfv;
    b.Kmb[o2] = kmbv;
    b.Vmax[o2] = vmv;
  }
  if (b.Q) b.Q[o2] = make_float4(vmv, kmfv, kmbv, kev);
}

template <int G>
__global__ void __launch_bounds__(kBlock) build_params_kernel(BuildArgs b) {
  const int lane = threadIdx.x % G;
  const long long n_eff = b.dn ? (long long)min(*b.dn, b.n) : (long long)b.n;
  const long long groups = n_eff * b.Pt, stride = (long long)gridDim.x * (blockDim.x / G);
  for (long long grp = ((long long)blockIdx.x * blockDim.x + threadIdx.x) / G; grp < groups; grp += stride)
    build_group<G>(b, grp, lane);  // whole groups iterate together
}


// ---------------------------------------------------------------------------------------------
// Host launchers

void cell_state_io(int n, int m, uintptr_t pos, int R, int C, uintptr_t map, int dtype, uintptr_t cell_mols,
                   uintptr_t buf, bool restore, uintptr_t stream);  // maps.hip

// LDS-path slots of `cps` cells per block for `blocks` blocks: in LDS when they fit (returns the
// dynamic LDS bytes), else in a device buffer (a cell with a proteome of ~900+ proteins: its slot alone
// exceeds the 160 KiB of LDS; long evolving runs grow such genomes by recombination) -- the same
// kernels, slower, and only for those launches. Sets `a`'s global-slot fields either way.
static std::unordered_map<int, std::pair<int*, size_t>> g_gslots;
static size_t lds_slots(IntegrateArgs& a, size_t slot_bytes, int cps, unsigned blocks) {
  const size_t lds = (size_t)cps * slot_bytes;
  if (lds <= 160 * 1024) {
    a.gslots = nullptr;
    a.gslot_stride = 0;
    return lds;
  }
  int dev = 0;
  MS_HIP_CHECK(hipGetDevice(&dev));
  auto& b = g_gslots[dev];
  const size_t need = (size_t)blocks * lds;
  if (b.second < need) {
    if (b.first) MS_HIP_CHECK(msd::dev_free(b.first));  // (synchronises: a queued launch may use it)
    b.first = nullptr;
    MS_HIP_CHECK(msd::dev_malloc((void**)&b.first, need));
    b.second = need;
  }
  a.gslots = b.first;
  a.gslot_stride = cps;
  return 0;
}

static int slot_words_for(int P, int s, int sp) {
  int w = P * sp + P * 8 + 3 * s + 1 + P + (P * s + 3) / 4;
  return (w + 3) & ~3;  // keep every slot 16-byte aligned
}

// Launch integration parts [part_begin, part_end) of trims.size() parts. X_io: if nonzero,
// integrate explicit signals X (c, s) and write the result back there (Kinetics.integrate_signals);
// otherwise gather from / scatter to the world state (cell_mols, molmap, positions). `masks` holds
// 4 flags per part plus a zero block; the caller may all-reduce (MAX) a part's flags across ranks
// between launches for the reference's global early exit over a domain-decomposed population.
// Would an integration of `s` signals in `nparts` parts take the speculative path (given the cell
// lists and the speculation buffer)? Every rank of a decomposed world sees the same answer, also a
// rank without cells (it still joins the all-reduces of the protocol it implies).
// Per stream: device memory for the register launch's argument blocks (two IntegrateArgs), written
// by the input kernel and read by integrate_spec_fused_kernel on the same stream.
std::vector<unsigned long long> int_prof_read(bool reset) {
#ifdef MS_INT_PROF
  std::vector<unsigned long long> v(64);
  MS_HIP_CHECK(msd::device_synchronize());
  MS_HIP_CHECK(hipMemcpyFromSymbol(v.data(), HIP_SYMBOL(g_int_prof), 64 * sizeof(unsigned long long)));
  if (reset) {
    std::vector<unsigned long long> z(64, 0ull);
    MS_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_int_prof), z.data(), 64 * sizeof(unsigned long long)));
  }
  return v;
#else
  (void)reset;
  return {};
#endif
}

static std::unordered_map<hipStream_t, IntegrateArgs*> g_args_dev;
static IntegrateArgs* args_block(hipStream_t st) {
  IntegrateArgs*& p = g_args_dev[st];
  if (!p) MS_HIP_CHECK(msd::dev_malloc((void**)&p, 2 * sizeof(IntegrateArgs)));
  return p;
}

bool integrate_spec_ok(int s, int nparts) {
  return s <= 128 && (g_integrate_mode & 8) == 0 && nparts >= 1 && nparts <= kMaxParts && (nparts & 1) == 1 &&
         (g_integrate_mode & 0xF8) == 0;
}

int integrate(int c, int P, int s, int m, int R, int C, uintptr_t W, uintptr_t Q, uintptr_t Kmr, uintptr_t cell_mols,
               uintptr_t molmap, uintptr_t positions, uintptr_t X_io, uintptr_t snap_a, uintptr_t snap_b,
               uintptr_t masks, const std::vector<float>& trims, int n_iters, int part_begin, int part_end,
               bool scatter, uintptr_t prow, uintptr_t lists, int map_dtype, uintptr_t map_corr, uintptr_t spec_buf,
               uintptr_t save_buf, int dist_stage, uintptr_t stream) {
  if (c <= 0) return 0;
  const float* corr = map_corr ? P_<float>(map_corr) : nullptr;
  if (n_iters < 0 || n_iters > ms::kEqIters) throw std::invalid_argument("n_iters must be in 0..4");
  const int nparts = (int)trims.size();
  if (part_begin < 0 || part_end > nparts || part_begin > part_end) throw std::invalid_argument("bad part range");
  hipStream_t st = S_(stream);
  unsigned* mk = P_<unsigned>(masks);
  unsigned* zero_flags = mk + ms::kEqIters * nparts;
  float* snaps[2] = {P_<float>(snap_a), P_<float>(snap_b)};
  const bool fast_path = lists != 0 && s <= 128 && (g_integrate_mode & 8) == 0;
  // Speculative all-parts path (s <= 128, the whole part range with the write-back, mode bits 3-7
  // clear): the reference's global exit (kinetics.py:846) cuts a part short only when no cell of the
  // whole population still has an impactful correction, which never happened in 40-step runs of any
  // BASELINE config (scripts/lab/spec_rate.py: all 3 parts at 4 iterations in every step at 10k-50k
  // cells; a 500-cell world ends early in about half the steps). So every cell runs all parts in one
  // launch, each part starting from the previous part's last candidate: the compaction and
  // stoichiometry staging happen once instead of once per part, no intermediate candidates are
  // stored, and the part boundaries' launch tails disappear. The flags the cells raise show whether
  // the assumption held; the LDS-path launches behind it redo the exact per-part integration from
  // the gathered input only if it did not (they return at once otherwise).
  unsigned* spec_w = P_<unsigned>(spec_buf);
  const bool spec_wb = (g_integrate_mode & 256) == 0;  // mode bit 8: final states via snap + write-back
  // (odd part counts: the final state lands in snap_a, and snap_b keeps the input for the fallback)
  //
  // Domain-decomposed callers (the flags all-reduced across ranks) split it into stages:
  //   dist_stage 1: the speculative launches only (input, register launches, LDS list); returns 1 if
  //                 they were issued (0: the caller uses the plain per-part protocol instead). The
  //                 caller then MAX-reduces the 4 * nparts speculative flags + the unfit word
  //                 (spec_buf[4 ..]) across ranks: "held" is then a global verdict.
  //   dist_stage 2: the exact fallback launches of parts [part_begin, part_end) (return at once when
  //                 the global speculation held; the caller all-reduces each part's flags as in the
  //                 per-part protocol), and with `scatter` the write-back of what is left.
  const bool spec_ok = fast_path && spec_w != nullptr && integrate_spec_ok(s, nparts);
  if (dist_stage < 0 || dist_stage > 2) throw std::invalid_argument("integrate: dist_stage must be 0, 1 or 2");
  if (dist_stage == 1 && !spec_ok) return 0;
  if (dist_stage == 2 && !spec_ok) throw std::invalid_argument("integrate: dist_stage 2 without the speculative path");
  const bool spec_path = spec_ok && (dist_stage == 1 || (dist_stage == 0 && part_begin == 0 && part_end == nparts &&
                                                         scatter));
  const bool spec_any = spec_path || dist_stage == 2;
  // save_buf: the state the activity changes (cell molecules, raw pixels under the cells) for a
  // speculative activity's rollback (World._speculate) -- written by the speculative path's input
  // kernel, else by a separate pass first
  if (save_buf && !X_io && part_begin == 0 && !spec_any)
    cell_state_io(c, m, positions, R, C, molmap, map_dtype, cell_mols, save_buf, false, stream);
  if (spec_any) {
    // LDS sizing of the list / fallback launches first: nothing may throw once the input kernel has
    // appended to the wide list (its count is only reset by the write-back at the end)
    const int sp = (s % 2 == 0) ? s + 1 : s;
    const int slot_words = slot_words_for(P, s, sp);
    const size_t slot_bytes = (size_t)slot_words * 4;
    const int Gs = s <= 32 ? 32 : 64;  // lanes per cell (64: s in 33..128, two signals per lane above 64)
    const bool two = s > 64;
    int cps = kBlock / Gs;
    while (cps > 1 && cps * slot_bytes > 64 * 1024) --cps;
    const size_t lds_full = cps * slot_bytes;  // (beyond 160 KiB the slots go to device memory, lds_slots)
    const long long per_cu =
        lds_full > 160 * 1024 ? kWideBlocksPerCU
                              : std::max<long long>(1, std::min<long long>(kWideBlocksPerCU, (160 * 1024) / (long long)lds_full));
    const unsigned grid = (unsigned)std::min<long long>(cdiv(c, cps), 256 * per_cu);
    const int nz = ms::kEqIters * (nparts + 1);
    int32_t* L = P_<int32_t>(lists);
    int32_t* wl = L + c;                    // wide list (more than 32 active proteins)
    int32_t* wl2 = L;                       // overflow list of the narrow blocks (non-zeros, exponents)
    int32_t* wc2 = L + 2 * (size_t)c;       // its count, cleared with the flags below
    int32_t* zwc = L + 2 * (size_t)c + 1;
    int32_t* wl3 = L + 2 * (size_t)c + 2 + 2 * kSortBuckets;  // what no register launch takes (the
    int32_t* wc3 = L + 2 * (size_t)c + 2;                      // sort order / histogram slots, unused here)
    unsigned* sflags = spec_w + 4;          // speculative flags (4 per part) + the unfit word
    if (spec_path) {
    IntegrateArgs a{};
    a.c = c; a.P = P; a.s = s;
    a.W = P_<int32_t>(W); a.Q = P_<float4>(Q); a.Kmr = P_<float>(Kmr);
    a.snap_prev = snaps[1];
    a.mask_prev = zero_flags;
    a.n_iters_prev = n_iters;
    a.snap_out = snaps[(nparts - 1) & 1];  // slot n_iters: where the write-back looks after a full run
    a.mask_out = sflags;
    a.trim = trims[0];
    a.n_iters = n_iters;
    a.sp = sp;
    a.prow = prow ? P_<int64_t>(prow) : nullptr;
    a.spec_parts = nparts;
    for (int p = 0; p < nparts; ++p) a.trims[p] = trims[p];
    a.unfit = sflags + ms::kEqIters * nparts;
    if (spec_wb) {
      a.wb = 1;
      a.wb_x = X_io ? P_<float>(X_io) : nullptr;
      a.wb_cm = P_<float>(cell_mols);
      a.wb_map = P_<void>(molmap);
      a.wb_corr = corr;
      a.wb_pos = P_<int32_t>(positions);
      a.wb_m = m; a.wb_R = R; a.wb_C = C; a.wb_dtype = map_dtype;
    }
    a.Ps = 32;
    a.prelisted = 1;
    a.ovf_list = wl2;
    a.ovf_count = wc2;
    IntegrateArgs aw = a;  // front blocks: the wide list on 64-lane slots
    aw.list = wl;
    aw.count = reinterpret_cast<const int32_t*>(spec_w);
    aw.Ps = 64;
    aw.prelisted = 0;
    aw.ovf_list = wl3;
    aw.ovf_count = wc3;
    IntegrateArgs ao = aw;  // the overflow list (rare) on 64-lane slots with 2 * kNzReg non-zeros
    ao.list = wl2;
    ao.count = wc2;
    // the input kernel also stores the register launch's argument blocks in device memory (32-lane
    // cells: narrow + wide for integrate_spec_fused_kernel; two signals per lane: the narrow block of
    // integrate_spl2_spec_kernel)
    IntegrateArgs an = a;
    an.Ps = 64;
    an.prelisted = 0;
    const bool spl2 = Gs == 64 && s > 64;
    IntegrateArgs* dargs = (Gs == 32 || spl2) ? args_block(st) : nullptr;
    if (Gs == 32)
      msd::kl(gather_bin_kernel<32>, cdiv(c, kBlock / 32), kBlock, 0, st)(
          c, s, m, R, C, P, X_io ? P_<float>(X_io) : nullptr, P_<float>(cell_mols), P_<void>(molmap), map_dtype, corr,
          P_<int32_t>(positions), P_<float4>(Q), prow ? P_<int64_t>(prow) : nullptr, trims[0], snaps[1], wl, spec_w, mk,
          nz, zwc, X_io ? nullptr : P_<float>(save_buf), nparts, (g_integrate_mode & 512) != 0, a, aw, dargs);
    else
      msd::kl(gather_bin_kernel<64>, cdiv(c, kBlock / 64), kBlock, 0, st)(
          c, s, m, R, C, P, X_io ? P_<float>(X_io) : nullptr, P_<float>(cell_mols), P_<void>(molmap), map_dtype, corr,
          P_<int32_t>(positions), P_<float4>(Q), prow ? P_<int64_t>(prow) : nullptr, trims[0], snaps[1], wl, spec_w, mk,
          nz, zwc, X_io ? nullptr : P_<float>(save_buf), nparts, (g_integrate_mode & 512) != 0, an, an, dargs);
    MS_LAUNCH_CHECK();
    if (Gs == 32) {
      const size_t lds_fast = (size_t)(kBlock / 32) * fast_slot_words<32, kNzReg>() * 4;
      const size_t lds_fw = (size_t)(kBlock / 64) * fast_slot_words<64, kNzWide>() * 4;
      // (6 waves per SIMD: measured faster than 5 -- 96 VGPRs, fewer spills -- by 3-5 % on the
      // flagship state, profiles/r5/ab_integrator_*.log)
      msd::kl(integrate_spec_fused_kernel<6>, cdiv(c, kBlock / 32), kBlock, lds_fast, st)(dargs);
      MS_LAUNCH_CHECK();
      if (dist_stage == 0 && g_rescue_mode && scatter) {
        // one launch for the overflow lists, the exact fallback and the write-back (see
        // integrate_rescue_kernel); the barrier counter was zeroed by the input kernel
        if (!g_rescue_blocks) {
          int dev = 0, cus = 0;
          MS_HIP_CHECK(hipGetDevice(&dev));
          MS_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
          g_rescue_blocks = (unsigned)std::max(1, std::min(cus, 256));
          MS_HIP_CHECK(hipHostMalloc((void**)&g_rescue_err, sizeof(unsigned), hipHostMallocMapped | hipHostMallocCoherent));
          *g_rescue_err = 0;
          MS_HIP_CHECK(hipHostGetDevicePointer((void**)&g_rescue_err_dev, g_rescue_err, 0));
        }
        msd::kl(integrate_fast_kernel<64, kNzWide, true, true>, g_ovf_blocks, kBlock, lds_fw, st)(ao, nullptr, nullptr);
        MS_LAUNCH_CHECK();
        RescueArgs r{};
        r.lb = a;
        r.lb.list = wl3;
        r.lb.count = wc3;
        r.lb.Ps = P;
        r.lb.slot_words = slot_words;
        r.lb.wb = 0;  // (phase D writes the list-B cells back)
        r.cps = std::min(cps, kBlock / 32);
        r.nparts = nparts;
        r.n_iters = n_iters;
        {
          IntegrateArgs& f = r.fb;
          f.c = c; f.P = P; f.s = s;
          f.W = P_<int32_t>(W); f.Q = P_<float4>(Q); f.Kmr = P_<float>(Kmr); f.prow = prow ? P_<int64_t>(prow) : nullptr;
          f.n_iters_prev = n_iters;
          f.n_iters = n_iters;
          f.sp = sp;
          f.slot_words = slot_words;
          f.Ps = P;
          for (int part = 0; part < nparts; ++part) {
            f.trims[part] = trims[part];
            r.fb_snap_prev[part] = part == 0 ? snaps[1] : snaps[(part - 1) & 1];
            r.fb_mask_prev[part] = part == 0 ? zero_flags : mk + ms::kEqIters * (part - 1);
            r.fb_snap_out[part] = snaps[part & 1];
            r.fb_mask_out[part] = mk + ms::kEqIters * part;
          }
        }
        r.sflags = sflags;
        r.masks = mk;
        r.barrier = spec_w + 1;
        r.err_host = g_rescue_err_dev;
        r.wide_reset = reinterpret_cast<int*>(spec_w);
        r.c = c; r.s = s; r.m = m; r.R = R; r.C = C; r.map_dtype = map_dtype;
        r.snap_spec = a.snap_out;
        r.snap_last = snaps[(nparts - 1) & 1];
        r.positions = P_<int32_t>(positions);
        r.cell_mols = P_<float>(cell_mols);
        r.molmap = P_<void>(molmap);
        r.corr = corr;
        r.X_out = X_io ? P_<float>(X_io) : nullptr;
        r.all_from_snap = spec_wb ? 0 : 1;
        const size_t lds_r = lds_slots(r.lb, slot_bytes, r.cps, g_rescue_blocks);
        r.fb.gslots = r.lb.gslots;
        r.fb.gslot_stride = r.lb.gslot_stride;
        msd::kl(integrate_rescue_kernel, g_rescue_blocks, kBlock, lds_r, st)(r);
        MS_LAUNCH_CHECK();
        return 1;
      }
      msd::kl(integrate_fast_kernel<64, kNzWide, true, true>, g_ovf_blocks, kBlock, lds_fw, st)(ao, nullptr, nullptr);
      MS_LAUNCH_CHECK();
    } else {
      // 64-lane cells: no wider register level for more than 64 active proteins, so the narrow
      // launch passes every cell it cannot take (too many proteins, non-zeros or large exponents) to
      // the overflow list; the 64-lane kNzWide launch passes what it cannot take on to the LDS list
      const size_t lds_n = (size_t)(kBlock / 64) *
                           (two ? fast_slot_words<64, kNzReg, 2>() : fast_slot_words<64, kNzReg>()) * 4;
      const size_t lds_fw =
          (size_t)(kBlock / 64) * (two ? fast_slot_words<64, kNzWide, 2>() : fast_slot_words<64, kNzWide>()) * 4;
      if (two) {
        const unsigned g2 = cdiv(c, kBlock / 64);
        if (g_spl2_waves == 2) msd::kl(integrate_spl2_spec_kernel<2>, g2, kBlock, lds_n, st)(dargs);
        else if (g_spl2_waves == 3) msd::kl(integrate_spl2_spec_kernel<3>, g2, kBlock, lds_n, st)(dargs);
        else msd::kl(integrate_spl2_spec_kernel<4>, g2, kBlock, lds_n, st)(dargs);
        MS_LAUNCH_CHECK();
        msd::kl(integrate_fast_kernel<64, kNzWide, true, true, 2>, g_ovf_blocks, kBlock, lds_fw, st)(ao, nullptr, nullptr);
      } else {
        msd::kl(integrate_fast_kernel<64, kNzReg, false, true>, cdiv(c, kBlock / 64), kBlock, lds_n, st)(an, nullptr,
                                                                                                 nullptr);
        MS_LAUNCH_CHECK();
        msd::kl(integrate_fast_kernel<64, kNzWide, true, true>, g_ovf_blocks, kBlock, lds_fw, st)(ao, nullptr, nullptr);
      }
      MS_LAUNCH_CHECK();
    }
    // the cells neither register launch took, all parts on the LDS path (rare: usually an empty list)
    {
      IntegrateArgs l = a;
      l.list = wl3;
      l.count = wc3;
      l.Ps = P;
      l.slot_words = slot_words;
      const unsigned gl = std::min<unsigned>(grid, 256);
      const size_t lds = lds_slots(l, slot_bytes, cps, gl);
      if (Gs == 32) msd::kl(integrate_spec_lds_kernel<32>, gl, cps * 32, lds, st)(l);
      else msd::kl(integrate_spec_lds_kernel<64>, gl, cps * 64, lds, st)(l);
      MS_LAUNCH_CHECK();
    }
    }  // spec_path
    if (dist_stage == 1) return 1;
    // exact fallback: the per-part LDS path over every cell, skipped when the speculation held
    const int fb0 = dist_stage == 2 ? part_begin : 0, fb1 = dist_stage == 2 ? part_end : nparts;
    for (int part = fb0; part < fb1; ++part) {
      IntegrateArgs f{};
      f.c = c; f.P = P; f.s = s;
      f.W = P_<int32_t>(W); f.Q = P_<float4>(Q); f.Kmr = P_<float>(Kmr); f.prow = prow ? P_<int64_t>(prow) : nullptr;
      f.snap_prev = part == 0 ? snaps[1] : snaps[(part - 1) & 1];
      f.mask_prev = part == 0 ? zero_flags : mk + ms::kEqIters * (part - 1);
      f.n_iters_prev = n_iters;
      f.snap_out = snaps[part & 1];
      f.mask_out = mk + ms::kEqIters * part;
      f.trim = trims[part];
      f.n_iters = n_iters;
      f.sp = sp;
      f.slot_words = slot_words;
      f.Ps = P;
      f.spec_check = sflags;
      f.spec_n = nparts;
      f.copy_to = part == nparts - 1 ? mk : nullptr;
      const size_t lds = lds_slots(f, slot_bytes, cps, grid);
      if (Gs == 32) msd::kl(integrate_part_kernel<32, true>, grid, cps * 32, lds, st)(f);
      else msd::kl(integrate_part_kernel<64, true>, grid, cps * 64, lds, st)(f);
      MS_LAUNCH_CHECK();
    }
  } else if (part_begin == 0) {
    // part 0 input -> candidate 0 of snap_b, selected through the zero flags; the same launch
    // clears all flag words and (register path) the wide-list counter
    const int nz = ms::kEqIters * (nparts + 1);
    if (nz > kBlock) throw std::invalid_argument("integrate: too many parts");
    int32_t* zwc = fast_path ? P_<int32_t>(lists) + 2 * (size_t)c + 1 : nullptr;
    if (X_io) {
      msd::kl(load_x_kernel, cdiv((long long)c * s, kBlock), kBlock, 0, st)(c, s, P_<float>(X_io), snaps[1], mk, nz, zwc);
    } else {
      msd::kl(gather_x_kernel, cdiv((long long)c * s, kBlock), kBlock, 0, st)(c, s, m, R, C, P_<float>(cell_mols),
                                                                          P_<void>(molmap), map_dtype, corr,
                                                                          P_<int32_t>(positions), snaps[1], mk, nz,
                                                                          zwc);
    }
    MS_LAUNCH_CHECK();
  }
  const int sp = (s % 2 == 0) ? s + 1 : s;
  auto part_args = [&](int part) {
    IntegrateArgs a{};
    a.c = c; a.P = P; a.s = s;
    a.W = P_<int32_t>(W); a.Q = P_<float4>(Q); a.Kmr = P_<float>(Kmr);
    a.snap_prev = part == 0 ? snaps[1] : snaps[(part - 1) & 1];
    a.mask_prev = part == 0 ? zero_flags : mk + ms::kEqIters * (part - 1);
    a.n_iters_prev = n_iters;
    a.snap_out = snaps[part & 1];
    a.mask_out = mk + ms::kEqIters * part;
    a.trim = trims[part];
    a.n_iters = n_iters;
    a.sp = sp;
    a.prow = prow ? P_<int64_t>(prow) : nullptr;
    return a;
  };
  // register-resident path (default for s <= 64, integrate_item_fast): one launch per part over
  // every cell with at most G active proteins and kNzReg non-zeros per protein. Part 0 lists the
  // others (wide list), which a strided 64-lane launch with 2 * kNzReg non-zeros per protein takes
  // next; what does not fit there either (more than 64 active proteins, more non-zeros, exponents
  // >= 32; part 0 lists it again) goes to a strided launch with LDS slots for all P proteins
  // (integrate_item). The 64-lane launch replaced the LDS path for the wide list: that path's
  // per-cell dependency chain made its launch ~40 us per part for a few hundred cells.
  if (spec_any) {
    // launched above
  } else if (fast_path) {
    int32_t* wl = P_<int32_t>(lists) + c;
    int32_t* wc = P_<int32_t>(lists) + 2 * (size_t)c + 1;  // cleared by the input kernel of part 0
    int32_t* wl2 = P_<int32_t>(lists);
    int32_t* wc2 = wc - 1;  // cleared with wc
    const int G = s <= 32 ? 32 : 64;
    const bool two = s > 64;  // two signals per lane (64-lane groups, s <= 128)
    const int cps = kBlock / G;
    const size_t lds_fast = (size_t)cps *
                            (G == 32 ? fast_slot_words<32, kNzReg>()
                                     : (two ? fast_slot_words<64, kNzReg, 2>() : fast_slot_words<64, kNzReg>())) * 4;
    const size_t lds_fw =
        (size_t)(kBlock / 64) * (two ? fast_slot_words<64, kNzWide, 2>() : fast_slot_words<64, kNzWide>()) * 4;
    const unsigned grid_fw = (unsigned)std::min<long long>(cdiv(c, kBlock / 64), 512);
    constexpr int kFusedWideBlocks = 64;
    const int slot_words = slot_words_for(P, s, sp);
    const size_t slot_bytes = (size_t)slot_words * 4;
    int cpsw = kBlock / G;
    while (cpsw > 1 && cpsw * slot_bytes > 64 * 1024) --cpsw;
    const size_t ldsw_full = cpsw * slot_bytes;
    const long long per_cu =
        ldsw_full > 160 * 1024 ? kWideBlocksPerCU
                               : std::max<long long>(1, std::min<long long>(kWideBlocksPerCU, (160 * 1024) / (long long)ldsw_full));
    const unsigned gridw = (unsigned)std::min<long long>(cdiv(c, cpsw), 256 * per_cu);
    // lists layout: [0, c) second-level wide list, [c, 2c) wide list, 2c / 2c + 1 their counts,
    // 2c + 2 .. histogram + cursors (cleared by the input kernel of part 0), then the sort order (c)
    // and per-cell counts (c bytes)
    int32_t* hist = wc + 1;
    int32_t* cursor = hist + kSortBuckets;
    int32_t* order = cursor + kSortBuckets;
    int32_t* total = order + c;  // = c (device count for the list launch)
    uint8_t* na = reinterpret_cast<uint8_t*>(total + 1);
    // off by default: on the flagship state the sorted order was 31 % slower (682 vs 521 us per
    // 3-part integration, scripts/lab/integrator_bench.py) -- neighbouring cells' parameter rows are
    // neighbours in memory, and losing that locality costs more than the wasted lanes
    const bool sorted = (g_integrate_mode & 16) != 0;
    // mode bit 5: skip the 64-lane level (the whole wide list takes the LDS path; for A/B)
    const bool fw = (g_integrate_mode & 32) == 0;
    if (sorted && part_begin == 0) {
      msd::kl(na_hist_kernel, cdiv(c, 256), 256, 0, st)(c, P, P_<float4>(Q), prow ? P_<int64_t>(prow) : nullptr, na, hist,
                                                    total);
      MS_LAUNCH_CHECK();
      msd::kl(na_scatter_kernel, cdiv(c, 256), 256, 0, st)(c, na, hist, cursor, order);
      MS_LAUNCH_CHECK();
    }
    for (int part = part_begin; part < part_end; ++part) {
      IntegrateArgs a = part_args(part);
      a.Ps = G;
      if (sorted) {
        a.list = order;
        a.count = total;
      }
      IntegrateArgs aw = a;
      aw.list = wl;
      aw.count = wc;
      aw.Ps = 64;
      // mode bit 6: parts >= 1 launch the wide list separately too (A/B of the fused launch)
      // (32-lane cells only: the 64-lane narrow path needs more registers than the fused kernel's
      // occupancy target leaves)
      const bool fused = G == 32 && fw && part > 0 && (g_integrate_mode & 64) == 0;
      if (fused) {
        msd::kl(integrate_fused_kernel<32>, cdiv(c, cps) + kFusedWideBlocks, kBlock, lds_fast, st)(a, aw, kFusedWideBlocks);
        MS_LAUNCH_CHECK();
      } else {
        if (G == 32)
          msd::kl(integrate_fast_kernel<32, kNzReg, false>, cdiv(c, cps), kBlock, lds_fast, st)(a, part == 0 ? wl : nullptr, wc);
        else if (two)
          msd::kl(integrate_fast_kernel<64, kNzReg, false, false, 2>, cdiv(c, cps), kBlock, lds_fast, st)(
              a, part == 0 ? wl : nullptr, wc);
        else
          msd::kl(integrate_fast_kernel<64, kNzReg, false>, cdiv(c, cps), kBlock, lds_fast, st)(a, part == 0 ? wl : nullptr, wc);
        MS_LAUNCH_CHECK();
        if (fw) {
          if (two)
            msd::kl(integrate_fast_kernel<64, kNzWide, true, false, 2>, grid_fw, kBlock, lds_fw, st)(
                aw, part == 0 ? wl2 : nullptr, wc2);
          else
            msd::kl(integrate_fast_kernel<64, kNzWide, true>, grid_fw, kBlock, lds_fw, st)(aw, part == 0 ? wl2 : nullptr, wc2);
          MS_LAUNCH_CHECK();
        }
      }
      a.list = fw ? wl2 : wl;
      a.count = fw ? wc2 : wc;
      a.Ps = P;
      a.slot_words = slot_words;
      const size_t ldsw = lds_slots(a, slot_bytes, cpsw, gridw);
      if (G == 32) msd::kl(integrate_part_kernel<32, true>, gridw, cpsw * G, ldsw, st)(a);
      else msd::kl(integrate_part_kernel<64, true>, gridw, cpsw * G, ldsw, st)(a);
      MS_LAUNCH_CHECK();
    }
  } else {
    // legacy LDS-staged launches (s > 64, or mode bit 3 for A/B): narrow / wide binning (only worth
    // it when P is well above the typical active count)
    const int G_wide = s <= 32 ? 32 : 64;
    // narrow launch: 16-lane groups (4 cells per wave) halve the idle lanes of the protein phases
    // (<= kNarrowP proteins); signal phases take s / 16 passes instead
    const int G_narrow = (g_integrate_mode & 4) ? 16 : G_wide;
    const bool binned = lists != 0 && P > kNarrowP;
    int32_t* lst = P_<int32_t>(lists);
    int32_t* cnt = lst ? lst + 2 * (size_t)c : nullptr;
    if (binned && part_begin == 0) {
      MS_HIP_CHECK(msd::memset_async(cnt, 0, 2 * sizeof(int32_t), st));
      msd::kl(bin_cells_kernel, cdiv(c, 256), 256, 0, st)(c, P, kNarrowP, P_<float4>(Q), prow ? P_<int64_t>(prow) : nullptr,
                                                     lst, cnt);
      MS_LAUNCH_CHECK();
    }
    struct Launch {
      int Ps;
      const int32_t* list;
      const int32_t* count;
    };
    Launch launches[2];
    int nl = 0;
    if (binned) {
      launches[nl++] = Launch{kNarrowP, lst, cnt};
      launches[nl++] = Launch{P, lst + c, cnt + 1};
    } else {
      launches[nl++] = Launch{P, nullptr, nullptr};
    }
    // Binned parts run the wide launch on a side stream concurrently with the narrow one: the wide
    // bin is small but its large proteomes are long per-cell dependency chains, which then overlap
    // with the narrow bin's throughput work instead of adding to it (fork / join per part; the next
    // part reads both bins' flags).
    hipStream_t& side = g_lds_side;
    hipEvent_t &ev_fork = g_lds_fork, &ev_join = g_lds_join;
    const bool conc = nl == 2 && (g_integrate_mode & 1) != 0;
    if (conc && !side) {
      MS_HIP_CHECK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
      MS_HIP_CHECK(hipEventCreateWithFlags(&ev_fork, hipEventDisableTiming));
      MS_HIP_CHECK(hipEventCreateWithFlags(&ev_join, hipEventDisableTiming));
    }
    for (int part = part_begin; part < part_end; ++part) {
      if (conc) {
        MS_HIP_CHECK(msd::event_record(ev_fork, st));
        MS_HIP_CHECK(msd::stream_wait_event(side, ev_fork, 0));
      }
      for (int li = nl - 1; li >= 0; --li) {  // wide first: its long chains start early
        const Launch& L = launches[li];
        const int G = (nl == 2 && li == 0) ? G_narrow : G_wide;
        hipStream_t ls = (conc && li == 1) ? side : st;
        const int slot_words = slot_words_for(L.Ps, s, sp);
        const size_t slot_bytes = (size_t)slot_words * 4;
        int cps = kBlock / G;
        while (cps > 1 && cps * slot_bytes > 64 * 1024) --cps;
        const size_t lds_full = cps * slot_bytes;
        const int threads = cps * G;
        const bool stride = nl == 2 && li == 1 && (g_integrate_mode & 2) != 0;
        unsigned grid = cdiv(c, cps);
        if (stride) {  // the wide bin: at most kWideBlocksPerCU resident blocks per CU, striding
          const long long per_cu =
              lds_full > 160 * 1024 ? kWideBlocksPerCU
                                    : std::max<long long>(1, std::min<long long>(kWideBlocksPerCU, (160 * 1024) / (long long)lds_full));
          grid = (unsigned)std::min<long long>(grid, 256 * per_cu);
        }
        IntegrateArgs a = part_args(part);
        a.slot_words = slot_words;
        const size_t lds = lds_slots(a, slot_bytes, cps, grid);
        a.list = L.list;
        a.count = L.count;
        a.Ps = L.Ps;
        if (G == 16) {
          msd::kl(integrate_part_kernel<16, false>, grid, threads, lds, ls)(a);
        } else if (G == 32) {
          if (stride) msd::kl(integrate_part_kernel<32, true>, grid, threads, lds, ls)(a);
          else msd::kl(integrate_part_kernel<32, false>, grid, threads, lds, ls)(a);
        } else {
          if (stride) msd::kl(integrate_part_kernel<64, true>, grid, threads, lds, ls)(a);
          else msd::kl(integrate_part_kernel<64, false>, grid, threads, lds, ls)(a);
        }
        MS_LAUNCH_CHECK();
      }
      if (conc) {
        MS_HIP_CHECK(msd::event_record(ev_join, side));
        MS_HIP_CHECK(msd::stream_wait_event(st, ev_join, 0));
      }
    }
  }
  // the write-back selects the last part's snapshot by its (possibly all-reduced) flags, so a
  // domain-decomposed caller runs it as a separate call once those flags are global
  if (scatter && part_end == nparts && nparts > 0) {
    const int last = nparts - 1;
    msd::kl(integrate_scatter_kernel, (unsigned)std::min<long long>(cdiv((long long)c * s, kBlock), 2048), kBlock, 0, st)(
        c, s, m, R, C, snaps[last & 1], mk + ms::kEqIters * last, n_iters, P_<int32_t>(positions),
        P_<float>(cell_mols), P_<void>(molmap), map_dtype, corr, X_io ? P_<float>(X_io) : nullptr,
        spec_any ? spec_w : nullptr, spec_any && spec_wb ? spec_w + 4 : nullptr, nparts,
        spec_any ? P_<int32_t>(lists) + 2 * (size_t)c + 2 + 2 * kSortBuckets : nullptr,
        spec_any ? P_<int32_t>(lists) + 2 * (size_t)c + 2 : nullptr);
    MS_LAUNCH_CHECK();
  }
  return spec_path ? 1 : 0;
}

void rccl_allreduce(uintptr_t comm, uintptr_t buf, long long count, int dtype, int op, uintptr_t stream);  // comm.hip

// The decomposed world's speculative protocol (integrate(), dist_stage 1 / 2) in one call, its flag
// all-reduces (int32 MAX) issued here on the native RCCL communicator `comm`: the speculative launch,
// one all-reduce of its 4 * nparts flags + unfit word, the exact per-part launches (return at once
// when the speculation held globally) each followed by its part's all-reduce, and the write-back.
// Returns 0 without issuing anything when the speculative path does not apply (the caller runs the
// per-part protocol instead; every rank decides alike, see integrate_spec_ok).
int integrate_dist(int c, int P, int s, int m, int R, int C, uintptr_t W, uintptr_t Q, uintptr_t Kmr,
                   uintptr_t cell_mols, uintptr_t molmap, uintptr_t positions, uintptr_t snap_a, uintptr_t snap_b,
                   uintptr_t masks, const std::vector<float>& trims, int n_iters, uintptr_t prow, uintptr_t lists,
                   int map_dtype, uintptr_t map_corr, uintptr_t spec_buf, uintptr_t save_buf, uintptr_t comm,
                   uintptr_t stream) {
  const int nparts = (int)trims.size();
  if (!integrate(c, P, s, m, R, C, W, Q, Kmr, cell_mols, molmap, positions, 0, snap_a, snap_b, masks, trims, n_iters,
                 0, 0, false, prow, lists, map_dtype, map_corr, spec_buf, save_buf, 1, stream))
    return 0;
  rccl_allreduce(comm, spec_buf + 4 * sizeof(unsigned), ms::kEqIters * nparts + 1, 0, 1, stream);
  for (int part = 0; part < nparts; ++part) {
    integrate(c, P, s, m, R, C, W, Q, Kmr, cell_mols, molmap, positions, 0, snap_a, snap_b, masks, trims, n_iters,
              part, part + 1, false, prow, lists, map_dtype, map_corr, spec_buf, 0, 2, stream);
    rccl_allreduce(comm, masks + (size_t)ms::kEqIters * part * sizeof(unsigned), ms::kEqIters, 0, 1, stream);
  }
  integrate(c, P, s, m, R, C, W, Q, Kmr, cell_mols, molmap, positions, 0, snap_a, snap_b, masks, trims, n_iters,
            nparts, nparts, true, prow, lists, map_dtype, map_corr, spec_buf, 0, 2, stream);
  return 1;
}

void pack_params(long long items, int s, uintptr_t N, uintptr_t Nf, uintptr_t Nb, uintptr_t A, uintptr_t Vmax,
                 uintptr_t Kmf, uintptr_t Kmb, uintptr_t Ke, uintptr_t W, uintptr_t Q, uintptr_t overflow,
                 uintptr_t stream) {
  if (items <= 0 || s <= 0) return;
  msd::kl(pack_params_kernel, cdiv(items * s, kBlock), kBlock, 0, S_(stream))(
      items, s, P_<int32_t>(N), P_<int32_t>(Nf), P_<int32_t>(Nb), P_<int32_t>(A), P_<float>(Vmax), P_<float>(Kmf),
      P_<float>(Kmb), P_<float>(Ke), P_<int32_t>(W), P_<float4>(Q), P_<int>(overflow));
  MS_LAUNCH_CHECK();
}

void build_params(int n, int P, int D, int Pt, int s, uintptr_t tokens, uintptr_t rows, uintptr_t vmax_w, int nw,
                  uintptr_t km_w, int nk, uintptr_t signs, int nsg, uintptr_t hills, int nh, uintptr_t RM,
                  uintptr_t TM, uintptr_t EM, int nv, uintptr_t energies, float abs_temp, float gas, uintptr_t N,
                  uintptr_t Nf, uintptr_t Nb, uintptr_t A, uintptr_t Kmr, uintptr_t Kmf, uintptr_t Kmb,
                  uintptr_t Vmax, uintptr_t Ke, uintptr_t nprot, uintptr_t W, uintptr_t Q, uintptr_t overflow,
                  uintptr_t dn, uintptr_t roff, uintptr_t stream) {
  if (n <= 0 || Pt <= 0) return;
  if ((W == 0) != (Q == 0) || (W != 0 && overflow == 0)) throw std::invalid_argument("build_params: W, Q, overflow");
  if ((N == 0 || Ke == 0) && W == 0) throw std::invalid_argument("build_params: no parameter layout to write");
  if (P > Pt) throw std::invalid_argument("build_params: token proteins exceed parameter capacity");
  BuildArgs b{};
  b.n = n; b.P = P; b.D = D; b.Pt = Pt; b.s = s;
  b.tokens = P_<int32_t>(tokens); b.rows = P_<int32_t>(rows);
  b.nprot = nprot ? P_<int32_t>(nprot) : nullptr;
  b.vmax_w = P_<float>(vmax_w); b.km_w = P_<float>(km_w);
  b.signs = P_<int32_t>(signs); b.hills = P_<int32_t>(hills);
  b.RM = P_<int32_t>(RM); b.TM = P_<int32_t>(TM); b.EM = P_<int32_t>(EM);
  b.nw = nw; b.nk = nk; b.nsg = nsg; b.nh = nh; b.nv = nv;
  b.energies = P_<float>(energies); b.abs_temp = abs_temp; b.gas = gas;
  b.N = P_<int32_t>(N); b.Nf = P_<int32_t>(Nf); b.Nb = P_<int32_t>(Nb); b.A = P_<int32_t>(A);
  b.Kmr = P_<float>(Kmr); b.Kmf = P_<float>(Kmf); b.Kmb = P_<float>(Kmb); b.Vmax = P_<float>(Vmax); b.Ke = P_<float>(Ke);
  b.W = W ? P_<int32_t>(W) : nullptr; b.Q = Q ? P_<float4>(Q) : nullptr; b.overflow = P_<int>(overflow);
  b.dn = dn ? P_<int>(dn) : nullptr;
  b.roff = roff ? P_<int64_t>(roff) : nullptr;
  if (b.roff && (b.N || b.Ke)) throw std::invalid_argument("build_params: ragged records hold the packed layout only");
  const long long groups = (long long)n * Pt;
  // with a device count the grid is capped and strides (the host passes the capacity as n)
  auto grid = [&](int g) { const unsigned full = cdiv(groups * g, kBlock); return dn ? std::min(full, 4096u) : full; };
  // (the group is the narrowest power of two covering the signals: 16 lanes for the 14-molecule
  // chemistry, where 32-lane groups left 18 of every 32 lanes idle; the energy butterfly only loses
  // exact zero terms, so the bits are the same)
  if (s <= 16) msd::kl(build_params_kernel<16>, grid(16), kBlock, 0, S_(stream))(b);
  else if (s <= 32) msd::kl(build_params_kernel<32>, grid(32), kBlock, 0, S_(stream))(b);
  else msd::kl(build_params_kernel<64>, grid(64), kBlock, 0, S_(stream))(b);
  MS_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------------------------
// Ragged parameter records (params.h): assignment, dense views, collection

__global__ void __launch_bounds__(1024) assign_records_kernel(int n, const int* dn, const int32_t* nprot,
                                                              const int64_t* cells, int64_t* slot, long long* rtop,
                                                              long long rcap, int width, int64_t* roff, int* flags) {
  const int ne = dn ? min(*dn, n) : n;
  assign_records_block(ne, nprot, cells, slot, rtop, rcap, width, roff, flags, 1);
}

// The dense (n, P, s) / (n, P) view of the records (Kinetics._materialize): protein p < count is its
// record, count <= p < width the build's padding (Vmax 0, Kmf = Kmb = EPS, Ke 1, Kmr 1, words 0 --
// what build_group computes for a protein without domains), beyond that zeros (a widening).
__global__ void __launch_bounds__(256) records_to_dense_kernel(int n, int P, int s, const int64_t* slot,
                                                               const int32_t* W, const float4* Q, const float* Kmr,
                                                               int32_t* Wd, float4* Qd, float* Kmrd) {
  const long long total = (long long)n * P * s;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const long long ip = t / s;
    const int j = (int)(t - ip * s);
    const int i = (int)(ip / P), p = (int)(ip - (long long)i * P);
    const long long v = slot ? slot[i] : rec_encode((long long)i * P, P, P);
    const int cnt = rec_cnt(v), wid = rec_width(v);
    const long long r = rec_off(v) + p;
    if (p < cnt) {
      Wd[t] = W[r * s + j];
      Kmrd[t] = Kmr[r * s + j];
    } else {
      Wd[t] = 0;
      Kmrd[t] = p < wid ? 1.0f : 0.0f;
    }
    if (j == 0)
      Qd[ip] = p < cnt ? Q[r] : (p < wid ? make_float4(0.0f, ms::kEps, ms::kEps, 1.0f) : make_float4(0.f, 0.f, 0.f, 0.f));
  }
}

// Collection: cell i's records move to new_off[i] (an exclusive scan of the counts) in fresh
// buffers, one 64-lane group per cell; the cell's new slot goes to slot_out (sharers of a record run
// get a copy each).
__global__ void __launch_bounds__(256) records_move_kernel(int n, int s, const int64_t* slot, const int64_t* new_off,
                                                           const int32_t* W, const float4* Q, const float* Kmr,
                                                           int32_t* W2, float4* Q2, float* Kmr2, int64_t* slot_out) {
  const int lane = threadIdx.x & 63;
  const int g0 = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, ng = (gridDim.x * blockDim.x) >> 6;
  for (int i = g0; i < n; i += ng) {
    const long long v = slot[i];
    const int cnt = rec_cnt(v);
    const long long src = rec_off(v), dst = new_off[i];
    const long long words = (long long)cnt * s;
    for (long long t = lane; t < words; t += 64) {
      W2[dst * s + t] = W[src * s + t];
      Kmr2[dst * s + t] = Kmr[src * s + t];
    }
    for (int p = lane; p < cnt; p += 64) Q2[dst + p] = Q[src + p];
    if (lane == 0) slot_out[i] = cnt ? rec_encode(dst, cnt, rec_width(v)) : 0;
  }
}

void assign_records(int n, uintptr_t dn, uintptr_t nprot, uintptr_t cells, uintptr_t slot, uintptr_t rtop,
                    long long rcap, int width, uintptr_t roff, uintptr_t flags, uintptr_t stream) {
  if (n <= 0) return;
  if (width < 0 || width > kRecMaxProteins) throw std::invalid_argument("assign_records: protein width too large");
  if (rcap > (long long)kRecOffMask) throw std::invalid_argument("assign_records: record capacity too large");
  msd::kl(assign_records_kernel, 1, 1024, 0, S_(stream))(n, dn ? P_<int>(dn) : nullptr, P_<int32_t>(nprot),
                                                    cells ? P_<int64_t>(cells) : nullptr, P_<int64_t>(slot),
                                                    P_<long long>(rtop), rcap, width, P_<int64_t>(roff), P_<int>(flags));
  MS_LAUNCH_CHECK();
}

void records_to_dense(int n, int P, int s, uintptr_t slot, uintptr_t W, uintptr_t Q, uintptr_t Kmr, uintptr_t Wd,
                      uintptr_t Qd, uintptr_t Kmrd, uintptr_t stream) {
  if (n <= 0 || P <= 0) return;
  const unsigned g = (unsigned)std::min<long long>(cdiv((long long)n * P * s, 256), 8192);
  msd::kl(records_to_dense_kernel, g, 256, 0, S_(stream))(n, P, s, slot ? P_<int64_t>(slot) : nullptr, P_<int32_t>(W),
                                                     P_<float4>(Q), P_<float>(Kmr), P_<int32_t>(Wd), P_<float4>(Qd),
                                                     P_<float>(Kmrd));
  MS_LAUNCH_CHECK();
}

void records_move(int n, int s, uintptr_t slot, uintptr_t new_off, uintptr_t W, uintptr_t Q, uintptr_t Kmr,
                  uintptr_t W2, uintptr_t Q2, uintptr_t Kmr2, uintptr_t slot_out, uintptr_t stream) {
  if (n <= 0) return;
  const unsigned g = (unsigned)std::min<long long>(cdiv((long long)n * 64, 256), 8192);
  msd::kl(records_move_kernel, g, 256, 0, S_(stream))(n, s, P_<int64_t>(slot), P_<int64_t>(new_off), P_<int32_t>(W),
                                                 P_<float4>(Q), P_<float>(Kmr), P_<int32_t>(W2), P_<float4>(Q2),
                                                 P_<float>(Kmr2), P_<int64_t>(slot_out));
  MS_LAUNCH_CHECK();
}

}  // namespace msd
