// gfx950 kernels for the cell geometry (map physics: maps.hip):
//   * placement: random free-pixel claims (spawn / add / reposition) and device-resolved
//     neighbour claims for division / movement (list priority via atomicMin per pixel);
//   * neighbour pairs via a pixel -> cell index map (O(n) instead of the reference's O(n^2));
//   * division bookkeeping.
//
// Geometry: a map is R x C pixels per molecule plane. Cells live in rows [r_lo, r_hi). A
// single-GPU world is R = C = map_size, r_lo = 0, r_hi = R with the x axis wrapping. A strip of a
// domain-decomposed world (magicsoup_amd.parallel) has one halo row above and below its owned rows
// (R = H + 2, r_lo = 1, r_hi = H + 1, no x wrap: the halo rows hold the neighbours' boundary rows).
// The y axis always wraps (columns are never split).
#include <unordered_map>

#include "hip_common.h"
#include "select_lb.h"

namespace msd {

struct Geom {
  int R, C, r_lo, r_hi, wrap;
  __device__ __forceinline__ int xup(int x) const { return (wrap && x == 0) ? R - 1 : x - 1; }
  __device__ __forceinline__ int xdn(int x) const { return (wrap && x == R - 1) ? 0 : x + 1; }
  __device__ __forceinline__ int yl(int y) const { return y == 0 ? C - 1 : y - 1; }
  __device__ __forceinline__ int yr(int y) const { return y == C - 1 ? 0 : y + 1; }
};

// Division bookkeeping after the rows were cloned (reference world.py:446-473): parent and child
// share the parent's molecules half-half, both get divisions + 1 and lifetime 0. One thread per
// (pair, molecule); molecule 0 threads also do the scalar fields.
__global__ void __launch_bounds__(256) split_cells_kernel(int k, int m, const int64_t* parents, const int64_t* children,
                                                          float* cell_mols, int32_t* divisions, int32_t* lifetimes) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)k * m) return;
  const int i = (int)(t / m), j = (int)(t - (long long)i * m);
  const long long p = parents[i], c = children[i];
  const float h = cell_mols[p * m + j] * 0.5f;
  cell_mols[p * m + j] = h;
  cell_mols[c * m + j] = h;
  if (j == 0) {
    const int32_t d = divisions[p] + 1;
    divisions[p] = d;
    divisions[c] = d;
    lifetimes[p] = 0;
    lifetimes[c] = 0;
  }
}

// Division commit with a device-side winner count (the host learns it after the launches): winner
// j (wins[j], j < *dn, ascending cell index) becomes parent of the new row n0 + j, which takes the
// claimed pixel; both get half the parent's molecules, divisions + 1 and lifetime 0 (the columns a
// row gather would copy are all overwritten here, so only genomes / labels / parameter-row map are
// gathered). Grid-stride over (*dn) x m.
__global__ void __launch_bounds__(256) divide_commit_kernel(const int* dn, const int64_t* wins, const long long* result,
                                                            int C, long long n0, const int* n0_dev, int m, int64_t* par,
                                                            int32_t* pos, float* cell_mols, int32_t* divisions,
                                                            int32_t* lifetimes) {
  const long long total = (long long)(*dn) * m;
  if (n0_dev) n0 += *n0_dev;  // (children after a device-side row count: a kill issued just before)
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const long long i = t / m;
    const int j = (int)(t - i * m);
    const long long p = wins[i], c = n0 + i;
    const float h = cell_mols[p * m + j] * 0.5f;
    cell_mols[p * m + j] = h;
    cell_mols[c * m + j] = h;
    if (j == 0) {
      par[i] = p;
      const long long px = result[p];
      pos[2 * c] = (int32_t)(px / C);
      pos[2 * c + 1] = (int32_t)(px - (px / C) * C);
      const int32_t d = divisions[p] + 1;
      divisions[p] = d;
      divisions[c] = d;
      lifetimes[p] = 0;
      lifetimes[c] = 0;
    }
  }
}

// The winner selection of divide_mask_dev_at and divide_commit_kernel in one launch (select_lb.h):
// the k-th parent p (result[p] >= 0, ascending) becomes parent of row n0 (+ *n0_dev) + k. Each
// tile (256 cells: one per thread, so the grid has as many workgroups as divide_commit_kernel
// needs for its latency-bound row updates) commits its own winners afterwards, the workgroup's
// threads over (winners x m).
__global__ void __launch_bounds__(kSelThreads) select_commit_kernel(int n, const long long* result,
                                                                    unsigned long long* status, uint32_t gen,
                                                                    unsigned* err, int64_t* wins, int32_t* dcount, long long* host64,
                                                                    int C, long long n0, const int* n0_dev, int m,
                                                                    int64_t* par, int32_t* pos, float* cell_mols,
                                                                    int32_t* divisions, int32_t* lifetimes) {
  int cnt = 0;
  const long long toff = select_lb_tile<1>(
      n, [&](long long i) { return result[i] >= 0; }, status, gen, err,
      [&](long long k, long long p) {
        wins[k] = p;
        par[k] = p;
      },
      [](long long, long long) {}, dcount, host64, &cnt);
  __syncthreads();  // the tile's wins[] entries (this workgroup's stores) are visible to all its waves
  const long long c0 = n0 + (n0_dev ? (long long)*n0_dev : 0ll) + toff;
  for (int t = threadIdx.x; t < cnt * m; t += blockDim.x) {
    const int q = t / m, j = t - q * m;
    const long long p = wins[toff + q], c = c0 + q;
    const float h = cell_mols[p * m + j] * 0.5f;
    cell_mols[p * m + j] = h;
    cell_mols[c * m + j] = h;
    if (j == 0) {
      const long long px = result[p];
      pos[2 * c] = (int32_t)(px / C);
      pos[2 * c + 1] = (int32_t)(px - (px / C) * C);
      const int32_t d = divisions[p] + 1;
      divisions[p] = d;
      divisions[c] = d;
      lifetimes[p] = 0;
      lifetimes[c] = 0;
    }
  }
}

// Division commit with a host count (decomposed worlds, after their one synchronisation): child
// n0 + j of parent par[j] takes pixel npos[j]; both halve the parent's molecules, divisions + 1,
// lifetime 0. Exporting parents (children created on a neighbour rank) halve their molecules and
// count the division too. Thread over (k + n_exp) x m.
__global__ void __launch_bounds__(256) divide_commit_list_kernel(int k, const int64_t* par, const int32_t* npos,
                                                                 long long n0, int n_exp, const int64_t* exp, int m,
                                                                 int32_t* pos, float* cell_mols, int32_t* divisions,
                                                                 int32_t* lifetimes) {
  const long long total = (long long)(k + n_exp) * m;
  for (long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (long long)gridDim.x * blockDim.x) {
    const long long i = t / m;
    const int j = (int)(t - i * m);
    const bool local = i < k;
    const long long p = local ? par[i] : exp[i - k];
    const long long c = local ? n0 + i : p;
    const float h = cell_mols[p * m + j] * 0.5f;
    cell_mols[p * m + j] = h;
    cell_mols[c * m + j] = h;
    if (j == 0) {
      if (local) {
        pos[2 * c] = npos[2 * i];
        pos[2 * c + 1] = npos[2 * i + 1];
      }
      const int32_t d = divisions[p] + 1;
      divisions[p] = d;
      divisions[c] = d;
      lifetimes[p] = 0;
      lifetimes[c] = 0;
    }
  }
}

void divide_commit_list(int k, uintptr_t par, uintptr_t npos, long long n0, int n_exp, uintptr_t exp, int m,
                        uintptr_t pos, uintptr_t cell_mols, uintptr_t divisions, uintptr_t lifetimes, uintptr_t stream) {
  if (k + n_exp <= 0 || m <= 0) return;
  const unsigned grid = std::min<unsigned>(cdiv((long long)(k + n_exp) * m, 256), 512u);
  msd::kl(divide_commit_list_kernel, grid, 256, 0, S_(stream))(k, P_<int64_t>(par), P_<int32_t>(npos), n0, n_exp,
                                                          P_<int64_t>(exp), m, P_<int32_t>(pos), P_<float>(cell_mols),
                                                          P_<int32_t>(divisions), P_<int32_t>(lifetimes));
  MS_LAUNCH_CHECK();
}

// ---------------------------------------------------------------- placement
// Claim k uniformly random free pixels of the owned rows by rejection: atomically set the pixel's
// byte in the (4-byte padded) bool occupancy map; out[i] = pixel or -1 after `attempts` misses.
__global__ void __launch_bounds__(256) claim_free_kernel(int k, Geom g, uint8_t* cell_map, uint64_t seed, uint64_t call,
                                                         int attempts, long long* out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= k) return;
  Philox rng(seed, call, (uint32_t)i);
  const long long base = (long long)g.r_lo * g.C, n_pix = (long long)(g.r_hi - g.r_lo) * g.C;
  long long got = -1;
  for (int t = 0; t < attempts; ++t) {
    const long long pix = base + (long long)rng.below64((uint64_t)n_pix);
    if (cell_map[pix]) continue;
    unsigned* word = reinterpret_cast<unsigned*>(cell_map + (pix & ~3ll));
    const unsigned bit = 1u << (8 * (pix & 3));
    const unsigned old = atomicOr(word, bit);
    if (!(old & (0xFFu << (8 * (pix & 3))))) {
      got = pix;
      break;
    }
  }
  out[i] = got;
}

// Moore neighbours in the reference order (w,n),(w,y),(w,s),(x,n),(x,s),(e,n),(e,y),(e,s) as
// pixel indices; duplicates (tiny maps) removed. Returns the count.
__device__ __forceinline__ int moore(int x, int y, const Geom& g, long long* nb) {
  const int w = g.xup(x), e = g.xdn(x), n = g.yl(y), s = g.yr(y);
  const int xs[8] = {w, w, w, x, x, e, e, e}, ys[8] = {n, y, s, n, s, n, y, s};
  int cnt = 0;
  for (int k = 0; k < 8; ++k) {
    const long long p = (long long)xs[k] * g.C + ys[k];
    bool dup = false;
    for (int q = 0; q < cnt; ++q) dup |= nb[q] == p;
    if (!dup) nb[cnt++] = p;
  }
  return cnt;
}

// Device-resolved placement rounds (divide / move): in a round every pending cell bids for a
// random free Moore neighbour with atomicMin(claim[pixel], list position); the lowest list position
// wins each pixel (the reference places cells in list order, rust/world.rs:59-146), losers retry
// next round against the updated occupancy. `claim` is an int32 per pixel kept at INT_MAX between
// rounds: the winner resets its pixel (a loser reading the reset value still sees "not mine").
// Cells without any free neighbour drop out. No host synchronisation between rounds.
constexpr int kNoClaim = 0x7FFFFFFF;

__global__ void __launch_bounds__(256) place_bid_kernel(int k, const int64_t* cells, const int32_t* pos, Geom g,
                                                        const uint8_t* cell_map, uint8_t* pending, uint64_t seed,
                                                        uint64_t call, long long* cand, int* claim) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= k || !pending[i]) return;
  const int c = cells ? (int)cells[i] : i;
  long long nb[8], fr[8];
  const int cnt = moore(pos[2 * c], pos[2 * c + 1], g, nb);
  int nf = 0;
  for (int q = 0; q < cnt; ++q)
    if (!cell_map[nb[q]]) fr[nf++] = nb[q];
  if (nf == 0) {
    pending[i] = 0;
    cand[i] = -1;
    return;
  }
  Philox rng(seed, call, (uint32_t)i);
  const long long px = fr[rng.below((uint32_t)nf)];
  cand[i] = px;
  atomicMin(claim + px, i);
}

__global__ void __launch_bounds__(256) place_resolve_kernel(int k, const int64_t* cells, const int32_t* pos, Geom g,
                                                            bool vacate, uint8_t* cell_map, uint8_t* pending,
                                                            const long long* cand, int* claim, long long* result) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= k || !pending[i]) return;
  const long long px = cand[i];
  if (px < 0 || claim[px] != i) return;
  claim[px] = kNoClaim;
  cell_map[px] = 1;
  result[i] = px;
  pending[i] = 0;
  // a move into a halo row is committed only after the owning rank accepts it: keep the pixel
  const int x = (int)(px / g.C);
  if (vacate && (g.wrap || (x >= g.r_lo && x < g.r_hi))) {
    const int c = cells ? (int)cells[i] : i;
    cell_map[(size_t)pos[2 * c] * g.C + pos[2 * c + 1]] = 0;
  }
}

// rounds path over a participation mask (cells 0..k-1): pending from the mask, no result yet
__global__ void __launch_bounds__(256) place_init_mask_kernel(int k, const uint8_t* mask, uint8_t* pending,
                                                              long long* result) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= k) return;
  pending[i] = mask[i] != 0;
  result[i] = -1;
}

// Winners of the placement rounds (wins = ascending list positions with result >= 0): the cell and
// its new pixel as (x, y).
__global__ void __launch_bounds__(256) place_collect_kernel(int k, const int64_t* wins, const int64_t* cells,
                                                            const long long* result, int C, int64_t* par,
                                                            int32_t* npos) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= k) return;
  const long long w = wins[i];
  const long long px = result[w];
  par[i] = cells ? cells[w] : w;
  npos[2 * i] = (int32_t)(px / C);
  npos[2 * i + 1] = (int32_t)(px - (px / C) * C);
}

// Small placement batches: all rounds in one workgroup (rounds separated by __syncthreads instead
// of kernel boundaries), same bids / priorities / RNG streams as the multi-launch path.
__global__ void __launch_bounds__(1024) place_rounds_wg_kernel(int k, const int64_t* cells, const int32_t* pos, Geom g,
                                                               bool vacate, uint8_t* cell_map, uint8_t* pending,
                                                               uint64_t seed, uint64_t call, long long* cand,
                                                               int* claim, long long* result, int rounds) {
  for (int r = 0; r < rounds; ++r) {
    const uint64_t rc = call + ((uint64_t)r << 48);
    for (int i = threadIdx.x; i < k; i += blockDim.x) {
      if (!pending[i]) continue;
      const int c = (int)cells[i];
      long long nb[8], fr[8];
      const int cnt = moore(pos[2 * c], pos[2 * c + 1], g, nb);
      int nf = 0;
      for (int q = 0; q < cnt; ++q)
        if (!cell_map[nb[q]]) fr[nf++] = nb[q];
      if (nf == 0) {
        pending[i] = 0;
        cand[i] = -1;
        continue;
      }
      Philox rng(seed, rc, (uint32_t)i);
      const long long px = fr[rng.below((uint32_t)nf)];
      cand[i] = px;
      atomicMin(claim + px, i);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < k; i += blockDim.x) {
      if (!pending[i]) continue;
      const long long px = cand[i];
      if (px < 0 || claim[px] != i) continue;
      result[i] = px;
      pending[i] = 0;
      cell_map[px] = 1;
      const int x = (int)(px / g.C);
      if (vacate && (g.wrap || (x >= g.r_lo && x < g.r_hi))) {
        const int c = (int)cells[i];
        cell_map[(size_t)pos[2 * c] * g.C + pos[2 * c + 1]] = 0;
      }
    }
    __syncthreads();
    // winners reset their pixel's claim only after every loser has compared against it
    for (int i = threadIdx.x; i < k; i += blockDim.x) {
      const long long px = cand[i];
      if (px >= 0 && result[i] == px) claim[px] = kNoClaim;
    }
    __syncthreads();
  }
  // losers of the last round may still hold claims
  for (int i = threadIdx.x; i < k; i += blockDim.x) {
    const long long px = cand[i];
    if (px >= 0) atomicCAS(claim + px, i, kNoClaim);
  }
}


// All placement rounds in ONE cooperative launch (co-resident workgroups, grid barriers between the
// phases of a round) with an early exit once no cell is left pending: same bids / priorities / RNG
// streams as place_bid / place_resolve. A winner's pixel becomes occupied, so no later bid targets
// it and its claim can stay set until the final reset (no reset phase between rounds): two grid
// barriers per round. The list is `cells` (list position = priority) or, with cells == nullptr,
// cell i itself for i < k with `mask[i]` selecting the cells that take part (divide_cells(mask):
// no index compaction and no host round trip before placement).
// ctl: unsigned[kCtlWords], zeroed before the launch (barrier counter, pending per round,
// barrier-timeout error word). A barrier timeout is also reported in `err_host` (pinned, mapped),
// which the host checks after the placement's one synchronisation (place_error_take).
constexpr int kMaxRounds = 16;
// control words per launch: barrier counter, pending per round, timeout error word, then the tail
// kernel's done-workgroup counter and list length
constexpr int kCtlDone = kMaxRounds + 2, kCtlList = kMaxRounds + 3, kCtlWords = kMaxRounds + 4;

// Grid-wide barrier of a cooperative launch. Data shared between workgroups of different XCDs
// (their L2s are not coherent for ordinary device memory) is only touched with device-scope atomics
// in the cooperative kernel, so the barrier needs no cache write-back / invalidation: each wave
// waits for its own memory operations, then one thread per workgroup arrives and spins.
__device__ __forceinline__ void grid_barrier(unsigned* ctr, unsigned nblocks, unsigned& phase, unsigned* err_host) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned target = (++phase) * nblocks;
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // bounded spin: a barrier that never completes (it cannot with a cooperative launch) ends the
    // wait after ~1 s instead of hanging the device; the error word tells the host
    for (long long spin = 0; __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target; ++spin) {
      if (spin > (1ll << 24)) {
        __hip_atomic_store(ctr + kMaxRounds + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (err_host) __hip_atomic_store(err_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  __syncthreads();
}

// occupancy byte px of the (4-byte padded) map, read / set / cleared coherently across XCDs
__device__ __forceinline__ unsigned map_get(const uint8_t* cell_map, long long px) {
  const unsigned w = __hip_atomic_load(reinterpret_cast<const unsigned*>(cell_map + (px & ~3ll)), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
  return (w >> (8 * (px & 3))) & 0xFFu;
}
__device__ __forceinline__ void map_set(uint8_t* cell_map, long long px) {
  atomicOr(reinterpret_cast<unsigned*>(cell_map + (px & ~3ll)), 1u << (8 * (px & 3)));
}
__device__ __forceinline__ void map_clear(uint8_t* cell_map, long long px) {
  atomicAnd(reinterpret_cast<unsigned*>(cell_map + (px & ~3ll)), ~(0xFFu << (8 * (px & 3))));
}

__global__ void __launch_bounds__(256) place_rounds_coop_kernel(int k, const int64_t* cells, const uint8_t* mask,
                                                                const int32_t* pos, Geom g, bool vacate,
                                                                uint8_t* cell_map, uint8_t* pending, uint64_t seed,
                                                                uint64_t call, long long* cand, int* claim,
                                                                long long* result, int rounds, unsigned* ctl,
                                                                unsigned* ctl_next, unsigned* err_host) {
  const unsigned nb = gridDim.x;
  // the other control buffer, used by the next launch on this stream (which starts after this one
  // ended), cleared here: no memset launch before every placement
  if (blockIdx.x == 0)
    for (int j = threadIdx.x; j < kCtlWords; j += blockDim.x) ctl_next[j] = 0u;
  const int stride = gridDim.x * blockDim.x, t0 = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned phase = 0;
  __shared__ int s_left;
  for (int r = 0; r < rounds; ++r) {
    const uint64_t rc = call + ((uint64_t)r << 48);
    for (int i = t0; i < k; i += stride) {
      if (r == 0) {  // own items only: no barrier needed before the first bids
        pending[i] = mask ? (mask[i] != 0) : 1;
        result[i] = -1;
        cand[i] = -1;
      }
      if (!pending[i]) continue;
      const int c = cells ? (int)cells[i] : i;
      long long nbh[8], fr[8];
      const int cnt = moore(pos[2 * c], pos[2 * c + 1], g, nbh);
      int nf = 0;
      for (int q = 0; q < cnt; ++q)
        if (!map_get(cell_map, nbh[q])) fr[nf++] = nbh[q];
      if (nf == 0) {
        pending[i] = 0;
        cand[i] = -1;
        continue;
      }
      Philox rng(seed, rc, (uint32_t)i);
      const long long px = fr[rng.below((uint32_t)nf)];
      cand[i] = px;
      atomicMin(claim + px, i);
    }
    grid_barrier(ctl, nb, phase, err_host);
    if (threadIdx.x == 0) s_left = 0;
    __syncthreads();
    int left = 0;
    for (int i = t0; i < k; i += stride) {
      if (!pending[i]) continue;
      const long long px = cand[i];
      if (px >= 0 && __hip_atomic_load(claim + px, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == i) {
        result[i] = px;
        pending[i] = 0;
        map_set(cell_map, px);
        const int x = (int)(px / g.C);
        if (vacate && (g.wrap || (x >= g.r_lo && x < g.r_hi))) {
          const int c = cells ? (int)cells[i] : i;
          map_clear(cell_map, (long long)pos[2 * c] * g.C + pos[2 * c + 1]);
        }
      } else {
        ++left;
      }
    }
    if (left) atomicAdd(&s_left, left);
    __syncthreads();
    if (threadIdx.x == 0 && s_left) atomicAdd(ctl + 1 + r, (unsigned)s_left);
    grid_barrier(ctl, nb, phase, err_host);
    if (__hip_atomic_load(ctl + 1 + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) break;
  }
  // winners release their pixels' claims (losers never hold one: a pixel's claim is its winner)
  for (int i = t0; i < k; i += stride) {
    const long long px = result[i];
    if (px >= 0) claim[px] = kNoClaim;
  }
}

// place_rounds_coop_kernel with the later rounds over round 0's losers only. Round 0 runs over all
// cells -- its bids read the map with plain loads (nothing in this launch has written it yet) --
// then a grid barrier, the round's resolution with the losers appended to a list (device-scope
// atomics), a second barrier, and the remaining rounds over that list: by workgroup 0 alone, rounds
// separated by __syncthreads, when the list is short (a sparse map: round 0 places almost every
// cell), else by the whole grid with two barriers per round. Same bids, priorities (claims:
// atomicMin of the cell's list position) and RNG streams as the other paths, so the same placement;
// the all-grid form paid two grid barriers per round over all cells, at least four in all.
// Cross-XCD rule (as above): data one workgroup writes and another reads goes through device-scope
// atomics (map, claims, list entries); a loser's result, pending state and later bids are written by
// the tail workgroup only (ls: per list entry -2 done, -1 pending, >= 0 the current bid pixel).
constexpr long long kLsDone = -2, kLsPending = -1;
constexpr int kTailAlone = 512;  // list entries one workgroup takes on (2 per thread)
__global__ void __launch_bounds__(256) place_tail_coop_kernel(int k, const int64_t* cells, const uint8_t* mask,
                                                              const int32_t* pos, Geom g, bool vacate,
                                                              uint8_t* cell_map, uint64_t seed, uint64_t call,
                                                              long long* cand, int* claim, long long* result,
                                                              int rounds, unsigned* ctl, unsigned* ctl_next,
                                                              unsigned* err_host, int* list, long long* ls) {
  const unsigned nb = gridDim.x;
  if (blockIdx.x == 0)
    for (int j = threadIdx.x; j < kCtlWords; j += blockDim.x) ctl_next[j] = 0u;
  const int stride = gridDim.x * blockDim.x, t0 = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned phase = 0;
  // round 0: bids (cand[i] >= 0 marks a bidder; the owner thread reads it back after the barrier)
  for (int i = t0; i < k; i += stride) {
    long long px = -1;
    if (mask ? (mask[i] != 0) : true) {
      const int c = cells ? (int)cells[i] : i;
      long long nbh[8], fr[8];
      const int cnt = moore(pos[2 * c], pos[2 * c + 1], g, nbh);
      int nf = 0;
      for (int q = 0; q < cnt; ++q)
        if (!cell_map[nbh[q]]) fr[nf++] = nbh[q];
      if (nf > 0) {
        Philox rng(seed, call, (uint32_t)i);
        px = fr[rng.below((uint32_t)nf)];
        atomicMin(claim + px, i);
      }
    }
    cand[i] = px;
  }
  grid_barrier(ctl, nb, phase, err_host);
  for (int i = t0; i < k; i += stride) {
    const long long px = cand[i];
    if (px < 0) {
      result[i] = -1;
      continue;
    }
    if (__hip_atomic_load(claim + px, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == i) {
      result[i] = px;
      map_set(cell_map, px);
      const int x = (int)(px / g.C);
      if (vacate && (g.wrap || (x >= g.r_lo && x < g.r_hi))) {
        const int c = cells ? (int)cells[i] : i;
        map_clear(cell_map, (long long)pos[2 * c] * g.C + pos[2 * c + 1]);
      }
    } else {
      const unsigned j = __hip_atomic_fetch_add(ctl + kCtlList, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(list + j, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  // the list is complete and round 0's claims / map bits are in once every workgroup is past this
  grid_barrier(ctl, nb, phase, err_host);
  // round-0 winners release their claims (a claimed pixel is occupied now: no later bid targets it)
  for (int i = t0; i < k; i += stride) {
    const long long px = cand[i];
    if (px >= 0 && result[i] == px) claim[px] = kNoClaim;
  }
  const int L = (int)__hip_atomic_load(ctl + kCtlList, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (L == 0) return;
  // a short list: workgroup 0 alone, rounds separated by __syncthreads; a long one (crowded maps,
  // where most bids collide): the whole grid over the list, two grid barriers per round as before
  const bool alone = L <= kTailAlone;
  if (alone && blockIdx.x != 0) return;
  const int j0 = alone ? (int)threadIdx.x : t0, js = alone ? (int)blockDim.x : stride;
  __shared__ int s_left;
  for (int j = j0; j < L; j += js) ls[j] = kLsPending;  // (entry j: always this thread's)
  for (int r = 1; r < rounds; ++r) {
    const uint64_t rc = call + ((uint64_t)r << 48);
    for (int j = j0; j < L; j += js) {
      if (ls[j] == kLsDone) continue;
      const int i = __hip_atomic_load(list + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int c = cells ? (int)cells[i] : i;
      long long nbh[8], fr[8];
      const int cnt = moore(pos[2 * c], pos[2 * c + 1], g, nbh);
      int nf = 0;
      for (int q = 0; q < cnt; ++q)
        if (!map_get(cell_map, nbh[q])) fr[nf++] = nbh[q];
      if (nf == 0) {
        ls[j] = kLsDone;
        result[i] = -1;
        continue;
      }
      Philox rng(seed, rc, (uint32_t)i);
      const long long px = fr[rng.below((uint32_t)nf)];
      ls[j] = px;
      atomicMin(claim + px, i);
    }
    if (threadIdx.x == 0) s_left = 0;
    if (alone)
      __syncthreads();
    else
      grid_barrier(ctl, nb, phase, err_host);
    int left = 0;
    for (int j = j0; j < L; j += js) {
      const long long px = ls[j];
      if (px < 0) continue;
      const int i = __hip_atomic_load(list + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__hip_atomic_load(claim + px, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == i) {
        result[i] = px;
        ls[j] = kLsDone;
        map_set(cell_map, px);
        const int x = (int)(px / g.C);
        if (vacate && (g.wrap || (x >= g.r_lo && x < g.r_hi))) {
          const int c = cells ? (int)cells[i] : i;
          map_clear(cell_map, (long long)pos[2 * c] * g.C + pos[2 * c + 1]);
        }
        claim[px] = kNoClaim;  // a loser comparing after this sees no claim of its own either
      } else {
        ls[j] = kLsPending;
        ++left;
      }
    }
    if (left) atomicAdd(&s_left, left);
    __syncthreads();
    if (alone) {
      const int tot = s_left;
      __syncthreads();  // read by every thread before thread 0 clears it in the next round
      if (tot == 0) break;
    } else {
      if (threadIdx.x == 0 && s_left) atomicAdd(ctl + 1 + r, (unsigned)s_left);
      grid_barrier(ctl, nb, phase, err_host);
      if (__hip_atomic_load(ctl + 1 + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) break;
    }
  }
  // cells still pending after the last round stay where they are
  for (int j = j0; j < L; j += js)
    if (ls[j] != kLsDone) result[__hip_atomic_load(list + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)] = -1;
}

// ---------------------------------------------------------------- neighbours
// The pixel -> cell index map is never cleared: index_map() writes every current cell's index, and a
// reader accepts an entry only if that cell still sits on the pixel (stale entries of dead or moved
// cells fail the check). Saves a clearing launch per neighbour query.
__device__ __forceinline__ int cell_at(const int32_t* idx_map, const int32_t* pos, int n, int C, long long px) {
  const int o = idx_map[px];
  if (o < 0 || o >= n) return -1;
  return ((long long)pos[2 * o] * C + pos[2 * o + 1]) == px ? o : -1;
}

__global__ void __launch_bounds__(256) index_map_kernel(int c, const int32_t* pos, int C, int32_t* idx_map, bool clear) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= c) return;
  idx_map[(size_t)pos[2 * i] * C + pos[2 * i + 1]] = clear ? -1 : i;
}

// the cell count of a chain issued before the host knows it (World._chain_bound): n is the bound,
// the count the sum of two device words (a kill_divide's survivors and placed children)
__device__ __forceinline__ int dev_count(int n, const int* na, const int* nb) {
  return na ? min(n, *na + *nb) : n;
}

// index_map_kernel + the longest genome of the c cells into `word` as (gen << 32) | length (one
// atomicMax per wave; a larger `gen` than the last call's overrides it, so the word is never reset):
// the bound of the recombination draws' thinning (rec_slot_draw), computed from the genomes alone so
// the device pipeline and the synchronous path draw against the same bound
__global__ void __launch_bounds__(256) index_map_lmax_kernel(int c, const int32_t* pos, int C, int32_t* idx_map,
                                                             const int32_t* lens, unsigned long long* word,
                                                             unsigned long long gen, const int* na, const int* nb) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  int l = 0;
  if (i < dev_count(c, na, nb)) {
    idx_map[(size_t)pos[2 * i] * C + pos[2 * i + 1]] = i;
    l = lens[i];
  }
  for (int o = 32; o > 0; o >>= 1) l = max(l, __shfl_xor(l, o));
  if ((threadIdx.x & 63) == 0) atomicMax(word, (gen << 32) | (unsigned long long)(unsigned)max(l, 0));
}
__device__ __forceinline__ int lmax_of(const unsigned long long* word) { return (int)(*word & 0xFFFFFFFFull); }

// Unique neighbour pairs (a < b) between the cells marked in_from and the cells marked in_to, in
// fixed slots: slot a*8 + j holds (a << 32) | b for the j-th smallest qualifying neighbour b > a of
// cell a (a pair belongs to its smaller cell: no pair twice, no atomics), else -1. An
// order-preserving compaction of the 8n slots then lists the pairs sorted by (a, b) -- no sort, no
// de-duplication pass (a neighbour met twice in a tiny wrapped map is kept once).
__global__ void __launch_bounds__(256) neighbor_pairs_sorted_kernel(int n, const int32_t* pos, Geom g,
                                                                    const int32_t* idx_map, const uint8_t* in_from,
                                                                    const uint8_t* in_to, int64_t* keys) {
  const int a = blockIdx.x * blockDim.x + threadIdx.x;
  if (a >= n) return;
  const bool fa = in_from[a] != 0, ta = in_to[a] != 0;
  int cand[8];
  int m = 0;
  if (fa || ta) {
    long long nb[8];
    const int cnt = moore(pos[2 * a], pos[2 * a + 1], g, nb);
    for (int q = 0; q < cnt; ++q) {
      const int o = cell_at(idx_map, pos, n, g.C, nb[q]);
      if (o <= a || !((fa && in_to[o]) || (ta && in_from[o]))) continue;
      int j = m;
      bool dup = false;
      for (int t = 0; t < m; ++t) dup |= cand[t] == o;
      if (dup) continue;
      while (j > 0 && cand[j - 1] > o) {  // insertion: cand stays ascending
        cand[j] = cand[j - 1];
        --j;
      }
      cand[j] = o;
      ++m;
    }
  }
  for (int j = 0; j < 8; ++j) keys[(size_t)a * 8 + j] = j < m ? (((int64_t)a << 32) | cand[j]) : -1;
}

// All neighbour pairs of all cells in fixed slots: slot c*8 + q holds (c << 32) | o for the q-th
// Moore neighbour o > c of cell c, else -1. Deterministic order (cell-major, reference neighbour
// order), no atomics, no counter read-back. One thread per slot: the index-map / position reads
// are two dependent random loads each, so 8x the threads hide their latency (one thread per cell
// ran 8 such chains back to back on a quarter-filled chip: ~70 us for 50k cells).
__global__ void __launch_bounds__(256) neighbor_slots_kernel(int n, const int32_t* pos, Geom g, const int32_t* idx_map,
                                                             int64_t* keys) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 8LL * n) return;
  const int c = (int)(t >> 3), q = (int)(t & 7);
  long long nb[8];
  const int cnt = moore(pos[2 * c], pos[2 * c + 1], g, nb);
  int64_t key = -1;
  if (q < cnt) {
    const int o = cell_at(idx_map, pos, n, g.C, nb[q]);
    if (o > c) key = ((int64_t)c << 32) | o;
  }
  keys[t] = key;
}

// The recombination draw of slot t (cell c = t / 8, its q-th Moore neighbour o), by thinning:
// N ~ Poisson(p * Lb), Lb = len(c) + lw >= len(c) + len(o) (lw: the longest genome, index_map_lmax),
// from the slot's Philox stream; each of the N events is kept with probability L / Lb (L = len(c) +
// len(o)), so the kept count is Poisson(p * L), the per-slot rate of the reference's pairs. Only the
// ~p * Lb of slots with N > 0 look up their neighbour: the 8n dependent random chains (position ->
// neighbour pixel -> index map -> its position -> its length) of a direct draw ran next to the
// diffusion stencil on the side stream, where every random load waits behind the stencil's HBM
// stream (rec_slots 20 us alone, 53-83 us beside it: profiles/r5/side_chain.txt). The same stream
// and draw order as rec_count_keys_kernel with lw >= 0 (the synchronous path): identical results.
// Returns the clamped event count (0: no recombination) and the pair key.
__device__ __forceinline__ int rec_slot_draw(long long t, int n, const int32_t* pos, const Geom& g,
                                             const int32_t* idx_map, const int32_t* lens, int lw, double p,
                                             uint64_t seed, uint64_t call, int kcap, int64_t& key) {
  const int c = (int)(t >> 3);
  const int lc = lens[c];
  const double lb = (double)lc + (double)lw;
  if (!(lb >= 1.0)) return 0;
  Philox rng(seed, call, (uint32_t)t);
  const long long nev = poisson(rng, p * lb);
  if (nev == 0) return 0;
  long long nb[8];
  const int nn = moore(pos[2 * c], pos[2 * c + 1], g, nb);
  const int q = (int)(t & 7);
  if (q >= nn) return 0;
  const int oo = cell_at(idx_map, pos, n, g.C, nb[q]);
  if (oo <= c) return 0;  // (the pair belongs to its smaller cell; -1: no cell there)
  const int L = lc + lens[oo];
  long long x = 0;
  for (long long e = 0; e < nev; ++e) x += rng.uniform_d() * lb < (double)L ? 1 : 0;
  if (kcap > 0 && x > kcap) x = kcap;
  key = ((int64_t)c << 32) | oo;
  return (int)(x > L ? L : x);
}

// Neighbour slots fused with the recombination draws of the device pipeline (gp_recombine) and
// the count pass of their selection: per tile of kSlotTile slots (16 per thread, the tiling of
// select.hip), the key and draw of slot t (rec_slot_draw: Poisson(p * (len a + len b)), the draws of
// rec_count_keys_kernel over neighbor_slots_kernel's keys), and the tile's
// number of slots with k > 0. One pass instead of three launches over the 8n slots; the write
// pass (select.hip) follows. A chain already broken by a narrow arena (gflags width bit) draws
// nothing and marks the call skipped, as gp_skip does.
constexpr int kSlotItems = 4, kSlotBlock = 256 * kSlotItems;  // 1024 slots per block: a count per
                                                                // quarter of select.hip's 4096-item tile
__global__ void __launch_bounds__(256) rec_slots_kernel(int n, const int32_t* pos, Geom g, const int32_t* idx_map,
                                                        const int32_t* lens, const unsigned long long* lw_word,
                                                        double p, uint64_t seed,
                                                        uint64_t call, int kcap, const int* gflags, int* opflags,
                                                        int64_t* keys, int32_t* kout, int32_t* tile_count,
                                                        int32_t* tile_max) {
  const bool skip = gflags && (*gflags & 8);  // mutations.hip kGpWidth
  if (skip && blockIdx.x == 0 && threadIdx.x == 0) atomicOr(opflags, 16);  // kGpSkipped
  const long long base = (long long)blockIdx.x * kSlotBlock, total = 8LL * n;
  const int lw = lmax_of(lw_word);
  int cnt = 0;
#pragma unroll
  for (int j = 0; j < kSlotItems; ++j) {
    const long long t = base + j * 256 + threadIdx.x;
    if (t >= total) continue;
    int64_t key = -1;
    const int kk = skip ? 0 : rec_slot_draw(t, n, pos, g, idx_map, lens, lw, p, seed, call, kcap, key);
    // (the pipeline reads keys only at the selected slots, kk > 0: ~1e-4 of them at the bench's
    // rate, so the other 8n - k key stores are skipped)
    if (kk > 0) keys[t] = key;
    kout[t] = kk;
    cnt += kk > 0;
  }
  __shared__ int s_cnt[4];
  for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
  if ((threadIdx.x & 63) == 0) s_cnt[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    tile_count[blockIdx.x] = s_cnt[0] + s_cnt[1] + s_cnt[2] + s_cnt[3];
    tile_max[blockIdx.x] = 0;
  }
}

// The selection of rec_slots_kernel's draws without its count array and selection pass (the default
// when the pair capacity fits rec_sort_kernel): the slots with events are appended (one atomic each,
// ~1e-4 of the slots at the bench's rate) and put in slot order by rec_sort_kernel.
constexpr int kRecSortCap = 4096;  // pair capacity of the thinned path (rec_sort_kernel's LDS)
__global__ void __launch_bounds__(256) rec_draw_kernel(int n, const int32_t* pos, Geom g, const int32_t* idx_map,
                                                       const int32_t* lens, const unsigned long long* lw_word,
                                                       double p, uint64_t seed,
                                                       uint64_t call, int kcap, const int* gflags, int* opflags,
                                                       int64_t* keys, int32_t* kout, int64_t* cand, int* cand_count,
                                                       int cap, const int* na, const int* nb) {
  const bool skip = gflags && (*gflags & 8);  // mutations.hip kGpWidth
  if (skip) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(opflags, 16);  // kGpSkipped
    return;
  }
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  n = dev_count(n, na, nb);
  if (t >= 8LL * n) return;
  int64_t key = -1;
  const int kk = rec_slot_draw(t, n, pos, g, idx_map, lens, lmax_of(lw_word), p, seed, call, kcap, key);
  if (kk <= 0) return;
  keys[t] = key;
  kout[t] = kk;
  const int j = atomicAdd(cand_count, 1);
  if (j < cap) cand[j] = t;
}

// One workgroup: the appended candidate slots into ascending slot order (bitonic sort in LDS) ->
// sel[0 : count] and out_dev = {count, 0}, as the capped selection pass writes them; more candidates
// than `cap` void the call (kGpSkipped / kGpWidth, the host replays it: select.hip cap semantics).
// The counter is reset for the next call on this stream. With `gather`: sel[i] = gather[sorted i].
__global__ void __launch_bounds__(1024) rec_sort_kernel(const int64_t* cand, int* cand_count, int cap, int64_t* sel,
                                                        int32_t* out_dev, int* gflags, int* opflags,
                                                        const int64_t* gather) {
  __shared__ int64_t s_v[kRecSortCap];
  __shared__ int s_total;
  if (threadIdx.x == 0) {
    s_total = *cand_count;
    *cand_count = 0;
  }
  __syncthreads();
  int total = s_total;
  if (total > cap) {
    if (threadIdx.x == 0) {
      if (opflags) atomicOr(opflags, 16);  // kGpSkipped
      if (gflags) atomicOr(gflags, 8);     // kGpWidth
      out_dev[0] = 0;
      out_dev[1] = 0;
    }
    return;
  }
  int np2 = 1;
  while (np2 < total) np2 <<= 1;
  for (int i = threadIdx.x; i < np2; i += blockDim.x) s_v[i] = i < total ? cand[i] : INT64_MAX;
  __syncthreads();
  for (int k = 2; k <= np2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < np2; i += blockDim.x) {
        const int l = i ^ j;
        if (l > i) {
          const int64_t a = s_v[i], b = s_v[l];
          const bool up = (i & k) == 0;
          if ((a > b) == up) {
            s_v[i] = b;
            s_v[l] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < total; i += blockDim.x) sel[i] = gather ? gather[s_v[i]] : s_v[i];
  if (threadIdx.x == 0) {
    out_dev[0] = total;
    out_dev[1] = 0;
  }
}

// ---------------------------------------------------------------- host launchers
static Geom geom(int R, int C, int r_lo, int r_hi, int wrap) {
  if (R <= 0 || C <= 0 || r_lo < 0 || r_hi > R || r_lo >= r_hi) throw std::invalid_argument("bad map geometry");
  if (!wrap && (r_lo < 1 || r_hi > R - 1)) throw std::invalid_argument("a non-wrapping strip needs halo rows");
  return Geom{R, C, r_lo, r_hi, wrap};
}

void split_cells(int k, int m, uintptr_t parents, uintptr_t children, uintptr_t cell_mols, uintptr_t divisions,
                 uintptr_t lifetimes, uintptr_t stream) {
  if (k <= 0 || m <= 0) return;
  msd::kl(split_cells_kernel, cdiv((long long)k * m, 256), 256, 0, S_(stream))(
      k, m, P_<int64_t>(parents), P_<int64_t>(children), P_<float>(cell_mols), P_<int32_t>(divisions),
      P_<int32_t>(lifetimes));
  MS_LAUNCH_CHECK();
}

void claim_free(int k, int R, int C, int r_lo, int r_hi, uintptr_t cell_map, uint64_t seed, uint64_t call,
                int attempts, uintptr_t out, uintptr_t stream) {
  if (k <= 0) return;
  const Geom g = geom(R, C, r_lo, r_hi, 1);
  msd::kl(claim_free_kernel, cdiv(k, 256), 256, 0, S_(stream))(k, g, P_<uint8_t>(cell_map), seed, call, attempts,
                                                           P_<long long>(out));
  MS_LAUNCH_CHECK();
}

constexpr int kPlaceWgMax = 2048;  // single-workgroup rounds up to this many cells (one CU: ~2 cells per thread)
static int g_coop_blocks = 256;    // co-resident workgroups of the single-launch placement (one per CU; 128: +18 % time)
// 0: the single-launch placement as an ordinary launch of at most as many workgroups as the device
// holds at once (its grid barrier is software: device-scope atomics with a bounded spin, see
// grid_barrier), 1: multi-launch rounds, 2: the same kernel through hipLaunchCooperativeKernel.
// Mode 2 was the default until it was traced as the cause of the SIGSEGV at exit of profiled
// processes: a cooperative launch makes the HIP runtime create its cooperative queue, and at exit
// the runtime's teardown of it (libamdhip64 -> libhsa-runtime64) touches a device mapping the
// already finalised rocprofiler-sdk tool released (profiles/r3/profexit: the faulting address is in
// a /dev/dri render-node mapping, frames hip exit handler -> hsa runtime -> fault). An ordinary
// launch never creates that queue, so profiles now time the production path.
static int g_place_mode = 0;
constexpr int kMaxDevices = 64;
// per device: two sets of control words of the cooperative launch, used in turn (a launch clears
// the set of the next one)
static unsigned* g_place_ctl[kMaxDevices] = {};
static int g_place_par[kMaxDevices] = {};
static unsigned* g_place_err = nullptr;           // pinned, mapped: a barrier timed out (any device)
static unsigned* g_place_err_dev = nullptr;
void set_place_mode(int mode) { g_place_mode = mode; }
// 1: the single-launch placement with one grid barrier and a one-workgroup tail (place_tail_coop_kernel)
static int g_place_tail = 1;
static char* g_place_list[kMaxDevices] = {};
static long long g_place_list_cap[kMaxDevices] = {};
void set_place_tail(int on) { g_place_tail = on; }

// 1 if a cooperative placement's grid barrier timed out since the last call (then its claims may
// have raced: the caller treats the world state as corrupt); clears the word.
int place_error_take() {
  if (!g_place_err) return 0;
  const unsigned v = __atomic_exchange_n(g_place_err, 0u, __ATOMIC_ACQ_REL);
  return v ? 1 : 0;
}
void set_coop_blocks(int n) { g_coop_blocks = std::max(1, std::min(n, 1024)); }

// Cooperative placement over `cells` (k entries) or over cells 0..k-1 selected by `mask`; returns
// false if the device refused the cooperative launch (the caller falls back to the rounds path).
static bool place_coop(int k, uintptr_t cells, uintptr_t mask, uintptr_t pos, const Geom& g, bool vacate,
                       uintptr_t cell_map, uintptr_t pending, uintptr_t cand, uintptr_t claim, uintptr_t result,
                       int rounds, uint64_t seed, uint64_t call, hipStream_t s) {
  int dev = 0;
  MS_HIP_CHECK(hipGetDevice(&dev));
  if (dev < 0 || dev >= kMaxDevices) throw std::runtime_error("place_coop: device index out of range");
  if (!g_place_ctl[dev]) {
    MS_HIP_CHECK(msd::dev_malloc((void**)&g_place_ctl[dev], 2 * kCtlWords * sizeof(unsigned)));
    MS_HIP_CHECK(msd::dev_memset(g_place_ctl[dev], 0, 2 * kCtlWords * sizeof(unsigned)));
    g_place_par[dev] = 0;
  }
  if (!g_place_err) {
    MS_HIP_CHECK(hipHostMalloc((void**)&g_place_err, sizeof(unsigned), hipHostMallocMapped | hipHostMallocCoherent));
    *g_place_err = 0;
    MS_HIP_CHECK(hipHostGetDevicePointer((void**)&g_place_err_dev, g_place_err, 0));
  }
  int kk = k;
  const int64_t* cp = cells ? P_<int64_t>(cells) : nullptr;
  const uint8_t* mp = mask ? P_<uint8_t>(mask) : nullptr;
  const int32_t* pp = P_<int32_t>(pos);
  uint8_t* cm = P_<uint8_t>(cell_map);
  uint8_t* pend = P_<uint8_t>(pending);
  long long* cd = P_<long long>(cand);
  int* cl = P_<int>(claim);
  long long* res = P_<long long>(result);
  int rr = std::min(rounds, kMaxRounds);
  unsigned* ctl = g_place_ctl[dev] + g_place_par[dev] * kCtlWords;
  unsigned* ctl_next = g_place_ctl[dev] + (1 - g_place_par[dev]) * kCtlWords;
  unsigned* err = g_place_err_dev;
  Geom gg = g;
  bool vac = vacate;
  void* args[] = {&kk, &cp, &mp, &pp, &gg, &vac, &cm, &pend, &seed, &call, &cd, &cl, &res, &rr, &ctl, &ctl_next, &err};
  unsigned grid = std::min<unsigned>(cdiv(k, 256), (unsigned)g_coop_blocks);
  if (g_place_tail && g_place_mode == 0) {
    // the list of round-0 losers + the tail workgroup's per-entry state (grown when k grows: the
    // stream is drained first, an earlier launch may still use the old buffer)
    if ((long long)k > g_place_list_cap[dev]) {
      if (g_place_list[dev]) {
        MS_HIP_CHECK(msd::stream_synchronize(s));
        MS_HIP_CHECK(msd::dev_free(g_place_list[dev]));
      }
      g_place_list_cap[dev] = std::max<long long>(k, 1ll << 16);
      MS_HIP_CHECK(msd::dev_malloc((void**)&g_place_list[dev], g_place_list_cap[dev] * 12));
    }
    long long* ls = reinterpret_cast<long long*>(g_place_list[dev]);
    int* list = reinterpret_cast<int*>(ls + g_place_list_cap[dev]);
    static int resident_t[kMaxDevices] = {};
    if (!resident_t[dev]) {
      int per_cu = 0, cus = 0;
      MS_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)place_tail_coop_kernel, 256, 0));
      MS_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
      resident_t[dev] = std::max(1, per_cu * cus);
    }
    grid = std::min<unsigned>(grid, (unsigned)resident_t[dev]);
    msd::kl(place_tail_coop_kernel, grid, 256, 0, s)(kk, cp, mp, pp, gg, vac, cm, seed, call, cd, cl, res, rr, ctl, ctl_next,
                                                err, list, ls);
    MS_LAUNCH_CHECK();
    g_place_par[dev] ^= 1;
    return true;
  }
  if (g_place_mode == 2) {
    const hipError_t e = msd::flushed_coop_launch((const void*)place_rounds_coop_kernel, dim3(grid), dim3(256), args,
                                                    0, s);
    if (e != hipSuccess) {
      (void)hipGetLastError();  // clear the sticky launch error; fall back
      return false;
    }
    g_place_par[dev] ^= 1;
    return true;
  }
  // ordinary launch: the grid must fit the device at once (every workgroup reaches the barriers)
  static int resident[kMaxDevices] = {};
  if (!resident[dev]) {
    int per_cu = 0, cus = 0;
    MS_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)place_rounds_coop_kernel, 256, 0));
    MS_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    resident[dev] = std::max(1, per_cu * cus);
  }
  grid = std::min<unsigned>(grid, (unsigned)resident[dev]);
  msd::kl(place_rounds_coop_kernel, grid, 256, 0, s)(kk, cp, mp, pp, gg, vac, cm, pend, seed, call, cd, cl, res, rr, ctl,
                                                 ctl_next, err);
  MS_LAUNCH_CHECK();
  g_place_par[dev] ^= 1;
  return true;
}

static void place_rounds_launches(int k, uintptr_t cells, uintptr_t mask, uintptr_t pos, const Geom& g, bool vacate,
                                  uintptr_t cell_map, uintptr_t pending, uintptr_t cand, uintptr_t claim,
                                  uintptr_t result, int rounds, uint64_t seed, uint64_t call, hipStream_t s);

// Deterministic spawn placement (spawn_cells on the GPU; the reference samples the free pixels with
// its RNG, world.py:910-920). New cell j draws up to kSpawnProbes uniform pixels of the owned rows
// per round from its own Philox stream and bids for the first free one (atomicMin of j on the claim
// map); the lowest bidder takes the pixel. Rounds are separated by grid barriers (a co-resident
// grid, as place_rounds_coop_kernel), so every bid reads the occupancy of the round's start: the
// winners, and so every position, are a function of the seed alone -- not of which wave's atomic
// landed first, as with the racing claims before. Cells still unplaced after kMaxRounds rounds (a
// nearly full map) are placed by one thread in index order, scanning from a drawn start. Winners
// release their claims at the end. result[j]: the pixel (-1 and `failed` set: no free pixel left).
constexpr int kSpawnProbes = 8;
__global__ void __launch_bounds__(256) spawn_claim_coop_kernel(int k, long long base, long long n_pix, uint8_t* cell_map,
                                                               uint64_t seed, uint64_t call, long long* cand, int* claim,
                                                               long long* result, unsigned* ctl, unsigned* ctl_next,
                                                               unsigned* err_host, int* failed) {
  const unsigned nb = gridDim.x;
  if (blockIdx.x == 0)
    for (int j = threadIdx.x; j < kCtlWords; j += blockDim.x) ctl_next[j] = 0u;
  const int stride = gridDim.x * blockDim.x, t0 = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned phase = 0;
  __shared__ int s_left;
  int r = 0;
  for (; r < kMaxRounds; ++r) {
    const uint64_t rc = call + ((uint64_t)r << 48);
    for (int i = t0; i < k; i += stride) {
      if (r == 0) __hip_atomic_store(result + i, -1ll, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else if (__hip_atomic_load(result + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= 0) continue;
      Philox rng(seed, rc, (uint32_t)i);
      long long px = -1;
      for (int t = 0; t < kSpawnProbes; ++t) {
        const long long q = base + (long long)rng.below64((uint64_t)n_pix);
        if (!map_get(cell_map, q)) {
          px = q;
          break;
        }
      }
      cand[i] = px;
      if (px >= 0) atomicMin(claim + px, i);
    }
    grid_barrier(ctl, nb, phase, err_host);
    if (threadIdx.x == 0) s_left = 0;
    __syncthreads();
    int left = 0;
    for (int i = t0; i < k; i += stride) {
      if (__hip_atomic_load(result + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= 0) continue;
      const long long px = cand[i];
      if (px >= 0 && __hip_atomic_load(claim + px, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == i) {
        __hip_atomic_store(result + i, px, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        map_set(cell_map, px);
      } else {
        ++left;
      }
    }
    if (left) atomicAdd(&s_left, left);
    __syncthreads();
    if (threadIdx.x == 0 && s_left) atomicAdd(ctl + 1 + r, (unsigned)s_left);
    grid_barrier(ctl, nb, phase, err_host);
    if (__hip_atomic_load(ctl + 1 + r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) break;
  }
  // winners release their claims (a claimed pixel's claim is its winner's)
  for (int i = t0; i < k; i += stride) {
    const long long px = __hip_atomic_load(result + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (px >= 0) claim[px] = kNoClaim;
  }
  // a nearly full map: what the rounds left, in index order by one thread (deterministic)
  if (r == kMaxRounds && blockIdx.x == 0 && threadIdx.x == 0) {
    for (int i = 0; i < k; ++i) {
      if (__hip_atomic_load(result + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= 0) continue;
      Philox rng(seed, call ^ 0x5DEECE66Dull, (uint32_t)i);
      const long long start = (long long)rng.below64((uint64_t)n_pix);
      long long got = -1;
      for (long long q = 0; q < n_pix && got < 0; ++q) {
        const long long px = base + (start + q) % n_pix;
        if (!map_get(cell_map, px)) got = px;
      }
      if (got < 0) {
        atomicOr(failed, 1);
        break;
      }
      map_set(cell_map, got);
      __hip_atomic_store(result + i, got, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Launcher of spawn_claim_coop_kernel (maps.hip spawn_dev): rows [r_lo, r_hi) of a C-wide map, the
// world's claim map (all kNoClaim between calls), per-cell scratch cand / result (k each).
void spawn_claims(int k, int C, int r_lo, int r_hi, uintptr_t cell_map, uintptr_t claim, uintptr_t cand,
                  uintptr_t result, uint64_t seed, uint64_t call, uintptr_t failed, hipStream_t s) {
  if (k <= 0) return;
  int dev = 0;
  MS_HIP_CHECK(hipGetDevice(&dev));
  if (dev < 0 || dev >= kMaxDevices) throw std::runtime_error("spawn_claims: device index out of range");
  if (!g_place_ctl[dev]) {
    MS_HIP_CHECK(msd::dev_malloc((void**)&g_place_ctl[dev], 2 * kCtlWords * sizeof(unsigned)));
    MS_HIP_CHECK(msd::dev_memset(g_place_ctl[dev], 0, 2 * kCtlWords * sizeof(unsigned)));
    g_place_par[dev] = 0;
  }
  if (!g_place_err) {
    MS_HIP_CHECK(hipHostMalloc((void**)&g_place_err, sizeof(unsigned), hipHostMallocMapped | hipHostMallocCoherent));
    *g_place_err = 0;
    MS_HIP_CHECK(hipHostGetDevicePointer((void**)&g_place_err_dev, g_place_err, 0));
  }
  static int resident[kMaxDevices] = {};
  if (!resident[dev]) {
    int per_cu = 0, cus = 0;
    MS_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, (const void*)spawn_claim_coop_kernel, 256, 0));
    MS_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    resident[dev] = std::max(1, per_cu * cus);
  }
  // (a co-resident grid: every workgroup reaches the barriers; grid-stride over the cells)
  const unsigned grid = std::min<unsigned>(std::min<unsigned>(cdiv(k, 256), (unsigned)g_coop_blocks),
                                           (unsigned)resident[dev]);
  unsigned* ctl = g_place_ctl[dev] + g_place_par[dev] * kCtlWords;
  unsigned* ctl_next = g_place_ctl[dev] + (1 - g_place_par[dev]) * kCtlWords;
  msd::kl(spawn_claim_coop_kernel, grid, 256, 0, s)(k, (long long)r_lo * C, (long long)(r_hi - r_lo) * C,
                                               P_<uint8_t>(cell_map), seed, call, P_<long long>(cand), P_<int>(claim),
                                               P_<long long>(result), ctl, ctl_next, g_place_err_dev, P_<int>(failed));
  MS_LAUNCH_CHECK();
  g_place_par[dev] ^= 1;
}

// Placement with a participation mask instead of a cell list (cells 0..n-1, priority = index).
void place_rounds_mask(int n, uintptr_t mask, uintptr_t pos, int R, int C, int r_lo, int r_hi, int wrap, bool vacate,
                       uintptr_t cell_map, uintptr_t pending, uintptr_t cand, uintptr_t claim, uintptr_t result,
                       int rounds, uint64_t seed, uint64_t call, uintptr_t stream) {
  if (n <= 0) return;
  const Geom g = geom(R, C, r_lo, r_hi, wrap);
  if (g_place_mode != 1 &&
      place_coop(n, 0, mask, pos, g, vacate, cell_map, pending, cand, claim, result, rounds, seed, call, S_(stream)))
    return;
  place_rounds_launches(n, 0, mask, pos, g, vacate, cell_map, pending, cand, claim, result, rounds, seed, call,
                        S_(stream));
}

// The multi-launch rounds (bid / resolve per round; the same draws and winners as the cooperative
// single launch). With a mask: cells 0..k-1 that take part.
static void place_rounds_launches(int k, uintptr_t cells, uintptr_t mask, uintptr_t pos, const Geom& g, bool vacate,
                                  uintptr_t cell_map, uintptr_t pending, uintptr_t cand, uintptr_t claim,
                                  uintptr_t result, int rounds, uint64_t seed, uint64_t call, hipStream_t s) {
  if (mask) {
    msd::kl(place_init_mask_kernel, cdiv(k, 256), 256, 0, s)(k, P_<uint8_t>(mask), P_<uint8_t>(pending), P_<long long>(result));
    MS_LAUNCH_CHECK();
  } else {
    MS_HIP_CHECK(msd::memset_async(P_<uint8_t>(pending), 1, (size_t)k, s));
    MS_HIP_CHECK(msd::memset_async(P_<long long>(result), 0xFF, (size_t)k * sizeof(long long), s));
  }
  const int64_t* cp = cells ? P_<int64_t>(cells) : nullptr;
  if (k <= kPlaceWgMax && cells) {
    msd::kl(place_rounds_wg_kernel, 1, 1024, 0, s)(k, cp, P_<int32_t>(pos), g, vacate, P_<uint8_t>(cell_map),
                                              P_<uint8_t>(pending), seed, call, P_<long long>(cand), P_<int>(claim),
                                              P_<long long>(result), rounds);
    MS_LAUNCH_CHECK();
    return;
  }
  const unsigned grid = cdiv(k, 256);
  for (int r = 0; r < rounds; ++r) {
    msd::kl(place_bid_kernel, grid, 256, 0, s)(k, cp, P_<int32_t>(pos), g, P_<uint8_t>(cell_map), P_<uint8_t>(pending),
                                          seed, call + ((uint64_t)r << 48), P_<long long>(cand), P_<int>(claim));
    MS_LAUNCH_CHECK();
    msd::kl(place_resolve_kernel, grid, 256, 0, s)(k, cp, P_<int32_t>(pos), g, vacate, P_<uint8_t>(cell_map),
                                              P_<uint8_t>(pending), P_<long long>(cand), P_<int>(claim),
                                              P_<long long>(result));
    MS_LAUNCH_CHECK();
  }
}

void place_rounds(int k, uintptr_t cells, uintptr_t pos, int R, int C, int r_lo, int r_hi, int wrap, bool vacate,
                  uintptr_t cell_map, uintptr_t pending, uintptr_t cand, uintptr_t claim, uintptr_t result, int rounds,
                  uint64_t seed, uint64_t call, uintptr_t stream) {
  if (k <= 0) return;
  const Geom g = geom(R, C, r_lo, r_hi, wrap);
  if (g_place_mode != 1 &&
      place_coop(k, cells, 0, pos, g, vacate, cell_map, pending, cand, claim, result, rounds, seed, call, S_(stream)))
    return;
  place_rounds_launches(k, cells, 0, pos, g, vacate, cell_map, pending, cand, claim, result, rounds, seed, call,
                        S_(stream));
}

int select_indices_async(long long n, int kind, uintptr_t src, uintptr_t sel, uintptr_t rest, uintptr_t out_dev,
                         uintptr_t stream);

// divide_cells over a mask, everything issued before the count is known: cooperative placement
// over the mask, winners (result >= 0) compacted with the count on the device and in a pinned
// status slot (returned), then the commit into rows n0.. (capacity for n more rows is the caller's).
// (n0_dev: optional device int added to n0 -- the survivor count of a kill issued just before)
int divide_mask_dev_at(int n, uintptr_t mask, uintptr_t pos, int R, int C, int r_lo, int r_hi, int wrap,
                       uintptr_t cell_map, uintptr_t pending, uintptr_t cand, uintptr_t claim, uintptr_t result,
                       int rounds, uint64_t seed, uint64_t call, uintptr_t wins, uintptr_t dcount, long long n0,
                       uintptr_t n0_dev, int m, uintptr_t par, uintptr_t cell_mols, uintptr_t divisions,
                       uintptr_t lifetimes, uintptr_t stream) {
  if (n <= 0) throw std::invalid_argument("divide_mask_dev: no cells");
  const Geom g = geom(R, C, r_lo, r_hi, wrap);
  hipStream_t s = S_(stream);
  if (g_place_mode == 1 ||
      !place_coop(n, 0, mask, pos, g, false, cell_map, pending, cand, claim, result, rounds, seed, call, s))
    place_rounds_launches(n, 0, mask, pos, g, false, cell_map, pending, cand, claim, result, rounds, seed, call, s);
  if (select_single_pass(n) && cdiv(n, kSelThreads) <= (unsigned)kLbMaxTiles) {
    long long* h64 = nullptr;
    const int slot = status_slot_new(&h64);
    const LbState lb = lb_begin(s);
    msd::kl(select_commit_kernel, cdiv(n, kSelThreads), kSelThreads, 0, s)(
        n, P_<long long>(result), lb.status, lb.gen, lb.err, P_<int64_t>(wins), P_<int32_t>(dcount), h64, C, n0,
        n0_dev ? P_<int>(n0_dev) : nullptr, m, P_<int64_t>(par), P_<int32_t>(pos), P_<float>(cell_mols),
        P_<int32_t>(divisions), P_<int32_t>(lifetimes));
    MS_LAUNCH_CHECK();
    return slot;
  }
  const int slot = select_indices_async(n, 3 /* int64 >= 0 */, result, wins, 0, dcount, stream);
  const unsigned grid = std::min<unsigned>(cdiv((long long)n * m, 256), 512u);
  msd::kl(divide_commit_kernel, grid, 256, 0, s)(P_<int>(dcount), P_<int64_t>(wins), P_<long long>(result), C, n0,
                                            n0_dev ? P_<int>(n0_dev) : nullptr, m,
                                            P_<int64_t>(par), P_<int32_t>(pos), P_<float>(cell_mols),
                                            P_<int32_t>(divisions), P_<int32_t>(lifetimes));
  MS_LAUNCH_CHECK();
  return slot;
}

int divide_mask_dev(int n, uintptr_t mask, uintptr_t pos, int R, int C, int r_lo, int r_hi, int wrap, uintptr_t cell_map,
                    uintptr_t pending, uintptr_t cand, uintptr_t claim, uintptr_t result, int rounds, uint64_t seed,
                    uint64_t call, uintptr_t wins, uintptr_t dcount, long long n0, int m, uintptr_t par,
                    uintptr_t cell_mols, uintptr_t divisions, uintptr_t lifetimes, uintptr_t stream) {
  return divide_mask_dev_at(n, mask, pos, R, C, r_lo, r_hi, wrap, cell_map, pending, cand, claim, result, rounds, seed,
                            call, wins, dcount, n0, 0, m, par, cell_mols, divisions, lifetimes, stream);
}

void place_collect(int k, uintptr_t wins, uintptr_t cells, uintptr_t result, int C, uintptr_t par, uintptr_t npos,
                   uintptr_t stream) {
  if (k <= 0) return;
  msd::kl(place_collect_kernel, cdiv(k, 256), 256, 0, S_(stream))(k, P_<int64_t>(wins), cells ? P_<int64_t>(cells) : nullptr,
                                                              P_<long long>(result), C, P_<int64_t>(par),
                                                              P_<int32_t>(npos));
  MS_LAUNCH_CHECK();
}

void index_map(int c, uintptr_t pos, int C, uintptr_t idx_map, bool clear, uintptr_t stream) {
  if (c <= 0) return;
  msd::kl(index_map_kernel, cdiv(c, 256), 256, 0, S_(stream))(c, P_<int32_t>(pos), C, P_<int32_t>(idx_map), clear);
  MS_LAUNCH_CHECK();
}

void index_map_lmax(int c, uintptr_t pos, int C, uintptr_t idx_map, uintptr_t lens, uintptr_t word, uint64_t gen,
                    uintptr_t na, uintptr_t nb, uintptr_t stream) {
  if (c <= 0) return;
  if (gen == 0 || gen >= (1ull << 31)) throw std::invalid_argument("index_map_lmax: generation out of range");
  if ((na == 0) != (nb == 0)) throw std::invalid_argument("index_map_lmax: give both device count words or neither");
  msd::kl(index_map_lmax_kernel, cdiv(c, 256), 256, 0, S_(stream))(c, P_<int32_t>(pos), C, P_<int32_t>(idx_map),
                                                               P_<int32_t>(lens), P_<unsigned long long>(word), gen,
                                                               na ? P_<int>(na) : nullptr, nb ? P_<int>(nb) : nullptr);
  MS_LAUNCH_CHECK();
}

void neighbor_slots(int n, uintptr_t pos, int R, int C, int r_lo, int r_hi, int wrap, uintptr_t idx_map, uintptr_t keys,
                    uintptr_t stream) {
  if (n <= 0) return;
  const Geom g = geom(R, C, r_lo, r_hi, wrap);
  msd::kl(neighbor_slots_kernel, cdiv(8LL * n, 256), 256, 0, S_(stream))(n, P_<int32_t>(pos), g, P_<int32_t>(idx_map),
                                                               P_<int64_t>(keys));
  MS_LAUNCH_CHECK();
}

std::pair<int32_t*, int32_t*> select_tiles(long long tiles, hipStream_t s);
void select_write_i32pos_capped(long long n, uintptr_t src, int32_t* tc, int32_t* tm, int sub, uintptr_t sel,
                                uintptr_t out_dev, int cap, uintptr_t gflags, uintptr_t opflags, hipStream_t s);

// per-stream append counters of the draw kernels (rec_draw_kernel, mutations.hip mut_draw_kernel):
// zero between calls, rec_sort_kernel resets them (the calls of one stream run one after another)
static std::unordered_map<hipStream_t, int*> g_sel_cnt;
int* append_counter(hipStream_t s) {
  int*& cnt = g_sel_cnt[s];
  if (!cnt) {
    MS_HIP_CHECK(msd::dev_malloc((void**)&cnt, sizeof(int)));
    MS_HIP_CHECK(msd::memset_async(cnt, 0, sizeof(int), s));
  }
  return cnt;
}
void sel_sort(uintptr_t cand, int* cnt, int cap, uintptr_t sel, uintptr_t out_dev, uintptr_t gflags, uintptr_t opflags,
              hipStream_t s, uintptr_t gather) {
  msd::kl(rec_sort_kernel, 1, 1024, 0, s)(P_<int64_t>(cand), cnt, cap, P_<int64_t>(sel), P_<int32_t>(out_dev),
                                     P_<int>(gflags), P_<int>(opflags), gather ? P_<int64_t>(gather) : nullptr);
  MS_LAUNCH_CHECK();
}
int sel_sort_cap() { return kRecSortCap; }
static int g_rec_thin = 1;  // 0: the count + selection passes for every capacity (A/B)
extern int g_mut_append;     // (mutations.hip: the same for the mutation draws)
void set_rec_thinning(int on) { g_rec_thin = g_mut_append = on; }

// The recombination draws of all slots (rec_slot_draw) + the capped selection of slots with k > 0
// into sel / out_dev (gp_recombine): appended and sorted (rec_draw_kernel + rec_sort_kernel) with a
// pair capacity of at most kRecSortCap, else rec_slots_kernel + the selection pass. `lw`: the
// longest genome (index_map_lmax's word). `cand`: 8 * cap bytes of scratch.
void rec_slots(int n, uintptr_t pos, int R, int C, int r_lo, int r_hi, int wrap, uintptr_t idx_map, uintptr_t lens,
               uintptr_t lw_word, double p, uint64_t seed, uint64_t call, int kcap, uintptr_t gflags,
               uintptr_t opflags, uintptr_t keys, uintptr_t k, uintptr_t sel, uintptr_t out_dev, int cap,
               uintptr_t cand, uintptr_t stream, uintptr_t na, uintptr_t nb) {
  if (n <= 0) throw std::invalid_argument("rec_slots: no cells");
  const Geom g = geom(R, C, r_lo, r_hi, wrap);
  hipStream_t s = S_(stream);
  const long long total = 8LL * n;
  if (!lw_word) throw std::invalid_argument("rec_slots: the longest-genome word of index_map_lmax is required");
  const auto* lw = P_<unsigned long long>(lw_word);
  if (g_rec_thin && cand && cap <= kRecSortCap) {
    int* cnt = append_counter(s);
    msd::kl(rec_draw_kernel, (unsigned)cdiv(total, 256), 256, 0, s)(
        n, P_<int32_t>(pos), g, P_<int32_t>(idx_map), P_<int32_t>(lens), lw, p, seed, call, kcap, P_<int>(gflags),
        P_<int>(opflags), P_<int64_t>(keys), P_<int32_t>(k), P_<int64_t>(cand), cnt, cap, na ? P_<int>(na) : nullptr,
        nb ? P_<int>(nb) : nullptr);
    MS_LAUNCH_CHECK();
    sel_sort(cand, cnt, cap, sel, out_dev, gflags, opflags, s, 0);
    return;
  }
  if (na) throw std::invalid_argument("rec_slots: a device cell count needs the append path (cap <= the sort's)");
  constexpr int kSelTile = 4096;  // select.hip
  const long long blocks = (total + kSelTile - 1) / kSelTile * (kSelTile / kSlotBlock);
  auto tiles = select_tiles(blocks, s);
  // (the blocks past the last slot write zero counts: the write pass reads whole tiles' counts)
  msd::kl(rec_slots_kernel, (unsigned)blocks, 256, 0, s)(n, P_<int32_t>(pos), g, P_<int32_t>(idx_map), P_<int32_t>(lens), lw,
                                                    p, seed, call, kcap, P_<int>(gflags), P_<int>(opflags),
                                                    P_<int64_t>(keys), P_<int32_t>(k), tiles.first, tiles.second);
  MS_LAUNCH_CHECK();
  select_write_i32pos_capped(total, k, tiles.first, tiles.second, kSelTile / kSlotBlock, sel, out_dev, cap, gflags,
                             opflags, s);
}

void neighbor_pairs_sorted(int n, uintptr_t pos, int R, int C, int r_lo, int r_hi, int wrap, uintptr_t idx_map,
                           uintptr_t in_from, uintptr_t in_to, uintptr_t keys, uintptr_t stream) {
  if (n <= 0) return;
  const Geom g = geom(R, C, r_lo, r_hi, wrap);
  msd::kl(neighbor_pairs_sorted_kernel, cdiv(n, 256), 256, 0, S_(stream))(n, P_<int32_t>(pos), g, P_<int32_t>(idx_map),
                                                                     P_<uint8_t>(in_from), P_<uint8_t>(in_to),
                                                                     P_<int64_t>(keys));
  MS_LAUNCH_CHECK();
}


void release_world_buffers() {
  int cur = 0;
  MS_HIP_CHECK(hipGetDevice(&cur));
  for (int d = 0; d < kMaxDevices; ++d) {
    if (!g_place_ctl[d]) continue;
    MS_HIP_CHECK(hipSetDevice(d));
    MS_HIP_CHECK(msd::dev_free(g_place_ctl[d]));
    g_place_ctl[d] = nullptr;
  }
  MS_HIP_CHECK(hipSetDevice(cur));
  if (g_place_err) MS_HIP_CHECK(hipHostFree(g_place_err));
  g_place_err = nullptr;
  g_place_err_dev = nullptr;
}

}  // namespace msd
