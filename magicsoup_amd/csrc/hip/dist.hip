// Kernels of the strip-decomposed world's exchange protocols (magicsoup_amd.parallel.dist_world).
//
// A rank owns rows 1..H of an (H + 2) x C strip; rows 0 and H + 1 are halo copies of the
// neighbours' boundary rows. Everything here exists so that one step needs no host round trip
// beyond the ones a single-GPU world already makes, and only fixed-size or header-sized messages:
//
//   strip_marks / strip_reserve   division: a byte per boundary column (occupied, dividing cell)
//                                 goes to the neighbour, which copies the occupancy into its halo
//                                 row and reserves its boundary pixels next to the neighbour's
//                                 dividing cells. Claims into halo rows are then conflict-free,
//                                 so the owner accepts them all (no verdict round trip).
//   place_split                   winners of the placement rounds split into local / up / down
//                                 children (order-preserving, counts + headers on the device)
//   rec_pack / rec_unpack         child / migrant records (position, lengths, counters,
//                                 molecules, label, genome) packed for and appended from the peers
//   halo_pack / halo_unpack       molecule-map boundary rows <-> contiguous exchange buffers
//   xb_prep / xb_events / xb_apply recombination across a strip boundary, computed identically on
//                                 both ranks from exchanged lengths and genomes (shared RNG stream)
#include <algorithm>

#include "hip_common.h"
#include "rec_common.h"
#include "select_lb.h"

namespace msd {

// ---------------------------------------------------------------- division: boundary marks
// marks[y] of the owned boundary rows: 1 = occupied, 3 = occupied by a dividing cell
__global__ void __launch_bounds__(256) strip_occ_kernel(int C, int H, const uint8_t* cell_map, uint8_t* up, uint8_t* dn) {
  const int y = blockIdx.x * blockDim.x + threadIdx.x;
  if (y >= C) return;
  up[y] = cell_map[(size_t)1 * C + y] ? 1 : 0;
  dn[y] = cell_map[(size_t)H * C + y] ? 1 : 0;
}

// dividing cells: a list (cells) or, with cells == nullptr, cells i < k with mask[i] != 0
__global__ void __launch_bounds__(256) strip_div_kernel(int k, const int64_t* cells, const uint8_t* mask,
                                                        const int32_t* pos, int C, int H, uint8_t* up, uint8_t* dn) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= k) return;
  if (!cells && !mask[i]) return;
  const int64_t c = cells ? cells[i] : i;
  const int x = pos[2 * c], y = pos[2 * c + 1];
  if (x == 1) up[y] = 3;
  if (x == H) dn[y] = 3;
}

// The upper neighbour's row H (from_up) and the lower one's row 1 (from_dn) arrived: halo rows get
// their occupancy; free owned boundary pixels next to a neighbour's dividing cell are reserved
// (value 2: occupied for the placement rounds, cleared by strip_clear).
__global__ void __launch_bounds__(256) strip_reserve_kernel(int C, int H, const uint8_t* from_up, const uint8_t* from_dn,
                                                            uint8_t* cell_map) {
  const int y = blockIdx.x * blockDim.x + threadIdx.x;
  if (y >= C) return;
  const int yl = y == 0 ? C - 1 : y - 1, yr = y == C - 1 ? 0 : y + 1;
  cell_map[y] = from_up[y] & 1;
  cell_map[(size_t)(H + 1) * C + y] = from_dn[y] & 1;
  if (!cell_map[(size_t)C + y] && ((from_up[yl] | from_up[y] | from_up[yr]) & 2)) cell_map[(size_t)C + y] = 2;
  if (!cell_map[(size_t)H * C + y] && ((from_dn[yl] | from_dn[y] | from_dn[yr]) & 2)) cell_map[(size_t)H * C + y] = 2;
}

// halo rows back to empty, reservations released (claimed pixels are 1 and stay)
__global__ void __launch_bounds__(256) strip_clear_kernel(int C, int H, uint8_t* cell_map) {
  const int y = blockIdx.x * blockDim.x + threadIdx.x;
  if (y >= C) return;
  cell_map[y] = 0;
  cell_map[(size_t)(H + 1) * C + y] = 0;
  if (cell_map[(size_t)C + y] == 2) cell_map[(size_t)C + y] = 0;
  if (cell_map[(size_t)H * C + y] == 2) cell_map[(size_t)H * C + y] = 0;
}

// ---------------------------------------------------------------- division: winners by destination
// Class of placement result i: -1 no pixel, 0 owned row, 1 upper halo (row 0), 2 lower halo (row H+1).
constexpr int kSplitThreads = 256, kSplitItems = 8, kSplitTile = kSplitThreads * kSplitItems;

__device__ __forceinline__ int split_class(long long px, int C, int H) {
  if (px < 0) return -1;
  const long long x = px / C;
  return x == 0 ? 1 : (x == H + 1 ? 2 : 0);
}

__global__ void __launch_bounds__(kSplitThreads) place_split_count_kernel(int k, const long long* result, int C, int H,
                                                                          int32_t* tile_counts) {
  __shared__ int s[3][kSplitThreads / 64];
  int c[3] = {0, 0, 0};
  const long long base = (long long)blockIdx.x * kSplitTile;
#pragma unroll
  for (int j = 0; j < kSplitItems; ++j) {
    const long long i = base + j * kSplitThreads + threadIdx.x;
    const int cls = i < k ? split_class(result[i], C, H) : -1;
    if (cls >= 0) ++c[cls];
  }
  for (int o = 32; o > 0; o >>= 1)
    for (int q = 0; q < 3; ++q) c[q] += __shfl_xor(c[q], o);
  if (lane_id() == 0)
    for (int q = 0; q < 3; ++q) s[q][threadIdx.x >> 6] = c[q];
  __syncthreads();
  if (threadIdx.x < 3) {
    int t = 0;
    for (int w = 0; w < kSplitThreads / 64; ++w) t += s[threadIdx.x][w];
    tile_counts[(size_t)blockIdx.x * 3 + threadIdx.x] = t;
  }
}

// par[cls * k + j] = cells[i], npos[(cls * k + j) * 2 + {0,1}] = pixel (x, y) of the j-th winner of
// class cls (in list order). The last tile writes counts[3] and the headers' first words.
__global__ void __launch_bounds__(kSplitThreads) place_split_write_kernel(int k, const long long* result,
                                                                          const int64_t* cells, int C, int H,
                                                                          const int32_t* tile_counts, int64_t* par,
                                                                          int32_t* npos, int32_t* counts,
                                                                          int32_t* hdr_up, int32_t* hdr_dn, int lw,
                                                                          int gw, int m) {
  constexpr int W = kSplitThreads / 64;
  __shared__ int s_off[3];
  __shared__ int s_wc[kSplitItems][3][W];
  __shared__ int s_pre[kSplitItems][3][W];
  const int w = threadIdx.x >> 6, lane = lane_id();
  const int b = blockIdx.x;
  if (threadIdx.x < 3) {
    int o = 0;
    for (int q = 0; q < b; ++q) o += tile_counts[(size_t)q * 3 + threadIdx.x];
    s_off[threadIdx.x] = o;
  }
  const long long base = (long long)b * kSplitTile;
  uint64_t bal[kSplitItems][3];
#pragma unroll
  for (int j = 0; j < kSplitItems; ++j) {
    const long long i = base + j * kSplitThreads + threadIdx.x;
    const int cls = i < k ? split_class(result[i], C, H) : -1;
    for (int q = 0; q < 3; ++q) {
      bal[j][q] = __ballot(cls == q);
      if (lane == 0) s_wc[j][q][w] = __popcll(bal[j][q]);
    }
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    int acc = 0;
    for (int j = 0; j < kSplitItems; ++j)
      for (int q = 0; q < W; ++q) {
        s_pre[j][threadIdx.x][q] = acc;
        acc += s_wc[j][threadIdx.x][q];
      }
  }
  __syncthreads();
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
  for (int j = 0; j < kSplitItems; ++j) {
    const long long i = base + j * kSplitThreads + threadIdx.x;
    if (i >= k) break;
    for (int q = 0; q < 3; ++q) {
      if (!((bal[j][q] >> lane) & 1ull)) continue;
      const long long o = (long long)q * k + s_off[q] + s_pre[j][q][w] + __popcll(bal[j][q] & lt);
      const long long px = result[i];
      par[o] = cells ? cells[i] : i;
      npos[2 * o] = (int32_t)(px / C);
      npos[2 * o + 1] = (int32_t)(px - (px / C) * C);
    }
  }
  if (b == (int)gridDim.x - 1 && threadIdx.x < 3) {
    int t = s_off[threadIdx.x];
    for (int j = 0; j < kSplitItems; ++j)
      for (int q = 0; q < W; ++q) t += s_wc[j][threadIdx.x][q];
    counts[threadIdx.x] = t;
    int32_t* hdr = threadIdx.x == 1 ? hdr_up : (threadIdx.x == 2 ? hdr_dn : nullptr);
    if (hdr) {
      hdr[0] = t;
      hdr[1] = lw;
      hdr[2] = gw;
      hdr[3] = m;
    }
  }
}

// place_split_count_kernel + place_split_write_kernel in one launch (select_lb.h's scheme with three
// classes): each tile publishes its three counts (12 bits each, a tile holds 2048 items) tagged with
// the call's generation, sums the earlier tiles' words and writes its winners. Same output.
__global__ void __launch_bounds__(kSplitThreads) place_split_lb_kernel(int k, const long long* result,
                                                                       const int64_t* cells, int C, int H,
                                                                       unsigned long long* status, uint32_t gen,
                                                                       unsigned* err, int64_t* par, int32_t* npos,
                                                                       int32_t* counts,
                                                                       int32_t* hdr_up, int32_t* hdr_dn, int lw,
                                                                       int gw, int m) {
  constexpr int W = kSplitThreads / 64;
  static_assert(kSplitTile < 4096, "tile counts are packed in 12 bits");
  __shared__ int s_wc[kSplitItems][3][W];
  __shared__ int s_pre[kSplitItems][3][W];
  __shared__ int s_tot[3];
  __shared__ int s_red[3][W];
  __shared__ int s_off[3];
  const int w = threadIdx.x >> 6, lane = lane_id();
  const int b = blockIdx.x;
  const long long base = (long long)b * kSplitTile;
  uint64_t bal[kSplitItems][3];
#pragma unroll
  for (int j = 0; j < kSplitItems; ++j) {
    const long long i = base + j * kSplitThreads + threadIdx.x;
    const int cls = i < k ? split_class(result[i], C, H) : -1;
    for (int q = 0; q < 3; ++q) {
      bal[j][q] = __ballot(cls == q);
      if (lane == 0) s_wc[j][q][w] = __popcll(bal[j][q]);
    }
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    int acc = 0;
    for (int j = 0; j < kSplitItems; ++j)
      for (int q = 0; q < W; ++q) {
        s_pre[j][threadIdx.x][q] = acc;
        acc += s_wc[j][threadIdx.x][q];
      }
    s_tot[threadIdx.x] = acc;
  }
  __syncthreads();
  const unsigned long long tag = gen & kLbGenMask;  // (lb_begin keeps gen within the 28 bits)
  if (threadIdx.x == 0)
    __hip_atomic_store(status + b,
                       (tag << 36) | (unsigned long long)s_tot[0] | ((unsigned long long)s_tot[1] << 12) |
                           ((unsigned long long)s_tot[2] << 24),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // the earlier tiles' counts (every tile publishes before it waits; bounded spin as in select_lb.h)
  int o[3] = {0, 0, 0};
  for (int q = threadIdx.x; q < b; q += kSplitThreads) {
    unsigned long long v = __hip_atomic_load(status + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int spin = 0; (v >> 36) != tag; ++spin) {
      if (spin >= (1 << 22)) {  // (reported through hip_ops.check_placement instead of a hang)
        if (err) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      v = __hip_atomic_load(status + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    o[0] += (int)(v & 0xFFFu);
    o[1] += (int)((v >> 12) & 0xFFFu);
    o[2] += (int)((v >> 24) & 0xFFFu);
  }
  for (int c = 0; c < 3; ++c) {
    for (int sh = 32; sh > 0; sh >>= 1) o[c] += __shfl_xor(o[c], sh);
    if (lane == 0) s_red[c][w] = o[c];
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    int t = 0;
    for (int q = 0; q < W; ++q) t += s_red[threadIdx.x][q];
    s_off[threadIdx.x] = t;
  }
  __syncthreads();
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
  for (int j = 0; j < kSplitItems; ++j) {
    const long long i = base + j * kSplitThreads + threadIdx.x;
    if (i >= k) break;
    for (int q = 0; q < 3; ++q) {
      if (!((bal[j][q] >> lane) & 1ull)) continue;
      const long long oo = (long long)q * k + s_off[q] + s_pre[j][q][w] + __popcll(bal[j][q] & lt);
      const long long px = result[i];
      par[oo] = cells ? cells[i] : i;
      npos[2 * oo] = (int32_t)(px / C);
      npos[2 * oo + 1] = (int32_t)(px - (px / C) * C);
    }
  }
  if (b == (int)gridDim.x - 1 && threadIdx.x < 3) {
    const int t = s_off[threadIdx.x] + s_tot[threadIdx.x];
    counts[threadIdx.x] = t;
    int32_t* hdr = threadIdx.x == 1 ? hdr_up : (threadIdx.x == 2 ? hdr_dn : nullptr);
    if (hdr) {
      hdr[0] = t;
      hdr[1] = lw;
      hdr[2] = gw;
      hdr[3] = m;
    }
  }
}

// ---------------------------------------------------------------- cell records
// Record layout (4-byte words): y, genome length, label length, divisions, lifetime, m molecules,
// then the label row (lw bytes) and the genome (gw bytes: the sender's genome length bound, zero
// padded); lw, gw are multiples of 4. Genomes come from / go to the genome pool (hip_common.h).
struct RecCols {
  float* mols;
  int32_t* pos;
  int32_t* life;
  int32_t* div;
  uint8_t* pool;
  int64_t* off;
  unsigned long long* top;
  long long pool_cap;
  int* pool_failed;
  int32_t* glen;
  int gw;
  uint8_t* ldata;
  int32_t* llen;
  int lw;
  int m;
};

__host__ __device__ __forceinline__ long long rec_bytes(int m, int lw, int gw) { return 4ll * (5 + m) + lw + gw; }

// One wavefront per record: records of cells par_up[0..k_up) go to out_up, par_dn[..] to out_dn.
// child: the record describes the cell's child (half the molecules, divisions + 1, lifetime 0).
__global__ void __launch_bounds__(64) rec_pack_kernel(int k_up, int k_dn, const int64_t* par_up, const int32_t* pos_up,
                                                      const int64_t* par_dn, const int32_t* pos_dn, RecCols w,
                                                      bool child, uint8_t* out_up, uint8_t* out_dn) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const bool up = b < k_up;
  const int j = up ? b : b - k_up;
  if (!up && j >= k_dn) return;
  const int64_t c = up ? par_up[j] : par_dn[j];
  const int y = up ? pos_up[2 * j + 1] : pos_dn[2 * j + 1];
  const long long B = rec_bytes(w.m, w.lw, w.gw);
  uint8_t* r = (up ? out_up : out_dn) + (size_t)j * B;
  int32_t* h = reinterpret_cast<int32_t*>(r);
  float* mol = reinterpret_cast<float*>(r + 20);
  if (lane == 0) {
    h[0] = y;
    h[1] = w.glen[c];
    h[2] = w.llen[c];
    h[3] = w.div[c] + (child ? 1 : 0);
    h[4] = child ? 0 : w.life[c];
  }
  for (int q = lane; q < w.m; q += 64) mol[q] = w.mols[(size_t)c * w.m + q] * (child ? 0.5f : 1.0f);
  const uint32_t* ls = reinterpret_cast<const uint32_t*>(w.ldata + (size_t)c * w.lw);
  uint32_t* ld = reinterpret_cast<uint32_t*>(r + 4 * (5 + w.m));
  for (int q = lane; q < w.lw / 4; q += 64) ld[q] = ls[q];
  const uint8_t* gs = w.pool + w.off[c];
  uint8_t* gd = r + 4 * (5 + w.m) + w.lw;
  const int gl = min(w.glen[c], w.gw);
  for (int q = lane; q < w.gw; q += 64) gd[q] = q < gl ? gs[q] : 0;
}

// Append k_up records from the upper neighbour (landing on row 1) and k_dn from the lower one
// (row H) as cells n0, n0 + 1, ...; the sender's label / genome row widths are slw / sgw.
__global__ void __launch_bounds__(64) rec_unpack_kernel(int n0, int k_up, const uint8_t* in_up, int up_lw, int up_gw,
                                                        int k_dn, const uint8_t* in_dn, int dn_lw, int dn_gw, int C,
                                                        int H, RecCols w, uint8_t* cell_map) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const bool up = b < k_up;
  const int j = up ? b : b - k_up;
  if (!up && j >= k_dn) return;
  const int slw = up ? up_lw : dn_lw, sgw = up ? up_gw : dn_gw;
  const long long B = rec_bytes(w.m, slw, sgw);
  const uint8_t* r = (up ? in_up : in_dn) + (size_t)j * B;
  const int32_t* h = reinterpret_cast<const int32_t*>(r);
  const float* mol = reinterpret_cast<const float*>(r + 20);
  const long long c = (long long)n0 + b;
  const int x = up ? 1 : H, y = h[0];
  const int gl = min(h[1], w.gw), ll = min(h[2], w.lw);
  if (lane == 0) {
    w.pos[2 * c] = x;
    w.pos[2 * c + 1] = y;
    w.glen[c] = gl;
    w.llen[c] = ll;
    w.div[c] = h[3];
    w.life[c] = h[4];
    cell_map[(size_t)x * C + y] = 1;
  }
  for (int q = lane; q < w.m; q += 64) w.mols[c * w.m + q] = mol[q];
  const uint8_t* ls = r + 4 * (5 + w.m);
  for (int q = lane; q < w.lw; q += 64) w.ldata[c * w.lw + q] = q < ll ? ls[q] : 0;
  const uint8_t* gs = ls + slw;
  // the genome into fresh pool space (the host made room for every record before the launch)
  long long o = 0;
  if (lane == 0) o = pool_alloc(w.top, w.pool_cap, gl);
  o = (long long)(((unsigned long long)(unsigned)__shfl((int)(o >> 32), 0) << 32) |
                  (unsigned long long)(unsigned)__shfl((int)(o & 0xFFFFFFFFll), 0));
  if (o < 0) {
    if (lane == 0) {
      if (w.pool_failed) atomicOr(w.pool_failed, 1);
      w.off[c] = 0;
      w.glen[c] = 0;
    }
    return;
  }
  for (int q = lane; q < gl; q += 64) w.pool[o + q] = gs[q];
  if (lane == 0) w.off[c] = o;
}

// ---------------------------------------------------------------- diffusion halo rows
// send_up[j, :] = map[j, 1, :], send_dn[j, :] = map[j, H, :] (elem-byte elements, copied as words)
template <class T>
__global__ void __launch_bounds__(256) halo_pack_kernel(int m, int C, int H, const T* map, T* send_up, T* send_dn) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)m * C) return;
  const int j = (int)(t / C), y = (int)(t - (long long)j * C);
  const size_t plane = (size_t)(H + 2) * C;
  send_up[t] = map[j * plane + (size_t)C + y];
  send_dn[t] = map[j * plane + (size_t)H * C + y];
}

template <class T>
__global__ void __launch_bounds__(256) halo_unpack_kernel(int m, int C, int H, T* map, const T* from_up, const T* from_dn) {
  const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (long long)m * C) return;
  const int j = (int)(t / C), y = (int)(t - (long long)j * C);
  const size_t plane = (size_t)(H + 2) * C;
  map[j * plane + y] = from_up[t];
  map[j * plane + (size_t)(H + 1) * C + y] = from_dn[t];
}


// ---------------------------------------------------------------- recombination across a boundary
// Every pair (upper cell at (its row H, y), lower cell at (its row 1, y + d)), d in {-1, 0, 1}, of the
// boundary between rank u and u + 1 is item 3 y + d + 1. Both ranks of a boundary know both rows'
// genome lengths (exchanged), draw the same Poisson counts from the boundary's stream (seed, call,
// item), keep the same first E events, swap the involved genomes and compute the same
// recombinations (rec_pair_apply); each keeps the result of its own cell.
__device__ __forceinline__ int strip_cell_at(const int32_t* idx_map, const int32_t* pos, int n, int C, long long px) {
  const int o = idx_map[px];
  if (o < 0 || o >= n) return -1;
  return ((long long)pos[2 * o] * C + pos[2 * o + 1]) == px ? o : -1;
}

// own boundary cells and their genome lengths (-1: no cell); word C of each length row = the
// genome length bound of the pool (PoolArena.width)
__global__ void __launch_bounds__(256) xb_prep_kernel(int C, int H, int n, const int32_t* pos, const int32_t* idx_map,
                                                      const int32_t* lens, int width, int32_t* len_up, int32_t* len_dn,
                                                      int32_t* own1, int32_t* ownH) {
  const int y = blockIdx.x * blockDim.x + threadIdx.x;
  if (y == 0) {
    len_up[C] = width;
    len_dn[C] = width;
  }
  if (y >= C) return;
  const int c1 = strip_cell_at(idx_map, pos, n, C, (long long)C + y);
  const int cH = strip_cell_at(idx_map, pos, n, C, (long long)H * C + y);
  own1[y] = c1;
  ownH[y] = cH;
  len_up[y] = c1 >= 0 ? lens[c1] : -1;
  len_dn[y] = cH >= 0 ? lens[cH] : -1;
}

struct XbEvents {
  int32_t* b;     // boundary of event j: 0 = below this rank (we are the upper side), 1 = above
  int32_t* item;  // item index within the boundary
  int32_t* k;     // strand breaks
  int32_t* own;   // our cell
  int32_t* slot;  // slot of the event within its boundary's exchange buffer
  int32_t* counts;  // {events below, events above, total, dropped (beyond E)}
};

constexpr int kXbThreads = 1024;

// One workgroup: draws of both boundaries, the first E events of each in item order, and a copy of
// our genome of every event into the boundary's outgoing slots ([int32 length | slot_w bytes]).
__global__ void __launch_bounds__(kXbThreads) xb_events_kernel(int C, int E, int slot_w, double p, int kcap,
                                                               uint64_t seed_dn, uint64_t seed_up, uint64_t call,
                                                               const int32_t* mine_dn, const int32_t* from_dn,
                                                               const int32_t* mine_up, const int32_t* from_up,
                                                               const int32_t* own1, const int32_t* ownH,
                                                               const uint8_t* arena, const int64_t* off, XbEvents ev,
                                                               uint8_t* slots_dn, uint8_t* slots_up) {
  constexpr int W = kXbThreads / 64;
  __shared__ int s_wc[W];
  __shared__ int s_base;
  __shared__ int s_cnt[2], s_tot[2];
  const int tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
  if (tid == 0) s_base = 0;
  for (int b = 0; b < 2; ++b) {
    // b = 0: we hold the upper cells (row H, lengths mine_dn), the lower rank the lower ones (from_dn)
    const int32_t* la_row = b == 0 ? mine_dn : from_up;
    const int32_t* lb_row = b == 0 ? from_dn : mine_up;
    const int wx = min(slot_w, min(mine_dn[C], b == 0 ? from_dn[C] : from_up[C]));
    const uint64_t seed = b == 0 ? seed_dn : seed_up;
    int found = 0;  // events of this boundary so far (uniform across the block)
    __syncthreads();
    const int base0 = s_base;
    for (int c0 = 0; c0 < 3 * C; c0 += kXbThreads) {
      const int i = c0 + tid;
      int kk = 0, own = -1;
      if (i < 3 * C) {
        const int y = i / 3, d = i - 3 * y - 1;
        const bool ok_d = d == 0 || (d == -1 && C >= 2) || (d == 1 && C >= 3);
        const int yb = (y + d + C) % C;
        const int la = la_row[y], lb = lb_row[yb];
        if (ok_d && la >= 0 && lb >= 0 && la <= wx && lb <= wx && la + lb > 0) {
          Philox rng(seed, call, (uint32_t)i);
          long long q = poisson(rng, p * (double)(la + lb));
          if (kcap > 0 && q > kcap) q = kcap;
          kk = (int)(q > la + lb ? la + lb : q);
          own = b == 0 ? ownH[y] : own1[yb];
        }
      }
      const uint64_t bal = __ballot(kk > 0);
      if (lane == 0) s_wc[w] = __popcll(bal);
      __syncthreads();
      int pre = 0, tot = 0;
      for (int q = 0; q < W; ++q) {
        if (q < w) pre += s_wc[q];
        tot += s_wc[q];
      }
      if (kk > 0) {
        const int jb = found + pre + __popcll(bal & lt);
        if (jb < E) {
          const int j = base0 + jb;
          ev.b[j] = b;
          ev.item[j] = i;
          ev.k[j] = kk;
          ev.own[j] = own;
          ev.slot[j] = jb;
        }
      }
      found += tot;
      __syncthreads();
    }
    if (tid == 0) {
      s_cnt[b] = min(found, E);
      s_tot[b] = found;
      s_base = base0 + min(found, E);
    }
  }
  __syncthreads();
  if (tid == 0) {
    ev.counts[0] = s_cnt[0];
    ev.counts[1] = s_cnt[1];
    ev.counts[2] = s_cnt[0] + s_cnt[1];
    ev.counts[3] += (s_tot[0] - s_cnt[0]) + (s_tot[1] - s_cnt[1]);
  }
  // our genome of each event into its slot (the pre-recombination copy both ranks work from)
  const int total = s_cnt[0] + s_cnt[1];
  for (int j = 0; j < total; ++j) {
    const int b = ev.b[j], jb = ev.slot[j], c = ev.own[j];
    uint8_t* slot = (b == 0 ? slots_dn : slots_up) + (size_t)jb * (4 + slot_w);
    const int32_t* lrow = b == 0 ? mine_dn : mine_up;
    const int item = ev.item[j];
    const int y = item / 3, d = item - 3 * y - 1;
    const int L = b == 0 ? lrow[y] : lrow[(y + d + C) % C];
    if (tid == 0) *reinterpret_cast<int32_t*>(slot) = L;
    const uint8_t* g = arena + off[c];
    for (int t = tid; t < L; t += kXbThreads) slot[4 + t] = g[t];
  }
}

// One wavefront per event: the recombination of (upper genome, lower genome) exactly as both ranks
// compute it; our cell's result goes to out row `base + j` (base = 2 * *pair_count when appending
// after the local pipeline's results, else 0) with its row; the other result to scratch.
// *nres = base + total (rows to commit).
__global__ void __launch_bounds__(64) xb_apply_kernel(int C, int slot_w, uint64_t seed_dn, uint64_t seed_up,
                                                      uint64_t call, XbEvents ev, const uint8_t* slots_dn,
                                                      const uint8_t* slots_up, const uint8_t* recv_dn,
                                                      const uint8_t* recv_up, int32_t* parts, int parts_cap,
                                                      const int* pair_count, uint8_t* out, int out_width,
                                                      int32_t* out_len, int64_t* out_rows, uint8_t* other,
                                                      int* nres) {
  __shared__ int32_t lparts[(kFloydMax + 2) * 3];
  __shared__ int meta[2];
  const int j = blockIdx.x, lane = threadIdx.x;
  const int total = ev.counts[2];
  const int base = pair_count ? 2 * *pair_count : 0;
  if (j == 0 && lane == 0) *nres = base + total;
  if (j >= total) return;
  const int b = ev.b[j], jb = ev.slot[j];
  const size_t so = (size_t)jb * (4 + slot_w);
  // b = 0: our cell is the upper one (its copy in slots_dn), the lower one arrived in recv_dn
  const uint8_t* ua = b == 0 ? slots_dn + so : recv_up + so;
  const uint8_t* lb = b == 0 ? recv_dn + so : slots_up + so;
  // (lengths clamped to the slot: a corrupted exchange must not send the pair past its buffers)
  const int n0 = min(max(*reinterpret_cast<const int32_t*>(ua), 0), slot_w);
  const int n1 = min(max(*reinterpret_cast<const int32_t*>(lb), 0), slot_w);
  uint8_t* mine = out + (size_t)(base + j) * out_width;
  uint8_t* theirs = other + (size_t)j * out_width;
  int w0, w1;
  rec_pair_apply(ua + 4, n0, lb + 4, n1, ev.k[j], b == 0 ? seed_dn : seed_up, call, (uint32_t)ev.item[j],
                 parts + (size_t)j * parts_cap * 3, lparts, meta, b == 0 ? mine : theirs, b == 0 ? theirs : mine,
                 out_width, w0, w1);
  if (lane == 0) {
    const int wm = b == 0 ? w0 : w1;
    out_len[base + j] = wm < out_width ? wm : out_width;
    out_rows[base + j] = ev.own[j];
  }
}

// ---------------------------------------------------------------- host launchers
namespace {
RecCols rec_cols(uintptr_t mols, uintptr_t pos, uintptr_t life, uintptr_t div, const GenomePoolArgs& g, uintptr_t glen,
                 int gw, uintptr_t ldata, uintptr_t llen, int lw, int m) {
  if (gw % 4 || lw % 4) throw std::invalid_argument("records: row widths must be multiples of 4");
  return RecCols{P_<float>(mols), P_<int32_t>(pos), P_<int32_t>(life), P_<int32_t>(div), P_<uint8_t>(g.pool),
                 P_<int64_t>(g.off), P_<unsigned long long>(g.top), g.cap, g.failed ? P_<int>(g.failed) : nullptr,
                 P_<int32_t>(glen), gw, P_<uint8_t>(ldata), P_<int32_t>(llen), lw, m};
}
int32_t* g_split_tiles = nullptr;
long long g_split_cap = 0;
int g_split_single = 1;  // place_split as one single-pass launch (0: count + write, A/B)
}  // namespace

void strip_marks(int C, int H, uintptr_t cell_map, int k, uintptr_t cells, uintptr_t mask, uintptr_t pos, uintptr_t up,
                 uintptr_t dn, uintptr_t stream) {
  if (H < 2 || C < 1) throw std::invalid_argument("strip_marks: bad strip");
  if (!cells && !mask && k > 0) throw std::invalid_argument("strip_marks: give cells or a mask");
  msd::kl(strip_occ_kernel, cdiv(C, 256), 256, 0, S_(stream))(C, H, P_<uint8_t>(cell_map), P_<uint8_t>(up), P_<uint8_t>(dn));
  MS_LAUNCH_CHECK();
  if (k > 0) {
    msd::kl(strip_div_kernel, cdiv(k, 256), 256, 0, S_(stream))(k, cells ? P_<int64_t>(cells) : nullptr,
                                                            mask ? P_<uint8_t>(mask) : nullptr, P_<int32_t>(pos), C,
                                                            H, P_<uint8_t>(up), P_<uint8_t>(dn));
    MS_LAUNCH_CHECK();
  }
}

void strip_reserve(int C, int H, uintptr_t from_up, uintptr_t from_dn, uintptr_t cell_map, uintptr_t stream) {
  msd::kl(strip_reserve_kernel, cdiv(C, 256), 256, 0, S_(stream))(C, H, P_<uint8_t>(from_up), P_<uint8_t>(from_dn),
                                                              P_<uint8_t>(cell_map));
  MS_LAUNCH_CHECK();
}

void strip_clear(int C, int H, uintptr_t cell_map, uintptr_t stream) {
  msd::kl(strip_clear_kernel, cdiv(C, 256), 256, 0, S_(stream))(C, H, P_<uint8_t>(cell_map));
  MS_LAUNCH_CHECK();
}

// par: int64[3 k], npos: int32[3 k * 2], counts: int32[3]; hdr_up / hdr_dn: {count, lw, gw, m}.
// k == 0 still runs one (empty) tile so that the counts and headers are written.
void place_split(int k, uintptr_t result, uintptr_t cells, int C, int H, uintptr_t par, uintptr_t npos, uintptr_t counts,
                 uintptr_t hdr_up, uintptr_t hdr_dn, int lw, int gw, int m, uintptr_t stream) {
  hipStream_t s = S_(stream);
  if (k < 0) throw std::invalid_argument("place_split: negative count");
  const long long tiles = std::max(1ll, ((long long)k + kSplitTile - 1) / kSplitTile);
  if (g_split_single && tiles <= kLbMaxTiles) {  // one launch (the status words of select_lb.h)
    const LbState lb = lb_begin(s);
    msd::kl(place_split_lb_kernel, (unsigned)tiles, kSplitThreads, 0, s)(
        k, P_<long long>(result), cells ? P_<int64_t>(cells) : nullptr, C, H, lb.status, lb.gen, lb.err,
        P_<int64_t>(par), P_<int32_t>(npos), P_<int32_t>(counts), P_<int32_t>(hdr_up), P_<int32_t>(hdr_dn), lw, gw, m);
    MS_LAUNCH_CHECK();
    return;
  }
  if (tiles > g_split_cap) {
    if (g_split_tiles) {
      MS_HIP_CHECK(msd::stream_synchronize(s));
      MS_HIP_CHECK(msd::dev_free(g_split_tiles));
    }
    g_split_cap = std::max(tiles, 64ll);
    MS_HIP_CHECK(msd::dev_malloc((void**)&g_split_tiles, 3 * g_split_cap * sizeof(int32_t)));
  }
  msd::kl(place_split_count_kernel, (unsigned)tiles, kSplitThreads, 0, s)(k, P_<long long>(result), C, H, g_split_tiles);
  MS_LAUNCH_CHECK();
  msd::kl(place_split_write_kernel, (unsigned)tiles, kSplitThreads, 0, s)(
      k, P_<long long>(result), cells ? P_<int64_t>(cells) : nullptr, C, H, g_split_tiles, P_<int64_t>(par),
      P_<int32_t>(npos),
      P_<int32_t>(counts), P_<int32_t>(hdr_up), P_<int32_t>(hdr_dn), lw, gw, m);
  MS_LAUNCH_CHECK();
}

long long rec_record_bytes(int m, int lw, int gw) { return rec_bytes(m, lw, gw); }

void set_split_single(int on) { g_split_single = on; }

void rec_pack(int k_up, int k_dn, uintptr_t par_up, uintptr_t pos_up, uintptr_t par_dn, uintptr_t pos_dn,
              uintptr_t mols, uintptr_t pos, uintptr_t life, uintptr_t div, const GenomePoolArgs& gp, uintptr_t glen,
              int gw, uintptr_t ldata, uintptr_t llen, int lw, int m, bool child, uintptr_t out_up, uintptr_t out_dn,
              uintptr_t stream) {
  if (k_up + k_dn <= 0) return;
  const RecCols w = rec_cols(mols, pos, life, div, gp, glen, gw, ldata, llen, lw, m);
  msd::kl(rec_pack_kernel, k_up + k_dn, 64, 0, S_(stream))(k_up, k_dn, P_<int64_t>(par_up), P_<int32_t>(pos_up),
                                                      P_<int64_t>(par_dn), P_<int32_t>(pos_dn), w, child,
                                                      P_<uint8_t>(out_up), P_<uint8_t>(out_dn));
  MS_LAUNCH_CHECK();
}

void rec_unpack(int n0, int k_up, uintptr_t in_up, int up_lw, int up_gw, int k_dn, uintptr_t in_dn, int dn_lw,
                int dn_gw, int C, int H, uintptr_t mols, uintptr_t pos, uintptr_t life, uintptr_t div,
                const GenomePoolArgs& gp, uintptr_t glen, int gw, uintptr_t ldata, uintptr_t llen, int lw, int m,
                uintptr_t cell_map, uintptr_t stream) {
  if (k_up + k_dn <= 0) return;
  if (up_lw % 4 || up_gw % 4 || dn_lw % 4 || dn_gw % 4) throw std::invalid_argument("rec_unpack: bad sender widths");
  const RecCols w = rec_cols(mols, pos, life, div, gp, glen, gw, ldata, llen, lw, m);
  msd::kl(rec_unpack_kernel, k_up + k_dn, 64, 0, S_(stream))(n0, k_up, P_<uint8_t>(in_up), up_lw, up_gw, k_dn,
                                                        P_<uint8_t>(in_dn), dn_lw, dn_gw, C, H, w,
                                                        P_<uint8_t>(cell_map));
  MS_LAUNCH_CHECK();
}

void halo_pack(int m, int C, int H, int elem, uintptr_t map, uintptr_t send_up, uintptr_t send_dn, uintptr_t stream) {
  const unsigned g = cdiv((long long)m * C, 256);
  if (elem == 4)
    msd::kl(halo_pack_kernel<uint32_t>, g, 256, 0, S_(stream))(m, C, H, P_<uint32_t>(map), P_<uint32_t>(send_up),
                                                          P_<uint32_t>(send_dn));
  else if (elem == 2)
    msd::kl(halo_pack_kernel<uint16_t>, g, 256, 0, S_(stream))(m, C, H, P_<uint16_t>(map), P_<uint16_t>(send_up),
                                                          P_<uint16_t>(send_dn));
  else
    throw std::invalid_argument("halo_pack: element size must be 2 or 4");
  MS_LAUNCH_CHECK();
}

void halo_unpack(int m, int C, int H, int elem, uintptr_t map, uintptr_t from_up, uintptr_t from_dn, uintptr_t stream) {
  const unsigned g = cdiv((long long)m * C, 256);
  if (elem == 4)
    msd::kl(halo_unpack_kernel<uint32_t>, g, 256, 0, S_(stream))(m, C, H, P_<uint32_t>(map), P_<uint32_t>(from_up),
                                                            P_<uint32_t>(from_dn));
  else if (elem == 2)
    msd::kl(halo_unpack_kernel<uint16_t>, g, 256, 0, S_(stream))(m, C, H, P_<uint16_t>(map), P_<uint16_t>(from_up),
                                                            P_<uint16_t>(from_dn));
  else
    throw std::invalid_argument("halo_unpack: element size must be 2 or 4");
  MS_LAUNCH_CHECK();
}


XbEvents xb_ev(uintptr_t evbuf, int E2) {
  int32_t* e = P_<int32_t>(evbuf);
  return XbEvents{e, e + E2, e + 2 * E2, e + 3 * E2, e + 4 * E2, e + 5 * E2};
}

// evbuf: int32[5 * 2E + 4] (event fields, then counts; counts[3] accumulates dropped events)
void xb_prep(int C, int H, int n, uintptr_t pos, uintptr_t idx_map, uintptr_t lens, int width, uintptr_t len_up,
             uintptr_t len_dn, uintptr_t own1, uintptr_t ownH, uintptr_t stream) {
  msd::kl(xb_prep_kernel, cdiv(C, 256), 256, 0, S_(stream))(C, H, n, P_<int32_t>(pos), P_<int32_t>(idx_map),
                                                        P_<int32_t>(lens), width, P_<int32_t>(len_up),
                                                        P_<int32_t>(len_dn), P_<int32_t>(own1), P_<int32_t>(ownH));
  MS_LAUNCH_CHECK();
}

void xb_events(int C, int E, int slot_w, double p, int kcap, uint64_t seed_dn, uint64_t seed_up, uint64_t call,
               uintptr_t mine_dn, uintptr_t from_dn, uintptr_t mine_up, uintptr_t from_up, uintptr_t own1,
               uintptr_t ownH, uintptr_t arena, uintptr_t off, uintptr_t evbuf, uintptr_t slots_dn, uintptr_t slots_up,
               uintptr_t stream) {
  if (E < 1 || slot_w < 4 || slot_w % 4) throw std::invalid_argument("xb_events: bad capacity / slot width");
  msd::kl(xb_events_kernel, 1, kXbThreads, 0, S_(stream))(C, E, slot_w, p, kcap, seed_dn, seed_up, call,
                                                     P_<int32_t>(mine_dn), P_<int32_t>(from_dn), P_<int32_t>(mine_up),
                                                     P_<int32_t>(from_up), P_<int32_t>(own1), P_<int32_t>(ownH),
                                                     P_<uint8_t>(arena), P_<int64_t>(off), xb_ev(evbuf, 2 * E),
                                                     P_<uint8_t>(slots_dn), P_<uint8_t>(slots_up));
  MS_LAUNCH_CHECK();
}

void xb_apply(int C, int E, int slot_w, uint64_t seed_dn, uint64_t seed_up, uint64_t call, uintptr_t evbuf,
              uintptr_t slots_dn, uintptr_t slots_up, uintptr_t recv_dn, uintptr_t recv_up, uintptr_t parts,
              int parts_cap, uintptr_t pair_count, uintptr_t out, int out_width, uintptr_t out_len,
              uintptr_t out_rows, uintptr_t other, uintptr_t nres, uintptr_t stream) {
  msd::kl(xb_apply_kernel, 2 * E, 64, 0, S_(stream))(C, slot_w, seed_dn, seed_up, call, xb_ev(evbuf, 2 * E),
                                                P_<uint8_t>(slots_dn), P_<uint8_t>(slots_up), P_<uint8_t>(recv_dn),
                                                P_<uint8_t>(recv_up), P_<int32_t>(parts), parts_cap,
                                                pair_count ? P_<int>(pair_count) : nullptr, P_<uint8_t>(out),
                                                out_width, P_<int32_t>(out_len), P_<int64_t>(out_rows),
                                                P_<uint8_t>(other), P_<int>(nres));
  MS_LAUNCH_CHECK();
}

void release_dist_buffers() {
  if (g_split_tiles) MS_HIP_CHECK(msd::dev_free(g_split_tiles));
  g_split_tiles = nullptr;
  g_split_cap = 0;
}

void index_map(int c, uintptr_t pos, int C, uintptr_t idx_map, bool clear, uintptr_t stream);
void rccl_exchange(uintptr_t comm, int up, int down, uintptr_t send_up, long long n_send_up, uintptr_t send_down,
                   long long n_send_down, uintptr_t recv_down, long long n_recv_down, uintptr_t recv_up,
                   long long n_recv_up, uintptr_t stream);

// The collective part of the strip-boundary recombination (parallel/dist_world.py
// _BoundaryRecombination) in one call over the native RCCL communicator `comm`: the index map, the
// boundary rows' genome lengths exchanged, the events drawn and the event genomes exchanged.
// lens: int32 4 (C + 1) = mine up | mine down | from down | from up; own: int32 2 C; slots: 4 E
// (4 + slot_w) bytes = to down | to up | from down | from up.
void xb_begin(int C, int H, int n, uintptr_t pos, uintptr_t idx_map, uintptr_t glens, uintptr_t gdata, uintptr_t goff,
              int width,
              uintptr_t lens, uintptr_t own, int E, int slot_w, double p, int kcap, uint64_t seed_dn, uint64_t seed_up,
              uint64_t call, uintptr_t evbuf, uintptr_t slots, uintptr_t comm, int up, int down, uintptr_t stream) {
  const size_t lb = 4ull * (C + 1);
  const uintptr_t mine_up = lens, mine_dn = lens + lb, from_dn = lens + 2 * lb, from_up = lens + 3 * lb;
  index_map(n, pos, C, idx_map, false, stream);
  xb_prep(C, H, n, pos, idx_map, glens, width, mine_up, mine_dn, own, own + 4ull * C, stream);
  rccl_exchange(comm, up, down, mine_up, lb, mine_dn, lb, from_dn, lb, from_up, lb, stream);
  const size_t sb = (size_t)E * (4 + slot_w);  // a slot: 4 header bytes + slot_w genome bytes
  const uintptr_t slots_dn = slots, slots_up = slots + sb, recv_dn = slots + 2 * sb, recv_up = slots + 3 * sb;
  xb_events(C, E, slot_w, p, kcap, seed_dn, seed_up, call, mine_dn, from_dn, mine_up, from_up, own, own + 4ull * C,
            gdata, goff, evbuf, slots_dn, slots_up, stream);
  rccl_exchange(comm, up, down, slots_up, sb, slots_dn, sb, recv_dn, sb, recv_up, sb, stream);
}

}  // namespace msd
