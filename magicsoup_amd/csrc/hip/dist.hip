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

namespace msd {

// ---------------------------------------------------------------- division: boundary marks
// marks[y] of the owned boundary rows: 1 = occupied, 3 = occupied by a dividing cell
__global__ void __launch_bounds__(256) strip_occ_kernel(int C, int H, const uint8_t* cell_map, uint8_t* up, uint8_t* dn) {
  const int y = blockIdx.x * blockDim.x + threadIdx.x;
  if (y >= C) return;
  up[y] = cell_map[(size_t)1 * C + y] ? 1 : 0;
  dn[y] = cell_map[(size_t)H * C + y] ? 1 : 0;
}

__global__ void __launch_bounds__(256) strip_div_kernel(int k, const int64_t* cells, const int32_t* pos, int C, int H,
                                                        uint8_t* up, uint8_t* dn) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= k) return;
  const int64_t c = cells[i];
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
      par[o] = cells[i];
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

// ---------------------------------------------------------------- cell records
// Record layout (4-byte words): y, genome length, label length, divisions, lifetime, m molecules,
// then the label row (lw bytes) and the genome row (gw bytes); lw, gw are multiples of 4.
struct RecCols {
  float* mols;
  int32_t* pos;
  int32_t* life;
  int32_t* div;
  uint8_t* gdata;
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
  const uint32_t* gs = reinterpret_cast<const uint32_t*>(w.gdata + (size_t)c * w.gw);
  uint32_t* gd = reinterpret_cast<uint32_t*>(r + 4 * (5 + w.m) + w.lw);
  for (int q = lane; q < w.gw / 4; q += 64) gd[q] = gs[q];
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
  for (int q = lane; q < w.gw; q += 64) w.gdata[c * w.gw + q] = q < gl ? gs[q] : 0;
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

// ---------------------------------------------------------------- host launchers
namespace {
RecCols rec_cols(uintptr_t mols, uintptr_t pos, uintptr_t life, uintptr_t div, uintptr_t gdata, uintptr_t glen, int gw,
                 uintptr_t ldata, uintptr_t llen, int lw, int m) {
  if (gw % 4 || lw % 4) throw std::invalid_argument("records: row widths must be multiples of 4");
  return RecCols{P_<float>(mols), P_<int32_t>(pos), P_<int32_t>(life), P_<int32_t>(div), P_<uint8_t>(gdata),
                 P_<int32_t>(glen), gw, P_<uint8_t>(ldata), P_<int32_t>(llen), lw, m};
}
int32_t* g_split_tiles = nullptr;
long long g_split_cap = 0;
}  // namespace

void strip_marks(int C, int H, uintptr_t cell_map, int k, uintptr_t cells, uintptr_t pos, uintptr_t up, uintptr_t dn,
                 uintptr_t stream) {
  if (H < 2 || C < 1) throw std::invalid_argument("strip_marks: bad strip");
  strip_occ_kernel<<<cdiv(C, 256), 256, 0, S_(stream)>>>(C, H, P_<uint8_t>(cell_map), P_<uint8_t>(up), P_<uint8_t>(dn));
  MS_LAUNCH_CHECK();
  if (k > 0) {
    strip_div_kernel<<<cdiv(k, 256), 256, 0, S_(stream)>>>(k, P_<int64_t>(cells), P_<int32_t>(pos), C, H,
                                                            P_<uint8_t>(up), P_<uint8_t>(dn));
    MS_LAUNCH_CHECK();
  }
}

void strip_reserve(int C, int H, uintptr_t from_up, uintptr_t from_dn, uintptr_t cell_map, uintptr_t stream) {
  strip_reserve_kernel<<<cdiv(C, 256), 256, 0, S_(stream)>>>(C, H, P_<uint8_t>(from_up), P_<uint8_t>(from_dn),
                                                              P_<uint8_t>(cell_map));
  MS_LAUNCH_CHECK();
}

void strip_clear(int C, int H, uintptr_t cell_map, uintptr_t stream) {
  strip_clear_kernel<<<cdiv(C, 256), 256, 0, S_(stream)>>>(C, H, P_<uint8_t>(cell_map));
  MS_LAUNCH_CHECK();
}

// par: int64[3 k], npos: int32[3 k * 2], counts: int32[3]; hdr_up / hdr_dn: {count, lw, gw, m}.
// k == 0 still runs one (empty) tile so that the counts and headers are written.
void place_split(int k, uintptr_t result, uintptr_t cells, int C, int H, uintptr_t par, uintptr_t npos, uintptr_t counts,
                 uintptr_t hdr_up, uintptr_t hdr_dn, int lw, int gw, int m, uintptr_t stream) {
  hipStream_t s = S_(stream);
  if (k < 0) throw std::invalid_argument("place_split: negative count");
  const long long tiles = std::max(1ll, ((long long)k + kSplitTile - 1) / kSplitTile);
  if (tiles > g_split_cap) {
    if (g_split_tiles) {
      MS_HIP_CHECK(hipStreamSynchronize(s));
      MS_HIP_CHECK(hipFree(g_split_tiles));
    }
    g_split_cap = std::max(tiles, 64ll);
    MS_HIP_CHECK(hipMalloc((void**)&g_split_tiles, 3 * g_split_cap * sizeof(int32_t)));
  }
  place_split_count_kernel<<<(unsigned)tiles, kSplitThreads, 0, s>>>(k, P_<long long>(result), C, H, g_split_tiles);
  MS_LAUNCH_CHECK();
  place_split_write_kernel<<<(unsigned)tiles, kSplitThreads, 0, s>>>(
      k, P_<long long>(result), P_<int64_t>(cells), C, H, g_split_tiles, P_<int64_t>(par), P_<int32_t>(npos),
      P_<int32_t>(counts), P_<int32_t>(hdr_up), P_<int32_t>(hdr_dn), lw, gw, m);
  MS_LAUNCH_CHECK();
}

long long rec_record_bytes(int m, int lw, int gw) { return rec_bytes(m, lw, gw); }

void rec_pack(int k_up, int k_dn, uintptr_t par_up, uintptr_t pos_up, uintptr_t par_dn, uintptr_t pos_dn,
              uintptr_t mols, uintptr_t pos, uintptr_t life, uintptr_t div, uintptr_t gdata, uintptr_t glen, int gw,
              uintptr_t ldata, uintptr_t llen, int lw, int m, bool child, uintptr_t out_up, uintptr_t out_dn,
              uintptr_t stream) {
  if (k_up + k_dn <= 0) return;
  const RecCols w = rec_cols(mols, pos, life, div, gdata, glen, gw, ldata, llen, lw, m);
  rec_pack_kernel<<<k_up + k_dn, 64, 0, S_(stream)>>>(k_up, k_dn, P_<int64_t>(par_up), P_<int32_t>(pos_up),
                                                      P_<int64_t>(par_dn), P_<int32_t>(pos_dn), w, child,
                                                      P_<uint8_t>(out_up), P_<uint8_t>(out_dn));
  MS_LAUNCH_CHECK();
}

void rec_unpack(int n0, int k_up, uintptr_t in_up, int up_lw, int up_gw, int k_dn, uintptr_t in_dn, int dn_lw,
                int dn_gw, int C, int H, uintptr_t mols, uintptr_t pos, uintptr_t life, uintptr_t div, uintptr_t gdata,
                uintptr_t glen, int gw, uintptr_t ldata, uintptr_t llen, int lw, int m, uintptr_t cell_map,
                uintptr_t stream) {
  if (k_up + k_dn <= 0) return;
  if (up_lw % 4 || up_gw % 4 || dn_lw % 4 || dn_gw % 4) throw std::invalid_argument("rec_unpack: bad sender widths");
  const RecCols w = rec_cols(mols, pos, life, div, gdata, glen, gw, ldata, llen, lw, m);
  rec_unpack_kernel<<<k_up + k_dn, 64, 0, S_(stream)>>>(n0, k_up, P_<uint8_t>(in_up), up_lw, up_gw, k_dn,
                                                        P_<uint8_t>(in_dn), dn_lw, dn_gw, C, H, w,
                                                        P_<uint8_t>(cell_map));
  MS_LAUNCH_CHECK();
}

void halo_pack(int m, int C, int H, int elem, uintptr_t map, uintptr_t send_up, uintptr_t send_dn, uintptr_t stream) {
  const unsigned g = cdiv((long long)m * C, 256);
  if (elem == 4)
    halo_pack_kernel<uint32_t><<<g, 256, 0, S_(stream)>>>(m, C, H, P_<uint32_t>(map), P_<uint32_t>(send_up),
                                                          P_<uint32_t>(send_dn));
  else if (elem == 2)
    halo_pack_kernel<uint16_t><<<g, 256, 0, S_(stream)>>>(m, C, H, P_<uint16_t>(map), P_<uint16_t>(send_up),
                                                          P_<uint16_t>(send_dn));
  else
    throw std::invalid_argument("halo_pack: element size must be 2 or 4");
  MS_LAUNCH_CHECK();
}

void halo_unpack(int m, int C, int H, int elem, uintptr_t map, uintptr_t from_up, uintptr_t from_dn, uintptr_t stream) {
  const unsigned g = cdiv((long long)m * C, 256);
  if (elem == 4)
    halo_unpack_kernel<uint32_t><<<g, 256, 0, S_(stream)>>>(m, C, H, P_<uint32_t>(map), P_<uint32_t>(from_up),
                                                            P_<uint32_t>(from_dn));
  else if (elem == 2)
    halo_unpack_kernel<uint16_t><<<g, 256, 0, S_(stream)>>>(m, C, H, P_<uint16_t>(map), P_<uint16_t>(from_up),
                                                            P_<uint16_t>(from_dn));
  else
    throw std::invalid_argument("halo_unpack: element size must be 2 or 4");
  MS_LAUNCH_CHECK();
}

}  // namespace msd
