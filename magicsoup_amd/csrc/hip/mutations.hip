// gfx950 point mutations and recombinations on the device genome arena
// (semantics of rust/mutations.rs:11-154).
//
// Both are two-phase: a cheap per-item Poisson draw over all genomes / neighbour pairs, then an
// apply kernel for the (usually few) items that drew at least one event. An apply kernel runs one
// wavefront per item: one lane draws the k event positions (Floyd's sorted sampling) into an LDS
// plan, then all 64 lanes stream the new sequence into a scratch row; arena_scatter commits the rows
// into fresh space of the genome pool.
#include <algorithm>

#include "hip_common.h"
#include "rec_common.h"

namespace msd {

__device__ __forceinline__ uint8_t rand_nt(Philox& rng) {
  const char nts[4] = {'A', 'C', 'T', 'G'};
  return (uint8_t)nts[rng.below(4)];
}

// k[i] ~ Poisson(p * len(row_i))
// Device pipelines (magicsoup_amd/ops/genome_pipeline.py): an op whose predecessor in the same
// pending chain could not commit a genome (arena too narrow) does nothing and is replayed by the
// host later, so the chain never works on a stale genome.
constexpr int kGpWidth = 8, kGpSkipped = 16;
__device__ __forceinline__ bool gp_skip(int i, const int* gflags, int* opflags) {
  if (!gflags || !(*gflags & kGpWidth)) return false;
  if (i == 0) atomicOr(opflags, kGpSkipped);
  return true;
}

__global__ void __launch_bounds__(256) mut_count_kernel(int n, const int64_t* rows, const int32_t* lens, double p,
                                                        uint64_t seed, uint64_t call, int32_t* k, int kcap,
                                                        const int* gflags, int* opflags) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (gp_skip(i, gflags, opflags)) {
    k[i] = 0;
    return;
  }
  const int64_t r = rows ? rows[i] : i;
  const int L = lens[r];
  if (L < 1) {
    k[i] = 0;
    return;
  }
  Philox rng(seed, call, (uint32_t)i);
  long long kk = poisson(rng, p * (double)L);
  if (kcap > 0 && kk > kcap) kk = kcap;
  k[i] = (int32_t)(kk > L ? L : kk);
}

// mut_count_kernel over all n genomes (rows = identity) that also writes each block's number of
// genomes with events into tile_count[block] (tile_max[block] = 0): the counts of the order-preserving
// selection that follows (select.hip select_write_i32pos_capped with 16 blocks per 4096-item tile),
// so the chain needs no separate count pass over k. The grid covers whole selection tiles; blocks
// past n write zero counts.
__global__ void __launch_bounds__(256) mut_count_tiles_kernel(int n, const int32_t* lens, double p, uint64_t seed,
                                                              uint64_t call, int32_t* k, int kcap, const int* gflags,
                                                              int* opflags, int32_t* tile_count, int32_t* tile_max) {
  __shared__ int s_cnt[4];
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  int kk = 0;
  if (i < n) {
    if (!gp_skip(i, gflags, opflags)) {
      const int L = lens[i];
      if (L >= 1) {
        Philox rng(seed, call, (uint32_t)i);
        long long d = poisson(rng, p * (double)L);
        if (kcap > 0 && d > kcap) d = kcap;
        kk = (int)(d > L ? L : d);
      }
    }
    k[i] = kk;
  }
  const int c = __popcll(__ballot(kk > 0));
  if ((threadIdx.x & 63) == 0) s_cnt[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    tile_count[blockIdx.x] = (s_cnt[0] + s_cnt[1]) + (s_cnt[2] + s_cnt[3]);
    tile_max[blockIdx.x] = 0;
  }
}

// mut_count_tiles_kernel's draws with the cells that mutate appended (one atomic each, ~n p L of the
// n cells) instead of a count array and a selection pass; world.hip sel_sort puts them in cell order.
__global__ void __launch_bounds__(256) mut_draw_kernel(int n, const int32_t* lens, double p, uint64_t seed,
                                                       uint64_t call, int32_t* k, int kcap, const int* gflags,
                                                       int* opflags, int64_t* cand, int* cand_count, int cap,
                                                       const int* na, const int* nb) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (na) n = min(n, *na + *nb);  // (a chain issued on a device cell count, world.hip dev_count)
  if (i >= n || gp_skip(i, gflags, opflags)) return;
  const int L = lens[i];
  if (L < 1) return;
  Philox rng(seed, call, (uint32_t)i);
  long long d = poisson(rng, p * (double)L);
  if (kcap > 0 && d > kcap) d = kcap;
  const int kk = (int)(d > L ? L : d);
  if (kk <= 0) return;
  k[i] = kk;
  const int j = atomicAdd(cand_count, 1);
  if (j < cap) cand[j] = i;
}

// One mutation event at nucleotide `ch`: the 0..2 nucleotides it emits (reference
// rust/mutations.rs:30-60: indel with p_indel, then deletion with p_del, else insertion before ch;
// otherwise a substitution that may repeat the old nucleotide).
__device__ __forceinline__ int mutate_at(Philox& rng, uint8_t ch, double p_indel, double p_del, uint8_t* lit) {
  if (rng.uniform_d() < p_indel) {
    if (rng.uniform_d() < p_del) return 0;  // deletion
    lit[0] = rand_nt(rng);                  // insertion before the current nucleotide
    lit[1] = ch;
    return 2;
  }
  lit[0] = rand_nt(rng);  // substitution
  return 1;
}

// One wavefront per selected genome: lane 0 draws the event positions and the emitted literals into
// an LDS plan (copy segment, literal, copy segment, ...); all lanes then stream the segments.
// Genomes with more than kFloydMax events (very high rates) take a serial selection-sampling path.
__device__ __forceinline__ void mut_apply_item(int j, const int64_t* sel, const int64_t* rows, const uint8_t* arena,
                                               const int64_t* off, const int32_t* lens, const int32_t* k, double p_indel,
                                               double p_del, uint64_t seed, uint64_t call, uint8_t* out, int out_width,
                                               int32_t* out_len, int* pos, uint8_t (*lit)[2], int* nlit) {
  const int lane = threadIdx.x;
  const int64_t i = sel[j];
  const int64_t r = rows ? rows[i] : i;
  const uint8_t* s = arena + off[r];
  const int L = lens[r];
  const int kk = k[i];
  uint8_t* o = out + (size_t)j * out_width;
  if (kk > kFloydMax) {
    if (lane == 0) {
      Philox rng(seed, call ^ kApplyStream, (uint32_t)i);
      int need = kk, w = 0;
      uint8_t l2[2];
      for (int t = 0; t < L; ++t) {
        // selection sampling: position t is chosen with chance need / (L - t)
        if (need > 0 && rng.below((uint32_t)(L - t)) < (uint32_t)need) {
          --need;
          const int nl = mutate_at(rng, s[t], p_indel, p_del, l2);
          for (int q = 0; q < nl; ++q)
            if (w < out_width) o[w++] = l2[q];
        } else if (w < out_width) {
          o[w++] = s[t];
        }
      }
      out_len[j] = w;
    }
    return;
  }
  if (lane == 0) {
    Philox rng(seed, call ^ kApplyStream, (uint32_t)i);
    floyd_sorted(rng, L, kk, pos);
    for (int q = 0; q < kk; ++q) nlit[q] = mutate_at(rng, s[pos[q]], p_indel, p_del, lit[q]);
  }
  __syncthreads();
  int prev = 0, w = 0;
  for (int q = 0; q < kk; ++q) {
    wave_copy(s, prev, pos[q], o, w, out_width, lane);
    w += pos[q] - prev;
    if (lane < nlit[q] && w + lane < out_width) o[w + lane] = lit[q][lane];
    w += nlit[q];
    prev = pos[q] + 1;
  }
  wave_copy(s, prev, L, o, w, out_width, lane);
  w += L - prev;
  if (lane == 0) out_len[j] = w < out_width ? w : out_width;
}

// dn: optional device-side item count (<= nsel): the grid strides over the items, so the host does
// not need to know how many genomes were selected.
__global__ void __launch_bounds__(64) mut_apply_kernel(int nsel, const int* dn, const int64_t* sel, const int64_t* rows,
                                                       const uint8_t* arena, const int64_t* off, const int32_t* lens,
                                                       const int32_t* k, double p_indel, double p_del, uint64_t seed,
                                                       uint64_t call, uint8_t* out, int out_width, int32_t* out_len) {
  __shared__ int pos[kFloydMax];
  __shared__ uint8_t lit[kFloydMax][2];
  __shared__ int nlit[kFloydMax];
  const int ne = dn ? min(*dn, nsel) : nsel;
  for (int j = blockIdx.x; j < ne; j += gridDim.x) {
    mut_apply_item(j, sel, rows, arena, off, lens, k, p_indel, p_del, seed, call, out, out_width, out_len, pos, lit,
                   nlit);
    __syncthreads();
  }
}

// k[i] ~ Poisson(p * (len(a) + len(b))) for neighbour pair i
__global__ void __launch_bounds__(256) rec_count_kernel(int n, const int32_t* pairs, const int32_t* lens, double p,
                                                        uint64_t seed, uint64_t call, int32_t* k) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int nb = lens[pairs[2 * i]] + lens[pairs[2 * i + 1]];
  if (nb < 1) {
    k[i] = 0;
    return;
  }
  Philox rng(seed, call, (uint32_t)i);
  long long kk = poisson(rng, p * (double)nb);
  k[i] = (int32_t)(kk > nb ? nb : kk);
}

// Same draw over fixed neighbour slots (int64 keys (a << 32) | b, -1 = empty slot). With `lw_word`
// (world.hip index_map_lmax: the longest genome): by thinning against the bound len(a) + longest,
// as world.hip rec_slot_draw (the device pipeline's draw: the same stream and order, so both paths
// select the same pairs); without: directly.
__global__ void __launch_bounds__(256) rec_count_keys_kernel(int n, const int64_t* keys, const int32_t* lens, double p,
                                                             uint64_t seed, uint64_t call, int32_t* k, int32_t* tot,
                                                             int kcap, const int* gflags, int* opflags,
                                                             const unsigned long long* lw_word) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (gp_skip(i, gflags, opflags)) {
    k[i] = 0;
    if (tot) tot[i] = 0;
    return;
  }
  const int64_t key = keys[i];
  if (key < 0) {
    k[i] = 0;
    if (tot) tot[i] = 0;
    return;
  }
  const int la = lens[key >> 32];
  const int nb = la + lens[key & 0xFFFFFFFF];
  if (tot) tot[i] = nb;
  long long kk = 0;
  if (lw_word) {
    const double lb = (double)la + (double)(int)(*lw_word & 0xFFFFFFFFull);
    if (lb >= 1.0) {
      Philox rng(seed, call, (uint32_t)i);
      const long long nev = poisson(rng, p * lb);
      for (long long e = 0; e < nev; ++e) kk += rng.uniform_d() * lb < (double)nb ? 1 : 0;
    }
  } else {
    if (nb < 1) {
      k[i] = 0;
      return;
    }
    Philox rng(seed, call, (uint32_t)i);
    kk = poisson(rng, p * (double)nb);
  }
  if (kcap > 0 && kk > kcap) kk = kcap;
  k[i] = (int32_t)(kk > nb ? nb : kk);
}

// Recombine pair sel[j] (rows ca, cb of the arena) into scratch rows 2j and 2j+1 (rec_pair_apply).
__device__ __forceinline__ void rec_apply_item(int j, const int64_t* sel, const int32_t* pairs, const int64_t* keys,
                                               const uint8_t* arena, const int64_t* off, const int32_t* lens,
                                               const int32_t* k,
                                               uint64_t seed, uint64_t call, int32_t* parts, int parts_cap,
                                               uint8_t* out, int out_width, int32_t* out_len, int64_t* out_rows,
                                               int32_t* lparts, int* meta) {
  const int lane = threadIdx.x;
  const int64_t i = sel[j];
  // pairs: int32 (a, b) rows, or int64 slot keys (a << 32) | b
  const int ca = keys ? (int)(keys[i] >> 32) : pairs[2 * i];
  const int cb = keys ? (int)(keys[i] & 0xFFFFFFFF) : pairs[2 * i + 1];
  int w0, w1;
  rec_pair_apply(arena + off[ca], lens[ca], arena + off[cb], lens[cb], k[i], seed, call,
                 (uint32_t)i, parts + (size_t)j * parts_cap * 3, lparts, meta, out + (size_t)(2 * j) * out_width,
                 out + (size_t)(2 * j + 1) * out_width, out_width, w0, w1);
  if (lane == 0) {
    out_len[2 * j] = w0 < out_width ? w0 : out_width;
    out_len[2 * j + 1] = w1 < out_width ? w1 : out_width;
    if (out_rows) {
      out_rows[2 * j] = ca;
      out_rows[2 * j + 1] = cb;
    }
  }
}

__global__ void __launch_bounds__(64) rec_apply_kernel(int nsel, const int* dn, const int64_t* sel, const int32_t* pairs,
                                                       const int64_t* keys, const uint8_t* arena, const int64_t* off,
                                                       const int32_t* lens, const int32_t* k, uint64_t seed,
                                                       uint64_t call, int32_t* parts, int parts_cap, uint8_t* out,
                                                       int out_width, int32_t* out_len, int64_t* out_rows) {
  __shared__ int32_t lparts[(kFloydMax + 2) * 3];
  __shared__ int meta[2];  // number of parts, split index
  const int ne = dn ? min(*dn, nsel) : nsel;
  for (int j = blockIdx.x; j < ne; j += gridDim.x) {
    rec_apply_item(j, sel, pairs, keys, arena, off, lens, k, seed, call, parts, parts_cap, out, out_width, out_len,
                   out_rows, lparts, meta);
    __syncthreads();
  }
}

// ---------------------------------------------------------------- arena commit
// Last writer wins among duplicate target rows (a cell in several recombined pairs keeps the
// result of the last pair, as the reference's sequential update does): generation-tagged 64-bit
// marks, so the mark array never needs clearing.
// dn (optional): device item count, scaled by dn_mul (2 for the two results of a recombined pair)
__device__ __forceinline__ int eff_count(int k, const int* dn, int dn_mul) { return dn ? min(*dn * dn_mul, k) : k; }

__global__ void __launch_bounds__(256) arena_mark_kernel(int k, const int* dn, int dn_mul, const int64_t* rows,
                                                         unsigned long long* mark, unsigned long long gen) {
  const int ke = eff_count(k, dn, dn_mul);
  for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < ke; q += gridDim.x * blockDim.x)
    atomicMax(mark + rows[q], (gen << 32) | (unsigned long long)q);
}

// One wavefront per result row: copy it over its arena row (zero-padding the rest of the row) and
// its length, if it won; flags[q] = won.
// Commit result rows into fresh space of the genome pool: every row that won its cell (mark: the
// last result per cell) gets a new 16-byte aligned allocation (pool_alloc), its bytes, and the
// cell's offset and length. A result longer than `width` (the pipeline's genome length bound) or a
// full pool is left for the host (flags; reconcile raises the bound / collects the pool and
// re-commits), so pending calls never see a genome longer than the bound they were sized for.
__global__ void __launch_bounds__(64) arena_scatter_kernel(int k, const int* dn, int dn_mul, const int64_t* rows,
                                                           const uint8_t* src, int src_width, const int32_t* src_len,
                                                           uint8_t* pool, int64_t* off, unsigned long long* top,
                                                           long long pool_cap, int width, int32_t* lens,
                                                           const unsigned long long* mark, unsigned long long gen,
                                                           uint8_t* flags, int* gflags, int* opflags,
                                                           int64_t* app_cand = nullptr, int* app_cnt = nullptr) {
  const int ke = eff_count(k, dn, dn_mul), lane = threadIdx.x;
  if (flags)  // entries past the live count read as "not won" (no separate clearing launch)
    for (int q = ke + blockIdx.x * 64 + lane; q < k; q += gridDim.x * 64) flags[q] = 0;
  const bool vec = (src_width & 15) == 0 && (reinterpret_cast<uintptr_t>(src) & 15) == 0;
  for (int q = blockIdx.x; q < ke; q += gridDim.x) {
    const int64_t r = rows[q];
    const bool won = !mark || mark[r] == ((gen << 32) | (unsigned long long)q);
    if (lane == 0 && flags) flags[q] = won;
    if (!won) continue;
    if (lane == 0 && app_cnt) app_cand[atomicAdd(app_cnt, 1)] = q;  // (winners appended: world.hip sel_sort)
    if (gflags && src_len[q] > width) {  // longer than the bound: left for the host (reconcile)
      if (lane == 0) {
        atomicOr(gflags, kGpWidth);
        atomicOr(opflags, kGpWidth);
      }
      continue;
    }
    const int L = min(src_len[q], width);
    long long o = 0;
    if (lane == 0) o = pool_alloc(top, pool_cap, L);
    o = (long long)(((unsigned long long)(unsigned)__shfl((int)(o >> 32), 0) << 32) |
                    (unsigned long long)(unsigned)__shfl((int)(o & 0xFFFFFFFFll), 0));
    if (o < 0) {  // pool full: the same route as a too long result
      if (lane == 0 && gflags) {
        atomicOr(gflags, kGpWidth);
        atomicOr(opflags, kGpWidth);
      }
      continue;
    }
    const uint8_t* s = src + (size_t)q * src_width;
    uint8_t* d = pool + o;
    if (vec) {
      for (int t = lane * 16; t < L; t += 64 * 16) *reinterpret_cast<uint4*>(d + t) = *reinterpret_cast<const uint4*>(s + t);
    } else {
      for (int t = lane; t < L; t += 64) d[t] = s[t];
    }
    if (lane == 0) {
      off[r] = o;
      lens[r] = L;
    }
  }
}

constexpr unsigned kDevGrid = 2048;
static unsigned item_grid(long long n, uintptr_t dn) {
  return dn ? (unsigned)std::min<long long>(n, kDevGrid) : (unsigned)n;
}

void mut_count(int n, uintptr_t rows, uintptr_t lens, double p, uint64_t seed, uint64_t call, uintptr_t k, int kcap,
               uintptr_t gflags, uintptr_t opflags, uintptr_t stream) {
  if (n <= 0) return;
  msd::kl(mut_count_kernel, cdiv(n, 256), 256, 0, S_(stream))(n, rows ? P_<int64_t>(rows) : nullptr, P_<int32_t>(lens), p,
                                                         seed, call, P_<int32_t>(k), kcap,
                                                         gflags ? P_<int>(gflags) : nullptr, P_<int>(opflags));
  MS_LAUNCH_CHECK();
}

std::pair<int32_t*, int32_t*> select_tiles(long long tiles, hipStream_t s);
void select_write_i32pos_capped(long long n, uintptr_t src, int32_t* tc, int32_t* tm, int sub, uintptr_t sel,
                                uintptr_t out_dev, int cap, uintptr_t gflags, uintptr_t opflags, hipStream_t s);

int* append_counter(hipStream_t s);
void sel_sort(uintptr_t cand, int* cnt, int cap, uintptr_t sel, uintptr_t out_dev, uintptr_t gflags, uintptr_t opflags,
              hipStream_t s, uintptr_t gather = 0);
int sel_sort_cap();
extern int g_mut_append;
int g_mut_append = 1;  // 0: the count + selection passes for every capacity (A/B, set_rec_thinning)

// mut_count over all n genomes + the capped selection of those with events into sel / out_dev (the
// device pipeline's mutation chain): the draws appended + sorted (mut_draw_kernel, world.hip
// sel_sort; `cand`: 8 * cap bytes of scratch) when the capacity fits the sort, else the fused count
// pass + the selection pass.
void mut_count_select(int n, uintptr_t lens, double p, uint64_t seed, uint64_t call, uintptr_t k, int kcap,
                      uintptr_t gflags, uintptr_t opflags, uintptr_t sel, uintptr_t out_dev, int cap, uintptr_t cand,
                      uintptr_t stream, uintptr_t na, uintptr_t nb) {
  if (n <= 0) throw std::invalid_argument("mut_count_select: no genomes");
  hipStream_t s = S_(stream);
  if (g_mut_append && cand && cap <= sel_sort_cap()) {
    int* cnt = append_counter(s);
    msd::kl(mut_draw_kernel, cdiv(n, 256), 256, 0, s)(n, P_<int32_t>(lens), p, seed, call, P_<int32_t>(k), kcap,
                                                 gflags ? P_<int>(gflags) : nullptr, P_<int>(opflags),
                                                 P_<int64_t>(cand), cnt, cap, na ? P_<int>(na) : nullptr,
                                                 nb ? P_<int>(nb) : nullptr);
    MS_LAUNCH_CHECK();
    sel_sort(cand, cnt, cap, sel, out_dev, gflags, opflags, s);
    return;
  }
  if (na) throw std::invalid_argument("mut_count_select: a device cell count needs the append path");
  constexpr int kSelTile = 4096, kBlock = 256;  // select.hip tile; 16 count blocks per tile
  const long long blocks = ((long long)n + kSelTile - 1) / kSelTile * (kSelTile / kBlock);
  auto tiles = select_tiles(blocks, s);
  msd::kl(mut_count_tiles_kernel, (unsigned)blocks, kBlock, 0, s)(n, P_<int32_t>(lens), p, seed, call, P_<int32_t>(k), kcap,
                                                            gflags ? P_<int>(gflags) : nullptr, P_<int>(opflags),
                                                            tiles.first, tiles.second);
  MS_LAUNCH_CHECK();
  select_write_i32pos_capped(n, k, tiles.first, tiles.second, kSelTile / kBlock, sel, out_dev, cap, gflags, opflags, s);
}

void mut_apply(int nsel, uintptr_t dn, uintptr_t sel, uintptr_t rows, uintptr_t arena, uintptr_t off, uintptr_t lens,
               uintptr_t k, double p_indel, double p_del, uint64_t seed, uint64_t call, uintptr_t out, int out_width,
               uintptr_t out_len, uintptr_t stream) {
  if (nsel <= 0) return;
  msd::kl(mut_apply_kernel, item_grid(nsel, dn), 64, 0, S_(stream))(
      nsel, dn ? P_<int>(dn) : nullptr, P_<int64_t>(sel), rows ? P_<int64_t>(rows) : nullptr, P_<uint8_t>(arena),
      P_<int64_t>(off), P_<int32_t>(lens), P_<int32_t>(k), p_indel, p_del, seed, call, P_<uint8_t>(out), out_width,
      P_<int32_t>(out_len));
  MS_LAUNCH_CHECK();
}

void rec_count(int n, uintptr_t pairs, uintptr_t lens, double p, uint64_t seed, uint64_t call, uintptr_t k,
               uintptr_t stream) {
  if (n <= 0) return;
  msd::kl(rec_count_kernel, cdiv(n, 256), 256, 0, S_(stream))(n, P_<int32_t>(pairs), P_<int32_t>(lens), p, seed, call,
                                                         P_<int32_t>(k));
  MS_LAUNCH_CHECK();
}

void rec_count_keys(int n, uintptr_t keys, uintptr_t lens, double p, uint64_t seed, uint64_t call, uintptr_t k,
                    uintptr_t tot, int kcap, uintptr_t gflags, uintptr_t opflags, uintptr_t stream,
                    uintptr_t lw_word) {
  if (n <= 0) return;
  msd::kl(rec_count_keys_kernel, cdiv(n, 256), 256, 0, S_(stream))(n, P_<int64_t>(keys), P_<int32_t>(lens), p, seed, call,
                                                              P_<int32_t>(k), tot ? P_<int32_t>(tot) : nullptr, kcap,
                                                              gflags ? P_<int>(gflags) : nullptr, P_<int>(opflags),
                                                              lw_word ? P_<unsigned long long>(lw_word) : nullptr);
  MS_LAUNCH_CHECK();
}

void rec_apply(int nsel, uintptr_t dn, uintptr_t sel, uintptr_t pairs, uintptr_t keys, uintptr_t arena, uintptr_t off,
               uintptr_t lens, uintptr_t k, uint64_t seed, uint64_t call, uintptr_t parts, int parts_cap, uintptr_t out,
               int out_width, uintptr_t out_len, uintptr_t out_rows, uintptr_t stream) {
  if (nsel <= 0) return;
  if ((pairs == 0) == (keys == 0)) throw std::invalid_argument("rec_apply: give exactly one of pairs / keys");
  msd::kl(rec_apply_kernel, item_grid(nsel, dn), 64, 0, S_(stream))(
      nsel, dn ? P_<int>(dn) : nullptr, P_<int64_t>(sel), pairs ? P_<int32_t>(pairs) : nullptr,
      keys ? P_<int64_t>(keys) : nullptr, P_<uint8_t>(arena), P_<int64_t>(off), P_<int32_t>(lens), P_<int32_t>(k), seed,
      call,
      P_<int32_t>(parts), parts_cap, P_<uint8_t>(out), out_width, P_<int32_t>(out_len),
      out_rows ? P_<int64_t>(out_rows) : nullptr);
  MS_LAUNCH_CHECK();
}

// k result rows (capacity when dn != 0: then *dn * dn_mul rows are live)
static void arena_scatter_impl(int k, uintptr_t dn, int dn_mul, uintptr_t rows, uintptr_t src, int src_width,
                               uintptr_t src_len, uintptr_t pool, uintptr_t off, uintptr_t top, long long pool_cap,
                               int width, uintptr_t lens, uintptr_t mark, uint64_t gen, uintptr_t flags,
                               uintptr_t gflags, uintptr_t opflags, uintptr_t stream, int64_t* app_cand,
                               int* app_cnt) {
  if (gflags && !opflags) throw std::invalid_argument("arena_scatter: gflags needs opflags");
  if (k <= 0) return;
  const int* d = dn ? P_<int>(dn) : nullptr;
  if (mark) {
    const unsigned g = dn ? std::min<unsigned>(cdiv(k, 256), 256u) : cdiv(k, 256);
    msd::kl(arena_mark_kernel, g, 256, 0, S_(stream))(k, d, dn_mul, P_<int64_t>(rows), P_<unsigned long long>(mark), gen);
    MS_LAUNCH_CHECK();
  }
  msd::kl(arena_scatter_kernel, item_grid(k, dn), 64, 0, S_(stream))(
      k, d, dn_mul, P_<int64_t>(rows), P_<uint8_t>(src), src_width, P_<int32_t>(src_len), P_<uint8_t>(pool),
      P_<int64_t>(off), P_<unsigned long long>(top), pool_cap, width, P_<int32_t>(lens), mark ? P_<unsigned long long>(mark) : nullptr, gen, flags ? P_<uint8_t>(flags) : nullptr,
      gflags ? P_<int>(gflags) : nullptr, opflags ? P_<int>(opflags) : nullptr, app_cand, app_cnt);
  MS_LAUNCH_CHECK();
}

void arena_scatter(int k, uintptr_t dn, int dn_mul, uintptr_t rows, uintptr_t src, int src_width, uintptr_t src_len,
                   uintptr_t pool, uintptr_t off, uintptr_t top, long long pool_cap, int width, uintptr_t lens,
                   uintptr_t mark, uint64_t gen, uintptr_t flags, uintptr_t gflags, uintptr_t opflags,
                   uintptr_t stream) {
  arena_scatter_impl(k, dn, dn_mul, rows, src, src_width, src_len, pool, off, top, pool_cap, width, lens, mark, gen,
                     flags, gflags, opflags, stream, nullptr, nullptr);
}

// arena_scatter with the winning result rows appended to `cand` (k int64 entries) on the stream's
// append counter instead of `won` flags for a selection pass (gp.hip: world.hip sel_sort orders them)
void arena_scatter_app(int k, uintptr_t dn, int dn_mul, uintptr_t rows, uintptr_t src, int src_width, uintptr_t src_len,
                       uintptr_t pool, uintptr_t off, uintptr_t top, long long pool_cap, int width, uintptr_t lens,
                       uintptr_t mark, uint64_t gen, uintptr_t gflags, uintptr_t opflags, uintptr_t cand,
                       uintptr_t stream) {
  arena_scatter_impl(k, dn, dn_mul, rows, src, src_width, src_len, pool, off, top, pool_cap, width, lens, mark, gen, 0,
                     gflags, opflags, stream, P_<int64_t>(cand), append_counter(S_(stream)));
}

}  // namespace msd
