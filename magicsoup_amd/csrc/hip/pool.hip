// The GPU genome pool (models/strings.py PoolArena): genomes of every length in one byte buffer at
// per-cell offsets, instead of rows as wide as the longest genome.
//
// The reference keeps each genome as its own Python string (python/magicsoup/world.py:192-194) and
// its Rust mutates strings one by one (rust/mutations.rs:11-154). Here a cell's genome is the
// lens[i] bytes at pool + off[i]; storage is allocated by an atomic bump of a device counter
// (hip_common.h pool_alloc, 16-byte aligned) and never written again: a mutated or recombined genome
// takes new space, a dividing cell's child shares its parent's bytes (only off / lens are copied), a
// killed cell only leaves its offset behind. The space of genomes nobody references any more is
// reclaimed by a compaction that keeps shared genomes shared (pool_compact, PoolArena.collect).
#include <pybind11/pybind11.h>

#include <algorithm>
#include <stdexcept>

#include "hip_common.h"
#include "bind_util.h"

namespace msd {

// Genome j: bytes rows[j, :lens[j]] (row stride L_in) -> a new allocation; cell dst[j] (or n0 + j)
// gets its offset and length. A workgroup takes kPwChunk genomes at a time: their (pool_alloc-sized)
// allocations are one atomic on the bump counter -- one per genome serialised ~10k atomics on one
// address (137 us for a 10.8k-cell top-up spawn) -- and its four waves copy them. A full pool sets
// *failed (the host sized the pool so that it never is; the flag makes a sizing bug loud).
constexpr int kPwChunk = 16;
__global__ void __launch_bounds__(256) pool_write_kernel(int k, int L_in, const uint8_t* rows, const int32_t* lens,
                                                         const int64_t* dst, long long n0, uint8_t* pool, int64_t* off,
                                                         unsigned long long* top, long long cap, int32_t* out_lens,
                                                         int* failed) {
  __shared__ long long s_off[kPwChunk];
  __shared__ int s_len[kPwChunk];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool vec = (L_in & 15) == 0 && (reinterpret_cast<uintptr_t>(rows) & 15) == 0;
  for (long long j0 = (long long)blockIdx.x * kPwChunk; j0 < k; j0 += (long long)gridDim.x * kPwChunk) {
    if (w == 0) {
      const long long j = j0 + lane;
      int L = 0, sz = 0;
      if (lane < kPwChunk && j < k) {
        L = min(max(lens[j], 0), L_in);
        sz = ((L > 1 ? L : 1) + 15) & ~15;  // (as pool_alloc: every allocation has its own offset)
      }
      int incl = sz;  // inclusive prefix over the chunk's lanes
      for (int o = 1; o < kPwChunk; o <<= 1) {
        const int v = __shfl_up(incl, o);
        if (lane >= o) incl += v;
      }
      const int total = __shfl(incl, kPwChunk - 1);
      unsigned long long base = 0;
      if (lane == 0) base = atomicAdd(top, (unsigned long long)total);
      const unsigned lo = __shfl((unsigned)(base & 0xFFFFFFFFull), 0), hi = __shfl((unsigned)(base >> 32), 0);
      base = ((unsigned long long)hi << 32) | lo;
      if (lane < kPwChunk) {
        s_off[lane] = (long long)(base + (unsigned long long)total) <= cap ? (long long)(base + incl - sz) : -1ll;
        s_len[lane] = L;
      }
    }
    __syncthreads();
    for (int q = w; q < kPwChunk; q += 4) {
      const long long j = j0 + q;
      if (j >= k) break;
      const long long o = s_off[q];
      const int L = s_len[q];
      const long long c = dst ? dst[j] : n0 + j;
      if (o < 0) {
        if (lane == 0) {
          if (failed) atomicOr(failed, 1);
          off[c] = 0;
          out_lens[c] = 0;
        }
        continue;
      }
      const uint8_t* src = rows + (size_t)j * L_in;
      uint8_t* d = pool + o;
      if (vec) {
        for (int t = lane * 16; t < L; t += 64 * 16)
          *reinterpret_cast<uint4*>(d + t) = *reinterpret_cast<const uint4*>(src + t);
      } else {
        for (int t = lane; t < L; t += 64) d[t] = src[t];
      }
      if (lane == 0) {
        off[c] = o;
        out_lens[c] = L;
      }
    }
    __syncthreads();  // (the chunk's offsets are read before the next chunk's wave 0 overwrites them)
  }
}

// Genomes of cells src[j] (or j) -> zero-padded rows out[j, :W] (at most W bytes each).
__global__ void __launch_bounds__(64) pool_read_kernel(int k, const int64_t* src, const uint8_t* pool,
                                                       const int64_t* off, const int32_t* lens, uint8_t* out, int W) {
  const int lane = threadIdx.x;
  for (int j = blockIdx.x; j < k; j += gridDim.x) {
    const long long c = src ? src[j] : j;
    const int L = min(lens[c], W);
    const uint8_t* s = pool + off[c];
    uint8_t* d = out + (size_t)j * W;
    for (int t = lane; t < W; t += 64) d[t] = t < L ? s[t] : 0;
  }
}

// Genomes of cells src[j] (or j) back to back: out[dst_off[j] : dst_off[j] + lens] (no padding;
// StringColumn materialisation copies exactly the genome bytes to the host).
__global__ void __launch_bounds__(64) pool_read_packed_kernel(int k, const int64_t* src, const uint8_t* pool,
                                                              const int64_t* off, const int32_t* lens,
                                                              const int64_t* dst_off, uint8_t* out) {
  const int lane = threadIdx.x;
  for (int j = blockIdx.x; j < k; j += gridDim.x) {
    const long long c = src ? src[j] : j;
    const int L = lens[c];
    const uint8_t* s = pool + off[c];
    uint8_t* d = out + dst_off[j];
    for (int t = lane * 16; t < L; t += 64 * 16) {  // 16-byte loads (allocations are 16-byte aligned)
      const uint4 q = *reinterpret_cast<const uint4*>(s + t);
      const uint8_t* b = reinterpret_cast<const uint8_t*>(&q);
      const int e = min(16, L - t);
      for (int u = 0; u < e; ++u) d[t + u] = b[u];
    }
  }
}

// Compaction: unique genome u (old offset old_off[u], size bytes) -> new_pool + new_off[u].
__global__ void __launch_bounds__(64) pool_compact_kernel(int nu, const uint8_t* old_pool, const int64_t* old_off,
                                                          const int64_t* sizes, uint8_t* new_pool,
                                                          const int64_t* new_off) {
  const int lane = threadIdx.x;
  for (int u = blockIdx.x; u < nu; u += gridDim.x) {
    const uint4* s = reinterpret_cast<const uint4*>(old_pool + old_off[u]);
    uint4* d = reinterpret_cast<uint4*>(new_pool + new_off[u]);
    const long long n16 = sizes[u] / 16;  // allocations are 16-byte multiples
    for (long long t = lane; t < n16; t += 64) d[t] = s[t];
  }
}

// ---- collection on the device (PoolArena.collect): no sort, no host loop over genomes.
// Pool space is in 16-byte granules. Every allocation starts at a granule that some cell's offset
// names; cells sharing an allocation (a parent and its children) name the same one. mark: per cell,
// the allocation's size (the longest genome naming it, at least one granule, as pool_alloc) and its
// owner (the lowest cell index naming it) into per-granule arrays; scan: exclusive prefix sum of the
// sizes over the granules = the allocations' new offsets, in old-offset order; move: the owner copies
// the allocation, every cell takes the new offset. The layout equals the one of sorting the distinct
// offsets and summing their sizes in that order.
__global__ void __launch_bounds__(256) pool_mark_kernel(int n, const int64_t* off, const int32_t* lens,
                                                        int32_t* size_g, int32_t* owner_g) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long long g = off[i] >> 4;
  const int sz = max(1, (max(lens[i], 0) + 15) >> 4);
  atomicMax(size_g + g, sz);
  atomicMin(owner_g + g, i);
}

constexpr int kScanThreads = 256, kScanItems = 4, kScanTile = kScanThreads * kScanItems;

__device__ __forceinline__ long long block_excl_scan(long long v, long long* s_w, long long& total) {
  // exclusive scan of one value per thread over the block (4 waves of 64)
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  long long x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const long long y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) s_w[w] = x;
  __syncthreads();
  long long base = 0;
  total = 0;
  for (int q = 0; q < kScanThreads / 64; ++q) {
    if (q < w) base += s_w[q];
    total += s_w[q];
  }
  __syncthreads();
  return base + x - v;
}

// tile t of the granules: exclusive scan within the tile -> new_g, the tile's total -> tile_sum[t]
__global__ void __launch_bounds__(kScanThreads) pool_scan_tiles_kernel(long long G, const int32_t* size_g,
                                                                       int32_t* new_g, long long* tile_sum) {
  __shared__ long long s_w[kScanThreads / 64];
  const long long base = (long long)blockIdx.x * kScanTile + (long long)threadIdx.x * kScanItems;
  int v[kScanItems];
  long long mine = 0;
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    v[j] = base + j < G ? size_g[base + j] : 0;
    mine += v[j];
  }
  long long total;
  long long pre = block_excl_scan(mine, s_w, total);
#pragma unroll
  for (int j = 0; j < kScanItems; ++j) {
    if (base + j < G) new_g[base + j] = (int32_t)pre;
    pre += v[j];
  }
  if (threadIdx.x == 0) tile_sum[blockIdx.x] = total;
}

// one block: exclusive scan of the tile totals in place; the grand total (granules) -> *total
__global__ void __launch_bounds__(kScanThreads) pool_scan_sums_kernel(long long tiles, long long* tile_sum,
                                                                      long long* total_out) {
  __shared__ long long s_w[kScanThreads / 64];
  __shared__ long long s_carry;
  if (threadIdx.x == 0) s_carry = 0;
  __syncthreads();
  for (long long b0 = 0; b0 < tiles; b0 += kScanThreads) {
    const long long t = b0 + threadIdx.x;
    const long long v = t < tiles ? tile_sum[t] : 0;
    long long total;
    const long long pre = block_excl_scan(v, s_w, total);
    const long long carry = s_carry;
    if (t < tiles) tile_sum[t] = carry + pre;
    __syncthreads();
    if (threadIdx.x == 0) s_carry = carry + total;
    __syncthreads();
  }
  if (threadIdx.x == 0) *total_out = s_carry;
}

__global__ void __launch_bounds__(kScanThreads) pool_scan_add_kernel(long long G, int32_t* new_g,
                                                                     const long long* tile_sum) {
  const long long g = (long long)blockIdx.x * kScanThreads + threadIdx.x;
  if (g < G) new_g[g] += (int32_t)tile_sum[g / kScanTile];
}

// one wavefront per cell: the owner of its allocation copies it; every cell takes the new offset
__global__ void __launch_bounds__(64) pool_move_kernel(int n, int64_t* off, const uint8_t* old_pool,
                                                       uint8_t* new_pool, const int32_t* size_g,
                                                       const int32_t* owner_g, const int32_t* new_g) {
  const int lane = threadIdx.x;
  for (int c = blockIdx.x; c < n; c += gridDim.x) {
    const long long g = off[c] >> 4;
    const long long d = (long long)new_g[g] << 4;
    if (owner_g[g] == c) {
      const uint4* s = reinterpret_cast<const uint4*>(old_pool + (g << 4));
      uint4* t = reinterpret_cast<uint4*>(new_pool + d);
      const int n16 = size_g[g];
      for (int q = lane; q < n16; q += 64) t[q] = s[q];
    }
    if (lane == 0) off[c] = d;
  }
}

static unsigned grid_for(long long k) { return (unsigned)std::max<long long>(1, std::min<long long>(k, 8192)); }

void pool_write(int k, int L_in, uintptr_t rows, uintptr_t lens, uintptr_t dst, long long n0, uintptr_t pool,
                uintptr_t off, uintptr_t top, long long cap, uintptr_t out_lens, uintptr_t failed, uintptr_t stream) {
  if (k <= 0) return;
  if (L_in < 0) throw std::invalid_argument("pool_write: negative row width");
  const unsigned grid = (unsigned)std::max<long long>(1, std::min<long long>(((long long)k + kPwChunk - 1) / kPwChunk, 4096));
  msd::kl(pool_write_kernel, grid, 256, 0, S_(stream))(k, L_in, P_<uint8_t>(rows), P_<int32_t>(lens),
                                                        dst ? P_<int64_t>(dst) : nullptr, n0, P_<uint8_t>(pool),
                                                        P_<int64_t>(off), P_<unsigned long long>(top), cap,
                                                        P_<int32_t>(out_lens), failed ? P_<int>(failed) : nullptr);
  MS_LAUNCH_CHECK();
}

void pool_read(int k, uintptr_t src, uintptr_t pool, uintptr_t off, uintptr_t lens, uintptr_t out, int W,
               uintptr_t stream) {
  if (k <= 0 || W <= 0) return;
  msd::kl(pool_read_kernel, grid_for(k), 64, 0, S_(stream))(k, src ? P_<int64_t>(src) : nullptr, P_<uint8_t>(pool),
                                                       P_<int64_t>(off), P_<int32_t>(lens), P_<uint8_t>(out), W);
  MS_LAUNCH_CHECK();
}

void pool_read_packed(int k, uintptr_t src, uintptr_t pool, uintptr_t off, uintptr_t lens, uintptr_t dst_off,
                      uintptr_t out, uintptr_t stream) {
  if (k <= 0) return;
  msd::kl(pool_read_packed_kernel, grid_for(k), 64, 0, S_(stream))(k, src ? P_<int64_t>(src) : nullptr, P_<uint8_t>(pool),
                                                              P_<int64_t>(off), P_<int32_t>(lens), P_<int64_t>(dst_off),
                                                              P_<uint8_t>(out));
  MS_LAUNCH_CHECK();
}

void pool_compact(int nu, uintptr_t old_pool, uintptr_t old_off, uintptr_t sizes, uintptr_t new_pool,
                  uintptr_t new_off, uintptr_t stream) {
  if (nu <= 0) return;
  if ((old_pool | new_pool) & 15) throw std::invalid_argument("pool_compact: pools must be 16-byte aligned");
  msd::kl(pool_compact_kernel, grid_for(nu), 64, 0, S_(stream))(nu, P_<uint8_t>(old_pool), P_<int64_t>(old_off),
                                                           P_<int64_t>(sizes), P_<uint8_t>(new_pool),
                                                           P_<int64_t>(new_off));
  MS_LAUNCH_CHECK();
}

// Phase 1 of a collection over the G granules below the pool's top: sizes / owners per granule and
// their exclusive scan; the total (granules) -> total_out (device int64). size_g, owner_g, new_g:
// int32[G]; tile_sum: int64[ceil(G / 1024)].
void pool_collect_plan(int n, uintptr_t off, uintptr_t lens, long long G, uintptr_t size_g, uintptr_t owner_g,
                       uintptr_t new_g, uintptr_t tile_sum, uintptr_t total_out, uintptr_t stream) {
  if (n <= 0 || G <= 0) throw std::invalid_argument("pool_collect_plan: empty pool");
  if (G >= (1ll << 31)) throw std::invalid_argument("pool_collect_plan: pool too large for int32 granule offsets");
  hipStream_t s = S_(stream);
  MS_HIP_CHECK(msd::memset_async(P_<int32_t>(size_g), 0, (size_t)G * 4, s));
  MS_HIP_CHECK(msd::memset_async(P_<int32_t>(owner_g), 0x7F, (size_t)G * 4, s));
  msd::kl(pool_mark_kernel, cdiv(n, 256), 256, 0, s)(n, P_<int64_t>(off), P_<int32_t>(lens), P_<int32_t>(size_g),
                                                P_<int32_t>(owner_g));
  MS_LAUNCH_CHECK();
  const long long tiles = (G + kScanTile - 1) / kScanTile;
  msd::kl(pool_scan_tiles_kernel, (unsigned)tiles, kScanThreads, 0, s)(G, P_<int32_t>(size_g), P_<int32_t>(new_g),
                                                                  P_<long long>(tile_sum));
  MS_LAUNCH_CHECK();
  msd::kl(pool_scan_sums_kernel, 1, kScanThreads, 0, s)(tiles, P_<long long>(tile_sum), P_<long long>(total_out));
  MS_LAUNCH_CHECK();
  msd::kl(pool_scan_add_kernel, (unsigned)cdiv(G, kScanThreads), kScanThreads, 0, s)(G, P_<int32_t>(new_g),
                                                                                P_<long long>(tile_sum));
  MS_LAUNCH_CHECK();
}

// Phase 2: copy every allocation into new_pool (sized for the total) and remap the offsets.
void pool_collect_move(int n, uintptr_t off, uintptr_t old_pool, uintptr_t new_pool, uintptr_t size_g,
                       uintptr_t owner_g, uintptr_t new_g, uintptr_t stream) {
  if (n <= 0) return;
  if ((old_pool | new_pool) & 15) throw std::invalid_argument("pool_collect_move: pools must be 16-byte aligned");
  msd::kl(pool_move_kernel, grid_for(n), 64, 0, S_(stream))(n, P_<int64_t>(off), P_<uint8_t>(old_pool),
                                                       P_<uint8_t>(new_pool), P_<int32_t>(size_g),
                                                       P_<int32_t>(owner_g), P_<int32_t>(new_g));
  MS_LAUNCH_CHECK();
}

void bind_pool(pybind11::module_& m) {
  namespace py = pybind11;
  py::class_<GenomePoolArgs>(m, "GenomePoolArgs", py::module_local())
      .def(py::init<>())
      .def_readwrite("pool", &GenomePoolArgs::pool)
      .def_readwrite("off", &GenomePoolArgs::off)
      .def_readwrite("top", &GenomePoolArgs::top)
      .def_readwrite("failed", &GenomePoolArgs::failed)
      .def_readwrite("cap", &GenomePoolArgs::cap);
  msd::gdef(m, "pool_write", &pool_write, "genome rows (k, L) -> new pool allocations of cells dst[j] (or n0 + j)");
  msd::gdef(m, "pool_read", &pool_read, "genomes of cells -> zero-padded rows (k, W)");
  msd::gdef(m, "pool_read_packed", &pool_read_packed, "genomes of cells back to back (no padding)");
  msd::gdef(m, "pool_compact", &pool_compact, "copy unique genomes into a new pool");
  msd::gdef(m, "pool_collect_plan", &pool_collect_plan, "collection phase 1: per-granule sizes / owners and their scan");
  msd::gdef(m, "pool_collect_move", &pool_collect_move, "collection phase 2: copy the allocations, remap the offsets");
}

}  // namespace msd
