// Order-preserving stream compaction with the count delivered to pinned host memory.
//
// Every population change of the API (kill_cells, divide_cells, the mutated / recombined subset of
// mutate_cells / recombinate_cells) needs "the ascending indices i with pred(i)" and, because the
// reference API returns Python-sized results, their count on the host. torch.nonzero does this with
// ~5 launches and a separate read-back; here it is two launches plus one stream synchronisation:
//
//   select_count_kernel   per 4096-item tile: selected count and max(vals) of selected items
//   select_write_kernel   per tile: exclusive offset from the preceding tiles' counts, wave-ballot
//                         prefix within the tile, write selected (and optionally the rejected)
//                         indices; the last tile writes {count, max} straight into pinned host memory
//
// Predicates: u8 mask != 0, u8 mask == 0, int32 > 0, int64 >= 0.
#include <unordered_map>
#include <algorithm>
#include <tuple>

#include <cstring>
#include <vector>

#include "hip_common.h"
#include "select_lb.h"

namespace msd {


enum SelKind { kMaskSet = 0, kMaskClear = 1, kI32Pos = 2, kI64NonNeg = 3 };

template <int K>
__device__ __forceinline__ bool sel_pred(const void* src, long long i) {
  if constexpr (K == kMaskSet) return reinterpret_cast<const uint8_t*>(src)[i] != 0;
  if constexpr (K == kMaskClear) return reinterpret_cast<const uint8_t*>(src)[i] == 0;
  if constexpr (K == kI32Pos) return reinterpret_cast<const int32_t*>(src)[i] > 0;
  return reinterpret_cast<const int64_t*>(src)[i] >= 0;
}

template <int K>
__global__ void __launch_bounds__(kSelThreads) select_count_kernel(long long n, const void* src, const int32_t* vals,
                                                                   int32_t* tile_count, int32_t* tile_max) {
  __shared__ int s_cnt[kSelThreads / 64], s_max[kSelThreads / 64];
  const long long base = (long long)blockIdx.x * kSelTile;
  int cnt = 0, mx = 0;
#pragma unroll
  for (int j = 0; j < kSelItems; ++j) {
    const long long i = base + j * kSelThreads + threadIdx.x;
    if (i < n && sel_pred<K>(src, i)) {
      ++cnt;
      if (vals) mx = max(mx, vals[i]);
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    cnt += __shfl_xor(cnt, o);
    mx = max(mx, __shfl_xor(mx, o));
  }
  const int w = threadIdx.x >> 6;
  if (lane_id() == 0) {
    s_cnt[w] = cnt;
    s_max[w] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int c = 0, m = 0;
    for (int q = 0; q < kSelThreads / 64; ++q) {
      c += s_cnt[q];
      m = max(m, s_max[q]);
    }
    tile_count[blockIdx.x] = c;
    tile_max[blockIdx.x] = m;
  }
}

template <int K>
__global__ void __launch_bounds__(kSelThreads) select_write_kernel(long long n, const void* src, const int32_t* tile_count,
                                                                   const int32_t* tile_max, int64_t* sel,
                                                                   int64_t* rest, int32_t* host_out,
                                                                   long long* host64, int cap, int* cap_gflags,
                                                                   int* cap_opflags, int sub) {
  constexpr int W = kSelThreads / 64;
  __shared__ long long s_red[W];
  __shared__ int s_wc[kSelItems][W];
  __shared__ int s_pre[kSelItems][W];
  const int w = threadIdx.x >> 6, lane = lane_id();
  const int b = blockIdx.x;
  // exclusive offset of this tile: sum of the preceding tiles' counts
  long long off = 0;
  // (sub: the count pass wrote `sub` counts per tile, e.g. world.hip rec_slots_kernel)
  for (int q = threadIdx.x; q < b * sub; q += kSelThreads) off += tile_count[q];
  for (int o = 32; o > 0; o >>= 1) off += __shfl_xor(off, o);
  if (lane == 0) s_red[w] = off;
  const long long base = (long long)b * kSelTile;
  uint64_t ballots[kSelItems];
#pragma unroll
  for (int j = 0; j < kSelItems; ++j) {
    const long long i = base + j * kSelThreads + threadIdx.x;
    const bool p = i < n && sel_pred<K>(src, i);
    ballots[j] = __ballot(p);
    if (lane == 0) s_wc[j][w] = __popcll(ballots[j]);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    long long t = 0;
    for (int q = 0; q < W; ++q) t += s_red[q];
    s_red[0] = t;
    int acc = 0;
    for (int j = 0; j < kSelItems; ++j)
      for (int q = 0; q < W; ++q) {
        s_pre[j][q] = acc;
        acc += s_wc[j][q];
      }
  }
  __syncthreads();
  const long long tile_off = s_red[0];
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
  for (int j = 0; j < kSelItems; ++j) {
    const long long i = base + j * kSelThreads + threadIdx.x;
    if (i >= n) break;
    const long long k = s_pre[j][w] + __popcll(ballots[j] & lt);  // selected before i within the tile
    if ((ballots[j] >> lane) & 1ull) {
      sel[tile_off + k] = i;
    } else if (rest) {
      rest[(base - tile_off) + (i - base - k)] = i;
    }
  }
  if (b == (int)gridDim.x - 1 && threadIdx.x == 0) {
    int total = (int)tile_off, m = 0;
    for (int j = 0; j < kSelItems; ++j)
      for (int q = 0; q < W; ++q) total += s_wc[j][q];
    for (int q = 0; q < (int)gridDim.x * sub; ++q) m = max(m, tile_max[q]);
    if (cap >= 0 && total > cap) {
      // capacity guard of a device-pipeline call (cap_skip semantics): the call becomes a no-op
      // that the host replays on the synchronous path, and the pending chain is broken
      total = 0;
      atomicOr(cap_opflags, 16);  // kGpSkipped
      atomicOr(cap_gflags, 8);    // kGpWidth
    }
    host_out[0] = total;
    host_out[1] = m;
    if (host64) {  // also into a pinned status slot (select_indices_async)
      host64[0] = total;
      host64[1] = m;
      host64[2] = 0;
      host64[3] = 0;
    }
  }
}

// Single-pass form of the two kernels above (select_lb.h): one launch per selection. Optional
// payload: pay_dst[k] = pay_src[i] for the k-th selected item i, and 0 for the rejected items from
// the end (pay_dst[n - 1 - r] for the r-th rejected), so pay_dst[dn..n) is all zeros (the division
// mask compacted with the survivors of kill_divide, fast.hip).
template <int K, int ITEMS>
__global__ void __launch_bounds__(kSelThreads) select_lb_kernel(long long n, const void* src, unsigned long long* status,
                                                                uint32_t gen, unsigned* err, int64_t* sel,
                                                                int64_t* rest, int32_t* out, long long* host64,
                                                                const uint8_t* pay_src, uint8_t* pay_dst) {
  select_lb_tile<ITEMS>(
      n, [&](long long i) { return sel_pred<K>(src, i); }, status, gen, err,
      [&](long long k, long long i) {
        sel[k] = i;
        if (pay_dst) pay_dst[k] = pay_src[i];
      },
      [&](long long r, long long i) {
        if (rest) rest[r] = i;
        if (pay_dst) pay_dst[n - 1 - r] = 0;
      },
      out, host64);
}

// Per-genome protein totals (fwd + rev) and the maxima a translate count pass needs on the host.
// Block maxima are combined with atomicMax in a device accumulator; the last block to finish
// (done counter) publishes {max proteins, max domains, long genomes} to pinned host memory and
// resets the accumulator for the next call.
__global__ void __launch_bounds__(256) translate_stats_kernel(int n, const int32_t* counts, const int32_t* ndom,
                                                              const int32_t* long_count, int32_t* per, int32_t* acc,
                                                              int32_t* host_out) {
  int mp = 0, md = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const int p = counts[2 * i] + counts[2 * i + 1];
    per[i] = p;
    mp = max(mp, p);
    md = max(md, max(ndom[2 * i], ndom[2 * i + 1]));
  }
  for (int o = 32; o > 0; o >>= 1) {
    mp = max(mp, __shfl_xor(mp, o));
    md = max(md, __shfl_xor(md, o));
  }
  if (lane_id() == 0) {
    atomicMax(acc, mp);
    atomicMax(acc + 1, md);
  }
  __threadfence();
  __syncthreads();
  __shared__ bool last;
  if (threadIdx.x == 0) last = atomicAdd(acc + 2, 1) == (int)gridDim.x - 1;
  __syncthreads();
  if (last && threadIdx.x == 0) {
    __threadfence();
    host_out[0] = atomicExch(acc, 0);
    host_out[1] = atomicExch(acc + 1, 0);
    host_out[2] = *long_count;
    acc[2] = 0;
  }
}

namespace {
int32_t* g_host = nullptr;  // pinned, coherent {count, max}
int32_t* g_host_dev = nullptr;
// device {count[tiles], max[tiles]} per stream: selections on different streams (the compute
// stream and the genome chains' side stream) may run at the same time
struct TileBuf {
  int32_t* p = nullptr;
  long long cap = 0;
};
std::unordered_map<hipStream_t, TileBuf> g_tiles;
// the tile buffer of stream s with room for `tiles` tiles: {counts, maxima}
std::pair<int32_t*, int32_t*> tiles_for(hipStream_t s, long long tiles) {
  TileBuf& b = g_tiles[s];
  if (tiles > b.cap) {
    if (b.p) {
      MS_HIP_CHECK(msd::stream_synchronize(s));  // the old buffer may still be read by this stream
      MS_HIP_CHECK(msd::dev_free(b.p));
    }
    b.cap = std::max(tiles, 256ll);
    MS_HIP_CHECK(msd::dev_malloc((void**)&b.p, 2 * b.cap * sizeof(int32_t)));
  }
  return {b.p, b.p + b.cap};
}
// per stream: the tile status words of select_lb_tile and the generation of its last call
struct LbBuf {
  unsigned long long* p = nullptr;
  uint32_t gen = 0;
};
std::unordered_map<hipStream_t, LbBuf> g_lb;
unsigned* g_lb_err = nullptr;  // pinned, mapped: a look-back spin timed out (LbState::err)
unsigned* g_lb_err_dev = nullptr;
int g_sel_single = 1;  // select_indices_async takes the single-pass kernel when the grid allows
int g_sel_items = 4;   // items per thread of its tiles (1, 4 or 16) while the status words suffice
int32_t* g_tacc = nullptr;  // device {max proteins, max domains, done blocks}, zero between calls

void ensure_host() {
  if (!g_host) {
    MS_HIP_CHECK(hipHostMalloc((void**)&g_host, 4 * sizeof(int32_t), hipHostMallocMapped | hipHostMallocCoherent));
    MS_HIP_CHECK(hipHostGetDevicePointer((void**)&g_host_dev, g_host, 0));
  }
}
}  // namespace

std::tuple<int, int, int> translate_stats(int n, uintptr_t counts, uintptr_t ndom, uintptr_t long_count, uintptr_t per,
                                          uintptr_t stream) {
  if (n <= 0) return {0, 0, 0};
  ensure_host();
  if (!g_tacc) {
    MS_HIP_CHECK(msd::dev_malloc((void**)&g_tacc, 4 * sizeof(int32_t)));
    MS_HIP_CHECK(msd::dev_memset(g_tacc, 0, 4 * sizeof(int32_t)));
  }
  g_host[0] = -1;
  const unsigned grid = std::min(cdiv(n, 256), 1024u);
  msd::kl(translate_stats_kernel, grid, 256, 0, S_(stream))(n, P_<int32_t>(counts), P_<int32_t>(ndom),
                                                      P_<int32_t>(long_count), P_<int32_t>(per), g_tacc, g_host_dev);
  MS_LAUNCH_CHECK();
  MS_HIP_CHECK(msd::stream_synchronize(S_(stream)));
  if (g_host[0] < 0) throw std::runtime_error("translate_stats: bad read-back");
  return {g_host[0], g_host[1], g_host[2]};
}

// ---------------------------------------------------------------- device-count pipelines
// Sync-free genome updates (mutate / recombinate on the GPU): the selected count stays on the
// device, later kernels stride over it, and overflow conditions the host could not rule out in
// advance raise flag bits that the host resolves at its next synchronisation point.

// Like select_indices, but {count, max} go to device memory (out_dev) and nothing is synchronised.
void select_indices_dev(long long n, int kind, uintptr_t src, uintptr_t vals, uintptr_t sel, uintptr_t rest,
                        uintptr_t out_dev, uintptr_t stream);

// dst[j] = src[idx[j]] for j < min(*dn, cap)
__global__ void __launch_bounds__(256) gather_dev_kernel(int cap, const int* dn, const int64_t* idx, const int64_t* src,
                                                         int64_t* dst) {
  const int n = min(*dn, cap);
  for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) dst[j] = src[idx[j]];
}

// Capacity guard of a device-pipeline call: a selected count above the buffers' capacity turns the
// call into a no-op (count 0) that the host replays on the synchronous path (opflags |= skipped)
// and breaks the pending chain (gflags |= the arena-width bit), so later calls replay too.
constexpr int kGpWidthBit = 8, kGpSkippedBit = 16;  // mutations.hip kGpWidth / kGpSkipped
__global__ void cap_skip_kernel(int* dn, int cap, int* gflags, int* opflags) {
  if (*dn > cap) {
    *dn = 0;
    atomicOr(opflags, kGpSkippedBit);
    atomicOr(gflags, kGpWidthBit);
  }
}

void cap_skip(uintptr_t dn, int cap, uintptr_t gflags, uintptr_t opflags, uintptr_t stream) {
  msd::kl(cap_skip_kernel, 1, 1, 0, S_(stream))(P_<int>(dn), cap, P_<int>(gflags), P_<int>(opflags));
  MS_LAUNCH_CHECK();
}

// Pinned status ring: a pipeline call's {count, flags, row counter, selected count} are written by
// one single-thread kernel straight into coherent host memory; the host reads the slot after the
// call's event completed (no copy launch, no staging tensors).
constexpr int kStatusSlots = 64;
long long* g_status = nullptr;
long long* g_status_dev = nullptr;
int g_status_next = 0;

__global__ void status_write_kernel(const int* dcnt, const int* opflags, const long long* d_rows, const int* cnt,
                                    long long* out) {
  out[0] = *dcnt;
  out[1] = *opflags;
  out[2] = *d_rows;
  out[3] = *cnt;
}

int status_write(uintptr_t dcnt, uintptr_t opflags, uintptr_t d_rows, uintptr_t cnt, uintptr_t stream) {
  if (!g_status) {
    MS_HIP_CHECK(hipHostMalloc((void**)&g_status, kStatusSlots * 4 * sizeof(long long),
                               hipHostMallocMapped | hipHostMallocCoherent));
    MS_HIP_CHECK(hipHostGetDevicePointer((void**)&g_status_dev, g_status, 0));
  }
  const int slot = g_status_next;
  g_status_next = (g_status_next + 1) % kStatusSlots;
  for (int i = 0; i < 4; ++i) g_status[slot * 4 + i] = -1;
  msd::kl(status_write_kernel, 1, 1, 0, S_(stream))(P_<int>(dcnt), P_<int>(opflags), P_<long long>(d_rows), P_<int>(cnt),
                                               g_status_dev + slot * 4);
  MS_LAUNCH_CHECK();
  return slot;
}

__global__ void count_to_host_kernel(const int* dcount, long long* out) {
  out[0] = dcount[0];
  out[1] = dcount[1];
  out[2] = 0;
  out[3] = 0;
}

// {count, max} of a device-count select into a pinned ring slot: the host launches the work that
// depends on the count first and reads the slot after one stream synchronisation
int count_to_host(uintptr_t dcount, uintptr_t stream) {
  if (!g_status) {
    MS_HIP_CHECK(hipHostMalloc((void**)&g_status, kStatusSlots * 4 * sizeof(long long),
                               hipHostMallocMapped | hipHostMallocCoherent));
    MS_HIP_CHECK(hipHostGetDevicePointer((void**)&g_status_dev, g_status, 0));
  }
  const int slot = g_status_next;
  g_status_next = (g_status_next + 1) % kStatusSlots;
  for (int i = 0; i < 4; ++i) g_status[slot * 4 + i] = -1;
  msd::kl(count_to_host_kernel, 1, 1, 0, S_(stream))(P_<int>(dcount), g_status_dev + slot * 4);
  MS_LAUNCH_CHECK();
  return slot;
}

int status_slot_new(long long** dev) {
  if (!g_status) {
    MS_HIP_CHECK(hipHostMalloc((void**)&g_status, kStatusSlots * 4 * sizeof(long long),
                               hipHostMallocMapped | hipHostMallocCoherent));
    MS_HIP_CHECK(hipHostGetDevicePointer((void**)&g_status_dev, g_status, 0));
  }
  const int slot = g_status_next;
  g_status_next = (g_status_next + 1) % kStatusSlots;
  for (int i = 0; i < 4; ++i) g_status[slot * 4 + i] = -1;
  *dev = g_status_dev + slot * 4;
  return slot;
}

std::tuple<long long, long long, long long, long long> status_read(int slot) {
  if (!g_status || slot < 0 || slot >= kStatusSlots) throw std::invalid_argument("status_read: bad slot");
  const long long* v = g_status + slot * 4;
  if (v[0] < 0) throw std::runtime_error("status_read: slot not written (event not complete?)");
  return {v[0], v[1], v[2], v[3]};
}

// One stream synchronisation, then the slot (what wait_count needs, without a Python stream object).
std::tuple<long long, long long, long long, long long> stream_sync_read(int slot, uintptr_t stream) {
  MS_HIP_CHECK(msd::stream_synchronize(S_(stream)));
  return status_read(slot);
}

// select_indices_dev whose last tile also writes {count, max} into a fresh pinned status slot
// (returned): the host launches the work that depends on the count with `out_dev` as device count
// and reads the slot after one stream synchronisation (no separate copy launch).
LbState lb_begin(hipStream_t s) {
  LbBuf& lb = g_lb[s];
  if (!lb.p) {
    MS_HIP_CHECK(msd::dev_malloc((void**)&lb.p, kLbMaxTiles * sizeof(unsigned long long)));
    MS_HIP_CHECK(msd::memset_async(lb.p, 0, kLbMaxTiles * sizeof(unsigned long long), s));
  }
  if (!g_lb_err) {
    MS_HIP_CHECK(hipHostMalloc((void**)&g_lb_err, sizeof(unsigned), hipHostMallocMapped | hipHostMallocCoherent));
    *g_lb_err = 0;
    MS_HIP_CHECK(hipHostGetDevicePointer((void**)&g_lb_err_dev, g_lb_err, 0));
  }
  // the tags wrapped (at the narrowest tag width of the kernels that share the words): clear the
  // words, so no stale tag can match gen 1 then
  if (++lb.gen > kLbGenMask) {
    MS_HIP_CHECK(msd::memset_async(lb.p, 0, kLbMaxTiles * sizeof(unsigned long long), s));
    lb.gen = 1;
  }
  return {lb.p, lb.gen, g_lb_err_dev};
}

int lb_error_take() {
  if (!g_lb_err) return 0;
  return __atomic_exchange_n(g_lb_err, 0u, __ATOMIC_ACQ_REL) ? 1 : 0;
}

bool select_single_pass(long long n) { return g_sel_single && (n + kSelTile - 1) / kSelTile <= kLbMaxTiles; }

void set_select_single_pass(int on, int items) {
  g_sel_single = on;
  if (items == 1 || items == 4 || items == kSelItems) g_sel_items = items;
}

// The payload of a two-pass selection (too many items for the single-pass status words): the same
// bytes select_lb_kernel writes, pay_dst[k] = pay_src[sel[k]] below the device count, 0 above.
__global__ void __launch_bounds__(256) select_payload_kernel(long long n, const int32_t* cnt, const int64_t* sel,
                                                             const uint8_t* pay_src, uint8_t* pay_dst) {
  const long long c = *cnt;
  for (long long k = (long long)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (long long)gridDim.x * blockDim.x)
    pay_dst[k] = k < c ? pay_src[sel[k]] : (uint8_t)0;
}

// select_indices_async with the payload of select_lb_kernel (pay_dst: n bytes)
int select_indices_async_pay(long long n, int kind, uintptr_t src, uintptr_t sel, uintptr_t rest, uintptr_t out_dev,
                             uintptr_t pay_src, uintptr_t pay_dst, uintptr_t stream);

static int select_async_impl(long long n, int kind, uintptr_t src, uintptr_t sel, uintptr_t rest, uintptr_t out_dev,
                             uintptr_t pay_src, uintptr_t pay_dst, uintptr_t stream) {
  if (!g_status) {
    MS_HIP_CHECK(hipHostMalloc((void**)&g_status, kStatusSlots * 4 * sizeof(long long),
                               hipHostMallocMapped | hipHostMallocCoherent));
    MS_HIP_CHECK(hipHostGetDevicePointer((void**)&g_status_dev, g_status, 0));
  }
  const int slot = g_status_next;
  g_status_next = (g_status_next + 1) % kStatusSlots;
  for (int i = 0; i < 4; ++i) g_status[slot * 4 + i] = -1;
  long long* h64 = g_status_dev + slot * 4;
  hipStream_t s = S_(stream);
  if (n <= 0) {
    MS_HIP_CHECK(msd::memset_async(P_<int32_t>(out_dev), 0, 2 * sizeof(int32_t), s));
    msd::kl(count_to_host_kernel, 1, 1, 0, s)(P_<int>(out_dev), h64);
    MS_LAUNCH_CHECK();
    return slot;
  }
  if (n >= (1ll << 40)) throw std::invalid_argument("select_indices_async: n too large");
  const long long tiles = (n + kSelTile - 1) / kSelTile;
  const void* sp = reinterpret_cast<const void*>(src);
  if (g_sel_single && tiles <= kLbMaxTiles) {
    const LbState lb = lb_begin(s);
    // smaller tiles while they fit the status words: more workgroups, shorter per-tile chains
    const int items = g_sel_items < kSelItems && n <= (long long)kLbMaxTiles * kSelThreads * g_sel_items ? g_sel_items
                                                                                                      : kSelItems;
    const unsigned grid = (unsigned)((n + (long long)kSelThreads * items - 1) / ((long long)kSelThreads * items));
#define MS_SEL1(K, I)                                                                                               \
  msd::kl(select_lb_kernel<K, I>, grid, kSelThreads, 0, s)(n, sp, lb.status, lb.gen, lb.err, P_<int64_t>(sel),           \
                                                      rest ? P_<int64_t>(rest) : nullptr, P_<int32_t>(out_dev), h64, \
                                                      P_<uint8_t>(pay_src), P_<uint8_t>(pay_dst));                  \
  MS_LAUNCH_CHECK();
#define MS_SELI(K)             \
  if (items == 1) {            \
    MS_SEL1(K, 1)              \
  } else if (items == 4) {     \
    MS_SEL1(K, 4)              \
  } else {                     \
    MS_SEL1(K, kSelItems)      \
  }
    switch (kind) {
      case kMaskSet: MS_SELI(kMaskSet) break;
      case kMaskClear: MS_SELI(kMaskClear) break;
      case kI32Pos: MS_SELI(kI32Pos) break;
      case kI64NonNeg: MS_SELI(kI64NonNeg) break;
      default: throw std::invalid_argument("select_indices_async: unknown predicate");
    }
#undef MS_SELI
#undef MS_SEL1
    return slot;
  }
  auto tb = tiles_for(s, tiles);
  int32_t* tc = tb.first;
  int32_t* tm = tb.second;
  int32_t* out = P_<int32_t>(out_dev);
#define MS_SEL(K)                                                                                                \
  msd::kl(select_count_kernel<K>, (unsigned)tiles, kSelThreads, 0, s)(n, sp, nullptr, tc, tm);                      \
  MS_LAUNCH_CHECK();                                                                                             \
  msd::kl(select_write_kernel<K>, (unsigned)tiles, kSelThreads, 0, s)(n, sp, tc, tm, P_<int64_t>(sel),              \
                                                                 rest ? P_<int64_t>(rest) : nullptr, out, h64, -1, nullptr, nullptr, 1);  \
  MS_LAUNCH_CHECK();
  switch (kind) {
    case kMaskSet: MS_SEL(kMaskSet) break;
    case kMaskClear: MS_SEL(kMaskClear) break;
    case kI32Pos: MS_SEL(kI32Pos) break;
    case kI64NonNeg: MS_SEL(kI64NonNeg) break;
    default: throw std::invalid_argument("select_indices_async: unknown predicate");
  }
#undef MS_SEL
  if (pay_dst) {
    const unsigned g = (unsigned)std::min<long long>((n + 255) / 256, 4096);
    msd::kl(select_payload_kernel, g, 256, 0, s)(n, out, P_<int64_t>(sel), P_<uint8_t>(pay_src), P_<uint8_t>(pay_dst));
    MS_LAUNCH_CHECK();
  }
  return slot;
}

int select_indices_async(long long n, int kind, uintptr_t src, uintptr_t sel, uintptr_t rest, uintptr_t out_dev,
                         uintptr_t stream) {
  return select_async_impl(n, kind, src, sel, rest, out_dev, 0, 0, stream);
}

int select_indices_async_pay(long long n, int kind, uintptr_t src, uintptr_t sel, uintptr_t rest, uintptr_t out_dev,
                             uintptr_t pay_src, uintptr_t pay_dst, uintptr_t stream) {
  if (!pay_src || !pay_dst) throw std::invalid_argument("select_indices_async_pay: no payload");
  return select_async_impl(n, kind, src, sel, rest, out_dev, pay_src, pay_dst, stream);
}

void gather_dev(int cap, uintptr_t dn, uintptr_t idx, uintptr_t src, uintptr_t dst, uintptr_t stream) {
  const unsigned g = std::min(cdiv(cap, 256), 64u);
  msd::kl(gather_dev_kernel, g, 256, 0, S_(stream))(cap, P_<int>(dn), P_<int64_t>(idx), P_<int64_t>(src), P_<int64_t>(dst));
  MS_LAUNCH_CHECK();
}

// Returns {count, max(vals over selected)}; synchronises `stream`. sel must hold n entries (rest too,
// when given). Writes nothing and returns {0, 0} for n == 0.
std::pair<long long, int> select_indices(long long n, int kind, uintptr_t src, uintptr_t vals, uintptr_t sel,
                                         uintptr_t rest, uintptr_t stream) {
  if (n <= 0) return {0, 0};
  if (n >= (1ll << 40)) throw std::invalid_argument("select_indices: n too large");
  ensure_host();
  const long long tiles = (n + kSelTile - 1) / kSelTile;
  g_host[0] = -1;
  hipStream_t s = S_(stream);
  const void* sp = reinterpret_cast<const void*>(src);
  const int32_t* vp = vals ? P_<int32_t>(vals) : nullptr;
  auto tb = tiles_for(s, tiles);
  int32_t* tc = tb.first;
  int32_t* tm = tb.second;
#define MS_SEL(K)                                                                                               \
  msd::kl(select_count_kernel<K>, (unsigned)tiles, kSelThreads, 0, s)(n, sp, vp, tc, tm);                          \
  MS_LAUNCH_CHECK();                                                                                            \
  msd::kl(select_write_kernel<K>, (unsigned)tiles, kSelThreads, 0, s)(n, sp, tc, tm, P_<int64_t>(sel),             \
                                                                 rest ? P_<int64_t>(rest) : nullptr, g_host_dev, nullptr, -1, nullptr, nullptr, 1); \
  MS_LAUNCH_CHECK();
  switch (kind) {
    case kMaskSet: MS_SEL(kMaskSet) break;
    case kMaskClear: MS_SEL(kMaskClear) break;
    case kI32Pos: MS_SEL(kI32Pos) break;
    case kI64NonNeg: MS_SEL(kI64NonNeg) break;
    default: throw std::invalid_argument("select_indices: unknown predicate");
  }
#undef MS_SEL
  MS_HIP_CHECK(msd::stream_synchronize(s));
  const long long cnt = g_host[0];
  if (cnt < 0 || cnt > n) throw std::runtime_error("select_indices: bad count read-back");
  return {cnt, g_host[1]};
}

// select_indices_dev with the pipeline capacity guard folded into the last tile (cap_skip).
void select_indices_capped(long long n, int kind, uintptr_t src, uintptr_t sel, uintptr_t out_dev, int cap,
                           uintptr_t gflags, uintptr_t opflags, uintptr_t stream) {
  hipStream_t s = S_(stream);
  if (n <= 0) {
    MS_HIP_CHECK(msd::memset_async(P_<int32_t>(out_dev), 0, 2 * sizeof(int32_t), s));
    return;
  }
  if (n >= (1ll << 40)) throw std::invalid_argument("select_indices_capped: n too large");
  const long long tiles = (n + kSelTile - 1) / kSelTile;
  const void* sp = reinterpret_cast<const void*>(src);
  auto tb = tiles_for(s, tiles);
  int32_t* tc = tb.first;
  int32_t* tm = tb.second;
#define MS_SEL(K)                                                                                                \
  msd::kl(select_count_kernel<K>, (unsigned)tiles, kSelThreads, 0, s)(n, sp, nullptr, tc, tm);                      \
  MS_LAUNCH_CHECK();                                                                                             \
  msd::kl(select_write_kernel<K>, (unsigned)tiles, kSelThreads, 0, s)(n, sp, tc, tm, P_<int64_t>(sel), nullptr,     \
                                                                 P_<int32_t>(out_dev), nullptr, cap,             \
                                                                 P_<int>(gflags), P_<int>(opflags), 1);             \
  MS_LAUNCH_CHECK();
  switch (kind) {
    case kMaskSet: MS_SEL(kMaskSet) break;
    case kI32Pos: MS_SEL(kI32Pos) break;
    default: throw std::invalid_argument("select_indices_capped: unsupported predicate");
  }
#undef MS_SEL
}

// The tile buffers ({count, max} per tile, `tiles` entries each) for a caller whose own kernel
// produces the selected counts of an int32 > 0 selection, `sub` per kSelTile items (world.hip
// rec_slots), and the write pass of select_indices_capped over them.
std::pair<int32_t*, int32_t*> select_tiles(long long tiles, hipStream_t s) { return tiles_for(s, tiles); }

void select_write_i32pos_capped(long long n, uintptr_t src, int32_t* tc, int32_t* tm, int sub, uintptr_t sel,
                                uintptr_t out_dev, int cap, uintptr_t gflags, uintptr_t opflags, hipStream_t s) {
  if (kSelTile % sub) throw std::invalid_argument("select_write_i32pos_capped: bad sub-tile count");
  const long long tiles = (n + kSelTile - 1) / kSelTile;
  msd::kl(select_write_kernel<kI32Pos>, (unsigned)tiles, kSelThreads, 0, s)(
      n, reinterpret_cast<const void*>(src), tc, tm, P_<int64_t>(sel), nullptr, P_<int32_t>(out_dev), nullptr, cap,
      P_<int>(gflags), P_<int>(opflags), sub);
  MS_LAUNCH_CHECK();
}

// Overflow lists beside the status ring (gp.hip gp_check_assign_kernel): a rebuild call's cells
// whose proteome outgrew the speculative token layout, {count, cell...}, written by the device into
// coherent host memory so the host rebuilds just those cells once the call's event completed.
constexpr int kBadWords = 256;
long long* g_bad = nullptr;
long long* g_bad_dev = nullptr;

long long* status_bad_dev(int slot) {
  if (!g_bad) {
    MS_HIP_CHECK(hipHostMalloc((void**)&g_bad, kStatusSlots * kBadWords * sizeof(long long),
                               hipHostMallocMapped | hipHostMallocCoherent));
    MS_HIP_CHECK(hipHostGetDevicePointer((void**)&g_bad_dev, g_bad, 0));
  }
  g_bad[slot * kBadWords] = -1;
  return g_bad_dev + slot * kBadWords;
}

int status_bad_cap() { return kBadWords - 1; }

std::vector<long long> status_bad_read(int slot) {
  if (!g_bad || slot < 0 || slot >= kStatusSlots) throw std::invalid_argument("status_bad_read: bad slot");
  const long long* v = g_bad + slot * kBadWords;
  if (v[0] < 0 || v[0] > kBadWords - 1) throw std::runtime_error("status_bad_read: list not written");
  return std::vector<long long>(v + 1, v + 1 + v[0]);
}

// A fresh pinned status slot: {device pointer of its 4 int64 words, slot index}.
std::pair<long long*, int> status_slot() {
  if (!g_status) {
    MS_HIP_CHECK(hipHostMalloc((void**)&g_status, kStatusSlots * 4 * sizeof(long long),
                               hipHostMallocMapped | hipHostMallocCoherent));
    MS_HIP_CHECK(hipHostGetDevicePointer((void**)&g_status_dev, g_status, 0));
  }
  const int slot = g_status_next;
  g_status_next = (g_status_next + 1) % kStatusSlots;
  for (int i = 0; i < 4; ++i) g_status[slot * 4 + i] = -1;
  return {g_status_dev + slot * 4, slot};
}

void select_indices_dev(long long n, int kind, uintptr_t src, uintptr_t vals, uintptr_t sel, uintptr_t rest,
                        uintptr_t out_dev, uintptr_t stream) {
  hipStream_t s = S_(stream);
  if (n <= 0) {
    MS_HIP_CHECK(msd::memset_async(P_<int32_t>(out_dev), 0, 2 * sizeof(int32_t), s));
    return;
  }
  if (n >= (1ll << 40)) throw std::invalid_argument("select_indices_dev: n too large");
  const long long tiles = (n + kSelTile - 1) / kSelTile;
  const void* sp = reinterpret_cast<const void*>(src);
  const int32_t* vp = vals ? P_<int32_t>(vals) : nullptr;
  auto tb = tiles_for(s, tiles);
  int32_t* tc = tb.first;
  int32_t* tm = tb.second;
  int32_t* out = P_<int32_t>(out_dev);
#define MS_SEL(K)                                                                                                \
  msd::kl(select_count_kernel<K>, (unsigned)tiles, kSelThreads, 0, s)(n, sp, vp, tc, tm);                           \
  MS_LAUNCH_CHECK();                                                                                             \
  msd::kl(select_write_kernel<K>, (unsigned)tiles, kSelThreads, 0, s)(n, sp, tc, tm, P_<int64_t>(sel),              \
                                                                 rest ? P_<int64_t>(rest) : nullptr, out, nullptr, -1, nullptr, nullptr, 1);       \
  MS_LAUNCH_CHECK();
  switch (kind) {
    case kMaskSet: MS_SEL(kMaskSet) break;
    case kMaskClear: MS_SEL(kMaskClear) break;
    case kI32Pos: MS_SEL(kI32Pos) break;
    case kI64NonNeg: MS_SEL(kI64NonNeg) break;
    default: throw std::invalid_argument("select_indices_dev: unknown predicate");
  }
#undef MS_SEL
}

// Mapped pinned int flags (kernels store into host memory; the host reads them without a copy or a
// synchronisation): handed out from blocks of kFlagBlock, never reused, freed at exit.
constexpr int kFlagBlock = 1024;
static std::vector<int*> g_flag_blocks;
static int g_flag_next = kFlagBlock;
std::pair<uintptr_t, uintptr_t> mapped_flag() {
  if (g_flag_next == kFlagBlock) {
    int* h = nullptr;
    MS_HIP_CHECK(hipHostMalloc((void**)&h, kFlagBlock * sizeof(int), hipHostMallocMapped | hipHostMallocCoherent));
    std::memset(h, 0, kFlagBlock * sizeof(int));
    g_flag_blocks.push_back(h);
    g_flag_next = 0;
  }
  int* h = g_flag_blocks.back() + g_flag_next++;
  int* d = nullptr;
  MS_HIP_CHECK(hipHostGetDevicePointer((void**)&d, h, 0));
  return {reinterpret_cast<uintptr_t>(h), reinterpret_cast<uintptr_t>(d)};
}
int mapped_flag_read(uintptr_t host) { return *reinterpret_cast<volatile const int*>(host); }

// Free the process-wide pinned / device buffers of this file (exit path, see release_static).
void release_select_buffers() {
  for (int* h : g_flag_blocks) MS_HIP_CHECK(hipHostFree(h));
  g_flag_blocks.clear();
  g_flag_next = kFlagBlock;
  if (g_host) MS_HIP_CHECK(hipHostFree(g_host));
  g_host = g_host_dev = nullptr;
  if (g_tacc) MS_HIP_CHECK(msd::dev_free(g_tacc));
  g_tacc = nullptr;
  if (g_status) MS_HIP_CHECK(hipHostFree(g_status));
  g_status = g_status_dev = nullptr;
  for (auto& kv : g_tiles)
    if (kv.second.p) MS_HIP_CHECK(msd::dev_free(kv.second.p));
  g_tiles.clear();
}

}  // namespace msd
