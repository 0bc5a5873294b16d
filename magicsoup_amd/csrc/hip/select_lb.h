// Single-pass order-preserving selection (select.hip select_lb_kernel, world.hip winners + commit).
//
// A grid of at most kLbMaxTiles tiles of kSelTile items: each tile ballots its items, publishes its
// selected count tagged with the call's generation (one 64-bit word per tile, never reset: a stale
// word carries an older tag), then sums the published counts of the tiles before it and hands every
// item its output position. Every tile publishes before it waits on anything and workgroups are
// dispatched in index order, so the spin on an earlier tile ends; it is bounded anyway: a tile that
// never publishes sets the mapped error word `err` (LbState::err, read by lb_error_take through
// hip_ops.check_placement) instead of hanging the device. One launch per selection instead
// of the count + write pair, and the caller's per-item work (a payload, a commit) rides along.
#pragma once
#include "hip_common.h"

namespace msd {

constexpr int kSelThreads = 256;
constexpr int kSelItems = 16;
constexpr int kSelTile = kSelThreads * kSelItems;  // 4096
constexpr int kLbMaxTiles = 1024;

// the tile status words of a stream and the tag of the call being issued (select.hip lb_begin)
// Tags are 28 bits wide (place_split_lb_kernel packs three 12-bit counts beside its tag): lb_begin
// clears the words whenever the generation wraps at 2^28, so no stale word carries a matching tag.
constexpr uint32_t kLbGenMask = 0x0FFFFFFFu;
struct LbState {
  unsigned long long* status;
  uint32_t gen;   // 1 .. kLbGenMask
  unsigned* err;  // mapped host word: a look-back spin timed out (the selection's offsets are wrong)
};
LbState lb_begin(hipStream_t s);
// whether select_indices_async takes the single-pass form for n items
bool select_single_pass(long long n);
// 1 if a single-pass selection's look-back spin timed out since the last call; clears the word
int lb_error_take();
// a fresh pinned status slot (select.hip ring) and its device pointer
int status_slot_new(long long** dev);

// pred(i) -> bool; on_sel(k, i): i is the k-th selected item; on_rest(r, i): the r-th rejected.
// The last tile writes the count to out[0] (0 to out[1]) and {count, 0, 0, 0} to host64 if given.
// Returns the tile's first output position; *tile_cnt (if given) gets its selected count.
// ITEMS per thread (tiles of 256 * ITEMS items): fewer items per tile mean more workgroups for the
// caller's per-tile work (world.hip select_commit_kernel commits a tile's winners in its workgroup).
template <int ITEMS = kSelItems, class Pred, class OnSel, class OnRest>
__device__ __forceinline__ long long select_lb_tile(long long n, Pred pred, unsigned long long* status, uint32_t gen,
                                                    unsigned* err, OnSel on_sel, OnRest on_rest, int32_t* out, long long* host64,
                                                    int* tile_cnt = nullptr) {
  constexpr int W = kSelThreads / 64;
  constexpr int kTile = kSelThreads * ITEMS;
  __shared__ long long s_red[W];
  __shared__ int s_wc[ITEMS][W];
  __shared__ int s_pre[ITEMS][W];
  __shared__ int s_tot;
  const int w = threadIdx.x >> 6, lane = lane_id();
  const int b = blockIdx.x;
  const long long base = (long long)b * kTile;
  uint64_t ballots[ITEMS];
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const long long i = base + j * kSelThreads + threadIdx.x;
    const bool p = i < n && pred(i);
    ballots[j] = __ballot(p);
    if (lane == 0) s_wc[j][w] = __popcll(ballots[j]);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int j = 0; j < ITEMS; ++j)
      for (int q = 0; q < W; ++q) {
        s_pre[j][q] = acc;
        acc += s_wc[j][q];
      }
    s_tot = acc;
    __hip_atomic_store(status + b, ((unsigned long long)gen << 32) | (unsigned)acc, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  long long off = 0;
  for (int q = threadIdx.x; q < b; q += kSelThreads) {
    unsigned long long v = __hip_atomic_load(status + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int spin = 0; (uint32_t)(v >> 32) != gen; ++spin) {
      if (spin >= (1 << 22)) {  // (never in a healthy grid: report, do not hang)
        if (err) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      v = __hip_atomic_load(status + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    off += (uint32_t)v;
  }
  for (int o = 32; o > 0; o >>= 1) off += __shfl_xor(off, o);
  if (lane == 0) s_red[w] = off;
  __syncthreads();
  long long tile_off = 0;
#pragma unroll
  for (int q = 0; q < W; ++q) tile_off += s_red[q];
  const uint64_t lt = lane == 0 ? 0ull : (~0ull >> (64 - lane));
#pragma unroll
  for (int j = 0; j < ITEMS; ++j) {
    const long long i = base + j * kSelThreads + threadIdx.x;
    if (i >= n) break;
    const long long k = s_pre[j][w] + __popcll(ballots[j] & lt);  // selected before i within the tile
    if ((ballots[j] >> lane) & 1ull)
      on_sel(tile_off + k, i);
    else
      on_rest((base - tile_off) + (i - base - k), i);
  }
  if (tile_cnt) *tile_cnt = s_tot;
  if (b == (int)gridDim.x - 1 && threadIdx.x == 0) {
    const int total = (int)(tile_off + s_tot);
    out[0] = total;
    out[1] = 0;
    if (host64) {
      host64[0] = total;
      host64[1] = 0;
      host64[2] = 0;
      host64[3] = 0;
    }
  }
  return tile_off;
}

}  // namespace msd
