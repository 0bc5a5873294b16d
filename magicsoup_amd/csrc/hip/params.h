// Ragged (CSR) parameter storage of the GPU kinetics (models/kinetics.py, slot mode).
//
// Every protein of a cell is one *record* of the record pool: its packed stoichiometry words W (s
// int32: int8 N / Nf / Nb / A), its Kmr row (s floats) and Q = (Vmax, Kmf, Kmb, Ke). A cell owns a
// contiguous run of records -- as many as its proteome has proteins, not the population's longest
// proteome -- named by one int64 per cell (the kinetics "slot", moved with the per-cell columns by
// every compaction / clone gather):
//
//   bits  0..31  offset of the first record (4 Gi records: past any record pool of 288 GB)
//   bits 32..47  record count (proteins, at most kRecMaxProteins)
//   bits 48..63  protein width of the build that wrote them (the dense API pads the proteins
//                [count, width) with the reference's build padding -- Vmax 0, Kmf = Kmb = EPS, Ke 1,
//                Kmr 1 -- and shows zeros beyond, as a later widening of the reference's tensors)
//
// Slot 0 is a cell without parameters (all zero, like unset_cell_params). A dense (c, P) layout is
// the special case offset i * P, count P, width P. Records are written once (a rebuild takes fresh
// ones, a division's child shares its parent's), taken by a device bump counter and compacted by a
// collection when the pool runs out (Kinetics._collect_records). The reference keeps dense (c, p, s)
// tensors padded to the longest proteome (python/magicsoup/kinetics.py:399-409, 705-723).
#pragma once
#include <stdint.h>

namespace msd {

constexpr int kRecOffBits = 32;
constexpr int kRecCntBits = 16;
constexpr int kRecMaxProteins = (1 << 15) - 1;  // (count and width; the width keeps the sign bit clear)
constexpr unsigned long long kRecOffMask = (1ull << kRecOffBits) - 1ull;

__host__ __device__ __forceinline__ long long rec_encode(long long off, int cnt, int width) {
  return (long long)(((unsigned long long)width << (kRecOffBits + kRecCntBits)) |
                     ((unsigned long long)cnt << kRecOffBits) | ((unsigned long long)off & kRecOffMask));
}
__host__ __device__ __forceinline__ long long rec_off(long long v) {
  return (long long)((unsigned long long)v & kRecOffMask);
}
__host__ __device__ __forceinline__ int rec_cnt(long long v) {
  return (int)(((unsigned long long)v >> kRecOffBits) & ((1ull << kRecCntBits) - 1ull));
}
__host__ __device__ __forceinline__ int rec_width(long long v) {
  return (int)((unsigned long long)v >> (kRecOffBits + kRecCntBits));
}

// The records of `cell`: the slot map `prow` (CSR), or the dense layout (prow == nullptr: cell i's P
// proteins at records i * P ..). Invalid items get an empty range.
__device__ __forceinline__ void prot_range(const int64_t* prow, int cell, int P, bool valid, size_t& base, int& cnt) {
  if (!valid) {
    base = 0;
    cnt = 0;
  } else if (prow) {
    const long long v = prow[cell];
    base = (size_t)rec_off(v);
    cnt = rec_cnt(v);
  } else {
    base = (size_t)cell * (size_t)P;
    cnt = P;
  }
}

}  // namespace msd

namespace msd {

// Records for items 0..ne-1 of a build, in item order, taken from the bump counter *rtop by ONE
// workgroup (1024 threads): an exclusive scan of the protein counts, chunk by chunk. Item j's cell
// (cells[j], or j) gets slot rec_encode(offset, np_j, width) and roff[j] = offset; an item without
// proteins gets slot 0 (no parameters) and roff[j] = -1; an item past `rcap` keeps its slot and gets
// roff[j] = -1 and flag bit `fbit` (the host rebuilds it after a collection). The counter ends past
// the last record taken. Every thread of the block must call it.
__device__ __forceinline__ void assign_records_block(int ne, const int32_t* nprot, const int64_t* cells, int64_t* slot,
                                                     long long* rtop, long long rcap, int width, int64_t* roff,
                                                     int* flags, int fbit) {
  __shared__ long long s_base, s_end;
  __shared__ int s_w[16];
  __shared__ int s_tot;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  if (threadIdx.x == 0) {
    s_base = *rtop;
    s_end = s_base;
  }
  __syncthreads();
  for (int c0 = 0; c0 < ne; c0 += blockDim.x) {
    const int j = c0 + (int)threadIdx.x;
    int np = j < ne ? nprot[j] : 0;
    if (np < 0) np = 0;
    if (np > kRecMaxProteins) {  // (a proteome the slot cannot name: the host path raises first)
      atomicOr(flags, fbit);
      np = 0;
    }
    int x = np;  // inclusive scan within the wave
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (lane == 63) s_w[wave] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
      int acc = 0;
      for (int w = 0; w < nw; ++w) {
        const int t = s_w[w];
        s_w[w] = acc;
        acc += t;
      }
      s_tot = acc;
    }
    __syncthreads();
    const long long off = s_base + s_w[wave] + x - np;
    if (j < ne) {
      const long long cell = cells ? cells[j] : (long long)j;
      if (np == 0) {
        slot[cell] = 0;
        roff[j] = -1;
      } else if (off + np > rcap) {
        atomicOr(flags, fbit);
        roff[j] = -1;
      } else {
        slot[cell] = rec_encode(off, np, width);
        roff[j] = off;
        atomicMax(reinterpret_cast<unsigned long long*>(&s_end), (unsigned long long)(off + np));
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) s_base += s_tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) *rtop = s_end;
}

}  // namespace msd
