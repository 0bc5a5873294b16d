// Multi-tensor row movement: one launch copies rows of up to kMaxDescs row-major tensors.
//
// A world operation touches every per-cell array at once -- cell molecules, positions, lifetimes,
// divisions, the genome and label arenas and the nine kinetics parameter tensors -- with the same
// row mapping (order-preserving compaction on kill_cells, parent -> child cloning on divide_cells).
// Instead of one gather launch per tensor (plus a copy back), all of them go through one kernel:
// the work is flattened over (descriptor, row, 16-byte chunk) with a prefix over descriptors, so
// large rows (kinetics (P, s) slices of a few KiB) and 4-byte rows share one grid.
#include <algorithm>
#include <tuple>
#include <vector>

#include "rows.h"

namespace msd {

// grid.y = descriptor: no per-element descriptor search; 32-bit index math within a descriptor
// (n * units < 2^31 is checked on the host).
template <class U>
__device__ __forceinline__ void copy_units(const RowDesc& d, unsigned total, const int64_t* src_rows,
                                           const int64_t* dst_rows, long long dst_off) {
  const unsigned units = (unsigned)d.units;
  for (unsigned t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const unsigned i = t / units, c = t - i * units;
    const long long sr = src_rows ? src_rows[i] : (long long)i;
    if (d.len && c * sizeof(U) >= (unsigned)d.len[sr]) continue;
    const long long dr = (dst_rows ? dst_rows[i] : (long long)i) + dst_off;
    const U v = reinterpret_cast<const U*>(d.src + sr * d.src_stride)[c];
    reinterpret_cast<U*>(d.dst + dr * d.dst_stride)[c] = v;
  }
}

__global__ void __launch_bounds__(256) gather_rows_kernel(RowArgs a) {
  const RowDesc& d = a.d[blockIdx.y];
  const unsigned n_eff = (unsigned)(a.dn ? min(*a.dn, a.n) : a.n);
  const unsigned total = n_eff * (unsigned)d.units;
  if (blockIdx.x * blockDim.x >= total) return;
  const long long off = a.dst_off + (a.dst_base ? (long long)*a.dst_base : 0ll);
  if (d.unit == 16)
    copy_units<uint4>(d, total, a.src_rows, a.dst_rows, off);
  else
    copy_units<uint32_t>(d, total, a.src_rows, a.dst_rows, off);
}

RowArgs make_row_args(const std::vector<RowDescTuple>& descs, size_t first, size_t* next) {
  RowArgs a{};
  int nd = 0;
  size_t q = first;
  for (; q < descs.size() && nd < kMaxDescs; ++q) {
    const auto& [sp, dp, ss, ds, rb, lp] = descs[q];
    if (rb <= 0) continue;
    if (rb % 4 || ss % 4 || ds % 4 || sp % 4 || dp % 4)
      throw std::invalid_argument("gather_rows: rows, strides and pointers must be 4-byte aligned");
    const bool vec = rb % 16 == 0 && ss % 16 == 0 && ds % 16 == 0 && sp % 16 == 0 && dp % 16 == 0;
    RowDesc& d = a.d[nd];
    d.src = P_<uint8_t>(sp);
    d.dst = P_<uint8_t>(dp);
    d.src_stride = ss;
    d.dst_stride = ds;
    d.unit = vec ? 16 : 4;
    d.units = (int)(rb / d.unit);
    d.len = lp ? P_<int32_t>(lp) : nullptr;
    ++nd;
  }
  a.nd = nd;
  if (next) *next = q;
  return a;
}

void launch_row_args(const RowArgs& plan, int n, const int* dn, const int64_t* src_rows, const int64_t* dst_rows,
                     long long dst_off, hipStream_t s, const int* dst_base) {
  if (n <= 0 || plan.nd == 0) return;
  RowArgs a = plan;
  a.n = n;
  a.dn = dn;
  a.src_rows = src_rows;
  a.dst_rows = dst_rows;
  a.dst_off = dst_off;
  a.dst_base = dst_base;
  long long widest = 0;
  for (int q = 0; q < a.nd; ++q) widest = std::max(widest, (long long)n * a.d[q].units);
  if (widest >= (1ll << 31)) throw std::invalid_argument("gather_rows: too many units per tensor");
  // enough blocks for the widest descriptor, capped (grid-stride beyond); ~2k blocks fill the chip
  const long long blocks = (widest + 255) / 256;
  const unsigned gx = (unsigned)(blocks < 2048 ? blocks : 2048);
  msd::kl(gather_rows_kernel, dim3(gx, a.nd), 256, 0, s)(a);
  MS_LAUNCH_CHECK();
}

// descs: (src_ptr, dst_ptr, src_stride_bytes, dst_stride_bytes, row_bytes) per tensor. Row bytes and
// strides must be multiples of 4 (of 16 for the vector path, chosen per tensor).
void gather_rows(int n, uintptr_t dn, uintptr_t src_rows, uintptr_t dst_rows, const std::vector<RowDescTuple>& descs,
                 uintptr_t stream) {
  if (n <= 0 || descs.empty()) return;
  size_t q = 0;
  while (q < descs.size()) {
    const RowArgs a = make_row_args(descs, q, &q);
    launch_row_args(a, n, dn ? P_<int>(dn) : nullptr, src_rows ? P_<int64_t>(src_rows) : nullptr,
                    dst_rows ? P_<int64_t>(dst_rows) : nullptr, 0, S_(stream));
  }
}

}  // namespace msd
