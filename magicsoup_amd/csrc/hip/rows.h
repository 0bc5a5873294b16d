// Multi-tensor row movement (rows.hip): descriptors of one gather launch, reusable as a prebuilt
// plan (fast.hip keeps plans for the compaction / clone gathers of a world's per-cell buffers).
#pragma once
#include <tuple>
#include <vector>

#include "hip_common.h"

namespace msd {

constexpr int kMaxDescs = 24;

struct RowDesc {
  const uint8_t* src;
  uint8_t* dst;
  long long src_stride, dst_stride;  // bytes between rows
  int units;                         // row size in units
  int unit;                          // 16 or 4 bytes
  const int32_t* len;                // optional: bytes used by source row r (string arenas); the
                                     // rest of the row is not copied (padding is never read)
};

struct RowArgs {
  RowDesc d[kMaxDescs];
  int nd, n;
  long long dst_off;        // added to every destination row
  const int* dst_base;      // optional device value, also added to every destination row
  const int* dn;            // optional device row count (<= n; n is then the capacity)
  const int64_t* src_rows;  // nullptr: identity
  const int64_t* dst_rows;  // nullptr: identity
};

using RowDescTuple = std::tuple<uintptr_t, uintptr_t, long long, long long, long long, uintptr_t>;

// Descriptors of up to kMaxDescs (src, dst, src stride, dst stride, row bytes, lens) tuples.
RowArgs make_row_args(const std::vector<RowDescTuple>& descs, size_t first = 0, size_t* next = nullptr);
// One launch of a prebuilt plan over rows [0, n) (device count dn optional).
void launch_row_args(const RowArgs& plan, int n, const int* dn, const int64_t* src_rows, const int64_t* dst_rows,
                     long long dst_off, hipStream_t s, const int* dst_base = nullptr);

}  // namespace msd
