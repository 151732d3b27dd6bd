// Chunk-range geometry of the partition's in-block prefix sums (gbdt_partition_atomic.h,
// kMode 3): host- and device-callable so the index math is checked on the CPU
// (tests/test_chunk_range.py) against a brute-force sum.
#pragma once
#include <hip/hip_runtime.h>

namespace ytk {

// The chunk counts of [f0, f1) (one split's chunks) summed as the partial group at each end
// read count by count plus the whole 32-chunk groups between them read from their group sums
// (gsum[g] = sum of chunks [32 g, 32 g + 32), all splits'): item t of ntot -> its address.
constexpr int kGrpShift = 5;
struct ChunkRange {
  int f0, g0, c1, na, nab, ntot;
  __host__ __device__ __forceinline__ ChunkRange(int f0_, int f1) : f0(f0_) {
    g0 = f0 >> kGrpShift;
    const int g1 = f1 >> kGrpShift;
    if (g0 == g1) {
      na = f1 - f0;
      nab = na;
      c1 = f1;
    } else {
      na = ((g0 + 1) << kGrpShift) - f0;
      nab = na + (g1 - g0 - 1);
      c1 = g1 << kGrpShift;
    }
    ntot = nab + (f1 - c1);
  }
  __host__ __device__ __forceinline__ const unsigned long long* item(const unsigned long long* cnt,
                                                                     const unsigned long long* gsum, int t) const {
    return t < na ? cnt + f0 + t : t < nab ? gsum + (g0 + 1 + t - na) : cnt + c1 + (t - nab);
  }
};

}  // namespace ytk
