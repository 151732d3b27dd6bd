// Histogram-sync helpers of the multi-GPU tree engines (gfx950).
//
// Reference: J/data/gbdt/HistogramBuilder.java:95 -- reduceScatterArray of the level's
// histograms by feature ownership (GBDTDataFlow.java:252-272 assigns each worker a
// contiguous feature range), plus the per-level child-count allreduce
// (DataParallelTreeMaker.java:518,538).
//
// Owner-computes sync: the level's built slots are [slot][bin][F][2] int64; rank r owns
// features [r*fr, min(F, (r+1)*fr)). A reduce-scatter needs the P feature blocks as P
// contiguous chunks, so ONE pack kernel writes x[r] = (the slots' block-r columns, zero
// padded to fr, then the level's count words, replicated into every chunk) into a
// persistent buffer, and ONE unpack kernel scatters this rank's reduced chunk back
// (instead of a zero fill plus one strided copy per rank every level).
#include "common.h"

namespace ytk {

// i in [0, P * (nb + C)): chunk r = i / (nb + C); inside a chunk, element
// ((slot * B + bin) * fr + fl) * 2 + c of the block, then the C count words.
__global__ __launch_bounds__(256) void owner_pack_kernel(const long long* __restrict__ hist, long long* __restrict__ x,
                                                         int nslots, int B, int F, int fr, int P,
                                                         const long long* __restrict__ cnt, int C) {
  const long long nb = (long long)nslots * B * fr * 2;
  const long long per = nb + C;
  const long long total = per * P;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int r = (int)(i / per);
    const long long j = i - (long long)r * per;
    long long v = 0;
    if (j < nb) {
      const int c = (int)(j & 1);
      const long long e = j >> 1;  // (slot * B + bin) * fr + fl
      const int fl = (int)(e % fr);
      const long long sb = e / fr;  // slot * B + bin
      const int f = r * fr + fl;
      if (f < F) v = hist[(sb * F + f) * 2 + c];
    } else {
      v = cnt[j - nb];
    }
    x[i] = v;
  }
}

__global__ __launch_bounds__(256) void owner_unpack_kernel(const long long* __restrict__ out, long long* __restrict__ hist,
                                                           int nslots, int B, int F, int fr, int rank,
                                                           long long* __restrict__ cnt, int C) {
  const long long nb = (long long)nslots * B * fr * 2;
  const long long total = nb + C;
  for (long long j = blockIdx.x * (long long)blockDim.x + threadIdx.x; j < total;
       j += (long long)gridDim.x * blockDim.x) {
    if (j < nb) {
      const int c = (int)(j & 1);
      const long long e = j >> 1;
      const int fl = (int)(e % fr);
      const long long sb = e / fr;
      const int f = rank * fr + fl;
      if (f < F) hist[(sb * F + f) * 2 + c] = out[j];
    } else {
      cnt[j - nb] = out[j];
    }
  }
}

static inline int grid_of(long long n) { return (int)std::min<long long>((n + 255) / 256, 256 * 8); }

}  // namespace ytk

using namespace ytk;

extern "C" {

// hist: the first of the nslots slots (slot stride B * F * 2 int64); cnt: C count words
// (0 when none); x: P * (nslots * B * fr * 2 + C) int64.
void ytk_owner_pack(uintptr_t hist, uintptr_t x, int nslots, int B, int F, int fr, int P, uintptr_t cnt, int C,
                    uintptr_t stream) {
  const long long total = ((long long)nslots * B * fr * 2 + C) * P;
  if (total <= 0) return;
  hipLaunchKernelGGL(owner_pack_kernel, dim3(grid_of(total)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     (const long long*)hist, (long long*)x, nslots, B, F, fr, P, (const long long*)cnt, C);
  YTK_LAUNCH_CHECK();
}

void ytk_owner_unpack(uintptr_t out, uintptr_t hist, int nslots, int B, int F, int fr, int rank, uintptr_t cnt, int C,
                      uintptr_t stream) {
  const long long total = (long long)nslots * B * fr * 2 + C;
  if (total <= 0) return;
  hipLaunchKernelGGL(owner_unpack_kernel, dim3(grid_of(total)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     (const long long*)out, (long long*)hist, nslots, B, F, fr, rank, (long long*)cnt, C);
  YTK_LAUNCH_CHECK();
}

}  // extern "C"
