// GBDT histogram build (gfx950 / CDNA4, wave64).
//
// Reference semantics: J/data/gbdt/HistogramBuilder.java:56-90 (sum of (g, h) per
// (feature, bin) over the rows of a node).
//
// Design:
//  * FEATURE-MINOR LDS layout lds[bin][32]: the 32 lanes of a half-wave own the
//    32 features of one row, so the bank of every ds_add_f32 is the feature lane.
//    A wave-instruction updates 2 rows x 32 features with zero bank conflicts
//    whatever the (random) bin values are. g and h are two 32 KiB planes.
//  * 1024-thread blocks, 64 KiB LDS -> 2 blocks = 32 waves per CU. Each half-wave
//    keeps kHistU rows in flight (row id, 32-B bin-row segment, position-ordered
//    (g, h)): ~20 KiB of loads outstanding per CU. (A first 256-thread / 4-rows
//    version was latency bound at ~115 GB/s -- profiles/README.md.)
//  * (g, h) is read in POSITION order (the partition kernel permutes it together
//    with the row ids), so the only gather left is the 32-B bin-row segment.
//  * One launch covers every node of a level: work[blk] = (slot, begin, end, 0).
//  * Block partials are merged with no-return global f32 atomics into
//    hist[slot][B][F] (float2 g,h interleaved), zero bins skipped.
#include "common.h"

namespace ytk {

constexpr int kHistThreads = 1024;
constexpr int kHistU = 8;

template <bool kIdentity>
__global__ __launch_bounds__(kHistThreads) void hist_u8_lds_kernel(
    const uint8_t* __restrict__ bins, long long stride, int F,
    const float2* __restrict__ ghp, const int* __restrict__ rows,
    const int4* __restrict__ work, float2* __restrict__ hist, int B, int nb_lds) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* lg = smem;
  float* lh = smem + nb_lds * 32;
  const int4 w = work[blockIdx.x];
  const int fg = blockIdx.y;
  const int tid = threadIdx.x;
  for (int i = tid; i < nb_lds * 64; i += kHistThreads) smem[i] = 0.f;
  __syncthreads();

  constexpr int HW = kHistThreads / 32;
  const int hw = tid >> 5;  // half-wave -> row offset
  const int fl = tid & 31;  // feature lane
  const int f = fg * 32 + fl;
  const bool active = f < F;
  const uint8_t* bcol = bins + fg * 32 + fl;
  const int end = w.z;
  int pos = w.y + hw;
  for (; pos + HW * (kHistU - 1) < end; pos += HW * kHistU) {
    int r[kHistU], b[kHistU];
    float2 v[kHistU];
#pragma unroll
    for (int j = 0; j < kHistU; ++j) r[j] = kIdentity ? pos + HW * j : rows[pos + HW * j];
#pragma unroll
    for (int j = 0; j < kHistU; ++j) {
      b[j] = bcol[(size_t)(unsigned)r[j] * stride];
      v[j] = ghp[pos + HW * j];
    }
    if (active) {
#pragma unroll
      for (int j = 0; j < kHistU; ++j) {
        atomicAdd(&lg[b[j] * 32 + fl], v[j].x);
        atomicAdd(&lh[b[j] * 32 + fl], v[j].y);
      }
    }
  }
  for (; pos < end; pos += HW) {
    const int r = kIdentity ? pos : rows[pos];
    const int b = bcol[(size_t)(unsigned)r * stride];
    const float2 v = ghp[pos];
    if (active) { atomicAdd(&lg[b * 32 + fl], v.x); atomicAdd(&lh[b * 32 + fl], v.y); }
  }
  __syncthreads();

  float2* out = hist + (size_t)w.x * B * F;
  for (int i = tid; i < nb_lds * 32; i += kHistThreads) {
    const int bin = i >> 5, l = i & 31, ff = fg * 32 + l;
    if (ff < F) {
      const float g = lg[i], h = lh[i];
      if (g != 0.f || h != 0.f) {
        float* o = reinterpret_cast<float*>(&out[(size_t)bin * F + ff]);
        atomicAdd(o, g);
        atomicAdd(o + 1, h);
      }
    }
  }
}

// Generic histogram (uint8 or uint16 bins, any bin count): direct global atomics.
// Fallback for > 256 bins (e.g. the 5000-bin communication-stress config).
template <typename BinT>
__global__ __launch_bounds__(256) void hist_global_kernel(
    const BinT* __restrict__ bins, long long stride, int F,
    const float2* __restrict__ ghp, const int* __restrict__ rows,
    const int4* __restrict__ work, float2* __restrict__ hist, int B) {
  const int4 w = work[blockIdx.x];
  const long long n = (long long)(w.z - w.y) * F;
  float2* out = hist + (size_t)w.x * B * F;
  for (long long i = threadIdx.x; i < n; i += 256) {
    const int pos = w.y + (int)(i / F);
    const int f = (int)(i % F);
    const int r = rows ? rows[pos] : pos;
    const int b = bins[(long long)r * stride + f];
    const float2 v = ghp[pos];
    float* o = reinterpret_cast<float*>(&out[(size_t)b * F + f]);
    atomicAdd(o, v.x);
    atomicAdd(o + 1, v.y);
  }
}

}  // namespace ytk

using namespace ytk;

extern "C" {

void ytk_hist_u8(uintptr_t bins, long long stride, int F, uintptr_t ghp, uintptr_t rows,
                 uintptr_t work, int nwork, uintptr_t hist, int B, uintptr_t stream) {
  if (nwork <= 0) return;
  const int groups = (F + 31) / 32;
  const int nb_lds = B;  // caller guarantees B <= 256
  const size_t lds = (size_t)nb_lds * 64 * sizeof(float);
  dim3 grid(nwork, groups);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (rows == 0) {
    hipLaunchKernelGGL(hist_u8_lds_kernel<true>, grid, dim3(kHistThreads), lds, s,
                       (const uint8_t*)bins, stride, F, (const float2*)ghp, (const int*)nullptr,
                       (const int4*)work, (float2*)hist, B, nb_lds);
  } else {
    hipLaunchKernelGGL(hist_u8_lds_kernel<false>, grid, dim3(kHistThreads), lds, s,
                       (const uint8_t*)bins, stride, F, (const float2*)ghp, (const int*)rows,
                       (const int4*)work, (float2*)hist, B, nb_lds);
  }
  YTK_LAUNCH_CHECK();
}

void ytk_hist_global(uintptr_t bins, int bin_bytes, long long stride, int F, uintptr_t ghp,
                     uintptr_t rows, uintptr_t work, int nwork, uintptr_t hist, int B,
                     uintptr_t stream) {
  if (nwork <= 0) return;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (bin_bytes == 1) {
    hipLaunchKernelGGL(hist_global_kernel<uint8_t>, dim3(nwork), dim3(256), 0, s,
                       (const uint8_t*)bins, stride, F, (const float2*)ghp, (const int*)rows,
                       (const int4*)work, (float2*)hist, B);
  } else {
    hipLaunchKernelGGL(hist_global_kernel<uint16_t>, dim3(nwork), dim3(256), 0, s,
                       (const uint16_t*)bins, stride, F, (const float2*)ghp, (const int*)rows,
                       (const int4*)work, (float2*)hist, B);
  }
  YTK_LAUNCH_CHECK();
}

}  // extern "C"
