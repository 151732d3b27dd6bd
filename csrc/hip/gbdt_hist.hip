// GBDT histogram build (gfx950 / CDNA4, wave64) -- exact int64 fixed point.
//
// Reference semantics: J/data/gbdt/HistogramBuilder.java:56-90 (sum of (g, h) per
// (feature, bin) over the rows of a node; the reference accumulates in double).
//
// Why fixed point: on gfx950 `ds_add_f32` measured ~33x slower than `ds_add_u32`
// for the same conflict-free pattern (profiles/hist_ablation.md). Each (g, h) is
// scaled by a per-tree power of two (2^k chosen so |sum over all rows| < 2^62) and
// rounded to int64 once; sums are then EXACT integers:
//   * deterministic and order independent (bitwise identical on 1 and N GPUs,
//     all-reduce of int64 is exact);
//   * parent - small child = large child exactly;
//   * resolution 2^-k ~ 1e-12 x max|g| -- finer than the fp32 gradients themselves.
//
// Layout / mapping:
//   * LDS: two int64 planes lds[bin][32] (g, h): 128 KiB at 256 bins, 1 block/CU,
//     1024 threads (16 waves).
//   * lane = (row r = lane/8, q = lane%8): one dword load = 4 features of a row, a
//     wave-instruction moves 8 rows x 32 B = 256 B; step k updates feature
//     4q + ((k + r) & 3) so the 32 lanes of each half-wave hit 32 distinct banks.
//   * (g, h) is read in POSITION order (the partition moves it with the row ids).
//   * One launch covers every node of a level: work[blk] = (slot, begin, end, 0).
//   * Block partials -> global int64 atomics (zero entries skipped).
#include "common.h"

#include <algorithm>
#include <stdexcept>

namespace ytk {

constexpr int kHistThreads = 1024;
constexpr int kHistU = 8;
constexpr int kHistUGather = 16; // gathered rows: more loads in flight per wave

template <bool kIdentity>
__global__ __launch_bounds__(kHistThreads) void hist_fx_kernel(
    const uint8_t* __restrict__ bins, long long stride, int F,
    const float2* __restrict__ ghp, const int* __restrict__ rows,
    const int4* __restrict__ work, long long* __restrict__ hist, int B, int nb_lds,
    float sg, float sh, const int* __restrict__ nwork_dev, const float* __restrict__ scales_dev,
    long long* __restrict__ staging, const int* __restrict__ work_off_dev) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long sm64[];
  unsigned long long* lg = sm64;
  unsigned long long* lh = sm64 + nb_lds * 32;
  // device-resident work count (fixed maximal grid launched by the level engine)
  // work_off_dev (optional): this launch covers work items [*work_off_dev, *nwork_dev) --
  // the second half of a level whose first half is already being all-reduced
  const int bx = (int)blockIdx.x + (work_off_dev ? *work_off_dev : 0);
  if (nwork_dev && bx >= *nwork_dev) return;
  if (scales_dev) {
    sg = scales_dev[0];
    sh = scales_dev[1];
  }
  const int4 w = work[bx];
  const int fg = blockIdx.y;
  const int tid = threadIdx.x;
  for (int i = tid; i < nb_lds * 64; i += kHistThreads) sm64[i] = 0ull;
  __syncthreads();

  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int wr = lane >> 3;  // row within the wave's 8
  const int q = lane & 7;    // dword (4 features) within the 32-B group segment
  constexpr int RW = (kHistThreads / 64) * 8;  // rows per block step
  const uint8_t* bseg = bins + fg * 32 + 4 * q;
  const int fbase = fg * 32 + 4 * q;
  constexpr int U = kIdentity ? kHistU : kHistUGather;
  for (int base = w.y + wave * 8; base < w.z; base += RW * U) {
    unsigned d[U];
    float2 v[U];
    bool ok[U];
#pragma unroll
    for (int j = 0; j < U; ++j) {
      const int pos = base + j * RW + wr;
      ok[j] = pos < w.z;
      const int p = ok[j] ? pos : w.y;
      const int r = kIdentity ? p : rows[p];
      d[j] = *reinterpret_cast<const unsigned*>(bseg + (size_t)(unsigned)r * stride);
      v[j] = ghp[p];
    }
#pragma unroll
    for (int j = 0; j < U; ++j) {
      if (!ok[j]) continue;
      const unsigned long long gi = (unsigned long long)__float2ll_rn(v[j].x * sg);
      const unsigned long long hi = (unsigned long long)__float2ll_rn(v[j].y * sh);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int c = (k + wr) & 3;
        const int bin = (d[j] >> (8 * c)) & 255;
        if (fbase + c < F) {
          atomicAdd(&lg[bin * 32 + 4 * q + c], gi);
          atomicAdd(&lh[bin * 32 + 4 * q + c], hi);
        }
      }
    }
  }
  __syncthreads();

  if (staging) {
    // two-stage flush: plain 16-B stores of this block's partial (g, h) pairs; the slot
    // sums are formed by hist_reduce_kernel. Global u64 atomics execute at the memory
    // side at ~1.3 TB/s chip-wide, which made the atomic flush the floor of every
    // launch (~45 us per level at 256 blocks); stores + one ordered read are ~4x cheaper.
    const int E = nb_lds * 32;
    longlong2* st = reinterpret_cast<longlong2*>(staging) + ((size_t)bx * gridDim.y + fg) * E;
    for (int i = tid; i < E; i += kHistThreads) st[i] = make_longlong2((long long)lg[i], (long long)lh[i]);
    return;
  }
  long long* out = hist + (size_t)w.x * B * F * 2;
  // Flush order rotated per block: every block of a level flushes into the SAME few
  // thousand addresses at about the same time; starting each block at a different
  // 1024-entry tile spreads the global atomics over the L2 channels instead of
  // serialising hundreds of blocks on one address at a time.
  const int E = nb_lds * 32;
  const int ntile = (E + kHistThreads - 1) / kHistThreads;
  const int rot = (int)((unsigned)bx % (unsigned)ntile);
  for (int t = 0; t < ntile; ++t) {
    const int i = ((t + rot) % ntile) * kHistThreads + tid;
    if (i >= E) continue;
    const int bin = i >> 5, l = i & 31, ff = fg * 32 + l;
    if (ff < F) {
      const unsigned long long g = lg[i], h = lh[i];
      if (g | h) {
        unsigned long long* o = reinterpret_cast<unsigned long long*>(&out[((size_t)bin * F + ff) * 2]);
        atomicAdd(o, g);
        atomicAdd(o + 1, h);
      }
    }
  }
}

// Second stage of the staged flush: hist[slot][bin][f] = sum over the work items of that
// slot of their block partials. One thread per (entry, slot, feature group); the items of
// the slot are collected into LDS first (<= 1024 items per level). Integer sums: exact and
// order independent. Every slot in [slot_base, slot_base + nslots) is written (zero when
// it has no items), so the built half of a level needs no zero fill.
// Split-K over the slot's items (blockIdx.z of kReduceSplit): each block sums a strided
// subset of the items with 8 independent 16-B loads in flight per thread and adds its
// partial with one int64 atomic per value (exact; kReduceSplit-way contention only).
// The slots must be zero on entry.
constexpr int kReduceSplit = 8;

__global__ __launch_bounds__(256) void hist_reduce_kernel(
    const long long* __restrict__ staging, const int4* __restrict__ work, int nwork,
    const int* __restrict__ nwork_dev, long long* __restrict__ hist, int B, int F, int nb_lds,
    int groups, int slot_base, const int* __restrict__ slot_ids) {
  __shared__ int s_sel[1024];
  __shared__ int s_wcnt[4];
  __shared__ int s_n;
  const int n = nwork_dev ? min(*nwork_dev, nwork) : nwork;
  // slot_ids (optional): explicit, possibly non-contiguous target slots (recycled slot pool)
  const int slot = slot_ids ? slot_ids[(int)blockIdx.y / groups] : slot_base + (int)blockIdx.y / groups;
  const int fg = (int)blockIdx.y % groups;
  // Ordered (stable) compaction of this slot's items: the kReduceSplit blocks of a slot
  // each take a strided subset s_sel[z], s_sel[z + 8], ..., so every block must see the
  // SAME order (an LDS-atomic compaction orders items differently per block whenever a
  // slot's items straddle waves, dropping and double counting items).
  // Fast path: every caller emits a slot's items contiguously -> one pass finds the
  // range [lo, hi] (min/max of matching indices) and the match count; contiguous iff
  // count == hi - lo + 1. Otherwise fall back to the ordered compaction below.
  __shared__ int s_lo, s_hi, s_cnt;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  if (tid == 0) { s_n = 0; s_lo = 0x7fffffff; s_hi = -1; s_cnt = 0; }
  __syncthreads();
  for (int k0 = 0; k0 < n; k0 += 256) {  // one LDS atomic per wave, not per item
    const int k = k0 + tid;
    const unsigned long long bal = __ballot(k < n && work[k].x == slot);
    if (lane == 0 && bal) {
      const int wbase = k0 + wid * 64;
      atomicMin(&s_lo, wbase + __ffsll((long long)bal) - 1);
      atomicMax(&s_hi, wbase + 63 - __clzll((long long)bal));
      atomicAdd(&s_cnt, __popcll(bal));
    }
  }
  __syncthreads();
  const bool contiguous = s_cnt == 0 || s_cnt == s_hi - s_lo + 1;
  if (contiguous) {
    if (tid == 0) s_n = s_cnt;
  }
  for (int k0 = 0; !contiguous && k0 < n; k0 += 256) {
    const int k = k0 + tid;
    const bool m = k < n && work[k].x == slot;
    const unsigned long long bal = __ballot(m);
    if (lane == 0) s_wcnt[wid] = __popcll(bal);
    __syncthreads();
    int off = s_n;
    for (int w = 0; w < wid; ++w) off += s_wcnt[w];
    const int p = off + __popcll(bal & ((lane == 0) ? 0ull : (~0ull >> (64 - lane))));
    if (m && p < 1024) s_sel[p] = k;
    __syncthreads();
    if (tid == 0) s_n += s_wcnt[0] + s_wcnt[1] + s_wcnt[2] + s_wcnt[3];
    __syncthreads();
  }
  __syncthreads();
  const int cnt = contiguous ? s_n : min(s_n, 1024);
  const int lo = s_lo;
  // t-th item of the slot
#define YTK_SEL(t) (contiguous ? lo + (t) : s_sel[(t)])
  const int E = nb_lds * 32;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= E || cnt == 0) return;
  const int bin = i >> 5, ff = fg * 32 + (i & 31);
  if (ff >= F || bin >= B) return;
  const longlong2* st = reinterpret_cast<const longlong2*>(staging);
  long long g = 0, h = 0;
  int t = (int)blockIdx.z;
  for (; t + 7 * kReduceSplit < cnt; t += 8 * kReduceSplit) {
    longlong2 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = st[((size_t)YTK_SEL(t + u * kReduceSplit) * groups + fg) * E + i];
#pragma unroll
    for (int u = 0; u < 8; ++u) { g += v[u].x; h += v[u].y; }
  }
  for (; t < cnt; t += kReduceSplit) {
    const longlong2 v = st[((size_t)YTK_SEL(t) * groups + fg) * E + i];
    g += v.x;
    h += v.y;
  }
  if (g | h) {
    unsigned long long* o = reinterpret_cast<unsigned long long*>(hist + (((size_t)slot * B + bin) * F + ff) * 2);
    atomicAdd(o, (unsigned long long)g);
    atomicAdd(o + 1, (unsigned long long)h);
  }
}
#undef YTK_SEL

// Generic histogram (uint8 or uint16 bins, any bin count): direct global int64
// atomics. Fallback for > 256 bins (e.g. the 5000-bin communication-stress config).
template <typename BinT>
__global__ __launch_bounds__(256) void hist_fx_global_kernel(
    const BinT* __restrict__ bins, long long stride, int F,
    const float2* __restrict__ ghp, const int* __restrict__ rows,
    const int4* __restrict__ work, long long* __restrict__ hist, int B, float sg, float sh) {
  const int4 w = work[blockIdx.x];
  const long long n = (long long)(w.z - w.y) * F;
  long long* out = hist + (size_t)w.x * B * F * 2;
  for (long long i = threadIdx.x; i < n; i += 256) {
    const int pos = w.y + (int)(i / F);
    const int f = (int)(i % F);
    const int r = rows ? rows[pos] : pos;
    const int b = bins[(long long)r * stride + f];
    const float2 v = ghp[pos];
    unsigned long long* o = reinterpret_cast<unsigned long long*>(&out[((size_t)b * F + f) * 2]);
    atomicAdd(o, (unsigned long long)__float2ll_rn(v.x * sg));
    atomicAdd(o + 1, (unsigned long long)__float2ll_rn(v.y * sh));
  }
}

// Wide-bin histogram (B > 256, uint16 bins -- e.g. the 5000-bin communication-stress
// config, docs/gbdt_experiments.md:156-168; reference loop HistogramBuilder.java:56-90).
// The 32-feature x B-bin LDS planes of hist_fx_kernel do not fit, so a block owns a
// GROUP of FG features (FG = floor(LDS budget / (B * 16 B)), >= 1) and reads their
// bins from the COLUMN-major matrix binsT [F][ncol] (2 B per row per feature,
// coalesced for the identity root, monotone row ids inside a node otherwise).
// LDS holds interleaved exact int64 (g, h) pairs lds[(f_in_group * B + bin) * 2 + {0,1}],
// accumulated with ds_add_u64 (same fixed point as hist_fx_kernel -> bitwise equal to
// the CPU path). Block partials are flushed with global int64 atomics, zero entries
// skipped (deep nodes touch few bins). grid = (work items, ceil(F / FG)).
constexpr int kWideThreads = 512;
constexpr int kWideU = 4;                    // rows in flight per thread
constexpr int kWideLdsBytes = 160 * 1024;    // one block per CU at the widest groups

template <bool kIdentity>
__global__ __launch_bounds__(kWideThreads) void hist_wide_kernel(
    const uint16_t* __restrict__ binsT, long long ncol, int F, int FG,
    const float2* __restrict__ ghp, const int* __restrict__ rows,
    const int4* __restrict__ work, long long* __restrict__ hist, int B,
    float sg, float sh, const int* __restrict__ nwork_dev, const float* __restrict__ scales_dev,
    const int* __restrict__ work_off_dev) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long wl[];
  const int bx = (int)blockIdx.x + (work_off_dev ? *work_off_dev : 0);
  if (nwork_dev && bx >= *nwork_dev) return;
  if (scales_dev) {
    sg = scales_dev[0];
    sh = scales_dev[1];
  }
  const int4 w = work[bx];
  const int f_lo = (int)blockIdx.y * FG;
  const int nf = min(FG, F - f_lo);
  const int tid = threadIdx.x;
  const int E = nf * B;
  for (int i = tid; i < 2 * E; i += kWideThreads) wl[i] = 0ull;
  __syncthreads();
  const uint16_t* col = binsT + (size_t)f_lo * ncol;
  for (int base = w.y + tid; base < w.z; base += kWideThreads * kWideU) {
    int r[kWideU];
    float2 v[kWideU];
    bool ok[kWideU];
#pragma unroll
    for (int j = 0; j < kWideU; ++j) {
      const int pos = base + j * kWideThreads;
      ok[j] = pos < w.z;
      const int p = ok[j] ? pos : w.y;
      r[j] = kIdentity ? p : rows[p];
      v[j] = ghp[p];
    }
#pragma unroll
    for (int j = 0; j < kWideU; ++j) {
      if (!ok[j]) continue;
      const unsigned long long gi = (unsigned long long)__float2ll_rn(v[j].x * sg);
      const unsigned long long hi = (unsigned long long)__float2ll_rn(v[j].y * sh);
      const uint16_t* c = col + (size_t)(unsigned)r[j];
      for (int fi = 0; fi < nf; ++fi) {
        const int bin = c[(size_t)fi * ncol];
        unsigned long long* e = &wl[(size_t)(fi * B + bin) * 2];
        atomicAdd(e, gi);
        atomicAdd(e + 1, hi);
      }
    }
  }
  __syncthreads();
  long long* out = hist + (size_t)w.x * B * F * 2;
  for (int i = tid; i < E; i += kWideThreads) {
    const unsigned long long g = wl[2 * i], h = wl[2 * i + 1];
    if (g | h) {
      const int fi = i / B, bin = i - fi * B;
      unsigned long long* o = reinterpret_cast<unsigned long long*>(&out[((size_t)bin * F + f_lo + fi) * 2]);
      atomicAdd(o, g);
      atomicAdd(o + 1, h);
    }
  }
}

}  // namespace ytk

using namespace ytk;

extern "C" {

int ytk_hist_wide_group(int B, int F);

// nwork_dev / scales_dev (optional): device-resident work count (grid = nwork is the
// maximum) and fixed-point scales, used by the GPU-resident level engine.
void ytk_hist_fx(uintptr_t bins, long long stride, int F, uintptr_t ghp, uintptr_t rows,
                 uintptr_t work, int nwork, uintptr_t hist, int B, float sg, float sh,
                 uintptr_t nwork_dev, uintptr_t scales_dev, uintptr_t stream) {
  if (nwork <= 0) return;
  const int groups = (F + 31) / 32;
  const int nb_lds = B;  // caller guarantees B <= 256
  const size_t lds = (size_t)nb_lds * 64 * sizeof(unsigned long long);
  dim3 grid(nwork, groups);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (rows == 0) {
    hipLaunchKernelGGL(hist_fx_kernel<true>, grid, dim3(kHistThreads), lds, s,
                       (const uint8_t*)bins, stride, F, (const float2*)ghp, (const int*)nullptr,
                       (const int4*)work, (long long*)hist, B, nb_lds, sg, sh,
                       (const int*)nwork_dev, (const float*)scales_dev, (long long*)nullptr,
                       (const int*)nullptr);
  } else {
    hipLaunchKernelGGL(hist_fx_kernel<false>, grid, dim3(kHistThreads), lds, s,
                       (const uint8_t*)bins, stride, F, (const float2*)ghp, (const int*)rows,
                       (const int4*)work, (long long*)hist, B, nb_lds, sg, sh,
                       (const int*)nwork_dev, (const float*)scales_dev, (long long*)nullptr,
                       (const int*)nullptr);
  }
  YTK_LAUNCH_CHECK();
}

// Staged variant: block partials to ``staging`` (>= nwork * groups * B * 32 * 16 bytes),
// then accumulated into the slots [slot_base, slot_base + nslots) -- or slot_ids[0..nslots)
// when given -- which must be zero.
void ytk_hist_fx_staged(uintptr_t bins, long long stride, int F, uintptr_t ghp, uintptr_t rows,
                        uintptr_t work, int nwork, uintptr_t hist, int B, float sg, float sh,
                        uintptr_t nwork_dev, uintptr_t scales_dev, uintptr_t staging,
                        int slot_base, int nslots, uintptr_t slot_ids, uintptr_t work_off_dev,
                        uintptr_t stream) {
  if (nwork <= 0 || nslots <= 0) return;
  const int groups = (F + 31) / 32;
  const int nb_lds = B;
  const size_t lds = (size_t)nb_lds * 64 * sizeof(unsigned long long);
  dim3 grid(nwork, groups);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (rows == 0) {
    hipLaunchKernelGGL(hist_fx_kernel<true>, grid, dim3(kHistThreads), lds, s,
                       (const uint8_t*)bins, stride, F, (const float2*)ghp, (const int*)nullptr,
                       (const int4*)work, (long long*)hist, B, nb_lds, sg, sh,
                       (const int*)nwork_dev, (const float*)scales_dev, (long long*)staging,
                       (const int*)work_off_dev);
  } else {
    hipLaunchKernelGGL(hist_fx_kernel<false>, grid, dim3(kHistThreads), lds, s,
                       (const uint8_t*)bins, stride, F, (const float2*)ghp, (const int*)rows,
                       (const int4*)work, (long long*)hist, B, nb_lds, sg, sh,
                       (const int*)nwork_dev, (const float*)scales_dev, (long long*)staging,
                       (const int*)work_off_dev);
  }
  YTK_LAUNCH_CHECK();
  const int E = nb_lds * 32;
  hipLaunchKernelGGL(hist_reduce_kernel, dim3((E + 255) / 256, nslots * groups, kReduceSplit), dim3(256), 0, s,
                     (const long long*)staging, (const int4*)work, nwork, (const int*)nwork_dev,
                     (long long*)hist, B, F, nb_lds, groups, slot_base, (const int*)slot_ids);
  YTK_LAUNCH_CHECK();
}

void ytk_hist_fx_global(uintptr_t bins, int bin_bytes, long long stride, int F, uintptr_t ghp,
                        uintptr_t rows, uintptr_t work, int nwork, uintptr_t hist, int B,
                        float sg, float sh, uintptr_t stream) {
  if (nwork <= 0) return;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (bin_bytes == 1) {
    hipLaunchKernelGGL(hist_fx_global_kernel<uint8_t>, dim3(nwork), dim3(256), 0, s,
                       (const uint8_t*)bins, stride, F, (const float2*)ghp, (const int*)rows,
                       (const int4*)work, (long long*)hist, B, sg, sh);
  } else {
    hipLaunchKernelGGL(hist_fx_global_kernel<uint16_t>, dim3(nwork), dim3(256), 0, s,
                       (const uint16_t*)bins, stride, F, (const float2*)ghp, (const int*)rows,
                       (const int4*)work, (long long*)hist, B, sg, sh);
  }
  YTK_LAUNCH_CHECK();
}

// Wide-bin histogram (uint16 binsT [F][ncol], any B up to the LDS budget of one feature:
// B * 16 <= 160 KiB). Target slots must be zero. Returns the feature-group size used.
int ytk_hist_wide(uintptr_t binsT, long long ncol, int F, uintptr_t ghp, uintptr_t rows,
                  uintptr_t work, int nwork, uintptr_t hist, int B, float sg, float sh,
                  uintptr_t nwork_dev, uintptr_t scales_dev, uintptr_t work_off_dev,
                  uintptr_t stream) {
  const int FG = ytk_hist_wide_group(B, F);
  if (FG <= 0) throw std::invalid_argument("hist_wide: one feature's bins exceed the LDS budget");
  if (nwork <= 0) return FG;
  const size_t lds = (size_t)FG * B * 2 * sizeof(unsigned long long);
  dim3 grid(nwork, (F + FG - 1) / FG);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (rows == 0) {
    hipLaunchKernelGGL(hist_wide_kernel<true>, grid, dim3(kWideThreads), lds, s, (const uint16_t*)binsT,
                       ncol, F, FG, (const float2*)ghp, (const int*)nullptr, (const int4*)work,
                       (long long*)hist, B, sg, sh, (const int*)nwork_dev, (const float*)scales_dev,
                       (const int*)work_off_dev);
  } else {
    hipLaunchKernelGGL(hist_wide_kernel<false>, grid, dim3(kWideThreads), lds, s, (const uint16_t*)binsT,
                       ncol, F, FG, (const float2*)ghp, (const int*)rows, (const int4*)work,
                       (long long*)hist, B, sg, sh, (const int*)nwork_dev, (const float*)scales_dev,
                       (const int*)work_off_dev);
  }
  YTK_LAUNCH_CHECK();
  return FG;
}

// Features per block of hist_wide_kernel (0: a single feature does not fit).
int ytk_hist_wide_group(int B, int F) {
  const long long per = (long long)B * 16;
  if (B <= 0 || per > kWideLdsBytes) return 0;
  return (int)std::min<long long>(F, kWideLdsBytes / per);
}

}  // extern "C"
