// L1 (least-absolute-deviation) leaf refinement on the device (gfx950).
//
// Reference: J/optimizer/gbdt/TreeRefiner.java:72-254 -- every leaf value becomes
// learning_rate x the weighted median of the residuals (label - score) of its rows:
// getLeafRefineValForLADPrecise (exact, PreciseQuantile.java:237-320) or
// getLeafRefineValForLADAppr (WeightApproximateQuantile summaries, eps 1e-5).
//
// The caller (models/gbdt/refine.py) sorts the rows by (leaf, residual) on the device and
// merges equal residuals of a leaf into entries (value v, weight wx), with each entry's
// rank interval inside its leaf (rmin, rmax = rmin + wx): exactly WQSummary::from_sorted
// per leaf (csrc/native/wquantile.cpp). Leaf s owns entries [seg[s], seg[s + 1]). These
// kernels then answer, per leaf, without copying a row to the host:
//   exact  (mode 0): the first entry whose rmax >= W / 2 (the sorted weighted median);
//   approx (mode 1): WQSummary::query(W / 2) on the leaf's summary PRUNED to `size`
//          entries when it holds more (WQSummary::prune) -- the pruned entry of target k is
//          a pure function of k (nearest entry to rank W k / (size - 1)), so the query
//          binary-searches k and never materialises the pruned summary.
// seg_prune_kernel materialises pruned summaries (multi-GPU approximate mode: the per-rank
// summaries are exchanged and merged like the reference's allreduceMap).
#include "common.h"

namespace ytk {

// first index i in [lo, hi) with a[i] >= x (hi if none); a non-decreasing on [lo, hi)
__device__ __forceinline__ long long lower_bound_d(const double* a, long long lo, long long hi, double x) {
  while (lo < hi) {
    const long long m = (lo + hi) >> 1;
    if (a[m] < x) lo = m + 1; else hi = m;
  }
  return lo;
}

// entry of target k (1 <= k <= size - 2) of WQSummary::prune on entries [b, b + n) of
// mid = (rmin + rmax) / 2 (leaf-local ranks), total W; returned as an offset from b
__device__ __forceinline__ long long prune_pick(const double* mid, long long b, long long n, double W, int size,
                                                long long k) {
  const double d = W * (double)k / (double)(size - 1);
  long long i = lower_bound_d(mid, b + 1, b + n, d) - b;  // first index >= 1 with mid >= d
  if (i > n - 1) i = n - 1;
  long long j = i;
  if (i > 1) {
    const double a = fabs(mid[b + i - 1] - d);
    const double c = fabs(mid[b + i] - d);
    if (a < c) j = i - 1;
  }
  return j;
}

__global__ __launch_bounds__(256) void seg_median_kernel(const double* __restrict__ v, const double* __restrict__ rmin,
                                                         const double* __restrict__ rmax, const double* __restrict__ mid,
                                                         const long long* __restrict__ seg, int nseg, int mode,
                                                         int size, double* __restrict__ out) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nseg) return;
  const long long b = seg[s], e = seg[s + 1], n = e - b;
  if (n <= 0) {
    out[s] = __builtin_nan("");
    return;
  }
  const double W = rmax[e - 1];
  if (mode == 0) {  // first entry with cumulative weight >= W / 2
    long long i = lower_bound_d(rmax, b, e, 0.5 * W);
    if (i >= e) i = e - 1;
    out[s] = v[i];
    return;
  }
  // WQSummary::query(rank = W / 2): d2 = 2 rank = W against rmin + rmax = 2 mid
  const double d2 = W;
  auto m2 = [&](long long i) { return rmin[i] + rmax[i]; };
  if (d2 <= m2(b)) { out[s] = v[b]; return; }
  if (d2 >= m2(e - 1)) { out[s] = v[e - 1]; return; }
  if (n <= size || size < 3) {
    long long lo = b, hi = e - 1;  // first entry with m2 >= d2 (exists: the last one)
    while (lo < hi) {
      const long long m = (lo + hi) >> 1;
      if (m2(m) < d2) lo = m + 1; else hi = m;
    }
    const double a = d2 - m2(lo - 1), c = m2(lo) - d2;
    out[s] = (a < c) ? v[lo - 1] : v[lo];
    return;
  }
  // pruned summary: seq[0] = 0, seq[t] = prune_pick(t) (1 <= t <= size - 2), seq[size - 1] = n - 1
  // (non-decreasing in t); first t with m2(seq[t]) >= d2, then its predecessor seq[t - 1]
  auto seq = [&](long long t) -> long long {
    if (t <= 0) return 0;
    if (t >= size - 1) return n - 1;
    return prune_pick(mid, b, n, W, size, t);
  };
  long long lo = 1, hi = size - 1;  // seq[0] fails (d2 > m2(b)), seq[size - 1] passes
  while (lo < hi) {
    const long long m = (lo + hi) >> 1;
    if (m2(b + seq(m)) < d2) lo = m + 1; else hi = m;
  }
  const long long jl = b + seq(lo), jp = b + seq(lo - 1);
  const double a = d2 - m2(jp), c = m2(jl) - d2;
  out[s] = (a < c) ? v[jp] : v[jl];
}

// pick[q] for q over the pruned leaves' targets: leaf list[q / per], k = q % per + 1
// (per = size - 2): the ENTRY index (global) WQSummary::prune keeps for that target
__global__ __launch_bounds__(256) void seg_prune_kernel(const double* __restrict__ mid, const double* __restrict__ rmax,
                                                        const long long* __restrict__ seg,
                                                        const int* __restrict__ leaves, int nleaves, int size,
                                                        long long* __restrict__ pick) {
  const long long per = size - 2;
  const long long total = per * nleaves;
  for (long long q = blockIdx.x * (long long)blockDim.x + threadIdx.x; q < total;
       q += (long long)gridDim.x * blockDim.x) {
    const int s = leaves[q / per];
    const long long k = q % per + 1;
    const long long b = seg[s], n = seg[s + 1] - b;
    pick[q] = b + prune_pick(mid, b, n, rmax[b + n - 1], size, k);
  }
}

}  // namespace ytk

using namespace ytk;

extern "C" {

void ytk_seg_median(uintptr_t v, uintptr_t rmin, uintptr_t rmax, uintptr_t mid, uintptr_t seg, int nseg, int mode,
                    int size, uintptr_t out, uintptr_t stream) {
  if (nseg <= 0) return;
  hipLaunchKernelGGL(seg_median_kernel, dim3((nseg + 255) / 256), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     (const double*)v, (const double*)rmin, (const double*)rmax, (const double*)mid,
                     (const long long*)seg, nseg, mode, size, (double*)out);
  YTK_LAUNCH_CHECK();
}

void ytk_seg_prune(uintptr_t mid, uintptr_t rmax, uintptr_t seg, uintptr_t leaves, int nleaves, int size,
                   uintptr_t pick, uintptr_t stream) {
  if (nleaves <= 0 || size < 3) return;
  const long long total = (long long)(size - 2) * nleaves;
  const int grid = (int)std::min<long long>((total + 255) / 256, 256 * 16);
  hipLaunchKernelGGL(seg_prune_kernel, dim3(grid), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     (const double*)mid, (const double*)rmax, (const long long*)seg, (const int*)leaves, nleaves, size,
                     (long long*)pick);
  YTK_LAUNCH_CHECK();
}

}  // extern "C"
