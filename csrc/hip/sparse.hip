// Sparse products for the L-BFGS model family (gfx950 / CDNA4, wave64).
//
// Reference hot loops:
//   z = X w (CSR SpMV)               J/optimizer/LinearHoagOptimizer.java:76-87
//   g = X^T (weight * l')            LinearHoagOptimizer.java:89-106
//   S = X W, G = X^T D (J columns)   MulticlassLinearHoagOptimizer.java:82-149,
//                                    FMHoagOptimizer.java:88-160, GBMLRHoagOptimizer.java:130-243
//   precision diag(X^T D X)          LinearHoagOptimizer.java:179-206
//
// One kernel covers all of them: a "segment" is a contiguous range [beg, end) of an
// index/value list; out[s, j] = sum_k val[k] * X[idx[k], j] (optionally val^2).
//  * CSR rows as segments -> X W.
//  * CSC column CHUNKS as segments -> partial sums of X^T D; a second kernel adds each
//    column's chunk partials in a fixed order. Long columns (the bias column holds every
//    row) are split into fixed-size chunks so the work is balanced, and no float atomics
//    are used anywhere: results are bitwise deterministic run to run and across GPU counts
//    (the reference's thread-order summation is not).
// Lane mapping: L lanes per segment (L = 64 / segments-per-wave). For J == 1 the L lanes
// split the nnz of a segment and finish with a shuffle tree; for J > 1 the lanes split the
// J output columns (coalesced gathers of W rows) and loop over the nnz.
#include "common.h"

namespace ytk {

template <int L, bool kSquare>
__global__ __launch_bounds__(256) void seg_spmv_kernel(
    const long long* __restrict__ beg, const long long* __restrict__ end, int nseg,
    const int* __restrict__ idx, const float* __restrict__ val, const float* __restrict__ x,
    float* __restrict__ out, float alpha, int accumulate) {
  const int gl = blockIdx.x * blockDim.x + threadIdx.x;
  const int seg = gl / L;
  const int sub = gl % L;
  if (seg >= nseg) return;  // whole groups exit together (L divides 64)
  const long long b = beg[seg], e = end[seg];
  float acc = 0.f;
  for (long long k = b + sub; k < e; k += L) {
    const float v = val ? val[k] : 1.f;
    acc += (kSquare ? v * v : v) * x[idx[k]];
  }
#pragma unroll
  for (int off = L / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off, L);
  if (sub == 0) out[seg] = accumulate ? out[seg] + alpha * acc : alpha * acc;
}

template <int L, bool kSquare>
__global__ __launch_bounds__(256) void seg_spmm_kernel(
    const long long* __restrict__ beg, const long long* __restrict__ end, int nseg,
    const int* __restrict__ idx, const float* __restrict__ val, const float* __restrict__ X,
    long long ldx, int J, float* __restrict__ out, long long ldo, float alpha, int accumulate) {
  const int gl = blockIdx.x * blockDim.x + threadIdx.x;
  const int seg = gl / L;
  const int sub = gl % L;
  if (seg >= nseg) return;
  const long long b = beg[seg], e = end[seg];
  for (int j0 = 0; j0 < J; j0 += L) {
    const int j = j0 + sub;
    float acc = 0.f;
    if (j < J) {
      for (long long k = b; k < e; ++k) {
        const float v = val ? val[k] : 1.f;
        acc += (kSquare ? v * v : v) * X[(long long)idx[k] * ldx + j];
      }
      float* o = out + (long long)seg * ldo + j;
      *o = accumulate ? *o + alpha * acc : alpha * acc;
    }
  }
}

// out[col, :] (+)= alpha * sum_{c in chunks of col, in order} part[c, :]
__global__ __launch_bounds__(256) void chunk_reduce_kernel(
    const long long* __restrict__ cbeg, int ncol, const float* __restrict__ part, int J,
    float* __restrict__ out, long long ldo, float alpha, int accumulate) {
  const long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (t >= (long long)ncol * J) return;
  const int col = (int)(t / J), j = (int)(t % J);
  float acc = 0.f;
  for (long long c = cbeg[col]; c < cbeg[col + 1]; ++c) acc += part[c * J + j];
  float* o = out + (long long)col * ldo + j;
  *o = accumulate ? *o + alpha * acc : alpha * acc;
}

}  // namespace ytk

using namespace ytk;

template <bool kSquare>
static void launch_spmv(int L, const long long* beg, const long long* end, int nseg, const int* idx,
                        const float* val, const float* x, float* out, float alpha, int acc,
                        hipStream_t s) {
  const long long threads = (long long)nseg * L;
  const int grid = (int)((threads + 255) / 256);
#define YTK_SPMV(LL)                                                                         \
  hipLaunchKernelGGL((seg_spmv_kernel<LL, kSquare>), dim3(grid), dim3(256), 0, s, beg, end, \
                     nseg, idx, val, x, out, alpha, acc)
  switch (L) {
    case 1: YTK_SPMV(1); break;
    case 2: YTK_SPMV(2); break;
    case 4: YTK_SPMV(4); break;
    case 8: YTK_SPMV(8); break;
    case 16: YTK_SPMV(16); break;
    case 32: YTK_SPMV(32); break;
    default: YTK_SPMV(64); break;
  }
#undef YTK_SPMV
}

template <bool kSquare>
static void launch_spmm(int L, const long long* beg, const long long* end, int nseg, const int* idx,
                        const float* val, const float* X, long long ldx, int J, float* out,
                        long long ldo, float alpha, int acc, hipStream_t s) {
  const long long threads = (long long)nseg * L;
  const int grid = (int)((threads + 255) / 256);
#define YTK_SPMM(LL)                                                                         \
  hipLaunchKernelGGL((seg_spmm_kernel<LL, kSquare>), dim3(grid), dim3(256), 0, s, beg, end, \
                     nseg, idx, val, X, ldx, J, out, ldo, alpha, acc)
  switch (L) {
    case 1: YTK_SPMM(1); break;
    case 2: YTK_SPMM(2); break;
    case 4: YTK_SPMM(4); break;
    case 8: YTK_SPMM(8); break;
    case 16: YTK_SPMM(16); break;
    case 32: YTK_SPMM(32); break;
    default: YTK_SPMM(64); break;
  }
#undef YTK_SPMM
}

extern "C" {

// out[s, 0:J] (=|+=) alpha * sum_{k in seg s} f(val[k]) * X[idx[k], 0:J]; f = id or square.
void ytk_seg_spmm(uintptr_t beg, uintptr_t end, int nseg, uintptr_t idx, uintptr_t val,
                  uintptr_t X, long long ldx, int J, uintptr_t out, long long ldo, float alpha,
                  int accumulate, int square, int lanes, uintptr_t stream) {
  if (nseg <= 0 || J <= 0) return;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int L = 1;
  while (L < lanes && L < 64) L <<= 1;
  if (J == 1) {
    if (square)
      launch_spmv<true>(L, (const long long*)beg, (const long long*)end, nseg, (const int*)idx,
                        (const float*)val, (const float*)X, (float*)out, alpha, accumulate, s);
    else
      launch_spmv<false>(L, (const long long*)beg, (const long long*)end, nseg, (const int*)idx,
                         (const float*)val, (const float*)X, (float*)out, alpha, accumulate, s);
  } else {
    if (square)
      launch_spmm<true>(L, (const long long*)beg, (const long long*)end, nseg, (const int*)idx,
                        (const float*)val, (const float*)X, ldx, J, (float*)out, ldo, alpha,
                        accumulate, s);
    else
      launch_spmm<false>(L, (const long long*)beg, (const long long*)end, nseg, (const int*)idx,
                         (const float*)val, (const float*)X, ldx, J, (float*)out, ldo, alpha,
                         accumulate, s);
  }
  YTK_LAUNCH_CHECK();
}

void ytk_chunk_reduce(uintptr_t cbeg, int ncol, uintptr_t part, int J, uintptr_t out,
                      long long ldo, float alpha, int accumulate, uintptr_t stream) {
  if (ncol <= 0 || J <= 0) return;
  const long long n = (long long)ncol * J;
  hipLaunchKernelGGL(chunk_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), (const long long*)cbeg, ncol,
                     (const float*)part, J, (float*)out, ldo, alpha, accumulate);
  YTK_LAUNCH_CHECK();
}

}  // extern "C"
