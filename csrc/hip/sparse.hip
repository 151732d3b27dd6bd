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

// J == 1: each lane takes the segment's entries sub, sub + L, ... in steps of 4L with all
// four index loads, value loads and x gathers of a step issued together (predicated),
// four independent accumulators; kOnes: one-hot values (every stored value is 1, e.g. the
// Criteo categorical fields) are not read at all. The lane count per segment is chosen
// on the host from the mean segment length (~4 entries per lane).
template <int L, bool kSquare, bool kOnes>
__global__ __launch_bounds__(256) void seg_spmv_kernel(
    const long long* __restrict__ beg, const long long* __restrict__ end, int nseg,
    const int* __restrict__ idx, const float* __restrict__ val, const float* __restrict__ x,
    float* __restrict__ out, float alpha, int accumulate, const int* __restrict__ perm) {
  const int gl = blockIdx.x * blockDim.x + threadIdx.x;
  const int sg = gl / L;
  const int sub = gl % L;
  if (sg >= nseg) return;  // whole groups exit together (L divides 64)
  // perm (optional): the launch covers segments perm[0..nseg) -- length buckets of the CSC
  // chunks, each launched with its own lane count
  const int seg = perm ? perm[sg] : sg;
  const long long b = beg[seg], e = end[seg];
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (long long k = b + sub; k < e; k += 4 * L) {
    int i[4];
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const long long kk = k + u * L;
      const bool ok = kk < e;
      i[u] = ok ? idx[kk] : 0;
      v[u] = ok ? (kOnes ? 1.f : val[kk]) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] += (kSquare ? v[u] * v[u] : v[u]) * x[i[u]];
  }
  float a = (acc[0] + acc[1]) + (acc[2] + acc[3]);
#pragma unroll
  for (int off = L / 2; off > 0; off >>= 1) a += __shfl_xor(a, off, L);
  if (sub == 0) out[seg] = accumulate ? out[seg] + alpha * a : alpha * a;
}

template <int L, bool kSquare>
__global__ __launch_bounds__(256) void seg_spmm_kernel(
    const long long* __restrict__ beg, const long long* __restrict__ end, int nseg,
    const int* __restrict__ idx, const float* __restrict__ val, const float* __restrict__ X,
    long long ldx, int J, float* __restrict__ out, long long ldo, float alpha, int accumulate,
    const int* __restrict__ perm) {
  const int gl = blockIdx.x * blockDim.x + threadIdx.x;
  const int sg = gl / L;
  const int sub = gl % L;
  if (sg >= nseg) return;
  const int seg = perm ? perm[sg] : sg;
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
// ids (optional): the chunk numbers of column col are ids[cbeg[col] .. cbeg[col + 1]) (row-
// tiled CSC: a column's chunks are spread over the tiles); otherwise they are contiguous.
__global__ __launch_bounds__(256) void chunk_reduce_kernel(
    const long long* __restrict__ cbeg, int ncol, const float* __restrict__ part, int J,
    float* __restrict__ out, long long ldo, float alpha, int accumulate, const long long* __restrict__ ids) {
  const long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (t >= (long long)ncol * J) return;
  const int col = (int)(t / J), j = (int)(t % J);
  float acc = 0.f;
  for (long long c = cbeg[col]; c < cbeg[col + 1]; ++c) acc += part[(ids ? ids[c] : c) * J + j];
  float* o = out + (long long)col * ldo + j;
  *o = accumulate ? *o + alpha * acc : alpha * acc;
}

}  // namespace ytk

using namespace ytk;

template <bool kSquare, bool kOnes>
static void launch_spmv(int L, const long long* beg, const long long* end, int nseg, const int* idx,
                        const float* val, const float* x, float* out, float alpha, int acc,
                        const int* perm, hipStream_t s) {
  const long long threads = (long long)nseg * L;
  const int grid = (int)((threads + 255) / 256);
#define YTK_SPMV(LL)                                                                                  \
  hipLaunchKernelGGL((seg_spmv_kernel<LL, kSquare, kOnes>), dim3(grid), dim3(256), 0, s, beg, end, \
                     nseg, idx, val, x, out, alpha, acc, perm)
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
                        long long ldo, float alpha, int acc, const int* perm, hipStream_t s) {
  const long long threads = (long long)nseg * L;
  const int grid = (int)((threads + 255) / 256);
#define YTK_SPMM(LL)                                                                         \
  hipLaunchKernelGGL((seg_spmm_kernel<LL, kSquare>), dim3(grid), dim3(256), 0, s, beg, end, \
                     nseg, idx, val, X, ldx, J, out, ldo, alpha, acc, perm)
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
// perm (optional, int32 [nseg]): segment ids covered by this launch.
void ytk_seg_spmm(uintptr_t beg, uintptr_t end, int nseg, uintptr_t idx, uintptr_t val,
                  uintptr_t X, long long ldx, int J, uintptr_t out, long long ldo, float alpha,
                  int accumulate, int square, int lanes, uintptr_t perm, uintptr_t stream) {
  if (nseg <= 0 || J <= 0) return;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int L = 1;
  while (L < lanes && L < 64) L <<= 1;
  if (J == 1) {
    // val == 0: one-hot matrix (all values 1) -- the values are never read
#define YTK_SPMV_L(SQ, ON)                                                                      \
  launch_spmv<SQ, ON>(L, (const long long*)beg, (const long long*)end, nseg, (const int*)idx,  \
                      (const float*)val, (const float*)X, (float*)out, alpha, accumulate, (const int*)perm, s)
    if (val == 0) {
      YTK_SPMV_L(false, true);  // 1^2 == 1: square is the same product
    } else if (square) {
      YTK_SPMV_L(true, false);
    } else {
      YTK_SPMV_L(false, false);
    }
#undef YTK_SPMV_L
  } else {
    if (square)
      launch_spmm<true>(L, (const long long*)beg, (const long long*)end, nseg, (const int*)idx,
                        (const float*)val, (const float*)X, ldx, J, (float*)out, ldo, alpha,
                        accumulate, (const int*)perm, s);
    else
      launch_spmm<false>(L, (const long long*)beg, (const long long*)end, nseg, (const int*)idx,
                         (const float*)val, (const float*)X, ldx, J, (float*)out, ldo, alpha,
                         accumulate, (const int*)perm, s);
  }
  YTK_LAUNCH_CHECK();
}

void ytk_chunk_reduce(uintptr_t cbeg, int ncol, uintptr_t part, int J, uintptr_t out,
                      long long ldo, float alpha, int accumulate, uintptr_t ids, uintptr_t stream) {
  if (ncol <= 0 || J <= 0) return;
  const long long n = (long long)ncol * J;
  hipLaunchKernelGGL(chunk_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), (const long long*)cbeg, ncol,
                     (const float*)part, J, (float*)out, ldo, alpha, accumulate, (const long long*)ids);
  YTK_LAUNCH_CHECK();
}

}  // extern "C"
