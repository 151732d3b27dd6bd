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

#include <stdexcept>

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
    if (j < J) {
      // 8 entries per step: their index / value loads, then their 8 row gathers, all in
      // flight together (one entry at a time left the kernel two dependent round trips per
      // entry: 8.8 -> 5.0 ms for a 164M-entry J = 32 product; 16 predicated entries per step
      // measured no better)
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
      long long k = b;
      for (; k + 8 <= e; k += 8) {
        int ii[8];
        float vv[8], xv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          ii[u] = idx[k + u];
          vv[u] = val ? val[k + u] : 1.f;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) xv[u] = X[(long long)ii[u] * ldx + j];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc[u & 3] += (kSquare ? vv[u] * vv[u] : vv[u]) * xv[u];
      }
      for (; k < e; ++k) {
        const float v = val ? val[k] : 1.f;
        acc[0] += (kSquare ? v * v : v) * X[(long long)idx[k] * ldx + j];
      }
      const float a = (acc[0] + acc[1]) + (acc[2] + acc[3]);
      float* o = out + (long long)seg * ldo + j;
      *o = accumulate ? *o + alpha * a : alpha * a;
    }
  }
}

// out[col, :] (+)= alpha * sum_{c in chunks of col, in order} part[c, :]
// ids (optional): the chunk numbers of column col are ids[cbeg[col] .. cbeg[col + 1]) (row-
// tiled CSC: a column's chunks are spread over the tiles); otherwise they are contiguous.
__global__ __launch_bounds__(256) void chunk_reduce_kernel(
    const long long* __restrict__ cbeg, int ncol, const float* __restrict__ part, int J,
    float* __restrict__ out, long long ldo, float alpha, int accumulate, const long long* __restrict__ ids,
    int skip_heavy) {
  const long long t = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  if (t >= (long long)ncol * J) return;
  const int col = (int)(t / J), j = (int)(t % J);
  if (skip_heavy && cbeg[col + 1] - cbeg[col] > 16) return;  // chunk_reduce_heavy_kernel's (kReduceLight)
  // 4 chunks per step in flight (ids, then the partials)
  float a4[4] = {0.f, 0.f, 0.f, 0.f};
  const long long c1 = cbeg[col + 1];
  long long c = cbeg[col];
  for (; c + 4 <= c1; c += 4) {
    long long q[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) q[u] = ids ? ids[c + u] : c + u;
#pragma unroll
    for (int u = 0; u < 4; ++u) a4[u] += part[q[u] * J + j];
  }
  for (; c < c1; ++c) a4[0] += part[(ids ? ids[c] : c) * J + j];
  const float acc = (a4[0] + a4[1]) + (a4[2] + a4[3]);
  float* o = out + (long long)col * ldo + j;
  *o = accumulate ? *o + alpha * acc : alpha * acc;
}

// ---------------------------------------------------------------------------------
// Entry-tiled segmented SpMV (J == 1) for segments that tile their entry list contiguously
// (CSR rows: row_end[s] == row_beg[s + 1]; the CSC chunks likewise). seg_spmv_kernel gives
// each segment its own L lanes: a wave of 4-16 short rows issues one round of loads and
// exits, so the Criteo-shaped products (40 entries per row, 1M-column tails of 1-4 entry
// chunks) ran latency bound at ~2.3 TB/s. Here a block takes a run of whole segments
// (<= 256 segments starting within one kTileCap-entry window; host-built table bseg) and
// streams the run's entries in passes of kTileCap (one pass unless the last segment reaches
// past the window: windows are kTileCap - 256 entries): every thread loads kTileCap / 256
// (index, value) pairs and their x gathers with all loads in flight, the products go to
// LDS, then G = 256 / segments threads per segment sum its slice of the pass from LDS.
// Per-segment order is fixed by (the table, G): bitwise deterministic run to run.
constexpr int kTileThreads = 256;
constexpr int kTileCap = 4096;
constexpr int kTileSegs = 256;  // segments per block at most (bseg construction)

template <bool kSquare, bool kOnes>
__global__ __launch_bounds__(kTileThreads) void seg_tile_spmv_kernel(
    const long long* __restrict__ beg, const long long* __restrict__ end, const int* __restrict__ bseg,
    const int* __restrict__ idx, const float* __restrict__ val, const float* __restrict__ x,
    float* __restrict__ out, float alpha, int accumulate) {
  __shared__ float sp[kTileCap];
  __shared__ float sred[kTileThreads];
  const int s0 = bseg[blockIdx.x], s1 = bseg[blockIdx.x + 1];
  const int ns = s1 - s0;
  if (ns <= 0) return;  // uniform per block
  const int t = threadIdx.x;
  int G = 1;  // threads per segment: the largest power of two with G * ns <= 256
  while (2 * G * ns <= kTileThreads) G <<= 1;
  const int ms = t / G, lane = t % G;
  const bool mine = ms < ns;
  const long long e0 = beg[s0], e1 = end[s1 - 1];
  const long long sb = mine ? beg[s0 + ms] : 0, se = mine ? end[s0 + ms] : 0;
  constexpr int K = kTileCap / kTileThreads;
  float acc = 0.f;
  for (long long p0 = e0; p0 < e1; p0 += kTileCap) {
    const int n = (int)min((long long)kTileCap, e1 - p0);
    int ii[K];
    float vv[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const int o = k * kTileThreads + t;
      const bool ok = o < n;
      ii[k] = ok ? idx[p0 + o] : 0;
      vv[k] = ok ? (kOnes ? 1.f : val[p0 + o]) : 0.f;
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const float xv = x[ii[k]];
      sp[k * kTileThreads + t] = (kSquare ? vv[k] * vv[k] : vv[k]) * xv;
    }
    __syncthreads();
    if (mine) {
      // this pass's slice of the segment, 4 independent LDS reads in flight (a serial
      // read-add chain left the kernel LDS-latency bound: 0.94 ms for a 164M-entry product)
      const int a = (int)(max(sb, p0) - p0), z = (int)(min(se, p0 + n) - p0);
      float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
      int e = a + lane;
      for (; e + 3 * G < z; e += 4 * G) {
        a0 += sp[e];
        a1 += sp[e + G];
        a2 += sp[e + 2 * G];
        a3 += sp[e + 3 * G];
      }
      for (; e < z; e += G) a0 += sp[e];
      acc += (a0 + a1) + (a2 + a3);
    }
    __syncthreads();
  }
  // the G partials of a segment, combined by a fixed tree
  if (G <= kWave) {
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1)
      if (off < G) acc += __shfl_xor(acc, off, kWave);
  } else {
    sred[t] = acc;
    __syncthreads();
    for (int off = G >> 1; off > 0; off >>= 1) {
      if (lane < off) sred[t] += sred[t + off];
      __syncthreads();
    }
    acc = sred[t];
  }
  if (mine && lane == 0) {
    const int s = s0 + ms;
    out[s] = accumulate ? out[s] + alpha * acc : alpha * acc;
  }
}

// Heavy columns of the chunk reduce (more than kReduceLight chunks: the bias column holds
// ~N / 4096 chunks): one block per column, threads = (chunk group g, output j); each thread
// sums chunks g, g + G, ... of its j (4 loads in flight), then the G group partials are
// added in group order through LDS. chunk_reduce_kernel skips these columns.
constexpr int kReduceLight = 16;

__global__ __launch_bounds__(256) void chunk_reduce_heavy_kernel(
    const long long* __restrict__ cbeg, const int* __restrict__ heavy, const float* __restrict__ part, int J,
    float* __restrict__ out, long long ldo, float alpha, int accumulate, const long long* __restrict__ ids) {
  __shared__ float s[256];
  const int col = heavy[blockIdx.x];
  const long long c0 = cbeg[col], c1 = cbeg[col + 1];
  const int JL = min(J, 256);
  const int G = 256 / JL;
  const int t = threadIdx.x, g = t / JL, jl = t % JL;
  for (int jb = 0; jb < J; jb += JL) {
    const int j = jb + jl;
    float acc = 0.f;
    if (g < G && j < J) {
      float a4[4] = {0.f, 0.f, 0.f, 0.f};
      long long c = c0 + g;
      for (; c + 3 * G < c1; c += 4 * G) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const long long cc = c + u * G;
          a4[u] += part[(ids ? ids[cc] : cc) * J + j];
        }
      }
      for (; c < c1; c += G) a4[0] += part[(ids ? ids[c] : c) * J + j];
      acc = (a4[0] + a4[1]) + (a4[2] + a4[3]);
    }
    if (G > 1) {
      __syncthreads();
      s[t] = acc;
      __syncthreads();
      if (g == 0 && j < J) {
        float tot = 0.f;
        for (int q = 0; q < G; ++q) tot += s[q * JL + jl];
        acc = tot;
      }
    }
    if (g == 0 && j < J) {
      float* o = out + (long long)col * ldo + j;
      *o = accumulate ? *o + alpha * acc : alpha * acc;
    }
  }
}

// ---------------------------------------------------------------------------------
// Fixed-layout rows (every row holds m entries; position j's columns all lie in
// [lo[j], lo[j] + span[j]), span <= kFixSpan -- the Criteo shape: the bias, then one entry
// per categorical field, each field a contiguous column range). X w is then computed
// position by position: position j's slice of w (<= 128 KiB) is staged in LDS once per
// block and the block's rows gather from LDS instead of from the whole 4 MB w in L2 (the
// per-row kernels are bound by those 164M random L2 gathers: ~550 of ~850 us). The index
// stream is the position-major transpose of the local column offsets as uint16
// (idxT[j][r] = idx[r][j] - lo[j]: half the bytes, coalesced per position). One 1024-thread
// block of kFixRows rows per CU; per row the positions are summed in order (deterministic).
constexpr int kFixThreads = 1024;
constexpr int kFixSpan = 32768;  // floats of LDS per position slice (128 KiB)
constexpr int kFixRPT = 16;      // rows per thread (kFixRows = 16384 rows per block)

template <bool kOnes, bool kSquare>
__global__ __launch_bounds__(kFixThreads) void fixed_spmv_kernel(
    const unsigned short* __restrict__ idxT, const float* __restrict__ valT, long long n, int m,
    const int* __restrict__ lo, const int* __restrict__ span, const float* __restrict__ x,
    float* __restrict__ out, float alpha, int accumulate) {
  extern __shared__ float sx[];
  const int t = threadIdx.x;
  const long long r0 = (long long)blockIdx.x * kFixThreads * kFixRPT;
  float acc[kFixRPT];
#pragma unroll
  for (int q = 0; q < kFixRPT; ++q) acc[q] = 0.f;
  for (int j = 0; j < m; ++j) {
    const int L = lo[j], S = span[j];
    // stage x[L, L + S): 8 independent loads per thread in flight per step
    for (int i0 = 0; i0 < S; i0 += kFixThreads * 8) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * kFixThreads + t;
        v[u] = i < S ? x[L + i] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * kFixThreads + t;
        if (i < S) sx[i] = v[u];
      }
    }
    __syncthreads();
    const unsigned short* ij = idxT + (size_t)j * n;
    const float* vj = kOnes ? nullptr : valT + (size_t)j * n;
    unsigned short c[kFixRPT];
    float v[kFixRPT];
#pragma unroll
    for (int q = 0; q < kFixRPT; ++q) {
      const long long r = r0 + (long long)q * kFixThreads + t;
      const bool ok = r < n;
      c[q] = ok ? ij[r] : (unsigned short)0;
      v[q] = ok ? (kOnes ? 1.f : vj[r]) : 0.f;
    }
#pragma unroll
    for (int q = 0; q < kFixRPT; ++q) acc[q] += (kSquare ? v[q] * v[q] : v[q]) * sx[c[q]];
    __syncthreads();  // sx is restaged for the next position
  }
#pragma unroll
  for (int q = 0; q < kFixRPT; ++q) {
    const long long r = r0 + (long long)q * kFixThreads + t;
    if (r < n) out[r] = accumulate ? out[r] + alpha * acc[q] : alpha * acc[q];
  }
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

// heavy (optional, int32 [nheavy]): the columns with more than kReduceLight chunks, reduced
// by chunk_reduce_heavy_kernel (one block each) instead of one serial thread per output
void ytk_chunk_reduce(uintptr_t cbeg, int ncol, uintptr_t part, int J, uintptr_t out,
                      long long ldo, float alpha, int accumulate, uintptr_t ids, uintptr_t heavy, int nheavy,
                      uintptr_t stream) {
  if (ncol <= 0 || J <= 0) return;
  const long long n = (long long)ncol * J;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(chunk_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                     (const long long*)cbeg, ncol, (const float*)part, J, (float*)out, ldo, alpha, accumulate,
                     (const long long*)ids, heavy ? 1 : 0);
  if (heavy && nheavy > 0)
    hipLaunchKernelGGL(chunk_reduce_heavy_kernel, dim3((unsigned)nheavy), dim3(256), 0, s, (const long long*)cbeg,
                       (const int*)heavy, (const float*)part, J, (float*)out, ldo, alpha, accumulate,
                       (const long long*)ids);
  YTK_LAUNCH_CHECK();
}

// Fixed-layout J == 1 row product (fixed_spmv_kernel). idxT: uint16 [m, n] local offsets,
// valT: float [m, n] (0: one-hot), lo / span: int32 [m] (span <= kFixSpan, checked by the caller).
void ytk_fixed_spmv(uintptr_t idxT, uintptr_t valT, long long n, int m, uintptr_t lo, uintptr_t span, int max_span,
                    uintptr_t x, uintptr_t out, float alpha, int accumulate, int square, uintptr_t stream) {
  if (n <= 0 || m <= 0) return;
  if (max_span > kFixSpan || max_span <= 0) throw std::invalid_argument("fixed_spmv: position span out of range");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const long long rows = (long long)kFixThreads * kFixRPT;
  const unsigned grid = (unsigned)((n + rows - 1) / rows);
  const size_t lds = (size_t)max_span * sizeof(float);
#define YTK_FIX(ON, SQ)                                                                                     \
  hipLaunchKernelGGL((fixed_spmv_kernel<ON, SQ>), dim3(grid), dim3(kFixThreads), lds, s, (const unsigned short*)idxT, \
                     (const float*)valT, n, m, (const int*)lo, (const int*)span, (const float*)x, (float*)out,   \
                     alpha, accumulate)
  if (valT == 0) YTK_FIX(true, false);
  else if (square) YTK_FIX(false, true);
  else YTK_FIX(false, false);
#undef YTK_FIX
  YTK_LAUNCH_CHECK();
}

// Entry-tiled J == 1 product over contiguous segments (seg_tile_spmv_kernel); bseg: int32
// [nblk + 1] block -> first segment. val == 0: one-hot values.
void ytk_seg_tile_spmv(uintptr_t beg, uintptr_t end, uintptr_t bseg, int nblk, uintptr_t idx, uintptr_t val,
                       uintptr_t x, uintptr_t out, float alpha, int accumulate, int square, uintptr_t stream) {
  if (nblk <= 0) return;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
#define YTK_TILE(SQ, ON)                                                                                    \
  hipLaunchKernelGGL((seg_tile_spmv_kernel<SQ, ON>), dim3((unsigned)nblk), dim3(kTileThreads), 0, s,        \
                     (const long long*)beg, (const long long*)end, (const int*)bseg, (const int*)idx,       \
                     (const float*)val, (const float*)x, (float*)out, alpha, accumulate)
  if (val == 0) YTK_TILE(false, true);
  else if (square) YTK_TILE(true, false);
  else YTK_TILE(false, false);
#undef YTK_TILE
  YTK_LAUNCH_CHECK();
}

}  // extern "C"
