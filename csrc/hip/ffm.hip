// Field-aware factorization machine pair interactions (gfx950 / CDNA4, wave64).
//
// Reference: J/optimizer/FFMHoagOptimizer.java:90-210
//   fx(row)  = sum_{p<q} <V[i_p, f_q, :], V[i_q, f_p, :]> x_p x_q   (+ linear part)
//   g[i_p, f_q, :] += c x_p x_q V[i_q, f_p, :],  g[i_q, f_p, :] += c x_p x_q V[i_p, f_q, :]
// with V stored after the F linear weights as [F][nfield][k] (dim = F + F*nfield*k).
//
// Mapping: one wave per row. Lane j caches entry j of the row (feature, value, field) in
// registers (rows longer than 64 entries are processed in 64-entry tiles); for each p the
// wave broadcasts p's entry and lanes take q = p+1+lane, so every lane owns one pair per
// step and the k-long dot products are independent gathers of contiguous k floats
// (L2-resident for hot features). Forward ends with a wave reduction; backward scatters
// with hardware float atomics (no-return global_atomic_add_f32) -- the only
// order-dependent reduction in the sparse family (documented).
#include "common.h"

namespace ytk {

__device__ __forceinline__ float pair_dot(const float* __restrict__ a, const float* __restrict__ b, int k,
                                          bool vec4) {
  float s = 0.f;
  int f = 0;
  if (vec4) {
    for (; f < k; f += 4) {
      const float4 va = *reinterpret_cast<const float4*>(a + f);
      const float4 vb = *reinterpret_cast<const float4*>(b + f);
      s += va.x * vb.x + va.y * vb.y + va.z * vb.z + va.w * vb.w;
    }
  } else {
    for (; f < k; ++f) s += a[f] * b[f];
  }
  return s;
}

template <bool kBackward>
__global__ __launch_bounds__(256) void ffm_pairs_kernel(
    const long long* __restrict__ indptr, const int* __restrict__ idx, const float* __restrict__ val,
    const int* __restrict__ fld, long long nrows, const float* __restrict__ V, int nfield, int k,
    float* __restrict__ fx, const float* __restrict__ coef, float* __restrict__ gV, int vec4) {
  const long long row = (blockIdx.x * (long long)blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (row >= nrows) return;
  const long long b = indptr[row];
  const int m = (int)(indptr[row + 1] - b);
  const long long stride = (long long)nfield * k;
  const float c = kBackward ? coef[row] : 0.f;
  float acc = 0.f;
  // tiles of 64 entries: (P tile, Q tile) with Q tile >= P tile
  for (int pt = 0; pt < m; pt += 64) {
    const int pj = pt + lane;
    int ip = 0, fp = 0;
    float xp = 0.f;
    if (pj < m) { ip = idx[b + pj]; xp = val[b + pj]; fp = fld[b + pj]; }
    for (int qt = pt; qt < m; qt += 64) {
      const int qj = qt + lane;
      int iq = 0, fq = 0;
      float xq = 0.f;
      if (qj < m) { iq = idx[b + qj]; xq = val[b + qj]; fq = fld[b + qj]; }
      const int pend = min(64, m - pt);
      for (int pp = 0; pp < pend; ++pp) {
        const int P = pt + pp;
        const int ipb = __shfl(ip, pp, 64), fpb = __shfl(fp, pp, 64);
        const float xpb = __shfl(xp, pp, 64);
        if (qj < m && qj > P) {
          const float* vp = V + (long long)ipb * stride + (long long)fq * k;  // V[i_p, f_q]
          const float* vq = V + (long long)iq * stride + (long long)fpb * k;  // V[i_q, f_p]
          const float xx = xpb * xq;
          if (!kBackward) {
            acc += pair_dot(vp, vq, k, vec4 != 0) * xx;
          } else {
            const float s = c * xx;
            float* gp = gV + (long long)ipb * stride + (long long)fq * k;
            float* gq = gV + (long long)iq * stride + (long long)fpb * k;
            for (int f = 0; f < k; ++f) {
              unsafeAtomicAdd(gp + f, s * vq[f]);
              unsafeAtomicAdd(gq + f, s * vp[f]);
            }
          }
        }
      }
    }
  }
  if (!kBackward) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (lane == 0) fx[row] = acc;
  }
}

}  // namespace ytk

using namespace ytk;

extern "C" {

// fx[row] = pair interaction sum (forward) or g += pair gradients scaled by coef[row].
void ytk_ffm_pairs(uintptr_t indptr, uintptr_t idx, uintptr_t val, uintptr_t fld, long long nrows,
                   uintptr_t V, int nfield, int k, uintptr_t fx, uintptr_t coef, uintptr_t gV,
                   int backward, uintptr_t stream) {
  if (nrows <= 0 || k <= 0) return;
  const long long threads = nrows * 64;
  const dim3 grid((unsigned)((threads + 255) / 256));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int vec4 = ((k & 3) == 0 && (V & 15) == 0) ? 1 : 0;  // 16-B gathers need aligned V
  if (backward)
    hipLaunchKernelGGL(ffm_pairs_kernel<true>, grid, dim3(256), 0, s, (const long long*)indptr,
                       (const int*)idx, (const float*)val, (const int*)fld, nrows, (const float*)V,
                       nfield, k, (float*)fx, (const float*)coef, (float*)gV, vec4);
  else
    hipLaunchKernelGGL(ffm_pairs_kernel<false>, grid, dim3(256), 0, s, (const long long*)indptr,
                       (const int*)idx, (const float*)val, (const int*)fld, nrows, (const float*)V,
                       nfield, k, (float*)fx, (const float*)coef, (float*)gV, vec4);
  YTK_LAUNCH_CHECK();
}

}  // extern "C"
