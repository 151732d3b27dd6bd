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

#include <algorithm>
#include <cstdlib>

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

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <bool kBackward>
__global__ __launch_bounds__(256) void ffm_pairs_kernel(
    const long long* __restrict__ indptr, const int* __restrict__ idx, const float* __restrict__ val,
    const int* __restrict__ fld, long long nrows, const float* __restrict__ V, int nfield, int k,
    float* __restrict__ fx, const float* __restrict__ coef, float* __restrict__ gV, int vec4,
    int skip_feat, const int* __restrict__ cnt) {
  // cnt (backward, optional): rows per feature of the SGD batch -- V[i, :] takes the
  // per-feature mean of the batch's steps (see fm_sgd_update_kernel)
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
        // skip_feat: a feature whose latent block is identically zero (the bias without a
        // latent factor): its pairs contribute nothing, and skipping them removes the
        // hottest atomic targets (the bias occurs in every row)
        if (qj < m && qj > P && ipb != skip_feat && iq != skip_feat) {
          const float* vp = V + (long long)ipb * stride + (long long)fq * k;  // V[i_p, f_q]
          const float* vq = V + (long long)iq * stride + (long long)fpb * k;  // V[i_q, f_p]
          const float xx = xpb * xq;
          if (!kBackward) {
            acc += pair_dot(vp, vq, k, vec4 != 0) * xx;
          } else {
            const float s = c * xx;
            const float sp = cnt ? s / (float)max(1, cnt[ipb]) : s;
            const float sq = cnt ? s / (float)max(1, cnt[iq]) : s;
            float* gp = gV + (long long)ipb * stride + (long long)fq * k;
            float* gq = gV + (long long)iq * stride + (long long)fpb * k;
            for (int f = 0; f < k; ++f) {
              unsafeAtomicAdd(gp + f, sp * vq[f]);
              unsafeAtomicAdd(gq + f, sq * vp[f]);
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


// Forward for k == 4 (one float4 per latent block), kPU pairs per lane in flight: the
// generic loop walks p one pair at a time, two dependent 16-B gathers per step, which left
// the forward latency bound (one wave per row, 39 serial gather round trips: 25 ms per
// Criteo-shape pass). Same pairs, same per-lane order of the adds.
//
// kE (SGD, fixed-layout rows of m <= 64 entries, ops/sgd.py): the kernel also writes the pair
// terms the batch gradient is made of, E[e_p][q] = x_p x_q V[i_q, f_p, :] for every ordered
// pair of positions (p, q) of the row (zero for q == p and for pairs with the skipped
// feature), e_p = the entry's offset from e_base. Both factors of every pair are already in
// registers for the dot product, so the gradient costs one row write here and one row read
// per entry in ffm_sgd_ecol_kernel -- instead of a second pass of 16-B gathers scattered over
// V. Step p's lanes q > p write E[p][q] as one coalesced segment; the transposed terms
// E[q][p] go to a per-wave LDS triangle first and leave as row segments after the row's last
// step (written straight from the lanes they were 16-B stores 640 B apart, whose lines were
// evicted from L2 half written).
constexpr int kPU = 4;
template <bool kE>
__global__ __launch_bounds__(256) void ffm_pairs_k4_kernel(
    const long long* __restrict__ indptr, const int* __restrict__ idx, const float* __restrict__ val,
    const int* __restrict__ fld, long long nrows, const float* __restrict__ V, int nfield,
    float* __restrict__ fx, int skip_feat, float4* __restrict__ E, long long e_base) {
  extern __shared__ float4 s_tri[];  // kE: [waves][m (m - 1) / 2], entry (q, p < q) at q (q - 1) / 2 + p
  const long long row = (blockIdx.x * (long long)blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (row >= nrows) return;
  const long long b = indptr[row];
  const int m = (int)(indptr[row + 1] - b);
  const long long stride = (long long)nfield * 4;
  float acc = 0.f;
  for (int pt = 0; pt < m; pt += 64) {
    const int pj = pt + lane;
    int ip = 0, fp = 0;
    float xp = 0.f;
    if (pj < m) { ip = idx[b + pj]; xp = val[b + pj]; fp = fld[b + pj]; }
    if (kE && pj < m) E[(b - e_base + pj) * m + pj] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int qt = pt; qt < m; qt += 64) {
      const int qj = qt + lane;
      int iq = 0, fq = 0;
      float xq = 0.f;
      if (qj < m) { iq = idx[b + qj]; xq = val[b + qj]; fq = fld[b + qj]; }
      const int pend = min(64, m - pt);
      for (int pp0 = 0; pp0 < pend; pp0 += kPU) {
        float4 va[kPU], vb[kPU];
        float xx[kPU];
        bool ok[kPU];
#pragma unroll
        for (int u = 0; u < kPU; ++u) {
          const int pp = min(pp0 + u, pend - 1);  // uniform; the duplicate is masked by ok
          const int P = pt + pp;
          const int ipb = __shfl(ip, pp, 64), fpb = __shfl(fp, pp, 64);
          const float xpb = __shfl(xp, pp, 64);
          ok[u] = pp0 + u < pend && qj < m && qj > P && ipb != skip_feat && iq != skip_feat;
          xx[u] = xpb * xq;
          va[u] = vb[u] = make_float4(0.f, 0.f, 0.f, 0.f);
          if (ok[u]) {
            va[u] = *reinterpret_cast<const float4*>(V + (long long)ipb * stride + (long long)fq * 4);
            vb[u] = *reinterpret_cast<const float4*>(V + (long long)iq * stride + (long long)fpb * 4);
          }
        }
#pragma unroll
        for (int u = 0; u < kPU; ++u)
          if (ok[u])
            acc += (va[u].x * vb[u].x + va[u].y * vb[u].y + va[u].z * vb[u].z + va[u].w * vb[u].w) * xx[u];
        if (kE) {
#pragma unroll
          for (int u = 0; u < kPU; ++u) {
            const int P = pt + pp0 + u;
            if (pp0 + u < pend && qj < m && qj > P) {  // every pair slot is written (zero if skipped)
              const float s = ok[u] ? xx[u] : 0.f;
              // E[p][q] = x_p x_q V[i_q, f_p]: lanes write consecutive slots of row p
              E[(b - e_base + P) * m + qj] = make_float4(s * vb[u].x, s * vb[u].y, s * vb[u].z, s * vb[u].w);
              // E[q][p] = x_p x_q V[i_p, f_q]: into the LDS triangle
              s_tri[(threadIdx.x >> 6) * (m * (m - 1) / 2) + qj * (qj - 1) / 2 + P] =
                  make_float4(s * va[u].x, s * va[u].y, s * va[u].z, s * va[u].w);
            }
          }
        }
      }
    }
  }
  if (kE) {  // the transposed terms, row by row: t -> (q, p) with t = q (q - 1) / 2 + p
    wave_sync();
    const int ntri = m * (m - 1) / 2;
    const float4* tri = s_tri + (threadIdx.x >> 6) * ntri;
    for (int t = lane; t < ntri; t += 64) {
      int q = (int)(0.5f * (1.f + sqrtf(1.f + 8.f * (float)t)));
      while (q * (q - 1) / 2 > t) --q;
      while ((q + 1) * q / 2 <= t) ++q;
      E[(b - e_base + q) * m + (t - q * (q - 1) / 2)] = tri[t];
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if (lane == 0) fx[row] = acc;
}

// Forward for k == 4 with the row's latent rows staged in LDS: one wave per row (64-thread
// blocks walking rows grid-stride), the m latent rows V[i_j, 0..nfield) of the row copied whole
// into LDS with coalesced 16-B loads, then the m (m - 1) / 2 pairs read from LDS, pair index
// pi = q (q - 1) / 2 + p (p < q) decoded per lane. ffm_pairs_k4_kernel gathers the same bytes
// as 16-B pieces, one per lane and pair: 64 distinct lines per load instruction for V[i_q, f_p]
// (every latent row is touched 2 (m - 1) times, in slices), so it is bound by the cache
// request rate, not by bytes. Rows of at most max_m entries (LDS: max_m * (nfield + 1) * 16 B;
// the padded row stride keeps a column read -- lanes q at slot f -- off one bank group).
// kE (SGD pair terms, as ffm_pairs_k4_kernel<true>): then E[e_p][q] = x_p x_q V[i_q, f_p] row by
// row, lanes q reading LDS column f_p -- every store a coalesced row, no transpose.
constexpr int kLdsU = 16;  // staging loads in flight per lane (4: 30.7 ms per 4M-row forward, bytes-in-flight bound)

// bf16 latent slots (k == 4: one 8-B uint2 of packed bf16 pairs per (feature, field)):
// widened exactly to fp32, narrowed round-to-nearest-even (finite values)
__device__ __forceinline__ float4 bf4_to_f4(uint2 h) {
  return make_float4(__uint_as_float(h.x << 16), __uint_as_float(h.x & 0xffff0000u), __uint_as_float(h.y << 16),
                     __uint_as_float(h.y & 0xffff0000u));
}
__device__ __forceinline__ unsigned f_to_bf(float f) {
  const unsigned u = __float_as_uint(f);
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ uint2 f4_to_bf4(float4 v) {
  return make_uint2(f_to_bf(v.x) | (f_to_bf(v.y) << 16), f_to_bf(v.z) | (f_to_bf(v.w) << 16));
}

// kBf (SGD dtype = bf16): V is the bf16 working copy (8-B slots, half the staging bytes)
// and the pair terms E are written as bf16 (half the bytes the chunk sums read back); the LDS
// rows, the pair dot products and the row sums stay fp32.
template <bool kE, bool kBf = false>
__global__ __launch_bounds__(64) void ffm_pairs_lds_kernel(
    const long long* __restrict__ indptr, const int* __restrict__ idx, const float* __restrict__ val,
    const int* __restrict__ fld, long long nrows, const void* __restrict__ Vv, int nfield,
    float* __restrict__ fx, int skip_feat, void* __restrict__ Ev, long long e_base) {
  // bf16: 8-B slot loads (16-B slot-pair loads widened into two LDS rows measured slower, 0.91
  // vs 0.70 ms per batch: this kernel is bound by its LDS and shuffle work, not by bytes)
  const float4* __restrict__ V = reinterpret_cast<const float4*>(Vv);
  const uint2* __restrict__ Vh = reinterpret_cast<const uint2*>(Vv);
  float4* __restrict__ E = reinterpret_cast<float4*>(Ev);
  extern __shared__ float4 s_v[];  // [m][nfield + 1]
  const int lane = threadIdx.x;
  const int S = nfield + 1;
  const int tn = nfield;  // staging units per entry
  const int step_j = 64 / tn, step_t = 64 - step_j * tn;
  const int lane_j = lane / tn, lane_t = lane - lane_j * tn;
  for (long long row = blockIdx.x; row < nrows; row += gridDim.x) {
    const long long b = indptr[row];
    const int m = (int)(indptr[row + 1] - b);
    int ij = 0, fj = 0;
    float xj = 0.f;
    if (lane < m) { ij = idx[b + lane]; fj = fld[b + lane]; xj = val[b + lane]; }
    const int tot = m * tn;
    int j = lane_j, t = lane_t;  // (entry, unit) of position s0 + u * 64 + lane
    for (int s0 = 0; s0 < tot; s0 += 64 * kLdsU) {
      float4 v[kLdsU];
      uint2 vh[kLdsU];  // bf16: raw slots, every load issued before any is widened (widening in
                        // this loop made the compiler wait on each load in turn)
      int dst[kLdsU];
#pragma unroll
      for (int u = 0; u < kLdsU; ++u) {
        const int sp = s0 + u * 64 + lane;
        const int i = __shfl(ij, min(j, 63), 64);
        dst[u] = sp < tot ? j * S + t : -1;
        if constexpr (kBf)
          vh[u] = sp < tot ? Vh[(long long)i * nfield + t] : make_uint2(0u, 0u);
        else
          v[u] = sp < tot ? V[(long long)i * nfield + t] : make_float4(0.f, 0.f, 0.f, 0.f);
        t += step_t;
        j += step_j;
        if (t >= tn) { t -= tn; ++j; }
      }
#pragma unroll
      for (int u = 0; u < kLdsU; ++u) {
        if (dst[u] >= 0) s_v[dst[u]] = kBf ? bf4_to_f4(vh[u]) : v[u];
      }
    }
    wave_sync();
    float acc = 0.f;
    const int np = m * (m - 1) / 2;
    // uniform trip count: the shuffles read lanes p, q, which must be active (a lane that left
    // a divergent loop returns no data to ds_bpermute)
    for (int base = 0; base < np; base += 64) {
      const int pi = min(base + lane, np - 1);
      int q = (int)(0.5f * (1.f + sqrtf(1.f + 8.f * (float)pi)));
      while (q * (q - 1) / 2 > pi) --q;
      while ((q + 1) * q / 2 <= pi) ++q;
      const int p = pi - q * (q - 1) / 2;
      const int ip = __shfl(ij, p, 64), iq = __shfl(ij, q, 64);
      const int fp = __shfl(fj, p, 64), fq = __shfl(fj, q, 64);
      const float xx = __shfl(xj, p, 64) * __shfl(xj, q, 64);
      if (base + lane < np && ip != skip_feat && iq != skip_feat) {
        const float4 a = s_v[p * S + fq], c = s_v[q * S + fp];  // V[i_p, f_q], V[i_q, f_p]
        acc += (a.x * c.x + a.y * c.y + a.z * c.z + a.w * c.w) * xx;
      }
    }
    if constexpr (kE && kBf) {  // E rows: entry p, lanes q, one 8-B bf16 slot each (16-B slot
      // pairs per lane measured slower: 1.02 vs 0.70 ms per batch -- twice the LDS reads per lane
      // at a doubled lane stride)
      uint2* Eq = reinterpret_cast<uint2*>(Ev);
      const bool qs = lane < m && ij != skip_feat;
      for (int p = 0; p < m; ++p) {  // p is wave-uniform: readlane, no LDS-routed shuffles
        const int fp = __builtin_amdgcn_readlane(fj, p), ip = __builtin_amdgcn_readlane(ij, p);
        const float xp = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(xj), p));
        if (lane < m) {
          const float s = (qs && lane != p && ip != skip_feat) ? xp * xj : 0.f;
          const float4 c = s_v[lane * S + fp];
          Eq[(b - e_base + p) * m + lane] = f4_to_bf4(make_float4(s * c.x, s * c.y, s * c.z, s * c.w));
        }
      }
    } else if constexpr (kE) {  // E rows: entry p, lanes q
      const bool qs = lane < m && ij != skip_feat;
      for (int p = 0; p < m; ++p) {
        const int fp = __builtin_amdgcn_readlane(fj, p), ip = __builtin_amdgcn_readlane(ij, p);
        const float xp = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(xj), p));
        if (lane < m) {
          const float s = (qs && lane != p && ip != skip_feat) ? xp * xj : 0.f;
          const float4 c = s_v[lane * S + fp];
          E[(b - e_base + p) * m + lane] = make_float4(s * c.x, s * c.y, s * c.z, s * c.w);
        }
      }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if (lane == 0) fx[row] = acc;
    wave_sync();  // the next row's staging overwrites s_v
  }
}

// Pair scatter backward for k == 4 (the SGD step's direct update of V: coef = -lr c_r):
// the generic backward walks p one pair at a time -- two dependent 16-B gathers, then the
// atomics -- so a Criteo-shape SGD epoch ran latency bound (~1.07 s). Here kPU pairs'
// gathers per lane are in flight before their atomics, as in ffm_pairs_k4_kernel. Same
// pairs and updates as ffm_pairs_kernel<true> (Hogwild!: the atomics race either way).
__global__ __launch_bounds__(256) void ffm_pairs_k4_bwd_kernel(
    const long long* __restrict__ indptr, const int* __restrict__ idx, const float* __restrict__ val,
    const int* __restrict__ fld, long long nrows, const float* __restrict__ V, int nfield,
    const float* __restrict__ coef, float* __restrict__ gV, int skip_feat, const int* __restrict__ cnt) {
  const long long row = (blockIdx.x * (long long)blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (row >= nrows) return;
  const float c = coef[row];
  if (c == 0.f) return;  // wave-uniform
  const long long b = indptr[row];
  const int m = (int)(indptr[row + 1] - b);
  const long long stride = (long long)nfield * 4;
  for (int pt = 0; pt < m; pt += 64) {
    const int pj = pt + lane;
    int ip = 0, fp = 0;
    float xp = 0.f, rp = 1.f;
    if (pj < m) {
      ip = idx[b + pj]; xp = val[b + pj]; fp = fld[b + pj];
      if (cnt) rp = 1.f / (float)max(1, cnt[ip]);
    }
    for (int qt = pt; qt < m; qt += 64) {
      const int qj = qt + lane;
      int iq = 0, fq = 0;
      float xq = 0.f, rq = 1.f;
      if (qj < m) {
        iq = idx[b + qj]; xq = val[b + qj]; fq = fld[b + qj];
        if (cnt) rq = 1.f / (float)max(1, cnt[iq]);
      }
      const int pend = min(64, m - pt);
      for (int pp0 = 0; pp0 < pend; pp0 += kPU) {
        float4 va[kPU], vb[kPU];
        float sp[kPU], sq[kPU];
        long long op[kPU], oq[kPU];
        bool ok[kPU];
#pragma unroll
        for (int u = 0; u < kPU; ++u) {
          const int pp = min(pp0 + u, pend - 1);  // uniform; the duplicate is masked by ok
          const int P = pt + pp;
          const int ipb = __shfl(ip, pp, 64), fpb = __shfl(fp, pp, 64);
          const float xpb = __shfl(xp, pp, 64), rpb = __shfl(rp, pp, 64);
          ok[u] = pp0 + u < pend && qj < m && qj > P && ipb != skip_feat && iq != skip_feat;
          const float s = c * xpb * xq;
          sp[u] = s * rpb;  // into V[i_p, f_q]
          sq[u] = s * rq;   // into V[i_q, f_p]
          op[u] = (long long)ipb * stride + (long long)fq * 4;
          oq[u] = (long long)iq * stride + (long long)fpb * 4;
          va[u] = vb[u] = make_float4(0.f, 0.f, 0.f, 0.f);
          if (ok[u]) {
            va[u] = *reinterpret_cast<const float4*>(V + op[u]);
            vb[u] = *reinterpret_cast<const float4*>(V + oq[u]);
          }
        }
#pragma unroll
        for (int u = 0; u < kPU; ++u) {
          if (!ok[u]) continue;
          float* gp = gV + op[u];
          float* gq = gV + oq[u];
          unsafeAtomicAdd(gp, sp[u] * vb[u].x);
          unsafeAtomicAdd(gp + 1, sp[u] * vb[u].y);
          unsafeAtomicAdd(gp + 2, sp[u] * vb[u].z);
          unsafeAtomicAdd(gp + 3, sp[u] * vb[u].w);
          unsafeAtomicAdd(gq, sq[u] * va[u].x);
          unsafeAtomicAdd(gq + 1, sq[u] * va[u].y);
          unsafeAtomicAdd(gq + 2, sq[u] * va[u].z);
          unsafeAtomicAdd(gq + 3, sq[u] * va[u].w);
        }
      }
    }
  }
}

// Column-ordered (gather) backward: no global atomics.
//   gV[i, f_q, :] = sum over entries e of feature i (row r, value x, field f_i) and every
//                   other entry q of row r:  c_r x x_q V[i_q, f_i, :]
// which is the same sum as the pair scatter above, regrouped by the target feature i.
// One wave per CSC chunk (<= CHUNK entries of one column), four independent waves per
// 256-thread block (64-thread blocks cap residency at ~12 waves/CU). The chunk's
// [nfield][k] accumulator lives in LDS and is written once to part[chunk] (an ordered
// chunk_reduce then sums the chunks of a column). Lane e of a 64-entry batch loads entry
// e's row descriptor; the wave then walks kUnroll entries at a time with lane = position
// q in the row, so the row's idx/val/fld loads are coalesced and kUnroll rows' gathers are
// in flight together. When every row has distinct fields (one-hot-per-field data such as
// Criteo) the lanes of one entry hit distinct accumulator slots and the update is a plain
// LDS read-add-write (b128 for k % 4 == 0); otherwise it falls back to ds_add_f32.
// All LDS traffic is wave-private: wave_sync() orders it.
constexpr int kCscUnroll = 4;
constexpr int kCscWaves = 4;

template <bool kVec4, bool kDistinct>
__global__ __launch_bounds__(256) void ffm_grad_csc_kernel(
    const long long* __restrict__ chunk_beg, const long long* __restrict__ chunk_end, long long nch,
    const int* __restrict__ csc_rows, const float* __restrict__ csc_vals,
    const long long* __restrict__ csc_pos, const long long* __restrict__ indptr,
    const unsigned* __restrict__ pk, int sh, const float* __restrict__ val,
    const float* __restrict__ Vt, long long nfeat, int nfield, int k, const float* __restrict__ coef,
    float* __restrict__ part, int skip_feat) {
  extern __shared__ float lds_acc[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long long ch = blockIdx.x * (long long)kCscWaves + wave;
  if (ch >= nch) return;  // no block-level barriers below
  const int J = nfield * k;
  const unsigned mask = (1u << sh) - 1u;
  const long long fstride = nfeat * k;  // Vt is [nfield][nfeat][k]
  float* acc = lds_acc + wave * J;  // [nfield][k]
  for (int j = lane; j < J; j += 64) acc[j] = 0.f;
  wave_sync();
  const long long e0 = chunk_beg[ch], e1 = chunk_end[ch];
  const int feat = (int)(pk[csc_pos[e0]] & mask);
  if (feat != skip_feat) {
    for (long long eb = e0; eb < e1; eb += 64) {
      const long long e = eb + lane;
      long long d_b = 0, d_pos = -1;
      int d_len = 0, d_f = 0;
      float d_s = 0.f;
      if (e < e1) {
        d_pos = csc_pos[e];
        const int r = csc_rows[e];
        d_b = indptr[r];
        d_len = (int)(indptr[r + 1] - d_b);
        d_s = coef[r] * csc_vals[e];
        d_f = (int)(pk[d_pos] >> sh);
      }
      const int nb = (int)min<long long>(64, e1 - eb);
      for (int e2 = 0; e2 < nb; e2 += kCscUnroll) {
        long long qb[kCscUnroll], qpos[kCscUnroll];
        int len[kCscUnroll];
        const float* vbase[kCscUnroll];
        float sc[kCscUnroll];
        int maxlen = 0;
#pragma unroll
        for (int u = 0; u < kCscUnroll; ++u) {
          const int src = min(e2 + u, nb - 1);
          len[u] = e2 + u < nb ? __shfl(d_len, src, 64) : 0;
          qb[u] = __shfl(d_b, src, 64);
          qpos[u] = __shfl(d_pos, src, 64);
          vbase[u] = Vt + (long long)__shfl(d_f, src, 64) * fstride;  // Vt[f_i]
          sc[u] = __shfl(d_s, src, 64);
          maxlen = max(maxlen, len[u]);
        }
        for (int qt = 0; qt < maxlen; qt += 64) {
          int slot[kCscUnroll];
          float tv[kCscUnroll];
          const float* vq[kCscUnroll];
#pragma unroll
          for (int u = 0; u < kCscUnroll; ++u) {
            const int q = qt + lane;
            slot[u] = -1;
            tv[u] = 0.f;
            vq[u] = Vt;
            if (q < len[u] && qb[u] + q != qpos[u]) {
              const long long g = qb[u] + q;
              const unsigned code = pk[g];
              const int iq = (int)(code & mask);
              if (iq != skip_feat) {
                slot[u] = (int)(code >> sh) * k;
                tv[u] = val ? sc[u] * val[g] : sc[u];
                vq[u] = vbase[u] + (long long)iq * k;  // V[i_q, f_i]
              }
            }
          }
          if (kVec4) {
            for (int f = 0; f < k; f += 4) {
              float4 v4[kCscUnroll];
#pragma unroll
              for (int u = 0; u < kCscUnroll; ++u)
                v4[u] = slot[u] >= 0 ? *reinterpret_cast<const float4*>(vq[u] + f) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
              for (int u = 0; u < kCscUnroll; ++u) {
                if (slot[u] < 0) continue;
                float* a = acc + slot[u] + f;
                if (kDistinct) {
                  float4 o = *reinterpret_cast<float4*>(a);
                  o.x += tv[u] * v4[u].x;
                  o.y += tv[u] * v4[u].y;
                  o.z += tv[u] * v4[u].z;
                  o.w += tv[u] * v4[u].w;
                  *reinterpret_cast<float4*>(a) = o;
                } else {
                  atomicAdd(a, tv[u] * v4[u].x);
                  atomicAdd(a + 1, tv[u] * v4[u].y);
                  atomicAdd(a + 2, tv[u] * v4[u].z);
                  atomicAdd(a + 3, tv[u] * v4[u].w);
                }
              }
            }
          } else {
#pragma unroll
            for (int u = 0; u < kCscUnroll; ++u) {
              if (slot[u] < 0) continue;
              float* a = acc + slot[u];
              for (int f = 0; f < k; ++f) {
                if (kDistinct) a[f] += tv[u] * vq[u][f];
                else atomicAdd(a + f, tv[u] * vq[u][f]);
              }
            }
          }
          wave_sync();
        }
      }
    }
  }
  wave_sync();
  float* out = part + ch * (long long)J;
  for (int j = lane; j < J; j += 64) out[j] = acc[j];
}

// Fixed-layout, XCD-split, streamed column-ordered backward. When every row holds the same m
// fields in the same order (one entry per field: Criteo-style data, the bias in position 0),
// the kernel above is L2-miss bound on two random streams: its 16-B latent gathers
// V[i_q, f_i] (one field's slice Vt[f_i] is nfeat*16 B = 16 MB at 1M features, four times an
// XCD's 4-MB L2; 274 GB fetched per Criteo-shape pass) and the row entries it re-reads for
// every column of the row. Here
//  * the row POSITIONS are split into 8 groups and group g's work runs on the blocks with
//    blockIdx % 8 == g -- one XCD (blocks are dealt round-robin over the XCDs) -- so an XCD
//    only gathers latent rows of its own ~m/8 fields: Vt[f_i] restricted to those fields'
//    features, an L2-sized working set;
//  * the row entries each group needs are a setup-time expansion exp_idx[g][e][0..G) of the
//    CSC entries (entry e's row's feature ids at the group's positions, -1 for the entry
//    itself and skipped features), read as a coalesced nontemporal stream instead of random
//    row reads (HBM capacity bought for bandwidth: nnz * 8G * 4 B), and the per-entry scale
//    s[e] = coef[row] * x_e is one gathered pass per evaluation.
// Lanes: G = ceil(m / 8) positions x E = 64 / G entries; each lane accumulates its position's
// k floats in registers over the chunk, then the E lanes of a position are summed in a fixed
// order through LDS -- deterministic, no atomics. A wave walks a contiguous range of chunks
// (wave_chunk, ~equal entries per wave) so small columns do not each pay a wave launch.
constexpr int kFixUnroll = 4;

template <int KV>
__global__ __launch_bounds__(256) void ffm_grad_stream_kernel(
    const long long* __restrict__ wave_chunk, long long nwaves, const long long* __restrict__ chunk_beg,
    const long long* __restrict__ chunk_end, const int* __restrict__ chunk_fa, const int* __restrict__ exp_idx,
    const float* __restrict__ exp_val, const float* __restrict__ se, long long nnz, int G,
    const int* __restrict__ lay_field, int m, const float* __restrict__ Vt, long long nfeat, int nfield,
    float* __restrict__ part) {
  __shared__ float4 red[kCscWaves][64 * KV];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int grp = blockIdx.x & 7;
  const long long w = (long long)(blockIdx.x >> 3) * kCscWaves + wave;
  if (w >= nwaves) return;  // no block-level barriers below
  constexpr int k = KV * 4;
  const long long J = (long long)nfield * k;
  const int E = 64 / G;
  const int es = lane / G, qi = lane - es * G;
  const bool lane_ok = es < E && grp * G + qi < m;
  const long long fstride = nfeat * k;  // Vt is [nfield][nfeat][k]
  const int* __restrict__ xi = exp_idx + (long long)grp * nnz * G;
  const float* __restrict__ xv = exp_val ? exp_val + (long long)grp * nnz * G : nullptr;
  const long long c0 = wave_chunk[w], c1 = wave_chunk[w + 1];
  for (long long ch = c0; ch < c1; ++ch) {
    const long long e0 = chunk_beg[ch], e1 = chunk_end[ch];
    const int fa = chunk_fa[ch];  // field of the chunk's column, -1: skipped column
    float4 acc[KV];
#pragma unroll
    for (int j = 0; j < KV; ++j) acc[j] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (fa >= 0 && lane_ok) {
      const float* vbase = Vt + (long long)fa * fstride;
      for (long long eb = e0; eb < e1; eb += (long long)E * kFixUnroll) {
        int iq[kFixUnroll];
        float s[kFixUnroll];
#pragma unroll
        for (int u = 0; u < kFixUnroll; ++u) {
          const long long e = eb + (long long)u * E + es;
          iq[u] = -1;
          s[u] = 0.f;
          if (e < e1) {
            iq[u] = __builtin_nontemporal_load(xi + e * G + qi);
            s[u] = __builtin_nontemporal_load(se + e);
            if (xv) s[u] *= __builtin_nontemporal_load(xv + e * G + qi);
          }
        }
#pragma unroll
        for (int u = 0; u < kFixUnroll; ++u) {
          if (iq[u] < 0) continue;
          const float* vq = vbase + (long long)iq[u] * k;  // V[i_q, f_i]
#pragma unroll
          for (int j = 0; j < KV; ++j) {
            const float4 v = *reinterpret_cast<const float4*>(vq + 4 * j);
            acc[j].x += s[u] * v.x;
            acc[j].y += s[u] * v.y;
            acc[j].z += s[u] * v.z;
            acc[j].w += s[u] * v.w;
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < KV; ++j) red[wave][lane * KV + j] = acc[j];
    wave_sync();
    if (lane < G && grp * G + lane < m) {
      const int f_out = lay_field[grp * G + lane];
#pragma unroll
      for (int j = 0; j < KV; ++j) {
        float4 t = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int e = 0; e < E; ++e) {
          const float4 a = red[wave][(e * G + lane) * KV + j];
          t.x += a.x; t.y += a.y; t.z += a.z; t.w += a.w;
        }
        *reinterpret_cast<float4*>(part + ch * J + (long long)f_out * k + 4 * j) = t;
      }
    }
    wave_sync();
  }
}

// SGD batch pair gradient (ops/sgd.py), fixed-layout rows (every row holds the same m ==
// nfield fields in the same order; each column sits in one position): one group of 8 lanes
// per CSC chunk of a batch column i (field fa, <= 64 entries: a batch's columns are short,
// hot ones are split), lane q owning the row positions q, q + 8, ... (< 8 per lane). For
// every entry (row r, value x_i, coefficient c_r) the lane gathers V[i_q, fa, :] of its
// positions straight from the model vector ([F][nfield][k]: 16-B aligned k-float slices)
// and accumulates c_r x_i x_q V[i_q, fa] into its positions' field slots in registers;
// the group then writes the chunk's [nfield][k] gradient row once. Against the L-BFGS
// streamed kernel (one wave per column, ~4 entries per column in a 65536-row batch: the
// per-column latency chain dominated) a wave works 8 columns at once and needs neither the
// setup-time row expansion nor a transposed copy of V.
template <int KV, bool kAligned>
__global__ __launch_bounds__(256) void ffm_sgd_grad_kernel(
    const long long* __restrict__ chunk_beg, const long long* __restrict__ chunk_end, long long nch,
    const int* __restrict__ csc_rows, const float* __restrict__ csc_vals, const int* __restrict__ chunk_fa,
    const int* __restrict__ chunk_col, const int* __restrict__ idx, const float* __restrict__ val, int m,
    const int* __restrict__ lay_field, const float* __restrict__ coef, const float* __restrict__ V, int nfield,
    float* __restrict__ part, long long vt_nfeat, int skip_feat) {
  constexpr int GL = 8, PM = 8, k = 4 * KV, U = 4;
  const long long g = (blockIdx.x * 256LL + threadIdx.x) / GL;
  const int q = threadIdx.x & (GL - 1);
  if (g >= nch) return;
  const long long e0 = chunk_beg[g], e1 = chunk_end[g];
  const int fa = chunk_fa[g], col = chunk_col[g];
  const long long J = (long long)nfield * k;
  float4 acc[PM][KV];
#pragma unroll
  for (int j = 0; j < PM; ++j)
#pragma unroll
    for (int v = 0; v < KV; ++v) acc[j][v] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (fa >= 0) {
    // V: the model's [F][nfield][k] (slice fa of row iq at iq * J + fa * k), or with vt_nfeat
    // > 0 the field-major copy [nfield][F][k] (row iq of slice fa at (fa * F + iq) * k: the
    // column's gathers then stay inside one 16-MB field slice)
    const float* vf = vt_nfeat > 0 ? V + (long long)fa * vt_nfeat * k : V + (long long)fa * k;
    const long long vs = vt_nfeat > 0 ? (long long)k : J;
    for (long long eb = e0; eb < e1; eb += U) {
      int r[U];
      float sc[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {  // U entries' row ids / scales in flight
        const long long e = eb + u;
        r[u] = e < e1 ? csc_rows[e] : -1;
        sc[u] = e < e1 ? csc_vals[e] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) sc[u] = r[u] >= 0 ? sc[u] * coef[r[u]] : 0.f;
      int iq[U][PM];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < PM; ++j) {
          const int p = q + GL * j;
          iq[u][j] = (r[u] >= 0 && p < m) ? idx[(long long)r[u] * m + p] : col;
        }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int j = 0; j < PM; ++j) {
          // the entry itself / a padded position / the skipped feature (the bias without a
          // latent factor: its V row need not be zero, e.g. continued from a model saved with one)
          if (iq[u][j] == col || iq[u][j] < 0 || iq[u][j] == skip_feat) continue;
          const float s = val ? sc[u] * val[(long long)r[u] * m + q + GL * j] : sc[u];
          const float* vrow = vf + (long long)iq[u][j] * vs;
#pragma unroll
          for (int v = 0; v < KV; ++v) {
            // V sits behind the F linear weights in the model vector: 16-B aligned iff F % 4 == 0
            const float4 x = kAligned ? reinterpret_cast<const float4*>(vrow)[v]
                                      : make_float4(vrow[4 * v], vrow[4 * v + 1], vrow[4 * v + 2], vrow[4 * v + 3]);
            acc[j][v].x += s * x.x;
            acc[j][v].y += s * x.y;
            acc[j][v].z += s * x.z;
            acc[j][v].w += s * x.w;
          }
        }
    }
  }
#pragma unroll
  for (int j = 0; j < PM; ++j) {
    const int p = q + GL * j;
    if (p < m) {
      float4* out = reinterpret_cast<float4*>(part + g * J + (long long)lay_field[p] * k);
#pragma unroll
      for (int v = 0; v < KV; ++v) out[v] = acc[j][v];
    }
  }
}

// SGD batch step from the forward's pair terms (ffm_pairs_lds_kernel<true> /
// ffm_pairs_k4_kernel<true>, k == 4, fixed-layout rows): a chunk's pair gradient is the sum
// over its entries e (CSC order: deterministic) of c_{row(e)} * E[perm(e)][q] into field slot
// f_q, its linear gradient sum c x. One 32-lane group per kEcolCpg consecutive chunks, lane q
// owning positions q and q + 32 (m <= 64): the group's chunk bounds / fields / columns are
// loaded by its lanes at once, the entries walked in order in windows of 32 whose positions,
// coefficients and values the lanes also load at once (one round trip per window instead of
// a dependent chain per chunk -- measured 717 -> 701 us per batch: the kernel is bound by the
// random 640-B row reads of E, ~2.4 TB/s), U entry rows of E in flight (contiguous m x 16 B
// each -- the 16-B gathers of V that ffm_sgd_grad_kernel makes are replaced by whole-line
// reads). Crossing a chunk end flushes the chunk: a chunk that is
// its column's only one (solo: most columns of a batch) applies the step here, exactly as
// sgd_apply_kernel would from a single chunk (w -= lri (g + cnt l2w w), V -= lri (gV + cnt
// l2v V), bias rules); the others write lat / lin = (sum c x, 0) for sgd_apply over the
// multi-chunk columns. The skipped column (chunk_fa < 0) has all-zero E rows: no latent step.
// kBf: E holds bf16 pair terms (packed 8-B slots; the sums stay fp32) and the bf16 working copy Vb of
// every updated latent slot is re-rounded from its new fp32 value.
constexpr int kEcolCpg = 8;
template <bool kBf = false>
__global__ __launch_bounds__(256) void ffm_sgd_ecol_kernel(
    const long long* __restrict__ chunk_beg, const long long* __restrict__ chunk_end, long long nch,
    const int* __restrict__ csc_rows, const float* __restrict__ csc_vals, const int* __restrict__ csc_perm,
    const int* __restrict__ chunk_fa, const int* __restrict__ chunk_col, const unsigned char* __restrict__ solo,
    const void* __restrict__ Ev, int m, const int* __restrict__ lay_field, const float* __restrict__ coef,
    float* __restrict__ lat, float* __restrict__ lin, float* __restrict__ w, float* __restrict__ V, float lr,
    float l2w, float l2v, int reg_skip, int upd_w, int bias_latent, int avg, uint2* __restrict__ Vb) {
  const float4* __restrict__ E = reinterpret_cast<const float4*>(Ev);
  const uint2* __restrict__ Eh = reinterpret_cast<const uint2*>(Ev);
  constexpr int GL = 32, U = kBf ? 8 : 4;  // bf16: half the registers per row in flight
  const long long grp = (blockIdx.x * 256LL + threadIdx.x) / GL;
  const int q = threadIdx.x & (GL - 1);
  const long long c0 = grp * kEcolCpg;
  if (c0 >= nch) return;  // group-uniform
  const int nc = (int)min<long long>(kEcolCpg, nch - c0);
  long long my_e1 = 0;
  int my_fa = -1, my_col = 0, my_solo = 0;
  if (q < nc) {
    my_e1 = chunk_end[c0 + q];
    my_fa = chunk_fa[c0 + q];
    my_col = chunk_col[c0 + q];
    my_solo = solo[c0 + q];
  }
  const long long E0 = chunk_beg[c0];
  const long long E1 = __shfl(my_e1, nc - 1, GL);
  // lane q owns positions (q, q + 32); bf16 (m even): the adjacent pair (2q, 2q + 1), read as
  // one 16-B load -- the chunk sums are bound by load requests, not bytes
  const int pos0 = kBf ? 2 * q : q, pos1 = kBf ? 2 * q + 1 : q + GL;
  const bool has0 = pos0 < m, has1 = pos1 < m;
  const int lf0 = has0 ? lay_field[pos0] : 0, lf1 = has1 ? lay_field[pos1] : 0;
  const long long J4 = m;  // float4 slots per feature (nfield == m, k == 4)
  int ci = 0;
  long long cbeg = E0, cend = __shfl(my_e1, 0, GL);
  float4 a0 = make_float4(0.f, 0.f, 0.f, 0.f), a1 = a0;
  float glin = 0.f;
  auto flush = [&]() {  // chunk c0 + ci, entries [cbeg, cend); group-uniform
    const long long gc = c0 + ci;
    const int fa = __shfl(my_fa, ci, GL), col = __shfl(my_col, ci, GL), sl = __shfl(my_solo, ci, GL);
    if (!sl) {
      float4* out = reinterpret_cast<float4*>(lat) + gc * J4;
      if (has0) out[lf0] = a0;
      if (has1) out[lf1] = a1;
      if (q == 0) { lin[2 * gc] = glin; lin[2 * gc + 1] = 0.f; }
      return;
    }
    const float cnt = (float)(cend - cbeg);
    const float lri = avg ? lr / fmaxf(cnt, 1.f) : lr;
    const bool is_bias = col == reg_skip;
    if (q == 0 && (upd_w || is_bias)) {
      const float wi = w[col];
      w[col] = wi - lri * (glin + (is_bias ? 0.f : cnt * l2w * wi));
    }
    if (fa < 0 || (is_bias && !bias_latent)) return;
    const float dec = is_bias ? 0.f : cnt * l2v;
    float4* vr = reinterpret_cast<float4*>(V) + (long long)col * J4;
    if (has0) {
      float4* p = vr + lf0;
      const float4 v = *p;
      const float4 nv = make_float4(v.x - lri * (a0.x + dec * v.x), v.y - lri * (a0.y + dec * v.y),
                                    v.z - lri * (a0.z + dec * v.z), v.w - lri * (a0.w + dec * v.w));
      *p = nv;
      if constexpr (kBf) Vb[(long long)col * J4 + lf0] = f4_to_bf4(nv);
    }
    if (has1) {
      float4* p = vr + lf1;
      const float4 v = *p;
      const float4 nv = make_float4(v.x - lri * (a1.x + dec * v.x), v.y - lri * (a1.y + dec * v.y),
                                    v.z - lri * (a1.z + dec * v.z), v.w - lri * (a1.w + dec * v.w));
      *p = nv;
      if constexpr (kBf) Vb[(long long)col * J4 + lf1] = f4_to_bf4(nv);
    }
  };
  for (long long wb = E0; wb < E1; wb += GL) {
    const int n = (int)min<long long>(GL, E1 - wb);
    int prL = -1;
    float scL = 0.f, xL = 0.f;
    if (q < n) {
      prL = csc_perm[wb + q];
      xL = csc_vals[wb + q];
      scL = coef[csc_rows[wb + q]];
    }
    for (int i = 0; i < n; i += U) {
      int pr[U];
      float sc[U], xv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int src = min(i + u, n - 1);
        pr[u] = __shfl(prL, src, GL);
        sc[u] = __shfl(scL, src, GL);
        xv[u] = __shfl(xL, src, GL);
      }
      float4 x0[U], x1[U];
      uint2 h0[U], h1[U];  // bf16: raw slots, every load issued before any is widened
#pragma unroll
      for (int u = 0; u < U; ++u) {
        x0[u] = x1[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        h0[u] = h1[u] = make_uint2(0u, 0u);
        if (i + u < n) {
          if constexpr (kBf) {
            if (has0) {  // m even: has0 implies has1
              const uint4 pair = reinterpret_cast<const uint4*>(Eh + (long long)pr[u] * m)[q];
              h0[u] = make_uint2(pair.x, pair.y);
              h1[u] = make_uint2(pair.z, pair.w);
            }
          } else {
            const float4* row = E + (long long)pr[u] * m;
            if (has0) x0[u] = row[q];
            if (has1) x1[u] = row[q + GL];
          }
        }
      }
      if constexpr (kBf) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          x0[u] = bf4_to_f4(h0[u]);
          x1[u] = bf4_to_f4(h1[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (i + u >= n) break;  // group-uniform
        const long long e = wb + i + u;
        while (e >= cend) {  // the entry opens the next chunk(s)
          flush();
          ++ci;
          cbeg = cend;
          cend = __shfl(my_e1, ci, GL);
          a0 = a1 = make_float4(0.f, 0.f, 0.f, 0.f);
          glin = 0.f;
        }
        glin += sc[u] * xv[u];
        a0.x += sc[u] * x0[u].x; a0.y += sc[u] * x0[u].y; a0.z += sc[u] * x0[u].z; a0.w += sc[u] * x0[u].w;
        a1.x += sc[u] * x1[u].x; a1.y += sc[u] * x1[u].y; a1.z += sc[u] * x1[u].z; a1.w += sc[u] * x1[u].w;
      }
    }
  }
  flush();
}

}  // namespace ytk

using namespace ytk;

static bool getenv_off(const char* name) {
  const char* e = getenv(name);
  return e && e[0] == '0';
}

extern "C" {

// fx[row] = pair interaction sum (forward) or g += pair gradients scaled by coef[row].
void ytk_ffm_pairs(uintptr_t indptr, uintptr_t idx, uintptr_t val, uintptr_t fld, long long nrows,
                   uintptr_t V, int nfield, int k, uintptr_t fx, uintptr_t coef, uintptr_t gV,
                   int backward, int skip_feat, uintptr_t stream, uintptr_t cnt) {
  if (nrows <= 0 || k <= 0) return;
  const long long threads = nrows * 64;
  const dim3 grid((unsigned)((threads + 255) / 256));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int vec4 = ((k & 3) == 0 && (V & 15) == 0) ? 1 : 0;  // 16-B gathers need aligned V
  if (backward && vec4 && k == 4 && (gV & 15) == 0 && !getenv_off("YTK_FFM_K4"))
    hipLaunchKernelGGL(ffm_pairs_k4_bwd_kernel, grid, dim3(256), 0, s, (const long long*)indptr, (const int*)idx,
                       (const float*)val, (const int*)fld, nrows, (const float*)V, nfield, (const float*)coef,
                       (float*)gV, skip_feat, (const int*)cnt);
  else if (backward)
    hipLaunchKernelGGL(ffm_pairs_kernel<true>, grid, dim3(256), 0, s, (const long long*)indptr,
                       (const int*)idx, (const float*)val, (const int*)fld, nrows, (const float*)V,
                       nfield, k, (float*)fx, (const float*)coef, (float*)gV, vec4, skip_feat, (const int*)cnt);
  else if (vec4 && k == 4 && !getenv_off("YTK_FFM_K4"))
    hipLaunchKernelGGL(ffm_pairs_k4_kernel<false>, grid, dim3(256), 0, s, (const long long*)indptr,
                       (const int*)idx, (const float*)val, (const int*)fld, nrows, (const float*)V, nfield,
                       (float*)fx, skip_feat, (float4*)nullptr, 0LL);
  else
    hipLaunchKernelGGL(ffm_pairs_kernel<false>, grid, dim3(256), 0, s, (const long long*)indptr,
                       (const int*)idx, (const float*)val, (const int*)fld, nrows, (const float*)V,
                       nfield, k, (float*)fx, (const float*)coef, (float*)gV, vec4, skip_feat, (const int*)nullptr);
  YTK_LAUNCH_CHECK();
}


// part[chunk, nfield*k] = per-chunk gradient blocks (column-ordered gather backward).
// pk[entry] = feature | field << sh; val may be 0 (all values 1); Vt is V transposed to
// [nfield][nfeat][k] so the gathers of one chunk stay inside one field's slice.
void ytk_ffm_grad_csc(uintptr_t chunk_beg, uintptr_t chunk_end, long long nch, uintptr_t csc_rows,
                      uintptr_t csc_vals, uintptr_t csc_pos, uintptr_t indptr, uintptr_t pk, int sh,
                      uintptr_t val, uintptr_t Vt, long long nfeat, int nfield, int k, uintptr_t coef,
                      uintptr_t part, int skip_feat, int distinct_fields, uintptr_t stream) {
  if (nch <= 0 || k <= 0) return;
  const int J = nfield * k;
  if (J > 2048) throw std::invalid_argument("ffm_grad_csc: nfield*k > 2048");  // 4 x 8 KB LDS
  if (sh <= 0 || sh > 31) throw std::invalid_argument("ffm_grad_csc: bad pack shift");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const size_t lds = (size_t)kCscWaves * J * sizeof(float);
  const bool vec4 = (k & 3) == 0 && (Vt & 15) == 0;  // 16-B gathers and b128 LDS updates
#define YTK_FFM_CSC(VEC, DIS)                                                                  \
  hipLaunchKernelGGL((ffm_grad_csc_kernel<VEC, DIS>),                                         \
                     dim3((unsigned)((nch + kCscWaves - 1) / kCscWaves)), dim3(64 * kCscWaves), \
                     lds, s, (const long long*)chunk_beg, (const long long*)chunk_end, nch,   \
                     (const int*)csc_rows, (const float*)csc_vals, (const long long*)csc_pos,  \
                     (const long long*)indptr, (const unsigned*)pk, sh, (const float*)val,     \
                     (const float*)Vt, nfeat, nfield, k, (const float*)coef, (float*)part,     \
                     skip_feat)
  if (vec4) {
    if (distinct_fields) YTK_FFM_CSC(true, true); else YTK_FFM_CSC(true, false);
  } else {
    if (distinct_fields) YTK_FFM_CSC(false, true); else YTK_FFM_CSC(false, false);
  }
#undef YTK_FFM_CSC
  YTK_LAUNCH_CHECK();
}

// Fixed-layout XCD-split streamed variant (see ffm_grad_stream_kernel): exp_idx / exp_val
// [8][nnz][G] (G = ceil(m / 8); exp_val may be 0 for unit values), se[nnz] the per-entry
// scales, chunk_fa[nch] the chunk's column field (-1: write zeros), lay_field[m] the field of
// each position (a permutation of 0..nfield-1), wave_chunk[nwaves+1] the chunk range of each
// wave. Writes every part[chunk] slot.
void ytk_ffm_grad_stream(uintptr_t wave_chunk, long long nwaves, uintptr_t chunk_beg, uintptr_t chunk_end,
                         uintptr_t chunk_fa, uintptr_t exp_idx, uintptr_t exp_val, uintptr_t se, long long nnz,
                         uintptr_t lay_field, int m, uintptr_t Vt, long long nfeat, int nfield, int k,
                         uintptr_t part, uintptr_t stream) {
  if (nwaves <= 0) return;
  if (m < 8 || m > 512 || m != nfield) throw std::invalid_argument("ffm_grad_stream: need 8 <= m == nfield <= 512");
  if ((Vt & 15) || (part & 15)) throw std::invalid_argument("ffm_grad_stream: Vt / part must be 16-B aligned");
  const int G = (m + 7) / 8;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid((unsigned)(8 * ((nwaves + kCscWaves - 1) / kCscWaves)));
#define YTK_FFM_STREAM(KV)                                                                         \
  hipLaunchKernelGGL((ffm_grad_stream_kernel<KV>), grid, dim3(64 * kCscWaves), 0, s,               \
                     (const long long*)wave_chunk, nwaves, (const long long*)chunk_beg,            \
                     (const long long*)chunk_end, (const int*)chunk_fa, (const int*)exp_idx,       \
                     (const float*)exp_val, (const float*)se, nnz, G, (const int*)lay_field, m,    \
                     (const float*)Vt, nfeat, nfield, (float*)part)
  if (k == 4) YTK_FFM_STREAM(1);
  else if (k == 8) YTK_FFM_STREAM(2);
  else if (k == 16) YTK_FFM_STREAM(4);
  else throw std::invalid_argument("ffm_grad_stream: k must be 4, 8 or 16");
#undef YTK_FFM_STREAM
  YTK_LAUNCH_CHECK();
}

// SGD batch pair gradient over fixed-layout rows (see ffm_sgd_grad_kernel); idx / val: the
// batch's CSR entries (rows of m entries; val null for unit values); skipped columns have
// chunk_fa < 0 (their rows of part are zero).
void ytk_ffm_sgd_grad(uintptr_t chunk_beg, uintptr_t chunk_end, long long nch, uintptr_t csc_rows, uintptr_t csc_vals,
                      uintptr_t chunk_fa, uintptr_t chunk_col, uintptr_t idx, uintptr_t val, int m, uintptr_t lay_field,
                      uintptr_t coef, uintptr_t V, int nfield, int k, uintptr_t part, long long vt_nfeat,
                      int skip_feat, uintptr_t stream) {
  if (nch <= 0) return;
  if (m < 1 || m > 64 || m != nfield) throw std::invalid_argument("ffm_sgd_grad: need 1 <= m == nfield <= 64");
  if ((V & 3) || (part & 15)) throw std::invalid_argument("ffm_sgd_grad: V 4-B / part 16-B aligned");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid((unsigned)((nch * 8 + 255) / 256));
  const bool al = (V & 15) == 0;
#define YTK_FFM_SGD(KV)                                                                                     \
  if (al) YTK_FFM_SGD2(KV, true); else YTK_FFM_SGD2(KV, false)
#define YTK_FFM_SGD2(KV, AL)                                                                                \
  hipLaunchKernelGGL((ffm_sgd_grad_kernel<KV, AL>), grid, dim3(256), 0, s, (const long long*)chunk_beg,     \
                     (const long long*)chunk_end, nch, (const int*)csc_rows, (const float*)csc_vals,        \
                     (const int*)chunk_fa, (const int*)chunk_col, (const int*)idx, (const float*)val, m,    \
                     (const int*)lay_field, (const float*)coef, (const float*)V, nfield, (float*)part, vt_nfeat, \
                     skip_feat)
  if (k == 4) YTK_FFM_SGD(1);
  else if (k == 8) YTK_FFM_SGD(2);
  else throw std::invalid_argument("ffm_sgd_grad: k must be 4 or 8");
#undef YTK_FFM_SGD
#undef YTK_FFM_SGD2
  YTK_LAUNCH_CHECK();
}

// Forward pair sums of fixed-layout rows (k == 4, V 16-B aligned) that also write the pair
// terms E[entry - e_base][m] (float4) for ffm_sgd_ecol (see ffm_pairs_k4_kernel).
void ytk_ffm_pairs_fwd_e(uintptr_t indptr, uintptr_t idx, uintptr_t val, uintptr_t fld, long long nrows,
                         uintptr_t V, int nfield, uintptr_t fx, int skip_feat, uintptr_t E, long long e_base, int m,
                         uintptr_t stream) {
  if (nrows <= 0) return;
  if ((V & 15) || (E & 15)) throw std::invalid_argument("ffm_pairs_fwd_e: V / E must be 16-B aligned");
  if (m < 1 || m > 64) throw std::invalid_argument("ffm_pairs_fwd_e: rows of 1..64 entries");
  const long long threads = nrows * 64;
  const size_t lds = (size_t)4 * (m * (m - 1) / 2) * sizeof(float4);  // 4 waves per block
  hipLaunchKernelGGL(ffm_pairs_k4_kernel<true>, dim3((unsigned)((threads + 255) / 256)), dim3(256), lds,
                     reinterpret_cast<hipStream_t>(stream), (const long long*)indptr, (const int*)idx,
                     (const float*)val, (const int*)fld, nrows, (const float*)V, nfield, (float*)fx, skip_feat,
                     (float4*)E, e_base);
  YTK_LAUNCH_CHECK();
}

// One SGD batch step's pair gradient + the update of every single-chunk column (see
// ffm_sgd_ecol_kernel); csc_perm: the batch-relative CSR position of each CSC entry (int32);
// nfield == m <= 64, k == 4; lat [nch][m * 4] / lin [nch][2]: the multi-chunk columns' partials.
void ytk_ffm_sgd_ecol(uintptr_t chunk_beg, uintptr_t chunk_end, long long nch, uintptr_t csc_rows, uintptr_t csc_vals,
                      uintptr_t csc_perm, uintptr_t chunk_fa, uintptr_t chunk_col, uintptr_t solo, uintptr_t E, int m,
                      uintptr_t lay_field, uintptr_t coef, uintptr_t lat, uintptr_t lin, uintptr_t w, uintptr_t V,
                      float lr, float l2w, float l2v, int reg_skip, int upd_w, int bias_latent, int avg,
                      uintptr_t Vb, uintptr_t stream) {
  // Vb != 0: E holds bf16 pair terms and the bf16 working copy Vb ([F][m] 8-B slots) is kept
  if (nch <= 0) return;
  if (m < 1 || m > 64) throw std::invalid_argument("ffm_sgd_ecol: need 1 <= m <= 64");
  if ((E & 15) || (lat & 15) || (V & 15) || (Vb & 7) || (Vb && (m & 1)))
    throw std::invalid_argument("ffm_sgd_ecol: E / lat / V 16-B aligned, Vb 8-B; bf16 needs an even m");
  const dim3 grid((unsigned)(((nch + kEcolCpg - 1) / kEcolCpg * 32 + 255) / 256));
#define YTK_ECOL(BF)                                                                                          \
  hipLaunchKernelGGL(ffm_sgd_ecol_kernel<BF>, grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream),     \
                     (const long long*)chunk_beg, (const long long*)chunk_end, nch, (const int*)csc_rows,     \
                     (const float*)csc_vals, (const int*)csc_perm, (const int*)chunk_fa, (const int*)chunk_col, \
                     (const unsigned char*)solo, (const void*)E, m, (const int*)lay_field, (const float*)coef, \
                     (float*)lat, (float*)lin, (float*)w, (float*)V, lr, l2w, l2v, reg_skip, upd_w, bias_latent, \
                     avg, (uint2*)Vb)
  if (Vb) YTK_ECOL(true);
  else YTK_ECOL(false);
#undef YTK_ECOL
  YTK_LAUNCH_CHECK();
}

// Forward pair sums with the row's latent rows staged in LDS (see ffm_pairs_lds_kernel):
// k == 4, V 16-B aligned, every row of <= max_m <= 64 entries, max_m * (nfield + 1) * 16 B of
// LDS. E != 0: fixed-layout rows of exactly max_m entries, also writing the SGD pair terms
// E[entry - e_base][max_m] (float4).
// bf16 = 1: V is the bf16 working copy ([F][nfield] 8-B slots) and E (SGD) is written as bf16.
void ytk_ffm_pairs_lds(uintptr_t indptr, uintptr_t idx, uintptr_t val, uintptr_t fld, long long nrows, uintptr_t V,
                       int nfield, uintptr_t fx, int skip_feat, int max_m, uintptr_t E, long long e_base,
                       int bf16, uintptr_t stream) {
  if (nrows <= 0) return;
  if ((V & 15) || (E & 15)) throw std::invalid_argument("ffm_pairs_lds: V / E must be 16-B aligned");
  if (bf16 && E && (max_m & 1)) throw std::invalid_argument("ffm_pairs_lds: bf16 pair terms need even rows");
  if (max_m < 1 || max_m > 64 || nfield < 1) throw std::invalid_argument("ffm_pairs_lds: 1 <= max_m <= 64");
  const size_t lds = (size_t)max_m * (nfield + 1) * sizeof(float4);
  if (lds > 64 * 1024) throw std::invalid_argument("ffm_pairs_lds: max_m * (nfield + 1) * 16 B > 64 KiB");
  const long long grid = std::min<long long>(nrows, 256LL * 32);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
#define YTK_LDS(KE, BF)                                                                                   \
  hipLaunchKernelGGL((ffm_pairs_lds_kernel<KE, BF>), dim3((unsigned)grid), dim3(64), lds, s,              \
                     (const long long*)indptr, (const int*)idx, (const float*)val, (const int*)fld, nrows, \
                     (const void*)V, nfield, (float*)fx, skip_feat, (void*)E, KE ? e_base : 0LL)
  if (E && bf16) YTK_LDS(true, true);
  else if (E) YTK_LDS(true, false);
  else if (bf16) YTK_LDS(false, true);
  else YTK_LDS(false, false);
#undef YTK_LDS
  YTK_LAUNCH_CHECK();
}

}  // extern "C"
