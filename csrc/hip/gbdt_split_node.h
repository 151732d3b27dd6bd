// Split-search definitions shared by the split kernels (gbdt_split.hip) and the fused
// split + level-planner kernel (gbdt_level.hip). See gbdt_split.hip for the reference
// semantics (DataParallelTreeMaker.java:598-637, UpdateStrategy.java:50-100).
#pragma once
#include "common.h"

namespace ytk {

struct SplitOut {
  float loss_chg;
  int feat;
  int bin_a;  // last non-empty bin going left
  int bin_b;  // first non-empty bin going right
  double gl, hl;  // left sums
  double g, h;    // node sums
};
static_assert(sizeof(SplitOut) == 48, "SplitOut layout");

struct GainParams {
  float mcw;  // min_child_hessian_sum
  float l1, l2;
  float max_abs_leaf;
  double inv_sg, inv_sh;  // fixed-point -> real
};

__device__ __forceinline__ double thr_l1(double w, double lam) {
  if (w > lam) return w - lam;
  if (w < -lam) return w + lam;
  return 0.0;
}

__device__ __forceinline__ double node_value(double g, double h, const GainParams& p) {
  if (h < (double)p.mcw) return 0.0;
  double v = (p.l1 == 0.f) ? -g / (h + p.l2) : -thr_l1(g, p.l1) / (h + p.l2);
  if (p.max_abs_leaf > 0.f) {
    if (v > p.max_abs_leaf) v = p.max_abs_leaf;
    else if (v < -p.max_abs_leaf) v = -p.max_abs_leaf;
  }
  return v;
}

__device__ __forceinline__ double calc_gain(double g, double h, const GainParams& p) {
  if (h < (double)p.mcw) return 0.0;
  if (p.max_abs_leaf <= 0.f) {
    if (p.l1 == 0.f) return g * g / (h + p.l2);
    const double t = thr_l1(g, p.l1);
    return t * t / (h + p.l2);
  }
  const double v = node_value(g, h, p);
  return -2.0 * (g * v + 0.5 * (h + p.l2) * v * v + p.l1 * fabs(v));
}

// (chg, feat, bin) lexicographic "better": larger chg, then lower feat, then lower bin.
__device__ __forceinline__ bool better(float c1, int f1, int b1, float c2, int f2, int b2) {
  if (c1 != c2) return c1 > c2;
  if (f1 != f2) return f1 < f2;
  return b1 < b2;
}

// ---------------------------------------------------------------------------------
// One block per NODE with the node's whole histogram resident in LDS (B * F small
// enough, e.g. 28 x 257 x 16 B = 115 KB) -- the default when it fits. The hist layout
// [bin][feature] makes a per-feature read a 16-byte gather at stride F*16 B: with one
// block per (node, feature) every block touches every cache line of the node's histogram
// (F-fold L2 traffic). Here the block streams the histogram ONCE, coalesced (fusing the
// parent - sibling subtraction and its write-back), transposes it into LDS as
// [feature][B+1] (odd 16-byte stride: the transposing stores spread over the banks, the
// per-feature reads are contiguous), then wave w scans features w, w+16, ...: a lane owns
// 4 consecutive bins, one DPP wave scan per feature (no LDS-routed shuffles -- with 16
// waves on one CU those were the bottleneck), and the per-wave argmax is one 64-bit DPP
// max over a packed (gain, -feature, -bin) key.
constexpr int kNodeThreads = 1024;
constexpr size_t kNodeLdsMax = 144 * 1024;  // of the 160 KB per CU
constexpr int kNodeLoads = 8;                // entries per thread: B * F <= 8192
constexpr int kNodeMaxF = 256;

// v from lane (l - s) within a row of 16 / broadcast row patterns (GFX9 DPP), `fill` where
// the source is outside the row or the row is masked off
template <int kCtrl, int kRowMask>
__device__ __forceinline__ int dpp32(int v, int fill) {
  return __builtin_amdgcn_update_dpp(fill, v, kCtrl, kRowMask, 0xf, false);
}
template <int kCtrl, int kRowMask>
__device__ __forceinline__ unsigned long long dpp64(unsigned long long v) {
  const int lo = dpp32<kCtrl, kRowMask>((int)(unsigned)v, 0);
  const int hi = dpp32<kCtrl, kRowMask>((int)(unsigned)(v >> 32), 0);
  return ((unsigned long long)(unsigned)hi << 32) | (unsigned)lo;
}
constexpr int kShr1 = 0x111, kShr2 = 0x112, kShr4 = 0x114, kShr8 = 0x118;
constexpr int kBcast15 = 0x142, kBcast31 = 0x143;

// inclusive wave scans (Hillis-Steele within rows of 16, then the two row broadcasts)
__device__ __forceinline__ long long dpp_scan_add(long long x) {
  unsigned long long u = (unsigned long long)x;
  u += dpp64<kShr1, 0xf>(u);
  u += dpp64<kShr2, 0xf>(u);
  u += dpp64<kShr4, 0xf>(u);
  u += dpp64<kShr8, 0xf>(u);
  u += dpp64<kBcast15, 0xa>(u);
  u += dpp64<kBcast31, 0xc>(u);
  return (long long)u;
}
__device__ __forceinline__ int dpp_scan_max(int x) {  // values >= -1
  x = max(x, dpp32<kShr1, 0xf>(x, -1));
  x = max(x, dpp32<kShr2, 0xf>(x, -1));
  x = max(x, dpp32<kShr4, 0xf>(x, -1));
  x = max(x, dpp32<kShr8, 0xf>(x, -1));
  x = max(x, dpp32<kBcast15, 0xa>(x, -1));
  x = max(x, dpp32<kBcast31, 0xc>(x, -1));
  return x;
}
__device__ __forceinline__ unsigned long long dpp_max_u64(unsigned long long x) {  // lane 63 = max
  unsigned long long o;
  o = dpp64<kShr1, 0xf>(x); x = o > x ? o : x;
  o = dpp64<kShr2, 0xf>(x); x = o > x ? o : x;
  o = dpp64<kShr4, 0xf>(x); x = o > x ? o : x;
  o = dpp64<kShr8, 0xf>(x); x = o > x ? o : x;
  o = dpp64<kBcast15, 0xa>(x); x = o > x ? o : x;
  o = dpp64<kBcast31, 0xc>(x); x = o > x ? o : x;
  return x;
}
__device__ __forceinline__ long long readlane64(long long v, int lane) {
  const unsigned lo = __builtin_amdgcn_readlane((int)(unsigned)(unsigned long long)v, lane);
  const unsigned hi = __builtin_amdgcn_readlane((int)(unsigned)((unsigned long long)v >> 32), lane);
  return (long long)(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ double readlane_f64(double v, int lane) {
  return __longlong_as_double(readlane64(__double_as_longlong(v), lane));
}

// One wave scans one feature's histogram row (LDS, bins [0, nb)): lane l owns bins 4l..4l+3,
// DPP prefix sums of the exact int64 (g, h), and the wave's best split (better() order) over
// the bins whose both sides hold >= mcw hessian, gains in double as the reference
// (UpdateStrategy.java:50-100). (A float pre-filter that evaluated only near-maximal bins in
// double was tried and measured no faster: the scan is latency bound, not fp64 bound --
// docs/performance.md, round 5.) tp (optional): wave-0 timestamps for tools/dbg_rs_prof.py.
__device__ __forceinline__ void wave_feature_scan(const longlong2* __restrict__ hrow, int nb, int f, long long Gq,
                                                  long long Hq, float root_gain, const GainParams& gp,
                                                  float& best_chg, int& best_f, int& best_a, int& best_b,
                                                  double& best_gl, double& best_hl,
                                                  unsigned long long* tp = nullptr) {
  const int l = lane_id();
  if (tp && l == 0) tp[0] = wall_clock64();
  longlong2 q[4];
  long long sg = 0, sh = 0;
  int lastne = -1;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int bin = 4 * l + k;
    q[k] = (bin < nb) ? hrow[bin] : make_longlong2(0, 0);
    sg += q[k].x;
    sh += q[k].y;
    if (q[k].x != 0 || q[k].y != 0) lastne = bin;
  }
  const long long ig = dpp_scan_add(sg), ih = dpp_scan_add(sh);
  const int im = dpp_scan_max(lastne);
  int prev = __shfl_up(im, 1, kWave);
  if (l == 0) prev = -1;
  long long pg = ig - sg, ph = ih - sh;
  if (tp && l == 0) tp[1] = wall_clock64() + (unsigned long long)(prev == 12345);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int bin = 4 * l + k;
    if (q[k].x != 0 || q[k].y != 0) {
      if (prev >= 0 && ph != 0) {
        const double dgl = (double)pg * gp.inv_sg, dhl = (double)ph * gp.inv_sh;
        const double dgr = (double)(Gq - pg) * gp.inv_sg, dhr = (double)(Hq - ph) * gp.inv_sh;
        if (dhl >= (double)gp.mcw && dhr >= (double)gp.mcw) {
          const float chg = (float)(calc_gain(dgl, dhl, gp) + calc_gain(dgr, dhr, gp) - (double)root_gain);
          if (better(chg, f, bin, best_chg, best_f, best_b)) {
            best_chg = chg; best_f = f; best_a = prev; best_b = bin;
            best_gl = dgl; best_hl = dhl;
          }
        }
      }
      pg += q[k].x;
      ph += q[k].y;
      prev = bin;
    }
  }
  if (tp && l == 0) tp[2] = wall_clock64() + (unsigned long long)(best_chg == 12345.f);
}

// The node-resident split search of one node by one kNodeThreads block: item `it`, result
// to *out. sh_hist: dynamic LDS of F * Bp longlong2; nb/fm: per-feature bin counts and
// feature mask (read into LDS here together with the histogram).
// Features [fbeg, fend) of the node only (feature groups: one node searched by several
// blocks, each writing its own record; the level planner keeps the best by better()).
// The node totals come from the group's copy of feature f0 when the group holds it, else
// from its first feature: every row adds its (g, h) to exactly one bin of EVERY feature, so
// the exact int64 sums are the same for all features.
// 16-B histogram pair; kCoh: read with device-coherent atomic loads (data just accumulated
// by other blocks' memory-side atomics in the same launch, no acquire fence)
template <bool kCoh>
__device__ __forceinline__ longlong2 hist_ld2(const longlong2* p) {
  if constexpr (kCoh) {
    long long* q = const_cast<long long*>(reinterpret_cast<const long long*>(p));
    return make_longlong2(__hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                          __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  } else {
    return *p;
  }
}

// kThreads: block size (1024 for the split kernels; 256 in the reduce + split tail of
// lv_reduce_split_kernel, which searches one 8-feature group). kCoh: the built slot (hn of a
// built item, hs of a derived one) is read with coherent loads (hist_ld2).
template <int kThreads = kNodeThreads, bool kCoh = false>
__device__ __forceinline__ void split_node_block(long long* __restrict__ hist, int B, int F, int Bp,
                                                 const int* __restrict__ nbins_f,
                                                 const uint8_t* __restrict__ fmask, int f0, int4 it,
                                                 SplitOut* __restrict__ out, const GainParams& gp,
                                                 longlong2* sh_hist, int fbeg = 0, int fend = -1) {
  if (fend < 0) fend = F;
  const int FG = fend - fbeg;
  constexpr int kW = kThreads / kWave;
  __shared__ float s_chg[kW];
  __shared__ int s_feat[kW], s_a[kW], s_b[kW];
  __shared__ double s_gl[kW], s_hl[kW];
  __shared__ int s_nb[kNodeMaxF];
  __shared__ uint8_t s_fm[kNodeMaxF];
  const int t = threadIdx.x, wid = t >> 6, l = lane_id();
  int nb_t = 0;
  uint8_t fm_t = 0;
  if (t < FG) { nb_t = nbins_f[fbeg + t]; fm_t = fmask[fbeg + t]; }
  const size_t slot_sz = (size_t)B * F * 2;
  longlong2* hn = reinterpret_cast<longlong2*>(hist + (size_t)it.x * slot_sz);
  const longlong2* hp = reinterpret_cast<const longlong2*>(hist + (size_t)it.y * slot_sz);
  const longlong2* hs = reinterpret_cast<const longlong2*>(hist + (size_t)it.z * slot_sz);
  const bool derived = it.w != 0;
  // ---- stream the node's histogram (this group's features) into LDS (all loads of a
  // thread in flight at once); local entry i = bin * FG + fl -> global bin * F + fbeg + fl
  const int total = B * FG;
  auto gidx = [&](int i) { const int bin = i / FG; return bin * F + fbeg + (i - bin * FG); };
  longlong2 v[kNodeLoads];
  if (derived) {
    longlong2 s[kNodeLoads];
#pragma unroll
    for (int j = 0; j < kNodeLoads; ++j) {
      const int i = t + j * kThreads;
      if (i < total) { const int gi = gidx(i); v[j] = hp[gi]; s[j] = hist_ld2<kCoh>(hs + gi); }
    }
#pragma unroll
    for (int j = 0; j < kNodeLoads; ++j) {
      const int i = t + j * kThreads;
      if (i < total) {
        v[j] = make_longlong2(v[j].x - s[j].x, v[j].y - s[j].y);
        hn[gidx(i)] = v[j];
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < kNodeLoads; ++j) {
      const int i = t + j * kThreads;
      if (i < total) v[j] = hist_ld2<kCoh>(hn + gidx(i));
    }
  }
#pragma unroll
  for (int j = 0; j < kNodeLoads; ++j) {
    const int i = t + j * kThreads;
    if (i < total) {
      const int bin = i / FG, f = i - bin * FG;
      sh_hist[f * Bp + bin] = v[j];
    }
  }
  if (t < FG) { s_nb[t] = nb_t; s_fm[t] = fm_t; }
  __syncthreads();
  // ---- node totals (exact int64, first sampled feature: DataParallelTreeMaker:543-573);
  // every wave computes them itself (no extra barrier)
  long long Gq, Hq;
  {
    const int ft = (f0 >= fbeg && f0 < fend) ? f0 - fbeg : 0;  // local feature of the totals
    const int nb0 = s_nb[ft];
    long long sg = 0, sh = 0;
    for (int bin = l; bin < nb0; bin += kWave) {
      const longlong2 q = sh_hist[ft * Bp + bin];
      sg += q.x;
      sh += q.y;
    }
    Gq = readlane64(dpp_scan_add(sg), kWave - 1);
    Hq = readlane64(dpp_scan_add(sh), kWave - 1);
  }
  const double G = (double)Gq * gp.inv_sg, H = (double)Hq * gp.inv_sh;
  const float root_gain = (float)calc_gain(G, H, gp);

  float best_chg = -INFINITY;
  int best_f = 0xffff, best_a = -1, best_b = 0xffff;
  double best_gl = 0.0, best_hl = 0.0;
  for (int fl = wid; fl < FG; fl += kW) {
    if (!s_fm[fl]) continue;  // wave-uniform
    wave_feature_scan(sh_hist + fl * Bp, s_nb[fl], fbeg + fl, Gq, Hq, root_gain, gp, best_chg, best_f, best_a, best_b,
                      best_gl, best_hl);
  }
  // ---- wave argmax: max of (ordered gain bits, ~feature, ~bin) == better()
  {
    const unsigned u = __float_as_uint(best_chg + 0.0f);  // -0 -> +0 (better() equates them)
    const unsigned ord = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
    const unsigned long long key = ((unsigned long long)ord << 32) |
                                   ((unsigned)(0xffff - best_f) << 16) | (unsigned)(0xffff - best_b);
    const unsigned long long kmax = (unsigned long long)readlane64((long long)dpp_max_u64(key), kWave - 1);
    const unsigned long long hit = __ballot(key == kmax);
    const int src = __builtin_ctzll(hit);
    if (l == 0) {
      s_chg[wid] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(best_chg), src));
      s_feat[wid] = __builtin_amdgcn_readlane(best_f, src);
      s_a[wid] = __builtin_amdgcn_readlane(best_a, src);
      s_b[wid] = __builtin_amdgcn_readlane(best_b, src);
    }
    const double gl = readlane_f64(best_gl, src), hl = readlane_f64(best_hl, src);
    if (l == 0) { s_gl[wid] = gl; s_hl[wid] = hl; }
  }
  __syncthreads();
  if (t == 0) {
    int bw = 0;
    for (int w = 1; w < kW; ++w)
      if (better(s_chg[w], s_feat[w], s_b[w], s_chg[bw], s_feat[bw], s_b[bw])) bw = w;
    SplitOut o;
    o.loss_chg = s_chg[bw];
    o.feat = (s_feat[bw] == 0xffff) ? -1 : s_feat[bw];
    o.bin_a = s_a[bw];
    o.bin_b = (s_b[bw] == 0xffff) ? -1 : s_b[bw];
    o.gl = s_gl[bw];
    o.hl = s_hl[bw];
    o.g = G;
    o.h = H;
    *out = o;
  }
}


}  // namespace ytk
