// GBDT best-split search over exact int64 fixed-point histograms (gfx950, wave64).
//
// Reference semantics:
//   split enumeration    J/optimizer/gbdt/DataParallelTreeMaker.java:598-637
//     (left-to-right bin scan, empty bins (g==0 && h==0) skipped, a hit on an
//      empty left sum (H==0) only initialises it, min_child_hessian_sum both sides)
//   gain / leaf value    J/optimizer/gbdt/UpdateStrategy.java:50-100
//   node totals          DataParallelTreeMaker.java:543-573 (first sampled feature)
//   tie-break            J/data/gbdt/SplitInfo.java:99-104 (max lossChg, then lower
//                        feature; within a feature the first bin)
//
// Design: one workgroup (4 waves) per node; wave w owns features w, w+4, ...; a lane
// owns 4 consecutive bins; int64 wave prefix scans (exact) -> prefix sums are
// converted to double only to evaluate gains; (chg, feature, bin) argmax is
// lexicographic -> deterministic. Sibling subtraction (parent - small child) is
// fused into the load (exact in int64) and written back for the node's children.
#include "common.h"

#include <rocprim/block/block_scan.hpp>

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

__device__ __forceinline__ long long wave_incl_scan_ll(long long v) {
  const int l = lane_id();
#pragma unroll
  for (int off = 1; off < kWave; off <<= 1) {
    const long long o = __shfl_up(v, off, kWave);
    if (l >= off) v += o;
  }
  return v;
}

__device__ __forceinline__ long long wave_sum_ll(long long v) {
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// hist: int64 [slot][B][F][2]. items[blk] = {slot, parent_slot, sibling_slot, derived}
constexpr int kSplitWaves = 8;   // 512 threads (<= 256 VGPRs): one block covers F <= 32 (<= 4 / wave)
constexpr int kFPW = 4;          // features per wave per block (hoisted loads)

// Latency design (a level's split search is a chain of dependent memory round trips,
// not bandwidth): each wave issues the loads of ALL its features (<= 4) plus the
// node-total feature up front -- one HBM/L2 round trip -- then scans/evaluates from
// registers. With F <= 32 one block owns a whole node: no cross-block combine.
// For F > 32 the features are spread over gridDim.y blocks and the last block of an
// item (device-scope counter) combines the per-block candidates (same tie-break).
__global__ __launch_bounds__(kSplitWaves * 64) void split_find_kernel(
    long long* __restrict__ hist, int B, int F, const int* __restrict__ nbins_f,
    const uint8_t* __restrict__ fmask, int f0, const int4* __restrict__ items,
    SplitOut* __restrict__ out, GainParams gp, const int* __restrict__ nitems_dev,
    const double* __restrict__ inv_dev, SplitOut* __restrict__ part, int* __restrict__ counters) {
  __shared__ float s_chg[kSplitWaves];
  __shared__ int s_feat[kSplitWaves], s_a[kSplitWaves], s_b[kSplitWaves];
  __shared__ double s_gl[kSplitWaves], s_hl[kSplitWaves];
  __shared__ int s_last;

  if (nitems_dev && (int)blockIdx.x >= *nitems_dev) return;
  const int ngroups = (int)gridDim.y;
  const int fstep = ngroups * kSplitWaves;
  if (inv_dev) {
    gp.inv_sg = inv_dev[0];
    gp.inv_sh = inv_dev[1];
  }
  const int4 it = items[blockIdx.x];
  const int wid = threadIdx.x >> 6;
  const int l = lane_id();
  const size_t slot_sz = (size_t)B * F * 2;
  longlong2* hn = reinterpret_cast<longlong2*>(hist + (size_t)it.x * slot_sz);
  const longlong2* hp = reinterpret_cast<const longlong2*>(hist + (size_t)it.y * slot_sz);
  const longlong2* hs = reinterpret_cast<const longlong2*>(hist + (size_t)it.z * slot_sz);
  const bool derived = it.w != 0;

  auto load = [&](int f, int bin) -> longlong2 {
    const size_t idx = (size_t)bin * F + f;
    if (derived) {
      const longlong2 p = hp[idx], s = hs[idx];
      return make_longlong2(p.x - s.x, p.y - s.y);
    }
    return hn[idx];
  };

  // this wave's features: fw[j] = blockIdx.y*kSplitWaves + wid + j*fstep
  int fw[kFPW];
  int nfw = 0;
#pragma unroll
  for (int j = 0; j < kFPW; ++j) {
    const int f = (int)blockIdx.y * kSplitWaves + wid + j * fstep;
    fw[j] = f;
    if (f < F) nfw = j + 1;
  }
  const bool one_chunk = B <= 4 * kWave;

  // ---- one batch of loads: node-total feature f0 + the first chunk of every feature
  longlong2 v0[4];
  longlong2 vf[kFPW][4];
  {
    const int nb0 = nbins_f[f0];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int bin = l + k * kWave;  // strided: only a sum is needed
      v0[k] = (bin < nb0 && bin < B) ? load(f0, bin) : make_longlong2(0, 0);
    }
  }
  if (one_chunk) {
#pragma unroll
    for (int j = 0; j < kFPW; ++j) {
      const int f = fw[j];
      const int nb = (j < nfw && fmask[f]) ? nbins_f[f] : 0;
      const int nbd = (j < nfw) ? B : 0;  // derived write-back covers every bin
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int bin = 4 * l + k;
        vf[j][k] = make_longlong2(0, 0);
        if (bin < nb || (derived && bin < nbd)) vf[j][k] = load(f, bin);
      }
    }
  }
  // node totals (exact int64; the first sampled feature, DataParallelTreeMaker:543-573)
  long long Gq, Hq;
  {
    long long sg = 0, sh = 0;
    const int nb0 = nbins_f[f0];
    for (int k = 0; k < 4; ++k) { sg += v0[k].x; sh += v0[k].y; }
    for (int bin = l + 4 * kWave; bin < nb0; bin += kWave) {  // B > 256 only
      const longlong2 v = load(f0, bin);
      sg += v.x;
      sh += v.y;
    }
    Gq = wave_sum_ll(sg);
    Hq = wave_sum_ll(sh);
  }
  const double G = (double)Gq * gp.inv_sg, H = (double)Hq * gp.inv_sh;
  const float root_gain = (float)calc_gain(G, H, gp);

  float best_chg = -INFINITY;
  int best_f = 0x7fffffff, best_a = -1, best_b = 0x7fffffff;
  double best_gl = 0.0, best_hl = 0.0;

#pragma unroll
  for (int j = 0; j < kFPW; ++j) {
    const int f = fw[j];
    const bool on = j < nfw && fmask[f] != 0;
    if (j >= nfw || (!on && !derived)) continue;
    const int nb = nbins_f[f];
    long long carry_g = 0, carry_h = 0;
    int carry_last = -1;
    for (int c = 0; c < B; c += 4 * kWave) {
      longlong2 v[4];
      long long sg = 0, sh = 0;
      int lastne = -1;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int bin = c + 4 * l + k;
        if (one_chunk) {
          v[k] = vf[j][k];
        } else {
          v[k] = make_longlong2(0, 0);
          if ((on && bin < nb) || (derived && bin < B)) v[k] = load(f, bin);
        }
        if (derived && bin < B) hn[(size_t)bin * F + f] = v[k];
        if (!on || bin >= nb) v[k] = make_longlong2(0, 0);
        sg += v[k].x;
        sh += v[k].y;
        if (v[k].x != 0 || v[k].y != 0) lastne = bin;
      }
      if (!on) continue;  // derived write-back only
      const long long ig = wave_incl_scan_ll(sg);
      const long long ih = wave_incl_scan_ll(sh);
      const int im = wave_incl_max(lastne);
      int em = __shfl_up(im, 1, kWave);
      if (l == 0) em = -1;
      long long pg = ig - sg + carry_g;
      long long ph = ih - sh + carry_h;
      int prev = max(em, carry_last);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int bin = c + 4 * l + k;
        const bool ne = (v[k].x != 0 || v[k].y != 0);
        if (ne) {
          const double dgl = (double)pg * gp.inv_sg, dhl = (double)ph * gp.inv_sh;
          if (prev >= 0 && ph != 0 && dhl >= (double)gp.mcw) {
            const double dgr = (double)(Gq - pg) * gp.inv_sg, dhr = (double)(Hq - ph) * gp.inv_sh;
            if (dhr >= (double)gp.mcw) {
              const float chg =
                  (float)(calc_gain(dgl, dhl, gp) + calc_gain(dgr, dhr, gp) - (double)root_gain);
              if (better(chg, f, bin, best_chg, best_f, best_b)) {
                best_chg = chg; best_f = f; best_a = prev; best_b = bin;
                best_gl = dgl; best_hl = dhl;
              }
            }
          }
          pg += v[k].x;
          ph += v[k].y;
          prev = bin;
        }
      }
      carry_g += __shfl(ig, kWave - 1, kWave);
      carry_h += __shfl(ih, kWave - 1, kWave);
      carry_last = max(carry_last, __shfl(im, kWave - 1, kWave));
    }
  }
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) {
    const float oc = __shfl_xor(best_chg, off, kWave);
    const int of = __shfl_xor(best_f, off, kWave);
    const int oa = __shfl_xor(best_a, off, kWave);
    const int ob = __shfl_xor(best_b, off, kWave);
    const double ogl = __shfl_xor(best_gl, off, kWave);
    const double ohl = __shfl_xor(best_hl, off, kWave);
    if (better(oc, of, ob, best_chg, best_f, best_b)) {
      best_chg = oc; best_f = of; best_a = oa; best_b = ob; best_gl = ogl; best_hl = ohl;
    }
  }
  if (l == 0) {
    s_chg[wid] = best_chg; s_feat[wid] = best_f; s_a[wid] = best_a; s_b[wid] = best_b;
    s_gl[wid] = best_gl; s_hl[wid] = best_hl;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int bw = 0;
    for (int w2 = 1; w2 < kSplitWaves; ++w2)
      if (better(s_chg[w2], s_feat[w2], s_b[w2], s_chg[bw], s_feat[bw], s_b[bw])) bw = w2;
    SplitOut o;
    o.loss_chg = s_chg[bw];
    o.feat = s_feat[bw];  // 0x7fffffff = none (mapped to -1 below)
    o.bin_a = s_a[bw];
    o.bin_b = s_b[bw];
    o.gl = s_gl[bw];
    o.hl = s_hl[bw];
    o.g = G;
    o.h = H;
    s_last = 1;
    if (ngroups > 1) {
      part[(size_t)blockIdx.x * ngroups + blockIdx.y] = o;
      __threadfence();
      const int prev = atomicAdd(&counters[blockIdx.x], 1);
      s_last = (prev == ngroups - 1);
      if (s_last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // see the other groups' parts
        counters[blockIdx.x] = 0;
        const volatile SplitOut* pp = part + (size_t)blockIdx.x * ngroups;
        for (int y = 0; y < ngroups; ++y) {
          const float c = pp[y].loss_chg;
          const int f = pp[y].feat, b = pp[y].bin_b;
          if (y == 0 || better(c, f, b, o.loss_chg, o.feat, o.bin_b)) {
            o.loss_chg = c; o.feat = f; o.bin_a = pp[y].bin_a; o.bin_b = b;
            o.gl = pp[y].gl; o.hl = pp[y].hl;
          }
        }
      }
    }
    if (s_last) {
      if (o.feat == 0x7fffffff) o.feat = -1;
      if (o.bin_b == 0x7fffffff) o.bin_b = -1;
      out[blockIdx.x] = o;
    }
  }
}


// ---------------------------------------------------------------------------------
// One block per (node, feature), one bin per thread (B <= 256) -- the default path.
// A level's split search is latency bound (tiny data, dependent steps), so the work is
// spread as wide as possible: nodes x F blocks; every block does ONE load round trip
// (its feature's bins + the node-total feature f0's bins), one rocPRIM (DPP) block scan
// of (g, h, last-non-empty-bin), the gain of its bin, and a block argmax. The last
// block of a node (device-scope counter) combines the F per-feature candidates with the
// reference tie-break (max lossChg, then lower feature, then lower bin).
struct ScanT {
  long long g, h;
  int last;
};
struct ScanOp {
  __device__ __forceinline__ ScanT operator()(const ScanT& a, const ScanT& b) const {
    return ScanT{a.g + b.g, a.h + b.h, max(a.last, b.last)};
  }
};
constexpr int kFeatThreads = 256;
using FeatScan = rocprim::block_scan<ScanT, kFeatThreads>;

__global__ __launch_bounds__(kFeatThreads) void split_feat_kernel(
    long long* __restrict__ hist, int B, int F, const int* __restrict__ nbins_f,
    const uint8_t* __restrict__ fmask, int f0, const int4* __restrict__ items,
    SplitOut* __restrict__ out, GainParams gp, const int* __restrict__ nitems_dev,
    const double* __restrict__ inv_dev, SplitOut* __restrict__ part, int* __restrict__ counters) {
  __shared__ typename FeatScan::storage_type s_scan;
  __shared__ long long s_tg[kFeatThreads / kWave], s_th[kFeatThreads / kWave];
  __shared__ float s_chg[kFeatThreads / kWave];
  __shared__ int s_bin[kFeatThreads / kWave], s_a[kFeatThreads / kWave];
  __shared__ double s_gl[kFeatThreads / kWave], s_hl[kFeatThreads / kWave];
  __shared__ int s_last;
  __shared__ SplitOut s_part[64];

  if (nitems_dev && (int)blockIdx.x >= *nitems_dev) return;
  if (inv_dev) {
    gp.inv_sg = inv_dev[0];
    gp.inv_sh = inv_dev[1];
  }
  const int f = (int)blockIdx.y;
  const int t = threadIdx.x, wid = t >> 6, l = lane_id();
  const int4 it = items[blockIdx.x];
  const size_t slot_sz = (size_t)B * F * 2;
  longlong2* hn = reinterpret_cast<longlong2*>(hist + (size_t)it.x * slot_sz);
  const longlong2* hp = reinterpret_cast<const longlong2*>(hist + (size_t)it.y * slot_sz);
  const longlong2* hs = reinterpret_cast<const longlong2*>(hist + (size_t)it.z * slot_sz);
  const bool derived = it.w != 0;
  auto load = [&](int ff, int bin) -> longlong2 {
    const size_t idx = (size_t)bin * F + ff;
    if (derived) {
      const longlong2 p = hp[idx], s = hs[idx];
      return make_longlong2(p.x - s.x, p.y - s.y);
    }
    return hn[idx];
  };
  const int nb = nbins_f[f], nb0 = nbins_f[f0];
  const bool on = fmask[f] != 0;
  // ---- one load round trip
  longlong2 v = make_longlong2(0, 0), v0 = make_longlong2(0, 0);
  if (t < B && (derived || (on && t < nb))) v = load(f, t);
  if (f != f0 && t < nb0) v0 = load(f0, t);
  if (derived && t < B) hn[(size_t)t * F + f] = v;  // materialise the derived histogram
  if (f == f0) v0 = (t < nb0) ? v : make_longlong2(0, 0);
  // ---- node totals (exact int64, first sampled feature: DataParallelTreeMaker:543-573)
  {
    const long long sg = wave_sum_ll(v0.x), sh = wave_sum_ll(v0.y);
    if (l == 0) { s_tg[wid] = sg; s_th[wid] = sh; }
  }
  __syncthreads();
  long long Gq = 0, Hq = 0;
#pragma unroll
  for (int w = 0; w < kFeatThreads / kWave; ++w) { Gq += s_tg[w]; Hq += s_th[w]; }
  const double G = (double)Gq * gp.inv_sg, H = (double)Hq * gp.inv_sh;

  float best_chg = -INFINITY;
  int best_b = 0x7fffffff, best_a = -1;
  double best_gl = 0.0, best_hl = 0.0;
  if (on) {  // block-uniform
    if (t >= nb) v = make_longlong2(0, 0);
    const bool ne = (v.x != 0 || v.y != 0);
    ScanT ex;
    FeatScan().exclusive_scan(ScanT{v.x, v.y, ne ? t : -1}, ex, ScanT{0, 0, -1}, s_scan, ScanOp());
    if (ne && ex.last >= 0 && ex.h != 0) {
      const double dgl = (double)ex.g * gp.inv_sg, dhl = (double)ex.h * gp.inv_sh;
      const double dgr = (double)(Gq - ex.g) * gp.inv_sg, dhr = (double)(Hq - ex.h) * gp.inv_sh;
      if (dhl >= (double)gp.mcw && dhr >= (double)gp.mcw) {
        const float root_gain = (float)calc_gain(G, H, gp);
        best_chg = (float)(calc_gain(dgl, dhl, gp) + calc_gain(dgr, dhr, gp) - (double)root_gain);
        best_b = t;
        best_a = ex.last;
        best_gl = dgl;
        best_hl = dhl;
      }
    }
  }
  // ---- block argmax (chg desc, bin asc)
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) {
    const float oc = __shfl_xor(best_chg, off, kWave);
    const int ob = __shfl_xor(best_b, off, kWave);
    const int oa = __shfl_xor(best_a, off, kWave);
    const double ogl = __shfl_xor(best_gl, off, kWave);
    const double ohl = __shfl_xor(best_hl, off, kWave);
    if (better(oc, 0, ob, best_chg, 0, best_b)) {
      best_chg = oc; best_b = ob; best_a = oa; best_gl = ogl; best_hl = ohl;
    }
  }
  if (l == 0) {
    s_chg[wid] = best_chg; s_bin[wid] = best_b; s_a[wid] = best_a; s_gl[wid] = best_gl; s_hl[wid] = best_hl;
  }
  __syncthreads();
  if (t == 0) {
    int bw = 0;
    for (int w = 1; w < kFeatThreads / kWave; ++w)
      if (better(s_chg[w], 0, s_bin[w], s_chg[bw], 0, s_bin[bw])) bw = w;
    SplitOut o;
    o.loss_chg = s_chg[bw];
    o.feat = (s_bin[bw] == 0x7fffffff) ? 0x7fffffff : f;
    o.bin_a = s_a[bw];
    o.bin_b = s_bin[bw];
    o.gl = s_gl[bw];
    o.hl = s_hl[bw];
    o.g = G;
    o.h = H;
    part[(size_t)blockIdx.x * F + f] = o;
    __threadfence();
    const int prev = atomicAdd(&counters[blockIdx.x], 1);
    s_last = (prev == F - 1);
  }
  __syncthreads();
  if (!s_last) return;
  // ---- last block of the node: combine the F feature candidates (64 per pass)
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  SplitOut best;
  best.loss_chg = -INFINITY;
  best.feat = 0x7fffffff;
  best.bin_a = -1;
  best.bin_b = 0x7fffffff;
  best.gl = best.hl = 0.0;
  for (int c0 = 0; c0 < F; c0 += 64) {
    const int n = min(64, F - c0);
    if (t < n) {
      const volatile SplitOut* pp = part + (size_t)blockIdx.x * F + c0 + t;
      SplitOut q;
      q.loss_chg = pp->loss_chg; q.feat = pp->feat; q.bin_a = pp->bin_a; q.bin_b = pp->bin_b;
      q.gl = pp->gl; q.hl = pp->hl; q.g = pp->g; q.h = pp->h;
      s_part[t] = q;
    }
    __syncthreads();
    if (t == 0)
      for (int y = 0; y < n; ++y)
        if (better(s_part[y].loss_chg, s_part[y].feat, s_part[y].bin_b, best.loss_chg, best.feat, best.bin_b))
          best = s_part[y];
    __syncthreads();
  }
  if (t == 0) {
    counters[blockIdx.x] = 0;
    best.g = G;
    best.h = H;
    if (best.feat == 0x7fffffff) best.feat = -1;
    if (best.bin_b == 0x7fffffff) best.bin_b = -1;
    out[blockIdx.x] = best;
  }
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

__global__ __launch_bounds__(kNodeThreads) void split_node_kernel(
    long long* __restrict__ hist, int B, int F, int Bp, const int* __restrict__ nbins_f,
    const uint8_t* __restrict__ fmask, int f0, const int4* __restrict__ items,
    SplitOut* __restrict__ out, GainParams gp, const int* __restrict__ nitems_dev,
    const double* __restrict__ inv_dev) {
  extern __shared__ __attribute__((aligned(16))) longlong2 sh_hist[];  // [F][Bp]
  constexpr int kW = kNodeThreads / kWave;
  __shared__ float s_chg[kW];
  __shared__ int s_feat[kW], s_a[kW], s_b[kW];
  __shared__ double s_gl[kW], s_hl[kW];
  __shared__ int s_nb[kNodeMaxF];
  __shared__ uint8_t s_fm[kNodeMaxF];

  // the dependent global round trips are a large part of this kernel: issue every
  // independent load together (items / counts / scales, then the histogram + per-feature
  // metadata) instead of one chain per use
  const int t = threadIdx.x, wid = t >> 6, l = lane_id();
  const int4 it = items[blockIdx.x];  // items is sized for the whole grid
  if (inv_dev) {
    gp.inv_sg = inv_dev[0];
    gp.inv_sh = inv_dev[1];
  }
  if (nitems_dev && (int)blockIdx.x >= *nitems_dev) return;
  int nb_t = 0;
  uint8_t fm_t = 0;
  if (t < F) { nb_t = nbins_f[t]; fm_t = fmask[t]; }
  const size_t slot_sz = (size_t)B * F * 2;
  longlong2* hn = reinterpret_cast<longlong2*>(hist + (size_t)it.x * slot_sz);
  const longlong2* hp = reinterpret_cast<const longlong2*>(hist + (size_t)it.y * slot_sz);
  const longlong2* hs = reinterpret_cast<const longlong2*>(hist + (size_t)it.z * slot_sz);
  const bool derived = it.w != 0;
  // ---- stream the node's histogram into LDS (all loads of a thread in flight at once)
  const int total = B * F;
  longlong2 v[kNodeLoads];
  if (derived) {
    longlong2 s[kNodeLoads];
#pragma unroll
    for (int j = 0; j < kNodeLoads; ++j) {
      const int i = t + j * kNodeThreads;
      if (i < total) { v[j] = hp[i]; s[j] = hs[i]; }
    }
#pragma unroll
    for (int j = 0; j < kNodeLoads; ++j) {
      const int i = t + j * kNodeThreads;
      if (i < total) {
        v[j] = make_longlong2(v[j].x - s[j].x, v[j].y - s[j].y);
        hn[i] = v[j];
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < kNodeLoads; ++j) {
      const int i = t + j * kNodeThreads;
      if (i < total) v[j] = hn[i];
    }
  }
#pragma unroll
  for (int j = 0; j < kNodeLoads; ++j) {
    const int i = t + j * kNodeThreads;
    if (i < total) {
      const int bin = i / F, f = i - bin * F;
      sh_hist[f * Bp + bin] = v[j];
    }
  }
  if (t < F) { s_nb[t] = nb_t; s_fm[t] = fm_t; }
  __syncthreads();
  // ---- node totals (exact int64, first sampled feature: DataParallelTreeMaker:543-573);
  // every wave computes them itself (no extra barrier)
  long long Gq, Hq;
  {
    const int nb0 = s_nb[f0];
    long long sg = 0, sh = 0;
    for (int bin = l; bin < nb0; bin += kWave) {
      const longlong2 q = sh_hist[f0 * Bp + bin];
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
  for (int f = wid; f < F; f += kW) {
    if (!s_fm[f]) continue;  // wave-uniform
    const int nb = s_nb[f];
    longlong2 q[4];
    long long sg = 0, sh = 0;
    int lastne = -1;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int bin = 4 * l + k;
      q[k] = (bin < nb) ? sh_hist[f * Bp + bin] : make_longlong2(0, 0);
      sg += q[k].x;
      sh += q[k].y;
      if (q[k].x != 0 || q[k].y != 0) lastne = bin;
    }
    const long long ig = dpp_scan_add(sg), ih = dpp_scan_add(sh);
    const int im = dpp_scan_max(lastne);
    int prev = __shfl_up(im, 1, kWave);  // exclusive: last non-empty bin of the lanes below
    if (l == 0) prev = -1;
    long long pg = ig - sg, ph = ih - sh;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int bin = 4 * l + k;
      if (q[k].x != 0 || q[k].y != 0) {
        if (prev >= 0 && ph != 0) {
          const double dgl = (double)pg * gp.inv_sg, dhl = (double)ph * gp.inv_sh;
          const double dgr = (double)(Gq - pg) * gp.inv_sg, dhr = (double)(Hq - ph) * gp.inv_sh;
          if (dhl >= (double)gp.mcw && dhr >= (double)gp.mcw) {
            const float chg =
                (float)(calc_gain(dgl, dhl, gp) + calc_gain(dgr, dhr, gp) - (double)root_gain);
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
    out[blockIdx.x] = o;
  }
}

}  // namespace ytk

using namespace ytk;

// "0" in the environment variable disables an optional kernel path (read once per process)
static bool getenv_flag_off(const char* name) {
  const char* v = getenv(name);
  return v && v[0] == '0' && v[1] == 0;
}

// part / counters (optional): scratch of nitems * F SplitOut and nitems zeroed ints. With
// them and B <= 256 the (node, feature)-parallel kernel runs; otherwise the wave-per-
// feature kernel (features spread over ceil(F/32) blocks when the scratch is given).
extern "C" void ytk_split_find(uintptr_t hist, int B, int F, uintptr_t nbins_f, uintptr_t fmask,
                               int f0, uintptr_t items, int nitems, uintptr_t out, float mcw,
                               float l1, float l2, float max_abs_leaf, double inv_sg,
                               double inv_sh, uintptr_t nitems_dev, uintptr_t inv_dev,
                               uintptr_t part, uintptr_t counters, uintptr_t stream) {
  if (nitems <= 0) return;
  GainParams gp{mcw, l1, l2, max_abs_leaf, inv_sg, inv_sh};
  // node-resident kernel: the transposed, padded histogram fits in LDS
  const int Bp = B + 1;
  const size_t node_lds = (size_t)F * Bp * sizeof(long long) * 2;
  if (node_lds <= kNodeLdsMax && B <= 4 * kWave && B * F <= kNodeLoads * kNodeThreads &&
      F <= kNodeMaxF && F < 0xffff && !getenv_flag_off("YTK_SPLIT_NODE")) {
    hipLaunchKernelGGL(split_node_kernel, dim3(nitems), dim3(kNodeThreads), node_lds,
                       reinterpret_cast<hipStream_t>(stream), (long long*)hist, B, F, Bp,
                       (const int*)nbins_f, (const uint8_t*)fmask, f0, (const int4*)items,
                       (SplitOut*)out, gp, (const int*)nitems_dev, (const double*)inv_dev);
    YTK_LAUNCH_CHECK();
    return;
  }
  if (B <= kFeatThreads && part && counters) {
    // part: >= nitems * F SplitOut; counters: nitems zeroed ints
    hipLaunchKernelGGL(split_feat_kernel, dim3(nitems, F), dim3(kFeatThreads), 0,
                       reinterpret_cast<hipStream_t>(stream), (long long*)hist, B, F,
                       (const int*)nbins_f, (const uint8_t*)fmask, f0, (const int4*)items,
                       (SplitOut*)out, gp, (const int*)nitems_dev, (const double*)inv_dev,
                       (SplitOut*)part, (int*)counters);
    YTK_LAUNCH_CHECK();
    return;
  }
  // F <= 32: one block per node; otherwise ceil(F / 32) blocks combined via part/counters
  const int need = (F + kSplitWaves * kFPW - 1) / (kSplitWaves * kFPW);
  if (need > 1 && !(part && counters))
    throw std::invalid_argument("split_find: F > 32 needs the part/counters scratch");
  const int groups = need;
  hipLaunchKernelGGL(split_find_kernel, dim3(nitems, groups), dim3(kSplitWaves * 64), 0,
                     reinterpret_cast<hipStream_t>(stream), (long long*)hist, B, F,
                     (const int*)nbins_f, (const uint8_t*)fmask, f0, (const int4*)items,
                     (SplitOut*)out, gp, (const int*)nitems_dev, (const double*)inv_dev,
                     (SplitOut*)part, (int*)counters);
  YTK_LAUNCH_CHECK();
}
