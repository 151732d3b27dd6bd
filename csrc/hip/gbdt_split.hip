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
#include "gbdt_split_node.h"

#include <rocprim/block/block_scan.hpp>

namespace ytk {

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
constexpr int kSplitFeatMaxBlocks = 2048;  // grid cap of split_feat_kernel (a multiple of 32)

// kR bins per thread: thread t owns the contiguous bins [t * kR, t * kR + kR) so one
// block of kT threads covers B <= kT * kR (kR > 1: the wide-bin configs; kT = 1024 above
// 1024 bins, so a thread's sequential run stays <= 8 bins). The exclusive block scan
// of the per-thread run totals gives each run its left prefix; the run is then walked
// bin by bin exactly like the wave kernel (same gain, same tie-break).
template <int kR, int kT>
__global__ __launch_bounds__(kT) void split_feat_kernel(
    long long* __restrict__ hist, int B, int F, const int* __restrict__ nbins_f,
    const uint8_t* __restrict__ fmask, int f0, const int4* __restrict__ items,
    SplitOut* __restrict__ out, GainParams gp, const int* __restrict__ nitems_dev,
    const double* __restrict__ inv_dev, SplitOut* __restrict__ part, int* __restrict__ counters, int nitems_max) {
  using Scan = rocprim::block_scan<ScanT, kT>;
  __shared__ typename Scan::storage_type s_scan;
  __shared__ long long s_tg[kT / kWave], s_th[kT / kWave];
  __shared__ float s_chg[kT / kWave];
  __shared__ int s_bin[kT / kWave], s_a[kT / kWave];
  __shared__ double s_gl[kT / kWave], s_hl[kT / kWave];
  __shared__ int s_last;
  __shared__ SplitOut s_part[64];

  // XCD-aware block order: the grid is 1-D; a "unit" is 4 neighbouring features of one
  // node, which share every 64-B line of the [bin][F] histogram (4 x 16 B). Units are dealt
  // round-robin over the XCDs (blocks L with L % 8 == x run on XCD x) and a unit's 4 blocks
  // run back to back on its XCD, so each line is fetched into one L2 once instead of once
  // per feature; consecutive units still spread a level's (possibly few, nitems_dev) nodes
  // over every XCD.
  //
  // Grid-stride over that block order: a device-counted launch (leaf-wise engine) is sized
  // for its item BOUND (2 x max leaves), and thousands of empty 1024-thread blocks with a
  // 80-KB LDS footprint cost more than the real ones (measured 213 us per 5000-bin call).
  // The grid is capped (a multiple of 32) and each block walks L, L + gridDim.x, ...; the
  // unit index grows with L, so the first item past the count ends the walk.
  const int nq = (F + 3) >> 2;
  const int nitems_live = nitems_dev ? min(*nitems_dev, nitems_max) : nitems_max;
  if (inv_dev) {
    gp.inv_sg = inv_dev[0];
    gp.inv_sh = inv_dev[1];
  }
  const int t = threadIdx.x, wid = t >> 6, l = lane_id();
  for (unsigned Lb = blockIdx.x;; Lb += gridDim.x) {
  const unsigned sb = Lb >> 3;
  const int unit = (int)((sb >> 2) * 8u + (Lb & 7u));
  const int item = unit / nq;
  const int f = (unit - item * nq) * 4 + (int)(sb & 3u);
  if (item >= nitems_live) break;
  if (f >= F) continue;
  __syncthreads();  // the previous unit's LDS (bins, scan, partials) is no longer read
  const int4 it = items[item];
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
  const int b0 = t * kR;
  // kR == 1: one load round trip (this feature's bin + the node-total feature's bin).
  // kR > 1 (wide bins): the bins are loaded bin = t + 256 j -- neighbouring lanes on
  // neighbouring bins -- into LDS and each thread then walks its contiguous run from LDS
  // (loading the runs directly put the 64 lanes of a load 32 bins x F x 16 B apart, a
  // stride that lands on a couple of memory channels, and held 2 x kR 16-B values in
  // registers: 256 VGPRs, one wave per SIMD)
  extern __shared__ longlong2 s_bins[];
  longlong2 v1 = make_longlong2(0, 0);
  long long tg = 0, th = 0;
  if constexpr (kR == 1) {
    longlong2 v0 = make_longlong2(0, 0);
    if (b0 < B && (derived || (on && b0 < nb))) v1 = load(f, b0);
    if (f != f0 && b0 < nb0) v0 = load(f0, b0);
    if (derived && b0 < B) hn[(size_t)b0 * F + f] = v1;  // materialise the derived histogram
    if (f == f0) v0 = (b0 < nb0) ? v1 : make_longlong2(0, 0);
    tg = v0.x;
    th = v0.y;
  } else {
#pragma unroll 4
    for (int bin = t; bin < B; bin += kT) {
      longlong2 x = make_longlong2(0, 0), x0 = make_longlong2(0, 0);
      if (derived || (on && bin < nb)) x = load(f, bin);
      if (f != f0 && bin < nb0) x0 = load(f0, bin);
      if (derived) hn[(size_t)bin * F + f] = x;
      if (f == f0) x0 = (bin < nb0) ? x : make_longlong2(0, 0);
      s_bins[bin] = x;
      tg += x0.x;
      th += x0.y;
    }
  }
  auto val = [&](int k) -> longlong2 {  // this thread's k-th bin (zero past nb)
    const int bin = b0 + k;
    if (bin >= nb || bin >= B) return make_longlong2(0, 0);
    if constexpr (kR == 1) return v1;
    else return s_bins[bin];
  };
  // ---- node totals (exact int64, first sampled feature: DataParallelTreeMaker:543-573)
  {
    const long long sg = wave_sum_ll(tg);
    const long long sh = wave_sum_ll(th);
    if (l == 0) { s_tg[wid] = sg; s_th[wid] = sh; }
  }
  __syncthreads();  // (also publishes s_bins)
  long long Gq = 0, Hq = 0;
#pragma unroll
  for (int w = 0; w < kT / kWave; ++w) { Gq += s_tg[w]; Hq += s_th[w]; }
  const double G = (double)Gq * gp.inv_sg, H = (double)Hq * gp.inv_sh;

  float best_chg = -INFINITY;
  int best_b = 0x7fffffff, best_a = -1;
  double best_gl = 0.0, best_hl = 0.0;
  if (on) {  // block-uniform
    long long rg = 0, rh = 0;
    int rlast = -1;
    for (int k = 0; k < kR; ++k) {
      const longlong2 x = val(k);
      rg += x.x;
      rh += x.y;
      if (x.x != 0 || x.y != 0) rlast = b0 + k;
    }
    ScanT ex;
    Scan().exclusive_scan(ScanT{rg, rh, rlast}, ex, ScanT{0, 0, -1}, s_scan, ScanOp());
    const float root_gain = (float)calc_gain(G, H, gp);
    long long pg = ex.g, ph = ex.h;
    int prev = ex.last;
    for (int k = 0; k < kR; ++k) {
      const longlong2 x = val(k);
      const bool ne = (x.x != 0 || x.y != 0);
      if (!ne) continue;
      if (prev >= 0 && ph != 0) {
        const double dgl = (double)pg * gp.inv_sg, dhl = (double)ph * gp.inv_sh;
        const double dgr = (double)(Gq - pg) * gp.inv_sg, dhr = (double)(Hq - ph) * gp.inv_sh;
        if (dhl >= (double)gp.mcw && dhr >= (double)gp.mcw) {
          const float chg = (float)(calc_gain(dgl, dhl, gp) + calc_gain(dgr, dhr, gp) - (double)root_gain);
          if (better(chg, 0, b0 + k, best_chg, 0, best_b)) {
            best_chg = chg;
            best_b = b0 + k;
            best_a = prev;
            best_gl = dgl;
            best_hl = dhl;
          }
        }
      }
      pg += x.x;
      ph += x.y;
      prev = b0 + k;
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
    for (int w = 1; w < kT / kWave; ++w)
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
    part[(size_t)item * F + f] = o;
    __threadfence();
    const int prev = atomicAdd(&counters[item], 1);
    s_last = (prev == F - 1);
  }
  __syncthreads();
  if (!s_last) continue;
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
      const volatile SplitOut* pp = part + (size_t)item * F + c0 + t;
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
    counters[item] = 0;
    best.g = G;
    best.h = H;
    if (best.feat == 0x7fffffff) best.feat = -1;
    if (best.bin_b == 0x7fffffff) best.bin_b = -1;
    out[item] = best;
  }
  }  // grid-stride unit loop
}

// ---------------------------------------------------------------------------------
// Wide-bin split search (256 < B <= 256 * kR): one 256 kFG-thread block per (node, group of
// kFG neighbouring features), the group's histogram held in registers.
//
// Why: the [slot][bin][F] layout puts one feature's consecutive bins F x 16 B apart, so
// split_feat_kernel's per-feature blocks fetched a separate line per 16-B (g, h) pair --
// at 5000 bins 3 x 80 KB of scattered lines per (derived node, feature), ~290 us per
// leaf-wise batch. Here thread t owns feature t % kFG of the contiguous bin run
// [(t / kFG) kR, (t / kFG) kR + kR): at every load instruction the kFG lanes of a bin read
// its kFG x 16 contiguous bytes, all kR loads of a thread are in flight together,
// and the derived (parent - sibling) histogram is written back the same way. The run
// totals go through ONE block scan per feature (stride-kFG lane scan -- features interleave
// with the lanes -- then wave 0 scans the wave totals), and each thread walks its run
// from registers exactly like split_feat_kernel (same gain, same empty-bin rule, same
// tie-break). Node totals: the group's copy of f0, else its first sampled feature (every
// row adds to exactly one bin of every feature, so the exact int64 totals agree); the
// item's last group block combines the groups' records and takes the totals from f0's group.
constexpr int kWideSplitMaxBlocks = 2048;  // grid cap (a multiple of 8; grid-stride inside)

// Derived (parent - sibling) histograms of a wide-bin item list, materialised by one
// streaming pass before split_wide_kernel: every block subtracts a contiguous 2048-pair
// slice of one derived item with all its loads in flight (inside split_wide_kernel the
// subtraction ran 4 bins per step per thread -- its register budget holds the whole run
// of a feature pair -- and dominated the leaf-wise 5000-bin split search). Blocks past the
// device item count, or on built items, exit.
constexpr int kDeriveThreads = 256;
constexpr int kDerivePer = 8;  // 16-B pairs per thread
constexpr int kDeriveMaxBlocks = 4096;  // grid cap: the work units are walked grid-stride
__global__ __launch_bounds__(kDeriveThreads) void derive_wide_kernel(
    long long* __restrict__ hist, long long pairs, const int4* __restrict__ items,
    const int* __restrict__ nitems_dev, int nitems_max, int blocks_per_item) {
  const int live = nitems_dev ? min(*nitems_dev, nitems_max) : nitems_max;
  const long long units = (long long)live * blocks_per_item;
  for (long long w = blockIdx.x; w < units; w += gridDim.x) {  // uniform per block
    const int item = (int)(w / blocks_per_item);
    const int4 it = items[item];
    if (it.w == 0) continue;
    const long long p0 = (w % blocks_per_item) * kDeriveThreads * kDerivePer;
    longlong2* hn = reinterpret_cast<longlong2*>(hist) + (size_t)it.x * pairs;
    const longlong2* hp = reinterpret_cast<const longlong2*>(hist) + (size_t)it.y * pairs;
    const longlong2* hs = reinterpret_cast<const longlong2*>(hist) + (size_t)it.z * pairs;
    longlong2 a[kDerivePer], c[kDerivePer];
#pragma unroll
    for (int u = 0; u < kDerivePer; ++u) {
      const long long i = p0 + (long long)u * kDeriveThreads + threadIdx.x;
      if (i < pairs) { a[u] = hp[i]; c[u] = hs[i]; }
    }
#pragma unroll
    for (int u = 0; u < kDerivePer; ++u) {
      const long long i = p0 + (long long)u * kDeriveThreads + threadIdx.x;
      if (i < pairs) hn[i] = make_longlong2(a[u].x - c[u].x, a[u].y - c[u].y);
    }
  }
}

// pre_derived: derive_wide_kernel has materialised every derived item's histogram, so all
// items are read like built ones
template <int kR, int kFG, bool kPreDerived>
__global__ __launch_bounds__(256 * kFG) void split_wide_kernel(
    long long* __restrict__ hist, int B, int F, const int* __restrict__ nbins_f,
    const uint8_t* __restrict__ fmask, int f0, const int4* __restrict__ items,
    SplitOut* __restrict__ out, GainParams gp, const int* __restrict__ nitems_dev,
    const double* __restrict__ inv_dev, SplitOut* __restrict__ part, int* __restrict__ counters, int nitems_max) {
  constexpr int kT = 256 * kFG;  // 256 bin runs per feature
  constexpr int kW = kT / kWave;
  static_assert(kW * kFG <= kWave, "wave 0 scans the (wave, feature) totals");
  __shared__ long long s_wg[kW][kFG], s_wh[kW][kFG];  // wave totals per feature -> exclusive prefixes
  __shared__ int s_wl[kW][kFG];
  __shared__ long long s_tg[kW], s_th[kW];
  __shared__ float s_chg[kW];
  __shared__ int s_f[kW], s_b[kW], s_a[kW];
  __shared__ double s_gl[kW], s_hl[kW];
  __shared__ int s_last;
  __shared__ SplitOut s_part[64];
  const int ng = (F + kFG - 1) / kFG;
  const int nitems_live = nitems_dev ? min(*nitems_dev, nitems_max) : nitems_max;
  if (inv_dev) {
    gp.inv_sg = inv_dev[0];
    gp.inv_sh = inv_dev[1];
  }
  const int t = threadIdx.x, wid = t >> 6, l = lane_id();
  const int fi = t % kFG, b0 = (t / kFG) * kR;
  // XCD-local (item, group): blocks L = 8 s + x run on XCD x; s enumerates (item / 8, group),
  // so all groups of item 8 (s / ng) + x share that XCD's L2 (neighbouring groups share
  // 128-B lines of each bin row)
  for (unsigned L = blockIdx.x;; L += gridDim.x) {
    const unsigned sb = L >> 3;
    const int grp = (int)(sb % (unsigned)ng);
    const int item = (int)((sb / (unsigned)ng) * 8u + (L & 7u));
    if (item >= nitems_live) break;  // item grows with L
    __syncthreads();  // the previous item's LDS records are no longer read
    const int4 it = items[item];
    const size_t slot_sz = (size_t)B * F * 2;
    longlong2* hn = reinterpret_cast<longlong2*>(hist + (size_t)it.x * slot_sz);
    const longlong2* hp = reinterpret_cast<const longlong2*>(hist + (size_t)it.y * slot_sz);
    const longlong2* hs = reinterpret_cast<const longlong2*>(hist + (size_t)it.z * slot_sz);
    const bool derived = !kPreDerived && it.w != 0;
    const int f_lo = grp * kFG, f = f_lo + fi;
    const bool fin = f < F;
    const int nb = fin ? nbins_f[f] : 0;
    const bool on = fin && fmask[f] != 0;
    int tf = -1;  // totals feature of the group (block-uniform)
    if (f0 >= f_lo && f0 < min(F, f_lo + kFG)) {
      tf = f0;
    } else {
      for (int q = f_lo; q < min(F, f_lo + kFG); ++q)
        if (fmask[q]) { tf = q; break; }
    }
    const bool want = on || f == tf;
    longlong2 v[kR];
    if (derived) {  // 4 bins per step: 8 loads in flight, not 2 kR (register budget); dead when kPreDerived
#pragma unroll
      for (int k0 = 0; k0 < kR; k0 += 4) {
        longlong2 a[4], c[4];
#pragma unroll
        for (int j = 0; j < 4 && k0 + j < kR; ++j) {
          const int bin = b0 + k0 + j;
          a[j] = c[j] = make_longlong2(0, 0);
          if (fin && bin < B) { a[j] = hp[(size_t)bin * F + f]; c[j] = hs[(size_t)bin * F + f]; }
        }
#pragma unroll
        for (int j = 0; j < 4 && k0 + j < kR; ++j) {
          const int bin = b0 + k0 + j;
          const longlong2 x = make_longlong2(a[j].x - c[j].x, a[j].y - c[j].y);
          if (fin && bin < B) hn[(size_t)bin * F + f] = x;  // materialise the derived histogram
          v[k0 + j] = bin < nb ? x : make_longlong2(0, 0);
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < kR; ++k) {
        const int bin = b0 + k;
        v[k] = (want && bin < nb) ? hn[(size_t)bin * F + f] : make_longlong2(0, 0);
      }
    }
    // ---- run totals, node totals (exact int64)
    long long rg = 0, rh = 0;
    int rl = -1;
#pragma unroll
    for (int k = 0; k < kR; ++k) {
      rg += v[k].x;
      rh += v[k].y;
      if ((v[k].x | v[k].y) != 0) rl = b0 + k;
    }
    {
      const long long tg = wave_sum_ll(f == tf ? rg : 0), th = wave_sum_ll(f == tf ? rh : 0);
      if (l == 0) { s_tg[wid] = tg; s_th[wid] = th; }
    }
    // ---- exclusive scan of the run totals per feature: lanes kFG j + fi
    long long ig = rg, ih = rh;
    int il = rl;
#pragma unroll
    for (int off = kFG; off < kWave; off <<= 1) {
      const long long og = __shfl_up(ig, off, kWave), oh = __shfl_up(ih, off, kWave);
      const int ol = __shfl_up(il, off, kWave);
      if (l >= off) { ig += og; ih += oh; il = max(il, ol); }
    }
    int el = __shfl_up(il, kFG, kWave);
    if (l < kFG) el = -1;
    if (l >= kWave - kFG) { s_wg[wid][fi] = ig; s_wh[wid][fi] = ih; s_wl[wid][fi] = il; }
    __syncthreads();
    if (t < kW * kFG) {  // wave 0: exclusive prefix of the wave totals per feature (lane = kFG w + fi)
      const long long a0 = (&s_wg[0][0])[t], c0 = (&s_wh[0][0])[t];
      long long a = a0, c = c0;
      int m = (&s_wl[0][0])[t];
#pragma unroll
      for (int off = kFG; off < kW * kFG; off <<= 1) {
        const long long oa = __shfl_up(a, off, kWave), oc = __shfl_up(c, off, kWave);
        const int om = __shfl_up(m, off, kWave);
        if (t >= off) { a += oa; c += oc; m = max(m, om); }
      }
      int em = __shfl_up(m, kFG, kWave);
      if (t < kFG) em = -1;
      (&s_wg[0][0])[t] = a - a0;
      (&s_wh[0][0])[t] = c - c0;
      (&s_wl[0][0])[t] = em;
    }
    __syncthreads();
    long long Gq = 0, Hq = 0;
#pragma unroll
    for (int w = 0; w < kW; ++w) { Gq += s_tg[w]; Hq += s_th[w]; }
    const double G = (double)Gq * gp.inv_sg, H = (double)Hq * gp.inv_sh;
    long long pg = s_wg[wid][fi] + ig - rg, ph = s_wh[wid][fi] + ih - rh;  // left of this run
    int prev = max(s_wl[wid][fi], el);
    float best_chg = -INFINITY;
    int best_b = 0x7fffffff, best_a = -1;
    double best_gl = 0.0, best_hl = 0.0;
    if (on) {
      const float root_gain = (float)calc_gain(G, H, gp);
#pragma unroll
      for (int k = 0; k < kR; ++k) {
        const longlong2 x = v[k];
        if ((x.x | x.y) == 0) continue;
        if (prev >= 0 && ph != 0) {
          const double dgl = (double)pg * gp.inv_sg, dhl = (double)ph * gp.inv_sh;
          const double dgr = (double)(Gq - pg) * gp.inv_sg, dhr = (double)(Hq - ph) * gp.inv_sh;
          if (dhl >= (double)gp.mcw && dhr >= (double)gp.mcw) {
            const float chg = (float)(calc_gain(dgl, dhl, gp) + calc_gain(dgr, dhr, gp) - (double)root_gain);
            if (better(chg, 0, b0 + k, best_chg, 0, best_b)) {
              best_chg = chg; best_b = b0 + k; best_a = prev; best_gl = dgl; best_hl = dhl;
            }
          }
        }
        pg += x.x;
        ph += x.y;
        prev = b0 + k;
      }
    }
    // ---- block argmax over (chg desc, feature asc, bin asc)
    int best_f = best_b == 0x7fffffff ? 0x7fffffff : f;
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) {
      const float oc = __shfl_xor(best_chg, off, kWave);
      const int of = __shfl_xor(best_f, off, kWave), ob = __shfl_xor(best_b, off, kWave);
      const int oa = __shfl_xor(best_a, off, kWave);
      const double ogl = __shfl_xor(best_gl, off, kWave), ohl = __shfl_xor(best_hl, off, kWave);
      if (better(oc, of, ob, best_chg, best_f, best_b)) {
        best_chg = oc; best_f = of; best_b = ob; best_a = oa; best_gl = ogl; best_hl = ohl;
      }
    }
    if (l == 0) {
      s_chg[wid] = best_chg; s_f[wid] = best_f; s_b[wid] = best_b; s_a[wid] = best_a;
      s_gl[wid] = best_gl; s_hl[wid] = best_hl;
    }
    __syncthreads();
    if (t == 0) {
      int bw = 0;
      for (int w = 1; w < kW; ++w)
        if (better(s_chg[w], s_f[w], s_b[w], s_chg[bw], s_f[bw], s_b[bw])) bw = w;
      SplitOut o;
      o.loss_chg = s_chg[bw]; o.feat = s_f[bw]; o.bin_a = s_a[bw]; o.bin_b = s_b[bw];
      o.gl = s_gl[bw]; o.hl = s_hl[bw]; o.g = G; o.h = H;
      part[(size_t)item * ng + grp] = o;
      __threadfence();
      const int pv = atomicAdd(&counters[item], 1);
      s_last = (pv == ng - 1);
    }
    __syncthreads();
    if (!s_last) continue;
    // ---- last group block of the item: combine the groups' records (64 per pass)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    SplitOut best;
    best.loss_chg = -INFINITY; best.feat = 0x7fffffff; best.bin_a = -1; best.bin_b = 0x7fffffff;
    best.gl = best.hl = best.g = best.h = 0.0;
    double tg = 0.0, th = 0.0;
    for (int c0 = 0; c0 < ng; c0 += 64) {
      const int n = min(64, ng - c0);
      if (t < n) {
        const volatile SplitOut* pp = part + (size_t)item * ng + c0 + t;
        SplitOut q;
        q.loss_chg = pp->loss_chg; q.feat = pp->feat; q.bin_a = pp->bin_a; q.bin_b = pp->bin_b;
        q.gl = pp->gl; q.hl = pp->hl; q.g = pp->g; q.h = pp->h;
        s_part[t] = q;
      }
      __syncthreads();
      if (t == 0) {
        for (int y = 0; y < n; ++y)
          if (better(s_part[y].loss_chg, s_part[y].feat, s_part[y].bin_b, best.loss_chg, best.feat, best.bin_b))
            best = s_part[y];
        const int g0 = f0 / kFG - c0;  // totals from f0's group
        if (g0 >= 0 && g0 < n) { tg = s_part[g0].g; th = s_part[g0].h; }
      }
      __syncthreads();
    }
    if (t == 0) {
      counters[item] = 0;
      best.g = tg;
      best.h = th;
      if (best.feat == 0x7fffffff) best.feat = -1;
      if (best.bin_b == 0x7fffffff) best.bin_b = -1;
      out[item] = best;
    }
  }
}

// the dependent global round trips are a large part of this kernel: every independent
// load is issued together (items / counts / scales, then the histogram + per-feature
// metadata) instead of one chain per use
__global__ __launch_bounds__(kNodeThreads) void split_node_kernel(
    long long* __restrict__ hist, int B, int F, int Bp, const int* __restrict__ nbins_f,
    const uint8_t* __restrict__ fmask, int f0, const int4* __restrict__ items,
    SplitOut* __restrict__ out, GainParams gp, const int* __restrict__ nitems_dev,
    const double* __restrict__ inv_dev) {
  extern __shared__ __attribute__((aligned(16))) longlong2 sh_hist[];  // [F][Bp]
  const int4 it = items[blockIdx.x];  // items is sized for the whole grid
  if (inv_dev) {
    gp.inv_sg = inv_dev[0];
    gp.inv_sh = inv_dev[1];
  }
  if (nitems_dev && (int)blockIdx.x >= *nitems_dev) return;
  // gridDim.y feature groups per node: block (x, y) searches features [y*FGs, (y+1)*FGs)
  // and writes record x * gridDim.y + y (the level planner keeps each node's best)
  const int G = (int)gridDim.y, FGs = (F + G - 1) / G;
  const int fbeg = (int)blockIdx.y * FGs, fend = min(F, fbeg + FGs);
  split_node_block(hist, B, F, Bp, nbins_f, fmask, f0, it, out + (size_t)blockIdx.x * G + blockIdx.y, gp, sh_hist,
                   fbeg, fend);
}

}  // namespace ytk

using namespace ytk;

// Owner-computes combine (multi-GPU, hist_sync = owner): every rank searched only the
// features it owns; ``all`` holds the P ranks' records ([P][cap]) after an allgather.
// The global best per item uses the kernels' own total order (better(): larger lossChg,
// then lower feature, then lower bin -- SplitInfo.needReplace), so the result is the
// record the all-reduce mode finds; node totals (g, h) come from rank ``tot_rank``, the
// first rank owning a sampled feature (exact int64 sums: equal for every feature).
__global__ __launch_bounds__(256) void split_combine_kernel(const SplitOut* __restrict__ all, int P, int cap,
                                                            const int* __restrict__ n_dev, int n_max,
                                                            int tot_rank, SplitOut* __restrict__ out) {
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int n = n_dev ? min(*n_dev, n_max) : n_max;
  if (i >= n) return;
  auto fkey = [](int f) { return f < 0 ? 0x7fffffff : f; };
  SplitOut best = all[i];
  for (int r = 1; r < P; ++r) {
    const SplitOut c = all[(size_t)r * cap + i];
    if (better(c.loss_chg, fkey(c.feat), fkey(c.bin_b), best.loss_chg, fkey(best.feat), fkey(best.bin_b))) best = c;
  }
  const SplitOut t = all[(size_t)tot_rank * cap + i];
  best.g = t.g;
  best.h = t.h;
  out[i] = best;
}

// "0" in the environment variable disables an optional kernel path (read once per process)
static bool getenv_flag_off(const char* name) {
  const char* v = getenv(name);
  return v && v[0] == '0' && v[1] == 0;
}

// part / counters (optional): scratch of nitems * F SplitOut and nitems zeroed ints. With
// them and B <= 256 the (node, feature)-parallel kernel runs; otherwise the wave-per-
// feature kernel (features spread over ceil(F/32) blocks when the scratch is given).
extern "C" void ytk_split_combine(uintptr_t all, int P, int cap, uintptr_t n_dev, int n_max, int tot_rank,
                                  uintptr_t out, uintptr_t stream) {
  if (n_max <= 0) return;
  hipLaunchKernelGGL(split_combine_kernel, dim3((n_max + 255) / 256), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), (const SplitOut*)all, P, cap, (const int*)n_dev,
                     n_max, tot_rank, (SplitOut*)out);
  YTK_LAUNCH_CHECK();
}

// Node-resident split search with `groups` feature groups per node (grid nitems x groups,
// records [item][group]); returns 0 (nothing launched) if the node-resident kernel does
// not apply (then use ytk_split_find with one record per item).
extern "C" int ytk_split_node_grouped(uintptr_t hist, int B, int F, uintptr_t nbins_f, uintptr_t fmask, int f0,
                                      uintptr_t items, int nitems, uintptr_t out, float mcw, float l1, float l2,
                                      float max_abs_leaf, uintptr_t nitems_dev, uintptr_t inv_dev, int groups,
                                      uintptr_t stream) {
  if (nitems <= 0) return 1;
  const int Bp = B + 1;
  const int FGs = (F + groups - 1) / std::max(1, groups);
  if (groups < 1 || groups > F || (groups - 1) * FGs >= F) return 0;  // every group non-empty
  const size_t node_lds = (size_t)FGs * Bp * sizeof(long long) * 2;
  if (!(node_lds <= kNodeLdsMax && B <= 4 * kWave && B * FGs <= kNodeLoads * kNodeThreads && F <= kNodeMaxF &&
        F < 0xffff))
    return 0;
  GainParams gp{mcw, l1, l2, max_abs_leaf, 1.0, 1.0};
  hipLaunchKernelGGL(split_node_kernel, dim3(nitems, groups), dim3(kNodeThreads), node_lds,
                     reinterpret_cast<hipStream_t>(stream), (long long*)hist, B, F, Bp, (const int*)nbins_f,
                     (const uint8_t*)fmask, f0, (const int4*)items, (SplitOut*)out, gp, (const int*)nitems_dev,
                     (const double*)inv_dev);
  YTK_LAUNCH_CHECK();
  return 1;
}

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
  if (B > kFeatThreads && B <= 20 * 256 && part && counters && F <= 256 && !getenv_flag_off("YTK_SPLIT_WIDE")) {
    // wide bins: the group's histogram in registers (split_wide_kernel); part: nitems x
    // ceil(F / kFG) records. 4 features per 1024-thread block up to 1024 bins, above that 2
    // per 512-thread block (kR 16-B pairs per thread + the walk within 256 VGPRs)
    // derived histograms first, in one streaming pass (YTK_WIDE_DERIVE=0: inside the split)
    static const bool pre = [] {
      const char* e = getenv("YTK_WIDE_DERIVE");
      return !(e && e[0] == '0');
    }();
    if (pre) {
      const long long pairs = (long long)B * F;
      const int bpi = (int)((pairs + kDeriveThreads * kDerivePer - 1) / (kDeriveThreads * kDerivePer));
      hipLaunchKernelGGL(derive_wide_kernel, dim3((unsigned)std::min<long long>((long long)bpi * nitems, kDeriveMaxBlocks)),
                         dim3(kDeriveThreads), 0,
                         reinterpret_cast<hipStream_t>(stream), (long long*)hist, pairs, (const int4*)items,
                         (const int*)nitems_dev, nitems, bpi);
    }
#define YTK_SPLIT_WIDE(R, FG)                                                                                  \
  do {                                                                                                         \
    const long long L = (long long)((F + FG - 1) / FG) * ((nitems + 7) / 8 * 8);                               \
    const unsigned nblk = (unsigned)std::min<long long>(L, kWideSplitMaxBlocks);                               \
    if (pre)                                                                                                   \
      hipLaunchKernelGGL((split_wide_kernel<R, FG, true>), dim3(nblk), dim3(256 * FG), 0,                      \
                         reinterpret_cast<hipStream_t>(stream), (long long*)hist, B, F, (const int*)nbins_f,   \
                         (const uint8_t*)fmask, f0, (const int4*)items, (SplitOut*)out, gp,                   \
                         (const int*)nitems_dev, (const double*)inv_dev, (SplitOut*)part, (int*)counters,      \
                         nitems);                                                                              \
    else                                                                                                       \
      hipLaunchKernelGGL((split_wide_kernel<R, FG, false>), dim3(nblk), dim3(256 * FG), 0,                     \
                         reinterpret_cast<hipStream_t>(stream), (long long*)hist, B, F, (const int*)nbins_f,   \
                         (const uint8_t*)fmask, f0, (const int4*)items, (SplitOut*)out, gp,                   \
                         (const int*)nitems_dev, (const double*)inv_dev, (SplitOut*)part, (int*)counters,      \
                         nitems);                                                                              \
  } while (0)
    // (4-feature groups in 1024-thread blocks -- 64 B of every bin row per load instead of
    // 32 B -- measured slower: leaf-wise 5000 bins 8.70 -> 10.45 ms/tree at the 128-VGPR cap)
    if (B <= 4 * 256) YTK_SPLIT_WIDE(4, 4);
    else if (B <= 8 * 256) YTK_SPLIT_WIDE(8, 2);
    else if (B <= 12 * 256) YTK_SPLIT_WIDE(12, 2);
    else if (B <= 16 * 256) YTK_SPLIT_WIDE(16, 2);
    else YTK_SPLIT_WIDE(20, 2);
#undef YTK_SPLIT_WIDE
    YTK_LAUNCH_CHECK();
    return;
  }
  if (B <= 8192 && part && counters) {
    // part: >= nitems * F SplitOut; counters: nitems zeroed ints
    const long long units = (long long)nitems * ((F + 3) / 4);
    if (units * 4 > 0x7fffffffLL - 64) throw std::invalid_argument("split_find: too many (node, feature) blocks");
    // 4 blocks per unit, whole XCD rounds; capped (grid-stride inside): kSplitFeatMaxBlocks
    const unsigned nblk = (unsigned)std::min<long long>((units + 7) / 8 * 32, kSplitFeatMaxBlocks);
#define YTK_SPLIT_FEAT(R, T)                                                                       \
  hipLaunchKernelGGL((split_feat_kernel<R, T>), dim3(nblk), dim3(T), R > 1 ? (size_t)B * 16 : 0,     \
                     reinterpret_cast<hipStream_t>(stream), (long long*)hist, B, F,                \
                     (const int*)nbins_f, (const uint8_t*)fmask, f0, (const int4*)items,           \
                     (SplitOut*)out, gp, (const int*)nitems_dev, (const double*)inv_dev,           \
                     (SplitOut*)part, (int*)counters, nitems)
    if (B <= kFeatThreads) YTK_SPLIT_FEAT(1, 256);
    else if (B <= 2 * kFeatThreads) YTK_SPLIT_FEAT(2, 256);
    else if (B <= 4 * kFeatThreads) YTK_SPLIT_FEAT(4, 256);
    else if (B <= 2048) YTK_SPLIT_FEAT(2, 1024);
    else if (B <= 4096) YTK_SPLIT_FEAT(4, 1024);
    else YTK_SPLIT_FEAT(8, 1024);
#undef YTK_SPLIT_FEAT
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
