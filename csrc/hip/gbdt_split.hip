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
constexpr int kSplitWaves = 8;  // 512 threads: 3-4 features per wave at F=28 (latency bound)

// Grid (items, feature groups): block y owns features y*kSplitWaves + wave (one wave per
// feature when F <= groups*8), so a level's nodes fill many CUs instead of one block each
// walking ~F/8 features serially. With more than one group, every block writes its best
// candidate to part[item][group]; the last block of an item (device-scope counter)
// combines them with the same lexicographic tie-break and resets the counter.
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
  const int fstart = (int)blockIdx.y * kSplitWaves;
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

  // Node totals from the first sampled feature (exact; every wave computes them).
  long long Gq = 0, Hq = 0;
  {
    const int nb0 = nbins_f[f0];
    long long sg = 0, sh = 0;
    for (int bin = l; bin < nb0; bin += kWave) {
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

  for (int f = fstart + wid; f < F; f += fstep) {
    if (!fmask[f]) continue;
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
        v[k] = make_longlong2(0, 0);
        if (bin < nb) v[k] = load(f, bin);
        if (derived && bin < B) hn[(size_t)bin * F + f] = v[k];
        sg += v[k].x;
        sh += v[k].y;
        if (v[k].x != 0 || v[k].y != 0) lastne = bin;
      }
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

}  // namespace ytk

using namespace ytk;

// part / counters (optional): scratch of nitems * ceil(F/8) SplitOut and nitems zeroed ints;
// when given, the features of a node are spread over ceil(F/8) blocks.
extern "C" void ytk_split_find(uintptr_t hist, int B, int F, uintptr_t nbins_f, uintptr_t fmask,
                               int f0, uintptr_t items, int nitems, uintptr_t out, float mcw,
                               float l1, float l2, float max_abs_leaf, double inv_sg,
                               double inv_sh, uintptr_t nitems_dev, uintptr_t inv_dev,
                               uintptr_t part, uintptr_t counters, uintptr_t stream) {
  if (nitems <= 0) return;
  GainParams gp{mcw, l1, l2, max_abs_leaf, inv_sg, inv_sh};
  const int groups = (part && counters) ? (F + kSplitWaves - 1) / kSplitWaves : 1;
  hipLaunchKernelGGL(split_find_kernel, dim3(nitems, groups), dim3(kSplitWaves * 64), 0,
                     reinterpret_cast<hipStream_t>(stream), (long long*)hist, B, F,
                     (const int*)nbins_f, (const uint8_t*)fmask, f0, (const int4*)items,
                     (SplitOut*)out, gp, (const int*)nitems_dev, (const double*)inv_dev,
                     (SplitOut*)part, (int*)counters);
  YTK_LAUNCH_CHECK();
}
